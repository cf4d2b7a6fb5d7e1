// Key-side attention gradients from the probabilities the backward kernel hands over (gfx950,
// wave64), head dim 512:
//     dV = P^T dO,   dK = dS^T Q       per (batch n, head h), P / dS [Lq][Lk] from attn_bwd_kernel
// Replaces the two batched TN GEMMs (M = Lk, N = 512, K = Lq, one per product) that ran at
// 250-270 TFLOP/s on the c3 shapes (b384 / b192 x 300 x 512 x 300: profiles/r03_dkdv.jsonl) —
// short contractions whose per-tile prologue and epilogue the generic tile kernel cannot hide.
// Reference: the dK / dV of autograd's backward of F.multi_head_attention_forward behind every
// nn.MultiheadAttention of mm_multi_transformers.py:57,142-167.
//
// Geometry: an item is (n, h, product, 128-key tile) — the product (dV from P and dO, or dK from
// dS and Q) is part of the item, so a block holds one product's 128 x 512 fp32 accumulator (128
// registers per wave) and streams one row operand: per 128 keys it fetches Lq x (1 KiB + 256 B)
// (the two-product 64-key item of the first version fetched Lq x (2 KiB + 256 B) per 64 keys and
// ran at 2.9 TB/s of LDS fill: profiles/r04/dkdv_v1_vs_gemm.jsonl).  Blocks are persistent (one
// per CU, attn.hip's XCD-contiguous item ranges: the key tiles of one head and product share its
// dO / Q rows in one L2) and stream the queries in chunks of 32:
//  * stage = 32 dO / Q rows (1 KiB each, the swizzled row image of attn_common.h) and the P / dS
//    tile of those rows (32 x 128 keys, 256-B rows, 16-B chunk c of row r at c ^ ((r & 7) << 1):
//    conflict-free transposed reads) = 40 KiB; 4 stages (160 KiB), filled by LDS-DMA from inline
//    asm three chunks ahead, across items too; every wait is an exact vmcnt;
//  * wave w owns head dims 64 w .. +63: per chunk one MFMA k-step of 16x16x32 over 8 key groups x
//    4 dim groups.  Both operands come from ds_read_b64_tr_b16 reads (the dims of dO / Q and the
//    keys of P / dS are columns of their images), in the k-slot order of attn.hip's P V product;
//  * queries past Lq (the last chunk) read a clamped row and are zeroed in the P / dS fragment;
//    keys past Lk compute on whatever the P / dS row holds there and are not stored;
//  * the accumulators go straight from registers to HBM (16-B buffer stores of paired subtiles;
//    the buffer range check drops rows past Lk, so every wave issues exactly 16 stores per item
//    and the waits that follow count them).
// HBM bytes per (n, h): Lq rows of dO and of Q (1 KiB each; once per head when its key tiles share
// the L2), Lq x 128 ceil(Lk / 128) x 2 B of P and of dS, Lk rows of dK and of dV written.
#include "attn_common.h"

namespace jmt {

constexpr int DK_KT = 128;                              // keys per item
constexpr int DK_QC = 32;                               // queries per chunk (one MFMA k-step)
constexpr int DK_PROW = 2 * DK_KT;                      // P / dS image row bytes
constexpr int DK_IMG = DK_QC * AT_ROWB;                 // dO or Q image (32 KiB)
constexpr int DK_PIMG = DK_QC * DK_PROW;                // P or dS image (8 KiB)
constexpr int DK_STAGE = DK_IMG + DK_PIMG;              // 40 KiB
#ifndef JMT_DKDV_NS
#define JMT_DKDV_NS 4                                   // (dev A/B: 3 -> 120 KiB)
#endif
constexpr int DK_NS = JMT_DKDV_NS;                      // stages
constexpr int DK_LDS = DK_NS * DK_STAGE;                // 160 KiB
static_assert(DK_NS >= 2 && DK_NS <= 4, "2-4 stages (the wait table covers 0-2 later stages)");
constexpr int DK_NDMA = DK_QC / 8 + 1;                  // DMA wave-instructions per wave per stage
constexpr int DK_NST = 16;                              // output stores per wave per item

struct AttnDkdvArgs {
  const void* p;
  const void* ds;
  const void* go;
  const void* q;
  const void* k;
  void* dk;
  void* dv;
  void* dq;
  int64_t ldp, sgo_l, sgo_n, sq_l, sq_n, sk_l, sk_n, sdk_l, sdk_n, sdv_l, sdv_n, sdq_l, sdq_n;
  int Lq, Lk, H, nkt, nqd, ipn, nitems;
};

// byte offset of 16-B chunk `c` of row `r` of a P / dS image
__device__ __forceinline__ int pimg_off(int r, int c) {
  return r * DK_PROW + ((c ^ ((r & 7) << 1)) << 4);
}

// byte offset of 16-B chunk `c` of row `r` of a dS image of the dQ product (128 query rows x 32
// keys, 64-B rows): chunk c ^ ((r >> 2) & 3), so the two ds_read_b64 of a fragment (rows li of a
// 16-row group, keys 4 g and 16 + 4 g) are conflict-free
__device__ __forceinline__ int qimg_off(int r, int c) {
  return r * 64 + ((c ^ ((r >> 2) & 3)) << 4);
}

// item -> (n H + h, n, h, product (0: dV, 1: dK, 2: dQ), first key (0, 1) or query (2), chunks).
// Per (n, h): nkt dV items, nkt dK items (128-key tiles, the contraction over queries in 32-row
// chunks), then nqd dQ items (128-query tiles, the contraction over keys in 32-key chunks).
struct DkItem {
  int nh, n, hd, role, k0, nch;
};
__device__ __forceinline__ DkItem dk_decode(const AttnDkdvArgs& a, int it) {
  DkItem d;
  d.nh = it / a.ipn;
  const int r = it - d.nh * a.ipn;
  if (r < 2 * a.nkt) {
    d.role = r >= a.nkt;
    d.k0 = (r - d.role * a.nkt) * DK_KT;
    d.nch = (a.Lq + DK_QC - 1) / DK_QC;
  } else {
    d.role = 2;
    d.k0 = (r - 2 * a.nkt) * DK_KT;
    d.nch = (a.Lk + DK_QC - 1) / DK_QC;
  }
  d.n = d.nh / a.H;
  d.hd = d.nh - d.n * a.H;
  return d;
}

// one stage: rows q0 .. q0+31 (clamped to Lq - 1) of dO or Q, and of the P or dS tile (keys
// k0 .. k0+127): 4 + 1 DMA wave-instructions per wave.  Row offsets in 32-bit byte arithmetic
// from a per-head base (the host checks Lq rows fit): the 64-bit row products of stage_rows cost
// ~25 scalar instructions per DMA, and the CU's one scalar unit serves all 8 waves.
template <typename T>
__device__ __forceinline__ void dkdv_stage(char* st, const AttnDkdvArgs& a, const DkItem& d,
                                           int q0) {
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (d.role == 2) {
    // dQ chunk: K rows q0 .. q0+31 (here q0 is the first KEY of the chunk) and the dS tile of the
    // item's 128 queries x those 32 keys (one wave-instruction per wave: 16 rows of 64 B)
    const char* kb = (const char*)((const T*)a.k + (int64_t)d.n * a.sk_n + d.hd * AT_DH);
    const int ldk = (int)(a.sk_l * (int64_t)sizeof(T));
#pragma unroll
    for (int i = 0; i < DK_QC / 8; ++i) {
      const int r = wu * (DK_QC / 8) + i;
      const int src = min(q0 + r, a.Lk - 1);
      const unsigned off = (unsigned)(lane ^ ((r & 7) << 1)) << 4;
      glds16_asm(kb + (unsigned)(src * ldk) + off, st + r * AT_ROWB);
    }
    const int r = 16 * wu + (lane >> 2);                // dS image row (query d.k0 + r)
    const int c = (lane & 3) ^ ((r >> 2) & 3);          // the logical chunk this lane's 16 B hold
    const int src_row = min(d.k0 + r, a.Lq - 1);
    JMT_DCHECK(src_row >= 0 && q0 + 8 * c + 8 <= a.ldp);
    // tile-major dS (jmt_attn_bwd with dq = NULL): [key tile q0 / 32][query][32 keys]
    const char* pb = (const char*)((const T*)a.ds + (int64_t)d.nh * a.Lq * a.ldp);
    glds16_asm(pb + (unsigned)(((q0 >> 5) * a.Lq + src_row) * 64) + 16 * c,
               st + DK_IMG + wu * 1024);
    return;
  }
  const char* rb;
  int ldb;
  if (d.role == 0) {
    rb = (const char*)((const T*)a.go + (int64_t)d.n * a.sgo_n + d.hd * AT_DH);
    ldb = (int)(a.sgo_l * (int64_t)sizeof(T));
  } else {
    rb = (const char*)((const T*)a.q + (int64_t)d.n * a.sq_n + d.hd * AT_DH);
    ldb = (int)(a.sq_l * (int64_t)sizeof(T));
  }
#pragma unroll
  for (int i = 0; i < DK_QC / 8; ++i) {
    const int r = wu * (DK_QC / 8) + i;
    const int src = min(q0 + r, a.Lq - 1);
    const unsigned off = (unsigned)(lane ^ ((r & 7) << 1)) << 4;
    glds16_asm(rb + (unsigned)(src * ldb) + off, st + r * AT_ROWB);
  }
  const int r = 4 * wu + (lane >> 4);                   // P / dS image row of this lane's 16 B
  const int cs = (lane & 15) ^ ((r & 7) << 1);          // the logical chunk it holds
  const int src_row = min(q0 + r, a.Lq - 1);
  JMT_DCHECK(src_row >= 0 && d.k0 + 8 * cs + 8 <= a.ldp);
  if (a.dq) {      // tile-major P / dS (jmt_attn_bwd with dq = NULL): [key tile][query][32 keys]
    const char* pb = (const char*)((const T*)(d.role == 0 ? a.p : a.ds) +
                                   (int64_t)d.nh * a.Lq * a.ldp);
    glds16_asm(pb + (unsigned)((((d.k0 >> 5) + (cs >> 2)) * a.Lq + src_row) * 64) +
                   16 * (cs & 3),
               st + DK_IMG + wu * 1024);
    return;
  }
  const char* pb = (const char*)((const T*)(d.role == 0 ? a.p : a.ds) +
                                 (int64_t)d.nh * a.Lq * a.ldp + d.k0);
  glds16_asm(pb + (unsigned)(src_row * (int)(a.ldp * sizeof(T))) + 16 * cs,
             st + DK_IMG + wu * 1024);
}

// s_waitcnt vmcnt(stages * DK_NDMA + stores * DK_NST) for the counts the chunk loop meets:
// 0-2 later stages and 0-3 items' output stores in flight behind the awaited stage
template <int S>
__device__ __forceinline__ void dkdv_wait_s(int stores) {
  switch (stores) {
    case 0: wait_vmcnt<S * DK_NDMA>(); break;
    case 1: wait_vmcnt<S * DK_NDMA + DK_NST>(); break;
    case 2: wait_vmcnt<S * DK_NDMA + 2 * DK_NST>(); break;
    default: wait_vmcnt<S * DK_NDMA + 3 * DK_NST>(); break;
  }
}
__device__ __forceinline__ void dkdv_wait(int stages, int stores) {
  if (stages == 0) dkdv_wait_s<0>(stores);
  else if (stages == 1) dkdv_wait_s<1>(stores);
  else dkdv_wait_s<2>(stores);
}

template <typename T>
__global__ __launch_bounds__(512, 2) void attn_dkdv_kernel(AttnDkdvArgs a) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  int item, iend, istride;
  item_range(a.nitems, item, iend, istride);
  if (item >= iend) return;

  int tb[4], pb[8];                                     // transposed-read lane bases
#pragma unroll
  for (int t = 0; t < 4; ++t) tb[t] = tr_base(4 * (w & 1) + t, li, g, 0) + 256 * (w >> 1);
#pragma unroll
  for (int kg = 0; kg < 8; ++kg)
    pb[kg] = pimg_off(4 * g + (li >> 2), 2 * kg + ((li & 3) >> 1)) + 8 * (li & 1);
  // dQ: dS fragment of query group qg = rows 16 qg + li, keys 4 g .. +3 (k-slots 0-3) and
  // 16 + 4 g .. +3 (k-slots 4-7): the k-slot order of the transposed K-row reads
  const int qb0 = qimg_off(li, g >> 1) + 8 * (g & 1);
  const int qb1 = qimg_off(li, 2 + (g >> 1)) + 8 * (g & 1);

  // issue cursor: the chunk whose stage goes out next (runs DK_NS - 1 chunks ahead of the compute)
  int is_item = item, is_c = 0;
  DkItem is_d = dk_decode(a, item);
  bool is_ok = true;
  int is_buf = 0;
  unsigned after = 0;      // 4 bits per buffer: store batches issued after the stage it holds
  int inflight = 0;        // stages issued and not yet waited for
  auto issue = [&]() {
    if (is_ok) {
      dkdv_stage<T>(smem + is_buf * DK_STAGE, a, is_d, DK_QC * is_c);
      after &= ~(15u << (4 * is_buf));
      ++inflight;
      if (++is_c == is_d.nch) {
        is_c = 0;
        is_item += istride;
        is_ok = is_item < iend;
        if (is_ok) is_d = dk_decode(a, is_item);
      }
    }
    is_buf = is_buf == DK_NS - 1 ? 0 : is_buf + 1;
  };
  for (int i = 0; i < DK_NS - 1; ++i) issue();
  int buf = 0;

  while (true) {
    const DkItem d = dk_decode(a, item);
    const bool more = item + istride < iend;
    f32x4 acc[8][4];
#pragma unroll
    for (int kg = 0; kg < 8; ++kg)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[kg][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c = 0; c < d.nch; ++c) {
      const char* cur = smem + buf * DK_STAGE;
      // this chunk's stage landed (the later stages and the output stores issued after it may
      // stay in flight), and every wave is done reading the buffer restaged below
      dkdv_wait(inflight - 1, (after >> (4 * buf)) & 15);
      --inflight;
      lds_barrier();
      issue();
      F kf[8];
      const int c0 = DK_QC * c;                         // first contraction index of the chunk
      const int clen = d.role == 2 ? a.Lk : a.Lq;       // contraction length
      if (d.role != 2) {
#pragma unroll
        for (int kg = 0; kg < 8; ++kg) {
          const Hf lo = tr_read<Hf>(cur + DK_IMG + pb[kg]);
          const Hf hi = tr_read<Hf>(cur + DK_IMG + pb[kg] + 16 * DK_PROW);
          kf[kg] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      } else {
#pragma unroll
        for (int qg = 0; qg < 8; ++qg) {
          const Hf lo = *(const Hf*)(cur + DK_IMG + qb0 + 1024 * qg);
          const Hf hi = *(const Hf*)(cur + DK_IMG + qb1 + 1024 * qg);
          kf[qg] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
      if (c0 + DK_QC > clen) {   // k-slot e holds contraction index c0 + 16 (e >> 2) + 4 g + (e & 3)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool in = c0 + 16 * (e >> 2) + 4 * g + (e & 3) < clen;
#pragma unroll
          for (int kg = 0; kg < 8; ++kg) kf[kg][e] = in ? kf[kg][e] : from_f<T>(0.f);
        }
      }
      F df[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const Hf lo = tr_read<Hf>(cur + tb[t]);
        const Hf hi = tr_read<Hf>(cur + tb[t] + 16 * AT_ROWB);
        df[t] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int kg = 0; kg < 8; ++kg) acc[kg][t] = mfma16(df[t], kf[kg], acc[kg][t]);
      buf = buf == DK_NS - 1 ? 0 : buf + 1;
    }

    // ---- outputs: lane = key (dQ: query) k0 + 16 kg + li, dims 64 w + 16 t + 4 g + r; subtiles
    // t, t + 1 paired by v_permlane16_swap into 8 consecutive dims per lane (store_acc_direct's
    // scheme)
    {
      T* ob = d.role == 0 ? (T*)a.dv + (int64_t)d.n * a.sdv_n
            : d.role == 1 ? (T*)a.dk + (int64_t)d.n * a.sdk_n : (T*)a.dq + (int64_t)d.n * a.sdq_n;
      const int64_t sl = d.role == 0 ? a.sdv_l : d.role == 1 ? a.sdk_l : a.sdq_l;
      ob += (int64_t)d.hd * AT_DH + (int64_t)d.k0 * sl;
      const uint64_t ba = (uint64_t)(uintptr_t)ob;
      const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)ba);
      const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(ba >> 32));
      const int nrows = min(DK_KT, (d.role == 2 ? a.Lq : a.Lk) - d.k0);
      const int bytes = __builtin_amdgcn_readfirstlane((int)(nrows * sl * (int64_t)sizeof(T)));
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((uint64_t)bhi << 32) | blo), 0, bytes, 0x00020000);
      const int sl32 = (int)sl;
#pragma unroll
      for (int kg = 0; kg < 8; ++kg) {
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          uint32_t pk[2][2];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh)
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
              T two[2] = {from_f<T>(acc[kg][2 * jp + hh][2 * qq]),
                          from_f<T>(acc[kg][2 * jp + hh][2 * qq + 1])};
              pk[hh][qq] = *(const uint32_t*)two;
            }
          const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
          const int col = 64 * w + 16 * (2 * jp + (g & 1)) + 8 * (g >> 1);
          const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
          const int off = ((16 * kg + li) * sl32 + col) * (int)sizeof(T);
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, 0, 0);
        }
      }
    }
    // these stores follow the stages in flight (the next two chunks'; the free buffer's count is
    // reset when it is restaged)
    after += 0x1111;
    if (!more) break;
    item += istride;
  }
  wait_vmcnt<0>();
}

static int dkdv_grid(int nitems) {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 8)
      v = 8;
    ncu = v / 8 * 8;
  }
  return nitems > ncu ? ncu : nitems;
}

}  // namespace jmt

using namespace jmt;

extern "C" int jmt_attn_dkdv(int dt, int N, int H, int Lq, int Lk, int dh, const void* p,
                             const void* ds, int64_t ldp, const void* go, int64_t sgo_l,
                             int64_t sgo_n, const void* q, int64_t sq_l, int64_t sq_n,
                             const void* k, int64_t sk_l, int64_t sk_n, void* dk, int64_t sdk_l,
                             int64_t sdk_n, void* dv, int64_t sdv_l, int64_t sdv_n, void* dq,
                             int64_t sdq_l, int64_t sdq_n, void* stream) {
  if (N == 0 || Lk == 0) return JMT_OK;
  if (!((dt == JMT_BF16 || dt == JMT_F16) && dh == AT_DH))
    return set_error(JMT_ERR_UNSUPPORTED, "jmt_attn_dkdv: dtype %d / head dim %d not supported",
                     dt, dh);
  JMT_CHECK_ARG(N > 0 && H > 0 && Lq > 0 && Lk > 0, "jmt_attn_dkdv: bad sizes");
  const void* ptrs[] = {p, ds, go, q, dk, dv};
  for (int i = 0; i < 6; ++i)
    JMT_CHECK_ARG(ptrs[i] != nullptr && ((uintptr_t)ptrs[i] & 15) == 0,
                  "jmt_attn_dkdv: operand %d null or not 16-B aligned", i);
  const int64_t strides[] = {ldp, sgo_l, sgo_n, sq_l, sq_n, sdk_l, sdk_n, sdv_l, sdv_n};
  for (int i = 0; i < 9; ++i)
    JMT_CHECK_ARG(strides[i] % 8 == 0, "jmt_attn_dkdv: stride %d not a multiple of 8", i);
  const int nkt = (Lk + DK_KT - 1) / DK_KT;
  JMT_CHECK_ARG(ldp >= (int64_t)nkt * DK_KT,
                "jmt_attn_dkdv: ldp must cover 128-key tiles (>= %d)", nkt * DK_KT);
  JMT_CHECK_ARG(sdk_l >= H * AT_DH && sdv_l >= H * AT_DH &&
                    (int64_t)DK_KT * sdk_l * 2 < (1LL << 31) &&
                    (int64_t)DK_KT * sdv_l * 2 < (1LL << 31),
                "jmt_attn_dkdv: dK / dV row stride out of range");
  const int nqd = dq ? (Lq + DK_KT - 1) / DK_KT : 0;   // dQ items per (n, h)
  if (dq) {
    JMT_CHECK_ARG(k != nullptr && ((uintptr_t)k & 15) == 0 && ((uintptr_t)dq & 15) == 0 &&
                      sk_l % 8 == 0 && sk_n % 8 == 0 && sdq_l % 8 == 0 && sdq_n % 8 == 0,
                  "jmt_attn_dkdv: k / dq null, misaligned or strides not multiples of 8");
    JMT_CHECK_ARG(sdq_l >= H * AT_DH && (int64_t)DK_KT * sdq_l * 2 < (1LL << 31) &&
                      (int64_t)Lk * sk_l * 2 < (1LL << 31),
                  "jmt_attn_dkdv: dQ / K row stride out of range");
  }
  JMT_CHECK_ARG((int64_t)N * H * (2 * nkt + nqd) < (1LL << 31), "jmt_attn_dkdv: too many items");
  JMT_CHECK_ARG((int64_t)Lq * sgo_l * 2 < (1LL << 31) && (int64_t)Lq * sq_l * 2 < (1LL << 31) &&
                    (int64_t)Lq * ldp * 2 < (1LL << 31),
                "jmt_attn_dkdv: Lq rows of dO / Q / P exceed 2 GiB");
  AttnDkdvArgs a = {};
  a.p = p; a.ds = ds; a.go = go; a.q = q; a.k = k; a.dk = dk; a.dv = dv; a.dq = dq;
  a.ldp = ldp; a.sgo_l = sgo_l; a.sgo_n = sgo_n; a.sq_l = sq_l; a.sq_n = sq_n;
  a.sk_l = sk_l; a.sk_n = sk_n;
  a.sdk_l = sdk_l; a.sdk_n = sdk_n; a.sdv_l = sdv_l; a.sdv_n = sdv_n;
  a.sdq_l = sdq_l; a.sdq_n = sdq_n;
  a.Lq = Lq; a.Lk = Lk; a.H = H; a.nkt = nkt; a.nqd = nqd; a.ipn = 2 * nkt + nqd;
  a.nitems = N * H * a.ipn;
  const dim3 grid(dkdv_grid(a.nitems));
  hipStream_t st = as_stream(stream);
  if (dt == JMT_BF16) {
    static bool once = ((void)hipFuncSetAttribute((const void*)attn_dkdv_kernel<__bf16>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, DK_LDS),
                        true);
    (void)once;
    hipLaunchKernelGGL((attn_dkdv_kernel<__bf16>), grid, dim3(512), (size_t)DK_LDS, st, a);
  } else {
    static bool once = ((void)hipFuncSetAttribute((const void*)attn_dkdv_kernel<_Float16>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, DK_LDS),
                        true);
    (void)once;
    hipLaunchKernelGGL((attn_dkdv_kernel<_Float16>), grid, dim3(512), (size_t)DK_LDS, st, a);
  }
  JMT_LAUNCH_CHECK("jmt_attn_dkdv");
  return JMT_OK;
}
