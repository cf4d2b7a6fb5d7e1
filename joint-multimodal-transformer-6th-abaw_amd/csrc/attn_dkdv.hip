// Key-side attention gradients from the probabilities the backward kernel hands over (gfx950,
// wave64), head dim 512:
//     dV = P^T dO,   dK = dS^T Q       per (batch n, head h), P / dS [Lq][Lk] from attn_bwd_kernel
// Replaces the two batched TN GEMMs (M = Lk, N = 512, K = Lq, one per product) that ran at
// 250-270 TFLOP/s on the c3 shapes (b384 / b192 x 300 x 512 x 300: profiles/r03_dkdv.jsonl) —
// short contractions whose per-tile prologue and epilogue the generic tile kernel cannot hide.
// Reference: the dK / dV of autograd's backward of F.multi_head_attention_forward behind every
// nn.MultiheadAttention of mm_multi_transformers.py:57,142-167.
//
// Geometry: an item is (n, h, 64-key tile); a block (8 waves, one per CU, persistent over items
// with attn.hip's XCD-contiguous item ranges, so the key tiles of one head share its dO / Q rows in
// one L2) streams the queries in chunks of 32:
//  * stage = dO rows, Q rows (32 x 1 KiB each, the swizzled row image of attn_common.h) and the
//    P / dS tile (32 queries x 64 keys, 128-B rows, 16-B chunk c of row r at c ^ ((r >> 1 & 3) << 1):
//    the transposed reads below are conflict-free) = 72 KiB, double-buffered (144 KiB), filled by
//    LDS-DMA issued from inline asm (every wait explicit) one chunk ahead, across items too;
//  * waves 0-3 compute dV, waves 4-7 dK, wave w the 128 head dims 128 (w & 3) ..: per chunk one
//    MFMA k-step of 16x16x32 over 4 key groups x 8 dim groups (128 accumulator registers).  Both
//    operands come from ds_read_b64_tr_b16 reads (the dims of dO / Q and the keys of P / dS are
//    columns of their images), in the k-slot order of attn.hip's P V product;
//  * queries past Lq (the last chunk) read a clamped row and are zeroed in the P / dS fragment;
//    keys past Lk compute on whatever the P / dS row holds there and are not stored;
//  * the accumulators go straight from registers to HBM (16-B buffer stores of paired subtiles;
//    the buffer range check drops rows past Lk, so every wave issues exactly 16 stores per item
//    and the next item's first wait can leave them in flight).
// HBM bytes per (n, h): Lq rows of dO and Q (1 KiB each; once per head when its key tiles share
// the L2), Lq x 64 ceil(Lk / 64) x 2 B of P and of dS, Lk rows of dK and dV written.
#include "attn_common.h"

namespace jmt {

constexpr int DK_KT = 64;                               // keys per item
constexpr int DK_QC = 32;                               // queries per chunk (one MFMA k-step)
constexpr int DK_PROW = 2 * DK_KT;                      // P / dS image row bytes
constexpr int DK_IMG = DK_QC * AT_ROWB;                 // dO or Q image (32 KiB)
constexpr int DK_PIMG = DK_QC * DK_PROW;                // P or dS image (4 KiB)
constexpr int DK_STAGE = 2 * DK_IMG + 2 * DK_PIMG;      // 72 KiB
constexpr int DK_LDS = 2 * DK_STAGE;                    // 144 KiB
constexpr int DK_NST = 16;                              // output stores per wave per item

struct AttnDkdvArgs {
  const void* p;
  const void* ds;
  const void* go;
  const void* q;
  void* dk;
  void* dv;
  int64_t ldp, sgo_l, sgo_n, sq_l, sq_n, sdk_l, sdk_n, sdv_l, sdv_n;
  int Lq, Lk, H, nkt, nitems;
};

// byte offset of 16-B chunk `c` of row `r` of a P / dS image
__device__ __forceinline__ int pimg_off(int r, int c) {
  return r * DK_PROW + ((c ^ (((r >> 1) & 3) << 1)) << 4);
}

// one stage: dO and Q rows q0 .. q0+31 (clamped to Lq - 1), the P (waves 0-3) / dS (waves 4-7)
// tile of those rows, keys k0 .. k0+63: 4 + 4 + 1 DMA wave-instructions per wave
template <typename T>
__device__ __forceinline__ void dkdv_stage(char* st, const AttnDkdvArgs& a, int nh, int n, int hd,
                                           int k0, int q0) {
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  stage_rows<T, DK_QC, 8, true>(st, (const T*)a.go + (int64_t)n * a.sgo_n + hd * AT_DH, a.sgo_l,
                                q0, a.Lq);
  stage_rows<T, DK_QC, 8, true>(st + DK_IMG, (const T*)a.q + (int64_t)n * a.sq_n + hd * AT_DH,
                                a.sq_l, q0, a.Lq);
  const int i = wu & 3;
  const int r = 8 * i + (lane >> 3);                    // image row of this lane's 16 B
  const int cs = (lane & 7) ^ (((r >> 1) & 3) << 1);    // the logical chunk it holds
  const int src_row = min(q0 + r, a.Lq - 1);
  JMT_DCHECK(src_row >= 0 && k0 + 8 * cs + 8 <= a.ldp);
  const T* src = (const T*)(wu < 4 ? a.p : a.ds) + ((int64_t)nh * a.Lq + src_row) * a.ldp + k0 +
                 8 * cs;
  glds16_asm(src, st + 2 * DK_IMG + (wu >> 2) * DK_PIMG + i * 1024);
}

// s_waitcnt vmcnt(n) for the few counts the item loop needs
__device__ __forceinline__ void dkdv_wait(int n) {
  if (n == 0) wait_vmcnt<0>();
  else wait_vmcnt<DK_NST>();
}

template <typename T>
__global__ __launch_bounds__(512, 2) void attn_dkdv_kernel(AttnDkdvArgs a) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int role = w >> 2, dq = w & 3;                  // role 0: dV from P, dO; 1: dK from dS, Q
  const int nqc = (a.Lq + DK_QC - 1) / DK_QC;
  int item, iend, istride;
  item_range(a.nitems, item, iend, istride);
  if (item >= iend) return;

  int tb[8], pb[4];                                     // transposed-read lane bases
#pragma unroll
  for (int t = 0; t < 8; ++t) tb[t] = tr_base(t, li, g, dq >> 1) + 256 * (dq & 1);
#pragma unroll
  for (int kg = 0; kg < 4; ++kg)
    pb[kg] = pimg_off(4 * g + (li >> 2), 2 * kg + ((li & 3) >> 1)) + 8 * (li & 1);

  auto decode = [&](int it, int& nh, int& n, int& hd, int& k0) {
    nh = it / a.nkt;
    n = nh / a.H;
    hd = nh - n * a.H;
    k0 = (it - nh * a.nkt) * DK_KT;
  };
  int nh, n, hd, k0;
  decode(item, nh, n, hd, k0);
  int buf = 0;
  dkdv_stage<T>(smem, a, nh, n, hd, k0, 0);
  int nst = 0;                                          // stores issued after this item's stage 0

  while (true) {
    const int nxt = item + istride;
    const bool more = nxt < iend;
    int nh2 = 0, n2 = 0, hd2 = 0, k02 = 0;
    if (more) decode(nxt, nh2, n2, hd2, k02);
    f32x4 acc[4][8];
#pragma unroll
    for (int kg = 0; kg < 4; ++kg)
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[kg][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c = 0; c < nqc; ++c) {
      const char* cur = smem + buf * DK_STAGE;
      // this chunk's stage landed (only the previous item's output stores may still be in
      // flight), and every wave is done reading the other buffer
      dkdv_wait(c == 0 ? nst : 0);
      lds_barrier();
      if (c + 1 < nqc) dkdv_stage<T>(smem + (buf ^ 1) * DK_STAGE, a, nh, n, hd, k0, DK_QC * (c + 1));
      else if (more) dkdv_stage<T>(smem + (buf ^ 1) * DK_STAGE, a, nh2, n2, hd2, k02, 0);
      const char* img = cur + role * DK_IMG;
      const char* pim = cur + 2 * DK_IMG + role * DK_PIMG;
      F kf[4];
#pragma unroll
      for (int kg = 0; kg < 4; ++kg) {
        const Hf lo = tr_read<Hf>(pim + pb[kg]);
        const Hf hi = tr_read<Hf>(pim + pb[kg] + 16 * DK_PROW);
        kf[kg] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      const int q0 = DK_QC * c;
      if (q0 + DK_QC > a.Lq) {                          // k-slot e holds query 16 (e >> 2) + 4 g + (e & 3)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool in = q0 + 16 * (e >> 2) + 4 * g + (e & 3) < a.Lq;
#pragma unroll
          for (int kg = 0; kg < 4; ++kg) kf[kg][e] = in ? kf[kg][e] : from_f<T>(0.f);
        }
      }
      {   // dim subtiles in double-buffered pairs (t = 2 b + i)
        F fa[2], fb[2];
        auto dbatch = [&](F* dst, int b) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const char* ad = img + tb[2 * b + i];
            const Hf lo = tr_read<Hf>(ad);
            const Hf hi = tr_read<Hf>(ad + 16 * AT_ROWB);
            dst[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          }
        };
        dbatch(fa, 0);
#pragma unroll
        for (int b = 0; b < 4; b += 2) {
          dbatch(fb, b + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int kg = 0; kg < 4; ++kg)
              acc[kg][2 * b + i] = mfma16(fa[i], kf[kg], acc[kg][2 * b + i]);
          __builtin_amdgcn_sched_barrier(0);
          if (b + 2 < 4) dbatch(fa, b + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int kg = 0; kg < 4; ++kg)
              acc[kg][2 * b + 2 + i] = mfma16(fb[i], kf[kg], acc[kg][2 * b + 2 + i]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      buf ^= 1;
    }

    // ---- outputs: lane = key k0 + 16 kg + li, dims 128 dq + 16 t + 4 g + r; subtiles t, t + 1
    // paired by v_permlane16_swap into 8 consecutive dims per lane (store_acc_direct's scheme)
    {
      T* ob = role == 0 ? (T*)a.dv + (int64_t)n * a.sdv_n : (T*)a.dk + (int64_t)n * a.sdk_n;
      const int64_t sl = role == 0 ? a.sdv_l : a.sdk_l;
      ob += (int64_t)hd * AT_DH + (int64_t)k0 * sl;
      const uint64_t ba = (uint64_t)(uintptr_t)ob;
      const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)ba);
      const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(ba >> 32));
      const int nrows = min(DK_KT, a.Lk - k0);
      const int bytes = __builtin_amdgcn_readfirstlane((int)(nrows * sl * (int64_t)sizeof(T)));
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((uint64_t)bhi << 32) | blo), 0, bytes, 0x00020000);
      const int sl32 = (int)sl;
#pragma unroll
      for (int kg = 0; kg < 4; ++kg) {
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
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
          const int col = 128 * dq + 16 * (2 * jp + (g & 1)) + 8 * (g >> 1);
          const u32x4 v = {r0[0], r1[0], r0[1], r1[1]};
          const int off = ((16 * kg + li) * sl32 + col) * (int)sizeof(T);
          __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, 0, 0);
        }
      }
    }
    nst = DK_NST;
    if (!more) break;
    item = nxt; nh = nh2; n = n2; hd = hd2; k0 = k02;
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
                             int64_t sgo_n, const void* q, int64_t sq_l, int64_t sq_n, void* dk,
                             int64_t sdk_l, int64_t sdk_n, void* dv, int64_t sdv_l,
                             int64_t sdv_n, void* stream) {
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
                "jmt_attn_dkdv: ldp must cover 64-key tiles (>= %d)", nkt * DK_KT);
  JMT_CHECK_ARG(sdk_l >= H * AT_DH && sdv_l >= H * AT_DH &&
                    (int64_t)DK_KT * sdk_l * 2 < (1LL << 31) &&
                    (int64_t)DK_KT * sdv_l * 2 < (1LL << 31),
                "jmt_attn_dkdv: dK / dV row stride out of range");
  JMT_CHECK_ARG((int64_t)N * H * nkt < (1LL << 31), "jmt_attn_dkdv: too many items");
  AttnDkdvArgs a = {};
  a.p = p; a.ds = ds; a.go = go; a.q = q; a.dk = dk; a.dv = dv;
  a.ldp = ldp; a.sgo_l = sgo_l; a.sgo_n = sgo_n; a.sq_l = sq_l; a.sq_n = sq_n;
  a.sdk_l = sdk_l; a.sdk_n = sdk_n; a.sdv_l = sdv_l; a.sdv_n = sdv_n;
  a.Lq = Lq; a.Lk = Lk; a.H = H; a.nkt = nkt; a.nitems = N * H * nkt;
  const dim3 grid(dkdv_grid(a.nitems));
  hipStream_t st = as_stream(stream);
  if (dt == JMT_BF16) {
    static bool once = (hipFuncSetAttribute((const void*)attn_dkdv_kernel<__bf16>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, DK_LDS),
                        true);
    (void)once;
    hipLaunchKernelGGL((attn_dkdv_kernel<__bf16>), grid, dim3(512), (size_t)DK_LDS, st, a);
  } else {
    static bool once = (hipFuncSetAttribute((const void*)attn_dkdv_kernel<_Float16>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, DK_LDS),
                        true);
    (void)once;
    hipLaunchKernelGGL((attn_dkdv_kernel<_Float16>), grid, dim3(512), (size_t)DK_LDS, st, a);
  }
  JMT_LAUNCH_CHECK("jmt_attn_dkdv");
  return JMT_OK;
}
