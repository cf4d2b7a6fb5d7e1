// LDS-tiled MFMA GEMM for gfx950 (CDNA4), wave64.
//
//   C[b] = epilogue( alpha * A[b] (M x K) . B[b] (K x N) )
//
// Serves every matmul on the JMT path: nn.Linear forward (NT), its dgrad
// (NN) and wgrad (TN, split-K over the B*T tokens), and the attention products S = Q K^T,
// O = P V and their backward (batched over (batch, head) with two batch strides).
//
// Design:
//  * 256 threads = 4 waves in a 2x2 grid, block tile 128x128, wave tile 64x64 = 4x4 MFMA tiles.
//  * 16-bit inputs: v_mfma_f32_16x16x32_{bf16,f16}, BK = 64.  f32 inputs (the fp32 parity mode):
//    v_mfma_f32_16x16x4_f32 (exact f32 fma chain), BK = 32.  Either way one K-tile is 128 bytes
//    per row, so the staging code is shared.
//  * Each operand is staged global -> registers -> LDS (double-buffered, loads of tile k+1 issued
//    before the MFMAs of tile k, LDS writes after them: T14).  The LDS image depends on the
//    operand's memory order:
//      K-major operand  -> image [row][k], 16-B chunks XOR-swizzled by (row>>1)&7, read with
//                          ds_read_b128 (conflict-free for the 16-row fragment reads);
//      MN-major operand -> image [k][row] copied straight (no register transpose), 32-B pairs
//                          swizzled by t(k), read with ds_read_b64_tr_b16 (T10) for 16-bit types.
//  * Operands may be K-concatenations of up to 8 tensors (cat(...) @ W^T without a concat copy)
//    or per-batch pointer tables; C may be a per-batch pointer table.
//  * split-K writes fp32 partial slabs to a caller-owned workspace; jmt_gemm launches the
//    reduce + epilogue kernel afterwards (deterministic, no atomics).
//  * XCD-aware block -> tile remap: blocks that share an A row panel run on the same XCD (T1).
#include "common.h"

namespace jmt {

constexpr int GT = 256;     // threads per block
constexpr int BMT = 128;    // block tile rows (M)
constexpr int BNT = 128;    // block tile cols (N)
constexpr int MAXP = 8;

struct GemmParams {
  const void* a_ptr[MAXP];
  const void* b_ptr[MAXP];
  void* c_ptr[MAXP];
  const float* bias;
  const void* aux;
  float* ws;
  int64_t lda, ldb, ldc, ldaux;
  int64_t sA0, sA1, sB0, sB1, sC0, sC1;
  int a_mode, b_mode, c_mode;   // 0 strided, 1 pointer per b0, 2 K-concat (a/b only)
  int a_kseg, b_kseg;           // K-concat segment length (multiple of BK)
  int M, N, K;
  int batch0, batch1;
  int splits, k_per_split;
  float alpha, beta;
  int bias_mode;                // 0 none, 1 per column n, 2 per row m
  int relu;
  int c_dtype;
  int aux_dtype;
  int tiles_m, tiles_n;
  int c_vec;                    // C (and aux) rows 16-B aligned for 16-B vector stores
  int dbg;                      // development ablations: 1 skip MFMA, 2 skip epilogue stores
};

template <typename T> struct Vec { static constexpr int n = 16 / sizeof(T); };

// ------------------------------------------------------------------ operand addressing
template <typename T>
__device__ __forceinline__ const T* operand_base(const void* const* ptrs, int mode, int64_t s0,
                                                 int64_t s1, int b0, int b1, int kseg, int k0,
                                                 int& kloc) {
  if (mode == 2) {
    const int seg = k0 / kseg;
    kloc = k0 - seg * kseg;
    return (const T*)ptrs[seg];
  }
  kloc = k0;
  const T* p = (const T*)ptrs[mode == 1 ? b0 : 0];
  return p + (mode == 1 ? 0 : (int64_t)b0 * s0) + (int64_t)b1 * s1;
}

// K-tile geometry: KB = bytes per operand row of one K-tile (128 or 64), BKE = KB / sizeof(T)
// K elements.  Register staging (used only for a trailing partial K-tile): each thread moves
// KB/32 chunks of 16 B per operand.  K-major image: 128 rows x KB/16 chunks; MN-major image:
// BKE rows x (128*sizeof(T)/16) chunks.
template <typename T, bool KMAJ, int KB>
__device__ __forceinline__ void stage_load(uint4 (&r)[KB / 32], const T* base, int64_t ld,
                                           int rows_lim, int r0, int k_lim, int kloc) {
  constexpr int V = Vec<T>::n;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < KB / 32; ++i) {
    const int id = tid + GT * i;
    int row, kk;
    if constexpr (KMAJ) {
      constexpr int CPRK = KB / 16;
      row = id / CPRK;
      kk = (id % CPRK) * V;
    } else {
      constexpr int CPR = BMT * (int)sizeof(T) / 16;   // chunks per image row
      kk = id / CPR;
      row = (id % CPR) * V;
    }
    const int gr = r0 + row;
    const int gk = kloc + kk;   // k index local to the operand segment
    uint4 v = make_uint4(0, 0, 0, 0);
    if constexpr (KMAJ) {
      if (gr < rows_lim && gk < k_lim) {
        const T* src = base + (int64_t)gr * ld + gk;
        if (gk + V <= k_lim) {
          v = *(const uint4*)src;
        } else {
          T tmp[V];
#pragma unroll
          for (int e = 0; e < V; ++e) tmp[e] = (gk + e < k_lim) ? src[e] : from_f<T>(0.f);
          v = *(uint4*)tmp;
        }
      }
    } else {
      if (gk < k_lim && gr < rows_lim) {
        const T* src = base + (int64_t)gk * ld + gr;
        if (gr + V <= rows_lim) {
          v = *(const uint4*)src;
        } else {
          T tmp[V];
#pragma unroll
          for (int e = 0; e < V; ++e) tmp[e] = (gr + e < rows_lim) ? src[e] : from_f<T>(0.f);
          v = *(uint4*)tmp;
        }
      }
    }
    r[i] = v;
  }
}

// byte offset of 16-B chunk `c` of image row `row` in a K-major image (KB-byte rows); the XOR
// makes the 16-row fragment reads (ds_read_b128) conflict-free.
template <int KB>
__device__ __forceinline__ int kmaj_off(int row, int c) {
  if constexpr (KB == 128) return row * 128 + ((c ^ ((row >> 1) & 7)) << 4);
  else return row * 64 + ((c ^ ((row >> 2) & 3)) << 4);
}
// byte offset of element column `m` (16-bit) of image row `k` in a 16-bit MN-major image
// (256-B rows, 32-B pairs swizzled by t(k): conflict-free ds_read_b64_tr_b16)
__device__ __forceinline__ int mnmaj16_off(int k, int m) {
  const int c = m >> 3;
  const int t = (k & 3) | (((k >> 3) & 1) << 2);
  const int cp = ((((c >> 1) ^ t)) << 1) | (c & 1);
  return k * 256 + (cp << 4) + ((m & 7) << 1);
}

template <typename T, bool KMAJ, int KB>
__device__ __forceinline__ void stage_store(char* img, const uint4 (&r)[KB / 32]) {
  constexpr int V = Vec<T>::n;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < KB / 32; ++i) {
    const int id = tid + GT * i;
    int off;
    if constexpr (KMAJ) {
      constexpr int CPRK = KB / 16;
      off = kmaj_off<KB>(id / CPRK, id % CPRK);
    } else if constexpr (sizeof(T) == 2) {
      constexpr int CPR = BMT * 2 / 16;
      off = mnmaj16_off(id / CPR, (id % CPR) * V);
    } else {
      constexpr int CPR = BMT * 4 / 16;
      off = (id / CPR) * (BMT * 4) + (id % CPR) * 16;
    }
    *(uint4*)(img + off) = r[i];
  }
}

// LDS-DMA staging of one FULL K-tile (global_load_lds_dwordx4, 1 KiB per wave-instruction, no
// VGPR round trip).  The LDS destination of a wave-instruction is linear (base + 16*lane), so the
// bank swizzles of kmaj_off / mnmaj16_off are applied to the per-lane GLOBAL source address
// (rule 21 of the CDNA guide).  Rows past the matrix edge are clamped to a valid row: their
// products only reach discarded outputs.  KB/32 instructions per wave per operand.
template <typename T, bool KMAJ, int KB>
__device__ __forceinline__ void glds_tile(char* img, const T* base, int64_t ld, int rows_lim,
                                          int r0, int kloc) {
  constexpr int V = Vec<T>::n;
  constexpr int NI = KB / 32;
  constexpr int BKE = KB / (int)sizeof(T);
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const T* src;
    char* dst;
    if constexpr (KMAJ) {                      // image [128 rows][KB]
      constexpr int RPI = 1024 / KB;           // rows per instruction
      constexpr int CPRK = KB / 16;
      const int row0 = 32 * w + RPI * i;
      const int row = row0 + lane / CPRK;
      const int cp = lane % CPRK;
      const int c = (KB == 128) ? (cp ^ ((row >> 1) & 7)) : (cp ^ ((row >> 2) & 3));
      const int gr = min(r0 + row, rows_lim - 1);
      src = base + (int64_t)gr * ld + kloc + c * V;
      dst = img + row0 * KB;
    } else if constexpr (sizeof(T) == 2) {     // image [BKE k][256 B]
      const int k0 = (BKE / 4) * w + 4 * i;
      const int k = k0 + (lane >> 4);
      const int cp = lane & 15;
      const int t = (k & 3) | (((k >> 3) & 1) << 2);
      const int c = ((((cp >> 1) ^ t)) << 1) | (cp & 1);
      int gm = r0 + c * V;
      if (gm >= rows_lim) gm = ((rows_lim - 1) / V) * V;
      src = base + (int64_t)(kloc + k) * ld + gm;
      dst = img + k0 * 256;
    } else {                                   // f32 image [BKE k][512 B]
      const int k0 = (BKE / 4) * w + 2 * i;
      const int k = k0 + (lane >> 5);
      int gm = r0 + (lane & 31) * V;
      if (gm >= rows_lim) gm = ((rows_lim - 1) / V) * V;
      src = base + (int64_t)(kloc + k) * ld + gm;
      dst = img + k0 * 512;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

// ------------------------------------------------------------------ fragment reads
template <typename T> struct Frag16;
template <> struct Frag16<__bf16> { typedef bf16x8 t; typedef bf16x4 h; };
template <> struct Frag16<_Float16> { typedef f16x8 t; typedef f16x4 h; };

typedef short i16x4 __attribute__((ext_vector_type(4)));
template <typename H>
__device__ __forceinline__ H tr_read(const char* p) {
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(i16x4, p));
  return __builtin_bit_cast(H, v);
}

// 16-bit A/B fragment of one 16-row subtile for k-step ks (32 wide) of the current K-tile.
template <typename T, bool KMAJ, int KB>
__device__ __forceinline__ typename Frag16<T>::t read_frag16(const char* img, int rbase, int ks) {
  typedef typename Frag16<T>::t F;
  typedef typename Frag16<T>::h Hf;
  const int lane = threadIdx.x & 63;
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return *(const F*)(img + kmaj_off<KB>(row, c));
  } else {
    const int i = lane & 15;
    const int k0 = ks * 32 + (lane >> 4) * 8 + (i >> 2);
    const int m = rbase + (i & 3) * 4;
    Hf lo = tr_read<Hf>(img + mnmaj16_off(k0, m));
    Hf hi = tr_read<Hf>(img + mnmaj16_off(k0 + 4, m));
    F f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
}

// f32 fragment: element s (0..3) is the operand value at k = seg*16 + 4*(lane>>4) + s.
template <bool KMAJ, int KB>
__device__ __forceinline__ f32x4 read_frag32(const char* img, int rbase, int seg) {
  const int lane = threadIdx.x & 63;
  if constexpr (KMAJ) {
    const int row = rbase + (lane & 15);
    const int c = seg * 4 + (lane >> 4);
    return *(const f32x4*)(img + kmaj_off<KB>(row, c));
  } else {
    const float* f = (const float*)img;
    const int m = rbase + (lane & 15);
    const int k = seg * 16 + 4 * (lane >> 4);
    f32x4 r;
    r[0] = f[(k + 0) * BMT + m];
    r[1] = f[(k + 1) * BMT + m];
    r[2] = f[(k + 2) * BMT + m];
    r[3] = f[(k + 3) * BMT + m];
    return r;
  }
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------ epilogue
__device__ __forceinline__ float epi_value(const GemmParams& p, float v, int m, int n,
                                           const void* cptr, int64_t coff, const void* auxp,
                                           int64_t auxoff) {
  v *= p.alpha;
  if (p.bias_mode == 1) v += p.bias[n];
  else if (p.bias_mode == 2) v += p.bias[m];
  if (p.beta != 0.f) v += p.beta * ld_dyn(cptr, coff, p.c_dtype);
  if (p.relu) v = fmaxf(v, 0.f);
  if (auxp) {
    if (!(ld_dyn(auxp, auxoff, p.aux_dtype) > 0.f)) v = 0.f;
  }
  return v;
}

__device__ __forceinline__ void c_addr(const GemmParams& p, int b0, int b1, void*& cp,
                                       int64_t& cbase, const void*& ap, int64_t& abase) {
  if (p.c_mode == 1) {
    cp = p.c_ptr[b0];
    cbase = (int64_t)b1 * p.sC1;
  } else {
    cp = p.c_ptr[0];
    cbase = (int64_t)b0 * p.sC0 + (int64_t)b1 * p.sC1;
  }
  ap = p.aux;
  abase = cbase;   // aux shares C's batch strides (only used unbatched)
}

// ------------------------------------------------------------------ main kernel
template <typename T, bool AK, bool BK, int KB>
__device__ __forceinline__ void compute_tile(const char* imgA, const char* imgB, int wm, int wn,
                                             f32x4 (&acc)[4][4]) {
  if constexpr (sizeof(T) == 2) {
    typedef typename Frag16<T>::t F;
#pragma unroll
    for (int ks = 0; ks < KB / 64; ++ks) {
      F fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag16<T, AK, KB>(imgA, wm * 64 + i * 16, ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag16<T, BK, KB>(imgB, wn * 64 + j * 16, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
    }
  } else {
#pragma unroll
    for (int seg = 0; seg < KB / 64; ++seg) {
      f32x4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag32<AK, KB>(imgA, wm * 64 + i * 16, seg);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag32<BK, KB>(imgB, wn * 64 + j * 16, seg);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][s], fb[j][s], acc[i][j], 0, 0,
                                                             0);
    }
  }
}

__device__ __forceinline__ void wait_vm(int n) {   // s_waitcnt vmcnt(n), n in {0,4,8,12,16}
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
  }
}

template <typename O> struct OutVec { static constexpr int n = 16 / sizeof(O); };

struct Epi {
  float alpha, beta;
  const float* bias;
  int bias_mode, relu, N;
  int64_t ldc, ldaux;
};

// Epilogue of one output row chunk of VO = 16/sizeof(O) columns at (m, n); v[] = fp32
// accumulators.  16-B vector accesses when the chunk is interior and aligned (vec).
template <typename O>
__device__ __forceinline__ void store_chunk(const Epi& e, O* cp, int64_t cbase, const O* aux,
                                            int m, int n, float (&v)[16 / sizeof(O)], bool vec) {
  constexpr int VO = 16 / sizeof(O);
  const int64_t co = cbase + (int64_t)m * e.ldc + n;
  const bool full = vec && (n + VO <= e.N);
  const int nv = min(VO, e.N - n);
  float add[VO];
#pragma unroll
  for (int i = 0; i < VO; ++i) add[i] = 0.f;
  if (e.bias_mode == 1) {
#pragma unroll
    for (int i = 0; i < VO; ++i) add[i] = (i < nv) ? e.bias[n + i] : 0.f;
  } else if (e.bias_mode == 2) {
    const float bm = e.bias[m];
#pragma unroll
    for (int i = 0; i < VO; ++i) add[i] = bm;
  }
  if (e.beta != 0.f) {
    O old[VO];
    if (full) {
      *(uint4*)old = *(const uint4*)(cp + co);
    } else {
#pragma unroll
      for (int i = 0; i < VO; ++i) old[i] = (i < nv) ? cp[co + i] : from_f<O>(0.f);
    }
#pragma unroll
    for (int i = 0; i < VO; ++i) add[i] += e.beta * to_f(old[i]);
  }
  O out[VO];
  if (aux) {
    const int64_t ao = cbase + (int64_t)m * e.ldaux + n;
    O av[VO];
    if (full) {
      *(uint4*)av = *(const uint4*)(aux + ao);
    } else {
#pragma unroll
      for (int i = 0; i < VO; ++i) av[i] = (i < nv) ? aux[ao + i] : from_f<O>(0.f);
    }
#pragma unroll
    for (int i = 0; i < VO; ++i) {
      float x = v[i] * e.alpha + add[i];
      if (e.relu) x = fmaxf(x, 0.f);
      out[i] = from_f<O>(to_f(av[i]) > 0.f ? x : 0.f);
    }
  } else {
#pragma unroll
    for (int i = 0; i < VO; ++i) {
      float x = v[i] * e.alpha + add[i];
      if (e.relu) x = fmaxf(x, 0.f);
      out[i] = from_f<O>(x);
    }
  }
  if (full) {
    *(uint4*)(cp + co) = *(const uint4*)out;
  } else {
#pragma unroll
    for (int i = 0; i < VO; ++i)
      if (i < nv) cp[co + i] = out[i];
  }
}

// KB: bytes per operand row of one K-tile (128 | 64); S: LDS stages (2: prefetch 1 tile, two
// barriers per tile; >= 3: prefetch S-1 tiles, one barrier per tile).
template <typename T, typename O, bool AK, bool BK, int KB, int S>
__global__ __launch_bounds__(GT, 2) void gemm_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TILE_BYTES = BMT * KB;  // one operand image per stage
  constexpr int BKE = KB / (int)sizeof(T);   // K elements per tile
  constexpr int VMT = 2 * (KB / 32);         // glds instructions per wave per tile

  // XCD-aware remap (bijective): consecutive logical tiles (same A row panel) on one XCD.
  const int nwg = p.tiles_m * p.tiles_n;
  const int bid = blockIdx.x;
  int wg = bid;
  if (nwg >= 16) {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int tm = wg / p.tiles_n;
  const int tn = wg % p.tiles_n;
  const int b = blockIdx.y;
  const int b0 = b / p.batch1, b1 = b % p.batch1;
  const int split = blockIdx.z;

  const int m0 = tm * BMT, n0 = tn * BNT;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int klen = max(0, kend - kbeg);
  const int nfull = klen / BKE;
  const bool tail = (klen % BKE) != 0;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt, int buf) {
    const int k0 = kbeg + kt * BKE;
    int ka, kb;
    const T* A = operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, b0, b1, p.a_kseg, k0, ka);
    const T* B = operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, b0, b1, p.b_kseg, k0, kb);
    char* base = smem + buf * 2 * TILE_BYTES;
    glds_tile<T, AK, KB>(base, A, p.lda, p.M, m0, ka);
    glds_tile<T, BK, KB>(base + TILE_BYTES, B, p.ldb, p.N, n0, kb);
  };

  if constexpr (S == 2) {
    if (nfull > 0) issue(0, 0);
    for (int kt = 0; kt < nfull; ++kt) {
      if (kt + 1 < nfull) {
        issue(kt + 1, (kt + 1) & 1);
        wait_vm(VMT);                          // tile kt landed (one newer tile in flight)
      } else {
        wait_vm(0);
      }
      __builtin_amdgcn_s_barrier();            // ... for every wave of the block
      const char* imgA = smem + (kt & 1) * 2 * TILE_BYTES;
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, KB>(imgA, imgA + TILE_BYTES, wm, wn, acc);
      __builtin_amdgcn_s_barrier();            // buffer (kt&1) free for tile kt+2
    }
  } else {
    constexpr int D = S - 1;                   // prefetch distance
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (i < nfull) issue(i, i);
    for (int kt = 0; kt < nfull; ++kt) {
      const int after = min(D - 1, nfull - 1 - kt);   // tiles issued after kt, in flight
      wait_vm(after * VMT);
      __builtin_amdgcn_s_barrier();            // tile kt landed for all waves; tile kt-1 consumed
      if (kt + D < nfull) issue(kt + D, (kt + D) % S);
      const char* imgA = smem + (kt % S) * 2 * TILE_BYTES;
      if (!(p.dbg & 1)) compute_tile<T, AK, BK, KB>(imgA, imgA + TILE_BYTES, wm, wn, acc);
    }
  }
  if (tail) {   // trailing partial K-tile: masked register staging
    uint4 ra[KB / 32], rb[KB / 32];
    const int k0 = kbeg + nfull * BKE;
    int ka, kb;
    const T* A = operand_base<T>(p.a_ptr, p.a_mode, p.sA0, p.sA1, b0, b1, p.a_kseg, k0, ka);
    const T* B = operand_base<T>(p.b_ptr, p.b_mode, p.sB0, p.sB1, b0, b1, p.b_kseg, k0, kb);
    const int ka_lim = (p.a_mode == 2) ? min(p.a_kseg, ka + (kend - k0)) : kend;
    const int kb_lim = (p.b_mode == 2) ? min(p.b_kseg, kb + (kend - k0)) : kend;
    stage_load<T, AK, KB>(ra, A, p.lda, p.M, m0, ka_lim, ka);
    stage_load<T, BK, KB>(rb, B, p.ldb, p.N, n0, kb_lim, kb);
    char* base = smem + (nfull % S) * 2 * TILE_BYTES;
    stage_store<T, AK, KB>(base, ra);
    stage_store<T, BK, KB>(base + TILE_BYTES, rb);
    __syncthreads();
    if (!(p.dbg & 1)) compute_tile<T, AK, BK, KB>(base, base + TILE_BYTES, wm, wn, acc);
  }
  __syncthreads();

  // ---- epilogue through LDS, one 64-row half at a time: C/D layout of 16x16 MFMA is
  //      col = lane&15, row = 4*(lane>>4) + r; the store pass writes 16-B row chunks.
  constexpr int CLD = 132;                  // padded fp32 row of the staged half tile
  float* ct = (float*)smem;
  const bool partial = p.splits > 1;
  O* cp;
  int64_t cbase;
  const void* ap = partial ? nullptr : p.aux;
  bool vec;
  if (partial) {
    const int nb = p.batch0 * p.batch1;
    cp = (O*)(p.ws + ((int64_t)split * nb + b) * (int64_t)p.M * p.N);
    cbase = 0;
    vec = (p.N % 4) == 0;
  } else {
    if (p.c_mode == 1) {
      cp = (O*)p.c_ptr[b0];
      cbase = (int64_t)b1 * p.sC1;
    } else {
      cp = (O*)p.c_ptr[0];
      cbase = (int64_t)b0 * p.sC0 + (int64_t)b1 * p.sC1;
    }
    vec = p.c_vec != 0;
  }
  if (p.dbg & 2) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (sum == 12345.678f) ((float*)cp)[0] = sum;   // keep acc live
    return;
  }
  Epi ep;
  ep.alpha = p.alpha; ep.beta = p.beta; ep.bias = p.bias; ep.bias_mode = p.bias_mode;
  ep.relu = p.relu; ep.N = p.N; ep.ldc = p.ldc; ep.ldaux = p.ldaux;
  if (partial) {   // raw partial sums: no epilogue ops, row stride N
    ep.alpha = 1.f; ep.beta = 0.f; ep.bias_mode = 0; ep.relu = 0; ep.ldc = p.N;
  }
  const O* auxp = (const O*)ap;
  constexpr int VO = OutVec<O>::n;
  constexpr int CPR = BNT / VO;                 // chunks per 128-col row
  constexpr int RPI = GT / CPR;                 // rows covered per pass
  constexpr int NIT = 64 / RPI;                 // passes per 64-row half
  // each thread owns ONE column chunk for the whole epilogue (GT is a multiple of CPR)
  const int cc = (threadIdx.x % CPR) * VO;
  const int r_in = threadIdx.x / CPR;
  const int n = n0 + cc;
  const bool col_ok = n < p.N;
  const int nv = min(VO, p.N - n);
  const bool full = vec && (n + VO <= p.N);
  float bvec[VO];
#pragma unroll
  for (int i = 0; i < VO; ++i) bvec[i] = 0.f;
  if (ep.bias_mode == 1 && col_ok) {
#pragma unroll
    for (int i = 0; i < VO; ++i) bvec[i] = (i < nv) ? ep.bias[n + i] : 0.f;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ct[(i * 16 + 4 * (lane >> 4) + r) * CLD + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
    // phase 1: LDS reads + every global load of the pass (C_old, aux) issued back to back
    float v[NIT][VO];
    O oldv[NIT][VO];
    O auxv[NIT][VO];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rr = r_in + RPI * it;
      const float* src = ct + rr * CLD + cc;
#pragma unroll
      for (int e = 0; e < VO; e += 4) {
        const float4 t = *(const float4*)(src + e);
        v[it][e] = t.x; v[it][e + 1] = t.y; v[it][e + 2] = t.z; v[it][e + 3] = t.w;
      }
      const int m = m0 + 64 * h + rr;
      const bool ok = col_ok && m < p.M;
      const int64_t co = cbase + (int64_t)m * ep.ldc + n;
      const int64_t ao = cbase + (int64_t)m * ep.ldaux + n;
      if (ep.beta != 0.f) {
        if (ok && full) *(uint4*)oldv[it] = *(const uint4*)(cp + co);
        else
#pragma unroll
          for (int i = 0; i < VO; ++i) oldv[it][i] = (ok && i < nv) ? cp[co + i] : from_f<O>(0.f);
      }
      if (auxp) {
        if (ok && full) *(uint4*)auxv[it] = *(const uint4*)(auxp + ao);
        else
#pragma unroll
          for (int i = 0; i < VO; ++i) auxv[it][i] = (ok && i < nv) ? auxp[ao + i] : from_f<O>(0.f);
      }
    }
    // phase 2: epilogue math + 16-B stores
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rr = r_in + RPI * it;
      const int m = m0 + 64 * h + rr;
      if (!(col_ok && m < p.M)) continue;
      const float bm = (ep.bias_mode == 2) ? ep.bias[m] : 0.f;
      O out[VO];
#pragma unroll
      for (int i = 0; i < VO; ++i) {
        float x = v[it][i] * ep.alpha + bvec[i] + bm;
        if (ep.beta != 0.f) x += ep.beta * to_f(oldv[it][i]);
        if (ep.relu) x = fmaxf(x, 0.f);
        if (auxp && !(to_f(auxv[it][i]) > 0.f)) x = 0.f;
        out[i] = from_f<O>(x);
      }
      const int64_t co = cbase + (int64_t)m * ep.ldc + n;
      if (full) {
        *(uint4*)(cp + co) = *(const uint4*)out;
      } else {
#pragma unroll
        for (int i = 0; i < VO; ++i)
          if (i < nv) cp[co + i] = out[i];
      }
    }
    __syncthreads();
  }
}

// split-K reduction + epilogue: one thread per output element (vector of 4 along n when possible)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmParams p) {
  const int nb = p.batch0 * p.batch1;
  const int64_t per = (int64_t)p.M * p.N;
  const int64_t total = per * nb;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(e / per);
    const int64_t mn = e - (int64_t)b * per;
    const int m = (int)(mn / p.N), n = (int)(mn - (int64_t)m * p.N);
    float v = 0.f;
    for (int s = 0; s < p.splits; ++s) v += p.ws[((int64_t)s * nb + b) * per + mn];
    const int b0 = b / p.batch1, b1 = b % p.batch1;
    void* cp;
    int64_t cbase, abase;
    const void* ap;
    c_addr(p, b0, b1, cp, cbase, ap, abase);
    const int64_t co = cbase + (int64_t)m * p.ldc + n;
    const int64_t ao = abase + (int64_t)m * p.ldaux + n;
    st_dyn(cp, co, p.c_dtype, epi_value(p, v, m, n, cp, co, ap, ao));
  }
}

template <typename T, typename O, bool AK, bool BK, int KB, int S>
static void launch_cfg(const GemmParams& p, dim3 grid, hipStream_t st) {
  constexpr size_t lds = (size_t)S * 2 * BMT * KB;
  auto fn = gemm_kernel<T, O, AK, BK, KB, S>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(fn, grid, dim3(GT), lds, st, p);
}

// GEMM configurations: (KB, S) = 1: (128, 2)  2: (128, 3)  3: (64, 3)  4: (64, 4)
template <typename T, typename O, bool AK, bool BK>
static void launch_layout(const GemmParams& p, int cfg, dim3 grid, hipStream_t st) {
  switch (cfg) {
    case 2: launch_cfg<T, O, AK, BK, 128, 3>(p, grid, st); break;
    case 3: launch_cfg<T, O, AK, BK, 64, 3>(p, grid, st); break;
    case 4: launch_cfg<T, O, AK, BK, 64, 4>(p, grid, st); break;
    default: launch_cfg<T, O, AK, BK, 128, 2>(p, grid, st); break;
  }
}

template <typename T, typename O>
static void launch_to(const GemmParams& p, int ak, int bk, int cfg, dim3 grid, hipStream_t st) {
  if (ak && bk) launch_layout<T, O, true, true>(p, cfg, grid, st);
  else if (ak && !bk) launch_layout<T, O, true, false>(p, cfg, grid, st);
  else if (!ak && bk) launch_layout<T, O, false, true>(p, cfg, grid, st);
  else launch_layout<T, O, false, false>(p, cfg, grid, st);
}

template <typename T>
static void launch_t(const GemmParams& p, int ak, int bk, int cfg, dim3 grid, hipStream_t st) {
  if (p.splits > 1 || p.c_dtype == JMT_F32) launch_to<T, float>(p, ak, bk, cfg, grid, st);
  else launch_to<T, T>(p, ak, bk, cfg, grid, st);
}

}  // namespace jmt

using namespace jmt;

static int g_gemm_dbg = 0;
static int g_gemm_cfg = 0;
extern "C" void jmt_gemm_set_debug(int flags) { g_gemm_dbg = flags & 0xff; g_gemm_cfg = flags >> 8; }

extern "C" size_t jmt_gemm_workspace_bytes(int M, int N, int batch, int splits) {
  if (splits <= 1) return 0;
  return (size_t)splits * (size_t)batch * (size_t)M * (size_t)N * sizeof(float);
}

extern "C" int jmt_gemm(const jmt_gemm_desc* d, void* stream) {
  JMT_CHECK_ARG(d != nullptr, "jmt_gemm: null descriptor");
  const int dt = d->ab_dtype;
  JMT_CHECK_ARG(dt == JMT_F32 || dt == JMT_BF16 || dt == JMT_F16, "jmt_gemm: bad ab_dtype %d", dt);
  JMT_CHECK_ARG(d->c_dtype == JMT_F32 || d->c_dtype == dt, "jmt_gemm: c_dtype must be f32 or ab");
  JMT_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0, "jmt_gemm: negative size");
  JMT_CHECK_ARG(d->aux == nullptr || d->aux_dtype == d->c_dtype,
                "jmt_gemm: aux (ReLU mask) must have the output dtype");
  if (d->M == 0 || d->N == 0) return JMT_OK;
  const int batch0 = d->batch0 < 1 ? 1 : d->batch0;
  const int batch1 = d->batch1 < 1 ? 1 : d->batch1;
  JMT_CHECK_ARG(batch0 * batch1 <= 65535, "jmt_gemm: batch too large");
  const int es = dtype_size(dt);
  const int V = 16 / es;
  // pipeline configuration (see launch_layout); K tiles must divide the K-concat segments
  int cfg = g_gemm_cfg ? g_gemm_cfg : 1;
  const int KBsel = (cfg == 3 || cfg == 4) ? 64 : 128;
  const int BKE = KBsel / es;
  JMT_CHECK_ARG(d->n_a >= 1 && d->n_a <= MAXP && d->n_b >= 1 && d->n_b <= MAXP &&
                    d->n_c >= 1 && d->n_c <= MAXP, "jmt_gemm: pointer table size");
  JMT_CHECK_ARG(d->lda % V == 0 && d->ldb % V == 0, "jmt_gemm: lda/ldb must be multiples of %d", V);
  JMT_CHECK_ARG((d->sA0 % V == 0) && (d->sA1 % V == 0) && (d->sB0 % V == 0) && (d->sB1 % V == 0),
                "jmt_gemm: batch strides must be multiples of %d elements", V);
  for (int i = 0; i < d->n_a; ++i)
    JMT_CHECK_ARG(((uintptr_t)d->a[i] & 15) == 0, "jmt_gemm: A[%d] not 16-B aligned", i);
  for (int i = 0; i < d->n_b; ++i)
    JMT_CHECK_ARG(((uintptr_t)d->b[i] & 15) == 0, "jmt_gemm: B[%d] not 16-B aligned", i);
  if (d->a_mode == 2) JMT_CHECK_ARG(d->a_kseg % BKE == 0 && d->a_kseg * d->n_a >= d->K,
                                    "jmt_gemm: A K-concat segment must be a multiple of %d", BKE);
  if (d->b_mode == 2) JMT_CHECK_ARG(d->b_kseg % BKE == 0 && d->b_kseg * d->n_b >= d->K,
                                    "jmt_gemm: B K-concat segment must be a multiple of %d", BKE);
  if (d->a_mode == 1) JMT_CHECK_ARG(d->n_a >= batch0, "jmt_gemm: A pointer table < batch0");
  if (d->b_mode == 1) JMT_CHECK_ARG(d->n_b >= batch0, "jmt_gemm: B pointer table < batch0");
  if (d->c_mode == 1) JMT_CHECK_ARG(d->n_c >= batch0, "jmt_gemm: C pointer table < batch0");

  GemmParams p;
  for (int i = 0; i < MAXP; ++i) {
    p.a_ptr[i] = i < d->n_a ? d->a[i] : nullptr;
    p.b_ptr[i] = i < d->n_b ? d->b[i] : nullptr;
    p.c_ptr[i] = i < d->n_c ? d->c[i] : nullptr;
  }
  p.bias = d->bias;
  p.aux = d->aux;
  p.lda = d->lda; p.ldb = d->ldb; p.ldc = d->ldc; p.ldaux = d->ldaux;
  p.sA0 = d->sA0; p.sA1 = d->sA1; p.sB0 = d->sB0; p.sB1 = d->sB1; p.sC0 = d->sC0; p.sC1 = d->sC1;
  p.a_mode = d->a_mode; p.b_mode = d->b_mode; p.c_mode = d->c_mode;
  p.a_kseg = d->a_mode == 2 ? d->a_kseg : 0;
  p.b_kseg = d->b_mode == 2 ? d->b_kseg : 0;
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.batch0 = batch0; p.batch1 = batch1;
  p.alpha = d->alpha; p.beta = d->beta;
  p.bias_mode = d->bias ? d->bias_mode : 0;
  p.relu = d->relu;
  p.c_dtype = d->c_dtype;
  p.aux_dtype = d->aux_dtype;
  p.tiles_m = (d->M + BMT - 1) / BMT;
  p.tiles_n = (d->N + BNT - 1) / BNT;
  p.dbg = g_gemm_dbg;
  {
    const int ces = dtype_size(d->c_dtype);
    const int VO = 16 / ces;
    bool cv = d->ldc % VO == 0 && d->sC0 % VO == 0 && d->sC1 % VO == 0;
    for (int i = 0; i < d->n_c; ++i) cv = cv && (((uintptr_t)d->c[i] & 15) == 0);
    if (d->aux) cv = cv && (((uintptr_t)d->aux & 15) == 0) && d->ldaux % VO == 0;
    p.c_vec = cv ? 1 : 0;
  }

  int splits = d->splits < 1 ? 1 : d->splits;
  // each split must own whole K-tiles, and a K-concat segment boundary must not cut a tile
  int kps = ((d->K + splits - 1) / splits + BKE - 1) / BKE * BKE;
  if (kps < BKE) kps = BKE;
  splits = (d->K + kps - 1) / kps;
  if (splits < 1) splits = 1;
  p.splits = splits;
  p.k_per_split = splits > 1 ? kps : (d->K > 0 ? d->K : 1);
  p.ws = (float*)d->workspace;
  if (splits > 1) {
    const size_t need = jmt_gemm_workspace_bytes(d->M, d->N, batch0 * batch1, splits);
    JMT_CHECK_ARG(d->workspace != nullptr && d->ws_bytes >= need,
                  "jmt_gemm: split-K needs %zu workspace bytes", need);
  }
  hipStream_t st = as_stream(stream);
  dim3 grid(p.tiles_m * p.tiles_n, batch0 * batch1, splits);
  if (dt == JMT_F32) launch_t<float>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
  else if (dt == JMT_BF16) launch_t<__bf16>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
  else launch_t<_Float16>(p, d->a_kmajor, d->b_kmajor, cfg, grid, st);
  JMT_LAUNCH_CHECK("jmt_gemm");
  if (splits > 1) {
    const int64_t total = (int64_t)d->M * d->N * batch0 * batch1;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, p);
    JMT_LAUNCH_CHECK("jmt_gemm(splitk_reduce)");
  }
  return JMT_OK;
}
