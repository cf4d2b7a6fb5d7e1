/*
 * jmt.h — C-ABI of libjmt_hip.so, the MI355X (gfx950) kernels of the Joint-Multimodal-Transformer
 * fusion hot path.
 *
 * The reference (PoloWlg/Joint-Multimodal-Transformer-6th-ABAW) has no FFI: its boundary is Python
 * module/class identity.  The Python drop-in modules under
 * joint-multimodal-transformer-6th-abaw_amd/{models,losses} bind these entry points with ctypes
 * (jmt/_lib.py); each entry point replaces the stock PyTorch op(s) the reference calls at the
 * cited lines.  Conventions:
 *   - every pointer is a device pointer owned by the caller (the PyTorch caching allocator),
 *     including workspaces; the library never allocates device memory and keeps no state;
 *   - every call is enqueued on `stream` (a hipStream_t); no host synchronisation;
 *   - return 0 on success or a negative JMT_ERR_*; jmt_last_error() describes the last failure
 *     (thread-local).
 */
#ifndef JMT_H_
#define JMT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JMT_ABI_VERSION 7
/* ABI 7 (round 6): jmt_attn_bwd with dq == NULL writes P and dS only (the 128-row kernel), and
 * jmt_attn_dkdv takes k / dq (+ strides) and computes dQ = dS K as its third product. */
/* ABI 6 (round 5): jmt_attn_bwd_km removed (the key-major P / dS hand-off measured slower than
 * jmt_attn_bwd + jmt_attn_dkdv); the split-K workspace holds the fp32 slabs only. */

enum { JMT_F32 = 0, JMT_BF16 = 1, JMT_F16 = 2 };
enum { JMT_OK = 0, JMT_ERR_ARG = -1, JMT_ERR_HIP = -2, JMT_ERR_UNSUPPORTED = -3 };

int jmt_abi_version(void);
const char* jmt_last_error(void);
/* number of gfx950 code objects / kernels compiled in (sanity probe, no GPU needed) */
int jmt_kernel_count(void);
/* Bounds-check build (csrc `make bounds`, -DJMT_BOUNDS=1, loaded with JMT_LIB=<path>): the
 * number of failed device-side index checks since the last reset (reset != 0 clears them; the
 * call synchronises the device); -1 in the default build, which compiles the checks out. */
long long jmt_bounds_violations(int reset);

/* ------------------------------------------------------------------ GEMM
 * C[b] = epilogue(alpha * A[b] . B[b]),  A: M x K, B: K x N, C: M x N.
 *   a_kmajor=1: A[m][k] at a + m*lda + k   (row-major activations)      a_kmajor=0: a + k*lda + m
 *   b_kmajor=1: B[k][n] at b + n*ldb + k   (nn.Linear weight, W^T)      b_kmajor=0: b + k*ldb + n
 * batch index b = (b0, b1), b0 < batch0, b1 < batch1.  Operand address modes:
 *   0 strided:   base[0] + b0*s0 + b1*s1
 *   1 table:     base[b0] + b1*s1                        (up to 8 tensors)
 *   2 K-concat:  K range [i*kseg, (i+1)*kseg) read from base[i]  (a torch.cat along the feature
 *                axis that is never materialised; kseg a multiple of 64 (16-bit) / 32 (f32))
 * Epilogue on the fp32 accumulator: *alpha, +bias (1: per column n, 2: per row m), +beta*C,
 * ReLU, then zeroed where aux <= 0 (ReLU backward mask), stored as c_dtype.
 * splits > 1: split-K with fp32 partial slabs in `workspace` (jmt_gemm_workspace_bytes), then a
 * deterministic reduce + epilogue launch.
 * Replaces: nn.Linear (fc_layer.py:6-12, two_transformers.py:56,104-114,
 * mm_multi_transformers.py:52-56,99,102), the in_proj/out_proj GEMMs and the bmm's of
 * F.multi_head_attention_forward behind every nn.MultiheadAttention, and
 * their autograd backward.
 */
typedef struct jmt_gemm_desc {
  int ab_dtype, c_dtype, aux_dtype;
  int M, N, K;
  const void* a[8];
  const void* b[8];
  void* c[8];
  int n_a, n_b, n_c;
  int a_mode, b_mode, c_mode;
  int a_kseg, b_kseg;
  int a_kmajor, b_kmajor;
  int64_t lda, ldb, ldc, ldaux;
  int batch0, batch1;
  int64_t sA0, sA1, sB0, sB1, sC0, sC1;
  float alpha, beta;
  const float* bias;
  int bias_mode;
  int relu;
  const void* aux;
  int splits;
  void* workspace;
  size_t ws_bytes;
  /* ABI 2: per-batch bias table (grouped GEMMs of several nn.Linear / in_proj modules in one
   * launch): when n_bias > 0, batch b0 uses bias_tab[b0] (bias_mode 1 or 2) instead of bias. */
  const float* bias_tab[8];
  int n_bias;
  /* ABI 4: A row sums — the bias gradient of a weight-gradient GEMM dW = dY^T X, db[m] =
   * sum_k A[m][k] = the column sums of dY (nn.Linear's bias.grad, autograd of the same
   * modules) — taken from the A fragments inside the GEMM instead of a second pass over dY:
   * when n_dbias > 0, dbias_tab[b0][m] (+)= (dbias_acc) the row sums of A[b0] (fp32; a NULL
   * entry skips b0 — the segments of a K-concatenated wgrad share one dY).  16-bit
   * MN-major A and B, fp32 C, batch1 = 1; split-K needs dbias_ws (splits * batch0 * M floats). */
  float* dbias_tab[8];
  int n_dbias;
  int dbias_acc;
  float* dbias_ws;
  size_t dbias_ws_bytes;
} jmt_gemm_desc;

int jmt_gemm(const jmt_gemm_desc* desc, void* stream);
size_t jmt_gemm_workspace_bytes(int M, int N, int batch, int splits);
/* split-K factor jmt_gemm's planner picks for this problem (1 = no split).  jmt_gemm chooses the
 * block tile (128x128 or 256x256) from the same cost model: waves x (tile FLOPs / per-block MFMA
 * rate + per-block overhead) + the split-K reduce traffic. */
int jmt_gemm_plan_splits(int ab_dtype, int M, int N, int K, int batch);
/* development only: low byte = GEMM ablation flags (1 = skip MFMA, 2 = skip epilogue stores),
 * flags >> 8 = forced tile config (1 128x128, 5 256x256, 6 256x128, 7 128x256), 0 = off */
void jmt_gemm_set_debug(int flags);
/* development: per-block s_memrealtime stamps (entry, first K-tile, loop end, epilogue end) of
 * the last launch made with debug flag 8; returns the number of blocks copied to host[4*n]. */
int jmt_gemm_trace_read(uint64_t* host, int nblocks);

/* ------------------------------------------------------------------ row-wise ops
 * Rows are `rows` vectors of length D at stride ld (elements). */

/* F.normalize(x, p=2, dim=-1, eps) (two_transformers.py:118-119): y = x / max(||x||, eps);
 * writes inv_norm[r] = 1 / max(||x_r||, eps) (fp32) for the backward. */
int jmt_l2norm_fwd(int x_dt, int y_dt, int64_t rows, int D, const void* x, int64_t ldx, void* y,
                   int64_t ldy, float* inv_norm, float eps, void* stream);
/* dx = (dy - y (y.dy)) * inv_norm when ||x|| > eps, else dy * inv_norm;  y = x * inv_norm. */
int jmt_l2norm_bwd(int x_dt, int dy_dt, int dx_dt, int64_t rows, int D, const void* x,
                   int64_t ldx, const void* dy, int64_t lddy, const float* inv_norm, float eps,
                   void* dx, int64_t lddx, void* stream);

/* Post-LN residual block (mm_multi_transformers.py:64-70): y = LayerNorm(x + r) * gamma + beta,
 * eps, biased variance.  r may be NULL.  Saves mean / rstd (fp32, per row). */
int jmt_layernorm_fwd(int dt_in, int dt_out, int64_t rows, int D, const void* x, int64_t ldx,
                      const void* r, int64_t ldr, const float* gamma, const float* beta, float eps,
                      void* y, int64_t ldy, float* mean, float* rstd, void* stream);
/* ds = d(x+r); dgamma/dbeta accumulated as fp32 partial slabs into `partials` (2 * nblk * D
 * floats, nblk = jmt_layernorm_bwd_blocks(rows)) and reduced into dgamma/dbeta (beta_acc=1 adds
 * to the existing values). */
int jmt_layernorm_bwd_blocks(int64_t rows);
int jmt_layernorm_bwd(int dt_in, int dt_dy, int dt_dx, int64_t rows, int D, const void* x,
                      int64_t ldx, const void* r, int64_t ldr, const void* dy, int64_t lddy,
                      const float* mean, const float* rstd, const float* gamma, void* dx,
                      int64_t lddx, float* dgamma, float* dbeta, int beta_acc, float* partials,
                      void* stream);

/* jmt_layernorm_bwd plus dsum (+)= the column sums of dx (the gradient of the bias of the linear
 * whose output entered the residual sum: FFN out / attention out_proj, mm_multi_transformers.py:
 * 52-70), reduced with dgamma / dbeta (partials: 3 * D * jmt_layernorm_bwd_blocks(rows) floats,
 * 16-B aligned).  D in {512, 768, 1024} with 4-element aligned rows; otherwise returns
 * JMT_ERR_UNSUPPORTED and writes nothing. */
int jmt_layernorm_bwd_dsum(int dt_in, int dt_dy, int dt_dx, int64_t rows, int D, const void* x,
                           int64_t ldx, const void* r, int64_t ldr, const void* dy, int64_t lddy,
                           const float* mean, const float* rstd, const float* gamma, void* dx,
                           int64_t lddx, float* dgamma, float* dbeta, float* dsum, int beta_acc,
                           float* partials, void* stream);

/* Grouped LayerNorm (round 3): G <= 8 same-shaped LayerNorms in one launch — the grouped
 * encoders' LN1 / LN2, one per stream (mm_multi_transformers.py:61-70).  Group g's rows start at
 * x + g*sx (r + g*sr; y or dx + g*sy / sdx; dy + g*sdy; elements), its statistics at
 * mean / rstd + g*rows, its parameters / gradients from the pointer tables (host arrays of G
 * device pointers).  Backward: dsum may be NULL (no column sums of dx); partials:
 * G * (dsum ? 3 : 2) * D * jmt_layernorm_bwd_grouped_blocks(rows) floats, 16-B aligned.  D in
 * {512, 768, 1024} with 4-element aligned rows and strides; otherwise JMT_ERR_UNSUPPORTED. */
int jmt_layernorm_fwd_grouped(int dt_in, int dt_out, int G, int64_t rows, int D, const void* x,
                              int64_t ldx, int64_t sx, const void* r, int64_t ldr, int64_t sr,
                              const float* const* gamma, const float* const* beta, float eps,
                              void* y, int64_t ldy, int64_t sy, float* mean, float* rstd,
                              void* stream);
int jmt_layernorm_bwd_grouped(int dt_in, int dt_dy, int dt_dx, int G, int64_t rows, int D,
                              const void* x, int64_t ldx, int64_t sx, const void* r, int64_t ldr,
                              int64_t sr, const void* dy, int64_t lddy, int64_t sdy,
                              const float* mean, const float* rstd, const float* const* gamma,
                              void* dx, int64_t lddx, int64_t sdx, float* const* dgamma,
                              float* const* dbeta, float* const* dsum, int beta_acc,
                              float* partials, void* stream);
/* ABI 5: the partials of jmt_layernorm_bwd_grouped hold G * (dsum ? 3 : 2) * D *
 * jmt_layernorm_bwd_grouped_blocks(rows) floats (the grouped kernel's rows per block). */
int jmt_layernorm_bwd_grouped_blocks(int64_t rows);

/* Attention softmax (F.multi_head_attention_forward): rows of length n of the
 * fp32 score matrix S (ld) -> P = softmax(scale * S) stored as p_dt at ldp; columns [n, ldp)
 * of P are zeroed. */
int jmt_softmax_fwd(int p_dt, int64_t rows, int n, const float* s, int64_t lds, float scale,
                    void* p, int64_t ldp, void* stream);
/* dS = scale * P o (dP - rowsum(P o dP)), dP fp32, dS stored as ds_dt (columns [n, ldds) = 0). */
int jmt_softmax_bwd(int p_dt, int ds_dt, int64_t rows, int n, const void* p, int64_t ldp,
                    const float* dp, int64_t lddp, float scale, void* ds, int64_t ldds,
                    void* stream);

/* Fused attention core (F.multi_head_attention_forward's softmax(Q K^T * scale) V per (n, h);
 * mm_multi_transformers.py:57,142-167,191, intra_modal_transformer_fusion.py):
 * element (l, n, h, d) of X in {q,k,v,o,go,dq} at X + l*sX_l + n*sX_n + h*dh + d.
 * jmt_attn_supported(dt, dh) != 0 for the configurations the fused kernels cover (16-bit,
 * dh = 512); otherwise the entry points return JMT_ERR_UNSUPPORTED and the caller uses the
 * GEMM + jmt_softmax path.
 * jmt_attn_fwd: writes o and, if lse != NULL, lse[(n*H + h)*Lq + l] = ln sum_k exp(scale s_lk).
 *   No probabilities are kept: the backward recomputes them from lse.
 * jmt_attn_bwd: given dO (go), the forward's o and lse, and q, k, v: recomputes
 *   P = exp(scale Q K^T - lse), writes p_out = P and ds_out = scale * P o (dO V^T - rowsum(dO o O))
 *   (N*H*Lq rows of ldp >= Lk, row (n*H + h)*Lq + l; columns [Lk, ldp) zero) and
 *   dq = ds K.  dK = ds^T Q and dV = P^T dO are left to jmt_gemm.
 *   dq == NULL (ABI 7): P and ds only, by the 128-query-row kernel (no dQ accumulator: the whole
 *   512-dim Q / dO rows of a wave stay in registers), in the TILE-MAJOR layout: the (n, h)
 *   region of Lq * ldp values holds ldp / 32 key tiles, tile t = [Lq queries][32 keys]
 *   (element ((n*H + h) * ldp / 32 + t) * Lq * 32 + l * 32 + c = key 32 t + c of query l);
 *   ldp a multiple of 32 >= Lk (keys [Lk, 32 ceil(Lk / 32)) written as zeros, later tiles
 *   untouched), (Lq + 128) ldp 16-bit values < 1 GiB; dq / sdq_* ignored.  dQ, dK and dV then
 *   come from jmt_attn_dkdv with dq != NULL.
 * (ABI 3: replaces ABI 2's jmt_attn_fwd p_out/mt outputs, jmt_attn_mt_floats and
 * jmt_attn_bwd_dq.) */
int jmt_attn_supported(int dt, int dh);
int jmt_attn_fwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* q, int64_t sq_l,
                 int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n, const void* v,
                 int64_t sv_l, int64_t sv_n, void* o, int64_t so_l, int64_t so_n, float scale,
                 float* lse, void* stream);
int jmt_attn_bwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* go, int64_t sgo_l,
                 int64_t sgo_n, const void* o, int64_t so_l, int64_t so_n, const void* q,
                 int64_t sq_l, int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n,
                 const void* v, int64_t sv_l, int64_t sv_n, const float* lse, void* p_out,
                 void* ds_out, int64_t ldp, void* dq, int64_t sdq_l, int64_t sdq_n, float scale,
                 void* stream);

/* Key-side attention gradients from the handed-over probabilities (round 4): per (n, h)
 * dV = P^T dO and dK = dS^T Q, P / dS as jmt_attn_bwd writes them (row (n*H + h)*Lq + q, keys in
 * columns, row stride ldp >= 128 ceil(Lk / 128): the kernel reads whole 128-key tiles; columns past
 * Lk only feed outputs that are not stored).  dO / Q / dK / dV seq-first views as jmt_attn_bwd's
 * operands (row stride s*_l, batch stride s*_n, head h at columns 512 h).  16-bit, dh = 512.
 * Replaces the two batched TN jmt_gemm calls (M = Lk, N = dh, K = Lq) of the same products.
 * ABI 7: when dq != NULL also dQ = dS K (k: the attention's K operand, a view like q; dq like
 * dk, rows Lq), as 128-query items beside the 128-key dK / dV items of the same launch, and P /
 * dS are read in the tile-major layout jmt_attn_bwd(dq = NULL) writes (the pair's contract);
 * dS keys [0, 32 ceil(Lk / 32)) feed dQ. */
int jmt_attn_dkdv(int dt, int N, int H, int Lq, int Lk, int dh, const void* p, const void* ds,
                  int64_t ldp, const void* go, int64_t sgo_l, int64_t sgo_n, const void* q,
                  int64_t sq_l, int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n, void* dk,
                  int64_t sdk_l, int64_t sdk_n, void* dv, int64_t sdv_l, int64_t sdv_n, void* dq,
                  int64_t sdq_l, int64_t sdq_n, void* stream);

/* Fused attention over short sequences, the whole backward in one kernel (Lq, Lk <= 32, 16-bit,
 * dh = 512; the batch-axis self-attention of mm_transformers.py:119-146 at B = 32 and every
 * attention of the T = 16 real-data configuration): same element addressing as jmt_attn_*,
 * one block per (n, h).  jmt_attn_short_supported(dt, dh, Lq, Lk) != 0 for the covered shapes.
 * jmt_attn_short_fwd: as jmt_attn_fwd (o and lse; bitwise the same values).
 * jmt_attn_short_bwd: dq = dS K, dk = dS^T Q, dv = P^T dO with P recomputed from lse and
 *   dS = scale * P o (dO V^T - rowsum(dO o O)); dq/dk/dv overwritten (they may be column slices
 *   of one buffer); no P / dS leave the chip (replaces jmt_attn_bwd + the two jmt_gemm calls).
 *   Rows 16-B aligned, strides multiples of 8.  (ABI 3, round 3 addition.) */
int jmt_attn_short_supported(int dt, int dh, int Lq, int Lk);
int jmt_attn_short_fwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* q, int64_t sq_l,
                       int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n, const void* v,
                       int64_t sv_l, int64_t sv_n, void* o, int64_t so_l, int64_t so_n,
                       float scale, float* lse, void* stream);
int jmt_attn_short_bwd(int dt, int N, int H, int Lq, int Lk, int dh, const void* go,
                       int64_t sgo_l, int64_t sgo_n, const void* o, int64_t so_l, int64_t so_n,
                       const void* q, int64_t sq_l, int64_t sq_n, const void* k, int64_t sk_l,
                       int64_t sk_n, const void* v, int64_t sv_l, int64_t sv_n, const float* lse,
                       void* dq, int64_t sdq_l, int64_t sdq_n, void* dk, int64_t sdk_l,
                       int64_t sdk_n, void* dv, int64_t sdv_l, int64_t sdv_n, float scale,
                       void* stream);

/* Attention over short sequences (Lq, Lk <= 8; E = H*dh = 512, E/8/H a power of two, dt any of
 * fp32/bf16/fp16): the SELF_ATTEN head's 6-token sequences (mm_multi_transformers.py:169-199)
 * and intra-modal fusion's 2-token ones (intra_modal_transformer_fusion.py:93-108), same element
 * addressing as jmt_attn_*, one wave per sequence n (HBM-bound; the 64-row fused kernels would
 * idle >90 % of every tile). Rows 16-B aligned (32-B for fp32), strides multiples of 8.
 * jmt_small_attn_fwd: o = softmax(scale Q K^T) V; if p_out != NULL the fp32 probabilities are
 *   kept at p_out[((n*H + h)*Lq + l)*Lk + k] (N*H*Lq*Lk floats) for the backward.
 * jmt_small_attn_bwd: dq = dS K, dk = dS^T Q, dv = P^T dO with dS = scale P o (dO V^T -
 *   rowsum(P o dO V^T)); dq/dk/dv overwritten (they may be column slices of one buffer). */
int jmt_small_attn_fwd(int dt, int N, int H, int Lq, int Lk, int E, const void* q, int64_t sq_l,
                       int64_t sq_n, const void* k, int64_t sk_l, int64_t sk_n, const void* v,
                       int64_t sv_l, int64_t sv_n, void* o, int64_t so_l, int64_t so_n,
                       float scale, float* p_out, void* stream);
int jmt_small_attn_bwd(int dt, int N, int H, int Lq, int Lk, int E, const void* go,
                       int64_t sgo_l, int64_t sgo_n, const void* q, int64_t sq_l, int64_t sq_n,
                       const void* k, int64_t sk_l, int64_t sk_n, const void* v, int64_t sv_l,
                       int64_t sv_n, const float* p, void* dq, int64_t sdq_l, int64_t sdq_n,
                       void* dk, int64_t sdk_l, int64_t sdk_n, void* dv, int64_t sdv_l,
                       int64_t sdv_n, float scale, void* stream);

/* Bias gradient: db[n] (+)= sum_m dy[m][n] (two-phase, deterministic, fp32 partial slabs of
 * jmt_colsum_blocks(rows) * N floats). */
int jmt_colsum_blocks(int64_t rows);
int jmt_colsum(int dt, int64_t rows, int N, const void* dy, int64_t ld, float* db, int beta_acc,
               float* partials, void* stream);
/* G column sums in one launch pair (bias gradients of G same-shaped nn.Linear / in_proj modules
 * run as one grouped GEMM): group g reads dy + g*sdy and reduces into db_tab[g] (G <= 8;
 * partials: G * jmt_colsum_blocks(rows) * N floats; N, ld, sdy multiples of 16/elem bytes). */
int jmt_colsum_grouped(int dt, int G, int64_t rows, int N, const void* dy, int64_t ld,
                       int64_t sdy, float* const* db_tab, int beta_acc, float* partials,
                       void* stream);

/* An empty one-block launch (measurement: the overhead of an event pair around a launch). */
int jmt_noop(void* stream);

/* Strided 2-D copy with dtype conversion and optional transpose (layout plumbing:
 * the (T,B) output of the FC head, torch.stack of the SELF_ATTEN head). dst may be accumulated
 * into (accumulate=1). */
int jmt_copy2d(int src_dt, int dst_dt, int64_t rows, int64_t cols, const void* src,
               int64_t src_rs, int64_t src_cs, void* dst, int64_t dst_rs, int64_t dst_cs,
               int accumulate, void* stream);

/* ------------------------------------------------------------------ regressor output layers
 * The second Linear(128, k) of the V and A regressors (two_transformers.py:104-114; k = 1, or
 * the digitize_num bins of configs[4]'s head, k <= 24) for both heads at once: they read the
 * halves of one hidden buffer h = [h_0 | h_1] (rows x 256, row stride ldh, bf16 / f16, ReLU
 * applied); W2_g (k x 128) in h's dtype, b2_g fp32 (NULL = no bias).
 * jmt_head_fwd: y_g[r][o] = sum_j h_g[r][j] W2_g[o][j] + b2_g[o] (fp32 accumulation), y_g at row
 *   stride ldy in y_dt (f32 or h's dtype).
 * jmt_head_bwd: dh[r][128 g + j] = [h > 0] sum_o gy_g[r][o] W2_g[o][j] (h's dtype, row stride
 *   lddh); dw2_g += sum_r gy_g[r][o] h_g[r][j] and db2_g += sum_r gy_g[r][o] (fp32, NULL =
 *   skip), deterministic two-phase sums through `partials`
 *   (jmt_head_bwd_workspace_bytes(rows) bytes). */
int jmt_head_fwd(int h_dt, int y_dt, int64_t rows, int hid, int k, const void* h, int64_t ldh,
                 const void* w2_0, const void* w2_1, const float* b2_0, const float* b2_1,
                 void* y_0, void* y_1, int64_t ldy, void* stream);
int jmt_head_bwd(int h_dt, int gy_dt, int64_t rows, int hid, int k, const void* h, int64_t ldh,
                 const void* w2_0, const void* w2_1, const void* gy_0, const void* gy_1,
                 int64_t ldgy, void* dh, int64_t lddh, float* dw2_0, float* dw2_1, float* db2_0,
                 float* db2_1, float* partials, void* stream);
size_t jmt_head_bwd_workspace_bytes(int64_t rows);

/* ------------------------------------------------------------------ CCC losses
 * kind 0: losses/loss.py:8-32 CCCLoss (digitize_num k; k>1: pred is (n,k) logits, softmax over
 *         bins = linspace(range) first)
 * kind 1: losses/CCCLoss.py:4-43 CCCLoss(ignore) (labels == ignore are masked; the ccc is
 *         divided by the pre-mask batch size `bs`: bs >= 1 as given — size(0) of the (1, B*T)
 *         view of train.py:303-307, the same on every rank —, bs < 0 = 1-D predictions: the
 *         gathered size(0) = sum over ranks of the pre-mask counts)
 * Local statistics (double[8]: n, mean_x, mean_y, M2x, M2y, Cxy, pre-mask count, 0) of this
 * rank's elements;
 * several ranks' statistics are combined exactly (Chan) by jmt_ccc_finish, which writes the loss
 * (fp32 scalar) and 8 doubles of gradient coefficients {c0, c1, c2, mean_x, mean_y, valid, 0, 0}
 * used by jmt_ccc_bwd: dL/dx_i = grad_loss * (c0 + c1 (x_i - mean_x) + c2 (y_i - mean_y)). */
int jmt_ccc_stats(int kind, int pred_dt, int64_t n, int k, const void* pred, const float* label,
                  float ignore, float lo, float hi, double* stats, void* stream);
int jmt_ccc_finish(int kind, int world, const double* stats_all, int64_t bs, float eps,
                   float* loss, double* coef, void* stream);
/* ABI 5: the same, writing *add + loss (one fp32 rounding, as torch's l1 + l2 of
 * train.py:311) when add != NULL: the two criteria of a training step summed in the finish
 * kernel instead of a separate add launch. */
int jmt_ccc_finish_add(int kind, int world, const double* stats_all, int64_t bs, float eps,
                       const float* add, float* loss, double* coef, void* stream);
int jmt_ccc_bwd(int kind, int pred_dt, int64_t n, int k, const void* pred, const float* label,
                float ignore, float lo, float hi, const double* coef, const float* grad_loss,
                void* dpred, void* stream);
/* CELoss (losses/loss.py:34-51; replaces its host numpy digitize + F.cross_entropy): labels
 * digitized on the device into k bins (np.digitize over linspace(lo, hi, k + 1) - 1, top bin
 * clamped), x (n, k) logits, optional class weights (k floats, NULL = none).
 * jmt_ce_stats: double[4] = (sum w nll, sum w, labels below lo, 0) of this rank's rows;
 * jmt_ce_finish: `world` ranks' stats (rank order) -> loss = sum w nll / sum w (fp32 scalar; NaN
 * when any label fell below lo, where the reference raises) and coef[0] = 1 / sum w;
 * jmt_ce_bwd: dx_ij = grad_loss w[c_i] coef[0] (softmax(x_i)_j - [j == c_i]);
 * jmt_ce_labels: the digitized labels (int64).  No host synchronisation. */
int jmt_ce_stats(int x_dt, int64_t n, int k, const void* x, const float* label, float lo, float hi,
                 const float* weights, double* stats, void* stream);
int jmt_ce_finish(int world, const double* stats_all, float* loss, double* coef, void* stream);
int jmt_ce_bwd(int x_dt, int64_t n, int k, const void* x, const float* label, float lo, float hi,
               const float* weights, const double* coef, const float* grad_loss, void* dx,
               void* stream);
int jmt_ce_labels(int64_t n, int k, const float* label, float lo, float hi, int64_t* out,
                  void* stream);
/* Mask indices (labels != ignore) in ascending order, count written to *count (device int64).
 * The bit-exact padding-mask indices of the ignore path. */
int jmt_mask_indices(int64_t n, const float* label, float ignore, int64_t* idx, int64_t* count,
                     void* stream);

/* ------------------------------------------------------------------ optimizer
 * torch.optim.SGD(momentum, dampening, weight_decay, nesterov) step over one flat fp32 buffer
 * (instantiator.py:32-38).  grad is multiplied by grad_scale first (GradScaler unscale); if
 * shadow != NULL the updated params are also written as shadow_dt (bf16/f16 compute copies). */
int jmt_sgd_step(int64_t n, float* param, const float* grad, float* momentum_buf, float lr,
                 float momentum, float dampening, float weight_decay, int nesterov,
                 int first_step, float grad_scale, void* shadow, int shadow_dt, void* stream);
/* ABI 5: the same step, then grad[i] = 0 in the same pass (the next step's optimizer.zero_grad()
 * folded into this kernel; for jmt_sgd_step_amp_zero also on a skipped, found_inf step). */
int jmt_sgd_step_zero(int64_t n, float* param, float* grad, float* momentum_buf, float lr,
                      float momentum, float dampening, float weight_decay, int nesterov,
                      int first_step, float grad_scale, void* shadow, int shadow_dt, void* stream);

/* GradScaler with device-resident state (train.py:89,314-316): amp[5] fp32 = {scale, inv_scale,
 * found_inf, growth_tracker, steps_taken}.  jmt_amp_check sets found_inf if any grad*inv_scale is
 * not finite; jmt_sgd_step_amp is jmt_sgd_step on the unscaled gradient, skipped when found_inf
 * (first-step momentum rule: allow_first && steps_taken == 0); jmt_amp_update is torch's _amp_update_scale_
 * (backoff on overflow, growth after growth_interval clean steps) and clears found_inf. */
int jmt_amp_check(int64_t n, const float* grad, float* amp, void* stream);
int jmt_sgd_step_amp(int64_t n, float* param, const float* grad, float* momentum_buf, float lr,
                     float momentum, float dampening, float weight_decay, int nesterov,
                     int allow_first, const float* amp, void* shadow, int shadow_dt,
                     void* stream);
int jmt_sgd_step_amp_zero(int64_t n, float* param, float* grad, float* momentum_buf, float lr,
                          float momentum, float dampening, float weight_decay, int nesterov,
                          int allow_first, const float* amp, void* shadow, int shadow_dt,
                          void* stream);
int jmt_amp_update(float* amp, float growth_factor, float backoff_factor, int growth_interval,
                   void* stream);

/* ------------------------------------------------------------------ validation post-processing
 * val.py:313-382 + EvaluationMetrics/cccmetric.py:4-21 on the GPU.
 * Per-video float64 arrays live in one flat buffer; video v occupies [off[v], off[v]+seglen[v]).
 * jmt_vp_scatter: element i (frame id fid[i], the entry's own vid_length len[i], video vid[i],
 *   predictions pv/pa, labels lv/la) is written to slot off[v] + fid - 1 (Python negative-index
 *   rule) unless a label equals `ignore` or fid > len; among hits of one slot the element with the
 *   largest sequence number seq0 + i wins (the reference loop's last write).  winner: one uint64
 *   per slot, zero-initialised once; seq0 must grow across calls (seq0 += n).
 * jmt_vp_smooth: y = uniform_filter1d(clip(x, -1, 1), size, mode='constant') per video.
 * jmt_vp_ccc: out2[0] = ccc(x0, y0), out2[1] = ccc(x1, y1) (population std, float64). */
int jmt_vp_scatter(int64_t n, const int* fid, const int* len, const int* vid, const int64_t* off,
                   const int* seglen, const float* pv, const float* pa, const float* lv,
                   const float* la, float ignore, int64_t seq0, uint64_t* winner, double* pred_v,
                   double* pred_a, double* lab_v, double* lab_a, void* stream);
int jmt_vp_smooth(int64_t total, int nseg, const int64_t* off, const int* seglen, const double* x,
                  int size, double* y, void* stream);
int jmt_vp_ccc(int64_t n, const double* x0, const double* y0, const double* x1, const double* y1,
               double* out2, void* stream);

/* ------------------------------------------------------------------ feature store gather
 * SURVEY.md §8f row 2 (replaces the per-clip np.load + torch.cat of train.py:150-171 and the
 * per-batch H2D copy): out[r, 0:D] = (dt_out) table[idx[r], 0:D] for r < rows, zero rows where
 * idx[r] < 0 or >= nrows_table (left padding).  ld's multiples of 8 elements, 16-B aligned. */
int jmt_gather_rows(int dt_table, int dt_out, int64_t rows, int D, const void* table, int64_t ldt,
                    int64_t nrows_table, const int64_t* idx, void* out, int64_t ldo,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* JMT_H_ */
