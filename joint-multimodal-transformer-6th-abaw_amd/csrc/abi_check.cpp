// Host-side ABI check, built with AddressSanitizer by `make asan` (host code only: the kernels
// are compiled out with --offload-host-only) and run by tests/test_abi.py on the CPU (SURVEY.md
// §5 "Race detection / sanitizers").  Every entry point of include/jmt.h that validates its
// arguments is driven with invalid ones (null / misaligned pointers, bad sizes, unsupported
// dtypes, oversized tables); each must return a negative JMT_ERR_* and leave a bounded,
// non-empty jmt_last_error() — all in the library's host code (argument checks, planners, error
// formatting), so ASan sees every host-side byte the ABI touches.  No GPU is needed.
#include <stdio.h>
#include <string.h>

#include "../../include/jmt.h"

static int g_fail = 0;

// the error message names the check (not a later failure, e.g. a launch without a device)
static void expect_msg(const char* what, const char* needle) {
  const char* e = jmt_last_error();
  if (!e || !strstr(e, needle)) {
    fprintf(stderr, "FAIL %s: err='%s' lacks '%s'\n", what, e ? e : "(null)", needle);
    ++g_fail;
  }
}

static void expect_err(const char* what, int rc) {
  const char* e = jmt_last_error();
  const size_t n = e ? strnlen(e, 1024) : 0;
  if (rc >= 0 || n == 0 || n >= 512) {
    fprintf(stderr, "FAIL %s: rc=%d err='%s'\n", what, rc, e ? e : "(null)");
    ++g_fail;
  }
}

int main() {
  if (jmt_abi_version() != JMT_ABI_VERSION) {
    fprintf(stderr, "FAIL abi version\n");
    return 1;
  }
  alignas(16) char buf[64];
  float* fnull = nullptr;
  void* misal = (void*)(buf + 1);
  void* algn = (void*)buf;        // aligned, never dereferenced (the checks fail first)

  // GEMM: descriptor validation and the host planners
  jmt_gemm_desc d;
  memset(&d, 0, sizeof(d));
  d.ab_dtype = JMT_BF16; d.c_dtype = JMT_BF16; d.M = 128; d.N = 128; d.K = 128;
  d.n_a = d.n_b = d.n_c = 1; d.batch0 = d.batch1 = 1; d.lda = d.ldb = d.ldc = 128;
  d.alpha = 1.f;
  expect_err("gemm null operands", jmt_gemm(&d, nullptr));
  d.a[0] = misal; d.b[0] = misal; d.c[0] = misal;
  expect_err("gemm misaligned operands", jmt_gemm(&d, nullptr));
  d.n_a = 9;
  expect_err("gemm pointer table > 8", jmt_gemm(&d, nullptr));
  d.n_a = 1; d.ab_dtype = 7;
  expect_err("gemm dtype", jmt_gemm(&d, nullptr));
  d.ab_dtype = JMT_BF16; d.M = -5;
  expect_err("gemm negative M", jmt_gemm(&d, nullptr));
  // A row sums (ABI 4): table entries, layout and table size are checked before any launch
  d.M = 128; d.a[0] = d.b[0] = d.c[0] = (void*)buf; d.c_dtype = JMT_F32;
  d.a_kmajor = 0; d.b_kmajor = 0; d.n_dbias = 1; d.dbias_tab[0] = nullptr;
  expect_err("gemm dbias null entry", jmt_gemm(&d, nullptr));
  expect_msg("gemm dbias null entry", "every dbias_tab entry");
  d.dbias_tab[0] = (float*)buf; d.a_kmajor = 1;
  expect_err("gemm dbias K-major A", jmt_gemm(&d, nullptr));
  expect_msg("gemm dbias K-major A", "row sums");
  d.a_kmajor = 0; d.n_dbias = 9;
  expect_err("gemm dbias table > 8", jmt_gemm(&d, nullptr));
  expect_msg("gemm dbias table > 8", "dbias table");
  d.n_dbias = 0;
  expect_err("gemm null desc", jmt_gemm(nullptr, nullptr));
  size_t ws = 0;
  for (int m = 1; m <= 1 << 16; m *= 7)
    for (int s = 1; s <= 256; s *= 4) ws += jmt_gemm_workspace_bytes(m, 512, 3, s);
  int splits = 0;
  for (int k = 16; k <= 1 << 20; k *= 5)
    splits += jmt_gemm_plan_splits(JMT_BF16, 1024, 512, k, 1) +
              jmt_gemm_plan_splits(JMT_F32, 7, 3, k, 6);
  if (ws == 0 || splits <= 0) {
    fprintf(stderr, "FAIL planners ws=%zu splits=%d\n", ws, splits);
    ++g_fail;
  }

  // row ops
  expect_err("l2norm_fwd null", jmt_l2norm_fwd(JMT_BF16, JMT_BF16, 8, 512, nullptr, 512, nullptr,
                                               512, fnull, 1e-12f, nullptr));
  expect_err("layernorm_fwd dtype", jmt_layernorm_fwd(9, JMT_BF16, 8, 512, misal, 512, nullptr, 0,
                                                      fnull, fnull, 1e-5f, misal, 512, fnull,
                                                      fnull, nullptr));
  expect_err("softmax_fwd null", jmt_softmax_fwd(JMT_BF16, 8, 300, nullptr, 304, 1.f, nullptr, 304,
                                                 nullptr));
  expect_err("colsum null", jmt_colsum(JMT_BF16, 64, 512, nullptr, 512, fnull, 0, fnull, nullptr));
  expect_err("copy2d dtype", jmt_copy2d(5, 6, 4, 4, misal, 4, 1, misal, 4, 1, 0, nullptr));

  // attention
  expect_err("attn_fwd head dim", jmt_attn_fwd(JMT_BF16, 2, 1, 300, 300, 64, misal, 512, 512,
                                               misal, 512, 512, misal, 512, 512, misal, 512, 512,
                                               0.1f, fnull, nullptr));
  expect_err("attn_fwd misaligned", jmt_attn_fwd(JMT_BF16, 2, 1, 300, 300, 512, misal, 512, 512,
                                                 misal, 512, 512, misal, 512, 512, misal, 512,
                                                 512, 0.1f, fnull, nullptr));
  expect_err("attn_bwd sizes", jmt_attn_bwd(JMT_BF16, -1, 1, 300, 300, 512, misal, 1, 1, misal, 1,
                                            1, misal, 1, 1, misal, 1, 1, misal, 1, 1, fnull,
                                            misal, misal, 8, misal, 1, 1, 0.1f, nullptr));
  expect_err("attn_dkdv ldp", jmt_attn_dkdv(JMT_BF16, 2, 1, 300, 300, 512, misal, misal, 320,
                                           misal, 512, 512, misal, 512, 512, nullptr, 0, 0,
                                           misal, 512, 512, misal, 512, 512, nullptr, 0, 0,
                                           nullptr));
  expect_err("attn_dkdv head dim", jmt_attn_dkdv(JMT_BF16, 2, 1, 300, 300, 64, misal, misal, 384,
                                                 misal, 512, 512, misal, 512, 512, nullptr, 0, 0,
                                                 misal, 512, 512, misal, 512, 512, nullptr, 0,
                                                 0, nullptr));
  expect_err("attn_dkdv dq misaligned", jmt_attn_dkdv(JMT_BF16, 2, 1, 300, 300, 512, algn, algn,
                                                      384, algn, 512, 512, algn, 512, 512, misal,
                                                      512, 512, algn, 512, 512, algn, 512, 512,
                                                      misal, 512, 512, nullptr));
  expect_err("attn_bwd pds ldp", jmt_attn_bwd(JMT_BF16, 2, 1, 300, 300, 512, algn, 512, 512,
                                              algn, 512, 512, algn, 512, 512, algn, 512, 512,
                                              algn, 512, 512, fnull, algn, algn, 300, nullptr,
                                              0, 0, 0.1f, nullptr));
  expect_err("small_attn_fwd null", jmt_small_attn_fwd(JMT_BF16, 4, 1, 6, 6, 512, nullptr, 512,
                                                       512, nullptr, 512, 512, nullptr, 512, 512,
                                                       nullptr, 512, 512, 0.1f, fnull, nullptr));

  // losses
  expect_err("ccc_stats kind", jmt_ccc_stats(3, JMT_F32, 10, 1, misal, fnull, 0.f, -1.f, 1.f,
                                             nullptr, nullptr));
  expect_err("ccc_stats bins", jmt_ccc_stats(0, JMT_F32, 10, 100, misal, fnull, 0.f, -1.f, 1.f,
                                             (double*)buf, nullptr));
  expect_err("ccc_finish null", jmt_ccc_finish(0, 0, nullptr, 1, 1e-8f, fnull, nullptr, nullptr));
  expect_err("ccc_finish_add null", jmt_ccc_finish_add(0, 1, nullptr, 1, 1e-8f, fnull, fnull,
                                                       nullptr, nullptr));
  expect_err("ce_stats bins", jmt_ce_stats(JMT_F32, 10, 1, misal, fnull, -1.f, 1.f, fnull,
                                           (double*)buf, nullptr));
  expect_err("ce_bwd null", jmt_ce_bwd(JMT_F32, 10, 5, nullptr, fnull, -1.f, 1.f, fnull, nullptr,
                                       fnull, nullptr, nullptr));
  expect_err("ce_labels null", jmt_ce_labels(10, 5, fnull, -1.f, 1.f, nullptr, nullptr));
  expect_err("mask_indices null", jmt_mask_indices(10, fnull, -5.f, nullptr, nullptr, nullptr));

  // optimizer, validation post-processing, feature store
  expect_err("sgd null", jmt_sgd_step(10, fnull, fnull, fnull, 0.1f, 0.9f, 0.f, 0.f, 1, 1, 1.f,
                                      nullptr, JMT_BF16, nullptr));
  expect_err("sgd_zero null", jmt_sgd_step_zero(10, fnull, nullptr, fnull, 0.1f, 0.9f, 0.f, 0.f,
                                                1, 1, 1.f, nullptr, JMT_BF16, nullptr));
  expect_err("sgd_amp_zero null", jmt_sgd_step_amp_zero(10, fnull, fnull, fnull, 0.1f, 0.9f,
                                                        0.f, 0.f, 1, 1, nullptr, nullptr,
                                                        JMT_BF16, nullptr));
  expect_err("vp_ccc null", jmt_vp_ccc(10, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr));
  expect_err("gather null", jmt_gather_rows(JMT_F32, JMT_BF16, 4, 512, nullptr, 512, 4, nullptr,
                                            nullptr, 512, nullptr));

  if (jmt_bounds_violations(0) != -1) {
    fprintf(stderr, "FAIL bounds counters present in the default build\n");
    ++g_fail;
  }
  printf("abi_check: %s (%d failures)\n", g_fail ? "FAIL" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
