// HBM-resident feature store gather: out[r, :] = table[idx[r], :] for a
// batch of window clips, converted to the compute dtype; idx < 0 -> zero row (left padding of
// padSequence.py:14-21).  Replaces the per-clip np.load + torch.cat of wavLM vectors inside the
// training loop (train.py:150-171) and the host->device copy of the batch: the whole feature
// table stays in HBM (288 GB per GPU) and a window batch is assembled on the device.
// HBM-bound: per row D*(|table| + |out|) bytes; one wave per row, 16-B loads / stores per lane.
#include "common.h"

namespace jmt {

constexpr int GB = 256;

template <typename TI, typename TO>
__global__ __launch_bounds__(GB) void gather_rows_kernel(int64_t rows, int D, const TI* table,
                                                         int64_t ldt, int64_t nrows_table,
                                                         const int64_t* idx, TO* out,
                                                         int64_t ldo) {
  constexpr int V = 16 / sizeof(TI) < 16 / sizeof(TO) ? 16 / sizeof(TI) : 16 / sizeof(TO);
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * (GB / 64) + (threadIdx.x >> 6); r < rows;
       r += (int64_t)gridDim.x * (GB / 64)) {
    const int64_t s = idx[r];
    const bool valid = s >= 0 && s < nrows_table;
    const TI* src = table + (valid ? s : 0) * ldt;
    TO* dst = out + r * ldo;
    typedef TI IV __attribute__((ext_vector_type(V)));
    typedef TO OV __attribute__((ext_vector_type(V)));
    for (int c = lane * V; c < D; c += 64 * V) {
      if (c + V <= D) {
        OV o;
        if (valid) {
          const IV iv = *(const IV*)(src + c);
#pragma unroll
          for (int e = 0; e < V; ++e) o[e] = from_f<TO>(to_f(iv[e]));
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e) o[e] = from_f<TO>(0.f);
        }
        *(OV*)(dst + c) = o;
      } else {
        for (int e = 0; e < V && c + e < D; ++e)
          dst[c + e] = from_f<TO>(valid ? to_f(src[c + e]) : 0.f);
      }
    }
  }
}

}  // namespace jmt

using namespace jmt;

extern "C" int jmt_gather_rows(int dt_table, int dt_out, int64_t rows, int D, const void* table,
                               int64_t ldt, int64_t nrows_table, const int64_t* idx, void* out,
                               int64_t ldo, void* stream) {
  if (rows == 0) return JMT_OK;
  JMT_CHECK_ARG(rows > 0 && D > 0 && table && idx && out && ldt >= D && ldo >= D,
                "jmt_gather_rows: bad args");
  JMT_CHECK_ARG(ldt % 8 == 0 && ldo % 8 == 0 && ((uintptr_t)table % 16) == 0 &&
                    ((uintptr_t)out % 16) == 0,
                "jmt_gather_rows: rows must be 16-B aligned (ld multiple of 8)");
  int64_t blocks = (rows + GB / 64 - 1) / (GB / 64);
  if (blocks > 65536) blocks = 65536;
  hipStream_t st = as_stream(stream);
#define JMT_GATHER(TI, TO)                                                                     \
  hipLaunchKernelGGL((gather_rows_kernel<TI, TO>), dim3((unsigned)blocks), dim3(GB), 0, st, rows, \
                     D, (const TI*)table, ldt, nrows_table, idx, (TO*)out, ldo)
  if (dt_table == JMT_F32 && dt_out == JMT_F32) JMT_GATHER(float, float);
  else if (dt_table == JMT_F32 && dt_out == JMT_BF16) JMT_GATHER(float, __bf16);
  else if (dt_table == JMT_F32 && dt_out == JMT_F16) JMT_GATHER(float, _Float16);
  else if (dt_table == JMT_F16 && dt_out == JMT_F32) JMT_GATHER(_Float16, float);
  else if (dt_table == JMT_F16 && dt_out == JMT_F16) JMT_GATHER(_Float16, _Float16);
  else if (dt_table == JMT_F16 && dt_out == JMT_BF16) JMT_GATHER(_Float16, __bf16);
  else if (dt_table == JMT_BF16 && dt_out == JMT_F32) JMT_GATHER(__bf16, float);
  else if (dt_table == JMT_BF16 && dt_out == JMT_BF16) JMT_GATHER(__bf16, __bf16);
  else if (dt_table == JMT_BF16 && dt_out == JMT_F16) JMT_GATHER(__bf16, _Float16);
  else return set_error(JMT_ERR_ARG, "jmt_gather_rows: dtype pair %d -> %d", dt_table, dt_out);
#undef JMT_GATHER
  JMT_LAUNCH_CHECK("jmt_gather_rows");
  return JMT_OK;
}
