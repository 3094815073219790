// FedAvg weighted partner aggregation, batched over coalitions (gfx950).
//
// Replaces mplc/mpl_utils.py:90-102 (Aggregator.aggregate_model_weights: per-layer
// np.average(np.array(weights_for_layer), axis=0, weights=aggregation_weights)) whose float64 result
// Keras' set_weights stores back as float32 (mplc/multi_partner_learning.py:100-104).
//
// numpy's np.average(a, axis=0, weights=w) = np.multiply(a, w).sum(axis=0) / w.sum(): each product is
// rounded to fp64, the axis-0 reduction adds rows sequentially, then one division.  The kernel does
// exactly that per element (fp-contract off: no FMA), so the fp32 result is bit-identical.
//
// Roofline: HBM-bound. Algorithmic bytes per coalition = 4 * n_param * (|S| read + 1 write
// [+ |S| broadcast writes, minus the skipped range of mplc_fedavg_aggregate_bcast_skip]).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mplc_hip.h"

#pragma clang fp contract(off)

namespace {

constexpr int TPB = 256;

__global__ __launch_bounds__(TPB) void fedavg_kernel(float* __restrict__ x, int64_t x_stride,
                                                     const int32_t* __restrict__ first, const double* __restrict__ w,
                                                     const double* __restrict__ scale, int64_t n_param,
                                                     float* __restrict__ out, int64_t out_stride, int broadcast,
                                                     int64_t skip_lo, int64_t skip_hi, int vec4, int skip_avg) {
  const int c = blockIdx.y;
  const int r0 = first[c];
  const int r1 = first[c + 1];
  const double scl = scale[c];
  const int64_t nthreads = (int64_t)gridDim.x * TPB;
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (vec4) {
    // skip_avg: the range [skip_lo, skip_hi) is not visited at all (the element index jumps over it)
    const int64_t lo4 = skip_lo >> 2, gap4 = skip_avg ? (skip_hi - skip_lo) >> 2 : 0;
    const int64_t n4 = (n_param >> 2) - gap4;
    for (int64_t kk = t; kk < n4; kk += nthreads) {
      const int64_t k = kk < lo4 ? kk : kk + gap4;
      const float4 a = reinterpret_cast<const float4*>(x + (int64_t)r0 * x_stride)[k];
      const double w0 = w[r0];
      double s0 = (double)a.x * w0, s1 = (double)a.y * w0, s2 = (double)a.z * w0, s3 = (double)a.w * w0;
      for (int r = r0 + 1; r < r1; ++r) {
        const float4 b = reinterpret_cast<const float4*>(x + (int64_t)r * x_stride)[k];
        const double wr = w[r];
        s0 = s0 + (double)b.x * wr;
        s1 = s1 + (double)b.y * wr;
        s2 = s2 + (double)b.z * wr;
        s3 = s3 + (double)b.w * wr;
      }
      const float4 res = make_float4((float)(s0 / scl), (float)(s1 / scl), (float)(s2 / scl), (float)(s3 / scl));
      if (out) reinterpret_cast<float4*>(out + (int64_t)c * out_stride)[k] = res;
      if (broadcast && (4 * k < skip_lo || 4 * k >= skip_hi))
        for (int r = r0; r < r1; ++r) reinterpret_cast<float4*>(x + (int64_t)r * x_stride)[k] = res;
    }
  } else {
    const int64_t gap = skip_avg ? skip_hi - skip_lo : 0;
    for (int64_t kk = t; kk < n_param - gap; kk += nthreads) {
      const int64_t k = kk < skip_lo ? kk : kk + gap;
      double s = (double)x[(int64_t)r0 * x_stride + k] * w[r0];
      for (int r = r0 + 1; r < r1; ++r) s = s + (double)x[(int64_t)r * x_stride + k] * w[r];
      const float res = (float)(s / scl);
      if (out) out[(int64_t)c * out_stride + k] = res;
      if (broadcast && (k < skip_lo || k >= skip_hi))
        for (int r = r0; r < r1; ++r) x[(int64_t)r * x_stride + k] = res;
    }
  }
}

}  // namespace

namespace {
int fedavg_launch(float* x, int64_t x_stride, const int32_t* first, const double* w, const double* scale,
                  int n_coalitions, int64_t n_param, float* out, int64_t out_stride, int broadcast, int64_t skip_lo,
                  int64_t skip_hi, void* stream, int skip_avg = 0) {
  if (x == nullptr || first == nullptr || w == nullptr || scale == nullptr) return MPLC_E_ARG;
  if (n_coalitions < 1 || n_coalitions > 65535 || n_param < 1 || x_stride < n_param) return MPLC_E_ARG;
  if (out == nullptr && !broadcast) return MPLC_E_ARG;
  if (out != nullptr && out_stride < n_param) return MPLC_E_ARG;
  if (skip_lo < 0 || skip_hi < skip_lo || skip_hi > n_param) return MPLC_E_ARG;
  const bool vec4 = ((skip_lo | skip_hi) & 3) == 0 && ((n_param & 3) == 0) && ((x_stride & 3) == 0) && (((uintptr_t)x & 15) == 0) &&
                    (out == nullptr || (((out_stride & 3) == 0) && (((uintptr_t)out & 15) == 0)));
  const int64_t work = (vec4 ? (n_param >> 2) : n_param) - (skip_avg ? (vec4 ? (skip_hi - skip_lo) >> 2 : skip_hi - skip_lo) : 0);
  int64_t bx = (work + TPB - 1) / TPB;
  // enough blocks to fill 256 CUs across all coalitions, grid-stride the rest
  const int64_t cap = (2048 + n_coalitions - 1) / n_coalitions;
  if (bx > cap) bx = cap < 1 ? 1 : cap;
  dim3 grid((unsigned)bx, (unsigned)n_coalitions);
  fedavg_kernel<<<grid, TPB, 0, (hipStream_t)stream>>>(x, x_stride, first, w, scale, n_param, out, out_stride,
                                                       broadcast, skip_lo, skip_hi, vec4 ? 1 : 0, skip_avg);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MPLC_OK : (int)e;
}
}  // namespace

extern "C" int mplc_fedavg_aggregate(float* x, int64_t x_stride, const int32_t* first, const double* w,
                                     const double* scale, int n_coalitions, int64_t n_param, float* out,
                                     int64_t out_stride, int broadcast, void* stream) {
  return fedavg_launch(x, x_stride, first, w, scale, n_coalitions, n_param, out, out_stride, broadcast, 0, 0, stream);
}

extern "C" int mplc_fedavg_aggregate_bcast_skip(float* x, int64_t x_stride, const int32_t* first, const double* w,
                                                const double* scale, int n_coalitions, int64_t n_param, float* out,
                                                int64_t out_stride, int64_t skip_lo, int64_t skip_hi, void* stream) {
  if (out == nullptr) return MPLC_E_ARG;  // the skipped range's only copy is the coalition row
  return fedavg_launch(x, x_stride, first, w, scale, n_coalitions, n_param, out, out_stride, 1, skip_lo, skip_hi,
                       stream);
}

extern "C" int mplc_fedavg_aggregate_skip(float* x, int64_t x_stride, const int32_t* first, const double* w,
                                          const double* scale, int n_coalitions, int64_t n_param, float* out,
                                          int64_t out_stride, int64_t skip_lo, int64_t skip_hi, void* stream) {
  if (out == nullptr || skip_hi <= skip_lo) return MPLC_E_ARG;
  return fedavg_launch(x, x_stride, first, w, scale, n_coalitions, n_param, out, out_stride, 1, skip_lo, skip_hi,
                       stream, 1);
}
