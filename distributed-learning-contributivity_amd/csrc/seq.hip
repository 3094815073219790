// Sequential multi-partner approaches (seq-pure / seq-with-final-agg / seqavg,
// mplc/multi_partner_learning.py:337-433) on the batched trainers: the member schedule lives in keyed.h
// (MPLC_REP_SEQ); this file holds the per-member weight snapshot that the aggregating variants average.
// Model-agnostic: rows are n_param floats at the trainer's stride.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keyed.h"
#include "mplc_hip.h"

namespace {

constexpr int SNAP_THREADS = 256;

__global__ __launch_bounds__(SNAP_THREADS) void seq_snapshot_kernel(
    const float* __restrict__ params, int64_t stride, int64_t n_param, const mplc_replica_t* __restrict__ reps,
    const int32_t* __restrict__ seq, const int32_t* __restrict__ splits, int step, int M, int round_len, int epochs,
    const int32_t* __restrict__ snap_first, float* __restrict__ snap) {
  const int r = blockIdx.y;
  const mplc_replica_t rep = reps[r];
  if (rep.kind != MPLC_REP_SEQ) return;
  SeqPos p;
  if (!seq_locate(rep, step, M, round_len, epochs, splits, seq, p) || p.tl != p.ns - 1) return;
  const float* src = params + (int64_t)r * stride;
  float* dst = snap + (int64_t)(snap_first[r] + p.mi) * stride;
  const int64_t n4 = n_param / 4;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(dst);
  for (int64_t i = (int64_t)blockIdx.x * SNAP_THREADS + threadIdx.x; i < n4; i += (int64_t)gridDim.x * SNAP_THREADS)
    d4[i] = s4[i];
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * SNAP_THREADS + threadIdx.x; i < n_param;
       i += (int64_t)gridDim.x * SNAP_THREADS)
    dst[i] = src[i];
}

}  // namespace

extern "C" {

int mplc_seq_snapshot(const float* params, int64_t stride, int64_t n_param, const mplc_replica_t* reps, int n_rep,
                      const int32_t* seq, const int32_t* splits, int step, int minibatch_count, int round_len,
                      int epochs, const int32_t* snap_first, float* snap, void* stream) {
  if (!params || !reps || !seq || !splits || !snap_first || !snap || n_rep < 1 || n_rep > 65535) return MPLC_E_ARG;
  if (stride < n_param || (stride & 3) || n_param < 1 || minibatch_count < 1 || round_len < 1) return MPLC_E_ARG;
  seq_snapshot_kernel<<<dim3(64, n_rep), SNAP_THREADS, 0, (hipStream_t)stream>>>(
      params, stride, n_param, reps, seq, splits, step, minibatch_count, round_len, epochs, snap_first, snap);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MPLC_OK : (int)e;
}

}  // extern "C"
