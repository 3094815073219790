// Phase timing for csrc/logreg.hip (scripts/lr_phases.py force-includes this into a timing copy of the library;
// never part of the product build).  LR_PHASE(i) charges the wall-clock ticks since the wave's previous mark (the
// mark's own bookkeeping excluded) to phase i and counts the mark; LR_PHASE(-1) only starts the clock.  One wave per workgroup, so lane 0 keeps the
// time of the previous mark in LDS.
#pragma once
#include <hip/hip_runtime.h>
__device__ unsigned long long lr_phase_ticks[16];
__device__ unsigned long long lr_phase_calls[16];
__device__ unsigned long long lr_phase_span[4096][3];  // per workgroup: start and end ticks, fits << 32 | iterations
__shared__ unsigned long long lr_phase_last;
__shared__ unsigned long long lr_phase_lt[16], lr_phase_lc[16];  // this wave's sums, flushed at the last mark
__device__ __forceinline__ void lr_phase_mark(int i) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = wall_clock64();
    if (i < 0) {
      for (int k = 0; k < 16; ++k) lr_phase_lt[k] = lr_phase_lc[k] = 0;
      if (blockIdx.x < 4096) lr_phase_span[blockIdx.x][0] = t;
    } else {
      lr_phase_lt[i] += t - lr_phase_last;
      lr_phase_lc[i] += 1;
    }
    if (i == 7 && blockIdx.x < 4096) {
      lr_phase_span[blockIdx.x][1] = t;
      lr_phase_span[blockIdx.x][2] = (lr_phase_lc[1] << 32) | lr_phase_lc[3];
    }
    if (i == 7) {  // the kernel's last mark: one atomic per phase per wave (no contention inside the timed code)
      for (int k = 0; k < 16; ++k) {
        atomicAdd(&lr_phase_ticks[k], lr_phase_lt[k]);
        atomicAdd(&lr_phase_calls[k], lr_phase_lc[k]);
      }
    }
    lr_phase_last = wall_clock64();
  }
  __syncthreads();
}
#define LR_PHASE(i) lr_phase_mark(i)
extern "C" int lr_phase_read(unsigned long long* ticks, unsigned long long* calls, int* wall_khz) {
  unsigned long long z[16] = {0};
  if (hipMemcpyFromSymbol(ticks, HIP_SYMBOL(lr_phase_ticks), sizeof(z)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(calls, HIP_SYMBOL(lr_phase_calls), sizeof(z)) != hipSuccess) return -1;
  hipMemcpyToSymbol(HIP_SYMBOL(lr_phase_ticks), z, sizeof(z));
  hipMemcpyToSymbol(HIP_SYMBOL(lr_phase_calls), z, sizeof(z));
  return hipDeviceGetAttribute(wall_khz, hipDeviceAttributeWallClockRate, 0) == hipSuccess ? 0 : -1;
}
extern "C" int lr_phase_spans(unsigned long long* out) {  // [4096][3]
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(lr_phase_span), sizeof(unsigned long long) * 4096 * 3) == hipSuccess ? 0 : -1;
}
