// Monte-Carlo Shapley over a bitmask v(S) table on gfx950: truncated permutation walks (TMCS / ITMCS,
// mplc/contributivity.py:195-322) with the truncation test on device.
//
// V is the dense table V[mask] (fp64, 2^n entries, bit i = partner i); an entry that is NaN is "not yet
// evaluated".  One thread walks one permutation exactly like the reference's inner loop:
//   char[0] = 0; for j: if |v_all - char[j]| < truncation: char[j+1] = char[j]            (TMCS)
//                                                         or char[j] + a * size[j]           (ITMCS, a fixed at the
//                                                            first truncation: (v_all - char[j]) / sum size[j..n-1])
//                        else char[j+1] = V[prefix mask]; row[perm[j]] = char[j+1] - char[j]
// in the reference's fp64 operation order (no contraction, see the pragma below).  A walk that
// reaches an unknown prefix stops and reports it (status = j, need = mask): the host trains that frontier in
// one batch and walks again.  This is how the contributivity engine finds the coalitions a wave of
// permutations needs (mplc/contributivity.py _prefetch_permutation_wave) and how it computes TMCS rows on a
// fully known table.
// The fused moments form (fixed permutation budget, permutations either given or drawn on device from a keyed
// counter) reduces sum(row) and sum(row^2) per partner with wavefront shuffles + a fixed-order block pass.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "keyed.h"
#include "mplc_hip.h"

// IEEE fp64 in the reference's operation order: no FMA contraction anywhere in this file (HIP's default
// -ffp-contract=fast would fuse char + a * size into one rounding).  Plain operators on purpose: the
// pragma governs the operations written here, not those inlined from library intrinsics.
#pragma clang fp contract(off)

namespace {

constexpr int MC_MAX_N = 30;
constexpr int MC_THREADS = 256;

// keyed Fisher-Yates permutation of [0, n) for permutation index k (device-drawn mode)
__device__ __forceinline__ void keyed_permutation(uint64_t seed, uint64_t k, int n, uint8_t* p) {
  for (int i = 0; i < n; ++i) p[i] = (uint8_t)i;
  uint64_t s = mix64(seed ^ mix64(k + 0x7A11ull));
  for (int i = n - 1; i > 0; --i) {
    s = mix64(s + 0x9E3779B97F4A7C15ull);
    const int j = (int)(((s >> 32) * (uint64_t)(i + 1)) >> 32);
    const uint8_t t = p[i];
    p[i] = p[j];
    p[j] = t;
  }
}

// One permutation walk; returns n when complete, else the first position whose prefix is unknown.
__device__ __forceinline__ int walk(const double* __restrict__ V, int n, const uint8_t* perm, double v_all,
                                    double trunc, int interpolate, const double* __restrict__ sizes, double* row,
                                    uint64_t* need) {
  double cur = 0.0;
  uint64_t mask = 0;
  bool first = true;
  double a = 0.0;
  for (int j = 0; j < n; ++j) {
    const int p = perm[j];
    mask |= 1ull << p;
    double nxt;
    if (fabs(v_all - cur) < trunc) {
      if (!interpolate) {
        nxt = cur;
      } else {
        if (first) {
          double rest = 0.0;  // integer sizes: exact
          for (int i = j; i < n; ++i) rest = rest + sizes[i];
          a = (v_all - cur) / rest;
          first = false;
        }
        nxt = cur + a * sizes[j];  // reference quirk: size of partner j (index order)
      }
    } else {
      const double v = V[mask];
      if (isnan(v)) {
        *need = mask;
        return j;
      }
      nxt = v;
    }
    row[p] = nxt - cur;
    cur = nxt;
  }
  return n;
}

__global__ __launch_bounds__(MC_THREADS) void tmc_walk_kernel(const double* __restrict__ V, int n,
                                                              const uint8_t* __restrict__ perms, int n_perms,
                                                              double v_all, double trunc, int interpolate,
                                                              const double* __restrict__ sizes,
                                                              double* __restrict__ rows, int32_t* __restrict__ status,
                                                              uint64_t* __restrict__ need) {
  const int k = blockIdx.x * MC_THREADS + threadIdx.x;
  if (k >= n_perms) return;
  uint8_t perm[MC_MAX_N];
  for (int j = 0; j < n; ++j) perm[j] = perms[(int64_t)k * n + j];
  double row[MC_MAX_N];
  for (int j = 0; j < n; ++j) row[j] = 0.0;
  uint64_t nd = 0;
  const int st = walk(V, n, perm, v_all, trunc, interpolate, sizes, row, &nd);
  status[k] = st;
  need[k] = nd;
  double* out = rows + (int64_t)k * n;
  for (int j = 0; j < n; ++j) out[j] = row[j];
}

// Fixed-budget moments: block b reduces permutations [b*256, b*256+256) into partial[b][2n+1]
// = {sum row_j (j < n), sum row_j^2 (j < n), complete walks}.  Deterministic (no atomics).
__global__ __launch_bounds__(MC_THREADS) void tmc_moments_kernel(const double* __restrict__ V, int n,
                                                                 const uint8_t* __restrict__ perms, uint64_t seed,
                                                                 uint64_t perm_base, int n_perms, double v_all,
                                                                 double trunc, int interpolate,
                                                                 const double* __restrict__ sizes,
                                                                 double* __restrict__ partial) {
  __shared__ double red[MC_THREADS / 64][2 * MC_MAX_N + 1];
  const int tid = threadIdx.x;
  const int k = blockIdx.x * MC_THREADS + tid;
  uint8_t perm[MC_MAX_N];
  double row[MC_MAX_N];
  for (int j = 0; j < n; ++j) row[j] = 0.0;
  double ok = 0.0;
  if (k < n_perms) {
    if (perms) {
      for (int j = 0; j < n; ++j) perm[j] = perms[(int64_t)k * n + j];
    } else {
      keyed_permutation(seed, perm_base + (uint64_t)k, n, perm);
    }
    uint64_t nd = 0;
    if (walk(V, n, perm, v_all, trunc, interpolate, sizes, row, &nd) == n) {
      ok = 1.0;
    } else {
      for (int j = 0; j < n; ++j) row[j] = 0.0;  // incomplete walks (unknown entries) are not counted
    }
  }
  const int lane = tid & 63, wave = tid >> 6;
  for (int q = 0; q < 2 * n + 1; ++q) {
    double v = q < n ? row[q] : (q < 2 * n ? row[q - n] * row[q - n] : ok);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[wave][q] = v;
  }
  __syncthreads();
  if (tid < 2 * n + 1) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < MC_THREADS / 64; ++w) s += red[w][tid];
    partial[(int64_t)blockIdx.x * (2 * n + 1) + tid] = s;
  }
}

__global__ void tmc_moments_reduce_kernel(const double* __restrict__ partial, int blocks, int width,
                                          double* __restrict__ out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= width) return;
  double s = 0.0;
  for (int b = 0; b < blocks; ++b) s += partial[(int64_t)b * width + q];
  out[q] = s;
}

inline int launch_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MPLC_OK : (int)e;
}

}  // namespace

extern "C" {

int mplc_tmc_walk(const double* V, int n, const uint8_t* perms, int n_perms, double v_all, double truncation,
                  int interpolate, const double* sizes, double* rows, int32_t* status, uint64_t* need, void* stream) {
  if (!V || !perms || !rows || !status || !need || n < 1 || n > MC_MAX_N || n_perms < 1) return MPLC_E_ARG;
  if (interpolate && !sizes) return MPLC_E_ARG;
  tmc_walk_kernel<<<(n_perms + MC_THREADS - 1) / MC_THREADS, MC_THREADS, 0, (hipStream_t)stream>>>(
      V, n, perms, n_perms, v_all, truncation, interpolate, sizes, rows, status, need);
  return launch_status();
}

size_t mplc_tmc_moments_workspace_bytes(int n, int n_perms) {
  if (n < 1 || n > MC_MAX_N || n_perms < 1) return 0;
  return (size_t)((n_perms + MC_THREADS - 1) / MC_THREADS) * (2 * n + 1) * sizeof(double);
}

int mplc_tmc_moments(const double* V, int n, const uint8_t* perms, uint64_t seed, uint64_t perm_base, int n_perms,
                     double v_all, double truncation, int interpolate, const double* sizes, double* moments_out,
                     void* workspace, size_t workspace_bytes, void* stream) {
  if (!V || !moments_out || n < 1 || n > MC_MAX_N || n_perms < 1) return MPLC_E_ARG;
  if (interpolate && !sizes) return MPLC_E_ARG;
  const int blocks = (n_perms + MC_THREADS - 1) / MC_THREADS;
  if (!workspace || workspace_bytes < mplc_tmc_moments_workspace_bytes(n, n_perms)) return MPLC_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  double* partial = (double*)workspace;
  tmc_moments_kernel<<<blocks, MC_THREADS, 0, s>>>(V, n, perms, seed, perm_base, n_perms, v_all, truncation,
                                                   interpolate, sizes, partial);
  tmc_moments_reduce_kernel<<<1, 64, 0, s>>>(partial, blocks, 2 * n + 1, moments_out);
  return launch_status();
}

}  // extern "C"
