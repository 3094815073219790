// Exact Shapley aggregation over a bitmask-ordered v(S) table (gfx950).
//
// Replaces mplc/contributivity.py:1210-1253 `shapley_value` (pure Python, O(n 4^n), called from
// compute_SV at mplc/contributivity.py:163) with a single HBM pass: every V[mask] is read once.
//
//   w(s) = s!(n-s-1)!/n! = 1/(n C(n-1,s)),  w(-1) = w(n) = 0
//   SV_i = sum_{S not i} w(|S|)(v(S+i) - v(S)) = A_i - B
//   A_i  = sum_{T contains i} v(T) (w(|T|-1) + w(|T|)),   B = sum_S v(S) w(|S|)
//
// Roofline: HBM-bound, algorithmic bytes = 8 * count (read once) + 16(n+1) written.
//
// Membership sums without per-element per-player work (n >= 16 path, 65536 masks per block):
//   mask bit 0          : element within a lane's 16-B load            -> in-thread accumulator
//   mask bits 1..6      : lane id                                      -> lane-bit masked wave sums
//   mask bit 7          : which of the wave's two 1-KiB loads          -> in-thread accumulator
//   mask bits 8..9      : wave id                                      -> wave-bit masked block sums
//   mask bits 10..12    : pass index low bits (unrolled, compile-time) -> in-thread accumulators
//   mask bits 13..15    : pass group (uniform loop)                    -> in-thread accumulators per group
//   mask bits >= 16     : block id (uniform)                           -> finalize kernel, from block totals
// so each element costs 2 multiplies + a handful of compensated adds, all hidden under the load.
// The popcount of every element is a per-thread constant + popc(g) (uniform) + a compile-time offset,
// so its weights come from a 6-entry register table refreshed once per 8 passes.
//
// Accuracy: in-thread sums are compensated (TwoSum); block trees are plain fp64 (<= 9 ulp relative
// of a sum of non-negative-weight terms); block partials are summed with double-double.  SV_i is a
// difference of two sums about H_n * v_bar apart from a result ~v_bar/n, so the relative error stays
// near 1e-14 at n = 28 (gate: 1e-12 vs the reference fp64 loop and a long-double oracle).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mplc_hip.h"

#pragma clang fp contract(off)

namespace {

constexpr int TPB = 256;
constexpr int PASSES = 64;
constexpr int SPAN = TPB * 4 * PASSES;  // 65536 masks per block
constexpr int LOG_SPAN = 16;
constexpr int NQ = 18;                  // per-block partials: mask bits 0..15, A_total, B
constexpr int MAX_N = 40;
typedef double dvec2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void two_sum_acc(double& s, double& c, double x) {
  const double t = s + x;
  const double bb = t - s;
  c += (s - (t - bb)) + (x - bb);
  s = t;
}

// Double-double add of (bh,bl) into (ah,al).
__device__ __forceinline__ void dd_add(double& ah, double& al, double bh, double bl) {
  const double s = ah + bh;
  const double bb = s - ah;
  const double e = (ah - (s - bb)) + (bh - bb);
  const double lo = e + al + bl;
  ah = s + lo;
  al = lo - (ah - s);
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// Weight tables cw[s] = w(s-1) + w(s), bw[s] = w(s), s = 0..n (zero beyond), computed once on the host (IEEE
// fp64, the same operation order for every launch) and passed by value as a kernel argument: a block copies
// them into LDS instead of re-deriving the binomials with fp64 divisions (that prologue used to cost more
// than the 512 KiB a block streams at n = 24).
struct Weights {
  double cw[MAX_N + 2];
  double bw[MAX_N + 2];
};

inline double weight_w(int n, int s) {  // w(s) = 1 / (n C(n-1, s)), 0 outside [0, n-1]
  if (s < 0 || s >= n) return 0.0;
  double C = 1.0;  // C(n-1, s), exact in fp64 for n <= 40
  for (int j = 0; j < s; ++j) C = C * (double)(n - 1 - j) / (double)(j + 1);
  return 1.0 / ((double)n * C);
}

inline Weights make_weights(int n) {
  Weights W;
  for (int s = 0; s < MAX_N + 2; ++s) {
    W.cw[s] = (s <= n) ? (weight_w(n, s - 1) + weight_w(n, s)) : 0.0;
    W.bw[s] = (s <= n) ? weight_w(n, s) : 0.0;
  }
  return W;
}

__device__ __forceinline__ void load_weights(const Weights& W, double* cw, double* bw) {
  const int s = threadIdx.x;
  if (s < 64) {
    cw[s] = s < MAX_N + 2 ? W.cw[s] : 0.0;
    bw[s] = s < MAX_N + 2 ? W.bw[s] : 0.0;
  }
}

// Pass groups (mask bits 13..15) are split over `gsplit` blocks when a range has few 65536-mask spans, so
// small tables (n < 24) still launch >= 256 blocks (one per CU); every block's partials are membership sums
// over its own masks, so the reduction is unchanged.  gsplit = 1 from 256 spans up (a finer split measured
// slower at n = 24-26: the per-block reductions outweigh the extra parallelism).
inline int gsplit_for(uint64_t nspans) {
  int g = 1;
  while (g < 8 && nspans * (uint64_t)g < 256) g *= 2;
  return g;
}

// ------------------------------------------------------------------------------------------------
// Main pass: one block = 65536 / gsplit masks of a 65536-mask span starting at a multiple of 65536.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(TPB) void shapley_block_kernel(const double* __restrict__ v, uint64_t mask_begin,
                                                            int n, int gsplit, const Weights W,
                                                            double* __restrict__ blockpart) {
  __shared__ double cw_s[64];
  __shared__ double bw_s[64];
  __shared__ double red_s[4][NQ];
  load_weights(W, cw_s, bw_s);
  __syncthreads();

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const uint64_t span = blockIdx.x / (unsigned)gsplit;
  const int gn = 8 / gsplit, g0 = (int)(blockIdx.x % (unsigned)gsplit) * gn;
  const uint64_t base = mask_begin + span * SPAN;
  // thread-constant mask bits: lane -> bits 1..6, wave -> bits 8..9
  const int s_thread = __popcll(base) + __popc(lane) + __popc(wave);

  // accumulators (sum, compensation)
  double a_tot = 0, a_tot_c = 0, b_tot = 0, b_tot_c = 0;
  double a_b0 = 0, a_b0_c = 0, a_b7 = 0, a_b7_c = 0;
  double a_p[6] = {0, 0, 0, 0, 0, 0}, a_p_c[6] = {0, 0, 0, 0, 0, 0};

  const dvec2* vb = reinterpret_cast<const dvec2*>(v + span * SPAN) + wave * 128 + lane;

  // pass p = 8 g + r: r (mask bits 10..12) unrolled at compile time, g (mask bits 13..15) a uniform loop.
  for (int g = g0; g < g0 + gn; ++g) {
    const int sg = s_thread + __popc(g);
    double cw[6], bw[6];  // weights for popcount sg + k, k = popc(r) + h + e in [0, 5]
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int idx = sg + k;
      cw[k] = idx < 64 ? cw_s[idx] : 0.0;
      bw[k] = idx < 64 ? bw_s[idx] : 0.0;
    }
    double gsum = 0.0, gsum_c = 0.0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int pr = __builtin_popcount(r);
      const int p = g * 8 + r;
      // element (half h, e) has mask low bits  p<<10 | wave<<8 | h<<7 | lane<<1 | e
      const dvec2 x0 = __builtin_nontemporal_load(vb + p * 512);       // h = 0
      const dvec2 x1 = __builtin_nontemporal_load(vb + p * 512 + 64);  // h = 1
      const double a00 = x0.x * cw[pr], a01 = x0.y * cw[pr + 1];
      const double a10 = x1.x * cw[pr + 1], a11 = x1.y * cw[pr + 2];
      const double b = (x0.x * bw[pr] + x0.y * bw[pr + 1]) + (x1.x * bw[pr + 1] + x1.y * bw[pr + 2]);
      const double e1 = a01 + a11;  // mask bit 0 set
      const double h1 = a10 + a11;  // mask bit 7 set
      const double tot = (a00 + a01) + h1;
      two_sum_acc(gsum, gsum_c, tot);
      two_sum_acc(b_tot, b_tot_c, b);
      two_sum_acc(a_b0, a_b0_c, e1);
      two_sum_acc(a_b7, a_b7_c, h1);
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (r & (1 << j)) two_sum_acc(a_p[j], a_p_c[j], tot);
    }
    const double gs = gsum + gsum_c;
    two_sum_acc(a_tot, a_tot_c, gs);
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if ((g >> j) & 1) two_sum_acc(a_p[3 + j], a_p_c[3 + j], gs);
  }

  const double tot = a_tot + a_tot_c;
  double q[NQ];
  q[0] = a_b0 + a_b0_c;
#pragma unroll
  for (int bit = 1; bit <= 6; ++bit) q[bit] = ((lane >> (bit - 1)) & 1) ? tot : 0.0;
  q[7] = a_b7 + a_b7_c;
  q[8] = 0.0;  // wave bits handled below from the wave totals
  q[9] = 0.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) q[10 + j] = a_p[j] + a_p_c[j];
  q[16] = tot;
  q[17] = b_tot + b_tot_c;

#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    if (k == 8 || k == 9) continue;
    const double s = wave_sum(q[k]);
    if (lane == 0) red_s[wave][k] = s;
  }
  __syncthreads();
  if (tid < NQ) {
    const int k = tid;
    double s;
    if (k == 8 || k == 9) {
      const int wb = k - 8;
      s = 0.0;
      for (int w = 0; w < 4; ++w)
        if ((w >> wb) & 1) s += red_s[w][16];
    } else {
      s = (red_s[0][k] + red_s[1][k]) + (red_s[2][k] + red_s[3][k]);
    }
    blockpart[(uint64_t)blockIdx.x * NQ + k] = s;
  }
}

// Reduce per-block partials into partial_out[2*(n+1)] (double-double).  One block per quantity.
__global__ __launch_bounds__(TPB) void shapley_reduce_blocks_kernel(const double* __restrict__ blockpart,
                                                                    uint64_t nblocks, int gsplit, uint64_t mask_begin,
                                                                    int n, double* __restrict__ partial_out) {
  __shared__ double hs[TPB], ls[TPB];
  const int qi = blockIdx.x;  // 0..n-1 players, n = B
  double s = 0.0, c = 0.0;
  for (uint64_t b = threadIdx.x; b < nblocks; b += TPB) {
    double x;
    if (qi == n) {
      x = blockpart[b * NQ + 17];
    } else if (qi < LOG_SPAN) {
      x = blockpart[b * NQ + qi];
    } else {
      const uint64_t base = mask_begin + (b / (uint64_t)gsplit) * SPAN;
      x = ((base >> qi) & 1ull) ? blockpart[b * NQ + 16] : 0.0;
    }
    two_sum_acc(s, c, x);
  }
  hs[threadIdx.x] = s;
  ls[threadIdx.x] = c;
  __syncthreads();
  for (int off = TPB / 2; off >= 1; off >>= 1) {
    if ((int)threadIdx.x < off) {
      double h = hs[threadIdx.x], l = ls[threadIdx.x];
      dd_add(h, l, hs[threadIdx.x + off], ls[threadIdx.x + off]);
      hs[threadIdx.x] = h;
      ls[threadIdx.x] = l;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial_out[2 * qi] = hs[0];
    partial_out[2 * qi + 1] = ls[0];
  }
}

// Small tables (n < 16, or any range): one block, generic per-element membership loop.
__global__ __launch_bounds__(TPB) void shapley_small_kernel(const double* __restrict__ v, uint64_t mask_begin,
                                                            uint64_t count, int n, const Weights W,
                                                            double* __restrict__ partial_out) {
  __shared__ double cw_s[64];
  __shared__ double bw_s[64];
  __shared__ double hs[TPB], ls[TPB];
  load_weights(W, cw_s, bw_s);
  __syncthreads();
  double as[16], ac[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { as[i] = 0.0; ac[i] = 0.0; }
  double bs = 0.0, bc = 0.0;
  for (uint64_t k = threadIdx.x; k < count; k += TPB) {
    const uint64_t m = mask_begin + k;
    const double x = v[k];
    const int s = __popcll(m);
    const double a = x * cw_s[s];
    two_sum_acc(bs, bc, x * bw_s[s]);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < n && ((m >> i) & 1ull)) two_sum_acc(as[i], ac[i], a);
  }
  for (int q = 0; q <= n; ++q) {
    double h = 0.0, l = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i == q) { h = as[i]; l = ac[i]; }
    if (q == n) { h = bs; l = bc; }
    hs[threadIdx.x] = h;
    ls[threadIdx.x] = l;
    __syncthreads();
    for (int off = TPB / 2; off >= 1; off >>= 1) {
      if ((int)threadIdx.x < off) {
        double hh = hs[threadIdx.x], ll = ls[threadIdx.x];
        dd_add(hh, ll, hs[threadIdx.x + off], ls[threadIdx.x + off]);
        hs[threadIdx.x] = hh;
        ls[threadIdx.x] = ll;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      partial_out[2 * q] = hs[0];
      partial_out[2 * q + 1] = ls[0];
    }
    __syncthreads();
  }
}

__global__ void shapley_finalize_kernel(const double* __restrict__ partial, int n, double* __restrict__ sv) {
  const int i = threadIdx.x;
  if (i < n) sv[i] = (partial[2 * i] - partial[2 * n]) + (partial[2 * i + 1] - partial[2 * n + 1]);
}

inline int hip_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MPLC_OK : (int)e;
}

}  // namespace

extern "C" {

int mplc_abi_version(void) { return MPLC_ABI_VERSION; }

size_t mplc_shapley_workspace_bytes(int n, uint64_t count) {
  if (n < 16) return 0;
  const uint64_t nspans = (count + SPAN - 1) / SPAN;
  return (size_t)(nspans * gsplit_for(nspans)) * NQ * sizeof(double);
}

int mplc_shapley_partial(const double* v, uint64_t mask_begin, uint64_t count, int n, double* partial_out,
                         void* workspace, size_t workspace_bytes, void* stream) {
  if (n < 1 || n > MAX_N || v == nullptr || partial_out == nullptr) return MPLC_E_ARG;
  if (count == 0) return MPLC_E_ARG;
  if (n < 64 && (mask_begin >= (1ull << n) || count > (1ull << n) - mask_begin)) return MPLC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (n < 16) {
    shapley_small_kernel<<<1, TPB, 0, s>>>(v, mask_begin, count, n, make_weights(n), partial_out);
    return hip_status();
  }
  if ((mask_begin % SPAN) != 0 || (count % SPAN) != 0) return MPLC_E_ARG;
  const uint64_t nspans = count / SPAN;
  const int gsplit = gsplit_for(nspans);
  const uint64_t nblocks = nspans * gsplit;
  if (workspace == nullptr || workspace_bytes < mplc_shapley_workspace_bytes(n, count)) return MPLC_E_WORKSPACE;
  if (nblocks > 0x7fffffffull) return MPLC_E_ARG;
  double* bp = (double*)workspace;
  shapley_block_kernel<<<(unsigned)nblocks, TPB, 0, s>>>(v, mask_begin, n, gsplit, make_weights(n), bp);
  int st = hip_status();
  if (st) return st;
  shapley_reduce_blocks_kernel<<<n + 1, TPB, 0, s>>>(bp, nblocks, gsplit, mask_begin, n, partial_out);
  return hip_status();
}

int mplc_shapley_finalize(const double* partial, int n, double* sv_out, void* stream) {
  if (n < 1 || n > MAX_N || partial == nullptr || sv_out == nullptr) return MPLC_E_ARG;
  shapley_finalize_kernel<<<1, 64, 0, (hipStream_t)stream>>>(partial, n, sv_out);
  return hip_status();
}

int mplc_shapley_exact(const double* v, int n, double* sv_out, void* workspace, size_t workspace_bytes,
                       void* stream) {
  if (n < 1 || n > MAX_N || v == nullptr || sv_out == nullptr) return MPLC_E_ARG;
  // partial_out lives at the tail of the workspace for n >= 16, else needs 2(n+1) doubles of workspace.
  const uint64_t count = 1ull << n;
  const size_t need = mplc_shapley_workspace_bytes(n, count);
  const size_t total = need + 2 * (size_t)(n + 1) * sizeof(double);
  if (workspace == nullptr || workspace_bytes < total) return MPLC_E_WORKSPACE;
  double* partial = (double*)((char*)workspace + need);
  int st = mplc_shapley_partial(v, 0, count, n, partial, workspace, need, stream);
  if (st) return st;
  return mplc_shapley_finalize(partial, n, sv_out, stream);
}

}  // extern "C"
