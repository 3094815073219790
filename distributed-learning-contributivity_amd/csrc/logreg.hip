// Batched FedAvg logistic regression (Titanic model) for gfx950.
//
// Replaces, per coalition, the reference's Titanic path (BASELINE config #2):
//   model   mplc/dataset.py:323-394  Titanic.LogisticRegression = sklearn LR (lbfgs, C=1, L2 on coef only)
//   FedAvg  mplc/multi_partner_learning.py:195-216, 285-334: per epoch, each partner's rows are permuted and
//           split into M minibatches (mplc/partner.py:155-167); per round every partner refits on its
//           minibatch (warm start), the [coef | intercept] rows are np.average'd (mplc/mpl_utils.py:90-115);
//           early stop compares the round-0 val loss of epoch e with e - 10 (mplc/multi_partner_learning.py:
//           177-193), where the never-fitted model of epoch 0 evaluates to [0, 0] (mplc/dataset.py:343-351)
//   score   accuracy of predict() = [w.x + b > 0] on the test set
// Every fit is solved EXACTLY (damped Newton in fp64, gradient < 1e-10), the optimum of the strictly convex
// problem sklearn approximates to tol 1e-4.  Work is tiny (28 unknowns, tens of rows): latency-bound; the point is
// running all coalitions' fits together and keeping each fit's dependent chain short.  Round 5: each FedAvg round is one launch whose waves take
// (coalition, partner) fits from a work queue, and one launch averages each coalition's fits (numpy's order, no
// fused multiply-add).  A fit: its rows staged in LDS as fp64 with the intercept's column of ones; the Hessian
// X^T diag(h) X and the gradient from v_mfma_f64_16x16x4 (2 x 2 tiles of 16, the gradient riding in the padding
// column 31); lane i factorises row i of H in registers (right-looking Cholesky, multipliers broadcast with
// v_readlane, the padding rows set to the identity so no loop needs a data-dependent guard); the solves on the
// lanes; wave sums as xor butterflies (the same bits on every lane, so every branch is uniform); the full Newton
// step once Armijo's decrease sinks under the objective's rounding; two waves per SIMD (19 KB of LDS: the rows staged
// as their fp32 values, 64 at a time).  The 1023-coalition sweep (config #2): 242 ms (one 256-thread workgroup per
// coalition, serial factorisation) -> 1.7 ms (three 0.56 ms rounds; profiles/r05_titanic_kernel_stats{,_rounds,
// _occ2}.csv; per-phase times: scripts/lr_phases.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "keyed.h"
#include "mplc_hip.h"

// Phase-timing hooks (scripts/lr_phases.py builds a timing copy of this file that defines them); no-ops here.
#ifndef LR_PHASE
#define LR_PHASE(i) ((void)0)
#endif

namespace {

constexpr int LR_THREADS = 64;   // one wave per fit (a fit kernel work item) / per coalition (averages)
constexpr int LR_MAXF = 32;      // D = n_features + 1 unknowns (coef | intercept) supported
constexpr int LR_MAXP = 64;      // partners per coalition
constexpr int LR_NMAX = 64;      // rows staged in LDS at a time (config #2's fits: 56-57 rows; larger fits stream)
constexpr int LR_XS = LR_MAXF + 1;  // staged row stride in floats (odd: per-lane row reads 2-way banked)
constexpr int LR_LS = LR_MAXF + 1;  // row stride of the Hessian / factor in LDS: lane li's row reads 2-way banked
typedef double f64x4 __attribute__((ext_vector_type(4)));

// 18.5 KB: two one-wave workgroups per SIMD fit a CU's 160 KB of LDS
struct Shared {
  double w[LR_MAXF];       // current Newton iterate (entries >= D stay 0)
  double trial[LR_MAXF];   // line-search trial point (entries >= D stay 0)
  double L[LR_MAXF * LR_LS];  // the Hessian's tiles, then the Cholesky factor (row-major, stride LR_LS)
  double hv[LR_NMAX];      // s (1 - s) of the staged rows, s = sigma(-y z)
  double sv[LR_NMAX];      // -y s
  float xs[LR_NMAX * LR_XS];  // staged rows [i][k] (the data's fp32): features k < F, 1 at k = F (intercept), 0 after
  float ys[LR_NMAX];       // +-1
  int rid[LR_NMAX];
};

// Sum over the wave: an xor butterfly, so every lane ends with the same bits (each level adds the same two
// partial sums on both partner lanes: a + b and b + a).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return v;
}

// lane l's value of v, for every lane (v_readlane into scalar registers; l uniform)
__device__ __forceinline__ double readlane(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// rows: global row ids of this fit are rowsel(i), i < n (row = rows[off + perm...]); X row-major [N][F]
struct RowSel {
  const int32_t* rows;
  int off, n_p, start, count;  // minibatch = permuted positions [start, start+count) of the partner's rows
  uint64_t perm_key;
  bool permute;
  __device__ int row(int i) const {
    const int pos = permute ? (int)keyed_perm(perm_key, (uint32_t)n_p, (uint32_t)(start + i)) : start + i;
    return rows[off + pos];
  }
};

// rows [c0, c0 + cn) of the fit into LDS as the data's fp32 (widened to fp64 exactly where read), the intercept's
// column of ones and zero padding appended, labels as +-1
__device__ void stage_rows(const RowSel& rs, int c0, int cn, const float* X, const float* Y, int F, Shared& sh) {
  const int lane = threadIdx.x;
  for (int i = lane; i < cn; i += LR_THREADS) {
    const int r = rs.row(c0 + i);
    sh.rid[i] = r;
    sh.ys[i] = Y[r] > 0.5f ? 1.0f : -1.0f;
  }
  __syncthreads();
  // (row, column) pairs over the lanes, 32 columns a row: no per-column address table for the compiler to keep
  // live across the kernel (an unrolled per-lane row loop held 32 offsets and 32 masks in registers)
#pragma unroll 4
  for (int e = lane; e < cn * LR_MAXF; e += LR_THREADS) {
    const int i = e >> 5, k = e & (LR_MAXF - 1);
    const float v = X[(int64_t)sh.rid[i] * F + min(k, F - 1)];
    sh.xs[i * LR_XS + k] = k < F ? v : (k == F ? 1.0f : 0.0f);
  }
  __syncthreads();
}

// w . [x | 1] over a staged row (w's entries >= D are 0, as are the row's)
__device__ __forceinline__ double row_z(const double* w, const float* xr) {
  double z = 0.0;
#pragma unroll
  for (int k = 0; k < LR_MAXF; ++k) z += w[k] * (double)xr[k];
  return z;
}

// sum_i log(1 + exp(-y_i z_i)) + 0.5 ||coef||^2 over the fit's rows (staged already when resident)
__device__ double objective(const double* w, const RowSel& rs, bool resident, const float* X, const float* Y, int F,
                            Shared& sh) {
  const int lane = threadIdx.x;
  double part = 0.0;
  for (int c0 = 0; c0 < rs.count; c0 += LR_NMAX) {
    const int cn = min(LR_NMAX, rs.count - c0);
    if (!resident) stage_rows(rs, c0, cn, X, Y, F, sh);
    for (int i = lane; i < cn; i += LR_THREADS) {
      const double t = -(double)sh.ys[i] * row_z(w, sh.xs + i * LR_XS);
      part += t > 0 ? t + log1p(exp(-t)) : log1p(exp(t));
    }
    if (!resident) __syncthreads();
  }
  const double reg = (lane < F) ? w[lane] * w[lane] : 0.0;
  return wave_sum(part) + 0.5 * wave_sum(reg);
}

// Exact L2-logistic fit (damped Newton with Armijo backtracking) into sh.w, warm-started from sh.w.
// Lane i (< D) owns row i of the Hessian in registers (h[k], k < LR_MAXF: fully unrolled, so every index is a
// compile-time constant), factorises it in place (right-looking Cholesky, column j's multipliers broadcast with
// v_readlane) and holds entry i of the gradient and of the Newton step.
__device__ void newton_fit(const RowSel& rs, const float* X, const float* Y, int F, Shared& sh) {
  const int lane = threadIdx.x;
  const int li = lane & (LR_MAXF - 1);  // the Hessian row this lane factorises (lanes >= 32 mirror lanes < 32)
  const int D = F + 1;
  const bool resident = rs.count <= LR_NMAX;
  if (resident) stage_rows(rs, 0, rs.count, X, Y, F, sh);
  LR_PHASE(9);
  double f0 = objective(sh.w, rs, resident, X, Y, F, sh);
  LR_PHASE(1);
  const int kk = lane >> 4, idx = lane & 15;  // the f64 MFMA's operand lane map: A[idx][kk], B[kk][idx]
  for (int it = 0; it < 100; ++it) {
    // H = sum_r x_r (h_r x_r)^T on the matrix cores: 32 x 32 as 2 x 2 tiles of v_mfma_f64_16x16x4, four rows per
    // step.  B's column 31 (the padding column: D <= 31) carries sv_r instead, so that column of the product is
    // the gradient's data term sum_r sv_r x_r.
    f64x4 t00 = {0.0, 0.0, 0.0, 0.0}, t01 = t00, t10 = t00, t11 = t00;
    for (int c0 = 0; c0 < rs.count; c0 += LR_NMAX) {
      const int cn = min(LR_NMAX, rs.count - c0);
      const int cn4 = (cn + 3) & ~3;
      if (!resident) stage_rows(rs, c0, cn, X, Y, F, sh);
      for (int i = lane; i < cn4; i += LR_THREADS) {  // per row: s = sigma(-y z), s (1 - s); 0 on the padding
        double sv = 0.0, hv = 0.0;
        if (i < cn) {
          const double yy = (double)sh.ys[i];
          const double sg = 1.0 / (1.0 + exp(yy * row_z(sh.w, sh.xs + i * LR_XS)));
          sv = -yy * sg;
          hv = sg * (1.0 - sg);
        }
        sh.sv[i] = sv;
        sh.hv[i] = hv;
      }
      __syncthreads();
      for (int r0 = 0; r0 < cn; r0 += 4) {
        const int r = r0 + kk;
        const bool ok = r < cn;
        const double a0 = ok ? (double)sh.xs[r * LR_XS + idx] : 0.0;
        const double a1 = ok ? (double)sh.xs[r * LR_XS + 16 + idx] : 0.0;
        const double hr = sh.hv[r];
        const double b0 = hr * a0;
        const double b1 = idx == 15 ? sh.sv[r] : hr * a1;
        t00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, t00, 0, 0, 0);
        t01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, t01, 0, 0, 0);
        t10 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, t10, 0, 0, 0);
        t11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, t11, 0, 0, 0);
      }
      __syncthreads();
    }
    // tiles -> LDS (result v of a lane: row kk + 4 v, column idx) -> lane li takes row li
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = kk + 4 * v;
      sh.L[row * LR_LS + idx] = t00[v];
      sh.L[row * LR_LS + 16 + idx] = t01[v];
      sh.L[(16 + row) * LR_LS + idx] = t10[v];
      sh.L[(16 + row) * LR_LS + 16 + idx] = t11[v];
    }
    __syncthreads();
    double h[LR_MAXF];
#pragma unroll
    for (int k = 0; k < LR_MAXF - 1; ++k) h[k] = sh.L[li * LR_LS + k];
    h[LR_MAXF - 1] = 0.0;
    const double gdata = sh.L[li * LR_LS + LR_MAXF - 1];
    __syncthreads();
    const double gk = li < D ? gdata + (li < F ? sh.w[li] : 0.0) : 0.0;
    LR_PHASE(2);
    if (wave_max(fabs(gk)) < 1e-10) break;
    LR_PHASE(3);
    // the L2 term on the coefficients, and the identity on the padding rows li >= D: the factor of [H 0; 0 I] is
    // [L 0; 0 I] exactly (every update of a padding entry subtracts an exact 0), so every loop below runs over all
    // LR_MAXF columns with no data-dependent guard and no exec-mask branches
#pragma unroll
    for (int k = 0; k < LR_MAXF; ++k) h[k] += (k == li && (li < F || li >= D)) ? 1.0 : 0.0;
    // Cholesky H = L L^T, right-looking: column j's multipliers l_ij = h[j] / l_jj on the lanes, then the trailing
    // update h[k] -= l_ij l_kj (on every lane: the entries above the diagonal are never read).  The diagonal keeps
    // 1 / l_jj, the only form the solves use.
#pragma unroll
    for (int j = 0; j < LR_MAXF; ++j) {
      const double rinv = 1.0 / sqrt(readlane(h[j], j));
      h[j] = (li == j) ? rinv : h[j] * rinv;
#pragma unroll
      for (int k = j + 1; k < LR_MAXF; ++k) h[k] -= h[j] * readlane(h[j], k);
    }
    LR_PHASE(4);
    // L y = g (forward, L's column q in registers), L^T d = y (backward, L's row q from LDS)
    if (lane < LR_MAXF) {
#pragma unroll
      for (int k = 0; k < LR_MAXF; ++k) sh.L[lane * LR_LS + k] = h[k];
    }
    double b = gk;
#pragma unroll
    for (int q = 0; q < LR_MAXF; ++q) {
      const double yq = readlane(b, q) * readlane(h[q], q);
      const double nb = b - h[q] * yq;
      b = li > q ? nb : (li == q ? yq : b);
    }
    __syncthreads();
#pragma unroll
    for (int q = LR_MAXF - 1; q >= 0; --q) {
      const double dq = readlane(b, q) * sh.L[q * LR_LS + q];
      const double nb = b - sh.L[q * LR_LS + li] * dq;
      b = li < q ? nb : (li == q ? dq : b);
    }
    const double dk = li < D ? b : 0.0;
    LR_PHASE(5);
    const double gd = wave_sum(lane < 32 ? gk * dk : 0.0);
    // backtracking line search on the objective; the accepted value is the next iteration's f0.  Near the optimum
    // the Armijo decrease 1e-4 t g.d sinks under the rounding of the objective's row sum (~1e-14 |f|): no step
    // could pass, and such fits used to spend their 100 iterations x 40 halvings stuck at |g| ~ 1e-9.  Once g.d <=
    // 1e-10 |f| the full Newton step is taken (the quadratic-convergence region: |g| ~ 1e-5 for this problem).
    const bool full = gd <= 1e-10 * fmax(1.0, fabs(f0));
    double t = 1.0, f1 = f0;
    for (int ls = 0; ls < 40; ++ls) {
      if (lane < D) sh.trial[lane] = sh.w[lane] - t * dk;
      __syncthreads();
      f1 = objective(sh.trial, rs, resident, X, Y, F, sh);
      if (full || f1 <= f0 - 1e-4 * t * gd) break;
      t *= 0.5;
    }
    if (lane < D) sh.w[lane] = sh.trial[lane];
    f0 = f1;
    LR_PHASE(6);
    __syncthreads();
  }
}

__device__ __forceinline__ double row_z_global(const double* w, const float* xr, int F) {
  double z = w[F];
  for (int k = 0; k < F; ++k) z += w[k] * (double)xr[k];
  return z;
}

__device__ int count_correct(const double* w, const float* X, const float* Y, int n, int F) {
  double c = 0.0;
  for (int i = threadIdx.x; i < n; i += LR_THREADS)
    c += ((row_z_global(w, X + (int64_t)i * F, F) > 0.0) == (Y[i] > 0.5f)) ? 1.0 : 0.0;
  return (int)(wave_sum(c) + 0.5);
}

__device__ int count_correct_rows(const double* w, const RowSel& rs, const float* X, const float* Y, int F) {
  double c = 0.0;
  for (int i = threadIdx.x; i < rs.count; i += LR_THREADS) {
    const int r = rs.row(i);
    c += ((row_z_global(w, X + (int64_t)r * F, F) > 0.0) == (Y[r] > 0.5f)) ? 1.0 : 0.0;
  }
  return (int)(wave_sum(c) + 0.5);
}

// Titanic.LogisticRegression.evaluate (mplc/dataset.py:343-351): [log_loss(y, predict(x)), accuracy] on hard
// 0/1 predictions, from the count of correct predictions.  log_loss clips the 0/1 "probabilities" at the
// machine epsilon of predict()'s dtype (sklearn's eps="auto", the version the reference runs with here and
// that tests/golden/lr_history.json pins; sklearn 0.22 clipped at 1e-15): a partner model fitted on the
// float32 labels predicts float32 classes (eps 2^-23), the aggregated model, built with int classes, float64
// ones (eps 2^-52)
constexpr double EPS_FITTED = 1.1920928955078125e-07, EPS_GLOBAL = 2.220446049250313e-16;
__device__ void lr_metrics(int n_correct, int n, double& loss, double& acc, double eps) {
  loss = ((double)(n - n_correct) * (-log(eps)) + (double)n_correct * (-log(1.0 - eps))) / (double)n;
  acc = (double)n_correct / (double)n;
}

// ------------------------------------------------------------------------------------------------
// The FedAvg rounds as launches over all coalitions at once.  One coalition's rounds are a chain (each partner
// fit warm-starts from the previous round's average), but within a round its |S| fits are independent: every
// round is one launch whose waves take (coalition, partner) fits from a work queue, then one launch averages each
// coalition's fits in partner order.  The sweep's length is then its total fit work over the machine plus one
// round's longest fit per round, not its longest coalition's E x M x |S| chain of fits.
// ------------------------------------------------------------------------------------------------
constexpr int LR_HAVE = 1, LR_STOPPED = 2;  // coalition state bits: fitted global model / early-stopped

struct LrJob {
  const float* X;
  const float* Y;
  int F, M, C, epochs, early_stopping, n_val, n_test;
  const int32_t* rows;
  const int32_t* rows_off;
  const int32_t* n_rows;
  const int32_t* splits;
  const uint64_t* masks;
  const uint64_t* keys;
  const double* agg_w;
  const double* agg_scale;
  const float* Xv;
  const float* Yv;
  const float* Xt;
  const float* Yt;
  double* hist;
  int64_t hist_stride;
  // workspace (one stream-ordered allocation per call)
  double* theta;     // [C][LR_MAXF] the coalition's global model
  double* wpart;     // [C][LR_MAXP][LR_MAXF] this round's partner fits
  double* val_hist;  // [C][64] early stopping: val loss at each epoch's start
  int32_t* item_off;  // [C + 1] first fit item of coalition c (exclusive prefix of |S|)
  int32_t* state;     // [C] LR_HAVE | LR_STOPPED
  int32_t* done;      // [C] epochs run
  uint32_t* counters;  // [epochs * M] work-queue heads, one per round
};

__device__ __forceinline__ double* hist_row(const LrJob& j, int c, int e, int m) {
  return j.hist + (int64_t)c * j.hist_stride + (int64_t)(e * j.M + m) * (2 + 4 * LR_MAXP);
}

// one block of 1024 threads: item offsets (exclusive prefix of the coalition sizes), state, queue heads
__global__ __launch_bounds__(1024) void lr_prep_kernel(LrJob j) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (j.C + 1023) / 1024;
  const int c0 = min(j.C, t * per), c1 = min(j.C, c0 + per);
  int s = 0;
  for (int c = c0; c < c1; ++c) s += __popcll(j.masks[c]);
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan of the 1024 chunk sums
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = t ? part[t - 1] : 0;
  for (int c = c0; c < c1; ++c) {
    j.item_off[c] = run;
    run += __popcll(j.masks[c]);
  }
  if (t == 1023) j.item_off[j.C] = part[1023];
  for (int c = t; c < j.C; c += 1024) {
    j.state[c] = 0;
    j.done[c] = j.epochs;
    j.val_hist[(int64_t)c * 64] = 0.0;  // epoch 0 starts unfitted: evaluate -> [0, 0]
  }
  for (int i = t; i < j.epochs * j.M; i += 1024) j.counters[i] = 0u;
  if (j.hist && t < j.C) {  // round (0, 0) starts unfitted; a singleton has no collective entries
    if (__popcll(j.masks[t]) > 1) hist_row(j, t, 0, 0)[0] = hist_row(j, t, 0, 0)[1] = 0.0;
  }
}

// round (e, m): waves take (coalition, partner) fits from the round's queue until it is empty
__global__ __launch_bounds__(LR_THREADS, 2) void lr_fit_kernel(LrJob j, int e, int m) {
  __shared__ Shared sh;
  const int lane = threadIdx.x;
  const int D = j.F + 1;
  const int total = j.item_off[j.C];
  uint32_t* head = j.counters + e * j.M + m;
  if (lane < LR_MAXF) { sh.w[lane] = 0.0; sh.trial[lane] = 0.0; }
  __syncthreads();
  LR_PHASE(-1);
  for (;;) {
    int got = 0;
    if (lane == 0) got = (int)atomicAdd(head, 1u);
    const int item = __shfl(got, 0);
    if (item >= total) break;  // every wave reaches this: the queue only grows past `total`
    int lo = 0, hi = j.C - 1;  // the coalition: last c with item_off[c] <= item
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (j.item_off[mid] <= item) lo = mid;
      else hi = mid - 1;
    }
    const int c = lo, pi = item - j.item_off[c];
    const uint64_t mask = j.masks[c];
    const int P = __popcll(mask);
    const int st = j.state[c];
    if (pi >= P || (st & LR_STOPPED) || (P == 1 && (e | m))) continue;  // a singleton fits once, in round (0, 0)
    uint64_t rem = mask;
    for (int k = 0; k < pi; ++k) rem &= rem - 1;
    const int p = __builtin_ctzll(rem);
    // singleton: one fit on the partner's full data (E refits of the same rows reach the same optimum)
    const int* sp = j.splits + p * (j.M + 1);
    const RowSel rs = P == 1 ? RowSel{j.rows, j.rows_off[p], j.n_rows[p], 0, j.n_rows[p], 0ull, false}
                             : RowSel{j.rows, j.rows_off[p], j.n_rows[p], sp[m], sp[m + 1] - sp[m],
                                      subkey(j.keys[(int64_t)c * LR_MAXP + pi], 0x10000u + (uint32_t)e, 0u), j.M > 1};
    if (lane < D) sh.w[lane] = (st & LR_HAVE) ? j.theta[(int64_t)c * LR_MAXF + lane] : 0.0;  // warm start
    __syncthreads();
    LR_PHASE(10);
    newton_fit(rs, j.X, j.Y, j.F, sh);
    if (lane < D) j.wpart[((int64_t)c * LR_MAXP + pi) * LR_MAXF + lane] = sh.w[lane];
    if (j.hist) {  // the partner's fit history: [loss, accuracy] on its rows, then on val (a singleton: round (0, 0))
      const int ct = count_correct_rows(sh.w, rs, j.X, j.Y, j.F);
      const int cv = count_correct(sh.w, j.Xv, j.Yv, j.n_val, j.F);
      if (lane == 0) {
        double* h = hist_row(j, c, e, m) + 2 + 4 * pi;
        lr_metrics(ct, rs.count, h[0], h[1], EPS_FITTED);
        lr_metrics(cv, j.n_val, h[2], h[3], EPS_FITTED);
      }
    }
    __syncthreads();
  }
  LR_PHASE(7);
}

// round (e, m), one wave per coalition: np.average of the partner fits (multiply, then sum in partner order, fp64);
// at an epoch's end the early-stopping test (mplc/multi_partner_learning.py:177-193: round-0 val loss of epoch e
// against e - 10), then the next round's start values from the new global model
__global__ __launch_bounds__(LR_THREADS) void lr_avg_kernel(LrJob j, int e, int m) {
  __shared__ double th[LR_MAXF];
  const int c = blockIdx.x, lane = threadIdx.x;
  const int D = j.F + 1;
  const int st = j.state[c];
  if (st & LR_STOPPED) return;
  const int P = __popcll(j.masks[c]);
  double* theta = j.theta + (int64_t)c * LR_MAXF;
  const double* wp = j.wpart + (int64_t)c * LR_MAXP * LR_MAXF;
  if (P == 1) {
    if (e == 0 && m == 0) {
      if (lane < D) theta[lane] = wp[lane];
      if (lane == 0) j.state[c] = LR_HAVE;
    }
    return;
  }
  if (lane < LR_MAXF) {
    // numpy multiplies, then adds: no fused multiply-add here (tests/test_lr.py pins it bit for bit)
#pragma clang fp contract(off)
    double acc = 0.0;
    if (lane < D) {
      for (int pi = 0; pi < P; ++pi) {
        const double prod = wp[pi * LR_MAXF + lane] * j.agg_w[(int64_t)c * LR_MAXP + pi];
        acc = (pi == 0) ? prod : acc + prod;
      }
      acc = acc / j.agg_scale[c];
      theta[lane] = acc;
    }
    th[lane] = acc;
  }
  __syncthreads();
  int state = LR_HAVE;
  double* vh = j.val_hist + (int64_t)c * 64;
  const bool es = j.early_stopping && j.epochs > 10;
  if (es && m == j.M - 1 && e >= 10 && e < 64 && vh[e] > vh[e - 10]) {
    state |= LR_STOPPED;
    if (lane == 0) j.done[c] = e + 1;
  }
  const int en = (m + 1 < j.M) ? e : e + 1, mn = (m + 1 < j.M) ? m + 1 : 0;  // the next round
  if (!(state & LR_STOPPED) && en < j.epochs) {
    if (es && mn == 0 && en < 64) {  // log_loss(y, predict(x)) on hard 0/1 predictions, sklearn eps 1e-15
      const int cv = count_correct(th, j.Xv, j.Yv, j.n_val, j.F);
      const double eps = 1e-15;
      if (lane == 0)
        vh[en] = (double)(j.n_val - cv) * (-log(eps)) / (double)j.n_val + (double)cv * (-log(1.0 - eps)) / (double)j.n_val;
    }
    if (j.hist) {  // the round-start collective model on val (eval_and_log_model_val_perf)
      const int cv = count_correct(th, j.Xv, j.Yv, j.n_val, j.F);
      if (lane == 0) {
        double* h = hist_row(j, c, en, mn);
        lr_metrics(cv, j.n_val, h[0], h[1], EPS_GLOBAL);
      }
    }
  }
  if (lane == 0) j.state[c] = state;
}

// the final model of every coalition: theta_out, test hits, epochs run
__global__ __launch_bounds__(LR_THREADS) void lr_final_kernel(LrJob j, int32_t* __restrict__ correct,
                                                              int32_t* __restrict__ epochs_done,
                                                              double* __restrict__ theta_out) {
  __shared__ double th[LR_MAXF];
  const int c = blockIdx.x, lane = threadIdx.x;
  const int D = j.F + 1;
  if (lane < LR_MAXF) th[lane] = lane < D ? j.theta[(int64_t)c * LR_MAXF + lane] : 0.0;
  __syncthreads();
  if (lane < D) theta_out[(int64_t)c * D + lane] = th[lane];
  const int cc = count_correct(th, j.Xt, j.Yt, j.n_test, j.F);
  if (lane == 0) {
    correct[c] = cc;
    epochs_done[c] = j.done[c];
  }
}

}  // namespace

extern "C" int mplc_lr_fedavg(const float* x, const float* y, int n_features, const int32_t* rows,
                              const int32_t* rows_off, const int32_t* n_rows, const int32_t* splits,
                              int minibatch_count, const uint64_t* masks, const uint64_t* keys, const double* agg_w,
                              const double* agg_scale, int n_coalitions, int epochs, int early_stopping,
                              const float* x_val, const float* y_val, int n_val, const float* x_test,
                              const float* y_test, int n_test, int32_t* correct, int32_t* epochs_done,
                              double* theta_out, double* hist, int64_t hist_stride, void* stream) {
  if (!x || !y || !rows || !rows_off || !n_rows || !splits || !masks || !keys || !agg_w || !agg_scale || !x_test ||
      !y_test || !correct || !epochs_done || !theta_out)
    return MPLC_E_ARG;
  if (hist && (!x_val || !y_val || n_val < 1 || hist_stride < (int64_t)epochs * minibatch_count * (2 + 4 * LR_MAXP)))
    return MPLC_E_ARG;
  // D = n_features + 1 unknowns <= LR_MAXF - 1 (the Hessian product's last column carries the gradient)
  if (n_features < 1 || n_features + 2 > LR_MAXF || n_coalitions < 1 || minibatch_count < 1 || epochs < 1 ||
      n_test < 1)
    return MPLC_E_ARG;
  if (early_stopping && (!x_val || !y_val || n_val < 1)) return MPLC_E_ARG;
  if (hist && n_coalitions > 1024) return MPLC_E_ARG;  // the history is for single coalitions
  const int64_t C = n_coalitions, R = (int64_t)epochs * minibatch_count;
  if (R > (1 << 20)) return MPLC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const size_t b_theta = (size_t)C * LR_MAXF * 8, b_wpart = (size_t)C * LR_MAXP * LR_MAXF * 8,
               b_vh = (size_t)C * 64 * 8, b_off = (size_t)(C + 1) * 4, b_st = (size_t)C * 4, b_ctr = (size_t)R * 4;
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t bytes = up(b_theta) + up(b_wpart) + up(b_vh) + up(b_off) + 2 * up(b_st) + up(b_ctr);
  char* ws = nullptr;
  hipError_t err = hipMallocAsync((void**)&ws, bytes, s);
  if (err != hipSuccess) return (int)err;
  LrJob j{};
  j.X = x, j.Y = y, j.F = n_features, j.M = minibatch_count, j.C = n_coalitions, j.epochs = epochs;
  j.early_stopping = early_stopping, j.n_val = n_val, j.n_test = n_test;
  j.rows = rows, j.rows_off = rows_off, j.n_rows = n_rows, j.splits = splits, j.masks = masks, j.keys = keys;
  j.agg_w = agg_w, j.agg_scale = agg_scale, j.Xv = x_val, j.Yv = y_val, j.Xt = x_test, j.Yt = y_test;
  j.hist = hist, j.hist_stride = hist_stride;
  char* q = ws;
  j.theta = (double*)q, q += up(b_theta);
  j.wpart = (double*)q, q += up(b_wpart);
  j.val_hist = (double*)q, q += up(b_vh);
  j.item_off = (int32_t*)q, q += up(b_off);
  j.state = (int32_t*)q, q += up(b_st);
  j.done = (int32_t*)q, q += up(b_st);
  j.counters = (uint32_t*)q;
  lr_prep_kernel<<<1, 1024, 0, s>>>(j);
  // the fit launches' persistent grid: 8 one-wave workgroups per CU (2 per SIMD) on the 256 CUs
  const int grid = (int)std::min<int64_t>(C * LR_MAXP, 2048);
  for (int e = 0; e < epochs; ++e)
    for (int m = 0; m < minibatch_count; ++m) {
      lr_fit_kernel<<<grid, LR_THREADS, 0, s>>>(j, e, m);
      lr_avg_kernel<<<n_coalitions, LR_THREADS, 0, s>>>(j, e, m);
    }
  lr_final_kernel<<<n_coalitions, LR_THREADS, 0, s>>>(j, correct, epochs_done, theta_out);
  err = hipGetLastError();
  const hipError_t ferr = hipFreeAsync(ws, s);
  if (err != hipSuccess) return (int)err;
  return ferr == hipSuccess ? MPLC_OK : (int)ferr;
}
