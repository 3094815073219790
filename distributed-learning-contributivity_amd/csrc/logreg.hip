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
// One workgroup = one coalition; every fit is solved EXACTLY (damped Newton in fp64, gradient < 1e-10),
// the optimum of the strictly convex problem sklearn approximates to tol 1e-4.
// Work is tiny (28 unknowns, tens of rows): latency-bound; the point is doing all coalitions in ONE launch and
// keeping each fit's dependent chain short.  Round 5: one wave per coalition.  The fit's rows are staged in LDS
// once per fit as fp64 with the intercept's column of ones (lanes over rows, each row's loads issued together); the
// Hessian X^T diag(h) X and the gradient come from v_mfma_f64_16x16x4 (2 x 2 tiles of 16, the gradient riding in
// the padding column 31); lane i factorises row i of H in registers (right-looking Cholesky, multipliers broadcast
// with v_readlane, the padding rows set to the identity so no loop needs a data-dependent guard); the solves run on
// the lanes; wave sums are xor butterflies (the same bits on every lane, so every branch is uniform); the line
// search's accepted objective is the next iteration's start value.  The 1023-coalition sweep (config #2):
// 242 ms (one 256-thread workgroup, serial single-thread factorisation) -> 14.7 ms
// (profiles/r05_titanic_kernel_stats{,_mfma}.csv; per-phase times: scripts/lr_phases.py, profiles/r05_lr_phases.json).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "keyed.h"
#include "mplc_hip.h"

// Phase-timing hooks (scripts/lr_phases.py builds a timing copy of this file that defines them); no-ops here.
#ifndef LR_PHASE
#define LR_PHASE(i) ((void)0)
#endif

namespace {

constexpr int LR_THREADS = 64;   // one wave per coalition
constexpr int LR_MAXF = 32;      // D = n_features + 1 unknowns (coef | intercept) supported
constexpr int LR_MAXP = 64;      // partners per coalition
constexpr int LR_NMAX = 96;      // rows staged in LDS at a time (a whole Titanic fit: <= 71 rows)
constexpr int LR_XS = LR_MAXF + 2;  // staged row stride in doubles: 16-byte aligned rows, 4-way banked per-lane reads
constexpr int LR_LS = LR_MAXF + 1;  // row stride of the Hessian / factor in LDS: lane li's row reads 2-way banked
typedef double f64x4 __attribute__((ext_vector_type(4)));

struct Shared {
  double theta[LR_MAXF];
  double w[LR_MAXF];       // current Newton iterate (entries >= D stay 0)
  double trial[LR_MAXF];   // line-search trial point (entries >= D stay 0)
  double acc[LR_MAXF];     // FedAvg accumulator
  double L[LR_MAXF * LR_LS];  // the Hessian's tiles, then the Cholesky factor (row-major, stride LR_LS)
  double hv[LR_NMAX];      // s (1 - s) of the staged rows, s = sigma(-y z)
  double sv[LR_NMAX];      // -y s
  double xs[LR_NMAX * LR_XS];  // staged rows [i][k]: features k < F, 1 at k = F (the intercept's column), 0 after
  double ys[LR_NMAX];      // +-1
  double val_hist[64];
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

// rows [c0, c0 + cn) of the fit into LDS as fp64 (exact widening of the fp32 data), the intercept's column of ones
// and zero padding appended, labels as +-1
__device__ void stage_rows(const RowSel& rs, int c0, int cn, const float* X, const float* Y, int F, Shared& sh) {
  // lanes over rows: each lane gathers its row's F features with independent loads (one memory latency per row,
  // not one per feature)
  for (int i = threadIdx.x; i < cn; i += LR_THREADS) {
    const int r = rs.row(c0 + i);
    sh.ys[i] = Y[r] > 0.5f ? 1.0 : -1.0;
    const float* xr = X + (int64_t)r * F;
    double* dst = sh.xs + i * LR_XS;
    float v[LR_MAXF];
#pragma unroll
    for (int k = 0; k < LR_MAXF; ++k) v[k] = xr[min(k, F - 1)];  // unconditional: the loads issue back to back
#pragma unroll
    for (int k = 0; k < LR_MAXF; ++k) dst[k] = k < F ? (double)v[k] : (k == F ? 1.0 : 0.0);
  }
  __syncthreads();
}

// w . [x | 1] over a staged row (w's entries >= D are 0, as are the row's)
__device__ __forceinline__ double row_z(const double* w, const double* xr) {
  double z = 0.0;
#pragma unroll
  for (int k = 0; k < LR_MAXF; ++k) z += w[k] * xr[k];
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
      const double t = -sh.ys[i] * row_z(w, sh.xs + i * LR_XS);
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
          const double yy = sh.ys[i];
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
        const double a0 = ok ? sh.xs[r * LR_XS + idx] : 0.0;
        const double a1 = ok ? sh.xs[r * LR_XS + 16 + idx] : 0.0;
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
    // backtracking line search on the objective; the accepted value is the next iteration's f0
    double t = 1.0, f1 = f0;
    for (int ls = 0; ls < 40; ++ls) {
      if (lane < D) sh.trial[lane] = sh.w[lane] - t * dk;
      __syncthreads();
      f1 = objective(sh.trial, rs, resident, X, Y, F, sh);
      if (f1 <= f0 - 1e-4 * t * gd) break;
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

__global__ __launch_bounds__(LR_THREADS) void lr_fedavg_kernel(
    const float* __restrict__ X, const float* __restrict__ Y, int F, const int32_t* __restrict__ rows,
    const int32_t* __restrict__ rows_off, const int32_t* __restrict__ n_rows, const int32_t* __restrict__ splits,
    int M, const uint64_t* __restrict__ masks, const uint64_t* __restrict__ keys, const double* __restrict__ agg_w,
    const double* __restrict__ agg_scale, int epochs, int early_stopping, const float* __restrict__ Xv,
    const float* __restrict__ Yv, int n_val, const float* __restrict__ Xt, const float* __restrict__ Yt, int n_test,
    int32_t* __restrict__ correct, int32_t* __restrict__ epochs_done, double* __restrict__ theta_out,
    double* __restrict__ hist, int64_t hist_stride) {
  __shared__ Shared sh;
  LR_PHASE(-1);
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  const int D = F + 1;
  const uint64_t mask = masks[c];
  const int P = __popcll(mask);  // partners in bit order (no per-lane array: it would live in scratch memory)
  if (tid < LR_MAXF) { sh.theta[tid] = 0.0; sh.w[tid] = 0.0; sh.trial[tid] = 0.0; }
  __syncthreads();
  int done_epochs = epochs;
  if (P == 1) {
    // singleton: one fit on the partner's full data (E refits of the same rows reach the same optimum)
    const int p = __builtin_ctzll(mask);
    RowSel rs{rows, rows_off[p], n_rows[p], 0, n_rows[p], 0ull, false};
    newton_fit(rs, X, Y, F, sh);
    if (tid < D) theta_out[(int64_t)c * D + tid] = sh.w[tid];
    __syncthreads();
    if (hist) {  // SinglePartnerLearning logs its fit at [0, 0]
      const int ct = count_correct_rows(sh.w, rs, X, Y, F);
      const int cv = count_correct(sh.w, Xv, Yv, n_val, F);
      if (tid == 0) {
        double* h = hist + (int64_t)c * hist_stride + 2;
        lr_metrics(ct, rs.count, h[0], h[1], EPS_FITTED);
        lr_metrics(cv, n_val, h[2], h[3], EPS_FITTED);
      }
    }
  } else {
    double* val_hist = sh.val_hist;
    int have = 0;  // the initial model is unfitted (coef_ None): evaluate -> [0, 0]
    for (int e = 0; e < epochs; ++e) {
      if (early_stopping && epochs > 10 && e < 64) {
        double vl = 0.0;
        if (have) {  // log_loss(y, predict(x)) on hard 0/1 predictions, sklearn eps 1e-15
          const int cv = count_correct(sh.theta, Xv, Yv, n_val, F);
          const double eps = 1e-15;
          vl = (double)(n_val - cv) * (-log(eps)) / (double)n_val + (double)cv * (-log(1.0 - eps)) / (double)n_val;
        }
        if (tid == 0) val_hist[e] = vl;
        __syncthreads();
      }
      for (int m = 0; m < M; ++m) {
        double* hrow = hist ? hist + (int64_t)c * hist_stride + (int64_t)(e * M + m) * (2 + 4 * LR_MAXP) : nullptr;
        if (hrow) {  // the round-start collective model on val (eval_and_log_model_val_perf); unfitted: [0, 0]
          const int cv = have ? count_correct(sh.theta, Xv, Yv, n_val, F) : 0;
          if (tid == 0) {
            if (have) lr_metrics(cv, n_val, hrow[0], hrow[1], EPS_GLOBAL);
            else hrow[0] = hrow[1] = 0.0;
          }
        }
        if (tid < D) sh.acc[tid] = 0.0;
        __syncthreads();
        uint64_t rem = mask;
        for (int pi = 0; pi < P; ++pi, rem &= rem - 1) {
          const int p = __builtin_ctzll(rem);
          const int* sp = splits + p * (M + 1);
          RowSel rs{rows, rows_off[p], n_rows[p], sp[m], sp[m + 1] - sp[m],
                    subkey(keys[(int64_t)c * LR_MAXP + pi], 0x10000u + (uint32_t)e, 0u), M > 1};
          if (tid < D) sh.w[tid] = have ? sh.theta[tid] : 0.0;  // warm start from the global model
          __syncthreads();
          LR_PHASE(10);
          newton_fit(rs, X, Y, F, sh);
          if (hrow) {  // the partner's fit history: [loss, accuracy] on its minibatch, then on val
            const int ct = count_correct_rows(sh.w, rs, X, Y, F);
            const int cv = count_correct(sh.w, Xv, Yv, n_val, F);
            if (tid == 0) {
              double* h = hrow + 2 + 4 * pi;
              lr_metrics(ct, rs.count, h[0], h[1], EPS_FITTED);
              lr_metrics(cv, n_val, h[2], h[3], EPS_FITTED);
            }
          }
          // np.average: multiply then sum in partner order (float64)
          if (tid < D) {
            const double prod = sh.w[tid] * agg_w[(int64_t)c * LR_MAXP + pi];
            sh.acc[tid] = (pi == 0) ? prod : sh.acc[tid] + prod;
          }
          __syncthreads();
        }
        if (tid < D) sh.theta[tid] = sh.acc[tid] / agg_scale[c];
        LR_PHASE(8);
        have = 1;
        __syncthreads();
      }
      if (early_stopping && epochs > 10 && e >= 10 && e < 64 && val_hist[e] > val_hist[e - 10]) {
        done_epochs = e + 1;
        break;
      }
    }
    if (tid < D) theta_out[(int64_t)c * D + tid] = sh.theta[tid];
    if (tid < D) sh.w[tid] = sh.theta[tid];
    __syncthreads();
  }
  LR_PHASE(7);
  const int cc = count_correct(sh.w, Xt, Yt, n_test, F);
  if (tid == 0) {
    correct[c] = cc;
    epochs_done[c] = done_epochs;
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
  lr_fedavg_kernel<<<n_coalitions, LR_THREADS, 0, (hipStream_t)stream>>>(
      x, y, n_features, rows, rows_off, n_rows, splits, minibatch_count, masks, keys, agg_w, agg_scale, epochs,
      early_stopping, x_val, y_val, n_val, x_test, y_test, n_test, correct, epochs_done, theta_out, hist,
      hist_stride);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MPLC_OK : (int)e;
}
