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
// keeping each fit's dependent chain short.  Round 5: one wave per coalition (reductions in registers, no block
// barriers), the fit's rows staged in LDS once per fit (the Newton iterations read them from LDS instead of
// re-gathering them through the keyed permutation from global memory), the Hessian's entries spread over the
// lanes, the Cholesky factorisation and the two triangular solves parallel over the rows (a single lane did them
// serially: 28^3/6 dependent LDS round trips per iteration), and the line search's accepted objective reused as
// the next iteration's start value.  The 1023-coalition sweep (config #2): 242 ms -> 40.3 ms
// (profiles/r05_titanic_kernel_stats{,_onewave}.csv).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "keyed.h"
#include "mplc_hip.h"

namespace {

constexpr int LR_THREADS = 64;   // one wave per coalition
constexpr int LR_MAXF = 32;      // D = n_features + 1 unknowns (coef | intercept) supported
constexpr int LR_MAXP = 64;      // partners per coalition
constexpr int LR_NMAX = 128;     // rows staged in LDS at a time (a whole Titanic fit: <= 71 rows)
constexpr int LR_NE = LR_MAXF * (LR_MAXF + 1) / 2 + LR_MAXF;  // Hessian upper triangle + gradient entries
constexpr int LR_EPL = (LR_NE + LR_THREADS - 1) / LR_THREADS;  // entries per lane

struct Shared {
  double theta[LR_MAXF];
  double w[LR_MAXF];       // current Newton iterate
  double trial[LR_MAXF];   // line-search trial point
  double acc[LR_MAXF];     // FedAvg accumulator
  double g[LR_MAXF];       // gradient
  double L[LR_MAXF * LR_MAXF];  // the Hessian's lower triangle, factorised in place (row-major)
  double hv[LR_NMAX];      // s (1 - s) of the staged rows, s = sigma(-y z)
  double sv[LR_NMAX];      // -y s
  float xs[LR_NMAX * LR_MAXF];  // staged rows [i][k], k < F
  float ys[LR_NMAX];       // +-1
  int rid[LR_NMAX];
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

// rows [c0, c0 + cn) of the fit into LDS: features as fp32 (the data's own precision), labels as +-1
__device__ void stage_rows(const RowSel& rs, int c0, int cn, const float* X, const float* Y, int F, Shared& sh) {
  const int lane = threadIdx.x;
  for (int i = lane; i < cn; i += LR_THREADS) {
    const int r = rs.row(c0 + i);
    sh.rid[i] = r;
    sh.ys[i] = Y[r] > 0.5f ? 1.0f : -1.0f;
  }
  __syncthreads();
  for (int e = lane; e < cn * F; e += LR_THREADS) {
    const int i = e / F, k = e % F;
    sh.xs[i * LR_MAXF + k] = X[(int64_t)sh.rid[i] * F + k];
  }
  __syncthreads();
}

__device__ __forceinline__ double row_z(const double* w, const float* xr, int F) {
  double z = w[F];
  for (int k = 0; k < F; ++k) z += w[k] * (double)xr[k];
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
      const double t = -(double)sh.ys[i] * row_z(w, sh.xs + i * LR_MAXF, F);
      part += t > 0 ? t + log1p(exp(-t)) : log1p(exp(t));
    }
  }
  const double reg = (lane < F) ? w[lane] * w[lane] : 0.0;
  return wave_sum(part) + 0.5 * wave_sum(reg);
}

// Exact L2-logistic fit (damped Newton with Armijo backtracking) into sh.w, warm-started from sh.w.
__device__ void newton_fit(const RowSel& rs, const float* X, const float* Y, int F, Shared& sh) {
  const int lane = threadIdx.x;
  const int D = F + 1;
  const int NE = D * (D + 1) / 2 + D;  // Hessian entries (k <= l) then the gradient
  const bool resident = rs.count <= LR_NMAX;
  if (resident) stage_rows(rs, 0, rs.count, X, Y, F, sh);
  double f0 = objective(sh.w, rs, resident, X, Y, F, sh);
  for (int it = 0; it < 100; ++it) {
    // gradient and Hessian: per staged row s and s (1 - s), then lane-owned entries summed over the rows in order
    double acc[LR_EPL];
#pragma unroll
    for (int u = 0; u < LR_EPL; ++u) acc[u] = 0.0;
    for (int c0 = 0; c0 < rs.count; c0 += LR_NMAX) {
      const int cn = min(LR_NMAX, rs.count - c0);
      if (!resident) stage_rows(rs, c0, cn, X, Y, F, sh);
      for (int i = lane; i < cn; i += LR_THREADS) {
        const double yy = (double)sh.ys[i];
        const double sg = 1.0 / (1.0 + exp(yy * row_z(sh.w, sh.xs + i * LR_MAXF, F)));
        sh.sv[i] = -yy * sg;
        sh.hv[i] = sg * (1.0 - sg);
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < LR_EPL; ++u) {
        const int e = lane + LR_THREADS * u;
        if (e >= NE) break;
        double s = 0.0;
        if (e >= NE - D) {  // gradient entry k
          const int k = e - (NE - D);
          for (int i = 0; i < cn; ++i) s += sh.sv[i] * (k < F ? (double)sh.xs[i * LR_MAXF + k] : 1.0);
        } else {  // Hessian entry (k, l), k <= l: the e-th of the row-major upper triangle
          int k = 0, rem = e;
          while (rem >= D - k) { rem -= D - k; ++k; }
          const int l = k + rem;
          for (int i = 0; i < cn; ++i) {
            const double xk = k < F ? (double)sh.xs[i * LR_MAXF + k] : 1.0;
            const double xl = l < F ? (double)sh.xs[i * LR_MAXF + l] : 1.0;
            s += sh.hv[i] * xk * xl;
          }
        }
        acc[u] += s;
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < LR_EPL; ++u) {
      const int e = lane + LR_THREADS * u;
      if (e >= NE) break;
      if (e >= NE - D) {
        const int k = e - (NE - D);
        sh.g[k] = acc[u] + (k < F ? sh.w[k] : 0.0);
      } else {
        int k = 0, rem = e;
        while (rem >= D - k) { rem -= D - k; ++k; }
        const int l = k + rem;
        sh.L[l * LR_MAXF + k] = acc[u] + ((k == l && k < F) ? 1.0 : 0.0);  // lower triangle, row l
      }
    }
    __syncthreads();
    const double gk = lane < D ? sh.g[lane] : 0.0;
    if (wave_max(fabs(gk)) < 1e-10) break;
    // Cholesky H = L L^T in place, left-looking: column j, lanes = rows i >= j
    for (int j = 0; j < D; ++j) {
      double sj = 0.0;
      if (lane >= j && lane < D) {
        sj = sh.L[lane * LR_MAXF + j];
        for (int q = 0; q < j; ++q) sj -= sh.L[lane * LR_MAXF + q] * sh.L[j * LR_MAXF + q];
      }
      const double ljj = sqrt(__shfl(sj, j));
      if (lane == j) sh.L[j * LR_MAXF + j] = ljj;
      else if (lane > j && lane < D) sh.L[lane * LR_MAXF + j] = sj / ljj;
      __syncthreads();
    }
    // L y = g (forward), L^T d = y (backward): lane k holds entry k; one row broadcast per step
    double b = gk;
    for (int q = 0; q < D; ++q) {
      const double yq = __shfl(b, q) / sh.L[q * LR_MAXF + q];
      if (lane == q) b = yq;
      else if (lane > q && lane < D) b -= sh.L[lane * LR_MAXF + q] * yq;
    }
    for (int q = D - 1; q >= 0; --q) {
      const double dq = __shfl(b, q) / sh.L[q * LR_MAXF + q];
      if (lane == q) b = dq;
      else if (lane < q) b -= sh.L[q * LR_MAXF + lane] * dq;
    }
    const double dk = lane < D ? b : 0.0;
    const double gd = wave_sum(gk * dk);
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
    __syncthreads();
  }
}

__device__ int count_correct(const double* w, const float* X, const float* Y, int n, int F) {
  double c = 0.0;
  for (int i = threadIdx.x; i < n; i += LR_THREADS)
    c += ((row_z(w, X + (int64_t)i * F, F) > 0.0) == (Y[i] > 0.5f)) ? 1.0 : 0.0;
  return (int)(wave_sum(c) + 0.5);
}

__device__ int count_correct_rows(const double* w, const RowSel& rs, const float* X, const float* Y, int F) {
  double c = 0.0;
  for (int i = threadIdx.x; i < rs.count; i += LR_THREADS) {
    const int r = rs.row(i);
    c += ((row_z(w, X + (int64_t)r * F, F) > 0.0) == (Y[r] > 0.5f)) ? 1.0 : 0.0;
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
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  const int D = F + 1;
  const uint64_t mask = masks[c];
  int parts[LR_MAXP];
  int P = 0;
  for (int p = 0; p < 64 && P < LR_MAXP; ++p)
    if ((mask >> p) & 1ull) parts[P++] = p;
  if (tid < D) { sh.theta[tid] = 0.0; sh.w[tid] = 0.0; }
  __syncthreads();
  int done_epochs = epochs;
  if (P == 1) {
    // singleton: one fit on the partner's full data (E refits of the same rows reach the same optimum)
    const int p = parts[0];
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
        for (int pi = 0; pi < P; ++pi) {
          const int p = parts[pi];
          const int* sp = splits + p * (M + 1);
          RowSel rs{rows, rows_off[p], n_rows[p], sp[m], sp[m + 1] - sp[m],
                    subkey(keys[(int64_t)c * LR_MAXP + pi], 0x10000u + (uint32_t)e, 0u), M > 1};
          if (tid < D) sh.w[tid] = have ? sh.theta[tid] : 0.0;  // warm start from the global model
          __syncthreads();
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
  // D = n_features + 1 unknowns <= LR_MAXF (the factor, the per-lane Hessian entries)
  if (n_features < 1 || n_features + 1 > LR_MAXF || n_coalitions < 1 || minibatch_count < 1 || epochs < 1 ||
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
