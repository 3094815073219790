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
// Work is tiny (28 unknowns, tens of rows): latency-bound; the point is doing all coalitions in ONE launch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "keyed.h"
#include "mplc_hip.h"

namespace {

constexpr int LR_THREADS = 256;
constexpr int LR_MAXF = 64;   // features (+1 intercept) supported
constexpr int LR_MAXP = 64;   // partners per coalition
constexpr int LR_CHUNK = 2048; // rows whose sigma is staged in LDS at a time

struct Shared {
  double theta[LR_MAXF];
  double w[LR_MAXF];       // current Newton iterate
  double g[LR_MAXF];
  double d[LR_MAXF];
  double H[LR_MAXF * LR_MAXF];
  double acc[LR_MAXF];      // FedAvg accumulator
  double red[LR_THREADS];
  double sg[LR_CHUNK];      // sigma(-y z) of the staged rows
  int rid[LR_CHUNK];        // their dataset row ids
  double val_hist[64];
  int done;
};

__device__ double block_sum(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int off = LR_THREADS / 2; off >= 1; off >>= 1) {
    if (tid < off) red[tid] += red[tid + off];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
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

__device__ double objective(const double* w, const RowSel& rs, const float* X, const float* Y, int F, Shared& sh) {
  double part = 0.0;
  for (int i = threadIdx.x; i < rs.count; i += LR_THREADS) {
    const int r = rs.row(i);
    const float* xr = X + (int64_t)r * F;
    double z = w[F];
    for (int k = 0; k < F; ++k) z += w[k] * (double)xr[k];
    const double yy = Y[r] > 0.5f ? 1.0 : -1.0;
    const double t = -yy * z;
    part += t > 0 ? t + log1p(exp(-t)) : log1p(exp(t));
  }
  double f = block_sum(part, sh.red);
  double reg = 0.0;
  for (int k = 0; k < F; ++k) reg += w[k] * w[k];
  return f + 0.5 * reg;
}

// Exact L2-logistic fit (damped Newton) into sh.w, warm-started from sh.w.
__device__ void newton_fit(const RowSel& rs, const float* X, const float* Y, int F, Shared& sh) {
  const int tid = threadIdx.x;
  const int D = F + 1;
  for (int it = 0; it < 100; ++it) {
    // gradient and Hessian: rows staged in chunks (sigma and row id in LDS); thread t owns entries
    // e = t, t+256, ... of [upper-triangular Hessian | gradient]
    double accum[4] = {0.0, 0.0, 0.0, 0.0};
    for (int c0 = 0; c0 < rs.count; c0 += LR_CHUNK) {
      const int cn = min(LR_CHUNK, rs.count - c0);
      for (int i = tid; i < cn; i += LR_THREADS) {
        const int r = rs.row(c0 + i);
        const float* xr = X + (int64_t)r * F;
        double z = sh.w[F];
        for (int q = 0; q < F; ++q) z += sh.w[q] * (double)xr[q];
        const double yy = Y[r] > 0.5f ? 1.0 : -1.0;
        sh.sg[i] = 1.0 / (1.0 + exp(yy * z));
        sh.rid[i] = r;
      }
      __syncthreads();
      for (int u = 0, e = tid; e < D * D + D; e += LR_THREADS, ++u) {
        const bool isg = e >= D * D;
        const int k = isg ? e - D * D : e / D;
        const int l = isg ? 0 : e % D;
        if (!isg && l < k) continue;  // upper triangle only
        double s = 0.0;
        for (int i = 0; i < cn; ++i) {
          const int r = sh.rid[i];
          const float* xr = X + (int64_t)r * F;
          const double sg = sh.sg[i];
          const double xk = k < F ? (double)xr[k] : 1.0;
          if (isg) {
            const double yy = Y[r] > 0.5f ? 1.0 : -1.0;
            s += -yy * sg * xk;
          } else {
            const double xl = l < F ? (double)xr[l] : 1.0;
            s += sg * (1.0 - sg) * xk * xl;
          }
        }
        accum[u] += s;
      }
      __syncthreads();
    }
    for (int u = 0, e = tid; e < D * D + D; e += LR_THREADS, ++u) {
      const bool isg = e >= D * D;
      const int k = isg ? e - D * D : e / D;
      const int l = isg ? 0 : e % D;
      if (!isg && l < k) continue;
      if (isg) {
        sh.g[k] = accum[u] + (k < F ? sh.w[k] : 0.0);
      } else {
        const double v = accum[u] + ((k == l && k < F) ? 1.0 : 0.0);
        sh.H[k * D + l] = v;
        sh.H[l * D + k] = v;
      }
    }
    __syncthreads();
    if (tid == 0) {
      double gmax = 0.0;
      for (int k = 0; k < D; ++k) gmax = fmax(gmax, fabs(sh.g[k]));
      sh.done = gmax < 1e-10 ? 1 : 0;
    }
    __syncthreads();
    if (sh.done) break;
    // Cholesky solve H d = g (single lane: D <= 64, negligible)
    if (tid == 0) {
      double* A = sh.H;
      for (int j = 0; j < D; ++j) {
        double s = A[j * D + j];
        for (int q = 0; q < j; ++q) s -= A[j * D + q] * A[j * D + q];
        const double Ljj = sqrt(s);
        A[j * D + j] = Ljj;
        for (int i = j + 1; i < D; ++i) {
          double t = A[i * D + j];
          for (int q = 0; q < j; ++q) t -= A[i * D + q] * A[j * D + q];
          A[i * D + j] = t / Ljj;
        }
      }
      for (int i = 0; i < D; ++i) {  // forward
        double t = sh.g[i];
        for (int q = 0; q < i; ++q) t -= A[i * D + q] * sh.d[q];
        sh.d[i] = t / A[i * D + i];
      }
      for (int i = D - 1; i >= 0; --i) {  // backward
        double t = sh.d[i];
        for (int q = i + 1; q < D; ++q) t -= A[q * D + i] * sh.d[q];
        sh.d[i] = t / A[i * D + i];
      }
    }
    __syncthreads();
    // backtracking line search on the objective
    const double f0 = objective(sh.w, rs, X, Y, F, sh);
    double gd = 0.0;
    for (int k = 0; k < D; ++k) gd += sh.g[k] * sh.d[k];
    double t = 1.0;
    for (int ls = 0; ls < 40; ++ls) {
      if (tid < D) sh.theta[tid] = sh.w[tid] - t * sh.d[tid];  // theta used as scratch trial point
      __syncthreads();
      const double f1 = objective(sh.theta, rs, X, Y, F, sh);
      if (f1 <= f0 - 1e-4 * t * gd) break;
      t *= 0.5;
      __syncthreads();
    }
    if (tid < D) sh.w[tid] = sh.theta[tid];
    __syncthreads();
  }
}

__device__ int count_correct(const double* w, const float* X, const float* Y, int n, int F, double* red) {
  double c = 0.0;
  for (int i = threadIdx.x; i < n; i += LR_THREADS) {
    double z = w[F];
    for (int k = 0; k < F; ++k) z += w[k] * (double)X[(int64_t)i * F + k];
    c += ((z > 0.0) == (Y[i] > 0.5f)) ? 1.0 : 0.0;
  }
  return (int)(block_sum(c, red) + 0.5);
}

__device__ int count_correct_rows(const double* w, const RowSel& rs, const float* X, const float* Y, int F,
                                  double* red) {
  double c = 0.0;
  for (int i = threadIdx.x; i < rs.count; i += LR_THREADS) {
    const int r = rs.row(i);
    double z = w[F];
    for (int k = 0; k < F; ++k) z += w[k] * (double)X[(int64_t)r * F + k];
    c += ((z > 0.0) == (Y[r] > 0.5f)) ? 1.0 : 0.0;
  }
  return (int)(block_sum(c, red) + 0.5);
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
      const int ct = count_correct_rows(sh.w, rs, X, Y, F, sh.red);
      const int cv = count_correct(sh.w, Xv, Yv, n_val, F, sh.red);
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
          const int cv = count_correct(sh.theta, Xv, Yv, n_val, F, sh.red);
          const double eps = 1e-15;
          vl = (double)(n_val - cv) * (-log(eps)) / (double)n_val + (double)cv * (-log(1.0 - eps)) / (double)n_val;
        }
        if (tid == 0) val_hist[e] = vl;
        __syncthreads();
      }
      for (int m = 0; m < M; ++m) {
        double* hrow = hist ? hist + (int64_t)c * hist_stride + (int64_t)(e * M + m) * (2 + 4 * LR_MAXP) : nullptr;
        if (hrow) {  // the round-start collective model on val (eval_and_log_model_val_perf); unfitted: [0, 0]
          const int cv = have ? count_correct(sh.theta, Xv, Yv, n_val, F, sh.red) : 0;
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
            const int ct = count_correct_rows(sh.w, rs, X, Y, F, sh.red);
            const int cv = count_correct(sh.w, Xv, Yv, n_val, F, sh.red);
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
  const int cc = count_correct(sh.w, Xt, Yt, n_test, F, sh.red);
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
  // (D*D + D) Hessian+gradient entries must fit 4 per thread: D = n_features + 1 <= 31
  if (n_features < 1 || n_features + 1 > 31 || n_coalitions < 1 || minibatch_count < 1 || epochs < 1 ||
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
