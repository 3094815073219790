/*
 * mplc_hip.h - C ABI of the MI355X-native MPLC coalition-evaluation engine (libmplc_hip.so).
 *
 * The reference (mshuaic/distributed-learning-contributivity, pure Python) has no FFI: its hot path is
 * Python calling Keras/TF and numpy.  Each entry point below REPLACES one reference interface on the
 * coalition-evaluation path; the replaced file:line is cited per function.  The Python host package
 * (distributed-learning-contributivity_amd/mplc) binds these with ctypes (mplc/_native.py).
 *
 * Conventions
 *  - All pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) unless a comment says "host".
 *  - Buffers are caller-owned.  The library allocates nothing persistent and keeps no pointer after
 *    return.  Work is enqueued on `stream` (a hipStream_t passed as void*; NULL = default stream);
 *    nothing synchronises except where stated.
 *  - Return value: 0 = success; > 0 = hipError_t from a launch; < 0 = MPLC_E_* argument error.
 *    No function calls exit()/abort().
 *  - Coalitions are bitmasks: bit i set <=> partner i in S.  v(S) tables are "bitmask order":
 *    V[mask], mask in [0, 2^n), V[0] = v(empty) = 0 (mplc/contributivity.py:74).
 */
#ifndef MPLC_HIP_H
#define MPLC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPLC_OK 0
#define MPLC_E_ARG (-1)        /* invalid argument (n out of range, misaligned range, NULL)       */
#define MPLC_E_WORKSPACE (-2)  /* workspace too small                                            */
#define MPLC_E_SHAPE (-3)      /* tensor geometry the kernel does not support                    */

/* Version / capability probe: returns MPLC_ABI_VERSION.  Version 2: the CIFAR10 Winograd weight workspace
 * (MPLC_CIFAR_WT 114688) and the layout queries mplc_cnn_layout / mplc_cifar_layout.  Version 3: the CIFAR10
 * pooled-gradient slots dz4 / dz2 at their pooled sizes (MPLC_CIFAR_DZ4 2304, MPLC_CIFAR_DZ2 7200).  Version 4: the
 * round's last step may fuse W3's FedAvg average into the MNIST dense pass (mplc_cnn_train_t.avg_*) and
 * mplc_fedavg_aggregate_skip aggregates the other layers. */
#define MPLC_ABI_VERSION 4
int mplc_abi_version(void);

/* ------------------------------------------------------------------------------------------------
 * Exact Shapley aggregation over the bitmask v(S) table.
 * Replaces: mplc/contributivity.py:1210-1253 `shapley_value(partners_count, char_func_list)` (pure
 *           Python, O(n 4^n)) as called from compute_SV mplc/contributivity.py:163.
 * Formulation (single pass, each V[mask] read once):
 *   w(s) = s!(n-s-1)!/n!,  A_i = sum_{T contains i} v(T) (w(|T|-1) + w(|T|)),  B = sum_S v(S) w(|S|)
 *   with w(-1) = w(n) = 0;  SV_i = A_i - B.
 * Sums are compensated (Kahan in-thread, double-double across threads/blocks).
 * ---------------------------------------------------------------------------------------------- */

/* Bytes of device workspace mplc_shapley_partial/exact need for `count` masks. */
size_t mplc_shapley_workspace_bytes(int n, uint64_t count);

/* Partial sums over masks [mask_begin, mask_begin + count) of an n-partner table.
 * v points at V[mask_begin].  Writes partial_out[2*(n+1)] doubles (device):
 *   {A_0.hi, A_0.lo, ..., A_{n-1}.hi, A_{n-1}.lo, B.hi, B.lo}.
 * Partials of disjoint ranges add (hi with hi, lo with lo): the range-sharded multi-GPU form is
 * partial per rank -> all_reduce(sum) -> mplc_shapley_finalize.
 * Requirements: 1 <= n <= 40; for n >= 16 mask_begin and count are multiples of 65536. */
int mplc_shapley_partial(const double* v, uint64_t mask_begin, uint64_t count, int n, double* partial_out,
                         void* workspace, size_t workspace_bytes, void* stream);

/* sv_out[i] = (A_i.hi - B.hi) + (A_i.lo - B.lo), i < n (device in, device out). */
int mplc_shapley_finalize(const double* partial, int n, double* sv_out, void* stream);

/* Whole table in one call: partial over [0, 2^n) + finalize.  v has 2^n entries, v[0] ignored (= 0). */
int mplc_shapley_exact(const double* v, int n, double* sv_out, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ------------------------------------------------------------------------------------------------
 * FedAvg weighted partner aggregation, batched over coalitions.
 * Replaces: mplc/mpl_utils.py:90-102 `Aggregator.aggregate_model_weights` (per-layer
 *           np.average(stack, axis=0, weights=w) in float64, stored back as float32 by set_weights,
 *           mplc/multi_partner_learning.py:100-104) for DataVolumeAggregator/UniformAggregator
 *           (mplc/mpl_utils.py:105-115).
 * For coalition c with replicas r in [first[c], first[c+1]):
 *   out[c][k] = float( ( ((double)x[r0][k]*w[r0] + (double)x[r1][k]*w[r1]) + ... ) / scale[c] )
 * products and sums rounded separately in replica order (numpy's multiply-then-sum, axis 0), then
 * one division and one fp64->fp32 rounding: bit-identical to the reference's numpy path.
 * If broadcast != 0 the result is also written into every replica row of the coalition
 * (x[r][k] = out[c][k]), which starts the next FedAvg round (mplc/multi_partner_learning.py:310-311).
 * ---------------------------------------------------------------------------------------------- */
int mplc_fedavg_aggregate(float* x, int64_t x_stride, const int32_t* first, const double* w,
                          const double* scale, int n_coalitions, int64_t n_param, float* out,
                          int64_t out_stride, int broadcast, void* stream);

/* As mplc_fedavg_aggregate with broadcast, except that parameters [skip_lo, skip_hi) are not written back
 * into the replica rows: their only copy is out[c] (required), which the next round's first step reads
 * instead (the MNIST trainer's W3, include/mplc_hip_cnn.h `glob` / `rep_glob`): 98 % of the broadcast bytes
 * of a FedAvg round are not written, and the replicas of a coalition read one shared row. */
int mplc_fedavg_aggregate_bcast_skip(float* x, int64_t x_stride, const int32_t* first, const double* w,
                                     const double* scale, int n_coalitions, int64_t n_param, float* out,
                                     int64_t out_stride, int64_t skip_lo, int64_t skip_hi, void* stream);

/* As mplc_fedavg_aggregate_bcast_skip, except that parameters [skip_lo, skip_hi) are neither averaged nor
 * written anywhere: out[c]'s range is left as it is (ABI 4: the MNIST trainer's W3, whose average the round's
 * last step already wrote there - mplc_cnn_train_t.avg_*).  Every other parameter is averaged into out[c] and
 * broadcast to the replica rows, bit-identical to mplc_fedavg_aggregate. */
int mplc_fedavg_aggregate_skip(float* x, int64_t x_stride, const int32_t* first, const double* w, const double* scale,
                               int n_coalitions, int64_t n_param, float* out, int64_t out_stride, int64_t skip_lo,
                               int64_t skip_hi, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Batched FedAvg logistic regression (Titanic model, BASELINE config #2), all coalitions at once: per FedAvg
 * round one launch whose waves take (coalition, partner) fits from a work queue and one launch that averages
 * each coalition's fits; a stream-ordered workspace (hipMallocAsync / hipFreeAsync on `stream`) holds the
 * coalitions' models between the launches.
 * Replaces, per coalition, FederatedAverageLearning.fit (mplc/multi_partner_learning.py:195-216,
 * 285-334) with the Titanic.LogisticRegression model (mplc/dataset.py:323-394: sklearn L2 LR, C=1),
 * np.average aggregation (mplc/mpl_utils.py:90-115) and the test accuracy (:158-169).  Every fit is the
 * exact optimum (damped Newton, fp64).  Singletons (the reference crashes there: callbacks= passed to the
 * LR fit, mplc/multi_partner_learning.py:254-260) are one fit on the partner's full data.
 *  x [N][n_features] fp32, y [N] fp32 0/1; rows/rows_off/n_rows: partners' row ids into x;
 *  splits: M+1 minibatch boundaries per partner (partner p at p*(M+1)); masks[c]: coalition bitmask;
 *  keys[c*64 + i], agg_w[c*64 + i]: shuffle key and aggregation weight of the i-th partner (ascending id)
 *  of coalition c; agg_scale[c]: np.average's weight sum.  Outputs: correct[c] test hits,
 *  epochs_done[c], theta_out[c][n_features+1] = [coef | intercept].  n_features <= 30.
 *  hist (NULL = off; needs x_val): the learning history (mplc/mpl_utils.py:11-27, logged by
 *  mplc/multi_partner_learning.py:130-156) of coalition c at hist + c * hist_stride, round (e, m) at
 *  offset (e*M + m) * (2 + 4*64): [collective val_loss, val_accuracy at the round start (0, 0 while
 *  unfitted)] then per partner pi (ascending id) [loss, accuracy on its minibatch, val_loss,
 *  val_accuracy] after its fit - Titanic.LogisticRegression.evaluate on hard predictions
 *  (mplc/dataset.py:329-351).  A singleton writes its partner block of round (0, 0).  Unvisited entries
 *  are left as the caller initialised them.  hist_stride >= epochs * M * (2 + 4 * 64).
 * ---------------------------------------------------------------------------------------------- */
int mplc_lr_fedavg(const float* x, const float* y, int n_features, const int32_t* rows, const int32_t* rows_off,
                   const int32_t* n_rows, const int32_t* splits, int minibatch_count, const uint64_t* masks,
                   const uint64_t* keys, const double* agg_w, const double* agg_scale, int n_coalitions, int epochs,
                   int early_stopping, const float* x_val, const float* y_val, int n_val, const float* x_test,
                   const float* y_test, int n_test, int32_t* correct, int32_t* epochs_done, double* theta_out,
                   double* hist, int64_t hist_stride, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Monte-Carlo Shapley over a dense bitmask v(S) table (csrc/mc_shapley.hip).  V has 2^n fp64 entries,
 * NaN = not evaluated yet; 1 <= n <= 30; perms are [n_perms][n] uint8 partner ids.
 * Replaces: the permutation walk of truncated_MC / interpol_TMC (mplc/contributivity.py:217-246,
 *           :278-316): char[j+1] = char[j] (TMCS) / char[j] + a*size[j] (ITMCS, sizes in partner-index
 *           order as the reference) once |v_all - char[j]| < truncation, else v(prefix); row[perm[j]] =
 *           char[j+1] - char[j], in the reference's fp64 operation order.
 * ---------------------------------------------------------------------------------------------- */

/* One thread per permutation: rows[k][n] increments; status[k] = n if the walk completed, else the first
 * position j whose prefix mask need[k] is NaN in V (rows[k] then incomplete). */
int mplc_tmc_walk(const double* V, int n, const uint8_t* perms, int n_perms, double v_all, double truncation,
                  int interpolate, const double* sizes, double* rows, int32_t* status, uint64_t* need, void* stream);

/* Fixed-budget form: moments_out[2n+1] = {sum_k row_k[j] (j<n), sum_k row_k[j]^2 (j<n), #complete walks}
 * over n_perms walks (incomplete walks contribute 0).  perms == NULL draws permutation perm_base + k on
 * device (keyed Fisher-Yates from `seed`).  Deterministic reduction (wavefront shuffles, fixed block order). */
size_t mplc_tmc_moments_workspace_bytes(int n, int n_perms);
int mplc_tmc_moments(const double* V, int n, const uint8_t* perms, uint64_t seed, uint64_t perm_base, int n_perms,
                     double v_all, double truncation, int interpolate, const double* sizes, double* moments_out,
                     void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Batched multi-model MNIST CNN trainer (mplc/dataset.py:457-479 architecture; Keras 2.3.1 Adam).
 * One "replica" = one (coalition, partner) model.  Replaces, for B replicas at once, the per-partner
 * Keras `model.fit(x_mb, y_mb, batch_size=bs_p, epochs=1)` of mplc/multi_partner_learning.py:319-332
 * (FedAvg round), the singleton `model.fit(epochs=E)` of mplc/multi_partner_learning.py:253-260 and
 * `model.evaluate(x_test, y_test)` of mplc/multi_partner_learning.py:158-169.
 * Declared in mplc_hip_cnn.h.
 * ---------------------------------------------------------------------------------------------- */

#ifdef __cplusplus
}
#endif

#include "mplc_hip_cnn.h"
#include "mplc_hip_cifar.h"

#endif /* MPLC_HIP_H */
