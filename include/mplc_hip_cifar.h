/*
 * mplc_hip_cifar.h - batched multi-model CIFAR10 CNN trainer (part of the mplc_hip.h C ABI).
 *
 * Model (mplc/dataset.py:167-200):
 *   Conv2D(32,3x3,same) ReLU -> Conv2D(32,3x3) ReLU -> MaxPool(2) -> Dropout(.25)
 *   -> Conv2D(64,3x3,same) ReLU -> Conv2D(64,3x3) ReLU -> MaxPool(2) -> Dropout(.25)
 *   -> Flatten(2304) -> Dense(512) ReLU -> Dropout(.5) -> Dense(10) softmax;
 *   categorical cross-entropy; Keras 2.3.1 RMSprop(learning_rate=1e-4, rho=0.9, eps=1e-7, decay=1e-6);
 *   glorot_uniform kernels, zero biases.
 *
 * Same replica model as mplc_hip_cnn.h (a REPLICA is one (coalition, partner) model; mplc_replica_t,
 * MPLC_REP_* and the keyed sample schedule are shared), with two additions:
 *   - Dropout masks are keyed counters: keep(layer, slot, element) of a replica at one Keras step is a
 *     pure function of (replica key, epoch, round, step) - restated bit for bit in oracle/cifar_cnn.py.
 *   - RMSprop keeps one accumulator per parameter; a FedAvg partner fit starts a fresh optimizer
 *     (accumulators 0, iterations 0: mplc/multi_partner_learning.py:319), a singleton keeps it.
 *
 * Replaces, for all replicas at once, the CIFAR10 instances of:
 *   - Keras `model.fit(x_mb, y_mb, batch_size=bs_p, epochs=1)` per partner per FedAvg round
 *     (mplc/multi_partner_learning.py:301-332),
 *   - the singleton `model.fit(x, y, batch_size=bs_p, epochs=E)` (mplc/multi_partner_learning.py:253-260),
 *   - `model.evaluate(x, y, batch_size=256)` (mplc/multi_partner_learning.py:142-169).
 */
#ifndef MPLC_HIP_CIFAR_H
#define MPLC_HIP_CIFAR_H

#include <stddef.h>
#include <stdint.h>

#include "mplc_hip_cnn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* parameter row layout (floats), Keras weight order per layer, 64-float aligned */
#define MPLC_CIFAR_OFF_W1 0          /* 3*3*3*32     */
#define MPLC_CIFAR_OFF_B1 896        /* 32           */
#define MPLC_CIFAR_OFF_W2 960        /* 3*3*32*32    */
#define MPLC_CIFAR_OFF_B2 10176      /* 32           */
#define MPLC_CIFAR_OFF_W3 10240      /* 3*3*32*64    */
#define MPLC_CIFAR_OFF_B3 28672      /* 64           */
#define MPLC_CIFAR_OFF_W4 28736      /* 3*3*64*64    */
#define MPLC_CIFAR_OFF_B4 65600      /* 64           */
#define MPLC_CIFAR_OFF_W5 65664      /* 2304*512     */
#define MPLC_CIFAR_OFF_B5 1245312    /* 512          */
#define MPLC_CIFAR_OFF_W6 1245824    /* 512*10       */
#define MPLC_CIFAR_OFF_B6 1250944    /* 10           */
#define MPLC_CIFAR_NPARAM 1250954
#define MPLC_CIFAR_STRIDE 1251008
/* per-sample activation sizes (floats; NHWC) */
#define MPLC_CIFAR_A1 32768          /* conv1 out 32x32x32 (ReLU)                 */
#define MPLC_CIFAR_D2 7200           /* pool2 + dropout out 15x15x32              */
#define MPLC_CIFAR_A3 14400          /* conv3 out 15x15x64 (ReLU)                 */
#define MPLC_CIFAR_D4 2304           /* pool4 + dropout out 6x6x64 (= flatten)    */
#define MPLC_CIFAR_H5 512            /* dense5 out (ReLU + dropout)               */
#define MPLC_CIFAR_DZ4 2304          /* slot stride of dz4: the pooled gradient 6x6x64 (ABI 3) */
#define MPLC_CIFAR_DZ3 14400         /* conv3 pre-activation gradient 15x15x64    */
#define MPLC_CIFAR_DZ2 7200          /* slot stride of dz2: the pooled gradient 15x15x32 (ABI 3) */
#define MPLC_CIFAR_DZ1 32768         /* conv1 pre-activation gradient 32x32x32    */
#define MPLC_CIFAR_WT 114688         /* W2|W3|W4 in Winograd form (16 x ci x co each): the forward's, then
                                        the data gradients' (rotated, channels swapped) */
#define MPLC_CIFAR_WPART 65664       /* partial gradient row of W1..b4 (= params layout prefix) */
#ifndef MPLC_CIFAR_WG_SAMPLES
#define MPLC_CIFAR_WG_SAMPLES 2      /* samples per weight-gradient split (fixed: reproducible sums) */
#endif

typedef struct {
  /* geometry */
  int32_t n_rep;          /* replicas                                                     */
  int32_t bmax;           /* max batch size over replicas (slot stride)                   */
  int32_t wg_splits;      /* = ceil(bmax / MPLC_CIFAR_WG_SAMPLES)                         */
  int32_t pad0;
  /* schedule (global step -> per-replica samples), as mplc_cnn_train_t */
  int32_t step;
  int32_t minibatch_count;
  int32_t round_len;
  int32_t epochs;
  const mplc_replica_t* reps;
  const int32_t* rows;
  const int32_t* splits;
  const int32_t* seq;     /* MPLC_REP_SEQ member records (NULL when there are none)        */
  /* data */
  const float* x;         /* [N][32][32][3] fp32 in [0,1]                                 */
  const int32_t* labels;  /* [N] class ids                                                */
  /* model state */
  float* params;          /* [n_rep][MPLC_CIFAR_STRIDE]                                   */
  float* rms;             /* [n_rep][MPLC_CIFAR_STRIDE] RMSprop accumulators              */
  /* workspaces (device), slot-major [n_rep][bmax][...] */
  int32_t* idx;           /* [n_rep][bmax] dataset rows of this step                      */
  int32_t* cnt;           /* [n_rep] samples this step (0 = idle)                         */
  int32_t* opt_t;         /* [n_rep] optimizer iteration of this step (1 = fresh)         */
  uint64_t* drop_key;     /* [n_rep] dropout key of this step                             */
  float* a1;              /* [.][MPLC_CIFAR_A1]                                           */
  float* d2;              /* [.][MPLC_CIFAR_D2]                                           */
  uint8_t* code2;         /* [.][MPLC_CIFAR_D2] argmax | 0x40 kept | 0x80 positive        */
  float* a3;              /* [.][MPLC_CIFAR_A3]                                           */
  float* d4;              /* [.][MPLC_CIFAR_D4]                                           */
  uint8_t* code4;         /* [.][MPLC_CIFAR_D4]                                           */
  float* d5;              /* [.][MPLC_CIFAR_H5] dropout(relu(dense5))                     */
  uint8_t* code5;         /* [.][MPLC_CIFAR_H5] 0x40 kept | 0x80 positive                 */
  float* dh5;             /* [.][MPLC_CIFAR_H5]                                           */
  float* dz4;             /* [.][MPLC_CIFAR_DZ4]: the POOLED dense5 input gradient [6][6][64],  */
                          /* un-pooled by conv4's gradient kernels (code4)                    */
  float* dz3;             /* [.][MPLC_CIFAR_DZ3]                                          */
  float* dz2;             /* [.][MPLC_CIFAR_DZ2]: the POOLED conv3 input gradient [15][15][32], */
                          /* un-pooled by conv2's gradient kernels (code2)                    */
  float* dz1;             /* [.][MPLC_CIFAR_DZ1]                                          */
  float* wt;              /* [n_rep][MPLC_CIFAR_WT] Winograd-form conv weights (workspace)  */
  float* wpart;           /* [n_rep][wg_splits][MPLC_CIFAR_WPART]                         */
  /* optimizer (Keras 2.3.1 RMSprop).  one_minus_rho is passed separately: Keras computes (1. - rho) on
   * the Python double (rho is not a backend variable) and rounds once, fp32(1 - 0.9) = 0.1f, which is
   * not 1 - fp32(0.9). */
  float lr, rho, one_minus_rho, decay, eps;
  /* optional in-stream timing of one launch of the step (bench roofline); ids in mplc/cifar.py.  prof_kernel =
   * MPLC_PROF_ALL times every launch k = 1 .. 15, prof_begin / prof_end then pointing to hipEvent_t arrays of 16 */
  int32_t prof_kernel;
  void* prof_begin;
  void* prof_end;
  /* optional training history (NULL = off): per replica, the step's [sum of per-sample CE before the
   * update, correct predictions, samples] (dropout active, as a Keras fit reports them); see
   * mplc_cnn_train_t.hstats */
  double* hstats;         /* [n_rep][3]                                                   */
  /* optional (NULL = off), as mplc_cnn_train_t.glob for W3: FedAvg replicas read W5 at the first step of a
   * round from their coalition's row of glob, which the aggregation then need not broadcast
   * (mplc_fedavg_aggregate_bcast_skip with [MPLC_CIFAR_OFF_W5, MPLC_CIFAR_OFF_B5)). */
  const float* glob;      /* [n_coalitions][MPLC_CIFAR_STRIDE] coalition models                   */
  const int32_t* rep_glob;  /* [n_rep] replica -> its coalition's row of glob                 */
  int32_t* w5src;         /* [n_rep] workspace: glob row W5 is read from this step, or -1      */
} mplc_cifar_train_t;

/* Parameter row stride in floats (== MPLC_CIFAR_STRIDE). */
int mplc_cifar_stride(void);

/* Samples per weight-gradient split: mplc_cifar_train_t.wg_splits must be ceil(bmax / this). */
int mplc_cifar_wgrad_split_samples(void);

/* Layout query (ABI check at load): the value of item `what` (MPLC_CIFAR_Q_*) as this library was built, or -1
 * for an unknown item.  The host compares every item with its own constants and refuses a mismatched pair. */
#define MPLC_CIFAR_Q_STRIDE 0
#define MPLC_CIFAR_Q_NPARAM 1
#define MPLC_CIFAR_Q_A1 2
#define MPLC_CIFAR_Q_D2 3
#define MPLC_CIFAR_Q_A3 4
#define MPLC_CIFAR_Q_D4 5
#define MPLC_CIFAR_Q_H5 6
#define MPLC_CIFAR_Q_DZ4 7
#define MPLC_CIFAR_Q_DZ3 8
#define MPLC_CIFAR_Q_DZ2 9
#define MPLC_CIFAR_Q_DZ1 10
#define MPLC_CIFAR_Q_WT 11
#define MPLC_CIFAR_Q_WPART 12
#define MPLC_CIFAR_Q_WG_SAMPLES 13
#define MPLC_CIFAR_Q_TRAIN_T_BYTES 14  /* sizeof(mplc_cifar_train_t) */
#define MPLC_CIFAR_Q_COUNT 15
int64_t mplc_cifar_layout(int what);

/* glorot_uniform kernels / zero biases for n_models rows, keyed per model. */
int mplc_cifar_init_params(float* params, int64_t stride, const uint64_t* keys, int n_models, void* stream);

/* Enqueue one lockstep training step of all replicas (schedule, forward, backward, RMSprop). */
int mplc_cifar_train_step(const mplc_cifar_train_t* t, void* stream);

/* Forward-only (inference: no dropout) evaluation of n_models models on samples [0, n_samples):
 * correct[m] += #argmax hits, loss_sum[m] += sum of per-sample CE (float64: per
 * block of 256 samples a fixed tree, the blocks added in sample order; with every chunk but the last a multiple
 * of 256 the sum does not depend on chunk or n_models).  ws is a workspace of
 * mplc_cifar_eval_workspace_floats(n_models, chunk) floats. */
int64_t mplc_cifar_eval_workspace_floats(int n_models, int chunk);
int mplc_cifar_evaluate(const float* params, int64_t stride, int n_models, const float* x, const int32_t* labels,
                        int n_samples, int chunk, float* ws, int32_t* correct, double* loss_sum, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MPLC_HIP_CIFAR_H */
