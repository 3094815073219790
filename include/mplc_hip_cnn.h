/*
 * mplc_hip_cnn.h - batched multi-model MNIST CNN trainer (part of the mplc_hip.h C ABI).
 *
 * Model (mplc/dataset.py:457-479): Conv2D(32,3x3,relu) -> Conv2D(64,3x3,relu) -> MaxPool(2) -> Flatten
 * -> Dense(128,relu) -> Dense(10,softmax); categorical cross-entropy; Keras 2.3.1 Adam (lr 1e-3,
 * beta 0.9/0.999, eps 1e-7); glorot_uniform kernels, zero biases.
 *
 * A MODEL is one flat fp32 parameter row of MPLC_CNN_STRIDE floats (Keras weight order per layer:
 * conv kernels [kh][kw][cin][cout], dense [in][out]; offsets below).  A REPLICA is one model being
 * trained on one partner's data: a (coalition, partner) pair of a FedAvg coalition or the single model
 * of a singleton coalition.  B replicas step in lockstep; each has its own batch size, sample schedule
 * and Adam step count (ragged batches are masked per replica).
 *
 * Replaces, for all replicas at once:
 *   - Keras `model.fit(x_mb, y_mb, batch_size=bs_p, epochs=1)` per partner per FedAvg round with a fresh
 *     optimizer (mplc/multi_partner_learning.py:301-332, partner.build_model mplc/partner.py:169-170),
 *   - the singleton `model.fit(x, y, batch_size=bs_p, epochs=E)` with persistent Adam
 *     (mplc/multi_partner_learning.py:253-260),
 *   - `model.evaluate(x, y, batch_size=256)` -> [loss, accuracy] (mplc/multi_partner_learning.py:142-169).
 * Sample order: epoch permutation of the partner's rows (PartnerMpl.split_minibatches,
 * mplc/partner.py:155-167), split at floor(k/M * n_p), then Keras' per-fit shuffle inside the minibatch;
 * both permutations are keyed bijections so v(S) is a deterministic function of
 * (S, seed) whatever the batch composition.
 */
#ifndef MPLC_HIP_CNN_H
#define MPLC_HIP_CNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* parameter row layout (floats) */
#define MPLC_CNN_OFF_W1 0          /* 3*3*1*32   */
#define MPLC_CNN_OFF_B1 288        /* 32         */
#define MPLC_CNN_OFF_W2 320        /* 3*3*32*64  */
#define MPLC_CNN_OFF_B2 18752      /* 64         */
#define MPLC_CNN_OFF_W3 18816      /* 9216*128   */
#define MPLC_CNN_OFF_B3 1198464    /* 128        */
#define MPLC_CNN_OFF_W4 1198592    /* 128*10     */
#define MPLC_CNN_OFF_B4 1199872    /* 10         */
#define MPLC_CNN_NPARAM 1199882
#define MPLC_CNN_STRIDE 1199936    /* row stride, multiple of 64 floats */
#define MPLC_PROF_ALL (-1)         /* mplc_cnn_train_t.prof_kernel: time every launch of the step */
#define MPLC_PROF_KERNELS 7
#define MPLC_PHASE_FRONT 1
#define MPLC_PHASE_DENSE 2
#define MPLC_PHASE_BACK 4
#define MPLC_CNN_W1_BANDS 3        /* data-gradient blocks per sample (64 Winograd tiles each) */
#define MPLC_CNN_W2T 32768         /* per-model W2 workspace: 16 Winograd planes x 32 x 64 floats */
#define MPLC_CNN_FEAT 9216         /* flattened pooled features */
#define MPLC_CNN_HID 128
#define MPLC_CNN_NCLS 10
#define MPLC_CNN_W1P 320           /* per-sample partial gradient of W1+b1 */
#define MPLC_CNN_W2P 18496         /* partial gradient row of W2+b2 */

/* replica kinds */
#define MPLC_REP_IDLE (-1)
#define MPLC_REP_FEDAVG 0     /* member of a FedAvg coalition: M rounds per epoch, fresh Adam per round */
#define MPLC_REP_SINGLE 1     /* singleton coalition: Keras fit over all rows, E epochs, persistent Adam  */
#define MPLC_REP_SEQ 2        /* sequential coalition model (seq-pure / seq-with-final-agg / seqavg): one
                               * model per coalition trained on its members' minibatches one after the
                               * other in a per-round shuffled member order, one optimizer per round
                               * (mplc/multi_partner_learning.py:337-433).  For this kind n_rows = member
                               * count k, rows_off = offset of the coalition's k member records in `seq`,
                               * batch = max member batch size, key = member-order key. */
#define MPLC_SEQ_REC 6        /* member record in `seq`: n_rows, batch, rows_off, split_off, key lo, key hi */

typedef struct {
  int32_t kind;       /* MPLC_REP_*                                                      */
  int32_t n_rows;     /* partner train size n_p                                          */
  int32_t batch;      /* partner batch size bs_p (mplc/scenario.py:705-724)              */
  int32_t rows_off;   /* offset of the partner's dataset row indices in `rows`           */
  int32_t split_off;  /* offset of the partner's M+1 minibatch boundaries in `splits`    */
  int32_t model;      /* index of the replica's parameter row                            */
  uint64_t key;       /* shuffle key (seed, coalition, partner)                          */
} mplc_replica_t;     /* 32 bytes */

typedef struct {
  /* geometry */
  int32_t n_rep;          /* replicas                                                     */
  int32_t bmax;           /* max batch size over replicas (slot stride)                   */
  int32_t w2_splits;      /* = ceil(bmax / mplc_cnn_wgrad_split_samples()): conv2 weight- */
                          /* gradient splits of that many samples per replica (9)           */
  int32_t pad0;
  /* schedule (global step -> per-replica samples) */
  int32_t step;           /* global step index                                            */
  int32_t minibatch_count;/* M                                                            */
  int32_t round_len;      /* steps per FedAvg round (max over replicas)                   */
  int32_t epochs;         /* E                                                            */
  const mplc_replica_t* reps;
  const int32_t* rows;    /* concatenated partner row indices into x/labels               */
  const int32_t* splits;  /* concatenated minibatch boundaries, M+1 per partner           */
  const int32_t* seq;     /* MPLC_REP_SEQ member records (NULL when there are none)        */
  /* data */
  const float* x;         /* [N][28][28] fp32 in [0,1]                                    */
  const int32_t* labels;  /* [N] class ids                                                */
  /* model state */
  float* params;          /* [n_rep][MPLC_CNN_STRIDE]                                     */
  float* adam_m;
  float* adam_v;
  /* workspaces (device) */
  int32_t* idx;           /* [n_rep][bmax]                                                */
  int32_t* cnt;           /* [n_rep]                                                      */
  int32_t* adam_t;        /* [n_rep]  (0 = idle this step)                                */
  float* pooled;          /* [n_rep][bmax][9216]                                          */
  uint8_t* code;          /* [n_rep][bmax][9216] argmax-in-window | 0x80 if positive      */
  float* hidden;          /* [n_rep][bmax][128]                                           */
  float* dhidden;         /* [n_rep][bmax][128]                                           */
  float* dpooled;         /* [n_rep][bmax][9216]                                          */
  float* w1_part;         /* [n_rep][bmax][MPLC_CNN_W1_BANDS][MPLC_CNN_W1P]: one [dW1 | db1]   */
                          /* partial per sample and band of output tiles                    */
  float* w2_part;         /* [n_rep][w2_splits][MPLC_CNN_W2P]                             */
  float* w2t;             /* [n_rep][MPLC_CNN_W2T]: W2 in Winograd form for the forward   */
                          /* conv, then the rotated kernel's Winograd form for the dgrad     */
  /* optimizer (Keras 2.3.1 Adam) */
  float lr, beta1, beta2, eps;
  /* optional in-stream timing of one kernel of the step (bench roofline): hipEvent_t recorded right
   * before / after launch number prof_kernel (1 conv_fwd, 2 dense_fwd, 3 head, 4 dense1_bwd_adam,
   * 5 conv_bwd_data, 6 conv_wgrad, 7 adam_small); 0 or NULL events = off.  prof_kernel = MPLC_PROF_ALL (-1):
   * every launch k is timed, prof_begin / prof_end then point to hipEvent_t arrays of MPLC_PROF_KERNELS + 1
   * entries indexed by k */
  int32_t prof_kernel;
  /* Which launches of the step to issue (bit mask; 0 = all, the whole step): MPLC_PHASE_FRONT = schedule,
   * W2 Winograd form, conv_fwd; MPLC_PHASE_DENSE = dense_fwd, head, dense1_bwd_adam; MPLC_PHASE_BACK = the
   * rotated W2, conv_bwd_data, conv_wgrad, adam_small.  Issuing the phases of one step separately, in order,
   * on one stream is the same computation; the host may interleave the phases of two replica ranges on two
   * streams (MFMA-bound convolutions beside the HBM-bound dense layer). */
  int32_t phases;
  void* prof_begin;
  void* prof_end;
  /* optional training history (NULL = off): per replica, the step's [sum of per-sample CE before the
   * update, correct predictions, samples] - the running 'loss' / 'accuracy' that a Keras fit reports
   * (mplc/multi_partner_learning.py:130-133 log_partner_perf); idle replicas write zeros */
  double* hstats;         /* [n_rep][3]                                                   */
  /* optional (NULL = off): FedAvg replicas read W3 at the first step of a round (Adam t = 1) from their
   * coalition's row of glob instead of their own row, which the round's aggregation then need not
   * overwrite (mplc_fedavg_aggregate_bcast_skip with [MPLC_CNN_OFF_W3, MPLC_CNN_OFF_B3)).  The step
   * writes the updated W3 into the replica's own row as usual. */
  const float* glob;      /* [n_coalitions][MPLC_CNN_STRIDE] coalition models                    */
  const int32_t* rep_glob;  /* [n_rep] replica -> its coalition's row of glob                 */
  int32_t* w3src;         /* [n_rep] workspace: glob row W3 is read from this step, or -1      */
  /* optional (ABI 4; avg_n = 0: off): the last step of a FedAvg round with W3's data-volume average fused into
   * the dense pass (replaces the W3 part of mplc_fedavg_aggregate, mplc/mpl_utils.py:90-115).  For each of the
   * avg_n coalitions (replicas avg_first[2c] .. avg_first[2c + 1] - 1, contiguous) the step computes every member's
   * updated W3 as usual and writes np.average of them - fp64 products x * avg_w[r] added in replica order, divided
   * by avg_scale[c], rounded once - into row avg_glob[c] of avg_out, not into the replicas' rows; the host then
   * aggregates the other layers with mplc_fedavg_aggregate_skip over [MPLC_CNN_OFF_W3, MPLC_CNN_OFF_B3).
   * avg_rep[r] != 0 marks the replicas of those coalitions.  Only a round's last step may carry it. */
  int32_t avg_n;
  int32_t pad1;
  const int32_t* avg_first;  /* [2 avg_n] the coalitions' replica ranges (begin, end)           */
  const double* avg_w;       /* [n_rep] the replica's aggregation weight (data volume / uniform)  */
  const double* avg_scale;   /* [avg_n] the coalition's sum of weights                          */
  const int32_t* avg_glob;   /* [avg_n] the coalition's row of avg_out                          */
  float* avg_out;            /* coalition rows (the same array as glob)                         */
  const int32_t* avg_rep;    /* [n_rep]                                                         */
} mplc_cnn_train_t;

/* Parameter row stride in floats (== MPLC_CNN_STRIDE). */
int mplc_cnn_stride(void);

/* Samples per conv2 weight-gradient split: mplc_cnn_train_t.w2_splits must be ceil(bmax / this). */
int mplc_cnn_wgrad_split_samples(void);

/* Layout query (ABI check at load): the value of item `what` (MPLC_CNN_Q_*) as this library was built, or -1
 * for an unknown item.  The host compares every item with its own constants and refuses a mismatched pair. */
#define MPLC_CNN_Q_STRIDE 0
#define MPLC_CNN_Q_NPARAM 1
#define MPLC_CNN_Q_FEAT 2
#define MPLC_CNN_Q_HID 3
#define MPLC_CNN_Q_W1P 4
#define MPLC_CNN_Q_W2P 5
#define MPLC_CNN_Q_W2T 6
#define MPLC_CNN_Q_W1_BANDS 7
#define MPLC_CNN_Q_WG_SAMPLES 8
#define MPLC_CNN_Q_PROF_KERNELS 9
#define MPLC_CNN_Q_TRAIN_T_BYTES 10    /* sizeof(mplc_cnn_train_t) */
#define MPLC_CNN_Q_REPLICA_T_BYTES 11  /* sizeof(mplc_replica_t)   */
#define MPLC_CNN_Q_COUNT 12
int64_t mplc_cnn_layout(int what);

/* glorot_uniform kernels / zero biases for n_models rows, keyed per model (deterministic counter RNG). */
int mplc_cnn_init_params(float* params, int64_t stride, const uint64_t* keys, int n_models, void* stream);

/* dst[i] = src[map[i]] row copies (start of training: replica rows <- coalition global rows). */
int mplc_cnn_copy_rows(float* dst, const float* src, int64_t stride, const int32_t* map, int n_rows,
                       void* stream);

/* Enqueue one lockstep training step of all replicas (schedule, forward, backward, Adam). */
int mplc_cnn_train_step(const mplc_cnn_train_t* t, void* stream);

/* Sequential approaches: after step `step`, copy params[r] into snap[snap_first[r] + i] for every
 * MPLC_REP_SEQ replica r whose member i (ascending partner order) finished its minibatch fit at this step
 * (partner.model_weights = model.get_weights(), mplc/multi_partner_learning.py:372-374).  The schedule
 * arguments are those of the train step. */
int mplc_seq_snapshot(const float* params, int64_t stride, int64_t n_param, const mplc_replica_t* reps, int n_rep,
                      const int32_t* seq, const int32_t* splits, int step, int minibatch_count, int round_len,
                      int epochs, const int32_t* snap_first, float* snap, void* stream);

/* Forward-only evaluation of n_models models on samples [0, n_samples) of x/labels:
 * correct[m] += #argmax hits, loss_sum[m] += sum of per-sample CE (float64: per
 * block of 256 samples a fixed tree, the blocks added in sample order; with every chunk but the last a multiple
 * of 256 the sum does not depend on chunk or n_models).  pooled/hidden/w2_wino are
 * workspaces of n_models * chunk * 9216, n_models * chunk * 128 and n_models * MPLC_CNN_W2T floats. */
int mplc_cnn_evaluate(const float* params, int64_t stride, int n_models, const float* x, const int32_t* labels,
                      int n_samples, int chunk, float* pooled, float* hidden, float* w2_wino, int32_t* correct,
                      double* loss_sum, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MPLC_HIP_CNN_H */
