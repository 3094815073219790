// Keyed counters shared by the batched trainers (bit-identical restatements in oracle/cnn.py and
// oracle/cifar_cnn.py): splitmix64 finaliser, keyed bijections of [0, n), and the per-replica sample
// schedule of one lockstep step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mplc_hip_cnn.h"

namespace {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t subkey(uint64_t key, uint32_t a, uint32_t b) {
  return mix64(key ^ mix64(((uint64_t)a << 32) | (uint64_t)b));
}

// Bijection of [0, n) (balanced 4-round Feistel on 2h bits + cycle walking).
__device__ __forceinline__ uint32_t keyed_perm(uint64_t key, uint32_t n, uint32_t i) {
  if (n <= 1) return 0;
  int bits = 32 - __clz(n - 1);  // ceil(log2 n)
  const int h = (bits + 1) >> 1;
  const uint32_t mask = (1u << h) - 1u;
  uint32_t x = i;
  do {
    uint32_t L = x >> h, R = x & mask;
#pragma unroll
    for (int rd = 0; rd < 4; ++rd) {
      const uint32_t F = (uint32_t)mix64(key ^ ((uint64_t)rd << 40) ^ (uint64_t)R) & mask;
      const uint32_t nl = R;
      R = L ^ F;
      L = nl;
    }
    x = (L << h) | R;
  } while (x >= n);
  return x;
}

// One replica slot of one lockstep step: how many samples the replica trains on (c), its optimizer
// iteration (at; 0 = idle), the dataset row of slot j (-1 if j >= c) and the step's dropout key.
//  FedAvg member: step -> (epoch e, round m, Keras step t) with round_len steps per round; the round's
//    samples are the epoch permutation of the partner's rows (PartnerMpl.split_minibatches,
//    mplc/partner.py:155-167) cut at the minibatch bounds, then Keras' per-fit shuffle.
//  Singleton: step -> (epoch e, step t) of one Keras fit over all rows, persistent optimizer.
struct SlotSched {
  int c, at, row;
  uint64_t dkey;
};

// Sequential coalition model at one step: which member trains (index mi in ascending partner order), the
// Keras step tl inside that member's fit, its step count ns, and the member record.  Round (e, m) visits
// the members in the keyed order keyed_perm(subkey(key, 0x60000 + e, m), k, .) (the reference draws
// np.random.permutation(partners_count), mplc/multi_partner_learning.py:365); each member fit runs
// ceil(L / bs) steps on its minibatch m, back to back from the start of the round.
struct SeqPos {
  int e, m, t, mi, tl, ns;
  const int32_t* rec;
};

__device__ __forceinline__ bool seq_locate(const mplc_replica_t& rep, int step, int M, int round_len, int epochs,
                                           const int32_t* __restrict__ splits, const int32_t* __restrict__ seq,
                                           SeqPos& p) {
  const int per_epoch = M * round_len;
  p.e = step / per_epoch;
  if (p.e >= epochs) return false;
  const int rem = step % per_epoch;
  p.m = rem / round_len;
  p.t = rem % round_len;
  const int k = rep.n_rows;
  const uint64_t okey = subkey(rep.key, 0x60000u + (uint32_t)p.e, (uint32_t)p.m);
  int acc = 0;
  for (int idx = 0; idx < k; ++idx) {
    const int mi = (int)keyed_perm(okey, (uint32_t)k, (uint32_t)idx);
    const int32_t* rec = seq + rep.rows_off + MPLC_SEQ_REC * mi;
    const int L = splits[rec[3] + p.m + 1] - splits[rec[3] + p.m];
    const int ns = (L + rec[1] - 1) / rec[1];
    if (p.t < acc + ns) {
      p.mi = mi;
      p.tl = p.t - acc;
      p.ns = ns;
      p.rec = rec;
      return true;
    }
    acc += ns;
  }
  return false;  // this coalition's round is shorter than round_len: idle
}

__device__ __forceinline__ SlotSched schedule_slot(const mplc_replica_t& rep, int j, int step, int M, int round_len,
                                                   int epochs, const int32_t* __restrict__ rows,
                                                   const int32_t* __restrict__ splits,
                                                   const int32_t* __restrict__ seq) {
  SlotSched s{0, 0, -1, 0ull};
  if (rep.kind == MPLC_REP_SEQ) {
    SeqPos p;
    if (seq_locate(rep, step, M, round_len, epochs, splits, seq, p)) {
      const int32_t* rec = p.rec;
      const int n_rows = rec[0], batch = rec[1], rows_off = rec[2], split_off = rec[3];
      const uint64_t mkey = (uint64_t)(uint32_t)rec[4] | ((uint64_t)(uint32_t)rec[5] << 32);
      const int s0 = splits[split_off + p.m];
      const int L = splits[split_off + p.m + 1] - s0;
      s.c = min(batch, L - p.tl * batch);
      s.at = p.t + 1;  // one optimizer for the whole round: its iterations run on across the members
      s.dkey = subkey(mkey, 0x40000u + (uint32_t)p.e, ((uint32_t)p.m << 16) | (uint32_t)p.tl);
      if (j < s.c) {
        const uint32_t q = keyed_perm(subkey(mkey, 0x20000u + (uint32_t)p.e, (uint32_t)p.m), (uint32_t)L,
                                      (uint32_t)(p.tl * batch + j));
        const uint32_t pos = keyed_perm(subkey(mkey, 0x10000u + (uint32_t)p.e, 0u), (uint32_t)n_rows,
                                        (uint32_t)s0 + q);
        s.row = rows[rows_off + (int)pos];
      }
    }
  } else if (rep.kind == MPLC_REP_FEDAVG) {
    const int per_epoch = M * round_len;
    const int e = step / per_epoch;
    const int rem = step % per_epoch;
    const int m = rem / round_len;
    const int t = rem % round_len;
    if (e < epochs) {
      const int s0 = splits[rep.split_off + m];
      const int s1 = splits[rep.split_off + m + 1];
      const int L = s1 - s0;
      const int nsteps = (L + rep.batch - 1) / rep.batch;
      if (t < nsteps) {
        s.c = min(rep.batch, L - t * rep.batch);
        s.at = t + 1;
        s.dkey = subkey(rep.key, 0x40000u + (uint32_t)e, ((uint32_t)m << 16) | (uint32_t)t);
        if (j < s.c) {
          const uint32_t q = keyed_perm(subkey(rep.key, 0x20000u + (uint32_t)e, (uint32_t)m), (uint32_t)L,
                                        (uint32_t)(t * rep.batch + j));
          const uint32_t pos = keyed_perm(subkey(rep.key, 0x10000u + (uint32_t)e, 0u), (uint32_t)rep.n_rows,
                                          (uint32_t)s0 + q);
          s.row = rows[rep.rows_off + (int)pos];
        }
      }
    }
  } else if (rep.kind == MPLC_REP_SINGLE) {
    const int spe = (rep.n_rows + rep.batch - 1) / rep.batch;
    const int e = step / spe;
    const int t = step % spe;
    if (e < epochs) {
      s.c = min(rep.batch, rep.n_rows - t * rep.batch);
      s.at = step + 1;
      s.dkey = subkey(rep.key, 0x50000u + (uint32_t)e, (uint32_t)t);
      if (j < s.c) {
        const uint32_t pos = keyed_perm(subkey(rep.key, 0x30000u + (uint32_t)e, 0u), (uint32_t)rep.n_rows,
                                        (uint32_t)(t * rep.batch + j));
        s.row = rows[rep.rows_off + (int)pos];
      }
    }
  }
  return s;
}

}  // namespace
