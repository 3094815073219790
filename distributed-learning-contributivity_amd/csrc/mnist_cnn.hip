// Batched multi-model MNIST CNN trainer for gfx950 (see include/mplc_hip_cnn.h for the contract).
//
// One lockstep step of B replicas = 10 launches:
//   schedule        per replica: this step's sample rows, batch count, Adam step     (index work)
//   winograd_w2     W2 in Winograd form (G g G^T per input/output channel pair)
//   conv_fwd        conv1 (recomputed, MFMA) -> conv2 in Winograd form F(2x2,3x3) on fp32 MFMA 16x16x4 (one
//                   output tile = one pooling window) -> +b, ReLU, 2x2 max-pool -> pooled + argmax code
//   dense_fwd       Dense(128)+ReLU: per-replica GEMM [b x 9216] x [9216 x 128], fp32 MFMA
//   head            Dense(10), softmax-CE gradient, dW4/db4 + Adam, dh = dlogits W4^T * relu'
//   dense1_bwd_adam per 32-row slice of W3: dp = dh W3^T, dW3 = p^T dh, Adam(W3) in the same pass
//                   (W3 = 98% of the parameters: read once, written once per step)
//   winograd_w2r    W2 rotated by 180 degrees, channels swapped, in Winograd form (dgrad B operand)
//   conv_bwd_data   dA1 = dZ2 (*) W2 in Winograd form F(2x2,3x3) on MFMA, V built directly from (dp, argmax
//                   code) of the 2x2 pooling windows a tile's patch covers; ReLU' of the recomputed conv1
//                   output and conv1's weight gradient fused in the epilogue
//   conv_wgrad      dW2 = A1^T dZ2 on MFMA over all pixels of a replica's samples (split-K partials)
//   adam_small      Adam on W1/b1/W2/b2 from the per-sample / per-split partials (fixed order: bitwise
//                   reproducible)
// Everything is fp32 (the reference's Keras float32), accumulation on the exact-f32 MFMA.
// conv1's output (86.5 KB/sample) is never written to HBM: it is recomputed (9 MACs/element) by the
// three kernels that need it.
#include "mnist_common.h"

namespace {

// ------------------------------------------------------------------------------------------------
// Initialisation: glorot_uniform kernels (Keras default), zero biases / padding.
// u = top 24 bits of mix64(key + i*golden) / 2^24;  w = (2u - 1) * limit  (fp32, exact restatable)
// ------------------------------------------------------------------------------------------------
__global__ void init_params_kernel(float* __restrict__ params, int64_t stride, const uint64_t* __restrict__ keys) {
  const int m = blockIdx.y;
  const uint64_t key = keys[m];
  float* row = params + (int64_t)m * stride;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < stride; i += (int64_t)gridDim.x * blockDim.x) {
    float lim = 0.0f;
    int64_t li = 0;
    if (i < OFF_B1) { lim = 0x1.23170ep-3f; li = i - OFF_W1; }
    else if (i >= OFF_W2 && i < OFF_B2) { lim = 0x1.555556p-4f; li = i - OFF_W2; }
    else if (i >= OFF_W3 && i < OFF_B3) { lim = 0x1.9f2c4cp-6f; li = i - OFF_W3; }
    else if (i >= OFF_W4 && i < OFF_B4) { lim = 0x1.ab099ap-3f; li = i - OFF_W4; }
    float w = 0.0f;
    if (lim != 0.0f) {
      const uint64_t hsh = mix64(key + (uint64_t)i * 0x9E3779B97F4A7C15ull);
      const float u = (float)(uint32_t)(hsh >> 40) * 0x1p-24f;
      w = (u * 2.0f - 1.0f) * lim;
    }
    (void)li;
    row[i] = w;
  }
}

__global__ void copy_rows_kernel(float* __restrict__ dst, const float* __restrict__ src, int64_t stride,
                                 const int32_t* __restrict__ map) {
  const int r = blockIdx.y;
  const float4* s = reinterpret_cast<const float4*>(src + (int64_t)map[r] * stride);
  float4* d = reinterpret_cast<float4*>(dst + (int64_t)r * stride);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < stride / 4; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

// ------------------------------------------------------------------------------------------------
// Schedule: global step -> per-replica sample rows (reference sample order, keyed permutations)
// ------------------------------------------------------------------------------------------------
__global__ void schedule_kernel(const mplc_replica_t* __restrict__ reps, int n_rep, int bmax,
                                const int32_t* __restrict__ rows, const int32_t* __restrict__ splits,
                                const int32_t* __restrict__ seq, int step,
                                int M, int round_len, int epochs, int32_t* __restrict__ idx,
                                int32_t* __restrict__ cnt, int32_t* __restrict__ adam_t,
                                const int32_t* __restrict__ rep_glob, int32_t* __restrict__ w3src) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)n_rep * bmax) return;
  const int r = (int)(gid / bmax);
  const int j = (int)(gid % bmax);
  const SlotSched ss = schedule_slot(reps[r], j, step, M, round_len, epochs, rows, splits, seq);
  const int c = ss.c, at = ss.at, row = ss.row;
  idx[gid] = row;
  if (j == 0) {
    cnt[r] = c;
    // the optimizer's last step: its next step is idle or starts a fresh optimizer (slot index bmax: no row
    // lookup, only the step's count and Adam iteration)
    const SlotSched nx = schedule_slot(reps[r], bmax, step + 1, M, round_len, epochs, rows, splits, seq);
    adam_t[r] = at | ((at > 0 && nx.at != at + 1) ? ADAM_LAST : 0);
    // a FedAvg partner's first step of a round starts from the coalition model: W3 from its glob row
    if (w3src) w3src[r] = (reps[r].kind == MPLC_REP_FEDAVG && at == 1) ? rep_glob[r] : -1;
  }
}

// ------------------------------------------------------------------------------------------------
// conv2 in Winograd form F(2x2, 3x3) (Lavin & Gray): per 4x4 input patch d and 3x3 kernel g,
//   Y[2x2] = A^T [ (G g G^T) (.) (B^T d B) ] A,   with one output tile = one 2x2 max-pool window.
// W2 is transformed once per model and step: U[xi = 4i + j][ci][co] = (G g G^T)[i][j] (winograd_w2_kernel).
// The conv becomes 16 independent GEMMs M[xi][tile][co] = sum_ci V[xi][tile][ci] U[xi][ci][co]: 2.25x fewer
// multiply-adds than the direct convolution (16 x 32 x 64 per tile of 4 outputs instead of 4 x 288 x 64).
// All arithmetic stays fp32 (the transforms are sums, differences and halvings; MFMA accumulation is f32).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void wino_g_rows(const float (&g)[3], float (&o)[4]) {  // o = G g (one column)
  o[0] = g[0];
  o[1] = 0.5f * ((g[0] + g[1]) + g[2]);
  o[2] = 0.5f * ((g[0] - g[1]) + g[2]);
  o[3] = g[2];
}

__global__ __launch_bounds__(256) void winograd_w2_kernel(const float* __restrict__ params, int64_t stride,
                                                          const int32_t* __restrict__ cnt, float* __restrict__ U) {
  const int r = blockIdx.y;
  if (cnt && cnt[r] == 0) return;
  const int e = blockIdx.x * 256 + threadIdx.x;  // (ci, co)
  if (e >= C1 * C2) return;
  const float* W2 = params + (int64_t)r * stride + OFF_W2 + e;  // [kyx][ci][co]: tap k at W2[k * C1 * C2]
  float g[3][3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) g[ky][kx] = W2[(ky * 3 + kx) * C1 * C2];
  float gg[4][3];  // G g: rows i, columns kx
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const float col[3] = {g[0][kx], g[1][kx], g[2][kx]};
    float o[4];
    wino_g_rows(col, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) gg[i][kx] = o[i];
  }
  float* Ur = U + (int64_t)r * MPLC_CNN_W2T + e;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float o[4];
    wino_g_rows(gg[i], o);  // (G g) G^T: row i
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) Ur[(4 * i + jj) * C1 * C2] = o[jj];
  }
}

// ------------------------------------------------------------------------------------------------
// conv1 (recompute) + conv2 (Winograd, MFMA) + bias + ReLU + 2x2 max-pool.  Block = (third of the image:
// 4 pool rows = 48 tiles, group of FWD_SPB samples, model), 4 waves; the block walks its samples in order.
// Wave i owns transform row i (xi = 4i .. 4i+3) of the three 16-tile groups x 4 channel groups: 48
// accumulators of v_mfma_f32_16x16x4_f32 (tile x co), K = 32 input channels in 8 steps of 4.  The wave's B
// operands (its transform row of U: 128 values) are loaded into registers once per block and serve every
// group of every sample; A operands (V) are computed in registers from the LDS conv1 tile (8 reads and 8 adds
// give a lane its 4 values of V for one (tile, ci)), software-pipelined one k-step ahead.  The next sample's
// image rows are loaded into registers while the current sample's GEMMs run.  Output: each wave folds its row
// of the output transform (T_i = M_i A, 2 values per (tile, co)) into LDS; then Y = sum_i A^T[.][i] T_i + bias,
// the max over the window (first max in scan order) and ReLU, written with the argmax code.
// ------------------------------------------------------------------------------------------------
constexpr int FWD_THREADS = 256;
constexpr int FWD_PR = 4;                          // pool rows per block
constexpr int FWD_PARTS = PL / FWD_PR;             // blocks per image
constexpr int FWD_C1R = 2 * FWD_PR + 2;            // conv1 rows per block
constexpr int FWD_IMR = FWD_C1R + 2;               // image rows per block
constexpr int FWD_C1T = (FWD_C1R * A1 + 31) / 32;  // conv1 tiles (9)
constexpr int FWD_TILES = FWD_PR * PL;             // 48 Winograd tiles (= pool windows) per block
constexpr int FWD_TS = C2 + 4;  // tile stride of a T plane: a half-wave writes tile quads kq, kq + 1 (4 TS apart) on opposite
                                // bank halves (4 TS = 16 mod 32; 65 gave 2-way conflicts): -1.5 %, bit-identical
constexpr int FWD_TQ = 16 * FWD_TS;                // one (row i, b) plane of T for a 16-tile group
constexpr int FWD_NIT = (FWD_IMR * IMG + FWD_THREADS - 1) / FWD_THREADS;  // image values per thread
constexpr int FWD_SPB = 9;  // samples per block (config #3's bs 27 = 3 groups; 3: +1 %, 14 / 27: +1.2 % / +3 %)

__global__ __launch_bounds__(FWD_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) CONV_REGS void conv_fwd_kernel(
    const float* __restrict__ x, const int32_t* __restrict__ idx, int row_base, const int32_t* __restrict__ cnt,
    int cnt_all, int bmax, const float* __restrict__ params, int64_t stride, const float* __restrict__ U,
    float* __restrict__ pooled, uint8_t* __restrict__ code) {
  __shared__ float img_s[2][FWD_IMR * IMG];  // double-buffered: the next sample's image goes in beside the current
  // padded to whole conv1 tiles: unconditional writes (rows >= 260 unread).  (Its rows padded to 12 (mod 16) floats
  // - conflict-free patch reads, as conv_bwd_data's - spilled 33 registers: the address arithmetic of the conv1
  // epilogue, p A1P + 2 (p / 26) per value, round 6)
  __shared__ float a1_s[FWD_C1T * 32 * A1P];
  __shared__ float t_s[8 * FWD_TQ];  // [i][b][16 tiles][64 co]
  const int64_t lb = xcd_block();  // logical block (part, sample group, r), replica-major
  const int part = (int)(lb % FWD_PARTS);
  const int jg = (int)((lb / FWD_PARTS) % gridDim.y);
  const int r = (int)(lb / ((int64_t)FWD_PARTS * gridDim.y));
  const int count = cnt ? cnt[r] : cnt_all;
  const int j_begin = jg * FWD_SPB;
  const int j_end = min(count, j_begin + FWD_SPB);
  if (j_begin >= j_end) return;
  const int tid = threadIdx.x;
  const float* P = params + (int64_t)r * stride;
  float imv[FWD_NIT];  // a sample's image rows, loaded one sample ahead
  auto load_img = [&](int jj) {
    const int row = idx ? idx[(int64_t)r * bmax + jj] : row_base + jj;
    const float* xs = x + (int64_t)row * (IMG * IMG) + part * 2 * FWD_PR * IMG;
#pragma unroll
    for (int k = 0; k < FWD_NIT; ++k) {
      const int e = tid + FWD_THREADS * k;
      imv[k] = xs[e < FWD_IMR * IMG ? e : 0];
    }
  };
  load_img(j_begin);
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int m = lane & 31;
  const int kh = lane >> 5;
  float w1r[5];
  load_w1r(P, kh, m, w1r);
  // ---- Winograd GEMM roles: wave = transform row i; lane (tl = lane & 15, kq = lane >> 4)
  const int wi = wave;
  const int tl = lane & 15, kq = lane >> 4;
  // B^T row i combines two input rows: t = d[ry] + sx d[rx] (row 0: d0 - d2, 1: d1 + d2, 2: d2 - d1, 3: d1 - d3),
  // one fused multiply-add by +-1 per value: the product is exact, so it rounds once, as the add or subtract does
  // (a VALU instruction costs an f32 MFMA stream 2.5-3.5 cycles, DESIGN.md 7f: this was a multiply and an fma)
  const int ry = (wi == 0) ? 0 : (wi == 2) ? 2 : 1;
  const int rx = (wi == 3) ? 3 : (wi == 2) ? 1 : 2;
  const float sx = (wi == 1) ? 1.0f : -1.0f;
  const int drow = (rx - ry) * A1 * A1P;
  // the wave's B operands of all 8 k-steps (its transform row of U), resident for the whole block
  const float* Ub = U + (int64_t)r * MPLC_CNN_W2T + (int64_t)(4 * wi) * C1 * C2 + kq * C2 + tl;
  const float bias = P[OFF_B2 + (tid & 63)];  // the output phase's channel co = tid & 63 in every pass
  float bw[8][16];
#pragma unroll
  for (int st = 0; st < 8; ++st)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int cg = 0; cg < 4; ++cg) bw[st][4 * jj + cg] = Ub[(int64_t)jj * C1 * C2 + (4 * st) * C2 + 16 * cg];
  auto store_img = [&](float* dst) {
#pragma unroll
    for (int k = 0; k < FWD_NIT; ++k)
      if (tid + FWD_THREADS * k < FWD_IMR * IMG) dst[tid + FWD_THREADS * k] = imv[k];
  };
  store_img(img_s[0]);
  if (j_begin + 1 < j_end) load_img(j_begin + 1);  // in flight during the first sample
  __syncthreads();
#pragma unroll 1
  for (int j = j_begin; j < j_end; ++j) {
    // a1_s is free (the previous sample's last two barriers follow its last GEMM read); this sample's image is
    // in img_s[b] since before the previous sample's barriers
    const int b = (j - j_begin) & 1;
    // conv1 + ReLU for local rows 0..FWD_C1R-1 (global 2*FWD_PR*part + lr): FWD_C1T MFMA tiles over 4 waves
    constexpr int NPOS1 = FWD_C1R * A1;
#pragma unroll
    for (int u = 0; u < (FWD_C1T + 3) / 4; ++u) {
      const int t = wave + 4 * u;
      if (t < FWD_C1T) {  // wave-uniform
        const int p = min(t * 32 + m, NPOS1 - 1);
        const floatx16 a = conv1_mfma(img_s[b], (p / A1) * IMG + p % A1, kh, w1r);
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int pw = t * 32 + acc_row(reg, kh);
          a1_s[pw * A1P + m] = fmaxf(a[reg], 0.0f);
        }
      }
    }
    if (j + 1 < j_end) {  // img_s[b ^ 1] was last read by the previous sample's conv1, two barriers ago
      store_img(img_s[b ^ 1]);
      if (j + 2 < j_end) load_img(j + 2);
    }
    __syncthreads();
    float* outp = pooled + ((int64_t)r * bmax + j) * FEAT;
    uint8_t* outc = code ? code + ((int64_t)r * bmax + j) * FEAT : nullptr;
#pragma unroll 1
    for (int g = 0; g < 3; ++g) {  // one 16-tile group at a time
      const int tile = 16 * g + tl;
      // this lane's patch origin (row 2ty + ry, col 2tx) in a1_s, + channel kq
      const int pa = ((2 * (tile / PL) + ry) * A1 + 2 * (tile % PL)) * A1P + kq;
      fvec4 acc[4][4];  // [j][channel group]
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int cg = 0; cg < 4; ++cg) acc[jj][cg] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
      // Software-pipelined k-loop: the next k-step's 8 patch values are read at the start of a k-step and
      // pinned (empty asm: the compiler cannot hoist their use) after its first two MFMA chunks, so that their
      // LDS latency is covered and the next k-step's V arithmetic fills the last two chunks' MFMA gaps.
      float pn[8];
      auto load_patch = [&](int st) {
        const float* d0 = a1_s + pa + 4 * st;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          pn[c] = d0[c * A1P];
          pn[4 + c] = d0[drow + c * A1P];
        }
      };
      auto make_v = [&](float (&v)[4]) {
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) t[c] = __builtin_fmaf(sx, pn[4 + c], pn[c]);
        v[0] = t[0] - t[2];
        v[1] = t[1] + t[2];
        v[2] = t[2] - t[1];
        v[3] = t[1] - t[3];
      };
      float vc[4], vn[4];
      load_patch(0);
      make_v(vc);
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        if (st + 1 < 8) load_patch(st + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          if (jj == 2) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(pn[k]));
          }
#pragma unroll
          for (int cg = 0; cg < 4; ++cg) acc[jj][cg] = mfma16(vc[jj], bw[st][4 * jj + cg], acc[jj][cg]);
        }
        if (st + 1 < 8) make_v(vn);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 4; ++q) vc[q] = vn[q];
      }
      // T_i[b] = sum_j M_ij A[j][b]: T_i0 = M_i0 + M_i1 + M_i2, T_i1 = M_i1 - M_i2 - M_i3.  Lane holds tiles
      // 4*kq + rr (rr = 0..3) of the group, channel 16*cg + tl.
#pragma unroll
      for (int cg = 0; cg < 4; ++cg)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const float m0 = acc[0][cg][rr], m1 = acc[1][cg][rr], m2 = acc[2][cg][rr], m3 = acc[3][cg][rr];
          const int o = (4 * kq + rr) * FWD_TS + 16 * cg + tl;
          t_s[(2 * wi) * FWD_TQ + o] = (m0 + m1) + m2;
          t_s[(2 * wi + 1) * FWD_TQ + o] = (m1 - m2) - m3;
        }
      __syncthreads();
      // Y[a][b] = sum_i A^T[a][i] T_i[b]: Y0b = T0b + T1b + T2b, Y1b = T1b - T2b - T3b; window pixel q = 2a + b
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int o = tid + FWD_THREADS * k;  // (tile in group, co)
        const int co = o & 63;
        const int tile_o = 16 * g + (o >> 6);
        float tv[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) tv[i][bb] = t_s[(2 * i + bb) * FWD_TQ + (o >> 6) * FWD_TS + co];
        float z[4];
        z[0] = ((tv[0][0] + tv[1][0]) + tv[2][0]) + bias;
        z[1] = ((tv[0][1] + tv[1][1]) + tv[2][1]) + bias;
        z[2] = ((tv[1][0] - tv[2][0]) - tv[3][0]) + bias;
        z[3] = ((tv[1][1] - tv[2][1]) - tv[3][1]) + bias;
        float best = z[0];
        int arg = 0;
#pragma unroll
        for (int qq = 1; qq < 4; ++qq)
          if (z[qq] > best) { best = z[qq]; arg = qq; }
        const int py = FWD_PR * part + tile_o / PL, px = tile_o % PL;
        const int pidx = (py * PL + px) * C2 + co;
        outp[pidx] = fmaxf(best, 0.0f);
        if (outc) outc[pidx] = (uint8_t)(arg | (best > 0.0f ? 0x80 : 0));
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Dense(128) + ReLU:  H[r][m][n] = relu(sum_k A[r][m][k] W3[r][k][n] + b3[n]).  Block = 32 rows x 128.
// ------------------------------------------------------------------------------------------------
constexpr int DF_K = 64;

__global__ __launch_bounds__(256) void dense_fwd_kernel(const float* __restrict__ A, int64_t a_rstride,
                                                        const int32_t* __restrict__ cnt, int cnt_all, int bmax,
                                                        const float* __restrict__ params, int64_t stride,
                                                        const float* __restrict__ glob,
                                                        const int32_t* __restrict__ w3src, float* __restrict__ H) {
  __shared__ float a_s[32 * (DF_K + 1)];
  const int r = blockIdx.y;
  const int m0 = blockIdx.x * 32;
  const int count = cnt ? cnt[r] : cnt_all;
  if (m0 >= count) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int n0 = wave * 32;
  const int kh = lane >> 5;
  const float* Ar = A + (int64_t)r * a_rstride;
  const int gsrc = w3src ? w3src[r] : -1;  // W3 of a round's first step: the coalition row (not broadcast)
  const float* W = (gsrc >= 0 ? glob + (int64_t)gsrc * stride : params + (int64_t)r * stride) + OFF_W3;
  floatx16 acc = zero16();
  // software pipeline over K chunks: the next chunk's A tile (8 values per thread) and W3 column slice
  // (32 values per lane) are loaded into registers while this chunk's 32 MFMAs run, so neither the LDS
  // staging nor the MFMA chain ever waits on a single exposed load
  constexpr int AIT = 32 * DF_K / 256;
  const float* wl = W + n0 + (lane & 31) + (int64_t)kh * HID;
  float av[AIT], bv[DF_K / 2];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
      const int e = tid + 256 * i;
      const int mm = e / DF_K, kk = e % DF_K;
      const bool ok = m0 + mm < count;
      const float t = Ar[(int64_t)(ok ? m0 + mm : m0) * FEAT + k0 + kk];
      av[i] = ok ? t : 0.0f;
    }
#pragma unroll
    for (int s = 0; s < DF_K / 2; ++s) bv[s] = wl[(int64_t)(k0 + 2 * s) * HID];
  };
  load(0);
  for (int k0 = 0; k0 < FEAT; k0 += DF_K) {
    __syncthreads();  // previous chunk's readers done
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
      const int e = tid + 256 * i;
      a_s[(e / DF_K) * (DF_K + 1) + e % DF_K] = av[i];
    }
    float bc[DF_K / 2];
#pragma unroll
    for (int s = 0; s < DF_K / 2; ++s) bc[s] = bv[s];
    load(min(k0 + DF_K, FEAT - DF_K));  // the last chunk re-loads itself (uniform, branch-free)
    __syncthreads();
#pragma unroll
    for (int s = 0; s < DF_K / 2; ++s) acc = mfma32(a_s[(lane & 31) * (DF_K + 1) + 2 * s + kh], bc[s], acc);
  }
  const float bias = params[(int64_t)r * stride + OFF_B3 + n0 + (lane & 31)];
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * kh;
    if (m0 + row < count)
      H[((int64_t)r * bmax + m0 + row) * HID + n0 + (lane & 31)] = fmaxf(acc[reg] + bias, 0.0f);
  }
}

// ------------------------------------------------------------------------------------------------
// Keras 2.3.1 Adam (fresh state when t == 1: FedAvg builds a new optimizer per partner fit)
// ------------------------------------------------------------------------------------------------
// adam_t[r] = the replica's Adam iteration t (1-based; 0 = idle) | ADAM_LAST on the optimizer's last step
struct AdamCfg {
  float lr_t, b1, b2, eps;
  int t;
  bool reset, last;
};

__device__ __forceinline__ AdamCfg adam_cfg(int t_flags, float lr, float b1, float b2, float eps) {
  AdamCfg c;
  c.t = t_flags & ~ADAM_LAST;
  const float tf = (float)c.t;
  c.lr_t = lr * (sqrtf(1.0f - powf(b2, tf)) / (1.0f - powf(b1, tf)));
  c.b1 = b1;
  c.b2 = b2;
  c.eps = eps;
  c.reset = (c.t == 1);
  c.last = (t_flags & ADAM_LAST) != 0;
  return c;
}

// The moments after a fresh optimizer's first step, m1 = (1 - b1) g and v1 = (1 - b2) g^2, are functions of
// that step's gradient alone: dense1_bwd_adam stores g there and rebuilds m1, v1 from it at step 2 with
// this same routine (bit-identical), which halves the moment traffic of those two steps.
__device__ __forceinline__ void adam_first_moments(float g, const AdamCfg& c, float& m1, float& v1) {
  m1 = __fmul_rn(1.0f - c.b1, g);
  v1 = __fmul_rn(1.0f - c.b2, __fmul_rn(g, g));
}

// Every operation rounded on its own, in Keras' order (keras/optimizers.py Adam.get_updates; oracle/cnn.py
// KerasAdam): m_t = (b1 m) + ((1 - b1) g), v_t = (b2 v) + ((1 - b2) g^2), p - (lr_t m_t) / (sqrt(v_t) + eps).  Under
// hipcc's default fp-contract=fast, `b1 * m + (1 - b1) * g` may become fma(b1, m, (1 - b1) g) OR fma(1 - b1, g, b1 m)
// - two roundings of the same sum, and which one the backend picks depended on the code around the inlined call: a
// refactor of dense1_bwd_adam_kernel that left its FP instruction multiset unchanged moved the MNIST models in their
// last bits (profiles/r06_adam_contraction.txt).  Contraction off here (as rms_apply, cifar_common.h; the __*_rn
// intrinsics do not stop the backend fusing) pins one rounding per operation.
__device__ __forceinline__ void adam_apply(float& p, float& m, float& v, float g, const AdamCfg& c) {
#pragma clang fp contract(off)
  float mt, vt;
  if (c.reset) {
    adam_first_moments(g, c, mt, vt);
  } else {
    mt = c.b1 * m + (1.0f - c.b1) * g;
    vt = c.b2 * v + (1.0f - c.b2) * (g * g);
  }
  p = p - c.lr_t * mt / (sqrtf(vt) + c.eps);
  m = mt;
  v = vt;
}

// ------------------------------------------------------------------------------------------------
// Head: Dense(10) + softmax-CE gradient (mean over the batch), dW4/db4 + Adam, dh = dlogits W4^T * relu'
// One block per replica.
// ------------------------------------------------------------------------------------------------
constexpr int HEAD_CHUNK = 256;

__global__ __launch_bounds__(256) void head_kernel(const float* __restrict__ H, const int32_t* __restrict__ idx,
                                                   const int32_t* __restrict__ labels, const int32_t* __restrict__ cnt,
                                                   const int32_t* __restrict__ adam_t, int bmax,
                                                   float* __restrict__ params, float* __restrict__ adam_m,
                                                   float* __restrict__ adam_v, int64_t stride,
                                                   float* __restrict__ dH, float lr, float b1, float b2, float eps,
                                                   double* __restrict__ hstats) {
  __shared__ float w4_s[HID * NCLS + NCLS];
  __shared__ float dl_s[HEAD_CHUNK * NCLS];
  __shared__ double hs_s[2][HEAD_CHUNK];
  const int r = blockIdx.x;
  const int count = cnt[r];
  const int tid = threadIdx.x;
  if (count == 0) {
    if (hstats && tid < 3) hstats[(int64_t)r * 3 + tid] = 0.0;
    return;
  }
  float* P = params + (int64_t)r * stride;
  for (int e = tid; e < HID * NCLS + NCLS; e += 256) w4_s[e] = P[OFF_W4 + e];
  __syncthreads();
  const float inv_b = 1.0f / (float)count;
  float gacc[6] = {0, 0, 0, 0, 0, 0};  // dW4 elements tid, tid+256, ... (1290 = W4 + b4)
  double hl = 0.0, hc = 0.0;           // this thread's training CE / correct sums (hstats)
  const float* Hr = H + (int64_t)r * bmax * HID;
  for (int c0 = 0; c0 < count; c0 += HEAD_CHUNK) {
    const int cn = min(HEAD_CHUNK, count - c0);
    if (tid < cn) {
      const int jj = c0 + tid;
      const float* h = Hr + (int64_t)jj * HID;
      float z[NCLS];
#pragma unroll
      for (int o = 0; o < NCLS; ++o) z[o] = w4_s[HID * NCLS + o];
      for (int c = 0; c < HID; ++c) {
        const float hv = h[c];
#pragma unroll
        for (int o = 0; o < NCLS; ++o) z[o] += hv * w4_s[c * NCLS + o];
      }
      const int y = labels[idx[(int64_t)r * bmax + jj]];
      int am = 0;  // first maximum (the evaluation's argmax)
      float mx = z[0];
#pragma unroll
      for (int o = 1; o < NCLS; ++o)
        if (z[o] > mx) { mx = z[o]; am = o; }
      float zy = z[0];
#pragma unroll
      for (int o = 1; o < NCLS; ++o) zy = (o == y) ? z[o] : zy;
      float s = 0.0f;
#pragma unroll
      for (int o = 0; o < NCLS; ++o) { z[o] = expf(z[o] - mx); s += z[o]; }
      hl += (double)(logf(s) + mx - zy);
      hc += (am == y) ? 1.0 : 0.0;
#pragma unroll
      for (int o = 0; o < NCLS; ++o) dl_s[tid * NCLS + o] = (z[o] / s - (o == y ? 1.0f : 0.0f)) * inv_b;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = tid + 256 * u;
      if (e < HID * NCLS) {
        const int c = e / NCLS, o = e % NCLS;
        float a = 0.0f;
        for (int jj = 0; jj < cn; ++jj) a += Hr[(int64_t)(c0 + jj) * HID + c] * dl_s[jj * NCLS + o];
        gacc[u] += a;
      } else if (e < HID * NCLS + NCLS) {
        const int o = e - HID * NCLS;
        float a = 0.0f;
        for (int jj = 0; jj < cn; ++jj) a += dl_s[jj * NCLS + o];
        gacc[u] += a;
      }
    }
    for (int e = tid; e < cn * HID; e += 256) {
      const int jj = e / HID, c = e % HID;
      const float hv = Hr[(int64_t)(c0 + jj) * HID + c];
      float a = 0.0f;
#pragma unroll
      for (int o = 0; o < NCLS; ++o) a += dl_s[jj * NCLS + o] * w4_s[c * NCLS + o];
      dH[((int64_t)r * bmax + c0 + jj) * HID + c] = hv > 0.0f ? a : 0.0f;
    }
    __syncthreads();
  }
  if (hstats) {  // the step's training loss / accuracy sums before the update (Keras fit history)
    hs_s[0][tid] = hl;
    hs_s[1][tid] = hc;
    __syncthreads();
    for (int off = HEAD_CHUNK / 2; off >= 1; off >>= 1) {
      if (tid < off) { hs_s[0][tid] += hs_s[0][tid + off]; hs_s[1][tid] += hs_s[1][tid + off]; }
      __syncthreads();
    }
    if (tid == 0) {
      hstats[(int64_t)r * 3] = hs_s[0][0];
      hstats[(int64_t)r * 3 + 1] = hs_s[1][0];
      hstats[(int64_t)r * 3 + 2] = (double)count;
    }
  }
  const AdamCfg cfg = adam_cfg(adam_t[r], lr, b1, b2, eps);
  float* Mr = adam_m + (int64_t)r * stride;
  float* Vr = adam_v + (int64_t)r * stride;
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const int e = tid + 256 * u;
    if (e < HID * NCLS + NCLS) {
      const int64_t o = OFF_W4 + e;  // W4 and b4 are contiguous
      float p = P[o], mm = Mr[o], vv = Vr[o];
      adam_apply(p, mm, vv, gacc[u], cfg);
      P[o] = p;
      Mr[o] = mm;
      Vr[o] = vv;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Dense(128) backward + Adam, per 32-row slice of W3 (block = 256 threads: row = tid/8, 16 cols each)
// dp[j][k] = sum_c dh[j][c] W3[k][c];  dW3[k][c] = sum_j p[j][k] dh[j][c];  db3 (slice 0 block)
// ------------------------------------------------------------------------------------------------
#ifndef MPLC_D1_MFMA
#define MPLC_D1_MFMA 0  // dense1_bwd_adam_mfma_kernel (bit-identical MFMA form) instead of the VALU form: -4.7 % on the
                        // 1260-replica probe but +1.9 % at the bench's 5120 replicas (memory-bound there), so off
#endif
constexpr int D1_ROWS = 32;    // W3 rows per block (8 threads per row)
constexpr int D1_SCHUNK = 32;  // samples staged in LDS at a time

// One replica's pass over one 32-row slice of W3 (the body of dense1_bwd_adam_kernel, shared with the fused
// averaging kernel below): dp rows written, W3's moments read / written by the optimizer step, b3 updated by the
// slice-0 block; the updated slice is returned in w (lane's fvec4 chunks c8 + 8 i) and, when Wout is given, stored
// there as each chunk is updated (the standalone kernel: its stores interleaved with the moments' stores, as before
// the slice was shared - storing after the b3 update instead cost the kernel 6 %, scripts/r06/gpu22.sh).
__device__ __forceinline__ void dense1_replica_slice(
    int r, int k0, int count, const float* __restrict__ Pool, const float* __restrict__ dH,
    const int32_t* __restrict__ adam_t, int bmax, float* __restrict__ params, float* __restrict__ adam_m,
    float* __restrict__ adam_v, int64_t stride, const float* __restrict__ glob, const int32_t* __restrict__ w3src,
    float* __restrict__ dPool, float lr, float b1, float b2, float eps, fvec4* dh_s, float* p_s, fvec4 (&w)[4],
    fvec4* Wout) {
  const int tid = threadIdx.x;
  const int rowl = tid >> 3;
  // the 8 threads of a row own interleaved fvec4 chunks q = c8 + 8*i (columns 4q..4q+3): each global
  // access instruction covers 128 contiguous bytes per row, each dh_s read 8 adjacent 16-B slots
  const int c8 = tid & 7;
  const AdamCfg cfg = adam_cfg(adam_t[r], lr, b1, b2, eps);
  // W3's moments: a fresh optimizer's first step (t = 1) reads none and stores its gradient g1 in the m slot
  // (not m1 and v1); step 2 reads g1 back and rebuilds m1, v1 (adam_first_moments); from step 3 on m and v
  // are read and written as usual; an optimizer's last step writes neither (the next step starts fresh)
  const bool fresh = cfg.reset, second = (cfg.t == 2);
  const int64_t roff = (int64_t)r * stride + OFF_W3 + (int64_t)(k0 + rowl) * HID;
  const fvec4* W = reinterpret_cast<const fvec4*>(params + roff) + c8;
  // a round's first step reads W3 from the coalition row (the aggregation did not broadcast it)
  const int gsrc = w3src ? w3src[r] : -1;
  const fvec4* Wsrc = gsrc >= 0 ? reinterpret_cast<const fvec4*>(glob + roff + (int64_t)(gsrc - r) * stride) + c8 : W;
  fvec4* Mr = reinterpret_cast<fvec4*>(adam_m + roff) + c8;
  fvec4* Vr = reinterpret_cast<fvec4*>(adam_v + roff) + c8;
  const fvec4 z4 = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  // every HBM read of the pass is issued up front; the moments land while the gradient is accumulated
  fvec4 g[4], mv[4], vv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = Wsrc[8 * i];
    g[i] = z4;
    mv[i] = z4;
    vv[i] = z4;
  }
  if (second) {
#pragma unroll
    for (int i = 0; i < 4; ++i) mv[i] = __builtin_nontemporal_load(Mr + 8 * i);  // g1
  } else if (!fresh) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mv[i] = __builtin_nontemporal_load(Mr + 8 * i);
      vv[i] = __builtin_nontemporal_load(Vr + 8 * i);
    }
  }
  const float* Pr = Pool + (int64_t)r * bmax * FEAT;
  const fvec4* dHr = reinterpret_cast<const fvec4*>(dH + (int64_t)r * bmax * HID);
  float* dPr = dPool + (int64_t)r * bmax * FEAT;
  for (int c0 = 0; c0 < count; c0 += D1_SCHUNK) {
    const int cn = min(D1_SCHUNK, count - c0);
    {  // every staging load in flight before the first LDS store (clamped index, no branch on the load)
      constexpr int HIT = D1_SCHUNK * (HID / 4) / 256, PIT = D1_SCHUNK * D1_ROWS / 256;
      fvec4 hv[HIT];
      float pv[PIT];
#pragma unroll
      for (int i = 0; i < HIT; ++i) {
        const int e = tid + 256 * i;
        hv[i] = dHr[(int64_t)c0 * (HID / 4) + (e < cn * (HID / 4) ? e : 0)];
      }
#pragma unroll
      for (int i = 0; i < PIT; ++i) {
        const int e = tid + 256 * i;
        const int jj = e < cn * D1_ROWS ? e / D1_ROWS : 0;
        pv[i] = Pr[(int64_t)(c0 + jj) * FEAT + k0 + e % D1_ROWS];
      }
#pragma unroll
      for (int i = 0; i < HIT; ++i)
        if (tid + 256 * i < cn * (HID / 4)) dh_s[tid + 256 * i] = hv[i];
#pragma unroll
      for (int i = 0; i < PIT; ++i)
        if (tid + 256 * i < cn * D1_ROWS) p_s[tid + 256 * i] = pv[i];
    }
    __syncthreads();
#pragma unroll 2
    for (int jj = 0; jj < cn; ++jj) {
      const float pv = p_s[jj * D1_ROWS + rowl];
      float d = 0.0f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const fvec4 dh = dh_s[jj * (HID / 4) + c8 + 8 * i];
        g[i].x += pv * dh.x; g[i].y += pv * dh.y; g[i].z += pv * dh.z; g[i].w += pv * dh.w;
        d += dh.x * w[i].x; d += dh.y * w[i].y; d += dh.z * w[i].z; d += dh.w * w[i].w;
      }
      d += dpp_partner<DPP_XOR1>(d);
      d += dpp_partner<DPP_XOR2>(d);
      d += dpp_partner<DPP_HALF_MIRROR>(d);
      if (c8 == 0) dPr[(int64_t)(c0 + jj) * FEAT + k0 + rowl] = d;
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    fvec4 pw = w[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float p1 = pw[q], m1 = mv[i][q], v1 = vv[i][q];
      if (second) adam_first_moments(mv[i][q], cfg, m1, v1);
      adam_apply(p1, m1, v1, g[i][q], cfg);
      pw[q] = p1;
      mv[i][q] = m1;
      vv[i][q] = v1;
    }
    w[i] = pw;
    if (Wout) Wout[8 * i] = pw;
    if (!cfg.last) {
      if (fresh) {
        __builtin_nontemporal_store(g[i], Mr + 8 * i);
      } else {
        __builtin_nontemporal_store(mv[i], Mr + 8 * i);
        __builtin_nontemporal_store(vv[i], Vr + 8 * i);
      }
    }
  }
  if (k0 == 0 && tid < HID) {  // the replica's slice-0 block (logical order)
    float gb = 0.0f;
    const float* dHs = dH + (int64_t)r * bmax * HID;
    for (int jj = 0; jj < count; ++jj) gb += dHs[(int64_t)jj * HID + tid];
    const int64_t o = (int64_t)r * stride + OFF_B3 + tid;
    adam_apply(params[o], adam_m[o], adam_v[o], gb, cfg);
  }
}

__global__ __launch_bounds__(256) void dense1_bwd_adam_kernel(
    const float* __restrict__ Pool, const float* __restrict__ dH, const int32_t* __restrict__ cnt,
    const int32_t* __restrict__ adam_t, int bmax, float* __restrict__ params, float* __restrict__ adam_m,
    float* __restrict__ adam_v, int64_t stride, const float* __restrict__ glob, const int32_t* __restrict__ w3src,
    float* __restrict__ dPool, float lr, float b1, float b2, float eps, const int32_t* __restrict__ avg_rep) {
  __shared__ fvec4 dh_s[D1_SCHUNK * (HID / 4)];
  __shared__ float p_s[D1_SCHUNK * D1_ROWS];
  const int64_t lb = xcd_block();  // logical block (slice, r), replica-major: dh and p stay in one L2
  const int r = (int)(lb / gridDim.x);
  const int k0 = (int)(lb % gridDim.x) * D1_ROWS;
  const int count = cnt[r];
  if (count == 0) return;
  if (avg_rep && avg_rep[r]) return;  // this step's pass of r belongs to dense1_bwd_adam_avg_kernel
  fvec4 w[4];
  fvec4* W = reinterpret_cast<fvec4*>(params + (int64_t)r * stride + OFF_W3 + (int64_t)(k0 + (threadIdx.x >> 3)) * HID) +
             (threadIdx.x & 7);
  dense1_replica_slice(r, k0, count, Pool, dH, adam_t, bmax, params, adam_m, adam_v, stride, glob, w3src, dPool, lr,
                       b1, b2, eps, dh_s, p_s, w, W);
}

// The last step of a FedAvg round with the coalition's W3 average fused in.
// Block = (32-row slice, fused coalition c): the coalition's replicas in order, each the pass of
// dense1_bwd_adam_kernel (the same code: dp rows, b3), and instead of storing the replica's updated slice, its
// np.average term: s = x_0 w_0, then s = s + x_r w_r in replica order in fp64, one division by the weights' sum,
// one rounding to fp32 - mplc_fedavg_aggregate's arithmetic (no contraction), written to the coalition row.  The
// replicas' own W3 rows are neither written here nor read by the aggregation (mplc_fedavg_aggregate_skip leaves
// W3 out), and the next round's first step reads W3 from the coalition row (w3src): every replica W3 store of the
// round's last step and the aggregation's W3 reads disappear.  A member without a step this time (it finished
// its round's fit earlier: fewer rows) enters with its own row, as the aggregation would read it.
#ifndef MPLC_D1AVG_WAVES
// waves per SIMD: 3 (168 VGPRs, 2 spilled) against the unconstrained 2 (172 VGPRs): 96.7 -> 84.7 ms over the config #3
// probe's 40 launches, bit-identical (profiles/r06_ab_avgw.txt).  Still ~0.4 of HBM: each block walks its
// coalition's replicas one after the other (load, stage, reduce, update per replica)
#define MPLC_D1AVG_WAVES 3
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MPLC_D1AVG_WAVES, MPLC_D1AVG_WAVES))) void dense1_bwd_adam_avg_kernel(
    const float* __restrict__ Pool, const float* __restrict__ dH, const int32_t* __restrict__ cnt,
    const int32_t* __restrict__ adam_t, int bmax, float* __restrict__ params, float* __restrict__ adam_m,
    float* __restrict__ adam_v, int64_t stride, const float* __restrict__ glob, const int32_t* __restrict__ w3src,
    float* __restrict__ dPool, float lr, float b1, float b2, float eps, const int32_t* __restrict__ avg_first,
    const double* __restrict__ avg_w, const double* __restrict__ avg_scale, const int32_t* __restrict__ avg_glob,
    float* __restrict__ avg_out) {
#pragma clang fp contract(off)
  __shared__ fvec4 dh_s[D1_SCHUNK * (HID / 4)];
  __shared__ float p_s[D1_SCHUNK * D1_ROWS];
  const int64_t lb = xcd_block();  // logical block (slice, coalition), coalition-major
  const int c = (int)(lb / gridDim.x);
  const int k0 = (int)(lb % gridDim.x) * D1_ROWS;
  const int r0 = avg_first[2 * c], r1 = avg_first[2 * c + 1];
  const int64_t soff = OFF_W3 + (int64_t)(k0 + (threadIdx.x >> 3)) * HID;
  const int c8 = threadIdx.x & 7;
  double s[4][4];
  for (int r = r0; r < r1; ++r) {
    const int count = cnt[r];  // block-uniform
    fvec4 w[4];
    if (count == 0) {
      const fvec4* W = reinterpret_cast<const fvec4*>(params + (int64_t)r * stride + soff) + c8;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = W[8 * i];
    } else {
      dense1_replica_slice(r, k0, count, Pool, dH, adam_t, bmax, params, adam_m, adam_v, stride, glob, w3src, dPool,
                           lr, b1, b2, eps, dh_s, p_s, w, nullptr);
    }
    const double wr = avg_w[r];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) s[i][q] = (r == r0) ? (double)w[i][q] * wr : s[i][q] + (double)w[i][q] * wr;
  }
  const double scl = avg_scale[c];
  fvec4* O = reinterpret_cast<fvec4*>(avg_out + (int64_t)avg_glob[c] * stride + soff) + c8;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    O[8 * i] = fvec4{(float)(s[i][0] / scl), (float)(s[i][1] / scl), (float)(s[i][2] / scl), (float)(s[i][3] / scl)};
}

// ------------------------------------------------------------------------------------------------
// The same pass with both products on v_mfma_f32_16x16x4_f32, bit-identical to dense1_bwd_adam_kernel: the
// matrix core accumulates D = C + sum_k A[m][k] B[k][n] as the fmaf chain k = 0, 1, 2, 3 (measured on every output
// of 4096 random tiles, scripts/probes/mfma_order.hip), so MFMAs chained in the VALU loop's order reproduce it.
//   dW3: the VALU form's chain per element runs over the samples in order (g += p_j dh_j): MFMA K = 4 samples,
//        chained over sample quads; padded samples (zero p and dh) add exact zeros.
//   dp:  the VALU form's thread c8 chains the 16 columns 4 c8 + 32 i + q (i outer, q inner) and the 8 partials
//        are added in a fixed tree ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)): per c8 an MFMA chain over
//        i with K = q (4 columns), then the same tree on the 8 accumulators, in registers.
// Block = 64 rows of W3 (16 per wave) x all 128 columns.  In the MFMA layout lane (tl, kq) holds row tl and the
// columns 16 tau + 4 v + kq (tau = 0..7, v = 0..3): W3 is brought into it (and dW3 out of it, for the Adam step in
// the row layout of the coalesced 16-B accesses) through an LDS transpose once per block.  The VALU loop's 32
// multiply-adds per sample and row-thread become 2 MFMAs per 4 samples per 16 x 16 tile; the pass is left with
// its HBM traffic (W3, m, v read and written).
// ------------------------------------------------------------------------------------------------
constexpr int D1M_ROWS = 64;     // W3 rows per block (16 per wave)
constexpr int D1M_SCHUNK = 32;   // samples staged in LDS at a time (two 16-sample tiles)
constexpr int D1M_DHS = HID + 20;  // dh row stride: conflict-free for the dp operand reads (20 * m + kq)
constexpr int D1M_PS = D1M_ROWS + 16;  // p row stride
constexpr int D1M_XS = HID + 4;  // transpose scratch row stride (4 tl + kq: conflict-free)
constexpr int D1M_STAGE = D1M_SCHUNK * (D1M_DHS + D1M_PS);
constexpr int D1M_LDS = (D1M_STAGE > 4 * 16 * D1M_XS) ? D1M_STAGE : 4 * 16 * D1M_XS;
static_assert(HID == 128 && FEAT % D1M_ROWS == 0, "dense1_bwd_adam_mfma_kernel: 8 column tiles, 64-row slices");

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void dense1_bwd_adam_mfma_kernel(
    const float* __restrict__ Pool, const float* __restrict__ dH, const int32_t* __restrict__ cnt,
    const int32_t* __restrict__ adam_t, int bmax, float* __restrict__ params, float* __restrict__ adam_m,
    float* __restrict__ adam_v, int64_t stride, const float* __restrict__ glob, const int32_t* __restrict__ w3src,
    float* __restrict__ dPool, float lr, float b1, float b2, float eps, const int32_t* __restrict__ avg_rep) {
  __shared__ float smem[D1M_LDS];
  float* const dh_s = smem;                            // [sample][D1M_DHS]
  float* const p_s = smem + D1M_SCHUNK * D1M_DHS;     // [sample][D1M_PS]
  const int64_t lb = xcd_block();  // logical block (slice, r), replica-major: dh and p stay in one L2
  const int r = (int)(lb / gridDim.x);
  const int k0 = (int)(lb % gridDim.x) * D1M_ROWS;
  const int count = cnt[r];
  if (count == 0) return;
  if (avg_rep && avg_rep[r]) return;  // this step's pass of r belongs to dense1_bwd_adam_avg_kernel
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int tl = lane & 15, kq = lane >> 4;
  float* const x_s = smem + wave * 16 * D1M_XS;  // this wave's transpose scratch [16 rows][D1M_XS] (aliases staging)
  const AdamCfg cfg = adam_cfg(adam_t[r], lr, b1, b2, eps);
  const bool fresh = cfg.reset, second = (cfg.t == 2);  // moments as in dense1_bwd_adam_kernel
  // row layout: lane's fvec4 f = lane + 64 u of the wave's 16 x 32 chunks (row f / 32, columns 4 (f % 32) ..)
  const int64_t roff = (int64_t)r * stride + OFF_W3 + (int64_t)(k0 + 16 * wave) * HID;
  fvec4* W = reinterpret_cast<fvec4*>(params + roff) + lane;
  const int gsrc = w3src ? w3src[r] : -1;
  const fvec4* Wsrc = gsrc >= 0 ? reinterpret_cast<const fvec4*>(glob + roff + (int64_t)(gsrc - r) * stride) + lane : W;
  fvec4* Mr = reinterpret_cast<fvec4*>(adam_m + roff) + lane;
  fvec4* Vr = reinterpret_cast<fvec4*>(adam_v + roff) + lane;
  const fvec4 z4 = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  fvec4 w[8], mv[8], vv[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    w[u] = Wsrc[64 * u];
    mv[u] = z4;
    vv[u] = z4;
  }
  if (second) {
#pragma unroll
    for (int u = 0; u < 8; ++u) mv[u] = __builtin_nontemporal_load(Mr + 64 * u);  // g1
  } else if (!fresh) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      mv[u] = __builtin_nontemporal_load(Mr + 64 * u);
      vv[u] = __builtin_nontemporal_load(Vr + 64 * u);
    }
  }
  // W3 into the MFMA layout: wd[tau][v] = W3[row tl][16 tau + 4 v + kq]
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int f = lane + 64 * u;
    *reinterpret_cast<fvec4*>(x_s + (f >> 5) * D1M_XS + 4 * (f & 31)) = w[u];
  }
  __syncthreads();
  float wd[8][4];
#pragma unroll
  for (int tau = 0; tau < 8; ++tau)
#pragma unroll
    for (int v = 0; v < 4; ++v) wd[tau][v] = x_s[tl * D1M_XS + 16 * tau + 4 * v + kq];
  fvec4 g[8];  // dW3 in the MFMA layout: g[tau][v] = row tl, column 16 tau + 4 v + kq
#pragma unroll
  for (int tau = 0; tau < 8; ++tau) g[tau] = z4;
  const float* Pr = Pool + (int64_t)r * bmax * FEAT;
  const float* dHr = dH + (int64_t)r * bmax * HID;
  float* dPr = dPool + (int64_t)r * bmax * FEAT;
  // operand columns: g's A row m = 4 a + b is column 16 tau + 4 b + a (the output's v <-> 4 v + kq)
  const int gcol = 4 * (tl & 3) + (tl >> 2);
  for (int c0 = 0; c0 < count; c0 += D1M_SCHUNK) {
    const int cn = min(D1M_SCHUNK, count - c0);
    __syncthreads();  // the transpose reads / the previous chunk's readers are done
    {  // stage dh [32][128] and p [32][64] (zero past the chunk's samples: the padded MFMA steps add zeros)
      constexpr int HIT = D1M_SCHUNK * (HID / 4) / 256, PIT = D1M_SCHUNK * (D1M_ROWS / 4) / 256;
      fvec4 hv[HIT], pv[PIT];
#pragma unroll
      for (int i = 0; i < HIT; ++i) {
        const int e = tid + 256 * i;  // (sample e / 32, chunk e % 32)
        const bool ok = e / (HID / 4) < cn;
        const fvec4 t = *reinterpret_cast<const fvec4*>(dHr + (int64_t)(c0 + (ok ? e / (HID / 4) : 0)) * HID +
                                                        4 * (e % (HID / 4)));
        hv[i] = ok ? t : z4;
      }
#pragma unroll
      for (int i = 0; i < PIT; ++i) {
        const int e = tid + 256 * i;  // (sample e / 16, rows 4 (e % 16) ..)
        const bool ok = e / (D1M_ROWS / 4) < cn;
        const fvec4 t = *reinterpret_cast<const fvec4*>(Pr + (int64_t)(c0 + (ok ? e / (D1M_ROWS / 4) : 0)) * FEAT +
                                                        k0 + 4 * (e % (D1M_ROWS / 4)));
        pv[i] = ok ? t : z4;
      }
#pragma unroll
      for (int i = 0; i < HIT; ++i) {
        const int e = tid + 256 * i;
        float* d = dh_s + (e / (HID / 4)) * D1M_DHS + 4 * (e % (HID / 4));
        d[0] = hv[i].x;
        d[1] = hv[i].y;
        d[2] = hv[i].z;
        d[3] = hv[i].w;
      }
#pragma unroll
      for (int i = 0; i < PIT; ++i) {
        const int e = tid + 256 * i;
        *reinterpret_cast<fvec4*>(p_s + (e / (D1M_ROWS / 4)) * D1M_PS + 4 * (e % (D1M_ROWS / 4))) = pv[i];
      }
    }
    __syncthreads();
    // dW3: sample quads in order
    for (int jq = 0; jq < cn; jq += 4) {
      const float bp = p_s[(jq + kq) * D1M_PS + 16 * wave + tl];
      const float* dq = dh_s + (jq + kq) * D1M_DHS + gcol;
#pragma unroll
      for (int tau = 0; tau < 8; ++tau) g[tau] = mfma16(dq[16 * tau], bp, g[tau]);
    }
    // dp: 16-sample tiles; per c8 the chain over i (K = 4 columns), then the VALU form's tree
    for (int j0 = 0; j0 < cn; j0 += 16) {
      const float* da = dh_s + (j0 + tl) * D1M_DHS + kq;
      fvec4 pc[8];
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8) {
        pc[c8] = z4;
#pragma unroll
        for (int i = 0; i < 4; ++i)  // column 4 c8 + 32 i + kq = 16 (c8 / 4 + 2 i) + 4 (c8 % 4) + kq
          pc[c8] = mfma16(da[4 * c8 + 32 * i], wd[c8 / 4 + 2 * i][c8 % 4], pc[c8]);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {  // lane holds sample j0 + 4 kq + v, row tl
        const float d = ((pc[0][v] + pc[1][v]) + (pc[2][v] + pc[3][v])) + ((pc[4][v] + pc[5][v]) + (pc[6][v] + pc[7][v]));
        const int jj = j0 + 4 * kq + v;
        if (jj < cn) dPr[(int64_t)(c0 + jj) * FEAT + k0 + 16 * wave + tl] = d;
      }
    }
  }
  // dW3 back to the row layout through the scratch (which aliases the staging: wait for its last readers)
  __syncthreads();
#pragma unroll
  for (int tau = 0; tau < 8; ++tau)
#pragma unroll
    for (int v = 0; v < 4; ++v) x_s[tl * D1M_XS + 16 * tau + 4 * v + kq] = g[tau][v];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int f = lane + 64 * u;
    const fvec4 gr = *reinterpret_cast<const fvec4*>(x_s + (f >> 5) * D1M_XS + 4 * (f & 31));
    fvec4 pw = w[u];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float p1 = pw[q], m1 = mv[u][q], v1 = vv[u][q];
      if (second) adam_first_moments(mv[u][q], cfg, m1, v1);
      adam_apply(p1, m1, v1, gr[q], cfg);
      pw[q] = p1;
      mv[u][q] = m1;
      vv[u][q] = v1;
    }
    W[64 * u] = pw;
    if (!cfg.last) {
      if (fresh) {
        __builtin_nontemporal_store(gr, Mr + 64 * u);
      } else {
        __builtin_nontemporal_store(mv[u], Mr + 64 * u);
        __builtin_nontemporal_store(vv[u], Vr + 64 * u);
      }
    }
  }
  if (k0 == 0 && tid < HID) {  // the replica's slice-0 block (logical order)
    float gb = 0.0f;
    const float* dHs = dH + (int64_t)r * bmax * HID;
    for (int jj = 0; jj < count; ++jj) gb += dHs[(int64_t)jj * HID + tid];
    const int64_t o = (int64_t)r * stride + OFF_B3 + tid;
    adam_apply(params[o], adam_m[o], adam_v[o], gb, cfg);
  }
}

// W2 for the data gradient in Winograd form: the data gradient is the correlation of the padded dZ2 with
// the kernel rotated by 180 degrees and its channels swapped, W2r[ky][kx][co][ci] = W2[2-ky][2-kx][ci][co];
// Ur[co][ci][xi = 4i + j] = (G W2r G^T)[i][j]: the 16 transform points of one (co, ci) pair are contiguous, so
// conv_bwd_data stages a channel quarter with 16-byte copies and a lane reads its 16 B operands as 4 x b128.
__global__ __launch_bounds__(256) void winograd_w2r_kernel(const float* __restrict__ params, int64_t stride,
                                                           const int32_t* __restrict__ cnt, float* __restrict__ Ur) {
  const int r = blockIdx.y;
  if (cnt && cnt[r] == 0) return;
  const int e = blockIdx.x * 256 + threadIdx.x;  // (ci, co): consecutive lanes read consecutive co of W2
  if (e >= C1 * C2) return;
  const int ci = e / C2, co = e % C2;
  const float* W2 = params + (int64_t)r * stride + OFF_W2 + ci * C2 + co;  // tap k at W2[k * C1 * C2]
  float g[3][3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) g[ky][kx] = W2[((2 - ky) * 3 + (2 - kx)) * C1 * C2];
  float gg[4][3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const float col[3] = {g[0][kx], g[1][kx], g[2][kx]};
    float o[4];
    wino_g_rows(col, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) gg[i][kx] = o[i];
  }
  fvec4* U = reinterpret_cast<fvec4*>(Ur + (int64_t)r * MPLC_CNN_W2T + (int64_t)(co * C1 + ci) * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float o[4];
    wino_g_rows(gg[i], o);
    U[i] = fvec4{o[0], o[1], o[2], o[3]};
  }
}

// ------------------------------------------------------------------------------------------------
// conv2 data gradient + conv1 backward, Winograd F(2x2, 3x3).  dA1[y][x][ci] = sum_{ky,kx,co} dZ2p[y+ky][x+kx][co]
// W2r[ky][kx][co][ci] (dZ2p = dZ2 padded by 2) over 13 x 13 output tiles of 2x2 (row-major), as 16 GEMMs
// M[xi][tile][ci] = sum_co V[xi][tile][co] Ur[xi][co][ci], V = B^T d B of the tile's 4x4 dZ2p patch, K = 64.
// Block = (band of 64 tiles, group of BWD_SPB samples, replica), 4 waves, walking its samples in order (the next
// sample's first (dp, code) quarter and its image are loaded while the current one finishes); wave w owns
// tiles 16w .. 16w+15 of the band and ALL 16
// transform points for both 16-channel halves of ci (32 accumulators of v_mfma_f32_16x16x4_f32).  Per k-step
// (4 output channels of conv2) a lane reads its tile's 4x4 patch at one channel (16 LDS reads), forms the 16
// values of V with 32 adds and issues 32 MFMAs with B operands read from the staged Ur quarter (4 x b128 per
// half): half an LDS read per MFMA (a wave per transform row read one per MFMA: 55 % MFMA issue).
// dZ2 (the max-pool gradient: one nonzero per window, at its argmax when positive) is un-pooled from
// (dp, code) into a dense LDS band one quarter of the channels (16) at a time, with zero rows / columns around
// the 12 x 12 grid, so a patch is read without tests; Ur's quarter is staged beside it, its 4 chunks of 4
// transform points XOR-swizzled by ci so that the b128 reads of a lane group hit 64 distinct banks.
// Epilogue, wave-local: the output transform Y = A^T M A of each (tile, ci) in registers; conv1's
// pre-activation at the same positions recomputed on 16x16x4 MFMAs in the accumulator layout (taps 0..8 and
// the bias in the order of conv1_mfma, so the ReLU' mask is the forward's); dZ1 = Y * ReLU'; [dW1 | db1] +=
// patch^T dZ1 on 16x16x4 MFMAs whose B operand is dZ1 straight from registers.  One partial per (sample,
// band), the waves' partials added in a fixed order.
// ------------------------------------------------------------------------------------------------
constexpr int BWD_THREADS = 256;
constexpr int BWD_TILES = 169;                 // 13 x 13 output tiles of 2 x 2 over the 26 x 26 conv1 grid
constexpr int BWD_BAND_TILES = 64;             // tiles per block (one 16-tile group per wave)
constexpr int BWD_BANDS = MPLC_CNN_W1_BANDS;   // ceil(169 / 64) = 3
constexpr int BWD_WR = 7;                      // window rows a band's patches touch (<= 6 tile rows + 1)
constexpr int BWD_DR = 2 * BWD_WR;             // dZ2 rows staged
constexpr int BWD_DC = Z2 + 4;                 // dZ2 columns staged: 2 zero columns each side
constexpr int BWD_CS = 17;                     // channel stride (16 channels of a quarter + 1: bank spread)
// staged row stride, padded to 13 (mod 16): with BWD_CS = 1 (mod 16) tile (tyl, tx) of the 13-wide tile rows starts
// on bank 2 (13 tyl + tx) = 2 tile (mod 32), so a half-wave's 16 tiles x 2 channels cover the 32 banks once (the
// unpadded 476 put a group's wrapped tile row on its first row's banks)
constexpr int BWD_RS = BWD_DC * BWD_CS + (((13 - BWD_DC * BWD_CS) % 16) + 16) % 16;
static_assert(BWD_CS % 16 == 1 && BWD_RS % 16 == 13, "conflict-free patch reads");
constexpr int BWD_PAIRS = BWD_WR * PL * 16;    // (dp, code) pairs of a quarter
constexpr int BWD_PRE = (BWD_PAIRS + BWD_THREADS - 1) / BWD_THREADS;
constexpr int BWD_UQ = 16 * C1 * 16;           // Ur floats of one channel quarter [co 16][ci 32][xi 16]
constexpr int BWD_NIT = (IMG * IMG + BWD_THREADS - 1) / BWD_THREADS;  // image values per thread
constexpr int BWD_SPB = 1;  // samples per block (9: +2 % on the probe, the sample loop spills 13 registers)
static_assert(BWD_BANDS * BWD_BAND_TILES >= BWD_TILES && (BWD_BANDS - 1) * BWD_BAND_TILES < BWD_TILES,
              "MPLC_CNN_W1_BANDS must be ceil(169 / 64)");

__global__ __launch_bounds__(BWD_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) CONV_REGS void conv_bwd_data_kernel(
    const float* __restrict__ x, const int32_t* __restrict__ idx, const int32_t* __restrict__ cnt, int bmax,
    const float* __restrict__ params, int64_t stride, const float* __restrict__ Ur,
    const float* __restrict__ dPool, const uint8_t* __restrict__ code, float* __restrict__ w1_part) {
  __shared__ float dz_s[BWD_DR * BWD_RS];
  __shared__ fvec4 ur_s[BWD_UQ / 4];
  __shared__ float img_s[IMG * IMG];
  __shared__ float red_s[4][10 * 32];
  const int64_t lb = xcd_block();  // logical block (band, sample group, r), replica-major
  const int band = (int)(lb % BWD_BANDS);
  const int jg = (int)((lb / BWD_BANDS) % gridDim.y);
  const int r = (int)(lb / ((int64_t)BWD_BANDS * gridDim.y));
  const int j_begin = jg * BWD_SPB;
  const int j_end = min(cnt[r], j_begin + BWD_SPB);
  if (j_begin >= j_end) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int tl = lane & 15, kq = lane >> 4;
  const float* P = params + (int64_t)r * stride;
  const int tile0 = band * BWD_BAND_TILES;
  const int ty0 = tile0 / 13;
  const int wy0 = ty0 - 1;  // first window row staged (local window row 0; rows outside 0..11 stay zero)
  const int gt0 = tile0 + 16 * wave;         // this wave's first tile
  const bool active = gt0 < BWD_TILES;       // wave-uniform: the last band's last wave has no tile
  const fvec4* Uq = reinterpret_cast<const fvec4*>(Ur + (int64_t)r * MPLC_CNN_W2T);
  // pair e of a quarter: channel e & 15, window column (e >> 4) % 12, local window row e / 192
  float pdv[BWD_PRE];
  uint32_t pcd[BWD_PRE];
  auto fetch = [&](int jj, int q) {
    const float* dp = dPool + ((int64_t)r * bmax + jj) * FEAT;
    const uint8_t* cd = code + ((int64_t)r * bmax + jj) * FEAT;
#pragma unroll
    for (int s = 0; s < BWD_PRE; ++s) {
      const int e = tid + BWD_THREADS * s;
      const int wy = wy0 + e / (PL * 16);
      const bool ok = e < BWD_PAIRS && wy >= 0 && wy < PL;
      const int pidx = (wy * PL + (e >> 4) % PL) * C2 + 16 * q + (e & 15);
      pdv[s] = ok ? dp[pidx] : 0.0f;
      pcd[s] = ok ? cd[pidx] : 0u;
    }
  };
  float imv[BWD_NIT];  // a sample's image, loaded ahead of its staging into img_s
  auto load_img = [&](int jj) {
    const float* xr = x + (int64_t)idx[(int64_t)r * bmax + jj] * IMG * IMG;
#pragma unroll
    for (int k = 0; k < BWD_NIT; ++k) {
      const int e = tid + BWD_THREADS * k;
      imv[k] = xr[e < IMG * IMG ? e : 0];
    }
  };
  fetch(j_begin, 0);
  load_img(j_begin);
  {
    // zero columns (2 each side) of every staged row; the interior is rewritten by every quarter
    for (int e = tid; e < BWD_DR * 4 * BWD_CS; e += BWD_THREADS) {
      const int rr = e / (4 * BWD_CS), c = (e / BWD_CS) % 4, k = e % BWD_CS;
      dz_s[rr * BWD_RS + (c < 2 ? c : BWD_DC - 4 + c) * BWD_CS + k] = 0.0f;
    }
  }
  // A operand (V): this lane's tile tl of the wave's group at channel kq of each k-step
  const int tcl = min(gt0 + tl, BWD_TILES - 1);
  const int pa = (2 * (tcl / 13 - ty0)) * BWD_RS + 2 * (tcl % 13) * BWD_CS + kq;
  // B operand (Ur): ci = 16h + tl, co = 4st + kq of the quarter; chunk m of the 16 transform points at
  // m ^ swz (the staging applies the same XOR)
  const int swz = (tl >> 2) & 3;
#pragma unroll 1
  for (int j = j_begin; j < j_end; ++j) {
  // img_s is free: the previous sample's epilogue reads end before its reduction barrier
#pragma unroll
  for (int k = 0; k < BWD_NIT; ++k)
    if (tid + BWD_THREADS * k < IMG * IMG) img_s[tid + BWD_THREADS * k] = imv[k];
  fvec4 acc[16][2];  // [xi][ci half]
#pragma unroll
  for (int xi = 0; xi < 16; ++xi)
#pragma unroll
    for (int h = 0; h < 2; ++h) acc[xi][h] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 1
  for (int q = 0; q < 4; ++q) {  // channel quarters
    __syncthreads();             // previous quarter's readers done (and the zero columns / image written)
#ifndef BWD_EXP_NOSTAGE  // timing experiment switch (garbage results): the quarter's staging compiled out
    {
      constexpr int UIT = BWD_UQ / 4 / BWD_THREADS;  // 8 chunks of 4 floats per thread
      fvec4 uv[UIT];  // the quarter's Ur: loads in flight while the band is un-pooled
#if !defined(BWD_EXP_NOSTAGE_UR)
#pragma unroll
      for (int s = 0; s < UIT; ++s) uv[s] = Uq[q * (BWD_UQ / 4) + tid + BWD_THREADS * s];
#endif
#ifndef BWD_EXP_NOSTAGE_DZ
#pragma unroll
      for (int s = 0; s < BWD_PRE; ++s) {  // un-pool the quarter's (dp, code) into the dense band
        const int e = tid + BWD_THREADS * s;
        if (e < BWD_PAIRS) {
          const int lwy = e / (PL * 16), wx = (e >> 4) % PL, ch = e & 15;
          const uint32_t c = pcd[s];
          const float v = (c & 0x80) ? pdv[s] : 0.0f;
          const int sel = c & 3;
          float* d = dz_s + (2 * lwy) * BWD_RS + (2 + 2 * wx) * BWD_CS + ch;
          // the window's 4 pixels zeroed, then the value at the argmax (same thread, same address: in order): no
          // per-pixel compare / select chain (SGPR-mask hazards padded with s_nop in every one)
          d[0] = 0.0f;
          d[BWD_CS] = 0.0f;
          d[BWD_RS] = 0.0f;
          d[BWD_RS + BWD_CS] = 0.0f;
          d[(sel >> 1) * BWD_RS + (sel & 1) * BWD_CS] = v;
        }
      }
#endif
#ifndef BWD_EXP_NOSTAGE_UR
#pragma unroll
      for (int s = 0; s < UIT; ++s) {  // chunk k = (co, ci, m): stored at m ^ ((ci >> 2) & 3)
        const int k = tid + BWD_THREADS * s;
        const int pair = k >> 2, m = k & 3;
        ur_s[pair * 4 + (m ^ ((pair >> 2) & 3))] = uv[s];
      }
#endif
    }
#endif
    {  // the next quarter's (dp, code), or the next sample's first quarter
      const int jn = q < 3 ? j : j + 1;
      if (jn < j_end) fetch(jn, (q + 1) & 3);
    }
    __syncthreads();
    if (active) {
      // Software-pipelined k-loop (same operands, same per-accumulator order: bit-identical results).  The
      // 32 MFMAs of a k-step run as 4 chunks of 8 (transform row i = chunk m: xi = 4m .. 4m+3, both ci
      // halves); during chunk m the B operands of the next chunk are read, and the next k-step's patch is
      // read in chunk 0 and turned into its V one transform row per chunk, so that every LDS read has a
      // chunk of MFMAs (256 cycles) to land and the VALU sits in the MFMA gaps.
      const float* dq = dz_s + pa;
      float pn[16];  // next k-step's 4x4 patch, [row][col]
      auto load_patch = [&](int st) {
#pragma unroll
        for (int rr2 = 0; rr2 < 4; ++rr2)
#pragma unroll
          for (int c = 0; c < 4; ++c) pn[4 * rr2 + c] = dq[4 * st + rr2 * BWD_RS + c * BWD_CS];
      };
      // transform row i of V from the patch: t_i[c] = (B^T d)[i][c], then v[4i + j] = (t_i B)[j]
      auto v_row = [&](int i, float (&v)[16]) {
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float d_0 = pn[c], d_1 = pn[4 + c], d_2 = pn[8 + c], d_3 = pn[12 + c];
          t[c] = (i == 0) ? d_0 - d_2 : (i == 1) ? d_1 + d_2 : (i == 2) ? d_2 - d_1 : d_1 - d_3;
        }
        v[4 * i + 0] = t[0] - t[2];
        v[4 * i + 1] = t[1] + t[2];
        v[4 * i + 2] = t[2] - t[1];
        v[4 * i + 3] = t[1] - t[3];
      };
      auto load_b = [&](int st, int m, fvec4 (&b)[2]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) b[h] = ur_s[((4 * st + kq) * C1 + 16 * h + tl) * 4 + (m ^ swz)];
      };
      float vc[16], vn[16];
      load_patch(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) v_row(i, vc);
      fvec4 bc[2], bn[2];
      load_b(0, 0, bc);
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        if (st < 3) load_patch(st + 1);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          if (m < 3) load_b(st, m + 1, bn);
          else if (st < 3) load_b(st + 1, 0, bn);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            // the patch values "change" here (an empty asm the compiler cannot see through), so the V
            // arithmetic of row m cannot be hoisted above this chunk and fills its MFMA gaps; in chunk 0
            // the pin sits after two MFMA pairs, which cover the patch reads issued just before
            if (x == (m == 0 ? 2 : 0)) {
              if (m == 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(pn[k]));
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[4 * m + x][h] = mfma16(vc[4 * m + x], bc[h][x], acc[4 * m + x][h]);
          }
          if (st < 3) v_row(m, vn);
          __builtin_amdgcn_sched_barrier(0);
          bc[0] = bn[0];
          bc[1] = bn[1];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) vc[i] = vn[i];
      }
    }
  }
  // ---- epilogue (wave-local).  Lane (tl, kq) holds M[xi][tile 4kq + rr][ci 16h + tl] in acc[xi][h][rr].
  if (j + 1 < j_end) load_img(j + 1);  // in flight during the epilogue
  // conv1 weights as the B operand of the 16x16x4 recompute: W1e[4s + kq][16h + tl], rows 0..8 = taps, 9 = bias
  float w1b[3][2];
#pragma unroll
  for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 4 * s3 + kq, ci = 16 * h + tl;
      w1b[s3][h] = (k < 9) ? P[OFF_W1 + k * C1 + ci] : ((k == 9) ? P[OFF_B1 + ci] : 0.0f);
    }
  fvec4 gacc = fvec4{0.0f, 0.0f, 0.0f, 0.0f};  // [dW1 | db1] partial: rows = tap 4kq + reg, col = ci 16h + tl
  fvec4 gacc1 = gacc;
#ifdef BWD_EXP_NOEPI  // timing experiment: the epilogue compiled out (the accumulators still consumed)
  if (active) {
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) gacc += acc[xi][0] + acc[xi][1];
  }
  if (false) {
#else
  if (active) {
#endif
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      // positions of the MFMA rows m = 4 kq' + q: tile 4kq' + rr of the group, window pixel q = 2a + b
      // A operands for this lane as a row (m = tl): its position's taps 4s + kq (conv1) ...
      const int tA = min(gt0 + 4 * (tl >> 2) + rr, BWD_TILES - 1);
      const int pyA = 2 * (tA / 13) + ((tl & 3) >> 1), pxA = 2 * (tA % 13) + (tl & 1);
      float a1v[3];
#pragma unroll
      for (int s3 = 0; s3 < 3; ++s3) {
        const int k = 4 * s3 + kq;
        a1v[s3] = (k < 9) ? img_s[(pyA + k / 3) * IMG + pxA + k % 3] : ((k == 9) ? 1.0f : 0.0f);
      }
      // ... and as a K index (k = kq) for dW1: position (tile 4kq + rr, q), tap tl
      const int tB = gt0 + 4 * kq + rr;
      const bool valid = tB < BWD_TILES && tB < tile0 + BWD_BAND_TILES;
      const int tBc = min(tB, BWD_TILES - 1);
      fvec4 z[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        fvec4 c1 = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) c1 = mfma16(a1v[s3], w1b[s3][h], c1);
        // output transform of (tile 4kq + rr, ci 16h + tl): T_i = M_i A, Y = A^T T
        float tv[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float m0 = acc[4 * i][h][rr], m1 = acc[4 * i + 1][h][rr], m2 = acc[4 * i + 2][h][rr],
                      m3 = acc[4 * i + 3][h][rr];
          tv[i][0] = (m0 + m1) + m2;
          tv[i][1] = (m1 - m2) - m3;
        }
        float y[4];
        y[0] = (tv[0][0] + tv[1][0]) + tv[2][0];
        y[1] = (tv[0][1] + tv[1][1]) + tv[2][1];
        y[2] = (tv[1][0] - tv[2][0]) - tv[3][0];
        y[3] = (tv[1][1] - tv[2][1]) - tv[3][1];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) z[h][qq] = (valid && c1[qq] > 0.0f) ? y[qq] : 0.0f;
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        // A: tap tl of position (tile 4kq + rr, q = qq); 1 for the bias row, 0 beyond
        const int py = 2 * (tBc / 13) + (qq >> 1), px = 2 * (tBc % 13) + (qq & 1);
        const float pv = (tl < 9) ? img_s[(py + tl / 3) * IMG + px + tl % 3] : 0.0f;
        const float av = (tl < 9) ? pv : ((tl == 9) ? 1.0f : 0.0f);
        gacc = mfma16(av, z[0][qq], gacc);
        gacc1 = mfma16(av, z[1][qq], gacc1);
      }
    }
  }
  // gacc / gacc1: rows = tap 4kq + reg (0..9 used), col = ci tl / 16 + tl
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int k = 4 * kq + reg;
    if (k < 10) {
      red_s[wave][k * 32 + tl] = gacc[reg];
      red_s[wave][k * 32 + 16 + tl] = gacc1[reg];
    }
  }
  __syncthreads();
  float* out = w1_part + (((int64_t)r * bmax + j) * BWD_BANDS + band) * MPLC_CNN_W1P;
  for (int e = tid; e < 10 * 32; e += BWD_THREADS)
    out[e] = (red_s[0][e] + red_s[1][e]) + (red_s[2][e] + red_s[3][e]);
  }  // samples
}

// Adam on W1 | b1 | W2 | b2 (params [0, 18816)) from the per-sample / per-split partial gradients.
__global__ void adam_small_kernel(const int32_t* __restrict__ cnt, const int32_t* __restrict__ adam_t, int bmax,
                                  int splits, const float* __restrict__ w1_part, const float* __restrict__ w2_part,
                                  float* __restrict__ params, float* __restrict__ adam_m, float* __restrict__ adam_v,
                                  int64_t stride, float lr, float b1, float b2, float eps) {
  const int r = blockIdx.y;
  const int count = cnt[r];
  if (count == 0) return;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= OFF_W3) return;
  float g = 0.0f;
  if (e < OFF_W2) {
    // (sample, band) order; the partials' loads issued 16 at a time ahead of their (sequential) adds
    const float* w = w1_part + (int64_t)r * bmax * BWD_BANDS * MPLC_CNN_W1P + e;
    const int n = BWD_BANDS * count;
    int jj = 0;
    for (; jj + 16 <= n; jj += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = w[(int64_t)(jj + u) * MPLC_CNN_W1P];
#pragma unroll
      for (int u = 0; u < 16; ++u) g += v[u];
    }
    for (; jj < n; ++jj) g += w[(int64_t)jj * MPLC_CNN_W1P];
  } else {
    const float* w = w2_part + (int64_t)r * splits * MPLC_CNN_W2P + (e - OFF_W2);
    const int used = (count + WG_SAMPLES - 1) / WG_SAMPLES;
    for (int s = 0; s < used; ++s) g += w[(int64_t)s * MPLC_CNN_W2P];
  }
  const AdamCfg cfg = adam_cfg(adam_t[r], lr, b1, b2, eps);
  const int64_t o = (int64_t)r * stride + e;
  adam_apply(params[o], adam_m[o], adam_v[o], g, cfg);
}

// ------------------------------------------------------------------------------------------------
// Evaluation head: logits, accuracy count and summed cross-entropy per model (deterministic order).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void eval_head_kernel(const float* __restrict__ H, int count, int chunk,
                                                        const int32_t* __restrict__ labels, int row_base,
                                                        const float* __restrict__ params, int64_t stride,
                                                        int32_t* __restrict__ correct, double* __restrict__ loss_sum) {
  __shared__ float w4_s[HID * NCLS + NCLS];
  __shared__ double ls[256];
  __shared__ int cs[256];
  const int mdl = blockIdx.x;
  const int tid = threadIdx.x;
  const float* P = params + (int64_t)mdl * stride;
  for (int e = tid; e < HID * NCLS + NCLS; e += 256) w4_s[e] = P[OFF_W4 + e];
  __syncthreads();
  // The loss is summed in fixed blocks of 256 samples (the tree below), added to the model's running total in
  // block order: with every chunk but the last a multiple of 256 samples (the host's rule), the total is the same
  // bits whatever the chunk size - and the chunk size depends on how many models share the evaluation.
  double run = (tid == 0) ? loss_sum[mdl] : 0.0;
  int csum = 0;
  for (int b0 = 0; b0 < count; b0 += 256) {
    const int jj = b0 + tid;
    double lv = 0.0;
    if (jj < count) {
      const float* h = H + ((int64_t)mdl * chunk + jj) * HID;
      float z[NCLS];
#pragma unroll
      for (int o = 0; o < NCLS; ++o) z[o] = w4_s[HID * NCLS + o];
      for (int c = 0; c < HID; ++c) {
        const float hv = h[c];
#pragma unroll
        for (int o = 0; o < NCLS; ++o) z[o] += hv * w4_s[c * NCLS + o];
      }
      int am = 0;
      float mx = z[0];
#pragma unroll
      for (int o = 1; o < NCLS; ++o)
        if (z[o] > mx) { mx = z[o]; am = o; }
      float s = 0.0f;
#pragma unroll
      for (int o = 0; o < NCLS; ++o) s += expf(z[o] - mx);
      const int y = labels[row_base + jj];
      lv = (double)(logf(s) + mx - z[y]);
      csum += (am == y) ? 1 : 0;
    }
    ls[tid] = lv;
    __syncthreads();
    for (int off = 128; off >= 1; off >>= 1) {
      if (tid < off) ls[tid] += ls[tid + off];
      __syncthreads();
    }
    if (tid == 0) run += ls[0];
    __syncthreads();  // ls is rewritten by the next block
  }
  cs[tid] = csum;
  __syncthreads();
  for (int off = 128; off >= 1; off >>= 1) {
    if (tid < off) cs[tid] += cs[tid + off];
    __syncthreads();
  }
  if (tid == 0) {
    correct[mdl] += cs[0];
    loss_sum[mdl] = run;
  }
}

inline int launch_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MPLC_OK : (int)e;
}

}  // namespace

extern "C" {

int mplc_cnn_stride(void) { return MPLC_CNN_STRIDE; }

int mplc_cnn_wgrad_split_samples(void) { return WG_SAMPLES; }

int64_t mplc_cnn_layout(int what) {
  switch (what) {
    case MPLC_CNN_Q_STRIDE: return MPLC_CNN_STRIDE;
    case MPLC_CNN_Q_NPARAM: return MPLC_CNN_NPARAM;
    case MPLC_CNN_Q_FEAT: return MPLC_CNN_FEAT;
    case MPLC_CNN_Q_HID: return MPLC_CNN_HID;
    case MPLC_CNN_Q_W1P: return MPLC_CNN_W1P;
    case MPLC_CNN_Q_W2P: return MPLC_CNN_W2P;
    case MPLC_CNN_Q_W2T: return MPLC_CNN_W2T;
    case MPLC_CNN_Q_W1_BANDS: return MPLC_CNN_W1_BANDS;
    case MPLC_CNN_Q_WG_SAMPLES: return WG_SAMPLES;
    case MPLC_CNN_Q_PROF_KERNELS: return MPLC_PROF_KERNELS;
    case MPLC_CNN_Q_TRAIN_T_BYTES: return (int64_t)sizeof(mplc_cnn_train_t);
    case MPLC_CNN_Q_REPLICA_T_BYTES: return (int64_t)sizeof(mplc_replica_t);
    default: return -1;
  }
}

int mplc_cnn_init_params(float* params, int64_t stride, const uint64_t* keys, int n_models, void* stream) {
  if (!params || !keys || n_models < 1 || n_models > 65535 || stride < MPLC_CNN_NPARAM) return MPLC_E_ARG;
  init_params_kernel<<<dim3(512, n_models), 256, 0, (hipStream_t)stream>>>(params, stride, keys);
  return launch_status();
}

int mplc_cnn_copy_rows(float* dst, const float* src, int64_t stride, const int32_t* map, int n_rows, void* stream) {
  if (!dst || !src || !map || n_rows < 1 || n_rows > 65535 || (stride & 3)) return MPLC_E_ARG;
  copy_rows_kernel<<<dim3(256, n_rows), 256, 0, (hipStream_t)stream>>>(dst, src, stride, map);
  return launch_status();
}

// In-stream kernel timing (bench.py): prof_kernel = k > 0 records the events prof_begin / prof_end around
// launch k; prof_kernel = MPLC_PROF_ALL records around every launch k, with prof_begin / prof_end then pointing
// to arrays of hipEvent_t indexed by k (1 .. MPLC_PROF_KERNELS).
static inline void prof_record(const mplc_cnn_train_t* t, int k, bool end, hipStream_t s) {
  void* ev = end ? t->prof_end : t->prof_begin;
  if (!ev) return;
  if (t->prof_kernel == k) (void)hipEventRecord((hipEvent_t)ev, s);
  else if (t->prof_kernel == MPLC_PROF_ALL) (void)hipEventRecord(static_cast<hipEvent_t*>(ev)[k], s);
}
#define PROF_BEGIN(k) prof_record(t, (k), false, s)
#define PROF_END(k) prof_record(t, (k), true, s)

int mplc_cnn_train_step(const mplc_cnn_train_t* t, void* stream) {
  if (!t || t->n_rep < 1 || t->n_rep > 65535 || t->bmax < 1) return MPLC_E_ARG;
  if (t->w2_splits != (t->bmax + WG_SAMPLES - 1) / WG_SAMPLES) return MPLC_E_SHAPE;
  if (!t->reps || !t->rows || !t->splits || !t->x || !t->labels || !t->params || !t->adam_m || !t->adam_v ||
      !t->idx || !t->cnt || !t->adam_t || !t->pooled || !t->code || !t->hidden || !t->dhidden || !t->dpooled ||
      !t->w1_part || !t->w2_part || !t->w2t)
    return MPLC_E_ARG;
  if (t->minibatch_count < 1 || t->round_len < 1 || t->epochs < 1) return MPLC_E_ARG;
  if (t->glob && (!t->rep_glob || !t->w3src)) return MPLC_E_ARG;
  if (t->phases & ~(MPLC_PHASE_FRONT | MPLC_PHASE_DENSE | MPLC_PHASE_BACK)) return MPLC_E_ARG;
  if (t->avg_n < 0 || t->avg_n > 65535 ||
      (t->avg_n > 0 && (!t->avg_first || !t->avg_w || !t->avg_scale || !t->avg_glob || !t->avg_out || !t->avg_rep)))
    return MPLC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int R = t->n_rep, B = t->bmax;
  const int64_t S = MPLC_CNN_STRIDE;
  const int64_t slots = (int64_t)R * B;
  const int ph = t->phases ? t->phases : (MPLC_PHASE_FRONT | MPLC_PHASE_DENSE | MPLC_PHASE_BACK);
  if (ph & MPLC_PHASE_FRONT) {
  schedule_kernel<<<(unsigned)((slots + 255) / 256), 256, 0, s>>>(t->reps, R, B, t->rows, t->splits, t->seq, t->step,
                                                                   t->minibatch_count, t->round_len, t->epochs,
                                                                   t->idx, t->cnt, t->adam_t, t->rep_glob,
                                                                   t->glob ? t->w3src : nullptr);
  // t->w2t holds W2 in Winograd form for the forward, then the rotated kernel's Winograd form for the dgrad
  winograd_w2_kernel<<<dim3(C1 * C2 / 256, R), 256, 0, s>>>(t->params, S, t->cnt, t->w2t);
  PROF_BEGIN(1);
  conv_fwd_kernel<<<dim3(FWD_PARTS, (B + FWD_SPB - 1) / FWD_SPB, R), FWD_THREADS, 0, s>>>(t->x, t->idx, 0, t->cnt, 0, B, t->params, S, t->w2t,
                                                         t->pooled, t->code);
  PROF_END(1);
  }
  const int32_t* w3src = t->glob ? t->w3src : nullptr;
  if (ph & MPLC_PHASE_DENSE) {
  PROF_BEGIN(2);
  dense_fwd_kernel<<<dim3((B + 31) / 32, R), 256, 0, s>>>(t->pooled, (int64_t)B * FEAT, t->cnt, 0, B, t->params, S,
                                                          t->glob, w3src, t->hidden);
  PROF_END(2);
  PROF_BEGIN(3);
  head_kernel<<<R, 256, 0, s>>>(t->hidden, t->idx, t->labels, t->cnt, t->adam_t, B, t->params, t->adam_m, t->adam_v,
                                S, t->dhidden, t->lr, t->beta1, t->beta2, t->eps, t->hstats);
  PROF_END(3);
  PROF_BEGIN(4);
  const int32_t* avg_rep = t->avg_n > 0 ? t->avg_rep : nullptr;
#if MPLC_D1_MFMA
  dense1_bwd_adam_mfma_kernel<<<dim3(FEAT / D1M_ROWS, R), 256, 0, s>>>(t->pooled, t->dhidden, t->cnt, t->adam_t, B,
                                                                       t->params, t->adam_m, t->adam_v, S, t->glob,
                                                                       w3src, t->dpooled,
                                                                       t->lr, t->beta1, t->beta2, t->eps, avg_rep);
#else
  dense1_bwd_adam_kernel<<<dim3(FEAT / D1_ROWS, R), 256, 0, s>>>(t->pooled, t->dhidden, t->cnt, t->adam_t, B,
                                                                  t->params, t->adam_m, t->adam_v, S, t->glob,
                                                                  w3src, t->dpooled,
                                                                  t->lr, t->beta1, t->beta2, t->eps, avg_rep);
#endif
  if (t->avg_n > 0)  // the round's last step of the fused coalitions: their W3 passes and the W3 average
    dense1_bwd_adam_avg_kernel<<<dim3(FEAT / D1_ROWS, t->avg_n), 256, 0, s>>>(
        t->pooled, t->dhidden, t->cnt, t->adam_t, B, t->params, t->adam_m, t->adam_v, S, t->glob, w3src, t->dpooled,
        t->lr, t->beta1, t->beta2, t->eps, t->avg_first, t->avg_w, t->avg_scale, t->avg_glob, t->avg_out);
  PROF_END(4);
  }
  if (ph & MPLC_PHASE_BACK) {
  winograd_w2r_kernel<<<dim3(C1 * C2 / 256, R), 256, 0, s>>>(t->params, S, t->cnt, t->w2t);
  PROF_BEGIN(5);
  conv_bwd_data_kernel<<<dim3(BWD_BANDS, (B + BWD_SPB - 1) / BWD_SPB, R), BWD_THREADS, 0, s>>>(t->x, t->idx, t->cnt, B, t->params, S, t->w2t, t->dpooled,
                                                          t->code, t->w1_part);
  PROF_END(5);
  PROF_BEGIN(6);
  mplc_mnist::launch_conv_wgrad(t->w2_splits, R, s, t->x, t->idx, t->cnt, B, t->params, S, t->dpooled, t->code,
                                t->w2_part);
  PROF_END(6);
  PROF_BEGIN(7);
  adam_small_kernel<<<dim3((OFF_W3 + 255) / 256, R), 256, 0, s>>>(t->cnt, t->adam_t, B, t->w2_splits, t->w1_part,
                                                                 t->w2_part, t->params, t->adam_m, t->adam_v, S,
                                                                 t->lr, t->beta1, t->beta2, t->eps);
  PROF_END(7);
  }
  return launch_status();
}

int mplc_cnn_evaluate(const float* params, int64_t stride, int n_models, const float* x, const int32_t* labels,
                      int n_samples, int chunk, float* pooled, float* hidden, float* w2_wino, int32_t* correct,
                      double* loss_sum, void* stream) {
  if (!params || !x || !labels || !pooled || !hidden || !w2_wino || !correct || !loss_sum) return MPLC_E_ARG;
  if (n_models < 1 || n_models > 65535 || n_samples < 1 || chunk < 1 || chunk > 65535 || stride != MPLC_CNN_STRIDE)
    return MPLC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  winograd_w2_kernel<<<dim3(C1 * C2 / 256, n_models), 256, 0, s>>>(params, stride, nullptr, w2_wino);
  for (int s0 = 0; s0 < n_samples; s0 += chunk) {
    const int cn = n_samples - s0 < chunk ? n_samples - s0 : chunk;
    conv_fwd_kernel<<<dim3(FWD_PARTS, (cn + FWD_SPB - 1) / FWD_SPB, n_models), FWD_THREADS, 0, s>>>(x, nullptr, s0, nullptr, cn, chunk, params, stride,
                                                                  w2_wino, pooled, nullptr);
    dense_fwd_kernel<<<dim3((cn + 31) / 32, n_models), 256, 0, s>>>(pooled, (int64_t)chunk * FEAT, nullptr, cn, chunk,
                                                                    params, stride, nullptr, nullptr, hidden);
    eval_head_kernel<<<n_models, 256, 0, s>>>(hidden, cn, chunk, labels, s0, params, stride, correct, loss_sum);
    const int st = launch_status();
    if (st) return st;
  }
  return MPLC_OK;
}

}  // extern "C"
