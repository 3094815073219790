// Batched multi-model CIFAR10 CNN trainer for gfx950 (contract: include/mplc_hip_cifar.h).
//
// One lockstep step of R replicas (each with its own weights, batch, schedule and dropout masks):
//   schedule       per replica: sample rows, batch count, optimizer iteration, dropout key
//   conv1_fwd      x -> a1 = relu(conv3x3 same, 3->32)                      implicit GEMM, fp32 MFMA
//   conv2_fwd      a1 -> d2 = dropout(pool(relu(conv3x3 valid, 32->32)))   pool fused in the accumulator
//   conv3_fwd      d2 -> a3 = relu(conv3x3 same, 32->64)
//   conv4_fwd      a3 -> d4 = dropout(pool(relu(conv3x3 valid, 64->64)))
//   dense5_fwd     d4 -> d5 = dropout(relu(d4 W5 + b5))                   A in LDS, W5 streamed
//   head           Dense(10) + softmax-CE gradient, dW6 + RMSprop, dh5 = (dl W6^T) * dropout' * relu'
//   dense5_bwd     per 16-row slice of W5: dd4 = dh5 W5^T, dW5 = d4^T dh5, RMSprop(W5) in one pass; the
//                  epilogue routes dd4 through dropout' and the pool's mask into the pooled dz4 (the conv4
//                  gradient kernels un-pool it, and conv3's data gradient writes dz2 pooled the same way)
//   wino_u<1>      W2|W3|W4 -> the rotated, channel-swapped kernels in Winograd form for the data gradients
//   conv4 wgrad/dgrad, conv3 wgrad/dgrad (epilogue: dropout' + un-pool into dz2), conv2 wgrad/dgrad,
//   conv1 wgrad    data gradients are Winograd F(2x2,3x3) like the forward (full/same padding, rotated
//                  weights) with a relu'-mask epilogue; weight gradients are split-K over fixed
//                  groups of MPLC_CIFAR_WG_SAMPLES samples (sums independent of the batch composition)
//   rmsprop_small  RMSprop on W1..b4 from the split partials (fixed order: bitwise reproducible)
// Everything is fp32 (the reference's Keras float32), accumulated on the exact-f32 MFMAs (32x32x2, 16x16x4).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keyed.h"
#include "xcd.h"
#include "mplc_hip.h"
#include "mplc_hip_cifar.h"
#include "cifar_common.h"

namespace {

// ------------------------------------------------------------------------------------------------
// init (glorot_uniform from mix64(key + i*golden), as mplc_cnn_init_params), schedule, flipped weights
// ------------------------------------------------------------------------------------------------
__global__ void init_params_kernel(float* __restrict__ params, int64_t stride, const uint64_t* __restrict__ keys) {
  const int m = blockIdx.y;
  const uint64_t key = keys[m];
  float* row = params + (int64_t)m * stride;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < stride; i += (int64_t)gridDim.x * blockDim.x) {
    float lim = 0.0f;
    if (i < OFF_W1 + 864) lim = 0x1.1aa69ep-3f;
    else if (i >= OFF_W2 && i < OFF_W2 + 9216) lim = 0x1.a20bd8p-4f;
    else if (i >= OFF_W3 && i < OFF_W3 + 18432) lim = 0x1.555556p-4f;
    else if (i >= OFF_W4 && i < OFF_W4 + 36864) lim = 0x1.279a74p-4f;
    else if (i >= OFF_W5 && i < OFF_W5 + 1179648) lim = 0x1.7a2316p-5f;
    else if (i >= OFF_W6 && i < OFF_W6 + 5120) lim = 0x1.b72326p-4f;
    float w = 0.0f;
    if (lim != 0.0f) {
      const uint64_t hsh = mix64(key + (uint64_t)i * 0x9E3779B97F4A7C15ull);
      const float u = (float)(uint32_t)(hsh >> 40) * 0x1p-24f;
      w = (u * 2.0f - 1.0f) * lim;
    }
    row[i] = w;
  }
}

__global__ void schedule_kernel(const mplc_replica_t* __restrict__ reps, int n_rep, int bmax,
                                const int32_t* __restrict__ rows, const int32_t* __restrict__ splits,
                                const int32_t* __restrict__ seq, int step,
                                int M, int round_len, int epochs, int32_t* __restrict__ idx,
                                int32_t* __restrict__ cnt, int32_t* __restrict__ opt_t,
                                uint64_t* __restrict__ drop_key, const int32_t* __restrict__ rep_glob,
                                int32_t* __restrict__ w5src) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)n_rep * bmax) return;
  const int r = (int)(gid / bmax);
  const int j = (int)(gid % bmax);
  const SlotSched ss = schedule_slot(reps[r], j, step, M, round_len, epochs, rows, splits, seq);
  idx[gid] = ss.row;
  if (j == 0) {
    cnt[r] = ss.c;
    opt_t[r] = ss.at;
    drop_key[r] = ss.dkey;
    // a FedAvg partner's first step of a round starts from the coalition model: W5 from its glob row
    if (w5src) w5src[r] = (reps[r].kind == MPLC_REP_FEDAVG && ss.at == 1) ? rep_glob[r] : -1;
  }
}

// ------------------------------------------------------------------------------------------------
// 3x3 stride-1 convolution as an implicit GEMM on v_mfma_f32_32x32x2f32:
//   out[y][x][n] = sum_{ky,kx,c} in[y+ky-PAD][x+kx-PAD][c] * B[(ky*3+kx)*CI + c][n]
// Forward: B = W [ky][kx][ci][co].  Data gradient: in = dZ of the layer, PAD' = 2 - PAD, B = flipped W.
// Block = (row band, sample slot j, replica r), NW waves; the band's input rows are staged in LDS
// ([rows][cols][CI|1], odd channel stride: the 32 lanes of a half read 32 pixels on 32 banks); B streams
// from L2.  GEMM rows: output pixels of the band, or for the pooled forward 2x2 windows x 4 pixels laid
// out so that the 4 pixels of a window are accumulator registers 4g..4g+3 of one lane (pool = register
// max).  Wave w owns the row tiles w + NW*u, u < UM, and all CO/32 column tiles.
// ------------------------------------------------------------------------------------------------
enum { EPI_FWD = 0, EPI_FWD_POOL = 1, EPI_BWD_MASK = 2, EPI_BWD_UNPOOL = 3 };

struct ConvArgs {
  const float* in;
  int in_mode;  // 0: slot-major activations [r*bmax + j]; 1: dataset row idx[r*bmax + j]; 2: row_base + j
  int row_base;
  const int32_t* idx;
  const int32_t* cnt;  // per replica sample count (NULL: cnt_all)
  int cnt_all;
  int bmax;
  const float* w;      // B operand of replica r: w + r * w_rstride
  int64_t w_rstride;
  const float* bias;   // forward: bias of replica r: bias + r * b_rstride
  int64_t b_rstride;
  const uint64_t* drop_key;  // pooled forward, train: per replica dropout key (NULL: inference)
  uint32_t drop_layer;
  const float* aux;          // BWD_MASK: the layer input activation (relu output) [slot][HO*WO*CO]
  const uint8_t* code_in;    // BWD_UNPOOL: pool/dropout code of the grid [slot][HO*WO*CO]
  float* out;
  uint8_t* code_out;         // pooled forward, train
};

// LDS offset of K index k = (ky*3 + kx)*3 + c of the 3-channel input (row stride rowp, pixel stride 3)
__host__ __device__ constexpr int ci3_off(int k, int rowp) { return (k / 9) * rowp + ((k / 3) % 3) * 3 + k % 3; }

// M tiles are 2-D: a 32-row tile is a 4 x 8 block of output pixels, or for the pooled forward a 2 x 4 block
// of pool windows with lane m = window * 4 + q (so the 4 pixels of a window are accumulator registers
// 4g..4g+3 of one lane: the pool is a register max).  With the LDS row stride = 8 (mod 32) dwords and an
// odd pixel stride, the 32 pixels of a tile fall on 32 distinct banks.
template <int HI, int WI, int CI, int CO, int PAD, int BR, int NW, int UM, int EPI, int CS = 1>
__global__ __launch_bounds__(NW * 64) void conv_kernel(const ConvArgs a) {
  static_assert(EPI == EPI_FWD || EPI == EPI_BWD_MASK, "the pooled-gradient epilogue (EPI_BWD_UNPOOL) is wino_kernel's");
  // CS channel slices: the input band is staged CI / CS channels at a time (K split), so a band (or a whole
  // sample) with many tiles per wave fits a small LDS footprint
  constexpr int HO = HI + 2 * PAD - 2, WO = WI + 2 * PAD - 2;
  constexpr bool POOL = (EPI == EPI_FWD_POOL);
  constexpr int PH = HO / 2, PW = WO / 2;
  constexpr int ROWS = POOL ? 2 * BR : BR;  // output rows per band (BR window rows when pooled)
  constexpr int TX = POOL ? (PW + 3) / 4 : (WO + 7) / 8;
  constexpr int TY = POOL ? BR / 2 : BR / 4;
  constexpr int TILES = TX * TY;
  constexpr int CIS = CI / CS;  // channels per slice
  constexpr int LR = ROWS + 2, WIP = WI + 2 * PAD, CIP = CIS | 1;
  constexpr int ROWP = WIP * CIP + ((8 - (WIP * CIP) % 32) + 32) % 32;
  constexpr int NT = CO / 32;
  constexpr int NTHR = NW * 64;
  static_assert(POOL ? BR % 2 == 0 : BR % 4 == 0, "bands are whole tile rows");
  static_assert(NW * UM >= TILES, "row tiles do not cover the band");
  static_assert(CO % 32 == 0 && (CI == 3 || CIS % 4 == 0) && CI % CS == 0, "unsupported channel counts");
  static_assert(CI != 3 || CS == 1, "the 3-channel input is not sliced");
  __shared__ float in_s[LR * ROWP];
  const int band = blockIdx.x, j = blockIdx.y, r = blockIdx.z;
  const int count = a.cnt ? a.cnt[r] : a.cnt_all;
  if (j >= count) return;
  const int tid = threadIdx.x;
  const int64_t slot = (int64_t)r * a.bmax + j;
  constexpr int IN_SZ = HI * WI * CI;
  const float* src = a.in_mode == 1 ? a.in + (int64_t)a.idx[slot] * IN_SZ
                     : a.in_mode == 2 ? a.in + (int64_t)(a.row_base + j) * IN_SZ
                                      : a.in + slot * IN_SZ;
  const int y0 = band * ROWS;
  // stage channels [cs * CIS, (cs + 1) * CIS) of the band's input rows
  auto stage = [&](int cs) {
    if constexpr (CI % 4 == 0) {
      // 16-B loads along the channels, all issued before the first LDS store (an exposed load -> wait ->
      // store chain per element would serialise the memory latency); out-of-image pixels load a valid
      // address and are zeroed by a select
      constexpr int C4 = CIS / 4;
      constexpr int TOT = LR * WIP * C4;
      constexpr int NIT = (TOT + NTHR - 1) / NTHR;
      fvec4 v[NIT];
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int e4 = tid + k * NTHR;
        const int pix = e4 / C4, c4 = e4 % C4;
        const int iy = y0 - PAD + pix / WIP, ix = pix % WIP - PAD;
        const bool ok = e4 < TOT && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
        const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? src + (iy * WI + ix) * CI + cs * CIS + 4 * c4 : src);
        v[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
      }
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int e4 = tid + k * NTHR;
        if (e4 < TOT) {
          const int pix = e4 / C4, c4 = e4 % C4;
          float* d = in_s + (pix / WIP) * ROWP + (pix % WIP) * CIP + 4 * c4;
          d[0] = v[k].x;
          d[1] = v[k].y;
          d[2] = v[k].z;
          d[3] = v[k].w;
        }
      }
    } else {
      constexpr int TOT = LR * WIP * CI;
      constexpr int NIT = (TOT + NTHR - 1) / NTHR;
      float v[NIT];
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int e = tid + k * NTHR;
        const int c = e % CI, pix = e / CI;
        const int iy = y0 - PAD + pix / WIP, ix = pix % WIP - PAD;
        const bool ok = e < TOT && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
        const float t = *(ok ? src + (iy * WI + ix) * CI + c : src);
        v[k] = ok ? t : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < NIT; ++k) {
        const int e = tid + k * NTHR;
        if (e < TOT) {
          const int c = e % CI, pix = e / CI;
          in_s[(pix / WIP) * ROWP + (pix % WIP) * CIP + c] = v[k];
        }
      }
    }
  };
  const int lane = tid & 63, wave = tid >> 6;
  const int n = lane & 31, kh = lane >> 5;
  int abase[UM];
#pragma unroll
  for (int u = 0; u < UM; ++u) {
    const int t = wave + NW * u;
    const int ty = t / TX, tx = t % TX;
    int yl, x;
    bool ok;
    if (POOL) {
      const int wi = n >> 2, q = n & 3;
      const int wy = ty * 2 + wi / 4, wx = tx * 4 + wi % 4;
      yl = 2 * wy + (q >> 1);
      x = 2 * wx + (q & 1);
      ok = t < TILES && wx < PW && band * BR + wy < PH;
    } else {
      yl = ty * 4 + n / 8;
      x = tx * 8 + n % 8;
      ok = t < TILES && x < WO && y0 + yl < HO;
    }
    if (!ok) { yl = 0; x = 0; }
    abase[u] = yl * ROWP + x * CIP + (CI == 3 ? 0 : kh);
  }
  floatx16 acc[UM][NT];
#pragma unroll
  for (int u = 0; u < UM; ++u)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[u][nt] = zero16();
  const float* W = a.w + (int64_t)r * a.w_rstride;
  if constexpr (CI == 3) {
    stage(0);
    __syncthreads();
    // K = 27 taps x channels, padded to 28: lane half kh takes k = 2s + kh
    const float* Wl = W + kh * CO + n;
#pragma unroll
    for (int s = 0; s < 14; ++s) {
      const bool valid = (2 * s + kh) < 27;
      const int off = kh ? (2 * s + 1 < 27 ? ci3_off(2 * s + 1, ROWP) : 0) : ci3_off(2 * s, ROWP);
      const float b = valid ? Wl[2 * s * CO] : 0.0f;
#pragma unroll
      for (int u = 0; u < UM; ++u) {
        const float av = valid ? in_s[abase[u] + off] : 0.0f;
        acc[u][0] = mfma32(av, b, acc[u][0]);
      }
    }
  } else {
    for (int cs = 0; cs < CS; ++cs) {
      if (cs) __syncthreads();  // the previous slice's readers are done
      stage(cs);
      __syncthreads();
#pragma unroll
      for (int kyx = 0; kyx < 9; ++kyx) {
        const int offA = (kyx / 3) * ROWP + (kyx % 3) * CIP;
        const float* Wk = W + (int64_t)(kyx * CI + cs * CIS + kh) * CO + n;
#pragma unroll
        for (int c2 = 0; c2 < CIS / 2; ++c2) {
          float b[NT];
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) b[nt] = Wk[2 * c2 * CO + nt * 32];
#pragma unroll
          for (int u = 0; u < UM; ++u) {
            const float av = in_s[abase[u] + offA + 2 * c2];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[u][nt] = mfma32(av, b[nt], acc[u][nt]);
          }
        }
      }
    }
  }
  // ---- epilogues: accumulator register -> tile row rt = acc_row(reg, kh) -> pixel / window ----
  if constexpr (EPI == EPI_FWD_POOL) {
    const float* bias = a.bias + (int64_t)r * a.b_rstride;
    float* o = a.out + slot * (PH * PW * CO);
    uint8_t* oc = a.drop_key ? a.code_out + slot * (PH * PW * CO) : nullptr;
    const uint32_t rseed = a.drop_key ? drop_row_seed(a.drop_key[r], a.drop_layer, (uint32_t)j) : 0u;
#pragma unroll
    for (int u = 0; u < UM; ++u) {
      const int t = wave + NW * u;
      const int ty = t / TX, tx = t % TX;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int co = nt * 32 + n;
        const float bv = bias[co];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int wi = 2 * g + kh;
          const int py = band * BR + ty * 2 + wi / 4, px = tx * 4 + wi % 4;
          if (t < TILES && px < PW && ty * 2 + wi / 4 < BR && py < PH) {
            float best = acc[u][nt][4 * g] + bv;
            int arg = 0;
#pragma unroll
            for (int q = 1; q < 4; ++q) {
              const float z = acc[u][nt][4 * g + q] + bv;
              if (z > best) { best = z; arg = q; }
            }
            const int pidx = (py * PW + px) * CO + co;
            const float av = fmaxf(best, 0.0f);
            if (oc) {
              const bool keep = drop_keep(rseed, (uint32_t)pidx, THR_25);
              o[pidx] = keep ? av * SCALE_25 : 0.0f;
              oc[pidx] = (uint8_t)(arg | (keep ? CODE_KEEP : 0) | (best > 0.0f ? CODE_POS : 0));
            } else {
              o[pidx] = av;
            }
          }
        }
      }
    }
  } else {
    const float* bias = (EPI == EPI_FWD) ? a.bias + (int64_t)r * a.b_rstride : nullptr;
    const float* act = (EPI == EPI_BWD_MASK) ? a.aux + slot * (HO * WO * CO) : nullptr;
    const uint8_t* cd = (EPI == EPI_BWD_UNPOOL) ? a.code_in + slot * (HO * WO * CO) : nullptr;
    float* o = a.out + slot * (HO * WO * CO);
#pragma unroll
    for (int u = 0; u < UM; ++u) {
      const int t = wave + NW * u;
      const int ty = t / TX, tx = t % TX;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int ch = nt * 32 + n;
        const float bv = (EPI == EPI_FWD) ? bias[ch] : 0.0f;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int rt = acc_row(reg, kh);
          const int y = y0 + ty * 4 + rt / 8, x = tx * 8 + rt % 8;
          if (!(t < TILES && x < WO && y < HO)) continue;
          const int o_i = (y * WO + x) * CO + ch;
          const float v = acc[u][nt][reg];
          if constexpr (EPI == EPI_FWD) {
            o[o_i] = fmaxf(v + bv, 0.0f);
          } else {
            o[o_i] = act[o_i] > 0.0f ? v : 0.0f;
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// conv1 forward (3 input channels, 'same', 32 output channels + ReLU; round 6): the implicit
// GEMM of conv_kernel<32, 32, 3, 32, 1, 8, 4, 2, EPI_FWD> with the operands' roles swapped - the output channels
// are the M rows of v_mfma_f32_32x32x2f32 (A = W1 transposed: lane (co, kh) holds W1[k][co], k = 2s + kh, loaded
// once for all 14 k-steps) and the band's pixels its N columns (B = the staged image, the same LDS reads).  Every
// output is the same fmaf chain over k = 0 .. 27 as before (a product's operands only trade places): bit-identical.
// What changes is the epilogue: a lane's 16 accumulators are 4 runs of 4 consecutive channels of ONE pixel (C/D
// rows 8j + 4kh .. +3), so the bias is 4 x 16-B loads per lane for the whole block, the ReLU'd activations leave as
// 4 x 16-B stores per tile (16 x 4-B stores and per-register pixel arithmetic before), and no tile needs a bounds
// test (4 bands x 2 x 4 tiles of 4 x 8 pixels cover the 32 x 32 output exactly).  conv1 is HBM-bound (K = 27:
// 12.3 flop/B): the stores are what it is made of.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const ConvArgs a) {
  constexpr int HI = 32, WI = 32, CI = 3, CO = 32, PAD = 1, BR = 8, NW = 4, UM = 2;
  constexpr int WO = WI, TX = WO / 8;  // 4 x 8-pixel tiles across, 2 down per band
  constexpr int LR = BR + 2, WIP = WI + 2 * PAD, CIP = CI;
  constexpr int ROWP = WIP * CIP + ((8 - (WIP * CIP) % 32) + 32) % 32;
  static_assert(NW * UM == TX * (BR / 4), "the band's tiles, one per (wave, u)");
  __shared__ float in_s[LR * ROWP];
  const int band = blockIdx.x, j = blockIdx.y, r = blockIdx.z;
  const int count = a.cnt ? a.cnt[r] : a.cnt_all;
  if (j >= count) return;
  const int tid = threadIdx.x;
  const int64_t slot = (int64_t)r * a.bmax + j;
  constexpr int IN_SZ = HI * WI * CI;
  const float* src = a.in_mode == 1 ? a.in + (int64_t)a.idx[slot] * IN_SZ
                     : a.in_mode == 2 ? a.in + (int64_t)(a.row_base + j) * IN_SZ
                                      : a.in + slot * IN_SZ;
  const int y0 = band * BR;
  {  // the band's 10 input rows (zero padded), as conv_kernel stages them
    constexpr int TOT = LR * WIP * CI;
    constexpr int NIT = (TOT + 255) / 256;
    float v[NIT];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e = tid + k * 256;
      const int c = e % CI, pix = e / CI;
      const int iy = y0 - PAD + pix / WIP, ix = pix % WIP - PAD;
      const bool ok = e < TOT && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
      const float t = *(ok ? src + (iy * WI + ix) * CI + c : src);
      v[k] = ok ? t : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e = tid + k * 256;
      if (e < TOT) {
        const int c = e % CI, pix = e / CI;
        in_s[(pix / WIP) * ROWP + (pix % WIP) * CIP + c] = v[k];
      }
    }
  }
  const int lane = tid & 63, wave = tid >> 6;
  const int n = lane & 31, kh = lane >> 5;
  // A operand: W1[k][co = n] for k = 2s + kh (0 past k = 26), the same for both tiles
  const float* W = a.w + (int64_t)r * a.w_rstride;
  float wa[14];
#pragma unroll
  for (int s = 0; s < 14; ++s) wa[s] = (2 * s + kh) < 27 ? W[(2 * s + kh) * CO + n] : 0.0f;
  const float* bias = a.bias + (int64_t)r * a.b_rstride;
  fvec4 bv[4];  // channels 8 jj + 4 kh .. + 3
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) bv[jj] = *reinterpret_cast<const fvec4*>(bias + 8 * jj + 4 * kh);
  __syncthreads();
  float* o = a.out + slot * (WO * WO * CO);
#pragma unroll
  for (int u = 0; u < UM; ++u) {
    const int t = wave + NW * u;
    const int ty = t / TX, tx = t % TX;
    const int yl = ty * 4 + n / 8, x = tx * 8 + n % 8;  // this lane's pixel (column n of the tile)
    const int ab = yl * ROWP + x * CIP;
    floatx16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 14; ++s) {
      const int k = 2 * s + kh;
      const int off = kh ? (2 * s + 1 < 27 ? ci3_off(2 * s + 1, ROWP) : 0) : ci3_off(2 * s, ROWP);
      const float bx = k < 27 ? in_s[ab + off] : 0.0f;
      acc = mfma32(wa[s], bx, acc);
    }
    fvec4* op = reinterpret_cast<fvec4*>(o + ((y0 + yl) * WO + x) * CO + 4 * kh);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      fvec4 z;
#pragma unroll
      for (int i = 0; i < 4; ++i) z[i] = fmaxf(acc[4 * jj + i] + bv[jj][i], 0.0f);
      op[2 * jj] = z;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// 3x3 stride-1 convolution in Winograd form F(2x2, 3x3) (Lavin & Gray) on v_mfma_f32_16x16x4_f32, for the
// layers with CI >= 32 (conv2..conv4 forward, and their data gradients = forward convolutions of dZ with the
// rotated, channel-swapped kernel, padding 2 - PAD):
//   out tile (2x2) = A^T [ (G g G^T) (.) (B^T d B) ] A  per 4x4 input patch d, summed over the input channels
// as 16 GEMMs M[xi][tile][co] = sum_ci V[xi][tile][ci] U[xi][ci][co]: 2.25x fewer multiply-adds than the
// direct implicit GEMM (16 per output tile of 4 instead of 36).  Everything stays fp32 (the transforms'
// coefficients are 0, +-1, +-1/2, exact; accumulation on the exact-f32 MFMA).  U is the per-replica,
// per-step Winograd form of the layer's weights (wino_u_kernel), read from L2.
// Tiles: the output in 2x2 tiles; for the pooled forward one tile IS one 2x2 max-pool window (pool = max
// over the tile's 4 outputs, no row/column of the unpooled output is computed that the pool drops).
// Block = (band of BTY tile rows, sample slot j, replica r), 4 waves; the band's input rows (zero padded)
// are staged in LDS once ([rows][cols][CI + 1]: the 32 lanes of a half-wave read 16 tiles x 2 channels on
// 32 banks).  Wave i owns transform row i (xi = 4i .. 4i+3) of every 16-tile group and all CO channels:
// 4 x CO/16 accumulators of 16x16x4; per k-step (4 input channels) a lane reads 8 staged values of its
// tile's patch, forms its 4 values of V with 12 adds and issues 4 x CO/16 MFMAs, the B operands (U) loaded
// one k-step ahead.  The waves fold their row of the output transform (T_i = M_i A) into LDS (32 output
// channels at a time); then every thread finishes Y = A^T T for (tile, channel) items and applies the layer's
// epilogue (same semantics as conv_kernel's).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ fvec4 mfma16(float a, float b, fvec4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Stage rows iy0 .. iy0 + NR - 1, columns ix0 .. ix0 + NC - 1 (iy0, ix0, NR, NC even: whole pooling windows) of a
// dense gradient held POOLED [HP][WP][C] with its pool codes (argmax = code & 3; dropout' and the pool's positive
// mask already applied by the producer) into an LDS image [NR][NC][CP floats], channels 0 .. C - 1: each window's
// value at its argmax pixel, 0 at the other three and outside the pooled grid (an odd dense size's last row / column
// belongs to no window).  Window-major: one (window, channel quad) per item, so one 16-B value load and one 4-B code
// load feed 4 pixels.  The LDS image is exactly what the dense un-pooled tensor held.
template <int C, int NR, int NC, int NTHR>
struct UnpoolShape {
  static constexpr int C4 = C / 4;
  static constexpr int TOT = (NR / 2) * (NC / 2) * C4;
  static constexpr int NIT = (TOT + NTHR - 1) / NTHR;
};
// the two halves of stage_unpool: the loads into registers (val, cw), then the LDS image from them
template <int HP, int WP, int C, int NR, int NC, int NTHR>
__device__ __forceinline__ void unpool_load(const float* __restrict__ pooled, const uint8_t* __restrict__ codes,
                                            int iy0, int ix0, int tid,
                                            fvec4 (&val)[UnpoolShape<C, NR, NC, NTHR>::NIT],
                                            uint32_t (&cw)[UnpoolShape<C, NR, NC, NTHR>::NIT]) {
  using S = UnpoolShape<C, NR, NC, NTHR>;
#pragma unroll
  for (int k = 0; k < S::NIT; ++k) {
    const int e = tid + k * NTHR;
    const int win = e / S::C4, c4 = e % S::C4;
    const int py = iy0 / 2 + win / (NC / 2), px = ix0 / 2 + win % (NC / 2);
    const bool ok = e < S::TOT && py >= 0 && py < HP && px >= 0 && px < WP;
    const int pidx = (py * WP + px) * C + 4 * c4;
    const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? pooled + pidx : pooled);
    const uint32_t c = *reinterpret_cast<const uint32_t*>(ok ? codes + pidx : codes);
    val[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
    cw[k] = c;
  }
}
template <int C, int NR, int NC, int CP, int NTHR, int RS = NC * CP>  // RS: the image's row stride (floats)
__device__ __forceinline__ void unpool_store(float* __restrict__ dst, int tid,
                                             const fvec4 (&val)[UnpoolShape<C, NR, NC, NTHR>::NIT],
                                             const uint32_t (&cw)[UnpoolShape<C, NR, NC, NTHR>::NIT]) {
  using S = UnpoolShape<C, NR, NC, NTHR>;
#pragma unroll
  for (int k = 0; k < S::NIT; ++k) {
    const int e = tid + k * NTHR;
    if (e < S::TOT) {
      const int win = e / S::C4, c4 = e % S::C4;
      float* d0 = dst + (2 * (win / (NC / 2))) * RS + (2 * (win % (NC / 2))) * CP + 4 * c4;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float* d = d0 + (p >> 1) * RS + (p & 1) * CP;
        d[0] = (cw[k] & 3) == (uint32_t)p ? val[k].x : 0.0f;
        d[1] = ((cw[k] >> 8) & 3) == (uint32_t)p ? val[k].y : 0.0f;
        d[2] = ((cw[k] >> 16) & 3) == (uint32_t)p ? val[k].z : 0.0f;
        d[3] = ((cw[k] >> 24) & 3) == (uint32_t)p ? val[k].w : 0.0f;
      }
    }
  }
}
template <int HP, int WP, int C, int NR, int NC, int CP, int NTHR, int RS = NC * CP>
__device__ __forceinline__ void stage_unpool(const float* __restrict__ pooled, const uint8_t* __restrict__ codes,
                                             int iy0, int ix0, float* __restrict__ dst, int tid) {
  using S = UnpoolShape<C, NR, NC, NTHR>;
  fvec4 val[S::NIT];
  uint32_t cw[S::NIT];
  unpool_load<HP, WP, C, NR, NC, NTHR>(pooled, codes, iy0, ix0, tid, val, cw);
  unpool_store<C, NR, NC, CP, NTHR, RS>(dst, tid, val, cw);
}

__device__ __forceinline__ void wino_g_rows(const float (&g)[3], float (&o)[4]) {  // o = G g (one column)
  o[0] = g[0];
  o[1] = 0.5f * ((g[0] + g[1]) + g[2]);
  o[2] = 0.5f * ((g[0] - g[1]) + g[2]);
  o[3] = g[2];
}

// U[xi][cin][cout] = (G g G^T)[i][j], xi = 4i + j, for the kernel g of channel pair (cin, cout):
// FLIP = 0: the layer's forward kernel, g[ky][kx] = W[ky][kx][cin][cout];
// FLIP = 1: the data gradient's kernel, g[ky][kx] = W[2 - ky][2 - kx][cout][cin] (in = the layer's co).
// XIL = 1 stores the pair's 16 transform points contiguously, U[cin][cout][xi] (conv2: the wave-local kernel reads a
// lane's 16 B operands of a k-step as 4 x 16 B instead of 16 scalar loads: conv2 forward -5 %); XIL = 0 the
// transform point first, U[xi][cin][cout] (conv3 / conv4: the row-per-wave kernel reads 4 of the 16 points per
// pair, coalesced across the lanes in this layout).
template <int CIN, int COUT, int FLIP, int XIL = 0>
__device__ __forceinline__ void wino_u_pair(const float* __restrict__ W, float* __restrict__ U, int e) {
  const int cin = e / COUT, cout = e % COUT;
  float g[3][3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
      g[ky][kx] = FLIP ? W[((2 - ky) * 3 + (2 - kx)) * CIN * COUT + cout * CIN + cin]
                       : W[(ky * 3 + kx) * CIN * COUT + cin * COUT + cout];
  float gg[4][3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const float col[3] = {g[0][kx], g[1][kx], g[2][kx]};
    float o[4];
    wino_g_rows(col, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) gg[i][kx] = o[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float o[4];
    wino_g_rows(gg[i], o);
    if (XIL) {
      reinterpret_cast<fvec4*>(U + (int64_t)e * 16)[i] = fvec4{o[0], o[1], o[2], o[3]};
    } else {
#pragma unroll
      for (int jx = 0; jx < 4; ++jx) U[(4 * i + jx) * CIN * COUT + e] = o[jx];
    }
  }
}

// Winograd-form weights of conv2 | conv3 | conv4 (layout MPLC_CIFAR_WT: WU_2, WU_3, WU_4) for the forward
// (FLIP = 0) or the data gradients (FLIP = 1), one thread per channel pair.
constexpr int WU_2 = 0, WU_3 = 16 * 32 * 32, WU_4 = WU_3 + 16 * 32 * 64;
static_assert(WU_4 + 16 * 64 * 64 == MPLC_CIFAR_WT, "MPLC_CIFAR_WT must hold conv2..conv4 in Winograd form");

// The data gradient's kernel (FLIP = 1) reads W transposed, W[k][cout][cin]: one thread per channel pair in
// U's order would read with a stride of CIN floats, so a block takes a 16 x 16 (cin, cout) tile, reads it
// cin-fastest, transforms it and writes U cout-fastest through an LDS transpose (same arithmetic per pair).
template <int CIN, int COUT, int XIL = 0>
__device__ __forceinline__ void wino_u_tile_flip(const float* __restrict__ W, float* __restrict__ U, int tile,
                                                 float (*sx)[16 * 17]) {
  const int tid = threadIdx.x;
  const int cin0 = 16 * (tile % (CIN / 16)), cout0 = 16 * (tile / (CIN / 16));
  const int cin = cin0 + (tid & 15), cout = cout0 + (tid >> 4);  // read order: cin fastest
  float g[3][3];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) g[ky][kx] = W[((2 - ky) * 3 + (2 - kx)) * CIN * COUT + cout * CIN + cin];
  float gg[4][3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const float col[3] = {g[0][kx], g[1][kx], g[2][kx]};
    float o[4];
    wino_g_rows(col, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) gg[i][kx] = o[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float o[4];
    wino_g_rows(gg[i], o);
#pragma unroll
    for (int jx = 0; jx < 4; ++jx) sx[4 * i + jx][(tid & 15) * 17 + (tid >> 4)] = o[jx];  // [xi][cin_l][cout_l], row stride 17
  }
  __syncthreads();
  const int wcin = cin0 + (tid >> 4), wcout = cout0 + (tid & 15);  // write order: cout fastest
  if (XIL) {  // the pair's 16 points contiguous (U[cin][cout][xi])
    fvec4* u4 = reinterpret_cast<fvec4*>(U + (int64_t)(wcin * COUT + wcout) * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = (tid >> 4) * 17 + (tid & 15);
      u4[i] = fvec4{sx[4 * i][c], sx[4 * i + 1][c], sx[4 * i + 2][c], sx[4 * i + 3][c]};
    }
    return;
  }
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) U[xi * CIN * COUT + wcin * COUT + wcout] = sx[xi][(tid >> 4) * 17 + (tid & 15)];
}

template <int FLIP>
__global__ __launch_bounds__(256) void wino_u_kernel(const float* __restrict__ params, int64_t stride,
                                                     const int32_t* __restrict__ cnt, float* __restrict__ U) {
  const int r = blockIdx.y;
  if (cnt && cnt[r] == 0) return;
  const float* P = params + (int64_t)r * stride;
  float* Ur = U + (int64_t)r * MPLC_CIFAR_WT;
  if (FLIP) {  // 16 x 16 tiles: conv2 4 | conv3 8 | conv4 16 (the grid's 28 blocks per replica)
    __shared__ float sx[16][16 * 17];
    const int b = blockIdx.x;
    if (b < 4) wino_u_tile_flip<32, 32, 1>(P + OFF_W2, Ur + WU_2, b, sx);
    else if (b < 12) wino_u_tile_flip<64, 32>(P + OFF_W3, Ur + WU_3, b - 4, sx);  // dgrad: in = conv3's 64 co
    else if (b < 28) wino_u_tile_flip<64, 64>(P + OFF_W4, Ur + WU_4, b - 12, sx);
    return;
  }
  const int e = blockIdx.x * 256 + threadIdx.x;  // pair index over conv2 (1024) | conv3 (2048) | conv4 (4096)
  if (e < 1024) {
    wino_u_pair<32, 32, FLIP, 1>(P + OFF_W2, Ur + WU_2, e);
  } else if (e < 3072) {
    if (FLIP) wino_u_pair<64, 32, 1>(P + OFF_W3, Ur + WU_3, e - 1024);   // dgrad: in = conv3's 64 co
    else wino_u_pair<32, 64, 0>(P + OFF_W3, Ur + WU_3, e - 1024);
  } else if (e < 7168) {
    wino_u_pair<64, 64, FLIP>(P + OFF_W4, Ur + WU_4, e - 3072);
  }
}

#ifndef MPLC_WINO_QUAD
#define MPLC_WINO_QUAD 1  // conv4_fwd's 4-tile remainder group on 4x4x1 MFMAs (0: a padded 16-tile group; same bits)
#endif


// Wave-index tag: a loop instantiated once per wave index (compile-time Winograd transform signs)
template <int V>
struct IntC {
  static constexpr int value = V;
};
template <int HI, int WI, int CI, int CO, int PAD, int BTY, int EPI, int UPI = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_kernel(const ConvArgs a) {
  constexpr bool POOL = (EPI == EPI_FWD_POOL);
  constexpr int HO = HI + 2 * PAD - 2, WO = WI + 2 * PAD - 2;
  constexpr int PH = HO / 2, PW = WO / 2;
  constexpr int TYT = POOL ? PH : (HO + 1) / 2;  // tile rows / columns computed
  constexpr int TXT = POOL ? PW : (WO + 1) / 2;
  constexpr int NG = (BTY * TXT + 15) / 16;      // 16-tile groups per band
  constexpr int LR = 2 * BTY + 2, LC = 2 * TXT + 2;
  constexpr int CIP = CI + 1;                    // odd channel stride
  // Row stride padded to ROWP = TXT (mod 16): with CIP = 1 (mod 16) tile (tyl, tx) then starts on bank
  // 2 (TXT tyl + tx) = 2 tile (mod 32), so a half-wave's 16 tiles x 2 channels (kq) fill the 32 banks once (the
  // unpadded LC CIP put a group's second tile row on its first row's banks: 2-way conflicts on every V read)
  constexpr int ROWP = LC * CIP + ((TXT - LC * CIP) % 16 + 16) % 16;
  static_assert(CIP % 16 == 1 && ROWP % 16 == TXT % 16, "conflict-free V reads");
  constexpr int NCG = CO / 16;
  constexpr int CH = CO > 32 ? 32 : CO;          // output channels per output-transform pass
  constexpr int NPASS = CO / CH;
  constexpr int TS = CH + 1;
  constexpr int TQ = 16 * TS;
  constexpr int NK = CI / 4;
  static_assert(CI % 4 == 0 && CO % 32 == 0, "channel counts");
  // one band whose last 16-tile group holds exactly 4 tiles, 64 output channels: that group on 4x4x1 MFMAs
  constexpr bool QUAD = MPLC_WINO_QUAD && BTY >= TYT && (BTY * TXT) % 16 == 4 && CO == 64;
  static_assert((16 * CH) % 256 == 0, "output items per thread");
  // the data gradients' epilogue operand (EPI_BWD_MASK: the ReLU' mask a > 0; EPI_BWD_UNPOOL: the pool codes) for
  // the band's 2 BTY output rows, staged as bytes with the input band: its global loads share the staging's latency
  // instead of stalling the output phase of every group
  constexpr bool STAGE_EPI = (EPI == EPI_BWD_MASK || EPI == EPI_BWD_UNPOOL);
  constexpr int ER = 2 * BTY;
  __shared__ float in_s[LR * ROWP];
  __shared__ float t_s[8 * TQ];
  __shared__ uint32_t e_s[STAGE_EPI ? ER * WO * CO / 4 : 1];
  constexpr bool STAGE_BIAS = (EPI == EPI_FWD || POOL);  // the forward's bias, staged with the input band
  __shared__ float b_s[STAGE_BIAS ? CO : 1];
  const LogicalBlock lbk = xcd_block3();  // (band, sample, replica): a replica's blocks share one XCD's L2 (its U)
  const int band = lbk.x, j = lbk.y, r = lbk.z;
  const int count = a.cnt ? a.cnt[r] : a.cnt_all;
  if (j >= count) return;
  const int tid = threadIdx.x;
  const int64_t slot = (int64_t)r * a.bmax + j;
  constexpr int IN_SZ = UPI ? (HI / 2) * (WI / 2) * CI : HI * WI * CI;  // UPI: a pooled gradient's slots
  const float* src = a.in_mode == 2 ? a.in + (int64_t)(a.row_base + j) * IN_SZ : a.in + slot * IN_SZ;
  const int ty0 = band * BTY;
  const int bty = min(BTY, TYT - ty0);  // tile rows of this band
  const int ntile = bty * TXT;
  if constexpr (UPI) {  // the input is a POOLED gradient [HI/2][WI/2][CI] with its pool codes: un-pooled here
    static_assert(PAD % 2 == 0 && LR % 2 == 0 && LC % 2 == 0, "the staged region must be whole pooling windows");
    stage_unpool<HI / 2, WI / 2, CI, LR, LC, CIP, 256, ROWP>(src, a.code_in + slot * ((HI / 2) * (WI / 2) * CI),
                                                             2 * ty0 - PAD, -PAD, in_s, tid);
  } else {  // stage input rows 2 ty0 - PAD .. + LR, columns -PAD .. + LC (zero outside the input)
    constexpr int C4 = CI / 4;
    constexpr int TOT = LR * LC * C4;
    constexpr int NIT = (TOT + 255) / 256;
    fvec4 v[NIT];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e4 = tid + k * 256;
      const int pix = e4 / C4, c4 = e4 % C4;
      const int iy = 2 * ty0 - PAD + pix / LC, ix = pix % LC - PAD;
      const bool ok = e4 < TOT && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
      const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? src + (iy * WI + ix) * CI + 4 * c4 : src);
      v[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e4 = tid + k * 256;
      if (e4 < TOT) {
        const int pix = e4 / C4, c4 = e4 % C4;
        float* d = in_s + (pix / LC) * ROWP + (pix % LC) * CIP + 4 * c4;
        d[0] = v[k].x;
        d[1] = v[k].y;
        d[2] = v[k].z;
        d[3] = v[k].w;
      }
    }
  }
  if constexpr (STAGE_BIAS) {
    if (tid < CO) b_s[tid] = a.bias[(int64_t)r * a.b_rstride + tid];
  }
  if constexpr (STAGE_EPI) {
    constexpr int TOT = ER * WO * (CO / 4);
    constexpr int NIT = (TOT + 255) / 256;
    const float* ax = a.aux + slot * (HO * WO * CO);
    const uint8_t* cx = a.code_in + slot * (HO * WO * CO);
    uint32_t ev[NIT];
    fvec4 fv[EPI == EPI_BWD_MASK ? NIT : 1];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e = tid + 256 * k;
      const int px = e / (CO / 4), c4 = e % (CO / 4);
      const int yy = 2 * ty0 + px / WO, xx = px % WO;
      const bool ok = e < TOT && yy < HO;
      const int64_t off = ok ? (int64_t)(yy * WO + xx) * CO + 4 * c4 : 0;
      if constexpr (EPI == EPI_BWD_MASK) {
        const fvec4 t = *reinterpret_cast<const fvec4*>(ax + off);
        fv[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
      } else {
        const uint32_t t = *reinterpret_cast<const uint32_t*>(cx + off);
        ev[k] = ok ? t : 0u;
      }
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e = tid + 256 * k;
      if (e < TOT) {
        if constexpr (EPI == EPI_BWD_MASK)
          ev[k] = (fv[k].x > 0.0f ? 1u : 0u) | (fv[k].y > 0.0f ? 0x100u : 0u) | (fv[k].z > 0.0f ? 0x10000u : 0u) |
                  (fv[k].w > 0.0f ? 0x1000000u : 0u);
        e_s[e] = ev[k];
      }
    }
  }
  const int lane = tid & 63, wave = tid >> 6;
  const int wi = wave;
  const int tl = lane & 15, kq = lane >> 4;
  // B operands of k-step st: U[4 wi + jj][4 st + kq][16 cg + tl] (the xi-first layout: a 16-lane group reads 64
  // contiguous bytes per transform point; the xi-last layout's one 16-B load per channel pair measured 5-10 % slower
  // here, scripts/r04/gpu_ab_cifar.sh)
  const float* Ub = a.w + (int64_t)r * a.w_rstride + (int64_t)(4 * wi) * CI * CO + kq * CO + tl;
  auto load_b = [&](int st, float (&bv)[4 * NCG]) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int cg = 0; cg < NCG; ++cg) bv[NCG * jj + cg] = Ub[(int64_t)jj * CI * CO + (4 * st) * CO + 16 * cg];
  };
  // EPI_BWD_UNPOOL writes the POOLED gradient [HO][WO][CO] of the layer below (its consumers un-pool it)
  float* o = a.out + slot * ((POOL ? PH * PW : HO * WO) * CO);
  const float* bias = (EPI == EPI_FWD || POOL) ? a.bias + (int64_t)r * a.b_rstride : nullptr;
  const float* act = (EPI == EPI_BWD_MASK) ? a.aux + slot * (HO * WO * CO) : nullptr;
  const uint8_t* cd = (EPI == EPI_BWD_UNPOOL) ? a.code_in + slot * (HO * WO * CO) : nullptr;
  uint8_t* oc = (POOL && a.drop_key) ? a.code_out + slot * (PH * PW * CO) : nullptr;
  const uint32_t rseed = (POOL && a.drop_key) ? drop_row_seed(a.drop_key[r], a.drop_layer, (uint32_t)j) : 0u;
  // The wave's transform row of U for the first KR k-steps (up to 128 values: all of conv3's, a quarter of conv4's)
  // is loaded once for all the band's groups instead of from L2 per group and k-step; the rest streams from L2
  // two k-steps ahead (same operands in the same order: bit-identical).
  constexpr int BREGS = (4 * NCG * NK <= 128) ? 128 : 64;  // conv4: 64 (128 spilled 41 registers)
  constexpr int KR = (BREGS / (4 * NCG)) < NK ? BREGS / (4 * NCG) : NK;
  static_assert(KR % 2 == 0 && (NK - KR) % 2 == 0, "k-steps in pairs");
  float bw[KR][4 * NCG];
#pragma unroll
  for (int st = 0; st < KR; ++st) load_b(st, bw[st]);
  __syncthreads();
  // B^T row i combines two patch rows: t = d[ry] + sx d[rx] (row 0: d0 - d2, 1: d1 + d2, 2: d2 - d1, 3: d1 - d3),
  // one fused multiply-add by +-1 per value (exact product, one rounding: the bits of the add or subtract).  This
  // replaced per-wave compiled copies of the group loop (compile-time signs, same instruction count), whose
  // barriers sat in wave-divergent code; now every barrier is in code all waves share.
  const int ry = (wi == 0) ? 0 : (wi == 2) ? 2 : 1;
  const int rx = (wi == 3) ? 3 : (wi == 2) ? 1 : 2;
  const float sx = (wi == 1) ? 1.0f : -1.0f;
  const int drow = (rx - ry) * ROWP;
  {
  // The QUAD group's GEMMs (4 tiles x 64 channels per transform point, K = CI) on 4x4x1 MFMAs: lane 4 b + i
  // supplies tile i's V (the same value in all 16 blocks), lane = output channel supplies U; the wave's 4 transform
  // points are 4 accumulators.  U streams from L2 in chunks of QC channels, the next chunk in flight.
  auto quad_group = [&](int t0, fvec4 (&q)[4]) __attribute__((always_inline)) {
    const int tile = t0 + (lane & 3);
    const int tyl = tile / TXT, tx = tile % TXT;
    const float* dpa = in_s + (2 * tyl + ry) * ROWP + 2 * tx * CIP;
    const float* Uq = a.w + (int64_t)r * a.w_rstride + (int64_t)(4 * wi) * CI * CO + (lane & (CO - 1));
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) q[jj] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int QC = 8;  // 16: 208 registers spilled
    constexpr int NCH = CI / QC;
    static_assert(CI % (2 * QC) == 0, "channel chunks in pairs");
    auto qload = [&](int ch, float (&b)[QC][4]) {
#pragma unroll
      for (int u = 0; u < QC; ++u)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) b[u][jj] = Uq[(int64_t)jj * CI * CO + (ch * QC + u) * CO];
    };
    auto qstep = [&](int ch, const float (&b)[QC][4]) {
#pragma unroll
      for (int u = 0; u < QC; ++u) {
        const float* d0 = dpa + ch * QC + u;
        float t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          t[c] = __builtin_fmaf(sx, d0[drow + c * CIP], d0[c * CIP]);
        }
        float v[4];
        v[0] = t[0] - t[2];
        v[1] = t[1] + t[2];
        v[2] = t[2] - t[1];
        v[3] = t[1] - t[3];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) q[jj] = mfma4(v[jj], b[u][jj], q[jj]);
      }
    };
    float qb0[QC][4], qb1[QC][4];
    qload(0, qb0);
#pragma unroll 1
    for (int ch = 0; ch < NCH; ch += 2) {
      qload(ch + 1, qb1);
      qstep(ch, qb0);
      if (ch + 2 < NCH) qload(ch + 2, qb0);
      qstep(ch + 1, qb1);
    }
  };
  // QUAD: the band's last group holds 4 tiles (conv4's 6 x 6 windows: 36 = 2 x 16 + 4).  Instead of a 16-row
  // MFMA group three quarters padding, its GEMMs run on v_mfma_f32_4x4x1f32 with the 4 tiles as rows and the 64
  // output channels as 16 blocks of 4 columns: a quarter of the matrix-core cycles.  Per output the products
  // chain over ci = 0, 1, .. 63 from zero exactly as the 16x16x4 form's k-steps do (fmaf per element in ci
  // order): the same bits.  The output transform below is shared.  The group runs after the loop, where the
  // register copy of U (bw) is dead.
  auto run_group = [&](int g, auto qtag) __attribute__((always_inline)) {
    constexpr bool quad = decltype(qtag)::value != 0;
    fvec4 acc4[4];
    fvec4 acc[4][NCG];
    if constexpr (quad) {
      quad_group(16 * g, acc4);
    } else {
    const int tile = min(16 * g + tl, ntile - 1);
    const int tyl = tile / TXT, tx = tile % TXT;
    const float* dpa = in_s + (2 * tyl + ry) * ROWP + 2 * tx * CIP + kq;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int cg = 0; cg < NCG; ++cg) acc[jj][cg] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
    // k-steps in pairs with two B buffers (the next step's operands in flight during this step's MFMAs);
    // not unrolled further: a fully unrolled CI = 64 loop lets the scheduler hoist every load and spill
    auto kstep = [&](int st, const float (&bv)[4 * NCG]) {
      const float* d0 = dpa + 4 * st;
      float t[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t[c] = __builtin_fmaf(sx, d0[drow + c * CIP], d0[c * CIP]);
      }
      float v[4];
      v[0] = t[0] - t[2];
      v[1] = t[1] + t[2];
      v[2] = t[2] - t[1];
      v[3] = t[1] - t[3];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) acc[jj][cg] = mfma16(v[jj], bv[NCG * jj + cg], acc[jj][cg]);
    };
    float b0[4 * NCG], b1[4 * NCG];
    if constexpr (KR < NK) load_b(KR, b0);  // in flight during the register k-steps
#pragma unroll
    for (int st = 0; st < KR; ++st) kstep(st, bw[st]);
    if constexpr (KR < NK) {
#pragma unroll 1
      for (int st = KR; st < NK; st += 2) {
        load_b(st + 1, b1);
        kstep(st, b0);
        if (st + 2 < NK) load_b(st + 2, b0);
        kstep(st + 1, b1);
      }
    }
    }  // 16-tile group
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
      if constexpr (quad) {
        // lane = output channel; register i = tile i of the group
        if ((lane >> 5) == pass) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float m0 = acc4[0][i], m1 = acc4[1][i], m2 = acc4[2][i], m3 = acc4[3][i];
            const int off = i * TS + (lane & 31);
            t_s[(2 * wi) * TQ + off] = (m0 + m1) + m2;
            t_s[(2 * wi + 1) * TQ + off] = (m1 - m2) - m3;
          }
        }
      } else {
      // T_i[b] = sum_j M_ij A[j][b]: lane holds tiles 4 kq + rr of the group, channel 16 cg + tl
#pragma unroll
      for (int cgl = 0; cgl < CH / 16; ++cgl)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int cg = pass * (CH / 16) + cgl;
          const float m0 = acc[0][cg][rr], m1 = acc[1][cg][rr], m2 = acc[2][cg][rr], m3 = acc[3][cg][rr];
          const int off = (4 * kq + rr) * TS + 16 * cgl + tl;
          t_s[(2 * wi) * TQ + off] = (m0 + m1) + m2;
          t_s[(2 * wi + 1) * TQ + off] = (m1 - m2) - m3;
        }
      }
      __syncthreads();
      // Y[a][b] = sum_i A^T[a][i] T_i[b]: Y0b = T0b + T1b + T2b, Y1b = T1b - T2b - T3b; tile pixel q = 2a + b
#pragma unroll
      for (int k = 0; k < 16 * CH / 256; ++k) {
        const int it = tid + 256 * k;
        const int col = it % CH, tg = it / CH;
        const int tt = 16 * g + tg;
        const int co = pass * CH + col;
        float tv[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) tv[i][bb] = t_s[(2 * i + bb) * TQ + tg * TS + col];
        float y[4];
        y[0] = (tv[0][0] + tv[1][0]) + tv[2][0];
        y[1] = (tv[0][1] + tv[1][1]) + tv[2][1];
        y[2] = (tv[1][0] - tv[2][0]) - tv[3][0];
        y[3] = (tv[1][1] - tv[2][1]) - tv[3][1];
        if (tt < ntile) {
          const int ty = ty0 + tt / TXT, tx2 = tt % TXT;
          if constexpr (POOL) {
            const float bv = STAGE_BIAS ? b_s[STAGE_BIAS ? co : 0] : bias[co];
            float best = y[0] + bv;
            int arg = 0;
#pragma unroll
            for (int q = 1; q < 4; ++q) {
              const float z = y[q] + bv;
              if (z > best) { best = z; arg = q; }
            }
            const int pidx = (ty * PW + tx2) * CO + co;
            const float av = fmaxf(best, 0.0f);
            if (oc) {
              const bool keep = drop_keep(rseed, (uint32_t)pidx, THR_25);
              o[pidx] = keep ? av * SCALE_25 : 0.0f;
              oc[pidx] = (uint8_t)(arg | (keep ? CODE_KEEP : 0) | (best > 0.0f ? CODE_POS : 0));
            } else {
              o[pidx] = av;
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int yy = 2 * ty + (q >> 1), xx = 2 * tx2 + (q & 1);
              if (yy >= HO || xx >= WO) continue;
              const int o_i = (yy * WO + xx) * CO + co;
              if constexpr (EPI == EPI_FWD) {
                o[o_i] = fmaxf(y[q] + (STAGE_BIAS ? b_s[STAGE_BIAS ? co : 0] : bias[co]), 0.0f);
              } else if constexpr (EPI == EPI_BWD_MASK) {
                if constexpr (STAGE_EPI) {
                  o[o_i] = reinterpret_cast<const uint8_t*>(e_s)[((yy - 2 * ty0) * WO + xx) * CO + co] ? y[q] : 0.0f;
                } else {
                  o[o_i] = act[o_i] > 0.0f ? y[q] : 0.0f;
                }
              } else {  // dropout' + the pool's positive mask: the POOLED gradient of the layer below, whose
                        // argmax (code & 3) the consumers un-pool on the fly (a quarter of the dense dZ's bytes)
                const uint32_t c =
                    STAGE_EPI ? reinterpret_cast<const uint8_t*>(e_s)[((yy - 2 * ty0) * WO + xx) * CO + co] : cd[o_i];
                const float dv = (c & CODE_KEEP) ? y[q] * SCALE_25 : 0.0f;
                o[o_i] = (c & CODE_POS) ? dv : 0.0f;
              }
            }
          }
        }
      }
      __syncthreads();
    }
  };
#pragma unroll 1
  for (int g = 0; g < NG - (QUAD ? 1 : 0); ++g) {
    if (16 * g >= ntile) break;  // block-uniform
    run_group(g, IntC<0>{});
  }
  if constexpr (QUAD) run_group(NG - 1, IntC<1>{});
  }

}

// ------------------------------------------------------------------------------------------------
// Weight gradient of a 3x3 conv: dW[kyx][ci][co] = sum_{samples, pixels} X[p + (ky,kx) - PAD][ci] dZ[p][co],
// db[co] = sum dZ.  Block = (split sp, replica r): samples [WGS*sp, WGS*sp + WGS) in order, row bands of BR
// output rows; X band and dZ band staged in LDS (dZ rows padded to an even width WOE with zeros so a
// k-pair never straddles rows); the band's K loop is fully unrolled (compile-time LDS offsets).  Only the
// first HOV x WOV output pixels are used (conv4: row/col 12 are dropped by the pool, their dZ is 0).
// Row tiles: (kyx, 32 input channels); wave w owns row tiles w + NW*u and all CO/32 column tiles.  For
// CI = 3 (conv1) the 27 rows fit one tile and the waves split the band's rows instead (KSPLIT), reduced in
// LDS in wave order.  db: each thread sums the dZ elements it stages (fixed channel), reduced in order.
// ------------------------------------------------------------------------------------------------
struct WgArgs {
  const float* x;
  int x_mode;  // 0 slot-major activations, 1 dataset rows via idx
  const int32_t* idx;
  const int32_t* cnt;
  int bmax;
  int splits;
  const float* dz;
  float* wpart;
  int off_w, off_b;
  const uint8_t* dz_code;  // UPZ (wino_wgrad_kernel): dz is the POOLED gradient, un-pooled with these argmax codes
};

template <int HI, int WI, int CI, int CO, int PAD, int HOV, int WOV, int BR, int NW, int WPE = 0>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE > 0 ? WPE : 1, WPE > 0 ? WPE : 8)))
void wgrad_kernel(const WgArgs a) {
  constexpr int HO = HI + 2 * PAD - 2, WO = WI + 2 * PAD - 2;
  constexpr int WOE = WOV + (WOV & 1);
  constexpr int WXP = WI + 2 * PAD + 1;
  constexpr int NT = CO / 32;
  constexpr bool KSPLIT = (CI == 3);
  constexpr int MT = KSPLIT ? 1 : 9 * CI / 32;
  constexpr int UMW = KSPLIT ? 1 : MT / NW;
  constexpr int NTHR = NW * 64;
  constexpr int NB = (HOV + BR - 1) / BR;
  constexpr int RW = KSPLIT ? BR / NW : BR;  // rows of the band per wave
  constexpr int SW = RW * WOE / 2;           // k-steps per wave per band
  static_assert(KSPLIT ? (BR % NW == 0 && NT == 1) : (MT % NW == 0), "bad wave split");
  static_assert(NTHR % (CO / 4) == 0, "db accumulation needs a fixed channel quad per thread");
  static_assert(!KSPLIT || NW * 1024 <= BR * WOE * CO, "reduction scratch aliases the dZ band");
  __shared__ float x_s[(BR + 2) * WXP * CI];
  __shared__ float z_s[BR * WOE * CO];
  __shared__ fvec4 gb_s[NTHR];
  const int sp = blockIdx.x, r = blockIdx.y;
  const int count = a.cnt[r];
  const int j_begin = sp * WGS, j_end = min(count, j_begin + WGS);
  if (j_begin >= j_end) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int m = lane & 31, kh = lane >> 5;
  // per-lane operand bases
  int ab[UMW];
  int ci0[UMW];
  float amask = 1.0f;
#pragma unroll
  for (int u = 0; u < UMW; ++u) {
    if (KSPLIT) {
      const int mm = m < 27 ? m : 0;
      amask = m < 27 ? 1.0f : 0.0f;
      const int kyx = mm / 3, c = mm % 3;
      ab[u] = ((kyx / 3) * WXP + kyx % 3 + kh) * CI + c + wave * RW * WXP * CI;
      ci0[u] = 0;
    } else {
      const int mt = wave + NW * u;
      const int kyx = mt / (CI / 32);
      ci0[u] = (mt % (CI / 32)) * 32;
      ab[u] = ((kyx / 3) * WXP + kyx % 3 + kh) * CI + ci0[u] + m;
    }
  }
  const int zb = kh * CO + m + (KSPLIT ? wave * RW * WOE * CO : 0);
  floatx16 acc[UMW][NT];
#pragma unroll
  for (int u = 0; u < UMW; ++u)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[u][nt] = zero16();
  fvec4 gb = fvec4{0.0f, 0.0f, 0.0f, 0.0f};  // db partial of channels 4*(tid % (CO/4)) .. +3
  for (int j = j_begin; j < j_end; ++j) {
    const int64_t slot = (int64_t)r * a.bmax + j;
    const float* X = a.x_mode == 1 ? a.x + (int64_t)a.idx[slot] * (HI * WI * CI) : a.x + slot * (HI * WI * CI);
    const float* Z = a.dz + slot * (HO * WO * CO);
    for (int band = 0; band < NB; ++band) {
      const int y0 = band * BR;
      __syncthreads();  // previous band's readers done
      if constexpr (CI % 4 == 0) {  // 16-B loads, all in flight before the ds_write_b128 stores
        constexpr int C4 = CI / 4;
        constexpr int TOT = (BR + 2) * WXP * C4;
        constexpr int NIT = (TOT + NTHR - 1) / NTHR;
        fvec4 v[NIT];
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int e4 = tid + k * NTHR;
          const int pix = e4 / C4, c4 = e4 % C4;
          const int iy = y0 - PAD + pix / WXP, ix = pix % WXP - PAD;
          const bool ok = e4 < TOT && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
          const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? X + (iy * WI + ix) * CI + 4 * c4 : X);
          v[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
        }
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int e4 = tid + k * NTHR;
          if (e4 < TOT) *reinterpret_cast<fvec4*>(x_s + 4 * e4) = v[k];
        }
      } else {
        constexpr int TOT = (BR + 2) * WXP * CI;
        constexpr int NIT = (TOT + NTHR - 1) / NTHR;
        float v[NIT];
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int e = tid + k * NTHR;
          const int c = e % CI, pix = e / CI;
          const int iy = y0 - PAD + pix / WXP, ix = pix % WXP - PAD;
          const bool ok = e < TOT && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
          const float t = *(ok ? X + (iy * WI + ix) * CI + c : X);
          v[k] = ok ? t : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int e = tid + k * NTHR;
          if (e < TOT) x_s[e] = v[k];
        }
      }
      {
        constexpr int Z4 = CO / 4;  // each thread: one channel quad of dZ (db too)
        constexpr int TOT = BR * WOE * Z4;
        constexpr int NIT = (TOT + NTHR - 1) / NTHR;
        fvec4 v[NIT];
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int e4 = tid + k * NTHR;
          const int pix = e4 / Z4, c4 = e4 % Z4;
          const int yy = y0 + pix / WOE, xx = pix % WOE;
          const bool ok = e4 < TOT && yy < HOV && xx < WOV;
          const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? Z + (yy * WO + xx) * CO + 4 * c4 : Z);
          v[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
        }
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          const int e4 = tid + k * NTHR;
          if (e4 < TOT) {
            *reinterpret_cast<fvec4*>(z_s + 4 * e4) = v[k];
            gb += v[k];  // channel quad e4 % (CO/4) == tid % (CO/4): NTHR is a multiple of CO/4
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int s = 0; s < SW; ++s) {
        const int yl = (2 * s) / WOE, xl = (2 * s) % WOE;
        float bz[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bz[nt] = z_s[zb + (yl * WOE + xl) * CO + nt * 32];
#pragma unroll
        for (int u = 0; u < UMW; ++u) {
          float av = x_s[ab[u] + (yl * WXP + xl) * CI];
          if (KSPLIT) av *= amask;
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[u][nt] = mfma32(av, bz[nt], acc[u][nt]);
        }
      }
    }
  }
  float* out = a.wpart + ((int64_t)r * a.splits + sp) * WPART;
  gb_s[tid] = gb;
  if (KSPLIT) {
    __syncthreads();  // all MFMA readers of z_s done: reuse it as the wave-reduction scratch
    float* red = z_s;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) red[wave * 1024 + acc_row(reg, kh) * 32 + m] = acc[0][0][reg];
    __syncthreads();
    for (int e = tid; e < 27 * 32; e += NTHR) {
      float s = 0.0f;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += red[w * 1024 + e];
      out[a.off_w + e] = s;  // row e/32 = kyx*3 + c, column co: Keras [ky][kx][ci][co] order
    }
  } else {
#pragma unroll
    for (int u = 0; u < UMW; ++u) {
      const int kyx = (wave + NW * u) / (CI / 32);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int ci = ci0[u] + acc_row(reg, kh);
          out[a.off_w + (kyx * CI + ci) * CO + nt * 32 + m] = acc[u][nt][reg];
        }
    }
    __syncthreads();
  }
  if (tid < CO) {  // channel tid: quad tid/4 of threads tid/4 + (CO/4)*i, summed in thread order
    constexpr int Z4 = CO / 4;
    float s = 0.0f;
    for (int i = 0; i < NTHR / Z4; ++i) s += gb_s[tid / 4 + Z4 * i][tid % 4];
    out[a.off_b + tid] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// Wave-local variant of wino_kernel for the CO = 32 layers (conv2 forward, conv2 and conv3 data gradients):
// each wave owns one 16-tile group and ALL 16 transform points for the 32 output channels (2 x 16 accumulators
// of 16x16x4), so the output transform and the epilogue stay in registers (no LDS round trip, no barrier after
// the staging).  Per k-step (4 input channels) a lane reads its tile's 4x4 patch (16 LDS values), forms the 16
// values of V with 32 adds and issues 32 MFMAs with U from L2 (32 B operands, loaded one k-step ahead):
// half the LDS reads and 2/3 of the VALU per MFMA of the row-per-wave form at CO = 32 (which issues 8 MFMAs
// per 8 reads and 12 adds).  NW waves per block = the band's 16-tile groups.
// ------------------------------------------------------------------------------------------------
template <int HI, int WI, int CI, int CO, int PAD, int BTY, int NW, int EPI, int UPI = 0>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_wl_kernel(const ConvArgs a) {
  static_assert(EPI != EPI_BWD_UNPOOL, "the pooled-gradient epilogue (EPI_BWD_UNPOOL) is wino_kernel's");
  constexpr bool POOL = (EPI == EPI_FWD_POOL);
  constexpr int HO = HI + 2 * PAD - 2, WO = WI + 2 * PAD - 2;
  constexpr int PH = HO / 2, PW = WO / 2;
  constexpr int TYT = POOL ? PH : (HO + 1) / 2;
  constexpr int TXT = POOL ? PW : (WO + 1) / 2;
  constexpr int LR = 2 * BTY + 2, LC = 2 * TXT + 2;
  constexpr int CIP = CI + 1;
  constexpr int ROWP = LC * CIP + ((TXT - LC * CIP) % 16 + 16) % 16;  // conflict-free V reads, as wino_kernel's
  static_assert(CIP % 16 == 1 && ROWP % 16 == TXT % 16, "conflict-free V reads");
  constexpr int NK = CI / 4;
  constexpr int NTHR = NW * 64;
  static_assert(CO == 32 && CI % 8 == 0, "wave-local form: 32 output channels");
  static_assert(NW * 16 >= BTY * TXT, "one 16-tile group per wave");
  __shared__ float in_s[LR * ROWP];
  // (plain block order: the XCD-aware order measured +1-2 % on these wave-local kernels, scripts/r04/gpu_wlpm_es.sh)
  const int band = blockIdx.x, j = blockIdx.y, r = blockIdx.z;
  const int count = a.cnt ? a.cnt[r] : a.cnt_all;
  if (j >= count) return;
  const int tid = threadIdx.x;
  const int64_t slot = (int64_t)r * a.bmax + j;
  constexpr int IN_SZ = UPI ? (HI / 2) * (WI / 2) * CI : HI * WI * CI;  // UPI: a pooled gradient's slots
  const float* src = a.in_mode == 2 ? a.in + (int64_t)(a.row_base + j) * IN_SZ : a.in + slot * IN_SZ;
  const int ty0 = band * BTY;
  const int bty = min(BTY, TYT - ty0);
  const int ntile = bty * TXT;
  if constexpr (UPI) {  // the input is a POOLED gradient [HI/2][WI/2][CI] with its pool codes: un-pooled here
    static_assert(PAD % 2 == 0 && LR % 2 == 0 && LC % 2 == 0, "the staged region must be whole pooling windows");
    stage_unpool<HI / 2, WI / 2, CI, LR, LC, CIP, NTHR, ROWP>(src, a.code_in + slot * ((HI / 2) * (WI / 2) * CI),
                                                              2 * ty0 - PAD, -PAD, in_s, tid);
  } else {
    constexpr int C4 = CI / 4;
    constexpr int TOT = LR * LC * C4;
    constexpr int NIT = (TOT + NTHR - 1) / NTHR;
    fvec4 v[NIT];
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e4 = tid + k * NTHR;
      const int pix = e4 / C4, c4 = e4 % C4;
      const int iy = 2 * ty0 - PAD + pix / LC, ix = pix % LC - PAD;
      const bool ok = e4 < TOT && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
      const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? src + (iy * WI + ix) * CI + 4 * c4 : src);
      v[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
    }
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int e4 = tid + k * NTHR;
      if (e4 < TOT) {
        const int pix = e4 / C4;
        float* d = in_s + (pix / LC) * ROWP + (pix % LC) * CIP + 4 * (e4 % C4);
        d[0] = v[k].x;
        d[1] = v[k].y;
        d[2] = v[k].z;
        d[3] = v[k].w;
      }
    }
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  if (16 * wave >= ntile) return;  // wave-uniform; no barrier follows
  const int tl = lane & 15, kq = lane >> 4;
  const int tile = min(16 * wave + tl, ntile - 1);
  const float* dpa = in_s + (2 * (tile / TXT)) * ROWP + 2 * (tile % TXT) * CIP + kq;
  // B operands of k-step st: U[4 st + kq][16 cg + tl][xi] (the xi-last layout of wino_u_kernel's conv2 section):
  // a lane's 16 transform points of one channel pair are 64 contiguous bytes, 4 x 16-B loads per cg
  const fvec4* Ub = reinterpret_cast<const fvec4*>(a.w + (int64_t)r * a.w_rstride) + (kq * CO + tl) * 4;
  auto load_b = [&](int st, float (&bv)[32]) {
#pragma unroll
    for (int cg = 0; cg < 2; ++cg)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const fvec4 u = Ub[((4 * st) * CO + 16 * cg) * 4 + q];
        bv[2 * (4 * q + 0) + cg] = u.x;
        bv[2 * (4 * q + 1) + cg] = u.y;
        bv[2 * (4 * q + 2) + cg] = u.z;
        bv[2 * (4 * q + 3) + cg] = u.w;
      }
  };
  fvec4 acc[16][2];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) acc[xi][0] = acc[xi][1] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  // The patch of k-step st + 1 is read right after k-step st's V is formed (its registers are free then), so
  // that its LDS latency is covered by k-step st's 32 MFMAs instead of stalling ahead of the next k-step's.
  float pn[16];  // [row][col]
  auto load_patch = [&](int st) {
    const float* d0 = dpa + 4 * st;
#pragma unroll
    for (int rr2 = 0; rr2 < 4; ++rr2)
#pragma unroll
      for (int c = 0; c < 4; ++c) pn[4 * rr2 + c] = d0[rr2 * ROWP + c * CIP];
  };
  load_patch(0);
  auto kstep = [&](int st, const float (&bv)[32]) {
    float t[4][4];  // t[i][c] = (B^T d)[i][c]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float d_0 = pn[c], d_1 = pn[4 + c], d_2 = pn[8 + c], d_3 = pn[12 + c];
      t[0][c] = d_0 - d_2;
      t[1][c] = d_1 + d_2;
      t[2][c] = d_2 - d_1;
      t[3][c] = d_1 - d_3;
    }
    __builtin_amdgcn_sched_barrier(0);
    if (st + 1 < NK) load_patch(st + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v0 = t[i][0] - t[i][2], v1 = t[i][1] + t[i][2], v2 = t[i][2] - t[i][1], v3 = t[i][1] - t[i][3];
#pragma unroll
      for (int cg = 0; cg < 2; ++cg) {
        acc[4 * i + 0][cg] = mfma16(v0, bv[2 * (4 * i + 0) + cg], acc[4 * i + 0][cg]);
        acc[4 * i + 1][cg] = mfma16(v1, bv[2 * (4 * i + 1) + cg], acc[4 * i + 1][cg]);
        acc[4 * i + 2][cg] = mfma16(v2, bv[2 * (4 * i + 2) + cg], acc[4 * i + 2][cg]);
        acc[4 * i + 3][cg] = mfma16(v3, bv[2 * (4 * i + 3) + cg], acc[4 * i + 3][cg]);
      }
    }
  };
  // EPI_BWD_MASK: the epilogue's ReLU' operand (the layer input a, 8 values per tile row and lane) is loaded during
  // the last k-step, so that its latency is covered by that k-step's 32 MFMAs (all 4 rows: conv2's data gradient
  // -40 %, 2 registers spilled; 2 rows -25 %, 1 row -13 %; the peeled loop alone -4 %; bit-identical)
  constexpr bool PRE_MASK = (EPI == EPI_BWD_MASK);
  constexpr int PRE_RR = 4;  // tile rows of the ReLU' operand loaded during the last k-step
  float mk[PRE_MASK && PRE_RR > 0 ? 8 * PRE_RR : 1];
  auto load_mask = [&]() {
    const float* ax = a.aux + slot * (HO * WO * CO);
#pragma unroll
    for (int rr = 0; rr < PRE_RR; ++rr) {
      const int tt = min(16 * wave + 4 * kq + rr, ntile - 1);
      const int ty = ty0 + tt / TXT, tx2 = tt % TXT;
#pragma unroll
      for (int cg = 0; cg < 2; ++cg)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int yy = min(2 * ty + (q >> 1), HO - 1), xx = min(2 * tx2 + (q & 1), WO - 1);
          mk[(rr * 2 + cg) * 4 + q] = ax[(yy * WO + xx) * CO + 16 * cg + tl];
        }
    }
  };
  // EPI_FWD_POOL: the lane's two bias values likewise (conv2 forward -4 %)
  constexpr bool PRE_BIAS = POOL;
  float bpre[2] = {0.0f, 0.0f};
  float b0[32], b1[32];
  load_b(0, b0);
  static_assert(NK % 2 == 0 && NK >= 2, "k-steps in pairs");
#pragma unroll 1
  for (int st = 0; st < NK - 2; st += 2) {
    load_b(st + 1, b1);
    kstep(st, b0);
    load_b(st + 2, b0);
    kstep(st + 1, b1);
  }
  // the last pair peeled: b0 is dead after k-step NK - 2, its registers take the mask operand
  load_b(NK - 1, b1);
  kstep(NK - 2, b0);
  if constexpr (PRE_MASK) load_mask();
  if constexpr (PRE_BIAS) {
    bpre[0] = a.bias[(int64_t)r * a.b_rstride + tl];
    bpre[1] = a.bias[(int64_t)r * a.b_rstride + 16 + tl];
  }
  kstep(NK - 1, b1);
  if constexpr (PRE_MASK) {  // the loads stay ahead of the last k-step (not sunk to their use)
#pragma unroll
    for (int i = 0; i < 8 * PRE_RR; ++i) asm volatile("" : "+v"(mk[i]));
  }
  if constexpr (PRE_BIAS) asm volatile("" : "+v"(bpre[0]), "+v"(bpre[1]));
  // output transform in registers: lane holds M[xi][tile 4 kq + rr][co 16 cg + tl]
  float* o = a.out + slot * ((POOL ? PH * PW : HO * WO) * CO);
  const uint32_t rseed = (POOL && a.drop_key) ? drop_row_seed(a.drop_key[r], a.drop_layer, (uint32_t)j) : 0u;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int tt = 16 * wave + 4 * kq + rr;
    if (tt >= ntile) continue;
    const int ty = ty0 + tt / TXT, tx2 = tt % TXT;
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
      const int co = 16 * cg + tl;
      float tv[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float m0 = acc[4 * i][cg][rr], m1 = acc[4 * i + 1][cg][rr], m2 = acc[4 * i + 2][cg][rr],
                    m3 = acc[4 * i + 3][cg][rr];
        tv[i][0] = (m0 + m1) + m2;
        tv[i][1] = (m1 - m2) - m3;
      }
      float y[4];
      y[0] = (tv[0][0] + tv[1][0]) + tv[2][0];
      y[1] = (tv[0][1] + tv[1][1]) + tv[2][1];
      y[2] = (tv[1][0] - tv[2][0]) - tv[3][0];
      y[3] = (tv[1][1] - tv[2][1]) - tv[3][1];
      if constexpr (POOL) {
        const float bv = PRE_BIAS ? bpre[cg] : a.bias[(int64_t)r * a.b_rstride + co];
        float best = y[0] + bv;
        int arg = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q) {
          const float z = y[q] + bv;
          if (z > best) { best = z; arg = q; }
        }
        const int pidx = (ty * PW + tx2) * CO + co;
        const float av = fmaxf(best, 0.0f);
        if (a.drop_key) {
          const bool keep = drop_keep(rseed, (uint32_t)pidx, THR_25);
          o[pidx] = keep ? av * SCALE_25 : 0.0f;
          a.code_out[slot * (PH * PW * CO) + pidx] =
              (uint8_t)(arg | (keep ? CODE_KEEP : 0) | (best > 0.0f ? CODE_POS : 0));
        } else {
          o[pidx] = av;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int yy = 2 * ty + (q >> 1), xx = 2 * tx2 + (q & 1);
          if (yy >= HO || xx >= WO) continue;
          const int o_i = (yy * WO + xx) * CO + co;
          if constexpr (EPI == EPI_BWD_MASK) {
            const float av = rr < PRE_RR ? mk[((rr < PRE_RR ? rr : 0) * 2 + cg) * 4 + q]
                                         : a.aux[slot * (HO * WO * CO) + o_i];
            o[o_i] = av > 0.0f ? y[q] : 0.0f;
          } else {
            o[o_i] = fmaxf(y[q] + a.bias[(int64_t)r * a.b_rstride + co], 0.0f);
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient of conv2..conv4 in Winograd form F(3x3, 2x2) (the transposed dual of the forward's
// F(2x2, 3x3)): with Y = A^T [U (.) V] A per 2x2 output tile, dL/dU = (A dY A^T) (.) V, so
//   dW[3x3] = G^T [ sum_tiles (A dY A^T) (.) (B^T d B) ] G
// per (ci, co), the sum over the tiles of the split's samples running in the transformed domain as 16 GEMMs
// M[xi][ci][co] = sum_tiles V[xi][tile][ci] D[xi][tile][co] on v_mfma_f32_16x16x4_f32 (K = tiles, 4 per
// k-step): 2.25x fewer multiply-adds than the direct sum.  Only the first HOV x WOV output pixels enter
// (conv4: row / column 12 are dropped by the pool, their dZ is 0); the tile grid covers them (zero beyond).
// Block = (split sp, replica r, input-channel chunk of CIB), 4 waves; wave i owns transform row i (xi = 4i ..
// 4i+3): 4 x CIB/16 x CO/16 accumulators.  Per band (BTY tile rows of one sample) the input rows (channels of
// the chunk) and the dZ rows are staged in LDS; per k-step a lane forms V of its tile for CIB/16 channels
// (8 reads, 12 adds each) and D = A dY A^T for CO/16 channels (4 reads, 6 adds each).  At the end the waves
// fold their row of the inverse transform (P_i = M_i G) and exchange it through LDS, 16 input channels at a
// time.  Samples, bands and tiles in a fixed order: sums independent of which replicas share the launch.
// ------------------------------------------------------------------------------------------------
template <int HI, int WI, int CI, int CO, int PAD, int HOV, int WOV, int BTY, int CIB, int UPZ = 0, int PIPE = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void wino_wgrad_kernel(const WgArgs a) {
  constexpr int HO = HI + 2 * PAD - 2, WO = WI + 2 * PAD - 2;
  constexpr int TY = (HOV + 1) / 2, TX = (WOV + 1) / 2;
  constexpr int NB = (TY + BTY - 1) / BTY;
  constexpr int LR = 2 * BTY + 2, LC = 2 * TX + 2;
  // channel strides padded by 8 (not 1): a half-wave reads 16 channels (tl) of 2 adjacent tiles (kq), 2 CIP apart;
  // 2 CIP = 16 (mod 32) puts the two tiles on opposite halves of the 32 banks (CIB + 1 gave 2-way conflicts):
  // conv2 / conv4 weight gradients -2.5 % / -2.7 %, bit-identical (profiles/r05_ab_wgrad_lds_pad.txt)
  constexpr int CIP = CIB + 8;
  constexpr int XROW = LC * CIP;
  constexpr int ZR = 2 * BTY, ZC = 2 * TX;
  constexpr int COP = CO + 8;
  constexpr int NH = CIB / 16, NCG = CO / 16;
  constexpr int XS = LR * XROW, ZS = ZR * ZC * COP;
  constexpr int PS = 4 * 3 * 16 * CO;  // the four waves' P_i for 16 input channels
  constexpr int SM = (XS + ZS > PS) ? XS + ZS : PS;
  static_assert(CI % CIB == 0 && CIB % 16 == 0 && CO % 16 == 0, "channel chunks");
  __shared__ float smem[SM];
  __shared__ fvec4 gb_s[256];
  float* const x_s = smem;
  float* const z_s = smem + XS;
  const int sp = blockIdx.x, r = blockIdx.y, chn = blockIdx.z;
  const int count = a.cnt[r];
  const int j_begin = sp * WGS, j_end = min(count, j_begin + WGS);
  if (j_begin >= j_end) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wi = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: the row's signs below live in SGPRs
  const int tl = lane & 15, kq = lane >> 4;
  // The wave's transform row as data (round 6: one loop for all waves, every barrier in code all waves share; round 5
  // compiled the sample loop once per wave with its barriers inside a wave-uniform switch).  V's row i of B^T d B is
  // s_a d[ra] + s_b d[rb], written as ONE fma by +-1 (the correctly rounded value of the same two exact terms: the
  // same bits as an add / subtract): t = fmaf(sq, d[tq], d[tp]).  D's row i of A dY (y0 | y0 + y1 | y0 - y1 | -y1)
  // likewise as fmaf(c, y[zq], y[zp]) with c = 0 for rows 0 and 3.  Row 3 computes -V and -D instead of V and D
  // (d3 - d1 and y1): every product V D is unchanged (a sign flip is exact on both factors), and the zero products
  // of c = 0 never reach a result (the accumulators start at +0; adding +-0 leaves a sum unchanged), so the
  // weight gradients are bit-identical to the per-wave copies.
  const int tp = wi;                                                     // + row of B^T: 0 | 1 | 2 | 3
  const int tq = (wi <= 1) ? 2 : 1;                                      // the other:    2 | 2 | 1 | 1
  const float sq = (wi == 1) ? 1.0f : -1.0f;
  const float cz = (wi == 1) ? 1.0f : ((wi == 2) ? -1.0f : 0.0f);       // A's row: y[zp] + cz y[zq]
  const int zpo = (wi == 3) ? ZC * COP : 0;                              // offsets of the y rows zp / zq in z_s
  const int zqo = (wi == 3) ? 0 : ZC * COP;
  fvec4 acc[4][NH][NCG];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj)
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int cg = 0; cg < NCG; ++cg) acc[jj][h][cg] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  fvec4 gb = fvec4{0.0f, 0.0f, 0.0f, 0.0f};  // db partial of channels 4 * (tid % (CO / 4)) .. + 3
  const int drow = (tq - tp) * XROW;
  // staging of (sample, band) in two halves: the global loads into registers, then the LDS images.  PIPE: the
  // next band's loads are issued right after this band's LDS stores, so that they land during this band's MFMAs
  // (the same values in the same places: bit-identical); otherwise loads and stores back to back.
  constexpr int C4X = CIB / 4;
  constexpr int TOTX = LR * LC * C4X;
  constexpr int NITX = (TOTX + 255) / 256;
  using ZU = UnpoolShape<CO, ZR, ZC, 256>;
  constexpr int Z4 = CO / 4;
  constexpr int TOTZ = ZR * ZC * Z4;
  constexpr int NITZ = UPZ ? ZU::NIT : (TOTZ + 255) / 256;
  static_assert(UPZ || 256 % Z4 == 0, "db needs a fixed channel quad per thread");
  static_assert(!UPZ || (ZR % 2 == 0 && ZC % 2 == 0 && HOV == 2 * (HO / 2) && WOV == 2 * (WO / 2)), "whole windows");
  fvec4 xv[NITX], zv[NITZ];
  uint32_t zc[UPZ ? NITZ : 1];
  auto stage_load = [&](int jj, int bnd) {
    const int64_t sl = (int64_t)r * a.bmax + jj;
    const float* X = a.x + sl * (HI * WI * CI) + chn * CIB;
    const float* Z = a.dz + sl * (UPZ ? (HO / 2) * (WO / 2) * CO : HO * WO * CO);  // UPZ: pooled slots
    const int ty0 = bnd * BTY;
#pragma unroll
    for (int k = 0; k < NITX; ++k) {  // input rows 2 ty0 - PAD .., columns -PAD .., the chunk's channels
      const int e4 = tid + k * 256;
      const int pix = e4 / C4X, c4 = e4 % C4X;
      const int iy = 2 * ty0 - PAD + pix / LC, ix = pix % LC - PAD;
      const bool ok = e4 < TOTX && iy >= 0 && iy < HI && ix >= 0 && ix < WI;
      const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? X + (iy * WI + ix) * CI + 4 * c4 : X);
      xv[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    if constexpr (UPZ) {  // pooled dZ [HO/2][WO/2][CO] with its codes, un-pooled window-major
      unpool_load<HO / 2, WO / 2, CO, ZR, ZC, 256>(Z, a.dz_code + sl * ((HO / 2) * (WO / 2) * CO), 2 * ty0, 0, tid,
                                                  zv, zc);
    } else {  // dZ rows 2 ty0 .. (zero beyond HOV x WOV)
#pragma unroll
      for (int k = 0; k < NITZ; ++k) {
        const int e4 = tid + k * 256;
        const int pix = e4 / Z4, c4 = e4 % Z4;
        const int yy = 2 * ty0 + pix / ZC, xx = pix % ZC;
        const bool ok = e4 < TOTZ && yy < HOV && xx < WOV;
        const fvec4 t = *reinterpret_cast<const fvec4*>(ok ? Z + (yy * WO + xx) * CO + 4 * c4 : Z);
        zv[k] = ok ? t : fvec4{0.0f, 0.0f, 0.0f, 0.0f};
      }
    }
  };
  auto stage_store = [&]() {
#pragma unroll
    for (int k = 0; k < NITX; ++k) {
      const int e4 = tid + k * 256;
      if (e4 < TOTX) {
        float* d = x_s + (e4 / C4X) * CIP + 4 * (e4 % C4X);
        d[0] = xv[k].x;
        d[1] = xv[k].y;
        d[2] = xv[k].z;
        d[3] = xv[k].w;
      }
    }
    if constexpr (UPZ) {
      unpool_store<CO, ZR, ZC, COP, 256>(z_s, tid, zv, zc);  // db below, from the staged image
    } else {
#pragma unroll
      for (int k = 0; k < NITZ; ++k) {
        const int e4 = tid + k * 256;
        if (e4 < TOTZ) {
          float* d = z_s + (e4 / Z4) * COP + 4 * (e4 % Z4);
          d[0] = zv[k].x;
          d[1] = zv[k].y;
          d[2] = zv[k].z;
          d[3] = zv[k].w;
          gb += zv[k];  // db from the same values (chunk 0 only); rows beyond HOV / WOV hold 0
        }
      }
    }
  };
  if constexpr (PIPE) stage_load(j_begin, 0);
  for (int j = j_begin; j < j_end; ++j) {
#pragma unroll 1
    for (int band = 0; band < NB; ++band) {
      const int ty0 = band * BTY;
      const int bty = min(BTY, TY - ty0);
      __syncthreads();  // the previous band's readers are done
      if constexpr (!PIPE) stage_load(j, band);
      stage_store();
      if constexpr (PIPE) {  // the next band (or the next sample's first) in flight during this band's MFMAs
        const bool last = band + 1 == NB;
        if (!last || j + 1 < j_end) stage_load(last ? j + 1 : j, last ? 0 : band + 1);
      }
      __syncthreads();
      if constexpr (UPZ) {  // db from the staged image, summed in the dense staging's order (bit-identical)
        if (chn == 0) {
          constexpr int Z4 = CO / 4;
          constexpr int TOT = ZR * ZC * Z4;
          static_assert(256 % Z4 == 0, "db needs a fixed channel quad per thread");
#pragma unroll
          for (int k = 0; k < (TOT + 255) / 256; ++k) {
            const int e4 = tid + k * 256;
            if (e4 < TOT) {
              const float* d = z_s + (e4 / Z4) * COP + 4 * (e4 % Z4);
              gb += fvec4{d[0], d[1], d[2], d[3]};
            }
          }
        }
      }
      const int ntile = bty * TX;
#pragma unroll 1
      for (int t0 = 0; t0 < ntile; t0 += 4) {
        const int tile = t0 + kq;
        const bool ok = tile < ntile;
        const int tc = ok ? tile : 0;
        const int tyl = tc / TX, tx = tc % TX;
        float va[NH][4];
        const float* d0 = x_s + ((2 * tyl + tp) * LC + 2 * tx) * CIP + tl;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          float t[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float da = d0[c * CIP + 16 * h], db = d0[drow + c * CIP + 16 * h];
            t[c] = fmaf(sq, db, da);
          }
          va[h][0] = ok ? t[0] - t[2] : 0.0f;
          va[h][1] = ok ? t[1] + t[2] : 0.0f;
          va[h][2] = ok ? t[2] - t[1] : 0.0f;
          va[h][3] = ok ? t[1] - t[3] : 0.0f;
        }
        float db[NCG][4];
        const float* z0 = z_s + ((2 * tyl) * ZC + 2 * tx) * COP + tl;
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) {
          const float yp0 = z0[zpo + 16 * cg], yp1 = z0[zpo + COP + 16 * cg];
          const float yq0 = z0[zqo + 16 * cg], yq1 = z0[zqo + COP + 16 * cg];
          const float r0 = fmaf(cz, yq0, yp0), r1 = fmaf(cz, yq1, yp1);  // row i of A dY (row 3: its negation)
          db[cg][0] = r0;
          db[cg][1] = r0 + r1;
          db[cg][2] = r0 - r1;
          db[cg][3] = -r1;
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) acc[jj][h][cg] = mfma16(va[h][jj], db[cg][jj], acc[jj][h][cg]);
      }
    }
  }
  // inverse transform dW[ky][kx] = sum_i G^T[ky][i] P_i[kx], P_i[kx] = sum_j M[i][j] G[j][kx]; lane holds
  // ci 16 h + 4 kq + rr (of the chunk), co 16 cg + tl
  float* out = a.wpart + ((int64_t)r * a.splits + sp) * WPART;
  gb_s[tid] = gb;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    __syncthreads();  // the last band's readers (or the previous chunk's) are done with smem
    float* px = smem + wi * (3 * 16 * CO);
#pragma unroll
    for (int cg = 0; cg < NCG; ++cg)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float m0 = acc[0][h][cg][rr], m1 = acc[1][h][cg][rr], m2 = acc[2][h][cg][rr], m3 = acc[3][h][cg][rr];
        const int o = (4 * kq + rr) * CO + 16 * cg + tl;
        px[o] = (m0 + 0.5f * m1) + 0.5f * m2;
        px[16 * CO + o] = 0.5f * m1 - 0.5f * m2;
        px[32 * CO + o] = (0.5f * m1 + 0.5f * m2) + m3;
      }
    __syncthreads();
    for (int e = tid; e < 16 * CO; e += 256) {  // (ci of the group, co)
      const int ci = chn * CIB + 16 * h + e / CO, co = e % CO;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float p0 = smem[0 * 3 * 16 * CO + kx * 16 * CO + e], p1 = smem[1 * 3 * 16 * CO + kx * 16 * CO + e];
        const float p2 = smem[2 * 3 * 16 * CO + kx * 16 * CO + e], p3 = smem[3 * 3 * 16 * CO + kx * 16 * CO + e];
        out[a.off_w + ((0 * 3 + kx) * CI + ci) * CO + co] = (p0 + 0.5f * p1) + 0.5f * p2;
        out[a.off_w + ((1 * 3 + kx) * CI + ci) * CO + co] = 0.5f * p1 - 0.5f * p2;
        out[a.off_w + ((2 * 3 + kx) * CI + ci) * CO + co] = (0.5f * p1 + 0.5f * p2) + p3;
      }
    }
  }
  __syncthreads();
  if (chn == 0 && tid < CO) {  // channel tid: quad tid / 4 of threads tid / 4 + (CO / 4) i, summed in thread order
    constexpr int Z4 = CO / 4;
    float s = 0.0f;
    for (int i = 0; i < 256 / Z4; ++i) s += gb_s[tid / 4 + Z4 * i][tid % 4];
    out[a.off_b + tid] = s;
  }
}

// RMSprop on W1..b4 (params [0, OFF_W5)) from the split partials, splits summed in order.
__device__ __forceinline__ bool small_param(int e) {
  return (e < OFF_W1 + 864) || (e >= OFF_B1 && e < OFF_B1 + 32) || (e >= OFF_W2 && e < OFF_B2 + 32) ||
         (e >= OFF_W3 && e < OFF_B3 + 64) || (e >= OFF_W4 && e < OFF_B4 + 64);
}

__global__ void rmsprop_small_kernel(const int32_t* __restrict__ cnt, const int32_t* __restrict__ opt_t, int splits,
                                     const float* __restrict__ wpart, float* __restrict__ params,
                                     float* __restrict__ rms, float lr, float rho, float omr, float decay, float eps) {
  const int r = blockIdx.y;
  const int count = cnt[r];
  if (count == 0) return;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= OFF_W5 || !small_param(e)) return;
  const float* w = wpart + (int64_t)r * splits * WPART + e;
  const int used = (count + WGS - 1) / WGS;
  float g = 0.0f;
  for (int s = 0; s < used; ++s) g += w[(int64_t)s * WPART];
  const RmsCfg cfg = rms_cfg(opt_t[r], lr, rho, omr, decay, eps);
  const int64_t o = (int64_t)r * STRIDE + e;
  rms_apply(params[o], rms[o], g, cfg);
}

// ------------------------------------------------------------------------------------------------
// Dense(512) + ReLU (+ dropout .5 when training): H[slot][n] = relu(sum_k D4[slot][k] W5[k][n] + b5[n]).
// Block = 32 samples x 128 columns (4 waves x 32); A staged in LDS, W5 streamed.
// ------------------------------------------------------------------------------------------------
constexpr int DF_K = 32;  // dense5_fwd: rows of W5 per K chunk (the MFMA chain order is the same for any): 32 -2 % vs
                          // 64 (76 registers, more waves); 128 / 192 +6 % / +30 % (219 / 256 registers)
static_assert(FEAT % DF_K == 0, "dense5_fwd K chunks");

__global__ __launch_bounds__(256) void dense5_fwd_kernel(const float* __restrict__ A, const int32_t* __restrict__ cnt,
                                                         int cnt_all, int bmax, const float* __restrict__ params,
                                                         int64_t stride, const float* __restrict__ glob,
                                                         const int32_t* __restrict__ w5src,
                                                         const uint64_t* __restrict__ drop_key,
                                                         float* __restrict__ H, uint8_t* __restrict__ code) {
  __shared__ float a_s[32 * (DF_K + 1)];
  const LogicalBlock lbk = xcd_block3();  // (sample tile, column slice, replica): a replica's W5 in one XCD's L2
  const int r = lbk.z;
  const int m0 = lbk.x * 32;
  const int count = cnt ? cnt[r] : cnt_all;
  if (m0 >= count) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int n0 = lbk.y * 128 + wave * 32;
  const int kh = lane >> 5;
  const float* Ar = A + (int64_t)r * bmax * FEAT;
  const int gsrc = w5src ? w5src[r] : -1;  // W5 of a round's first step: the coalition row (not broadcast)
  const float* W = (gsrc >= 0 ? glob + (int64_t)gsrc * stride : params + (int64_t)r * stride) + OFF_W5;
  floatx16 acc = zero16();
  // software pipeline over K chunks: the next chunk's A tile (8 values per thread) and W5 column slice
  // (32 values per lane) load into registers while this chunk's 32 MFMAs run
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
  const int col = n0 + (lane & 31);
  const float bias = params[(int64_t)r * stride + OFF_B5 + col];
  const uint64_t dkey = drop_key ? drop_key[r] : 0ull;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = m0 + acc_row(reg, kh);
    if (row < count) {
      const float z = acc[reg] + bias;
      const float h = fmaxf(z, 0.0f);
      const int64_t o = ((int64_t)r * bmax + row) * HID + col;
      if (drop_key) {
        const bool keep = drop_keep(drop_row_seed(dkey, DROP_L5, (uint32_t)row), (uint32_t)col, THR_50);
        H[o] = keep ? h * SCALE_50 : 0.0f;
        code[o] = (uint8_t)((keep ? CODE_KEEP : 0) | (z > 0.0f ? CODE_POS : 0));
      } else {
        H[o] = h;
      }
    }
  }
}

// The same Dense(512) forward in blocks of 16 samples x 64 columns on v_mfma_f32_16x16x4f32 (wave = 16 columns):
// at TMCS batch sizes (15-16 samples per replica) one m-tile without idle rows, and twice the waves of the 32 x 128
// form streaming W5: -13 % at 260 replicas, -18 % at 140 (profiles/r05_ab_dense5_fwd16.txt).  Bit-identical to it:
// both matrix-core forms accumulate each output as the fmaf chain over k in order.  Launched for
// B <= MPLC_D5F16_MAX slots; larger B (the evaluation's sample chunks) keeps the 32-row form, which reads W5 half as
// often.  The variant library (build_native.VARIANTS, MPLC_D5F16_MAX=0) runs the 32-row form everywhere, and
// tests/test_variants_gpu.py holds the two to the same bits.
#ifndef MPLC_D5F16_MAX
#define MPLC_D5F16_MAX 16
#endif
__global__ __launch_bounds__(256) void dense5_fwd16_kernel(const float* __restrict__ A, const int32_t* __restrict__ cnt,
                                                           int cnt_all, int bmax, const float* __restrict__ params,
                                                           int64_t stride, const float* __restrict__ glob,
                                                           const int32_t* __restrict__ w5src,
                                                           const uint64_t* __restrict__ drop_key,
                                                           float* __restrict__ H, uint8_t* __restrict__ code) {
  // A rows at a stride of DF_K + 2 (round 6): a half-wave's ds_read_b32 takes rows tl = 0..15 at
  // k-offsets kq and kq + 1, banks 2 tl + kq: 32 distinct (DF_K + 1 put row tl + 1's kq on row tl's kq + 1: 2-way,
  // PMC conflict ratio 0.44).  Layout only: bit-identical.
  constexpr int AS = DF_K + 2;
  __shared__ float a_s[16 * AS];
  const LogicalBlock lbk = xcd_block3();  // (sample tile, column slice, replica): a replica's W5 in one XCD's L2
  const int r = lbk.z;
  const int m0 = lbk.x * 16;
  const int count = cnt ? cnt[r] : cnt_all;
  if (m0 >= count) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int n0 = lbk.y * 64 + wave * 16;
  const int tl = lane & 15, kq = lane >> 4;
  const float* Ar = A + (int64_t)r * bmax * FEAT;
  const int gsrc = w5src ? w5src[r] : -1;
  const float* W = (gsrc >= 0 ? glob + (int64_t)gsrc * stride : params + (int64_t)r * stride) + OFF_W5;
  fvec4 acc = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  constexpr int AIT = 16 * DF_K / 256;
  const float* wl = W + n0 + tl + (int64_t)kq * HID;
  float av[AIT], bv[DF_K / 4];
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
    for (int s = 0; s < DF_K / 4; ++s) bv[s] = wl[(int64_t)(k0 + 4 * s) * HID];
  };
  load(0);
  for (int k0 = 0; k0 < FEAT; k0 += DF_K) {
    __syncthreads();  // previous chunk's readers done
#pragma unroll
    for (int i = 0; i < AIT; ++i) {
      const int e = tid + 256 * i;
      a_s[(e / DF_K) * AS + e % DF_K] = av[i];
    }
    float bc[DF_K / 4];
#pragma unroll
    for (int s = 0; s < DF_K / 4; ++s) bc[s] = bv[s];
    load(min(k0 + DF_K, FEAT - DF_K));  // the last chunk re-loads itself (uniform, branch-free)
    __syncthreads();
#pragma unroll
    for (int s = 0; s < DF_K / 4; ++s) acc = mfma16(a_s[tl * AS + 4 * s + kq], bc[s], acc);
  }
  const int col = n0 + tl;
  const float bias = params[(int64_t)r * stride + OFF_B5 + col];
  const uint64_t dkey = drop_key ? drop_key[r] : 0ull;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int row = m0 + 4 * kq + v;
    if (row < count) {
      const float z = acc[v] + bias;
      const float h = fmaxf(z, 0.0f);
      const int64_t o = ((int64_t)r * bmax + row) * HID + col;
      if (drop_key) {
        const bool keep = drop_keep(drop_row_seed(dkey, DROP_L5, (uint32_t)row), (uint32_t)col, THR_50);
        H[o] = keep ? h * SCALE_50 : 0.0f;
        code[o] = (uint8_t)((keep ? CODE_KEEP : 0) | (z > 0.0f ? CODE_POS : 0));
      } else {
        H[o] = h;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Dense(512) backward + RMSprop, per 32-row slice of W5, 8 rows at a time (32 threads per row, 4 fvec4
// each: every access instruction covers 512 contiguous bytes of a row); dh5 is staged in LDS once per
// block for its 4 row groups:
//   dd4[j][k] = sum_n dh5[j][n] W5[k][n];  dW5[k][n] = sum_j d4[j][k] dh5[j][n];  db5 (slice-0 block).
// dd4 goes through dropout'(.25) and the pool's positive mask into the POOLED dz4 [6][6][64] (conv4's gradient
// kernels un-pool it with code4's argmax while staging).
// HBM-bound: W5 and its accumulator are read and written once per step (the accumulator is not read on a
// fresh optimizer's first step).
// ------------------------------------------------------------------------------------------------
#ifndef MPLC_D5_MFMA
#define MPLC_D5_MFMA 1  // dense5_bwd_kernel (bit-identical MFMA form) instead of the VALU form
#endif
constexpr int D5_ROWS = 8;      // rows in flight (one per 32 threads)
constexpr int D5_GROUPS = 4;   // row groups per block (1 / 2: -8 % .. +2.5 % on two probes, not kept)
constexpr int D5_SCHUNK = 16;  // samples staged at a time (12: no gain)

__global__ __launch_bounds__(256) void dense5_bwd_valu_kernel(
    const float* __restrict__ D4, const uint8_t* __restrict__ code4, const float* __restrict__ dH,
    const int32_t* __restrict__ cnt, const int32_t* __restrict__ opt_t, int bmax, float* __restrict__ params,
    float* __restrict__ rms, const float* __restrict__ glob, const int32_t* __restrict__ w5src,
    float* __restrict__ dZ4, float lr, float rho, float omr, float decay, float eps) {
  constexpr int KB = D5_ROWS * D5_GROUPS;
  __shared__ fvec4 dh_s[D5_SCHUNK * (HID / 4)];
  __shared__ float p_s[D5_SCHUNK * KB];
  __shared__ uint8_t c_s[D5_SCHUNK * KB];
  const LogicalBlock lbk = xcd_block3();  // (row slice, replica): a replica's dh5 rows in one XCD's L2
  const int r = lbk.y;
  const int kb = lbk.x * KB;
  const int count = cnt[r];
  if (count == 0) return;
  const int tid = threadIdx.x;
  const int rowl = tid >> 5;
  const int c32 = tid & 31;
  const RmsCfg cfg = rms_cfg(opt_t[r], lr, rho, omr, decay, eps);
  const float* Pr = D4 + (int64_t)r * bmax * FEAT;
  const uint8_t* Cr = code4 + (int64_t)r * bmax * FEAT;
  const fvec4* dHr = reinterpret_cast<const fvec4*>(dH + (int64_t)r * bmax * HID);
  const fvec4 z4 = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  // staged per sample chunk: dh5 rows, the block's 32 d4 values and their pool/dropout codes
  auto stage = [&](int c0, int cn) {
    for (int e = tid; e < cn * (HID / 4); e += 256) dh_s[e] = dHr[(int64_t)c0 * (HID / 4) + e];
    for (int e = tid; e < cn * KB; e += 256) {
      const int64_t g = (int64_t)(c0 + e / KB) * FEAT + kb + e % KB;
      p_s[e] = Pr[g];
      c_s[e] = Cr[g];
    }
  };
  const bool one_chunk = count <= D5_SCHUNK;  // the usual case: staged once for all row groups
  auto row_ptrs = [&](int grp, fvec4*& W, fvec4*& Ra) {
    const int64_t roff = (int64_t)r * STRIDE + OFF_W5 + (int64_t)(kb + grp * D5_ROWS + rowl) * HID;
    W = reinterpret_cast<fvec4*>(params + roff) + c32;
    Ra = reinterpret_cast<fvec4*>(rms + roff) + c32;
  };
  // software pipeline: the next row group's W5 / accumulator loads are in flight while this one computes
  fvec4 w[4], av[4], wn[4], avn[4];
  // a round's first step reads W5 from the coalition row (the aggregation did not broadcast it); the update is
  // written into the replica's own row
  const int gsrc = w5src ? w5src[r] : -1;
  const int64_t src_shift = gsrc >= 0 ? (int64_t)(gsrc - r) * STRIDE : 0;
  auto wsrc = [&](const fvec4* Wp) {
    return gsrc >= 0 ? reinterpret_cast<const fvec4*>(glob + (reinterpret_cast<const float*>(Wp) - params) + src_shift)
                     : Wp;
  };
  fvec4 *W, *Ra;
  row_ptrs(0, W, Ra);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = wsrc(W)[32 * i];
    av[i] = cfg.reset ? z4 : __builtin_nontemporal_load(Ra + 32 * i);
  }
  if (one_chunk) {
    stage(0, count);
    __syncthreads();
  }
  for (int grp = 0; grp < D5_GROUPS; ++grp) {
    fvec4 *Wn = W, *Ran = Ra;
    if (grp + 1 < D5_GROUPS) {
      row_ptrs(grp + 1, Wn, Ran);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        wn[i] = wsrc(Wn)[32 * i];
        avn[i] = cfg.reset ? z4 : __builtin_nontemporal_load(Ran + 32 * i);
      }
    }
    const int k = kb + grp * D5_ROWS + rowl;  // the d4 element (flatten order: pooled row, column, channel)
    fvec4 g[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) g[i] = z4;
    for (int c0 = 0; c0 < count; c0 += D5_SCHUNK) {
      const int cn = min(D5_SCHUNK, count - c0);
      if (!one_chunk) {
        __syncthreads();
        stage(c0, cn);
        __syncthreads();
      }
      for (int jj = 0; jj < cn; ++jj) {
        const float pv = p_s[jj * KB + grp * D5_ROWS + rowl];
        float d = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const fvec4 dh = dh_s[jj * (HID / 4) + c32 + 32 * i];
          g[i].x += pv * dh.x; g[i].y += pv * dh.y; g[i].z += pv * dh.z; g[i].w += pv * dh.w;
          d += dh.x * w[i].x; d += dh.y * w[i].y; d += dh.z * w[i].z; d += dh.w * w[i].w;
        }
        d += dpp_partner<DPP_XOR1>(d);
        d += dpp_partner<DPP_XOR2>(d);
        d += dpp_partner<DPP_HALF_MIRROR>(d);
        d += dpp_partner<DPP_MIRROR>(d);
        d += __shfl_xor(d, 16, 64);
        if (c32 == 0) {  // dropout' and the pool's positive mask: the POOLED dz4 (conv4's gradients un-pool it)
          const uint32_t c = c_s[jj * KB + grp * D5_ROWS + rowl];
          const float v = (c & CODE_KEEP) ? d * SCALE_25 : 0.0f;
          dZ4[((int64_t)r * bmax + c0 + jj) * MPLC_CIFAR_DZ4 + k] = (c & CODE_POS) ? v : 0.0f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fvec4 pw = w[i];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float p1 = pw[q], a1 = av[i][q];
        rms_apply(p1, a1, g[i][q], cfg);
        pw[q] = p1;
        av[i][q] = a1;
      }
      W[32 * i] = pw;
      __builtin_nontemporal_store(av[i], Ra + 32 * i);
    }
    W = Wn;
    Ra = Ran;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = wn[i];
      av[i] = avn[i];
    }
  }
  if (lbk.x == 0) {
    const float* dHs = dH + (int64_t)r * bmax * HID;
    for (int c = tid; c < HID; c += 256) {
      float gb = 0.0f;
      for (int jj = 0; jj < count; ++jj) gb += dHs[(int64_t)jj * HID + c];
      const int64_t o = (int64_t)r * STRIDE + OFF_B5 + c;
      rms_apply(params[o], rms[o], gb, cfg);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// dense5_bwd with both products on v_mfma_f32_16x16x4_f32, bit-identical to dense5_bwd_valu_kernel (the matrix core
// accumulates as the fmaf chain in k order, scripts/probes/mfma_order.hip; same reasoning as mnist_cnn.hip's
// dense1_bwd_adam_mfma_kernel):
//   dW5: the VALU chain over the samples in order -> MFMA K = 4 samples chained over sample quads;
//   dd4: the VALU form's 32 partials (lane c32 of a row: columns 4 c32 + 128 i + q, i outer, q inner) -> per c32
//        an MFMA chain over i with K = q, then the same 5-level tree over c32: levels 0-2 in registers (a wave owns
//        c32 = 8 w .. 8 w + 7), levels 3-4 ((S0 + S1) + (S2 + S3)) across the 4 waves through LDS.
// Block = 16 rows of W5 x 512 columns; wave w owns the columns 128 i + 32 w + [0, 32) (8 tiles of 16): lane (tl,
// kq) holds row tl and, per tile, the columns base + 4 v + kq.  W5 comes into that layout (and dW5 out of it, for
// RMSprop in the row layout of the 16-B accesses) through a wave-private LDS transpose once per block.
// ------------------------------------------------------------------------------------------------
constexpr int D5M_ROWS = 16;
constexpr int D5M_SCHUNK = 16;          // samples staged at a time (one 16-sample tile)
constexpr int D5M_DHS = HID + 20;       // dh row stride: conflict-free dd4 operand reads
constexpr int D5M_XS = 128 + 4;         // transpose scratch row stride (a wave's 128 columns)
constexpr int D5M_STAGE = D5M_SCHUNK * D5M_DHS;
constexpr int D5M_LDS = (D5M_STAGE > 4 * 16 * D5M_XS) ? D5M_STAGE : 4 * 16 * D5M_XS;
static_assert(HID == 512 && FEAT % D5M_ROWS == 0, "dense5_bwd_kernel: 4 waves x 128 columns, 16-row slices");

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void dense5_bwd_kernel(
    const float* __restrict__ D4, const uint8_t* __restrict__ code4, const float* __restrict__ dH,
    const int32_t* __restrict__ cnt, const int32_t* __restrict__ opt_t, int bmax, float* __restrict__ params,
    float* __restrict__ rms, const float* __restrict__ glob, const int32_t* __restrict__ w5src,
    float* __restrict__ dZ4, float lr, float rho, float omr, float decay, float eps) {
  __shared__ float smem[D5M_LDS];
  __shared__ float p_s[D5M_SCHUNK * D5M_ROWS];
  __shared__ uint8_t c_s[D5M_SCHUNK * D5M_ROWS];
  __shared__ float t_s[4 * 4 * 64];  // the waves' level-2 sums [w][v][lane]
  float* const dh_s = smem;          // [sample][D5M_DHS]
  const LogicalBlock lbk = xcd_block3();  // (row slice, replica): a replica's dh5 rows in one XCD's L2
  const int r = lbk.y;
  const int k0 = lbk.x * D5M_ROWS;
  const int count = cnt[r];
  if (count == 0) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int tl = lane & 15, kq = lane >> 4;
  float* const x_s = smem + wave * 16 * D5M_XS;  // this wave's transpose scratch (aliases the staging)
  const RmsCfg cfg = rms_cfg(opt_t[r], lr, rho, omr, decay, eps);
  const fvec4 z4 = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  // row layout: lane's fvec4 f = lane + 64 u (u = 0..7): row f / 32, column chunk i = (f % 32) / 8, columns
  // 128 i + 32 w + 4 (f % 8) ..
  auto rl_off = [&](int u) {
    const int f = lane + 64 * u;
    return (int64_t)(k0 + (f >> 5)) * HID + 128 * ((f & 31) >> 3) + 32 * wave + 4 * (f & 7);
  };
  const int gsrc = w5src ? w5src[r] : -1;
  const float* Wsrc = gsrc >= 0 ? glob + (int64_t)gsrc * STRIDE + OFF_W5 : params + (int64_t)r * STRIDE + OFF_W5;
  float* const Wr = params + (int64_t)r * STRIDE + OFF_W5;
  float* const Rr = rms + (int64_t)r * STRIDE + OFF_W5;
  fvec4 w[8], av[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    w[u] = *reinterpret_cast<const fvec4*>(Wsrc + rl_off(u));
    av[u] = cfg.reset ? z4 : __builtin_nontemporal_load(reinterpret_cast<const fvec4*>(Rr + rl_off(u)));
  }
  // W5 into the MFMA layout: tile tau = 2 i + h (columns 128 i + 32 w + 16 h ..): wd[tau][v] = W5[tl][base + 4 v + kq]
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int f = lane + 64 * u;
    *reinterpret_cast<fvec4*>(x_s + (f >> 5) * D5M_XS + 32 * ((f & 31) >> 3) + 4 * (f & 7)) = w[u];
  }
  __syncthreads();
  float wd[8][4];
#pragma unroll
  for (int tau = 0; tau < 8; ++tau)
#pragma unroll
    for (int v = 0; v < 4; ++v) wd[tau][v] = x_s[tl * D5M_XS + 16 * tau + 4 * v + kq];
  fvec4 g[8];
#pragma unroll
  for (int tau = 0; tau < 8; ++tau) g[tau] = z4;
  const float* Pr = D4 + (int64_t)r * bmax * FEAT;
  const uint8_t* Cr = code4 + (int64_t)r * bmax * FEAT;
  const float* dHr = dH + (int64_t)r * bmax * HID;
  const int gcol = 4 * (tl & 3) + (tl >> 2);  // g's A row m = 4 a + b is column base + 4 b + a
  for (int c0 = 0; c0 < count; c0 += D5M_SCHUNK) {
    const int cn = min(D5M_SCHUNK, count - c0);
    __syncthreads();  // the transpose reads / the previous chunk's readers are done
    {
      constexpr int HIT = D5M_SCHUNK * (HID / 4) / 256;
      fvec4 hv[HIT];
#pragma unroll
      for (int i = 0; i < HIT; ++i) {
        const int e = tid + 256 * i;  // (sample e / 128, chunk e % 128)
        const bool ok = e / (HID / 4) < cn;
        const fvec4 t = *reinterpret_cast<const fvec4*>(dHr + (int64_t)(c0 + (ok ? e / (HID / 4) : 0)) * HID +
                                                        4 * (e % (HID / 4)));
        hv[i] = ok ? t : z4;
      }
      float pv = 0.0f;
      uint8_t cv = 0;
      {  // (sample tid / 16, row tid % 16)
        const bool ok = tid / D5M_ROWS < cn;
        const int64_t gi = (int64_t)(c0 + (ok ? tid / D5M_ROWS : 0)) * FEAT + k0 + tid % D5M_ROWS;
        const float t = Pr[gi];
        const uint8_t cc = Cr[gi];
        pv = ok ? t : 0.0f;
        cv = ok ? cc : (uint8_t)0;
      }
#pragma unroll
      for (int i = 0; i < HIT; ++i) {
        const int e = tid + 256 * i;
        float* d = dh_s + (e / (HID / 4)) * D5M_DHS + 4 * (e % (HID / 4));
        d[0] = hv[i].x;
        d[1] = hv[i].y;
        d[2] = hv[i].z;
        d[3] = hv[i].w;
      }
      p_s[tid] = pv;
      c_s[tid] = cv;
    }
    __syncthreads();
    // dW5: sample quads in order
    for (int jq = 0; jq < cn; jq += 4) {
      const float bp = p_s[(jq + kq) * D5M_ROWS + tl];
      const float* dq = dh_s + (jq + kq) * D5M_DHS + 32 * wave + gcol;
#pragma unroll
      for (int tau = 0; tau < 8; ++tau) g[tau] = mfma16(dq[128 * (tau >> 1) + 16 * (tau & 1)], bp, g[tau]);
    }
    // dd4: per c32 = 8 w + c (columns 128 i + 32 w + 4 c + q) the chain over i, then tree levels 0-2
    {
      const float* da = dh_s + tl * D5M_DHS + 32 * wave + kq;
      fvec4 pc[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        pc[c] = z4;
#pragma unroll
        for (int i = 0; i < 4; ++i) pc[c] = mfma16(da[128 * i + 4 * c], wd[2 * i + (c >> 2)][c & 3], pc[c]);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v)
        t_s[(wave * 4 + v) * 64 + lane] =
            ((pc[0][v] + pc[1][v]) + (pc[2][v] + pc[3][v])) + ((pc[4][v] + pc[5][v]) + (pc[6][v] + pc[7][v]));
    }
    __syncthreads();
    {  // levels 3-4 across the waves; wave w finishes register v = w: sample 4 kq + w, row tl
      const int v = wave;
      const float d = (t_s[(0 * 4 + v) * 64 + lane] + t_s[(1 * 4 + v) * 64 + lane]) +
                      (t_s[(2 * 4 + v) * 64 + lane] + t_s[(3 * 4 + v) * 64 + lane]);
      const int jj = 4 * kq + v;
      if (jj < cn) {  // dropout' and the pool's positive mask: the POOLED dz4 (conv4's gradients un-pool it)
        const uint32_t c = c_s[jj * D5M_ROWS + tl];
        const float dv = (c & CODE_KEEP) ? d * SCALE_25 : 0.0f;
        dZ4[((int64_t)r * bmax + c0 + jj) * MPLC_CIFAR_DZ4 + k0 + tl] = (c & CODE_POS) ? dv : 0.0f;
      }
    }
  }
  __syncthreads();  // the last readers of the staging (and t_s) are done: the scratch takes dW5
#pragma unroll
  for (int tau = 0; tau < 8; ++tau)
#pragma unroll
    for (int v = 0; v < 4; ++v) x_s[tl * D5M_XS + 16 * tau + 4 * v + kq] = g[tau][v];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int f = lane + 64 * u;
    const fvec4 gr = *reinterpret_cast<const fvec4*>(x_s + (f >> 5) * D5M_XS + 32 * ((f & 31) >> 3) + 4 * (f & 7));
    fvec4 pw = w[u];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float p1 = pw[q], a1 = av[u][q];
      rms_apply(p1, a1, gr[q], cfg);
      pw[q] = p1;
      av[u][q] = a1;
    }
    *reinterpret_cast<fvec4*>(Wr + rl_off(u)) = pw;
    __builtin_nontemporal_store(av[u], reinterpret_cast<fvec4*>(Rr + rl_off(u)));
  }
  if (lbk.x == 0) {
    const float* dHs = dH + (int64_t)r * bmax * HID;
    for (int c = tid; c < HID; c += 256) {
      float gb = 0.0f;
      for (int jj = 0; jj < count; ++jj) gb += dHs[(int64_t)jj * HID + c];
      const int64_t o = (int64_t)r * STRIDE + OFF_B5 + c;
      rms_apply(params[o], rms[o], gb, cfg);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// layer instantiations: <HI, WI, CI, CO, PAD, BR, NW, UM, EPI> (conv) and <HI, WI, CI, CO, PAD, HOV, WOV,
// BR, NW> (wgrad); geometry checked by static_asserts, LDS per block in the comment
// ------------------------------------------------------------------------------------------------
#define CONV1_FWD conv1_fwd_kernel  /* 4 bands, 4.1 KB; conv_kernel<32, 32, 3, 32, 1, 8, 4, 2, EPI_FWD> with the channels as M rows */
// Winograd F(2x2,3x3): <HI, WI, CI, CO, PAD, tile rows per band, EPI>; bands = ceil(tile rows / BTY)
// wave-local form: <HI, WI, CI, CO, PAD, BTY, waves, EPI>; reads conv2's Winograd weights in the xi-last layout
#define CONV2_FWD wino_wl_kernel<32, 32, 32, 32, 0, 4, 4, EPI_FWD_POOL>      /* 60 tiles, 4 bands, 42 KB */
// conv3's data gradient keeps the row form: its bands hold 2 tile groups, and the wave-local form with 2-wave
// blocks measured slower (4585 vs 4264 ms over a config #4 run, profiles/r03_driver_bench_v2.json)
#define CONV3_DGRAD wino_kernel<15, 15, 64, 32, 1, 4, EPI_BWD_UNPOOL>        /* 8x8 tiles, 2 bands, 63.7 KB */
// conv2's data / weight gradients read dZ2 POOLED (conv3's data gradient writes [15][15][32] + the pool codes) and
// un-pool it while staging: a quarter of the dense gradient's HBM bytes
#define CONV2_DGRAD wino_wl_kernel<30, 30, 32, 32, 2, 4, 4, EPI_BWD_MASK, 1> /* 64 tiles, 4 bands, 44.9 KB */
#define CONV3_DGRAD_NT 256
#define CONV3_FWD wino_kernel<15, 15, 32, 64, 1, 8, EPI_FWD>          /* 8x8 tiles,    1 band,  59.7 KB */
#define CONV4_FWD wino_kernel<15, 15, 64, 64, 0, 6, EPI_FWD_POOL>     /* 6x6 windows,  1 band,  67.9 KB */
// conv4's gradients read dz4 POOLED ([6][6][64] + code4, written by dense5_bwd) and un-pool it while staging
#define CONV4_DGRAD wino_kernel<13, 13, 64, 64, 2, 4, EPI_BWD_MASK, 1>   /* 8x8 tiles,    2 bands, 63.7 KB */
#define CONV1_WGRAD wgrad_kernel<32, 32, 3, 32, 1, 32, 32, 8, 4>
// Winograd F(3x3,2x2) weight gradients: <HI, WI, CI, CO, PAD, HOV, WOV, tile rows per band, ci per block>
#define CONV2_WGRAD wino_wgrad_kernel<32, 32, 32, 32, 0, 30, 30, 3, 32, 1, 0>  /* 15x15 tiles, 5 bands, 73.9 KB */
#define CONV3_WGRAD wino_wgrad_kernel<15, 15, 32, 64, 1, 15, 15, 4, 32>  /* 8x8 tiles,   2 bands, 69.8 KB */
#define CONV4_WGRAD wino_wgrad_kernel<15, 15, 64, 64, 0, 12, 12, 6, 32, 1, 1>  /* 6x6 tiles, 1 band, 2 ci chunks, 76.9 KB */
// dz2 / dz4 slots hold the pooled gradients: conv3's data gradient (out [15][15][32]) and dense5_bwd write them,
// conv2's / conv4's data (UPI: in [HI/2][WI/2][CI]) and weight (UPZ: dz [HO/2][WO/2][CO]) gradients read them
static_assert(15 * 15 * 32 == MPLC_CIFAR_DZ2 && (30 / 2) * (30 / 2) * 32 == MPLC_CIFAR_DZ2, "dz2 slot stride");
static_assert(6 * 6 * 64 == MPLC_CIFAR_DZ4 && (13 / 2) * (13 / 2) * 64 == MPLC_CIFAR_DZ4, "dz4 slot stride");

inline int launch_status() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? MPLC_OK : (int)e;
}

ConvArgs conv_args(const float* in, int in_mode, int row_base, const int32_t* idx, const int32_t* cnt, int cnt_all,
                   int bmax, const float* w, int64_t w_rstride) {
  ConvArgs a{};
  a.in = in;
  a.in_mode = in_mode;
  a.row_base = row_base;
  a.idx = idx;
  a.cnt = cnt;
  a.cnt_all = cnt_all;
  a.bmax = bmax;
  a.w = w;
  a.w_rstride = w_rstride;
  return a;
}

// In-stream kernel timing (bench.py): prof = k > 0 records the event ev before / after launch k; prof =
// MPLC_PROF_ALL records around every launch k, ev then pointing to an array of hipEvent_t indexed by k (1 .. 15).
inline void cifar_prof_record(int prof, void* ev, int k, hipStream_t s) {
  if (!ev) return;
  if (prof == k) (void)hipEventRecord((hipEvent_t)ev, s);
  else if (prof == MPLC_PROF_ALL) (void)hipEventRecord(static_cast<hipEvent_t*>(ev)[k], s);
}

// forward of conv1..dense5 for R models x B slots (train: dropout + codes; eval: inference)
void enqueue_forward(hipStream_t s, int R, int B, const float* x, int in_mode, int row_base, const int32_t* idx,
                     const int32_t* cnt, int cnt_all, const float* params, int64_t stride, const uint64_t* drop_key,
                     float* a1, float* d2, uint8_t* code2, float* a3, float* d4, uint8_t* code4, float* h5,
                     uint8_t* code5, int prof, void* pb, void* pe, float* wu, const float* glob = nullptr,
                     const int32_t* w5src = nullptr, bool make_wu = true) {
#define PB(k) cifar_prof_record(prof, pb, (k), s)
#define PE(k) cifar_prof_record(prof, pe, (k), s)
  // conv2..conv4 weights in Winograd form (U = G g G^T per channel pair); the evaluation makes them once for
  // all its sample chunks (make_wu = false here)
  if (make_wu) wino_u_kernel<0><<<dim3(7168 / 256, R), 256, 0, s>>>(params, stride, cnt, wu);
  ConvArgs c1 = conv_args(x, in_mode, row_base, idx, cnt, cnt_all, B, params + OFF_W1, stride);
  c1.bias = params + OFF_B1;
  c1.b_rstride = stride;
  c1.out = a1;
  PB(1);
  CONV1_FWD<<<dim3(4, B, R), 256, 0, s>>>(c1);
  PE(1);
  ConvArgs c2 = conv_args(a1, 0, 0, nullptr, cnt, cnt_all, B, wu + WU_2, MPLC_CIFAR_WT);
  c2.bias = params + OFF_B2;
  c2.b_rstride = stride;
  c2.drop_key = drop_key;
  c2.drop_layer = DROP_L2;
  c2.out = d2;
  c2.code_out = code2;
  PB(2);
  CONV2_FWD<<<dim3(4, B, R), 256, 0, s>>>(c2);
  PE(2);
  ConvArgs c3 = conv_args(d2, 0, 0, nullptr, cnt, cnt_all, B, wu + WU_3, MPLC_CIFAR_WT);
  c3.bias = params + OFF_B3;
  c3.b_rstride = stride;
  c3.out = a3;
  PB(3);
  CONV3_FWD<<<dim3(1, B, R), 256, 0, s>>>(c3);
  PE(3);
  ConvArgs c4 = conv_args(a3, 0, 0, nullptr, cnt, cnt_all, B, wu + WU_4, MPLC_CIFAR_WT);
  c4.bias = params + OFF_B4;
  c4.b_rstride = stride;
  c4.drop_key = drop_key;
  c4.drop_layer = DROP_L4;
  c4.out = d4;
  c4.code_out = code4;
  PB(4);
  CONV4_FWD<<<dim3(1, B, R), 256, 0, s>>>(c4);
  PE(4);
  PB(5);
  if (B <= MPLC_D5F16_MAX)
    dense5_fwd16_kernel<<<dim3(1, HID / 64, R), 256, 0, s>>>(d4, cnt, cnt_all, B, params, stride, glob, w5src,
                                                             drop_key, h5, code5);
  else
    dense5_fwd_kernel<<<dim3((B + 31) / 32, HID / 128, R), 256, 0, s>>>(d4, cnt, cnt_all, B, params, stride, glob,
                                                                        w5src, drop_key, h5, code5);
  PE(5);
#undef PB
#undef PE
}

}  // namespace

extern "C" {

int mplc_cifar_stride(void) { return MPLC_CIFAR_STRIDE; }

int mplc_cifar_wgrad_split_samples(void) { return WGS; }

int64_t mplc_cifar_layout(int what) {
  switch (what) {
    case MPLC_CIFAR_Q_STRIDE: return MPLC_CIFAR_STRIDE;
    case MPLC_CIFAR_Q_NPARAM: return MPLC_CIFAR_NPARAM;
    case MPLC_CIFAR_Q_A1: return MPLC_CIFAR_A1;
    case MPLC_CIFAR_Q_D2: return MPLC_CIFAR_D2;
    case MPLC_CIFAR_Q_A3: return MPLC_CIFAR_A3;
    case MPLC_CIFAR_Q_D4: return MPLC_CIFAR_D4;
    case MPLC_CIFAR_Q_H5: return MPLC_CIFAR_H5;
    case MPLC_CIFAR_Q_DZ4: return MPLC_CIFAR_DZ4;
    case MPLC_CIFAR_Q_DZ3: return MPLC_CIFAR_DZ3;
    case MPLC_CIFAR_Q_DZ2: return MPLC_CIFAR_DZ2;
    case MPLC_CIFAR_Q_DZ1: return MPLC_CIFAR_DZ1;
    case MPLC_CIFAR_Q_WT: return MPLC_CIFAR_WT;
    case MPLC_CIFAR_Q_WPART: return MPLC_CIFAR_WPART;
    case MPLC_CIFAR_Q_WG_SAMPLES: return WGS;
    case MPLC_CIFAR_Q_TRAIN_T_BYTES: return (int64_t)sizeof(mplc_cifar_train_t);
    default: return -1;
  }
}

int mplc_cifar_init_params(float* params, int64_t stride, const uint64_t* keys, int n_models, void* stream) {
  if (!params || !keys || n_models < 1 || n_models > 65535 || stride != MPLC_CIFAR_STRIDE) return MPLC_E_ARG;
  init_params_kernel<<<dim3(512, n_models), 256, 0, (hipStream_t)stream>>>(params, stride, keys);
  return launch_status();
}

#define PROF_BEGIN(k) cifar_prof_record(t->prof_kernel, t->prof_begin, (k), s)
#define PROF_END(k) cifar_prof_record(t->prof_kernel, t->prof_end, (k), s)

int mplc_cifar_train_step(const mplc_cifar_train_t* t, void* stream) {
  if (!t || t->n_rep < 1 || t->n_rep > 65535 || t->bmax < 1 || t->bmax > 65535) return MPLC_E_ARG;
  if (t->wg_splits != (t->bmax + WGS - 1) / WGS) return MPLC_E_SHAPE;
  if (!t->reps || !t->rows || !t->splits || !t->x || !t->labels || !t->params || !t->rms || !t->idx || !t->cnt ||
      !t->opt_t || !t->drop_key || !t->a1 || !t->d2 || !t->code2 || !t->a3 || !t->d4 || !t->code4 || !t->d5 ||
      !t->code5 || !t->dh5 || !t->dz4 || !t->dz3 || !t->dz2 || !t->dz1 || !t->wt || !t->wpart)
    return MPLC_E_ARG;
  if (t->minibatch_count < 1 || t->round_len < 1 || t->epochs < 1) return MPLC_E_ARG;
  if (t->glob && (!t->rep_glob || !t->w5src)) return MPLC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int R = t->n_rep, B = t->bmax;
  const int64_t slots = (int64_t)R * B;
  schedule_kernel<<<(unsigned)((slots + 255) / 256), 256, 0, s>>>(t->reps, R, B, t->rows, t->splits, t->seq, t->step,
                                                                   t->minibatch_count, t->round_len, t->epochs,
                                                                   t->idx, t->cnt, t->opt_t, t->drop_key,
                                                                   t->rep_glob, t->glob ? t->w5src : nullptr);
  const int32_t* w5src = t->glob ? t->w5src : nullptr;
  enqueue_forward(s, R, B, t->x, 1, 0, t->idx, t->cnt, 0, t->params, STRIDE, t->drop_key, t->a1, t->d2, t->code2,
                  t->a3, t->d4, t->code4, t->d5, t->code5, t->prof_kernel, t->prof_begin, t->prof_end, t->wt,
                  t->glob, w5src);
  PROF_BEGIN(6);
  cifar_launch_head(R, s, t->d5, t->code5, t->idx, t->labels, t->cnt, t->opt_t, B, t->params, t->rms, t->dh5, t->lr,
                    t->rho, t->one_minus_rho, t->decay, t->eps, t->hstats);
  PROF_END(6);
  PROF_BEGIN(7);
#if MPLC_D5_MFMA
  dense5_bwd_kernel<<<dim3(FEAT / D5M_ROWS, R), 256, 0, s>>>(t->d4, t->code4, t->dh5, t->cnt, t->opt_t, B,
                                                                  t->params, t->rms, t->glob, w5src, t->dz4, t->lr,
                                                                  t->rho, t->one_minus_rho, t->decay, t->eps);
#else
  dense5_bwd_valu_kernel<<<dim3(FEAT / (D5_ROWS * D5_GROUPS), R), 256, 0, s>>>(t->d4, t->code4, t->dh5, t->cnt, t->opt_t, B, t->params,
                                                            t->rms, t->glob, w5src, t->dz4, t->lr, t->rho,
                                                            t->one_minus_rho, t->decay, t->eps);
#endif
  PROF_END(7);
  // the data gradients' kernels (rotated, channels swapped) in Winograd form, over the forward's
  wino_u_kernel<1><<<dim3(7168 / 256, R), 256, 0, s>>>(t->params, STRIDE, t->cnt, t->wt);
  const int SP = t->wg_splits;
  WgArgs w4{t->a3, 0, t->idx, t->cnt, B, SP, t->dz4, t->wpart, (int)OFF_W4, (int)OFF_B4, t->code4};  // dz4 pooled
  PROF_BEGIN(8);
  CONV4_WGRAD<<<dim3(SP, R, 2), 256, 0, s>>>(w4);
  PROF_END(8);
  ConvArgs g4 = conv_args(t->dz4, 0, 0, nullptr, t->cnt, 0, B, t->wt + WU_4, MPLC_CIFAR_WT);
  g4.code_in = t->code4;  // dz4 is pooled: un-pooled while staging
  g4.aux = t->a3;
  g4.out = t->dz3;
  PROF_BEGIN(9);
  CONV4_DGRAD<<<dim3(2, B, R), 256, 0, s>>>(g4);
  PROF_END(9);
  WgArgs w3{t->d2, 0, t->idx, t->cnt, B, SP, t->dz3, t->wpart, (int)OFF_W3, (int)OFF_B3};
  PROF_BEGIN(10);
  CONV3_WGRAD<<<dim3(SP, R, 1), 256, 0, s>>>(w3);
  PROF_END(10);
  ConvArgs g3 = conv_args(t->dz3, 0, 0, nullptr, t->cnt, 0, B, t->wt + WU_3, MPLC_CIFAR_WT);
  g3.code_in = t->code2;
  g3.out = t->dz2;
  PROF_BEGIN(11);
  CONV3_DGRAD<<<dim3(2, B, R), CONV3_DGRAD_NT, 0, s>>>(g3);
  PROF_END(11);
  WgArgs w2{t->a1, 0, t->idx, t->cnt, B, SP, t->dz2, t->wpart, (int)OFF_W2, (int)OFF_B2, t->code2};  // dz2 pooled
  PROF_BEGIN(12);
  CONV2_WGRAD<<<dim3(SP, R, 1), 256, 0, s>>>(w2);
  PROF_END(12);
  ConvArgs g2 = conv_args(t->dz2, 0, 0, nullptr, t->cnt, 0, B, t->wt + WU_2, MPLC_CIFAR_WT);
  g2.aux = t->a1;
  g2.code_in = t->code2;  // dz2 is pooled: un-pooled while staging
  g2.out = t->dz1;
  PROF_BEGIN(13);
  CONV2_DGRAD<<<dim3(4, B, R), 256, 0, s>>>(g2);
  PROF_END(13);
  WgArgs w1{t->x, 1, t->idx, t->cnt, B, SP, t->dz1, t->wpart, (int)OFF_W1, (int)OFF_B1};
  PROF_BEGIN(14);
  CONV1_WGRAD<<<dim3(SP, R), 256, 0, s>>>(w1);
  PROF_END(14);
  PROF_BEGIN(15);
  rmsprop_small_kernel<<<dim3((OFF_W5 + 255) / 256, R), 256, 0, s>>>(t->cnt, t->opt_t, SP, t->wpart, t->params,
                                                                      t->rms, t->lr, t->rho, t->one_minus_rho, t->decay, t->eps);
  PROF_END(15);
  return launch_status();
}

int64_t mplc_cifar_eval_workspace_floats(int n_models, int chunk) {
  return (int64_t)n_models * chunk * (MPLC_CIFAR_A1 + MPLC_CIFAR_D2 + MPLC_CIFAR_A3 + MPLC_CIFAR_D4 + MPLC_CIFAR_H5) +
         (int64_t)n_models * MPLC_CIFAR_WT;
}

int mplc_cifar_evaluate(const float* params, int64_t stride, int n_models, const float* x, const int32_t* labels,
                        int n_samples, int chunk, float* ws, int32_t* correct, double* loss_sum, void* stream) {
  if (!params || !x || !labels || !ws || !correct || !loss_sum) return MPLC_E_ARG;
  if (n_models < 1 || n_models > 65535 || n_samples < 1 || chunk < 1 || chunk > 65535 || stride != MPLC_CIFAR_STRIDE)
    return MPLC_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t mc = (int64_t)n_models * chunk;
  float* a1 = ws;
  float* d2 = a1 + mc * MPLC_CIFAR_A1;
  float* a3 = d2 + mc * MPLC_CIFAR_D2;
  float* d4 = a3 + mc * MPLC_CIFAR_A3;
  float* h5 = d4 + mc * MPLC_CIFAR_D4;
  float* wu = h5 + mc * MPLC_CIFAR_H5;  // [n_models][MPLC_CIFAR_WT] conv2..conv4 in Winograd form
  // the weights do not change between chunks: their Winograd form once for the whole evaluation
  wino_u_kernel<0><<<dim3(7168 / 256, n_models), 256, 0, s>>>(params, stride, nullptr, wu);
  for (int s0 = 0; s0 < n_samples; s0 += chunk) {
    const int cn = n_samples - s0 < chunk ? n_samples - s0 : chunk;
    enqueue_forward(s, n_models, chunk, x, 2, s0, nullptr, nullptr, cn, params, stride, nullptr, a1, d2, nullptr, a3,
                    d4, nullptr, h5, nullptr, 0, nullptr, nullptr, wu, nullptr, nullptr, false);
    cifar_launch_eval_head(n_models, s, h5, cn, chunk, labels, s0, params, stride, correct, loss_sum);
    const int st = launch_status();
    if (st) return st;
  }
  return MPLC_OK;
}

}  // extern "C"
