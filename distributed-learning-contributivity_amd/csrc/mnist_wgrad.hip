// conv2 weight gradient of the batched MNIST CNN trainer (one launch per lockstep step; see csrc/mnist_cnn.hip for
// the step and include/mplc_hip_cnn.h for the contract).  A translation unit of its own: compiled together with
// conv_fwd_kernel it made the register allocator spill 4 of conv_fwd's registers.
#include "mnist_common.h"

namespace {

// ------------------------------------------------------------------------------------------------
// conv2 weight gradient in Winograd form F(3x3, 2x2): per 2x2 tile of dZ2 (= one pooling window) and the
// 4x4 conv1 patch it sees,  dW2[3x3] += G^T [ (A delta A^T) (.) (B^T d B) ] G  (the transposed dual of the
// forward's F(2x2, 3x3); A, B, G are the forward's matrices).  The sum over tiles runs in the transformed
// domain: 16 GEMMs M[xi][ci][co] = sum_tiles V[xi][tile][ci] D[xi][tile][co], then one inverse transform per
// split: 2.25x fewer multiply-adds than the direct sum (16 per tile instead of 4 positions x 9 taps).
// delta is the max-pool gradient of one window: a single nonzero v at the argmax (dy, dx) when positive,
// so D = v * A[:, dy] (x) A[:, dx] is a sign pattern of v.
// Block = (split s, replica r): samples [9s, 9s+9) (WG_SAMPLES); 4 waves, wave i owns transform row i (xi = 4i .. 4i+3) x
// 32 ci x 64 co (32 accumulators of v_mfma_f32_16x16x4_f32).  The work is a stream of bands (sample, 2 window
// rows = 24 tiles): conv1 rows recomputed on MFMA (conv1_mfma, bit-identical to the forward's activations)
// and the windows' (value, argmax) staged in LDS; per k-step of 4 tiles a lane forms 8 values of V (its
// tile, two ci) and 16 of D (its tile, four co), for 32 MFMAs.  At the end the waves fold their row of the
// inverse transform (P_i = M_i G) and exchange it through LDS.  Fixed-order sums: independent of which
// other replicas share the launch.
// ------------------------------------------------------------------------------------------------
constexpr int WG_PRE = 2 * PL * C2 / WG_THREADS;  // (dp, code) pairs per thread per band: 2 rows x 12 x 64
// Staged operands are read as 8-byte pairs: a lane needs channels ci and 16 + ci of a conv1 position (stored
// adjacent: slot 2 * (ci & 15) + (ci >> 4)) and (value, argmax) of a window channel (one int2), so a k-step's
// 32 MFMAs take 12 ds_read_b64 instead of 24 4-byte reads.  The strides put the two lane halves of a b64 read
// group (tiles kq, kq + 1: 2 positions or 1 window apart) on opposite halves of the 64 banks.
constexpr int WG_CS = 48;                         // a1 position stride (32 channels + pad; 2 * 48 = 32 mod 64)
constexpr int WG_A1 = 6 * A1 * WG_CS;             // one band's conv1 rows [6][26][48]
constexpr int WG_VS = 80;                         // window stride of the staged (value, argmax) pairs (int2)
constexpr int WG_PX = 3 * 16 * C2 + 16;           // one wave's P_i for one ci half: [3][16 ci][64 co] (+pad)

__global__ __launch_bounds__(WG_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2))) CONV_REGS void conv_wgrad_kernel(
    const float* __restrict__ x, const int32_t* __restrict__ idx, const int32_t* __restrict__ cnt, int bmax,
    int splits, const float* __restrict__ params, int64_t stride, const float* __restrict__ dPool,
    const uint8_t* __restrict__ code, float* __restrict__ w2_part) {
  __shared__ float smem[(WG_A1 + 24 * WG_VS * 2 > 4 * WG_PX) ? WG_A1 + 24 * WG_VS * 2 : 4 * WG_PX];
  __shared__ float img_s[IMG * IMG];
  __shared__ float gb_s[4][C2];
  float* const a1_s = smem;            // [6][26][WG_CS]
  int2* const vq_s = reinterpret_cast<int2*>(smem + WG_A1);  // [24 windows][WG_VS]: (value bits, argmax)
  const int sp = blockIdx.x;
  const int r = blockIdx.y;
  const int count = cnt[r];
  // samples [sp*WG_SAMPLES, (sp+1)*WG_SAMPLES): the split of a replica depends only on its own batch,
  // so its summation order (and v(S)) does not depend on which other replicas share the launch
  const int j_begin = sp * WG_SAMPLES;
  const int j_end = min(count, j_begin + WG_SAMPLES);
  if (j_begin >= j_end) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int m = lane & 31;
  const int kh = lane >> 5;
  const float* P = params + (int64_t)r * stride;
  float w1r[5];
  load_w1r(P, kh, m, w1r);
  float gb = 0.0f;  // db2 partial of channel tid & 63 (every pair this thread stages has that channel)
  float pdv[WG_PRE];
  uint32_t pcd[WG_PRE];
  // window rows 2*band, 2*band+1 of sample jj: pair e = tid + 256*s is element 24*64*band + e (contiguous)
  auto fetch = [&](int jj, int band) {
    const int64_t base = ((int64_t)r * bmax + jj) * FEAT + band * 2 * PL * C2;
#pragma unroll
    for (int s = 0; s < WG_PRE; ++s) {
      const int e = tid + WG_THREADS * s;
      pdv[s] = dPool[base + e];
      pcd[s] = code[base + e];
    }
  };
  constexpr int IMG_PRE = (IMG * IMG + WG_THREADS - 1) / WG_THREADS;
  float imgv[IMG_PRE];
  auto fetch_img = [&](int jj) {
    const float* xr = x + (int64_t)idx[(int64_t)r * bmax + jj] * (IMG * IMG);
#pragma unroll
    for (int k = 0; k < IMG_PRE; ++k) {
      const int e = tid + WG_THREADS * k;
      imgv[k] = xr[e < IMG * IMG ? e : 0];
    }
  };
  // GEMM roles: wave = transform row i; lane (tl = lane & 15: ci / co in a group of 16, kq = lane >> 4: tile)
  const int wi = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: the row's signs below live in SGPRs
  const int tl = lane & 15, kq = lane >> 4;
  // The wave's transform row as data (round 6: one loop for all waves, every barrier in code all waves share).
  // Row i of B^T takes patch rows ra, rb: t = s_a d[ra] + s_b d[rb], written as ONE fma by +-1 on the row whose sign
  // is + (tp) and the other (tq): fmaf(sq, d[tq], d[tp]) is the correctly rounded s_a d[ra] + s_b d[rb], the same bits
  // as round 5's per-wave add / subtract.  Row i of A gives delta's row dy the factor A[i][dy] in {0, +-1}: v times
  // that factor is v, -v or a zero, and a zero's sign never reaches a result (the MFMA accumulators start at +0 and
  // a product of +-0 leaves a sum unchanged), so v(S) is bit-identical to the per-wave copies.
  const int tp = (wi == 0) ? 0 : ((wi == 2) ? 2 : 1);   // the + row:  0 | 1 | 2 | 1
  const int tq = (wi == 0) ? 2 : ((wi == 2) ? 1 : ((wi == 3) ? 3 : 2));  // the other: 2 | 2 | 1 | 3
  const float sq = (wi == 1) ? 1.0f : -1.0f;
  const float fa0 = (wi == 3) ? 0.0f : 1.0f;                             // A[i][0]
  const float fa1 = (wi == 0) ? 0.0f : ((wi == 1) ? 1.0f : -1.0f);       // A[i][1]
  fvec4 acc[4][2][4];  // [j][ci half][co group]
#pragma unroll
  for (int jj = 0; jj < 4; ++jj)
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int cg = 0; cg < 4; ++cg) acc[jj][ch][cg] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  fetch(j_begin, 0);
  fetch_img(j_begin);
  for (int j = j_begin; j < j_end; ++j) {
    for (int band = 0; band < 6; ++band) {
      __syncthreads();  // previous band's readers (a1_s, vq_s; and img_s by its staging) done
      if (band == 0) {
#pragma unroll
        for (int k = 0; k < IMG_PRE; ++k)
          if (tid + WG_THREADS * k < IMG * IMG) img_s[tid + WG_THREADS * k] = imgv[k];
        if (j + 1 < j_end) fetch_img(j + 1);
        __syncthreads();
      }
      // windows of the band: (value masked by the positive bit, argmax)
#pragma unroll
      for (int s = 0; s < WG_PRE; ++s) {
        const int e = tid + WG_THREADS * s;  // window e >> 6 of the band (row-major), channel e & 63
        const uint32_t c = pcd[s];
        const float v = (c & 0x80) ? pdv[s] : 0.0f;
        gb += v;
        vq_s[(e >> 6) * WG_VS + (e & 63)] = int2{__float_as_int(v), (int)(c & 3)};
      }
      // conv1 + ReLU of rows 4*band .. 4*band+5: 156 positions = 4 tiles of 32 (one per wave, 32x32x2) and the
      // last 28 positions as 2 x 16 positions x 2 channel halves on 16x16x4 (one piece per wave; a fifth 32x32
      // tile on wave 0 was 1/8 padding and doubled that wave's share).  Taps and bias in conv1_mfma's k order on
      // both forms (an exact fmaf chain): bit-identical activations.
#ifndef WG_EXP_NOCONV1  // timing experiment switch (garbage results): conv1 recompute compiled out
      {
        const int p = wave * 32 + m;
        const floatx16 a = conv1_mfma(img_s, (4 * band + p / A1) * IMG + p % A1, kh, w1r);
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
          a1_s[(wave * 32 + acc_row(reg, kh)) * WG_CS + 2 * (m & 15) + (m >> 4)] = fmaxf(a[reg], 0.0f);
      }
      {
        const int mt = wave >> 1, h = wave & 1, tl = lane & 15, kq = lane >> 4;
        const int p = min(128 + 16 * mt + tl, 6 * A1 - 1);
        fvec4 c1 = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
          const int k = 4 * s3 + kq;
          const float av = (k < 9) ? img_s[(4 * band + p / A1 + k / 3) * IMG + p % A1 + k % 3] : ((k == 9) ? 1.0f : 0.0f);
          const float wv = (k < 9) ? P[OFF_W1 + k * C1 + 16 * h + tl] : ((k == 9) ? P[OFF_B1 + 16 * h + tl] : 0.0f);
          c1 = mfma16(av, wv, c1);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {  // rows past 155 are position 155 again: the same value rewritten
          const int pw = min(128 + 16 * mt + 4 * kq + reg, 6 * A1 - 1);
          a1_s[pw * WG_CS + 2 * tl + h] = fmaxf(c1[reg], 0.0f);
        }
      }
#endif
      if (band < 5) fetch(j, band + 1);
      else if (j + 1 < j_end) fetch(j + 1, 0);
      __syncthreads();
      // 6 k-steps of 4 tiles (window (wr, wc) = tile 12*wr + wc of the band; lane kq takes tile 4*st + kq)
#pragma unroll 1
#ifdef WG_EXP_NOGEMM  // timing experiment switch (garbage results; the dead staging is compiled out with it)
      for (int st = 0; st < 0; ++st) {
#else
      for (int st = 0; st < 6; ++st) {
#endif
        const int tb = 4 * st + kq;
        const int wr = tb / PL, wc = tb % PL;
        // V: B^T d B of the tile's 4x4 conv1 patch (rows 2*wr .., columns 2*wc ..), channels tl, 16 + tl
        const fvec2* d0 = reinterpret_cast<const fvec2*>(a1_s + ((2 * wr + tp) * A1 + 2 * wc) * WG_CS) + tl;
        const int drow = (tq - tp) * A1 * (WG_CS / 2);
        fvec2 pa[4], pb[4];  // rows tp, tq of the patch, columns c: (ci tl, ci 16 + tl)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          pa[c] = d0[c * (WG_CS / 2)];
          pb[c] = d0[drow + c * (WG_CS / 2)];
        }
        float va[2][4];
#pragma unroll
        for (int ch = 0; ch < 2; ++ch) {
          float t[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) t[c] = fmaf(sq, pb[c][ch], pa[c][ch]);
          va[ch][0] = t[0] - t[2];
          va[ch][1] = t[1] + t[2];
          va[ch][2] = t[2] - t[1];
          va[ch][3] = t[1] - t[3];
        }
        // D: delta's single nonzero v at (dy, dx): D[i][j] = v * A[i][dy] * A[j][dx], channels 16*cg + tl
        float db[4][4];
#pragma unroll
        for (int cg = 0; cg < 4; ++cg) {
          const int2 vs = vq_s[tb * WG_VS + 16 * cg + tl];
          const float v = __int_as_float(vs.x);
          const int sl = vs.y;
          const float vi = v * ((sl & 2) ? fa1 : fa0);  // v * A[i][dy]: exact
          const bool dx = (sl & 1) != 0;
          db[cg][0] = dx ? 0.0f : vi;
          db[cg][1] = vi;
          db[cg][2] = dx ? -vi : vi;
          db[cg][3] = dx ? -vi : 0.0f;
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int ch = 0; ch < 2; ++ch)
#pragma unroll
            for (int cg = 0; cg < 4; ++cg) acc[jj][ch][cg] = mfma16(va[ch][jj], db[cg][jj], acc[jj][ch][cg]);
      }
    }
  }
  // inverse transform dW2[ky][kx] = sum_i G^T[ky][i] P_i[kx], P_i[kx] = sum_j M[i][j] G[j][kx]: wave i folds
  // its row (P_i0 = M_i0 + .5 M_i1 + .5 M_i2, P_i1 = .5 M_i1 - .5 M_i2, P_i2 = .5 M_i1 + .5 M_i2 + M_i3), the
  // waves exchange P through LDS, one ci half at a time.  Lane holds ci 16*ch + 4*kq + rr, co 16*cg + tl.
  gb_s[wave][lane] = gb;
  float* out = w2_part + ((int64_t)r * splits + sp) * MPLC_CNN_W2P;
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    __syncthreads();  // previous readers of smem (the last band, or the previous half) done
    float* px = smem + wi * WG_PX;
#pragma unroll
    for (int cg = 0; cg < 4; ++cg)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float m0 = acc[0][ch][cg][rr], m1 = acc[1][ch][cg][rr], m2 = acc[2][ch][cg][rr],
                    m3 = acc[3][ch][cg][rr];
        const int o = (4 * kq + rr) * C2 + 16 * cg + tl;
        px[o] = (m0 + 0.5f * m1) + 0.5f * m2;
        px[16 * C2 + o] = 0.5f * m1 - 0.5f * m2;
        px[32 * C2 + o] = (0.5f * m1 + 0.5f * m2) + m3;
      }
    __syncthreads();
    for (int e = tid; e < 16 * C2; e += WG_THREADS) {  // (ci in half, co)
      const int ci = 16 * ch + (e >> 6), co = e & 63;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float p0 = smem[0 * WG_PX + kx * 16 * C2 + e], p1 = smem[1 * WG_PX + kx * 16 * C2 + e];
        const float p2 = smem[2 * WG_PX + kx * 16 * C2 + e], p3 = smem[3 * WG_PX + kx * 16 * C2 + e];
        const float w0 = (p0 + 0.5f * p1) + 0.5f * p2;
        const float w1 = 0.5f * p1 - 0.5f * p2;
        const float w2 = (0.5f * p1 + 0.5f * p2) + p3;
        out[((0 * 3 + kx) * C1 + ci) * C2 + co] = w0;
        out[((1 * 3 + kx) * C1 + ci) * C2 + co] = w1;
        out[((2 * 3 + kx) * C1 + ci) * C2 + co] = w2;
      }
    }
  }
  if (tid < C2) out[9 * C1 * C2 + tid] = (gb_s[0][tid] + gb_s[1][tid]) + (gb_s[2][tid] + gb_s[3][tid]);
}

}  // namespace

namespace mplc_mnist {
void launch_conv_wgrad(int splits, int n_rep, hipStream_t s, const float* x, const int32_t* idx, const int32_t* cnt,
                       int bmax, const float* params, int64_t stride, const float* dPool, const uint8_t* code,
                       float* w2_part) {
  conv_wgrad_kernel<<<dim3(splits, n_rep), WG_THREADS, 0, s>>>(x, idx, cnt, bmax, splits, params, stride, dPool, code,
                                                               w2_part);
}
}  // namespace mplc_mnist
