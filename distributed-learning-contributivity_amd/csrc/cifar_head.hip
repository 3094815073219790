// CIFAR10 trainer: the training head (Dense(10) + softmax-CE gradient + RMSprop of W6) and the evaluation head,
// in their own translation unit.  The rest of the trainer (cifar_cnn.hip) is compiled without SLP vectorisation,
// which takes the v_mov_b32-fed v_pk_add_f32 out of its Winograd loops; these two kernels keep the default flags,
// under which their expf / logf and dot products compile to the instruction sequence every earlier round's
// results were produced with (same bits: the v(S) probe hashes, scripts/r05/gpu_ab_noslp.sh).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mplc_hip.h"
#include "cifar_common.h"

namespace {

// ------------------------------------------------------------------------------------------------
// Head: Dense(10) + softmax-CE gradient (mean over the batch), dW6/db6 + RMSprop, dh5 through dropout'
// and relu'.  One block per replica.
// ------------------------------------------------------------------------------------------------
constexpr int HEAD_CHUNK = 256;
constexpr int W6N = HID * NCLS + NCLS;  // W6 and b6 are contiguous
constexpr int HEAD_G = (W6N + 255) / 256;

__global__ __launch_bounds__(256) void head_kernel(const float* __restrict__ D5, const uint8_t* __restrict__ code5,
                                                   const int32_t* __restrict__ idx, const int32_t* __restrict__ labels,
                                                   const int32_t* __restrict__ cnt, const int32_t* __restrict__ opt_t,
                                                   int bmax, float* __restrict__ params, float* __restrict__ rms,
                                                   float* __restrict__ dH, float lr, float rho, float omr,
                                                   float decay, float eps, double* __restrict__ hstats) {
  __shared__ float w6_s[W6N];
  __shared__ float dl_s[HEAD_CHUNK * NCLS];
  __shared__ double hs_s[2][HEAD_CHUNK];
  const int r = blockIdx.x;
  const int count = cnt[r];
  const int tid = threadIdx.x;
  if (count == 0) {
    if (hstats && tid < 3) hstats[(int64_t)r * 3 + tid] = 0.0;
    return;
  }
  float* P = params + (int64_t)r * STRIDE;
  for (int e = tid; e < W6N; e += 256) w6_s[e] = P[OFF_W6 + e];
  __syncthreads();
  const float inv_b = 1.0f / (float)count;
  float gacc[HEAD_G];
#pragma unroll
  for (int u = 0; u < HEAD_G; ++u) gacc[u] = 0.0f;
  double hl = 0.0, hc = 0.0;  // this thread's training CE / correct sums (hstats)
  const float* Dr = D5 + (int64_t)r * bmax * HID;
  for (int c0 = 0; c0 < count; c0 += HEAD_CHUNK) {
    const int cn = min(HEAD_CHUNK, count - c0);
    if (tid < cn) {
      const int jj = c0 + tid;
      const float* h = Dr + (int64_t)jj * HID;
      float z[NCLS];
#pragma unroll
      for (int o = 0; o < NCLS; ++o) z[o] = w6_s[HID * NCLS + o];
      for (int c = 0; c < HID; ++c) {
        const float hv = h[c];
#pragma unroll
        for (int o = 0; o < NCLS; ++o) z[o] += hv * w6_s[c * NCLS + o];
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
    for (int u = 0; u < HEAD_G; ++u) {
      const int e = tid + 256 * u;
      if (e < HID * NCLS) {
        const int c = e / NCLS, o = e % NCLS;
        float acc = 0.0f;
        for (int jj = 0; jj < cn; ++jj) acc += Dr[(int64_t)(c0 + jj) * HID + c] * dl_s[jj * NCLS + o];
        gacc[u] += acc;
      } else if (e < W6N) {
        const int o = e - HID * NCLS;
        float acc = 0.0f;
        for (int jj = 0; jj < cn; ++jj) acc += dl_s[jj * NCLS + o];
        gacc[u] += acc;
      }
    }
    const uint8_t* cd = code5 + (int64_t)r * bmax * HID;
    for (int e = tid; e < cn * HID; e += 256) {
      const int jj = e / HID, c = e % HID;
      float acc = 0.0f;
#pragma unroll
      for (int o = 0; o < NCLS; ++o) acc += dl_s[jj * NCLS + o] * w6_s[c * NCLS + o];
      const uint32_t k = cd[(int64_t)(c0 + jj) * HID + c];
      dH[((int64_t)r * bmax + c0 + jj) * HID + c] =
          ((k & CODE_KEEP) && (k & CODE_POS)) ? acc * SCALE_50 : 0.0f;
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
  const RmsCfg cfg = rms_cfg(opt_t[r], lr, rho, omr, decay, eps);
  float* Rr = rms + (int64_t)r * STRIDE;
#pragma unroll
  for (int u = 0; u < HEAD_G; ++u) {
    const int e = tid + 256 * u;
    if (e < W6N) {
      const int64_t o = OFF_W6 + e;
      float p = P[o], aa = Rr[o];
      rms_apply(p, aa, gacc[u], cfg);
      P[o] = p;
      Rr[o] = aa;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Evaluation head: logits, accuracy count and summed cross-entropy per model (deterministic order).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void eval_head_kernel(const float* __restrict__ H, int count, int chunk,
                                                        const int32_t* __restrict__ labels, int row_base,
                                                        const float* __restrict__ params, int64_t stride,
                                                        int32_t* __restrict__ correct, double* __restrict__ loss_sum) {
  __shared__ float w6_s[W6N];
  __shared__ double ls[256];
  __shared__ int cs[256];
  const int mdl = blockIdx.x;
  const int tid = threadIdx.x;
  const float* P = params + (int64_t)mdl * stride;
  for (int e = tid; e < W6N; e += 256) w6_s[e] = P[OFF_W6 + e];
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
      for (int o = 0; o < NCLS; ++o) z[o] = w6_s[HID * NCLS + o];
      for (int c = 0; c < HID; ++c) {
        const float hv = h[c];
#pragma unroll
        for (int o = 0; o < NCLS; ++o) z[o] += hv * w6_s[c * NCLS + o];
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

}  // namespace

void cifar_launch_head(int R, hipStream_t s, const float* D5, const uint8_t* code5, const int32_t* idx,
                       const int32_t* labels, const int32_t* cnt, const int32_t* opt_t, int bmax, float* params,
                       float* rms, float* dH, float lr, float rho, float omr, float decay, float eps, double* hstats) {
  head_kernel<<<R, 256, 0, s>>>(D5, code5, idx, labels, cnt, opt_t, bmax, params, rms, dH, lr, rho, omr, decay, eps,
                                hstats);
}

void cifar_launch_eval_head(int n_models, hipStream_t s, const float* H, int count, int chunk, const int32_t* labels,
                            int row_base, const float* params, int64_t stride, int32_t* correct, double* loss_sum) {
  eval_head_kernel<<<n_models, 256, 0, s>>>(H, count, chunk, labels, row_base, params, stride, correct, loss_sum);
}
