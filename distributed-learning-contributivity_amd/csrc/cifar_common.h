// Definitions shared by the CIFAR10 trainer's translation units (cifar_cnn.hip: every kernel but the head;
// cifar_head.hip: the training and evaluation heads, compiled with different flags, build_native.py FILE_FLAGS).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mplc_hip_cifar.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float fvec4 __attribute__((ext_vector_type(4)));

constexpr int64_t OFF_W1 = MPLC_CIFAR_OFF_W1, OFF_B1 = MPLC_CIFAR_OFF_B1, OFF_W2 = MPLC_CIFAR_OFF_W2,
                  OFF_B2 = MPLC_CIFAR_OFF_B2, OFF_W3 = MPLC_CIFAR_OFF_W3, OFF_B3 = MPLC_CIFAR_OFF_B3,
                  OFF_W4 = MPLC_CIFAR_OFF_W4, OFF_B4 = MPLC_CIFAR_OFF_B4, OFF_W5 = MPLC_CIFAR_OFF_W5,
                  OFF_B5 = MPLC_CIFAR_OFF_B5, OFF_W6 = MPLC_CIFAR_OFF_W6, OFF_B6 = MPLC_CIFAR_OFF_B6;
constexpr int64_t STRIDE = MPLC_CIFAR_STRIDE;
constexpr int IMG_SZ = 32 * 32 * 3;
constexpr int FEAT = MPLC_CIFAR_D4;  // 2304
constexpr int HID = MPLC_CIFAR_H5;   // 512
constexpr int NCLS = 10;
constexpr int WGS = MPLC_CIFAR_WG_SAMPLES;
constexpr int WPART = MPLC_CIFAR_WPART;

// dropout (Keras Dropout -> tf.nn.dropout: (x * (1/(1-rate))) * (u >= rate)); u = 24-bit keyed counter
constexpr uint32_t DROP_L2 = 2, DROP_L4 = 4, DROP_L5 = 5;
constexpr uint32_t THR_25 = 1u << 22;  // 0.25 * 2^24
constexpr uint32_t THR_50 = 1u << 23;  // 0.5 * 2^24
constexpr float SCALE_25 = 0x1.555556p+0f;  // float(1 / 0.75)
constexpr float SCALE_50 = 2.0f;
constexpr uint8_t CODE_KEEP = 0x40, CODE_POS = 0x80;

// 32-bit finaliser (lowbias32): a bijection with full avalanche; 2 multiplies, cheap next to the 64-bit mix.
__host__ __device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// keep(element e) = top 24 bits of hash32(row_seed ^ e) >= rate * 2^24, row_seed = drop_row_seed(step key,
// layer, slot j): one hash per element (restated in oracle/cifar_cnn.py).
__device__ __forceinline__ uint32_t drop_row_seed(uint64_t dkey, uint32_t layer, uint32_t j) {
  return hash32((uint32_t)dkey ^ hash32((uint32_t)(dkey >> 32) ^ (layer << 24) ^ j));
}

__device__ __forceinline__ bool drop_keep(uint32_t row_seed, uint32_t e, uint32_t thr) {
  return (hash32(row_seed ^ e) >> 8) >= thr;
}

// Cross-lane add within rows of 16 lanes on DPP (VALU, no LDS round trip).  Each level adds the partner's
// value exactly as `d += __shfl_xor(d, m)` does (commutative adds of the same operands: bit-identical).
template <int CTRL>
__device__ __forceinline__ float dpp_partner(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
constexpr int DPP_XOR1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141;  // lane i <-> 7 - i within 8 (the other quad after two levels)
constexpr int DPP_MIRROR = 0x140;       // lane i <-> 15 - i within 16 (the other 8 after three levels)

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// v_mfma_f32_4x4x1f32: 16 blocks of 4x4, K = 1.  Block b takes A[b][i] from lane 4b + i and B[b][j] from lane
// 4b + j; D[b][i][j] lands in lane 4b + j, register i.  Each output is fmaf(a, b, c) (measured on 2^20 outputs,
// scripts/probes/mfma_4x4.hip), issued in 8-10 cycles per SIMD: the rate of the 16x16x4 form at a quarter of its M.
__device__ __forceinline__ fvec4 mfma4(float a, float b, fvec4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.0f;
  return z;
}

// accumulator register -> row within a 32-row tile (v_mfma_f32_32x32x2f32 C/D layout)
__device__ __forceinline__ int acc_row(int reg, int kh) { return (reg & 3) + 8 * (reg >> 2) + 4 * kh; }

// ------------------------------------------------------------------------------------------------
// Keras 2.3.1 RMSprop (keras/optimizers.py): lr_t = lr / (1 + decay * iterations) with the iteration
// count before this update; a = rho a + (1 - rho) g^2; p -= lr_t g / (sqrt(a) + eps).  (1 - rho) comes
// from the host (a Python double rounded once to fp32, as Keras does).  A fresh optimizer (FedAvg partner
// fit, t == 1) has a == 0.
// ------------------------------------------------------------------------------------------------
struct RmsCfg {
  float lr_t, rho, one_m_rho, eps;
  bool reset;
};

__device__ __forceinline__ RmsCfg rms_cfg(int t, float lr, float rho, float omr, float decay, float eps) {
  RmsCfg c;
  const float it = (float)(t - 1);
  c.lr_t = lr * (1.0f / (1.0f + decay * it));
  c.rho = rho;
  c.one_m_rho = omr;
  c.eps = eps;
  c.reset = (t == 1);
  return c;
}

__device__ __forceinline__ void rms_apply(float& p, float& a, float g, const RmsCfg& c) {
  // Keras evaluates rho a + (1 - rho) g^2 as separate multiplies and an add: no fused multiply-add here, in every
  // kernel (the compiler's contraction otherwise depends on how it vectorised the caller)
#pragma clang fp contract(off)
  const float a0 = c.reset ? 0.0f : a;
  const float an = c.rho * a0 + c.one_m_rho * (g * g);
  p = p - c.lr_t * g / (sqrtf(an) + c.eps);
  a = an;
}

}  // namespace

// launches of the head kernels (cifar_head.hip) on stream s
void cifar_launch_head(int R, hipStream_t s, const float* D5, const uint8_t* code5, const int32_t* idx,
                       const int32_t* labels, const int32_t* cnt, const int32_t* opt_t, int bmax, float* params,
                       float* rms, float* dH, float lr, float rho, float omr, float decay, float eps, double* hstats);
void cifar_launch_eval_head(int n_models, hipStream_t s, const float* H, int count, int chunk, const int32_t* labels,
                            int row_base, const float* params, int64_t stride, int32_t* correct, double* loss_sum);
