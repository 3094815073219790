// Shared definitions of the batched MNIST CNN kernels (csrc/mnist_cnn.hip, csrc/mnist_wgrad.hip): layer
// geometry, model-row offsets, MFMA wrappers and the conv1 recompute that every kernel needing conv1's output
// uses (so forward and backward agree bit for bit).  Internal to the library; the contract is
// include/mplc_hip_cnn.h.
#ifndef MPLC_MNIST_COMMON_H
#define MPLC_MNIST_COMMON_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mplc_hip.h"
#include "keyed.h"
#include "xcd.h"

// Wave-index tag: a barrier-free loop body instantiated once per wave index (compile-time Winograd transform
// signs), dispatched by a wave-uniform switch
template <int V>
struct IntC {
  static constexpr int value = V;
};

// Timing-experiment switches compile parts of a kernel out and give WRONG results by design (A/B probes of
// where a kernel's time goes).  A product build must never carry one.
#if (defined(BWD_EXP_NOSTAGE) || defined(BWD_EXP_NOSTAGE_UR) || defined(BWD_EXP_NOSTAGE_DZ) || \
     defined(BWD_EXP_NOEPI) || defined(WG_EXP_NOCONV1) || defined(WG_EXP_NOGEMM)) && !defined(MPLC_EXPERIMENT)
#error "a *_EXP_* timing switch produces wrong results: define MPLC_EXPERIMENT for an A/B experiment build"
#endif

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float fvec4 __attribute__((ext_vector_type(4)));
typedef float fvec2 __attribute__((ext_vector_type(2)));

constexpr int IMG = 28;
constexpr int A1 = 26;
constexpr int C1 = 32;
constexpr int Z2 = 24;
constexpr int C2 = 64;
constexpr int PL = 12;
constexpr int FEAT = 9216;
constexpr int HID = 128;
constexpr int NCLS = 10;
constexpr int64_t OFF_W1 = MPLC_CNN_OFF_W1, OFF_B1 = MPLC_CNN_OFF_B1, OFF_W2 = MPLC_CNN_OFF_W2,
                  OFF_B2 = MPLC_CNN_OFF_B2, OFF_W3 = MPLC_CNN_OFF_W3, OFF_B3 = MPLC_CNN_OFF_B3,
                  OFF_W4 = MPLC_CNN_OFF_W4, OFF_B4 = MPLC_CNN_OFF_B4;
constexpr int ADAM_LAST = 1 << 30;  // adam_t flag: the optimizer's last step
constexpr int A1P = 33;  // padded channel stride of conv1 output tiles in LDS (bank-conflict-free A reads)

// Register cap of the three convolution kernels (build experiments: -DCONV_VGPR_CAP=N leaves 512 - 2N registers
// per SIMD lane beside two convolution waves, room for a wave of another kernel)
#ifdef CONV_VGPR_CAP
#define CONV_REGS __attribute__((amdgpu_num_vgpr(CONV_VGPR_CAP)))
#else
#define CONV_REGS
#endif

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

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.0f;
  return z;
}

// conv1 weights as the MFMA B operand: lane (kh, ci) holds W1e[2s + kh][ci], s = 0..4, where W1e rows 0..8
// are the 3x3 taps (ky*3 + kx) and row 9 is the bias.
__device__ __forceinline__ void load_w1r(const float* __restrict__ P, int kh, int ci, float (&w1r)[5]) {
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int k = 2 * s + kh;
    w1r[s] = (k < 9) ? P[OFF_W1 + k * C1 + ci] : P[OFF_B1 + ci];
  }
}

// conv1 + bias (pre-ReLU) of 32 positions on the fp32 MFMA: K = 9 taps + bias (patch value 1) in 5 k-steps.
// Lane (kh, i) passes `pix`, the img_s offset of its position's top-left pixel (row stride IMG).
// Result in accumulator layout: reg -> tile row (reg&3) + 8*(reg>>2) + 4*kh, column = channel lane&31.
// All kernels that need conv1's output use this one routine, so forward and backward agree bit for bit.
__device__ __forceinline__ floatx16 conv1_mfma(const float* img_s, int pix, int kh, const float (&w1r)[5]) {
  floatx16 acc = zero16();
  // tap k = 2s + kh at (k / 3) * IMG + k % 3
  acc = mfma32(img_s[pix + (kh ? 1 : 0)], w1r[0], acc);
  acc = mfma32(img_s[pix + (kh ? IMG : 2)], w1r[1], acc);
  acc = mfma32(img_s[pix + (kh ? IMG + 2 : IMG + 1)], w1r[2], acc);
  acc = mfma32(img_s[pix + (kh ? 2 * IMG + 1 : 2 * IMG)], w1r[3], acc);
  const float a8 = img_s[pix + 2 * IMG + 2];
  acc = mfma32(kh ? 1.0f : a8, w1r[4], acc);
  return acc;
}

// accumulator register -> row within a 32-row tile (v_mfma_f32_32x32x2f32 C/D layout)
__device__ __forceinline__ int acc_row(int reg, int kh) { return (reg & 3) + 8 * (reg >> 2) + 4 * kh; }

__device__ __forceinline__ fvec4 mfma16(float a, float b, fvec4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// conv2 weight gradient (csrc/mnist_wgrad.hip): samples per split-K block, fixed so that a replica's sums do not
// depend on the batch (bs 27 of config #3 = 3 equal splits: no short split block; 8 -> 8, 8, 8, 3: +18 % wgrad)
constexpr int WG_THREADS = 256;
constexpr int WG_SAMPLES = 9;

}  // namespace

// Launch of the conv2 weight gradient, compiled in its own translation unit (csrc/mnist_wgrad.hip): in the same
// unit as conv_fwd_kernel it made the register allocator spill 4 of conv_fwd's registers (12 B of scratch per
// lane, 0.13 GB more HBM traffic per launch at config #3's size).
namespace mplc_mnist {
void launch_conv_wgrad(int splits, int n_rep, hipStream_t s, const float* x, const int32_t* idx, const int32_t* cnt,
                       int bmax, const float* params, int64_t stride, const float* dPool, const uint8_t* code,
                       float* w2_part);
}  // namespace mplc_mnist

#endif  // MPLC_MNIST_COMMON_H
