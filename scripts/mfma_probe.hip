// Sustained fp32-MFMA rate of the whole chip (the practical roofline under DVFS), on random register
// operands: every CU runs 2 waves per SIMD of back-to-back v_mfma_f32_16x16x4f32 / v_mfma_f32_32x32x2f32 on
// independent accumulators.  Build: hipcc -O3 --offload-arch=gfx950 scripts/mfma_probe.hip -o mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma16(const float* in, float* out, int iters) {
  float a = in[threadIdx.x], b = in[threadIdx.x + 256];
  f4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void mfma32(const float* in, float* out, int iters) {
  float a = in[threadIdx.x], b = in[threadIdx.x + 256];
  f16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 16; ++j) s += acc[i][j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float *in, *out;
  hipMalloc(&in, 4096);
  hipMalloc(&out, 256 * 4 * 4096);
  float h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 0.5f + (i % 97) * 0.001f;
  hipMemcpy(in, h, 4096, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 2;  // 2 blocks of 4 waves per CU = 2 waves per SIMD
  const int iters = 20000;
  for (int k = 0; k < 2; ++k) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (k == 0) mfma16<<<blocks, 256>>>(in, out, iters);
      else mfma32<<<blocks, 256>>>(in, out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // 16x16x4: 2048 FLOP per wave-MFMA, 8 per iteration; 32x32x2: 4096 FLOP, 4 per iteration
      const double flop = (double)blocks * 4 * iters * (k == 0 ? 8 * 2048.0 : 4 * 4096.0);
      if (rep == 2) printf("%s: %.2f ms, %.1f TF/s\n", k == 0 ? "mfma_f32_16x16x4" : "mfma_f32_32x32x2", ms, flop / ms / 1e9);
    }
  }
  return 0;
}
