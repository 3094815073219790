// Probe: v_mfma_f32_4x4x1f32 (16 blocks of 4x4, K = 1) on gfx950.
//  1. what it computes per output element against fmaf(a, b, c), and its lane layout (assumed: A and B of block
//     b, row / column i at lane 4b + i; D of block b, row i, column j at lane 4b + j, register i);
//  2. issue cost per instruction, one wave and two waves per SIMD, beside v_mfma_f32_16x16x4f32;
//  3. whether independent f32 VALU work in the same wave slows the f32 MFMA stream (shared issue or pipe).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

typedef float fvec4 __attribute__((ext_vector_type(4)));

__global__ void exact_probe(const float* A, const float* B, const float* C, float* D) {
  const int l = threadIdx.x, t = blockIdx.x;
  const float a = A[t * 64 + l], b = B[t * 64 + l];
  fvec4 c;
  for (int v = 0; v < 4; ++v) c[v] = C[t * 256 + (l >> 2) * 16 + v * 4 + (l & 3)];  // [blk][row v][col l&3]
  fvec4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int v = 0; v < 4; ++v) D[t * 256 + (l >> 2) * 16 + v * 4 + (l & 3)] = d[v];
}

// FORM 0: 16x16x4, FORM 1: 4x4x1; NV independent VALU fmas per MFMA
template <int FORM, int NV>
__global__ void rate_probe(float* out, long long* cyc, int iters) {
  const int l = threadIdx.x;
  float a = 1e-3f * (l + 1), b = 2e-3f * (l + 3);
  fvec4 acc[8];
  for (int k = 0; k < 8; ++k) acc[k] = fvec4{0.0f, 0.0f, 0.0f, 0.0f};
  float v[8];
  for (int k = 0; k < 8; ++k) v[k] = 1e-4f * (k + l);
  __syncthreads();
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (FORM == 0)
        acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[k], 0, 0, 0);
      else
        acc[k] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[k], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < NV; ++q) v[(k + q) & 7] = fmaf(v[(k + q) & 7], 0.999f, 1e-7f);
    }
    asm volatile("" : "+v"(a), "+v"(b));
  }
  const long long t1 = clock64();
  float s = 0.0f;
  for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3] + v[k];
  out[blockIdx.x * blockDim.x + l] = s;
  if ((l & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int FORM, int NV>
static void run_rate(const char* name, int threads) {
  const int iters = 4096;
  float* out;
  long long* cyc;
  hipMalloc(&out, 1024 * 4);
  hipMalloc(&cyc, 16 * 8);
  rate_probe<FORM, NV><<<1, threads>>>(out, cyc, iters);
  if (hipDeviceSynchronize() != hipSuccess) { printf("rate kernel failed\n"); exit(1); }
  long long h[16];
  hipMemcpy(h, cyc, 16 * 8, hipMemcpyDeviceToHost);
  const int waves = threads / 64;
  long long mx = 0;
  for (int w = 0; w < waves; ++w) mx = h[w] > mx ? h[w] : mx;
  // waves of one block are spread over the CU's 4 SIMDs: waves / 4 (at least 1) per SIMD
  const int per_simd = waves > 4 ? waves / 4 : 1;
  printf("%-10s valu/mfma %2d  waves/SIMD %d: %.2f cycles per MFMA per SIMD (clock64)\n", name, NV, per_simd,
         (double)mx / ((double)iters * 8 * per_simd));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  const int T = 4096;
  std::mt19937 g(11);
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  float *A = (float*)malloc(T * 64 * 4), *B = (float*)malloc(T * 64 * 4), *C = (float*)malloc(T * 256 * 4),
        *D = (float*)malloc(T * 256 * 4);
  for (int i = 0; i < T * 64; ++i) { A[i] = u(g); B[i] = u(g); }
  for (int i = 0; i < T * 256; ++i) C[i] = u(g) * ((i % 3) ? 1.0f : 1e-3f);
  float *dA, *dB, *dC, *dD;
  hipMalloc(&dA, T * 64 * 4); hipMalloc(&dB, T * 64 * 4); hipMalloc(&dC, T * 256 * 4); hipMalloc(&dD, T * 256 * 4);
  hipMemcpy(dA, A, T * 64 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B, T * 64 * 4, hipMemcpyHostToDevice);
  hipMemcpy(dC, C, T * 256 * 4, hipMemcpyHostToDevice);
  exact_probe<<<T, 64>>>(dA, dB, dC, dD);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  hipMemcpy(D, dD, T * 256 * 4, hipMemcpyDeviceToHost);
  long n = 0, fma_hyp = 0, fma_tr = 0, muladd = 0;
  for (int t = 0; t < T; ++t)
    for (int blk = 0; blk < 16; ++blk)
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          const float c = C[t * 256 + blk * 16 + i * 4 + j], d = D[t * 256 + blk * 16 + i * 4 + j];
          const float a = A[t * 64 + 4 * blk + i], b = B[t * 64 + 4 * blk + j];
          const float at = A[t * 64 + 4 * blk + j], bt = B[t * 64 + 4 * blk + i];
          ++n;
          fma_hyp += (d == fmaf(a, b, c));
          fma_tr += (d == fmaf(at, bt, c));
          volatile float pr = a * b;
          muladd += (d == c + pr);
        }
  printf("4x4x1f32 outputs %ld: fmaf (A row at lane 4b+i, B col at lane 4b+j) %ld, transposed layout %ld, "
         "mul then add %ld\n", n, fma_hyp, fma_tr, muladd);
  run_rate<0, 0>("16x16x4", 64);
  run_rate<1, 0>("4x4x1", 64);
  run_rate<0, 0>("16x16x4", 512);
  run_rate<1, 0>("4x4x1", 512);
  run_rate<0, 2>("16x16x4", 64);
  run_rate<0, 4>("16x16x4", 64);
  run_rate<0, 8>("16x16x4", 64);
  run_rate<0, 16>("16x16x4", 64);
  run_rate<0, 4>("16x16x4", 512);
  run_rate<0, 8>("16x16x4", 512);
  run_rate<0, 16>("16x16x4", 512);
  run_rate<1, 1>("4x4x1", 64);
  run_rate<1, 2>("4x4x1", 64);
  run_rate<1, 2>("4x4x1", 512);
  return 0;
}
