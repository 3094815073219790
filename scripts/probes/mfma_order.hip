// Probe: what v_mfma_f32_16x16x4f32 computes per output element, compared with scalar fp32 chains over K = 4:
// a sequential fmaf chain in k order from C, the same chain in reverse order, products summed first then added
// to C, and an fp64 reference rounded once.  Prints how many of 256 x trials outputs each form matches exactly.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

typedef float fvec4 __attribute__((ext_vector_type(4)));

__global__ void probe(const float* A, const float* B, const float* C, float* D) {
  // lane l: A[l % 16][l / 16] (row i, k), B[l / 16][l % 16] (k, col j); D lane l holds rows 4 (l/16) + v, col l % 16
  const int l = threadIdx.x;
  const int t = blockIdx.x;
  const float a = A[t * 64 + (l % 16) * 4 + l / 16];
  const float b = B[t * 64 + (l / 16) * 16 + l % 16];
  fvec4 c;
  for (int v = 0; v < 4; ++v) c[v] = C[t * 256 + (4 * (l / 16) + v) * 16 + l % 16];
  fvec4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int v = 0; v < 4; ++v) D[t * 256 + (4 * (l / 16) + v) * 16 + l % 16] = d[v];
}

int main() {
  const int T = 4096;
  std::mt19937 g(7);
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
  probe<<<T, 64>>>(dA, dB, dC, dD);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  hipMemcpy(D, dD, T * 256 * 4, hipMemcpyDeviceToHost);
  long n = 0, seq = 0, rev = 0, prod = 0, f64 = 0, seqm = 0;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        const float* a = A + t * 64 + i * 4;  // A[i][k]
        float b[4];
        for (int k = 0; k < 4; ++k) b[k] = B[t * 64 + k * 16 + j];
        const float c = C[t * 256 + i * 16 + j], d = D[t * 256 + i * 16 + j];
        float s = c;
        for (int k = 0; k < 4; ++k) s = fmaf(a[k], b[k], s);
        float r = c;
        for (int k = 3; k >= 0; --k) r = fmaf(a[k], b[k], r);
        float p = 0.0f;
        for (int k = 0; k < 4; ++k) p = fmaf(a[k], b[k], p);
        p = p + c;
        float m = c;  // multiply then add, separately rounded, k order
        for (int k = 0; k < 4; ++k) { volatile float pr = a[k] * b[k]; m = m + pr; }
        double e = c;
        for (int k = 0; k < 4; ++k) e += (double)a[k] * (double)b[k];
        ++n;
        seq += (d == s); rev += (d == r); prod += (d == p); f64 += (d == (float)e); seqm += (d == m);
      }
  printf("outputs %ld: fma chain k order %ld, reverse %ld, products-then-C %ld, fp64 rounded once %ld, "
         "mul+add k order %ld\n", n, seq, rev, prod, f64, seqm);
  return 0;
}
