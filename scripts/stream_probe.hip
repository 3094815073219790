// HBM ceiling of dense1_bwd_adam's access pattern (MNIST W3 slices of many replicas), measured without its
// arithmetic: per 32-row x 128-col slice of every replica's W3, read W, m, v and write them back (the
// Adam pass), with the same block shape, fvec4 layout and nontemporal moments as the kernel.
// Variants: rmw3 (the pattern), rmw3_plain (no nontemporal hints), read3 (reads only), copy1 (one stream
// read, one written), rmw3_allnt (W nontemporal too), rmw3_pipe<S> (S slices per block, the next slice's loads
// in flight during the current slice's stores).  Build: hipcc -O3 --offload-arch=gfx950 scripts/stream_probe.hip -o stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float fvec4 __attribute__((ext_vector_type(4)));
constexpr int64_t STRIDE = 1199936, OFF_W3 = 18816;
constexpr int ROWS = 32, HID = 128, FEAT = 9216;

template <bool NT>
__global__ __launch_bounds__(256) void rmw3(float* P, float* M, float* V) {
  const int r = blockIdx.y, k0 = blockIdx.x * ROWS, tid = threadIdx.x, rowl = tid >> 3, c8 = tid & 7;
  const int64_t off = (int64_t)r * STRIDE + OFF_W3 + (int64_t)(k0 + rowl) * HID;
  fvec4* W = reinterpret_cast<fvec4*>(P + off) + c8;
  fvec4* Mr = reinterpret_cast<fvec4*>(M + off) + c8;
  fvec4* Vr = reinterpret_cast<fvec4*>(V + off) + c8;
  fvec4 w[4], m[4], v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = W[8 * i];
    m[i] = NT ? __builtin_nontemporal_load(Mr + 8 * i) : Mr[8 * i];
    v[i] = NT ? __builtin_nontemporal_load(Vr + 8 * i) : Vr[8 * i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    W[8 * i] = w[i] + 1e-7f;
    if (NT) {
      __builtin_nontemporal_store(m[i] * 0.9f, Mr + 8 * i);
      __builtin_nontemporal_store(v[i] * 0.99f, Vr + 8 * i);
    } else {
      Mr[8 * i] = m[i] * 0.9f;
      Vr[8 * i] = v[i] * 0.99f;
    }
  }
}

// every access nontemporal (W too)
__global__ __launch_bounds__(256) void rmw3_allnt(float* P, float* M, float* V) {
  const int r = blockIdx.y, k0 = blockIdx.x * ROWS, tid = threadIdx.x, rowl = tid >> 3, c8 = tid & 7;
  const int64_t off = (int64_t)r * STRIDE + OFF_W3 + (int64_t)(k0 + rowl) * HID;
  fvec4* W = reinterpret_cast<fvec4*>(P + off) + c8;
  fvec4* Mr = reinterpret_cast<fvec4*>(M + off) + c8;
  fvec4* Vr = reinterpret_cast<fvec4*>(V + off) + c8;
  fvec4 w[4], m[4], v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = __builtin_nontemporal_load(W + 8 * i);
    m[i] = __builtin_nontemporal_load(Mr + 8 * i);
    v[i] = __builtin_nontemporal_load(Vr + 8 * i);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    __builtin_nontemporal_store(w[i] + 1e-7f, W + 8 * i);
    __builtin_nontemporal_store(m[i] * 0.9f, Mr + 8 * i);
    __builtin_nontemporal_store(v[i] * 0.99f, Vr + 8 * i);
  }
}

// S consecutive slices per block, the loads of slice s+1 issued before the stores of slice s
template <int S>
__global__ __launch_bounds__(256) void rmw3_pipe(float* P, float* M, float* V) {
  const int r = blockIdx.y, tid = threadIdx.x, rowl = tid >> 3, c8 = tid & 7;
  fvec4 w[2][4], m[2][4], v[2][4];
  auto ld = [&](int s, int b) {
    const int64_t off = (int64_t)r * STRIDE + OFF_W3 + (int64_t)((blockIdx.x * S + s) * ROWS + rowl) * HID;
    fvec4* W = reinterpret_cast<fvec4*>(P + off) + c8;
    fvec4* Mr = reinterpret_cast<fvec4*>(M + off) + c8;
    fvec4* Vr = reinterpret_cast<fvec4*>(V + off) + c8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[b][i] = W[8 * i];
      m[b][i] = __builtin_nontemporal_load(Mr + 8 * i);
      v[b][i] = __builtin_nontemporal_load(Vr + 8 * i);
    }
  };
  auto st = [&](int s, int b) {
    const int64_t off = (int64_t)r * STRIDE + OFF_W3 + (int64_t)((blockIdx.x * S + s) * ROWS + rowl) * HID;
    fvec4* W = reinterpret_cast<fvec4*>(P + off) + c8;
    fvec4* Mr = reinterpret_cast<fvec4*>(M + off) + c8;
    fvec4* Vr = reinterpret_cast<fvec4*>(V + off) + c8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      W[8 * i] = w[b][i] + 1e-7f;
      __builtin_nontemporal_store(m[b][i] * 0.9f, Mr + 8 * i);
      __builtin_nontemporal_store(v[b][i] * 0.99f, Vr + 8 * i);
    }
  };
  ld(0, 0);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) ld(s + 1, (s + 1) & 1);
    st(s, s & 1);
  }
}

__global__ __launch_bounds__(256) void read3(const float* P, const float* M, const float* V, float* out) {
  const int r = blockIdx.y, k0 = blockIdx.x * ROWS, tid = threadIdx.x, rowl = tid >> 3, c8 = tid & 7;
  const int64_t off = (int64_t)r * STRIDE + OFF_W3 + (int64_t)(k0 + rowl) * HID;
  const fvec4* W = reinterpret_cast<const fvec4*>(P + off) + c8;
  const fvec4* Mr = reinterpret_cast<const fvec4*>(M + off) + c8;
  const fvec4* Vr = reinterpret_cast<const fvec4*>(V + off) + c8;
  fvec4 s = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) s += W[8 * i] + Mr[8 * i] + Vr[8 * i];
  if (s.x == 12345.0f) out[tid] = s.y + s.z + s.w;
}

__global__ __launch_bounds__(256) void copy1(const float* P, float* Q) {
  const int r = blockIdx.y, k0 = blockIdx.x * ROWS, tid = threadIdx.x, rowl = tid >> 3, c8 = tid & 7;
  const int64_t off = (int64_t)r * STRIDE + OFF_W3 + (int64_t)(k0 + rowl) * HID;
  const fvec4* W = reinterpret_cast<const fvec4*>(P + off) + c8;
  fvec4* D = reinterpret_cast<fvec4*>(Q + off) + c8;
  fvec4 w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = W[8 * i];
#pragma unroll
  for (int i = 0; i < 4; ++i) D[8 * i] = w[i];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 2048;
  const size_t n = (size_t)R * STRIDE;
  float *P, *M, *V, *out;
  CK(hipMalloc(&P, n * 4));
  CK(hipMalloc(&M, n * 4));
  CK(hipMalloc(&V, n * 4));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(P, 0, n * 4));
  CK(hipMemset(M, 0, n * 4));
  CK(hipMemset(V, 0, n * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const dim3 grid(FEAT / ROWS, R);
  const double slice = (double)R * FEAT * HID * 4;  // bytes of one stream
  const int reps = 10;
  const char* names[] = {"rmw3_nt", "rmw3_plain", "read3", "copy1", "rmw3_allnt", "rmw3_pipe2", "rmw3_pipe4"};
  for (int variant = 0; variant < 7; ++variant) {
    for (int rep = 0; rep < 2; ++rep) {  // first pass warms
      CK(hipEventRecord(a));
      for (int i = 0; i < reps; ++i) {
        if (variant == 0) rmw3<true><<<grid, 256>>>(P, M, V);
        if (variant == 1) rmw3<false><<<grid, 256>>>(P, M, V);
        if (variant == 2) read3<<<grid, 256>>>(P, M, V, out);
        if (variant == 3) copy1<<<grid, 256>>>(P, M);
        if (variant == 4) rmw3_allnt<<<grid, 256>>>(P, M, V);
        if (variant == 5) rmw3_pipe<2><<<dim3(FEAT / ROWS / 2, R), 256>>>(P, M, V);
        if (variant == 6) rmw3_pipe<4><<<dim3(FEAT / ROWS / 4, R), 256>>>(P, M, V);
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const double bytes = slice * (variant == 2 ? 3 : variant == 3 ? 2 : 6);
      if (rep == 1)
        printf("%-12s R=%d  %.3f ms/launch  %.2f TB/s\n",
               names[variant], R,
               ms / reps, bytes / (ms / reps * 1e-3) / 1e12);
    }
  }
  return 0;
}
