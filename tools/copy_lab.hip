// copy_lab: float4 streaming-copy variants on a 1 GiB buffer (read + write bytes / time), to
// pick the form of ppgat_stream_copy (bench.py's achievable-HBM yardstick).
//   hipcc --offload-arch=gfx950 -O3 -o tools/copy_lab tools/copy_lab.hip && tools/copy_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));

// U float4 per thread, consecutive lanes on consecutive 16 B, one pass (grid covers the buffer)
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_pass(const f4v* __restrict__ s, f4v* __restrict__ d, long n4) {
  const long base = (long)blockIdx.x * 256 * U + threadIdx.x;
  f4v v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + 256L * u;
    if (i < n4) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + 256L * u;
    if (i < n4) {
      if (NT) __builtin_nontemporal_store(v[u], d + i);
      else d[i] = v[u];
    }
  }
}

// grid-stride: a fixed grid of B blocks per CU, U float4 in flight per thread per iteration
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_stride(const f4v* __restrict__ s, f4v* __restrict__ d, long n4) {
  const long step = (long)gridDim.x * 256 * U;
  for (long base = (long)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += step) {
    f4v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      if (i < n4) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + 256L * u;
      if (i < n4) {
        if (NT) __builtin_nontemporal_store(v[u], d + i);
        else d[i] = v[u];
      }
    }
  }
}

template <typename F>
static double time_gbs(F launch, size_t bytes) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  const int reps = 20;
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return 2.0 * bytes * reps / (ms / 1e3) / 1e9;
}

int main() {
  const size_t bytes = 1ull << 30;
  const long n4 = bytes / 16;
  f4v *s, *d;
  if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipMemset(s, 0, bytes);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
#define PASS(U, NT)                                                                                        \
  printf("pass   U=%d nt=%d: %7.1f GB/s\n", U, NT, time_gbs([&] {                                        \
           hipLaunchKernelGGL((k_pass<U, NT>), dim3((unsigned)((n4 + 256L * U - 1) / (256L * U))), dim3(256), \
                              0, 0, s, d, n4);                                                              \
         }, bytes))
#define STRIDE(U, NT, B)                                                                                   \
  printf("stride U=%d nt=%d blocks/CU=%d: %7.1f GB/s\n", U, NT, B, time_gbs([&] {                          \
           hipLaunchKernelGGL((k_stride<U, NT>), dim3((unsigned)(cus * B)), dim3(256), 0, 0, s, d, n4);     \
         }, bytes))
  PASS(1, false); PASS(2, false); PASS(4, false); PASS(8, false);
  PASS(1, true); PASS(2, true); PASS(4, true); PASS(8, true);
  STRIDE(4, false, 4); STRIDE(4, false, 8); STRIDE(4, true, 8); STRIDE(8, true, 4); STRIDE(2, true, 16);
  hipFree(s);
  hipFree(d);
  return 0;
}
