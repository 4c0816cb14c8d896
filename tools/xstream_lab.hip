// Lab (not product code): read bandwidth of the X-operand stream of the NN / FusionMLP GEMMs on
// gfx950 -- X [M x K] fp32, row-major, read by workgroups of 8 waves x 32 rows (256 rows), one
// workgroup per CU (LDS padded to 120 KB as the GEMMs hold), K in 32-deep chunks as the GEMM
// main loop consumes it.  Modes:
//   0  lane owns a row (the GEMMs' layout): per chunk 4 float4 per lane, 32 B of each of 32 rows
//      per instruction, D chunks in flight (register sets)
//   1  coalesced rows: 8 lanes per row, each instruction 8 whole 128-B row segments
//   2  contiguous sweep of the same bytes (each wave streams its 32 rows' memory in order, 1 KB
//      per instruction): the DRAM-friendly bound for this traffic
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xstream_lab.hip -o tools/xstream_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ float4 ld4c(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int MODE, int D>
__global__ void __launch_bounds__(512, 1) k_stream(const float* __restrict__ X, int64_t M, int K, float* out) {
  __shared__ float pad[30 * 1024];  // 120 KB: one workgroup per CU, as the GEMMs
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int64_t rb = blockIdx.x;
  const int chunks = K / 32;
  float s = 0.f;
  if (MODE == 0) {
    const int64_t m = rb * 256 + wv * 32 + r;
    const float* xrow = X + (m < M ? m : M - 1) * (int64_t)K + 4 * hf;
    float4 x[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int g = 0; g < 4; ++g) x[d][g] = ld4c(xrow + d * 32 + 8 * g);
    for (int c = 0; c < chunks; c += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int g = 0; g < 4; ++g) s += x[d][g].x + x[d][g].y + x[d][g].z + x[d][g].w;
        const int cn = c + d + D < chunks ? c + d + D : chunks - 1;
#pragma unroll
        for (int g = 0; g < 4; ++g) x[d][g] = ld4c(xrow + cn * 32 + 8 * g);
      }
    }
  } else if (MODE == 1) {
    const float* xr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = rb * 256 + wv * 32 + (lane >> 3) + 8 * j;
      xr[j] = X + (row < M ? row : M - 1) * (int64_t)K + 4 * (lane & 7);
    }
    float4 x[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int j = 0; j < 4; ++j) x[d][j] = ld4c(xr[j] + d * 32);
    for (int c = 0; c < chunks; c += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s += x[d][j].x + x[d][j].y + x[d][j].z + x[d][j].w;
        const int cn = c + d + D < chunks ? c + d + D : chunks - 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) x[d][j] = ld4c(xr[j] + cn * 32);
      }
    }
  } else {
    const int64_t r0 = rb * 256 + wv * 32;
    const int64_t r1 = r0 + 32 < M ? r0 + 32 : M;
    if (r1 > r0) {
      const float* base = X + r0 * (int64_t)K;
      const int64_t n4 = (r1 - r0) * (int64_t)K / 4;
      for (int64_t i = lane; i < n4; i += 64 * 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = (i + 64 * u < n4) ? ld4c(base + 4 * (i + 64 * u)) : float4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u].x + v[u].y + v[u].z + v[u].w;
      }
    }
  }
  if (s == 1.2345f) pad[tid] = s;  // keep the loads
  if (s == 1.2345f) out[tid] = pad[(tid * 7) & 1023];
}

template <int MODE, int D>
static float run(const float* X, int64_t M, int K, float* out, int iters) {
  const unsigned grid = (unsigned)((M + 255) / 256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_stream<MODE, D>), dim3(grid), dim3(512), 0, 0, X, M, K, out);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k_stream<MODE, D>), dim3(grid), dim3(512), 0, 0, X, M, K, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main() {
  const struct { int64_t M; int K; const char* what; } shapes[] = {
      {498196, 896, "fusion x (498k x 896)"}, {1875000, 1024, "cfg5 agg (1.9M x 1024)"}, {1875000, 256, "cfg5 x (1.9M x 256)"}};
  float* out;
  CHECK(hipMalloc(&out, 4096 * 4));
  for (const auto& sh : shapes) {
    float* X;
    const size_t bytes = (size_t)sh.M * sh.K * 4;
    CHECK(hipMalloc(&X, bytes));
    CHECK(hipMemset(X, 0, bytes));
    const double gb = bytes / 1e9;
    const float t0 = run<0, 2>(X, sh.M, sh.K, out, 10), t0d = run<0, 4>(X, sh.M, sh.K, out, 10);
    const float t1 = run<1, 2>(X, sh.M, sh.K, out, 10), t1d = run<1, 4>(X, sh.M, sh.K, out, 10);
    const float t2 = run<2, 1>(X, sh.M, sh.K, out, 10);
    printf("{\"shape\": \"%s\", \"GB\": %.3f, \"lane_row_D2\": [%.3f, %.0f], \"lane_row_D4\": [%.3f, %.0f], "
           "\"coalesced_D2\": [%.3f, %.0f], \"coalesced_D4\": [%.3f, %.0f], \"contiguous\": [%.3f, %.0f]}\n",
           sh.what, gb, t0, gb / t0 * 1e3, t0d, gb / t0d * 1e3, t1, gb / t1 * 1e3, t1d, gb / t1d * 1e3, t2,
           gb / t2 * 1e3);
    CHECK(hipFree(X));
  }
  return 0;
}
