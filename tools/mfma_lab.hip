// Calibration of v_mfma_f32_32x32x2_f32 issue rates on gfx950 (one workgroup of 4 waves
// per CU, persistent): constant operands vs operands cycling through registers.
#include <hip/hip_runtime.h>
#include <stdio.h>
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int MODE>
__global__ void __launch_bounds__(256, 1) k_mfma(float* out, int iters, float a0, float b0) {
  f32x16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int q = 0; q < 16; ++q) acc[i][q] = 0.f;
  float bq[4][32];
  float x[32];
  for (int i = 0; i < 32; ++i) {
    x[i] = a0 + i * threadIdx.x;
    for (int n = 0; n < 4; ++n) bq[n][i] = b0 - i * n + threadIdx.x;
  }
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int u = 0; u < 32; ++u)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[0], bq[0][0], acc[n], 0, 0, 0);
    } else {
#pragma unroll
      for (int u = 0; u < 32; ++u)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[u], bq[n][u], acc[n], 0, 0, 0);
    }
    if (MODE == 2) {  // perturb x so the loop is not invariant
#pragma unroll
      for (int u = 0; u < 32; ++u) x[u] += 1.f;
    }
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int q = 0; q < 16; ++q) s += acc[i][q];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(int iters) {
  float* out;
  const int blocks = 256;
  (void)hipMalloc(&out, blocks * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_mfma<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.f, 2.f);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_mfma<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.f, 2.f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double flop = (double)blocks * 4 * iters * 32 * 4 * 32 * 32 * 2 * 2;
  printf("MODE=%d %.3f ms  %.1f TFLOP/s\n", MODE, ms, flop / ms / 1e9);
  (void)hipFree(out);
}

int main() {
  run<0>(100);
  run<1>(100);
  run<2>(100);
  return 0;
}
