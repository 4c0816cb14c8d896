// Issue rate of v_mfma_f32_32x32x16_bf16 on gfx950 for the two accumulation orders a split-bf16
// x6 GEMM step can use: six dependent MFMAs into one accumulator, then the next accumulator
// (CHAIN), or the six products of two tiles interleaved (PAIR), or every product across 8
// accumulators (ROUND).  One persistent workgroup per CU, WAVES waves.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_chain_lab.hip -o /tmp/mfma_chain_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
using f32x16 = __attribute__((ext_vector_type(16))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

template <int MODE>
__global__ void __launch_bounds__(512, 1) k_lab(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) uint4 lds[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = make_uint4(i, i + 1, i + 2, i + 3);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  bf16x8 a[3], b[3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
    for (int j = 0; j < 8; ++j) {
      a[p][j] = (__bf16)(0.001f * (threadIdx.x + j + p));
      b[p][j] = (__bf16)(0.002f * (threadIdx.x - j + p));
    }
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc[t], 0, 0, 0);
      }
    } else if (MODE == 1) {
#pragma unroll
      for (int t = 0; t < 8; t += 2) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const int pa = q < 3 ? q : (q == 3 ? 1 : 0), pb = q < 3 ? 2 - q : (q == 3 ? 0 : 1);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa], b[pb], acc[t], 0, 0, 0);
          acc[t + 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa], b[pb], acc[t + 1], 0, 0, 0);
        }
      }
    } else if (MODE == 3 || MODE == 4) {
      // B fragments from LDS: MODE 3 reads three 16-B fragments per six MFMAs, MODE 4 per twelve
      bf16x8 f[2][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) f[0][p] = __builtin_bit_cast(bf16x8, lds[(lane + 64 * p + it) & 4095]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (MODE == 3 || (t & 1)) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            f[MODE == 3 ? (t + 1) & 1 : ((t >> 1) + 1) & 1][p] =
                __builtin_bit_cast(bf16x8, lds[(lane + 64 * (p + 3 * t) + it) & 4095]);
        }
        const int s = MODE == 3 ? (t & 1) : ((t >> 1) & 1);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], f[s][0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], f[s][2], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], f[s][1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], f[s][0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], f[s][1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], f[s][0], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const int pa = q < 3 ? q : (q == 3 ? 1 : 0), pb = q < 3 ? 2 - q : (q == 3 ? 0 : 1);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa], b[pb], acc[t], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t)
    for (int q = 0; q < 16; ++q) s += acc[t][q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, int waves, int iters) {
  float* out;
  int cus = 256;
  (void)hipMalloc(&out, cus * 512 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_lab<MODE>, dim3(cus), dim3(64 * waves), 0, 0, out, iters);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_lab<MODE>, dim3(cus), dim3(64 * waves), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 16 * 48.0 * iters * waves * cus;
  printf("{\"order\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.3f, \"bf16_tflops\": %.1f}\n", name, waves, ms,
         flops / ms / 1e9);
  (void)hipFree(out);
}

int main() {
  const int iters = 20000;
  for (int w : {4, 8}) {
    run<0>("chain6", w, iters);
    run<1>("pair", w, iters);
    run<2>("round8", w, iters);
    run<3>("lds_3per6", w, iters);
    run<4>("lds_3per12", w, iters);
  }
  return 0;
}
