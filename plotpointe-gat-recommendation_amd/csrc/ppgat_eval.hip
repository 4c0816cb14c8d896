// ppgat_eval.hip -- sampled ranking for evaluation (A9 consumer of the inference forward).
//
// Replaces the per-user Python loop of eval_sampled (scripts/train_gat_pyg.py:160-175):
//   scores = I[cand] @ U[u];  rank = #(scores > scores[0]) + 1     (strict '>', :171)
// one device pass for all users instead of ~192k GEMVs and 192k device->host syncs.
// One wave per user; the user row stays in registers; candidates are gathered by C/4-lane
// subgroups with 8 rows in flight per wave.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppgat_internal.h"

namespace ppgat {
namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}
__device__ __forceinline__ int64_t clampi(int64_t v, int64_t n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }
__device__ __forceinline__ int64_t zrow(const int32_t* m, int64_t v) { return m ? m[v] : v; }

template <int C>
__global__ void __launch_bounds__(256) k_sampled_rank(const float* __restrict__ Z, int64_t n_users, int64_t n_items,
                                                      const int32_t* __restrict__ row_map,
                                                      const int64_t* __restrict__ users,
                                                      const int64_t* __restrict__ cands, int64_t B, int64_t K1,
                                                      int32_t* __restrict__ rank) {
  constexpr int LPR = C / 4, EPW = 64 / LPR, U = EPW >= 8 ? 1 : 8 / EPW;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= B) return;
  const int sg = lane / LPR, sl = lane % LPR;
  const int64_t ur = zrow(row_map, clampi(users[b], n_users));
  const float4 uv = ld4(Z + ur * C + sl * 4);
  const int64_t* cb = cands + b * K1;
  float s0 = dot4(uv, ld4(Z + zrow(row_map, n_users + clampi(cb[0], n_items)) * C + sl * 4));
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) s0 += __shfl_xor(s0, off);
  int cnt = 0;
  for (int64_t q0 = 1; q0 < K1; q0 += EPW * U) {
    float s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = q0 + u * EPW + sg;
      s[u] = q < K1 ? dot4(uv, ld4(Z + zrow(row_map, n_users + clampi(cb[q], n_items)) * C + sl * 4)) : 0.f;
    }
#pragma unroll
    for (int off = LPR / 2; off > 0; off >>= 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) s[u] += __shfl_xor(s[u], off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = q0 + u * EPW + sg;
      if (sl == 0 && q < K1 && s[u] > s0) ++cnt;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (lane == 0) rank[b] = cnt + 1;
}

}  // namespace

hipError_t sampled_rank(const float* Z, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                        const int64_t* users, const int64_t* cands, int64_t B, int64_t K1, int32_t* rank,
                        hipStream_t st) {
  if (B == 0) return hipSuccess;
  const unsigned g = (unsigned)((B + 3) / 4);
  switch (C) {
    case 32: hipLaunchKernelGGL(k_sampled_rank<32>, dim3(g), dim3(256), 0, st, Z, n_users, n_items, row_map, users,
                                cands, B, K1, rank); break;
    case 64: hipLaunchKernelGGL(k_sampled_rank<64>, dim3(g), dim3(256), 0, st, Z, n_users, n_items, row_map, users,
                                cands, B, K1, rank); break;
    case 128: hipLaunchKernelGGL(k_sampled_rank<128>, dim3(g), dim3(256), 0, st, Z, n_users, n_items, row_map,
                                 users, cands, B, K1, rank); break;
    case 256: hipLaunchKernelGGL(k_sampled_rank<256>, dim3(g), dim3(256), 0, st, Z, n_users, n_items, row_map,
                                 users, cands, B, K1, rank); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace ppgat
