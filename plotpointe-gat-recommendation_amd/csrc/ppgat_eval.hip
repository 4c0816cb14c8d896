// ppgat_eval.hip -- sampled ranking for evaluation (A9 consumer of the inference forward).
//
// Replaces the per-user Python loop of eval_sampled (scripts/train_gat_pyg.py:160-175):
//   scores = I[cand] @ U[u];  rank = #(scores > scores[0]) + 1     (strict '>', :171)
// one device pass for all users instead of ~192k GEMVs and 192k device->host syncs.
// One wave per user; the user row stays in registers; candidates are gathered by C/4-lane
// subgroups with 8 rows in flight per wave.
#include <hip/hip_runtime.h>
#include <math.h>
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

// ---------------------------------------------------------------------------
// Serving top-K (serving/runtime.py:56-76): user vector = mean of the history rows, scores =
// item_vecs @ user_vec, history masked to -1e9, top-k descending (ties: smaller index first,
// by ppgat_knn_topk's selection).  Batched over B users.
// ---------------------------------------------------------------------------
// U[b] = (sum of item_vecs[hist[k]] over the user's history, in order) / len  (numpy's
// float32 mean over axis 0: rows added one after another, then divided by the count)
template <int C>
__global__ void __launch_bounds__(256) k_user_mean(const float* __restrict__ iv, int64_t n_items,
                                                   const int64_t* __restrict__ hptr,
                                                   const int64_t* __restrict__ hist, int64_t B,
                                                   float* __restrict__ U) {
  constexpr int LPR = C / 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t b = t / LPR;
  if (b >= B) return;
  const int sl = (int)(t % LPR);
  const int64_t k0 = hptr[b], k1 = hptr[b + 1];
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t k = k0; k < k1; ++k) {
    const float4 v = ld4(iv + clampi(hist[k], n_items) * C + sl * 4);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float n = (float)(k1 - k0);
  *reinterpret_cast<float4*>(U + b * C + sl * 4) = make_float4(s.x / n, s.y / n, s.z / n, s.w / n);
}

// scores[b][i] = <iv[i], U[b]>: a C/4-lane subgroup per item, the users' rows in LDS
template <int C>
__global__ void __launch_bounds__(256) k_serve_scores(const float* __restrict__ iv, int64_t n_items,
                                                      const float* __restrict__ U, int B,
                                                      float* __restrict__ scores) {
  constexpr int LPR = C / 4, IPB = 256 / LPR;
  extern __shared__ float4 sU[];
  for (int e = threadIdx.x; e < B * LPR; e += 256) sU[e] = ld4(U + (int64_t)e * 4);
  __syncthreads();
  const int sg = threadIdx.x / LPR, sl = threadIdx.x % LPR;
  for (int64_t i0 = (int64_t)blockIdx.x * IPB; i0 < n_items; i0 += (int64_t)gridDim.x * IPB) {
    const int64_t i = i0 + sg;
    const float4 v = ld4(iv + (i < n_items ? i : n_items - 1) * C + sl * 4);
    for (int b = 0; b < B; ++b) {
      float d = dot4(v, sU[b * LPR + sl]);
#pragma unroll
      for (int off = LPR / 2; off > 0; off >>= 1) d += __shfl_xor(d, off);
      if (sl == 0 && i < n_items) scores[(int64_t)b * n_items + i] = d;
    }
  }
}

__global__ void __launch_bounds__(256) k_mask_history(const int64_t* __restrict__ hptr,
                                                      const int64_t* __restrict__ hist, int64_t B, int64_t n_items,
                                                      float* __restrict__ scores) {
  const int64_t b = blockIdx.y;
  const int64_t k = hptr[b] + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b < B && k < hptr[b + 1]) scores[b * n_items + clampi(hist[k], n_items)] = -1e9f;
}

}  // namespace

hipError_t serve_topk(const float* iv, int64_t n_items, int C, const int64_t* hptr, const int64_t* hist,
                      int64_t max_hist, int B, int k, float* U, float* scores, int32_t* out_idx, float* out_score,
                      hipStream_t st) {
  if (B <= 0) return hipSuccess;
  const int64_t th = (int64_t)B * (C / 4);
  const unsigned gm = (unsigned)((th + 255) / 256);
  const int64_t ipb = 256 / (C / 4);
  int64_t gs = (n_items + ipb - 1) / ipb;
  if (gs > 2048) gs = 2048;
  // the users' rows live in LDS: at most 64 KB per launch (256 users at C = 64, 64 at C = 256)
  const int ub = 65536 / (C * 4);
  for (int b0 = 0; b0 < B; b0 += ub) {
    const int nb = B - b0 < ub ? B - b0 : ub;
    const size_t lds = (size_t)nb * C * 4;
    const float* Ub = U + (int64_t)b0 * C;
    float* sb = scores + (int64_t)b0 * n_items;
    switch (C) {
      case 64:
        if (b0 == 0)
          hipLaunchKernelGGL(k_user_mean<64>, dim3(gm), dim3(256), 0, st, iv, n_items, hptr, hist, (int64_t)B, U);
        hipLaunchKernelGGL(k_serve_scores<64>, dim3((unsigned)gs), dim3(256), lds, st, iv, n_items, Ub, nb, sb);
        break;
      case 128:
        if (b0 == 0)
          hipLaunchKernelGGL(k_user_mean<128>, dim3(gm), dim3(256), 0, st, iv, n_items, hptr, hist, (int64_t)B, U);
        hipLaunchKernelGGL(k_serve_scores<128>, dim3((unsigned)gs), dim3(256), lds, st, iv, n_items, Ub, nb, sb);
        break;
      case 256:
        if (b0 == 0)
          hipLaunchKernelGGL(k_user_mean<256>, dim3(gm), dim3(256), 0, st, iv, n_items, hptr, hist, (int64_t)B, U);
        hipLaunchKernelGGL(k_serve_scores<256>, dim3((unsigned)gs), dim3(256), lds, st, iv, n_items, Ub, nb, sb);
        break;
      default:
        return hipErrorInvalidValue;
    }
  }
  if (max_hist > 0)
    hipLaunchKernelGGL(k_mask_history, dim3((unsigned)((max_hist + 255) / 256), (unsigned)B), dim3(256), 0, st, hptr,
                       hist, (int64_t)B, n_items, scores);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // selection: q0 = n_items puts "self" outside the columns; every score counts (min -inf)
  return knn_topk(scores, n_items, B, n_items, n_items, k, -INFINITY, out_idx, out_score, nullptr, st);
}

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
