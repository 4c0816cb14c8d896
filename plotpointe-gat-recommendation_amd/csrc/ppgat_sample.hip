// ppgat_sample.hip -- BPR triple sampler.
//
// Replaces the per-epoch Python loop of sample_bpr_epoch (scripts/train_gat_pyg.py:179-190):
//   u = random.choice(users with >= 1 train item)
//   i = random.choice(train_pos_idx[u])
//   j = random.randrange(n_items), redrawn while j in train_pos_idx[u]
// Same distribution, counter-based stream: every draw is a hash of (seed, triple index t,
// draw number), so triple t does not depend on how the S triples are cut into launches and
// the numpy restatement (oracle/sampler_oracle.py) reproduces the triples bit for bit.
// Membership of j is a binary search over the user's items sorted once per graph
// (bpr_sampler_prepare: rocPRIM segmented radix sort + the list of users with items).
// One thread per triple: a few dependent 4-8 B loads each (HBM latency bound, S = 200k
// triples is ~10 us); no reshaping into anything wider pays here.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "ppgat_internal.h"

namespace ppgat {
namespace {

constexpr int kMaxNegDraws = 1024;  // rejection cap: only a user holding ~all items reaches it

inline size_t align_up(size_t b) { return (b + 255) & ~size_t(255); }

// splitmix64 finaliser over (seed, t, k); the numpy restatement is oracle/sampler_oracle.py
__device__ __forceinline__ uint64_t draw64(uint64_t seed, uint64_t t, uint64_t k) {
  uint64_t z = seed + (t + 1) * 0x9E3779B97F4A7C15ull;
  z ^= (k + 1) * 0xD1B54A32D192ED03ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in [0, n): high word of the 128-bit product (bias < n / 2^64)
__device__ __forceinline__ int64_t below(uint64_t r, int64_t n) { return (int64_t)__umul64hi(r, (uint64_t)n); }

__device__ __forceinline__ bool member(const int32_t* __restrict__ items, int64_t lo, int64_t hi, int32_t v) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int32_t x = items[mid];
    if (x == v) return true;
    if (x < v) lo = mid + 1; else hi = mid;
  }
  return false;
}

__global__ void __launch_bounds__(256) k_has_items(const int64_t* __restrict__ ptr, int64_t n_users,
                                                   uint8_t* __restrict__ flag) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < n_users) flag[v] = ptr[v + 1] > ptr[v] ? 1 : 0;
}

__global__ void __launch_bounds__(256) k_bpr_sample(const int64_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ items,
                                                    const int32_t* __restrict__ eligible,
                                                    const int64_t* __restrict__ n_eligible, int64_t n_items,
                                                    int64_t S, uint64_t seed, int64_t t0, int64_t* __restrict__ u,
                                                    int64_t* __restrict__ i, int64_t* __restrict__ j,
                                                    int32_t* __restrict__ bad) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const uint64_t t = (uint64_t)(t0 + s);
  const int64_t ne = *n_eligible;
  if (ne <= 0 || n_items <= 0) {
    u[s] = 0; i[s] = 0; j[s] = 0;
    atomicOr(bad, 1);
    return;
  }
  const int64_t uu = eligible[below(draw64(seed, t, 0), ne)];
  const int64_t lo = ptr[uu], hi = ptr[uu + 1];
  const int64_t ii = items[lo + below(draw64(seed, t, 1), hi - lo)];
  int64_t jj = -1;
  for (int k = 0; k < kMaxNegDraws; ++k) {
    const int32_t c = (int32_t)below(draw64(seed, t, 2 + k), n_items);
    if (!member(items, lo, hi, c)) { jj = c; break; }
  }
  if (jj < 0) { jj = 0; atomicOr(bad, 2); }
  u[s] = uu; i[s] = ii; j[s] = jj;
}

// Sampled-evaluation candidates (eval_sampled, scripts/train_gat_pyg.py:157-167): row b holds
// the held-out positive, then n_neg negatives; negative k is the first draw d = 0, 1, ... of
// the stream (seed, t = b * n_neg + k, d) that is neither one of the user's train items nor
// the positive -- the reference's rule (np.random.randint(0, n_items) redrawn while in
// train_pos | {pos}), drawn independently per negative.  One thread per negative.
__global__ void __launch_bounds__(256) k_eval_sample(const int64_t* __restrict__ ptr,
                                                     const int32_t* __restrict__ items,
                                                     const int64_t* __restrict__ users,
                                                     const int64_t* __restrict__ pos, int64_t n_eval, int64_t n_neg,
                                                     int64_t n_items, uint64_t seed, int64_t* __restrict__ cands,
                                                     int32_t* __restrict__ bad) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_eval * (n_neg + 1)) return;
  const int64_t b = t / (n_neg + 1), k = t % (n_neg + 1);
  const int64_t p = pos[b];
  if (k == 0) {
    cands[t] = p;
    return;
  }
  const int64_t u = users[b];
  const int64_t lo = ptr[u], hi = ptr[u + 1];
  const uint64_t tt = (uint64_t)(b * n_neg + k - 1);
  int64_t c = -1;
  for (int d = 0; d < kMaxNegDraws; ++d) {
    const int32_t x = (int32_t)below(draw64(seed, tt, d), n_items);
    if (x != p && !member(items, lo, hi, x)) { c = x; break; }
  }
  if (c < 0) { c = 0; atomicOr(bad, 2); }
  cands[t] = c;
}

size_t sort_bytes(int64_t n_users, int64_t nnz) {
  size_t b = 0;
  (void)rocprim::segmented_radix_sort_keys(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr,
                                           (unsigned)(nnz > 0 ? nnz : 1), (unsigned)(n_users > 0 ? n_users : 1),
                                           (const int64_t*)nullptr, (const int64_t*)nullptr);
  return b;
}

size_t select_bytes(int64_t n_users) {
  size_t b = 0;
  (void)rocprim::select(nullptr, b, rocprim::counting_iterator<int32_t>(0), (const uint8_t*)nullptr,
                        (int32_t*)nullptr, (int64_t*)nullptr, (size_t)(n_users > 0 ? n_users : 1));
  return b;
}

}  // namespace

size_t bpr_sampler_workspace_bytes(int64_t n_users, int64_t nnz) {
  const size_t a = sort_bytes(n_users, nnz), b = select_bytes(n_users);
  return align_up((size_t)(n_users > 0 ? n_users : 1)) + align_up(a > b ? a : b);
}

hipError_t bpr_sampler_prepare(const int64_t* ptr, const int32_t* items, int64_t n_users, int64_t nnz,
                               int32_t* items_sorted, int32_t* eligible, int64_t* n_eligible, void* ws,
                               size_t ws_bytes, hipStream_t st) {
  if (ws_bytes < bpr_sampler_workspace_bytes(n_users, nnz)) return hipErrorInvalidValue;
  hipError_t err = hipMemsetAsync(n_eligible, 0, sizeof(int64_t), st);
  if (err != hipSuccess || n_users <= 0) return err;
  uint8_t* flag = static_cast<uint8_t*>(ws);
  void* tmp = static_cast<char*>(ws) + align_up((size_t)n_users);
  size_t tmp_bytes = ws_bytes - align_up((size_t)n_users);
  if (nnz > 0) {
    err = rocprim::segmented_radix_sort_keys(tmp, tmp_bytes, items, items_sorted, (unsigned)nnz, (unsigned)n_users,
                                             ptr, ptr + 1, 0u, 32u, st);
    if (err != hipSuccess) return err;
  }
  hipLaunchKernelGGL(k_has_items, dim3((unsigned)((n_users + 255) / 256)), dim3(256), 0, st, ptr, n_users, flag);
  tmp_bytes = ws_bytes - align_up((size_t)n_users);
  return rocprim::select(tmp, tmp_bytes, rocprim::counting_iterator<int32_t>(0), flag, eligible, n_eligible,
                         (size_t)n_users, st);
}

hipError_t bpr_sample(const int64_t* ptr, const int32_t* items_sorted, const int32_t* eligible,
                      const int64_t* n_eligible, int64_t n_items, int64_t S, uint64_t seed, int64_t t0, int64_t* u,
                      int64_t* i, int64_t* j, int32_t* bad, hipStream_t st) {
  hipError_t err = hipMemsetAsync(bad, 0, sizeof(int32_t), st);
  if (err != hipSuccess || S <= 0) return err;
  hipLaunchKernelGGL(k_bpr_sample, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, ptr, items_sorted, eligible,
                     n_eligible, n_items, S, seed, t0, u, i, j, bad);
  return hipGetLastError();
}

hipError_t eval_sample(const int64_t* ptr, const int32_t* items_sorted, const int64_t* users, const int64_t* pos,
                       int64_t n_eval, int64_t n_neg, int64_t n_items, uint64_t seed, int64_t* cands, int32_t* bad,
                       hipStream_t st) {
  hipError_t err = hipMemsetAsync(bad, 0, sizeof(int32_t), st);
  const int64_t th = n_eval * (n_neg + 1);
  if (err != hipSuccess || th <= 0) return err;
  hipLaunchKernelGGL(k_eval_sample, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, ptr, items_sorted, users, pos,
                     n_eval, n_neg, n_items, seed, cands, bad);
  return hipGetLastError();
}

}  // namespace ppgat
