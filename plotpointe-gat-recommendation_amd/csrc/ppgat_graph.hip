// ppgat_graph.hip -- COO edge_index (int64 [2,E]) -> CSR-by-dst + CSC-by-src on the device.
//
// The reference feeds the unsorted COO edge_index straight to PyG propagate / index_add_
// (scripts/train_gat_pyg.py:139-147,293; train_gat_custom.py:86-92).  Here the graph is
// static for the whole run, so it is sorted once (LSD radix sort = stable, so in-segment
// order is the original column order and every later sum has a fixed order) and cached
// by the caller.  The only host sync the library ever needs is the caller's one-time read
// of `bad` (out-of-range index count).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>

#include "ppgat_internal.h"

namespace ppgat {

static inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

static unsigned key_bits(int64_t n) {
  unsigned b = 1;
  while (b < 31 && ((int64_t)1 << b) < n) ++b;
  return b;
}

__global__ void k_keys(const int64_t* __restrict__ ei, int64_t E, int64_t N, int which, int32_t* __restrict__ key,
                       int32_t* __restrict__ iota, int32_t* __restrict__ bad) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= E) return;
  int64_t v = ei[which * E + k];
  if (bad != nullptr) {
    const int64_t o = ei[(1 - which) * E + k];
    const int nb = (v < 0 || v >= N) + (o < 0 || o >= N);
    if (nb) atomicAdd(bad, nb);  // integer count: order-independent
  }
  if (v < 0 || v >= N) v = 0;
  key[k] = (int32_t)v;
  iota[k] = (int32_t)k;
}

// ptr[r] = first sorted slot whose key >= r, for r in [0, N]
__global__ void k_ptr(const int32_t* __restrict__ skey, int64_t E, int64_t N, int32_t* __restrict__ ptr) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > E) return;
  if (k < E) {
    const int64_t d = skey[k];
    const int64_t prev = k == 0 ? -1 : skey[k - 1];
    for (int64_t r = prev + 1; r <= d; ++r) ptr[r] = (int32_t)k;
  } else {
    const int64_t last = E == 0 ? -1 : skey[E - 1];
    for (int64_t r = last + 1; r <= N; ++r) ptr[r] = (int32_t)E;
  }
}

__global__ void k_csr_cols(const int64_t* __restrict__ ei, int64_t E, int64_t N, const int32_t* __restrict__ eid,
                           int32_t* __restrict__ col, int32_t* __restrict__ pos) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= E) return;
  const int32_t e = eid[k];
  int64_t s = ei[e];
  if (s < 0 || s >= N) s = 0;
  col[k] = (int32_t)s;
  pos[e] = (int32_t)k;
}

__global__ void k_csc_rows(const int64_t* __restrict__ ei, int64_t E, int64_t N, const int32_t* __restrict__ eid,
                           const int32_t* __restrict__ pos, int32_t* __restrict__ row, int32_t* __restrict__ c2r) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= E) return;
  const int32_t e = eid[k];
  int64_t d = ei[E + e];
  if (d < 0 || d >= N) d = 0;
  row[k] = (int32_t)d;
  c2r[k] = pos[e];
}

static size_t sort_temp_bytes(int64_t N, int64_t E) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr,
                            (int32_t*)nullptr, (size_t)(E > 0 ? E : 1), 0u, key_bits(N));
  return bytes;
}

size_t csr_workspace_bytes(int64_t N, int64_t E) {
  const size_t e4 = align_up((size_t)(E > 0 ? E : 1) * 4);
  return 4 * e4 + align_up(sort_temp_bytes(N, E));
}

hipError_t csr_build(const int64_t* ei, int64_t E, int64_t N, int32_t* rowptr, int32_t* col, int32_t* csr_eid,
                     int32_t* colptr, int32_t* row, int32_t* csc_eid, int32_t* csc2csr, int32_t* bad, void* ws,
                     size_t ws_bytes, hipStream_t st) {
  if (ws_bytes < csr_workspace_bytes(N, E)) return hipErrorInvalidValue;
  const size_t e4 = align_up((size_t)(E > 0 ? E : 1) * 4);
  char* p = static_cast<char*>(ws);
  int32_t* key_in = reinterpret_cast<int32_t*>(p);
  int32_t* key_out = reinterpret_cast<int32_t*>(p + e4);
  int32_t* iota = reinterpret_cast<int32_t*>(p + 2 * e4);
  int32_t* pos = reinterpret_cast<int32_t*>(p + 3 * e4);
  void* tmp = p + 4 * e4;
  size_t tmp_bytes = ws_bytes - 4 * e4;
  const unsigned bits = key_bits(N);
  hipError_t err = hipMemsetAsync(bad, 0, sizeof(int32_t), st);
  if (err != hipSuccess) return err;
  const unsigned gE = (unsigned)((E + 255) / 256 > 0 ? (E + 255) / 256 : 1);
  const unsigned gE1 = (unsigned)((E + 1 + 255) / 256);
  // CSR by destination
  if (E > 0) {
    hipLaunchKernelGGL(k_keys, dim3(gE), dim3(256), 0, st, ei, E, N, 1, key_in, iota, bad);
    err = rocprim::radix_sort_pairs(tmp, tmp_bytes, key_in, key_out, iota, csr_eid, (size_t)E, 0u, bits, st);
    if (err != hipSuccess) return err;
  }
  hipLaunchKernelGGL(k_ptr, dim3(gE1), dim3(256), 0, st, key_out, E, N, rowptr);
  if (E > 0) hipLaunchKernelGGL(k_csr_cols, dim3(gE), dim3(256), 0, st, ei, E, N, csr_eid, col, pos);
  // CSC by source
  if (E > 0) {
    hipLaunchKernelGGL(k_keys, dim3(gE), dim3(256), 0, st, ei, E, N, 0, key_in, iota, (int32_t*)nullptr);
    err = rocprim::radix_sort_pairs(tmp, tmp_bytes, key_in, key_out, iota, csc_eid, (size_t)E, 0u, bits, st);
    if (err != hipSuccess) return err;
  }
  hipLaunchKernelGGL(k_ptr, dim3(gE1), dim3(256), 0, st, key_out, E, N, colptr);
  if (E > 0) hipLaunchKernelGGL(k_csc_rows, dim3(gE), dim3(256), 0, st, ei, E, N, csc_eid, pos, row, csc2csr);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Work schedule for the fused edge kernels (see ppgat_kernels.hip "Work items"):
// rows with deg > T become ceil(deg/T) hub pieces, listed first (hubs in row order);
// the other rows follow in descending degree (stable).
// counts = {n_hubs, n_hub_items, n_items, non-hub rows with more than kShortItemEdges edges}.
// ---------------------------------------------------------------------------
int64_t schedule_capacity(int64_t N, int64_t E, int32_t T) { return N + (E + T - 1) / T + 1; }

__global__ void k_sched_keys(const int32_t* __restrict__ ptr, int64_t N, int32_t T, int32_t* __restrict__ key,
                             int32_t* __restrict__ iota, int32_t* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t deg = i < N ? ptr[i + 1] - ptr[i] : 0;
  const bool hub = i < N && deg > T;
  const bool lng = i < N && !hub && deg > kShortItemEdges;
  if (i < N) {
    key[i] = hub ? 0 : (T + 1 - deg);
    iota[i] = (int32_t)i;
  }
  // one atomic per wave and counter (tens of thousands of rows count as long)
  const uint64_t bh = __ballot(hub), bl = __ballot(lng);
  if ((threadIdx.x & 63) == 0) {
    if (bh) atomicAdd(&counts[0], (int32_t)__popcll(bh));
    if (bl) atomicAdd(&counts[3], (int32_t)__popcll(bl));
  }
}

__global__ void k_sched_np(const int32_t* __restrict__ order, const int32_t* __restrict__ ptr, int64_t N, int32_t T,
                           int32_t* __restrict__ np) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= N) return;
  const int32_t r = order[s];
  const int32_t deg = ptr[r + 1] - ptr[r];
  np[s] = deg > T ? (deg + T - 1) / T : 1;
}

__global__ void k_sched_fill(const int32_t* __restrict__ order, const int32_t* __restrict__ ptr, int64_t N,
                             int32_t T, const int32_t* __restrict__ offs, const int32_t* __restrict__ np,
                             int32_t* __restrict__ item_row, int32_t* __restrict__ item_beg,
                             int32_t* __restrict__ item_end, int32_t* __restrict__ hub_row,
                             int32_t* __restrict__ hub_ptr, int32_t* __restrict__ counts) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= N) return;
  const int32_t r = order[s];
  const int32_t d0 = ptr[r], d1 = ptr[r + 1];
  const int32_t base = offs[s], n = np[s];
  for (int32_t q = 0; q < n; ++q) {
    item_row[base + q] = r;
    item_beg[base + q] = d0 + q * T;
    item_end[base + q] = min(d0 + (q + 1) * T, d1);
  }
  const bool hub = d1 - d0 > T;
  bool next_hub = false;
  if (s + 1 < N) {
    const int32_t r2 = order[s + 1];
    next_hub = ptr[r2 + 1] - ptr[r2] > T;
  }
  if (hub) {
    hub_row[s] = r;
    hub_ptr[s] = base;
    if (!next_hub) {
      hub_ptr[s + 1] = base + n;
      counts[1] = base + n;
    }
  } else if (s == 0) {
    hub_ptr[0] = 0;
    counts[1] = 0;
  }
  if (s == N - 1) counts[2] = base + n;
}

static size_t sched_temp_bytes(int64_t N, int32_t T) {
  size_t a = 0, b = 0;
  const size_t n = (size_t)(N > 0 ? N : 1);
  (void)rocprim::radix_sort_pairs(nullptr, a, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr,
                                  (int32_t*)nullptr, n, 0u, key_bits((int64_t)T + 2));
  (void)rocprim::exclusive_scan(nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr, (int32_t)0, n,
                                rocprim::plus<int32_t>());
  return a > b ? a : b;
}

size_t schedule_workspace_bytes(int64_t N) {
  const size_t n4 = align_up((size_t)(N > 0 ? N : 1) * 4);
  // temp size depends on T only through key_bits; use the widest key we allow (T < 2^20)
  return 5 * n4 + align_up(sched_temp_bytes(N, (1 << 20) - 2));
}

hipError_t schedule_build(const int32_t* ptr, int64_t N, int32_t T, int32_t* item_row, int32_t* item_beg,
                          int32_t* item_end, int32_t* hub_row, int32_t* hub_ptr, int32_t* counts, void* ws,
                          size_t ws_bytes, hipStream_t st) {
  if (T < 1 || T >= (1 << 20) - 2 || ws_bytes < schedule_workspace_bytes(N)) return hipErrorInvalidValue;
  hipError_t err = hipMemsetAsync(counts, 0, 4 * sizeof(int32_t), st);
  if (err != hipSuccess) return err;
  err = hipMemsetAsync(hub_ptr, 0, sizeof(int32_t), st);
  if (err != hipSuccess) return err;
  if (N == 0) return hipSuccess;
  const size_t n4 = align_up((size_t)N * 4);
  char* p = static_cast<char*>(ws);
  int32_t* key = reinterpret_cast<int32_t*>(p);
  int32_t* key_out = reinterpret_cast<int32_t*>(p + n4);
  int32_t* iota = reinterpret_cast<int32_t*>(p + 2 * n4);
  int32_t* order = reinterpret_cast<int32_t*>(p + 3 * n4);
  int32_t* np = reinterpret_cast<int32_t*>(p + 4 * n4);
  int32_t* offs = key;  // key is dead after the sort
  void* tmp = p + 5 * n4;
  size_t tmp_bytes = ws_bytes - 5 * n4;
  const unsigned g = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(k_sched_keys, dim3(g), dim3(256), 0, st, ptr, N, T, key, iota, counts);
  err = rocprim::radix_sort_pairs(tmp, tmp_bytes, key, key_out, iota, order, (size_t)N, 0u, key_bits((int64_t)T + 2),
                                  st);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(k_sched_np, dim3(g), dim3(256), 0, st, order, ptr, N, T, np);
  tmp_bytes = ws_bytes - 5 * n4;
  err = rocprim::exclusive_scan(tmp, tmp_bytes, np, offs, (int32_t)0, (size_t)N, rocprim::plus<int32_t>(), st);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(k_sched_fill, dim3(g), dim3(256), 0, st, order, ptr, N, T, offs, np, item_row, item_beg,
                     item_end, hub_row, hub_ptr, counts);
  return hipGetLastError();
}

}  // namespace ppgat
