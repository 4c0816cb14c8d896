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

}  // namespace ppgat
