// ppgat_debug.hip -- index-range validation (include/ppgat.h ppgat_check_index_range) and the
// checks a PPGAT_DEBUG build (make debug -> libppgat_debug.so) runs inside the entry points.
//
// Counting is deterministic and atomic-free: each workgroup reduces its slice to one count in
// a fixed order, one workgroup sums the per-block counts.  The counts live in a library-owned
// device array (no allocation); the check synchronises the stream to read the result, so it is
// a validation tool, not something to put inside a captured graph.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppgat_internal.h"

namespace ppgat {
namespace {

constexpr int kDbgBlocks = 1024;
__device__ long long g_dbg_counts[kDbgBlocks + 1];

template <typename T>
__global__ void __launch_bounds__(256) k_range_count(const T* __restrict__ p, int64_t n, int64_t lo, int64_t hi) {
  __shared__ long long red[256];
  long long c = 0;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int64_t v = (int64_t)p[t];
    c += (v < lo || v >= hi) ? 1 : 0;
  }
  red[threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) g_dbg_counts[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(64) k_count_sum(int blocks) {
  if (threadIdx.x != 0) return;
  long long s = 0;
  for (int b = 0; b < blocks; ++b) s += g_dbg_counts[b];
  g_dbg_counts[kDbgBlocks] = s;
}

}  // namespace

hipError_t count_out_of_range(const void* idx, int elem_bytes, int64_t n, int64_t lo, int64_t hi, int64_t* n_bad,
                              hipStream_t st) {
  *n_bad = 0;
  if (n <= 0) return hipSuccess;
  int blocks = (int)((n + 255) / 256);
  if (blocks > kDbgBlocks) blocks = kDbgBlocks;
  if (elem_bytes == 4)
    hipLaunchKernelGGL(k_range_count<int32_t>, dim3(blocks), dim3(256), 0, st, static_cast<const int32_t*>(idx), n, lo,
                       hi);
  else
    hipLaunchKernelGGL(k_range_count<int64_t>, dim3(blocks), dim3(256), 0, st, static_cast<const int64_t*>(idx), n, lo,
                       hi);
  hipLaunchKernelGGL(k_count_sum, dim3(1), dim3(64), 0, st, blocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  long long host = 0;
  void* sym = nullptr;
  e = hipGetSymbolAddress(&sym, HIP_SYMBOL(g_dbg_counts));
  if (e != hipSuccess) return e;
  e = hipMemcpyAsync(&host, static_cast<long long*>(sym) + kDbgBlocks, sizeof(host), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  *n_bad = (int64_t)host;
  return e;
}

}  // namespace ppgat
