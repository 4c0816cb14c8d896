// ppgat_dist.hip -- cross-rank merge of the replicated item rows (dist.py, replicated-item
// partition).  Each rank's fused forward (ppgat_fwd) leaves, for every item destination,
// the softmax state of the in-edges it holds (those of its own users): max m_r, sum l_r
// (as 1/(l_r + eps)) and the normalised aggregate a_r.  The exact merged row is the
// log-sum-exp combination the single-GPU kernel forms over all in-edges:
//   m = max_r m_r,  c_r = l_r exp(m_r - m),  L = sum_r c_r,  a = sum_r c_r a_r / (L + eps)
//   out = mean_h a + bias,  1/l = 1 / (L + eps)
// with the two sums taken by all_reduce(MAX) of m' and all_reduce(SUM) of [c a | c].
// Elementwise over [n_items, heads, C]: HBM-bound, one float4 per thread.
//
// Halo exchange of the row-sharded partition (dist.py ExchangePlan): the send buffer of an
// all_to_all_single is packed from the rank's own rows (k_rows_gather), and the gradients
// the peers return for those rows are added back in a fixed order (k_rows_return_add):
// row o gets its returned copies in peer order, so the sum is deterministic.  Both are
// row copies of `cols` floats (16-B vectors when aligned), HBM-bound.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ppgat_internal.h"

namespace ppgat {
namespace {

__device__ __forceinline__ bool live_row(const int32_t* rowptr, int64_t i) { return rowptr[i + 1] > rowptr[i]; }

// phase 0: mx = live ? m : -inf
__global__ void __launch_bounds__(256) k_rep_max(const float* __restrict__ m, const int32_t* __restrict__ rowptr,
                                                 int64_t n, int heads, float* __restrict__ mx) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * heads) return;
  mx[t] = live_row(rowptr, t / heads) ? m[t] : -INFINITY;
}

// phase 1: pack_a[i, h, :] = c a_r,  pack_c[i, h] = c  (after all_reduce MAX of mx).
// One thread per float4 of the [n * heads, C] pack: consecutive threads, consecutive
// 16-B columns (C/4 threads per (row, head)).
__global__ void __launch_bounds__(256) k_rep_pack(const float* __restrict__ out, const float* __restrict__ agg,
                                                  const float* __restrict__ bias, const float* __restrict__ m,
                                                  const float* __restrict__ invl, const int32_t* __restrict__ rowptr,
                                                  const float* __restrict__ mx, int64_t n, int heads, int C, float eps,
                                                  float* __restrict__ pack_a, float* __restrict__ pack_c) {
  const int Q = C / 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * heads * Q) return;
  const int64_t w = t / Q;  // (row, head)
  const int q = (int)(t % Q);
  const int64_t i = w / heads;
  float c = 0.f;
  if (live_row(rowptr, i)) c = (1.f / invl[w] - eps) * expf(m[w] - mx[w]);
  float4 v = agg != nullptr ? reinterpret_cast<const float4*>(agg + w * C)[q]
                            : reinterpret_cast<const float4*>(out + i * C)[q];
  if (agg == nullptr && bias != nullptr) {
    const float4 b = reinterpret_cast<const float4*>(bias)[q];
    v.x -= b.x; v.y -= b.y; v.z -= b.z; v.w -= b.w;
  }
  v.x *= c; v.y *= c; v.z *= c; v.w *= c;
  reinterpret_cast<float4*>(pack_a + w * C)[q] = v;
  if (q == 0) pack_c[w] = c;
}

// phase 2 (after all_reduce SUM of the pack): the merged rows; one thread per float4 of
// the [n, C] output, looping over the heads
__global__ void __launch_bounds__(256) k_rep_finish(const float* __restrict__ pack_a, const float* __restrict__ pack_c,
                                                    const float* __restrict__ mx, const float* __restrict__ bias,
                                                    int64_t n, int heads, int C, float eps, float* __restrict__ out,
                                                    float* __restrict__ m, float* __restrict__ invl,
                                                    float* __restrict__ agg) {
  const int Q = C / 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n * Q) return;
  const int64_t i = t / Q;
  const int q = (int)(t % Q);
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int hd = 0; hd < heads; ++hd) {
    const int64_t w = i * heads + hd;
    const float L = pack_c[w];
    const float r = 1.f / (L + eps);
    float4 v = reinterpret_cast<const float4*>(pack_a + w * C)[q];
    v.x *= r; v.y *= r; v.z *= r; v.w *= r;
    if (agg != nullptr) reinterpret_cast<float4*>(agg + w * C)[q] = v;
    o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
    if (q == 0) {
      invl[w] = r;
      m[w] = L > 0.f ? mx[w] : 0.f;
    }
  }
  if (heads > 1) {
    const float inv_h = 1.f / (float)heads;
    o.x *= inv_h; o.y *= inv_h; o.z *= inv_h; o.w *= inv_h;
  }
  if (bias != nullptr) {
    const float4 b = reinterpret_cast<const float4*>(bias)[q];
    o.x += b.x; o.y += b.y; o.z += b.z; o.w += b.w;
  }
  reinterpret_cast<float4*>(out + i * C)[q] = o;
}

// dst[r, :] = src[idx[r], :]; one 64-lane wave per row, float4 per lane when cols % 4 == 0
__global__ void __launch_bounds__(256) k_rows_gather(const float* __restrict__ src, int64_t lds,
                                                     const int64_t* __restrict__ idx, int64_t n, int cols,
                                                     float* __restrict__ dst, int64_t ldd, int vec) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = threadIdx.x & 63;
  const float* s = src + idx[r] * lds;
  float* d = dst + r * ldd;
  if (vec) {
    for (int c = lane * 4; c < cols; c += 256)
      *reinterpret_cast<float4*>(d + c) = *reinterpret_cast<const float4*>(s + c);
  } else {
    for (int c = lane; c < cols; c += 64) d[c] = s[c];
  }
}

// dst[o, :] += sum_{k in [ptr[o], ptr[o+1])} ret[pos[k], :], k ascending (peer order)
__global__ void __launch_bounds__(256) k_rows_return_add(float* __restrict__ dst, int64_t ldd,
                                                         const float* __restrict__ ret, int64_t ldr,
                                                         const int32_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ pos, int64_t n, int cols,
                                                         int vec) {
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= n) return;
  const int k0 = ptr[o], k1 = ptr[o + 1];
  if (k0 == k1) return;
  const int lane = threadIdx.x & 63;
  float* d = dst + o * ldd;
  if (vec) {
    // the copies' loads eight at a time, all in flight before the first add (one row gets at
    // most world - 1 copies); the adds in k order as before (bitwise the same sums)
    for (int c = lane * 4; c < cols; c += 256) {
      float4 a = *reinterpret_cast<const float4*>(d + c);
      for (int kb = k0; kb < k1; kb += 8) {
        float4 b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (kb + j < k1) b[j] = *reinterpret_cast<const float4*>(ret + (int64_t)pos[kb + j] * ldr + c);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (kb + j < k1) {
            a.x += b[j].x; a.y += b[j].y; a.z += b[j].z; a.w += b[j].w;
          }
      }
      *reinterpret_cast<float4*>(d + c) = a;
    }
  } else {
    for (int c = lane; c < cols; c += 64) {
      float a = d[c];
      for (int k = k0; k < k1; ++k) a += ret[(int64_t)pos[k] * ldr + c];
      d[c] = a;
    }
  }
}

// narrow rows (cols <= 16, 16-B aligned): L = cols / 4 lanes per row (rounded up to a power of
// two), 64 / L rows per wave -- the halo layer's nstate rows (4 H floats) and partial sums (H)
template <int L>
__global__ void __launch_bounds__(256) k_rows_gather_narrow(const float* __restrict__ src, int64_t lds,
                                                            const int64_t* __restrict__ idx, int64_t n, int cols,
                                                            float* __restrict__ dst, int64_t ldd) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = t / L;
  const int c = 4 * (int)(t % L);
  if (r >= n || c >= cols) return;
  *reinterpret_cast<float4*>(dst + r * ldd + c) = *reinterpret_cast<const float4*>(src + idx[r] * lds + c);
}

// one thread per row, the row's float4 columns in a loop; copies added in k order
__global__ void __launch_bounds__(256) k_rows_return_add_narrow(float* __restrict__ dst, int64_t ldd,
                                                                const float* __restrict__ ret, int64_t ldr,
                                                                const int32_t* __restrict__ ptr,
                                                                const int32_t* __restrict__ pos, int64_t n,
                                                                int cols) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= n) return;
  const int k0 = ptr[o], k1 = ptr[o + 1];
  if (k0 == k1) return;
  float* d = dst + o * ldd;
  for (int c = 0; c < cols; c += 4) {
    float4 a = *reinterpret_cast<const float4*>(d + c);
    for (int k = k0; k < k1; ++k) {
      const float4 b = *reinterpret_cast<const float4*>(ret + (int64_t)pos[k] * ldr + c);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *reinterpret_cast<float4*>(d + c) = a;
  }
}

}  // namespace

static bool vec_ok(const void* a, int64_t lda, const void* b, int64_t ldb, int cols) {
  return cols % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && (reinterpret_cast<uintptr_t>(a) % 16) == 0 &&
         (reinterpret_cast<uintptr_t>(b) % 16) == 0;
}

hipError_t rows_gather(const float* src, int64_t lds, const int64_t* idx, int64_t n, int cols, float* dst,
                       int64_t ldd, hipStream_t st) {
  if (n <= 0 || cols <= 0) return hipSuccess;
  if (cols <= 16 && vec_ok(src, lds, dst, ldd, cols)) {  // narrow rows: several rows per wave
    const int L = cols <= 4 ? 1 : cols <= 8 ? 2 : 4;
    const unsigned g = (unsigned)((n * L + 255) / 256);
    if (L == 1) hipLaunchKernelGGL(k_rows_gather_narrow<1>, dim3(g), dim3(256), 0, st, src, lds, idx, n, cols, dst, ldd);
    else if (L == 2) hipLaunchKernelGGL(k_rows_gather_narrow<2>, dim3(g), dim3(256), 0, st, src, lds, idx, n, cols, dst, ldd);
    else hipLaunchKernelGGL(k_rows_gather_narrow<4>, dim3(g), dim3(256), 0, st, src, lds, idx, n, cols, dst, ldd);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_rows_gather, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, src, lds, idx, n, cols, dst, ldd,
                     vec_ok(src, lds, dst, ldd, cols) ? 1 : 0);
  return hipGetLastError();
}

hipError_t rows_return_add(float* dst, int64_t ldd, const float* ret, int64_t ldr, const int32_t* ptr,
                           const int32_t* pos, int64_t n, int cols, hipStream_t st) {
  if (n <= 0 || cols <= 0) return hipSuccess;
  if (cols <= 16 && vec_ok(dst, ldd, ret, ldr, cols)) {  // narrow rows: one thread per row
    hipLaunchKernelGGL(k_rows_return_add_narrow, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, dst, ldd, ret,
                       ldr, ptr, pos, n, cols);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_rows_return_add, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, dst, ldd, ret, ldr, ptr, pos,
                     n, cols, vec_ok(dst, ldd, ret, ldr, cols) ? 1 : 0);
  return hipGetLastError();
}

hipError_t rep_merge(int phase, const int32_t* rowptr, int64_t n, int heads, int C, float eps, float* out, float* agg,
                     const float* bias, float* m, float* invl, float* mx, float* pack_a, float* pack_c,
                     hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t rows = n * heads;
  if (phase == 0) {
    hipLaunchKernelGGL(k_rep_max, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, m, rowptr, n, heads, mx);
  } else if (phase == 1) {
    const int64_t th = rows * (C / 4);
    hipLaunchKernelGGL(k_rep_pack, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, out, agg, bias, m, invl,
                       rowptr, mx, n, heads, C, eps, pack_a, pack_c);
  } else {
    const int64_t th = n * (C / 4);
    hipLaunchKernelGGL(k_rep_finish, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, pack_a, pack_c, mx, bias,
                       n, heads, C, eps, out, m, invl, agg);
  }
  return hipGetLastError();
}

}  // namespace ppgat
