// ppgat_knn.hip -- neighbour selection of the I-I kNN build (graphs/build_ii_knn.py:76-99),
// after the cosine-similarity block S = E_q E^T (library GEMM, the only dense part):
// per query row, the k largest similarities excluding the item itself, sorted descending
// (ties: smaller item index first), and how many of them reach min_similarity.
//
// One wave per row.  Each lane scans a strided slice of the row (coalesced 256-B loads,
// 4 in flight) keeping its own sorted top-k list in LDS ([slot][lane] so the 64 lanes hit
// 64 banks); an insertion happens only when a value beats the lane's current k-th, i.e.
// O(k log(n/64k)) times per lane.  The 64 lists are then merged by k rounds of a wave
// argmax (value desc, index asc).  No atomics: the result is deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "ppgat_internal.h"

namespace ppgat {

namespace {

template <int K>
__global__ void __launch_bounds__(256) k_knn_topk(const float* __restrict__ S, int64_t ld, int64_t rows,
                                                  int64_t n_cols, int64_t q0, int k, float min_sim,
                                                  int32_t* __restrict__ out_idx, float* __restrict__ out_sim,
                                                  int32_t* __restrict__ out_cnt) {
  __shared__ float lv[4][K][64];
  __shared__ int32_t li[4][K][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 4 + wv;
  if (r >= rows) return;  // whole wave
  for (int t = 0; t < k; ++t) {
    lv[wv][t][lane] = -INFINITY;
    li[wv][t][lane] = INT32_MAX;
  }
  float thr = -INFINITY;  // this lane's current k-th value
  const float* srow = S + r * ld;
  const int64_t self = q0 + r;
  for (int64_t j0 = 0; j0 < n_cols; j0 += 256) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = j0 + u * 64 + lane;
      v[u] = j < n_cols ? srow[j] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = j0 + u * 64 + lane;
      const float s = j == self ? -INFINITY : v[u];
      if (s > thr) {  // strict: an equal later value (larger index) does not displace
        int p = k - 1;
        while (p > 0 && lv[wv][p - 1][lane] < s) {
          lv[wv][p][lane] = lv[wv][p - 1][lane];
          li[wv][p][lane] = li[wv][p - 1][lane];
          --p;
        }
        lv[wv][p][lane] = s;
        li[wv][p][lane] = (int32_t)j;
        thr = lv[wv][k - 1][lane];
      }
    }
  }
  // merge the 64 sorted lists: k rounds of a wave argmax over the lanes' heads
  int h = 0;
  int cnt = 0;
  for (int t = 0; t < k; ++t) {
    float bv = h < k ? lv[wv][h][lane] : -INFINITY;
    int32_t bi = h < k ? li[wv][h][lane] : INT32_MAX;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float ov = __shfl_xor(bv, off);
      const int32_t oi = __shfl_xor(bi, off);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (h < k && li[wv][h][lane] == bi && lv[wv][h][lane] == bv) ++h;  // indices are unique per row
    if (lane == 0) {
      out_sim[r * k + t] = bv;
      out_idx[r * k + t] = bi == INT32_MAX ? -1 : bi;
    }
    cnt += bv >= min_sim ? 1 : 0;  // sorted descending: the kept entries are a prefix
  }
  if (lane == 0 && out_cnt != nullptr) out_cnt[r] = cnt;
}

}  // namespace

int knn_max_k() { return 64; }

hipError_t knn_topk(const float* S, int64_t ld, int64_t rows, int64_t n_cols, int64_t q0, int k, float min_sim,
                    int32_t* out_idx, float* out_sim, int32_t* out_cnt, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  if (k <= 8) hipLaunchKernelGGL(k_knn_topk<8>, grid, block, 0, st, S, ld, rows, n_cols, q0, k, min_sim, out_idx, out_sim, out_cnt);
  else if (k <= 16) hipLaunchKernelGGL(k_knn_topk<16>, grid, block, 0, st, S, ld, rows, n_cols, q0, k, min_sim, out_idx, out_sim, out_cnt);
  else if (k <= 32) hipLaunchKernelGGL(k_knn_topk<32>, grid, block, 0, st, S, ld, rows, n_cols, q0, k, min_sim, out_idx, out_sim, out_cnt);
  else hipLaunchKernelGGL(k_knn_topk<64>, grid, block, 0, st, S, ld, rows, n_cols, q0, k, min_sim, out_idx, out_sim, out_cnt);
  return hipGetLastError();
}

}  // namespace ppgat
