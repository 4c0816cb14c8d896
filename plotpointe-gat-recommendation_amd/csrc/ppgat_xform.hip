// ppgat_xform.hip -- the multi-head GAT layer in the aggregate-then-transform formulation,
// and the fp32 matrix-core GEMMs it (and the row-sharded config-5 path) runs on (gfx950).
//
// GATConv(C_in, C, heads=H, concat=False) (scripts/train_gat_pyg.py:77)
// computes out_i = 1/H sum_h sum_{j->i} alpha_ij^h W_h x_j + bias with W_h = lin.weight rows
// [h C, (h+1) C).  The message is linear in x_j, so
//     out_i = 1/H sum_h W_h ax_i^h + bias,   ax_i^h = sum_{j->i} alpha_ij^h x_j   [H, C_in]
// and the attention logits only need s_src_j^h = x_j . A_src^h with A_src^h = W_h^T att_src^h
// (likewise s_dst).  With H*C > C_in (config 5: 4*256 = 1024 against 256) the edge pass
// gathers x_j (C_in floats) instead of h_j (H*C floats), h is never materialised, and a
// row-sharded rank exchanges x for its halo rows (dist.py).  Backward, with g = dOut:
//     gt_i^h = W_h^T g_i / H                  (GEMM [n, C] x [C, H C_in])
//     D_i^h  = gt_i^h . ax_i^h                (= sum_k beta dalpha, Appendix B)
//     per edge k = (j -> i): dz = alpha (d gt_i^h . x_j - D_i^h) lrelu'
//     dx_j   = sum_k sum_h beta_k^h gt_i^h + sum_h ds_src_j^h A_src^h + sum_h ds_dst_j^h A_dst^h
//     dW_h   = g^T ax^h / H + att_src^h (x) (ds_src^h)^T x + att_dst^h (x) (ds_dst^h)^T x
//     datt_src^h = W_h (ds_src^h)^T x, datt_dst^h likewise,  dbias = sum_i g_i.
// One edge pass by source (CSC) produces dx_msg, ds_src and the per-edge dz (at its CSR
// slot, summed per destination by k_dst_sum); no atomics anywhere, fixed summation orders.
//
// GEMMs (v_mfma_f32_32x32x2_f32, exact fp32 FMA chains; 157 TF peak):
//  * k_gemm_nn: Y = alpha X B (+ bias), X [M, K] row-major streamed from HBM straight into
//    the A-operand layout (float4 per lane = 4 MFMA steps, reduction index permuted),
//    B [K, N] (row-major) or [N, K] (X W^T) staged per 32-deep k chunk in LDS; each wave owns
//    32 rows x BN columns (NT 32x32 accumulator tiles), workgroups mapped XCD-aware so the
//    column blocks of one row block share an L2.
//  * k_gemm_tn: G = A^T B over M rows (weight gradients): 128 x 256 output tile per
//    workgroup, 32-row chunks staged in LDS, row splits summed in split order (deterministic);
//    the tiles of one row split run on one XCD, so the rows leave HBM once.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "ppgat_internal.h"
#include "ppgat_lanes.h"
#include "ppgat_split.h"
#include "ppgat_nnh_pipe.h"

namespace ppgat {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 fma4(float s, float4 v, float4 a) {
  return make_float4(fmaf(s, v.x, a.x), fmaf(s, v.y, a.y), fmaf(s, v.z, a.z), fmaf(s, v.w, a.w));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 mul4(float4 a, float s) { return make_float4(a.x * s, a.y * s, a.z * s, a.w * s); }
__device__ __forceinline__ float4 absmax4(float4 m, float4 v) {
  return make_float4(fmaxf(m.x, fabsf(v.x)), fmaxf(m.y, fabsf(v.y)), fmaxf(m.z, fabsf(v.z)), fmaxf(m.w, fabsf(v.w)));
}
// merge a lane's maxima of |v| for columns c0 .. c0 + 3 into bits (IEEE bits, ordered as unsigned
// for v >= 0): read first, atomic only where larger -- after the first waves almost never.  A max
// is order-free, so the result is deterministic.
__device__ __forceinline__ void colmax_merge4(unsigned* bits, int c0, float4 m) {
  const uint4 cur = *reinterpret_cast<const uint4*>(bits + c0);
  if (__float_as_uint(m.x) > cur.x) atomicMax(bits + c0, __float_as_uint(m.x));
  if (__float_as_uint(m.y) > cur.y) atomicMax(bits + c0 + 1, __float_as_uint(m.y));
  if (__float_as_uint(m.z) > cur.z) atomicMax(bits + c0 + 2, __float_as_uint(m.z));
  if (__float_as_uint(m.w) > cur.w) atomicMax(bits + c0 + 3, __float_as_uint(m.w));
}
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}
__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// logit / dropout rules shared with ppgat_kernels.hip (PyG mode only here)
__device__ __forceinline__ float lrelu(float z, float slope) { return z > 0.f ? z : z * slope; }
__device__ __forceinline__ float dlrelu(float z, float slope) { return z > 0.f ? 1.f : slope; }
__device__ __forceinline__ float drop_scale(uint64_t seed, uint32_t eid, uint32_t head, float p, float inv_keep) {
  uint64_t x = seed ^ ((uint64_t)eid * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)head * 0xC2B2AE3D27D4EB4Full);
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  const float u = (float)(x >> 40) * (1.0f / 16777216.0f);
  return u >= p ? inv_keep : 0.f;
}

// ===========================================================================
// NN GEMM: Y[M, N] = alpha X[M, K] B + bias
// ===========================================================================
constexpr int kGBM = 128;  // rows per workgroup (4 waves x 32)
constexpr int kGBK = 32;   // reduction chunk
constexpr int kNkLd = kGBK + 4;  // LDS row stride of the [n][k] image (NK mode): conflict-free b128 reads

struct NnArg {
  const float* X;
  int64_t ldx;
  int64_t M;
  int K;
  const float* B;
  int64_t ldb;
  int N;
  float alpha;
  const float* bias;
  float* Y;
  int64_t ldy;
  int n_blocks;
  int64_t row_blocks;
  int splits;     // > 1: split-K, raw partial tiles to part[split][M][N] (k_nn_split_sum finishes)
  int k_per;      // reduction length per split (multiple of kGBK)
  float* part;
  // optional rank update fused into k_gemm_nnh's epilogue: Y += rS[row][:nv] rA[:nv][col]
  // (v ascending, after alpha and bias -- the order of k_rank_update, so the same bits)
  const float* rS;
  int64_t ldrs;
  int nv;
  const float* rA;
  int64_t ldra;
};

// BMODE 0: B[k][n] = B[k * ldb + n] (image [k][n], b32 reads); 1: B[k][n] = B[n * ldb + k] (X W^T,
// image [n][k], b128 reads).  MFMA 32x32x2 lane maps (r = lane & 31, hf = lane >> 5): A operand
// X[row r][k], B operand B[k][col r], accumulator q at row (q & 3) + 8 (q >> 2) + 4 hf, col r;
// within a group of 8 k, lane half hf supplies k = 8g + 4 hf + s at MFMA step s.
template <int NT, int BMODE>
__global__ void __launch_bounds__(256, 2) k_gemm_nn(NnArg a) {
  constexpr int BN = 32 * NT;
  constexpr int IMG = BMODE == 0 ? kGBK * BN : BN * kNkLd;
  __shared__ float sB[IMG];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  // XCD-aware order: blocks b, b + 8, b + 16, ... land on one XCD; the n blocks of a row block
  // are consecutive there, so its X rows are fetched from HBM once
  const int64_t b = blockIdx.x;
  int64_t rb;
  int n0, split = 0;
  if (a.splits > 1) {  // small M: (row block, n block, k split), splits fastest
    split = (int)(b % a.splits);
    const int64_t rest = b / a.splits;
    n0 = (int)(rest % a.n_blocks) * BN;
    rb = rest / a.n_blocks;
  } else {
    const int64_t idx = b >> 3;
    rb = (idx / a.n_blocks) * 8 + (b & 7);
    n0 = (int)(idx % a.n_blocks) * BN;
  }
  if (rb >= a.row_blocks) return;
  const int64_t M = a.M;
  const int kbeg = split * a.k_per;
  const int K = a.splits > 1 ? (kbeg + a.k_per < a.K ? kbeg + a.k_per : a.K) : a.K;
  const int64_t m = rb * kGBM + wv * 32 + r;
  const float* xrow = a.X + (m < M ? m : M - 1) * a.ldx + 4 * hf;  // rows past M re-read row M-1 (never stored)

  float4 bst[NT];
  auto load_b = [&](int kc) {
#pragma unroll
    for (int s = 0; s < NT; ++s) {
      const int e = tid + 256 * s;
      if (BMODE == 0) {
        const int k = e / (BN / 4), n4 = (e % (BN / 4)) * 4;
        bst[s] = ld4(a.B + (int64_t)(kc + k) * a.ldb + n0 + n4);
      } else {
        const int n = e >> 3, k4 = (e & 7) * 4;
        bst[s] = ld4(a.B + (int64_t)(n0 + n) * a.ldb + kc + k4);
      }
    }
  };
  auto store_b = [&]() {
#pragma unroll
    for (int s = 0; s < NT; ++s) {
      const int e = tid + 256 * s;
      if (BMODE == 0) {
        const int k = e / (BN / 4), n4 = (e % (BN / 4)) * 4;
        st4(&sB[k * BN + n4], bst[s]);
      } else {
        const int n = e >> 3, k4 = (e & 7) * 4;
        st4(&sB[n * kNkLd + k4], bst[s]);
      }
    }
  };
  float4 xa[4], xn[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) xa[g] = ld4(xrow + 8 * g);
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
  if (kbeg > 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) xa[g] = ld4(xrow + kbeg + 8 * g);
  }
  load_b(kbeg);
  store_b();
  __syncthreads();
  for (int kc = kbeg; kc < K; kc += kGBK) {
    const bool more = kc + kGBK < K;
    if (more) {
      load_b(kc + kGBK);
#pragma unroll
      for (int g = 0; g < 4; ++g) xn[g] = ld4(xrow + kc + kGBK + 8 * g);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (BMODE == 1) {
        float4 bv[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) bv[t] = ld4(&sB[(32 * t + r) * kNkLd + 8 * g + 4 * hf]);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = mfma32(comp(xa[g], s), comp(bv[t], s), acc[t]);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float* brow = &sB[(8 * g + 4 * hf + s) * BN + r];
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = mfma32(comp(xa[g], s), brow[32 * t], acc[t]);
        }
      }
    }
    __syncthreads();
    if (more) {
      store_b();
#pragma unroll
      for (int g = 0; g < 4; ++g) xa[g] = xn[g];
    }
    __syncthreads();
  }
  const int64_t row0 = rb * kGBM + wv * 32;
  if (a.splits > 1) {
    float* part = a.part + (int64_t)split * M * a.N;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        if (row < M) part[row * a.N + col] = acc[t][q];
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 32 * t + r;
    const float bv = a.bias != nullptr ? a.bias[col] : 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
      if (row < M) a.Y[row * a.ldy + col] = fmaf(a.alpha, acc[t][q], bv);
    }
  }
}

// NN GEMM on the split bf16 matrix cores (ppgat_split.h), same contract, block order and
// split-K partials as k_gemm_nn.  v_mfma_f32_32x32x16_bf16: lane (r, hf) holds A[row r][8 hf + j]
// and B[8 hf + j][col r]; a 32-deep k chunk is two MFMA steps u, and lane half hf's element j
// of step u is k = 16 u + 4 hf + (j & 3) + 8 (j >> 2) -- exactly the two float4 xa[2u], xa[2u+1]
// a lane already streams from its X row.  The B chunk is split once per workgroup while being
// staged: three bf16 images [n][kk] with kk the position of k in that order (80-B rows: the 16
// lanes of every ds_read_b128 group hit distinct bank slots), one b128 read per part per tile.
template <int NT, int BMODE, int KC>
__global__ void __launch_bounds__(256, 2) k_gemm_nnx(NnArg a) {
  constexpr int BN = 32 * NT;
  constexpr int LDK = KC + 8;             // bf16 per image row (KC + 8 pad: an odd number of 16-B units)
  constexpr int PART = BN * LDK;          // bf16 per part
  constexpr int G = BN * (KC / 4) / 256;  // 4-k groups staged per thread per chunk
  constexpr int XG = KC / 8;              // float4 of X per lane per chunk
  __shared__ __attribute__((aligned(16))) uint16_t sB[3 * PART];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int64_t b = blockIdx.x;
  int64_t rb;
  int n0, split = 0;
  if (a.splits > 1) {
    split = (int)(b % a.splits);
    const int64_t rest = b / a.splits;
    n0 = (int)(rest % a.n_blocks) * BN;
    rb = rest / a.n_blocks;
  } else {
    const int64_t idx = b >> 3;
    rb = (idx / a.n_blocks) * 8 + (b & 7);
    n0 = (int)(idx % a.n_blocks) * BN;
  }
  if (rb >= a.row_blocks) return;
  const int64_t M = a.M;
  const int kbeg = split * a.k_per;
  const int K = a.splits > 1 ? (kbeg + a.k_per < a.K ? kbeg + a.k_per : a.K) : a.K;
  const int64_t m = rb * kGBM + wv * 32 + r;
  const float* xrow = a.X + (m < M ? m : M - 1) * a.ldx + 4 * hf;

  // staged group e = tid + 256 s: column n, reduction indices 4 q .. 4 q + 3 of the chunk
  auto grp = [&](int s, int& n, int& q) {
    const int e = tid + 256 * s;
    if (BMODE == 0) { n = e % BN; q = e / BN; }                   // a k row is contiguous in n
    else if (KC == 32) {  // an n row is contiguous in k; rows n, n + 4 share a 16-lane write group
      n = 8 * (e >> 6) + ((((e >> 3) & 1) << 2) | ((e >> 4) & 3));  // (80 dwords apart: no bank conflict)
      q = e & 7;
    } else { n = e / (KC / 4); q = e % (KC / 4); }
  };
  float4 bst[G];
  auto load_b = [&](int kc) {
#pragma unroll
    for (int s = 0; s < G; ++s) {
      int n, q;
      grp(s, n, q);
      if (BMODE == 0) {
        const float* p = a.B + (int64_t)(kc + 4 * q) * a.ldb + n0 + n;
        bst[s] = make_float4(p[0], p[a.ldb], p[2 * a.ldb], p[3 * a.ldb]);
      } else {
        bst[s] = ld4(a.B + (int64_t)(n0 + n) * a.ldb + kc + 4 * q);
      }
    }
  };
  auto store_b = [&]() {
#pragma unroll
    for (int s = 0; s < G; ++s) {
      int n, q;
      grp(s, n, q);
      const int kk = 16 * (q >> 2) + 8 * (q & 1) + 4 * ((q >> 1) & 1);
      const float v[4] = {bst[s].x, bst[s].y, bst[s].z, bst[s].w};
      uint2 h, mm, l;
      uint32_t* ph = &h.x;
      uint32_t* pm = &mm.x;
      uint32_t* pl = &l.x;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint32_t hh = split::pk_bf16(v[2 * i], v[2 * i + 1]);
        const float r0 = v[2 * i] - split::bf_lo(hh), r1 = v[2 * i + 1] - split::bf_hi(hh);
        const uint32_t m2 = split::pk_bf16(r0, r1);
        ph[i] = hh;
        pm[i] = m2;
        pl[i] = split::pk_bf16(r0 - split::bf_lo(m2), r1 - split::bf_hi(m2));
      }
      const int off = n * LDK + kk;
      *reinterpret_cast<uint2*>(&sB[off]) = h;
      *reinterpret_cast<uint2*>(&sB[PART + off]) = mm;
      *reinterpret_cast<uint2*>(&sB[2 * PART + off]) = l;
    }
  };
  float4 xa[XG], xn[XG];
#pragma unroll
  for (int g = 0; g < XG; ++g) xa[g] = ld4(xrow + kbeg + 8 * g);
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
  load_b(kbeg);
  store_b();
  __syncthreads();
  for (int kc = kbeg; kc < K; kc += KC) {
    const bool more = kc + KC < K;
    if (more) {
      load_b(kc + KC);
#pragma unroll
      for (int g = 0; g < XG; ++g) xn[g] = ld4(xrow + kc + KC + 8 * g);
    }
    // (u, t) steps in order; the next step's three B units are read from LDS while the
    // current step's six MFMAs run (a read waited on right before its MFMAs exposes the LDS
    // latency against only six MFMAs)
    auto read_b = [&](int idx, split::u32x4 (&f)[3]) {
      const int off = (32 * (idx % NT) + r) * LDK + 16 * (idx / NT) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&sB[p * PART + off]);
    };
    split::u32x4 fx[3], fb[3];
    read_b(0, fb);
#pragma unroll
    for (int idx = 0; idx < (KC / 16) * NT; ++idx) {
      const int u = idx / NT, t = idx % NT;
      if (t == 0) split::split3(xa[2 * u], xa[2 * u + 1], fx[0], fx[1], fx[2]);
      split::u32x4 fn[3];
      if (idx + 1 < (KC / 16) * NT) read_b(idx + 1, fn);
      acc[t] = split::mfma32_x6(fx, fb, acc[t]);
      __builtin_amdgcn_sched_barrier(0);
      if (idx + 1 < (KC / 16) * NT) {
        fb[0] = fn[0];
        fb[1] = fn[1];
        fb[2] = fn[2];
      }
    }
    __syncthreads();
    if (more) {
      store_b();
#pragma unroll
      for (int g = 0; g < XG; ++g) xa[g] = xn[g];
    }
    __syncthreads();
  }
  const int64_t row0 = rb * kGBM + wv * 32;
  if (a.splits > 1) {
    float* part = a.part + (int64_t)split * M * a.N;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        if (row < M) part[row * a.N + col] = acc[t][q];
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 32 * t + r;
    const float bv = a.bias != nullptr ? a.bias[col] : 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
      if (row < M) a.Y[row * a.ldy + col] = fmaf(a.alpha, acc[t][q], bv);
    }
  }
}

// ---------------------------------------------------------------------------
// NN GEMM on the split bf16 matrix cores, B pre-split once per call (the large-M shapes:
// config 5's [1.9M x 1024] x [1024 x 256] and [1.9M x 256] x [256 x 1024]).
//
// k_gemm_nnx splits its 32-deep B chunk while staging it (per workgroup, per chunk: ~1.8 VALU
// instructions per MFMA, PMC profiles/r03/v1_gemm_nnx_cfg5_pmc.json: MFMA busy 0.49) and
// stages it through registers with two barriers per chunk.  Here:
//  * k_nnx_presplit writes the three bf16 images of every (column block, k chunk) to the
//    workspace ONCE per call, in exactly the LDS layout k_gemm_nnx uses (80-B rows, the
//    permuted reduction order), so the products are the same -- bitwise equal results;
//  * k_gemm_nnp stages them with global_load_lds_dwordx4 (an image is a contiguous byte
//    range, so the lane-linear LDS destination is the image itself), two LDS buffers, one
//    barrier per chunk, 8 waves (256 rows) sharing every staged chunk.
// ---------------------------------------------------------------------------
constexpr int kPBM = 256;  // rows per k_gemm_nnp workgroup (8 waves x 32)

template <int NT>
struct NnpImg {
  static constexpr int KC = 32, BN = 32 * NT, LDK = KC + 8, PART = BN * LDK, ELEMS = 3 * PART, BYTES = 2 * ELEMS;
  static_assert(BYTES % 1024 == 0, "an image is a whole number of 1-KB wave copies");
};

template <int NT, int BMODE>
__global__ void __launch_bounds__(256) k_nnx_presplit(const float* __restrict__ B, int64_t ldb, int K, int N,
                                                      uint16_t* __restrict__ img) {
  using I = NnpImg<NT>;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * (K / 4)) return;
  const int ng = (int)(t % N), kq = (int)(t / N);
  const int k0 = 4 * kq, c = k0 / I::KC, q = (k0 % I::KC) / 4;
  const int nb = ng / I::BN, n = ng % I::BN;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = BMODE == 0 ? B[(int64_t)(k0 + j) * ldb + ng] : B[(int64_t)ng * ldb + k0 + j];
  uint2 h, mm, l;
  uint32_t* ph = &h.x;
  uint32_t* pm = &mm.x;
  uint32_t* pl = &l.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const uint32_t hh = split::pk_bf16(v[2 * i], v[2 * i + 1]);
    const float r0 = v[2 * i] - split::bf_lo(hh), r1 = v[2 * i + 1] - split::bf_hi(hh);
    const uint32_t m2 = split::pk_bf16(r0, r1);
    ph[i] = hh;
    pm[i] = m2;
    pl[i] = split::pk_bf16(r0 - split::bf_lo(m2), r1 - split::bf_hi(m2));
  }
  const int kk = 16 * (q >> 2) + 8 * (q & 1) + 4 * ((q >> 1) & 1);
  uint16_t* base = img + ((int64_t)nb * (K / I::KC) + c) * I::ELEMS + n * I::LDK + kk;
  *reinterpret_cast<uint2*>(base) = h;
  *reinterpret_cast<uint2*>(base + I::PART) = mm;
  *reinterpret_cast<uint2*>(base + 2 * I::PART) = l;
}

template <int NT>
__global__ void __launch_bounds__(512, 1) k_gemm_nnp(NnArg a, const uint16_t* __restrict__ img) {
  using I = NnpImg<NT>;
  constexpr int KC = I::KC, LDK = I::LDK, PART = I::PART, NI = I::BYTES / 1024;
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][I::ELEMS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int64_t b = blockIdx.x;
  const int64_t idx = b >> 3;
  const int64_t rb = (idx / a.n_blocks) * 8 + (b & 7);  // XCD-aware: a row block's column blocks share an L2
  const int nb = (int)(idx % a.n_blocks);
  if (rb >= a.row_blocks) return;
  const int64_t M = a.M;
  const int K = a.K, chunks = K / KC;
  const int64_t m = rb * kPBM + wv * 32 + r;
  const float* xrow = a.X + (m < M ? m : M - 1) * a.ldx + 4 * hf;  // rows past M re-read row M-1 (never stored)
  // buffer_load ... lds (MUBUF), not global_load_lds: the compiler counts a FLAT LDS-DMA as a
  // pending LDS access, and every LDS-read wait behind it became lgkmcnt(0) -- the ds_reads of
  // step i + 1 could not overlap step i's MFMAs.  A MUBUF LDS-DMA is tracked on vmcnt only.
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(img + (int64_t)nb * chunks * I::ELEMS), 0, chunks * I::BYTES, 0x00020000);
  auto issue = [&](int c, int buf) {  // chunk c's three images -> sB[buf], 1 KB per wave instruction
    const int src = c * I::BYTES + lane * 16;
    char* dst = reinterpret_cast<char*>(sB[buf]);
    for (int i = wv; i < NI; i += 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + i * 1024), 16,
                                               src + i * 1024, 0, 0, 0);
  };
  float4 xa[4], xn[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) xa[g] = ld4(xrow + 8 * g);
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
  issue(0, 0);
  __syncthreads();  // vmcnt(0): chunk 0 and the first x fragments have landed
  for (int c = 0; c < chunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < chunks;
    if (more) {
      issue(c + 1, buf ^ 1);  // the buffer every wave finished reading before the last barrier
#pragma unroll
      for (int g = 0; g < 4; ++g) xn[g] = ld4(xrow + (c + 1) * KC + 8 * g);
    }
    const uint16_t* sb = sB[buf];
    auto read_b = [&](int i, split::u32x4 (&f)[3]) {
      const int off = (32 * (i % NT) + r) * LDK + 16 * (i / NT) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&sb[p * PART + off]);
    };
    // B fragments in two register sets used alternately (no copy between them, so the register
    // allocator cannot merge them): the reads of step i + 1 issue before the six MFMAs of step i
    // and have those ~190 cycles to land (with one merged set they were scheduled after the
    // step's fifth MFMA and the next step waited on the LDS latency)
    split::u32x4 fx[3], fb[2][3];
    read_b(0, fb[0]);
#pragma unroll
    for (int i = 0; i < (KC / 16) * NT; ++i) {
      const int u = i / NT, t = i % NT;
      if (t == 0) split::split3(xa[2 * u], xa[2 * u + 1], fx[0], fx[1], fx[2]);
      if (i + 1 < (KC / 16) * NT) read_b(i + 1, fb[(i + 1) & 1]);
      acc[t] = split::mfma32_x6(fx, fb[i & 1], acc[t]);
      // order inside the step: the next step's three LDS reads first, then the six MFMAs
      if (i + 1 < (KC / 16) * NT) __builtin_amdgcn_sched_group_barrier(0x0100, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 6, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // vmcnt(0): chunk c + 1 has landed; every wave is done with sB[buf]
    if (more) {
#pragma unroll
      for (int g = 0; g < 4; ++g) xa[g] = xn[g];
    }
  }
  const int64_t row0 = rb * kPBM + wv * 32;
  const int n0 = nb * I::BN;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = n0 + 32 * t + r;
    const float bv = a.bias != nullptr ? a.bias[col] : 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
      if (row < M) a.Y[row * a.ldy + col] = fmaf(a.alpha, acc[t][q], bv);
    }
  }
}

// ---------------------------------------------------------------------------
// NN GEMM on the fp16 matrix cores through the scaled two-term split (ppgat_split.h): three
// MFMAs per product instead of six.  B is pre-split once per call with a power-of-two scale per
// column (k_colscale16 + k_nnh_presplit: two fp16 images per (column block, k chunk), the same
// 80-B rows and permuted reduction order as the bf16 images).  X streams in 32-deep chunks, so a
// row's scale is set ONLINE: by the first chunk in which the row is nonzero (largest |x| s in
// [2^9, 2^10)), and lowered only when a later chunk would reach 2^15 (fp16 overflows at 65,520,
// so 32x headroom) -- then that row's accumulators are multiplied by the exact power of two
// s_new / s_old (a wave-uniform branch, rare on real data: first-chunk maxima within 32x of the
// row's).  Elements far below their row's max keep an absolute error <= 2^-34 of that max.
// ---------------------------------------------------------------------------

// per column of B [K x N]: the scale exponent (largest |b| 2^e in [2^9, 2^10); 0 for a zero column)
template <int BMODE>
__global__ void __launch_bounds__(256) k_colscale16(const float* __restrict__ B, int64_t ldb, int K, int N,
                                                    int* __restrict__ ecol) {
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  float m = 0.f;
  for (int k = lane; k < K; k += 64) m = fmaxf(m, fabsf(BMODE == 0 ? B[(int64_t)k * ldb + n] : B[(int64_t)n * ldb + k]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) ecol[n] = m > 0.f && m <= 3.4e38f ? split::scale_exp16(m) : 0;
}

template <int NT, int BMODE>
__global__ void __launch_bounds__(256) k_nnh_presplit(const float* __restrict__ B, int64_t ldb, int K, int N,
                                                      const int* __restrict__ ecol, uint16_t* __restrict__ img) {
  using I = NnhImg<NT>;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * (K / 4)) return;
  const int ng = (int)(t % N), kq = (int)(t / N);
  const int k0 = 4 * kq, c = k0 / I::KC, q = (k0 % I::KC) / 4;
  const int nb = ng / I::BN, n = ng % I::BN;
  const float s = ldexpf(1.f, ecol[ng]);
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (BMODE == 0 ? B[(int64_t)(k0 + j) * ldb + ng] : B[(int64_t)ng * ldb + k0 + j]) * s;
  uint2 h, l;
  uint32_t* ph = &h.x;
  uint32_t* pl = &l.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const uint32_t hh = split::pk_f16(v[2 * i], v[2 * i + 1]);
    const split::f32x2e back = __builtin_convertvector(__builtin_bit_cast(split::f16x2, hh), split::f32x2e);
    ph[i] = hh;
    pl[i] = split::pk_f16(v[2 * i] - back.x, v[2 * i + 1] - back.y);
  }
  const int kk = 16 * (q >> 2) + 8 * (q & 1) + 4 * ((q >> 1) & 1);
  uint16_t* base = img + ((int64_t)nb * (K / I::KC) + c) * I::ELEMS + n * I::LDK + kk;
  *reinterpret_cast<uint2*>(base) = h;
  *reinterpret_cast<uint2*>(base + I::PART) = l;
}

constexpr int kNnhRank = 8;  // rank terms the fused epilogue keeps in registers

template <int NT, bool RK>
__global__ void __launch_bounds__(512, 1) k_gemm_nnh(NnArg a, const uint16_t* __restrict__ img,
                                                     const int* __restrict__ ecol) {
  using I = NnhImg<NT>;
  constexpr int KC = I::KC, LDK = I::LDK, PART = I::PART, NI = I::BYTES / 1024;
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][I::ELEMS];
  __shared__ __attribute__((aligned(16))) float sF[8][32];  // per wave: a factor per row (rescale, epilogue)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int64_t b = blockIdx.x;
  const int64_t idx = b >> 3;
  const int64_t rb = (idx / a.n_blocks) * 8 + (b & 7);  // XCD-aware: a row block's column blocks share an L2
  const int nb = (int)(idx % a.n_blocks);
  if (rb >= a.row_blocks) return;
  const int64_t M = a.M;
  const int K = a.K, chunks = K / KC;
  const int64_t m = rb * kPBM + wv * 32 + r;
  const float* xrow = a.X + (m < M ? m : M - 1) * a.ldx + 4 * hf;  // rows past M re-read row M-1 (never stored)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(img + (int64_t)nb * chunks * I::ELEMS), 0, chunks * I::BYTES, 0x00020000);
  auto issue = [&](int c, int buf) {  // chunk c's two images -> sB[buf], 1 KB per wave instruction
    const int src = c * I::BYTES + lane * 16;
    char* dst = reinterpret_cast<char*>(sB[buf]);
    for (int i = wv; i < NI; i += 8)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + i * 1024), 16,
                                               src + i * 1024, 0, 0, 0);
  };
  float4 xa[4], xn[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) xa[g] = ld4(xrow + 8 * g);
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
  int erow = 0;
  bool set = false;  // the row has had a nonzero element (its scale is fixed until an overflow)
  issue(0, 0);
  __syncthreads();  // vmcnt(0): chunk 0 and the first x fragments have landed
  for (int c = 0; c < chunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < chunks;
    if (more) {
      issue(c + 1, buf ^ 1);  // the buffer every wave finished reading before the last barrier
#pragma unroll
      for (int g = 0; g < 4; ++g) xn[g] = ld4(xrow + (c + 1) * KC + 8 * g);
    }
    const float s = split::row_scale_online<NT>(xa, erow, set, acc, sF[wv], r, hf);  // chunk c's row scales
    const uint16_t* sb = sB[buf];
    auto read_b = [&](int i, split::u32x4 (&f)[2]) {
      const int off = (32 * (i % NT) + r) * LDK + 16 * (i / NT) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&sb[p * PART + off]);
    };
    // two fragment sets used alternately; each step issues the next step's two LDS reads before
    // its three MFMAs (see k_gemm_nnp)
    split::u32x4 fx[2], fb[2][2];
    read_b(0, fb[0]);
#pragma unroll
    for (int i = 0; i < (KC / 16) * NT; ++i) {
      const int u = i / NT, t = i % NT;
      if (t == 0) split::split2h(xa[2 * u], xa[2 * u + 1], s, fx[0], fx[1]);
      if (i + 1 < (KC / 16) * NT) read_b(i + 1, fb[(i + 1) & 1]);
      acc[t] = split::mfma32_h3(fx, fb[i & 1], acc[t]);
      if (i + 1 < (KC / 16) * NT) __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 3, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // vmcnt(0): chunk c + 1 has landed; every wave is done with sB[buf]
    if (more) {
#pragma unroll
      for (int g = 0; g < 4; ++g) xa[g] = xn[g];
    }
  }
  float fr[16];  // unscale: 1 / (s_row s_col), both exact powers of two
  split::row_unscale(erow, sF[wv], r, hf, fr);
  const int64_t row0 = rb * kPBM + wv * 32;
  const int n0 = nb * I::BN;
  if constexpr (RK) {
    // + S A (nv <= kNnhRank): this lane's columns of A in registers, each row's S terms loaded
    // once (broadcast over the 32 lanes of the row), the terms added in v order after alpha, bias
    const int nv = a.nv;
    float ra[NT][kNnhRank], bv[NT], ic[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
      bv[t] = a.bias != nullptr ? a.bias[col] : 0.f;
      ic[t] = ldexpf(a.alpha, -ecol[col]);
#pragma unroll
      for (int v = 0; v < kNnhRank; ++v) ra[t][v] = v < nv ? a.rA[v * a.ldra + col] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
      const int64_t rr = row < M ? row : M - 1;
      float sv[kNnhRank];
#pragma unroll
      for (int v = 0; v < kNnhRank; ++v) sv[v] = v < nv ? a.rS[rr * a.ldrs + v] : 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float y = fmaf(acc[t][q] * fr[q], ic[t], bv[t]);
#pragma unroll
        for (int v = 0; v < kNnhRank; ++v)
          if (v < nv) y = fmaf(sv[v], ra[t][v], y);
        if (row < M) a.Y[row * a.ldy + n0 + 32 * t + r] = y;
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
      const float bv = a.bias != nullptr ? a.bias[col] : 0.f;
      const float ic = ldexpf(a.alpha, -ecol[col]);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        if (row < M) a.Y[row * a.ldy + col] = fmaf(acc[t][q] * fr[q], ic, bv);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_gemm_nnh2: k_gemm_nnh's arithmetic (the same products in the same order: bitwise equal
// results) with a deeper pipeline.  In k_gemm_nnh the compiler waits for the whole vector-memory
// queue twice per 32-deep chunk -- before the first LDS read after an LDS-DMA issue (it cannot
// tell the DMA target from the buffer being read) and at every __syncthreads (its workgroup
// fence) -- so the next chunk's X rows, streamed from HBM one chunk ahead, had only part of a
// chunk to arrive (MFMA busy 0.41, 46 % of the wave cycles waiting; profiles/r03/v27_nnh_pmc.json).
// Here:
//  * B chunks go to LDS by LDS-DMA issued in inline asm (the compiler sees no memory access, so
//    it adds no wait before LDS reads), three buffers, issued two chunks ahead;
//  * X rows stream two chunks ahead in two register sets; a chunk's rows are scaled and split
//    into their fp16 fragments at the top of the chunk, which frees the set for chunk c + 2;
//  * the chunk barrier is a bare s_barrier after an explicit vmcnt wait for exactly this
//    wave's DMA of chunk c + 1 (the only operation the barrier must cover: everything issued
//    after it -- X of c + 1, DMA and X of c + 2 -- stays in flight).
// Global issue order per wave: DMA(0) X(0) DMA(1) X(1) | chunk c: DMA(c+2) X(c+2) ...
// ---------------------------------------------------------------------------

// LAB (diagnostics only, lab builds -DPPGAT_LAB_BUILD=1, never in libppgat.so; PPGAT_NNH2_LAB;
// results wrong), bits: 1 = no X loads after the first
// two chunks (registers reused), 2 = no B DMA after the first two chunks (LDS reused), 4 = no
// epilogue stores (a row is stored only if its first accumulator is NaN), 8 = no chunk barrier
template <int NT, bool RK, int LAB = 0>
__global__ void __launch_bounds__(512, 1) k_gemm_nnh2(NnArg a, const uint16_t* __restrict__ img,
                                                      const int* __restrict__ ecol) {
  using I = NnhImg<NT>;
  constexpr int KC = I::KC, LDK = I::LDK, PART = I::PART, NI = I::BYTES / 1024;
  __shared__ __attribute__((aligned(16))) uint16_t sB[3][I::ELEMS];
  __shared__ __attribute__((aligned(16))) float sF[8][32];  // per wave: a factor per row (rescale, epilogue)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int64_t b = blockIdx.x;
  const int64_t idx = b >> 3;
  const int64_t rb = (idx / a.n_blocks) * 8 + (b & 7);  // XCD-aware: a row block's column blocks share an L2
  const int nb = (int)(idx % a.n_blocks);
  if (rb >= a.row_blocks) return;
  const int64_t M = a.M;
  const int K = a.K, chunks = K / KC;
  const int64_t m = rb * kPBM + wv * 32 + r;
  const float* xrow = a.X + (m < M ? m : M - 1) * a.ldx + 4 * hf;  // rows past M re-read row M-1 (never stored)
  // buffer resource of this column block's images (stride 0, raw bytes), wave-uniform
  const uint64_t base = reinterpret_cast<uint64_t>(img + (int64_t)nb * chunks * I::ELEMS);
  const i32x4 rsrc = {__builtin_amdgcn_readfirstlane((int)(uint32_t)base),
                      __builtin_amdgcn_readfirstlane((int)((base >> 32) & 0xffff)),
                      __builtin_amdgcn_readfirstlane(chunks * I::BYTES), 0x00020000};
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(&sB[0][0]);
  const uint32_t voff = (uint32_t)lane * 16u;
  constexpr int ND = (NI + 7) / 8;  // DMA instructions of waves 0 .. (NI % 8) - 1 (one fewer for the rest)
  const bool full = (NI % 8 == 0) || wv < NI % 8;
  auto issue = [&](int c) {  // chunk c's two images -> sB[c % 3], 1 KB per wave instruction
    const uint32_t dst = lds0 + (uint32_t)((c % 3) * I::ELEMS * 2);
    for (int i = wv; i < NI; i += 8) dma_lds16(rsrc, dst + i * 1024, voff, (uint32_t)(c * I::BYTES + i * 1024));
  };
  auto loadx = [&](int c, float4 (&x)[4]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) x[g] = ld4(xrow + c * KC + 8 * g);
  };
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{};
  int erow = 0;
  bool set = false;  // the row has had a nonzero element (its scale is fixed until an overflow)
  // chunks is even (>= 2; the launcher checks): the loop below runs chunk pairs (xA, xB) and
  // every chunk loads an X set, the last two re-reading chunk chunks - 1, so the compiler sees
  // the same four loads per chunk on every path and waits for exactly the set it reads
  float4 xA[4], xB[4];
  issue(0);
  loadx(0, xA);
  issue(1);
  loadx(1, xB);
  if (full) wait_vm<4 + ND + 4>(); else wait_vm<4 + ND - 1 + 4>();  // DMA(0) has landed
  __builtin_amdgcn_s_barrier();

  auto body = [&](const int c, float4 (&xc)[4]) {
    // X(c): this chunk's row scales and fp16 fragments (both k steps), then the set is free
    const float s = split::row_scale_online<NT>(xc, erow, set, acc, sF[wv], r, hf);
    split::u32x4 fx[2][2];
    split::split2h(xc[0], xc[1], s, fx[0][0], fx[0][1]);
    split::split2h(xc[2], xc[3], s, fx[1][0], fx[1][1]);
    const bool ahead = c + 2 < chunks;
    if (ahead && !(LAB & 2)) issue(c + 2);
    if (!(LAB & 1)) loadx(ahead ? c + 2 : chunks - 1, xc);
    const uint16_t* sb = sB[c % 3];
    auto read_b = [&](int i, split::u32x4 (&f)[2]) {
      const int off = (32 * (i % NT) + r) * LDK + 16 * (i / NT) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&sb[p * PART + off]);
    };
    split::u32x4 fb[2][2];
    read_b(0, fb[0]);
#pragma unroll
    for (int i = 0; i < (KC / 16) * NT; ++i) {
      const int u = i / NT, t = i % NT;
      if (i + 1 < (KC / 16) * NT) read_b(i + 1, fb[(i + 1) & 1]);
      acc[t] = split::mfma32_h3(fx[u], fb[i & 1], acc[t]);
      if (i + 1 < (KC / 16) * NT) __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 3, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // DMA(c + 1) must have landed before any wave reads it, and every wave must be done with
    // sB[c % 3] before chunk c + 3's DMA (issued in chunk c + 1) overwrites it.  Issued after
    // DMA(c + 1): X(c + 1), and in this chunk DMA(c + 2) (if any) and an X set.
    if (LAB) {
      wait_vm<0>();
    } else if (ahead) {
      if (full) wait_vm<4 + ND + 4>(); else wait_vm<4 + ND - 1 + 4>();
    } else {
      wait_vm<4 + 4>();
    }
    if (!(LAB & 8)) __builtin_amdgcn_s_barrier();
  };
  for (int c = 0; c < chunks; c += 2) {
    body(c, xA);
    body(c + 1, xB);
  }
  float fr[16];  // unscale: 1 / (s_row s_col), both exact powers of two
  split::row_unscale(erow, sF[wv], r, hf, fr);
  const int64_t row0 = rb * kPBM + wv * 32;
  const int n0 = nb * I::BN;
  if constexpr (RK) {
    const int nv = a.nv;
    float ra[NT][kNnhRank], bv[NT], ic[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
      bv[t] = a.bias != nullptr ? a.bias[col] : 0.f;
      ic[t] = ldexpf(a.alpha, -ecol[col]);
#pragma unroll
      for (int v = 0; v < kNnhRank; ++v) ra[t][v] = v < nv ? a.rA[v * a.ldra + col] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
      const int64_t rr = row < M ? row : M - 1;
      float sv[kNnhRank];
#pragma unroll
      for (int v = 0; v < kNnhRank; ++v) sv[v] = v < nv ? a.rS[rr * a.ldrs + v] : 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float y = fmaf(acc[t][q] * fr[q], ic[t], bv[t]);
#pragma unroll
        for (int v = 0; v < kNnhRank; ++v)
          if (v < nv) y = fmaf(sv[v], ra[t][v], y);
        if (row < M) a.Y[row * a.ldy + n0 + 32 * t + r] = y;
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
      const float bv = a.bias != nullptr ? a.bias[col] : 0.f;
      const float ic = ldexpf(a.alpha, -ecol[col]);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        if (row < M && (!(LAB & 4) || acc[0][q] != acc[0][q])) a.Y[row * a.ldy + col] = fmaf(acc[t][q] * fr[q], ic, bv);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_gemm_nnh3: k_gemm_nnh2's pipeline with the next chunk prepared inside the current chunk's
// MFMA sequence (ppgat_nnh_pipe.h: nnh3_loop), same products in the same order as k_gemm_nnh.
// ---------------------------------------------------------------------------
// E4 (lab builds, PPGAT_NNH_E4=1): the epilogue without rank terms through a per-wave LDS
// transpose -- each lane's column of 16 rows is written to the (now idle) B buffers and read back
// as float4 pieces of rows, so a wave stores its 32 x 32 block per column tile in 4 float4
// instructions (8 rows x 128 B each) instead of 16 scalar ones; the same values (same bits).
// OCC (lab, PPGAT_NNH_OCC2=1 with NT = 4): at least OCC waves per SIMD (HIP's launch_bounds), i.e. two
// workgroups per CU at OCC = 4, so one's epilogue stores can run beside the other's products.
template <int NT, bool RK, int BD = 1, bool PRIO = false, int LAB = 0, bool XT = false, bool E4 = false, int OCC = 1>
__global__ void __launch_bounds__(512, OCC) k_gemm_nnh3(NnArg a, const uint16_t* __restrict__ img,
                                                      const int* __restrict__ ecol) {
  using I = NnhImg<NT>;
  constexpr int KC = I::KC;
  __shared__ __attribute__((aligned(16))) uint16_t sB[3 * I::ELEMS];
  __shared__ __attribute__((aligned(16))) float sF[8][32];  // per wave: a factor per row (rescale, epilogue)
  __shared__ __attribute__((aligned(16))) float sX[XT ? 8 : 1][XT ? 32 * 36 : 4];  // per wave: X transpose (XT)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int64_t b = blockIdx.x;
  const int64_t idx = b >> 3;
  const int64_t rb = (idx / a.n_blocks) * 8 + (b & 7);  // XCD-aware: a row block's column blocks share an L2
  const int nb = (int)(idx % a.n_blocks);
  if (rb >= a.row_blocks) return;
  const int64_t M = a.M;
  const int chunks = a.K / KC;
  const int64_t m = rb * kPBM + wv * 32 + r;
  const float* xrow = a.X + (m < M ? m : M - 1) * a.ldx + 4 * hf;  // rows past M re-read row M-1 (never stored)
  f32x16 acc[NT];
  int erow = 0;
  if constexpr (XT) {
    // coalesced: lane l reads floats [4 (l & 7), +4) of rows (l >> 3) + 8 j of the wave's 32
    const float* xr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t row = rb * kPBM + wv * 32 + (lane >> 3) + 8 * j;
      xr[j] = a.X + (row < M ? row : M - 1) * a.ldx + 4 * (lane & 7);
    }
    auto loadx = [&](int c, float4 (&x)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = ld4(xr[j] + c * KC);
    };
    nnh3_loop<NT, BD, PRIO, LAB, true>(img + (int64_t)nb * chunks * I::ELEMS, sB, chunks, loadx, acc, erow, sF[wv],
                                       wv, lane, sX[wv]);
  } else {
    auto loadx = [&](int c, float4 (&x)[4]) {
#pragma unroll
      for (int g = 0; g < 4; ++g) x[g] = ld4(xrow + c * KC + 8 * g);
    };
    nnh3_loop<NT, BD, PRIO, LAB>(img + (int64_t)nb * chunks * I::ELEMS, sB, chunks, loadx, acc, erow, sF[wv], wv,
                                 lane);
  }
  float fr[16];  // unscale: 1 / (s_row s_col), both exact powers of two
  split::row_unscale(erow, sF[wv], r, hf, fr);
  const int64_t row0 = rb * kPBM + wv * 32;
  const int n0 = nb * I::BN;
  if constexpr (RK) {
    const int nv = a.nv;
    float ra[NT][kNnhRank], bv[NT], ic[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
      bv[t] = a.bias != nullptr ? a.bias[col] : 0.f;
      ic[t] = ldexpf(a.alpha, -ecol[col]);
#pragma unroll
      for (int v = 0; v < kNnhRank; ++v) ra[t][v] = v < nv ? a.rA[v * a.ldra + col] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
      const int64_t rr = row < M ? row : M - 1;
      float sv[kNnhRank];
#pragma unroll
      for (int v = 0; v < kNnhRank; ++v) sv[v] = v < nv ? a.rS[rr * a.ldrs + v] : 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        float y = fmaf(acc[t][q] * fr[q], ic[t], bv[t]);
#pragma unroll
        for (int v = 0; v < kNnhRank; ++v)
          if (v < nv) y = fmaf(sv[v], ra[t][v], y);
        if (row < M) a.Y[row * a.ldy + n0 + 32 * t + r] = y;
      }
    }
  } else if constexpr (E4) {
    // the B buffers are idle: every wave passed the last chunk's barrier after its last B reads
    float* T = reinterpret_cast<float*>(sB) + wv * (32 * 40);  // this wave's [32 rows][40] tile
    const int rl = lane >> 3, c4 = 4 * (lane & 7);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
      const float bv = a.bias != nullptr ? a.bias[col] : 0.f;
      const float ic = ldexpf(a.alpha, -ecol[col]);
#pragma unroll
      for (int q = 0; q < 16; ++q) T[((q & 3) + 8 * (q >> 2) + 4 * hf) * 40 + r] = fmaf(acc[t][q] * fr[q], ic, bv);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t row = row0 + rl + 8 * j;
        const float4 v = *reinterpret_cast<const float4*>(T + (rl + 8 * j) * 40 + c4);
        if (row < M) *reinterpret_cast<float4*>(a.Y + row * a.ldy + n0 + 32 * t + c4) = v;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = n0 + 32 * t + r;
      const float bv = a.bias != nullptr ? a.bias[col] : 0.f;
      const float ic = ldexpf(a.alpha, -ecol[col]);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        if (row < M && (!(LAB & 4) || acc[0][q] != acc[0][q])) a.Y[row * a.ldy + col] = fmaf(acc[t][q] * fr[q], ic, bv);
      }
    }
  }
}

// split-K finish: Y = alpha * sum_s part[s] (split order) + bias, float4 per thread
__global__ void __launch_bounds__(256) k_nn_split_sum(const float* __restrict__ part, int64_t M, int N, int splits,
                                                      float alpha, const float* __restrict__ bias,
                                                      float* __restrict__ Y, int64_t ldy) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int n4 = N / 4;
  if (e >= M * n4) return;
  const int64_t row = e / n4;
  const int c = (int)(e % n4) * 4;
  const size_t stride = (size_t)M * N;
  float4 s = ld4(part + row * N + c);
  for (int k = 1; k < splits; ++k) s = add4(s, ld4(part + k * stride + row * N + c));
  float4 o;
  o.x = fmaf(alpha, s.x, bias ? bias[c] : 0.f);
  o.y = fmaf(alpha, s.y, bias ? bias[c + 1] : 0.f);
  o.z = fmaf(alpha, s.z, bias ? bias[c + 2] : 0.f);
  o.w = fmaf(alpha, s.w, bias ? bias[c + 3] : 0.f);
  st4(Y + row * ldy + c, o);
}

// ===========================================================================
// TN GEMM: part[split] = A[rows of split]^T B[rows of split], A [M, Ma], B [M, Nb]
// ===========================================================================
constexpr int kTA = 128;  // a-tile (output rows)
constexpr int kTR = 32;   // rows per LDS chunk

struct TnArg {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  int64_t M;
  int Ma, Nb;
  int tiles_a, tiles_b, splits;
  int64_t rows_per_split;  // multiple of kTR
  float* part;             // [splits, Ma, Nb]
};

// BT: b-tile width (256 or 128).  Waves 2 x 2: wave (wa, wb) owns a-columns [64 wa, +64) (2 MFMA
// tiles) x b-columns [BT/2 wb, +BT/2) (BT/64 tiles).  MFMA: i = a column, j = b column, kk = row.
template <int BT>
__global__ void __launch_bounds__(256, 2) k_gemm_tn(TnArg a) {
  constexpr int NB = BT / 64;  // b tiles per wave
  constexpr int LA = kTA + 4, LB = BT + 4;
  __shared__ float sA[kTR * LA];
  __shared__ float sB[kTR * LB];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int wa = wv & 1, wb = wv >> 1;
  const int T = a.tiles_a * a.tiles_b;
  const int64_t b = blockIdx.x;
  const int64_t idx = b >> 3;
  const int tile = (int)(idx % T);
  const int64_t split = (b & 7) + 8 * (idx / T);  // one split's tiles share an XCD (and its L2)
  if (split >= a.splits) return;
  const int ta = tile % a.tiles_a, tb = tile / a.tiles_a;
  const int64_t r0 = split * a.rows_per_split;
  const int64_t r1 = min(a.M, r0 + a.rows_per_split);
  constexpr int A4 = kTR * kTA / 4 / 256;  // float4 per thread per chunk (4)
  constexpr int B4 = kTR * BT / 4 / 256;   // (8 or 4)
  float4 ar[A4], br[B4];
  auto load = [&](int64_t c0) {
#pragma unroll
    for (int s = 0; s < A4; ++s) {
      const int e = tid + 256 * s;
      const int rr = e / (kTA / 4), c4 = (e % (kTA / 4)) * 4;
      const int64_t row = c0 + rr;
      ar[s] = row < r1 ? ld4(a.A + row * a.lda + ta * kTA + c4) : f4(0.f);
    }
#pragma unroll
    for (int s = 0; s < B4; ++s) {
      const int e = tid + 256 * s;
      const int rr = e / (BT / 4), c4 = (e % (BT / 4)) * 4;
      const int64_t row = c0 + rr;
      br[s] = row < r1 ? ld4(a.B + row * a.ldb + tb * BT + c4) : f4(0.f);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int s = 0; s < A4; ++s) {
      const int e = tid + 256 * s;
      st4(&sA[(e / (kTA / 4)) * LA + (e % (kTA / 4)) * 4], ar[s]);
    }
#pragma unroll
    for (int s = 0; s < B4; ++s) {
      const int e = tid + 256 * s;
      st4(&sB[(e / (BT / 4)) * LB + (e % (BT / 4)) * 4], br[s]);
    }
  };
  f32x16 acc[2][NB];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int t = 0; t < NB; ++t) acc[u][t] = f32x16{};
  if (r0 < r1) {
    load(r0);
    store();
  }
  __syncthreads();
  for (int64_t c0 = r0; c0 < r1; c0 += kTR) {
    const bool more = c0 + kTR < r1;
    if (more) load(c0 + kTR);
#pragma unroll 4
    for (int s = 0; s < kTR / 2; ++s) {
      const int row = 2 * s + hf;
      float av[2], bv[NB];
#pragma unroll
      for (int u = 0; u < 2; ++u) av[u] = sA[row * LA + 64 * wa + 32 * u + r];
#pragma unroll
      for (int t = 0; t < NB; ++t) bv[t] = sB[row * LB + (BT / 2) * wb + 32 * t + r];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[u][t] = mfma32(av[u], bv[t], acc[u][t]);
    }
    __syncthreads();
    if (more) store();
    __syncthreads();
  }
  float* P = a.part + (size_t)split * a.Ma * a.Nb;
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int col = tb * BT + (BT / 2) * wb + 32 * t + r;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int arow = ta * kTA + 64 * wa + 32 * u + (q & 3) + 8 * (q >> 2) + 4 * hf;
        P[(size_t)arow * a.Nb + col] = acc[u][t][q];
      }
    }
}

// out[e] = scale * sum_s part[s][e] (split order) -- float4 per thread
__global__ void __launch_bounds__(256) k_split_sum(const float* __restrict__ part, int64_t n4, int splits,
                                                   float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n4) return;
  float4 s = ld4(part + e * 4);
#pragma unroll 8
  for (int k = 1; k < splits; ++k) s = add4(s, ld4(part + ((size_t)k * n4 + e) * 4));  // (loads in flight, adds in order)
  st4(out + e * 4, s);
}

// ===========================================================================
// TN GEMM on the fp16 matrix cores: two-term split with per-column power-of-two scales
// ===========================================================================
// part[split] = A[rows of split]^T B[rows of split] as in k_gemm_tn, but the reduction runs
// over rows, so a row-wise online scale (k_gemm_nnh) cannot apply: each column of A and of B
// gets ONE scale over all M rows -- the power of two that puts the column's largest |v| in
// [2^9, 2^10) (ppgat_split.h scale_exp16) -- from a max pre-pass (k_colmax_bits: the max of
// the IEEE bits of |v|, order-free, so deterministic).  Elements far below their column's max
// keep an absolute error <= 2^-34 of that max; the rest carry 22 bits (2^-21 per product, as
// k_gemm_nnh).  Workgroup tile 128 (A columns) x 256 (B columns), 8 waves (4 x 2), each wave
// one 32-column A block against four 32-column B blocks (64 accumulators); the rows of a
// 32-row chunk are split ONCE by the staging threads into swizzled row-major fp16 images (A:
// [32][128], B: two [32][128] halves; hi and lo terms) and both operands -- columns over the
// chunk's rows -- come back through the transposing ds_read_b64_tr_b16 (conflict-free, see
// k_dxw).  The tiles of one row split run on one XCD, so the rows leave HBM once.
constexpr int kThImg = kTR * 128 * 2;       // bytes per fp16 image [32][128]
constexpr int kThBuf = 6 * kThImg;          // A hi/lo, B half 0 hi/lo, B half 1 hi/lo (48 KB)
constexpr size_t kThLds = 2 * kThBuf + (2 * 128 + 2 * 256 + 16 * 128) * sizeof(float);  // + sC (colsum)

// column maxima of |X| over rows [r0, r1) of a row block, merged into out[] as IEEE bits;
// with rp (CSC pointers [M + 1]) only over the rows that are the source of an edge
__global__ void __launch_bounds__(256) k_colmax_bits(const float* __restrict__ X, int64_t ldx, int64_t M, int C,
                                                     int64_t rows_per_block, const int32_t* __restrict__ rp,
                                                     unsigned* __restrict__ out) {
  __shared__ float4 red[256];
  const int T = C >> 2, P = 256 / T, t = threadIdx.x, cg = t % T, rl = t / T;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float4 m = f4(0.f);
  auto mx = [](float4 a, float4 v) {
    return make_float4(fmaxf(a.x, fabsf(v.x)), fmaxf(a.y, fabsf(v.y)), fmaxf(a.z, fabsf(v.z)), fmaxf(a.w, fabsf(v.w)));
  };
  if (rl < P && rp == nullptr) {  // eight rows' loads in flight per thread (a max: any order, same bits)
    int64_t r = r0 + rl;
    for (; r + 7 * P < r1; r += 8 * P) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld4(X + (r + u * P) * ldx + 4 * cg);
#pragma unroll
      for (int u = 0; u < 8; ++u) m = mx(m, v[u]);
    }
    for (; r < r1; r += P) m = mx(m, ld4(X + r * ldx + 4 * cg));
  } else if (rl < P) {
    for (int64_t r = r0 + rl; r < r1; r += P) {
      if (rp != nullptr && rp[r + 1] == rp[r]) continue;
      const float4 v = ld4(X + r * ldx + 4 * cg);
      m = make_float4(fmaxf(m.x, fabsf(v.x)), fmaxf(m.y, fabsf(v.y)), fmaxf(m.z, fabsf(v.z)), fmaxf(m.w, fabsf(v.w)));
    }
  }
  red[t] = m;
  __syncthreads();
  if (t < T) {
    for (int q = 1; q < P; ++q) {
      const float4 v = red[q * T + t];
      m = make_float4(fmaxf(m.x, v.x), fmaxf(m.y, v.y), fmaxf(m.z, v.z), fmaxf(m.w, v.w));
    }
    atomicMax(out + 4 * t, __float_as_uint(m.x));
    atomicMax(out + 4 * t + 1, __float_as_uint(m.y));
    atomicMax(out + 4 * t + 2, __float_as_uint(m.z));
    atomicMax(out + 4 * t + 3, __float_as_uint(m.w));
  }
}

struct TnhArg {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  int64_t M;
  int Ma, Nb;
  int tiles_a, tiles_b, splits;
  int64_t rows_per_split;
  const unsigned* amax;  // [Ma] column maxima (IEEE bits of |v|)
  int aclamp;            // amax covers only the rows whose B row is nonzero: clamp A's scaled values
  const unsigned* bmax;  // B column n's bound: bmax[n % bperiod] * bscale
  int bperiod;
  float bscale;
  float* part;           // [splits, Ma, Nb]
  float* cpart;          // nullable: [splits, Ma] column sums of A (the workgroups of B tile 0)
};

__device__ __forceinline__ int th_off(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

using th_s16x4 = __attribute__((ext_vector_type(4))) short;
__device__ __forceinline__ uint2 th_tr16(const unsigned char* p) {
  const th_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) th_s16x4*)(p));
  return __builtin_bit_cast(uint2, v);
}

// 4 values times their column scales -> two fp16x4 terms (split2h's arithmetic); clamp: the
// scaled values limited to the fp16 range first (rows a caller's bound does not cover, whose
// product partners are zero: they add 0 instead of inf * 0)
__device__ __forceinline__ void split2h_4(const float4& v, const float4& s, uint2& h, uint2& l, bool clamp = false) {
  float e[4] = {v.x * s.x, v.y * s.y, v.z * s.z, v.w * s.w};
  if (clamp) {
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = fminf(fmaxf(e[i], -65504.f), 65504.f);
  }
  uint32_t hh[2], ll[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    hh[i] = split::pk_f16(e[2 * i], e[2 * i + 1]);
    const split::f32x2e back = __builtin_convertvector(__builtin_bit_cast(split::f16x2, hh[i]), split::f32x2e);
    ll[i] = split::pk_f16(e[2 * i] - back.x, e[2 * i + 1] - back.y);
  }
  h = make_uint2(hh[0], hh[1]);
  l = make_uint2(ll[0], ll[1]);
}

__global__ void __launch_bounds__(512, 1) k_gemm_tnh(TnhArg a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char th_lds[];
  float* const sFa = reinterpret_cast<float*>(th_lds + 2 * kThBuf);  // [0,128): 2^e, [128,256): 2^-e
  float* const sFb = sFa + 2 * 128;                                  // [0,256): 2^e, [256,512): 2^-e
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int wa = w & 3, wb = w >> 2;
  const int T = a.tiles_a * a.tiles_b;
  const int64_t b = blockIdx.x;
  const int64_t idx = b >> 3;
  const int tile = (int)(idx % T);
  const int64_t split = (b & 7) + 8 * (idx / T);  // one split's tiles share an XCD (and its L2)
  if (split >= a.splits) return;
  const int ta = tile % a.tiles_a, tb = tile / a.tiles_a;
  const int64_t r0 = split * a.rows_per_split;
  const int64_t r1 = min(a.M, r0 + a.rows_per_split);
  const int steps = r1 > r0 ? (int)((r1 - r0 + kTR - 1) / kTR) : 0;
  if (tid < 128) {
    const float m = __uint_as_float(a.amax[ta * 128 + tid]);
    const int e = (m > 0.f && m <= 3.4e38f) ? split::scale_exp16(m) : 0;
    sFa[tid] = ldexpf(1.f, e);
    sFa[128 + tid] = ldexpf(1.f, -e);
  }
  if (tid < 256) {
    const float m = __uint_as_float(a.bmax[(tb * 256 + tid) % a.bperiod]) * a.bscale;
    const int e = (m > 0.f && m <= 3.4e38f) ? split::scale_exp16(m) : 0;
    sFb[tid] = ldexpf(1.f, e);
    sFb[256 + tid] = ldexpf(1.f, -e);
  }
  __syncthreads();

  // ---- staging: thread t -> rows t / 32 and t / 32 + 16 of the chunk, columns 4 (t % 32) .. +3
  // of the A tile and of both B halves ----
  const int sc = (tid & 31) * 4, slr = tid >> 5;
  const float4 sa = *reinterpret_cast<const float4*>(sFa + sc);
  const float4 sb0 = *reinterpret_cast<const float4*>(sFb + sc);
  const float4 sb1 = *reinterpret_cast<const float4*>(sFb + 128 + sc);
  const float* const Ab = a.A + ta * 128 + sc;
  const float* const Bb = a.B + tb * 256 + sc;
  struct Stage {
    float4 a[2], b0[2], b1[2];
  };
  auto load = [&](int64_t row0, Stage& S) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int64_t row = min(row0 + slr + 16 * p, r1 - 1);
      S.a[p] = ld4(Ab + row * a.lda);
      S.b0[p] = ld4(Bb + row * a.ldb);
      S.b1[p] = ld4(Bb + row * a.ldb + 128);
    }
  };
  // column sums of A over this split's rows (cpart; the B tile 0 workgroups of each A tile): the
  // staging thread's 4 columns over its rows in chunk order, the raw values (before any clamp),
  // kept in its own LDS slot sC[slr][sc .. +3] (no registers held across the loop)
  const bool csum = a.cpart != nullptr && tb == 0;
  float4* const sCs = reinterpret_cast<float4*>(sFb + 2 * 256) + slr * 32 + (sc >> 2);  // sC: [16][128]
  if (csum) *sCs = f4(0.f);
  auto put = [&](int buf, int64_t row0, const Stage& S) {
    unsigned char* img = th_lds + buf * kThBuf;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int lr = slr + 16 * p;
      const bool ok = row0 + lr < r1;
      const int off = th_off(lr, sc >> 3) + 8 * ((sc >> 2) & 1);
      if (csum && ok) {
        const float4 c = *sCs;
        *sCs = make_float4(c.x + S.a[p].x, c.y + S.a[p].y, c.z + S.a[p].z, c.w + S.a[p].w);
      }
      uint2 h, l;
      split2h_4(ok ? S.a[p] : f4(0.f), sa, h, l, a.aclamp != 0);
      *reinterpret_cast<uint2*>(img + off) = h;
      *reinterpret_cast<uint2*>(img + kThImg + off) = l;
      split2h_4(ok ? S.b0[p] : f4(0.f), sb0, h, l);
      *reinterpret_cast<uint2*>(img + 2 * kThImg + off) = h;
      *reinterpret_cast<uint2*>(img + 3 * kThImg + off) = l;
      split2h_4(ok ? S.b1[p] : f4(0.f), sb1, h, l);
      *reinterpret_cast<uint2*>(img + 4 * kThImg + off) = h;
      *reinterpret_cast<uint2*>(img + 5 * kThImg + off) = l;
    }
  };

  // transposed-read lane address (see k_dxw): lane 4 q + p of 16-lane group g reads row q of a
  // 4-row block, columns 4 p .. +3 of the group's 16 (16 (g & 1) within a 32-column block)
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  int oa[4], ob[4][4];  // [2 ks + t] for A; [t'][2 ks + t] for B's four blocks (image-relative)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = 16 * (u >> 1) + 8 * (tg >> 1) + 4 * (u & 1) + tq;
    const int ca = 32 * wa + 16 * (tg & 1) + 4 * tp;
    oa[u] = th_off(row, ca >> 3) + 8 * ((ca >> 2) & 1);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int cb = 32 * t + 16 * (tg & 1) + 4 * tp;
      ob[t][u] = th_off(row, cb >> 3) + 8 * ((cb >> 2) & 1);
    }
  }
  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x16{};

  auto compute = [&](const int buf) {
    const unsigned char* img = th_lds + buf * kThBuf;
    const unsigned char* bimg = img + (2 + 2 * wb) * kThImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      split::u32x4 fa[2], fb[4][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint2 v = th_tr16(img + e * kThImg + oa[2 * ks + t]);
          fa[e][2 * t] = v.x;
          fa[e][2 * t + 1] = v.y;
        }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint2 v = th_tr16(bimg + e * kThImg + ob[q][2 * ks + t]);
            fb[q][e][2 * t] = v.x;
            fb[q][e][2 * t + 1] = v.y;
          }
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = split::mfma32_h3(fa, fb[q], acc[q]);
    }
  };

  // two register stages (S0 / S1): chunks c + 1 and c + 2 are in flight while chunk c computes
  // (one stage left the kernel waiting on HBM latency: 48 KB in flight per CU)
  Stage S0, S1;
  if (steps > 0) {
    load(r0, S0);
    load(r0 + kTR, S1);
    put(0, r0, S0);
    __syncthreads();
  }
  for (int st = 0; st < steps; st += 2) {
    load(r0 + (int64_t)(st + 2) * kTR, S0);
    compute(0);
    if (st + 1 < steps) put(1, r0 + (int64_t)(st + 1) * kTR, S1);
    __syncthreads();
    if (st + 1 >= steps) break;
    load(r0 + (int64_t)(st + 3) * kTR, S1);
    compute(1);
    if (st + 2 < steps) put(0, r0 + (int64_t)(st + 2) * kTR, S0);
    __syncthreads();
  }
  // ---- unscale (exact powers of two) and store this split's partial ----
  float* P = a.part + (size_t)split * a.Ma * a.Nb;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int nl = 128 * wb + 32 * t + r;
    const float fb = sFb[256 + nl];
    const int col = tb * 256 + nl;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ml = 32 * wa + (q & 3) + 8 * (q >> 2) + 4 * hf;
      P[(size_t)(ta * 128 + ml) * a.Nb + col] = acc[t][q] * sFa[128 + ml] * fb;
    }
  }
  if (csum) {  // (workgroup-uniform) the 16 row threads of each column in row-thread order
    const float* sC = sFb + 2 * 256;
    __syncthreads();
    if (tid < 128) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) s += sC[q * 128 + tid];
      a.cpart[(size_t)split * a.Ma + ta * 128 + tid] = s;
    }
  }
}

// ---------------------------------------------------------------------------
// k_gemm_tnh256: k_gemm_tnh with a 256 x 256 output tile (A's 256 columns x B's 256) when Ma is a
// multiple of 256 (config 5's weight gradient G = g^T agg: Ma = 256, Nb = 1024).  The 128 x 256
// tile split every staged A row once per B tile (four times) and every B row once per A tile
// (twice): 3,072 fp16 splits per row of the product against 2,048 here (A four times, B once).
// 16 waves (1,024 threads, four per SIMD, <= 128 registers): wave w owns A block w & 7 (32
// columns) x B half w >> 3 (128 columns), acc[4] as in k_gemm_tnh; threads 0-511 stage the two
// A halves, 512-1023 the two B halves, two rows x four columns of each per thread, one register
// stage (chunk c + 1 loads while chunk c computes).  LDS: two buffers of eight [32][128] fp16
// images (A half 0/1 and B half 0/1, hi/lo each) = 128 KB, + scales + colsum slots.  The row
// splits are tnh_splits(M, tiles of the 128 x 256 kernel) and every output element takes
// k_gemm_tnh's products in k_gemm_tnh's order: the same bits (tests/test_gpu_gemm_f16.py).
// ---------------------------------------------------------------------------
constexpr int kTh2Buf = 8 * kThImg;  // 64 KB
constexpr size_t kTh2Lds = 2 * kTh2Buf + (2 * 256 + 2 * 256 + 16 * 256) * sizeof(float);

__global__ void __launch_bounds__(1024, 1) k_gemm_tnh256(TnhArg a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char th_lds[];
  float* const sFa = reinterpret_cast<float*>(th_lds + 2 * kTh2Buf);  // [0,256): 2^e, [256,512): 2^-e
  float* const sFb = sFa + 2 * 256;                                   // [0,256): 2^e, [256,512): 2^-e
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int wa = w & 7, wb = w >> 3;
  const int T = a.tiles_a * a.tiles_b;
  const int64_t b = blockIdx.x;
  const int64_t idx = b >> 3;
  const int tile = (int)(idx % T);
  const int64_t split = (b & 7) + 8 * (idx / T);  // one split's tiles share an XCD (and its L2)
  if (split >= a.splits) return;
  const int ta = tile % a.tiles_a, tb = tile / a.tiles_a;
  const int64_t r0 = split * a.rows_per_split;
  const int64_t r1 = min(a.M, r0 + a.rows_per_split);
  const int steps = r1 > r0 ? (int)((r1 - r0 + kTR - 1) / kTR) : 0;
  if (tid < 256) {
    const float m = __uint_as_float(a.amax[ta * 256 + tid]);
    const int e = (m > 0.f && m <= 3.4e38f) ? split::scale_exp16(m) : 0;
    sFa[tid] = ldexpf(1.f, e);
    sFa[256 + tid] = ldexpf(1.f, -e);
  } else if (tid < 512) {
    const int c = tid - 256;
    const float m = __uint_as_float(a.bmax[(tb * 256 + c) % a.bperiod]) * a.bscale;
    const int e = (m > 0.f && m <= 3.4e38f) ? split::scale_exp16(m) : 0;
    sFb[c] = ldexpf(1.f, e);
    sFb[256 + c] = ldexpf(1.f, -e);
  }
  __syncthreads();

  // ---- staging: thread t -> operand t >> 9 (A / B), rows (t >> 5) & 15 and + 16 of the chunk,
  // columns 4 (t % 32) .. +3 of both 128-column halves of that operand ----
  const int sc = (tid & 31) * 4, slr = (tid >> 5) & 15, isb = tid >> 9;
  const float* const src = isb ? a.B + tb * 256 + sc : a.A + ta * 256 + sc;
  const int64_t ld = isb ? a.ldb : a.lda;
  const float* const scl = (isb ? sFb : sFa) + sc;
  const bool clamp = !isb && a.aclamp != 0;
  float4 S[2][2];  // [row p][half]
  auto load = [&](int64_t row0) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int64_t row = min(row0 + slr + 16 * p, r1 - 1);
      S[p][0] = ld4(src + row * ld);
      S[p][1] = ld4(src + row * ld + 128);
    }
  };
  // column sums of A (cpart; the B tile 0 workgroups): the A staging thread's 4 columns of each
  // half over its rows in chunk order, raw values, in its own LDS slots sC[slr][256]
  const bool csum = a.cpart != nullptr && tb == 0 && !isb;
  float4* const sCs = reinterpret_cast<float4*>(sFb + 2 * 256) + slr * 64 + (sc >> 2);  // sC: [16][256]
  if (csum) {
    sCs[0] = f4(0.f);
    sCs[32] = f4(0.f);
  }
  auto put = [&](int buf, int64_t row0) {
    unsigned char* img = th_lds + buf * kTh2Buf + 4 * isb * kThImg;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int lr = slr + 16 * p;
      const bool ok = row0 + lr < r1;
      const int off = th_off(lr, sc >> 3) + 8 * ((sc >> 2) & 1);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if (csum && ok) {
          const float4 c = sCs[32 * hh];
          sCs[32 * hh] = make_float4(c.x + S[p][hh].x, c.y + S[p][hh].y, c.z + S[p][hh].z, c.w + S[p][hh].w);
        }
        uint2 h, l;
        split2h_4(ok ? S[p][hh] : f4(0.f), *reinterpret_cast<const float4*>(scl + 128 * hh), h, l, clamp);
        *reinterpret_cast<uint2*>(img + 2 * hh * kThImg + off) = h;
        *reinterpret_cast<uint2*>(img + (2 * hh + 1) * kThImg + off) = l;
      }
    }
  };

  // transposed-read lane address (as k_gemm_tnh): lane 4 q + p of 16-lane group g reads row q of
  // a 4-row block, columns 4 p .. +3 of the group's 16 (16 (g & 1) within a 32-column block)
  // th_off(row, (32 blk + c0) >> 3) + 8 ((c0 >> 2) & 1) with c0 = 16 (tg & 1) + 4 tp splits into a
  // row part and a block part: the row's swizzle is (tq << 2) | (2 (tg >> 1) + (u & 1)) for every
  // row this lane reads, so block blk sits at 64 (blk ^ tq) -- 9 registers instead of 20
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  const int c0 = 16 * (tg & 1) + 4 * tp;
  int obase[4], oq[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = 16 * (u >> 1) + 8 * (tg >> 1) + 4 * (u & 1) + tq;
    obase[u] = 256 * row + 16 * ((c0 >> 3) ^ (2 * (tg >> 1) + (u & 1))) + 8 * ((c0 >> 2) & 1);
    oq[u] = 64 * (u ^ tq);
  }
  const int oqa = 64 * ((wa & 3) ^ tq);
  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x16{};

  auto compute = [&](const int buf) {
    const unsigned char* img = th_lds + buf * kTh2Buf;
    const unsigned char* aimg = img + 2 * (wa >> 2) * kThImg;
    const unsigned char* bimg = img + (4 + 2 * wb) * kThImg;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      split::u32x4 fa[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint2 v = th_tr16(aimg + e * kThImg + obase[2 * ks + t] + oqa);
          fa[e][2 * t] = v.x;
          fa[e][2 * t + 1] = v.y;
        }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        split::u32x4 fb[2];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint2 v = th_tr16(bimg + e * kThImg + obase[2 * ks + t] + oq[q]);
            fb[e][2 * t] = v.x;
            fb[e][2 * t + 1] = v.y;
          }
        acc[q] = split::mfma32_h3(fa, fb, acc[q]);
      }
    }
  };

  if (steps > 0) {
    load(r0);
    put(0, r0);
    __syncthreads();
  }
  for (int st = 0; st < steps; ++st) {
    const bool more = st + 1 < steps;
    if (more) load(r0 + (int64_t)(st + 1) * kTR);
    compute(st & 1);
    if (more) put((st + 1) & 1, r0 + (int64_t)(st + 1) * kTR);
    __syncthreads();
  }
  // ---- unscale (exact powers of two) and store this split's partial ----
  float* P = a.part + (size_t)split * a.Ma * a.Nb;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int nl = 128 * wb + 32 * t + r;
    const float fb = sFb[256 + nl];
    const int col = tb * 256 + nl;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ml = 32 * wa + (q & 3) + 8 * (q >> 2) + 4 * hf;
      P[(size_t)(ta * 256 + ml) * a.Nb + col] = acc[t][q] * sFa[256 + ml] * fb;
    }
  }
  if (a.cpart != nullptr && tb == 0) {  // (workgroup-uniform) the 16 row threads of each column in order
    const float* sC = sFb + 2 * 256;
    __syncthreads();
    if (tid < 256) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) s += sC[q * 256 + tid];
      a.cpart[(size_t)split * a.Ma + ta * 256 + tid] = s;
    }
  }
}

// ===========================================================================
// aggregate-then-transform layer pieces
// ===========================================================================
// A[v][h][k] = sum_c att_v[h][c] W[h C + c][k]  (v = 0: src, 1: dst) -> [2, H, K]
// (16 outputs per block, the c sum split over 16 threads in fixed 16-wide chunks and combined in
// chunk order: 128 blocks instead of eight, each with 256-long serial chains, which left the
// kernel at 98 us)
__global__ void __launch_bounds__(256) k_att_proj(const float* __restrict__ W, const float* __restrict__ att_src,
                                                  const float* __restrict__ att_dst, int H, int C, int K,
                                                  float* __restrict__ A) {
  __shared__ float red[16][16];
  const int kl = threadIdx.x & 15, cq = threadIdx.x >> 4;
  const int64_t t = (int64_t)blockIdx.x * 16 + kl;
  const bool live = t < (int64_t)2 * H * K;
  float s = 0.f;
  if (live) {
    const int v = (int)(t / ((int64_t)H * K));
    const int h = (int)((t / K) % H), k = (int)(t % K);
    const float* att = (v == 0 ? att_src : att_dst) + h * C;
    const int cw = (C + 15) / 16, c0 = cq * cw, c1 = min(C, c0 + cw);
    for (int c = c0; c < c1; ++c) s = fmaf(att[c], W[(int64_t)(h * C + c) * K + k], s);
  }
  red[cq][kl] = s;
  __syncthreads();
  if (cq == 0 && live) {
    float a = red[0][kl];
#pragma unroll
    for (int q = 1; q < 16; ++q) a += red[q][kl];
    A[t] = a;
  }
}

// Wt[h K + k][c] = W[h C + c][k]  (the transform, [H K, C]) and Wg[c][h K + k] = W[h C + c][k] / H
__global__ void __launch_bounds__(256) k_wperm(const float* __restrict__ W, int H, int C, int K,
                                               float* __restrict__ Wt, float* __restrict__ Wg) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)H * C * K) return;
  const int hc = (int)(t / K), k = (int)(t % K);
  const int h = hc / C, c = hc % C;
  const float w = W[t];
  if (Wt) Wt[((int64_t)h * K + k) * C + c] = w;
  if (Wg) Wg[(int64_t)c * H * K + (int64_t)h * K + k] = w * (1.f / (float)H);
}

// s_src[n][h] = x_n . A_src[h] (n < n_rows), s_dst[n][h] = x_n . A_dst[h] (n < n_dst).
// K = 256: a row is one float4 per lane; a wave takes 4 rows per iteration (their loads in
// flight together), and each row's 2H lane partials are summed by one transposing butterfly
// (lanes 64 / 2H * v .. hold score v): 2H - 1 exchanges + a short reduction instead of 2H
// full-wave reductions.  (One row at a time with 2H six-step reductions ran at 3.0 TB/s.)
template <int K, int H>
__global__ void __launch_bounds__(256) k_xscores(const float* __restrict__ x, int64_t ldx, int64_t n_rows,
                                                 int64_t n_dst, const float* __restrict__ A, float* __restrict__ s_src,
                                                 float* __restrict__ s_dst) {
  static_assert(K == 256 && (H == 2 || H == 4), "k_xscores: K = 256, H in {2, 4}");
  constexpr int V = 2 * H, R = 4, LV = 64 / V;
  const int lane = threadIdx.x & 63;
  float4 av[V];
#pragma unroll
  for (int v = 0; v < V; ++v) av[v] = ld4(A + v * K + lane * 4);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int vi = lane / LV;  // the score this lane ends with
  for (int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * R; base < n_rows; base += nw * R) {
    float4 xv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t n = base + r;
      xv[r] = ld4(x + (n < n_rows ? n : n_rows - 1) * ldx + lane * 4);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float pv[V];
#pragma unroll
      for (int v = 0; v < V; ++v) pv[v] = dot4(xv[r], av[v]);
      const float sum = transpose_reduce<64, V>(pv, lane);
      const int64_t n = base + r;
      if (n < n_rows && lane % LV == 0) {
        if (vi < H) s_src[n * H + vi] = sum;
        else if (n < n_dst) s_dst[n * H + vi - H] = sum;
      }
    }
  }
}

struct XItems {
  const int32_t* row;
  const int32_t* beg;
  const int32_t* end;
  int64_t n_items;
  int64_t n_hub_items;
};

// ---------------------------------------------------------------------------
// forward edge pass: one wave per destination item (CSR), the neighbour row x_j (K floats)
// gathered ONCE per edge for all H heads: ax^h += p^h x_j with the online softmax per head.
// K = 256: one float4 per lane, one edge at a time across the wave, U rows in flight.
// Hub pieces leave [ax^h (K) | m | l | - -] per (item, head) for k_fwd_merge_wg.
// ---------------------------------------------------------------------------
// U rows in flight per wave: 4 (96 VGPRs, five waves per SIMD) -- 8 rows (144 VGPRs, three waves)
// left the pass at 7.1 ms per call on the config-5 share, 4 gives 6.0-6.3 (profiles/r06/x2/x3_bench5_fwdx_u*.log;
// 2, 3 and 6 within noise of 4); the FMA order per lane is the same for every U (same bits)
template <int K, int H, int U = 4>
__global__ void __launch_bounds__(256) k_fwd_x(XItems it, const int32_t* __restrict__ col,
                                               const int32_t* __restrict__ eid, const float* __restrict__ x,
                                               int64_t ldx, const float* __restrict__ s_src,
                                               const float* __restrict__ s_dst, float slope, float p, float inv_keep,
                                               uint64_t seed, const uint64_t* __restrict__ seed_in,
                                               float* __restrict__ agg, float* __restrict__ m_out,
                                               float* __restrict__ invl_out, float* __restrict__ partial,
                                               unsigned* __restrict__ xmax) {
  // xmax != NULL: the column maxima of |x_j| over the gathered rows (every source of an edge)
  // merged into it -- the bound of |agg| the weight gradient's fp16 split needs, for free
  static_assert(K == 256, "k_fwd_x: K == 256 (one float4 per lane)");
  if (p > 0.f) seed = *seed_in;
  __shared__ int recj[4][64];
  __shared__ float recw[4][H][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;
  if (w >= it.n_items) return;
  const int64_t i = it.row[w];
  const int rs = it.beg[w], re = it.end[w];
  const bool hub = w < it.n_hub_items;
  float sd[H], mh[H], lh[H];
  float4 acc[H];
  float4 xm = f4(0.f);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    sd[h] = s_dst[i * H + h];
    mh[h] = -INFINITY;
    lh[h] = 0.f;
    acc[h] = f4(0.f);
  }
  for (int base = rs; base < re; base += 64) {
    const int k = base + lane;
    const bool valid = k < re;
    const int j = valid ? col[k] : 0;
    const uint32_t e_id = (valid && p > 0.f) ? (uint32_t)eid[k] : 0u;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float e = valid ? lrelu(s_src[(int64_t)j * H + h] + sd[h], slope) : -INFINITY;
      const float mn = fmaxf(mh[h], wave_max(e));
      const float sc = expf(mh[h] - mn);
      const float pe = valid ? expf(e - mn) : 0.f;
      lh[h] = fmaf(lh[h], sc, wave_sum(pe));
      acc[h] = mul4(acc[h], sc);
      mh[h] = mn;
      float pw = pe;
      if (p > 0.f && valid) pw *= drop_scale(seed, e_id, (uint32_t)h, p, inv_keep);
      recw[wv][h][lane] = pw;
    }
    recj[wv][lane] = j;
    wave_sync();
    const int n = min(64, re - base);
    for (int q0 = 0; q0 < n; q0 += U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u;
        v[u] = q < n ? ld4(x + (int64_t)recj[wv][q] * ldx + lane * 4) : f4(0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = min(q0 + u, 63);
#pragma unroll
        for (int h = 0; h < H; ++h) acc[h] = fma4(q0 + u < n ? recw[wv][h][q] : 0.f, v[u], acc[h]);
        xm = absmax4(xm, v[u]);
      }
    }
    wave_sync();
  }
  if (xmax != nullptr) colmax_merge4(xmax, lane * 4, xm);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    if (hub) {
      float* slot = partial + (w * H + h) * (K + 4);
      st4(slot + lane * 4, acc[h]);
      if (lane == 0) st4(slot + K, make_float4(mh[h], lh[h], 0.f, 0.f));
      continue;
    }
    const float invl = 1.f / (lh[h] + 1e-16f);
    st4(agg + (i * H + h) * K + lane * 4, mul4(acc[h], invl));
    if (lane == 0) {
      m_out[i * H + h] = re > rs ? mh[h] : 0.f;
      invl_out[i * H + h] = invl;
    }
  }
}

// backward prologue: nstate[i][h] = {s_dst, m, inv_l, D = gt_i^h . ax_i^h}; one wave per row
template <int K, int H>
__global__ void __launch_bounds__(256) k_bwd_x_pro(const float* __restrict__ gt, const float* __restrict__ agg,
                                                   const float* __restrict__ s_dst, const float* __restrict__ m,
                                                   const float* __restrict__ invl, int64_t n,
                                                   float4* __restrict__ nstate) {
  static_assert(K == 256, "k_bwd_x_pro: K == 256");
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += nw) {
    float d[16];
#pragma unroll
    for (int h = 0; h < 16; ++h) d[h] = 0.f;
#pragma unroll
    for (int h = 0; h < H; ++h)
      d[h] = dot4(ld4(gt + (i * H + h) * K + lane * 4), ld4(agg + (i * H + h) * K + lane * 4));
#pragma unroll
    for (int h = 0; h < H; ++h) d[h] = wave_sum(d[h]);
    if (lane < H) {
      float dv = d[0];
#pragma unroll
      for (int h = 1; h < H; ++h) dv = lane == h ? d[h] : dv;
      const int64_t pr = i * H + lane;
      nstate[pr] = make_float4(s_dst[pr], m[pr], invl[pr], dv);
    }
  }
}

// ---------------------------------------------------------------------------
// backward edge pass by SOURCE (CSC): one wave per source item; x_j in registers (float4
// per lane), per out-edge the destination's gt_i (H x K floats) and packed state gathered
// once.  Per group of 4 edges the 16 partial dots <gt_i^h, x_j> are summed over the wave
// with a transposing butterfly.  Writes dx_j = sum beta gt + sum_h ds_src^h A_src^h (hub
// pieces: [msg (K) | ds_h (H <= 4)] partials), ds_src[j][h], and dz at each edge's CSR slot.
// ---------------------------------------------------------------------------
template <int OFF, int N>
__device__ __forceinline__ int tr_reduce(float (&v)[16], int sl, int& base) {
  if constexpr (OFF >= 8 && N > 1) {
    constexpr int Hh = N / 2;
    const bool bit = (sl & OFF) != 0;
#pragma unroll
    for (int t = 0; t < Hh; ++t) {
      if constexpr (OFF >= 16) {
        float r0, r1;
        row_swap<OFF>(v[t], v[Hh + t], r0, r1);
        v[t] = r0 + r1;
      } else {
        const float send = bit ? v[t] : v[Hh + t];
        const float keep = bit ? v[Hh + t] : v[t];
        v[t] = keep + dpp<0x128>(send);
      }
    }
    if (bit) base += Hh;
    return tr_reduce<OFF / 2, Hh>(v, sl, base);
  } else {
#pragma unroll
    for (int t = 0; t < N; ++t) v[t] = group_reduce<Op::Sum, 1, 4>(v[t]);
    return N;
  }
}

template <int K, int H>
__global__ void __launch_bounds__(256) k_bwd_x(XItems it, const int32_t* __restrict__ row,
                                               const int32_t* __restrict__ csc_eid,
                                               const int32_t* __restrict__ csc2csr, const float* __restrict__ x,
                                               int64_t ldx, const float* __restrict__ s_src,
                                               const float4* __restrict__ nstate, const float* __restrict__ gt,
                                               const float* __restrict__ A_src, float slope, float p, float inv_keep,
                                               uint64_t seed, const uint64_t* __restrict__ seed_in,
                                               float* __restrict__ dx, int64_t lddx, float* __restrict__ S,
                                               int64_t lds, float* __restrict__ dz, float* __restrict__ partial) {
  static_assert(K == 256 && H <= 4, "k_bwd_x: K == 256, H <= 4");
  constexpr int U = 16 / H;  // edges per reduction group (16 partial dots per lane)
  if (p > 0.f) seed = *seed_in;
  __shared__ int2 recA[4][64];          // {dst row, CSR slot}
  __shared__ float4 recH[4][H][64];     // per head {beta, c1, c0, -}
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;
  if (w >= it.n_items) return;
  const int64_t j = it.row[w];
  const int cs = it.beg[w], ce = it.end[w];
  const bool hub = w < it.n_hub_items;
  const float4 xv = ld4(x + j * ldx + lane * 4);
  float ss[H], dsa[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    ss[h] = s_src[j * H + h];
    dsa[h] = 0.f;
  }
  float4 acc = f4(0.f);
  for (int base = cs; base < ce; base += 64) {
    const int k = base + lane;
    const bool valid = k < ce;
    const int i = valid ? row[k] : 0;
    const int slot = valid ? (csc2csr != nullptr ? csc2csr[k] : k) : 0;  // NULL: dz in CSC order
    const uint32_t e_id = (valid && p > 0.f) ? (uint32_t)csc_eid[k] : 0u;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float bg = 0.f, c1 = 0.f, c0 = 0.f;
      if (valid) {
        const float4 st = nstate[(int64_t)i * H + h];  // {s_dst, m, inv_l, D}
        const float z = ss[h] + st.x;
        const float af = expf(lrelu(z, slope) - st.y) * st.z;
        const float dm = p > 0.f ? drop_scale(seed, e_id, (uint32_t)h, p, inv_keep) : 1.f;
        bg = af * dm;
        const float a1 = af * dlrelu(z, slope);
        c1 = a1 * dm;
        c0 = a1 * st.w;
      }
      recH[wv][h][lane] = make_float4(bg, c1, c0, 0.f);
    }
    recA[wv][lane] = make_int2(i, slot);
    wave_sync();
    const int n = min(64, ce - base);
    for (int q0 = 0; q0 < n; q0 += U) {
      float4 g[U][H];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u;
        const int64_t ii = recA[wv][min(q, 63)].x;
#pragma unroll
        for (int h = 0; h < H; ++h) g[u][h] = q < n ? ld4(gt + (ii * H + h) * K + lane * 4) : f4(0.f);
      }
      float part[16];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = min(q0 + u, 63);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const float bq = q0 + u < n ? recH[wv][h][q].x : 0.f;
          acc = fma4(bq, g[u][h], acc);
          part[u * H + h] = dot4(g[u][h], xv);
        }
      }
      int vbase = 0;
      const int R = tr_reduce<32, 16>(part, lane, vbase);
      const int t = lane & 7;
      if (t < R) {
        float dot = part[0];
#pragma unroll
        for (int c = 1; c < 8; ++c)
          if (c == t) dot = part[c];
        const int vi = vbase + t;
        const int u = vi / H, h = vi % H;
        const int q = q0 + u;
        if (q < n) {
          const float4 rb = recH[wv][h][q];
          const float dzv = fmaf(rb.y, dot, -rb.z);
#pragma unroll
          for (int c = 0; c < H; ++c)
            if (c == h) dsa[c] += dzv;
          dz[(int64_t)recA[wv][q].y * H + h] = dzv;
        }
      }
    }
    wave_sync();
  }
  float ds[H];
#pragma unroll
  for (int h = 0; h < H; ++h) ds[h] = wave_sum(dsa[h]);
  if (hub) {
    float* sp = partial + w * (K + 4);
    st4(sp + lane * 4, acc);
    if (lane == 0) {
      float4 d = f4(0.f);
      d.x = ds[0];
      if (H > 1) d.y = ds[1];
      if (H > 2) d.z = ds[2];
      if (H > 3) d.w = ds[3];
      st4(sp + K, d);
    }
    return;
  }
#pragma unroll
  for (int h = 0; h < H; ++h) acc = fma4(ds[h], ld4(A_src + h * K + lane * 4), acc);
  st4(dx + j * lddx + lane * 4, acc);
  if (lane < H) {
    float v = ds[0];
#pragma unroll
    for (int h = 1; h < H; ++h) v = lane == h ? ds[h] : v;
    S[j * lds + lane] = v;
  }
}

// hub sources: sum the pieces in order, add the attention term
template <int K, int H>
__global__ void __launch_bounds__(256) k_bwd_x_merge(const int32_t* __restrict__ hub_row,
                                                     const int32_t* __restrict__ hub_ptr, int64_t n_hubs,
                                                     const float* __restrict__ partial, const float* __restrict__ A_src,
                                                     float* __restrict__ dx, int64_t lddx, float* __restrict__ S,
                                                     int64_t lds) {
  const int lane = threadIdx.x & 63;
  const int64_t hb = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (hb >= n_hubs) return;
  const int64_t j = hub_row[hb];
  float4 acc = f4(0.f), d = f4(0.f);
  for (int q = hub_ptr[hb]; q < hub_ptr[hb + 1]; ++q) {
    acc = add4(acc, ld4(partial + (int64_t)q * (K + 4) + lane * 4));
    d = add4(d, ld4(partial + (int64_t)q * (K + 4) + K));
  }
  const float ds[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
  for (int h = 0; h < H; ++h) acc = fma4(ds[h], ld4(A_src + h * K + lane * 4), acc);
  st4(dx + j * lddx + lane * 4, acc);
  if (lane < H) S[j * lds + lane] = ds[lane];
}

// ---------------------------------------------------------------------------
// The backward edge pass gathering g_i (C floats per edge) instead of gt_i (H x C_in):
// dalpha^h_ij = gt^h_i . x_j = g_i . hs^h_j with hs^h_j = W_h x_j / H (one GEMM over the
// sources, read once per source here), and the message gradient is accumulated per head as
// acc^h_j = sum_i beta^h_ij g_i (written once per source, [n_src, H, C]); then
// dx_j = acc_j . W (one NN GEMM, rows h C + c of W = W_h) + the attention terms.  Per edge
// 1 KB instead of 4 KB of gathers at config 5.  Summation orders as k_bwd_x (edges in CSC
// order, hub pieces merged in piece order): deterministic.
// ---------------------------------------------------------------------------
template <int C, int H>
__global__ void __launch_bounds__(256) k_bwd_g(XItems it, const int32_t* __restrict__ row,
                                               const int32_t* __restrict__ csc_eid,
                                               const int32_t* __restrict__ csc2csr, const float* __restrict__ hs,
                                               const float* __restrict__ s_src, const float4* __restrict__ nstate,
                                               const float* __restrict__ g, int64_t ldg, float slope, float p,
                                               float inv_keep, uint64_t seed, const uint64_t* __restrict__ seed_in,
                                               float* __restrict__ acc_out, float* __restrict__ S, int64_t lds,
                                               float* __restrict__ dz, float* __restrict__ partial,
                                               float* __restrict__ pz, unsigned* __restrict__ gmax) {
  // pz != NULL (deferred D): dz receives dalpha = g_i . hs_j and pz beta * dalpha per edge and
  // head (D_i = sum_j beta dalpha by a destination sum, dz by k_xgat_dz); no ds_src here.
  // gmax != NULL: the column maxima of |g_i| over the gathered rows (every destination of an
  // edge) merged into it
  static_assert(C == 256 && H <= 4, "k_bwd_g: C == 256, H <= 4");
  constexpr int U = 16 / H;  // edges per reduction group (16 partial dots per lane)
  if (p > 0.f) seed = *seed_in;
  __shared__ int2 recA[4][64];          // {dst row, dz slot}
  __shared__ float4 recH[4][H][64];     // per head {beta, c1, c0, -}
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * 4 + wv;
  if (w >= it.n_items) return;
  const int64_t j = it.row[w];
  const int cs = it.beg[w], ce = it.end[w];
  const bool hub = w < it.n_hub_items;
  float4 hv[H], acc[H];
  float4 gm = f4(0.f);
  float ss[H], dsa[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    hv[h] = ld4(hs + (j * H + h) * C + lane * 4);
    acc[h] = f4(0.f);
    ss[h] = s_src[j * H + h];
    dsa[h] = 0.f;
  }
  for (int base = cs; base < ce; base += 64) {
    const int k = base + lane;
    const bool valid = k < ce;
    const int i = valid ? row[k] : 0;
    const int slot = valid ? (csc2csr != nullptr ? csc2csr[k] : k) : 0;  // NULL: dz in CSC order
    const uint32_t e_id = (valid && p > 0.f) ? (uint32_t)csc_eid[k] : 0u;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float bg = 0.f, c1 = 0.f, c0 = 0.f;
      if (valid) {
        const float4 st = nstate[(int64_t)i * H + h];  // {s_dst, m, inv_l, D}
        const float z = ss[h] + st.x;
        const float af = expf(lrelu(z, slope) - st.y) * st.z;
        const float dm = p > 0.f ? drop_scale(seed, e_id, (uint32_t)h, p, inv_keep) : 1.f;
        bg = af * dm;
        const float a1 = af * dlrelu(z, slope);
        c1 = a1 * dm;
        c0 = a1 * st.w;
      }
      recH[wv][h][lane] = make_float4(bg, c1, c0, 0.f);
    }
    recA[wv][lane] = make_int2(i, slot);
    wave_sync();
    const int n = min(64, ce - base);
    for (int q0 = 0; q0 < n; q0 += U) {
      float4 gq[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u;
        const int64_t ii = recA[wv][min(q, 63)].x;
        gq[u] = q < n ? ld4(g + ii * ldg + lane * 4) : f4(0.f);
        gm = absmax4(gm, gq[u]);
      }
      float part[16];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = min(q0 + u, 63);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const float bq = q0 + u < n ? recH[wv][h][q].x : 0.f;
          acc[h] = fma4(bq, gq[u], acc[h]);
          part[u * H + h] = dot4(gq[u], hv[h]);
        }
      }
      int vbase = 0;
      const int R = tr_reduce<32, 16>(part, lane, vbase);
      const int t = lane & 7;
      if (t < R) {
        float dot = part[0];
#pragma unroll
        for (int c = 1; c < 8; ++c)
          if (c == t) dot = part[c];
        const int vi = vbase + t;
        const int u = vi / H, h = vi % H;
        const int q = q0 + u;
        if (q < n) {
          const float4 rb = recH[wv][h][q];
          const int64_t o = (int64_t)recA[wv][q].y * H + h;
          if (pz != nullptr) {
            dz[o] = dot;
            pz[o] = rb.x * dot;
          } else {
            const float dzv = fmaf(rb.y, dot, -rb.z);
#pragma unroll
            for (int c = 0; c < H; ++c)
              if (c == h) dsa[c] += dzv;
            dz[o] = dzv;
          }
        }
      }
    }
    wave_sync();
  }
  if (gmax != nullptr) colmax_merge4(gmax, lane * 4, gm);
  float ds[H];
#pragma unroll
  for (int h = 0; h < H; ++h) ds[h] = wave_sum(dsa[h]);
  if (hub) {
    float* sp = partial + w * (H * C + 4);
#pragma unroll
    for (int h = 0; h < H; ++h) st4(sp + h * C + lane * 4, acc[h]);
    if (lane == 0) {
      float4 d = f4(0.f);
      d.x = ds[0];
      if (H > 1) d.y = ds[1];
      if (H > 2) d.z = ds[2];
      if (H > 3) d.w = ds[3];
      st4(sp + H * C, d);
    }
    return;
  }
#pragma unroll
  for (int h = 0; h < H; ++h) st4(acc_out + (j * H + h) * C + lane * 4, acc[h]);
  if (lane < H && S != nullptr) {  // deferred D: ds_src comes from k_xgat_dz
    float v = ds[0];
#pragma unroll
    for (int h = 1; h < H; ++h) v = lane == h ? ds[h] : v;
    S[j * lds + lane] = v;
  }
}

// nstate[i][h] = {s_dst, m, inv_l, D or 0} (the deferred-D backward builds it twice: without D
// for k_bwd_g, with D for k_xgat_dz)
__global__ void __launch_bounds__(256) k_xgat_nstate(const float* __restrict__ s_dst, const float* __restrict__ m,
                                                     const float* __restrict__ invl, const float* __restrict__ D,
                                                     int64_t n, float4* __restrict__ nstate) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  nstate[t] = make_float4(s_dst[t], m[t], invl[t], D != nullptr ? D[t] : 0.f);
}

// deferred-D backward, by SOURCE over the CSC: dz = alpha e'(z) (dm dalpha - D_i) per edge and
// head, in place over dalpha (the formula and rounding of k_bwd_g's dz), and ds_src_j = sum of
// the source's dz.  LPI lanes per source item over items [w0, w1): 16 for the hub and long items,
// 4 for the short ones (<= 16 edges: four rows per lane group keep four times as many items in
// flight).  Each lane takes every LPI-th edge, four at a time with all their loads issued
// first, summed in edge order, then the LPI-lane tree; hub pieces leave a partial that
// k_xgat_dz_merge_wg adds up (pieces dealt to the waves, combined in wave order).
template <int H, int LPI>
__global__ void __launch_bounds__(256) k_xgat_dz(XItems it, int64_t w0, int64_t w1, const int32_t* __restrict__ row,
                                                 const int32_t* __restrict__ csc_eid,
                                                 const int32_t* __restrict__ csc2csr, const float* __restrict__ s_src,
                                                 const float4* __restrict__ nstate, float slope, float p,
                                                 float inv_keep, uint64_t seed, const uint64_t* __restrict__ seed_in,
                                                 float* __restrict__ dz, float* __restrict__ S, int64_t lds,
                                                 float* __restrict__ partial) {
  if (p > 0.f) seed = *seed_in;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t w = w0 + t / LPI;
  const int l = (int)(t % LPI);
  const bool live = w < w1;
  float ds[H];
#pragma unroll
  for (int h = 0; h < H; ++h) ds[h] = 0.f;
  int64_t j = 0;
  if (live) {
    j = it.row[w];
    float ss[H];
#pragma unroll
    for (int h = 0; h < H; ++h) ss[h] = s_src[j * H + h];
    const int ce = it.end[w];
    for (int k0 = it.beg[w] + l; k0 < ce; k0 += 4 * LPI) {
      int64_t ii[4], sl[4];
      uint32_t e_id[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u * LPI < ce ? k0 + u * LPI : k0;
        ii[u] = row[k];
        sl[u] = csc2csr != nullptr ? (int64_t)csc2csr[k] : (int64_t)k;
        e_id[u] = p > 0.f ? (uint32_t)csc_eid[k] : 0u;
      }
      float4 st[4][H];
      float dv[4][H];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int h = 0; h < H; ++h) {
          st[u][h] = nstate[ii[u] * H + h];  // {s_dst, m, inv_l, D}
          dv[u][h] = dz[sl[u] * H + h];
        }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u * LPI < ce) {
#pragma unroll
          for (int h = 0; h < H; ++h) {
            const float z = ss[h] + st[u][h].x;
            const float af = expf(lrelu(z, slope) - st[u][h].y) * st[u][h].z;
            const float dm = p > 0.f ? drop_scale(seed, e_id[u], (uint32_t)h, p, inv_keep) : 1.f;
            const float a1 = af * dlrelu(z, slope);
            const float dzv = fmaf(a1 * dm, dv[u][h], -(a1 * st[u][h].w));
            dz[sl[u] * H + h] = dzv;
            ds[h] += dzv;
          }
        }
      }
    }
  }
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float x = group_reduce<Op::Sum, 1, LPI / 2>(ds[h]);  // the LPI lanes of the item
    if (live && l == 0) {
      if (w < it.n_hub_items) partial[w * H + h] = x;
      else S[j * lds + h] = x;
    }
  }
}

// ---------------------------------------------------------------------------
// Hub merges with a whole workgroup on each hub: the pieces are dealt to the kMW waves in
// turn (each wave keeps several partial rows in flight), and the waves' sums are combined in
// wave order through LDS -- a fixed order, deterministic.  One wave per hub (k_fwd_merge,
// k_bwd_g_merge, k_xgat_dz_merge: pieces in a single wave's loop) left config 5's top item --
// 1M edges = 3,900 pieces of 256 edges, on the rank that owns it -- merging for 4 ms per call,
// 10 ms per step of that rank (profiles/r04/v16_probe5_r0_kernel_stats.csv).
// ---------------------------------------------------------------------------
constexpr int kMW = 8;    // waves per hub in the dz merge
constexpr int kMWf = 16;  // waves per (hub, head) in the forward merge (its hubs all above kSmallP pieces)
constexpr int kMWb = 8;   // waves per (hub, component) in the backward merge (16: 27.4 us per call at the config-5 share, 8: 23.1)
// Hubs of at most kSmallP pieces (most of them: config 5's share has 3,740 hubs, few above a
// dozen pieces) are merged by one wave per (hub, head) instead -- a workgroup of 8-16 waves on
// a 3-piece hub leaves most of its waves idle through three barriers.  The workgroup kernels
// skip those hubs.
constexpr int kSmallP = 16;

// one wave per (hub, head) for the small hubs: lanes hold the pieces' m and l, then the rows
// in piece order, four loads in flight
__global__ void __launch_bounds__(256) k_fwd_merge_small(const int32_t* __restrict__ hub_row,
                                                         const int32_t* __restrict__ hub_ptr, int64_t n_hubs,
                                                         int heads, const float* __restrict__ partial, float eps,
                                                         float* __restrict__ m_out, float* __restrict__ invl_out,
                                                         float* __restrict__ agg_out) {
  constexpr int C = 256;
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= n_hubs * heads) return;
  const int64_t hb = u / heads;
  const int hd = (int)(u - hb * heads);
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  if (p1 - p0 > kSmallP) return;
  const int64_t i = hub_row[hb];
  auto slot = [&](int q) { return partial + ((int64_t)q * heads + hd) * (C + 4); };
  float mq = -INFINITY, lq = 0.f;
  if (p0 + lane < p1) {
    mq = slot(p0 + lane)[C];
    lq = slot(p0 + lane)[C + 1];
  }
  const float M = wave_max(mq);
  const float l = wave_sum(p0 + lane < p1 ? lq * expf(mq - M) : 0.f);
  float4 a0 = f4(0.f), a1 = f4(0.f), a2 = f4(0.f), a3 = f4(0.f);
  int q = p0;
  for (; q + 3 < p1; q += 4) {
    const float4 v0 = ld4(slot(q) + lane * 4), v1 = ld4(slot(q + 1) + lane * 4), v2 = ld4(slot(q + 2) + lane * 4),
                 v3 = ld4(slot(q + 3) + lane * 4);
    a0 = fma4(expf(__shfl(mq, q - p0) - M), v0, a0);
    a1 = fma4(expf(__shfl(mq, q + 1 - p0) - M), v1, a1);
    a2 = fma4(expf(__shfl(mq, q + 2 - p0) - M), v2, a2);
    a3 = fma4(expf(__shfl(mq, q + 3 - p0) - M), v3, a3);
  }
  for (; q < p1; ++q) a0 = fma4(expf(__shfl(mq, q - p0) - M), ld4(slot(q) + lane * 4), a0);
  const float invl = 1.f / (l + eps);
  st4(agg_out + (i * heads + hd) * C + lane * 4, mul4(add4(add4(a0, a1), add4(a2, a3)), invl));
  if (lane == 0) {
    m_out[i * heads + hd] = M;
    invl_out[i * heads + hd] = invl;
  }
}

// aggregate-then-transform forward: agg[i,h] = sum_q e^(m_q - M) ax_q / sum_q e^(m_q - M) l_q
__global__ void __launch_bounds__(64 * kMWf) k_fwd_merge_wg(const int32_t* __restrict__ hub_row,
                                                           const int32_t* __restrict__ hub_ptr, int heads,
                                                           const float* __restrict__ partial, float eps,
                                                           float* __restrict__ m_out, float* __restrict__ invl_out,
                                                           float* __restrict__ agg_out) {
  constexpr int C = 256;
  __shared__ float4 red[kMWf][64];
  __shared__ float sr[kMWf];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t hb = blockIdx.x;
  const int64_t i = hub_row[hb];
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  if (p1 - p0 <= kSmallP) return;  // k_fwd_merge_small's
  auto slot = [&](int q, int hd) { return partial + ((int64_t)q * heads + hd) * (C + 4); };
  {
    const int hd = blockIdx.y;  // one workgroup per (hub, head): 3,740 hubs x 4 heads at the config-5 share
    float M = -INFINITY;
    for (int q = p0 + tid; q < p1; q += 64 * kMWf) M = fmaxf(M, slot(q, hd)[C]);
    M = wave_max(M);
    if (lane == 0) sr[w] = M;
    __syncthreads();
    M = sr[0];
    for (int k = 1; k < kMWf; ++k) M = fmaxf(M, sr[k]);
    __syncthreads();
    float t = 0.f;
    for (int q = p0 + tid; q < p1; q += 64 * kMWf) t += slot(q, hd)[C + 1] * expf(slot(q, hd)[C] - M);
    t = wave_sum(t);
    if (lane == 0) sr[w] = t;
    float4 a0 = f4(0.f), a1 = f4(0.f), a2 = f4(0.f), a3 = f4(0.f);
    int q = p0 + w;
    for (; q + 3 * kMWf < p1; q += 4 * kMWf) {
      const float* s0 = slot(q, hd);
      const float* s1 = slot(q + kMWf, hd);
      const float* s2 = slot(q + 2 * kMWf, hd);
      const float* s3 = slot(q + 3 * kMWf, hd);
      const float4 v0 = ld4(s0 + lane * 4), v1 = ld4(s1 + lane * 4), v2 = ld4(s2 + lane * 4), v3 = ld4(s3 + lane * 4);
      a0 = fma4(expf(s0[C] - M), v0, a0);
      a1 = fma4(expf(s1[C] - M), v1, a1);
      a2 = fma4(expf(s2[C] - M), v2, a2);
      a3 = fma4(expf(s3[C] - M), v3, a3);
    }
    for (; q < p1; q += kMWf) a0 = fma4(expf(slot(q, hd)[C] - M), ld4(slot(q, hd) + lane * 4), a0);
    red[w][lane] = add4(add4(a0, a1), add4(a2, a3));
    __syncthreads();
    if (w == 0) {
      float l = 0.f;
      for (int k = 0; k < kMWf; ++k) l += sr[k];
      float4 acc = red[0][lane];
      for (int k = 1; k < kMWf; ++k) acc = add4(acc, red[k][lane]);
      const float invl = 1.f / (l + eps);
      st4(agg_out + (i * heads + hd) * C + lane * 4, mul4(acc, invl));
      if (lane == 0) {
        m_out[i * heads + hd] = M;
        invl_out[i * heads + hd] = invl;
      }
    }
  }
}

// hub sources of k_bwd_g: the pieces' [acc^h (C) x H | ds] summed, waves in order; one workgroup
// per (hub, component): blockIdx.y = h < H sums head h's row, blockIdx.y = H the ds quad
template <int C, int H>
__global__ void __launch_bounds__(64 * kMWb) k_bwd_g_merge_wg(const int32_t* __restrict__ hub_row,
                                                             const int32_t* __restrict__ hub_ptr,
                                                             const float* __restrict__ partial,
                                                             float* __restrict__ acc_out, float* __restrict__ S,
                                                             int64_t lds) {
  static_assert(C == 256, "one float4 per lane");
  __shared__ float4 red[kMWb][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t hb = blockIdx.x;
  const int h = blockIdx.y;
  if (h == H && S == nullptr) return;
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  if (p1 - p0 <= kSmallP) return;  // k_bwd_g_merge_small's
  const int64_t j = hub_row[hb];
  const int off = h < H ? h * C + lane * 4 : H * C;
  float4 a = f4(0.f), b = f4(0.f);
  int q = p0 + w;
  // eight, then four pieces' loads in flight per wave (the first half into a, the rest into b)
  for (; q + 7 * kMWb < p1; q += 8 * kMWb) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld4(partial + (int64_t)(q + u * kMWb) * (H * C + 4) + off);
    a = add4(add4(add4(add4(a, v[0]), v[1]), v[2]), v[3]);
    b = add4(add4(add4(add4(b, v[4]), v[5]), v[6]), v[7]);
  }
  for (; q + 3 * kMWb < p1; q += 4 * kMWb) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld4(partial + (int64_t)(q + u * kMWb) * (H * C + 4) + off);
    a = add4(add4(a, v[0]), v[1]);
    b = add4(add4(b, v[2]), v[3]);
  }
  for (; q + kMWb < p1; q += 2 * kMWb) {
    const float4 v0 = ld4(partial + (int64_t)q * (H * C + 4) + off);
    const float4 v1 = ld4(partial + (int64_t)(q + kMWb) * (H * C + 4) + off);
    a = add4(a, v0);
    b = add4(b, v1);
  }
  if (q < p1) a = add4(a, ld4(partial + (int64_t)q * (H * C + 4) + off));
  red[w][lane] = add4(a, b);
  __syncthreads();
  if (w != 0) return;
  float4 acc = red[0][lane];
  for (int k = 1; k < kMWb; ++k) acc = add4(acc, red[k][lane]);
  if (h < H) {
    st4(acc_out + (j * H + h) * C + lane * 4, acc);
  } else if (lane < H) {
    const float ds[4] = {acc.x, acc.y, acc.z, acc.w};
    S[j * lds + lane] = ds[lane];
  }
}

// one wave per (hub, component) for the small hubs: the pieces in order, four loads in flight
template <int C, int H>
__global__ void __launch_bounds__(256) k_bwd_g_merge_small(const int32_t* __restrict__ hub_row,
                                                           const int32_t* __restrict__ hub_ptr, int64_t n_hubs,
                                                           const float* __restrict__ partial,
                                                           float* __restrict__ acc_out, float* __restrict__ S,
                                                           int64_t lds) {
  static_assert(C == 256, "one float4 per lane");
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= n_hubs * (H + 1)) return;
  const int64_t hb = u / (H + 1);
  const int h = (int)(u - hb * (H + 1));
  if (h == H && S == nullptr) return;
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  if (p1 - p0 > kSmallP) return;
  const int64_t j = hub_row[hb];
  const int off = h < H ? h * C + lane * 4 : H * C;
  float4 a0 = f4(0.f), a1 = f4(0.f), a2 = f4(0.f), a3 = f4(0.f);
  int q = p0;
  for (; q + 3 < p1; q += 4) {
    const float* s = partial + (int64_t)q * (H * C + 4) + off;
    const float4 v0 = ld4(s), v1 = ld4(s + (H * C + 4)), v2 = ld4(s + 2 * (H * C + 4)), v3 = ld4(s + 3 * (H * C + 4));
    a0 = add4(a0, v0);
    a1 = add4(a1, v1);
    a2 = add4(a2, v2);
    a3 = add4(a3, v3);
  }
  for (; q < p1; ++q) a0 = add4(a0, ld4(partial + (int64_t)q * (H * C + 4) + off));
  const float4 acc = add4(add4(a0, a1), add4(a2, a3));
  if (h < H) {
    st4(acc_out + (j * H + h) * C + lane * 4, acc);
  } else if (lane < H) {
    const float ds[4] = {acc.x, acc.y, acc.z, acc.w};
    S[j * lds + lane] = ds[lane];
  }
}

// hub sources of k_xgat_dz: ds_src = the pieces' partial sums, threads over pieces, then the
// lanes (tree) and the waves (in order)
template <int H>
__global__ void __launch_bounds__(64 * kMW) k_xgat_dz_merge_wg(const int32_t* __restrict__ hub_row,
                                                               const int32_t* __restrict__ hub_ptr,
                                                               const float* __restrict__ partial, float* __restrict__ S,
                                                               int64_t lds) {
  __shared__ float sr[kMW][H];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t hb = blockIdx.x;
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  float x[H];
#pragma unroll
  for (int h = 0; h < H; ++h) x[h] = 0.f;
  for (int q = p0 + tid; q < p1; q += 64 * kMW) {
#pragma unroll
    for (int h = 0; h < H; ++h) x[h] += partial[(int64_t)q * H + h];
  }
#pragma unroll
  for (int h = 0; h < H; ++h) {
    x[h] = wave_sum(x[h]);
    if (lane == 0) sr[w][h] = x[h];
  }
  __syncthreads();
  if (tid < H) {
    float v = 0.f;
    for (int k = 0; k < kMW; ++k) v += sr[k][tid];
    S[(int64_t)hub_row[hb] * lds + tid] = v;
  }
}

// dx_i += sum_h ds_dst_i^h A_dst[h] over the destination rows (S[i][H + h] = ds_dst)
template <int K, int H>
__global__ void __launch_bounds__(256) k_bwd_x_epi(const float* __restrict__ S, int64_t lds,
                                                   const float* __restrict__ A_dst, int64_t n, float* __restrict__ dx,
                                                   int64_t lddx) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t i = t / (K / 4);
  if (i >= n) return;
  const int c4 = (int)(t % (K / 4)) * 4;
  float4 v = ld4(dx + i * lddx + c4);
#pragma unroll
  for (int h = 0; h < H; ++h) v = fma4(S[i * lds + H + h], ld4(A_dst + h * K + c4), v);
  st4(dx + i * lddx + c4, v);
}

// dx[i][k] += sum_{v < nv} S[i][v] A[v][k] (v ascending): the rank-nv attention terms of a
// multi-head layer's input gradient, dx = D W + S [A_src; A_dst], after the D W GEMM.  One
// thread per float4 of dx, nv <= 16 runtime (the transform-then-aggregate layer, any K % 4).
__global__ void __launch_bounds__(256) k_rank_update(const float* __restrict__ S, int64_t lds, int nv,
                                                     const float* __restrict__ A, int64_t lda, int64_t n, int K,
                                                     float* __restrict__ dx, int64_t lddx) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int q = K / 4;
  const int64_t i = t / q;
  if (i >= n) return;
  const int c4 = (int)(t % q) * 4;
  float4 v = ld4(dx + i * lddx + c4);
  for (int r = 0; r < nv; ++r) v = fma4(S[i * lds + r], ld4(A + r * lda + c4), v);
  st4(dx + i * lddx + c4, v);
}

// dW[h C + c][k] = G[c][h K + k] * gs + att_src[h][c] GV[h][k] + att_dst[h][c] GV[H + h][k];
// datt_v[h][c] = sum_k W[h C + c][k] GV[v H + h][k].  One wave per (h, c) row of W.
__global__ void __launch_bounds__(256) k_wgrad_x(const float* __restrict__ G, const float* __restrict__ GV,
                                                 const float* __restrict__ W, const float* __restrict__ att_src,
                                                 const float* __restrict__ att_dst, int H, int C, int K, float gs,
                                                 float* __restrict__ dW, float* __restrict__ datt_src,
                                                 float* __restrict__ datt_dst) {
  const int lane = threadIdx.x & 63;
  const int64_t hc = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (hc >= (int64_t)H * C) return;
  const int h = (int)(hc / C), c = (int)(hc % C);
  const float as = att_src[hc], ad = att_dst[hc];
  float ps = 0.f, pd = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float gs_ = GV[(int64_t)h * K + k], gd = GV[(int64_t)(H + h) * K + k];
    const float w = W[hc * K + k];
    dW[hc * K + k] = fmaf(G[(int64_t)c * H * K + (int64_t)h * K + k], gs, fmaf(as, gs_, ad * gd));
    ps = fmaf(w, gs_, ps);
    pd = fmaf(w, gd, pd);
  }
  ps = wave_sum(ps);
  pd = wave_sum(pd);
  if (lane == 0) {
    datt_src[hc] = ps;
    datt_dst[hc] = pd;
  }
}

// block partial column sums of Y [n, C] (dbias); reduced by k_col_reduce in block order
template <int C>
__global__ void __launch_bounds__(256) k_colsum_part(const float* __restrict__ Y, int64_t ldy, int64_t n,
                                                     float* __restrict__ part) {
  constexpr int LPR = C / 4, SPB = 256 / LPR;
  __shared__ float4 red[SPB][LPR];
  const int sg = threadIdx.x / LPR, sl = threadIdx.x % LPR;
  float4 s = f4(0.f);
  for (int64_t i = (int64_t)blockIdx.x * SPB + sg; i < n; i += (int64_t)gridDim.x * SPB)
    s = add4(s, ld4(Y + i * ldy + sl * 4));
  red[sg][sl] = s;
  __syncthreads();
  if (threadIdx.x < LPR) {
    float4 t = red[0][threadIdx.x];
    for (int q = 1; q < SPB; ++q) t = add4(t, red[q][threadIdx.x]);
    st4(part + ((int64_t)blockIdx.x * LPR + threadIdx.x) * 4, t);
  }
}

}  // namespace

// ===========================================================================
// host launchers
// ===========================================================================
bool gemm_nn_shape_ok(int64_t M, int K, int N, int bmode) {
  return M >= 0 && K >= kGBK && K % kGBK == 0 && N >= 128 && N % 128 == 0 && (bmode == 0 || bmode == 1);
}

// split-K for small M (few row blocks, long K): the partial tiles go to the caller's workspace
int gemm_nn_splits(int64_t M, int K, int N) {
  const int64_t tiles = (M + kGBM - 1) / kGBM * (N / (N % 256 == 0 ? 256 : 128));
  if (tiles >= 128 || K < 4 * kGBK) return 1;
  int s = 1;
  while (s * 2 * tiles <= 256 && (K / kGBK) >= 4 * s * 2 && s < 32) s *= 2;  // >= 4 chunks per split
  return s;
}

// the three bf16 images of B [K x N] (bmode 0: B[k][n] = B[k ldb + n]; 1: B[n ldb + k]) per
// (column block of 32 nt columns, 32-deep k chunk), in the LDS layout the split kernels read
#ifdef PPGAT_LAB_BUILD
hipError_t nnx_presplit(const float* B, int64_t ldb, int bmode, int K, int N, int nt, uint16_t* img, hipStream_t st) {
  const int64_t groups = (int64_t)N * (K / 4);
  const unsigned gp = (unsigned)((groups + 255) / 256);
  if (groups <= 0) return hipSuccess;
  if (nt == 8) {
    if (bmode == 0) hipLaunchKernelGGL((k_nnx_presplit<8, 0>), dim3(gp), dim3(256), 0, st, B, ldb, K, N, img);
    else hipLaunchKernelGGL((k_nnx_presplit<8, 1>), dim3(gp), dim3(256), 0, st, B, ldb, K, N, img);
  } else {
    if (bmode == 0) hipLaunchKernelGGL((k_nnx_presplit<4, 0>), dim3(gp), dim3(256), 0, st, B, ldb, K, N, img);
    else hipLaunchKernelGGL((k_nnx_presplit<4, 1>), dim3(gp), dim3(256), 0, st, B, ldb, K, N, img);
  }
  return hipGetLastError();
}

#endif

size_t nnx_image_bytes(int K, int N, int nt) {
  const size_t img = nt == 8 ? (size_t)NnpImg<8>::BYTES : (size_t)NnpImg<4>::BYTES;
  return (size_t)(N / (32 * nt)) * (size_t)(K / 32) * img;
}

// the pre-split path: large M, K % 32 == 0.  libppgat.so runs it on k_gemm_nnh3 only, which takes
// the K chunks in pairs: other shapes go to the general x6 kernel (k_gemm_nnx).  The superseded
// generations -- k_gemm_nnh (any chunk count), k_gemm_nnh2 and the bf16 x6 k_gemm_nnp
// (PPGAT_GEMM_NNP / PPGAT_GEMM_F16 / PPGAT_NNH2) -- exist only in the lab build (make lab).
static bool nnp_ok(int64_t M, int K, int N) {
#ifdef PPGAT_LAB_BUILD
  static const bool off = [] {
    const char* e = getenv("PPGAT_GEMM_NNP");
    return e && strcmp(e, "0") == 0;
  }();
  if (off) return false;
#else
  if ((K / kGBK) % 2 != 0) return false;
#endif
  return gemm_split_enabled() && M >= 4 * kPBM && K % 32 == 0 && N % 128 == 0 && gemm_nn_splits(M, K, N) == 1;
}

static size_t nnp_image_bytes(int K, int N) { return nnx_image_bytes(K, N, N % 256 == 0 ? 8 : 4); }

// the fp16 two-term family on the pre-split path; lab builds: PPGAT_GEMM_F16=0 runs the bf16 x6 k_gemm_nnp
static bool nnh_enabled() {
#ifdef PPGAT_LAB_BUILD
  static const bool off = [] {
    const char* e = getenv("PPGAT_GEMM_F16");
    return e && strcmp(e, "0") == 0;
  }();
  return !off;
#else
  return true;
#endif
}

bool gemm_f16_enabled() { return nnh_enabled(); }

size_t nnh_image_bytes(int K, int N, int nt) {
  const size_t img = nt == 8 ? (size_t)NnhImg<8>::BYTES : (size_t)NnhImg<4>::BYTES;
  return (size_t)(N / (32 * nt)) * (size_t)(K / 32) * img;
}

// B's column scales and two fp16 images (layout as nnx_presplit's, two parts instead of three)
hipError_t nnh_presplit(const float* B, int64_t ldb, int bmode, int K, int N, int nt, uint16_t* img, int* ecol,
                        hipStream_t st) {
  const int64_t groups = (int64_t)N * (K / 4);
  if (groups <= 0) return hipSuccess;
  const unsigned gc = (unsigned)((N + 3) / 4), gp = (unsigned)((groups + 255) / 256);
  if (bmode == 0) hipLaunchKernelGGL((k_colscale16<0>), dim3(gc), dim3(256), 0, st, B, ldb, K, N, ecol);
  else hipLaunchKernelGGL((k_colscale16<1>), dim3(gc), dim3(256), 0, st, B, ldb, K, N, ecol);
#define PPGAT_NNH_PRE(NT_, BM_) \
  hipLaunchKernelGGL((k_nnh_presplit<NT_, BM_>), dim3(gp), dim3(256), 0, st, B, ldb, K, N, ecol, img)
  if (nt == 8) {
    if (bmode == 0) PPGAT_NNH_PRE(8, 0); else PPGAT_NNH_PRE(8, 1);
  } else {
    if (bmode == 0) PPGAT_NNH_PRE(4, 0); else PPGAT_NNH_PRE(4, 1);
  }
#undef PPGAT_NNH_PRE
  return hipGetLastError();
}

// the NN fp16 two-term kernel: k_gemm_nnh3; in lab builds PPGAT_NNH2=0 k_gemm_nnh, =2 k_gemm_nnh2
// (and k_fusion_fwdh3; the default: 2-3 % faster than k_gemm_nnh2 at config-5 shapes, profiles/
// r04/v8_gemm5_nnh*.log).  All three compute the same products in the same order (bitwise equal,
// tests/test_gpu_gemm_f16.py::test_nnh2_bitwise_equals_nnh, a lab test).  Read once per process.
// The measured-negative nnh3 variants (4: B read two steps ahead, 5: + s_setprio, 6: X through
// LDS; all within 1-2 % of 3, v8/v22_gemm5_nnh*.log) and the diagnostic lab kernels
// (PPGAT_NNH2_LAB: parts of the loop removed, results WRONG) exist only in a lab build:
// tools/build_variants.sh ppgat_xform.hip lab:"-DPPGAT_LAB_BUILD=1" -- never in libppgat.so.
int nnh_pipeline_variant() {
#ifdef PPGAT_LAB_BUILD
  static const int v = [] {
    const char* e = getenv("PPGAT_NNH2");
    if (e && strcmp(e, "0") == 0) return 1;
    if (e && strcmp(e, "2") == 0) return 2;
    if (e && (strcmp(e, "4") == 0 || strcmp(e, "5") == 0 || strcmp(e, "6") == 0)) return e[0] - '0';
    return 3;
  }();
  return v;
#else
  return 3;
#endif
}

#ifdef PPGAT_LAB_BUILD
static int nnh2_lab() {
  static const int lab = [] {
    const char* e = getenv("PPGAT_NNH2_LAB");
    return e ? atoi(e) : 0;
  }();
  return lab;
}
#endif

static size_t nnq_bytes(int K, int N) {  // image + column exponents, either family
  const int nt = N % 256 == 0 ? 8 : 4;
  return nnh_enabled() ? align_up(nnh_image_bytes(K, N, nt)) + align_up((size_t)N * 4) : nnp_image_bytes(K, N);
}

size_t gemm_nn_workspace_bytes(int64_t M, int K, int N) {
  if (nnp_ok(M, K, N)) return align_up(nnq_bytes(K, N));
  const int s = gemm_nn_splits(M, K, N);
  return s > 1 ? align_up((size_t)s * M * N * 4) : 0;
}

hipError_t gemm_nn(const float* X, int64_t ldx, int64_t M, int K, const float* B, int64_t ldb, int bmode, int N,
                   float alpha, const float* bias, float* Y, int64_t ldy, hipStream_t st, void* ws, const float* rS,
                   int64_t ldrs, int nv, const float* rA, int64_t ldra) {
  if (M <= 0) return hipSuccess;
  if (nv > 0 && !(ws != nullptr && nnp_ok(M, K, N) && nnh_enabled() && nv <= kNnhRank)) {
    // no fused epilogue on this path: the GEMM, then the rank update as its own pass
    hipError_t e = gemm_nn(X, ldx, M, K, B, ldb, bmode, N, alpha, bias, Y, ldy, st, ws);
    if (e != hipSuccess) return e;
    return rank_update(rS, ldrs, nv, rA, ldra, M, N, Y, ldy, st);
  }
  NnArg a{};
  a.rS = rS; a.ldrs = ldrs; a.nv = nv; a.rA = rA; a.ldra = ldra;
  a.X = X; a.ldx = ldx; a.M = M; a.K = K; a.B = B; a.ldb = ldb; a.N = N; a.alpha = alpha; a.bias = bias;
  a.Y = Y; a.ldy = ldy;
  if (ws != nullptr && nnp_ok(M, K, N)) {  // B pre-split once, then the glds-staged kernel
    const bool w8 = N % 256 == 0;
    uint16_t* img = static_cast<uint16_t*>(ws);
    a.row_blocks = (M + kPBM - 1) / kPBM;
    a.n_blocks = N / (w8 ? 256 : 128);
    a.splits = 1;
    const unsigned grid = (unsigned)((a.row_blocks + 7) / 8 * 8 * a.n_blocks);
    if (nnh_enabled()) {  // fp16 two-term split: three MFMAs per product
      int* ecol = reinterpret_cast<int*>(reinterpret_cast<char*>(ws) + align_up(nnh_image_bytes(K, N, w8 ? 8 : 4)));
      hipError_t e = nnh_presplit(B, ldb, bmode, K, N, w8 ? 8 : 4, img, ecol, st);
      if (e != hipSuccess) return e;
      if (nnh_pipeline_variant() >= 3 && (K / kGBK) % 2 == 0) {  // k_gemm_nnh3 runs chunk pairs
        const int v = nnh_pipeline_variant();
#ifdef PPGAT_LAB_BUILD
        if (const int lab = nnh2_lab(); lab > 0 && nv == 0 && w8) {  // diagnostics (results wrong)
#define PPGAT_LAB3(L) \
  if (lab == L) hipLaunchKernelGGL((k_gemm_nnh3<8, false, 1, false, L>), dim3(grid), dim3(512), 0, st, a, img, ecol)
          PPGAT_LAB3(1); PPGAT_LAB3(3); PPGAT_LAB3(7); PPGAT_LAB3(23); PPGAT_LAB3(39); PPGAT_LAB3(55);
#undef PPGAT_LAB3
          return hipGetLastError();
        }
#endif
#define PPGAT_NNH3(BD, PR, XT)                                                                                   \
  do {                                                                                                           \
    if (nv > 0) {                                                                                                \
      if (w8) hipLaunchKernelGGL((k_gemm_nnh3<8, true, BD, PR, 0, XT>), dim3(grid), dim3(512), 0, st, a, img, ecol); \
      else hipLaunchKernelGGL((k_gemm_nnh3<4, true, BD, PR, 0, XT>), dim3(grid), dim3(512), 0, st, a, img, ecol);    \
    } else if (w8) {                                                                                             \
      hipLaunchKernelGGL((k_gemm_nnh3<8, false, BD, PR, 0, XT>), dim3(grid), dim3(512), 0, st, a, img, ecol);        \
    } else {                                                                                                     \
      hipLaunchKernelGGL((k_gemm_nnh3<4, false, BD, PR, 0, XT>), dim3(grid), dim3(512), 0, st, a, img, ecol);        \
    }                                                                                                            \
  } while (0)
#ifdef PPGAT_LAB_BUILD
        static const bool e4 = [] {
          const char* e = getenv("PPGAT_NNH_E4");
          return e != nullptr && atoi(e) == 1;
        }();
        static const bool occ2 = [] {  // two workgroups per CU on the 128-column tile (<= 128 VGPRs)
          const char* e = getenv("PPGAT_NNH_OCC2");
          return e != nullptr && atoi(e) == 1;
        }();
        if (occ2 && nv == 0) {
          NnArg b2 = a;
          b2.n_blocks = N / 128;
          const unsigned g2 = (unsigned)((b2.row_blocks + 7) / 8 * 8 * b2.n_blocks);
          int* ecol4 = reinterpret_cast<int*>(reinterpret_cast<char*>(ws) + align_up(nnh_image_bytes(K, N, 4)));
          if (w8) {  // re-split B for the 128-column tile
            hipError_t e2 = nnh_presplit(B, ldb, bmode, K, N, 4, img, ecol4, st);
            if (e2 != hipSuccess) return e2;
          }
          hipLaunchKernelGGL((k_gemm_nnh3<4, false, 1, false, 0, false, false, 4>), dim3(g2), dim3(512), 0, st, b2, img,
                             w8 ? ecol4 : ecol);
          return hipGetLastError();
        }
        if (e4 && nv == 0 && a.ldy % 4 == 0 && reinterpret_cast<uintptr_t>(Y) % 16 == 0) {
          if (w8) hipLaunchKernelGGL((k_gemm_nnh3<8, false, 1, false, 0, false, true>), dim3(grid), dim3(512), 0, st, a, img, ecol);
          else hipLaunchKernelGGL((k_gemm_nnh3<4, false, 1, false, 0, false, true>), dim3(grid), dim3(512), 0, st, a, img, ecol);
          return hipGetLastError();
        }
        if (v == 4) PPGAT_NNH3(2, false, false);
        else if (v == 5) PPGAT_NNH3(2, true, false);
        else if (v == 6) PPGAT_NNH3(1, false, true);
        else
#endif
        PPGAT_NNH3(1, false, false);
        (void)v;
#undef PPGAT_NNH3
        return hipGetLastError();
      }
#ifdef PPGAT_LAB_BUILD
      if (nnh_pipeline_variant() == 2 && (K / kGBK) % 2 == 0) {  // k_gemm_nnh2 runs chunk pairs
#ifdef PPGAT_LAB_BUILD
        if (const int lab = nnh2_lab(); lab > 0 && nv == 0 && w8) {
#define PPGAT_LAB(L) \
  if (lab == L) hipLaunchKernelGGL((k_gemm_nnh2<8, false, L>), dim3(grid), dim3(512), 0, st, a, img, ecol)
          PPGAT_LAB(1); PPGAT_LAB(2); PPGAT_LAB(3); PPGAT_LAB(7); PPGAT_LAB(15);
#undef PPGAT_LAB
          return hipGetLastError();
        }
#endif
        if (nv > 0) {
          if (w8) hipLaunchKernelGGL((k_gemm_nnh2<8, true>), dim3(grid), dim3(512), 0, st, a, img, ecol);
          else hipLaunchKernelGGL((k_gemm_nnh2<4, true>), dim3(grid), dim3(512), 0, st, a, img, ecol);
        } else if (w8) {
          hipLaunchKernelGGL((k_gemm_nnh2<8, false>), dim3(grid), dim3(512), 0, st, a, img, ecol);
        } else {
          hipLaunchKernelGGL((k_gemm_nnh2<4, false>), dim3(grid), dim3(512), 0, st, a, img, ecol);
        }
        return hipGetLastError();
      }
      if (nv > 0) {
        if (w8) hipLaunchKernelGGL((k_gemm_nnh<8, true>), dim3(grid), dim3(512), 0, st, a, img, ecol);
        else hipLaunchKernelGGL((k_gemm_nnh<4, true>), dim3(grid), dim3(512), 0, st, a, img, ecol);
      } else if (w8) {
        hipLaunchKernelGGL((k_gemm_nnh<8, false>), dim3(grid), dim3(512), 0, st, a, img, ecol);
      } else {
        hipLaunchKernelGGL((k_gemm_nnh<4, false>), dim3(grid), dim3(512), 0, st, a, img, ecol);
      }
      return hipGetLastError();
#else
      return hipErrorInvalidValue;  // unreachable: nnp_ok admits chunk pairs only
#endif
    }
#ifdef PPGAT_LAB_BUILD
    hipError_t e = nnx_presplit(B, ldb, bmode, K, N, w8 ? 8 : 4, img, st);
    if (e != hipSuccess) return e;
    if (w8) hipLaunchKernelGGL((k_gemm_nnp<8>), dim3(grid), dim3(512), 0, st, a, img);
    else hipLaunchKernelGGL((k_gemm_nnp<4>), dim3(grid), dim3(512), 0, st, a, img);
    return hipGetLastError();
#else
    return hipErrorInvalidValue;  // unreachable: the product's pre-split path is fp16
#endif
  }
  a.row_blocks = (M + kGBM - 1) / kGBM;
  const int64_t padded = (a.row_blocks + 7) / 8 * 8;
  const bool wide = N % 256 == 0;
  a.n_blocks = N / (wide ? 256 : 128);
  a.splits = ws != nullptr ? gemm_nn_splits(M, K, N) : 1;
  if (a.splits > 1) {  // every split non-empty: splits = ceil(chunks / chunks per split)
    const int chunks = K / kGBK;
    const int per = (chunks + a.splits - 1) / a.splits;
    a.k_per = per * kGBK;
    a.splits = (chunks + per - 1) / per;
    a.part = static_cast<float*>(ws);
  }
  if (gemm_split_enabled()) {  // split bf16 matrix cores, two workgroups per CU
    a.n_blocks = N / 128;
    // 256-wide tiles when N allows (measured at config-5 shapes: 5.6-6.5 ms against 5.9-7.0 for
    // 128-wide tiles or 64-deep k chunks, profiles/r02/v13_gemm_split_cfg5.log)
    const bool w8 = N % 256 == 0;
    if (w8) a.n_blocks = N / 256;
    const unsigned gv = a.splits > 1 ? (unsigned)(a.row_blocks * a.n_blocks * a.splits)
                                     : (unsigned)(padded * a.n_blocks);
#define PPGAT_NNX(NT_, KC_)                                                                     \
  do {                                                                                          \
    if (bmode == 0) hipLaunchKernelGGL((k_gemm_nnx<NT_, 0, KC_>), dim3(gv), dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((k_gemm_nnx<NT_, 1, KC_>), dim3(gv), dim3(256), 0, st, a);            \
  } while (0)
    if (w8) PPGAT_NNX(8, 32);
    else PPGAT_NNX(4, 32);
#undef PPGAT_NNX
  } else {
  const unsigned grid = a.splits > 1 ? (unsigned)(a.row_blocks * a.n_blocks * a.splits)
                                     : (unsigned)(padded * a.n_blocks);
#define PPGAT_NN(NT_, BM_) hipLaunchKernelGGL((k_gemm_nn<NT_, BM_>), dim3(grid), dim3(256), 0, st, a)
  if (wide) {
    if (bmode == 0) PPGAT_NN(8, 0); else PPGAT_NN(8, 1);
  } else {
    if (bmode == 0) PPGAT_NN(4, 0); else PPGAT_NN(4, 1);
  }
#undef PPGAT_NN
  }
  if (a.splits > 1) {
    const int64_t n4 = M * (N / 4);
    hipLaunchKernelGGL(k_nn_split_sum, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, a.part, M, N, a.splits,
                       alpha, bias, Y, ldy);
  }
  return hipGetLastError();
}

static int tn_splits(int64_t M, int T) {
  int s = 8;
  while (s < 512 && (int64_t)s * T < 512 && M / (2 * s) >= 4 * kTR) s *= 2;
  return s;
}

bool gemm_tn_big_shape_ok(int Ma, int Nb) { return Ma >= 128 && Ma % 128 == 0 && Nb >= 128 && Nb % 128 == 0; }

// the fp16 two-term TN kernel (k_gemm_tnh): Nb % 256 == 0, with the fp16 family on, and long
// reductions only -- below ~64k rows its three extra launches (max buffer clear, two column-max
// passes) cost more than the fp32 kernel's MFMA time (the FusionMLP training batch of 512 rows)
static bool tnh_ok(int64_t M, int Ma, int Nb) {
  return gemm_split_enabled() && nnh_enabled() && M >= 65536 && Ma % 128 == 0 && Nb % 256 == 0;
}
static int tnh_splits(int64_t M, int T) {  // one workgroup per CU: splits * tiles <= 256, >= 128 rows per split
  // two workgroup rounds per CU: the same time as one (3.96 vs 3.98 ms at the config-5 share,
  // profiles/r03/v16_tnh_*), half the rows per fp32 accumulator chain: 3.3e-6 vs 5.3e-6
  // max-abs/max-abs on 1.875M-row reductions (fp32 MFMA kernel: 3.5e-6).  PPGAT_TNH_WAVES
  // overrides (lab builds).
#ifdef PPGAT_LAB_BUILD
  static const int waves = [] {
    const char* e = getenv("PPGAT_TNH_WAVES");
    const int v = e ? atoi(e) : 2;
    return v >= 1 && v <= 16 ? v : 2;
  }();
#else
  constexpr int waves = 2;
#endif
  int s = 256 * waves / T;
  if (s < 1) s = 1;
  while (s > 1 && M / s < 4 * kTR) s /= 2;
  return s;
}

// (+ the column sums' partials: [splits, Ma] on the fp16 path, the colsum kernel's otherwise)
size_t gemm_tn_big_workspace_bytes(int64_t M, int Ma, int Nb) {
  if (tnh_ok(M, Ma, Nb)) {
    const int T = (Ma / 128) * (Nb / 256);
    const int s = tnh_splits(M, T);
    return align_up((size_t)s * Ma * Nb * 4) + align_up((size_t)(Ma + Nb) * 4) + align_up((size_t)s * Ma * 4);
  }
  const int T = (Ma / kTA) * (Nb / (Nb % 256 == 0 ? 256 : 128));
  return align_up((size_t)tn_splits(M, T) * Ma * Nb * 4) + align_up((size_t)colsum_blocks(M) * 256 * 4);
}

static hipError_t colmax_bits(const float* X, int64_t ldx, int64_t M, int C, unsigned* out, hipStream_t st,
                              const int32_t* rp = nullptr) {
  // C columns in slices of <= 1024 (256 float4 lanes per row pass)
  for (int c0 = 0; c0 < C; c0 += 1024) {
    const int c = C - c0 < 1024 ? C - c0 : 1024;
    int64_t blocks = (M + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    const int64_t rpb = (M + blocks - 1) / blocks;
    blocks = (M + rpb - 1) / rpb;
    hipLaunchKernelGGL(k_colmax_bits, dim3((unsigned)blocks), dim3(256), 0, st, X + c0, ldx, M, c, rpb, rp, out + c0);
  }
  return hipGetLastError();
}

hipError_t colmax_abs(const float* X, int64_t ldx, int64_t M, int C, unsigned* out, hipStream_t st,
                      const int32_t* src_ptr) {
  hipError_t e = hipMemsetAsync(out, 0, (size_t)C * 4, st);
  if (e == hipSuccess && M > 0) e = colmax_bits(X, ldx, M, C, out, st, src_ptr);
  return e;
}

hipError_t gemm_tn_big(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int Ma, int Nb, float* out,
                       void* ws, hipStream_t st, const unsigned* b_bound, int b_period, float b_scale,
                       const unsigned* a_bound, float* colsum_out) {
  if (M <= 0) {  // empty sums (no partials)
    hipError_t e = hipMemsetAsync(out, 0, (size_t)Ma * Nb * 4, st);
    if (e == hipSuccess && colsum_out) e = hipMemsetAsync(colsum_out, 0, (size_t)Ma * 4, st);
    return e;
  }
  if (tnh_ok(M, Ma, Nb)) {
    static const bool attr = [] {
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_tnh), hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)kThLds) == hipSuccess;
    }();
    (void)attr;
    TnhArg a{};
    a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.M = M; a.Ma = Ma; a.Nb = Nb;
    a.tiles_a = Ma / 128;
    a.tiles_b = Nb / 256;
    const int T = a.tiles_a * a.tiles_b;
    a.splits = tnh_splits(M, T);
    a.rows_per_split = ((M + a.splits - 1) / a.splits + kTR - 1) / kTR * kTR;
    a.part = static_cast<float*>(ws);
    unsigned* mx = reinterpret_cast<unsigned*>(static_cast<char*>(ws) + align_up((size_t)a.splits * Ma * Nb * 4));
    a.amax = a_bound ? a_bound : mx;       // a caller's bound of |A| (rows with nonzero B) skips A's pass
    a.aclamp = a_bound ? 1 : 0;
    a.bmax = b_bound ? b_bound : mx + Ma;  // a caller's bound of |B| per column skips B's pass
    a.bperiod = b_bound ? b_period : Nb;
    a.bscale = b_bound ? b_scale : 1.f;
    a.cpart = colsum_out ? reinterpret_cast<float*>(reinterpret_cast<char*>(mx) + align_up((size_t)(Ma + Nb) * 4))
                         : nullptr;
    hipError_t e = hipSuccess;
    if (!a_bound || !b_bound) e = hipMemsetAsync(mx, 0, (size_t)(Ma + Nb) * 4, st);
    if (e == hipSuccess && !a_bound) e = colmax_bits(A, lda, M, Ma, mx, st);
    if (e == hipSuccess && !b_bound) e = colmax_bits(B, ldb, M, Nb, mx + Ma, st);
    if (e != hipSuccess) return e;
#ifdef PPGAT_LAB_BUILD
    static const bool t256 = [] {  // PPGAT_TNH256=0: the 128 x 256 tile everywhere (A/B runs)
      const char* e = getenv("PPGAT_TNH256");
      return !(e && strcmp(e, "0") == 0);
    }();
#else
    constexpr bool t256 = true;
#endif
    if (t256 && Ma % 256 == 0) {  // the 256 x 256 tile, the same row splits (the same bits)
      static const bool attr2 = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_tnh256),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)kTh2Lds) == hipSuccess;
      }();
      (void)attr2;
      a.tiles_a = Ma / 256;
      const int T2 = a.tiles_a * a.tiles_b;
      hipLaunchKernelGGL(k_gemm_tnh256, dim3((unsigned)(8 * T2 * ((a.splits + 7) / 8))), dim3(1024), kTh2Lds, st, a);
    } else {
      const unsigned grid = (unsigned)(8 * T * ((a.splits + 7) / 8));
      hipLaunchKernelGGL(k_gemm_tnh, dim3(grid), dim3(512), kThLds, st, a);
    }
    const int64_t n4 = (int64_t)Ma * Nb / 4;
    hipLaunchKernelGGL(k_split_sum, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, a.part, n4, a.splits, out);
    if (colsum_out)
      hipLaunchKernelGGL(k_split_sum, dim3((unsigned)((Ma / 4 + 255) / 256)), dim3(256), 0, st, a.cpart,
                         (int64_t)Ma / 4, a.splits, colsum_out);
    return hipGetLastError();
  }
  const bool wide = Nb % 256 == 0;
  TnArg a{};
  a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.M = M; a.Ma = Ma; a.Nb = Nb;
  a.tiles_a = Ma / kTA;
  a.tiles_b = Nb / (wide ? 256 : 128);
  const int T = a.tiles_a * a.tiles_b;
  a.splits = tn_splits(M, T);
  a.rows_per_split = ((M + a.splits - 1) / a.splits + kTR - 1) / kTR * kTR;
  a.part = static_cast<float*>(ws);
  const unsigned grid = (unsigned)(8 * T * ((a.splits + 7) / 8));
  if (wide) hipLaunchKernelGGL((k_gemm_tn<256>), dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((k_gemm_tn<128>), dim3(grid), dim3(256), 0, st, a);
  const int64_t n4 = (int64_t)Ma * Nb / 4;
  hipLaunchKernelGGL(k_split_sum, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, a.part, n4, a.splits, out);
  if (colsum_out) {  // the colsum kernel over 256- (or 128-) column slabs of A
    float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + align_up((size_t)a.splits * Ma * Nb * 4));
    for (int c0 = 0; c0 < Ma; c0 += 256) {
      const hipError_t e = colsum(A + c0, lda, M, Ma - c0 >= 256 ? 256 : 128, colsum_out + c0, part, st);
      if (e != hipSuccess) return e;
    }
  }
  return hipGetLastError();
}

bool xgat_shape_ok(int K, int H, int C) { return K == 256 && (H == 2 || H == 4) && C >= 128 && C % 128 == 0; }

#define PPGAT_XH(H_, ...)                                   \
  do {                                                      \
    if ((H_) == 2) { constexpr int HH = 2; __VA_ARGS__; }   \
    else { constexpr int HH = 4; __VA_ARGS__; }             \
  } while (0)

hipError_t xgat_weights(const float* W, const float* att_src, const float* att_dst, int H, int C, int K, float* A,
                        float* Wt, float* Wg, hipStream_t st) {
  const int64_t na = (int64_t)2 * H * K;
  if (A) hipLaunchKernelGGL(k_att_proj, dim3((unsigned)((na + 15) / 16)), dim3(256), 0, st, W, att_src, att_dst, H, C,
                            K, A);
  const int64_t nw = (int64_t)H * C * K;
  if (Wt || Wg) hipLaunchKernelGGL(k_wperm, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, W, H, C, K, Wt, Wg);
  return hipGetLastError();
}

hipError_t xgat_scores(const float* x, int64_t ldx, int64_t n_rows, int64_t n_dst, int K, int H, const float* A,
                       float* s_src, float* s_dst, hipStream_t st) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows + 15) / 16;  // four rows per wave and iteration (K = 256), grid-stride
  if (blocks > 4096) blocks = 4096;
  PPGAT_XH(H, hipLaunchKernelGGL((k_xscores<256, HH>), dim3((unsigned)blocks), dim3(256), 0, st, x, ldx, n_rows, n_dst,
                                 A, s_src, s_dst));
  (void)K;
  return hipGetLastError();
}

hipError_t xgat_fwd(const ItemsArg& it, const int32_t* col, const int32_t* eid, const float* x, int64_t ldx, int K,
                    int H, const float* s_src, const float* s_dst, float slope, float p, uint64_t seed,
                    const uint64_t* seed_in, float* agg, float* m, float* invl, float* partial,
                    const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st, unsigned* xmax) {
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const XItems its{it.row, it.beg, it.end, it.n_items, it.n_hub_items};
#ifdef PPGAT_LAB_BUILD
  static const int fu = [] {  // rows in flight per wave (PPGAT_FWDX_U: 2 / 3 / 4 / 5 / 6 / 8)
    const char* e = getenv("PPGAT_FWDX_U");
    return e ? atoi(e) : 4;
  }();
#define PPGAT_FWDX(U_)                                                                                               \
  PPGAT_XH(H, hipLaunchKernelGGL((k_fwd_x<256, HH, U_>), dim3((unsigned)((it.n_items + 3) / 4)), dim3(256), 0, st, \
                                 its, col, eid, x, ldx, s_src, s_dst, slope, p, inv_keep, seed, seed_in, agg, m, invl, \
                                 partial, xmax))
  if (it.n_items > 0) {
    if (fu == 2) PPGAT_FWDX(2);
    else if (fu == 3) PPGAT_FWDX(3);
    else if (fu == 5) PPGAT_FWDX(5);
    else if (fu == 6) PPGAT_FWDX(6);
    else if (fu == 8) PPGAT_FWDX(8);
    else PPGAT_FWDX(4);
  }
#undef PPGAT_FWDX
#else
  if (it.n_items > 0)
    PPGAT_XH(H, hipLaunchKernelGGL((k_fwd_x<256, HH>), dim3((unsigned)((it.n_items + 3) / 4)), dim3(256), 0, st, its,
                                   col, eid, x, ldx, s_src, s_dst, slope, p, inv_keep, seed, seed_in, agg, m, invl,
                                   partial, xmax));
#endif
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  (void)K;
  if (n_hubs > 0) {
    hipLaunchKernelGGL(k_fwd_merge_small, dim3((unsigned)((n_hubs * H + 3) / 4)), dim3(256), 0, st, hub_row, hub_ptr,
                       (int64_t)n_hubs, H, partial, 1e-16f, m, invl, agg);
    hipLaunchKernelGGL(k_fwd_merge_wg, dim3((unsigned)n_hubs, (unsigned)H), dim3(64 * kMWf), 0, st, hub_row, hub_ptr, H, partial,
                       1e-16f, m, invl, agg);
  }
  return hipGetLastError();
}

hipError_t xgat_bwd_pro(const float* gt, const float* agg, const float* s_dst, const float* m, const float* invl,
                        int64_t n, int K, int H, float* nstate, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  PPGAT_XH(H, hipLaunchKernelGGL((k_bwd_x_pro<256, HH>), dim3((unsigned)blocks), dim3(256), 0, st, gt, agg, s_dst, m,
                                 invl, n, reinterpret_cast<float4*>(nstate)));
  (void)K;
  return hipGetLastError();
}

hipError_t xgat_bwd_edges(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr,
                          const float* x, int64_t ldx, int K, int H, const float* s_src, const float* nstate,
                          const float* gt, const float* A_src, float slope, float p, uint64_t seed,
                          const uint64_t* seed_in, float* dx, int64_t lddx, float* S, int64_t lds, float* dz,
                          float* partial, const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs,
                          hipStream_t st) {
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const XItems its{it.row, it.beg, it.end, it.n_items, it.n_hub_items};
  if (it.n_items > 0)
    PPGAT_XH(H, hipLaunchKernelGGL((k_bwd_x<256, HH>), dim3((unsigned)((it.n_items + 3) / 4)), dim3(256), 0, st, its,
                                   row, csc_eid, csc2csr, x, ldx, s_src, reinterpret_cast<const float4*>(nstate), gt,
                                   A_src, slope, p, inv_keep, seed, seed_in, dx, lddx, S, lds, dz, partial));
  if (n_hubs > 0)
    PPGAT_XH(H, hipLaunchKernelGGL((k_bwd_x_merge<256, HH>), dim3((unsigned)((n_hubs + 3) / 4)), dim3(256), 0, st,
                                   hub_row, hub_ptr, n_hubs, partial, A_src, dx, lddx, S, lds));
  (void)K;
  return hipGetLastError();
}

hipError_t xgat_bwd_edges_g(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr,
                            const float* hs, int C, int H, const float* s_src, const float* nstate, const float* g,
                            int64_t ldg, float slope, float p, uint64_t seed, const uint64_t* seed_in, float* acc,
                            float* S, int64_t lds, float* dz, float* partial, const int32_t* hub_row,
                            const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st, float* pz, unsigned* gmax) {
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const XItems its{it.row, it.beg, it.end, it.n_items, it.n_hub_items};
  if (it.n_items > 0)
    PPGAT_XH(H, hipLaunchKernelGGL((k_bwd_g<256, HH>), dim3((unsigned)((it.n_items + 3) / 4)), dim3(256), 0, st, its,
                                   row, csc_eid, csc2csr, hs, s_src, reinterpret_cast<const float4*>(nstate), g, ldg,
                                   slope, p, inv_keep, seed, seed_in, acc, S, lds, dz, partial, pz, gmax));
  if (n_hubs > 0)
    PPGAT_XH(H, {
      hipLaunchKernelGGL((k_bwd_g_merge_small<256, HH>), dim3((unsigned)((n_hubs * (HH + 1) + 3) / 4)), dim3(256), 0,
                         st, hub_row, hub_ptr, (int64_t)n_hubs, partial, acc, S, lds);
      hipLaunchKernelGGL((k_bwd_g_merge_wg<256, HH>), dim3((unsigned)n_hubs, HH + 1), dim3(64 * kMWb), 0, st, hub_row,
                         hub_ptr, partial, acc, S, lds);
    });
  (void)C;
  return hipGetLastError();
}

// nstate[i][h].w = D[i][h] for every row of a table whose {s_dst, m, inv_l} came by exchange (the
// halo partition's deferred D: the completed D arrives as its own [rows, H] table).  One thread
// per (row, head); replaces a strided torch copy that ran at ~1 TB/s.
__global__ void __launch_bounds__(256) k_xgat_nstate_set_d(float* __restrict__ nstate, const float* __restrict__ D,
                                                           int64_t nh) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < nh) nstate[t * 4 + 3] = D[t];
}

hipError_t xgat_nstate_set_d(float* nstate, const float* D, int64_t n, int H, hipStream_t st) {
  const int64_t nh = n * H;
  if (nh > 0)
    hipLaunchKernelGGL(k_xgat_nstate_set_d, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, nstate, D, nh);
  return hipGetLastError();
}

hipError_t xgat_nstate(const float* s_dst, const float* m, const float* invl, const float* D, int64_t n, int H,
                       float* nstate, hipStream_t st) {
  const int64_t nh = n * H;
  if (nh > 0)
    hipLaunchKernelGGL(k_xgat_nstate, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, s_dst, m, invl, D, nh,
                       reinterpret_cast<float4*>(nstate));
  return hipGetLastError();
}

hipError_t xgat_bwd_dz(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr, int H,
                       const float* s_src, const float* nstate, float slope, float p, uint64_t seed,
                       const uint64_t* seed_in, float* dz, float* S, int64_t lds, float* partial,
                       const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st) {
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const XItems its{it.row, it.beg, it.end, it.n_items, it.n_hub_items};
  // [0, wl): hub pieces and long items, 16 lanes each; [wl, n_items): short items, 4 lanes each
  const int64_t wl = it.n_long_items >= it.n_hub_items && it.n_long_items <= it.n_items ? it.n_long_items
                                                                                         : it.n_items;
  if (wl > 0)
    PPGAT_XH(H, hipLaunchKernelGGL((k_xgat_dz<HH, 16>), dim3((unsigned)((wl * 16 + 255) / 256)), dim3(256), 0, st,
                                   its, (int64_t)0, wl, row, csc_eid, csc2csr, s_src,
                                   reinterpret_cast<const float4*>(nstate), slope, p, inv_keep, seed, seed_in, dz, S,
                                   lds, partial));
  if (it.n_items > wl)
    PPGAT_XH(H, hipLaunchKernelGGL((k_xgat_dz<HH, 4>), dim3((unsigned)(((it.n_items - wl) * 4 + 255) / 256)),
                                   dim3(256), 0, st, its, wl, it.n_items, row, csc_eid, csc2csr, s_src,
                                   reinterpret_cast<const float4*>(nstate), slope, p, inv_keep, seed, seed_in, dz, S,
                                   lds, partial));
  if (n_hubs > 0)
    PPGAT_XH(H, hipLaunchKernelGGL((k_xgat_dz_merge_wg<HH>), dim3((unsigned)n_hubs), dim3(64 * kMW), 0, st, hub_row,
                                   hub_ptr, partial, S, lds));
  return hipGetLastError();
}

hipError_t xgat_bwd_epi(const float* S, int64_t lds, const float* A_dst, int64_t n, int K, int H, float* dx,
                        int64_t lddx, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t th = n * (K / 4);
  PPGAT_XH(H, hipLaunchKernelGGL((k_bwd_x_epi<256, HH>), dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, S, lds,
                                 A_dst, n, dx, lddx));
  return hipGetLastError();
}

hipError_t att_proj(const float* W, const float* att_src, const float* att_dst, int H, int C, int K, float* A,
                    hipStream_t st) {
  const int64_t na = (int64_t)2 * H * K;
  if (na > 0) hipLaunchKernelGGL(k_att_proj, dim3((unsigned)((na + 15) / 16)), dim3(256), 0, st, W, att_src, att_dst,
                                 H, C, K, A);
  return hipGetLastError();
}

hipError_t rank_update(const float* S, int64_t lds, int nv, const float* A, int64_t lda, int64_t n, int K, float* dx,
                       int64_t lddx, hipStream_t st) {
  if (n <= 0 || nv <= 0) return hipSuccess;
  const int64_t th = n * (K / 4);
  hipLaunchKernelGGL(k_rank_update, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, st, S, lds, nv, A, lda, n, K, dx,
                     lddx);
  return hipGetLastError();
}

hipError_t xgat_wgrad(const float* G, const float* GV, const float* W, const float* att_src, const float* att_dst,
                      int H, int C, int K, float* dW, float* datt_src, float* datt_dst, hipStream_t st) {
  const int64_t rows = (int64_t)H * C;
  hipLaunchKernelGGL(k_wgrad_x, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, G, GV, W, att_src, att_dst, H, C,
                     K, 1.f / (float)H, dW, datt_src, datt_dst);
  return hipGetLastError();
}

int64_t colsum_blocks(int64_t n) {
  int64_t b = (n + 63) / 64;
  return b < 1 ? 1 : (b > 1024 ? 1024 : b);
}

hipError_t colsum(const float* Y, int64_t ldy, int64_t n, int C, float* out, float* part, hipStream_t st) {
  const int64_t blocks = colsum_blocks(n);
  if (C == 256) hipLaunchKernelGGL((k_colsum_part<256>), dim3((unsigned)blocks), dim3(256), 0, st, Y, ldy, n, part);
  else if (C == 128) hipLaunchKernelGGL((k_colsum_part<128>), dim3((unsigned)blocks), dim3(256), 0, st, Y, ldy, n, part);
  else return hipErrorInvalidValue;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_col_reduce(part, blocks, C, C, out, nullptr, st);
}

}  // namespace ppgat
