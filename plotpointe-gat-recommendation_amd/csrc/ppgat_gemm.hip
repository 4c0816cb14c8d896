// ppgat_gemm.hip -- the GAT layer's projection GEMMs on the fp32 matrix cores, with the
// layer's per-node work fused into their epilogues, the weight-gradient GEMM, the
// weight-gradient assembly and the optimizer update (gfx950 / MI355X).
//
//  * k_proj<0>: h = x W^T (+ bias) for x [N, K<=128], W [128, K]  -- GATConv.lin / item_proj
//    (scripts/train_gat_pyg.py:74,77,81; train_gat_custom.py:66,77), with the node attention
//    terms s_src = h.att_src, s_dst = h.att_dst (PyG alpha_src/alpha_dst; custom :79) in the
//    epilogue, so h is never re-read for them.  x may come from two row segments (users from
//    user_emb, items from the item projection: train_gat_pyg.py:79-82) -- no concatenation.
//  * k_proj<1>: dx = D W + ds_src (x) A_src + ds_dst (x) A_dst (heads = 1), the input
//    gradient of the layer with the attention-logit terms folded in as a rank-2 epilogue
//    (A = att W, computed per workgroup from W in LDS).
//  * k_tn128: out = A^T B for A [N, M<=128], B [N, K<=128] (dW of every projection), one
//    128 x 128 fp32 accumulator per wave in the accumulation registers, rows streamed
//    straight from HBM into the MFMA operand layout (no LDS staging), + V^T B (nv <= 2) and
//    colsum(A) on the VALU; workgroup partials reduced through LDS, then an ordered
//    split reduction (deterministic).
//  * k_wgrad: dW = G + att_src (x) G_s + att_dst (x) G_d and datt = W G_{s,d} (one launch).
//  * k_adam: torch.optim.Adam's update (L2 weight decay, bias corrections; the arithmetic of
//    ATen's fused Adam) over up to 16 tensors per launch.
//
// MFMA: v_mfma_f32_32x32x2_f32, exact fp32 FMA chains (MI355X_MICROARCH.md: 157 TF peak,
// 64 cycles per instruction per SIMD).  Lane maps (l = lane, r = l & 31, hf = l >> 5):
//   A operand A'[i = r][kk = hf], B operand B'[kk = hf][j = r],
//   accumulator register q: row (q & 3) + 8 (q >> 2) + 4 hf, column r.
// The reduction index of each MFMA is free to permute as long as A and B agree, which is
// what lets every operand come from one contiguous float4 per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "ppgat_internal.h"
#include "ppgat_lanes.h"

// Experiment hook for tools/bench_gemm.py (0 in every product build): bit 0 skips the x
// loads of the projection kernel, bit 1 its MFMAs, bit 2 its epilogue stores.
#ifndef PPGAT_PROJ_VARIANT
#define PPGAT_PROJ_VARIANT 0
#endif

namespace ppgat {

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using u32x4 = __attribute__((__vector_size__(4 * sizeof(unsigned int)))) unsigned int;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int acc_row(int q, int hf) { return (q & 3) + 8 * (q >> 2) + 4 * hf; }

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// ---------------------------------------------------------------------------
// projection GEMM with fused epilogues
// ---------------------------------------------------------------------------
constexpr int kPT = 128;       // output columns (one tile)
constexpr int kPLd = kPT + 4;  // LDS row stride: 16 lanes of a ds_read_b128 hit 64 distinct banks

struct ProjArg {
  const float* x0;  // rows [0, split)
  int64_t ldx0;
  const float* x1;  // rows [split, n) (row - split)
  int64_t ldx1;
  int64_t split;
  int64_t n;
  int K;            // reduction length (<= 128, % 4 == 0)
  const float* W;   // mode 0: [128, K] (x W^T); mode 1: [K, 128] (x W)
  int64_t ldw;
  const float* bias;     // mode 0, nullable: + bias[col]
  const float* att_src;  // nullable: mode 0 scores; mode 1 A_src = att_src W
  const float* att_dst;
  const float* ds;       // mode 1: ds_src at ds[row * ldds], ds_dst at ds[row * ldds + 1]
  int64_t ldds;
  float* y;
  int64_t ldy;
  float* s_src;  // mode 0 with att: [n]
  float* s_dst;
};

// 8 per-lane partial values, each summed over the 32 lanes of its half-wave.  On return
// v[t] (t < 2) holds the full sum of value index ((l >> 4) & 1) * 4 + ((l >> 3) & 1) * 2 + t.
__device__ __forceinline__ void reduce8_over32(float (&v)[8], int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float r0, r1;
    row_swap<16>(v[t], v[4 + t], r0, r1);
    v[t] = r0 + r1;
  }
  const bool b8 = (lane & 8) != 0;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float send = b8 ? v[t] : v[2 + t];
    const float keep = b8 ? v[2 + t] : v[t];
    v[t] = keep + dpp<0x128>(send);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) v[t] = group_reduce<Op::Sum, 1, 4>(v[t]);
}

// Workgroup = 4 waves = 2 pairs, one workgroup per CU, persistent over 32-row tiles.  The two
// waves of a pair split the reduction (k) in halves and keep their half of B in registers
// for the whole launch (128 VGPRs: 4 column blocks x 32 k-steps), so the MFMA loop reads no
// LDS; x rows stream from HBM with the next tile in flight.  Per tile both waves publish
// their partial 32 x 128 tile row-major to LDS, then each finalises 16 rows: the two
// partials added in a fixed order, epilogue, float4 stores of whole row segments, scores.
// k mapping: step s of wave half kh, lane half hf covers k = 64 kh + 32 hf + s.
constexpr int kXLd = kPT + 8;  // exchange row stride: rows 4 apart land 32 banks apart
constexpr int kXTile = 32 * kXLd;
constexpr int kProjLds = 2 * 2 * 2 * kXTile;  // [slot][pair][half] partial tiles (floats)
static_assert(kProjLds >= kPT * kPLd, "the W staging image aliases the exchange buffers");

template <int MODE>
__global__ void __launch_bounds__(256, 1) k_proj(ProjArg a) {
  __shared__ float4 lds4[kProjLds / 4];
  __shared__ float sV[2][kPT];  // att (mode 0) / A = att W (mode 1)
  float* lds = reinterpret_cast<float*>(lds4);
  float (*sW)[kPLd] = reinterpret_cast<float (*)[kPLd]>(lds);  // W as stored (prologue only)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: buffer descriptors stay in SGPRs
  const int r = lane & 31, hf = lane >> 5;
  const int kh = w & 1, pr = w >> 1;
  const int K = a.K;
  // ---- stage W (zero-padded to 128 x 128), the attention vectors ----
  if (MODE == 0) {
    for (int idx = tid; idx < kPT * 32; idx += 256) {
      const int j = idx >> 5, k4 = (idx & 31) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k4 < K) v = ld4(a.W + (int64_t)j * a.ldw + k4);
      st4(&sW[j][k4], v);
    }
  } else {
    for (int idx = tid; idx < kPT * 32; idx += 256) {
      const int k = idx >> 5, j4 = (idx & 31) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < K) v = ld4(a.W + (int64_t)k * a.ldw + j4);
      st4(&sW[k][j4], v);
    }
  }
  const bool vec = a.att_src != nullptr;
  if (vec && tid < 2 * kPT) {
    const int k = tid & 127;
    sV[tid >> 7][k] = (MODE == 1 && k >= K) ? 0.f : (tid < kPT ? a.att_src : a.att_dst)[k];
  }
  __syncthreads();
  if (MODE == 1 && vec) {  // A[j] = sum_k att[k] W[k][j]
    float s = 0.f;
    const int j = tid & 127, v = tid >> 7;
    for (int k = 0; k < kPT; ++k) s = fmaf(sV[v][k], sW[k][j], s);
    __syncthreads();
    sV[v][j] = s;
  }
  // ---- B fragments into registers: bq[nb][s] = B[k = 64 kh + 32 hf + s][j = 32 nb + r] ----
  float bq[4][32];
  const int kb = 64 * kh + 32 * hf;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int s4 = 0; s4 < 32; s4 += 4) {
      if (MODE == 0) {
        const float4 v = *reinterpret_cast<const float4*>(&sW[nb * 32 + r][kb + s4]);
        bq[nb][s4] = v.x; bq[nb][s4 + 1] = v.y; bq[nb][s4 + 2] = v.z; bq[nb][s4 + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) bq[nb][s4 + e] = sW[kb + s4 + e][nb * 32 + r];
      }
    }
  __syncthreads();  // sW is dead from here on: its bytes become the exchange buffers
  // epilogue lane map: lane owns columns c4 .. c4 + 3 of rows 16 kh + 2 i + hf (i < 8)
  const int c4 = 4 * r;
  float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va, bias4 = va;
  if (vec) {
    va = make_float4(sV[0][c4], sV[0][c4 + 1], sV[0][c4 + 2], sV[0][c4 + 3]);
    vb = make_float4(sV[1][c4], sV[1][c4 + 1], sV[1][c4 + 2], sV[1][c4 + 3]);
  }
  if (MODE == 0 && a.bias) bias4 = ld4(a.bias + c4);

  const int64_t tiles = (a.n + 31) / 32;
  const int64_t iters = (tiles + 2 * (int64_t)gridDim.x - 1) / (2 * (int64_t)gridDim.x);  // same for every wave
  // x loads are unconditional (a select on a loaded value makes the compiler wait for the
  // load right there, which would serialise the prefetch): rows past n read row n - 1 (their
  // outputs are never stored), columns past K read in-row columns < K that meet zero B rows.
  auto load_x = [&](int64_t tile, float4 (&xv)[8]) {
    if (PPGAT_PROJ_VARIANT & 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[q] = make_float4(tile, q, r, 1.f);
      return;
    }
    int64_t row = tile * 32 + r;
    row = row < a.n ? row : a.n - 1;
    const float* src = row < a.split ? a.x0 + row * a.ldx0 : a.x1 + (row - a.split) * a.ldx1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = kb + 4 * q;
      xv[q] = ld4(src + (c < K ? c : K - 4));
    }
  };
  // Finalise tile tt from exchange slot sl: rows 16 kh + 2 i + hf, columns c4..c4+3.  Branch
  // free so hipcc can interleave it with the next tile's MFMAs: stores go through buffer
  // descriptors whose record count clips rows past n (and a whole tile past the last one).
  auto finalize = [&](int64_t tt, int sl) {
    const float* X = lds + ((sl * 2 + pr) * 2) * kXTile;
    const int64_t row0 = tt * 32;
    // rows of this tile that exist (0 for tt < 0 or past the last tile), min/max only: a
    // branch here would split the basic block the MFMAs share with this code
    const int64_t live = min(min(max(a.n - row0, (int64_t)0), (int64_t)32), max(row0 + 32, (int64_t)0));
    const int64_t base = max(row0, (int64_t)0);
    const auto ry = __builtin_amdgcn_make_buffer_rsrc(a.y + base * a.ldy, 0,
                                                      (int)(live * a.ldy * 4), 0x00020000);
    float4 y[8];
    float ps[8], pd[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rr = 16 * kh + 2 * i + hf;
      const float4 p0 = *reinterpret_cast<const float4*>(X + rr * kXLd + c4);
      const float4 p1 = *reinterpret_cast<const float4*>(X + kXTile + rr * kXLd + c4);
      float4 v = make_float4(p0.x + p1.x, p0.y + p1.y, p0.z + p1.z, p0.w + p1.w);
      if (MODE == 1) {
        const int64_t row = min(max(row0 + rr, (int64_t)0), a.n - 1);
        const float2 d = *reinterpret_cast<const float2*>(a.ds + row * a.ldds);
        v.x = fmaf(d.y, vb.x, fmaf(d.x, va.x, v.x));
        v.y = fmaf(d.y, vb.y, fmaf(d.x, va.y, v.y));
        v.z = fmaf(d.y, vb.z, fmaf(d.x, va.z, v.z));
        v.w = fmaf(d.y, vb.w, fmaf(d.x, va.w, v.w));
      } else {
        ps[i] = fmaf(v.w, va.w, fmaf(v.z, va.z, fmaf(v.y, va.y, v.x * va.x)));
        pd[i] = fmaf(v.w, vb.w, fmaf(v.z, vb.z, fmaf(v.y, vb.y, v.x * vb.x)));
        v = make_float4(v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w);
      }
      y[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rr = 16 * kh + 2 * i + hf;
      if (!(PPGAT_PROJ_VARIANT & 4) || y[i].x == 12345.f)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(y[i].x), __float_as_uint(y[i].y),
                                                      __float_as_uint(y[i].z), __float_as_uint(y[i].w)},
                                               ry, (int)((rr * a.ldy + c4) * 4), 0, 0);
    }
    if (MODE == 0 && vec) {
      reduce8_over32(ps, lane);
      reduce8_over32(pd, lane);
      const int o = lane & 7;
      const int i = ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + (o & 1);
      const int off = o < 2 ? (16 * kh + 2 * i + hf) * 4 : 0x40000000;  // non-writers fall outside
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.s_src + base, 0, (int)(live * 4), 0x00020000);
      const auto rd = __builtin_amdgcn_make_buffer_rsrc(a.s_dst + base, 0, (int)(live * 4), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((o & 1) ? ps[1] : ps[0]), rs, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((o & 1) ? pd[1] : pd[0]), rd, off, 0, 0);
    }
  };
  float4 xr[8];
  load_x((int64_t)blockIdx.x * 2 + pr, xr);
  // iteration it: MFMAs of tile it interleaved with the finalisation of tile it - 1 (a no-op
  // at it = 0: its descriptors have no records), then the partial of tile it is published;
  // one barrier per iteration (two exchange slots).  No branches inside, so the scheduler
  // can fill the MFMA shadows with the finalisation.
  for (int64_t it = 0; it < iters; ++it) {
    const int64_t t = (it * gridDim.x + blockIdx.x) * 2 + pr;
    float4 xn[8];
    load_x(t + 2 * (int64_t)gridDim.x, xn);  // next tile in flight
    f32x16 acc[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[nb][q] = 0.f;
    if (!(PPGAT_PROJ_VARIANT & 2)) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) acc[nb] = mfma(comp(xr[q], e), bq[nb][4 * q + e], acc[nb]);
    } else {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][0] = xr[nb].x + bq[nb][0];
    }
    finalize(t - 2 * (int64_t)gridDim.x, (int)((it + 1) & 1));
#pragma unroll
    for (int g = 0; g < 128; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x366, 2, 0);  // then up to two VALU/SALU/DS/VMEM
    }
    // ---- publish the partial tile row-major: X[slot][pr][kh][row][col] ----
    float* mine = lds + (((int)(it & 1) * 2 + pr) * 2 + kh) * kXTile;
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) mine[acc_row(q, hf) * kXLd + nb * 32 + r] = acc[nb][q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) xr[q] = xn[q];
  }
  finalize(((iters - 1) * gridDim.x + blockIdx.x) * 2 + pr, (int)((iters - 1) & 1));
}

// ---------------------------------------------------------------------------
// out[M, K] = A^T B (+ V^T B, colsum A), M, K <= 128
// ---------------------------------------------------------------------------
constexpr int kTnPairs = 8;  // row pairs per prefetch batch

struct TnArg {
  const float* A;
  int64_t lda;
  const float* B;   // rows [0, split)
  int64_t ldb;
  const float* B1;  // rows [split, n) (row - split)
  int64_t ldb1;
  int64_t split;
  const float* V;  // nullable, [N, nv] at ldv (nv <= 2)
  int64_t ldv;
  int nv;
  int64_t n;
  int M, K;
  int64_t rows_per_wave;  // even
  float* part;   // [gridDim.x][128][128] (m-major)
  float* vpart;  // [gridDim.x][2][128]
  float* cpart;  // nullable: [gridDim.x][128]
};

// One batch of kTnPairs row pairs: lane (r, hf) takes row base + 2p + hf.
template <int NV, bool MASK>
__device__ __forceinline__ void tn_load(const float* pa, const float* pb, const float* pv, int64_t sa, int64_t sb,
                                        int64_t sv, bool am, bool bk, float4 (&av)[kTnPairs], float4 (&bv)[kTnPairs],
                                        float2 (&vv)[kTnPairs]) {
#pragma unroll
  for (int p = 0; p < kTnPairs; ++p) {
    av[p] = ld4(pa + p * sa);
    bv[p] = ld4(pb + p * sb);
    if (NV == 2) vv[p] = *reinterpret_cast<const float2*>(pv + p * sv);
    else if (NV == 1) vv[p] = make_float2(pv[p * sv], 0.f);
    else vv[p] = make_float2(0.f, 0.f);
    if (MASK) {
      if (!am) av[p] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!bk) bv[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

template <int NV>
__device__ __forceinline__ void tn_compute(f32x16 (&acc)[4][4], float4& vacc0, float4& vacc1, float4& csum,
                                           const float4 (&av)[kTnPairs], const float4 (&bv)[kTnPairs],
                                           const float2 (&vv)[kTnPairs]) {
#pragma unroll
  for (int p = 0; p < kTnPairs; ++p) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma(comp(av[p], i), comp(bv[p], j), acc[i][j]);
    if (NV > 0) {
      vacc0.x = fmaf(vv[p].x, bv[p].x, vacc0.x);
      vacc0.y = fmaf(vv[p].x, bv[p].y, vacc0.y);
      vacc0.z = fmaf(vv[p].x, bv[p].z, vacc0.z);
      vacc0.w = fmaf(vv[p].x, bv[p].w, vacc0.w);
    }
    if (NV > 1) {
      vacc1.x = fmaf(vv[p].y, bv[p].x, vacc1.x);
      vacc1.y = fmaf(vv[p].y, bv[p].y, vacc1.y);
      vacc1.z = fmaf(vv[p].y, bv[p].z, vacc1.z);
      vacc1.w = fmaf(vv[p].y, bv[p].w, vacc1.w);
    }
    csum.x += av[p].x;
    csum.y += av[p].y;
    csum.z += av[p].z;
    csum.w += av[p].w;
  }
}

template <int NV, bool MASK>
__global__ void __launch_bounds__(256, 1) k_tn128(TnArg a) {
  __shared__ float sR[kPT][kPT + 4];
  __shared__ float sVr[4][2][kPT];
  __shared__ float sC[4][kPT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int64_t wid = (int64_t)blockIdx.x * 4 + w;
  const int64_t n_beg = wid * a.rows_per_wave;
  const int64_t n_end = min(a.n, n_beg + a.rows_per_wave);
  const bool am = !MASK || 4 * r < a.M, bk = !MASK || 4 * r < a.K;
  const int acol = am ? 4 * r : 0, bcol = bk ? 4 * r : 0;  // masked lanes read column 0, zeroed after
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  float4 vacc0 = make_float4(0.f, 0.f, 0.f, 0.f), vacc1 = vacc0, csum = vacc0;
  // two B segments: rows [n_beg, split) from B, [split, n_end) from B1
  for (int seg = 0; seg < 2; ++seg) {
    const int64_t r0 = seg == 0 ? n_beg : max(n_beg, a.split);
    const int64_t r1 = seg == 0 ? min(n_end, a.split) : n_end;
    if (r0 >= r1) continue;
    const float* bbase = seg == 0 ? a.B : a.B1;
    const int64_t ldb = seg == 0 ? a.ldb : a.ldb1;
    const int64_t boff = seg == 0 ? 0 : a.split;
    const int64_t sa = 2 * a.lda, sb = 2 * ldb, sv = 2 * a.ldv;
    const int64_t full = (r1 - r0) / (2 * kTnPairs);
    const float* pa = a.A + (r0 + hf) * a.lda + acol;
    const float* pb = bbase + (r0 - boff + hf) * ldb + bcol;
    const float* pv = a.V + (r0 + hf) * a.ldv;
    float4 av[kTnPairs], bv[kTnPairs];
    float2 vv[kTnPairs];
    if (full > 0) {
      tn_load<NV, MASK>(pa, pb, pv, sa, sb, sv, am, bk, av, bv, vv);
      for (int64_t bt = 1; bt < full; ++bt) {
        pa += kTnPairs * sa;
        pb += kTnPairs * sb;
        pv += kTnPairs * sv;
        float4 an[kTnPairs], bn[kTnPairs];
        float2 vn[kTnPairs];
        tn_load<NV, MASK>(pa, pb, pv, sa, sb, sv, am, bk, an, bn, vn);  // in flight during the MFMAs
        __builtin_amdgcn_sched_barrier(0);
        tn_compute<NV>(acc, vacc0, vacc1, csum, av, bv, vv);
#pragma unroll
        for (int p = 0; p < kTnPairs; ++p) {
          av[p] = an[p];
          bv[p] = bn[p];
          vv[p] = vn[p];
        }
      }
      tn_compute<NV>(acc, vacc0, vacc1, csum, av, bv, vv);
    }
    // tail (< 2 kTnPairs rows): out-of-range pairs read the segment's first row, zeroed
    const int64_t t0 = r0 + full * 2 * kTnPairs;
    if (t0 < r1) {
#pragma unroll
      for (int p = 0; p < kTnPairs; ++p) {
        const bool ok = t0 + 2 * p + hf < r1;
        const int64_t row = ok ? t0 + 2 * p + hf : r0;
        const float4 va = ld4(a.A + row * a.lda + acol);
        const float4 vb = ld4(bbase + (row - boff) * ldb + bcol);
        av[p] = (ok && am) ? va : make_float4(0.f, 0.f, 0.f, 0.f);
        bv[p] = (ok && bk) ? vb : make_float4(0.f, 0.f, 0.f, 0.f);
        float2 v = make_float2(0.f, 0.f);
        if (NV == 2) v = *reinterpret_cast<const float2*>(a.V + row * a.ldv);
        if (NV == 1) v.x = a.V[row * a.ldv];
        vv[p] = ok ? v : make_float2(0.f, 0.f);
      }
      tn_compute<NV>(acc, vacc0, vacc1, csum, av, bv, vv);
    }
  }
  // ---- workgroup reduction through LDS, waves in order 0..3 ----
  // acc[i][j][q]: m = 4 * acc_row(q, hf) + i, k = 4 * r + j
  auto put = [&](bool add) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = 4 * acc_row(q, hf) + i;
        float4 v = make_float4(acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]);
        float* dst = &sR[m][4 * r];
        if (add) {
          const float4 o = *reinterpret_cast<const float4*>(dst);
          v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        }
        st4(dst, v);
      }
  };
  // (no loop over turns: a loop lets the compiler hoist all 256 accumulator reads)
  if (w == 0) put(false);
  __syncthreads();
  if (w == 1) put(true);
  __syncthreads();
  if (w == 2) put(true);
  __syncthreads();
  if (w == 3) put(true);
  __syncthreads();
  // V and colsum: combine the two half-waves (lane, lane ^ 32), then the waves in order
  {
    float t0[4] = {vacc0.x, vacc0.y, vacc0.z, vacc0.w}, t1[4] = {vacc1.x, vacc1.y, vacc1.z, vacc1.w};
    float c[4] = {csum.x, csum.y, csum.z, csum.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x0, x1;
      row_swap<32>(t0[e], t0[e], x0, x1);
      t0[e] = x0 + x1;
      row_swap<32>(t1[e], t1[e], x0, x1);
      t1[e] = x0 + x1;
      row_swap<32>(c[e], c[e], x0, x1);
      c[e] = x0 + x1;
    }
    if (hf == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sVr[w][0][4 * r + e] = t0[e];
        sVr[w][1][4 * r + e] = t1[e];
        sC[w][4 * r + e] = c[e];
      }
    }
  }
  __syncthreads();
  float* P = a.part + (int64_t)blockIdx.x * kPT * kPT;
  for (int idx = tid; idx < kPT * kPT / 4; idx += 256) {
    const int m = idx >> 5, k4 = (idx & 31) * 4;
    st4(P + m * kPT + k4, *reinterpret_cast<const float4*>(&sR[m][k4]));
  }
  {
    const int v = tid >> 7, k = tid & 127;
    a.vpart[((int64_t)blockIdx.x * 2 + v) * kPT + k] =
        ((sVr[0][v][k] + sVr[1][v][k]) + sVr[2][v][k]) + sVr[3][v][k];
    if (a.cpart && tid < kPT)
      a.cpart[(int64_t)blockIdx.x * kPT + tid] = ((sC[0][tid] + sC[1][tid]) + sC[2][tid]) + sC[3][tid];
  }
}

// Ordered reduction of the k_tn128 partials: block b owns 64 consecutive elements of the
// concatenated [part | vpart | cpart] element space; 16 thread groups take splits
// g, g + 16, ... and are combined in group order (deterministic).  Elements outside
// [M] x [K] are dropped when writing.
struct TnReduceArg {
  const float* part;
  const float* vpart;
  const float* cpart;
  int64_t splits;
  int M, K, nv;
  float* out;    // [M, K]
  float* vout;   // [nv, K]
  float* colsum; // [M]
};

__global__ void __launch_bounds__(1024) k_tn_reduce(TnReduceArg a) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  int64_t e = (int64_t)blockIdx.x * 64 + lane;
  const float* src;
  int64_t stride, off;
  int kind;
  if (e < kPT * kPT) {
    src = a.part; stride = kPT * kPT; off = e; kind = 0;
  } else if (e < kPT * kPT + 2 * kPT) {
    src = a.vpart; stride = 2 * kPT; off = e - kPT * kPT; kind = 1;
  } else {
    src = a.cpart; stride = kPT; off = e - kPT * kPT - 2 * kPT; kind = 2;
  }
  const bool live = kind != 2 || a.cpart != nullptr;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (live) {
    int64_t k = g;
    for (; k + 48 < a.splits; k += 64) {
      s0 += src[k * stride + off];
      s1 += src[(k + 16) * stride + off];
      s2 += src[(k + 32) * stride + off];
      s3 += src[(k + 48) * stride + off];
    }
    for (; k < a.splits; k += 16) s0 += src[k * stride + off];
  }
  red[g][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && live) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][lane];
    if (kind == 0) {
      const int m = (int)(off >> 7), k = (int)(off & 127);
      if (m < a.M && k < a.K) a.out[(int64_t)m * a.K + k] = t;
    } else if (kind == 1) {
      const int v = (int)(off >> 7), k = (int)(off & 127);
      if (v < a.nv && k < a.K) a.vout[(int64_t)v * a.K + k] = t;
    } else {
      if (off < a.M) a.colsum[off] = t;
    }
  }
}

// ---------------------------------------------------------------------------
// dW / datt assembly (one workgroup per 8 rows of W; datt by the rows' owners)
//   dW[hc][k] = G[hc][k] + att_src[hc] GV[h][k] + att_dst[hc] GV[H + h][k]
//   datt_src[hc] = sum_k W[hc][k] GV[h][k],  datt_dst[hc] = sum_k W[hc][k] GV[H + h][k]
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_wgrad(const float* __restrict__ G, const float* __restrict__ GV,
                                               const float* __restrict__ W, const float* __restrict__ att_src,
                                               const float* __restrict__ att_dst, int heads, int C, int K,
                                               float* __restrict__ dW, float* __restrict__ datt_src,
                                               float* __restrict__ datt_dst) {
  const int HC = heads * C;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int hc = blockIdx.x * 4 + w; hc < HC; hc += gridDim.x * 4) {
    const int h = hc / C;
    const float as = att_src[hc], ad = att_dst[hc];
    const float* gs = GV + (int64_t)h * K;
    const float* gd = GV + (int64_t)(heads + h) * K;
    float ps = 0.f, pd = 0.f;
    for (int k = lane; k < K; k += 64) {
      const float wv = W[(int64_t)hc * K + k];
      dW[(int64_t)hc * K + k] = fmaf(ad, gd[k], fmaf(as, gs[k], G[(int64_t)hc * K + k]));
      ps = fmaf(wv, gs[k], ps);
      pd = fmaf(wv, gd[k], pd);
    }
    ps = wave_sum(ps);
    pd = wave_sum(pd);
    if (lane == 0) {
      datt_src[hc] = ps;
      datt_dst[hc] = pd;
    }
  }
}

// ---------------------------------------------------------------------------
// Adam (torch.optim.Adam, amsgrad=False, maximize=False; L2 weight decay added to the
// gradient; the arithmetic order of ATen's fused Adam)
// ---------------------------------------------------------------------------
constexpr int kAdamMax = 16;
constexpr int kAdamPerBlock = 256 * 8;  // elements per block (2 float4 per thread)

struct AdamArg {
  float* p[kAdamMax];
  const float* g[kAdamMax];
  float* m[kAdamMax];
  float* v[kAdamMax];
  int64_t n[kAdamMax];
  int64_t blk_end[kAdamMax];
  float step_size[kAdamMax];
  float bc2_sqrt[kAdamMax];
  int count;
  float beta1, beta2, omb1, omb2, eps, wd;  // omb = 1 - beta, rounded once from double on the host
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1, float b2, float omb1,
                                          float omb2, float eps, float wd, float step_size, float bc2s) {
  if (wd != 0.f) g = g + p * wd;
  m = b1 * m + omb1 * g;
  v = b2 * v + omb2 * g * g;
  const float denom = sqrtf(v) / bc2s + eps;
  p = p - step_size * m / denom;
}

__global__ void __launch_bounds__(256) k_adam(AdamArg a) {
  int ti = 0;
  int64_t b = blockIdx.x;
  while (ti < a.count - 1 && b >= a.blk_end[ti]) ++ti;
  if (ti > 0) b -= a.blk_end[ti - 1];
  float* __restrict__ P = a.p[ti];
  const float* __restrict__ Gr = a.g[ti];
  float* __restrict__ M = a.m[ti];
  float* __restrict__ V = a.v[ti];
  const int64_t n = a.n[ti];
  const float ss = a.step_size[ti], bc = a.bc2_sqrt[ti];
  const int64_t base = b * kAdamPerBlock;
  const bool aligned = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(Gr) |
                         reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(V)) & 15) == 0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t e = base + ((int64_t)u * 256 + threadIdx.x) * 4;
    if (aligned && e + 3 < n) {
      float4 p = ld4(P + e), g = ld4(Gr + e), m = ld4(M + e), v = ld4(V + e);
      adam_elem(p.x, g.x, m.x, v.x, a.beta1, a.beta2, a.omb1, a.omb2, a.eps, a.wd, ss, bc);
      adam_elem(p.y, g.y, m.y, v.y, a.beta1, a.beta2, a.omb1, a.omb2, a.eps, a.wd, ss, bc);
      adam_elem(p.z, g.z, m.z, v.z, a.beta1, a.beta2, a.omb1, a.omb2, a.eps, a.wd, ss, bc);
      adam_elem(p.w, g.w, m.w, v.w, a.beta1, a.beta2, a.omb1, a.omb2, a.eps, a.wd, ss, bc);
      st4(P + e, p);
      st4(M + e, m);
      st4(V + e, v);
    } else {
      for (int64_t x = e; x < e + 4 && x < n; ++x) {
        float p = P[x], m = M[x], v = V[x];
        adam_elem(p, Gr[x], m, v, a.beta1, a.beta2, a.omb1, a.omb2, a.eps, a.wd, ss, bc);
        P[x] = p;
        M[x] = m;
        V[x] = v;
      }
    }
  }
}

}  // namespace

// ---- host launchers ----
bool proj_shape_ok(int K, int ncols) { return K >= 4 && K <= kPT && K % 4 == 0 && ncols == kPT; }

static unsigned proj_grid(int64_t n) {
  const int64_t tiles = (n + 31) / 32;
  int64_t g = (tiles + 1) / 2;
  if (g > 256) g = 256;  // one workgroup per CU, persistent over the row tiles
  return (unsigned)(g < 1 ? 1 : g);
}

hipError_t proj_fwd(const float* x0, int64_t ldx0, const float* x1, int64_t ldx1, int64_t split, int64_t n, int K,
                    const float* W, int64_t ldw, const float* bias, const float* att_src, const float* att_dst,
                    float* y, int64_t ldy, float* s_src, float* s_dst, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  ProjArg a{};
  a.x0 = x0; a.ldx0 = ldx0; a.x1 = x1 ? x1 : x0; a.ldx1 = x1 ? ldx1 : ldx0; a.split = x1 ? split : n; a.n = n;
  a.K = K; a.W = W; a.ldw = ldw; a.bias = bias; a.att_src = att_src; a.att_dst = att_dst;
  a.y = y; a.ldy = ldy; a.s_src = s_src; a.s_dst = s_dst;
  hipLaunchKernelGGL(k_proj<0>, dim3(proj_grid(n)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t proj_dx(const float* D, int64_t ldd, int64_t n, int K, const float* W, int64_t ldw, const float* att_src,
                   const float* att_dst, const float* S, int64_t lds, float* y, int64_t ldy, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  ProjArg a{};
  a.x0 = D; a.ldx0 = ldd; a.x1 = D; a.ldx1 = ldd; a.split = n; a.n = n; a.K = K; a.W = W; a.ldw = ldw;
  a.att_src = att_src; a.att_dst = att_dst; a.ds = S; a.ldds = lds; a.y = y; a.ldy = ldy;
  hipLaunchKernelGGL(k_proj<1>, dim3(proj_grid(n)), dim3(256), 0, st, a);
  return hipGetLastError();
}

bool tn128_shape_ok(int M, int K, int nv, const float* V, int64_t ldv) {
  return M >= 4 && M <= kPT && M % 4 == 0 && K >= 4 && K <= kPT && K % 4 == 0 && nv >= 0 && nv <= 2 &&
         (nv < 2 || ((ldv % 2) == 0 && (reinterpret_cast<uintptr_t>(V) % 8) == 0));
}

static int64_t tn_blocks(int64_t N) {
  int64_t b = 256;                     // one workgroup (4 waves) per CU
  const int64_t min_rows = 16;         // >= 16 rows per wave
  while (b > 1 && b * 4 * min_rows > N) b /= 2;
  return b;
}

size_t tn128_workspace_bytes(int64_t N) {
  const int64_t b = tn_blocks(N);
  return align_up((size_t)b * kPT * kPT * 4) + align_up((size_t)b * 2 * kPT * 4) + align_up((size_t)b * kPT * 4);
}

hipError_t tn128(const float* A, int64_t lda, const float* B, int64_t ldb, const float* B1, int64_t ldb1, int64_t split,
                 int64_t N, int M, int K, float* out, float* colsum, const float* V, int64_t ldv, int nv, float* vout,
                 void* ws, hipStream_t st) {
  const int64_t nb = tn_blocks(N);
  char* p = static_cast<char*>(ws);
  TnArg a{};
  if (N <= 0) {  // empty sum: zero outputs
    hipError_t e = hipMemsetAsync(out, 0, (size_t)M * K * 4, st);
    if (e == hipSuccess && colsum) e = hipMemsetAsync(colsum, 0, (size_t)M * 4, st);
    if (e == hipSuccess && nv > 0) e = hipMemsetAsync(vout, 0, (size_t)nv * K * 4, st);
    return e;
  }
  a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.B1 = B1 ? B1 : B; a.ldb1 = B1 ? ldb1 : ldb; a.split = B1 ? split : N;
  a.V = nv > 0 ? V : A; a.ldv = nv > 0 ? ldv : lda; a.nv = nv; a.n = N;
  a.M = M; a.K = K;
  const int64_t waves = nb * 4;
  a.rows_per_wave = ((N + waves - 1) / waves + 1) / 2 * 2;
  a.part = reinterpret_cast<float*>(p);
  a.vpart = reinterpret_cast<float*>(p + align_up((size_t)nb * kPT * kPT * 4));
  a.cpart = colsum ? reinterpret_cast<float*>(p + align_up((size_t)nb * kPT * kPT * 4) +
                                              align_up((size_t)nb * 2 * kPT * 4))
                   : nullptr;
  const bool mask = M != kPT || K != kPT;
  const bool v2 = nv == 2 && (a.ldv % 2) == 0 && (reinterpret_cast<uintptr_t>(a.V) % 8) == 0;
  const int NVk = nv == 0 ? 0 : (nv == 1 || !v2) ? 1 : 2;
  if (nv == 2 && !v2) return hipErrorInvalidValue;  // caller guarantees 8-byte aligned V pairs
#define PPGAT_TN(NV_, MASK_) hipLaunchKernelGGL((k_tn128<NV_, MASK_>), dim3((unsigned)nb), dim3(256), 0, st, a)
  if (mask) {
    if (NVk == 0) PPGAT_TN(0, true); else if (NVk == 1) PPGAT_TN(1, true); else PPGAT_TN(2, true);
  } else {
    if (NVk == 0) PPGAT_TN(0, false); else if (NVk == 1) PPGAT_TN(1, false); else PPGAT_TN(2, false);
  }
#undef PPGAT_TN
  TnReduceArg ra{};
  ra.part = a.part; ra.vpart = a.vpart; ra.cpart = a.cpart; ra.splits = nb; ra.M = M; ra.K = K; ra.nv = nv;
  ra.out = out; ra.vout = vout; ra.colsum = colsum;
  const int64_t elems = kPT * kPT + 2 * kPT + (colsum ? kPT : 0);
  hipLaunchKernelGGL(k_tn_reduce, dim3((unsigned)((elems + 63) / 64)), dim3(1024), 0, st, ra);
  return hipGetLastError();
}

hipError_t wgrad_assemble(const float* G, const float* GV, const float* W, const float* att_src, const float* att_dst,
                          int heads, int C, int K, float* dW, float* datt_src, float* datt_dst, hipStream_t st) {
  const int HC = heads * C;
  const unsigned g = (unsigned)((HC + 3) / 4 < 256 ? (HC + 3) / 4 : 256);
  hipLaunchKernelGGL(k_wgrad, dim3(g), dim3(256), 0, st, G, GV, W, att_src, att_dst, heads, C, K, dW, datt_src,
                     datt_dst);
  return hipGetLastError();
}

int adam_max_tensors() { return kAdamMax; }

hipError_t adam_step(int count, float* const* p, const float* const* g, float* const* m, float* const* v,
                     const int64_t* n, const float* step_size, const float* bc2_sqrt, double beta1, double beta2,
                     float eps, float wd, hipStream_t st) {
  AdamArg a{};
  a.count = count;
  a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.omb1 = (float)(1.0 - beta1); a.omb2 = (float)(1.0 - beta2);
  a.eps = eps; a.wd = wd;
  int64_t blocks = 0;
  for (int t = 0; t < count; ++t) {
    a.p[t] = p[t]; a.g[t] = g[t]; a.m[t] = m[t]; a.v[t] = v[t]; a.n[t] = n[t];
    a.step_size[t] = step_size[t]; a.bc2_sqrt[t] = bc2_sqrt[t];
    blocks += (n[t] + kAdamPerBlock - 1) / kAdamPerBlock;
    a.blk_end[t] = blocks;
  }
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace ppgat
