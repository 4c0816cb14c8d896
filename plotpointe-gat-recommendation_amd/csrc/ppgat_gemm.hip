// ppgat_gemm.hip -- the GAT layer's projection GEMMs on the fp32 matrix cores, with the
// layer's per-node work fused into their epilogues, the weight-gradient GEMM, the
// weight-gradient assembly and the optimizer update (gfx950 / MI355X).
//
//  * k_proj16<0>: h = x W^T (+ bias) for x [N, K<=128], W [128, K]  -- GATConv.lin / item_proj
//    (scripts/train_gat_pyg.py:74,77,81; train_gat_custom.py:66,77), with the node attention
//    terms s_src = h.att_src, s_dst = h.att_dst (PyG alpha_src/alpha_dst; custom :79) in the
//    epilogue, so h is never re-read for them.  x may come from two row segments (users from
//    user_emb, items from the item projection: train_gat_pyg.py:79-82) -- no concatenation.
//  * k_proj16<1>: dx = D W + ds_src (x) A_src + ds_dst (x) A_dst (heads = 1), the input
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
// MFMA: v_mfma_f32_16x16x4_f32 (projections) and v_mfma_f32_32x32x2_f32 (k_tn128), exact
// fp32 FMA chains (MI355X_MICROARCH.md: 157 TF peak; 32 / 64 cycles per instruction per
// SIMD).  32x32x2 lane maps (l = lane, r = l & 31, hf = l >> 5):
//   A operand A'[i = r][kk = hf], B operand B'[kk = hf][j = r],
//   accumulator register q: row (q & 3) + 8 (q >> 2) + 4 hf, column r.
// The reduction index of each MFMA is free to permute as long as A and B agree, which is
// what lets every operand come from one contiguous float4 per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ppgat_internal.h"
#include "ppgat_lanes.h"
#include "ppgat_split.h"

// Projection kernel occupancy: 2 waves per SIMD (256 VGPRs, two workgroups per CU).
#ifndef PPGAT_PROJ16_OCC
#define PPGAT_PROJ16_OCC 2
#endif
// Experiment hook for tools/bench_gemm.py (0 in every product build): bit 0 skips the x
// loads of the projection kernel, bit 1 its MFMAs, bit 2 its epilogue stores, bit 3 its LDS
// reads of W.
#ifndef PPGAT_PROJ_VARIANT
#define PPGAT_PROJ_VARIANT 0
#endif

namespace ppgat {

#if PPGAT_CLOCK_PROBE
// Diagnostic builds only (tools/build_variants.sh -DPPGAT_CLOCK_PROBE=1): per-wave shader
// clock and 100 MHz real-time deltas of the projection / weight-gradient kernels, read by
// ppgat_debug_clock_mhz.  Nothing else reads these words.
__device__ unsigned long long g_probe[2][4096][2];
#define PPGAT_PROBE_BEGIN                                            \
  const unsigned long long probe_t0 = __builtin_amdgcn_s_memtime(); \
  const unsigned long long probe_r0 = __builtin_amdgcn_s_memrealtime();
#define PPGAT_PROBE_END(SLOT, WAVE)                                                            \
  if ((threadIdx.x & 63) == 0 && (WAVE) < 4096) {                                              \
    volatile unsigned long long* pp = &g_probe[SLOT][WAVE][0];                                 \
    pp[0] = __builtin_amdgcn_s_memtime() - probe_t0;                                           \
    pp[1] = __builtin_amdgcn_s_memrealtime() - probe_r0;                                       \
  }
#else
#define PPGAT_PROBE_BEGIN
#define PPGAT_PROBE_END(SLOT, WAVE)
#endif

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

// wave-uniform 64-bit value forced into scalar registers
__device__ __forceinline__ int64_t sgpr(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
// ... and as a global-address-space pointer (plain loads, not flat ones that also count
// against the LDS wait counter)
using gfloat = __attribute__((address_space(1))) const float;
__device__ __forceinline__ gfloat* sgpr(const float* p) {
  return (gfloat*)(uintptr_t)sgpr((int64_t)reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ float4 ld4(gfloat* p) {
  using v4 = __attribute__((ext_vector_type(4))) float;
  const v4 v = *(__attribute__((address_space(1))) const v4*)p;
  return make_float4(v.x, v.y, v.z, v.w);
}

// ---------------------------------------------------------------------------
// projection GEMM with fused epilogues
// ---------------------------------------------------------------------------
constexpr int kPT = 128;       // output columns (one tile)

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

// ---------------------------------------------------------------------------
// projection GEMM, one wave per 16-row tile (v_mfma_f32_16x16x4_f32)
//
// Every wave owns whole output rows: a 16 x 128 tile with the full reduction (K <= 128), so
// no partial tiles are exchanged and the waves never synchronise after the prologue.  W is
// staged once per workgroup in LDS as B'[j][k] (row stride 132 floats: the 16 lanes of a
// ds_read_b128 row hit 64 distinct banks) and re-read per tile, one ds_read_b128 per four
// MFMAs.  Lane l = (jl = l & 15, kq = l >> 4): A operand x[row jl][k = 32 kq + s], B operand
// B'[col 16 cb + jl][k = 32 kq + s] (the reduction index is permuted: each lane reads 128
// contiguous bytes of its x row), accumulator q = row 4 kq + q, column 16 cb + jl.
// Software pipeline per iteration (tile t): x (and ds) of tile t + nw in flight; the MFMAs
// of tile t; the epilogue of tile t - nw (its raw accumulators kept from the previous
// iteration) -- bias / rank-2 terms, node scores, stores clipped by buffer descriptors --
// scheduled into the MFMA shadows.
// ---------------------------------------------------------------------------
constexpr int kP16Ld = kPT + 4;
// LDS column of reduction index k in a B' row: the 32-wide k chunks 1 and 2 trade places, so
// the two k chunks met by each 16-lane group of a ds_read_b128 ({0-3,12-15,20-27}, ...) start
// on the same bank slot and the group's 16 lanes cover 16 distinct slots (no 2-way conflict)
__host__ __device__ constexpr int p16_col(int k) {
  return ((k >> 5) == 1 ? 64 : (k >> 5) == 2 ? 32 : (k & ~31)) + (k & 31);
}
using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// 8 per-lane values (index v = 4 h + q), each summed over the 16 lanes of a row.  On return
// lane jl holds the full sum for index 4 ((jl >> 3) & 1) + 2 ((jl >> 2) & 1) + ((jl >> 1) & 1)
// (lanes jl and jl ^ 1 agree).  Pairing: ror 8, half-row mirror, xor 2, xor 1 -- every final
// value covers all 16 lanes exactly once.
__device__ __forceinline__ float reduce8_over16(float (&v)[8], int jl) {
  const bool b3 = (jl & 8) != 0, b2 = (jl & 4) != 0, b1 = (jl & 2) != 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float send = b3 ? v[t] : v[4 + t];
    const float keep = b3 ? v[4 + t] : v[t];
    v[t] = keep + dpp<0x128>(send);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const float send = b2 ? v[t] : v[2 + t];
    const float keep = b2 ? v[2 + t] : v[t];
    v[t] = keep + dpp<0x141>(send);
  }
  {
    const float send = b1 ? v[0] : v[1];
    const float keep = b1 ? v[1] : v[0];
    v[0] = keep + dpp<0x4E>(send);
  }
  return v[0] + dpp<0xB1>(v[0]);
}

template <int MODE>
__global__ void __launch_bounds__(256, PPGAT_PROJ16_OCC) k_proj16(ProjArg a) {
  __shared__ float4 sW4[kPT * kP16Ld / 4];
  __shared__ float sV[2][kPT];  // att (mode 0) / A = att W (mode 1)
  float* sW = reinterpret_cast<float*>(sW4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int jl = lane & 15, kq = lane >> 4;
  const int K = a.K;
  // ---- stage B'[j][k] (zero-padded to 128 x 128) and the attention vectors ----
  if (MODE == 0) {
    for (int idx = tid; idx < kPT * 32; idx += 256) {
      const int j = idx >> 5, k4 = (idx & 31) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k4 < K) v = ld4(a.W + (int64_t)j * a.ldw + k4);
      st4(&sW[j * kP16Ld + p16_col(k4)], v);
    }
  } else {
    for (int idx = tid; idx < kPT * 32; idx += 256) {
      const int k = idx >> 5, j4 = (idx & 31) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < K) v = ld4(a.W + (int64_t)k * a.ldw + j4);
      const int c = p16_col(k);
      sW[(j4 + 0) * kP16Ld + c] = v.x;
      sW[(j4 + 1) * kP16Ld + c] = v.y;
      sW[(j4 + 2) * kP16Ld + c] = v.z;
      sW[(j4 + 3) * kP16Ld + c] = v.w;
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
    for (int k = 0; k < kPT; ++k) s = fmaf(sV[v][k], sW[j * kP16Ld + p16_col(k)], s);
    __syncthreads();
    sV[v][j] = s;
    __syncthreads();
  }
  PPGAT_PROBE_BEGIN
  float va[8], vb[8], bias[8];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) {
    const int c = 16 * cb + jl;
    va[cb] = vec ? sV[0][c] : 0.f;
    vb[cb] = vec ? sV[1][c] : 0.f;
    bias[cb] = (MODE == 0 && a.bias) ? a.bias[c] : 0.f;
  }
  gfloat* const x0 = sgpr(a.x0);
  gfloat* const x1 = sgpr(a.x1);
  const int64_t ldx0 = sgpr(a.ldx0), ldx1 = sgpr(a.ldx1), split = sgpr(a.split), n = sgpr(a.n);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t wave = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t tiles = (n + 15) / 16;
  const int64_t iters = (tiles + nw - 1) / nw;  // the same for every wave
  const float* sWl = sW + jl * kP16Ld + p16_col(32 * kq);

  // x loads are unconditional (a select on a loaded value makes hipcc wait for the load right
  // there, serialising the prefetch): rows past n read row n - 1 (never stored), columns
  // past K read in-row columns < K that meet zero rows of B'
  auto load_x = [&](int64_t tile, float4 (&xv)[8]) {
    if (PPGAT_PROJ_VARIANT & 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) xv[q] = make_float4(tile, q, jl, 1.f);
      return;
    }
    int64_t row = tile * 16 + jl;
    row = row < n ? row : n - 1;
    gfloat* src = row < split ? x0 + row * ldx0 : x1 + (row - split) * ldx1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = 32 * kq + 4 * q;
      xv[q] = ld4(src + (c < K ? c : K - 4));
    }
  };
  auto load_d = [&](int64_t tile, float2 (&dv)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int64_t row = tile * 16 + 4 * kq + q;
      row = min(max(row, (int64_t)0), n - 1);
      dv[q] = *reinterpret_cast<const float2*>(a.ds + row * a.ldds);
    }
  };
  // epilogue of tile tt from its raw accumulators (a no-op store-wise for tt < 0 or past
  // the last tile: the descriptors then hold no records)
  auto finalize = [&](int64_t tt, const f32x4 (&ac)[8], const float2 (&dv)[4]) {
    const int64_t row0 = tt * 16;
    const int64_t live = min(min(max(n - row0, (int64_t)0), (int64_t)16), max(row0 + 16, (int64_t)0));
    const int64_t base = max(row0, (int64_t)0);
    const auto ry = __builtin_amdgcn_make_buffer_rsrc(a.y + base * a.ldy, 0, (int)(live * a.ldy * 4), 0x00020000);
    float ps[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) { ps[q] = 0.f; ps[4 + q] = 0.f; }
#pragma unroll
    for (int cb = 0; cb < 8; ++cb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = ac[cb][q];
        if (MODE == 1) {
          v = fmaf(dv[q].y, vb[cb], fmaf(dv[q].x, va[cb], v));
        } else {
          ps[q] = fmaf(v, va[cb], ps[q]);
          ps[4 + q] = fmaf(v, vb[cb], ps[4 + q]);
          v += bias[cb];
        }
        if (!(PPGAT_PROJ_VARIANT & 4) || v == 12345.f)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ry,
                                                (int)(((4 * kq + q) * a.ldy + 16 * cb + jl) * 4), 0, 0);
      }
    if (MODE == 0 && vec) {
      const float sv = reduce8_over16(ps, jl);
      const int rr = 4 * kq + 2 * ((jl >> 2) & 1) + ((jl >> 1) & 1);
      const bool wr = (jl & 1) == 0, dst = (jl & 8) != 0;
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.s_src + base, 0, (int)(live * 4), 0x00020000);
      const auto rd = __builtin_amdgcn_make_buffer_rsrc(a.s_dst + base, 0, (int)(live * 4), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sv), rs, (wr && !dst) ? rr * 4 : 0x40000000, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sv), rd, (wr && dst) ? rr * 4 : 0x40000000, 0, 0);
    }
  };

  float4 xr[8];
  float2 dcur[4], dprev[4];
  f32x4 accp[8];
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) accp[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) dcur[q] = dprev[q] = make_float2(0.f, 0.f);
  load_x(wave, xr);
  if (MODE == 1) load_d(wave, dcur);
  for (int64_t it = 0; it < iters; ++it) {
    const int64_t t = wave + it * nw;
    float4 xn[8];
    float2 dn[4];
    load_x(t + nw, xn);  // next tile in flight
    if (MODE == 1) load_d(t + nw, dn);
    f32x4 acc[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < 8; ++s4) {
      float4 bf[8];
#pragma unroll
      for (int cb = 0; cb < 8; ++cb)
        bf[cb] = (PPGAT_PROJ_VARIANT & 8) ? make_float4(va[cb], vb[cb], s4, cb)
                                          : *reinterpret_cast<const float4*>(sWl + cb * 16 * kP16Ld + 4 * s4);
      if (!(PPGAT_PROJ_VARIANT & 2)) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int cb = 0; cb < 8; ++cb) acc[cb] = mfma16(comp(xr[s4], e), comp(bf[cb], e), acc[cb]);
      } else {
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) acc[cb][0] += xr[s4].x * bf[cb].y;
      }
    }
    finalize(t - nw, accp, dprev);
#pragma unroll
    for (int g = 0; g < 256; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x3F6, 2, 0);  // then up to two other instructions
    }
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) accp[cb] = acc[cb];
#pragma unroll
    for (int q = 0; q < 8; ++q) xr[q] = xn[q];
    if (MODE == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) { dprev[q] = dcur[q]; dcur[q] = dn[q]; }
    }
  }
  finalize(wave + (iters - 1) * nw, accp, dprev);
  PPGAT_PROBE_END(0, wave)
}

// ---------------------------------------------------------------------------
// projection GEMM, one wave per 32-row tile (v_mfma_f32_32x32x2_f32), K in {64, 128}
//
// Same contract as k_proj16 (both modes, both epilogues).  Each wave owns 32 x 128 output
// tiles with the full reduction: four 32 x 32 accumulator blocks (64 accumulation registers).
// Reduction order per lane (r, hf): step s = 4 q + e takes k = 8 q + 4 hf + e, so lane (r, hf)
// holds x[row r][8 q + 4 hf .. + 3] as one float4 per q (a wave's load q covers 32 B of each
// of its 32 rows) and reads B'[32 cb + r][8 q + 4 hf .. + 3] from LDS as one ds_read_b128 per
// four MFMAs of 64 cycles -- half the LDS reads per MFMA cycle of the 16 x 16 x 4 design.  The
// next tile's x is loaded into each float4 right after its last use (one tile of x in
// registers), the epilogue runs while the SIMD's other wave keeps the matrix pipe busy.
// Node scores: 32 per-lane partial sums (16 rows x {src, dst}) reduced over the 32 lanes of
// each half by transposing butterflies; each lane then stores one (row, vector) value.
// ---------------------------------------------------------------------------
template <int MODE, int KQ>
__global__ void __launch_bounds__(256, 2) k_proj32(ProjArg a) {
  constexpr int K = 8 * KQ;
  constexpr int LD = K + 4;  // B' row stride: the 16 lanes of a ds_read_b128 group hit 64 banks
  __shared__ float4 sW4[kPT * LD / 4];
  __shared__ float sV[2][kPT];
  float* sW = reinterpret_cast<float*>(sW4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int r = lane & 31, hf = lane >> 5;
  if (MODE == 0) {
    for (int idx = tid; idx < kPT * K / 4; idx += 256) {
      const int j = idx / (K / 4), k4 = (idx % (K / 4)) * 4;
      st4(&sW[j * LD + k4], ld4(a.W + (int64_t)j * a.ldw + k4));
    }
  } else {
    for (int idx = tid; idx < kPT * K / 4; idx += 256) {
      const int k = idx >> 5, j4 = (idx & 31) * 4;
      const float4 v = ld4(a.W + (int64_t)k * a.ldw + j4);
      sW[(j4 + 0) * LD + k] = v.x;
      sW[(j4 + 1) * LD + k] = v.y;
      sW[(j4 + 2) * LD + k] = v.z;
      sW[(j4 + 3) * LD + k] = v.w;
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
    for (int k = 0; k < K; ++k) s = fmaf(sV[v][k], sW[j * LD + k], s);
    __syncthreads();
    sV[v][j] = s;
    __syncthreads();
  }
  float va[4], vb[4], bias[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int c = 32 * cb + r;
    va[cb] = vec ? sV[0][c] : 0.f;
    vb[cb] = vec ? sV[1][c] : 0.f;
    bias[cb] = (MODE == 0 && a.bias) ? a.bias[c] : 0.f;
  }
  gfloat* const x0 = sgpr(a.x0);
  gfloat* const x1 = sgpr(a.x1);
  const int64_t ldx0 = sgpr(a.ldx0), ldx1 = sgpr(a.ldx1), split = sgpr(a.split), n = sgpr(a.n);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t wave = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t tiles = (n + 31) / 32;
  const int64_t iters = (tiles + nw - 1) / nw;  // the same for every wave
  const float* sWl = sW + r * LD + 4 * hf;
  // rows past n read row n - 1 (never stored)
  auto row_src = [&](int64_t tile) -> gfloat* {
    int64_t row = tile * 32 + r;
    row = row < n ? row : n - 1;
    return row < split ? x0 + row * ldx0 : x1 + (row - split) * ldx1;
  };
  float4 xr[KQ];
  {
    gfloat* src = row_src(wave);
#pragma unroll
    for (int q = 0; q < KQ; ++q) xr[q] = ld4(src + 8 * q + 4 * hf);
  }
  for (int64_t it = 0; it < iters; ++it) {
    const int64_t t = wave + it * nw;
    const int64_t row0 = t * 32;
    float2 dv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) dv[q] = make_float2(0.f, 0.f);
    if (MODE == 1 && a.ds != nullptr) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        int64_t row = row0 + (q & 3) + 8 * (q >> 2) + 4 * hf;
        row = row < n ? row : n - 1;
        dv[q] = *reinterpret_cast<const float2*>(a.ds + row * a.ldds);
      }
    }
    gfloat* nsrc = row_src(t + nw);
    f32x16 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[cb][i] = 0.f;
    // B' fragments one q ahead; the scheduling barrier keeps the compiler from hoisting every
    // LDS read of the tile (256 registers) above the MFMAs, or sinking them onto their use
    float4 bq[4], bn[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) bq[cb] = *reinterpret_cast<const float4*>(sWl + cb * 32 * LD);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      if (q + 1 < KQ) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) bn[cb] = *reinterpret_cast<const float4*>(sWl + cb * 32 * LD + 8 * (q + 1));
      }
      __builtin_amdgcn_sched_barrier(0);  // the q + 1 reads stay ahead of the q MFMAs
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] = mfma(comp(xr[q], e), comp(bq[cb], e), acc[cb]);
      xr[q] = ld4(nsrc + 8 * q + 4 * hf);  // next tile, into the registers just consumed
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) bq[cb] = bn[cb];
    }
    // ---- epilogue ----
    const int64_t live = row0 < n ? (n - row0 < 32 ? n - row0 : 32) : 0;
    const auto ry = __builtin_amdgcn_make_buffer_rsrc(a.y + (live ? row0 * a.ldy : 0), 0, (int)(live * a.ldy * 4),
                                                      0x00020000);
    const int64_t ldy = sgpr(a.ldy);
    int voff = (int)((4 * hf * ldy + r) * 4);
    asm volatile("" : "+v"(voff));  // per tile: keeps the 16 row offsets from being hoisted
    float ps[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) ps[i] = 0.f;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        float v = acc[cb][q];
        if (MODE == 1) {
          v = fmaf(dv[q].y, vb[cb], fmaf(dv[q].x, va[cb], v));
        } else {
          ps[q] = fmaf(v, va[cb], ps[q]);
          ps[16 + q] = fmaf(v, vb[cb], ps[16 + q]);
          v += bias[cb];
        }
        // every offset in the VGPR operand (the descriptor's range check clips the tail rows);
        // the column block goes to the instruction's immediate offset
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ry,
                                              voff + (int)(((q & 3) + 8 * (q >> 2)) * ldy * 4) + 128 * cb, 0, 0);
      }
    if (MODE == 0 && vec) {
      float res = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float v4[4] = {ps[4 * c], ps[4 * c + 1], ps[4 * c + 2], ps[4 * c + 3]};
        const float s = transpose_reduce<32, 4>(v4, r);  // value 4 c + (r >> 3)
        res = (r & 7) == c ? s : res;
      }
      const int v = 4 * (r & 7) + (r >> 3);
      const int q = v & 15;
      const int row = (q & 3) + 8 * (q >> 2) + 4 * hf;
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((v < 16 ? a.s_src : a.s_dst) + (live ? row0 : 0), 0,
                                                        (int)(live * 4), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(res), rs, row * 4, 0, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// out[M, K] = A^T B (+ V^T B, colsum A), M, K <= 128
//
// Workgroup = 8 waves = 4 pairs, one workgroup per CU (two waves per SIMD).  A pair owns a
// contiguous range of rows; its wave mh accumulates the m-half [64 mh, 64 mh + 64) of the
// 128 x 128 output (128 accumulation registers), streaming float2 of A and float4 of B per
// lane straight from HBM into the MFMA operand layout: lane (r, hf) takes row base + 2p + hf,
// A'[m = 64 mh + 2 r + i][kk = hf], B'[kk = hf][k = 4 r + j].  Wave mh also forms V[:, mh]^T B
// (on the VALU) and colsum over its m-half.  Pair partials are summed through LDS in pair
// order, then an ordered split reduction across workgroups (deterministic).
// ---------------------------------------------------------------------------
constexpr int kTnPairs = 4;  // row pairs per prefetch batch
constexpr int kTnWaves = 8;

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
  int64_t rows_per_pair;  // even
  float* part;   // [gridDim.x][128][128] (m-major)
  float* vpart;  // [gridDim.x][2][128]
  float* cpart;  // nullable: [gridDim.x][128]
};

// One batch of kTnPairs row pairs: lane (r, hf) takes row base + 2p + hf.
template <bool MASK>
__device__ __forceinline__ void tn_load(const float* pa, const float* pb, const float* pv, int64_t sa, int64_t sb,
                                        int64_t sv, bool am, bool bk, float2 (&av)[kTnPairs], float4 (&bv)[kTnPairs],
                                        float (&vv)[kTnPairs]) {
#pragma unroll
  for (int p = 0; p < kTnPairs; ++p) {
    av[p] = *reinterpret_cast<const float2*>(pa + p * sa);
    bv[p] = ld4(pb + p * sb);
    vv[p] = pv[p * sv];
    if (MASK) {
      if (!am) av[p] = make_float2(0.f, 0.f);
      if (!bk) bv[p] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

template <bool HASV>
__device__ __forceinline__ void tn_compute(f32x16 (&acc)[2][4], float4& vacc, float2& csum,
                                           const float2 (&av)[kTnPairs], const float4 (&bv)[kTnPairs],
                                           const float (&vv)[kTnPairs]) {
#pragma unroll
  for (int p = 0; p < kTnPairs; ++p) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma(i ? av[p].y : av[p].x, comp(bv[p], j), acc[i][j]);
    if (HASV) {
      vacc.x = fmaf(vv[p], bv[p].x, vacc.x);
      vacc.y = fmaf(vv[p], bv[p].y, vacc.y);
      vacc.z = fmaf(vv[p], bv[p].z, vacc.z);
      vacc.w = fmaf(vv[p], bv[p].w, vacc.w);
    }
    csum.x += av[p].x;
    csum.y += av[p].y;
  }
}

template <int NV, bool MASK>
__global__ void __launch_bounds__(64 * kTnWaves, 1) k_tn128(TnArg a) {
  __shared__ float sR[kPT][kPT + 4];
  __shared__ float sVr[kTnWaves / 2][2][kPT];
  __shared__ float sC[kTnWaves / 2][kPT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int mh = w & 1, pr = w >> 1;
  const int64_t pid = (int64_t)blockIdx.x * (kTnWaves / 2) + pr;
  const int64_t n_beg = pid * a.rows_per_pair;
  const int64_t n_end = min(a.n, n_beg + a.rows_per_pair);
  const int mcol = 64 * mh + 2 * r;
  const bool am = !MASK || mcol < a.M, bk = !MASK || 4 * r < a.K;
  const int acol = am ? mcol : 0, bcol = bk ? 4 * r : 0;  // masked lanes read column 0, zeroed after
  const bool hasv = mh < NV;
  const int vcol = hasv ? mh : 0;
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  float4 vacc = make_float4(0.f, 0.f, 0.f, 0.f);
  float2 csum = make_float2(0.f, 0.f);
  PPGAT_PROBE_BEGIN
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
    const float* pv = a.V + (r0 + hf) * a.ldv + vcol;
    float2 av[kTnPairs];
    float4 bv[kTnPairs];
    float vv[kTnPairs];
    if (full > 0) {
      tn_load<MASK>(pa, pb, pv, sa, sb, sv, am, bk, av, bv, vv);
      for (int64_t bt = 1; bt < full; ++bt) {
        pa += kTnPairs * sa;
        pb += kTnPairs * sb;
        pv += kTnPairs * sv;
        float2 an[kTnPairs];
        float4 bn[kTnPairs];
        float vn[kTnPairs];
        tn_load<MASK>(pa, pb, pv, sa, sb, sv, am, bk, an, bn, vn);  // in flight during the MFMAs
        __builtin_amdgcn_sched_barrier(0);
        tn_compute<NV != 0>(acc, vacc, csum, av, bv, vv);
#pragma unroll
        for (int p = 0; p < kTnPairs; ++p) {
          av[p] = an[p];
          bv[p] = bn[p];
          vv[p] = vn[p];
        }
      }
      tn_compute<NV != 0>(acc, vacc, csum, av, bv, vv);
    }
    // tail (< 2 kTnPairs rows): out-of-range pairs read the segment's first row, zeroed
    const int64_t t0 = r0 + full * 2 * kTnPairs;
    if (t0 < r1) {
#pragma unroll
      for (int p = 0; p < kTnPairs; ++p) {
        const bool ok = t0 + 2 * p + hf < r1;
        const int64_t row = ok ? t0 + 2 * p + hf : r0;
        const float2 va = *reinterpret_cast<const float2*>(a.A + row * a.lda + acol);
        const float4 vb = ld4(bbase + (row - boff) * ldb + bcol);
        av[p] = (ok && am) ? va : make_float2(0.f, 0.f);
        bv[p] = (ok && bk) ? vb : make_float4(0.f, 0.f, 0.f, 0.f);
        const float v = NV > 0 ? a.V[row * a.ldv + vcol] : 0.f;
        vv[p] = ok ? v : 0.f;
      }
      tn_compute<NV != 0>(acc, vacc, csum, av, bv, vv);
    }
  }
  PPGAT_PROBE_END(1, blockIdx.x * kTnWaves + w)
  // ---- workgroup reduction through LDS, pairs in order 0..3 ----
  // acc[i][j][q]: m = 64 mh + 2 acc_row(q, hf) + i, k = 4 r + j
  auto put = [&](bool add) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = 64 * mh + 2 * acc_row(q, hf) + i;
        float4 v = make_float4(acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]);
        float* dst = &sR[m][4 * r];
        if (add) {
          const float4 o = *reinterpret_cast<const float4*>(dst);
          v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        }
        st4(dst, v);
      }
  };
  // (no loop over turns: a loop lets the compiler hoist all accumulator reads)
  if (pr == 0) put(false);
  __syncthreads();
  if (pr == 1) put(true);
  __syncthreads();
  if (pr == 2) put(true);
  __syncthreads();
  if (pr == 3) put(true);
  // V and colsum: combine the two half-waves (lane, lane ^ 32), then the pairs in order
  {
    float t[4] = {vacc.x, vacc.y, vacc.z, vacc.w};
    float c[2] = {csum.x, csum.y};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x0, x1;
      row_swap<32>(t[e], t[e], x0, x1);
      t[e] = x0 + x1;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float x0, x1;
      row_swap<32>(c[e], c[e], x0, x1);
      c[e] = x0 + x1;
    }
    if (hf == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sVr[pr][mh][4 * r + e] = hasv ? t[e] : 0.f;
      sC[pr][mcol] = c[0];
      sC[pr][mcol + 1] = c[1];
    }
  }
  __syncthreads();
  float* P = a.part + (int64_t)blockIdx.x * kPT * kPT;
  for (int idx = tid; idx < kPT * kPT / 4; idx += 64 * kTnWaves) {
    const int m = idx >> 5, k4 = (idx & 31) * 4;
    st4(P + m * kPT + k4, *reinterpret_cast<const float4*>(&sR[m][k4]));
  }
  if (tid < 2 * kPT) {
    const int v = tid >> 7, k = tid & 127;
    a.vpart[((int64_t)blockIdx.x * 2 + v) * kPT + k] =
        ((sVr[0][v][k] + sVr[1][v][k]) + sVr[2][v][k]) + sVr[3][v][k];
  } else if (a.cpart && tid < 3 * kPT) {
    const int m = tid - 2 * kPT;
    a.cpart[(int64_t)blockIdx.x * kPT + m] = ((sC[0][m] + sC[1][m]) + sC[2][m]) + sC[3][m];
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
  const float* tstep[kAdamMax];  // non-null: step_size / bc2_sqrt from tensor t's device step count (graph replays)
  double lr, b1d, b2d;
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
  float ss = a.step_size[ti], bc = a.bc2_sqrt[ti];
  if (a.tstep[ti] != nullptr) {  // the host formulas of optim.Adam, in double, rounded once
    const double t = (double)*a.tstep[ti];
    ss = (float)(a.lr / (1.0 - pow(a.b1d, t)));
    bc = (float)sqrt(1.0 - pow(a.b2d, t));
  }
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

// ---------------------------------------------------------------------------
// fp32 GEMMs on the bf16 matrix cores: three-term split ("bf16x6", ppgat_split.h)
// ---------------------------------------------------------------------------
using split::mfma32_x6;
using split::mfma_x6;
using split::split3;

// LDS image of the split B' (three parts, [128 rows][128 k] bf16, 256-B rows, no padding).
// 16-B unit of (row n, reduction index k) within its row: the lane (jl = l & 15, kq = l >> 4)
// reads unit 4 kq + s of row 16 cb + jl for k step s; rotating by jl and swapping the kq
// pairs {0,1}, {2,3} of rows jl in [4, 12) makes the 16 lanes of every ds_read_b128 group
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) land on 16 distinct 16-B bank slots.
__host__ __device__ constexpr int xs_unit(int n, int k) {
  return (4 * ((k >> 5) ^ ((((n & 15) >= 4) && ((n & 15) < 12)) ? 1 : 0)) + ((k >> 3) & 3) + (n & 15)) & 15;
}
constexpr int kXsPart = kPT * kPT * 2;  // bytes per split part
constexpr int kXsWaves = 8;

// ---------------------------------------------------------------------------
// projection GEMM on the split bf16 matrix cores (same contract as k_proj16, both modes)
//
// One workgroup per CU (96 KB of split B' in LDS), 8 waves, each wave persistent over 16-row
// tiles.  The product is computed transposed: A = B' (output column n on the lane's row
// slot), B = x (row jl of the tile on the lane's column slot), so the accumulator of column
// block cb holds y[row jl][16 cb + 4 kq + q] in register q -- one float4 store per block --
// and the node scores reduce over the four kq lane groups only.  x: lane (jl, kq) loads
// x[row][32 kq .. 32 kq + 31] (8 float4, the reduction index permuted as in k_proj16), the
// next tile's x in flight during the MFMAs; k step s uses its float4 pair 2 s, 2 s + 1.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ void __launch_bounds__(64 * kXsWaves, 1) k_projx(ProjArg a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char xs_lds[];
  unsigned char* sW = xs_lds;                                          // 3 parts
  float* sV = reinterpret_cast<float*>(xs_lds + 3 * kXsPart);          // [2][128] att / A
  float* sB = sV + 2 * kPT;                                            // [128] bias
  float* sP = sB + kPT;  // mode 1: [2][16][128] partial A = att W per 8-k chunk
  const int tid = threadIdx.x, lane = tid & 63;
  const int jl = lane & 15, kq = lane >> 4;
  const int K = a.K;
  gfloat* const x0 = sgpr(a.x0);
  gfloat* const x1 = sgpr(a.x1);
  const int64_t ldx0 = sgpr(a.ldx0), ldx1 = sgpr(a.ldx1), split = sgpr(a.split), n = sgpr(a.n);
  const int64_t nw = (int64_t)gridDim.x * kXsWaves;
  const int64_t wave = (int64_t)blockIdx.x * kXsWaves + __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t tiles = (n + 15) / 16;
  int aoff[4];  // byte offset of this lane's A unit for k step s (column block 0)
#pragma unroll
  for (int s = 0; s < 4; ++s) aoff[s] = jl * 256 + xs_unit(jl, 32 * kq + 8 * s) * 16;

  auto load_x = [&](int64_t tile, float4 (&xv)[8]) {
    int64_t row = tile * 16 + jl;
    row = row < n ? row : n - 1;
    gfloat* src = row < split ? x0 + row * ldx0 : x1 + (row - split) * ldx1;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = 32 * kq + 4 * q;
      xv[q] = ld4(src + (c < K ? c : K - 4));
    }
  };

  // the first tile's x is in flight while B' is staged
  float4 xa[8], xb[8];
  if (wave < tiles) load_x(wave, xa);
  // ---- stage split B'[n][k] (zero past K) ----
  for (int idx = tid; idx < kPT * 16; idx += 64 * kXsWaves) {
    const int n = idx & 127, c = idx >> 7, k0 = 8 * c;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f), q = p;
    if (MODE == 0) {
      if (k0 < K) p = ld4(a.W + (int64_t)n * a.ldw + k0);
      if (k0 + 4 < K) q = ld4(a.W + (int64_t)n * a.ldw + k0 + 4);
    } else {
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = (k0 + j < K) ? a.W[(int64_t)(k0 + j) * a.ldw + n] : 0.f;
      p = make_float4(t[0], t[1], t[2], t[3]);
      q = make_float4(t[4], t[5], t[6], t[7]);
      if (a.att_src) {  // partial A_v[n] over this 8-k chunk (summed over the chunks in order below)
        float ps = 0.f, pd = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (k0 + j < K) {
            ps = fmaf(a.att_src[k0 + j], t[j], ps);
            pd = fmaf(a.att_dst[k0 + j], t[j], pd);
          }
        }
        sP[c * kPT + n] = ps;
        sP[16 * kPT + c * kPT + n] = pd;
      }
    }
    u32x4 h, m, l;
    split3(p, q, h, m, l);
    const int off = n * 256 + xs_unit(n, k0) * 16;
    *reinterpret_cast<u32x4*>(sW + off) = h;
    *reinterpret_cast<u32x4*>(sW + kXsPart + off) = m;
    *reinterpret_cast<u32x4*>(sW + 2 * kXsPart + off) = l;
  }
  const bool vec = a.att_src != nullptr;
  if (tid < 2 * kPT) {
    const int j = tid & 127, v = tid >> 7;
    float s = 0.f;
    if (vec) {
      const float* att = v ? a.att_dst : a.att_src;
      if (MODE == 0) {
        s = att[j];
      }
    }
    sV[v * kPT + j] = s;
  } else if (tid < 3 * kPT) {
    const int j = tid - 2 * kPT;
    sB[j] = (MODE == 0 && a.bias) ? a.bias[j] : 0.f;
  }
  __syncthreads();
  if (MODE == 1 && vec && tid < 2 * kPT) {  // A_v[j] = sum_k att_v[k] W[k][j], 8-k chunks in order
    const int j = tid & 127, v = tid >> 7;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += sP[v * 16 * kPT + c * kPT + j];
    sV[v * kPT + j] = s;
  }
  if (MODE == 1) __syncthreads();

  // one tile's MFMAs and epilogue; the caller keeps the next tile's x in flight in the other
  // register buffer (ping-pong, so no copy makes the loop wait for the prefetch)
  auto tile_body = [&](int64_t t, const float4 (&xr)[8]) {
    float2 dv = make_float2(0.f, 0.f);
    const int64_t row = t * 16 + jl;
    if (MODE == 1) dv = *reinterpret_cast<const float2*>(a.ds + (row < n ? row : n - 1) * a.ldds);
    f32x4 acc[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 32 (k step, column block) steps; the next step's three A units are read from LDS while
    // the current step's six MFMAs run
    auto read_a = [&](int idx, u32x4 (&f)[3]) {
      const unsigned char* pa = sW + aoff[idx >> 3] + (idx & 7) * 16 * 256;
      f[0] = *reinterpret_cast<const u32x4*>(pa);
      f[1] = *reinterpret_cast<const u32x4*>(pa + kXsPart);
      f[2] = *reinterpret_cast<const u32x4*>(pa + 2 * kXsPart);
    };
    u32x4 fa[3], bh, bm, bl;
    read_a(0, fa);
#pragma unroll
    for (int idx = 0; idx < 32; ++idx) {
      const int s = idx >> 3, cb = idx & 7;
      if (cb == 0) split3(xr[2 * s], xr[2 * s + 1], bh, bm, bl);
      u32x4 fn[3];
      if (idx < 31) read_a(idx + 1, fn);
      acc[cb] = mfma_x6(fa[0], fa[1], fa[2], bh, bm, bl, acc[cb]);
      __builtin_amdgcn_sched_barrier(0);  // keep each LDS read one step ahead (no hoisting)
      if (idx < 31) {
        fa[0] = fn[0];
        fa[1] = fn[1];
        fa[2] = fn[2];
      }
    }
    // ---- epilogue: lane holds y[row][16 cb + 4 kq + q] ----
    float ps = 0.f, pd = 0.f;
    float* yrow = a.y + (row < n ? row : 0) * a.ldy;
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
      const int c0 = 16 * cb + 4 * kq;
      const float4 va = *reinterpret_cast<const float4*>(sV + c0);
      const float4 vb = *reinterpret_cast<const float4*>(sV + kPT + c0);
      float4 o;
      if (MODE == 0) {
        const float4 bb = *reinterpret_cast<const float4*>(sB + c0);
        ps = fmaf(acc[cb][0], va.x, fmaf(acc[cb][1], va.y, fmaf(acc[cb][2], va.z, fmaf(acc[cb][3], va.w, ps))));
        pd = fmaf(acc[cb][0], vb.x, fmaf(acc[cb][1], vb.y, fmaf(acc[cb][2], vb.z, fmaf(acc[cb][3], vb.w, pd))));
        o = make_float4(acc[cb][0] + bb.x, acc[cb][1] + bb.y, acc[cb][2] + bb.z, acc[cb][3] + bb.w);
      } else {
        o = make_float4(fmaf(dv.y, vb.x, fmaf(dv.x, va.x, acc[cb][0])), fmaf(dv.y, vb.y, fmaf(dv.x, va.y, acc[cb][1])),
                        fmaf(dv.y, vb.z, fmaf(dv.x, va.z, acc[cb][2])), fmaf(dv.y, vb.w, fmaf(dv.x, va.w, acc[cb][3])));
      }
      if (row < n) st4(yrow + c0, o);
    }
    if (MODE == 0 && vec) {
      ps += __shfl_xor(ps, 16);
      pd += __shfl_xor(pd, 16);
      ps += __shfl_xor(ps, 32);
      pd += __shfl_xor(pd, 32);
      if (row < n && kq == 0) a.s_src[row] = ps;
      if (row < n && kq == 1) a.s_dst[row] = pd;
    }
  };
  int64_t t = wave;
  while (t < tiles) {
    if (t + nw < tiles) load_x(t + nw, xb);
    tile_body(t, xa);
    t += nw;
    if (t >= tiles) break;
    if (t + nw < tiles) load_x(t + nw, xa);
    tile_body(t, xb);
    t += nw;
  }
}
constexpr size_t kXsLds = 3 * kXsPart + (3 + 32) * kPT * sizeof(float);

// ---------------------------------------------------------------------------
// weight-gradient GEMM on the split bf16 matrix cores (same contract and partial layout as
// k_tn128): out = A^T B, + V^T B and colsum(A) on the VALU in fp32.
//
// v_mfma_f32_32x32x16_bf16 sums over 16 rows per instruction: lane (r, hf) holds rows
// 8 hf + j (j = 0..7) of a 16-row step.  A'[m = 64 mh + 2 r + i] and B'[k = 4 r + kb] as in
// k_tn128, so per row a lane loads one float2 of A and one float4 of B, and the three bf16
// terms of each operand fragment are formed from eight rows of one column.  WV = 8 waves per
// workgroup (four pairs of m halves, two waves per SIMD), one workgroup per CU: 128
// accumulators and one 16-row batch per wave, the SIMD's other wave hiding the load latency.
// WV = 4 (masked shapes): 512 registers per wave, a ring of three batches (two in flight).
// Pair partials are summed through LDS in pair order, then the ordered split reduction
// k_tn_reduce (deterministic).
// ---------------------------------------------------------------------------

constexpr int kTnxSteps = 1;              // MFMA k steps (16 rows each) per batch
constexpr int kTnxRows = 16 * kTnxSteps;  // rows per batch

struct TnxBatch {
  float2 av[kTnxSteps][8];
  float4 bv[kTnxSteps][8];
  float vv[kTnxSteps][8];
};

template <bool HASV>
__device__ __forceinline__ void tnx_compute(f32x16 (&acc)[2][4], float4& vacc, float2& csum, const TnxBatch& b) {
#pragma unroll
  for (int t = 0; t < kTnxSteps; ++t) {
    u32x4 fa[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = i ? b.av[t][j].y : b.av[t][j].x;
      split3(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), fa[i][0], fa[i][1], fa[i][2]);
    }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = comp(b.bv[t][j], kb);
      u32x4 fb[3];
      split3(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), fb[0], fb[1], fb[2]);
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i][kb] = mfma32_x6(fa[i], fb, acc[i][kb]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (HASV) {
        vacc.x = fmaf(b.vv[t][j], b.bv[t][j].x, vacc.x);
        vacc.y = fmaf(b.vv[t][j], b.bv[t][j].y, vacc.y);
        vacc.z = fmaf(b.vv[t][j], b.bv[t][j].z, vacc.z);
        vacc.w = fmaf(b.vv[t][j], b.bv[t][j].w, vacc.w);
      }
      csum.x += b.av[t][j].x;
      csum.y += b.av[t][j].y;
    }
  }
}

template <int NV, bool MASK, int WV>
__global__ void __launch_bounds__(64 * WV, 1) k_tnx(TnArg a) {
  constexpr bool RING = WV == 4;  // 8 waves (2 per SIMD): no batches in flight, the other wave hides latency
  __shared__ float sR[kPT][kPT + 4];
  __shared__ float sVr[WV / 2][2][kPT];
  __shared__ float sC[WV / 2][kPT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int mh = w & 1, pr = w >> 1;
  const int64_t pid = (int64_t)blockIdx.x * (WV / 2) + pr;
  const int64_t n_beg = pid * a.rows_per_pair;
  const int64_t n_end = min(a.n, n_beg + a.rows_per_pair);
  const int mcol = 64 * mh + 2 * r;
  const bool am = !MASK || mcol < a.M, bk = !MASK || 4 * r < a.K;
  const int acol = am ? mcol : 0, bcol = bk ? 4 * r : 0;
  const bool hasv = mh < NV;
  const int vcol = hasv ? mh : 0;
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  float4 vacc = make_float4(0.f, 0.f, 0.f, 0.f);
  float2 csum = make_float2(0.f, 0.f);
  for (int seg = 0; seg < 2; ++seg) {
    const int64_t r0 = seg == 0 ? n_beg : max(n_beg, a.split);
    const int64_t r1 = seg == 0 ? min(n_end, a.split) : n_end;
    if (r0 >= r1) continue;
    const float* bbase = seg == 0 ? a.B : a.B1;
    const int64_t ldb = seg == 0 ? a.ldb : a.ldb1;
    const int64_t boff = seg == 0 ? 0 : a.split;
    const int64_t full = (r1 - r0) / kTnxRows;
    // lane's row for (t, j) of a batch starting at row b: b + 16 t + 8 hf + j
    auto load = [&](int64_t b0, TnxBatch& bt, bool tail) {
#pragma unroll
      for (int t = 0; t < kTnxSteps; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          int64_t row = b0 + 16 * t + 8 * hf + j;
          const bool ok = !tail || row < r1;
          row = ok ? row : r0;
          const float2 va = *reinterpret_cast<const float2*>(a.A + row * a.lda + acol);
          const float4 vb = ld4(bbase + (row - boff) * ldb + bcol);
          const float vv = NV > 0 ? a.V[row * a.ldv + vcol] : 0.f;
          if (MASK || tail) {
            bt.av[t][j] = (ok && am) ? va : make_float2(0.f, 0.f);
            bt.bv[t][j] = (ok && bk) ? vb : make_float4(0.f, 0.f, 0.f, 0.f);
            bt.vv[t][j] = ok ? vv : 0.f;
          } else {
            bt.av[t][j] = va;
            bt.bv[t][j] = vb;
            bt.vv[t][j] = vv;
          }
        }
    };
    // fast path: buffer loads from descriptors based at the batch's first row, so a lane's
    // addresses are one 32-bit lane offset plus a scalar row offset (no 64-bit address
    // registers per row)
    const uint32_t lane_a = (uint32_t)((8 * hf * a.lda + acol) * 4);
    const uint32_t lane_b = (uint32_t)((8 * hf * ldb + bcol) * 4);
    const uint32_t lane_v = (uint32_t)((8 * hf * a.ldv + vcol) * 4);
    auto load_fast = [&](int64_t b0, TnxBatch& bt) {
      const auto rA = __builtin_amdgcn_make_buffer_rsrc((void*)(a.A + b0 * a.lda), 0, 0x7fffffff, 0x00020000);
      const auto rB = __builtin_amdgcn_make_buffer_rsrc((void*)(bbase + (b0 - boff) * ldb), 0, 0x7fffffff, 0x00020000);
      const auto rV = __builtin_amdgcn_make_buffer_rsrc((void*)(a.V + b0 * a.ldv), 0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int t = 0; t < kTnxSteps; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int rr = 16 * t + j;
          const auto va = __builtin_amdgcn_raw_buffer_load_b64(rA, lane_a, (int)(rr * a.lda * 4), 0);
          const auto vb = __builtin_amdgcn_raw_buffer_load_b128(rB, lane_b, (int)(rr * ldb * 4), 0);
          bt.av[t][j] = make_float2(__uint_as_float(va[0]), __uint_as_float(va[1]));
          bt.bv[t][j] = make_float4(__uint_as_float(vb[0]), __uint_as_float(vb[1]), __uint_as_float(vb[2]),
                                    __uint_as_float(vb[3]));
          bt.vv[t][j] = NV > 0 ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rV, lane_v, (int)(rr * a.ldv * 4), 0))
                               : 0.f;
        }
    };
    if (!MASK && !RING) {
      for (int64_t bi = 0; bi < full; ++bi) {
        TnxBatch cur;
        load_fast(r0 + bi * kTnxRows, cur);
        tnx_compute<NV != 0>(acc, vacc, csum, cur);
      }
    } else if (MASK) {  // rare shapes (M or K < 128): no batch in flight (the masks cost the registers)
      for (int64_t bi = 0; bi < full; ++bi) {
        TnxBatch cur;
        load(r0 + bi * kTnxRows, cur, false);
        tnx_compute<NV != 0>(acc, vacc, csum, cur);
      }
    } else if (full > 0) {  // ring of three buffers: two batches in flight during the MFMAs
      TnxBatch b0, b1, b2;
      load_fast(r0, b0);
      if (full > 1) load_fast(r0 + kTnxRows, b1);
      int64_t bi = 0;
      while (true) {
        if (bi + 2 < full) load_fast(r0 + (bi + 2) * kTnxRows, b2);
        __builtin_amdgcn_sched_barrier(0);
        tnx_compute<NV != 0>(acc, vacc, csum, b0);
        __builtin_amdgcn_sched_barrier(0);
        if (++bi >= full) break;
        if (bi + 2 < full) load_fast(r0 + (bi + 2) * kTnxRows, b0);
        __builtin_amdgcn_sched_barrier(0);
        tnx_compute<NV != 0>(acc, vacc, csum, b1);
        __builtin_amdgcn_sched_barrier(0);
        if (++bi >= full) break;
        if (bi + 2 < full) load_fast(r0 + (bi + 2) * kTnxRows, b1);
        __builtin_amdgcn_sched_barrier(0);
        tnx_compute<NV != 0>(acc, vacc, csum, b2);
        __builtin_amdgcn_sched_barrier(0);
        if (++bi >= full) break;
      }
    }
    const int64_t t0 = r0 + full * kTnxRows;
    if (t0 < r1) {
      TnxBatch tb;
      load(t0, tb, true);
      tnx_compute<NV != 0>(acc, vacc, csum, tb);
    }
  }
  // ---- workgroup reduction through LDS, pairs in order ----
  auto put = [&](bool add) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = 64 * mh + 2 * acc_row(q, hf) + i;
        float4 v = make_float4(acc[i][0][q], acc[i][1][q], acc[i][2][q], acc[i][3][q]);
        float* dst = &sR[m][4 * r];
        if (add) {
          const float4 o = *reinterpret_cast<const float4*>(dst);
          v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
        }
        st4(dst, v);
      }
  };
  if (pr == 0) put(false);
  __syncthreads();
  if (pr == 1) put(true);
  if (WV == 8) {
    __syncthreads();
    if (pr == 2) put(true);
    __syncthreads();
    if (pr == 3) put(true);
  }
  {
    float t[4] = {vacc.x, vacc.y, vacc.z, vacc.w};
    float c[2] = {csum.x, csum.y};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x0, x1;
      row_swap<32>(t[e], t[e], x0, x1);
      t[e] = x0 + x1;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float x0, x1;
      row_swap<32>(c[e], c[e], x0, x1);
      c[e] = x0 + x1;
    }
    if (hf == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sVr[pr][mh][4 * r + e] = hasv ? t[e] : 0.f;
      sC[pr][mcol] = c[0];
      sC[pr][mcol + 1] = c[1];
    }
  }
  __syncthreads();
  float* P = a.part + (int64_t)blockIdx.x * kPT * kPT;
  for (int idx = tid; idx < kPT * kPT / 4; idx += 64 * WV) {
    const int m = idx >> 5, k4 = (idx & 31) * 4;
    st4(P + m * kPT + k4, *reinterpret_cast<const float4*>(&sR[m][k4]));
  }
  if (tid < 2 * kPT) {
    const int v = tid >> 7, k = tid & 127;
    float sv = sVr[0][v][k] + sVr[1][v][k];
    if (WV == 8) sv = (sv + sVr[2][v][k]) + sVr[3][v][k];
    a.vpart[((int64_t)blockIdx.x * 2 + v) * kPT + k] = sv;
  }
  if (a.cpart && tid < kPT) {
    float sc = sC[0][tid] + sC[1][tid];
    if (WV == 8) sc = (sc + sC[2][tid]) + sC[3][tid];
    a.cpart[(int64_t)blockIdx.x * kPT + tid] = sc;
  }
}

// ---------------------------------------------------------------------------
// The heads = 1 layer backward's two GEMMs in ONE pass over D and x (split bf16, §4.3):
//   dx = D W + ds_src (x) A_src + ds_dst (x) A_dst     (k_projx<1>'s product, A_v = att_v W)
//   G  = D^T x,   GV = S^T x  (S = [ds_src | ds_dst])   (k_tnx's products)
// D [n, 128] is read from HBM once instead of twice (k_projx<1> + k_tnx), x once.
//
// One workgroup per CU, 8 waves, a contiguous row range per workgroup in 32-row steps; step
// st + 1's rows are in flight in registers while step st computes.  The staging threads split
// every D and x element ONCE into its three bf16 terms and store them as row-major images
// [32 rows][128] (256-B rows, 16-B chunk ch of row r at chunk ch ^ sw(r), sw(r) = (r & 3) << 2
// | (r >> 2) & 3), so no wave splits an operand itself:
//  * dx (16x16x32, transposed product as in k_projx): wave w owns output columns 16 w .. +15;
//    its split W' fragments (A operand) live in 48 registers for the whole kernel; the B
//    operand is D[row jl][32 kq + 8 s .. +7], one ds_read_b128 per term -- with the swizzle the
//    kq pairs met by each 16-lane group of a ds_read_b128 sit on complementary bank slots.
//  * G (32x32x16): wave w owns the 32 x 64 block (channels 32 (w & 3), columns 64 (w >> 2));
//    both operands are COLUMNS of the images (rows k = 8 h + j of column r), read with the
//    transposing ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group), conflict-free.
//  * GV: each staging thread accumulates S^T x over its own rows and 4 columns in fp32.
// Partials per workgroup (G [128][128] from the accumulators, GV over the 16 row lanes in
// order) go through the ordered split reduction k_tn_reduce -- deterministic.
// ---------------------------------------------------------------------------
constexpr int kDxwWaves = 8;
constexpr int kDxwRows = 32;                        // rows per step
constexpr int kDxwImg = kDxwRows * kPT * 2;         // bytes per bf16 term image (8 KB)
constexpr int kDxwBuf = 6 * kDxwImg;                // D and x, three terms each (48 KB)
constexpr size_t kDxwLds = 2 * kDxwBuf + (2 * kDxwRows * 2 + 2 * kPT + 2 * kDxwWaves * kDxwRows) * sizeof(float);

struct DxwArg {
  const float* D;   // [n, 128] at ldd
  int64_t ldd;
  const float* S;   // [n, 2] at lds: ds_src, ds_dst
  int64_t lds;
  const float* x0;  // rows [0, split)
  int64_t ldx0;
  const float* x1;  // rows [split, n) (row - split)
  int64_t ldx1;
  int64_t split;
  int64_t n;
  const float* W;   // [128 (channels), 128] at ldw: dx = D W
  int64_t ldw;
  const float* att_src;
  const float* att_dst;
  float* dx;        // nullable: [n, 128] at lddx
  int64_t lddx;
  int64_t rows_per_wg;
  float* part;      // [gridDim.x][128][128]
  float* vpart;     // [gridDim.x][2][128]
  // the producer layer's backward prologue (x = its output, heads = 1), from dx = its grad_out:
  // pnstate[r] = {p_sdst, p_m, p_invl, pgscale <dx_r, x_r - p_bias>}; pbpart = block partial
  // column sums of dx (its dbias).  pnstate NULL: off.
  const float* p_bias;  // nullable
  const float* p_sdst;
  const float* p_m;
  const float* p_invl;
  float pgscale;
  float4* pnstate;
  float* pbpart;        // nullable: [gridDim.x][128]
};

struct DxwRegs {
  float4 d[2];
  float4 x[2];
  float2 s[2];
};

// byte offset of 16-B chunk ch (0..15) of image row r
__device__ __forceinline__ int dxw_off(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

// 4 fp32 -> three bf16x4 terms (split3's arithmetic)
__device__ __forceinline__ void split3_4(const float4& v, uint2& h, uint2& m, uint2& l) {
  const float e[4] = {v.x, v.y, v.z, v.w};
  uint32_t hh[2], mm[2], ll[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    hh[i] = split::pk_bf16(e[2 * i], e[2 * i + 1]);
    const float r0 = e[2 * i] - split::bf_lo(hh[i]), r1 = e[2 * i + 1] - split::bf_hi(hh[i]);
    mm[i] = split::pk_bf16(r0, r1);
    ll[i] = split::pk_bf16(r0 - split::bf_lo(mm[i]), r1 - split::bf_hi(mm[i]));
  }
  h = make_uint2(hh[0], hh[1]);
  m = make_uint2(mm[0], mm[1]);
  l = make_uint2(ll[0], ll[1]);
}

using s16x4 = __attribute__((ext_vector_type(4))) short;
__device__ __forceinline__ uint2 ld_tr16(const unsigned char* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(uint2, v);
}

// PPGAT_DXW_LAB (lab builds only, results WRONG): 1 = no MFMA work (compute skipped), 2 = no
// global loads after the first step (registers reused), 4 = no staging after the first step
#ifndef PPGAT_DXW_LAB
#define PPGAT_DXW_LAB 0
#endif
__global__ void __launch_bounds__(64 * kDxwWaves, 1) k_dxw(DxwArg a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dxw_lds[];
  float* const sS = reinterpret_cast<float*>(dxw_lds + 2 * kDxwBuf);  // [2][32][2]
  float* const sA = sS + 2 * kDxwRows * 2;                            // [2][128]: A_src, A_dst
  float* const sDp = sA + 2 * kPT;  // [2][waves][32]: per-wave partial <dx_r, x_r - p_bias> (producer prologue)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int jl = lane & 15, kq = lane >> 4;  // dx lane roles
  const int r = lane & 31, hf = lane >> 5;   // G lane roles
  const int64_t n = a.n, split = a.split;
  const int64_t rbeg = (int64_t)blockIdx.x * a.rows_per_wg;
  const int64_t rend = min(n, rbeg + a.rows_per_wg);
  const int steps = rend > rbeg ? (int)((rend - rbeg + kDxwRows - 1) / kDxwRows) : 0;
  if (steps == 0) return;  // (no such workgroup: the grid gives every one rows)

  // ---- staging: thread t moves float4 units t and t + 512 of the step's D and x rows (row
  // lr = t / 32 and lr + 16, columns 4 (t % 32) .. +3).  Bases and strides in scalar
  // registers; loads unconditional (rows clamped into the workgroup's range, zeroed when
  // put), so two steps never wait on each other's counts ----
  gfloat* const Dg = sgpr(a.D);
  gfloat* const X0 = sgpr(a.x0);
  gfloat* const X1 = sgpr(a.x1);
  gfloat* const Sg = sgpr(a.S);
  const int64_t ldd = sgpr(a.ldd), ldx0 = sgpr(a.ldx0), ldx1 = sgpr(a.ldx1), lds = sgpr(a.lds);
  const int sc = (tid & 31) * 4, slr = tid >> 5;  // staging column, first staging row
  auto load = [&](int64_t row0, DxwRegs& R) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int64_t row = min(row0 + slr + 16 * p, rend - 1);
      R.d[p] = ld4(Dg + row * ldd + sc);
      gfloat* xs = row < split ? X0 + row * ldx0 : X1 + (row - split) * ldx1;
      R.x[p] = ld4(xs + sc);
      using v2 = __attribute__((ext_vector_type(2))) float;
      const v2 v = *(__attribute__((address_space(1))) const v2*)(Sg + row * lds);
      R.s[p] = make_float2(v.x, v.y);
    }
  };
  float gv[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};  // S^T x over this thread's rows
  auto put = [&](int b, int64_t row0, const DxwRegs& R) {
    unsigned char* img = dxw_lds + b * kDxwBuf;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int lr = slr + 16 * p;
      const bool ok = row0 + lr < rend;
      const float4 d = ok ? R.d[p] : z4, x = ok ? R.x[p] : z4;
      const float2 s = ok ? R.s[p] : make_float2(0.f, 0.f);
      const int off = dxw_off(lr, sc >> 3) + 8 * ((sc >> 2) & 1);
      uint2 h, m, l;
      split3_4(d, h, m, l);
      *reinterpret_cast<uint2*>(img + off) = h;
      *reinterpret_cast<uint2*>(img + kDxwImg + off) = m;
      *reinterpret_cast<uint2*>(img + 2 * kDxwImg + off) = l;
      split3_4(x, h, m, l);
      *reinterpret_cast<uint2*>(img + 3 * kDxwImg + off) = h;
      *reinterpret_cast<uint2*>(img + 4 * kDxwImg + off) = m;
      *reinterpret_cast<uint2*>(img + 5 * kDxwImg + off) = l;
      gv[0][0] = fmaf(s.x, x.x, gv[0][0]); gv[0][1] = fmaf(s.x, x.y, gv[0][1]);
      gv[0][2] = fmaf(s.x, x.z, gv[0][2]); gv[0][3] = fmaf(s.x, x.w, gv[0][3]);
      gv[1][0] = fmaf(s.y, x.x, gv[1][0]); gv[1][1] = fmaf(s.y, x.y, gv[1][1]);
      gv[1][2] = fmaf(s.y, x.z, gv[1][2]); gv[1][3] = fmaf(s.y, x.w, gv[1][3]);
      if (sc == 0) *reinterpret_cast<float2*>(sS + (b * kDxwRows + lr) * 2) = s;
    }
  };

  DxwRegs R0;
  load(rbeg, R0);

  // ---- W' fragments of this wave's 16 output columns, split once (registers): lane (jl, kq),
  // k step s covers channels 32 kq + 8 s .. +7.  The lane's 32 channels also give its part of
  // A_v[col] = sum_k att_v[k] W[k][col], summed over the four kq lanes (fixed order) ----
  const bool want_dx = a.dx != nullptr;
  u32x4 wh[4], wm[4], wl[4];
  {
    const int col = 16 * w + jl;
    float ps = 0.f, pd = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c0 = 32 * kq + 8 * s;
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = a.W[(int64_t)(c0 + j) * a.ldw + col];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ps = fmaf(a.att_src[c0 + j], t[j], ps);
        pd = fmaf(a.att_dst[c0 + j], t[j], pd);
      }
      split3(make_float4(t[0], t[1], t[2], t[3]), make_float4(t[4], t[5], t[6], t[7]), wh[s], wm[s], wl[s]);
    }
    ps += __shfl_xor(ps, 16);
    pd += __shfl_xor(pd, 16);
    ps += __shfl_xor(ps, 32);
    pd += __shfl_xor(pd, 32);
    if (kq == 0) {
      sA[col] = ps;
      sA[kPT + col] = pd;
    }
  }
  put(0, rbeg, R0);
  __syncthreads();

  f32x16 accg[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) accg[i][q] = 0.f;
  const int mb = w & 3, nb0 = 2 * (w >> 2);
  // transposed-read lane address: lane 4 q + p of its 16-lane group g reads row q of the block,
  // columns 4 p .. +3 of the group's 16 (16 (g & 1) within the 32-column operand block)
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;

  // LDS byte offsets of this lane's fragments (loop invariant): dx B operand per (rb, s), and
  // the transposed reads of G per (ks, t) for the A block and per (ks, i, t) for the B blocks
  int odx[8], ota[4], otb[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) odx[g] = dxw_off(16 * (g >> 2) + jl, 4 * kq + (g & 3));
  {
    const int ca = 32 * mb + 16 * (tg & 1) + 4 * tp;
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // u = 2 ks + t
      const int row = 16 * (u >> 1) + 8 * (tg >> 1) + 4 * (u & 1) + tq;
      ota[u] = dxw_off(row, ca >> 3) + 8 * ((ca >> 2) & 1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int cb = 32 * (nb0 + i) + 16 * (tg & 1) + 4 * tp;
        otb[2 * u + i] = 3 * kDxwImg + dxw_off(row, cb >> 3) + 8 * ((cb >> 2) & 1);
      }
    }
  }

  // producer prologue (a.pnstate): this lane's 4 dx columns of p_bias, and its column sums of dx
  const bool pro = want_dx && a.pnstate != nullptr;
  const float4 pbias = (pro && a.p_bias) ? *reinterpret_cast<const float4*>(a.p_bias + 16 * w + 4 * kq)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 pbsum = make_float4(0.f, 0.f, 0.f, 0.f);

  // One step's 12 MFMA groups in a fixed order -- dx (rb, s) for 8 groups, then G (ks, i) --
  // each group's LDS reads issued one group ahead, during the previous group's MFMAs.
  auto compute = [&](const int b, int64_t row0) {
    const unsigned char* img = dxw_lds + b * kDxwBuf;
    auto rd_dx = [&](int g, u32x4 (&f)[3]) {
#pragma unroll
      for (int e = 0; e < 3; ++e) f[e] = *reinterpret_cast<const u32x4*>(img + e * kDxwImg + odx[g]);
    };
    auto rd_tr = [&](const int (&o)[2], u32x4 (&f)[3]) {  // o[t]: rows 4 t + tq of the k step
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          const uint2 v = ld_tr16(img + e * kDxwImg + o[t]);
          f[e][2 * t] = v.x;
          f[e][2 * t + 1] = v.y;
        }
    };
    auto rd_ga = [&](int ks, u32x4 (&f)[3]) {
      const int o[2] = {ota[2 * ks], ota[2 * ks + 1]};
      rd_tr(o, f);
    };
    auto rd_gb = [&](int ks, int i, u32x4 (&f)[3]) {
      const int o[2] = {otb[4 * ks + i], otb[4 * ks + 2 + i]};
      rd_tr(o, f);
    };
    u32x4 fb[2][3], fa[2][3];
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    if (want_dx) {
      rd_dx(0, fb[0]);
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        if (g < 7) {
          rd_dx(g + 1, fb[(g + 1) & 1]);
        } else {
          rd_ga(0, fa[0]);
          rd_gb(0, 0, fb[0]);
        }
        __builtin_amdgcn_sched_barrier(0);
        const int s = g & 3;
        acc = mfma_x6(wh[s], wm[s], wl[s], fb[g & 1][0], fb[g & 1][1], fb[g & 1][2], acc);
        __builtin_amdgcn_sched_barrier(0);
        if (s == 3) {  // epilogue of row block rb = g / 4
          const int lr = 16 * (g >> 2) + jl;
          const int64_t row = row0 + lr;
          const float2 dv = *reinterpret_cast<const float2*>(sS + (b * kDxwRows + lr) * 2);
          const int c0 = 16 * w + 4 * kq;
          const float4 va = *reinterpret_cast<const float4*>(sA + c0);
          const float4 vb = *reinterpret_cast<const float4*>(sA + kPT + c0);
          const float4 o = make_float4(fmaf(dv.y, vb.x, fmaf(dv.x, va.x, acc[0])), fmaf(dv.y, vb.y, fmaf(dv.x, va.y, acc[1])),
                                       fmaf(dv.y, vb.z, fmaf(dv.x, va.z, acc[2])), fmaf(dv.y, vb.w, fmaf(dv.x, va.w, acc[3])));
          if (row < rend) st4(a.dx + row * a.lddx + c0, o);
          if (pro) {
            // x[row][c0 .. +3] = hi + mid + lo of its bf16 images (the three-term split is exact);
            // rows past rend were staged as zeros, so o = 0 there and they add nothing
            const unsigned char* xi = img + 3 * kDxwImg + dxw_off(lr, c0 >> 3) + 8 * ((c0 >> 2) & 1);
            const uint2 th = *reinterpret_cast<const uint2*>(xi);
            const uint2 tm = *reinterpret_cast<const uint2*>(xi + kDxwImg);
            const uint2 tl = *reinterpret_cast<const uint2*>(xi + 2 * kDxwImg);
            const float x0v = (split::bf_lo(th.x) + split::bf_lo(tm.x)) + split::bf_lo(tl.x);
            const float x1v = (split::bf_hi(th.x) + split::bf_hi(tm.x)) + split::bf_hi(tl.x);
            const float x2v = (split::bf_lo(th.y) + split::bf_lo(tm.y)) + split::bf_lo(tl.y);
            const float x3v = (split::bf_hi(th.y) + split::bf_hi(tm.y)) + split::bf_hi(tl.y);
            float d = o.x * (x0v - pbias.x);
            d = fmaf(o.y, x1v - pbias.y, d);
            d = fmaf(o.z, x2v - pbias.z, d);
            d = fmaf(o.w, x3v - pbias.w, d);
            d += __shfl_xor(d, 16);  // (kq 0 + 1) and (2 + 3), then their sum: the same bits in every lane
            d += __shfl_xor(d, 32);
            if (kq == 0) sDp[(b * kDxwWaves + w) * kDxwRows + lr] = d;
            pbsum = make_float4(pbsum.x + o.x, pbsum.y + o.y, pbsum.z + o.z, pbsum.w + o.w);
          }
          acc = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    } else {
      rd_ga(0, fa[0]);
      rd_gb(0, 0, fb[0]);
    }
    // ---- G = D^T x: groups (ks, i) = (0, 0), (0, 1), (1, 0), (1, 1) ----
    rd_gb(0, 1, fb[1]);
    __builtin_amdgcn_sched_barrier(0);
    accg[0] = mfma32_x6(fa[0], fb[0], accg[0]);
    __builtin_amdgcn_sched_barrier(0);
    rd_ga(1, fa[1]);
    rd_gb(1, 0, fb[0]);
    __builtin_amdgcn_sched_barrier(0);
    accg[1] = mfma32_x6(fa[0], fb[1], accg[1]);
    __builtin_amdgcn_sched_barrier(0);
    rd_gb(1, 1, fb[1]);
    __builtin_amdgcn_sched_barrier(0);
    accg[0] = mfma32_x6(fa[1], fb[0], accg[0]);
    __builtin_amdgcn_sched_barrier(0);
    accg[1] = mfma32_x6(fa[1], fb[1], accg[1]);
  };

  // producer prologue of a finished step (after its barrier): the 8 wave partials of each row
  // in wave order, packed with the producer's forward state (buffer b is next written two
  // barriers later)
  // (the producer's forward state of a step's rows is loaded one step ahead, so the wave that
  // packs it never waits on HBM in front of the next barrier)
  float pf_s = 0.f, pf_m = 0.f, pf_l = 0.f;
  auto pro_pref = [&](int64_t row0) {
    const int64_t row = min(row0 + tid, rend - 1);
    pf_s = a.p_sdst[row];
    pf_m = a.p_m[row];
    pf_l = a.p_invl[row];
  };
  if (pro && tid < kDxwRows) pro_pref(rbeg);
  auto pro_fin = [&](const int b, int64_t row0) {
    if (!pro || tid >= kDxwRows) return;
    const int64_t row = row0 + tid;
    if (row < rend) {
      const float* s = sDp + b * kDxwWaves * kDxwRows + tid;
      float d = s[0];
#pragma unroll
      for (int q = 1; q < kDxwWaves; ++q) d += s[q * kDxwRows];
      a.pnstate[row] = make_float4(pf_s, pf_m, pf_l, d * a.pgscale);
    }
    pro_pref(row0 + kDxwRows);
  };

  // one register stage, the loop unrolled by two so each half's LDS buffer is a constant
  for (int st = 0; st < steps; st += 2) {
    if (!(PPGAT_DXW_LAB & 2)) load(rbeg + (int64_t)(st + 1) * kDxwRows, R0);
    if (!(PPGAT_DXW_LAB & 1)) compute(0, rbeg + (int64_t)st * kDxwRows);
    if (st + 1 < steps && !(PPGAT_DXW_LAB & 4)) put(1, rbeg + (int64_t)(st + 1) * kDxwRows, R0);
    __syncthreads();
    pro_fin(0, rbeg + (int64_t)st * kDxwRows);
    if (st + 1 >= steps) break;
    if (!(PPGAT_DXW_LAB & 2)) load(rbeg + (int64_t)(st + 2) * kDxwRows, R0);
    if (!(PPGAT_DXW_LAB & 1)) compute(1, rbeg + (int64_t)(st + 1) * kDxwRows);
    if (st + 2 < steps && !(PPGAT_DXW_LAB & 4)) put(0, rbeg + (int64_t)(st + 2) * kDxwRows, R0);
    __syncthreads();
    pro_fin(1, rbeg + (int64_t)(st + 1) * kDxwRows);
  }
  if (pro && a.pbpart != nullptr) {  // column sums of dx over this workgroup's rows: the 16 row lanes, fixed tree
    float t[4] = {pbsum.x, pbsum.y, pbsum.z, pbsum.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int sh = 1; sh < 16; sh <<= 1) t[e] += __shfl_xor(t[e], sh);
    if (jl == 0) st4(a.pbpart + (int64_t)blockIdx.x * kPT + 16 * w + 4 * kq, make_float4(t[0], t[1], t[2], t[3]));
  }

  // ---- partials: G straight from the accumulators, GV through LDS in row-lane order ----
  float* P = a.part + (int64_t)blockIdx.x * kPT * kPT;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int q = 0; q < 16; ++q) P[(32 * mb + acc_row(q, hf)) * kPT + 32 * (nb0 + i) + r] = accg[i][q];
  float* sG = reinterpret_cast<float*>(dxw_lds);  // [16][2][128] (every wave is past the last barrier)
#pragma unroll
  for (int v = 0; v < 2; ++v)
    st4(sG + (slr * 2 + v) * kPT + sc, make_float4(gv[v][0], gv[v][1], gv[v][2], gv[v][3]));
  __syncthreads();
  if (tid < 2 * kPT) {
    const int v = tid >> 7, c = tid & 127;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += sG[(q * 2 + v) * kPT + c];
    a.vpart[((int64_t)blockIdx.x * 2 + v) * kPT + c] = s;
  }
}

}  // namespace

// ---- host launchers ----
bool proj_shape_ok(int K, int ncols) { return K >= 4 && K <= kPT && K % 4 == 0 && ncols == kPT; }

// k_proj32 (32 x 32 x 2, K in {64, 128}) is built with PPGAT_PROJ_KERNEL=32 only: measured at
// config 2 (profiles/r02/v4_gemm_ab.log) it is slower than k_proj16 -- 105.8 vs 99.4 us (x W^T
// with scores) and 120.5 vs 104.6 us (dx) -- so k_proj16 stays the product kernel
#ifndef PPGAT_PROJ_KERNEL
#define PPGAT_PROJ_KERNEL 16
#endif
static bool proj32_ok(int K, int64_t ld0, int64_t ld1) {
  return PPGAT_PROJ_KERNEL == 32 && (K == 64 || K == 128) && (ld0 % 4) == 0 && (ld1 % 4) == 0;
}

static unsigned proj32_grid(int64_t n) {
  const int64_t tiles = (n + 31) / 32;
  int64_t g = (tiles + 3) / 4;
  if (g > 512) g = 512;  // persistent: two workgroups per CU over the 32-row tiles
  return (unsigned)(g < 1 ? 1 : g);
}

// Which projection kernel runs: the split-bf16 matrix-core kernel k_projx (default) or the
// fp32 MFMA kernel k_proj16 (PPGAT_GEMM=fp32: exact fp32 FMA chains).  Read once per process.
bool gemm_split_enabled() {
  static const bool on = [] {
    const char* e = getenv("PPGAT_GEMM");
    return !(e && strcmp(e, "fp32") == 0);
  }();
  return on;
}

static bool projx_ok(const float* y, int64_t ldy) {
  return gemm_split_enabled() && (ldy % 4) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
}

template <int MODE>
static void launch_projx(const ProjArg& a, hipStream_t st) {
  static const bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_projx<MODE>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kXsLds) == hipSuccess;
  }();
  (void)attr;
  const int64_t tiles = (a.n + 15) / 16;
  int64_t g = (tiles + kXsWaves - 1) / kXsWaves;
  if (g > 256) g = 256;  // one workgroup per CU, persistent over the 16-row tiles
  hipLaunchKernelGGL(k_projx<MODE>, dim3((unsigned)(g < 1 ? 1 : g)), dim3(64 * kXsWaves), kXsLds, st, a);
}

static unsigned proj16_grid(int64_t n) {
  const int64_t tiles = (n + 15) / 16;
  int64_t g = (tiles + 3) / 4;
  if (g > 256 * PPGAT_PROJ16_OCC) g = 256 * PPGAT_PROJ16_OCC;  // persistent over the 16-row tiles
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
  if (projx_ok(y, ldy)) {
    launch_projx<0>(a, st);
  } else if (proj32_ok(K, ldx0, x1 ? ldx1 : ldx0)) {
    if (K == 128) hipLaunchKernelGGL((k_proj32<0, 16>), dim3(proj32_grid(n)), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_proj32<0, 8>), dim3(proj32_grid(n)), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(k_proj16<0>, dim3(proj16_grid(n)), dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t proj_dx(const float* D, int64_t ldd, int64_t n, int K, const float* W, int64_t ldw, const float* att_src,
                   const float* att_dst, const float* S, int64_t lds, float* y, int64_t ldy, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  ProjArg a{};
  a.x0 = D; a.ldx0 = ldd; a.x1 = D; a.ldx1 = ldd; a.split = n; a.n = n; a.K = K; a.W = W; a.ldw = ldw;
  a.att_src = att_src; a.att_dst = att_dst; a.ds = S; a.ldds = lds; a.y = y; a.ldy = ldy;
  if (projx_ok(y, ldy)) {
    launch_projx<1>(a, st);
    return hipGetLastError();
  }
  if (proj32_ok(K, ldd, ldd)) {
    if (K == 128) hipLaunchKernelGGL((k_proj32<1, 16>), dim3(proj32_grid(n)), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_proj32<1, 8>), dim3(proj32_grid(n)), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_proj16<1>, dim3(proj16_grid(n)), dim3(256), 0, st, a);
  return hipGetLastError();
}

bool tn128_shape_ok(int M, int K, int nv, const float* V, int64_t ldv) {
  return M >= 4 && M <= kPT && M % 4 == 0 && K >= 4 && K <= kPT && K % 4 == 0 && nv >= 0 && nv <= 2 &&
         (nv < 2 || ((ldv % 2) == 0 && (reinterpret_cast<uintptr_t>(V) % 8) == 0));
}

static int64_t tn_blocks(int64_t N) {
  int64_t b = 256;                     // one workgroup (4 wave pairs) per CU
  const int64_t min_rows = 16;         // >= 16 rows per pair
  while (b > 1 && b * (kTnWaves / 2) * min_rows > N) b /= 2;
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
  const int64_t pairs = nb * (kTnWaves / 2);
  a.rows_per_pair = ((N + pairs - 1) / pairs + 1) / 2 * 2;
  a.part = reinterpret_cast<float*>(p);
  a.vpart = reinterpret_cast<float*>(p + align_up((size_t)nb * kPT * kPT * 4));
  a.cpart = colsum ? reinterpret_cast<float*>(p + align_up((size_t)nb * kPT * kPT * 4) +
                                              align_up((size_t)nb * 2 * kPT * 4))
                   : nullptr;
  const bool mask = M != kPT || K != kPT;
  const int NVk = nv;
  if (gemm_split_enabled()) {
    // 8 waves (two per SIMD, no batch in flight: the other wave hides the latency) measured
    // 84.5 vs 94-96 us at config 2 against 4 waves with two batches in flight
    // (profiles/r02/v17_tnx_waves.log); the masked shapes keep 4 waves (8 would spill)
    const int wv = mask ? 4 : 8;
    const int64_t pairs_x = nb * (wv / 2);
    a.rows_per_pair = ((N + pairs_x - 1) / pairs_x + kTnxRows - 1) / kTnxRows * kTnxRows;
#define PPGAT_TNX(NV_, MASK_)                                                                        \
  do {                                                                                               \
    if (wv == 8) hipLaunchKernelGGL((k_tnx<NV_, MASK_, 8>), dim3((unsigned)nb), dim3(512), 0, st, a); \
    else hipLaunchKernelGGL((k_tnx<NV_, MASK_, 4>), dim3((unsigned)nb), dim3(256), 0, st, a);         \
  } while (0)
    if (mask) {
      if (NVk == 0) PPGAT_TNX(0, true); else if (NVk == 1) PPGAT_TNX(1, true); else PPGAT_TNX(2, true);
    } else {
      if (NVk == 0) PPGAT_TNX(0, false); else if (NVk == 1) PPGAT_TNX(1, false); else PPGAT_TNX(2, false);
    }
#undef PPGAT_TNX
  } else {
#define PPGAT_TN(NV_, MASK_) \
  hipLaunchKernelGGL((k_tn128<NV_, MASK_>), dim3((unsigned)nb), dim3(64 * kTnWaves), 0, st, a)
  if (mask) {
    if (NVk == 0) PPGAT_TN(0, true); else if (NVk == 1) PPGAT_TN(1, true); else PPGAT_TN(2, true);
  } else {
    if (NVk == 0) PPGAT_TN(0, false); else if (NVk == 1) PPGAT_TN(1, false); else PPGAT_TN(2, false);
  }
#undef PPGAT_TN
  }
  TnReduceArg ra{};
  ra.part = a.part; ra.vpart = a.vpart; ra.cpart = a.cpart; ra.splits = nb; ra.M = M; ra.K = K; ra.nv = nv;
  ra.out = out; ra.vout = vout; ra.colsum = colsum;
  const int64_t elems = kPT * kPT + 2 * kPT + (colsum ? kPT : 0);
  hipLaunchKernelGGL(k_tn_reduce, dim3((unsigned)((elems + 63) / 64)), dim3(1024), 0, st, ra);
  return hipGetLastError();
}

// ---- fused dx + G + GV (k_dxw) ----
static int64_t dxw_blocks(int64_t n) {
  int64_t nb = (n + kDxwRows - 1) / kDxwRows;
  if (nb > 256) nb = 256;  // one workgroup per CU
  return nb < 1 ? 1 : nb;
}
static int64_t dxw_rows_per_wg(int64_t n) {
  const int64_t nb = dxw_blocks(n);
  return (n + nb - 1) / nb;
}

bool dxw_ok(int hc, int k) { return gemm_split_enabled() && hc == kPT && k == kPT; }

size_t dxw_workspace_bytes(int64_t n) {
  const int64_t nb = dxw_blocks(n);
  return align_up((size_t)nb * kPT * kPT * 4) + align_up((size_t)nb * 2 * kPT * 4) + align_up((size_t)nb * kPT * 4);
}

hipError_t dxw(const float* D, int64_t ldd, const float* S, int64_t lds, const float* x0, int64_t ldx0, const float* x1,
               int64_t ldx1, int64_t split, int64_t n, const float* W, int64_t ldw, const float* att_src,
               const float* att_dst, float* dx, int64_t lddx, float* G, float* GV, void* ws, hipStream_t st,
               const DxwProducer* prod) {
  if (n <= 0) {
    hipError_t e = hipMemsetAsync(G, 0, (size_t)kPT * kPT * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(GV, 0, (size_t)2 * kPT * 4, st);
    if (e == hipSuccess && prod && prod->grad_bias) e = hipMemsetAsync(prod->grad_bias, 0, (size_t)kPT * 4, st);
    return e;
  }
  static const bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dxw), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)kDxwLds) == hipSuccess;
  }();
  (void)attr;
  const int64_t rpw = dxw_rows_per_wg(n);
  const int64_t nb = (n + rpw - 1) / rpw;  // every workgroup gets rows
  char* p = static_cast<char*>(ws);
  DxwArg a{};
  a.D = D; a.ldd = ldd; a.S = S; a.lds = lds;
  a.x0 = x0; a.ldx0 = ldx0; a.x1 = x1 ? x1 : x0; a.ldx1 = x1 ? ldx1 : ldx0; a.split = x1 ? split : n; a.n = n;
  a.W = W; a.ldw = ldw; a.att_src = att_src; a.att_dst = att_dst; a.dx = dx; a.lddx = lddx;
  a.rows_per_wg = rpw;
  a.part = reinterpret_cast<float*>(p);
  a.vpart = reinterpret_cast<float*>(p + align_up((size_t)dxw_blocks(n) * kPT * kPT * 4));
  if (prod != nullptr && dx != nullptr) {
    a.p_bias = prod->bias; a.p_sdst = prod->s_dst; a.p_m = prod->m; a.p_invl = prod->inv_l;
    a.pgscale = prod->gscale;
    a.pnstate = reinterpret_cast<float4*>(prod->nstate);
    a.pbpart = prod->grad_bias ? reinterpret_cast<float*>(p + align_up((size_t)dxw_blocks(n) * kPT * kPT * 4) +
                                                          align_up((size_t)dxw_blocks(n) * 2 * kPT * 4))
                               : nullptr;
  }
  hipLaunchKernelGGL(k_dxw, dim3((unsigned)nb), dim3(64 * kDxwWaves), kDxwLds, st, a);
  TnReduceArg ra{};
  // (the producer's dbias partials ride along as the reduction's column-sum rows)
  ra.part = a.part; ra.vpart = a.vpart; ra.cpart = a.pbpart; ra.splits = nb; ra.M = kPT; ra.K = kPT; ra.nv = 2;
  ra.out = G; ra.vout = GV; ra.colsum = a.pbpart ? prod->grad_bias : nullptr;
  const int64_t elems = kPT * kPT + 2 * kPT + (a.pbpart ? kPT : 0);
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
                     float eps, float wd, const float* const* tstep, double lr, hipStream_t st) {
  AdamArg a{};
  a.count = count;
  a.lr = lr; a.b1d = beta1; a.b2d = beta2;
  a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.omb1 = (float)(1.0 - beta1); a.omb2 = (float)(1.0 - beta2);
  a.eps = eps; a.wd = wd;
  int64_t blocks = 0;
  for (int t = 0; t < count; ++t) {
    a.p[t] = p[t]; a.g[t] = g[t]; a.m[t] = m[t]; a.v[t] = v[t]; a.n[t] = n[t];
    a.tstep[t] = tstep ? tstep[t] : nullptr;
    a.step_size[t] = step_size ? step_size[t] : 0.f; a.bc2_sqrt[t] = bc2_sqrt ? bc2_sqrt[t] : 1.f;
    blocks += (n[t] + kAdamPerBlock - 1) / kAdamPerBlock;
    a.blk_end[t] = blocks;
  }
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace ppgat

#if PPGAT_CLOCK_PROBE
// median over waves of (shader cycles / real time) in MHz for slot 0 (k_proj16) / 1 (k_tn128)
extern "C" int ppgat_debug_clock_mhz(int slot, int waves, double* mhz) {
  static unsigned long long h[2][4096][2];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(ppgat::g_probe), sizeof(h)) != hipSuccess) return 3;
  double v[4096];
  int n = 0;
  for (int w = 0; w < waves && w < 4096; ++w)
    if (h[slot][w][1] > 0) v[n++] = (double)h[slot][w][0] / (double)h[slot][w][1] * 100.0;
  if (n == 0) return 1;
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && v[j - 1] > v[j]; --j) { const double t = v[j]; v[j] = v[j - 1]; v[j - 1] = t; }
  *mhz = v[n / 2];
  return 0;
}
#endif
