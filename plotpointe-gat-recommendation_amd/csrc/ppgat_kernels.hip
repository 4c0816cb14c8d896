// ppgat_kernels.hip -- fused GAT message-passing kernels for CDNA4 (gfx950, MI355X).
//
// Hot path of BASELINE.json north_star: one GAT layer = per-node attention terms,
// per-edge LeakyReLU logit, per-destination segmented softmax, alpha-weighted
// neighbour aggregation (forward), and its atomic-free backward.
//
// Reference semantics restated (oracle/gat_oracle.py):
//   PyG GATConv (scripts/train_gat_pyg.py:77, concat=False, add_self_loops=False)
//   SimpleGATLayer.forward (scripts/train_gat_custom.py:75-93)
//
// Layout in HBM (all fp32 row-major, int32 indices):
//   h      [N, H, C]  projected node rows (one 512 B row per node at H=1, C=128)
//   s_src, s_dst, m, inv_l, D, ds_src  [N, H]
//   CSR by dst: rowptr[N+1], col[E] (src), csr_eid[E]
//   CSC by src: colptr[N+1], row[E] (dst), csc_eid[E], csc2csr[E]
//   dz     [E, H]  per-edge logit gradient, stored in CSR slot order
//
// Work decomposition: one 64-lane wavefront per node row.  A row of C floats is
// C/4 lanes x float4 (a "subgroup"); 64/(C/4) subgroups take different edges of
// the same row, each keeping U gathers in flight, so a wave has 8 neighbour rows
// (4 KB at C=128) outstanding.  Softmax state is wave-uniform (online max/sum over
// 64-edge chunks); subgroup partial aggregates merge with xor-shuffles at the end.
// No float atomics anywhere: every sum is owned by one wave in a fixed order, so
// results are bitwise reproducible run to run.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "ppgat_internal.h"
#include "ppgat_lanes.h"

#ifndef PPGAT_PRO_UP
#define PPGAT_PRO_UP 4
#endif
#ifndef PPGAT_SHORT_U
#define PPGAT_SHORT_U 4  // neighbour rows in flight per short item (per 16-lane row)
#endif

namespace ppgat {

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
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}
__device__ __forceinline__ float4 shfl_xor4(float4 v, int m) {
  return make_float4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m), __shfl_xor(v.w, m));
}
// attention logit e(z) and de/dz, per mode (torch leaky_relu / clamp backward rules:
// slope where z <= 0; clamp passes gradient where min <= e <= max).
__device__ __forceinline__ float logit(float z, float slope, int mode) {
  float e = z > 0.f ? z : z * slope;
  if (mode == kModeCustom) e = fminf(fmaxf(e, -10.f), 10.f);
  return e;
}
__device__ __forceinline__ float dlogit(float z, float slope, int mode) {
  const float e = z > 0.f ? z : z * slope;
  float d = z > 0.f ? 1.f : slope;
  if (mode == kModeCustom && (e < -10.f || e > 10.f)) d = 0.f;
  return d;
}

// Dropout epoch: a device-side counter folded into every dropout seed, so a step captured
// once in a hipGraph draws fresh masks on each replay (ppgat_dropout_advance enqueues the
// increment on the stream; 0 -- the default -- leaves the seeds as passed).  The effective
// seed is seed + epoch * kDropEpochMul (mod 2^64), restated in oracle/gat_oracle.py.
__device__ uint64_t g_drop_epoch = 0;
constexpr uint64_t kDropEpochMul = 0xD1B54A32D192ED03ull;
__device__ __forceinline__ uint64_t epoch_seed(uint64_t seed) {
  return seed + *(volatile const uint64_t*)&g_drop_epoch * kDropEpochMul;
}

// The seed the forward's masks use, stored for the backward (ppgat_fwd seed_used): the
// backward then reads it instead of the epoch counter, so an epoch advance enqueued between
// a forward and its backward (another captured step replayed in between, a recompute) does
// not change the backward's mask.
__global__ void k_seed_snap(uint64_t seed, uint64_t* __restrict__ out) {
  if (threadIdx.x == 0) out[0] = epoch_seed(seed);
}

// Counter-based dropout mask on alpha (restated in oracle/gat_oracle.py:dropout_scale).
__device__ __forceinline__ float drop_scale(uint64_t seed, uint32_t eid, uint32_t head, float p,
                                            float inv_keep) {
  uint64_t x = seed ^ ((uint64_t)eid * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)head * 0xC2B2AE3D27D4EB4Full);
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  const float u = (float)(x >> 40) * (1.0f / 16777216.0f);
  return u >= p ? inv_keep : 0.f;
}

// Streamed (once-touched) rows of the edge kernels -- the forward's output rows, pass B's own
// source rows h_j and dh_j -- with the non-temporal hint when PPGAT_NT_STREAM=1, so they do
// not push the gathered table (h forward, grad_out in pass B) out of the Infinity Cache.
#ifndef PPGAT_NT_STREAM
#define PPGAT_NT_STREAM 1
#endif
__device__ __forceinline__ float4 ld4s(const float* p) {
#if PPGAT_NT_STREAM
  using v4 = __attribute__((ext_vector_type(4))) float;
  const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
#else
  return *reinterpret_cast<const float4*>(p);
#endif
}
__device__ __forceinline__ void st4s(float* p, float4 a) {
#if PPGAT_NT_STREAM
  using v4 = __attribute__((ext_vector_type(4))) float;
  __builtin_nontemporal_store(v4{a.x, a.y, a.z, a.w}, reinterpret_cast<v4*>(p));
#else
  *reinterpret_cast<float4*>(p) = a;
#endif
}

template <int C>
struct Geo {
  static constexpr int LPR = C / 4;              // lanes per row (float4 each)
  static constexpr int EPW = 64 / LPR;           // edges handled side by side per wave
  static constexpr int U = EPW >= 8 ? 1 : 8 / EPW;  // unroll: 8 gathers in flight per wave
  static_assert(C % 4 == 0 && LPR <= 64 && 64 % LPR == 0, "C must be 4*2^k <= 256");
  static_assert(64 % (EPW * U) == 0, "chunk tiling");
};

// ---------------------------------------------------------------------------
// s_src[n,h] = <h[n,h,:], att_src[h,:]>, s_dst likewise.  One subgroup per (n,h).
// ---------------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(256) k_scores(const float* __restrict__ h, const float* __restrict__ att_src,
                                                const float* __restrict__ att_dst, int64_t pairs, int heads,
                                                float* __restrict__ s_src, float* __restrict__ s_dst) {
  using G = Geo<C>;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pr = t / G::LPR;
  const int sl = (int)(t % G::LPR);
  const bool valid = pr < pairs;
  const int hd = valid ? (int)(pr % heads) : 0;
  const float4 v = valid ? ld4(h + pr * C + sl * 4) : f4(0.f);
  float x = dot4(v, ld4(att_src + hd * C + sl * 4));
  float y = dot4(v, ld4(att_dst + hd * C + sl * 4));
  x = group_reduce<Op::Sum, 1, G::LPR / 2>(x);
  y = group_reduce<Op::Sum, 1, G::LPR / 2>(y);
  if (valid && sl == 0) {
    s_src[pr] = x;
    s_dst[pr] = y;
  }
}

// ---------------------------------------------------------------------------
// Work items.  Rows (dst rows for the forward, src rows for backward pass B) are
// cut into items of at most T edges by ppgat_schedule_build: hub rows (deg > T) become
// ceil(deg/T) pieces that write partial state to a scratch slab and are merged in
// piece order by a second small kernel (deterministic); all other rows are one item.
// Items are ordered hub pieces first, then rows by descending degree, so the longest
// work starts first and the tail is short (largest in-degree on config 2: 5,180).
// ---------------------------------------------------------------------------
struct Items {
  const int32_t* row;
  const int32_t* beg;
  const int32_t* end;
  int64_t n_items;
  int64_t n_hub_items;  // items [0, n_hub_items) are hub pieces, slot = item index
};

// ---------------------------------------------------------------------------
// Fused forward: one wave per item (destination row or hub piece), CSR by dst.
//   e_k = logit(s_src[j] + s_dst[i]);  online softmax over 64-edge chunks;
//   acc = sum_k exp(e_k - m) * d_k * h[j]  (d_k = dropout multiplier)
// partial slab (hub pieces) per (item, head): [acc C | m | l | pad pad]
// ---------------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(256) k_fwd(Items it, const int32_t* __restrict__ col,
                                             const int32_t* __restrict__ eid, int heads,
                                             const float* __restrict__ h, const float* __restrict__ s_src,
                                             const float* __restrict__ s_dst, const float* __restrict__ bias,
                                             int mode, float slope, float eps, float p, float inv_keep,
                                             uint64_t seed, float* __restrict__ out, float* __restrict__ m_out,
                                             float* __restrict__ invl_out, float* __restrict__ agg_out,
                                             float* __restrict__ partial, uint64_t* __restrict__ seed_out) {
  if (p > 0.f) seed = epoch_seed(seed);
  if (seed_out != nullptr && blockIdx.x == 0 && threadIdx.x == 0) seed_out[0] = seed;  // the backward's mask seed
  using G = Geo<C>;
  __shared__ int2 rec[4][64];  // per wave: chunk edges {src row, weight}
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w >= it.n_items) return;  // wave-uniform
  const int sg = lane / G::LPR, sl = lane % G::LPR;
  const int64_t i = it.row[w];
  const int rs = it.beg[w], re = it.end[w];
  const bool hub = w < it.n_hub_items;
  const bool pyg = mode == kModePyg;
  float4 osum = f4(0.f);
  for (int hd = 0; hd < heads; ++hd) {
    const float sd = s_dst[i * heads + hd];
    float m = pyg ? -INFINITY : 0.f, l = 0.f;
    float4 acc = f4(0.f);
    for (int base = rs; base < re; base += 64) {
      const int k = base + lane;
      const bool valid = k < re;
      const int j = valid ? col[k] : 0;
      float e = -INFINITY;
      if (valid) e = logit(s_src[(int64_t)j * heads + hd] + sd, slope, mode);
      float pe;
      if (pyg) {
        const float mn = fmaxf(m, wave_max(e));
        const float sc = expf(m - mn);
        pe = valid ? expf(e - mn) : 0.f;
        l = fmaf(l, sc, wave_sum(pe));
        acc = mul4(acc, sc);
        m = mn;
      } else {
        pe = valid ? expf(e) : 0.f;
        l += wave_sum(pe);
      }
      float pw = pe;
      if (p > 0.f && valid) pw *= drop_scale(seed, (uint32_t)eid[k], (uint32_t)hd, p, inv_keep);
      rec[wv][lane] = make_int2(j, __float_as_int(pw));
      wave_sync();
      const int n = min(64, re - base);
      for (int q0 = 0; q0 < n; q0 += G::EPW * G::U) {
        float4 v[G::U];
        float pq[G::U];
#pragma unroll
        for (int u = 0; u < G::U; ++u) {
          const int q = q0 + u * G::EPW + sg;
          const int2 r = rec[wv][q];
          pq[u] = __int_as_float(r.y);
          v[u] = q < n ? ld4(h + ((int64_t)r.x * heads + hd) * C + sl * 4) : f4(0.f);
        }
#pragma unroll
        for (int u = 0; u < G::U; ++u) acc = fma4(pq[u], v[u], acc);
      }
      wave_sync();
    }
    acc = across_subgroups<G::LPR>(acc);
    if (hub) {
      float* slot = partial + (w * heads + hd) * (C + 4);
      if (sg == 0) st4(slot + sl * 4, acc);
      if (lane == 0) st4(slot + C, make_float4(m, l, 0.f, 0.f));
      continue;
    }
    const float invl = 1.f / (l + eps);
    const float4 a = mul4(acc, invl);
    if (agg_out != nullptr && sg == 0) st4(agg_out + (i * heads + hd) * C + sl * 4, a);
    osum = add4(osum, a);
    if (lane == 0) {
      m_out[i * heads + hd] = (pyg && re > rs) ? m : 0.f;
      invl_out[i * heads + hd] = invl;
    }
  }
  if (hub) return;
  if (heads > 1) osum = mul4(osum, 1.f / (float)heads);
  if (bias != nullptr) osum = add4(osum, ld4(bias + sl * 4));
  if (sg == 0) st4s(out + i * C + sl * 4, osum);
}

// ---------------------------------------------------------------------------
// Short items (<= kShortItemEdges edges, heads = 1): four items per wave, one per 16-lane
// row of the wave.  With one item per wave a short row leaves the wave waiting on a chain
// of dependent loads (item -> edge -> node terms -> neighbour rows) for a handful of
// edges; four per wave put four times the neighbour rows in flight (4 rows x 4 items per
// wave).  Lane ql of a 16-lane row takes the edge rs + ql for the softmax terms (16-lane
// DPP reductions) and the float4 columns ql, ql + 16, ... of every neighbour row.
// ---------------------------------------------------------------------------
constexpr int kSU = PPGAT_SHORT_U;
static_assert(kSU == 4 || kSU == 8 || kSU == 16, "short-item unroll");

template <int C>
__device__ __forceinline__ void fwd_merge_wave(int64_t hb, const int32_t* __restrict__ hub_row,
                                               const int32_t* __restrict__ hub_ptr, int heads,
                                               const float* __restrict__ partial, const float* __restrict__ bias,
                                               int mode, float eps, float* __restrict__ out, float* __restrict__ m_out,
                                               float* __restrict__ invl_out, float* __restrict__ agg_out);

// hub merges riding at the head of a short-item launch (the hub pieces come from the long-item
// kernel launched before it): blocks [0, mblocks) merge hubs 4 per block, one per wave
struct HubMerge {
  const int32_t* hub_row;
  const int32_t* hub_ptr;
  int64_t n_hubs;
  int heads;
  const float* partial;
  int64_t mblocks;
};

template <int C>
__global__ void __launch_bounds__(256) k_fwd_short(Items it, int64_t first, const int32_t* __restrict__ col,
                                                   const int32_t* __restrict__ eid, const float* __restrict__ h,
                                                   const float* __restrict__ s_src, const float* __restrict__ s_dst,
                                                   const float* __restrict__ bias, int mode, float slope, float eps,
                                                   float p, float inv_keep, uint64_t seed, float* __restrict__ out,
                                                   float* __restrict__ m_out, float* __restrict__ invl_out,
                                                   float* __restrict__ agg_out, uint64_t* __restrict__ seed_out,
                                                   HubMerge mg) {
  if (p > 0.f) seed = epoch_seed(seed);
  if (seed_out != nullptr && blockIdx.x == 0 && threadIdx.x == 0) seed_out[0] = seed;  // the backward's mask seed
  constexpr int NV = C / 64;  // float4 columns per lane
  static_assert(NV >= 1, "k_fwd_short: C >= 64");
  __shared__ int2 rec[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if ((int64_t)blockIdx.x < mg.mblocks) {
    const int64_t hb = (int64_t)blockIdx.x * 4 + wv;
    if (hb < mg.n_hubs)
      fwd_merge_wave<C>(hb, mg.hub_row, mg.hub_ptr, mg.heads, mg.partial, bias, mode, eps, out, m_out, invl_out,
                        agg_out);
    return;
  }
  const int qr = lane >> 4, ql = lane & 15;
  const int64_t item = first + (((int64_t)blockIdx.x - mg.mblocks) * 4 + wv) * 4 + qr;
  const bool live = item < it.n_items;
  const int64_t ic = live ? item : first;
  const int64_t i = it.row[ic];
  const int rs = it.beg[ic], re = live ? it.end[ic] : rs;
  const bool pyg = mode == kModePyg;
  const int k = rs + ql;
  const bool valid = k < re;
  const int j = valid ? col[k] : 0;
  const float e = valid ? logit(s_src[j] + s_dst[i], slope, mode) : -INFINITY;
  float m = 0.f, pe;
  if (pyg) {
    m = group_reduce<Op::Max, 1, 8>(e);
    pe = valid ? expf(e - m) : 0.f;
  } else {
    pe = valid ? expf(e) : 0.f;
  }
  const float l = group_reduce<Op::Sum, 1, 8>(pe);
  float pw = pe;
  if (p > 0.f && valid) pw *= drop_scale(seed, (uint32_t)eid[k], 0u, p, inv_keep);
  rec[wv][lane] = make_int2(j, __float_as_int(pw));
  wave_sync();
  const int2* rq = &rec[wv][qr * 16];
  const int n = re - rs;
  float4 acc[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) acc[c] = f4(0.f);
  for (int t0 = 0; t0 < n; t0 += kSU) {
    float4 v[kSU][NV];
    float wt[kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      const int t = t0 + u;
      const int2 r = rq[t & 15];
      wt[u] = t < n ? __int_as_float(r.y) : 0.f;
#pragma unroll
      for (int c = 0; c < NV; ++c) v[u][c] = t < n ? ld4(h + (int64_t)r.x * C + (ql + 16 * c) * 4) : f4(0.f);
    }
#pragma unroll
    for (int u = 0; u < kSU; ++u)
#pragma unroll
      for (int c = 0; c < NV; ++c) acc[c] = fma4(wt[u], v[u][c], acc[c]);
  }
  if (!live) return;
  const float invl = 1.f / (l + eps);
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col4 = (ql + 16 * c) * 4;
    const float4 a = mul4(acc[c], invl);
    if (agg_out != nullptr) st4(agg_out + i * C + col4, a);
    st4s(out + i * C + col4, bias != nullptr ? add4(a, ld4(bias + col4)) : a);
  }
  if (ql == 0) {
    m_out[i] = (pyg && re > rs) ? m : 0.f;
    invl_out[i] = invl;
  }
}

// Merge the pieces of each hub row.  One wave per hub row: the piece maxima and
// rescaled sums are lane-parallel (wave reductions), the C-wide partial rows are taken
// by the subgroups in turn (piece q -> subgroup q mod EPW, two loads in flight each) and
// combined across subgroups -- a fixed order, so the merge is deterministic.  One wave's
// share, called by k_fwd_merge or by the merge blocks at the head of k_fwd_short.
template <int C>
__device__ __forceinline__ void fwd_merge_wave(int64_t hb, const int32_t* __restrict__ hub_row,
                                               const int32_t* __restrict__ hub_ptr, int heads,
                                               const float* __restrict__ partial, const float* __restrict__ bias,
                                               int mode, float eps, float* __restrict__ out, float* __restrict__ m_out,
                                               float* __restrict__ invl_out, float* __restrict__ agg_out) {
  using G = Geo<C>;
  const int lane = threadIdx.x & 63;
  const int sg = lane / G::LPR, sl = lane % G::LPR;
  const int64_t i = hub_row[hb];
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  float4 osum = f4(0.f);
  for (int hd = 0; hd < heads; ++hd) {
    float M = 0.f;
    if (mode == kModePyg) {
      M = -INFINITY;
      for (int q = p0 + lane; q - lane < p1; q += 64)
        M = fmaxf(M, q < p1 ? partial[((int64_t)q * heads + hd) * (C + 4) + C] : -INFINITY);
      M = wave_max(M);
    }
    float l = 0.f;
    for (int q = p0 + lane; q - lane < p1; q += 64) {
      float t = 0.f;
      if (q < p1) {
        const float* slot = partial + ((int64_t)q * heads + hd) * (C + 4);
        t = slot[C + 1] * expf(slot[C] - M);
      }
      l += wave_sum(t);
    }
    float4 acc = f4(0.f), acc2 = f4(0.f);
    int q = p0 + sg;
    for (; q + G::EPW < p1; q += 2 * G::EPW) {
      const float* s0 = partial + ((int64_t)q * heads + hd) * (C + 4);
      const float* s1 = partial + ((int64_t)(q + G::EPW) * heads + hd) * (C + 4);
      const float4 v0 = ld4(s0 + sl * 4), v1 = ld4(s1 + sl * 4);
      acc = fma4(expf(s0[C] - M), v0, acc);
      acc2 = fma4(expf(s1[C] - M), v1, acc2);
    }
    if (q < p1) {
      const float* s0 = partial + ((int64_t)q * heads + hd) * (C + 4);
      acc = fma4(expf(s0[C] - M), ld4(s0 + sl * 4), acc);
    }
    acc = across_subgroups<G::LPR>(add4(acc, acc2));
    const float invl = 1.f / (l + eps);
    const float4 a = mul4(acc, invl);
    if (agg_out != nullptr && sg == 0) st4(agg_out + (i * heads + hd) * C + sl * 4, a);
    osum = add4(osum, a);
    if (lane == 0) {
      m_out[i * heads + hd] = M;
      invl_out[i * heads + hd] = invl;
    }
  }
  if (out == nullptr) return;  // aggregate-then-transform: the per-head aggregates only
  if (heads > 1) osum = mul4(osum, 1.f / (float)heads);
  if (bias != nullptr) osum = add4(osum, ld4(bias + sl * 4));
  if (sg == 0) st4s(out + i * C + sl * 4, osum);
}

template <int C>
__global__ void __launch_bounds__(256) k_fwd_merge(const int32_t* __restrict__ hub_row,
                                                   const int32_t* __restrict__ hub_ptr, int64_t n_hubs, int heads,
                                                   const float* __restrict__ partial,
                                                   const float* __restrict__ bias, int mode, float eps,
                                                   float* __restrict__ out, float* __restrict__ m_out,
                                                   float* __restrict__ invl_out, float* __restrict__ agg_out) {
  const int64_t hb = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (hb >= n_hubs) return;
  fwd_merge_wave<C>(hb, hub_row, hub_ptr, heads, partial, bias, mode, eps, out, m_out, invl_out, agg_out);
}

// ---------------------------------------------------------------------------
// Backward prologue, one subgroup per (n, h), grid-stride over a fixed grid:
//   D[n,h] = <g_n, agg[n,h]>, g = gscale * grad_out   (= sum_k alpha_k dalpha_k, Appendix B)
// and the per-node state pass B gathers once per edge, packed as one float4:
//   nstate[n,h] = {s_dst, m, inv_l, D}
// When bias_part != NULL also the block partial column sums of grad_out (dbias), in a
// fixed order (subgroups in order within a block, blocks reduced by k_col_reduce).
// ---------------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(256) k_bwd_pro(const float* __restrict__ grad_out, const float* __restrict__ out,
                                                 const float* __restrict__ agg, const float* __restrict__ bias,
                                                 const float* __restrict__ s_dst, const float* __restrict__ m_in,
                                                 const float* __restrict__ invl_in, int64_t pairs, int heads,
                                                 float gscale, float4* __restrict__ nstate,
                                                 float* __restrict__ bias_part) {
  using G = Geo<C>;
  constexpr int SPB = 256 / G::LPR;
  constexpr int UP = PPGAT_PRO_UP;  // pairs per subgroup per iteration (2 UP row loads in flight)
  __shared__ float4 red[SPB][G::LPR];
  const int sg = threadIdx.x / G::LPR, sl = threadIdx.x % G::LPR;
  float4 bsum = f4(0.f);
  for (int64_t pr0 = (int64_t)blockIdx.x * SPB * UP; pr0 < pairs; pr0 += (int64_t)gridDim.x * SPB * UP) {
    float4 g[UP], a[UP];
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const int64_t pr = pr0 + u * SPB + sg;
      g[u] = a[u] = f4(0.f);
      if (pr < pairs) {
        const int64_t n = pr / heads;
        g[u] = ld4(grad_out + n * C + sl * 4);
        a[u] = agg != nullptr ? ld4s(agg + pr * C + sl * 4) : ld4s(out + n * C + sl * 4);  // read once here
      }
    }
#pragma unroll
    for (int u = 0; u < UP; ++u) {
      const int64_t pr = pr0 + u * SPB + sg;
      const bool valid = pr < pairs;
      if (valid && pr % heads == 0) bsum = add4(bsum, g[u]);
      float4 av = a[u];
      if (agg == nullptr && bias != nullptr) {
        const float4 b = ld4(bias + sl * 4);
        av = make_float4(av.x - b.x, av.y - b.y, av.z - b.z, av.w - b.w);
      }
      float x = group_reduce<Op::Sum, 1, G::LPR / 2>(dot4(g[u], av));
      if (valid && sl == 0) nstate[pr] = make_float4(s_dst[pr], m_in[pr], invl_in[pr], x * gscale);
    }
  }
  if (bias_part == nullptr) return;
  red[sg][sl] = bsum;
  __syncthreads();
  for (int t = threadIdx.x; t < G::LPR; t += blockDim.x) {
    float4 s = red[0][t];
    for (int q = 1; q < SPB; ++q) s = add4(s, red[q][t]);
    st4(bias_part + ((int64_t)blockIdx.x * G::LPR + t) * 4, s);
  }
}

// ---------------------------------------------------------------------------
// Backward pass B: one wave per item (SOURCE row j or hub piece), CSC by src.
//   dh_j     = sum_k beta_k g_{i_k}                              (message term)
//   dz_k     = alpha_k (d_k gscale <dOut_i, h_j> - D_i) e'(z_k)  (logit gradient)
//   ds_src_j = sum_k dz_k ;  dz_k stored at its CSR slot for the dst-side sum.
// alpha is recomputed from the saved (m, inv_l): nothing [E]-sized was saved.
// hub-piece partial slab per (item, head): [dh C | ds | pad pad pad]
// ---------------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(256) k_bwd_src(Items it, const int32_t* __restrict__ row,
                                                 const int32_t* __restrict__ csc_eid,
                                                 const int32_t* __restrict__ csc2csr, int heads,
                                                 const float* __restrict__ h, const float* __restrict__ s_src,
                                                 const float4* __restrict__ nstate,
                                                 const float* __restrict__ grad_out, int mode, float slope,
                                                 float gscale, float p, float inv_keep, uint64_t seed,
    const uint64_t* __restrict__ seed_in,
                                                 float* __restrict__ dh, int64_t ld_dh, float* __restrict__ ds_src,
                                                 int64_t ld_ds, float* __restrict__ dz, float* __restrict__ partial) {
  if (p > 0.f) seed = seed_in != nullptr ? *seed_in : epoch_seed(seed);
  using G = Geo<C>;
  constexpr int GRP = G::LPR / G::U;  // lanes sharing one reduced edge value
  // per wave, per chunk edge: {dst row, beta * gscale} and {c1, c0, CSR slot}, where
  // dz = c1 <g_i, h_j> - c0  (c1 = alpha e' d gscale, c0 = alpha e' D_i)
  __shared__ int2 recA[4][64];
  __shared__ float4 recB[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w >= it.n_items) return;
  const int sg = lane / G::LPR, sl = lane % G::LPR;
  const int myu = sl / GRP;
  const bool writer = (sl % GRP) == 0;
  const int64_t j = it.row[w];
  const int cs = it.beg[w], ce = it.end[w];
  const bool hub = w < it.n_hub_items;
  for (int hd = 0; hd < heads; ++hd) {
    const float ss = s_src[j * heads + hd];
    const float4 hv = ld4s(h + (j * heads + hd) * C + sl * 4);
    float4 acc = f4(0.f);
    float ds = 0.f;
    for (int base = cs; base < ce; base += 64) {
      const int k = base + lane;
      const bool valid = k < ce;
      const int i = valid ? row[k] : 0;
      float bg = 0.f, c1 = 0.f, c0 = 0.f;
      int slot = 0;
      if (valid) {
        const float4 st = nstate[(int64_t)i * heads + hd];  // {s_dst, m, inv_l, D}
        const float z = ss + st.x;
        const float e = logit(z, slope, mode);
        const float af = expf(e - st.y) * st.z;
        const float dm = p > 0.f ? drop_scale(seed, (uint32_t)csc_eid[k], (uint32_t)hd, p, inv_keep) : 1.f;
        slot = csc2csr != nullptr ? csc2csr[k] : k;  // NULL: dz in CSC order
        bg = af * dm * gscale;
        const float a1 = af * dlogit(z, slope, mode);
        c1 = a1 * dm * gscale;
        c0 = a1 * st.w;
      }
      recA[wv][lane] = make_int2(i, __float_as_int(bg));
      recB[wv][lane] = make_float4(c1, c0, __int_as_float(slot), 0.f);
      wave_sync();
      const int n = min(64, ce - base);
      for (int q0 = 0; q0 < n; q0 += G::EPW * G::U) {
        float4 g[G::U];
        float bq[G::U], part[G::U];
#pragma unroll
        for (int u = 0; u < G::U; ++u) {
          const int q = q0 + u * G::EPW + sg;
          const int2 r = recA[wv][q];
          bq[u] = __int_as_float(r.y);
          g[u] = q < n ? ld4(grad_out + (int64_t)r.x * C + sl * 4) : f4(0.f);
        }
#pragma unroll
        for (int u = 0; u < G::U; ++u) {
          acc = fma4(bq[u], g[u], acc);
          part[u] = dot4(g[u], hv);
        }
        const float dot = transpose_reduce<G::LPR, G::U>(part, sl);
        const int q = q0 + myu * G::EPW + sg;
        if (writer && q < n) {
          const float4 rb = recB[wv][q];
          const float dzv = fmaf(rb.x, dot, -rb.y);
          ds += dzv;
          dz[(int64_t)__float_as_int(rb.z) * heads + hd] = dzv;
        }
      }
      wave_sync();
    }
    acc = across_subgroups<G::LPR>(acc);
    ds = wave_sum(ds);
    if (hub) {
      float* s = partial + (w * heads + hd) * (C + 4);
      if (sg == 0) st4(s + sl * 4, acc);
      if (lane == 0) s[C] = ds;
      continue;
    }
    if (sg == 0) st4s(dh + j * ld_dh + hd * C + sl * 4, acc);
    if (lane == 0) ds_src[j * ld_ds + hd] = ds;
  }
}

// Pass B for short items (<= kShortItemEdges edges, heads = 1): four source rows per wave,
// one per 16-lane row, as k_fwd_short.  Lane ql builds the record of edge rs + ql and, after
// the 16-lane reduction of <g_i, h_j> for its edge, writes that edge's dz.
template <int C>
__device__ __forceinline__ void bwd_merge_wave(int64_t hb, const int32_t* __restrict__ hub_row,
                                               const int32_t* __restrict__ hub_ptr, int heads,
                                               const float* __restrict__ partial, float* __restrict__ dh,
                                               int64_t ld_dh, float* __restrict__ ds_src, int64_t ld_ds);

template <int C>
__global__ void __launch_bounds__(256) k_bwd_src_short(Items it, int64_t first, const int32_t* __restrict__ row,
                                                       const int32_t* __restrict__ csc_eid,
                                                       const int32_t* __restrict__ csc2csr,
                                                       const float* __restrict__ h, const float* __restrict__ s_src,
                                                       const float4* __restrict__ nstate,
                                                       const float* __restrict__ grad_out, int mode, float slope,
                                                       float gscale, float p, float inv_keep, uint64_t seed,
    const uint64_t* __restrict__ seed_in,
                                                       float* __restrict__ dh, int64_t ld_dh,
                                                       float* __restrict__ ds_src, int64_t ld_ds,
                                                       float* __restrict__ dz, HubMerge mg) {
  if (p > 0.f) seed = seed_in != nullptr ? *seed_in : epoch_seed(seed);
  constexpr int NV = C / 64;
  static_assert(NV >= 1, "k_bwd_src_short: C >= 64");
  __shared__ int2 rec[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if ((int64_t)blockIdx.x < mg.mblocks) {  // hub merges first (the long-item kernel ran before)
    const int64_t hb = (int64_t)blockIdx.x * 4 + wv;
    if (hb < mg.n_hubs) bwd_merge_wave<C>(hb, mg.hub_row, mg.hub_ptr, mg.heads, mg.partial, dh, ld_dh, ds_src, ld_ds);
    return;
  }
  const int qr = lane >> 4, ql = lane & 15;
  const int64_t item = first + (((int64_t)blockIdx.x - mg.mblocks) * 4 + wv) * 4 + qr;
  const bool live = item < it.n_items;
  const int64_t ic = live ? item : first;
  const int64_t j = it.row[ic];
  const int rs = it.beg[ic], re = live ? it.end[ic] : rs;
  const float ss = s_src[j];
  float4 hv[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) hv[c] = ld4s(h + j * C + (ql + 16 * c) * 4);
  const int k = rs + ql;
  const bool valid = k < re;
  const int i = valid ? row[k] : 0;
  float bg = 0.f, c1 = 0.f, c0 = 0.f;
  int slot = 0;
  if (valid) {
    const float4 st = nstate[i];  // {s_dst, m, inv_l, D}
    const float z = ss + st.x;
    const float af = expf(logit(z, slope, mode) - st.y) * st.z;
    const float dm = p > 0.f ? drop_scale(seed, (uint32_t)csc_eid[k], 0u, p, inv_keep) : 1.f;
    slot = csc2csr != nullptr ? csc2csr[k] : k;  // NULL: dz in CSC order
    bg = af * dm * gscale;
    const float a1 = af * dlogit(z, slope, mode);
    c1 = a1 * dm * gscale;
    c0 = a1 * st.w;
  }
  rec[wv][lane] = make_int2(i, __float_as_int(bg));
  wave_sync();
  const int2* rq = &rec[wv][qr * 16];
  const int n = re - rs;
  float4 acc[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) acc[c] = f4(0.f);
  float ds = 0.f;
  for (int t0 = 0; t0 < n; t0 += kSU) {
    float4 g[kSU][NV];
    float bq[kSU], part[kSU];
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      const int t = t0 + u;
      const int2 r = rq[t & 15];
      bq[u] = t < n ? __int_as_float(r.y) : 0.f;
#pragma unroll
      for (int c = 0; c < NV; ++c)
        g[u][c] = t < n ? ld4(grad_out + (int64_t)r.x * C + (ql + 16 * c) * 4) : f4(0.f);
    }
#pragma unroll
    for (int u = 0; u < kSU; ++u) {
      part[u] = 0.f;
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        acc[c] = fma4(bq[u], g[u][c], acc[c]);
        part[u] += dot4(g[u][c], hv[c]);
      }
    }
#pragma unroll
    for (int u = 0; u < kSU; ++u) part[u] = group_reduce<Op::Sum, 1, 8>(part[u]);
    const int my = ql - t0;
    if (valid && my >= 0 && my < kSU) {
      float dot = part[0];
#pragma unroll
      for (int u = 1; u < kSU; ++u) dot = my == u ? part[u] : dot;
      const float dzv = fmaf(c1, dot, -c0);
      ds += dzv;
      dz[slot] = dzv;
    }
  }
  ds = group_reduce<Op::Sum, 1, 8>(ds);
  if (!live) return;
#pragma unroll
  for (int c = 0; c < NV; ++c) st4s(dh + j * ld_dh + (ql + 16 * c) * 4, acc[c]);
  if (ql == 0) ds_src[j * ld_ds] = ds;
}

// ---------------------------------------------------------------------------
// Pass B for heads > 1: the same decomposition as k_bwd_src, but every head of an edge is
// handled in one pass, so each grad_out row g_i (C floats, shared by the heads: the output
// is the head mean) is gathered ONCE per edge instead of once per edge and head.  Per
// chunk of 64 edges a lane builds the records of one edge for all heads; per group of
// U x EPW edges the lane reduces U x H partial dots <g_i, h_j^hd> over its subgroup with a
// transposing butterfly (mh_reduce).  Requires C >= 32.
// ---------------------------------------------------------------------------
// V per-lane values, each summed over the LPR lanes of a subgroup.  Transposing steps at
// offsets LPR/2 .. 8 (while more than one value is left), then a DPP reduction over the
// 8-lane octet for the R values left.  Returns R; v[t] (t < R) holds the sum of value
// index base + t, base = sum over steps of (lane bit set ? half the values then : 0).
template <int OFF, int N>
__device__ __forceinline__ int mh_transpose(float (&v)[16], int sl, int& base) {
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
    return mh_transpose<OFF / 2, Hh>(v, sl, base);
  } else {
#pragma unroll
    for (int t = 0; t < N; ++t) v[t] = group_reduce<Op::Sum, 1, 4>(v[t]);
    return N;
  }
}

template <int C, int H>
__global__ void __launch_bounds__(256) k_bwd_src_mh(Items it, const int32_t* __restrict__ row,
                                                    const int32_t* __restrict__ csc_eid,
                                                    const int32_t* __restrict__ csc2csr,
                                                    const float* __restrict__ h, const float* __restrict__ s_src,
                                                    const float4* __restrict__ nstate,
                                                    const float* __restrict__ grad_out, int mode, float slope,
                                                    float gscale, float p, float inv_keep, uint64_t seed,
    const uint64_t* __restrict__ seed_in,
                                                    float* __restrict__ dh, int64_t ld_dh, float* __restrict__ ds_src,
                                                    int64_t ld_ds, float* __restrict__ dz, float* __restrict__ partial) {
  if (p > 0.f) seed = seed_in != nullptr ? *seed_in : epoch_seed(seed);
  using G = Geo<C>;
  static_assert(C >= 32, "k_bwd_src_mh: C >= 32");
  constexpr int U = G::U * H > 16 ? (16 / H > 0 ? 16 / H : 1) : G::U;  // <= 16 partial dots per lane
  constexpr int V = U * H;
  static_assert(V <= 16, "values per lane");
  static_assert(64 % (G::EPW * U) == 0, "chunk tiling");
  __shared__ int2 recA[4][64];       // {dst row, CSR slot}
  __shared__ float4 recH[4][H][64];  // per head {beta * gscale, c1, c0, -}
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  if (w >= it.n_items) return;
  const int sg = lane / G::LPR, sl = lane % G::LPR;
  const int64_t j = it.row[w];
  const int cs = it.beg[w], ce = it.end[w];
  const bool hub = w < it.n_hub_items;
  float ss[H];
  float4 hv[H], acc[H];
  float dsa[H];
#pragma unroll
  for (int hd = 0; hd < H; ++hd) {
    ss[hd] = s_src[j * H + hd];
    hv[hd] = ld4(h + (j * H + hd) * C + sl * 4);
    acc[hd] = f4(0.f);
    dsa[hd] = 0.f;
  }
  for (int base = cs; base < ce; base += 64) {
    const int k = base + lane;
    const bool valid = k < ce;
    const int i = valid ? row[k] : 0;
    const int slot = valid ? (csc2csr != nullptr ? csc2csr[k] : k) : 0;  // NULL: dz in CSC order
    const uint32_t eid = (valid && p > 0.f) ? (uint32_t)csc_eid[k] : 0u;
#pragma unroll
    for (int hd = 0; hd < H; ++hd) {
      float bg = 0.f, c1 = 0.f, c0 = 0.f;
      if (valid) {
        const float4 st = nstate[(int64_t)i * H + hd];  // {s_dst, m, inv_l, D}
        const float z = ss[hd] + st.x;
        const float e = logit(z, slope, mode);
        const float af = expf(e - st.y) * st.z;
        const float dm = p > 0.f ? drop_scale(seed, eid, (uint32_t)hd, p, inv_keep) : 1.f;
        bg = af * dm * gscale;
        const float a1 = af * dlogit(z, slope, mode);
        c1 = a1 * dm * gscale;
        c0 = a1 * st.w;
      }
      recH[wv][hd][lane] = make_float4(bg, c1, c0, 0.f);
    }
    recA[wv][lane] = make_int2(i, slot);
    wave_sync();
    const int n = min(64, ce - base);
    for (int q0 = 0; q0 < n; q0 += G::EPW * U) {
      float4 g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u * G::EPW + sg;
        g[u] = q < n ? ld4(grad_out + (int64_t)recA[wv][q].x * C + sl * 4) : f4(0.f);
      }
      float part[16];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u * G::EPW + sg;
#pragma unroll
        for (int hd = 0; hd < H; ++hd) {
          acc[hd] = fma4(recH[wv][hd][q].x, g[u], acc[hd]);
          part[u * H + hd] = dot4(g[u], hv[hd]);
        }
      }
#pragma unroll
      for (int t = V; t < 16; ++t) part[t] = 0.f;
      int vbase = 0;
      const int R = mh_transpose<G::LPR / 2, V>(part, sl, vbase);
      const int t = sl & 7;
      if (t < R) {
        float dot = part[0];
#pragma unroll
        for (int x = 1; x < 8; ++x)
          if (x == t) dot = part[x];
        const int vi = vbase + t;
        const int u = vi / H, hd = vi % H;
        const int q = q0 + u * G::EPW + sg;
        if (q < n) {
          const float4 rb = recH[wv][hd][q];
          const float dzv = fmaf(rb.y, dot, -rb.z);
#pragma unroll
          for (int x = 0; x < H; ++x)
            if (x == hd) dsa[x] += dzv;
          dz[(int64_t)recA[wv][q].y * H + hd] = dzv;
        }
      }
    }
    wave_sync();
  }
#pragma unroll
  for (int hd = 0; hd < H; ++hd) {
    const float4 a = across_subgroups<G::LPR>(acc[hd]);
    const float ds = wave_sum(dsa[hd]);
    if (hub) {
      float* sp = partial + (w * H + hd) * (C + 4);
      if (sg == 0) st4(sp + sl * 4, a);
      if (lane == 0) sp[C] = ds;
    } else {
      if (sg == 0) st4(dh + j * ld_dh + hd * C + sl * 4, a);
      if (lane == 0) ds_src[j * ld_ds + hd] = ds;
    }
  }
}

template <int C>
__device__ __forceinline__ void bwd_merge_wave(int64_t hb, const int32_t* __restrict__ hub_row,
                                               const int32_t* __restrict__ hub_ptr, int heads,
                                               const float* __restrict__ partial, float* __restrict__ dh,
                                               int64_t ld_dh, float* __restrict__ ds_src, int64_t ld_ds) {
  using G = Geo<C>;
  const int lane = threadIdx.x & 63;
  const int sg = lane / G::LPR, sl = lane % G::LPR;
  const int64_t j = hub_row[hb];
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  for (int hd = 0; hd < heads; ++hd) {
    float ds = 0.f;
    for (int q = p0 + lane; q - lane < p1; q += 64)
      ds += wave_sum(q < p1 ? partial[((int64_t)q * heads + hd) * (C + 4) + C] : 0.f);
    float4 acc = f4(0.f), acc2 = f4(0.f);
    int q = p0 + sg;
    for (; q + G::EPW < p1; q += 2 * G::EPW) {
      acc = add4(acc, ld4(partial + ((int64_t)q * heads + hd) * (C + 4) + sl * 4));
      acc2 = add4(acc2, ld4(partial + ((int64_t)(q + G::EPW) * heads + hd) * (C + 4) + sl * 4));
    }
    if (q < p1) acc = add4(acc, ld4(partial + ((int64_t)q * heads + hd) * (C + 4) + sl * 4));
    acc = across_subgroups<G::LPR>(add4(acc, acc2));
    if (sg == 0) st4s(dh + j * ld_dh + hd * C + sl * 4, acc);
    if (lane == 0) ds_src[j * ld_ds + hd] = ds;
  }
}

template <int C>
__global__ void __launch_bounds__(256) k_bwd_merge(const int32_t* __restrict__ hub_row,
                                                   const int32_t* __restrict__ hub_ptr, int64_t n_hubs, int heads,
                                                   const float* __restrict__ partial, float* __restrict__ dh,
                                                   int64_t ld_dh, float* __restrict__ ds_src, int64_t ld_ds) {
  const int64_t hb = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (hb >= n_hubs) return;
  bwd_merge_wave<C>(hb, hub_row, hub_ptr, heads, partial, dh, ld_dh, ds_src, ld_ds);
}

// ---------------------------------------------------------------------------
// Backward node epilogue (grid-stride over nodes, fixed partition => deterministic):
//   ds_dst_i = sum_{k in CSR(i)} dz_k            (ordered segment sum)
//   dh_i    += ds_src_i att_src + ds_dst_i att_dst
//   block partial datt_src += ds_src_i h_i, datt_dst += ds_dst_i h_i
// block partial layout [blocks, 2, H, C]; heads <= kMaxHeads.
// ---------------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(256) k_bwd_epi(const int32_t* __restrict__ rowptr, int64_t n_nodes, int heads,
                                                 const float* __restrict__ h, const float* __restrict__ att_src,
                                                 const float* __restrict__ att_dst,
                                                 const float* __restrict__ ds_src, const float* __restrict__ dz,
                                                 float* __restrict__ dh, float* __restrict__ partial) {
  using G = Geo<C>;
  __shared__ float4 red[4][2 * kMaxHeads * (C / 4)];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int sg = lane / G::LPR, sl = lane % G::LPR;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
  const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  float4 pa_s[kMaxHeads], pa_d[kMaxHeads];
#pragma unroll
  for (int hd = 0; hd < kMaxHeads; ++hd) { pa_s[hd] = f4(0.f); pa_d[hd] = f4(0.f); }
  for (int64_t base = wave * G::EPW; base < n_nodes; base += n_waves * G::EPW) {
    const int64_t i = base + sg;
    const bool valid = i < n_nodes;
    int rs = 0, re = 0;
    if (valid) { rs = rowptr[i]; re = rowptr[i + 1]; }
#pragma unroll
    for (int hd = 0; hd < kMaxHeads; ++hd) {
      if (hd >= heads) break;
      float x = 0.f;
      for (int k = rs + sl; k < re; k += G::LPR) x += dz[(int64_t)k * heads + hd];
#pragma unroll
      for (int off = G::LPR / 2; off > 0; off >>= 1) x += __shfl_xor(x, off);
      if (valid) {
        const int64_t pr = i * heads + hd;
        const float dsd = x, dss = ds_src[pr];
        const float4 hv = ld4(h + pr * C + sl * 4);
        float4 d = ld4(dh + pr * C + sl * 4);
        d = fma4(dss, ld4(att_src + hd * C + sl * 4), d);
        d = fma4(dsd, ld4(att_dst + hd * C + sl * 4), d);
        st4(dh + pr * C + sl * 4, d);
        pa_s[hd] = fma4(dss, hv, pa_s[hd]);
        pa_d[hd] = fma4(dsd, hv, pa_d[hd]);
      }
    }
  }
  // wave combine (subgroups), then block combine in wave order via LDS
#pragma unroll
  for (int hd = 0; hd < kMaxHeads; ++hd) {
    if (hd >= heads) break;
    float4 a = pa_s[hd], b = pa_d[hd];
#pragma unroll
    for (int off = G::LPR; off < 64; off <<= 1) {
      a = add4(a, shfl_xor4(a, off));
      b = add4(b, shfl_xor4(b, off));
    }
    if (sg == 0) {
      red[wv][(0 * heads + hd) * (C / 4) + sl] = a;
      red[wv][(1 * heads + hd) * (C / 4) + sl] = b;
    }
  }
  __syncthreads();
  const int nv = 2 * heads * (C / 4);
  for (int t = threadIdx.x; t < nv; t += blockDim.x) {
    float4 s = red[0][t];
    s = add4(s, red[1][t]);
    s = add4(s, red[2][t]);
    s = add4(s, red[3][t]);
    st4(partial + ((int64_t)blockIdx.x * nv + t) * 4, s);
  }
}

// Ordered column reduction of block partials [rows, cols] -> out_a[0:split], out_b[0:cols-split].
// One 1024-thread block per 64 columns: wave w sums rows w, w+16, ... in that order (16 loads
// in flight: the few hundred partial rows of a launch are one or two HBM round trips, not a
// chain of them); then the 16 wave sums are added in wave order.
__global__ void __launch_bounds__(1024) k_col_reduce(const float* __restrict__ partial, int64_t rows, int cols,
                                                     int split, float* __restrict__ out_a,
                                                     float* __restrict__ out_b) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < cols) {
    int64_t r = wv;
    for (; r + 15 * 16 < rows; r += 16 * 16) {
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = partial[(r + 16 * k) * cols + c];
#pragma unroll
      for (int k = 0; k < 16; ++k) s += v[k];
    }
    for (; r < rows; r += 16) s += partial[r * cols + c];
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && c < cols) {
    float t = 0.f;
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    if (c < split) out_a[c] = t;
    else out_b[c - split] = t;
  }
}

// ---------------------------------------------------------------------------
// ds_dst[i, h] = sum_{k in CSR(i)} dz[k, h] over the forward (destination) schedule:
// 16 lanes per (item, head), items hold <= max_edges edges, so no group waits on a hub;
// hub pieces leave a partial that k_dst_merge adds up in piece order (deterministic).
// Written with row stride ld.
// ---------------------------------------------------------------------------
// The dz gathers of the destination sums.  AUX != 0 (lab builds only, PPGAT_DST_AUX): the same
// gather as a buffer load carrying that cache policy (sc0 = 1, nt = 2, sc1 = 16), to measure
// whether the L2 then fetches less than a whole 128-B line per 4- / 16-B gather.
template <int AUX>
__device__ __forceinline__ float dz_ld(const float* dz, int64_t i) {
  if constexpr (AUX == 0) {
    return dz[i];
  } else {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)dz, (short)0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4), 0, AUX));
  }
}

template <int AUX, class V>
__device__ __forceinline__ V dz_ldv(const V* dzv, int64_t i) {
  if constexpr (AUX == 0 || sizeof(V) != 16) {
    return dzv[i];
  } else {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)dzv, (short)0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, AUX));
  }
}

template <bool PERM, int AUX = 0>
__global__ void __launch_bounds__(256) k_dst_sum(Items it, int heads, const float* __restrict__ dz,
                                                 const int32_t* __restrict__ csr2csc,
                                                 float* __restrict__ ds_dst, int64_t ld,
                                                 float* __restrict__ partial) {
  // PERM: dz is in CSC (source) order, as pass B wrote it contiguously; CSR slot k reads
  // dz[csr2csc[k]] (same summation order as the CSR-order layout: bitwise equal results)
  auto at = [&](int k) -> int64_t { return PERM ? (int64_t)csr2csc[k] : (int64_t)k; };
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pr = t >> 4;
  const int l = (int)(t & 15);
  const bool live = pr < it.n_items * heads;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f;
  int64_t w = 0;
  int hd = 0;
  if (live) {
    w = pr / heads;
    hd = (int)(pr % heads);
    const int rs = it.beg[w], re = it.end[w];
    int k = rs + l;
    for (; k + 48 < re; k += 64) {
      x0 += dz_ld<AUX>(dz, at(k) * heads + hd);
      x1 += dz_ld<AUX>(dz, at(k + 16) * heads + hd);
      x2 += dz_ld<AUX>(dz, at(k + 32) * heads + hd);
      x3 += dz_ld<AUX>(dz, at(k + 48) * heads + hd);
    }
    for (; k < re; k += 16) x0 += dz_ld<AUX>(dz, at(k) * heads + hd);
  }
  float x = (x0 + x1) + (x2 + x3);
  x = group_reduce<Op::Sum, 1, 8>(x);  // the 16 lanes of a DPP row
  if (live && l == 0) {
    if (w < it.n_hub_items) partial[w * heads + hd] = x;
    else ds_dst[(int64_t)it.row[w] * ld + hd] = x;
  }
}

// heads in {2, 4}: one 16-lane group per item for all heads, each edge's H logit gradients
// loaded as one vector (dz rows of H floats), the same per-head summation order as k_dst_sum
template <bool PERM, int H, int AUX = 0>
__global__ void __launch_bounds__(256) k_dst_sum_vh(Items it, const float* __restrict__ dz,
                                                    const int32_t* __restrict__ csr2csc, float* __restrict__ ds_dst,
                                                    int64_t ld, float* __restrict__ partial) {
  using V = __attribute__((ext_vector_type(H))) float;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t w = t >> 4;
  const int l = (int)(t & 15);
  const bool live = w < it.n_items;
  auto at = [&](int k) -> int64_t { return PERM ? (int64_t)csr2csc[k] : (int64_t)k; };
  const V* dzv = reinterpret_cast<const V*>(dz);
  V x0 = {}, x1 = {}, x2 = {}, x3 = {};
  if (live) {
    const int rs = it.beg[w], re = it.end[w];
    int k = rs + l;
    for (; k + 48 < re; k += 64) {
      x0 += dz_ldv<AUX>(dzv, at(k));
      x1 += dz_ldv<AUX>(dzv, at(k + 16));
      x2 += dz_ldv<AUX>(dzv, at(k + 32));
      x3 += dz_ldv<AUX>(dzv, at(k + 48));
    }
    for (; k < re; k += 16) x0 += dz_ldv<AUX>(dzv, at(k));
  }
  const V xs = (x0 + x1) + (x2 + x3);
#pragma unroll
  for (int hd = 0; hd < H; ++hd) {
    const float x = group_reduce<Op::Sum, 1, 8>(xs[hd]);
    if (live && l == 0) {
      if (w < it.n_hub_items) partial[w * H + hd] = x;
      else ds_dst[(int64_t)it.row[w] * ld + hd] = x;
    }
  }
}

// The short items (<= 16 edges: the schedule's [n_long_items, n_items), by descending degree)
// of k_dst_sum_vh<true, H>, one thread per item: every index and dz load of the item in flight
// at once, then the 16-lane group's butterfly (xor 1, 2, 4, 8 on slots l = edge k - beg) restated
// as the same balanced tree over the thread's 16 slots, empty slots +0 -- the same bits as
// k_dst_sum_vh (each slot 0 + dz, as the group's x0, so no slot is -0 and the empty ones add
// exactly nothing).  The halo partition's partial sums run over ~11M table rows of ~2 edges each
// at world 8 on config 5, where 16 lanes per item left 14 of them idle behind three dependent loads.
template <int H, int AUX = 0>
__global__ void __launch_bounds__(256) k_dst_sum_vh_short(Items it, int64_t w0, const float* __restrict__ dz,
                                                          const int32_t* __restrict__ csr2csc,
                                                          float* __restrict__ ds_dst, int64_t ld) {
  using V = __attribute__((ext_vector_type(H))) float;
  const int64_t w = w0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= it.n_items) return;
  const int rs = it.beg[w], n = it.end[w] - rs;
  const V* dzv = reinterpret_cast<const V*>(dz);
  int k[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) k[l] = l < n ? csr2csc[rs + l] : 0;
  V v[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) v[l] = l < n ? V{} + dz_ldv<AUX>(dzv, k[l]) : V{};
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int l = 0; l < 16; l += 2 * o) v[l] = v[l] + v[l + o];
  float* out = ds_dst + (int64_t)it.row[w] * ld;
#pragma unroll
  for (int hd = 0; hd < H; ++hd) out[hd] = v[0][hd];
}

// One wave per hub: lane l sums pieces l, l + 64, ... (piece order), per head, then the 64
// lanes in a fixed butterfly -- deterministic.  (One thread per (hub, head) walking every piece
// in turn took 134 us per call at the config-5 share, whose top item is 490 pieces.)
__global__ void __launch_bounds__(256) k_dst_merge(const int32_t* __restrict__ hub_row,
                                                   const int32_t* __restrict__ hub_ptr, int64_t n_hubs, int heads,
                                                   const float* __restrict__ partial, float* __restrict__ ds_dst,
                                                   int64_t ld) {
  const int lane = threadIdx.x & 63;
  const int64_t hb = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (hb >= n_hubs) return;  // (wave-uniform)
  const int p0 = hub_ptr[hb], p1 = hub_ptr[hb + 1];
  for (int hd = 0; hd < heads; ++hd) {
    float x = 0.f;
    for (int q = p0 + lane; q < p1; q += 64) x += partial[(int64_t)q * heads + hd];
    x = group_reduce<Op::Sum, 1, 32>(x);
    if (lane == 0) ds_dst[(int64_t)hub_row[hb] * ld + hd] = x;
  }
}

// ---------------------------------------------------------------------------
// host-side launchers (called from ppgat_abi.cpp)
// ---------------------------------------------------------------------------
#define PPGAT_DISPATCH_C(C_, ...)                      \
  switch (C_) {                                        \
    case 4: { constexpr int CC = 4; __VA_ARGS__; break; }     \
    case 8: { constexpr int CC = 8; __VA_ARGS__; break; }     \
    case 16: { constexpr int CC = 16; __VA_ARGS__; break; }   \
    case 32: { constexpr int CC = 32; __VA_ARGS__; break; }   \
    case 64: { constexpr int CC = 64; __VA_ARGS__; break; }   \
    case 128: { constexpr int CC = 128; __VA_ARGS__; break; } \
    case 256: { constexpr int CC = 256; __VA_ARGS__; break; } \
    default: return hipErrorInvalidValue;              \
  }

static inline unsigned blocks_for(int64_t threads) { return (unsigned)((threads + 255) / 256); }

hipError_t launch_scores(const float* h, const float* as, const float* ad, int64_t n, int heads, int C, float* ss,
                         float* sd, hipStream_t st) {
  const int64_t pairs = n * heads;
  if (pairs == 0) return hipSuccess;
  PPGAT_DISPATCH_C(C, hipLaunchKernelGGL(k_scores<CC>, dim3(blocks_for(pairs * (CC / 4))), dim3(256), 0, st, h, as,
                                         ad, pairs, heads, ss, sd));
  return hipGetLastError();
}

// First item of the four-per-wave short path, or n_items when every item takes the
// one-per-wave kernel (heads > 1, C < 64, or a schedule without n_long_items).
static int64_t short_begin(const ItemsArg& it, int heads, int C) {
  if (heads != 1 || (C != 64 && C != 128 && C != 256)) return it.n_items;
  if (it.n_long_items < it.n_hub_items || it.n_long_items > it.n_items) return it.n_items;
  return it.n_long_items;
}

#define PPGAT_DISPATCH_C64(C, ...)                             \
  do {                                                         \
    if ((C) == 64) { constexpr int CC = 64; __VA_ARGS__; }     \
    else if ((C) == 128) { constexpr int CC = 128; __VA_ARGS__; } \
    else { constexpr int CC = 256; __VA_ARGS__; }              \
  } while (0)

hipError_t launch_fwd(const ItemsArg& it, const int32_t* col, const int32_t* eid, int heads, int C,
                      const float* h, const float* ss, const float* sd, const float* bias, int mode, float slope,
                      float eps, float p, uint64_t seed, uint64_t* seed_out, float* out, float* m, float* invl,
                      float* agg, float* partial, const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs,
                      hipStream_t st) {
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  // the effective mask seed is written by block 0 of the first edge kernel launched (no
  // separate launch); a graph without items snapshots it with k_seed_snap
  const int64_t n_long = short_begin(it, heads, C);
  const Items its{it.row, it.beg, it.end, n_long, it.n_hub_items};
  if (seed_out != nullptr && it.n_items == 0) hipLaunchKernelGGL(k_seed_snap, dim3(1), dim3(64), 0, st, seed, seed_out);
  if (n_long > 0) {
    PPGAT_DISPATCH_C(C, hipLaunchKernelGGL(k_fwd<CC>, dim3(blocks_for(n_long * 64)), dim3(256), 0, st, its, col,
                                           eid, heads, h, ss, sd, bias, mode, slope, eps, p, inv_keep, seed, out, m,
                                           invl, agg, partial, seed_out));
  }
  // the hub merges ride at the head of the short-item launch when there is one (one launch fewer)
  const bool fold = n_long < it.n_items;
  if (fold) {
    const Items all{it.row, it.beg, it.end, it.n_items, it.n_hub_items};
    const HubMerge mg{hub_row, hub_ptr, n_hubs, heads, partial, n_hubs > 0 ? (n_hubs + 3) / 4 : 0};
    const unsigned g = (unsigned)((it.n_items - n_long + 15) / 16 + mg.mblocks);  // 4 waves x 4 items per block
    PPGAT_DISPATCH_C64(C, hipLaunchKernelGGL(k_fwd_short<CC>, dim3(g), dim3(256), 0, st, all, n_long, col, eid, h,
                                             ss, sd, bias, mode, slope, eps, p, inv_keep, seed, out, m, invl, agg,
                                             n_long > 0 ? nullptr : seed_out, mg));
  }
  if (n_hubs > 0 && !fold) {
    PPGAT_DISPATCH_C(C, hipLaunchKernelGGL(k_fwd_merge<CC>, dim3(blocks_for(n_hubs * 64)), dim3(256), 0, st,
                                           hub_row, hub_ptr, n_hubs, heads, partial, bias, mode, eps, out, m, invl,
                                           agg));
  }
  return hipGetLastError();
}

hipError_t launch_bwd_pro(const float* go, const float* out, const float* agg, const float* bias, const float* sd,
                          const float* m, const float* invl, int64_t n, int heads, int C, float gscale,
                          float* nstate, float* bias_part, int64_t blocks, hipStream_t st) {
  const int64_t pairs = n * heads;
  PPGAT_DISPATCH_C(C, hipLaunchKernelGGL(k_bwd_pro<CC>, dim3((unsigned)blocks), dim3(256), 0, st, go, out, agg, bias,
                                         sd, m, invl, pairs, heads, gscale, reinterpret_cast<float4*>(nstate),
                                         bias_part));
  return hipGetLastError();
}

hipError_t launch_bwd_src(const ItemsArg& it, const int32_t* row, const int32_t* csc_eid, const int32_t* csc2csr,
                          int heads, int C, const float* h, const float* ss, const float* nstate, const float* go,
                          int mode, float slope, float gscale, float p, uint64_t seed, const uint64_t* seed_in,
                          float* dh, int64_t ld_dh,
                          float* ds_src, int64_t ld_ds, float* dz, float* partial, const int32_t* hub_row,
                          const int32_t* hub_ptr, int64_t n_hubs, hipStream_t st) {
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int64_t n_long = short_begin(it, heads, C);
  const Items its{it.row, it.beg, it.end, n_long, it.n_hub_items};
  if (n_long > 0) {
    const bool mh = heads > 1 && C >= 32 && (heads == 2 || heads == 4 || heads == 8);
    if (mh) {  // every head of an edge in one pass (one grad_out gather per edge)
#define PPGAT_MH(HH)                                                                                           \
  PPGAT_DISPATCH_C(C, if constexpr (CC >= 32) {                                                             \
    hipLaunchKernelGGL((k_bwd_src_mh<CC, HH>), dim3(blocks_for(n_long * 64)), dim3(256), 0, st, its, row,      \
                       csc_eid, csc2csr, h, ss, reinterpret_cast<const float4*>(nstate), go, mode, slope, gscale, \
                       p, inv_keep, seed, seed_in, dh, ld_dh, ds_src, ld_ds, dz, partial);                    \
  })
      if (heads == 2) { PPGAT_MH(2); } else if (heads == 4) { PPGAT_MH(4); } else { PPGAT_MH(8); }
#undef PPGAT_MH
    } else {
      PPGAT_DISPATCH_C(C, hipLaunchKernelGGL(k_bwd_src<CC>, dim3(blocks_for(n_long * 64)), dim3(256), 0, st, its,
                                             row, csc_eid, csc2csr, heads, h, ss,
                                             reinterpret_cast<const float4*>(nstate), go, mode, slope, gscale, p,
                                             inv_keep, seed, seed_in, dh, ld_dh, ds_src, ld_ds, dz, partial));
    }
  }
  // the short items after the long ones, with the hub merges at the head of that launch
  const bool fold = n_long < it.n_items;
  if (fold) {
    const Items all{it.row, it.beg, it.end, it.n_items, it.n_hub_items};
    const HubMerge mg{hub_row, hub_ptr, n_hubs, heads, partial, n_hubs > 0 ? (n_hubs + 3) / 4 : 0};
    const unsigned g = (unsigned)((it.n_items - n_long + 15) / 16 + mg.mblocks);
    PPGAT_DISPATCH_C64(C, hipLaunchKernelGGL(k_bwd_src_short<CC>, dim3(g), dim3(256), 0, st, all, n_long, row,
                                             csc_eid, csc2csr, h, ss, reinterpret_cast<const float4*>(nstate), go,
                                             mode, slope, gscale, p, inv_keep, seed, seed_in, dh, ld_dh, ds_src, ld_ds,
                                             dz, mg));
  }
  if (n_hubs > 0 && !fold) {
    PPGAT_DISPATCH_C(C, hipLaunchKernelGGL(k_bwd_merge<CC>, dim3(blocks_for(n_hubs * 64)), dim3(256), 0, st,
                                           hub_row, hub_ptr, n_hubs, heads, partial, dh, ld_dh, ds_src, ld_ds));
  }
  return hipGetLastError();
}

int64_t epi_blocks(int64_t n) {
  // fixed partition: >= 4 blocks per CU when N allows, capped so the block-partial
  // slab (blocks x 2 x H x C floats) stays small
  int64_t b = (n + 31) / 32;
  if (b < 1) b = 1;
  if (b > kEpiMaxBlocks) b = kEpiMaxBlocks;
  return b;
}

hipError_t launch_bwd_epi(const int32_t* rowptr, int64_t n, int heads, int C, const float* h, const float* as,
                          const float* ad, const float* ds_src, const float* dz, float* dh, float* partial,
                          int64_t blocks, hipStream_t st) {
  PPGAT_DISPATCH_C(C, hipLaunchKernelGGL(k_bwd_epi<CC>, dim3((unsigned)blocks), dim3(256), 0, st, rowptr, n, heads,
                                         h, as, ad, ds_src, dz, dh, partial));
  return hipGetLastError();
}

hipError_t launch_dst_sum(const ItemsArg& it, int heads, const float* dz, const int32_t* csr2csc, float* ds_dst,
                          int64_t ld, float* partial, const int32_t* hub_row, const int32_t* hub_ptr, int64_t n_hubs,
                          hipStream_t st) {
  const int64_t pairs = it.n_items * heads;
  if (pairs == 0) return hipSuccess;
  const Items items{it.row, it.beg, it.end, it.n_items, it.n_hub_items};
  const bool aligned = (reinterpret_cast<uintptr_t>(dz) % (4 * heads)) == 0;
#ifdef PPGAT_LAB_BUILD
  static const int aux = [] {
    const char* e = getenv("PPGAT_DST_AUX");
    return e ? atoi(e) : 0;
  }();
  if (aux != 0 && csr2csc != nullptr && (heads == 1 || (heads == 4 && aligned))) {
    if (heads == 1) {
#define PPGAT_DST_LAB(A) hipLaunchKernelGGL((k_dst_sum<true, A>), dim3(blocks_for(pairs * 16)), dim3(256), 0, st, \
                                            items, heads, dz, csr2csc, ds_dst, ld, partial)
      if (aux == 2) PPGAT_DST_LAB(2);
      else if (aux == 17) PPGAT_DST_LAB(17);
      else if (aux == 19) PPGAT_DST_LAB(19);
      else PPGAT_DST_LAB(1);
#undef PPGAT_DST_LAB
    } else {
      const int64_t nl = it.n_long_items >= 0 ? it.n_long_items : it.n_items;
      const Items lng{it.row, it.beg, it.end, nl, it.n_hub_items};
      const dim3 gl(blocks_for(nl * 16)), gs(blocks_for(it.n_items - nl));
#define PPGAT_DST_LAB(A)                                                                                        \
  do {                                                                                                          \
    if (nl > 0)                                                                                                 \
      hipLaunchKernelGGL((k_dst_sum_vh<true, 4, A>), gl, dim3(256), 0, st, lng, dz, csr2csc, ds_dst, ld, partial); \
    if (it.n_items > nl)                                                                                        \
      hipLaunchKernelGGL((k_dst_sum_vh_short<4, A>), gs, dim3(256), 0, st, items, nl, dz, csr2csc, ds_dst, ld);    \
  } while (0)
      if (aux == 2) PPGAT_DST_LAB(2);
      else if (aux == 17) PPGAT_DST_LAB(17);
      else if (aux == 19) PPGAT_DST_LAB(19);
      else PPGAT_DST_LAB(1);
#undef PPGAT_DST_LAB
    }
    if (n_hubs > 0)
      hipLaunchKernelGGL(k_dst_merge, dim3((unsigned)((n_hubs + 3) / 4)), dim3(256), 0, st, hub_row, hub_ptr, n_hubs,
                         heads, partial, ds_dst, ld);
    return hipGetLastError();
  }
#endif
  if (csr2csc != nullptr && (heads == 2 || heads == 4) && aligned) {
    // the long items (and hub pieces) 16 lanes each; the short ones (known when the schedule
    // counted them) one thread each, the same bits (k_dst_sum_vh_short)
    const int64_t nl = it.n_long_items >= 0 ? it.n_long_items : it.n_items;
    const Items lng{it.row, it.beg, it.end, nl, it.n_hub_items};
    if (nl > 0) {
      if (heads == 2)
        hipLaunchKernelGGL((k_dst_sum_vh<true, 2>), dim3(blocks_for(nl * 16)), dim3(256), 0, st, lng, dz, csr2csc,
                           ds_dst, ld, partial);
      else
        hipLaunchKernelGGL((k_dst_sum_vh<true, 4>), dim3(blocks_for(nl * 16)), dim3(256), 0, st, lng, dz, csr2csc,
                           ds_dst, ld, partial);
    }
    if (it.n_items > nl) {
      const dim3 g(blocks_for(it.n_items - nl));
      if (heads == 2)
        hipLaunchKernelGGL((k_dst_sum_vh_short<2>), g, dim3(256), 0, st, items, nl, dz, csr2csc, ds_dst, ld);
      else
        hipLaunchKernelGGL((k_dst_sum_vh_short<4>), g, dim3(256), 0, st, items, nl, dz, csr2csc, ds_dst, ld);
    }
  } else if (csr2csc != nullptr)
    hipLaunchKernelGGL(k_dst_sum<true>, dim3(blocks_for(pairs * 16)), dim3(256), 0, st, items, heads, dz, csr2csc,
                       ds_dst, ld, partial);
  else
    hipLaunchKernelGGL(k_dst_sum<false>, dim3(blocks_for(pairs * 16)), dim3(256), 0, st, items, heads, dz, csr2csc,
                       ds_dst, ld, partial);
  if (n_hubs > 0)
    hipLaunchKernelGGL(k_dst_merge, dim3((unsigned)((n_hubs + 3) / 4)), dim3(256), 0, st, hub_row, hub_ptr, n_hubs,
                       heads, partial, ds_dst, ld);
  return hipGetLastError();
}

// the achievable-HBM yardstick (ppgat_stream_copy): one float4 per thread, non-temporal load and
// store, the grid covering the buffer in one pass -- the fastest of the variants measured
// (tools/copy_lab.hip, profiles/r06/x3_copy_lab.log: 6.58 TB/s on a 1 GiB copy; 2-8 float4 per
// thread, default-policy accesses or a grid-stride loop 4.3-6.2 TB/s)
typedef float stream_f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_stream_copy(const stream_f4* __restrict__ src, stream_f4* __restrict__ dst,
                                                     int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

hipError_t launch_stream_copy(const void* src, void* dst, int64_t n_bytes, hipStream_t st) {
  const int64_t n4 = n_bytes / 16;
  if (n4 <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st,
                     static_cast<const stream_f4*>(src), static_cast<stream_f4*>(dst), n4);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_invert_index(const int32_t* __restrict__ p, int64_t n,
                                                      int32_t* __restrict__ inv) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) inv[p[k]] = (int32_t)k;
}

hipError_t launch_invert_index(const int32_t* p, int64_t n, int32_t* inv, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_invert_index, dim3(blocks_for(n)), dim3(256), 0, st, p, n, inv);
  return hipGetLastError();
}

hipError_t launch_col_reduce(const float* partial, int64_t rows, int cols, int split, float* out_a, float* out_b,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_col_reduce, dim3((unsigned)((cols + 63) / 64)), dim3(1024), 0, st, partial, rows, cols, split,
                     out_a, out_b);
  return hipGetLastError();
}

namespace {
__global__ void k_drop_epoch(int set, uint64_t value) {
  if (threadIdx.x == 0) g_drop_epoch = set ? value : g_drop_epoch + 1;
}
}  // namespace

hipError_t seed_snapshot(uint64_t seed, uint64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_seed_snap, dim3(1), dim3(64), 0, st, seed, out);
  return hipGetLastError();
}

hipError_t dropout_epoch(int set, uint64_t value, hipStream_t st) {
  hipLaunchKernelGGL(k_drop_epoch, dim3(1), dim3(64), 0, st, set, value);
  return hipGetLastError();
}

}  // namespace ppgat
