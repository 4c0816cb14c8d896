// ppgat_train.hip -- the rest of the training step around the GAT layers, for CDNA4.
//
//  * BPR / BCE loss over sampled triples (scripts/train_gat_pyg.py:313-322): fused gather
//    of U[u], I[i], I[j] + dot products + loss terms (forward), and the gradient
//    dZ = A Z where A has 4 nonzeros per triple, computed deterministically by sorting
//    the 4S contributions by destination row and summing fixed 32-entry chunks with an
//    ordered fix-up for rows that span chunks (no float atomics).
//  * dW = A^T B for tall-skinny fp32 operands (A [N,M], B [N,K], N ~ 10^5..10^7, M,K <= 1024):
//    the weight gradient of every projection (GATConv.lin, item_proj).  hipBLASLt picks a
//    16-workgroup tile for this shape; here N is split over ~512 workgroups, each
//    accumulating a 128x128 tile with v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains),
//    followed by an ordered reduction of the split partials.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>
#include <math.h>

#include "ppgat_internal.h"
#include "ppgat_lanes.h"

namespace ppgat {

namespace {

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}
__device__ __forceinline__ float4 fma4(float s, float4 v, float4 a) {
  return make_float4(fmaf(s, v.x, a.x), fmaf(s, v.y, a.y), fmaf(s, v.z, a.z), fmaf(s, v.w, a.w));
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

unsigned key_bits(int64_t n) {
  unsigned b = 1;
  while (b < 31 && ((int64_t)1 << b) < n) ++b;
  return b;
}

__device__ __forceinline__ int64_t clamp_idx(int64_t v, int64_t n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); }
// Z row of node id v (users [0, n_users), items n_users + i); row_map != NULL remaps (sharded
// runs keep Z in a padded per-rank row space)
__device__ __forceinline__ int64_t zrow(const int32_t* row_map, int64_t v) { return row_map ? row_map[v] : v; }

// ---------------------------------------------------------------------------
// BPR forward: one subgroup (C/4 lanes) per triple.
//   pos = <U[u], I[i]>, neg = <U[u], I[j]>
//   bpr: l = -log(sigmoid(pos - neg) + 1e-8); dl/dpos = -dl/dneg = -s(1-s)/(s+1e-8)/S
//   bce: l = bce_logits(pos, 1) + bce_logits(neg, 0); dl/dpos = (s(pos)-1)/2S, dl/dneg = s(neg)/2S
// coef[t] = {dl/dpos, dl/dneg} (before the upstream scalar grad); per-block loss sums.
// ---------------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(256) k_bpr_fwd(const float* __restrict__ Z, int64_t n_users, int64_t n_items,
                                                 const int64_t* __restrict__ u, const int64_t* __restrict__ ii,
                                                 const int64_t* __restrict__ jj, int64_t S, int kind,
                                                 float2* __restrict__ coef, float* __restrict__ block_loss,
                                                 int32_t* __restrict__ block_bad, const int32_t* __restrict__ row_map) {
  constexpr int LPR = C / 4;
  constexpr int SPB = 256 / LPR;  // subgroups (triples in flight) per block
  __shared__ float sl_loss[SPB];
  __shared__ int sl_bad[SPB];
  int nbad = 0;  // out-of-range triples of this subgroup (counted per block: no zeroed counter needed)
  const int tid = threadIdx.x;
  const int sg = tid / LPR, sl = tid % LPR;
  float lsum = 0.f;  // this subgroup's triples, in order (fixed grid => fixed partition)
  for (int64_t t = (int64_t)blockIdx.x * SPB + sg; t - sg < S; t += (int64_t)gridDim.x * SPB) {
    const bool valid = t < S;
    float pos = 0.f, neg = 0.f;
    bool skip = false;  // row_map -1: user not held here (row-sharded loss), triple contributes 0
    if (valid) {
      const int64_t u0 = u[t], i0 = ii[t], j0 = jj[t];
      const bool oob = u0 < 0 || u0 >= n_users || i0 < 0 || i0 >= n_items || j0 < 0 || j0 >= n_items;
      const int64_t ur = zrow(row_map, clamp_idx(u0, n_users));
      const int64_t ir = zrow(row_map, n_users + clamp_idx(i0, n_items));
      const int64_t jr = zrow(row_map, n_users + clamp_idx(j0, n_items));
      skip = ur < 0;
      if (!skip) {
        const float4 a = ld4(Z + ur * C + sl * 4);
        pos = dot4(a, ld4(Z + ir * C + sl * 4));
        neg = dot4(a, ld4(Z + jr * C + sl * 4));
      }
      nbad += oob ? 1 : 0;  // indices were clamped; the caller raises
    }
    pos = group_reduce<Op::Sum, 1, LPR / 2>(pos);  // DPP / permlane steps, no LDS round trips
    neg = group_reduce<Op::Sum, 1, LPR / 2>(neg);
    if (sl == 0 && valid && skip) coef[t] = make_float2(0.f, 0.f);
    if (sl == 0 && valid && !skip) {
      float l;
      float2 cf;
      if (kind == 0) {
        const float x = pos - neg;
        const float s = 1.f / (1.f + expf(-x));
        l = -logf(s + 1e-8f);
        const float d = -(s * (1.f - s)) / (s + 1e-8f) / (float)S;
        cf = make_float2(d, -d);
      } else {
        const float sp = 1.f / (1.f + expf(-pos)), sn = 1.f / (1.f + expf(-neg));
        l = (fmaxf(pos, 0.f) - pos + log1pf(expf(-fabsf(pos)))) + (fmaxf(neg, 0.f) + log1pf(expf(-fabsf(neg))));
        cf = make_float2((sp - 1.f) / (2.f * S), sn / (2.f * S));
      }
      coef[t] = cf;
      lsum += l;
    }
  }
  if (sl == 0) {
    sl_loss[sg] = lsum;
    sl_bad[sg] = nbad;
  }
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    int b = 0;
    for (int k = 0; k < SPB; ++k) {
      s += sl_loss[k];
      b += sl_bad[k];
    }
    block_loss[blockIdx.x] = s;
    block_bad[blockIdx.x] = b;
  }
}

// ordered sum of the block losses -> loss (mean)
// (and the total of the blocks' out-of-range counts -> *bad, when asked)
__global__ void __launch_bounds__(1024) k_bpr_loss(const float* __restrict__ block_loss,
                                                   const int32_t* __restrict__ block_bad, int64_t nb, float denom,
                                                   float* __restrict__ loss, int32_t* __restrict__ bad) {
  __shared__ float red[1024];
  __shared__ int redb[1024];
  float s = 0.f;
  int c = 0;
  for (int64_t b = threadIdx.x; b < nb; b += 1024) {
    s += block_loss[b];
    c += block_bad[b];
  }
  red[threadIdx.x] = s;
  redb[threadIdx.x] = c;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[threadIdx.x] += red[threadIdx.x + w];
      redb[threadIdx.x] += redb[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss[0] = red[0] / denom;
    if (bad != nullptr) bad[0] = redb[0];
  }
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort of (key, value) int32 pairs, keys < 2^bits, for the loss backward
// (4S contributions by destination row).  ceil(bits / 10) passes of db <= 10 bits; per pass
//   k_rs_hist    tile digit counts (LDS int atomics: exact), digit-major [nd][tiles]
//   exclusive scan of the counts (rocPRIM) -> global digit/tile offsets
//   k_rs_scatter stable rank inside the tile: tile items are taken round-major (round r,
//                wave w, lane l), a lane's same-digit peers come from db ballots, the
//                per-(wave, digit) counts are scanned over waves in LDS, and the tile's
//                running digit totals carry from round to round.
// A handful of launches instead of rocPRIM's ~20-launch merge sort at this size.
// ---------------------------------------------------------------------------
#ifndef PPGAT_RS_THREADS
#define PPGAT_RS_THREADS 1024
#endif
#ifndef PPGAT_RS_ROUNDS
#define PPGAT_RS_ROUNDS 4
#endif
constexpr int kRsThreads = PPGAT_RS_THREADS;
constexpr int kRsWaves = kRsThreads / 64;
constexpr int kRsRounds = PPGAT_RS_ROUNDS;
constexpr int kRsTile = kRsThreads * kRsRounds;

__global__ void __launch_bounds__(kRsThreads) k_rs_hist(const int32_t* __restrict__ keys, int64_t n, int shift, int db,
                                                        int32_t* __restrict__ ghist, int64_t tiles) {
  extern __shared__ int32_t h[];
  const int nd = 1 << db;
  for (int d = threadIdx.x; d < nd; d += kRsThreads) h[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
#pragma unroll
  for (int r = 0; r < kRsRounds; ++r) {
    const int64_t p = base + r * kRsThreads + threadIdx.x;
    if (p < n) atomicAdd(&h[(keys[p] >> shift) & (nd - 1)], 1);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nd; d += kRsThreads) ghist[(int64_t)d * tiles + blockIdx.x] = h[d];
}

__global__ void __launch_bounds__(kRsThreads) k_rs_scatter(const int32_t* __restrict__ kin,
                                                           const int32_t* __restrict__ vin, int64_t n, int shift,
                                                           int db, const int32_t* __restrict__ goff, int64_t tiles,
                                                           int32_t* __restrict__ kout, int32_t* __restrict__ vout,
                                                           uint8_t* __restrict__ mark, int64_t mark_n) {
  extern __shared__ int32_t sm[];
  const int nd = 1 << db;
  int32_t* wc = sm;                   // [kRsWaves][nd]
  int32_t* tot = sm + kRsWaves * nd;  // [nd] running position of each digit
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int d = threadIdx.x; d < nd; d += kRsThreads) tot[d] = goff[(int64_t)d * tiles + blockIdx.x];
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
  for (int r = 0; r < kRsRounds; ++r) {
    if (base + (int64_t)r * kRsThreads >= n) break;  // block-uniform
    for (int q = threadIdx.x; q < kRsWaves * nd; q += kRsThreads) wc[q] = 0;
    __syncthreads();
    const int64_t p = base + (int64_t)r * kRsThreads + threadIdx.x;
    const bool valid = p < n;
    const int32_t k = valid ? kin[p] : 0;
    const int32_t v = valid ? vin[p] : 0;
    const int d = (k >> shift) & (nd - 1);
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < db; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(bit);
      peers &= bit ? bb : ~bb;
    }
    const int rank = __popcll(peers & below);
    if (valid && rank == 0) wc[w * nd + d] = __popcll(peers);
    __syncthreads();
    for (int dd = threadIdx.x; dd < nd; dd += kRsThreads) {
      int32_t run = tot[dd];
#pragma unroll
      for (int ww = 0; ww < kRsWaves; ++ww) {
        const int32_t t = wc[ww * nd + dd];
        wc[ww * nd + dd] = run;
        run += t;
      }
      tot[dd] = run;
    }
    __syncthreads();
    if (valid) {
      const int64_t pos = wc[w * nd + d] + rank;
      kout[pos] = k;
      vout[pos] = v;
      if (mark != nullptr && k < mark_n) mark[k] = 1;  // (last pass, when asked: the keys present)
    }
    __syncthreads();
  }
}

struct RsPlan {
  int passes, db;
  int64_t tiles, cells;  // cells = nd * tiles
  size_t scan_bytes;
};

RsPlan rs_plan(int64_t n, unsigned bits) {
  RsPlan pl{};
  pl.passes = (int)((bits + 9) / 10);
  if (pl.passes < 1) pl.passes = 1;
  pl.db = (int)((bits + pl.passes - 1) / pl.passes);
  pl.tiles = (n + kRsTile - 1) / kRsTile;
  if (pl.tiles < 1) pl.tiles = 1;
  pl.cells = ((int64_t)1 << pl.db) * pl.tiles;
  size_t b = 0;
  (void)rocprim::exclusive_scan(nullptr, b, (int32_t*)nullptr, (int32_t*)nullptr, 0, (size_t)pl.cells,
                                rocprim::plus<int32_t>());
  pl.scan_bytes = b;
  return pl;
}

size_t rs_workspace_bytes(int64_t n, unsigned bits) {
  const RsPlan pl = rs_plan(n, bits);
  return 2 * align_up((size_t)pl.cells * 4) + align_up(pl.scan_bytes);
}

// sorts (k0, v0) using (k1, v1) as the ping-pong pair; *result_in_1 says where it ended.
// mark != NULL: the last pass also sets mark[k] = 1 for every key k < mark_n.
hipError_t rs_sort(int32_t* k0, int32_t* v0, int32_t* k1, int32_t* v1, int64_t n, unsigned bits, void* ws,
                   bool* result_in_1, hipStream_t st, uint8_t* mark = nullptr, int64_t mark_n = 0) {
  const RsPlan pl = rs_plan(n, bits);
  char* p = static_cast<char*>(ws);
  int32_t* ghist = reinterpret_cast<int32_t*>(p);
  int32_t* goff = reinterpret_cast<int32_t*>(p + align_up((size_t)pl.cells * 4));
  void* tmp = p + 2 * align_up((size_t)pl.cells * 4);
  size_t tmp_bytes = pl.scan_bytes;
  const int nd = 1 << pl.db;
  bool in1 = false;
  for (int ps = 0; ps < pl.passes; ++ps) {
    const int shift = ps * pl.db;
    int32_t* ki = in1 ? k1 : k0;
    int32_t* vi = in1 ? v1 : v0;
    int32_t* ko = in1 ? k0 : k1;
    int32_t* vo = in1 ? v0 : v1;
    hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)pl.tiles), dim3(kRsThreads), nd * 4, st, ki, n, shift, pl.db, ghist,
                       pl.tiles);
    hipError_t e = rocprim::exclusive_scan(tmp, tmp_bytes, ghist, goff, 0, (size_t)pl.cells,
                                           rocprim::plus<int32_t>(), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)pl.tiles), dim3(kRsThreads), (kRsWaves + 1) * nd * 4, st, ki, vi,
                       n, shift, pl.db, goff, pl.tiles, ko, vo, ps + 1 == pl.passes ? mark : nullptr, mark_n);
    in1 = !in1;
  }
  *result_in_1 = in1;
  return hipGetLastError();
}

// contribution c = 4t + kind -> destination row (sort key)
// (contributions of triples whose user row is -1 -- not held here -- get the sentinel key
// n_rows: they sort last and are never written)
__global__ void k_bpr_keys(const int64_t* __restrict__ u, const int64_t* __restrict__ ii,
                           const int64_t* __restrict__ jj, int64_t S, int64_t n_users, int64_t n_items,
                           const int32_t* __restrict__ row_map, int64_t n_rows, int32_t* __restrict__ key,
                           int32_t* __restrict__ val, uint8_t* __restrict__ touched) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the touched-row map cleared here (16 B per thread; the region is a multiple of 16 B), set by
  // the sort's last pass: no fill or mark launch of its own
  if (c * 16 < n_rows) *reinterpret_cast<uint4*>(touched + c * 16) = make_uint4(0u, 0u, 0u, 0u);
  if (c >= 4 * S) return;
  const int64_t t = c >> 2;
  const int kd = (int)(c & 3);
  int64_t d;
  if (kd < 2) d = clamp_idx(u[t], n_users);
  else if (kd == 2) d = n_users + clamp_idx(ii[t], n_items);
  else d = n_users + clamp_idx(jj[t], n_items);
  const bool skip = zrow(row_map, clamp_idx(u[t], n_users)) < 0;
  key[c] = skip ? (int32_t)n_rows : (int32_t)zrow(row_map, d);
  val[c] = (int32_t)c;
}

// ---------------------------------------------------------------------------
// BPR backward, chunk pass: a subgroup owns 32 consecutive sorted contributions.
// Segments (runs of one destination row) complete inside the chunk are written to dZ;
// a segment touching the chunk start while continuing from the previous chunk goes to
// slot "head"; one touching the chunk end and continuing goes to slot "tail".
// ---------------------------------------------------------------------------
constexpr int kChunk = 32;

// The backward prologue of the GAT layer that produced Z (heads = 1; the layer's own
// ppgat_bwd_prologue, done here while the finished dZ row is in registers): for every row r
//   nstate[r] = {s_dst[r], m[r], inv_l[r], gscale <dZ_r, Z_r - bias>}
// (Z_r loaded with the segment's contributions, so the dot costs no extra round trip), and
// grad_bias = sum_r dZ_r = the sum of every contribution (block partials bpart, reduced in block
// order).  nstate == NULL: off.
struct BprPro {
  const float* bias;   // nullable
  const float* sdst;
  const float* m;
  const float* invl;
  float gscale;
  float4* nstate;
  float* bpart;        // nullable: [chunk blocks][C]
  int64_t nbpart;      // chunk blocks
  float* groups;       // [ceil(nbpart / kBpGroup)][C]: stage 1 of the ordered dbias sum (k_bpr_fixup)
  float* grad_bias;    // stage 2 (k_bpr_zero_untouched)
};

// <a, z> over the LPR lanes of a subgroup (4 columns per lane), accumulated in fp64 over a fixed
// tree: the prologue's D feeds the logit gradients alpha (d - D), whose destination sums
// cancel -- D is rounded once, from the fp32 dZ and Z values, not at every partial sum
constexpr int kBpGroup = 32;  // chunk-block partials per stage-1 group of the producer's dbias

template <int LPR>
__device__ __forceinline__ float subgroup_dot(float4 a, float4 z) {
  double v = fma((double)a.w, (double)z.w, fma((double)a.z, (double)z.z, fma((double)a.y, (double)z.y,
                                                                              (double)a.x * (double)z.x)));
#pragma unroll
  for (int sh = 1; sh < LPR; sh <<= 1) v += __shfl_xor(v, sh);
  return (float)v;
}

template <int C>
__global__ void __launch_bounds__(256) k_bpr_chunks(const int32_t* __restrict__ skey, const int32_t* __restrict__ scid,
                                                    int64_t total, const int64_t* __restrict__ u,
                                                    const int64_t* __restrict__ ii, const int64_t* __restrict__ jj,
                                                    int64_t n_users, int64_t n_items,
                                                    const int32_t* __restrict__ row_map,
                                                    const float2* __restrict__ coef,
                                                    const float* __restrict__ grad_loss, const float* __restrict__ Z,
                                                    int64_t n_rows, float* __restrict__ dZ, float* __restrict__ slots,
                                                    BprPro pro) {
  constexpr int LPR = C / 4;
  constexpr int SPB = 256 / LPR;
  __shared__ int32_t s_src[SPB][kChunk];
  __shared__ int32_t s_dst[SPB][kChunk];
  __shared__ float s_cf[SPB][kChunk];
  __shared__ float4 s_bp[SPB][LPR];
  const int tid = threadIdx.x;
  const int sg = tid / LPR, sl = tid % LPR;
  const int64_t ch = (int64_t)blockIdx.x * SPB + sg;
  const int64_t b0 = ch * kChunk;
  const float g = grad_loss[0];
  const bool pon = pro.nstate != nullptr;
  if (b0 < total) {
    for (int q = sl; q < kChunk; q += LPR) {
      const int64_t p = b0 + q;
      int32_t src = 0, dst = -1;
      float cf = 0.f;
      if (p < total) {
        const int32_t c = scid[p];
        const int64_t t = c >> 2;
        const int kd = c & 3;
        const float2 tc = coef[t];
        dst = skey[p];
        if (dst < n_rows) {
          if (kd == 0) { src = (int32_t)zrow(row_map, n_users + clamp_idx(ii[t], n_items)); cf = tc.x; }
          else if (kd == 1) { src = (int32_t)zrow(row_map, n_users + clamp_idx(jj[t], n_items)); cf = tc.y; }
          else { src = (int32_t)zrow(row_map, clamp_idx(u[t], n_users)); cf = kd == 2 ? tc.x : tc.y; }
        }
      }
      s_src[sg][q] = src;
      s_dst[sg][q] = dst;
      s_cf[sg][q] = cf * g;
    }
  }
  __syncthreads();
  float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);  // producer dbias: every contribution of this subgroup
  const float4 bb = (pon && pro.bias) ? ld4(pro.bias + sl * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  if (b0 < total) {
    const int len = (int)min((int64_t)kChunk, total - b0);
    const bool starts_before = b0 > 0 && skey[b0 - 1] == s_dst[sg][0];
    const bool ends_after = b0 + len < total && skey[b0 + len] == s_dst[sg][len - 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int seg_start = 0;
    constexpr int U = 4;
    for (int q0 = 0; q0 < len; q0 += U) {
      float4 v[U], zd[U];
      float ps[U], pm[U], pl[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int q = q0 + k;
        v[k] = q < len ? ld4(Z + (int64_t)s_src[sg][q] * C + sl * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        // where a segment finishing in this chunk ends: the destination row itself and its
        // forward state (prologue), loaded with the contributions -- no round trip at the end
        const int32_t rq = s_dst[sg][q < len ? q : 0];
        const bool fin = pon && q < len && (q == len - 1 ? !ends_after : s_dst[sg][q + 1] != rq) && rq < n_rows;
        zd[k] = fin ? ld4(Z + (int64_t)rq * C + sl * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool fin0 = fin && sl == 0;
        ps[k] = fin0 ? pro.sdst[rq] : 0.f;
        pm[k] = fin0 ? pro.m[rq] : 0.f;
        pl[k] = fin0 ? pro.invl[rq] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int q = q0 + k;
        if (q >= len) break;
        acc = fma4(s_cf[sg][q], v[k], acc);
        const bool last_of_seg = q == len - 1 || s_dst[sg][q + 1] != s_dst[sg][q];
        if (last_of_seg) {
          const int32_t r = s_dst[sg][q];
          const bool first = seg_start == 0, last = q == len - 1;
          if (first && starts_before) st4(slots + (ch * 2 + 0) * C + sl * 4, acc);
          else if (last && ends_after) st4(slots + (ch * 2 + 1) * C + sl * 4, acc);
          else if (r < n_rows) {
            st4(dZ + (int64_t)r * C + sl * 4, acc);
            if (pon) {  // (uniform over the subgroup: its lanes share the segment)
              const float4 zr = make_float4(zd[k].x - bb.x, zd[k].y - bb.y, zd[k].z - bb.z, zd[k].w - bb.w);
              const float d = subgroup_dot<LPR>(acc, zr);
              if (sl == 0) pro.nstate[r] = make_float4(ps[k], pm[k], pl[k], d * pro.gscale);
            }
          }
          if (pon) bsum = add4(bsum, acc);
          acc = make_float4(0.f, 0.f, 0.f, 0.f);
          seg_start = q + 1;
        }
      }
    }
  }
  if (!pon || pro.bpart == nullptr) return;
  s_bp[sg][sl] = bsum;
  __syncthreads();
  if (tid < LPR) {  // the block's subgroups in order
    float4 s = s_bp[0][tid];
    for (int q = 1; q < SPB; ++q) s = add4(s, s_bp[q][tid]);
    st4(pro.bpart + (int64_t)blockIdx.x * C + tid * 4, s);
  }
}

// Rows no contribution reaches are zeroed by a row-parallel pass over a byte map of the rows
// (whatever the key distribution: a rank whose triples are all sentinels, few triples, a huge
// Z): k_bpr_keys clears the map, the sort's last scatter pass sets touched[key] for every key
// (plain byte stores of one value, no atomics needed), k_bpr_zero_untouched writes zero rows
// where the byte is clear.  Every row of [0, n_rows) is still written exactly once
// (k_bpr_chunks / k_bpr_fixup, or here).
template <int C>
__global__ void __launch_bounds__(256) k_bpr_zero_untouched(const uint8_t* __restrict__ touched, int64_t n_rows,
                                                            float* __restrict__ dZ, BprPro pro) {
  constexpr int LPR = C / 4;
  constexpr int SPB = 256 / LPR;
  const int sg = threadIdx.x / LPR, sl = threadIdx.x % LPR;
  if (pro.bpart != nullptr && blockIdx.x == 0 && (int)threadIdx.x < C) {  // the producer's dbias, stage 2
    const int64_t ng = (pro.nbpart + kBpGroup - 1) / kBpGroup;
    float t = 0.f;
    for (int64_t q0 = 0; q0 < ng; q0 += 16) {  // 16 loads in flight, summed in order
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = q0 + k < ng ? pro.groups[(q0 + k) * C + threadIdx.x] : 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) t += v[k];
    }
    pro.grad_bias[threadIdx.x] = t;
  }
  for (int64_t r = (int64_t)blockIdx.x * SPB + sg; r < n_rows; r += (int64_t)gridDim.x * SPB)
    if (!touched[r]) {
      st4(dZ + r * C + sl * 4, make_float4(0.f, 0.f, 0.f, 0.f));
      if (pro.nstate != nullptr && sl == 0) pro.nstate[r] = make_float4(pro.sdst[r], pro.m[r], pro.invl[r], 0.f);
    }
}

// Fix-up: the chunk in which a chunk-spanning segment starts sums its tail slot and the
// head slots of the following chunks, in chunk order, and writes the row.
template <int C>
__global__ void __launch_bounds__(256) k_bpr_fixup(const int32_t* __restrict__ skey, int64_t total,
                                                   const float* __restrict__ slots, const float* __restrict__ Z,
                                                   int64_t n_rows, float* __restrict__ dZ, BprPro pro) {
  constexpr int LPR = C / 4;
  constexpr int SPB = 256 / LPR;
  const int sg = threadIdx.x / LPR, sl = threadIdx.x % LPR;
  if (pro.bpart != nullptr && (int64_t)blockIdx.x * kBpGroup < pro.nbpart && (int)threadIdx.x < C) {
    // the producer's dbias, stage 1: column c of chunk-block partials [32 b, 32 b + 32), every
    // load in flight at once, summed in order
    const int64_t q0 = (int64_t)blockIdx.x * kBpGroup;
    float v[kBpGroup];
#pragma unroll
    for (int k = 0; k < kBpGroup; ++k) v[k] = q0 + k < pro.nbpart ? pro.bpart[(q0 + k) * C + threadIdx.x] : 0.f;
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kBpGroup; ++k) t += v[k];
    pro.groups[(int64_t)blockIdx.x * C + threadIdx.x] = t;
  }
  const int64_t ch = (int64_t)blockIdx.x * SPB + sg;
  const int64_t b0 = ch * kChunk;
  if (b0 >= total) return;
  const int64_t b1 = min(b0 + kChunk, total);
  if (b1 >= total) return;
  const int32_t r = skey[b1 - 1];
  if (skey[b1] != r || r >= n_rows) return;            // last segment does not continue / sentinel
  if (skey[b0] == r && b0 > 0 && skey[b0 - 1] == r) return;  // segment started in an earlier chunk
  const bool pon = pro.nstate != nullptr;
  const float4 zd = pon ? ld4(Z + (int64_t)r * C + sl * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 acc = ld4(slots + (ch * 2 + 1) * C + sl * 4);
  for (int64_t c2 = ch + 1;; ++c2) {
    const int64_t e0 = c2 * kChunk;
    const int64_t e1 = min(e0 + kChunk, total);
    acc = add4(acc, ld4(slots + (c2 * 2 + 0) * C + sl * 4));
    if (!(skey[e1 - 1] == r && e1 < total && skey[e1] == r)) break;
  }
  st4(dZ + (int64_t)r * C + sl * 4, acc);
  if (pon) {
    const float4 bb = pro.bias ? ld4(pro.bias + sl * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 zr = make_float4(zd.x - bb.x, zd.y - bb.y, zd.z - bb.z, zd.w - bb.w);
    const float d = subgroup_dot<LPR>(acc, zr);
    if (sl == 0) pro.nstate[r] = make_float4(pro.sdst[r], pro.m[r], pro.invl[r], d * pro.gscale);
  }
}

// ---------------------------------------------------------------------------
// dW = A^T B.  Block = 256 threads (4 waves) -> 128x128 output tile over rows
// [n0, n1) of A and B; wave (wm, wk) owns a 64x64 sub-tile = 2x2 MFMA 32x32 tiles.
// LDS stages of 32 rows x 128 columns of A and B (16 KB each), double-buffered.
// v_mfma_f32_32x32x2_f32 lane maps: A operand A'[i=l&31][k=l>>5] = A[n+(l>>5)][m0+(l&31)],
// B operand B'[k=l>>5][j=l&31] = B[n+(l>>5)][k0+(l&31)]; C/D: col = l&31,
// row = (r&3) + 8*(r>>2) + 4*(l>>5) for r in [0,16).
// ---------------------------------------------------------------------------
using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int kTN = 128;  // output tile edge
constexpr int kNB = 32;   // rows per LDS stage

constexpr int kMaxV = 16;  // extra row-weighted column sums V^T B (2 * heads <= 16)

__global__ void __launch_bounds__(256) k_gemm_tn(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                                 int64_t ldb, int64_t N, int M, int K, int64_t rows_per_split,
                                                 float* __restrict__ part, float* __restrict__ colsum_part,
                                                 const float* __restrict__ V, int64_t ldv, int nv,
                                                 float* __restrict__ vpart) {
  __shared__ float sA[2][kNB][kTN];
  __shared__ float sB[2][kNB][kTN];
  __shared__ float sV[2][kNB][kMaxV];
  const int tiles_k = (K + kTN - 1) / kTN;
  const int tile = blockIdx.x;
  const int split = blockIdx.y;
  const int m0 = (tile / tiles_k) * kTN, k0 = (tile % tiles_k) * kTN;
  const int64_t n_beg = (int64_t)split * rows_per_split;
  const int64_t n_end = min(N, n_beg + rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wk = w & 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  float csum = 0.f;  // colsum of A for column m0 + tid (tid < 128), waves 0-1 only
  // (V^T B)[j][k0 + vc] for j = vg, vg + 2, ... < nv (m0 == 0 tiles): all 256 threads
  const int vc = tid & (kTN - 1), vg = tid >> 7;
  float vacc[kMaxV / 2];
#pragma unroll
  for (int q = 0; q < kMaxV / 2; ++q) vacc[q] = 0.f;
  const bool do_v = V != nullptr && m0 == 0;
  // register prefetch: stage s+1's global loads are in flight while stage s's MFMAs run
  float4 ra[4], rb[4];
  float rv[2];
  auto load_regs = [&](int64_t n0) {
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int idx = pass * 256 + tid;  // float4 index within the stage
      const int r = idx >> 5, c4 = (idx & 31) * 4;
      const int64_t n = n0 + r;
      float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
      if (n < n_end) {
        if (m0 + c4 + 3 < M) va = ld4(A + n * lda + m0 + c4);
        else {
          float t[4] = {0.f, 0.f, 0.f, 0.f};
          for (int e = 0; e < 4; ++e) if (m0 + c4 + e < M) t[e] = A[n * lda + m0 + c4 + e];
          va = make_float4(t[0], t[1], t[2], t[3]);
        }
        if (k0 + c4 + 3 < K) vb = ld4(B + n * ldb + k0 + c4);
        else {
          float t[4] = {0.f, 0.f, 0.f, 0.f};
          for (int e = 0; e < 4; ++e) if (k0 + c4 + e < K) t[e] = B[n * ldb + k0 + c4 + e];
          vb = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
      ra[pass] = va;
      rb[pass] = vb;
    }
    if (do_v) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = q * 256 + tid;  // (row, j) of the kNB x kMaxV stage
        const int r = idx / kMaxV, j = idx % kMaxV;
        const int64_t n = n0 + r;
        rv[q] = (j < nv && n < n_end) ? V[n * ldv + j] : 0.f;
      }
    }
  };
  auto store_lds = [&](int buf) {
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int idx = pass * 256 + tid;
      const int r = idx >> 5, c4 = (idx & 31) * 4;
      *reinterpret_cast<float4*>(&sA[buf][r][c4]) = ra[pass];
      *reinterpret_cast<float4*>(&sB[buf][r][c4]) = rb[pass];
    }
    if (do_v) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = q * 256 + tid;
        sV[buf][idx / kMaxV][idx % kMaxV] = rv[q];
      }
    }
  };
  int buf = 0;
  if (n_beg < n_end) {
    load_regs(n_beg);
    store_lds(0);
  }
  __syncthreads();
  for (int64_t n0 = n_beg; n0 < n_end; n0 += kNB) {
    const bool has_next = n0 + kNB < n_end;
    if (has_next) load_regs(n0 + kNB);
#pragma unroll 4
    for (int kk = 0; kk < kNB; kk += 2) {
      const int r = kk + (lane >> 5);
      const float a0 = sA[buf][r][wm * 64 + (lane & 31)];
      const float a1 = sA[buf][r][wm * 64 + 32 + (lane & 31)];
      const float b0 = sB[buf][r][wk * 64 + (lane & 31)];
      const float b1 = sB[buf][r][wk * 64 + 32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (colsum_part != nullptr && k0 == 0 && tid < kTN) {
      for (int r = 0; r < kNB; ++r) csum += sA[buf][r][tid];
    }
    if (do_v) {
      for (int r = 0; r < kNB; ++r) {
        const float b = sB[buf][r][vc];
#pragma unroll
        for (int q = 0; q < kMaxV / 2; ++q) {
          if (vg + 2 * q >= nv) break;
          vacc[q] = fmaf(sV[buf][r][vg + 2 * q], b, vacc[q]);
        }
      }
    }
    if (has_next) store_lds(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // write the split partial tile: part[split][M][K]
  float* P = part + (int64_t)split * M * K;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = k0 + wk * 64 + b * 32 + (lane & 31);
        if (row < M && col < K) P[(int64_t)row * K + col] = acc[a][b][r];
      }
  if (colsum_part != nullptr && k0 == 0 && tid < kTN && m0 + tid < M)
    colsum_part[(int64_t)split * M + m0 + tid] = csum;
  if (do_v && k0 + vc < K) {
#pragma unroll
    for (int q = 0; q < kMaxV / 2; ++q) {
      const int j = vg + 2 * q;
      if (j >= nv) break;
      vpart[((int64_t)split * nv + j) * K + k0 + vc] = vacc[q];
    }
  }
}

// out[e] = sum_s part[s][e] for up to three partial arrays in one launch.  A 1024-thread
// block owns 64 consecutive elements of one array; thread group g (16 of them) sums splits
// g, g + 16, ... with 4 interleaved accumulators, then the 16 group sums are added in
// group order through LDS -- a fixed tree, so the result is deterministic.
struct SplitReduceArg {
  const float* part[3];
  float* out[3];
  int64_t elems[3];
  int64_t blocks[3];  // prefix block offsets: array a owns blocks [blocks[a-1], blocks[a])
};

__global__ void __launch_bounds__(1024) k_split_reduce(SplitReduceArg arg, int64_t splits) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  int a = 0;
  int64_t b = blockIdx.x;
  while (a < 2 && b >= arg.blocks[a]) ++a;
  if (a > 0) b -= arg.blocks[a - 1];
  const float* __restrict__ part = arg.part[a];
  const int64_t elems = arg.elems[a];
  const int64_t e = b * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (e < elems) {
    int64_t k = g;
    for (; k + 48 < splits; k += 64) {
      s0 += part[k * elems + e];
      s1 += part[(k + 16) * elems + e];
      s2 += part[(k + 32) * elems + e];
      s3 += part[(k + 48) * elems + e];
    }
    for (; k < splits; k += 16) s0 += part[k * elems + e];
  }
  red[g][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && e < elems) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][lane];
    arg.out[a][e] = t;
  }
}

}  // namespace

#define PPGAT_DISPATCH_LOSS_C(C_, ...)                         \
  switch (C_) {                                                \
    case 32: { constexpr int CC = 32; __VA_ARGS__; break; }    \
    case 64: { constexpr int CC = 64; __VA_ARGS__; break; }    \
    case 128: { constexpr int CC = 128; __VA_ARGS__; break; }  \
    case 256: { constexpr int CC = 256; __VA_ARGS__; break; }  \
    default: return hipErrorInvalidValue;                      \
  }

bool bpr_channels_ok(int C) { return C == 32 || C == 64 || C == 128 || C == 256; }

// fixed grid (a function of S only): <= 1024 block partials for the one-block loss sum
// one subgroup per triple up to 16384 workgroups: each triple is a chain of dependent loads
// (ids -> row map -> rows), so the loss is latency-bound unless every triple is in flight at
// once (1024 workgroups left 25 rounds of that chain at 200k triples: 44 us, now ~2 rounds)
static int64_t bpr_fwd_blocks(int64_t S, int C) {
  const int64_t b = (S + 256 / (C / 4) - 1) / (256 / (C / 4));
  return b < 16384 ? b : 16384;
}

// workspace: block_loss | keys | vals | skeys | scid | slots | radix sort | touched | producer
// prologue (block partials [chunk blocks][C] | their group sums [groups][C])
static int64_t bpr_chunk_blocks(int64_t S, int C) {
  const int64_t chunks = (4 * S + kChunk - 1) / kChunk;
  const int64_t spb = 256 / (C / 4);
  return (chunks + spb - 1) / spb;
}

// the forward's block partials: loss [nb] floats | out-of-range counts [nb] int32
static size_t bpr_fwd_region(int64_t S, int C) { return align_up((size_t)bpr_fwd_blocks(S, C) * 8 + 4); }

static size_t bpr_base_bytes(int64_t N, int64_t S, int C) {
  const int64_t c4 = 4 * S > 0 ? 4 * S : 1;
  const int64_t chunks = (c4 + kChunk - 1) / kChunk;
  return bpr_fwd_region(S, C) + 4 * align_up((size_t)c4 * 4) +
         align_up((size_t)chunks * 2 * C * 4) + rs_workspace_bytes(c4, key_bits(N + 1)) + align_up((size_t)N + 1);
}

struct BprExtra {
  float* bpart;
  float* groups;
};

// byte offsets of the producer-prologue region: bpart, groups, end
static void bpr_extra_offsets(int64_t N, int64_t S, int C, size_t off[3]) {
  const int64_t blocks = bpr_chunk_blocks(S, C);
  const int64_t groups = (blocks + kBpGroup - 1) / kBpGroup;
  off[0] = bpr_base_bytes(N, S, C);
  off[1] = off[0] + align_up((size_t)(blocks > 0 ? blocks : 1) * C * 4);
  off[2] = off[1] + align_up((size_t)(groups > 0 ? groups : 1) * C * 4);
}

static BprExtra bpr_extra(void* ws, int64_t N, int64_t S, int C) {
  size_t off[3];
  bpr_extra_offsets(N, S, C, off);
  char* p = static_cast<char*>(ws);
  return BprExtra{reinterpret_cast<float*>(p + off[0]), reinterpret_cast<float*>(p + off[1])};
}

size_t bpr_workspace_bytes(int64_t N, int64_t S, int C) {
  size_t off[3];
  bpr_extra_offsets(N, S, C, off);
  return off[2];
}

hipError_t bpr_fwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                   const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, int kind, float* loss,
                   float* coef, int32_t* bad, void* ws, hipStream_t st) {
  float* block_loss = static_cast<float*>(ws);
  (void)n_rows;
  const int64_t nb = bpr_fwd_blocks(S, C);
  int32_t* block_bad = reinterpret_cast<int32_t*>(block_loss + nb);
  if (S > 0) {
    PPGAT_DISPATCH_LOSS_C(C, hipLaunchKernelGGL(k_bpr_fwd<CC>, dim3((unsigned)nb), dim3(256), 0, st, Z, n_users,
                                                n_items, u, i, j, S, kind, reinterpret_cast<float2*>(coef),
                                                block_loss, block_bad, row_map));
  }
  const float denom = kind == 0 ? (float)S : 2.f * (float)S;
  hipLaunchKernelGGL(k_bpr_loss, dim3(1), dim3(1024), 0, st, block_loss, block_bad, S > 0 ? nb : 0,
                     denom > 0 ? denom : 1.f, loss, bad);
  return hipGetLastError();
}

// the backward's part of the workspace (after the forward's block partials)
struct BprWs {
  int32_t *keys, *vals, *skeys, *scid;  // (skeys, scid): where the sorted pairs end up
  float* slots;
  void* tmp;
  uint8_t* touched;
};

static BprWs bpr_ws(void* ws, int64_t N, int64_t S, int C) {
  const int64_t total = 4 * S;
  const int64_t chunks = (total + kChunk - 1) / kChunk;
  char* p = static_cast<char*>(ws) + bpr_fwd_region(S, C);
  const size_t e4 = align_up((size_t)total * 4);
  BprWs w;
  w.keys = reinterpret_cast<int32_t*>(p);
  w.vals = reinterpret_cast<int32_t*>(p + e4);
  const bool in1 = (rs_plan(total, key_bits(N + 1)).passes & 1) != 0;  // odd pass count: in the second pair
  w.skeys = in1 ? reinterpret_cast<int32_t*>(p + 2 * e4) : w.keys;
  w.scid = in1 ? reinterpret_cast<int32_t*>(p + 3 * e4) : w.vals;
  w.slots = reinterpret_cast<float*>(p + 4 * e4);
  w.tmp = p + 4 * e4 + align_up((size_t)chunks * 2 * C * 4);
  w.touched = static_cast<uint8_t*>(w.tmp) + rs_workspace_bytes(total, key_bits(N + 1));
  return w;
}

// The part of the backward that depends on the triples only (not on Z or the loss): the
// contributions' destination rows, sorted, and the touched-row bytes.  Launched on its own
// stream it runs beside the model's forward (bench.py / train.epoch_step).
hipError_t bpr_bwd_prepare(int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                           const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, void* ws,
                           size_t ws_bytes, hipStream_t st) {
  const int64_t N = n_rows;
  if (S == 0) return hipSuccess;
  if (ws_bytes < bpr_workspace_bytes(N, S, C)) return hipErrorInvalidValue;
  const int64_t total = 4 * S;
  const BprWs w = bpr_ws(ws, N, S, C);
  hipError_t err = hipSuccess;
  const int64_t kthreads = total > (N + 15) / 16 ? total : (N + 15) / 16;  // (enough threads to clear the map)
  hipLaunchKernelGGL(k_bpr_keys, dim3((unsigned)((kthreads + 255) / 256)), dim3(256), 0, st, u, i, j, S, n_users,
                     n_items, row_map, N, w.keys, w.vals, w.touched);
  int32_t* k1 = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(w.keys) + 2 * align_up((size_t)total * 4));
  int32_t* v1 = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(w.keys) + 3 * align_up((size_t)total * 4));
  bool in1 = false;
  err = rs_sort(w.keys, w.vals, k1, v1, total, key_bits(N + 1), w.tmp, &in1, st, w.touched, N);
  if (err != hipSuccess) return err;
  if ((in1 ? k1 : w.keys) != w.skeys) return hipErrorUnknown;  // bpr_ws's parity rule disagrees with rs_sort
  return hipGetLastError();
}

// The rest, after bpr_bwd_prepare on the same workspace (stream-ordered after it).  prod !=
// NULL: also the producer layer's backward prologue (BprPro, row_map must be NULL).
hipError_t bpr_bwd_finish(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map,
                          int C, const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, const float* coef,
                          const float* grad_loss, float* dZ, void* ws, size_t ws_bytes, hipStream_t st,
                          const BprProducer* prod) {
  const int64_t N = n_rows;
  if (ws_bytes < bpr_workspace_bytes(N, S, C)) return hipErrorInvalidValue;
  BprPro pk{};
  if (prod != nullptr) {
    const BprExtra x = bpr_extra(ws, N, S, C);
    pk.bias = prod->bias; pk.sdst = prod->s_dst; pk.m = prod->m; pk.invl = prod->inv_l;
    pk.gscale = prod->gscale; pk.nstate = reinterpret_cast<float4*>(prod->nstate);
    pk.bpart = (prod->grad_bias && S > 0) ? x.bpart : nullptr;
    pk.nbpart = bpr_chunk_blocks(S, C);
    pk.groups = x.groups;
    pk.grad_bias = prod->grad_bias;
  }
  const BprWs w = bpr_ws(ws, N, S, C);
  if (S == 0) {
    if (prod == nullptr) return hipMemsetAsync(dZ, 0, (size_t)N * C * 4, st);  // otherwise k_bpr_zero_untouched
    hipError_t e = hipMemsetAsync(w.touched, 0, ((size_t)N + 15) & ~(size_t)15, st);
    if (e == hipSuccess && prod->grad_bias) e = hipMemsetAsync(prod->grad_bias, 0, (size_t)C * 4, st);
    if (e != hipSuccess) return e;
  }
  const int64_t total = 4 * S;
  const int64_t chunks = (total + kChunk - 1) / kChunk;
  PPGAT_DISPATCH_LOSS_C(C, {
    constexpr int SPB = 256 / (CC / 4);
    const unsigned g = (unsigned)((chunks + SPB - 1) / SPB);
    if (S > 0) {
      hipLaunchKernelGGL(k_bpr_chunks<CC>, dim3(g), dim3(256), 0, st, w.skeys, w.scid, total, u, i, j, n_users,
                         n_items, row_map, reinterpret_cast<const float2*>(coef), grad_loss, Z, N, dZ, w.slots, pk);
      hipLaunchKernelGGL(k_bpr_fixup<CC>, dim3(g), dim3(256), 0, st, w.skeys, total, w.slots, Z, N, dZ, pk);
    }
    if (N > 0) {
      int64_t gz = (N + SPB - 1) / SPB;
      if (gz > 4096) gz = 4096;
      hipLaunchKernelGGL(k_bpr_zero_untouched<CC>, dim3((unsigned)gz), dim3(256), 0, st, w.touched, N, dZ, pk);
    }
  });
  return hipGetLastError();
}

hipError_t bpr_bwd(const float* Z, int64_t n_rows, int64_t n_users, int64_t n_items, const int32_t* row_map, int C,
                   const int64_t* u, const int64_t* i, const int64_t* j, int64_t S, const float* coef,
                   const float* grad_loss, float* dZ, void* ws, size_t ws_bytes, hipStream_t st,
                   const BprProducer* prod) {
  hipError_t err = bpr_bwd_prepare(n_rows, n_users, n_items, row_map, C, u, i, j, S, ws, ws_bytes, st);
  if (err != hipSuccess) return err;
  return bpr_bwd_finish(Z, n_rows, n_users, n_items, row_map, C, u, i, j, S, coef, grad_loss, dZ, ws, ws_bytes, st,
                        prod);
}

// ---- skinny A^T B (M <= 16): the multi-head layer's GV = S^T x (S = [ds_src | ds_dst], 2H
// columns) -- a 128 x 128 MFMA tile would be 94 % padding there.  Thread (row lane, float4
// column group of B): fp32 FMAs over the block's rows in order, the row lanes summed in lane
// order, block partials through the ordered split reduction (deterministic). ----
template <int MV>
__global__ void __launch_bounds__(256) k_tn_skinny(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                                   int64_t ldb, int64_t N, int M, int K, int64_t rows_per_block,
                                                   float* __restrict__ part) {
  __shared__ float4 red[256];
  const int T = K >> 2, P = 256 / T, t = threadIdx.x, cg = t % T, rl = t / T;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block, r1 = min(N, r0 + rows_per_block);
  float4 acc[MV];
#pragma unroll
  for (int m = 0; m < MV; ++m) acc[m] = make_float4(0.f, 0.f, 0.f, 0.f);
  auto fma_row = [&](const float4& bv, const float (&av)[MV]) {
#pragma unroll
    for (int m = 0; m < MV; ++m)
      if (m < M)
        acc[m] = make_float4(fmaf(av[m], bv.x, acc[m].x), fmaf(av[m], bv.y, acc[m].y), fmaf(av[m], bv.z, acc[m].z),
                             fmaf(av[m], bv.w, acc[m].w));
  };
  if (rl < P) {
    int64_t r = r0 + rl;
    // four rows' loads in flight together, their FMAs in row order (the same order and bits as
    // one row at a time, which left the kernel waiting on each row's load: 2.5 TB/s)
    for (; r + 3 * P < r1; r += 4 * P) {
      float4 bv[4];
      float av[4][MV];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t ru = r + u * P;
        bv[u] = ld4(B + ru * ldb + 4 * cg);
#pragma unroll
        for (int m = 0; m < MV; ++m) av[u][m] = m < M ? A[ru * lda + m] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) fma_row(bv[u], av[u]);
    }
    for (; r < r1; r += P) {
      float av[MV];
#pragma unroll
      for (int m = 0; m < MV; ++m) av[m] = m < M ? A[r * lda + m] : 0.f;
      fma_row(ld4(B + r * ldb + 4 * cg), av);
    }
  }
  float* out = part + (int64_t)blockIdx.x * M * K;
#pragma unroll
  for (int m = 0; m < MV; ++m) {
    if (m < M) {  // uniform
      red[t] = acc[m];
      __syncthreads();
      if (t < T) {
        float4 s = red[t];
        for (int q = 1; q < P; ++q) s = add4(s, red[q * T + t]);
        st4(out + (int64_t)m * K + 4 * t, s);
      }
      __syncthreads();
    }
  }
}

// A^T B with M <= 16 always takes the skinny kernel, extras or not, so the product's bits do
// not depend on whether colsum(A) / V^T B are requested: V^T B is a second skinny product
// (nv <= 16) and colsum(A) = A^T 1 a third one against a broadcast row of ones (ldb = 0)
static bool skinny_ok(int M, int K, int nv) { return M <= 16 && K % 4 == 0 && K <= 1024 && nv <= 16; }
static int64_t skinny_blocks(int64_t N) {
  int64_t b = (N + 511) / 512;
  if (b > 2048) b = 2048;
  return b < 1 ? 1 : b;
}
static size_t skinny_ws(int64_t N, int K) {
  const int Kp = K < 4 ? 4 : K;
  return align_up((size_t)skinny_blocks(N) * 16 * Kp * 4) + align_up(16 + 16 * 4 * 4);
}

// ---- dW = A^T B ----
static int64_t gemm_splits(int64_t N, int M, int K) {
  const int64_t tiles = (int64_t)((M + kTN - 1) / kTN) * ((K + kTN - 1) / kTN);
  int64_t s = 512 / tiles;
  if (s < 1) s = 1;
  const int64_t max_s = (N + 255) / 256;  // >= 256 rows per split
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  return s;
}

size_t gemm_tn_workspace_bytes(int64_t N, int M, int K, int nv) {
  const int64_t s = gemm_splits(N, M, K);
  const size_t tiled = align_up((size_t)s * M * K * 4) + align_up((size_t)s * M * 4) +
                       align_up((size_t)s * (nv > 0 ? nv : 1) * K * 4);
  const size_t skinny = skinny_ok(M, K, nv) ? skinny_ws(N, K) : 0;
  return tiled > skinny ? tiled : skinny;
}

// out [M, K] = A^T B through k_tn_skinny + the ordered split reduction (part: workspace)
static hipError_t skinny_product(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t N, int M, int K,
                                 float* out, float* part, hipStream_t st) {
  int64_t blocks = skinny_blocks(N);
  const int64_t rpb = (N + blocks - 1) / blocks;
  blocks = (N + rpb - 1) / rpb;
  const int MV = M <= 1 ? 1 : M <= 2 ? 2 : M <= 4 ? 4 : M <= 8 ? 8 : 16;
#define PPGAT_SKINNY(MV_) \
  hipLaunchKernelGGL((k_tn_skinny<MV_>), dim3((unsigned)blocks), dim3(256), 0, st, A, lda, B, ldb, N, M, K, rpb, part)
  if (MV == 1) PPGAT_SKINNY(1); else if (MV == 2) PPGAT_SKINNY(2); else if (MV == 4) PPGAT_SKINNY(4);
  else if (MV == 8) PPGAT_SKINNY(8); else PPGAT_SKINNY(16);
#undef PPGAT_SKINNY
  SplitReduceArg ra{};
  const int64_t elems = (int64_t)M * K;
  ra.part[0] = part; ra.out[0] = out; ra.elems[0] = elems; ra.blocks[0] = (elems + 63) / 64;
  for (int q = 1; q < 3; ++q) { ra.part[q] = part; ra.out[q] = out; ra.elems[q] = 0; ra.blocks[q] = ra.blocks[0]; }
  hipLaunchKernelGGL(k_split_reduce, dim3((unsigned)ra.blocks[0]), dim3(1024), 0, st, ra, blocks);
  return hipGetLastError();
}

hipError_t gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t N, int M, int K, float* out,
                   float* colsum, const float* V, int64_t ldv, int nv, float* vout, void* ws, hipStream_t st) {
  if (M <= 0 || K <= 0) return hipSuccess;  // nothing to write (the ABI refuses these sizes; internal callers too)
  if (skinny_ok(M, K, (V && nv > 0) ? nv : 0) && N > 0) {
    // workspace: [split partials | ones float4 | colsum staging M x 4] (skinny_ws)
    char* p = static_cast<char*>(ws);
    float* part = reinterpret_cast<float*>(p);
    float* ones = reinterpret_cast<float*>(p + align_up((size_t)skinny_blocks(N) * 16 * K * 4));
    float* cs4 = ones + 4;
    hipError_t e = skinny_product(A, lda, B, ldb, N, M, K, out, part, st);
    if (e == hipSuccess && V && nv > 0) e = skinny_product(V, ldv, B, ldb, N, nv, K, vout, part, st);
    if (e == hipSuccess && colsum) {
      e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ones), 0x3f800000, 4, st);
      if (e == hipSuccess) e = skinny_product(A, lda, ones, 0, N, M, 4, cs4, part, st);
      if (e == hipSuccess)
        e = hipMemcpy2DAsync(colsum, sizeof(float), cs4, 4 * sizeof(float), sizeof(float), M, hipMemcpyDeviceToDevice, st);
    }
    return e;
  }
  const int64_t s = gemm_splits(N, M, K);
  const int64_t rows = ((N + s - 1) / s + kNB - 1) / kNB * kNB;
  char* p = static_cast<char*>(ws);
  float* part = reinterpret_cast<float*>(p);
  float* cpart = colsum ? reinterpret_cast<float*>(p + align_up((size_t)s * M * K * 4)) : nullptr;
  float* vpart = (V && nv > 0) ? reinterpret_cast<float*>(p + align_up((size_t)s * M * K * 4) +
                                                          align_up((size_t)s * M * 4))
                               : nullptr;
  const int tiles = ((M + kTN - 1) / kTN) * ((K + kTN - 1) / kTN);
  hipLaunchKernelGGL(k_gemm_tn, dim3((unsigned)tiles, (unsigned)s), dim3(256), 0, st, A, lda, B, ldb, N, M, K, rows,
                     part, cpart, vpart ? V : nullptr, ldv, vpart ? nv : 0, vpart);
  SplitReduceArg ra{};
  int na = 0;
  int64_t nb = 0;
  auto add = [&](const float* pp, float* o, int64_t elems) {
    ra.part[na] = pp;
    ra.out[na] = o;
    ra.elems[na] = elems;
    nb += (elems + 63) / 64;
    ra.blocks[na] = nb;
    ++na;
  };
  add(part, out, (int64_t)M * K);
  if (colsum) add(cpart, colsum, (int64_t)M);
  if (vpart) add(vpart, vout, (int64_t)nv * K);
  for (int q = na; q < 3; ++q) { ra.part[q] = ra.part[0]; ra.out[q] = ra.out[0]; ra.elems[q] = 0; ra.blocks[q] = nb; }
  hipLaunchKernelGGL(k_split_reduce, dim3((unsigned)nb), dim3(1024), 0, st, ra, s);
  return hipGetLastError();
}

}  // namespace ppgat
