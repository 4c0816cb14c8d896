// ppgat_infonce.hip -- the FusionMLP training step's contrastive loss and its backward on the
// device (embeddings/fuse_modal.py:39-72 contrastive_fusion_loss, trained by :179-214).
//
// Per batch of B rows (B <= 1024) with F = fused [B, D], T = txt_proj [B, D], I = img_proj [B, D]:
//   Fn = F / max(|F|, 1e-12)  (torch F.normalize), likewise Tn, In
//   S_t = Fn Tn^T / tau,  S_i = Fn In^T / tau                      [B, B]
//   loss_t = mean_b (logsumexp_c S_t[b, c] - S_t[b, b]),  loss_i likewise
//   loss = (loss_t + loss_i) / 2                        (F.cross_entropy with labels = arange)
// Backward with dS = (softmax(S) - onehot) / (2B):
//   dFn = (dS_t Tn + dS_i In) / tau,  dTn = dS_t^T Fn / tau,  dIn = dS_i^T Fn / tau
//   dx = (dy - y (y . dy)) / |x| for |x| > 1e-12, dy / 1e-12 otherwise   (normalize backward)
// The MLP around it (Linear 896 -> 256, ReLU, Dropout, Linear 256 -> 128; txt_proj, img_proj)
// runs on the matrix-core GEMMs (ppgat_gemm_nn / ppgat_gemm_tn); this file holds the small
// dense pieces: row norms, the two B x B similarity products (LDS-tiled fp32 FMA: 2 * 2 B^2 D
// = 134 MFLOP at B = 512, microseconds), the row-wise cross-entropy with its gradient, the
// transposed products of the backward, the dropout mask (counter hash, as ppgat_fwd) and ReLU.
// Every reduction has a fixed order: deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "ppgat_internal.h"
#include "ppgat_lanes.h"

namespace ppgat {
namespace {

constexpr int kD = 128;      // embedding width (output_dim)
constexpr float kNormEps = 1e-12f;

// y[r] = x[r] / max(|x[r]|, eps), nrm[r] = |x[r]|; one wave per row of one of three matrices
__global__ void __launch_bounds__(256) k_rownorm3(const float* __restrict__ x0, const float* __restrict__ x1,
                                                  const float* __restrict__ x2, int64_t B, float* __restrict__ y,
                                                  float* __restrict__ nrm) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= 3 * B) return;
  const int mtx = (int)(w / B);
  const int64_t r = w % B;
  const float* x = (mtx == 0 ? x0 : mtx == 1 ? x1 : x2) + r * kD;
  const float2 v = reinterpret_cast<const float2*>(x)[lane];
  const float s = wave_sum(fmaf(v.x, v.x, v.y * v.y));
  const float n = sqrtf(s);
  const float inv = 1.f / fmaxf(n, kNormEps);
  reinterpret_cast<float2*>(y + w * kD)[lane] = make_float2(v.x * inv, v.y * inv);
  if (lane == 0) nrm[w] = n;
}

// S1 = A B1^T * scale, S2 = A B2^T * scale for A, B1, B2 [B, kD]: 32 x 32 output tiles (B^2/1024
// workgroups: 256 at B = 512), 2 x 2 per thread per matrix, k staged through LDS in chunks of 32
__global__ void __launch_bounds__(256) k_sim2(const float* __restrict__ A, const float* __restrict__ B1,
                                              const float* __restrict__ B2, int64_t B, float scale,
                                              float* __restrict__ S1, float* __restrict__ S2) {
  __shared__ float sa[32][33], sb1[32][33], sb2[32][33];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  float acc1[2][2] = {}, acc2[2][2] = {};
  for (int k0 = 0; k0 < kD; k0 += 32) {
    for (int e = threadIdx.x; e < 32 * 32; e += 256) {
      const int rr = e >> 5, kk = e & 31;
      const int64_t ra = r0 + rr, rb = c0 + rr;
      sa[kk][rr] = ra < B ? A[ra * kD + k0 + kk] : 0.f;
      sb1[kk][rr] = rb < B ? B1[rb * kD + k0 + kk] : 0.f;
      sb2[kk][rr] = rb < B ? B2[rb * kD + k0 + kk] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < 32; ++kk) {
      const float a0 = sa[kk][ty], a1 = sa[kk][ty + 16];
      const float p0 = sb1[kk][tx], p1 = sb1[kk][tx + 16];
      const float q0 = sb2[kk][tx], q1 = sb2[kk][tx + 16];
      acc1[0][0] = fmaf(a0, p0, acc1[0][0]); acc1[0][1] = fmaf(a0, p1, acc1[0][1]);
      acc1[1][0] = fmaf(a1, p0, acc1[1][0]); acc1[1][1] = fmaf(a1, p1, acc1[1][1]);
      acc2[0][0] = fmaf(a0, q0, acc2[0][0]); acc2[0][1] = fmaf(a0, q1, acc2[0][1]);
      acc2[1][0] = fmaf(a1, q0, acc2[1][0]); acc2[1][1] = fmaf(a1, q1, acc2[1][1]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t r = r0 + ty + 16 * i, c = c0 + tx + 16 * j;
      if (r < B && c < B) {
        S1[r * B + c] = acc1[i][j] * scale;
        S2[r * B + c] = acc2[i][j] * scale;
      }
    }
}

// block reductions (256 threads, fixed order)
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// per row b and matrix m in {S1, S2}: l[m][b] = logsumexp_c S[b, c] - S[b, b] and
// dS[b, c] = (softmax(S[b])[c] - [c == b]) * gscale, written in place over S
__global__ void __launch_bounds__(256) k_ce_rows(float* __restrict__ S1, float* __restrict__ S2, int64_t B,
                                                 float gscale, float* __restrict__ l) {
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  float* S = (blockIdx.y == 0 ? S1 : S2) + b * B;
  float mx = -INFINITY;
  for (int64_t c = threadIdx.x; c < B; c += 256) mx = fmaxf(mx, S[c]);
  mx = block_max(mx, red);
  float se = 0.f;
  for (int64_t c = threadIdx.x; c < B; c += 256) se += expf(S[c] - mx);
  se = block_sum(se, red);
  const float lse = mx + logf(se);
  const float diag = S[b];
  __syncthreads();
  for (int64_t c = threadIdx.x; c < B; c += 256) S[c] = (expf(S[c] - lse) - (c == b ? 1.f : 0.f)) * gscale;
  if (threadIdx.x == 0) l[blockIdx.y * B + b] = lse - diag;
}

// loss = (mean l_t + mean l_i) / 2 -> out[0] = loss, out[1] = loss_t, out[2] = loss_i
__global__ void __launch_bounds__(256) k_ce_mean(const float* __restrict__ l, int64_t B, float* __restrict__ out) {
  __shared__ float red[4];
  float st = 0.f, si = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += 256) {
    st += l[b];
    si += l[B + b];
  }
  st = block_sum(st, red);
  si = block_sum(si, red);
  if (threadIdx.x == 0) {
    const float lt = st / (float)B, li = si / (float)B;
    out[0] = (lt + li) / 2.f;
    out[1] = lt;
    out[2] = li;
  }
}

// part[z][r, d] = sum_{k in split z} P(r, k) Q[k, d], P(r, k) = P[r * B + k] (TRANS 0) or
// P[k * B + r] (TRANS 1); P [B, B], Q [B, kD]; 16-row x 64-col output tiles, the reduction split
// over gridDim.z (kper each, a multiple of 32) so a 512-row batch fills the chip; 2 x 2 per
// thread, k staged through LDS in chunks of 32.  k_mm_sum adds the splits in order.
template <int TRANS>
__global__ void __launch_bounds__(256) k_mm_bd(const float* __restrict__ P, const float* __restrict__ Q, int64_t B,
                                               int64_t kper, float* __restrict__ part) {
  __shared__ float sp[32][17];
  __shared__ float sq[32][65];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // cols tx, tx + 32; rows ty, ty + 8
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  const int c0 = blockIdx.y * 64;
  const int64_t kb = (int64_t)blockIdx.z * kper;
  const int64_t ke = kb + kper < B ? kb + kper : B;
  float acc[2][2] = {};
  for (int64_t k0 = kb; k0 < ke; k0 += 32) {
    for (int e = threadIdx.x; e < 16 * 32; e += 256) {
      // consecutive threads along P's contiguous index: k for TRANS 0, r for TRANS 1
      const int rr = TRANS ? (e & 15) : (e >> 5), kk = TRANS ? (e >> 4) : (e & 31);
      const int64_t r = r0 + rr, k = k0 + kk;
      sp[kk][rr] = (r < B && k < ke) ? (TRANS ? P[k * B + r] : P[r * B + k]) : 0.f;
    }
    for (int e = threadIdx.x; e < 32 * 64; e += 256) {
      const int kk = e >> 6, d = e & 63;
      const int64_t k = k0 + kk;
      sq[kk][d] = k < ke ? Q[k * kD + c0 + d] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < 32; ++kk) {
      const float p0 = sp[kk][ty], p1 = sp[kk][ty + 8];
      const float q0 = sq[kk][tx], q1 = sq[kk][tx + 32];
      acc[0][0] = fmaf(p0, q0, acc[0][0]); acc[0][1] = fmaf(p0, q1, acc[0][1]);
      acc[1][0] = fmaf(p1, q0, acc[1][0]); acc[1][1] = fmaf(p1, q1, acc[1][1]);
    }
    __syncthreads();
  }
  float* out = part + (int64_t)blockIdx.z * B * kD;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int64_t r = r0 + ty + 8 * i;
    if (r >= B) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) out[r * kD + c0 + tx + 32 * j] = acc[i][j];
  }
}

// out[e] = scale * sum_{p < nparts} part[p][e]  (parts in order), float4 per thread
__global__ void __launch_bounds__(256) k_mm_sum(const float* __restrict__ part, int nparts, int64_t n4, float scale,
                                                float* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n4) return;
  float4 s = reinterpret_cast<const float4*>(part)[e];
  for (int p = 1; p < nparts; ++p) {
    const float4 v = reinterpret_cast<const float4*>(part)[(int64_t)p * n4 + e];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  reinterpret_cast<float4*>(out)[e] = make_float4(s.x * scale, s.y * scale, s.z * scale, s.w * scale);
}

// dx = (dy - y (y . dy)) / |x| (|x| > eps), dy / eps otherwise; one wave per row of the three
// matrices, in place (g_m holds dL/d(normalised m) on entry, dL/dm on exit)
__global__ void __launch_bounds__(256) k_norm_bwd3(const float* __restrict__ y, const float* __restrict__ nrm,
                                                   int64_t B, float* g0, float* g1, float* g2) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= 3 * B) return;
  const int mtx = (int)(w / B);
  float* g = (mtx == 0 ? g0 : mtx == 1 ? g1 : g2) + (w % B) * kD;
  const float2 yv = reinterpret_cast<const float2*>(y + w * kD)[lane];
  const float2 gv = reinterpret_cast<const float2*>(g)[lane];
  const float n = nrm[w];
  float2 o;
  if (n > kNormEps) {
    const float dot = wave_sum(fmaf(yv.x, gv.x, yv.y * gv.y));
    const float inv = 1.f / n;
    o = make_float2((gv.x - yv.x * dot) * inv, (gv.y - yv.y * dot) * inv);
  } else {
    o = make_float2(gv.x / kNormEps, gv.y / kNormEps);
  }
  reinterpret_cast<float2*>(g)[lane] = o;
}

__device__ __forceinline__ float drop_keep(uint64_t seed, uint64_t idx, float p, float inv_keep) {
  uint64_t x = seed ^ (idx * 0x9E3779B97F4A7C15ull);
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  const float u = (float)(x >> 40) * (1.0f / 16777216.0f);
  return u >= p ? inv_keep : 0.f;
}

// forward: a = relu(z) * mask (mask = 0 or 1/(1-p), counter hash of (seed, element));
// backward (dir 1): dz = dA * mask * [z > 0]   (in place over dA)
__global__ void __launch_bounds__(256) k_relu_drop(const float* __restrict__ z, int64_t n, float p, uint64_t seed,
                                                   int dir, float* __restrict__ a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const float inv_keep = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const float m = p > 0.f ? drop_keep(seed, (uint64_t)t, p, inv_keep) : 1.f;
  const float zv = z[t];
  if (dir == 0) a[t] = (zv > 0.f ? zv : 0.f) * m;
  else a[t] = zv > 0.f ? a[t] * m : 0.f;
}

}  // namespace

bool infonce_shape_ok(int64_t B, int D) { return B >= 1 && B <= 4096 && D == kD; }

// reduction splits of the B x B products: k ranges of >= 64 (two LDS chunks), at most 8
static int64_t mm_splits(int64_t B) {
  int64_t s = (B + 63) / 64;
  return s < 8 ? (s < 1 ? 1 : s) : 8;
}
static int64_t mm_kper(int64_t B) { return ((B + mm_splits(B) - 1) / mm_splits(B) + 31) / 32 * 32; }

size_t infonce_workspace_bytes(int64_t B) {
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  return al(3 * B * kD * 4) + al(3 * B * 4) + 2 * al(B * B * 4) + al(2 * B * 4) +
         al((size_t)4 * mm_splits(B) * B * kD * 4);
}

// loss[3] = {loss, loss_t, loss_i}; dF, dT, dI = gradients of loss w.r.t. F, T, I (pre-normalisation)
hipError_t infonce(const float* F, const float* T, const float* I, int64_t B, float tau, float* loss, float* dF,
                   float* dT, float* dI, void* ws, hipStream_t st) {
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  char* p = static_cast<char*>(ws);
  float* Y = reinterpret_cast<float*>(p);                 // [3, B, D] normalised rows
  p += al(3 * B * kD * 4);
  float* nrm = reinterpret_cast<float*>(p);               // [3, B]
  p += al(3 * B * 4);
  float* S1 = reinterpret_cast<float*>(p);
  p += al(B * B * 4);
  float* S2 = reinterpret_cast<float*>(p);
  p += al(B * B * 4);
  float* l = reinterpret_cast<float*>(p);                 // [2, B]
  p += al(2 * B * 4);
  float* part = reinterpret_cast<float*>(p);              // [4 products][splits][B, D]
  const float* Fn = Y;
  const float* Tn = Y + B * kD;
  const float* In = Y + 2 * B * kD;
  const unsigned w3 = (unsigned)((3 * B + 3) / 4);
  hipLaunchKernelGGL(k_rownorm3, dim3(w3), dim3(256), 0, st, F, T, I, B, Y, nrm);
  const unsigned t32 = (unsigned)((B + 31) / 32);
  hipLaunchKernelGGL(k_sim2, dim3(t32, t32), dim3(256), 0, st, Fn, Tn, In, B, 1.f / tau, S1, S2);
  hipLaunchKernelGGL(k_ce_rows, dim3((unsigned)B, 2), dim3(256), 0, st, S1, S2, B, 1.f / (2.f * (float)B), l);
  hipLaunchKernelGGL(k_ce_mean, dim3(1), dim3(256), 0, st, l, B, loss);
  // dFn = (dS_t Tn + dS_i In) / tau; dTn = dS_t^T Fn / tau; dIn = dS_i^T Fn / tau  (into dF, dT, dI)
  const float s = 1.f / tau;
  const int64_t ns = mm_splits(B), kper = mm_kper(B);
  const int64_t nz = (B + kper - 1) / kper;  // non-empty splits
  const size_t pstride = (size_t)ns * B * kD;
  const dim3 gm((unsigned)((B + 15) / 16), kD / 64, (unsigned)nz);
  hipLaunchKernelGGL(k_mm_bd<0>, gm, dim3(256), 0, st, S1, Tn, B, kper, part);
  hipLaunchKernelGGL(k_mm_bd<0>, gm, dim3(256), 0, st, S2, In, B, kper, part + (size_t)nz * B * kD);
  hipLaunchKernelGGL(k_mm_bd<1>, gm, dim3(256), 0, st, S1, Fn, B, kper, part + 2 * pstride);
  hipLaunchKernelGGL(k_mm_bd<1>, gm, dim3(256), 0, st, S2, Fn, B, kper, part + 3 * pstride);
  const int64_t n4 = B * kD / 4;
  const unsigned g4 = (unsigned)((n4 + 255) / 256);
  hipLaunchKernelGGL(k_mm_sum, dim3(g4), dim3(256), 0, st, part, (int)(2 * nz), n4, s, dF);  // S1 Tn + S2 In
  hipLaunchKernelGGL(k_mm_sum, dim3(g4), dim3(256), 0, st, part + 2 * pstride, (int)nz, n4, s, dT);
  hipLaunchKernelGGL(k_mm_sum, dim3(g4), dim3(256), 0, st, part + 3 * pstride, (int)nz, n4, s, dI);
  // normalisation backward, in place
  hipLaunchKernelGGL(k_norm_bwd3, dim3(w3), dim3(256), 0, st, Y, nrm, B, dF, dT, dI);
  return hipGetLastError();
}

hipError_t relu_dropout(const float* z, int64_t n, float p, uint64_t seed, int backward, float* a, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_relu_drop, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, z, n, p, seed, backward, a);
  return hipGetLastError();
}

}  // namespace ppgat
