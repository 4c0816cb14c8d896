// ppgat_fusion.hip -- FusionMLP inference on the matrix cores (the north
// star's MFMA target): embeddings/fuse_modal.py:18-36 + :220-244
//
//   x_b   = [txt_b | img_b]            img_b = img[img_index[b]] or img_fallback (mean image)
//   h_b   = relu(x_b W1^T + b1)        W1 [H1, Dt+Di]
//   y_b   = h_b W2^T + b2              W2 [Do, H1]
//   out_b = y_b / (||y_b|| + 1e-8)     (normalize != 0)
//
// fp32 in, fp32 out, v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains, no reduced precision, so
// the result matches the fp32 reference to accumulation-order rounding).
//
// One 256-thread workgroup = 128 rows, wave w owns rows [32 w, 32 w + 32) end to end:
//  GEMM1  x streams from HBM straight into MFMA operands (lane (r, hf) holds x[row r][k0 + 8 g
//         + 4 hf .. + 3] as a float4: the reduction index is permuted identically on both
//         operands), next chunk's x and W1 in flight while the current chunk's MFMAs run;
//         W1 chunks (256 x 32) staged in LDS as [n][k] with row stride 36 (b128 reads, no bank
//         conflicts); the wave's 32 x 256 pre-activation lives in 8 accumulator tiles.  The
//         cat() and the per-row image copy loop of the reference become the row pointers.
//  GEMM2  per 64 hidden columns: bias + ReLU, the wave's h slice transposed through its own LDS
//         patch into the A-operand layout, W2's 128 x 64 slice staged once per workgroup, 4 x 4
//         x 8 MFMAs into the 32 x 128 output tiles.
//  norm   row sums of squares reduced inside the wave (DPP over the 32 column lanes).
// LDS: max(W1 stage 36.9 KB, h patches 34.8 KB + W2 slice 34.8 KB) = 69.6 KB -> two
// workgroups per CU (8 waves); 4 waves x 32 rows amortise each W1 chunk over 128 rows.
// Shapes: H1 == 256, Do == 128, Dt % 32 == 0, Di % 32 == 0 (the reference's
// 384 + 512 -> 256 -> 128).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "ppgat_internal.h"
#include "ppgat_lanes.h"
#include "ppgat_split.h"
#include "ppgat_nnh_pipe.h"

namespace ppgat {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int BM = 128, BK = 32, H1 = 256, DO = 128;
constexpr int LW1 = BK + 4;   // W1 stage row stride ([n][k] image)
constexpr int HC = 64;        // hidden columns per GEMM2 step
constexpr int LH = HC + 4;    // h patch / W2 slice row stride
constexpr int kW1Floats = H1 * LW1;
constexpr int kG2Floats = 4 * 32 * LH + DO * LH;
constexpr int kLdsFloats = kW1Floats > kG2Floats ? kW1Floats : kG2Floats;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float comp(const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; }
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int row_of(int q, int hf) { return (q & 3) + 8 * (q >> 2) + 4 * hf; }

__global__ void __launch_bounds__(256, 2) k_fusion_fwd(const float* __restrict__ txt, const float* __restrict__ img,
                                                       const int32_t* __restrict__ img_index,
                                                       const float* __restrict__ img_fallback, int64_t B, int Dt,
                                                       int Di, const float* __restrict__ W1,
                                                       const float* __restrict__ b1, const float* __restrict__ W2,
                                                       const float* __restrict__ b2, int normalize,
                                                       float* __restrict__ out, float* __restrict__ z1_out) {
  __shared__ __attribute__((aligned(16))) float lds[kLdsFloats];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * BM + 32 * w;
  const int K = Dt + Di;
  // this lane's x row (rows past B re-read row B - 1, never stored)
  const int64_t b = row0 + r < B ? row0 + r : B - 1;
  const float* trow = txt + b * Dt + 4 * hf;
  const float* irow;
  if (Di > 0) {
    const int32_t ii = img_index ? img_index[b] : (int32_t)b;
    irow = (ii >= 0 ? img + (int64_t)ii * Di : img_fallback) + 4 * hf;
  } else {
    irow = trow;
  }
  auto load_x = [&](int k0, float4 (&xv)[4]) {
    const float* src = k0 < Dt ? trow + k0 : irow + (k0 - Dt);
#pragma unroll
    for (int g = 0; g < 4; ++g) xv[g] = ld4(src + 8 * g);
  };
  float4 wst[8];
  auto load_w1 = [&](int k0) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int e = tid + 256 * s;
      const int n = e >> 3, k4 = (e & 7) * 4;
      wst[s] = ld4(W1 + (int64_t)n * K + k0 + k4);
    }
  };
  auto store_w1 = [&]() {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int e = tid + 256 * s;
      st4(&lds[(e >> 3) * LW1 + (e & 7) * 4], wst[s]);
    }
  };

  // ---- GEMM1: z[32 rows x 256] per wave ----
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  float4 xa[4], xn[4];
  load_x(0, xa);
  load_w1(0);
  store_w1();
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) {
      load_w1(k0 + BK);
      load_x(k0 + BK, xn);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float4 bv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) bv[t] = ld4(&lds[(32 * t + r) * LW1 + 8 * g + 4 * hf]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma(comp(xa[g], s), comp(bv[t], s), acc[t]);
    }
    __syncthreads();
    if (more) {
      store_w1();
#pragma unroll
      for (int g = 0; g < 4; ++g) xa[g] = xn[g];
    }
    __syncthreads();
  }

  // ---- GEMM2: out[32 rows x 128] per wave, over four 64-column slices of h ----
  float* hp = lds + w * 32 * LH;   // this wave's h patch [32 rows][LH]
  float* w2s = lds + 4 * 32 * LH;  // W2 slice [128][LH]
  f32x16 acc2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc2[u] = f32x16{};
#pragma unroll
  for (int c = 0; c < H1 / HC; ++c) {
    // bias + ReLU of accumulator tiles 2c, 2c + 1 -> the patch (and z for a training backward)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int col = HC * c + 32 * tt + r;
      const float bias = b1[col];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = row_of(q, hf);
        const float z = acc[2 * c + tt][q] + bias;
        hp[row * LH + 32 * tt + r] = fmaxf(z, 0.f);
        if (z1_out != nullptr && row0 + row < B) z1_out[(row0 + row) * H1 + col] = z;
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // W2[:, 64 c .. 64 c + 63]: 2048 float4, 8 per thread
      const int e = tid + 256 * s;
      const int j = e >> 4, k4 = (e & 15) * 4;
      st4(&w2s[j * LH + k4], ld4(W2 + (int64_t)j * H1 + HC * c + k4));
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < HC / 8; ++g) {
      const float4 av = ld4(&hp[r * LH + 8 * g + 4 * hf]);
      float4 bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) bv[u] = ld4(&w2s[(32 * u + r) * LH + 8 * g + 4 * hf]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc2[u] = mfma(comp(av, s), comp(bv[u], s), acc2[u]);
    }
    __syncthreads();
  }

  // ---- bias, row L2 norm (inside the wave), store ----
  float ss[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) ss[q] = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float bias2 = b2[32 * u + r];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc2[u][q] += bias2;
      ss[q] = fmaf(acc2[u][q], acc2[u][q], ss[q]);
    }
  }
  if (normalize) {
#pragma unroll
    for (int q = 0; q < 16; ++q) ss[q] = 1.f / (sqrtf(group_reduce<Op::Sum, 1, 16>(ss[q])) + 1e-8f);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t row = row0 + row_of(q, hf);
    if (row >= B) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) out[row * DO + 32 * u + r] = normalize ? acc2[u][q] * ss[q] : acc2[u][q];
  }
}


// ---------------------------------------------------------------------------
// The same MLP on the split bf16 matrix cores (ppgat_split.h: fp32 products as six bf16
// MFMAs of three-term splits, fp32 accumulation), same contract and row ownership.
//  GEMM1  v_mfma_f32_32x32x16_bf16, 32-deep k chunks = two MFMA steps u; lane half hf's
//         element j of step u is k = 16 u + 4 hf + (j & 3) + 8 (j >> 2), i.e. the float4 pair
//         xa[2u], xa[2u + 1] the lane streams from its x row; the W1 chunk is split once per
//         workgroup while staged: three bf16 images [n][kk] (80-B rows, conflict-free b128 reads).
//  GEMM2  per 32 hidden columns (one accumulator tile): bias + ReLU into the wave's fp32 patch,
//         W2's 128 x 32 slice staged split; the patch is read back as float4 pairs in the same
//         k order and split per lane.
// LDS 61.4 KB (GEMM1 images; GEMM2 reuses it: patches 18.4 KB + W2 images 30.7 KB) -> two
// workgroups per CU.
// ---------------------------------------------------------------------------
constexpr int XLD = BK + 8;                 // bf16 per image row
constexpr int XP1 = H1 * XLD;               // bf16 per W1 image part
constexpr int XP2 = DO * XLD;               // bf16 per W2 image part
constexpr int XLH = BK + 4;                 // fp32 patch row stride
constexpr int kXLdsBytes = 3 * XP1 * 2;

__device__ __forceinline__ int xkk(int q) { return 16 * (q >> 2) + 8 * (q & 1) + 4 * ((q >> 1) & 1); }
// staging group e (8 per image row: k groups q = e & 7) -> image row.  Rows n and n + 4 share
// each 16-lane ds_write_b64 group, 80 dwords apart (16 mod 32): conflict-free writes, and every
// 8 lanes still read one 128-B row segment from global memory.
__device__ __forceinline__ int xrow(int e) { return 8 * (e >> 6) + ((((e >> 3) & 1) << 2) | ((e >> 4) & 3)); }

// split 4 consecutive-k values of one image row into the three parts at kk position xkk(q)
__device__ __forceinline__ void put_split4(uint16_t* img, int part, int row, int q, const float4& f) {
  const float v[4] = {f.x, f.y, f.z, f.w};
  uint2 h, m, l;
  uint32_t* ph = &h.x;
  uint32_t* pm = &m.x;
  uint32_t* pl = &l.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const uint32_t hh = split::pk_bf16(v[2 * i], v[2 * i + 1]);
    const float e0 = v[2 * i] - split::bf_lo(hh), e1 = v[2 * i + 1] - split::bf_hi(hh);
    const uint32_t mm = split::pk_bf16(e0, e1);
    ph[i] = hh;
    pm[i] = mm;
    pl[i] = split::pk_bf16(e0 - split::bf_lo(mm), e1 - split::bf_hi(mm));
  }
  const int off = row * XLD + xkk(q);
  *reinterpret_cast<uint2*>(&img[off]) = h;
  *reinterpret_cast<uint2*>(&img[part + off]) = m;
  *reinterpret_cast<uint2*>(&img[2 * part + off]) = l;
}

__global__ void __launch_bounds__(256, 2) k_fusion_fwdx(const float* __restrict__ txt, const float* __restrict__ img,
                                                        const int32_t* __restrict__ img_index,
                                                        const float* __restrict__ img_fallback, int64_t B, int Dt,
                                                        int Di, const float* __restrict__ W1,
                                                        const float* __restrict__ b1, const float* __restrict__ W2,
                                                        const float* __restrict__ b2, int normalize,
                                                        float* __restrict__ out, float* __restrict__ z1_out) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[kXLdsBytes / 2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hf = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * BM + 32 * w;
  const int K = Dt + Di;
  const int64_t b = row0 + r < B ? row0 + r : B - 1;
  const float* trow = txt + b * Dt + 4 * hf;
  const float* irow;
  if (Di > 0) {
    const int32_t ii = img_index ? img_index[b] : (int32_t)b;
    irow = (ii >= 0 ? img + (int64_t)ii * Di : img_fallback) + 4 * hf;
  } else {
    irow = trow;
  }
  auto load_x = [&](int k0, float4 (&xv)[4]) {
    const float* src = k0 < Dt ? trow + k0 : irow + (k0 - Dt);
#pragma unroll
    for (int g = 0; g < 4; ++g) xv[g] = ld4(src + 8 * g);
  };
  float4 wst[8];  // W1 chunk: group e = tid + 256 s -> row xrow(e), k group q = e & 7
  auto load_w1 = [&](int k0) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int e = tid + 256 * s;
      wst[s] = ld4(W1 + (int64_t)xrow(e) * K + k0 + (e & 7) * 4);
    }
  };
  auto store_w1 = [&]() {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int e = tid + 256 * s;
      put_split4(lds, XP1, xrow(e), e & 7, wst[s]);
    }
  };

  // ---- GEMM1 ----
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  float4 xa[4], xn[4];
  load_x(0, xa);
  load_w1(0);
  store_w1();
  __syncthreads();
  for (int k0 = 0; k0 < K; k0 += BK) {
    const bool more = k0 + BK < K;
    if (more) {
      load_w1(k0 + BK);
      load_x(k0 + BK, xn);
    }
    // (u, t) steps; the next step's W1 units are read while this step's six MFMAs run
    auto read_w = [&](int idx, split::u32x4 (&f)[3]) {
      const int off = (32 * (idx & 7) + r) * XLD + 16 * (idx >> 3) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&lds[p * XP1 + off]);
    };
    // two fragment sets used alternately; each step issues the next step's three LDS reads
    // before its six MFMAs (see k_gemm_nnp)
    split::u32x4 fx[3], fb[2][3];
    read_w(0, fb[0]);
#pragma unroll
    for (int idx = 0; idx < 16; ++idx) {
      const int u = idx >> 3, t = idx & 7;
      if (t == 0) split::split3(xa[2 * u], xa[2 * u + 1], fx[0], fx[1], fx[2]);
      if (idx + 1 < 16) read_w(idx + 1, fb[(idx + 1) & 1]);
      acc[t] = split::mfma32_x6(fx, fb[idx & 1], acc[t]);
      if (idx + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x0100, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 6, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    if (more) {
      store_w1();
#pragma unroll
      for (int g = 0; g < 4; ++g) xa[g] = xn[g];
    }
    __syncthreads();
  }

  // ---- GEMM2 over eight 32-column slices of h ----
  float* hp = reinterpret_cast<float*>(lds) + w * 32 * XLH;     // this wave's patch [32][XLH]
  uint16_t* w2i = lds + (4 * 32 * XLH * 4) / 2;                 // W2 slice images [3][128][XLD]
  f32x16 acc2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc2[u] = f32x16{};
#pragma unroll
  for (int c = 0; c < H1 / BK; ++c) {
    const int col = BK * c + r;
    const float bias = b1[col];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = row_of(q, hf);
      const float z = acc[c][q] + bias;
      hp[row * XLH + r] = fmaxf(z, 0.f);
      if (z1_out != nullptr && row0 + row < B) z1_out[(row0 + row) * H1 + col] = z;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {  // W2[:, 32 c .. 32 c + 31]: 1024 groups of 4 k, 4 per thread
      const int e = tid + 256 * s;
      put_split4(w2i, XP2, xrow(e), e & 7, ld4(W2 + (int64_t)xrow(e) * H1 + BK * c + (e & 7) * 4));
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      split::u32x4 fh[3];
      split::split3(ld4(&hp[r * XLH + 16 * u + 4 * hf]), ld4(&hp[r * XLH + 16 * u + 8 + 4 * hf]), fh[0], fh[1],
                    fh[2]);
#pragma unroll
      for (int uu = 0; uu < 4; ++uu) {
        const int off = (32 * uu + r) * XLD + 16 * u + 8 * hf;
        split::u32x4 fb[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) fb[p] = *reinterpret_cast<const split::u32x4*>(&w2i[p * XP2 + off]);
        acc2[uu] = split::mfma32_x6(fh, fb, acc2[uu]);
      }
    }
    __syncthreads();
  }

  // ---- bias, row L2 norm (inside the wave), store ----
  float ss[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) ss[q] = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float bias2 = b2[32 * u + r];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc2[u][q] += bias2;
      ss[q] = fmaf(acc2[u][q], acc2[u][q], ss[q]);
    }
  }
  if (normalize) {
#pragma unroll
    for (int q = 0; q < 16; ++q) ss[q] = 1.f / (sqrtf(group_reduce<Op::Sum, 1, 16>(ss[q])) + 1e-8f);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t row = row0 + row_of(q, hf);
    if (row >= B) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) out[row * DO + 32 * u + r] = normalize ? acc2[u][q] * ss[q] : acc2[u][q];
  }
}

// ---------------------------------------------------------------------------
// The same MLP with W1 and W2 pre-split once per call (ppgat::nnx_presplit: the three bf16
// images per 32-deep chunk in exactly the layout k_fusion_fwdx builds in LDS, so the products
// and results are bitwise those of k_fusion_fwdx) and staged by global_load_lds_dwordx4:
// 8 waves = 256 rows per workgroup share every staged chunk, two LDS buffers, one barrier
// per chunk.  k_fusion_fwdx splits each chunk while staging it (VALU beside the MFMAs) and
// waits at two barriers per chunk (PMC: MFMA busy 0.51, profiles/r02/v15_fusion_fwdx_pmc.json).
// LDS: GEMM1 2 x 61,440 B; GEMM2 reuses it: 8 wave patches (36,864 B) + 2 x 30,720 B W2 slices.
// ---------------------------------------------------------------------------
constexpr int PBM = 256;                       // rows per k_fusion_fwdp workgroup
constexpr int kW1Img = 3 * XP1;                // bf16 per W1 chunk image
constexpr int kW2Img = 3 * XP2;                // bf16 per W2 slice image
constexpr int kPatchB = 8 * 32 * XLH * 4;      // bytes of the 8 wave patches

// buffer_load ... lds (MUBUF LDS-DMA, tracked on vmcnt only): with global_load_lds the compiler
// turned every LDS-read wait behind it into lgkmcnt(0), so no fragment read overlapped an MFMA
__device__ __forceinline__ void glds_copy(const uint16_t* src, uint16_t* dst, int bytes, int wv, int lane) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(src), 0, bytes, 0x00020000);
  char* d = reinterpret_cast<char*>(dst);
  for (int i = wv; i < bytes / 1024; i += 8)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(d + i * 1024), 16,
                                             lane * 16 + i * 1024, 0, 0, 0);
}

#ifdef PPGAT_LAB_BUILD  // superseded by k_fusion_fwdh3 (lab builds only)
__global__ void __launch_bounds__(512, 1) k_fusion_fwdp(const float* __restrict__ txt, const float* __restrict__ img,
                                                        const int32_t* __restrict__ img_index,
                                                        const float* __restrict__ img_fallback, int64_t B, int Dt,
                                                        int Di, const uint16_t* __restrict__ w1i,
                                                        const float* __restrict__ b1, const uint16_t* __restrict__ w2i_g,
                                                        const float* __restrict__ b2, int normalize,
                                                        float* __restrict__ out, float* __restrict__ z1_out) {
  static_assert(kW1Img * 2 % 1024 == 0 && kW2Img * 2 % 1024 == 0, "1-KB wave copies");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * kW1Img];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * PBM + 32 * w;
  const int K = Dt + Di, chunks = K / BK;
  const int64_t b = row0 + r < B ? row0 + r : B - 1;
  const float* trow = txt + b * Dt + 4 * hf;
  const float* irow;
  if (Di > 0) {
    const int32_t ii = img_index ? img_index[b] : (int32_t)b;
    irow = (ii >= 0 ? img + (int64_t)ii * Di : img_fallback) + 4 * hf;
  } else {
    irow = trow;
  }
  auto load_x = [&](int k0, float4 (&xv)[4]) {
    const float* src = k0 < Dt ? trow + k0 : irow + (k0 - Dt);
#pragma unroll
    for (int g = 0; g < 4; ++g) xv[g] = ld4(src + 8 * g);
  };

  // ---- GEMM1 ----
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  float4 xa[4], xn[4];
  load_x(0, xa);
  glds_copy(w1i, lds, kW1Img * 2, w, lane);
  __syncthreads();  // vmcnt(0): chunk 0 and the first x fragments have landed
  for (int c = 0; c < chunks; ++c) {
    const uint16_t* sb = lds + (c & 1) * kW1Img;
    const bool more = c + 1 < chunks;
    if (more) {
      glds_copy(w1i + (int64_t)(c + 1) * kW1Img, lds + ((c + 1) & 1) * kW1Img, kW1Img * 2, w, lane);
      load_x((c + 1) * BK, xn);
    }
    auto read_w = [&](int idx, split::u32x4 (&f)[3]) {
      const int off = (32 * (idx & 7) + r) * XLD + 16 * (idx >> 3) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&sb[p * XP1 + off]);
    };
    // two fragment sets used alternately; each step issues the next step's three LDS reads
    // before its six MFMAs (see k_gemm_nnp)
    split::u32x4 fx[3], fb[2][3];
    read_w(0, fb[0]);
#pragma unroll
    for (int idx = 0; idx < 16; ++idx) {
      const int u = idx >> 3, t = idx & 7;
      if (t == 0) split::split3(xa[2 * u], xa[2 * u + 1], fx[0], fx[1], fx[2]);
      if (idx + 1 < 16) read_w(idx + 1, fb[(idx + 1) & 1]);
      acc[t] = split::mfma32_x6(fx, fb[idx & 1], acc[t]);
      if (idx + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x0100, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 6, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // chunk c + 1 landed; every wave is done with this buffer
    if (more) {
#pragma unroll
      for (int g = 0; g < 4; ++g) xa[g] = xn[g];
    }
  }

  // ---- GEMM2 over eight 32-column slices of h (W2 slice images double-buffered after the patches) ----
  float* hp = reinterpret_cast<float*>(lds) + w * 32 * XLH;                   // this wave's patch [32][XLH]
  uint16_t* w2s = lds + kPatchB / 2;                                           // [2][3][128][XLD]
  f32x16 acc2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc2[u] = f32x16{};
  glds_copy(w2i_g, w2s, kW2Img * 2, w, lane);
#pragma unroll
  for (int c = 0; c < H1 / BK; ++c) {
    const int col = BK * c + r;
    const float bias = b1[col];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = row_of(q, hf);
      const float z = acc[c][q] + bias;
      hp[row * XLH + r] = fmaxf(z, 0.f);
      if (z1_out != nullptr && row0 + row < B) z1_out[(row0 + row) * H1 + col] = z;
    }
    __syncthreads();  // vmcnt(0): slice c landed; the patch is written
    if (c + 1 < H1 / BK) glds_copy(w2i_g + (int64_t)(c + 1) * kW2Img, w2s + ((c + 1) & 1) * kW2Img, kW2Img * 2, w, lane);
    const uint16_t* ws2 = w2s + (c & 1) * kW2Img;
    auto read_w2 = [&](int i, split::u32x4 (&f)[3]) {
      const int off = (32 * (i & 3) + r) * XLD + 16 * (i >> 2) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&ws2[p * XP2 + off]);
    };
    split::u32x4 fh[3], fb2[2][3];
    read_w2(0, fb2[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int u = i >> 2, uu = i & 3;
      if (uu == 0)
        split::split3(ld4(&hp[r * XLH + 16 * u + 4 * hf]), ld4(&hp[r * XLH + 16 * u + 8 + 4 * hf]), fh[0], fh[1],
                      fh[2]);
      if (i + 1 < 8) read_w2(i + 1, fb2[(i + 1) & 1]);
      acc2[uu] = split::mfma32_x6(fh, fb2[i & 1], acc2[uu]);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // the patch and this slice's buffer are free again
  }

  // ---- bias, row L2 norm (inside the wave), store ----
  float ss[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) ss[q] = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float bias2 = b2[32 * u + r];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc2[u][q] += bias2;
      ss[q] = fmaf(acc2[u][q], acc2[u][q], ss[q]);
    }
  }
  if (normalize) {
#pragma unroll
    for (int q = 0; q < 16; ++q) ss[q] = 1.f / (sqrtf(group_reduce<Op::Sum, 1, 16>(ss[q])) + 1e-8f);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t row = row0 + row_of(q, hf);
    if (row >= B) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) out[row * DO + 32 * u + r] = normalize ? acc2[u][q] * ss[q] : acc2[u][q];
  }
}


#endif  // PPGAT_LAB_BUILD

// ---------------------------------------------------------------------------
// The same MLP on the fp16 matrix cores: the scaled two-term split of ppgat_split.h, three
// MFMAs per product instead of six.  W1 and W2 are pre-split once per call with per-column
// power-of-two scales (ppgat::nnh_presplit: k_gemm_nnh's images, two parts of [n][40]); x rows
// are scaled online per row as they stream (split::row_scale_online, as k_gemm_nnh); the rows
// of h = relu(.) are scaled by their max over the 256 hidden columns before GEMM2.  Every scale
// is a power of two, so unscaling is exact.  Row ownership, LDS-DMA staging (8 waves x 32 rows
// share each chunk, two buffers, one barrier per chunk) and GEMM2's per-wave patch as
// k_fusion_fwdp.  LDS: GEMM1 2 x 40,960 B; GEMM2 reuses it: the 8 wave patches (36,864 B) +
// 2 x 20,480 B W2 slices.
// ---------------------------------------------------------------------------
constexpr int HLDK = 40;                 // fp16 per image row (NnhImg LDK)
constexpr int kH1Part = H1 * HLDK;       // fp16 per W1 image part
constexpr int kH1Img = 2 * kH1Part;      // per 32-deep W1 chunk (NnhImg<8>::ELEMS)
constexpr int kH2Part = DO * HLDK;
constexpr int kH2Img = 2 * kH2Part;      // per 32-deep W2 chunk (NnhImg<4>::ELEMS)

#ifdef PPGAT_LAB_BUILD  // superseded by k_fusion_fwdh3 (lab builds only; the bitwise reference of the lab test)
__global__ void __launch_bounds__(512, 1) k_fusion_fwdh(const float* __restrict__ txt, const float* __restrict__ img,
                                                        const int32_t* __restrict__ img_index,
                                                        const float* __restrict__ img_fallback, int64_t B, int Dt,
                                                        int Di, const uint16_t* __restrict__ w1i,
                                                        const int* __restrict__ e1, const float* __restrict__ b1,
                                                        const uint16_t* __restrict__ w2i_g, const int* __restrict__ e2,
                                                        const float* __restrict__ b2, int normalize,
                                                        float* __restrict__ out, float* __restrict__ z1_out) {
  static_assert(kH1Img * 2 % 1024 == 0 && kH2Img * 2 % 1024 == 0, "1-KB wave copies");
  static_assert(kPatchB + 2 * kH2Img * 2 <= 2 * kH1Img * 2, "GEMM2 fits GEMM1's LDS");
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * kH1Img];
  __shared__ __attribute__((aligned(16))) float sF[8][32];  // per wave: a factor per row
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * PBM + 32 * w;
  const int K = Dt + Di, chunks = K / BK;
  const int64_t b = row0 + r < B ? row0 + r : B - 1;
  const float* trow = txt + b * Dt + 4 * hf;
  const float* irow;
  if (Di > 0) {
    const int32_t ii = img_index ? img_index[b] : (int32_t)b;
    irow = (ii >= 0 ? img + (int64_t)ii * Di : img_fallback) + 4 * hf;
  } else {
    irow = trow;
  }
  auto load_x = [&](int k0, float4 (&xv)[4]) {
    const float* src = k0 < Dt ? trow + k0 : irow + (k0 - Dt);
#pragma unroll
    for (int g = 0; g < 4; ++g) xv[g] = ld4(src + 8 * g);
  };

  // ---- GEMM1: rows scaled online, W1 columns by their pre-split scales ----
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  float4 xa[4], xn[4];
  int erow = 0;
  bool set = false;
  load_x(0, xa);
  glds_copy(w1i, lds, kH1Img * 2, w, lane);
  __syncthreads();  // vmcnt(0): chunk 0 and the first x fragments have landed
  for (int c = 0; c < chunks; ++c) {
    const uint16_t* sb = lds + (c & 1) * kH1Img;
    const bool more = c + 1 < chunks;
    if (more) {
      glds_copy(w1i + (int64_t)(c + 1) * kH1Img, lds + ((c + 1) & 1) * kH1Img, kH1Img * 2, w, lane);
      load_x((c + 1) * BK, xn);
    }
    const float s = split::row_scale_online<8>(xa, erow, set, acc, sF[w], r, hf);
    auto read_w = [&](int idx, split::u32x4 (&f)[2]) {
      const int off = (32 * (idx & 7) + r) * HLDK + 16 * (idx >> 3) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&sb[p * kH1Part + off]);
    };
    split::u32x4 fx[2], fb[2][2];
    read_w(0, fb[0]);
#pragma unroll
    for (int idx = 0; idx < 16; ++idx) {
      const int u = idx >> 3, t = idx & 7;
      if (t == 0) split::split2h(xa[2 * u], xa[2 * u + 1], s, fx[0], fx[1]);
      if (idx + 1 < 16) read_w(idx + 1, fb[(idx + 1) & 1]);
      acc[t] = split::mfma32_h3(fx, fb[idx & 1], acc[t]);
      if (idx + 1 < 16) __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 3, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // chunk c + 1 landed; every wave is done with this buffer
    if (more) {
#pragma unroll
      for (int g = 0; g < 4; ++g) xa[g] = xn[g];
    }
  }

  // ---- h = relu(z), z = acc / (s_row s_col) + b1 (exact unscale); h's row maxima ----
  float fr[16];
  split::row_unscale(erow, sF[w], r, hf, fr);
  float hm[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) hm[q] = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int col = BK * t + r;
    const float fc = ldexpf(1.f, -e1[col]), bias = b1[col];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float z = fmaf(acc[t][q] * fr[q], fc, bias);
      const int row = row_of(q, hf);
      if (z1_out != nullptr && row0 + row < B) z1_out[(row0 + row) * H1 + col] = z;
      const float h = fmaxf(z, 0.f);
      acc[t][q] = h;
      hm[q] = fmaxf(hm[q], h);
    }
  }
  float fr2[16];  // 1 / s_h of this lane's accumulator rows (GEMM2 epilogue)
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float m = group_reduce<Op::Max, 1, 16>(hm[q]);
    const int e = (m > 0.f && m <= 3.4e38f) ? split::scale_exp16(m) : 0;
    fr2[q] = ldexpf(1.f, -e);
    if (r == q) sF[w][row_of(q, hf)] = ldexpf(1.f, e);  // s_h for the A-operand lanes
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float sh = sF[w][r];  // this lane's GEMM2 A-operand row is row r

  // ---- GEMM2 over eight 32-column slices of h ----
  float* hp = reinterpret_cast<float*>(lds) + w * 32 * XLH;   // this wave's patch [32][XLH]
  uint16_t* w2s = lds + kPatchB / 2;                           // [2][kH2Img]
  f32x16 acc2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc2[u] = f32x16{};
  glds_copy(w2i_g, w2s, kH2Img * 2, w, lane);
#pragma unroll
  for (int c = 0; c < H1 / BK; ++c) {
#pragma unroll
    for (int q = 0; q < 16; ++q) hp[row_of(q, hf) * XLH + r] = acc[c][q];
    __syncthreads();  // vmcnt(0): slice c landed; the patch is written
    if (c + 1 < H1 / BK) glds_copy(w2i_g + (int64_t)(c + 1) * kH2Img, w2s + ((c + 1) & 1) * kH2Img, kH2Img * 2, w, lane);
    const uint16_t* ws2 = w2s + (c & 1) * kH2Img;
    auto read_w2 = [&](int i, split::u32x4 (&f)[2]) {
      const int off = (32 * (i & 3) + r) * HLDK + 16 * (i >> 2) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&ws2[p * kH2Part + off]);
    };
    split::u32x4 fh[2], fb2[2][2];
    read_w2(0, fb2[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int u = i >> 2, uu = i & 3;
      if (uu == 0) split::split2h(ld4(&hp[r * XLH + 16 * u + 4 * hf]), ld4(&hp[r * XLH + 16 * u + 8 + 4 * hf]), sh, fh[0], fh[1]);
      if (i + 1 < 8) read_w2(i + 1, fb2[(i + 1) & 1]);
      acc2[uu] = split::mfma32_h3(fh, fb2[i & 1], acc2[uu]);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // the patch and this slice's buffer are free again
  }

  // ---- unscale, bias, row L2 norm (inside the wave), store ----
  float ss[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) ss[q] = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int col = 32 * u + r;
    const float fc = ldexpf(1.f, -e2[col]), bias2 = b2[col];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc2[u][q] = fmaf(acc2[u][q] * fr2[q], fc, bias2);
      ss[q] = fmaf(acc2[u][q], acc2[u][q], ss[q]);
    }
  }
  if (normalize) {
#pragma unroll
    for (int q = 0; q < 16; ++q) ss[q] = 1.f / (sqrtf(group_reduce<Op::Sum, 1, 16>(ss[q])) + 1e-8f);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t row = row0 + row_of(q, hf);
    if (row >= B) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) out[row * DO + 32 * u + r] = normalize ? acc2[u][q] * ss[q] : acc2[u][q];
  }
}

#endif  // PPGAT_LAB_BUILD

// ---------------------------------------------------------------------------
// k_fusion_fwdh with GEMM1 on the pipelined loop of k_gemm_nnh3 (ppgat_nnh_pipe.h: W1 chunks by
// LDS-DMA into three buffers two chunks ahead, x two chunks ahead, the next chunk's row scale
// and fp16 split inside the current chunk's MFMA sequence, one bare barrier per chunk) -- the
// same products in the same order (bitwise equal outputs).  Even chunk counts (the reference's
// 384 + 512 = 28 chunks); LDS 3 x 40,960 B.
// GEMM2 (round 5): k_fusion_fwdh waited for every 20-KB W2 slice at a __syncthreads (vmcnt(0))
// right after issuing it, eight exposed L2 round trips per workgroup.  Here the four first slices
// go out by LDS-DMA the moment GEMM1's loop has released its buffers, into four buffers beside the
// wave patches, and slice c + 4 follows as soon as every wave is done with slice c; each slice
// waits only for its own DMA (exact per-wave vmcnt counts); b1 / e1 / b2 / e2 are staged in LDS
// by LDS-DMA ahead of GEMM1, so the h epilogue issues no global load behind the W2 DMAs.
// ---------------------------------------------------------------------------
constexpr int kH2Bytes = kH2Img * 2;           // one 32-deep W2 slice image
constexpr int kH2Pieces = kH2Bytes / 1024;     // 1-KB wave copies per slice (20)

template <int K>
__device__ __forceinline__ void wait_w2(bool full) {  // this wave's DMA of K later slices may stay in flight
  constexpr int F = (kH2Pieces + 7) / 8, P = kH2Pieces / 8;
  if (full) wait_vm<K * F>();
  else wait_vm<K * P>();
}

__device__ __forceinline__ i32x4 raw_rsrc(const void* p, uint32_t bytes) {
  const uint64_t base = reinterpret_cast<uint64_t>(p);
  return {__builtin_amdgcn_readfirstlane((int)(uint32_t)base), __builtin_amdgcn_readfirstlane((int)((base >> 32) & 0xffff)),
          __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}

__global__ void __launch_bounds__(512, 1) k_fusion_fwdh3(const float* __restrict__ txt, const float* __restrict__ img,
                                                        const int32_t* __restrict__ img_index,
                                                        const float* __restrict__ img_fallback, int64_t B, int Dt,
                                                        int Di, const uint16_t* __restrict__ w1i,
                                                        const int* __restrict__ e1, const float* __restrict__ b1,
                                                        const uint16_t* __restrict__ w2i_g, const int* __restrict__ e2,
                                                        const float* __restrict__ b2, int normalize,
                                                        float* __restrict__ out, float* __restrict__ z1_out) {
  static_assert(kH1Img * 2 % 1024 == 0 && kH2Bytes % 1024 == 0, "1-KB wave copies");
  static_assert(kPatchB % 1024 == 0 && kPatchB + 4 * kH2Bytes <= 3 * kH1Img * 2, "GEMM2 fits GEMM1's LDS");
  static_assert(kH1Img == NnhImg<8>::ELEMS, "W1 chunks are k_gemm_nnh's 256-column images");
  static_assert(H1 == 256 && DO == 128 && H1 / BK == 8, "staged parameter rows: 1 KB (H1) / 512 B (DO)");
  __shared__ __attribute__((aligned(16))) uint16_t lds[3 * kH1Img];
  __shared__ __attribute__((aligned(16))) float sF[8][32];  // per wave: a factor per row
  __shared__ __attribute__((aligned(16))) float sPar[4][256];  // b1 | e1 (int bits) | b2 | e2 (int bits)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hf = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * PBM + 32 * w;
  const int K = Dt + Di, chunks = K / BK;
  const int64_t b = row0 + r < B ? row0 + r : B - 1;
  const float* trow = txt + b * Dt + 4 * hf;
  const float* irow;
  if (Di > 0) {
    const int32_t ii = img_index ? img_index[b] : (int32_t)b;
    irow = (ii >= 0 ? img + (int64_t)ii * Di : img_fallback) + 4 * hf;
  } else {
    irow = trow;
  }
  auto load_x_chunk = [&](int c, float4 (&xv)[4]) {  // a chunk never straddles txt | img (Dt % 32 == 0)
    const int k0 = c * BK;
    const float* src = k0 < Dt ? trow + k0 : irow + (k0 - Dt);
#pragma unroll
    for (int g = 0; g < 4; ++g) xv[g] = ld4(src + 8 * g);
  };
  const uint32_t voff = (uint32_t)lane * 16u;
  // b1, e1, b2, e2 -> sPar by LDS-DMA (one wave each; older than GEMM1's first DMA, so the loop's
  // first wait covers them, and its barriers publish them; lanes past a 512-B row read zeros)
  if (w < 4) {
    const void* src = w == 0 ? (const void*)b1 : w == 1 ? (const void*)e1 : w == 2 ? (const void*)b2 : (const void*)e2;
    dma_lds16(raw_rsrc(src, w < 2 ? 4 * H1 : 4 * DO), (uint32_t)reinterpret_cast<uintptr_t>(&sPar[w][0]), voff, 0);
  }

  // ---- GEMM1: the pipelined fp16 two-term loop (ppgat_nnh_pipe.h), rows scaled online ----
  f32x16 acc[8];
  int erow = 0;
  nnh3_loop<8>(w1i, lds, chunks, load_x_chunk, acc, erow, sF[w], w, lane);

  // ---- W2 slices 0..3 -> buffers 0..3 beside the patches (the loop ended on a barrier after
  // every wave's last reads of its buffers) ----
  const uint32_t w2l = (uint32_t)reinterpret_cast<uintptr_t>(lds) + (uint32_t)kPatchB;
  const i32x4 rs2 = raw_rsrc(w2i_g, (uint32_t)(H1 / BK) * kH2Bytes);
  const bool full2 = (kH2Pieces % 8 == 0) || w < kH2Pieces % 8;
  auto issue2 = [&](int c) {
    const uint32_t dst = w2l + (uint32_t)((c & 3) * kH2Bytes);
    for (int i = w; i < kH2Pieces; i += 8) dma_lds16(rs2, dst + i * 1024, voff, (uint32_t)(c * kH2Bytes + i * 1024));
  };
#pragma unroll
  for (int c = 0; c < 4; ++c) issue2(c);

  // ---- h = relu(z), z = acc / (s_row s_col) + b1 (exact unscale); h's row maxima ----
  float fr[16];
  split::row_unscale(erow, sF[w], r, hf, fr);
  float hm[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) hm[q] = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int col = BK * t + r;
    const float fc = ldexpf(1.f, -__float_as_int(sPar[1][col])), bias = sPar[0][col];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float z = fmaf(acc[t][q] * fr[q], fc, bias);
      const int row = row_of(q, hf);
      if (z1_out != nullptr && row0 + row < B) z1_out[(row0 + row) * H1 + col] = z;
      const float h = fmaxf(z, 0.f);
      acc[t][q] = h;
      hm[q] = fmaxf(hm[q], h);
    }
  }
  if (z1_out != nullptr) wait_vm<0>();  // training forward: stores share the counter; keep the slice counts exact
  float fr2[16];  // 1 / s_h of this lane's accumulator rows (GEMM2 epilogue)
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float m = group_reduce<Op::Max, 1, 16>(hm[q]);
    const int e = (m > 0.f && m <= 3.4e38f) ? split::scale_exp16(m) : 0;
    fr2[q] = ldexpf(1.f, -e);
    if (r == q) sF[w][row_of(q, hf)] = ldexpf(1.f, e);  // s_h for the A-operand lanes
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float sh = sF[w][r];  // this lane's GEMM2 A-operand row is row r

  // ---- GEMM2 over eight 32-column slices of h ----
  float* hp = reinterpret_cast<float*>(lds) + w * 32 * XLH;   // this wave's patch [32][XLH]
  const uint16_t* w2s = lds + kPatchB / 2;                     // [4][kH2Img]
  f32x16 acc2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc2[u] = f32x16{};
#pragma unroll
  for (int c = 0; c < H1 / BK; ++c) {
#pragma unroll
    for (int q = 0; q < 16; ++q) hp[row_of(q, hf) * XLH + r] = acc[c][q];  // own patch: in-order LDS
    // slice c has landed: this wave's DMAs of up to three later slices may still be in flight
    if (c <= 4) wait_w2<3>(full2);
    else if (c == 5) wait_w2<2>(full2);
    else if (c == 6) wait_w2<1>(full2);
    else wait_w2<0>(full2);
    __builtin_amdgcn_s_barrier();  // every wave's part of slice c
    const uint16_t* ws2 = w2s + (c & 3) * kH2Img;
    auto read_w2 = [&](int i, split::u32x4 (&f)[2]) {
      const int off = (32 * (i & 3) + r) * HLDK + 16 * (i >> 2) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&ws2[p * kH2Part + off]);
    };
    split::u32x4 fh[2], fb2[2][2];
    read_w2(0, fb2[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int u = i >> 2, uu = i & 3;
      if (uu == 0) split::split2h(ld4(&hp[r * XLH + 16 * u + 4 * hf]), ld4(&hp[r * XLH + 16 * u + 8 + 4 * hf]), sh, fh[0], fh[1]);
      if (i + 1 < 8) read_w2(i + 1, fb2[(i + 1) & 1]);
      acc2[uu] = split::mfma32_h3(fh, fb2[i & 1], acc2[uu]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c + 4 < H1 / BK) {
      __builtin_amdgcn_s_barrier();  // every wave is done with buffer c & 3
      issue2(c + 4);
    }
  }

  // ---- unscale, bias, row L2 norm (inside the wave), store ----
  float ss[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) ss[q] = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int col = 32 * u + r;
    const float fc = ldexpf(1.f, -__float_as_int(sPar[3][col])), bias2 = sPar[2][col];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      acc2[u][q] = fmaf(acc2[u][q] * fr2[q], fc, bias2);
      ss[q] = fmaf(acc2[u][q], acc2[u][q], ss[q]);
    }
  }
  if (normalize) {
#pragma unroll
    for (int q = 0; q < 16; ++q) ss[q] = 1.f / (sqrtf(group_reduce<Op::Sum, 1, 16>(ss[q])) + 1e-8f);
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int64_t row = row0 + row_of(q, hf);
    if (row >= B) continue;
#pragma unroll
    for (int u = 0; u < 4; ++u) out[row * DO + 32 * u + r] = normalize ? acc2[u][q] * ss[q] : acc2[u][q];
  }
}

}  // namespace


bool fusion_shape_ok(int Dt, int Di, int h1, int d_out) {
  return h1 == H1 && d_out == DO && Dt >= 0 && Di >= 0 && Dt % BK == 0 && Di % BK == 0 && Dt + Di > 0;
}

// fp16 family: the two nnh images + the column exponents (4 KB, aligned); bf16 family: the
// three-part nnx images -- the workspace covers either
static size_t fusion_h_bytes(int Dt, int Di) { return nnh_image_bytes(Dt + Di, H1, 8) + nnh_image_bytes(H1, DO, 4); }
size_t fusion_workspace_bytes(int Dt, int Di) {
  const size_t x = nnx_image_bytes(Dt + Di, H1, 8) + nnx_image_bytes(H1, DO, 4) + 256;
  const size_t h = fusion_h_bytes(Dt, Di) + 4096;
  return x > h ? x : h;
}

hipError_t fusion_fwd(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                      int64_t B, int Dt, int Di, const float* W1, const float* b1, const float* W2, const float* b2,
                      int normalize, float* out, float* z1_out, hipStream_t st, void* ws) {
  if (B == 0) return hipSuccess;
#ifdef PPGAT_LAB_BUILD
  const bool pairs = nnh_pipeline_variant() >= 3 && ((Dt + Di) / BK) % 2 == 0;
  if (ws != nullptr && gemm_split_enabled() && gemm_f16_enabled()) {  // fp16 two-term family
#else
  // libppgat.so: k_fusion_fwdh3 (the K chunks in pairs: the reference's 384 + 512 = 28), else the
  // bf16 x6 k_fusion_fwdx; k_fusion_fwdh and k_fusion_fwdp are lab-build kernels
  const bool pairs = ((Dt + Di) / BK) % 2 == 0;
  if (ws != nullptr && gemm_split_enabled() && pairs) {
#endif
    uint16_t* w1i = static_cast<uint16_t*>(ws);
    uint16_t* w2i = w1i + nnh_image_bytes(Dt + Di, H1, 8) / 2;
    int* e1 = reinterpret_cast<int*>(static_cast<char*>(ws) + fusion_h_bytes(Dt, Di));
    int* e2 = e1 + H1;
    hipError_t e = nnh_presplit(W1, Dt + Di, 1, Dt + Di, H1, 8, w1i, e1, st);
    if (e == hipSuccess) e = nnh_presplit(W2, H1, 1, H1, DO, 4, w2i, e2, st);
    if (e != hipSuccess) return e;
#ifdef PPGAT_LAB_BUILD
    if (!pairs)
      hipLaunchKernelGGL(k_fusion_fwdh, dim3((unsigned)((B + PBM - 1) / PBM)), dim3(512), 0, st, txt, img,
                         img_index, img_fallback, B, Dt, Di, w1i, e1, b1, w2i, e2, b2, normalize, out, z1_out);
    else
#endif
      hipLaunchKernelGGL(k_fusion_fwdh3, dim3((unsigned)((B + PBM - 1) / PBM)), dim3(512), 0, st, txt, img,
                         img_index, img_fallback, B, Dt, Di, w1i, e1, b1, w2i, e2, b2, normalize, out, z1_out);
    return hipGetLastError();
  }
#ifdef PPGAT_LAB_BUILD
  if (ws != nullptr && gemm_split_enabled()) {  // W1 / W2 pre-split once, then the glds-staged kernel
    uint16_t* w1i = static_cast<uint16_t*>(ws);
    uint16_t* w2i = w1i + nnx_image_bytes(Dt + Di, H1, 8) / 2;
    hipError_t e = nnx_presplit(W1, Dt + Di, 1, Dt + Di, H1, 8, w1i, st);
    if (e == hipSuccess) e = nnx_presplit(W2, H1, 1, H1, DO, 4, w2i, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fusion_fwdp, dim3((unsigned)((B + PBM - 1) / PBM)), dim3(512), 0, st, txt, img, img_index,
                       img_fallback, B, Dt, Di, w1i, b1, w2i, b2, normalize, out, z1_out);
    return hipGetLastError();
  }
#endif
  if (gemm_split_enabled())
    hipLaunchKernelGGL(k_fusion_fwdx, dim3((unsigned)((B + BM - 1) / BM)), dim3(256), 0, st, txt, img, img_index,
                       img_fallback, B, Dt, Di, W1, b1, W2, b2, normalize, out, z1_out);
  else
    hipLaunchKernelGGL(k_fusion_fwd, dim3((unsigned)((B + BM - 1) / BM)), dim3(256), 0, st, txt, img, img_index,
                       img_fallback, B, Dt, Di, W1, b1, W2, b2, normalize, out, z1_out);
  return hipGetLastError();
}

}  // namespace ppgat
