// ppgat_fusion.hip -- FusionMLP inference on the matrix cores (the north
// star's MFMA target): embeddings/fuse_modal.py:18-36 + :220-244
//
//   x_b   = [txt_b | img_b]            img_b = img[img_index[b]] or img_fallback (mean image)
//   h_b   = relu(x_b W1^T + b1)        W1 [H1, Dt+Di]
//   y_b   = h_b W2^T + b2              W2 [Do, H1]
//   out_b = y_b / (||y_b|| + 1e-8)     (normalize != 0)
//
// fp32 in, fp32 out, v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains, no reduced precision, so
// the result matches the fp32 reference to accumulation-order rounding).  One 256-thread
// block = 64 rows: GEMM1 wave w owns hidden columns [64w, 64w+64) (2x2 tiles of 32x32),
// K streamed in 32-wide LDS chunks (the cat() and the per-row image copy loop of the
// reference are folded into the chunk loader); h stays on chip (LDS) for GEMM2 (wave w owns
// output columns [32w, 32w+32)); bias, ReLU and the row L2 norm are epilogues.
// Shapes: H1 == 4*64 = 256, Do == 4*32 = 128, Dt % 32 == 0, Di % 32 == 0 (the reference's
// 384 + 512 -> 256 -> 128).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "ppgat_internal.h"

namespace ppgat {
namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;
constexpr int BM = 64, BK = 32, H1 = 256, DO = 128;
constexpr int SXP = BK + 1;   // padded row stride (floats) of the LDS chunks
constexpr int SHP = H1 + 1;   // padded row stride of the on-chip hidden tile

__device__ __forceinline__ int row_of(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

__global__ void __launch_bounds__(256) k_fusion_fwd(const float* __restrict__ txt, const float* __restrict__ img,
                                                    const int32_t* __restrict__ img_index,
                                                    const float* __restrict__ img_fallback, int64_t B, int Dt, int Di,
                                                    const float* __restrict__ W1, const float* __restrict__ b1,
                                                    const float* __restrict__ W2, const float* __restrict__ b2,
                                                    int normalize, float* __restrict__ out,
                                                    float* __restrict__ z1_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sX = smem;                       // [BM][SXP]
  float* sW = smem + BM * SXP;            // [H1][SXP]  (GEMM2: [DO][SXP])
  float* sH = sW + H1 * SXP;              // [BM][SHP]
  float* sN = sH + BM * SHP;              // [4][BM] row sums of squares
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t row0 = (int64_t)blockIdx.x * BM;
  const int K = Dt + Di;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // ---- GEMM1: [BM x K] x [K x H1] ----
  for (int k0 = 0; k0 < K; k0 += BK) {
    // X chunk: BM x BK = 512 float4; 2 per thread
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int idx = t * 256 + tid;
      const int r = idx >> 3, c4 = (idx & 7) * 4;
      const int64_t b = row0 + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (b < B) {
        const int k = k0 + c4;
        if (k < Dt) {
          v = *reinterpret_cast<const float4*>(txt + b * Dt + k);
        } else {
          const int32_t ii = img_index ? img_index[b] : (int32_t)b;
          const float* src = ii >= 0 ? img + (int64_t)ii * Di : img_fallback;
          v = *reinterpret_cast<const float4*>(src + (k - Dt));
        }
      }
      float* d = sX + r * SXP + c4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    // W1 chunk: H1 x BK = 2048 float4; 8 per thread
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int idx = t * 256 + tid;
      const int j = idx >> 3, c4 = (idx & 7) * 4;
      const float4 v = *reinterpret_cast<const float4*>(W1 + (int64_t)j * K + k0 + c4);
      float* d = sW + j * SXP + c4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < BK; kk += 2) {
      const int kq = kk + (lane >> 5);
      const float a0 = sX[(lane & 31) * SXP + kq];
      const float a1 = sX[(32 + (lane & 31)) * SXP + kq];
      const float w0 = sW[(64 * w + (lane & 31)) * SXP + kq];
      const float w1 = sW[(64 * w + 32 + (lane & 31)) * SXP + kq];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, w0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, w1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, w0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, w1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  // bias + ReLU -> sH (and the pre-activation for a training backward)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int col = 64 * w + 32 * b + (lane & 31);
      const float bias = b1[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * a + row_of(r, lane);
        const float z = acc[a][b][r] + bias;
        sH[row * SHP + col] = fmaxf(z, 0.f);
        if (z1_out != nullptr && row0 + row < B) z1_out[(row0 + row) * H1 + col] = z;
      }
    }
  // ---- GEMM2: [BM x H1] x [H1 x DO] ----
  f32x16 acc2[2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[a][r] = 0.f;
  for (int k0 = 0; k0 < H1; k0 += BK) {
    // W2 chunk: DO x BK = 1024 float4; 4 per thread
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int idx = t * 256 + tid;
      const int j = idx >> 3, c4 = (idx & 7) * 4;
      const float4 v = *reinterpret_cast<const float4*>(W2 + (int64_t)j * H1 + k0 + c4);
      float* d = sW + j * SXP + c4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < BK; kk += 2) {
      const int kq = kk + (lane >> 5);
      const float a0 = sH[(lane & 31) * SHP + k0 + kq];
      const float a1 = sH[(32 + (lane & 31)) * SHP + k0 + kq];
      const float w0 = sW[(32 * w + (lane & 31)) * SXP + kq];
      acc2[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, w0, acc2[0], 0, 0, 0);
      acc2[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, w0, acc2[1], 0, 0, 0);
    }
    __syncthreads();
  }
  // bias, row L2 norm (over the 4 waves' 32 columns each), store
  const int col = 32 * w + (lane & 31);
  const float bias2 = b2[col];
  float ss[2][16];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc2[a][r] += bias2;
      ss[a][r] = acc2[a][r] * acc2[a][r];
    }
  if (normalize) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = ss[a][r];
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off);  // within the 32-lane half
        ss[a][r] = v;
      }
    if ((lane & 31) == 0) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int r = 0; r < 16; ++r) sN[w * BM + 32 * a + row_of(r, lane)] = ss[a][r];
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * a + row_of(r, lane);
      float v = acc2[a][r];
      if (normalize) {
        const float n2 = ((sN[row] + sN[BM + row]) + sN[2 * BM + row]) + sN[3 * BM + row];
        v = v / (sqrtf(n2) + 1e-8f);
      }
      if (row0 + row < B) out[(row0 + row) * DO + col] = v;
    }
}

}  // namespace

size_t fusion_lds_bytes() { return (size_t)(BM * SXP + H1 * SXP + BM * SHP + 4 * BM) * 4; }

bool fusion_shape_ok(int Dt, int Di, int h1, int d_out) {
  return h1 == H1 && d_out == DO && Dt >= 0 && Di >= 0 && Dt % BK == 0 && Di % BK == 0 && Dt + Di > 0;
}

hipError_t fusion_fwd(const float* txt, const float* img, const int32_t* img_index, const float* img_fallback,
                      int64_t B, int Dt, int Di, const float* W1, const float* b1, const float* W2, const float* b2,
                      int normalize, float* out, float* z1_out, hipStream_t st) {
  if (B == 0) return hipSuccess;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_fusion_fwd),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)fusion_lds_bytes());
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(k_fusion_fwd, dim3((unsigned)((B + BM - 1) / BM)), dim3(256), fusion_lds_bytes(), st, txt, img,
                     img_index, img_fallback, B, Dt, Di, W1, b1, W2, b2, normalize, out, z1_out);
  return hipGetLastError();
}

}  // namespace ppgat
