// ppgat_split.h -- fp32 products on the bf16 matrix cores through a three-term split (gfx950).
//
// Every fp32 operand v is cut into three bf16 terms, h = rne(v), m = rne(v - h),
// l = rne(v - h - m) (the two differences are exact), so v = h + m + l + e with
// |e| <= 2^-24 |v| -- fp32's own rounding unit.  A product a b is formed as the six terms of
// order <= 2 (l_a h_b, h_a l_b, m_a m_b, m_a h_b, h_a m_b, h_a h_b, smallest first) on
// v_mfma_f32_{16x16x32,32x32x16}_bf16 with fp32 accumulation; the dropped terms (m l, l m, l l)
// are <= 2^-24 |a b| together.  Each bf16 product is exact in fp32, so the result carries fp32
// GEMM accuracy at 16/6 = 2.7x the fp32 MFMA rate (MI355X_MICROARCH.md: 16x16x32 bf16 = 16,
// 32x32x16 bf16 = 32, 16x16x4 f32 = 32, 32x32x2 f32 = 64 cycles per SIMD).  Not bitwise equal
// to an fp32 FMA chain (different summation order).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ppgat {
namespace split {

using u32x4 = __attribute__((__vector_size__(4 * sizeof(unsigned int)))) unsigned int;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;
using bf16x2 = __attribute__((ext_vector_type(2))) __bf16;
using f32x2e = __attribute__((ext_vector_type(2))) float;

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {  // v_cvt_pk_bf16_f32 (rne)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2e{a, b}, bf16x2));
}
__device__ __forceinline__ float bf_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// 8 fp32 values (element j of the fragment = p.x, p.y, ..., q.w) -> three bf16x8 terms
__device__ __forceinline__ void split3(const float4& p, const float4& q, u32x4& h, u32x4& m, u32x4& l) {
  const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t hh = pk_bf16(v[2 * i], v[2 * i + 1]);
    const float r0 = v[2 * i] - bf_lo(hh), r1 = v[2 * i + 1] - bf_hi(hh);
    const uint32_t mm = pk_bf16(r0, r1);
    h[i] = hh;
    m[i] = mm;
    l[i] = pk_bf16(r0 - bf_lo(mm), r1 - bf_hi(mm));
  }
}
__device__ __forceinline__ f32x4 mfma_bf(const u32x4& a, const u32x4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_x6(const u32x4& ah, const u32x4& am, const u32x4& al, const u32x4& bh,
                                         const u32x4& bm, const u32x4& bl, f32x4 c) {
  c = mfma_bf(al, bh, c);
  c = mfma_bf(ah, bl, c);
  c = mfma_bf(am, bm, c);
  c = mfma_bf(am, bh, c);
  c = mfma_bf(ah, bm, c);
  return mfma_bf(ah, bh, c);
}

__device__ __forceinline__ f32x16 mfma32_bf(const u32x4& a, const u32x4& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32_x6(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
  c = mfma32_bf(a[2], b[0], c);
  c = mfma32_bf(a[0], b[2], c);
  c = mfma32_bf(a[1], b[1], c);
  c = mfma32_bf(a[1], b[0], c);
  c = mfma32_bf(a[0], b[1], c);
  return mfma32_bf(a[0], b[0], c);
}

// ---------------------------------------------------------------------------
// Scaled two-term fp16 split (the large-M NN GEMMs and the FusionMLP).  With a power-of-two
// scale s per row of X (per column of B) that puts the largest |v| s of the row in [2^9, 2^10),
// v s = h + l + e, h = rne16(v s), l = rne16(v s - h) (the difference is exact in fp32):
// 11 + 11 bits, |e| <= 2^-22 |v s| for elements whose l is a normal fp16 (|v s| >= 2^-2) and
// <= 2^-25 absolutely (2^-34 of the row's max) below that.  A product takes three fp16 MFMAs,
// l_a h_b + h_a l_b + h_a h_b (the dropped l_a l_b <= 2^-22 |ab|), fp32 accumulation, and the
// tile is unscaled by 1 / (s_a s_b) in the epilogue (exact: powers of two) -- half the MFMAs of
// the bf16 three-term split above, at 2^-21 instead of 2^-24 per product.
// ---------------------------------------------------------------------------
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;

__device__ __forceinline__ uint32_t pk_f16(float a, float b) {  // v_cvt_pk_f16_f32 (rne)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2e{a, b}, f16x2));
}

// the power-of-two scale that puts m (> 0, finite) in [2^9, 2^10); exponent clamped to [-126, 126]
__device__ __forceinline__ int scale_exp16(float m) {
  const int e = __builtin_amdgcn_frexp_expf(m);  // m in [2^(e-1), 2^e)
  const int s = 10 - e;
  return s > 126 ? 126 : (s < -126 ? -126 : s);
}

// 8 fp32 values (fragment order as split3) times s -> the two fp16x8 terms
__device__ __forceinline__ void split2h(const float4& p, const float4& q, float s, u32x4& h, u32x4& l) {
  const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = v[2 * i] * s, b = v[2 * i + 1] * s;
    const uint32_t hh = pk_f16(a, b);
    const f32x2e back = __builtin_convertvector(__builtin_bit_cast(f16x2, hh), f32x2e);
    h[i] = hh;
    l[i] = pk_f16(a - back.x, b - back.y);
  }
}

// Online row scales for an A operand streamed in 32-deep chunks, lane (r, hf) holding 16 values of
// row r (r = lane & 31, hf = lane >> 5) as 4 float4.  A row's scale exponent is set by the first
// chunk in which the row is nonzero and lowered only when a later chunk would reach 2^15 (fp16
// overflows at 65,520: 32x headroom); then the row's accumulators -- element q of each 32x32
// tile sits at row (q & 3) + 8 (q >> 2) + 4 hf -- are multiplied by the exact power of two
// 2^(new - old), through the wave's 32-float LDS scratch sFw.  Wave-uniform branch, taken rarely
// on real data.  Returns the scale 2^erow for this chunk's split.
template <int NT>
__device__ __forceinline__ float row_scale_online(const float4 (&xa)[4], int& erow, bool& set,
                                                  f32x16 (&acc)[NT], float* sFw, int r, int hf) {
  float mx = 0.f;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(xa[g].x), fabsf(xa[g].y)), fmaxf(fabsf(xa[g].z), fabsf(xa[g].w))));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  const bool need = mx <= 3.4e38f && (set ? mx * __builtin_ldexpf(1.f, erow) >= 32768.f : mx > 0.f);
  if (__builtin_amdgcn_ballot_w64(need)) {
    const int enew = need ? scale_exp16(mx) : erow;
    if (hf == 0) sFw[r] = set ? __builtin_ldexpf(1.f, enew - erow) : 1.f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float f[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 v = *reinterpret_cast<const float4*>(&sFw[8 * j + 4 * hf]);
      f[4 * j] = v.x; f[4 * j + 1] = v.y; f[4 * j + 2] = v.z; f[4 * j + 3] = v.w;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] *= f[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    erow = enew;
    set = set || need;
  }
  return __builtin_ldexpf(1.f, erow);
}

// row_scale_online in two halves, for a caller that prepares chunk c + 1 while chunk c's
// products run: absmax4 folds (the same expression and order as row_scale_online), row_scale_plan
// gives the chunk's per-lane exponent and whether its row rescales, and row_rescale applies the
// rescale to the accumulators once chunk c's products are in them (bitwise the same arithmetic)
__device__ __forceinline__ float absmax4(const float4& v) {
  return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}
__device__ __forceinline__ bool row_scale_plan(float mx, int erow, bool set, int& enew) {
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  // branch-free (the caller interleaves this with MFMAs): every term evaluated, combined bitwise
  const bool over = mx * __builtin_ldexpf(1.f, erow) >= 32768.f, pos = mx > 0.f, fin = mx <= 3.4e38f;
  const bool need = fin & ((set & over) | (!set & pos));
  enew = need ? scale_exp16(mx) : erow;
  return need;
}
template <int NT>
__device__ __forceinline__ void row_rescale(int erow, int enew, bool set, f32x16 (&acc)[NT], float* sFw, int r,
                                            int hf) {
  if (hf == 0) sFw[r] = set ? __builtin_ldexpf(1.f, enew - erow) : 1.f;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float f[16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 v = *reinterpret_cast<const float4*>(&sFw[8 * j + 4 * hf]);
    f[4 * j] = v.x; f[4 * j + 1] = v.y; f[4 * j + 2] = v.z; f[4 * j + 3] = v.w;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[t][q] *= f[q];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// half of split2h: the 4 values of p -> terms [2 j0, 2 j0 + 1] of h and l
__device__ __forceinline__ void split2h_half(const float4& p, float s, u32x4& h, u32x4& l, int j0) {
  const float v[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float a = v[2 * i] * s, b = v[2 * i + 1] * s;
    const uint32_t hh = pk_f16(a, b);
    const f32x2e back = __builtin_convertvector(__builtin_bit_cast(f16x2, hh), f32x2e);
    h[j0 + i] = hh;
    l[j0 + i] = pk_f16(a - back.x, b - back.y);
  }
}

// the per-row unscale factors 2^-erow of this lane's 16 accumulator rows (through sFw)
__device__ __forceinline__ void row_unscale(int erow, float* sFw, int r, int hf, float (&f)[16]) {
  if (hf == 0) sFw[r] = __builtin_ldexpf(1.f, -erow);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 v = *reinterpret_cast<const float4*>(&sFw[8 * j + 4 * hf]);
    f[4 * j] = v.x; f[4 * j + 1] = v.y; f[4 * j + 2] = v.z; f[4 * j + 3] = v.w;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ f32x16 mfma32_h(const u32x4& a, const u32x4& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                0, 0);
}
__device__ __forceinline__ f32x16 mfma32_h3(const u32x4 (&a)[2], const u32x4 (&b)[2], f32x16 c) {
  c = mfma32_h(a[1], b[0], c);
  c = mfma32_h(a[0], b[1], c);
  return mfma32_h(a[0], b[0], c);
}

}  // namespace split
}  // namespace ppgat
