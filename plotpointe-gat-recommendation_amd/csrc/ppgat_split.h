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


}  // namespace split
}  // namespace ppgat
