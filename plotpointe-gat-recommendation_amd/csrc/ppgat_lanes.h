// ppgat_lanes.h -- cross-lane reductions for 64-lane CDNA4 wavefronts without the LDS pipe.
//
// __shfl_xor lowers to ds_bpermute (an LDS round trip per step).  The reductions in the
// hot kernels use instead:
//   xor 1, 2       DPP quad_perm            (exact lane ^ 1, lane ^ 2)
//   "xor 4"        DPP row_half_mirror      (lane i <-> 7 - i; equal to lane ^ 4 once the
//                                            value is uniform within each quad, which the
//                                            ascending-order reductions below guarantee)
//   xor 8          DPP row_ror:8            (exact lane ^ 8 inside a 16-lane row)
//   xor 16, 32     v_permlane16_swap / v_permlane32_swap (gfx950): one VALU op swaps the
//                  odd 16-lane rows of a with the even rows of b (resp. the upper half of a
//                  with the lower half of b), so a lane sees its partner's value.
// Sums are formed as a + b with commutative IEEE adds, so both lanes of a pair hold the
// bitwise-identical result and every reduction is deterministic.
#pragma once
#include <hip/hip_runtime.h>

namespace ppgat {

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

// {own-or-partner} pair across rows: r[0] + r[1] == a_self + a_partner on lanes whose OFF
// bit is 0 and b_partner + b_self on lanes whose OFF bit is 1.
template <int OFF>
__device__ __forceinline__ void row_swap(float a, float b, float& r0, float& r1) {
  // Inline asm: hipcc (ROCm 7.2) returned the vdst half for both members of the
  // __builtin_amdgcn_permlane{16,32}_swap pair here (tools/lane_selftest.hip shows it).  The
  // two v_nop are the VALU-write -> v_permlane-read wait states.
  static_assert(OFF == 16 || OFF == 32, "row_swap: 16 or 32");
  if constexpr (OFF == 16) {
    asm volatile("v_nop\n\tv_nop\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  } else {
    asm volatile("v_nop\n\tv_nop\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  }
  r0 = a;
  r1 = b;
}

enum class Op { Sum, Max };

template <Op O>
__device__ __forceinline__ float combine(float a, float b) {
  if constexpr (O == Op::Sum) return a + b;
  else return fmaxf(a, b);
}

// one butterfly step at offset OFF (OFF == 4 requires quad-uniform v)
template <Op O, int OFF>
__device__ __forceinline__ float xstep(float v) {
  if constexpr (OFF == 1) return combine<O>(v, dpp<0xB1>(v));
  else if constexpr (OFF == 2) return combine<O>(v, dpp<0x4E>(v));
  else if constexpr (OFF == 4) return combine<O>(v, dpp<0x141>(v));
  else if constexpr (OFF == 8) return combine<O>(v, dpp<0x128>(v));
  else {
    float r0, r1;
    row_swap<OFF>(v, v, r0, r1);
    return combine<O>(r0, r1);
  }
}

// reduce over the lane-index bits [LO, HI] (powers of two), ascending; every lane of a
// group ends with the group's result.  LO must be 1 if HI >= 4 (quad uniformity).
template <Op O, int LO, int HI>
__device__ __forceinline__ float group_reduce(float v) {
  if constexpr (LO <= HI && LO >= 1) {
    v = xstep<O, LO>(v);
    return group_reduce<O, LO * 2, HI>(v);
  } else {
    return v;
  }
}

__device__ __forceinline__ float wave_sum(float v) { return group_reduce<Op::Sum, 1, 32>(v); }
__device__ __forceinline__ float wave_max(float v) { return group_reduce<Op::Max, 1, 32>(v); }

// sum over subgroups: lanes l, l + LPR, l + 2 LPR, ... (offsets LPR .. 32; offset 4 here is
// not quad-uniform, so it takes the exact bpermute xor)
template <int LPR>
__device__ __forceinline__ float4 across_subgroups(float4 a) {
  if constexpr (LPR >= 64) {
    return a;
  } else if constexpr (LPR != 4) {
    a.x = xstep<Op::Sum, LPR>(a.x);
    a.y = xstep<Op::Sum, LPR>(a.y);
    a.z = xstep<Op::Sum, LPR>(a.z);
    a.w = xstep<Op::Sum, LPR>(a.w);
    return across_subgroups<LPR * 2>(a);
  } else {
    a.x += __shfl_xor(a.x, LPR);
    a.y += __shfl_xor(a.y, LPR);
    a.z += __shfl_xor(a.z, LPR);
    a.w += __shfl_xor(a.w, LPR);
    return across_subgroups<LPR * 2>(a);
  }
}

// Transposing butterfly: U partial values per lane, each to be summed over the LPR lanes of
// a subgroup.  The first log2(U) steps exchange halves of the value set with the partner
// (U - 1 exchanges in all instead of U log2(LPR)); then a plain reduction over the
// remaining LPR / U lanes.  On return every lane holds the full sum for value index
// sl / (LPR / U).  Transposing offsets are LPR/2 .. LPR/U, all >= 8 for the geometries used.
template <int LPR, int U, int OFF = LPR / 2, int N = U>
__device__ __forceinline__ float transpose_reduce(float (&v)[U], int sl) {
  if constexpr (N > 1) {
    static_assert(OFF >= 8, "transposing steps need an exact xor (offset >= 8)");
    constexpr int H = N / 2;
    const bool bit = (sl & OFF) != 0;
#pragma unroll
    for (int t = 0; t < H; ++t) {
      if constexpr (OFF >= 16) {
        float r0, r1;
        row_swap<OFF>(v[t], v[H + t], r0, r1);
        v[t] = r0 + r1;
      } else {
        const float send = bit ? v[t] : v[H + t];
        const float keep = bit ? v[H + t] : v[t];
        v[t] = keep + dpp<0x128>(send);  // OFF == 8
      }
    }
    return transpose_reduce<LPR, U, OFF / 2, H>(v, sl);
  } else {
    return group_reduce<Op::Sum, 1, OFF>(v[0]);
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace ppgat
