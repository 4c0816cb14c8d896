// ppgat_nnh_pipe.h -- the pipelined main loop of the fp16 two-term NN products (k_gemm_nnh3 and
// the FusionMLP's GEMM1, k_fusion_fwdh3): A [rows x K] fp32 streamed by each lane from its row,
// B pre-split into NnhImg<NT> images (ppgat_xform.hip: nnh_presplit), 8 waves x 32 rows per
// workgroup sharing every staged B chunk.
//
// Per 32-deep chunk c (`chunks` even, >= 2):
//  * B chunk c + 2 goes to LDS by LDS-DMA (buffer_load ... lds in inline asm: the compiler sees no
//    memory access, so it adds no wait before LDS reads), three buffers;
//  * X(c + 2) streams into the register set X(c) came from (two sets, two chunks ahead);
//  * the 16 / 8 MFMA steps of chunk c (three fp16 MFMAs each) run from the fragments prepared
//    during chunk c - 1, and the second half of those steps carries chunk c + 1's preparation in
//    its gaps: row maxima, the online row scale (split::row_scale_plan), the fp16 split -- the
//    independent VALU work issues while the wave's MFMAs run, so no chunk starts with the MFMA
//    pipe idle behind ~100 VALU instructions (k_gemm_nnh2 did that at the top of every chunk);
//  * after the products: the rare accumulator rescale (split::row_rescale), then an explicit
//    vmcnt wait for this wave's DMA of chunk c + 1 and a bare s_barrier.
// The products and their order are k_gemm_nnh's (bitwise equal results).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ppgat_split.h"

namespace ppgat {

template <int NT>
struct NnhImg {
  static constexpr int KC = 32, BN = 32 * NT, LDK = KC + 8, PART = BN * LDK, ELEMS = 2 * PART, BYTES = 2 * ELEMS;
  static_assert(BYTES % 1024 == 0, "an image is a whole number of 1-KB wave copies");
};

using i32x4 = __attribute__((ext_vector_type(4))) int;

// one buffer_load_dwordx4 ... lds: 16 B per lane from rsrc at voff + soff into LDS at m0 = lds
__device__ __forceinline__ void dma_lds16(const i32x4& rsrc, uint32_t lds, uint32_t voff, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(lds), "v"(voff), "s"(rsrc), "s"(soff)
               : "memory", "m0");
}

// s_waitcnt vmcnt(n) (gfx9 encoding; expcnt / lgkmcnt left open)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// acc (NT 32x32 tiles of this wave's 32 rows) = sum over chunks of X chunk x B chunk, scaled:
// acc = (X s_row) (B s_col) with erow the row's final exponent (s_row = 2^erow).  img: this
// column block's chunk images (chunks x NnhImg<NT>::ELEMS); sB: LDS, 3 x ELEMS; sFw: this wave's
// 32-float LDS scratch; loadx(c, x): this lane's 16 values of chunk c (4 float4, the fragment
// order of split2h: x[g] = row[32 c + 8 g + 4 hf .. + 3]).
// BD: B fragments read BD MFMA steps ahead (1: the step before, as k_gemm_nnh2; 2: two steps,
// eight more VGPRs, for LDS latency under eight waves of reads).  PRIO: waves 4-7 (the second-
// dispatched half, the issue-arbitration loser) at s_setprio 1 for the whole loop.
// LAB (diagnostics only, instantiated in lab builds -DPPGAT_LAB_BUILD=1, never in libppgat.so;
// PPGAT_NNH2_LAB with PPGAT_NNH2=3; results wrong), bits: 1 = no X loads
// after the first two chunks, 2 = no B DMA after the first two chunks, 16 = no B fragment reads
// inside a chunk's MFMA steps (the first BD per chunk only), 32 = no preparation of the next
// chunk (its fragments reused)
// XT: loadx(c, x) delivers the chunk COALESCED -- lane l holds floats [4 (l & 7), +4) of rows
// (l >> 3) + 8 j, j = 0..3 (each load instruction reads 8 whole 128-B row segments, not 32-B
// pieces of 32 rows) -- and the preparation turns it into the fragment layout through this
// wave's LDS scratch sXw [32 rows][36 floats] (4 ds_write_b128 + 4 ds_read_b128 per chunk,
// conflict-free with the 36-float row stride).  The same values in the same fragment slots: the
// products are bitwise those of the direct layout.
template <int NT, int BD = 1, bool PRIO = false, int LAB = 0, bool XT = false, class LoadX>
__device__ __forceinline__ void nnh3_loop(const uint16_t* img, uint16_t* sB, int chunks, const LoadX& loadx,
                                          split::f32x16 (&acc)[NT], int& erow, float* sFw, int wv, int lane,
                                          float* sXw = nullptr) {
  static_assert(BD == 1 || BD == 2, "B read depth");
  using I = NnhImg<NT>;
  constexpr int LDK = I::LDK, PART = I::PART, NI = I::BYTES / 1024;
  constexpr int STEPS = (I::KC / 16) * NT;  // MFMA steps (three products each) per chunk
  constexpr int PH = 8;                     // preparation phases of the next chunk, in the second half
  constexpr int PPS = PH / (STEPS / 2);     // phases per step
  static_assert(PPS >= 1 && PPS * (STEPS / 2) == PH, "phases");
  const int r = lane & 31, hf = lane >> 5;
  const uint64_t base = reinterpret_cast<uint64_t>(img);
  const i32x4 rsrc = {__builtin_amdgcn_readfirstlane((int)(uint32_t)base),
                      __builtin_amdgcn_readfirstlane((int)((base >> 32) & 0xffff)),
                      __builtin_amdgcn_readfirstlane(chunks * I::BYTES), 0x00020000};
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(sB);
  const uint32_t voff = (uint32_t)lane * 16u;
  constexpr int ND = (NI + 7) / 8;  // DMA instructions of waves 0 .. (NI % 8) - 1 (one fewer for the rest)
  const bool full = (NI % 8 == 0) || wv < NI % 8;
  auto issue = [&](int c) {  // chunk c's two images -> buffer c % 3, 1 KB per wave instruction
    const uint32_t dst = lds0 + (uint32_t)((c % 3) * I::ELEMS * 2);
    for (int i = wv; i < NI; i += 8) dma_lds16(rsrc, dst + i * 1024, voff, (uint32_t)(c * I::BYTES + i * 1024));
  };
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = split::f32x16{};
  bool set = false;  // the row has had a nonzero element (its scale is fixed until an overflow)
  // the next chunk's preparation state
  float pmx = 0.f;
  int pen = 0;
  bool pneed = false;
  float ps = 1.f;
  // the prepared fragments materialised where they are computed (the compiler would otherwise
  // sink the split past the MFMAs to its use in the next chunk)
  auto pin = [](split::u32x4 (&f)[2]) { asm volatile("" : "+v"(f[0]), "+v"(f[1])); };
  // phase ph of preparing the chunk in xn into fragments fxn (phases 0..7; 7 is empty)
  auto prep = [&](int ph, float4 (&xn)[4], split::u32x4 (&fxn)[2][2]) {
    switch (ph) {
      case 0:
        if constexpr (XT) {  // coalesced rows -> fragment layout, in place
#pragma unroll
          for (int j = 0; j < 4; ++j)
            *reinterpret_cast<float4*>(sXw + ((lane >> 3) + 8 * j) * 36 + 4 * (lane & 7)) = xn[j];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
          for (int g = 0; g < 4; ++g) xn[g] = *reinterpret_cast<const float4*>(sXw + r * 36 + 8 * g + 4 * hf);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
          pmx = fmaxf(fmaxf(0.f, split::absmax4(xn[0])), split::absmax4(xn[1]));
        }
        break;
      case 1:
        if constexpr (XT)
          pmx = fmaxf(fmaxf(fmaxf(fmaxf(0.f, split::absmax4(xn[0])), split::absmax4(xn[1])), split::absmax4(xn[2])),
                      split::absmax4(xn[3]));
        else
          pmx = fmaxf(fmaxf(pmx, split::absmax4(xn[2])), split::absmax4(xn[3]));
        break;
      case 2:
        pneed = split::row_scale_plan(pmx, erow, set, pen);
        ps = __builtin_ldexpf(1.f, pen);
        break;
      case 3: split::split2h_half(xn[0], ps, fxn[0][0], fxn[0][1], 0); break;
      case 4:
        split::split2h_half(xn[1], ps, fxn[0][0], fxn[0][1], 2);
        pin(fxn[0]);
        break;
      case 5: split::split2h_half(xn[2], ps, fxn[1][0], fxn[1][1], 0); break;
      case 6:
        split::split2h_half(xn[3], ps, fxn[1][0], fxn[1][1], 2);
        pin(fxn[1]);
        break;
      default: break;
    }
  };
  // after the chunk's products: the rows whose scale changed rescale their accumulators
  auto commit = [&]() {
    if (__builtin_amdgcn_ballot_w64(pneed)) split::row_rescale<NT>(erow, pen, set, acc, sFw, r, hf);
    erow = pen;
    set = set || pneed;
  };
  if (PRIO && wv >= 4) __builtin_amdgcn_s_setprio(1);
  float4 xA[4], xB[4];
  split::u32x4 fxA[2][2], fxB[2][2];
  issue(0);
  loadx(0, xA);
  issue(1);
  loadx(1, xB);
#pragma unroll
  for (int ph = 0; ph < PH; ++ph) prep(ph, xA, fxA);
  commit();
  if (full) wait_vm<4 + ND + 4>(); else wait_vm<4 + ND - 1 + 4>();  // DMA(0) has landed
  __builtin_amdgcn_s_barrier();

  // chunk c from fxc; X(c + 2) -> xl (the set chunk c came from); chunk c + 1 prepared from xn
  auto body = [&](const int c, float4 (&xl)[4], float4 (&xn)[4], const split::u32x4 (&fxc)[2][2],
                  split::u32x4 (&fxn)[2][2], auto has_next) {
    constexpr bool NEXT = decltype(has_next)::value;
    const bool ahead = c + 2 < chunks;
    if (ahead && !(LAB & 2)) issue(c + 2);
    if (!(LAB & 1)) loadx(ahead ? c + 2 : chunks - 1, xl);  // the last two chunks re-read chunk chunks - 1
    const uint16_t* sb = sB + (c % 3) * I::ELEMS;
    auto read_b = [&](int i, split::u32x4 (&f)[2]) {
      const int off = (32 * (i % NT) + r) * LDK + 16 * (i / NT) + 8 * hf;
#pragma unroll
      for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const split::u32x4*>(&sb[p * PART + off]);
    };
    split::u32x4 fb[BD + 1][2];
#pragma unroll
    for (int i = 0; i < BD; ++i) read_b(i, fb[i]);
#pragma unroll
    for (int i = 0; i < STEPS; ++i) {
      const int u = i / NT, t = i % NT;
      if (!(LAB & 16) && i + BD < STEPS) read_b(i + BD, fb[(i + BD) % (BD + 1)]);
      acc[t] = split::mfma32_h3(fxc[u], fb[(LAB & 16) ? 0 : i % (BD + 1)], acc[t]);
      if constexpr (NEXT && !(LAB & 32)) {
        if (i >= STEPS / 2) {
#pragma unroll
          for (int k = 0; k < PPS; ++k) prep((i - STEPS / 2) * PPS + k, xn, fxn);
        }
      }
      if (i + BD < STEPS) __builtin_amdgcn_sched_group_barrier(0x0100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x0002, 6, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x0002, 6, 0);
      __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (NEXT && !(LAB & 32)) commit();
    // DMA(c + 1) has landed (issued after it: X(c + 1), DMA(c + 2) if any, X(c + 2)) and every
    // wave is done with buffer c % 3 before DMA(c + 3) (issued in chunk c + 1) overwrites it
    if (LAB) {
      wait_vm<0>();
    } else if (ahead) {
      if (full) wait_vm<4 + ND + 4>(); else wait_vm<4 + ND - 1 + 4>();
    } else {
      wait_vm<4 + 4>();
    }
    __builtin_amdgcn_s_barrier();
  };
  using yes = std::integral_constant<bool, true>;
  using no = std::integral_constant<bool, false>;
  for (int c = 0; c < chunks - 2; c += 2) {
    body(c, xA, xB, fxA, fxB, yes{});
    body(c + 1, xB, xA, fxB, fxA, yes{});
  }
  body(chunks - 2, xA, xB, fxA, fxB, yes{});
  body(chunks - 1, xB, xA, fxB, fxA, no{});
  if (PRIO && wv >= 4) __builtin_amdgcn_s_setprio(0);
}

}  // namespace ppgat
