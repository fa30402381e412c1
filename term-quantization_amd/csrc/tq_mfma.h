// MFMA-engine building blocks shared by the term-pair conv kernels on the matrix cores
// (tr_conv_mfma.hip: gather engines; tr_conv_patch.hip: input-patch engine).  The exactness
// argument for fp16 term-sum codes on v_mfma_f32_32x32x16_f16 is in tr_conv_mfma.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tq {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float float16v __attribute__((ext_vector_type(16)));
// Native vector (not HIP's union-based uint4, which defeats SROA: arrays of it become
// allocas that the backend promotes to LDS).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kKStep = 64;  // codes per K-step

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 8 + (chunk ^ ((row >> 1) & 7));
}

// Accumulator state of one wave: MB x 2 blocks of 32 x 32, fp32 (exact window) + int32.
template <int MB>
struct MfmaAcc {
  float16v f[MB][2];
  int i[MB][2][16];
};

template <int MB>
__device__ __forceinline__ void acc_zero(MfmaAcc<MB>& acc) {
#pragma unroll
  for (int bm = 0; bm < MB; ++bm)
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc.f[bm][bn][r] = 0.0f;
        acc.i[bm][bn][r] = 0;
      }
    }
}

// fp32 partial sums are exact integers below 2^24: move them into the int32 sums.
template <int MB>
__device__ __forceinline__ void acc_flush(MfmaAcc<MB>& acc) {
#pragma unroll
  for (int bm = 0; bm < MB; ++bm)
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc.i[bm][bn][r] += (int)acc.f[bm][bn][r];
        acc.f[bm][bn][r] = 0.0f;
      }
    }
}

// LDS staging by global_load_lds_dwordx4 (LDS-DMA: no VGPR destination; the LDS image of
// one wave-instruction is lane-linear, base + lane * 16).
__device__ u32x4 g_zero_page[64];  // static storage: all zeros, never written

__device__ __forceinline__ void glds16(const void* src, u32x4* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, lds_wave_base, 16, 0, 0);
}

// The same LDS-DMA issued as inline asm, invisible to the compiler's wait-count pass.  With
// the builtin, any LDS-DMA in flight makes that pass wait for vmcnt(0) before the first use
// of ANY vector-register load (it cannot order the two kinds of vmcnt event), which drains
// a kernel's register prefetch (checked on a two-load test kernel: vmcnt(0) with a DMA in
// flight, vmcnt(2) without).  Safe for the compiler's own waits: an untracked DMA only makes
// them wait longer (vmcnt retires in order).  The caller retires the DMA itself (counted
// TQ_WAIT_VM + barrier) and must keep LDS reads of the slot behind a compiler barrier
// ("memory" clobber: this asm is one).
__device__ __forceinline__ void glds16_asm(const void* src, u32x4* lds_wave_base) {
  const uint32_t la = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)lds_wave_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(la)
               : "memory", "m0");
}

// s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt[3:0] | expcnt 7 << 4 | lgkmcnt 15 << 8 |
// vmcnt[5:4] << 14), other counters untouched.
#define TQ_WAIT_VM(n) \
  __builtin_amdgcn_s_waitcnt(((n) & 15) | (7 << 4) | (15 << 8) | ((((n) >> 4) & 3) << 14))

// s_waitcnt vmcnt(n) for a runtime n in [0, 63] (larger n waits for 63: stricter, correct).
template <int N>
__device__ __forceinline__ void wait_vm_upto(int n) {
  if constexpr (N < 0) {
    TQ_WAIT_VM(0);
  } else {
    if (n >= N) {
      TQ_WAIT_VM(N);
    } else {
      wait_vm_upto<N - 1>(n);
    }
  }
}

__device__ __forceinline__ void wait_vm_dyn(int n) {
  if (n >= 15) {
    wait_vm_upto<63>(n);
  } else {
    wait_vm_upto<15>(n);
  }
}

}  // namespace
}  // namespace tq
