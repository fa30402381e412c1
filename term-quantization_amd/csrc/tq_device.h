// Device-side building blocks of the term-revealing (TR) path on CDNA4 (gfx950).
//
// Every function here restates one step of the reference kernel
// (kernels/tr_cuda_kernel.cu) in a form that suits a 64-lane wavefront: no per-element
// 64-slot term array, no data-dependent 64-iteration loop -- the HESE terms of an element
// are two 32-bit masks computed in registers, and term selection works on those masks.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tq {

constexpr int kMaxGroupSize = 32;  // kernels/tr_cuda_kernel.cu:9 (MAX_GROUP_SIZE)
constexpr int kMaxBitwidth = 24;   // keeps every partial sum exact in fp32

// a1 -- quantize: kernels/tr_cuda_kernel.cu:21-23.
//   q = min(sat_int32(double(fp32(|x| / sf)) + 0.5), 2^bw - 1), NaN -> 0.
// The +0.5 is a double add in the reference (the literal 0.5 promotes); doing it in fp32
// rounds |x|/sf = 0.49999997f up to 1.  With maxv <= 2^24 - 1 (exact in fp32) the
// reference's fminf(float(int), maxv) round trip equals an integer min.
//
// Both steps are computed without the IEEE fp32 division sequence and without fp64 adds:
//  * fp32(|x| / sf) == fp32(double(|x|) * RN64(1/sf)).  The double product is within
//    2^-52 (relative) of the exact quotient, while an exact quotient of two fp32 numbers
//    that is not itself a rounding midpoint lies at least ~2^-49 (relative) away from every
//    fp32 midpoint (its distance is (a - m*b)/b, a nonzero multiple of the 49-bit grid of
//    m*b), and it is never a midpoint in the normal range (odd part of m*b >= 2^24 + 1 >
//    odd part of a).  So both round to the same fp32 value; the only exceptions are
//    quotients below 2^-126, which quantize to 0 either way.  
//  * floor(double(r) + 0.5) == floor(r) + (r - floor(r) >= 0.5) exactly in fp32 (r - floor(r)
//    is exact; for r >= 2^23 r is an integer and the fraction is 0).
__device__ __forceinline__ float quotient_f32(float ax, double inv_sf) {
  return (float)((double)ax * inv_sf);
}

__device__ __forceinline__ uint32_t round_half_up_clamp(float r, float maxv) {
  const float fl = floorf(r);
  const float q0 = fl + ((r - fl) >= 0.5f ? 1.0f : 0.0f);  // +inf stays +inf (NaN compare)
  return (r == r) ? (uint32_t)fminf(q0, maxv) : 0u;
}

__device__ __forceinline__ uint32_t quantize_mag_inv(float x, double inv_sf, float maxv) {
  return round_half_up_clamp(quotient_f32(fabsf(x), inv_sf), maxv);
}

__device__ __forceinline__ uint32_t quantize_mag(float x, float sf, float maxv) {
  return quantize_mag_inv(x, 1.0 / (double)sf, maxv);
}

// The float64 instantiation of the reference kernel divides in double.
__device__ __forceinline__ uint32_t quantize_mag(double x, float sf, float maxv) {
  const double t = fabs(x) / (double)sf + 0.5;
  return (t == t) ? (uint32_t)fmin(t, (double)maxv) : 0u;
}

// a2 -- HESE encode: kernels/tr_cuda_kernel.cu:25-55 and bit_utils.hese (bit_utils.py:10-44).
// The reference scans bit windows (b[i+1], b[i], b[i-1]) from bit 63 down:
//   010 -> +2^i (and skip bit i-1), 011 -> +2^(i+1), 110 -> -2^i.
// Closed form on the whole word (checked against bit_utils.hese for every q < 2^17):
//   P = (q & ~(q>>1) & ~(q<<1)) | ((q & ~(q>>1) & (q<<1)) << 1),  N = q & (q>>1) & ~(q<<1)
// so q == P - N with P & N == 0: each set bit of P (N) is a +2^e (-2^e) term and all term
// exponents are distinct.  Terms come out of the reference in strictly decreasing
// exponent order, i.e. the order of the set bits of (P | N) from the top.
__device__ __forceinline__ void hese_masks(uint32_t q, uint32_t& pos, uint32_t& neg) {
  const uint32_t hi = q >> 1;
  const uint32_t lo = q << 1;
  const uint32_t a = q & ~hi;
  pos = (a & ~lo) | ((a & lo) << 1);
  neg = q & hi & ~lo;
}

// a3 for group_size == 1: the greedy of kernels/tr_cuda_kernel.cu:92-116 over a single
// element keeps its k largest-exponent terms.  Drop the (popcount - k) lowest set bits.
__device__ __forceinline__ uint32_t keep_top_terms(uint32_t mask, int k) {
  int drop = __popc(mask) - k;
  while (drop > 0) {
    mask &= mask - 1u;
    --drop;
  }
  return mask;
}

// Largest HESE term count of a bw-bit magnitude: floor(2 (bw + 1) / 3) -- runs "11" followed
// by one zero give two terms per three bits (brute-forced for bw <= 20 in
// tests/test_host.py::test_hese_max_terms).  Peeling the top set bit that many times empties
// any mask, so the fast path below caps its peel count there.
__host__ __device__ constexpr int hese_max_terms(int bw) { return 2 * (bw + 1) / 3; }

// a4 -- value of the kept terms, with the element's sign: kernels/tr_cuda_kernel.cu:112.
__device__ __forceinline__ int32_t kept_value(uint32_t pos, uint32_t neg, uint32_t keep,
                                              bool negative) {
  const int32_t v = (int32_t)(pos & keep) - (int32_t)(neg & keep);
  return negative ? -v : v;
}

__device__ __forceinline__ int32_t tr_value_of_q(uint32_t q, int k, bool negative) {
  uint32_t pos, neg;
  hese_masks(q, pos, neg);
  const uint32_t keep = keep_top_terms(pos | neg, k);
  return kept_value(pos, neg, keep, negative);
}

// One element through quantize -> encode -> keep top k -> signed integer value.
template <typename T>
__device__ __forceinline__ int32_t tr_value_g1(T x, float sf, float maxv, int k) {
  return tr_value_of_q(quantize_mag(x, sf, maxv), k, x < (T)0);
}

// fp32 element with a precomputed inv_sf = RN64(1 / sf) (hoisted out of per-element loops).
__device__ __forceinline__ int32_t tr_value_g1_inv(float x, double inv_sf, float maxv, int k) {
  return tr_value_of_q(quantize_mag_inv(x, inv_sf, maxv), k, x < 0.0f);
}

// Epilogue fast path for 4 values the epilogue has just passed through ReLU (y >= 0, never
// NaN) with 0 < sf < inf (finite, nonzero inv_sf): no sign, no NaN test, and the a1 rounding as
//   q = cvt(min(r, maxv)) + (fract(min(r, maxv)) >= 0.5)
// (exact: floor(r + 0.5) = floor(r) + (r - floor(r) >= 0.5); the clamp keeps +inf out of
// fract, and at the clamp fract(maxv) = 0 since maxv is an integer).  Top-k selection
// without popcount or a divergent loop: peel the highest set bit npeel times (wave-uniform:
// one scalar loop for all 4 values, 3 VALU per peel) and keep what was peeled; once a mask
// is empty its find-first-bit-high is 0xffffffff and the peel clears bit 0 of 0, a no-op.  v[i] == tr_value_g1_inv(y[i], inv_sf, maxv, k) for
// npeel = min(k, hese_max_terms(bw)).
__device__ __forceinline__ void tr_values_relu4(const float y[4], double inv_sf, float maxv,
                                                int npeel, int32_t v[4]) {
  uint32_t pos[4], neg[4], rest[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float r = fminf(quotient_f32(y[i], inv_sf), maxv);
    const uint32_t q = (uint32_t)r + (__builtin_amdgcn_fractf(r) >= 0.5f ? 1u : 0u);
    hese_masks(q, pos[i], neg[i]);
    rest[i] = pos[i] | neg[i];
  }
  for (int p = 0; p < npeel; ++p) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t lz;  // v_ffbh_u32: leading zeros, 0xffffffff for 0 (defined, unlike clz(0))
      asm("v_ffbh_u32 %0, %1" : "=v"(lz) : "v"(rest[i]));
      rest[i] &= ~(0x80000000u >> (lz & 31));
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t keep = (pos[i] | neg[i]) ^ rest[i];
    v[i] = (int32_t)(pos[i] & keep) - (int32_t)(neg[i] & keep);
  }
}

// Peel count of the fast path for code maxv = 2^bw - 1 and k kept terms.
__device__ __forceinline__ int relu_peels(float maxv, int k) {
  const int bw = 32 - __builtin_clz((uint32_t)maxv | 1u);
  return k < hese_max_terms(bw) ? k : hese_max_terms(bw);
}

// Epilogue code table.  On the ReLU fast path (y >= 0, 0 < sf < inf) the next layer's code is
// a function of the quantized magnitude q alone, so each workgroup builds code[q] for q <=
// maxv once in LDS (tr_value_of_q -> code bits) and an epilogue value costs the a1 rounding
// plus one ds_read_u16 instead of the HESE masks, the top-bit peels and the conversion to the
// code format (about 20 VALU per value).  Tables cover bit widths <= 11 (the MFMA code range).
constexpr int kLutMax = 2048;

__device__ __forceinline__ uint32_t relu_q(float y, double inv_sf, float maxv) {
  const float r = fminf(quotient_f32(y, inv_sf), maxv);
  return (uint32_t)r + (__builtin_amdgcn_fractf(r) >= 0.5f ? 1u : 0u);
}

// Epilogue arithmetic of the term-pair kernels (TQ_EPI_F32, default 0: the fp64 fold ships;
// 1 is an A/B build, measured no faster).
//   fold_acc: y = fp32(acc * sc + sh) of the exact integer sum -- with TQ_EPI_F32=1 in fp32
//     (one fma of the int -> fp32 converted sum: (float)acc is itself inexact once |acc| >=
//     2^24, which the int32 sums allow up to 2^31, so the error bound is ~3 ulp of
//     max(|acc sc|, |y|) plus that conversion's half ulp of |acc sc|, still far inside the
//     1e-5 parity bound) instead of fp64 (6 fp64-rate operations per value); every engine uses
//     the same fold, so their outputs stay bit-identical.
//   relu_q_epi: relu_q (q = round(fp32(y / sf)), exact as the reference rounds) from an fp32
//     product y * fp32(1/sf): |r_fast - fp32(y / sf)| <= 3 * 2^-24 r, so the rounded integer
//     can differ only when r_fast lies within that of a half-integer; those values (about
//     one in 4000) take the exact fp64 quotient.  The codes are TR of the stored y either way.
#ifndef TQ_EPI_F32
#define TQ_EPI_F32 0
#endif
#if TQ_EPI_F32
typedef float coef_t;
__device__ __forceinline__ float fold_acc(int acc, float sc, float sh) {
  return fmaf((float)acc, sc, sh);
}
// N values at once: one (rare) exact fallback block for the group
template <int N>
__device__ __forceinline__ void relu_q_epi(const float* y, double inv_sf, float maxv,
                                           uint32_t* q) {
  const float inv = (float)inv_sf;
  bool near = false;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float r = fminf(y[i] * inv, maxv + 1.0f);  // y >= 0, not NaN (after ReLU)
    const float fr = __builtin_amdgcn_fractf(r);
    const uint32_t qi = (uint32_t)r + (fr >= 0.5f ? 1u : 0u);
    q[i] = qi < (uint32_t)maxv ? qi : (uint32_t)maxv;
    near |= fabsf(fr - 0.5f) <= r * 0x1p-21f;
  }
  if (__builtin_expect(near, 0)) {
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = relu_q(y[i], inv_sf, maxv);
  }
}
#else
typedef double coef_t;
__device__ __forceinline__ float fold_acc(int acc, double sc, double sh) {
  return (float)((double)acc * sc + sh);
}
template <int N>
__device__ __forceinline__ void relu_q_epi(const float* y, double inv_sf, float maxv,
                                           uint32_t* q) {
#pragma unroll
  for (int i = 0; i < N; ++i) q[i] = relu_q(y[i], inv_sf, maxv);
}
#endif

// Codes of N epilogue values from the code table lut[q] (q <= maxv).  nonneg: the values
// passed a ReLU / ReLU6 (y >= 0, never NaN).  Otherwise (no activation, swish) the table
// still applies, as TR is odd in its input: TR(y) = sign(y) TR(|y|) (the reference quantizes
// |x| and applies the sign, kernels/tr_cuda_kernel.cu:21-23,112), so the code of y < 0 is the
// table's code of q(|y|) negated -- fp16 sign bit / int16 two's complement, zero stays +0 --
// and a NaN quantizes to q = 0 (code 0), as tr_value_g1_inv has it.
template <int N>
__device__ __forceinline__ void lut_codes(const float* y, double inv_sf, float maxv, int fmt,
                                          bool nonneg, const uint16_t* lut, uint32_t* bits) {
  uint32_t q[N];
  if (nonneg) {
    relu_q_epi<N>(y, inv_sf, maxv, q);
  } else {
    float ay[N];
#pragma unroll
    for (int i = 0; i < N; ++i) ay[i] = y[i] == y[i] ? fabsf(y[i]) : 0.0f;
    relu_q_epi<N>(ay, inv_sf, maxv, q);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    uint32_t v = lut[q[i]];
    if (!nonneg && y[i] < 0.0f && v != 0u)
      v = fmt == 1 /* kCodesF16 */ ? (v ^ 0x8000u) : ((0u - v) & 0xFFFFu);
    bits[i] = v;
  }
}

// Fused-epilogue activation (DwConvArgs relu, tq_act_encode_act): 0 none, 1 ReLU, 2 ReLU6,
// 3 swish y * sigmoid(y) (EfficientNet's MemoryEfficientSwish, with torch's fp32 sigmoid
// 1 / (1 + exp(-y))).  y becomes the value the next layer's codes encode, o the stored value:
// ReLU / ReLU6 keep a NaN in the stored value as torch.relu does (its codes are 0 either way:
// TR(NaN) = 0).
constexpr int kActSwish = 3;

// torch's own fp32 composition, operation for operation: sigmoid as 1 / (1 + expf(-y)) with
// the device library's full-precision expf and an IEEE division (torch's sigmoid kernel),
// then y * sigmoid(y) (MemoryEfficientSwish), so the stored value -- and the codes, TR of
// it -- are the module path's bit for bit (tests/test_gpu_fused_effnet.py).  (Used by the
// depthwise and encode kernels and the direct engine's SWISH instantiation only: a swish
// branch in the shared term-pair epilogue put the unrolled epilogue arrays of the strip and
// register-staged engines into scratch.)
__device__ __forceinline__ float swish_f32(float y) {
  const float s = 1.0f / (1.0f + expf(-y));
  return y * s;
}

__device__ __forceinline__ void act_apply(int act, float& y, float& o) {
  o = y;
  if (act == kActSwish) {
    y = swish_f32(y);
    o = y;
  } else if (act) {
    y = y > 0.0f ? y : 0.0f;
    if (act == 2) y = y < 6.0f ? y : 6.0f;
    o = o != o ? o : y;
  }
}

// True when the activation leaves y >= 0 and never NaN, so the next layer's codes may take
// the ReLU fast path and the code tables.
__host__ __device__ inline bool act_nonneg(int act) { return act == 1 || act == 2; }

// Activation / weight code formats of the term-pair kernels (include/tq.h TQ_CODES_*):
// the same signed integer term sum v stored as int16 (VALU dot2 engine) or as the fp16
// value v (MFMA engine; exact for |v| <= 2048, i.e. bitwidth <= 11).
constexpr int kCodesI16 = 0;
constexpr int kCodesF16 = 1;

__device__ __forceinline__ uint32_t code_bits(int32_t v, int fmt) {
  // |v| <= 2^bitwidth <= 2^14 (max_code_bits), so the int16 -> fp16 conversion
  // (v_cvt_f16_i16, one rounding) equals the int32 -> fp16 one
  return fmt == kCodesF16 ? (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(int16_t)v)
                          : ((uint32_t)v & 0xFFFFu);
}

// code[q] = code bits of TR(q * sf) for q in [0, n) (k >= 0 kept terms), by the threads of a
// workgroup; visible after the caller's next barrier.
__device__ __forceinline__ void lut_build(uint16_t* lut, int n, int k, int fmt, int tid,
                                          int nthreads) {
  for (int q = tid; q < n; q += nthreads)
    lut[q] = (uint16_t)code_bits(tr_value_of_q((uint32_t)q, k, false), fmt);
}

}  // namespace tq
