// Fused ResNet stem on the matrix cores: conv 7x7/2 (3 -> 64, pad 3, no bias) -> eval BN ->
// ReLU -> max-pool 3x3/2 (pad 1) -> fp32 output + the first TR layer's activation codes.
//
// The reference keeps the stem conv a plain fp32 conv (cnn_models/__init__.py:34-36 never
// converts it) followed by bn1 / relu / maxpool (torchvision ResNet.forward) and the first
// TRConv2dLayer's input TR (tr_layer.py:96-99).  Run as library calls that is an fp32 conv
// writing a 256x64x112x112 tensor (822 MB), a pass reading it back, and the pool output; here
// the conv output never leaves the chip: HBM sees the 154 MB input and the pooled outputs.
//
// Near-fp32 arithmetic on fp16 matrix cores ("fp16x2").  Every fp32 value is split exactly
// into two fp16 parts, v = v0 + v1 + e with v0 = RN16(v), v1 = RN16(v - v0) (the remainder is
// exact in fp32), |e| <= 2^-22 |v| while v1 is a normal fp16.  fp16 needs a range: the host
// packs the weights as w * 2^10 (|w| <= 32), and each tile's inputs are scaled in LDS by a
// power of two 2^kx chosen from the tile's max |x| (reduced while staging) so that it lies
// in [2^13, 2^14); the sums are scaled back by 2^-(kx + 10) (exact) before BN.  The products
// x0w0 + x0w1 + x1w0 (3 MFMAs) are exact in fp32 and accumulate in fp32; dropped terms and
// split errors are below ~3 * 2^-22 |x||w| (~7e-7: an fp32 conv's accumulation-order
// differences are ~1e-7, a TF32 conv -- cuDNN's default for convs on Ampere -- ~5e-4).  Input
// values below 2^-17 of their tile's max lose relative precision (fp16 subnormal remainder,
// absolute error <= 2^-25 in scaled units); the test bound 1e-5 * sum |x||w| holds unless a
// whole 7x7 window sits below ~2^-22 of its tile's max.  An earlier split-bf16 version
// (three parts, 6 MFMAs, 2^-25) measured 610 us for the bench batch.
//
// Layout.  Space-to-depth turns the stride-2 7x7 conv into a stride-1 4x4 conv over 12
// channels: the kernel padded to 8x8 (a zero tap in front), s2d pixel (R, C) = input rows
// 2R, 2R+1 x cols 2C, 2C+1 x 3 channels = 12 values; conv pixel (oy, ox) reads s2d rows
// oy-2..oy+1 and cols ox-2..ox+1, so K = 4 x 4 x 12 = 192 in the order (sy, sx, sub_r, sub_c,
// c), and any 8 consecutive K values are 8 consecutive fp32 in an s2d row ([col][12] rows).
//   LDS: weights [2 splits][64 rows of 208 fp16] (53 KB, staged once per workgroup) and
//        the input tile pre-split into two fp16 planes x0 = RN16(x), x1 = RN16(x - x0) of
//        s2d rows [2TP+4][SC][12] each (the split of a value is done once, when its tile is
//        staged, not per fragment read: every value feeds up to 16 taps x 4 Cout blocks)
//   wave = one strip of 16 conv columns (7 pool columns) x 2TP+1 conv rows, four rows at a
//        time; per row 6 K-steps x (4 Cout blocks x 3 split products)
//        v_mfma_f32_16x16x32_f16, each weight fragment read once for the four rows (the
//        kernel is bound by LDS fragment reads: two-row passes read the weights twice as
//        often)
//   epilogue: vertical max over the 3 conv rows of each pool row in registers, horizontal
//        max by lane shuffles (width 16), the strip's 7 pool pixels x 64 channels compacted
//        through LDS (1.8 KB per wave), then BN (fp32 fma, as the stem-tail kernel) + ReLU
//        of each pooled value, contiguous fp32 stores + TR codes, every lane finishing 4
//        channels of <= 2 quads.  Pooling the raw sums first is exact: the weights of
//        channels with a negative BN scale are negated when staged, so BN (with |scale|) and
//        ReLU are non-decreasing in the pooled value and commute with max.  Conv positions in
//        the pool's padding are -inf, as in torch's max-pool.
#include <type_traits>

#include "tq_device.h"
#include "tq_launch.h"

#ifndef STEM_AB
#define STEM_AB 0  // timing-only ablation builds (tools/ab/variant1.sh); 0 = the product kernel
#endif
#ifndef STEM_CARRY
#define STEM_CARRY 1  // 1: a tile's first conv row carried from the tile above (one strip per wave)
#endif
#ifndef STEM_TRACE
#define STEM_TRACE 0  // timing-only builds: per-tile phase stamps of wave 0 (tools/stem_trace.py)
#endif
#ifndef STEM_PF
#define STEM_PF 0  // 1: the next K-step's input slices read during this step's MFMAs
#endif
#ifndef STEM_NRM_MFMA
#define STEM_NRM_MFMA 0  // window norms: 1 the diagonal of an MFMA, 0 v_dot2 on the VALU
                         // (r06: with the fix-up as the tail phase the VALU form is 12-14 us
                         // faster per 256-image call, equal in the two-chunk bench;
                         // profiles/r06_fixup_ab.txt)
#endif
#ifndef STEM_QF32
#define STEM_QF32 0  // 1: the code-table index from an fp32 product (exact fp64 quotient only
                     // near a rounding midpoint); 0: every quotient in fp64 (r06: the fp32
                     // form made the stem 12-18 us slower in the bench, profiles/r06_stem_q_ab.txt)
#endif
#ifndef FIXUP_AB
#define FIXUP_AB 0  // timing-only builds of the fix-up kernel: 1 no sums, 2 no window staging,
                    // 3 the workgroup setup only
#endif
#ifndef FIX_FUSED
#define FIX_FUSED 1  // 1: the exact fix-up as the stem kernel's tail phase; 0: its own launch
#endif
#ifndef STEM_FIXAB
#define STEM_FIXAB 0  // timing-only builds of the fix-up listing: 1 no window norms, 2 no flags
#endif

namespace tq {

#if STEM_TRACE
// [workgroup][tile of its run < 16][top, barrier A passed, barrier B passed, tile done]
// (s_memrealtime ticks, 100 MHz) of the last traced launch
__device__ unsigned long long g_stem_trace[1024 * 16 * 4];
// [workgroup][tile < 16][wave][after the prefetch issue, after pass 0, tile done]
__device__ unsigned long long g_stem_trace_waves[1024 * 16 * 8 * 3];
#endif

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kStemThreads = 512;
constexpr int kStemK = 192;     // s2d K
constexpr int kStemWRow = 208;  // LDS weight row (bf16): 416 B makes the A reads conflict-free
constexpr int kStemWBytes = 2 * 64 * kStemWRow * 2;
constexpr int kStemWExp = 10;   // weights are split as w * 2^10 (tq_ops.pack_stem_weight)
constexpr int kStemXMag = 14;   // a tile's inputs are scaled to max |x| < 2^14
constexpr int kStemDynLds = 160 * 1024 - 1024;  // the rest of the CU's LDS: static arrays

// __shfl_down(v, D, 16) as a DPP row shift (no LDS permute): lane i of each 16-lane row
// reads lane i + D; lanes whose source is past the row end keep their own value.
template <int D>
__device__ __forceinline__ float row_down(float v) {
  const int b = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(b, b, 0x100 + D, 0xf, 0xf, false));
}

// ONE: one strip per wave (nb <= 8 waves: Wo <= 56), the strip's last conv row carried to
// the next tile (STEM_CARRY)
// relu_q (tq_device.h: q = round(fp32(y / sf)), y >= 0, clamped to maxv) from an fp32
// product y * fp32(1 / sf): |r_fast - fp32(y / sf)| <= 3 * 2^-24 r, so the rounded integer
// can differ only when r_fast lies within that of a half-integer; those values (about one in
// 4000) take the exact fp64 quotient (as tq_device.h's TQ_EPI_F32 relu_q_epi)
__device__ __forceinline__ uint32_t stem_relu_q(float y, double inv_sf, float maxv) {
  if (!STEM_QF32) return relu_q(y, inv_sf, maxv);
  const float r = fminf(y * (float)inv_sf, maxv + 1.0f);
  const float fr = __builtin_amdgcn_fractf(r);
  if (__builtin_expect(fabsf(fr - 0.5f) <= r * 0x1p-21f, 0)) return relu_q(y, inv_sf, maxv);
  const uint32_t q = (uint32_t)r + (fr >= 0.5f ? 1u : 0u);
  return q < (uint32_t)maxv ? q : (uint32_t)maxv;
}

// sum of squares of an 8-value fp16 slice, added to acc (v_dot2_f32_f16)
__device__ __forceinline__ float sq8(const f16x8& v, float acc) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const h2 p = {v[2 * i], v[2 * i + 1]};
    acc = __builtin_amdgcn_fdot2(p, p, acc, false);
  }
  return acc;
}

// Exact fix-up of the listed outputs (the FIX stem kernel's tail phase, FIX_FUSED; or one
// launch after the stem, same stream).  Each entry
// names a pool pixel p and a 4-bit mask of channels in quad cq; for each such channel the
// nine conv outputs of its pool window are recomputed exactly -- fp32 x times fp32 w is exact
// in fp64 and a 147-term fp64 sum is within 2^-46 of its magnitude sum, then one rounding to
// fp32 -- and the pooled value goes through the same BN fma, ReLU and code path as the
// stem's epilogue.  Workgroup g walks the entries of stem workgroup g's segment, 7 per wave
// and pass: the wave stages the 7 pool windows' 11 x 11 x 3 input values in LDS (one
// coalesced sweep), then lane 9 slot + j computes window position j from LDS (weights staged
// once per workgroup, fp32 [64][7][22], rows padded for 8-byte pairs), and the slot's max is
// gathered by lane shuffles.
__device__ float g_fix_zero[4];  // static storage: zeros, never written
constexpr int kFixWaves = 8;
constexpr int kFixThreads = 64 * kFixWaves;
constexpr int kFixWRow = 22;                       // floats per weight kernel row (21 + pad)
constexpr int kFixWFloats = 64 * 7 * kFixWRow;     // 9856
constexpr int kFixXRow = 34;                       // floats per window row (33 + pad)
constexpr int kFixXFloats = 11 * kFixXRow;         // per slot
constexpr int kFixEnts = 4096;                     // entries staged in LDS (more: read global)
constexpr int kFixLds = (kFixWFloats + kFixWaves * 7 * kFixXFloats + kFixEnts + kFixWaves * 32) * 4;

// one workgroup's segment (seg, cnt entries) with fix_lds >= kFixLds bytes of dynamic LDS:
// the tail phase of the FIX stem kernel (FIX_FUSED) or the body of stem_fixup_kernel
__device__ __forceinline__ void stem_fixup_run(const PoolArgs& a, const uint32_t* seg, int cnt,
                                               float* fix_lds) {
  float* wl = fix_lds;
  uint32_t* ents = reinterpret_cast<uint32_t*>(fix_lds + kFixWFloats + kFixWaves * 7 * kFixXFloats);
  if (cnt == 0) return;  // (uniform: before the barrier)
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  float* xw = fix_lds + kFixWFloats + wave * 7 * kFixXFloats;
  // weights [c][ky][kx * 3 + ci] from w64 (exact in fp32: they are the fp32 weights), and
  // the segment's entries
  for (int i = tid; i < 64 * 147; i += kFixThreads) {
    const int c = i / 147, k = i - c * 147, ky = k / 21;
    wl[c * 7 * kFixWRow + ky * kFixWRow + (k - ky * 21)] = (float)a.w64[i];
  }
  for (int i = tid; i < cnt && i < kFixEnts; i += kFixThreads) ents[i] = seg[i];
  __syncthreads();
  if (FIXUP_AB == 3) return;
  auto entry = [&](int i) __attribute__((always_inline)) {
    return i < kFixEnts ? ents[i] : seg[i];
  };
  const int slot = lane / 9;
  const int j = lane - 9 * slot;
  const int dy = j / 3, dx = j - 3 * (j / 3);
  const int Hc = a.H / 2, Wc = a.W / 2;

  // The pool windows of pass i0 (input rows 4 py - 5 .. 4 py + 5, columns 4 px - 5 .. 4 px +
  // 5, 363 values each): value e of the pass -> slot e / 363, row, float, so consecutive
  // lanes load consecutive floats of one input row (a wave instruction touches a few cache
  // lines); every lane issues its 40 loads with no branch around a load (positions outside
  // the image read the zero page).  Software-pipelined: a pass's loads are issued before the
  // previous pass computes.  Per slot and pass: [iy0, ix0, element offset of (iy0, ix0)]
  // in the wave's LDS scratch (decoded once by lanes 0..6).
  int* sinfo = reinterpret_cast<int*>(ents + kFixEnts) + wave * 32;
  constexpr int kFixPer = (7 * 363 + 63) / 64;  // 40 values per lane
  float v[kFixPer];
  auto fetch = [&](int i0) __attribute__((always_inline)) {
    const int ns = i0 < cnt ? min(7, cnt - i0) : 0;
    if (lane < ns) {
      const int pp = (int)(entry(i0 + lane) >> 8);  // pool pixel (< 2^24)
      const int px = pp % a.Wo;
      const int t = pp / a.Wo;
      const int py = t % a.Ho, n = t / a.Ho;
      sinfo[4 * lane] = 4 * py - 5;
      sinfo[4 * lane + 1] = 4 * px - 5;
      sinfo[4 * lane + 2] = n;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < kFixPer; ++k) {
      const int e = lane + 64 * k;
      const bool live = e < ns * 363;
      const int sl = live ? e / 363 : 0;
      const int rem = e - 363 * sl, r = rem / 33, f = rem - 33 * r;
      const int iy = sinfo[4 * sl] + r, ix = sinfo[4 * sl + 1] + f / 3;
      const bool ok = live && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const float* sp =
          ok ? a.x + (((int64_t)sinfo[4 * sl + 2] * a.H + iy) * a.W + ix) * 3 + (f - 3 * (f / 3))
             : g_fix_zero;
      v[k] = *sp;
    }
  };
  auto store = [&](int i0) __attribute__((always_inline)) {
    const int ns = min(7, cnt - i0);
#pragma unroll
    for (int k = 0; k < kFixPer; ++k) {
      const int e = lane + 64 * k;
      if (e < ns * 363) {
        const int sl = e / 363, rem = e - 363 * sl, r = rem / 33, f = rem - 33 * r;
        xw[sl * kFixXFloats + r * kFixXRow + f] = v[k];
      }
    }
  };

  int i0 = wave * 7;
  if (FIXUP_AB != 2) fetch(i0);
  for (; i0 < cnt; i0 += kFixWaves * 7) {
    const int ns = min(7, cnt - i0);  // entries of this pass (uniform)
    if (FIXUP_AB != 2) store(i0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    if (FIXUP_AB != 2) fetch(i0 + kFixWaves * 7);  // the next pass's windows in flight
    const bool act = slot < ns;
    const uint32_t ent = act ? entry(i0 + slot) : 0u;
    uint32_t m = ent & 15u;
    const uint32_t pq = ent >> 4;
    const int pp = (int)(pq >> 4);  // pool pixel (< 2^24)
    const int64_t p = pp;
    const int cq = (int)(pq & 15u);
    const int px = pp % a.Wo;
    const int py = (pp / a.Wo) % a.Ho;
    const int oy = 2 * py - 1 + dy, ox = 2 * px - 1 + dx;
    const bool valid = act && oy >= 0 && oy < Hc && ox >= 0 && ox < Wc;
    // this position's window: rows 2 dy .. 2 dy + 6, floats 6 dx .. 6 dx + 20 of each
    const float* xr = xw + (act ? slot : 0) * kFixXFloats + 2 * dy * kFixXRow + 6 * dx;
    while (__ballot(m != 0u)) {  // the wave's entries, one channel each round
      const bool has = m != 0u;
      const int c = 4 * cq + (has ? __builtin_ctz(m) : 0);
      m &= m - 1u;
      const float* wc = wl + c * 7 * kFixWRow;
      double acc0 = 0.0, acc1 = 0.0;
#pragma unroll 1
      for (int ky = 0; ky < (FIXUP_AB == 1 ? 0 : 7); ++ky) {
        const float* xk = xr + ky * kFixXRow;
        const float* wk = wc + ky * kFixWRow;
#pragma unroll
        for (int k = 0; k < 20; k += 2) {
          const float2 xv = *reinterpret_cast<const float2*>(xk + k);
          const float2 wv = *reinterpret_cast<const float2*>(wk + k);
          acc0 = fma((double)xv.x, (double)wv.x, acc0);
          acc1 = fma((double)xv.y, (double)wv.y, acc1);
        }
        acc0 = fma((double)xk[20], (double)wk[20], acc0);
      }
      const double acc = acc0 + acc1;
      float vv = (has && valid) ? (float)(__builtin_signbit(a.scale[c]) ? -acc : acc)
                                : -__builtin_inff();
      // window max on lane 9 slot (the shuffles read lanes of the same slot; lane 63's
      // reads wrap and are unused)
      float vm = vv;
#pragma unroll
      for (int jj = 1; jj < 9; ++jj) vm = fmaxf(vm, __shfl(vv, lane + jj));
      if (has && j == 0) {
        const float y = fmaxf(fmaf(vm, fabsf(a.scale[c]), a.shift[c]), 0.0f);
        a.out[p * 64 + c] = y;
        if (a.codes_a)
          a.codes_a[p * a.cp_a + c] =
              (int16_t)code_bits(tr_value_g1_inv(y, a.inv_a, a.maxv_a, a.k_a), a.fmt_a);
        if (a.codes_b)
          a.codes_b[p * a.cp_b + c] =
              (int16_t)code_bits(tr_value_g1_inv(y, a.inv_b, a.maxv_b, a.k_b), a.fmt_b);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this pass's window reads are done
    __builtin_amdgcn_wave_barrier();     // before the next pass restages the windows
  }
}

__global__ __launch_bounds__(kFixThreads) void stem_fixup_kernel(PoolArgs a, int tp,
                                                                 int tiles) {
  extern __shared__ __attribute__((aligned(16))) float fix_lds[];
  const int g = blockIdx.x;
  const int t_begin = (int)((int64_t)g * tiles / gridDim.x);
  stem_fixup_run(a, a.fix_list + (int64_t)t_begin * tp * a.Wo * 16, (int)a.fix_counts[g],
                 fix_lds);
}
static_assert(kFixThreads == kStemThreads && kFixLds <= kStemDynLds,
              "the fix-up runs as the stem kernel's tail phase in its workgroup and LDS");

// FIX: the exact fix-up's listing (a.fix_list): each conv output's input-window norm is summed
// beside its MFMAs, pooled like the values, and bounds the split conv's error.
template <int TP, int QMAX, bool ONE, bool FIX>
__global__ __launch_bounds__(kStemThreads, 1) void stem_conv_pool_kernel(PoolArgs a, int sc,
                                                                         int nb, int tiles) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds_raw[];
  __shared__ uint32_t tile_max[2];  // max |x| (fp32 bits) of a tile's rows, by tile parity
  __shared__ uint32_t fix_n;        // near-midpoint outputs this workgroup listed (fix-up)
  __shared__ float fix_ew[2][64];   // per side and channel: quotient error per unit norm
  __shared__ float fix_sh[2];       // per side: 2^-23 max |shift| / sf + 2^-30 (flag slack)
  __shared__ float fix_nrm[8][8];   // per wave: pooled window norms^2 of the strip's 7 pixels
  uint16_t* ws = reinterpret_cast<uint16_t*>(lds_raw);
  float* xs = reinterpret_cast<float*>(reinterpret_cast<char*>(lds_raw) + kStemWBytes);
  // per-wave pool staging: 7 pixels x 64 channels fp32 behind the input rows
  float* pb = xs + (2 * TP + 4) * sc * 12 + (threadIdx.x >> 6) * (7 * 64);
  // epilogue code tables behind the pool staging (the launcher sized the LDS for them or
  // cleared lut_a / lut_b); visible after the first barrier
  uint16_t* lut_a = a.lut_a ? reinterpret_cast<uint16_t*>(
                                  xs + (2 * TP + 4) * sc * 12 + (kStemThreads / 64) * (7 * 64))
                            : nullptr;
  uint16_t* lut_b = a.lut_b ? reinterpret_cast<uint16_t*>(
                                  xs + (2 * TP + 4) * sc * 12 + (kStemThreads / 64) * (7 * 64)) +
                                  a.lut_a
                            : nullptr;
  if (lut_a) lut_build(lut_a, a.lut_a, a.k_a, a.fmt_a, threadIdx.x, kStemThreads);
  if (lut_b) lut_build(lut_b, a.lut_b, a.k_b, a.fmt_b, threadIdx.x, kStemThreads);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int i16 = lane & 15;
  const int g = lane >> 4;
  const int Hc = a.H / 2, Wc = a.W / 2;  // conv output
  const int tpi = (a.Ho + TP - 1) / TP;  // tiles per image

  // weights once per workgroup: [2][64][192] fp16 -> rows of kStemWRow, each output channel's
  // row negated where its BN scale is negative (exact), so that every channel's BN is
  // non-decreasing in its (sign-adjusted) conv sum and the max-pool can run before BN
  for (int i = tid; i < 2 * 64 * (kStemK / 8); i += kStemThreads) {
    const int row = i / (kStemK / 8);
    const int ch = i - row * (kStemK / 8);
    u32x4 v = *reinterpret_cast<const u32x4*>(a.wsplit + row * kStemK + ch * 8);
    if (__builtin_signbit(a.scale[row & 63])) v ^= (u32x4)0x80008000u;
    *reinterpret_cast<u32x4*>(ws + row * kStemWRow + ch * 8) = v;
  }
  // BN coefficients (|scale|, shift) of the channels 4 (lane % 16) .. +3 this lane finishes
  float bsc[4], bsh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bsc[i] = fabsf(a.scale[4 * i16 + i]);
    bsh[i] = a.shift[4 * i16 + i];
  }
  // Exact fix-up (FIX): the split conv of channel c at a conv position is within wbound[c] *
  // |x| of the exact sum (|x| the 2-norm of the position's input window; wbound[c] = the
  // relative error bound times |w[c]|_2, Cauchy-Schwarz), so a pooled output whose quotient
  // y / sf lies within that (through BN, with the window norms pooled like the values, +
  // two ulps of slack for the BN fma and the quotient's rounding) of a rounding midpoint is
  // the only kind whose code can differ from the exact conv's; those are listed for
  // stem_fixup_kernel, which recomputes them exactly.
  constexpr bool fix = FIX;
  if (fix && tid < 128) {  // visible after the first barrier
    const int c = tid & 63;
    const float inv = (float)(tid < 64 ? a.inv_a : a.inv_b);
    const float wb = a.wbound[c] * fabsf(a.scale[c]) * 1.00390625f;
    fix_ew[tid >> 6][c] = wb * inv;
    float sh = fabsf(a.shift[c]) * inv;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sh = fmaxf(sh, __shfl_xor(sh, o));
    if (c == 0) fix_sh[tid >> 6] = fmaf(sh, 0x1p-23f, 0x1p-30f);
  }

  // Input staging, software-pipelined across tiles: the next tile's rows are loaded into
  // registers while this tile computes, and written to LDS between the two.  Wave w moves
  // (s2d row, sub row) pairs w, w + 8, ...; lane l float4s l, l + 64, ... of an input row
  // (3W floats).  The s2d halo columns (input columns outside the image) stay zero.
  constexpr int ROWS = 2 * (2 * TP + 4);
  constexpr int RPW = (ROWS + 7) / 8;
  // QMAX float4 per lane and input row: W <= 64 * QMAX * 4 / 3 (3: W <= 256, 4: W <= 340,
  // 6: W <= 512; the launcher checks it)
  const int f4n = 3 * a.W / 4;
  for (int i = tid; i < (2 * TP + 4) * sc * 3; i += kStemThreads)
    reinterpret_cast<float4*>(xs)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 pre[RPW][QMAX];
  auto prefetch = [&](int t) {
    const int tn = t / tpi;
    const int srow0 = 2 * (t - tn * tpi) * TP - 3;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int rid = wave + 8 * r;
      const int ir = 2 * (srow0 + (rid >> 1)) + (rid & 1);
      const bool rok = rid < ROWS && ir >= 0 && ir < a.H;
      const float4* src =
          reinterpret_cast<const float4*>(a.x + ((int64_t)tn * a.H + (rok ? ir : 0)) * a.W * 3);
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        const int idx = lane + 64 * q;
        pre[r][q] = (rok && idx < f4n) ? src[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  // The s2d tile is held pre-split: two fp16 planes x0 = RN16(x), x1 = RN16(x - x0) of the
  // scaled inputs, each [2TP + 4][sc][12] (the bytes of the fp32 tile).  Every input value
  // feeds up to 16 taps x 4 Cout blocks of MFMAs, so splitting it once here instead of per
  // fragment read takes the split's VALU out of the main loop.
  _Float16* xs0 = reinterpret_cast<_Float16*>(xs);
  _Float16* xs1 = xs0 + (2 * TP + 4) * sc * 12;
  auto commit = [&](int kx) {  // rows scaled by 2^kx (exact while no underflow), then split
    auto put2 = [&](int e, float u, float v) {
      const float xu = ldexpf(u, kx), xv = ldexpf(v, kx);
      const _Float16 u0 = (_Float16)xu, v0 = (_Float16)xv;
      const _Float16 u1 = (_Float16)(xu - (float)u0), v1 = (_Float16)(xv - (float)v0);
      typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
      *reinterpret_cast<f16x2*>(xs0 + e) = (f16x2){u0, v0};
      *reinterpret_cast<f16x2*>(xs1 + e) = (f16x2){u1, v1};
    };
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int rid = wave + 8 * r;
      if (rid >= ROWS) continue;
      const int row = (rid >> 1) * sc * 12 + (rid & 1) * 6;
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {
        const int idx = lane + 64 * q;
        if (idx >= f4n) continue;
        // flat input-row float f -> s2d column 3 + f / 6, slot f % 6 of the sub row
        const int f = 4 * idx;
        put2(row + (3 + f / 6) * 12 + f % 6, pre[r][q].x, pre[r][q].y);
        put2(row + (3 + (f + 2) / 6) * 12 + (f + 2) % 6, pre[r][q].z, pre[r][q].w);
      }
    }
  };
  if (tid == 0) {
    tile_max[0] = 0u;
    tile_max[1] = 0u;
    fix_n = 0u;
  }
  // Each workgroup walks a contiguous run of tiles (top to bottom through its images): the
  // 2 TP + 4 s2d rows of a tile overlap the previous tile's by 4, and those halo rows were
  // fetched by this workgroup one tile earlier, so they come from L2 instead of HBM (a
  // strided tile order put vertically adjacent tiles on different XCDs: 1.47x input FETCH).
  const int t_begin = (int)((int64_t)blockIdx.x * tiles / gridDim.x);
  const int t_end = (int)((int64_t)(blockIdx.x + 1) * tiles / gridDim.x);
  if (t_begin < t_end) prefetch(t_begin);
  // this workgroup's segment of the fix-up list: one entry at most per (pool pixel, 4-channel
  // quad) of its tiles
  uint32_t* fix_seg = fix ? a.fix_list + (int64_t)t_begin * TP * a.Wo * 16 : nullptr;
  __syncthreads();

  // fp16 operands need a range: each tile's inputs are scaled by 2^kx so that max |x| <
  // 2^14 (a power of two: exact), and the conv sums are scaled back by 2^-(kx + kStemWExp)
  // before BN.  The tile max is reduced while the rows are still in registers; slot
  // (it & 1) is written before barrier A and read between A and B, the other slot is
  // cleared between A and B for the next tile.
  int it = 0;
  // one strip per wave (Wo <= 56): each wave keeps its strip's last conv row for the next tile
  constexpr bool one = ONE;
  f32x4 carry[4];
  float carry_n = 0.0f;  // (FIX) the carried row's window norm^2
  int prev_tile = -2, prev_kx = 0;
  for (int tile = t_begin; tile < t_end; ++tile, ++it) {
#if STEM_TRACE
    const unsigned long long tr0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int n = tile / tpi;
    const int py0 = (tile - n * tpi) * TP;
    {
      uint32_t lm = 0u;
#pragma unroll
      for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int q = 0; q < QMAX; ++q) {
          lm = max(lm, __float_as_uint(pre[r][q].x) & 0x7fffffffu);
          lm = max(lm, __float_as_uint(pre[r][q].y) & 0x7fffffffu);
          lm = max(lm, __float_as_uint(pre[r][q].z) & 0x7fffffffu);
          lm = max(lm, __float_as_uint(pre[r][q].w) & 0x7fffffffu);
        }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) lm = max(lm, (uint32_t)__shfl_xor((int)lm, off));
      if (lane == 0) atomicMax(&tile_max[it & 1], lm);
    }
    __syncthreads();  // A: the previous tile's s2d rows are no longer read, tile max is final
#if STEM_TRACE
    const unsigned long long tr1 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t mbits = tile_max[it & 1];
    int kx = 0;  // all-zero or non-finite tiles stay unscaled
    if (mbits != 0u && mbits < 0x7f800000u) {
      int e;
      frexpf(__uint_as_float(mbits), &e);  // max |x| in [2^(e-1), 2^e)
      kx = kStemXMag - e;
    }
    const int kback = -(kx + kStemWExp);
    const float unscale = ldexpf(1.0f, -kx);  // (FIX) window norms back to input units
    if (STEM_AB != 3) commit(kx);  // (3: timing only, no input staging)
    if (tid == 0) tile_max[(it + 1) & 1] = 0u;
    __syncthreads();  // B
#if STEM_TRACE
    const unsigned long long tr2 = __builtin_amdgcn_s_memrealtime();
#endif
    if (STEM_AB != 3 && tile + 1 < t_end) prefetch(tile + 1);
#if STEM_TRACE
    const unsigned long long trw0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long trw1 = 0;
#endif

    for (int b = wave; b < nb; b += ONE ? nb : kStemThreads / 64) {
      const int c0 = 14 * b - 1;  // first conv column of the strip
      const int ox = c0 + i16;
      const bool colok = ox >= 0 && ox < Wc;

      // BN + ReLU of conv rows (2*py0 - 1 + rr + r), r < NR, at column ox, channels
      // mb*16 + 4g + i.  Rows in pairs share every weight fragment read (LDS traffic), and
      // the input slices of step ks+1 are read during step ks's MFMAs.
      // the lane's 8-value K slice of step ks at row rr, both split planes (8-byte aligned:
      // slices start at multiples of 4 values)
      typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
      auto load_x = [&](int rr, int ks, f16x8& h0, f16x8& h1) {
        const int j = 4 * ks + g;
        const int sy = j / 6;
        const int off = (j - sy * 6) * 8;
        const int e = ((rr + sy) * sc + (ox + 1)) * 12 + off;
        const f16x4 a0 = *reinterpret_cast<const f16x4*>(xs0 + e);
        const f16x4 b0 = *reinterpret_cast<const f16x4*>(xs0 + e + 4);
        const f16x4 a1 = *reinterpret_cast<const f16x4*>(xs1 + e);
        const f16x4 b1 = *reinterpret_cast<const f16x4*>(xs1 + e + 4);
        h0 = __builtin_shufflevector(a0, b0, 0, 1, 2, 3, 4, 5, 6, 7);
        h1 = __builtin_shufflevector(a1, b1, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      // (FIX) nrm[r]: sum of x0^2 over the input window of conv row r at column ox (scaled
      // units; 0 outside the image): the diagonal of one more MFMA per row and K-step, the
      // slice against itself (D[i][j] = sum_k x_i[k] x_j[k] over the 16 columns i, j)
      auto conv_rows = [&](auto nr_tag, int rr, f32x4 (&y)[4][4], float (&nrm)[4]) {
        constexpr int NR = decltype(nr_tag)::value;
        f32x4 acc[NR][4];
        f32x4 sq[FIX && STEM_NRM_MFMA ? NR : 1];
        float sqv[FIX && !STEM_NRM_MFMA ? NR : 1];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          if constexpr (FIX && STEM_NRM_MFMA) sq[r] = (f32x4)0.0f;
          if constexpr (FIX && !STEM_NRM_MFMA) sqv[r] = 0.0f;
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) acc[r][mb] = (f32x4)0.0f;
        }
        auto mfmas = [&](int ks, const f16x8 (&x0)[NR], const f16x8 (&x1)[NR])
            __attribute__((always_inline)) {
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) {
            const uint16_t* wr = ws + (mb * 16 + i16) * kStemWRow + 32 * ks + 8 * g;
            const f16x8 w0 = *reinterpret_cast<const f16x8*>(wr);
            const f16x8 w1 = *reinterpret_cast<const f16x8*>(wr + 64 * kStemWRow);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
              f32x4 c = acc[r][mb];
#if STEM_AB == 2  // timing only: no MFMA
              asm volatile("" : "+v"(c) : "v"(w0), "v"(w1), "v"(x0[r]), "v"(x1[r]));
#else
              c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, x0[r], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0, x1[r], c, 0, 0, 0);
              c = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1, x0[r], c, 0, 0, 0);
#endif
              acc[r][mb] = c;
            }
          }
        };
#if STEM_PF
        // the next K-step's input slices are read before this step's MFMAs (two register
        // buffers, the K loop unrolled so both stay in registers)
        f16x8 xa0[NR], xa1[NR], xb0[NR], xb1[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) load_x(rr + r, 0, xa0[r], xa1[r]);
#pragma unroll
        for (int ks = 0; ks < kStemK / 32; ks += 2) {
#pragma unroll
          for (int r = 0; r < NR; ++r) load_x(rr + r, ks + 1, xb0[r], xb1[r]);
          mfmas(ks, xa0, xa1);
          if (ks + 2 < kStemK / 32) {
#pragma unroll
            for (int r = 0; r < NR; ++r) load_x(rr + r, ks + 2, xa0[r], xa1[r]);
          }
          mfmas(ks + 1, xb0, xb1);
        }
#else
#pragma unroll 1
        for (int ks = 0; ks < kStemK / 32; ++ks) {
          // (no register double buffer of the input slices: with four rows in flight their
          // loads' latency hides behind the other rows' MFMAs, and the registers are full)
          f16x8 x0[NR], x1[NR];
#pragma unroll
          for (int r = 0; r < NR; ++r) load_x(rr + r, ks, x0[r], x1[r]);
          mfmas(ks, x0, x1);
          if constexpr (FIX && STEM_FIXAB != 1) {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
              if constexpr (STEM_NRM_MFMA)
                sq[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(x0[r], x0[r], sq[r], 0, 0, 0);
              else
                sqv[r] = sq8(x0[r], sqv[r]);
            }
          }
        }
#endif
        // raw (sign-adjusted) sums; conv positions outside the image pool as -inf
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int oy = 2 * py0 - 1 + rr + r;
          const bool ok = colok && oy >= 0 && oy < Hc;
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int i = 0; i < 4; ++i) y[r][mb][i] = ok ? acc[r][mb][i] : -__builtin_inff();
          if constexpr (FIX) {
            float t;
            if constexpr (STEM_NRM_MFMA) {
              // D[i16][i16] sits in lane (i16, i16 / 4), element i16 % 4
              const int e = i16 & 3;
              const float d =
                  e == 0 ? sq[r][0] : e == 1 ? sq[r][1] : e == 2 ? sq[r][2] : sq[r][3];
              t = __shfl(d, i16 + 16 * (i16 >> 2));
            } else {
              t = sqv[r] + __shfl_xor(sqv[r], 16);
              t += __shfl_xor(t, 32);
            }
            nrm[r] = ok ? t : 0.0f;
          }
        }
      };

      // Pool row j = max over conv rows rr = 2j, 2j+1, 2j+2: rows are computed in pairs
      // (2i, 2i+1); row 2i closes pool row i-1 and, with row 2i+1, opens pool row i.
      auto emit_pool = [&](int j, const f32x4 (&run)[4], const f32x4 (&last)[4], float run_n,
                           float last_n) {
        const int py = py0 + j;
        if (STEM_AB == 1) {  // timing only: no pool / BN / stores (every conv sum kept live)
          float keep = 0.0f;
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int i = 0; i < 4; ++i) keep += run[mb][i] + last[mb][i];
          asm volatile("" ::"v"(keep));
          return;
        }
        float m[4][4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = fmaxf(run[mb][i], last[mb][i]);
            const float v1 = row_down<1>(v);
            const float v2 = row_down<2>(v);
            m[mb][i] = fmaxf(fmaxf(v, v1), v2);
          }
        // compact the strip's 7 pool pixels x 64 channels through LDS, then every lane
        // finishes 4 consecutive channels of up to two of the 112 quads: contiguous stores
        // and no TR work on the 9 lanes of each row that hold no pool output
        float mn = 0.0f;  // (FIX) the pool window's largest input-window norm^2
        if constexpr (FIX) {
          const float v = fmaxf(run_n, last_n);
          mn = fmaxf(fmaxf(v, row_down<1>(v)), row_down<2>(v));
        }
        if (py >= a.Ho) return;
        const int q = i16 >> 1;
        if (!(i16 & 1) && i16 <= 12) {
#pragma unroll
          for (int mb = 0; mb < 4; ++mb)
            *reinterpret_cast<f32x4*>(pb + q * 64 + mb * 16 + 4 * g) =
                (f32x4){m[mb][0], m[mb][1], m[mb][2], m[mb][3]};
          if (FIX && g == 0) fix_nrm[wave][q] = mn;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the strip is in LDS
        __builtin_amdgcn_wave_barrier();
        const int npx = min(7, a.Wo - 7 * b);
        const int64_t p0 = ((int64_t)n * a.Ho + py) * a.Wo + 7 * b;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int f = lane + 64 * h;  // quad: pixel f / 16, channels 4 (f % 16) .. +3
          uint32_t ent = 0u;             // fix-up list entry of this quad (0: none)
          if (f < 16 * npx) {
          const int co = 4 * (f & 15);
          const int64_t p = p0 + (f >> 4);
          const f32x4 v4 = *reinterpret_cast<const f32x4*>(pb + 4 * f);
          // BN + ReLU of the pooled sum: both are non-decreasing in it (scale >= 0 after the
          // weight sign flip, fp32 rounding is monotone), so relu(bn(max)) == max(relu(bn))
          // bit for bit -- one BN per pool output instead of one per conv output
          float yv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) yv[i] = fmaxf(fmaf(ldexpf(v4[i], kback), bsc[i], bsh[i]), 0.0f);
          if (STEM_AB == 4) {  // timing only: no stores (values kept live)
            asm volatile("" ::"v"(yv[0]), "v"(yv[1]), "v"(yv[2]), "v"(yv[3]));
          } else {
            *reinterpret_cast<float4*>(a.out + p * 64 + co) =
                make_float4(yv[0], yv[1], yv[2], yv[3]);
          }
#pragma unroll
          for (int side = 0; side < 2; ++side) {
            int16_t* codes = side ? a.codes_b : a.codes_a;
            if (!codes) continue;
            const double inv = side ? a.inv_b : a.inv_a;
            const float maxv = side ? a.maxv_b : a.maxv_a;
            const int k = side ? a.k_b : a.k_a;
            const int cp = side ? a.cp_b : a.cp_a;
            const int fmt = side ? a.fmt_b : a.fmt_a;
            uint32_t v[4];
            const uint16_t* lut = side ? lut_b : lut_a;
            if constexpr (FIX) {  // near-midpoint quotients, listed for the exact fix-up
              uint32_t fm = 0u;
              const f32x4 ew = *reinterpret_cast<const f32x4*>(&fix_ew[side][co]);
              // (+ 0.5 scaled units: the fp16 subnormal remainders of inputs below ~2^-17 of
              // the tile's max, at most 2^-25 each, are not relative to the norm)
              const float wn = (sqrtf(fix_nrm[wave][f >> 4]) + 0.5f) * unscale;
              // Rounding slack in quotient units (r = y / sf; codes differ only if the exact
              // quotients y_split / sf and y_exact / sf straddle a half-integer, and fp32
              // rounding is monotone): this fp32 product vs y_split / sf <= 2^-23 r (1/sf
              // rounded to fp32, the product rounded); the BN fma's rounding on either side
              // <= 2^-23 r together; the correctly rounded conv's own rounding <= 2^-24 |s v|
              // <= 2^-24 (r + |shift| / sf).  In all 5 * 2^-24 r + 2^-24 |shift| / sf, taken
              // as 2^-21 r + 2^-23 max|shift| / sf + 2^-30 (fix_sh).  (Before: a flat 2^-12, enough only for
              // r < ~600 and 2-10x more than needed below ~200.)  Past the clamp every code
              // is maxv's, so a flag there is only a harmless recompute.
              const float invf = (float)inv;
              const float shs = fix_sh[side];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const float r = yv[i] * invf;
                const float slack = fmaf(r, 0x1p-21f, shs);
                if (STEM_FIXAB != 2 &&
                    fabsf(__builtin_amdgcn_fractf(r) - 0.5f) <= fmaf(wn, ew[i], slack))
                  fm |= 1u << i;
              }
              if (fm) ent = ((uint32_t)(p * 16 + (f & 15)) << 4) | (ent & 15u) | fm;
            }
            if (lut) {  // the fast path's codes from the LDS table
#pragma unroll
              for (int i = 0; i < 4; ++i) v[i] = lut[stem_relu_q(yv[i], inv, maxv)];
            } else if (inv > 0.0 && inv <= 1.0e308) {  // yv >= 0 (ReLU, max), 0 < sf < inf
              int32_t t[4];
              tr_values_relu4(yv, inv, maxv, relu_peels(maxv, k), t);
#pragma unroll
              for (int i = 0; i < 4; ++i) v[i] = code_bits(t[i], fmt);
            } else {
#pragma unroll
              for (int i = 0; i < 4; ++i)
                v[i] = code_bits(tr_value_g1_inv(yv[i], inv, maxv, k), fmt);
            }
            if (STEM_AB == 4) {
              asm volatile("" ::"v"(v[0] | (v[1] << 16)), "v"(v[2] | (v[3] << 16)));
            } else {
              *reinterpret_cast<int2*>(codes + p * cp + co) =
                  make_int2((int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)));
            }
          }
          }
          if constexpr (FIX) {  // append the wave's entries to the workgroup's segment
            const uint64_t bal = __ballot(ent != 0u);
            if (bal) {
              uint32_t base = 0u;
              if (lane == 0) base = atomicAdd(&fix_n, (uint32_t)__popcll(bal));
              base = __builtin_amdgcn_readfirstlane(base);
              if (ent) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                fix_seg[base + rank] = ent;
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();  // pb is rewritten by the next pool row
      };

      // conv rows in passes of four (4p .. 4p+3), every weight fragment read once per pass:
      // pass p closes pool row 2p-1 (rows 4p-2, 4p-1 carried in run, and 4p) and pool row 2p
      // (rows 4p .. 4p+2), and carries rows 4p+2, 4p+3; the last conv row 2TP closes pool
      // row TP-1.
      f32x4 run[4];
      f32x4 y[4][4];
      float yn[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // (FIX) the rows' window norms^2
      float run_n = 0.0f;
      if constexpr (STEM_CARRY && one) {
        // conv row 2 py0 - 1 (rr = 0) is the previous tile's last one (rr = 2 TP) when this
        // wave's previous tile was the one above in the same image (a workgroup walks its
        // tiles top to bottom) and scaled its inputs by the same 2^kx (the raw sums are in
        // the tile's scale; equal scales give the same fp16 splits, so the carried sums are
        // bit for bit the ones this tile would compute), -inf above the image, else computed:
        // 2 TP conv rows per tile instead of 2 TP + 1
        if (py0 == 0) {
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) carry[mb] = (f32x4)(-__builtin_inff());
          carry_n = 0.0f;
        } else if (!(tile == prev_tile + 1 && n == prev_tile / tpi && kx == prev_kx)) {
          conv_rows(std::integral_constant<int, 1>(), 0, y, yn);
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) carry[mb] = y[0][mb];
          carry_n = yn[0];
        }
#pragma unroll 1
        for (int p = 0; p < TP / 2; ++p) {
          conv_rows(std::integral_constant<int, 4>(), 4 * p + 1, y, yn);
#if STEM_TRACE
          if (p == 0) trw1 = __builtin_amdgcn_s_memrealtime();
#endif
          // pool row 2p: rr 4p (carry), 4p + 1, 4p + 2; pool row 2p + 1: rr 4p + 2 .. 4p + 4
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) run[mb] = __builtin_elementwise_max(carry[mb], y[0][mb]);
          emit_pool(2 * p, run, y[1], fmaxf(carry_n, yn[0]), yn[1]);
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) run[mb] = __builtin_elementwise_max(y[1][mb], y[2][mb]);
          emit_pool(2 * p + 1, run, y[3], fmaxf(yn[1], yn[2]), yn[3]);
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) carry[mb] = y[3][mb];
          carry_n = yn[3];
        }
        continue;
      } else {
#pragma unroll 1
      for (int p = 0; p < TP / 2; ++p) {
        conv_rows(std::integral_constant<int, 4>(), 4 * p, y, yn);
        if (p > 0) emit_pool(2 * p - 1, run, y[0], run_n, yn[0]);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) run[mb] = __builtin_elementwise_max(y[0][mb], y[1][mb]);
        emit_pool(2 * p, run, y[2], fmaxf(yn[0], yn[1]), yn[2]);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) run[mb] = __builtin_elementwise_max(y[2][mb], y[3][mb]);
        run_n = fmaxf(yn[2], yn[3]);
      }
      conv_rows(std::integral_constant<int, 1>(), 2 * TP, y, yn);
      emit_pool(TP - 1, run, y[0], run_n, yn[0]);
      }
    }
#if STEM_TRACE
    if (threadIdx.x == 0 && blockIdx.x < 1024 && it < 16) {
      unsigned long long* r = g_stem_trace + ((int64_t)blockIdx.x * 16 + it) * 4;
      r[0] = tr0;
      r[1] = tr1;
      r[2] = tr2;
      r[3] = __builtin_amdgcn_s_memrealtime();
    }
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024 && it < 16) {
      unsigned long long* rw =
          g_stem_trace_waves + (((int64_t)blockIdx.x * 16 + it) * 8 + (threadIdx.x >> 6)) * 3;
      rw[0] = trw0;
      rw[1] = trw1;
      rw[2] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    prev_tile = tile;
    prev_kx = kx;
  }
  if (fix) {
    __syncthreads();  // (also: every output store of the workgroup has completed)
    if (tid == 0) a.fix_counts[blockIdx.x] = fix_n;
    // the workgroup's own segment, right after its last tile: no second launch, and the
    // workgroups that finish early overlap it with the others' tiles
    if (FIX_FUSED) stem_fixup_run(a, fix_seg, (int)fix_n, reinterpret_cast<float*>(lds_raw));
  }
}

template <int TP, int QMAX, bool ONE, bool FIX>
hipError_t launch_stem_one(const PoolArgs& a, hipStream_t stream) {
  const int nb = (a.Wo + 6) / 7;
  const int sc = (14 * nb + 5 + 3) / 4 * 4;  // s2d columns -3 .. 14 nb + 1, padded
  int64_t bytes =
      kStemWBytes + (int64_t)(2 * TP + 4) * sc * 12 * 4 + (kStemThreads / 64) * 7 * 64 * 4;
  if (bytes > kStemDynLds) return hipErrorInvalidConfiguration;
  if (3 * a.W / 4 > 64 * QMAX) return hipErrorInvalidValue;  // an input row per lane group
  PoolArgs b = a;  // the epilogue code tables when they fit
  const int64_t lut = ((int64_t)(a.lut_a + a.lut_b) * 2 + 15) / 16 * 16;
  if (bytes + lut <= kStemDynLds) {
    bytes += lut;
  } else {
    b.lut_a = b.lut_b = 0;
  }
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&stem_conv_pool_kernel<TP, QMAX, ONE, FIX>),
        hipFuncAttributeMaxDynamicSharedMemorySize, kStemDynLds);
    if (e == hipSuccess && FIX && !FIX_FUSED)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_fixup_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kFixLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int tiles = a.N * ((a.Ho + TP - 1) / TP);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const int grid = tiles < cus ? tiles : cus;
  if (grid <= 0) return hipSuccess;
  if (a.fix_list && grid * 4 > kStemFixCountsBytes) return hipErrorInvalidValue;
  // the fix-up tail phase reuses the dynamic LDS with its own layout (LDS past the launch's
  // allocation is not the workgroup's: writes there are dropped, reads return zero)
  if (FIX && FIX_FUSED && bytes < kFixLds) bytes = kFixLds;
  stem_conv_pool_kernel<TP, QMAX, ONE, FIX>
      <<<dim3(grid), kStemThreads, (size_t)bytes, stream>>>(b, sc, nb, tiles);
  if (FIX && !FIX_FUSED) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    stem_fixup_kernel<<<dim3(grid), kFixThreads, kFixLds, stream>>>(b, TP, tiles);
  }
  return hipGetLastError();
}

template <int TP, int QMAX>
hipError_t launch_stem_tp(const PoolArgs& a, hipStream_t stream) {
  const int nb = (a.Wo + 6) / 7;
  if (a.fix_list)
    return nb <= kStemThreads / 64 ? launch_stem_one<TP, QMAX, true, true>(a, stream)
                                   : launch_stem_one<TP, QMAX, false, true>(a, stream);
  return nb <= kStemThreads / 64 ? launch_stem_one<TP, QMAX, true, false>(a, stream)
                                 : launch_stem_one<TP, QMAX, false, false>(a, stream);
}

}  // namespace

// Shape contract (checked by the C-ABI layer): 3 input channels, H % 4 == 0, W % 4 == 0,
// conv 7x7/2 pad 3 -> 64 channels, pool 3x3/2 pad 1 -> Ho = H/4, Wo = W/4, Wo <= 112.
// Four pool rows per tile when the input tile fits in LDS (W <= 224: 9 conv rows for 4 pool
// rows), else two (measured 717 vs 793 us for the ResNet-18 bench batch).
hipError_t launch_stem_conv_pool(const PoolArgs& a, hipStream_t stream) {
  static const char* tp = getenv("TQ_STEM_TP");  // A/B override (tools only)
  const bool narrow = 3 * a.W <= 64 * 3 * 4;  // every input row in 3 float4 per lane
  // W > 340: 6 float4 per lane (the 4-float4 form dropped the input columns past 340); such
  // a tile never fits four pool rows in the LDS
  if (3 * a.W > 64 * 4 * 4) return launch_stem_tp<2, 6>(a, stream);
  if (!(tp && atoi(tp) == 2)) {
    const hipError_t e = narrow ? launch_stem_tp<4, 3>(a, stream) : launch_stem_tp<4, 4>(a, stream);
    if (e != hipErrorInvalidConfiguration) return e;
  }
  return narrow ? launch_stem_tp<2, 3>(a, stream) : launch_stem_tp<2, 4>(a, stream);
}

#if STEM_TRACE
extern "C" int tq_stem_trace_waves_read(void* dst, int64_t n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stem_trace_waves), (size_t)n * 8, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int tq_stem_trace_read(void* dst, int64_t n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stem_trace), (size_t)n * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

}  // namespace tq
