// Depthwise term-pair Conv2d (groups == C_in == C_out) for MobileNet-V2 / EfficientNet-b0,
// whose depthwise layers keep (16, 1, 16) settings (cnn_models/__init__.py:57-58): 16-bit
// weight term sums do not fit int16, so weights stay int32 and each product is one
// v_mad_i32_i24 (|v_x| <= 2^14, |v_w| <= 2^16, both inside 24-bit operands; a 7x7 window
// sums to < 2^37 only for 16+14 bits -- the host checks the int32 bound).
//
// One lane per (output pixel, 8 channels): KH*KW 16-byte activation-code loads (NHWC, the
// 8 channels of one tap are contiguous), 8 int32 weights per tap from the [KH*KW][C] weight
// table (L1/L2-resident), exact int32 sums, one rounding in the epilogue.  HBM-bound: the
// activation tile is re-read from cache per tap, the output written once.
// Padding is implicit (any tap outside the input reads 0), so asymmetric "same" padding
// (Conv2dStaticSamePadding) is expressed by pad_top / pad_left and the output size.
#include <stdlib.h>

#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

__device__ int4 g_dw_zero;  // zero-initialised static storage, never written: padding taps

// Operands known to fit 24 signed bits let the compiler emit v_mad_i32_i24 (full rate).
__device__ __forceinline__ int sext24(int v) { return (v << 8) >> 8; }

// Epilogue of output pixel p (image img, in-image index rem), channels c0 .. c0 + CPL - 1,
// from the exact int32 sums: one fp64 -> fp32 rounding, activation, fp32 store and/or next
// codes.  CPL = 4 or 8 channels per lane.
// Epilogue coefficients of channels c0 .. c0 + CPL - 1: y = fold_acc(acc, sc, sh) (pad
// channels: sc = sh = 0, so y = 0).
template <int CPL>
__device__ __forceinline__ void dw_coef(const DwConvArgs& a, int c0, coef_t sc[CPL],
                                        coef_t sh[CPL]) {
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = c0 + i;
    if (a.ch_scale) {  // folded BN
      sc[i] = c < a.C ? (coef_t)a.ch_scale[c] : (coef_t)0;
      sh[i] = c < a.C ? (coef_t)a.ch_shift[c] : (coef_t)0;
    } else {
      sc[i] = c < a.C ? (coef_t)a.scale : (coef_t)0;
      sh[i] = (a.bias && c < a.C) ? (coef_t)(double)a.bias[c] : (coef_t)0;
    }
  }
}

// FAST: the fused executors' two forms with the generic path's operations for that form only
// (its runtime branches and unused stored values cost VALU the kernel is short of):
//   1 = ReLU / ReLU6 (a.relu), the next layer's codes from the table, no fp32 output, C == Cp
//   2 = swish, fp32 output only (EfficientNet-b0: the squeeze-excite branch pools it)
template <int CPL, int FAST = 0>
__device__ __forceinline__ void dw_emit_coef(const DwConvArgs& a, const uint16_t* lut,
                                             int64_t p, int64_t img, int rem, int c0,
                                             const int acc[CPL], const coef_t sc[CPL],
                                             const coef_t sh[CPL]) {
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  float y[CPL];
#pragma unroll
  for (int i = 0; i < CPL; ++i) y[i] = fold_acc(acc[i], sc[i], sh[i]);
  if constexpr (FAST == 1) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      y[i] = y[i] > 0.0f ? y[i] : 0.0f;
      if (a.relu == 2) y[i] = y[i] < 6.0f ? y[i] : 6.0f;
    }
    uint32_t qv[CPL], v[CPL];
    relu_q_epi<CPL>(y, a.inv_c, a.maxv_c, qv);
#pragma unroll
    for (int i = 0; i < CPL; ++i) v[i] = lut[qv[i]];
    int16_t* dst = a.codes + p * a.cp_c + c0;
    if (CPL == 4)
      *reinterpret_cast<uint2*>(dst) =
          make_uint2(v[0] | (v[1 % CPL] << 16), v[2 % CPL] | (v[3 % CPL] << 16));
    else
      *reinterpret_cast<uint32_t*>(dst) = v[0] | (v[1 % CPL] << 16);
    return;
  }
  if constexpr (FAST == 2) {
    float o[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) o[i] = swish_f32(y[i]);
    float* dst = a.out + p * a.C + c0;
    if (CPL == 4)
      *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1 % CPL], o[2 % CPL], o[3 % CPL]);
    else
      *reinterpret_cast<float2*>(dst) = make_float2(o[0], o[1 % CPL]);
    return;
  }
  const bool full = (a.C % CPL) == 0;
  auto store_nhwc = [&](const float (&v)[CPL]) {
    float* dst = a.out + p * a.C + c0;  // NHWC (fused epilogue)
    if (full) {  // a whole chunk inside [0, C), or a pad chunk (nothing to store)
      if (c0 >= a.C) return;
      if (CPL == 2) {
        *reinterpret_cast<float2*>(dst) = make_float2(v[0], v[1 % CPL]);
      } else {
#pragma unroll
        for (int i = 0; i < CPL; i += 4)
          *reinterpret_cast<float4*>(dst + i) =
              make_float4(v[i], v[(i + 1) % CPL], v[(i + 2) % CPL], v[(i + 3) % CPL]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        if (c0 + i < a.C) dst[i] = v[i];
    }
  };
  if (a.relu) {  // ReLU / ReLU6 / swish; the stored value keeps a NaN (torch.relu / hardtanh)
    float o[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) act_apply(a.relu, y[i], o[i]);
    if (a.out) store_nhwc(o);
  }
  if (a.codes) {  // next layer's codes of channels c0 .. c0 + CPL - 1 (cp_c == Cp)
    uint32_t v[CPL];
    if (a.lut_c) {
      uint32_t qv[CPL];
      relu_q_epi<CPL>(y, a.inv_c, a.maxv_c, qv);
#pragma unroll
      for (int i = 0; i < CPL; ++i) v[i] = lut[qv[i]];
    } else {
#pragma unroll
      for (int i = 0; i < CPL; ++i)
        v[i] = code_bits(tr_value_g1_inv(y[i], a.inv_c, a.maxv_c, a.k_c), a.fmt_c);
    }
#pragma unroll
    for (int i = 0; i < CPL; ++i)
      if (c0 + i >= a.C) v[i] = 0u;  // pad channels: zero codes
    if (CPL == 8)
      *reinterpret_cast<uint4*>(a.codes + p * a.cp_c + c0) =
          make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4 % CPL] | (v[5 % CPL] << 16),
                     v[6 % CPL] | (v[7 % CPL] << 16));
    else if (CPL == 4)
      *reinterpret_cast<uint2*>(a.codes + p * a.cp_c + c0) =
          make_uint2(v[0] | (v[1 % CPL] << 16), v[2 % CPL] | (v[3 % CPL] << 16));
    else
      *reinterpret_cast<uint32_t*>(a.codes + p * a.cp_c + c0) = v[0] | (v[1 % CPL] << 16);
  }
  if (a.relu || !a.out) return;
  if (a.out_nhwc) {
    store_nhwc(y);
  } else {
#pragma unroll
    for (int i = 0; i < CPL; ++i)
      if (c0 + i < a.C) a.out[(img * a.C + c0 + i) * HoWo + rem] = y[i];
  }
}

template <int CPL>
__device__ __forceinline__ void dw_emit(const DwConvArgs& a, const uint16_t* lut, int64_t p,
                                        int64_t img, int rem, int c0, const int acc[CPL]) {
  coef_t sc[CPL], sh[CPL];
  dw_coef<CPL>(a, c0, sc, sh);
  dw_emit_coef<CPL>(a, lut, p, img, rem, c0, acc, sc, sh);
}

__device__ __forceinline__ void dw_emit8(const DwConvArgs& a, const uint16_t* lut, int64_t p,
                                         int64_t img, int rem, int c0, const int acc[8]) {
  dw_emit<8>(a, lut, p, img, rem, c0, acc);
}

__global__ __launch_bounds__(256) void dwconv_tp_kernel(DwConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lut[];  // next-layer code table
  if (a.lut_c) {
    lut_build(lut, a.lut_c, a.k_c, a.fmt_c, threadIdx.x, 256);
    __syncthreads();
  }
  const int chunks = a.Cp / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t P = (int64_t)a.N * a.Ho * a.Wo;
  if (t >= P * chunks) return;
  const int64_t p = t / chunks;
  const int c0 = (int)(t - p * chunks) * 8;
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  const int64_t img = p / HoWo;
  const int rem = (int)(p - img * HoWo);
  const int oh = rem / a.Wo;
  const int ow = rem - oh * a.Wo;
  int acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0;
  for (int r = 0; r < a.KH; ++r) {
    const int ih = oh * a.sh - a.ph + r * a.dh;
    if (ih < 0 || ih >= a.H) continue;
    for (int s = 0; s < a.KW; ++s) {
      const int iw = ow * a.sw - a.pw + s * a.dw;
      if (iw < 0 || iw >= a.W) continue;
      const int4 xv =
          *reinterpret_cast<const int4*>(a.x + ((img * a.H + ih) * a.W + iw) * a.Cp + c0);
      const int32_t* wt = a.w + (int64_t)(r * a.KW + s) * a.Cp + c0;
      const int4 w0 = *reinterpret_cast<const int4*>(wt);
      const int4 w1 = *reinterpret_cast<const int4*>(wt + 4);
      const int xs[4] = {xv.x, xv.y, xv.z, xv.w};
      const int ws[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int lo = (int)(short)(xs[i] & 0xFFFF);
        const int hi = xs[i] >> 16;
        acc[2 * i] += lo * sext24(ws[2 * i]);
        acc[2 * i + 1] += hi * sext24(ws[2 * i + 1]);
      }
    }
  }
  dw_emit8(a, a.lut_c ? lut : nullptr, p, img, rem, c0, acc);
}

// Row-blocked variant for KH x KW taps known at compile time (3x3, 5x5, dilation 1): a lane
// owns channels c0 .. c0 + 7 of kDwRows vertically adjacent output pixels, so each tap's
// weights are loaded once for kDwRows outputs and every load of a tap row is issued
// unrolled (no per-tap dependent branch chain).  Lanes run chunk-fastest, then along the
// output row: a wave's loads of one tap cover contiguous NHWC bytes.
template <int KH, int KW, int kDwRows>
__global__ __launch_bounds__(256) void dwconv_tp_rows_kernel(DwConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lut[];  // next-layer code table
  if (a.lut_c) {
    lut_build(lut, a.lut_c, a.k_c, a.fmt_c, threadIdx.x, 256);
    __syncthreads();
  }
  const int chunks = a.Cp / 8;
  const int hb = (a.Ho + kDwRows - 1) / kDwRows;  // row blocks per image
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t lanes = (int64_t)a.N * hb * a.Wo * chunks;
  if (t >= lanes) return;
  int64_t q = t / chunks;
  const int c0 = (int)(t - q * chunks) * 8;
  const int ow = (int)(q % a.Wo);
  q /= a.Wo;
  const int bh = (int)(q % hb);
  const int64_t img = q / hb;
  const int oh0 = bh * kDwRows;
  const int iw0 = ow * a.sw - a.pw;
  int acc[kDwRows][8];
#pragma unroll
  for (int r = 0; r < kDwRows; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[r][i] = 0;
  const int16_t* xb = a.x + img * a.H * a.W * a.Cp + c0;
  // every load is unconditional (taps in the padding read a zero block): all of a tap row's
  // loads issue back to back instead of one branch-guarded round trip per tap (one tap row
  // at a time: unrolling the rows too holds every load in flight, 244+ VGPRs)
#pragma unroll 1
  for (int kr = 0; kr < KH; ++kr) {
#pragma unroll
    for (int ks = 0; ks < KW; ++ks) {
      const int iw = iw0 + ks;
      const bool wok = iw >= 0 && iw < a.W;
      const int32_t* wt = a.w + (int64_t)(kr * KW + ks) * a.Cp + c0;
      const int4 w0 = *reinterpret_cast<const int4*>(wt);
      const int4 w1 = *reinterpret_cast<const int4*>(wt + 4);
      const int ws[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int r = 0; r < kDwRows; ++r) {
        const int ih = (oh0 + r) * a.sh - a.ph + kr;
        const bool ok = wok && ih >= 0 && ih < a.H;
        const int4* src = ok ? reinterpret_cast<const int4*>(
                                   xb + ((int64_t)ih * a.W + iw) * a.Cp)
                             : &g_dw_zero;
        const int4 xv = *src;
        const int xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int lo = (int)(short)(xs[i] & 0xFFFF);
          const int hi = xs[i] >> 16;
          acc[r][2 * i] += lo * sext24(ws[2 * i]);
          acc[r][2 * i + 1] += hi * sext24(ws[2 * i + 1]);
        }
      }
    }
  }
  const uint16_t* l = a.lut_c ? lut : nullptr;
#pragma unroll
  for (int r = 0; r < kDwRows; ++r) {
    const int oh = oh0 + r;
    if (oh >= a.Ho) break;
    const int rem = oh * a.Wo + ow;
    dw_emit8(a, l, (img * a.Ho + oh) * a.Wo + ow, img, rem, c0, acc[r]);
  }
}

// Window-blocked 3x3 depthwise kernel (dilation 1, stride S = 1 or 2): a lane owns CPL
// channels of one output column over R consecutive output rows.  The nine taps' weights stay
// in registers for all R rows, and the (R - 1) S + 3 input rows of the block (each the three
// column taps, CPL codes apiece) are all loaded up front, so every input row is loaded once
// per lane and a lane keeps ~30 loads in flight (the kernel is bound by bytes in flight).
// Taps in the padding read a zero block (unconditional loads).  Lanes run chunk-fastest,
// then along the output row, so a wave's load of one tap covers contiguous NHWC bytes.
template <int S, int R, int CPL>
__global__ __launch_bounds__(256) void dwconv3_slide_kernel(DwConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lut[];  // next-layer code table
  if (a.lut_c) {
    lut_build(lut, a.lut_c, a.k_c, a.fmt_c, threadIdx.x, 256);
    __syncthreads();
  }
  typedef int v4i __attribute__((ext_vector_type(CPL / 2)));  // CPL int16 codes
  const int chunks = a.Cp / CPL;
  const int nrb = (a.Ho + R - 1) / R;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t lanes = (int64_t)a.N * nrb * a.Wo * chunks;
  if (t >= lanes) return;
  int64_t q = t / chunks;
  const int c0 = (int)(t - q * chunks) * CPL;
  const int ow = (int)(q % a.Wo);
  q /= a.Wo;
  const int rb = (int)(q % nrb);
  const int64_t img = q / nrb;
  const int oh0 = rb * R;
  const int iw0 = ow * S - a.pw;
  int w[9][CPL];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int32_t* wt = a.w + (int64_t)k * a.Cp + c0;
#pragma unroll
    for (int i = 0; i < CPL; i += 4) {
      const int4 wv = *reinterpret_cast<const int4*>(wt + i);
      w[k][i] = sext24(wv.x);
      w[k][i + 1] = sext24(wv.y);
      w[k][i + 2] = sext24(wv.z);
      w[k][i + 3] = sext24(wv.w);
    }
  }
  bool cok[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) cok[ks] = iw0 + ks >= 0 && iw0 + ks < a.W;
  const int16_t* xb = a.x + (int64_t)img * a.H * a.W * a.Cp + c0;
  const v4i* zero = reinterpret_cast<const v4i*>(&g_dw_zero);
  auto load_row = [&](int ih, v4i (&dst)[3]) {
    const bool rok = ih >= 0 && ih < a.H;
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const bool ok = rok && cok[ks];
      dst[ks] = *(ok ? reinterpret_cast<const v4i*>(xb + ((int64_t)ih * a.W + iw0 + ks) * a.Cp)
                     : zero);
    }
  };
  const uint16_t* l = a.lut_c ? lut : nullptr;
  const int ih0 = oh0 * S - a.ph;  // first tap row of output row oh0
  // every input row of the block's window is issued up front (NROW x 3 loads in flight per
  // lane: the bytes in flight, not the VALU, bound this kernel), then the rows are consumed
  constexpr int NROW = (R - 1) * S + 3;
  v4i rows[NROW][3];
#pragma unroll
  for (int k = 0; k < NROW; ++k) load_row(ih0 + k, rows[k]);
#pragma unroll
  for (int j = 0; j < R; ++j) {
    int acc[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) acc[i] = 0;
#pragma unroll
    for (int kr = 0; kr < 3; ++kr)
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const v4i xv = rows[j * S + kr][ks];
#pragma unroll
        for (int i = 0; i < CPL / 2; ++i) {
          const int lo = (int)(short)(xv[i] & 0xFFFF);
          const int hi = xv[i] >> 16;
          acc[2 * i] += lo * w[kr * 3 + ks][2 * i];
          acc[2 * i + 1] += hi * w[kr * 3 + ks][2 * i + 1];
        }
      }
    const int oh = oh0 + j;
    if (oh < a.Ho)
      dw_emit<CPL>(a, l, (img * a.Ho + oh) * a.Wo + ow, img, oh * a.Wo + ow, c0, acc);
  }
}

// Streaming K x K depthwise kernel (K = 3 or 5, dilation 1, stride S = 1 or 2).  A lane owns
// CPL channels of one output column over a segment of output rows, walked in blocks of R rows:
// the block's NIN = (R - 1) S + K input rows are in registers (K column taps each), the NEXT
// block's R S new input rows are loaded before the block's MACs and epilogue run, and the
// block's last K - S rows are kept for the next one.  So every input row is loaded once per lane (the
// sliding-window kernel reloads the (3 - S)-row halo of every block), a lane has a block of
// loads in flight for its whole segment instead of one load-then-compute shot, and the
// weights and epilogue coefficients are loaded once per segment.  Same exact int32 sums and
// epilogue as the other depthwise kernels (bit-identical outputs).
template <int K, int S, int R, int CPL, int FAST = 0>
__global__ __launch_bounds__(256) void dwconv_stream_kernel(DwConvArgs a, int seg) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lut[];  // next-layer code table
  if (a.lut_c) {
    lut_build(lut, a.lut_c, a.k_c, a.fmt_c, threadIdx.x, 256);
    __syncthreads();
  }
  constexpr int NIN = (R - 1) * S + K;  // input rows of a block
  constexpr int NEW = R * S;            // rows the next block adds
  constexpr int KEEP = NIN - NEW;       // rows shared with the next block (K - S)
  typedef int v4i __attribute__((ext_vector_type(CPL / 2)));  // CPL int16 codes
  const int chunks = a.Cp / CPL;
  const int nseg = (a.Ho + seg - 1) / seg;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t lanes = (int64_t)a.N * nseg * a.Wo * chunks;
  if (t >= lanes) return;
  int64_t q = t / chunks;
  const int c0 = (int)(t - q * chunks) * CPL;
  const int ow = (int)(q % a.Wo);
  q /= a.Wo;
  const int sg = (int)(q % nseg);
  const int64_t img = q / nseg;
  const int oh_begin = sg * seg;
  const int oh_end = oh_begin + seg < a.Ho ? oh_begin + seg : a.Ho;
  const int iw0 = ow * S - a.pw;
  int w[K * K][CPL];
#pragma unroll
  for (int k = 0; k < K * K; ++k) {
    const int32_t* wt = a.w + (int64_t)k * a.Cp + c0;
    if (CPL == 2) {
      const int2 wv = *reinterpret_cast<const int2*>(wt);
      w[k][0] = sext24(wv.x);
      w[k][1 % CPL] = sext24(wv.y);
    } else {
#pragma unroll
      for (int i = 0; i < CPL; i += 4) {
        const int4 wv = *reinterpret_cast<const int4*>(wt + i);
        w[k][i] = sext24(wv.x);
        w[k][(i + 1) % CPL] = sext24(wv.y);
        w[k][(i + 2) % CPL] = sext24(wv.z);
        w[k][(i + 3) % CPL] = sext24(wv.w);
      }
    }
  }
  coef_t sc[CPL], sh[CPL];
  dw_coef<CPL>(a, c0, sc, sh);
  bool cok[K];
#pragma unroll
  for (int ks = 0; ks < K; ++ks) cok[ks] = iw0 + ks >= 0 && iw0 + ks < a.W;
  const int16_t* xb = a.x + (int64_t)img * a.H * a.W * a.Cp + c0;
  const v4i* zero = reinterpret_cast<const v4i*>(&g_dw_zero);
  // unconditional loads: rows outside the image (or wanted == false) read the zero block
  auto load_row = [&](int ih, bool wanted, v4i (&dst)[K]) {
    const bool rok = wanted && ih >= 0 && ih < a.H;
#pragma unroll
    for (int ks = 0; ks < K; ++ks) {
      const bool ok = rok && cok[ks];
      dst[ks] = *(ok ? reinterpret_cast<const v4i*>(xb + ((int64_t)ih * a.W + iw0 + ks) * a.Cp)
                     : zero);
    }
  };
  const uint16_t* l = a.lut_c ? lut : nullptr;
  int ih0 = oh_begin * S - a.ph;  // first tap row of the block's first output row
  v4i cur[NIN][K];
#pragma unroll
  for (int k = 0; k < NIN; ++k) load_row(ih0 + k, true, cur[k]);
  for (int oh0 = oh_begin; oh0 < oh_end; oh0 += R) {
    v4i nxt[NEW][K];  // the next block's new rows, in flight during this block
    const bool more = oh0 + R < oh_end;
#pragma unroll
    for (int k = 0; k < NEW; ++k) load_row(ih0 + NIN + k, more, nxt[k]);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      int acc[CPL];
#pragma unroll
      for (int i = 0; i < CPL; ++i) acc[i] = 0;
#pragma unroll
      for (int kr = 0; kr < K; ++kr)
#pragma unroll
        for (int ks = 0; ks < K; ++ks) {
          const v4i xv = cur[j * S + kr][ks];
#pragma unroll
          for (int i = 0; i < CPL / 2; ++i) {
            const int lo = (int)(short)(xv[i] & 0xFFFF);
            const int hi = xv[i] >> 16;
            acc[2 * i] += lo * w[kr * K + ks][2 * i];
            acc[2 * i + 1] += hi * w[kr * K + ks][2 * i + 1];
          }
        }
      const int oh = oh0 + j;
      if (oh < oh_end)
        dw_emit_coef<CPL, FAST>(a, l, (img * a.Ho + oh) * a.Wo + ow, img, oh * a.Wo + ow, c0,
                                acc, sc, sh);
    }
#pragma unroll
    for (int k = 0; k < KEEP; ++k)
#pragma unroll
      for (int ks = 0; ks < K; ++ks) cur[k][ks] = cur[NEW + k][ks];
#pragma unroll
    for (int k = 0; k < NEW; ++k)
#pragma unroll
      for (int ks = 0; ks < K; ++ks) cur[KEEP + k][ks] = nxt[k][ks];
    ih0 += NEW;
  }
}

// One streaming-kernel shape with the epilogue form (dw_emit_coef FAST) the arguments allow.
template <int K, int S, int R, int CPL>
void launch_stream(const DwConvArgs& a, dim3 grid, size_t lds, int seg, hipStream_t stream) {
  const bool fast1 = (a.relu == 1 || a.relu == 2) && a.out == nullptr && a.codes != nullptr &&
                     a.lut_c > 0;
  const bool fast2 = a.relu == kActSwish && a.out != nullptr && a.out_nhwc &&
                     a.codes == nullptr && a.C % CPL == 0 && a.Cp == a.C;
  const char* env = getenv("TQ_DW_FAST");  // 0: the generic epilogue (tests, A/B)
  const bool on = !(env && atoi(env) == 0);
  if (on && fast1) dwconv_stream_kernel<K, S, R, CPL, 1><<<grid, 256, lds, stream>>>(a, seg);
  else if (on && fast2) dwconv_stream_kernel<K, S, R, CPL, 2><<<grid, 256, lds, stream>>>(a, seg);
  else dwconv_stream_kernel<K, S, R, CPL, 0><<<grid, 256, lds, stream>>>(a, seg);
}

}  // namespace

hipError_t launch_dwconv_tp(const DwConvArgs& a, hipStream_t stream) {
  const int64_t n = (int64_t)a.N * a.Ho * a.Wo * (a.Cp / 8);
  if (n == 0) return hipSuccess;
  // A/B override (tools only): TQ_DW_ROWS=0 the flat kernel, =4 four rows for 5x5 too;
  // TQ_DW_SLIDE=0 keeps 3x3 convs on the row-blocked kernel, =4 four channels per lane
  static const char* rows_env = getenv("TQ_DW_ROWS");
  const char* slide_env = getenv("TQ_DW_SLIDE");  // read per launch: tests switch it
  const int slide = slide_env ? atoi(slide_env) : 4;
  // the streaming kernel (default for 3x3 stride 1/2): TQ_DW_STREAM=0 falls back to the
  // sliding-window / row-blocked kernels (tests and A/B); =8 / =2 eight (four) / two (one)
  // rows per block at stride 1 (2) instead of the defaults below (A/B)
  const char* stream_env = getenv("TQ_DW_STREAM");
  const int stream_mode = stream_env ? atoi(stream_env) : 1;
  // 5x5 on the streaming kernel (TQ_DW_STREAM5=0: the row-blocked kernel, A/B): EfficientNet-b0
  // depthwise launches 133 -> 103 us average, fused 28.4k -> 29.9k img/s (r03ah)
  const char* s5_env = getenv("TQ_DW_STREAM5");
  const bool s5 = !s5_env || atoi(s5_env) != 0;
  if (stream_mode && a.KH == a.KW && (a.KH == 3 || (a.KH == 5 && s5)) && a.dh == 1 &&
      a.dw == 1 && a.sh == a.sw && (a.sh == 1 || a.sh == 2) && a.Cp % 4 == 0) {
    const int S = a.sh;
    // rows per block: fewer rows, fewer VGPRs, more waves.  Stride 1: 4 rows (168 VGPRs, 3
    // waves per SIMD) on the large maps, 2 below 56 rows; stride 2: 1 row (122 VGPRs, 4
    // waves).  Each 10-20 % faster than 8 / 4 rows (216 / 203 VGPRs, 2 waves) on the
    // MobileNet-V2 shapes (profiles/r03ae_dw_probe.txt, r03af_dw_probe.txt).
    const int R = a.KH == 5 ? (S == 1 && stream_mode == 8 ? 2 : 1)  // 5x5: 1 row (2: A/B)
                : stream_mode == 8 ? (S == 1 ? 8 : 4)
                : stream_mode == 2 ? (S == 1 ? 2 : 1)
                                   : (S == 1 ? (a.Ho >= 56 ? 4 : 2) : 1);
    // segments: enough lanes for about two rounds of 3 waves per SIMD, each lane walking
    // as many R-row blocks as that leaves (one segment = a whole image column if it fits)
    const int cpl = a.KH == 5 ? 2 : 4;  // channels per lane
    const int64_t base = (int64_t)a.N * a.Wo * (a.Cp / cpl);
    const int64_t want = (int64_t)device_cus() * 4 * 3 * 64 * 2;  // 3 waves per SIMD
    const int nblk = (a.Ho + R - 1) / R;
    int64_t nseg = (want + base - 1) / base;
    if (nseg < 1) nseg = 1;
    if (nseg > nblk) nseg = nblk;
    int bps = (int)((nblk + nseg - 1) / nseg);  // blocks per segment
    const char* seg_env = getenv("TQ_DW_SEG");   // tests: force multi-block segments
    if (seg_env && atoi(seg_env) > 0) bps = atoi(seg_env);
    const int seg = bps * R;
    const int64_t lanes = base * ((a.Ho + seg - 1) / seg);
    const dim3 grid((unsigned)((lanes + 255) / 256));
    const size_t lds = (size_t)a.lut_c * 2;
    if (a.KH == 5) {
      // two channels per lane (4-byte loads): the 25 taps' weights of four channels would
      // take 100 VGPRs
      if (S == 2) launch_stream<5, 2, 1, 2>(a, grid, lds, seg, stream);
      else if (R == 2) launch_stream<5, 1, 2, 2>(a, grid, lds, seg, stream);
      else launch_stream<5, 1, 1, 2>(a, grid, lds, seg, stream);
    } else if (S == 2) {
      if (R == 1) launch_stream<3, 2, 1, 4>(a, grid, lds, seg, stream);
      else if (R == 2) launch_stream<3, 2, 2, 4>(a, grid, lds, seg, stream);
      else launch_stream<3, 2, 4, 4>(a, grid, lds, seg, stream);
    } else {
      if (R == 2) launch_stream<3, 1, 2, 4>(a, grid, lds, seg, stream);
      else if (R == 4) launch_stream<3, 1, 4, 4>(a, grid, lds, seg, stream);
      else launch_stream<3, 1, 8, 4>(a, grid, lds, seg, stream);
    }
    return hipGetLastError();
  }
  if (slide && !(rows_env && atoi(rows_env) == 0) && a.KH == 3 && a.KW == 3 && a.dh == 1 &&
      a.dw == 1 && a.sh == a.sw && (a.sh == 1 || a.sh == 2) && a.Cp % slide == 0) {
    // rows per lane: 8 at stride 1 (10 input rows in flight), 4 at stride 2 (9 rows)
    const int R = a.sh == 1 ? 8 : 4;
    const int cpl = slide == 8 ? 8 : 4;
    const int64_t lanes = (int64_t)a.N * ((a.Ho + R - 1) / R) * a.Wo * (a.Cp / cpl);
    const dim3 grid((unsigned)((lanes + 255) / 256));
    const size_t lds = (size_t)a.lut_c * 2;
    if (cpl == 8) {
      if (a.sh == 1) dwconv3_slide_kernel<1, 8, 8><<<grid, 256, lds, stream>>>(a);
      else dwconv3_slide_kernel<2, 4, 8><<<grid, 256, lds, stream>>>(a);
    } else {
      if (a.sh == 1) dwconv3_slide_kernel<1, 8, 4><<<grid, 256, lds, stream>>>(a);
      else dwconv3_slide_kernel<2, 4, 4><<<grid, 256, lds, stream>>>(a);
    }
    return hipGetLastError();
  }
  if (!(rows_env && atoi(rows_env) == 0) && a.dh == 1 && a.dw == 1 &&
      ((a.KH == 3 && a.KW == 3) || (a.KH == 5 && a.KW == 5))) {
    // four output rows per lane for 3x3, two for 5x5 (four would need 180 VGPRs)
    const int rows = a.KH == 3 ? 4 : (rows_env && atoi(rows_env) == 4 ? 4 : 2);
    const int64_t lanes = (int64_t)a.N * ((a.Ho + rows - 1) / rows) * a.Wo * (a.Cp / 8);
    const dim3 grid((unsigned)((lanes + 255) / 256));
    if (a.KH == 3)
      dwconv_tp_rows_kernel<3, 3, 4><<<grid, 256, (size_t)a.lut_c * 2, stream>>>(a);
    else if (rows == 4)
      dwconv_tp_rows_kernel<5, 5, 4><<<grid, 256, (size_t)a.lut_c * 2, stream>>>(a);
    else
      dwconv_tp_rows_kernel<5, 5, 2><<<grid, 256, (size_t)a.lut_c * 2, stream>>>(a);
    return hipGetLastError();
  }
  dwconv_tp_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, (size_t)a.lut_c * 2, stream>>>(a);
  return hipGetLastError();
}

}  // namespace tq
