// Epilogue building blocks shared by the term-pair conv kernels (VALU dot2 engine,
// tr_conv.hip, and MFMA engine, tr_conv_mfma.hip): both finish EXACT integer term-pair sums
// the same way, so their outputs are bit-identical for the same accumulators.
//
//   y = fp32(double(acc) * ch_scale[c] + ch_shift[c])   (conv scale, bias, folded eval BN)
//     | fp32(double(acc) * scale + bias[c])
//   y += residual (fp32), relu, fp32 store, next TR layers' activation codes
//   (tr_layer.py:96-99 applied to y) in the consumer's code format.  ReLU propagates NaN
//   into the stored value as torch.relu does; the codes of a NaN are 0, as TR(NaN) = 0.
#pragma once

#include <stdlib.h>

#include "tq_device.h"
#include "tq_launch.h"

namespace tq {
namespace {

// Per-channel epilogue coefficients of channels co..co+3: y = acc * sc + sh (fp64).
__device__ __forceinline__ void load_coef(const ConvArgs& a, int co, coef_t sc[4],
                                          coef_t sh[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = co + i < a.Cout;
    if (a.ch_scale) {
      sc[i] = (coef_t)(ok ? a.ch_scale[co + i] : 0.0);
      sh[i] = (coef_t)(ok ? a.ch_shift[co + i] : 0.0);
    } else {
      sc[i] = (coef_t)a.scale;
      sh[i] = (coef_t)((a.bias && ok) ? (double)a.bias[co + i] : 0.0);
    }
  }
}

// Codes of channels co..co+3 of pixel p.  The lane owning the last quad (co + 4 == cout) also
// zeroes the pad channels [cout, cp) (cp = roundup(cout, 8), so at most 4): a consumer
// multiplies them by zero weights, and stale fp16 bits decoding as Inf/NaN would turn 0 * Inf
// into NaN in its fp32 window.
__device__ __forceinline__ void store_codes4(int16_t* codes, int cp, int cout, int64_t p, int co,
                                             const float y[4], double inv_sf, float maxv,
                                             int k, int fmt, bool relu,
                                             const uint16_t* lut = nullptr) {
  uint32_t v[4];
  if (lut) {  // codes from the LDS table (signed values too: tq_device.h lut_codes)
    lut_codes<4>(y, inv_sf, maxv, fmt, relu, lut, v);
  } else if (relu && inv_sf > 0.0 && inv_sf <= 1.0e308) {  // y >= 0, 0 < sf < inf: fast path
    int32_t t[4];
    tr_values_relu4(y, inv_sf, maxv, relu_peels(maxv, k), t);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = code_bits(t[i], fmt);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = code_bits(tr_value_g1_inv(y[i], inv_sf, maxv, k), fmt);
  }
  *reinterpret_cast<int2*>(codes + p * cp + co) =
      make_int2((int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)));
  if (co + 4 == cout && cp > cout) *reinterpret_cast<int2*>(codes + p * cp + co + 4) = make_int2(0, 0);
}

// emit4_nhwc with the residual already loaded (rv = residual[p][co..co+3], or the fused
// downsample's identity, or zeros when there is neither): the epilogue issues every residual
// load of a tile before its first store, so the loads' latency is paid once, not once per
// output quad.  Cout % 4 == 0.
// SWISH: the activation is swish (relu == 3; only the direct engine's SWISH instantiation,
// so the other instantiations' code is unchanged -- a runtime swish branch here put the
// strip and register-staged engines' epilogue arrays in scratch).
template <bool SWISH = false>
__device__ __forceinline__ void emit4_nhwc_res(const ConvArgs& a, int64_t p, int co,
                                               const int acc[4], const coef_t sc[4],
                                               const coef_t sh[4], const float4 rv,
                                               const uint16_t* lut_a = nullptr,
                                               const uint16_t* lut_b = nullptr) {
  float y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = fold_acc(acc[i], sc[i], sh[i]);
  if (a.residual || a.ds_x) {
    y[0] += rv.x;
    y[1] += rv.y;
    y[2] += rv.z;
    y[3] += rv.w;
  }
  float o[4];  // stored value: ReLU keeps NaN like torch.relu; the codes see 0 (TR(NaN) = 0)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = y[i];
    if (SWISH) {
      y[i] = swish_f32(y[i]);
      o[i] = y[i];
    } else if (a.relu) {
      y[i] = y[i] > 0.0f ? y[i] : 0.0f;
      if (a.relu == 2) y[i] = y[i] < 6.0f ? y[i] : 6.0f;  // ReLU6 (MobileNet-V2)
      o[i] = o[i] != o[i] ? o[i] : y[i];
    }
  }
  if (a.out)
    *reinterpret_cast<float4*>(a.out + p * a.Cout + co) = make_float4(o[0], o[1], o[2], o[3]);
  if (a.codes_a) store_codes4(a.codes_a, a.cp_a, a.Cout, p, co, y, a.inv_a, a.maxv_a, a.k_a, a.fmt_a,
                               SWISH ? false : (bool)a.relu, lut_a);
  if (a.codes_b) store_codes4(a.codes_b, a.cp_b, a.Cout, p, co, y, a.inv_b, a.maxv_b, a.k_b, a.fmt_b,
                               SWISH ? false : (bool)a.relu, lut_b);
}

// emit4_nhwc_res for the ResNet executors' form -- ReLU, the code outputs served by their
// tables (a.lut_a, and a.lut_b when codes_b) -- with that form's operations only: the same
// values and stores without the runtime branches (and registers) of the other forms'.
// RELU6: the ReLU6 form (MobileNet-V2's expand convs, epilogue_form 5).
template <bool RELU6 = false>
__device__ __forceinline__ void emit4_relu_lut(const ConvArgs& a, int64_t p, int co,
                                               const int acc[4], const coef_t sc[4],
                                               const coef_t sh[4], const float4 rv,
                                               const uint16_t* lut_a, const uint16_t* lut_b) {
  const float r[4] = {rv.x, rv.y, rv.z, rv.w};
  float y[4], o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    y[i] = fold_acc(acc[i], sc[i], sh[i]);
    if (a.residual || a.ds_x) y[i] += r[i];
    o[i] = y[i];
    y[i] = y[i] > 0.0f ? y[i] : 0.0f;
    if (RELU6) y[i] = y[i] < 6.0f ? y[i] : 6.0f;
    o[i] = o[i] != o[i] ? o[i] : y[i];
  }
  if (a.out)
    *reinterpret_cast<float4*>(a.out + p * a.Cout + co) = make_float4(o[0], o[1], o[2], o[3]);
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    int16_t* codes = side ? a.codes_b : a.codes_a;
    if (side && !codes) break;
    const int cp = side ? a.cp_b : a.cp_a;
    const uint16_t* lut = side ? lut_b : lut_a;
    uint32_t q[4];
    relu_q_epi<4>(y, side ? a.inv_b : a.inv_a, side ? a.maxv_b : a.maxv_a, q);
    uint32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = lut[q[i]];
    *reinterpret_cast<int2*>(codes + p * cp + co) =
        make_int2((int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)));
    if (co + 4 == a.Cout && cp > a.Cout)
      *reinterpret_cast<int2*>(codes + p * cp + co + 4) = make_int2(0, 0);
  }
}

// The identity form (a downsample conv: no activation, no residual, no codes, fp32 output
// only) of emit4_nhwc_res: the fold and the store.
__device__ __forceinline__ void emit4_identity(const ConvArgs& a, int64_t p, int co,
                                               const int acc[4], const coef_t sc[4],
                                               const coef_t sh[4]) {
  *reinterpret_cast<float4*>(a.out + p * a.Cout + co) =
      make_float4(fold_acc(acc[0], sc[0], sh[0]), fold_acc(acc[1], sc[1], sh[1]),
                  fold_acc(acc[2], sc[2], sh[2]), fold_acc(acc[3], sc[3], sh[3]));
}

// The linear form (no activation: a depthwise net's projection conv, optional residual and
// fp32 output, one code output from its table -- signed values, tq_device.h lut_codes) of
// emit4_nhwc_res.
__device__ __forceinline__ void emit4_linear_lut(const ConvArgs& a, int64_t p, int co,
                                                 const int acc[4], const coef_t sc[4],
                                                 const coef_t sh[4], const float4 rv,
                                                 const uint16_t* lut_a) {
  const float r[4] = {rv.x, rv.y, rv.z, rv.w};
  float y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    y[i] = fold_acc(acc[i], sc[i], sh[i]);
    if (a.residual) y[i] += r[i];
  }
  if (a.out)
    *reinterpret_cast<float4*>(a.out + p * a.Cout + co) = make_float4(y[0], y[1], y[2], y[3]);
  uint32_t v[4];
  lut_codes<4>(y, a.inv_a, a.maxv_a, a.fmt_a, false, lut_a, v);
  *reinterpret_cast<int2*>(a.codes_a + p * a.cp_a + co) =
      make_int2((int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)));
  if (co + 4 == a.Cout && a.cp_a > a.Cout)
    *reinterpret_cast<int2*>(a.codes_a + p * a.cp_a + co + 4) = make_int2(0, 0);
}

// The swish form with one table-served code output and nothing else (EfficientNet-b0's
// expand convs: no residual, no fp32 output, no second code output) of emit4_nhwc_res<true>.
__device__ __forceinline__ void emit4_swish_lut(const ConvArgs& a, int64_t p, int co,
                                                const int acc[4], const coef_t sc[4],
                                                const coef_t sh[4], const uint16_t* lut_a) {
  float y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = swish_f32(fold_acc(acc[i], sc[i], sh[i]));
  uint32_t v[4];
  lut_codes<4>(y, a.inv_a, a.maxv_a, a.fmt_a, false, lut_a, v);
  *reinterpret_cast<int2*>(a.codes_a + p * a.cp_a + co) =
      make_int2((int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)));
  if (co + 4 == a.Cout && a.cp_a > a.Cout)
    *reinterpret_cast<int2*>(a.codes_a + p * a.cp_a + co + 4) = make_int2(0, 0);
}

// 4 = emit4_swish_lut's form (the direct engine's swish instantiation picks it: swish_form)
__host__ inline bool swish_lut_form(const ConvArgs& a) {
  const char* env = getenv("TQ_EPI_FAST");
  return !(env && atoi(env) == 0) && (a.Cout & 3) == 0 && !a.ds_x && !a.residual && !a.out &&
         a.codes_a && a.lut_a > 0 && !a.codes_b;
}

// Epilogue form of a conv launch the engines specialise (0 = the generic emit4_nhwc(_res)):
// 1 = ReLU with every code output from its table (emit4_relu_lut), 2 = the identity form
// (emit4_identity), 3 = the linear form with one table-served code output (emit4_linear_lut),
// 5 = form 1 with ReLU6 (emit4_relu_lut<true>) -- 3 and 5 in the direct engine only, the
// others run 0 for them.  TQ_EPI_FAST=0 keeps the generic
// epilogue (tests, A/B).
__host__ inline int epilogue_form(const ConvArgs& a) {
  const char* env = getenv("TQ_EPI_FAST");
  if ((env && atoi(env) == 0) || (a.Cout & 3) || a.ds_x) return 0;
  if (a.relu == 1 && a.codes_a && a.lut_a > 0 && (a.codes_b == nullptr || a.lut_b > 0))
    return 1;
  if (a.relu == 0 && a.out && !a.codes_a && !a.codes_b && !a.residual) return 2;
  if (a.relu == 0 && a.codes_a && a.lut_a > 0 && !a.codes_b) return 3;
  if (a.relu == 2 && a.codes_a && a.lut_a > 0 && (a.codes_b == nullptr || a.lut_b > 0))
    return 5;
  return 0;
}

// Finish channels co..co+3 of output pixel p (channels_last) from exact integer sums:
// one fp64->fp32 rounding, residual add and ReLU in fp32, fp32 store, next layers' TR codes
// (tr_layer.py:96-99 applied to the stored value).
__device__ __forceinline__ void emit4_nhwc(const ConvArgs& a, int64_t p, int co,
                                           const int acc[4], const coef_t sc[4],
                                           const coef_t sh[4], bool vec,
                                           const uint16_t* lut_a = nullptr,
                                           const uint16_t* lut_b = nullptr) {
  float y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = fold_acc(acc[i], sc[i], sh[i]);
  if (a.residual) {
    const float* r = a.residual + p * a.Cout + co;
    if (vec) {
      const float4 rv = *reinterpret_cast<const float4*>(r);
      y[0] += rv.x;
      y[1] += rv.y;
      y[2] += rv.z;
      y[3] += rv.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (co + i < a.Cout) y[i] += r[i];
    }
  }
  float o[4];  // as emit4_nhwc_res: NaN-propagating ReLU for the stored value
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = y[i];
    if (a.relu) {
      y[i] = y[i] > 0.0f ? y[i] : 0.0f;
      if (a.relu == 2) y[i] = y[i] < 6.0f ? y[i] : 6.0f;  // ReLU6 (MobileNet-V2)
      o[i] = o[i] != o[i] ? o[i] : y[i];
    }
  }
  if (a.out) {
    float* dst = a.out + p * a.Cout + co;
    if (vec) {
      *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (co + i < a.Cout) dst[i] = o[i];
    }
  }
  if (a.codes_a) store_codes4(a.codes_a, a.cp_a, a.Cout, p, co, y, a.inv_a, a.maxv_a, a.k_a, a.fmt_a,
                               a.relu, lut_a);
  if (a.codes_b) store_codes4(a.codes_b, a.cp_b, a.Cout, p, co, y, a.inv_b, a.maxv_b, a.k_b, a.fmt_b,
                               a.relu, lut_b);
}

// Epilogue code tables of a conv launch in LDS at `base` (a.lut_a then a.lut_b entries),
// built by the workgroup's threads; the caller's next barrier makes them visible.
__device__ __forceinline__ void conv_luts(const ConvArgs& a, uint16_t* base, uint16_t*& la,
                                          uint16_t*& lb) {
  la = a.lut_a ? base : nullptr;
  lb = a.lut_b ? base + a.lut_a : nullptr;
  const int nt = blockDim.x;
  if (la) lut_build(la, a.lut_a, a.k_a, a.fmt_a, threadIdx.x, nt);
  if (lb) lut_build(lb, a.lut_b, a.k_b, a.fmt_b, threadIdx.x, nt);
}

__host__ __device__ inline int64_t conv_lut_bytes(const ConvArgs& a) {
  return ((int64_t)(a.lut_a + a.lut_b) * 2 + 15) / 16 * 16;
}

// Bijective XCD-aware remap of the block index: blocks are dealt round-robin to the 8 XCDs
// (bid % 8), so hand each XCD a contiguous run of logical work items (neighbouring pixel
// tiles share halo rows, Cout tiles of a pixel tile share its activation tile, both then
// hit one L2).  Placement is a speed choice only.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q8 = nblk >> 3, r8 = nblk & 7, xcd = bid & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

}  // namespace
}  // namespace tq
