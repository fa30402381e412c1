// C-ABI entry points of libtq_hip.so (declared in include/tq.h).  Argument validation
// lives here so every kernel can assume its contract; nothing here allocates or syncs, so
// the calls are capturable in a hipGraph.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/tq.h"
#include "tq_device.h"
#include "tq_launch.h"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// Largest bitwidth whose term sums (|v| <= 2^bitwidth) a code format holds exactly.
int max_code_bits(int fmt) { return fmt == TQ_CODES_F16 ? 11 : 14; }

int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return TQ_OK;
  return fail(TQ_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

int check_tr_args(int64_t ndim, const int64_t* shape, float sf, int32_t bitwidth,
                  int32_t group_size, int64_t* B, int64_t* C, int64_t* WH, int64_t* numel) {
  if (ndim < 2 || shape == nullptr)
    return fail(TQ_ERR_INVALID_ARGUMENT, "tr: input must have at least 2 dimensions (got %lld)",
                (long long)ndim);
  int64_t n = 1;
  for (int64_t d = 0; d < ndim; ++d) {
    if (shape[d] < 0) return fail(TQ_ERR_INVALID_ARGUMENT, "tr: negative size");
    n *= shape[d];
  }
  if (!(sf >= 0.0f))
    return fail(TQ_ERR_INVALID_ARGUMENT, "tr: sf must be >= 0 (got %g)", (double)sf);
  if (bitwidth < 0 || bitwidth > tq::kMaxBitwidth)
    return fail(TQ_ERR_UNSUPPORTED, "tr: bitwidth must be in [0, %d] (got %d)",
                tq::kMaxBitwidth, bitwidth);
  if (group_size < 1 || group_size > 32)
    return fail(TQ_ERR_INVALID_ARGUMENT, "tr: group_size must be in [1, 32] (got %d)",
                group_size);
  *B = shape[0];
  *C = shape[1];
  *WH = ndim == 4 ? shape[2] * shape[3] : 1;  // kernels/tr_cuda_kernel.cu:133-141
  *numel = n;
  return TQ_OK;
}

template <typename T>
int tr_impl(const T* in, T* out, int32_t* codes, int64_t ndim, const int64_t* shape, float sf,
            int32_t bitwidth, int32_t group_size, int32_t k, void* stream) {
  int64_t B, C, WH, numel;
  int rc = check_tr_args(ndim, shape, sf, bitwidth, group_size, &B, &C, &WH, &numel);
  if (rc != TQ_OK) return rc;
  if (numel == 0) return TQ_OK;
  if (in == nullptr || out == nullptr)
    return fail(TQ_ERR_INVALID_ARGUMENT, "tr: null tensor pointer");
  // num_keep_terms < 0 runs no selection step in the reference: nothing is kept.
  const int kk = k < 0 ? 0 : k;
  return hip_status(tq::launch_tr<T>(in, out, codes, B, C, WH, numel, sf, bitwidth, group_size,
                                     kk, (hipStream_t)stream),
                    "tr launch");
}

}  // namespace

extern "C" {

const char* tq_version(void) { return "tq-hip 0.1.0 gfx950"; }

const char* tq_last_error(void) { return g_err; }

int tq_sync_faults(uint32_t* count) {
  if (count == nullptr) return fail(TQ_ERR_INVALID_ARGUMENT, "sync_faults: count is null");
  return hip_status(tq::strip_sync_faults(count), "sync_faults");
}

int tq_tr_f32(const float* input, float* output, int64_t ndim, const int64_t* shape, float sf,
              int32_t bitwidth, int32_t group_size, int32_t num_keep_terms, void* stream) {
  return tr_impl<float>(input, output, nullptr, ndim, shape, sf, bitwidth, group_size,
                        num_keep_terms, stream);
}

int tq_tr_f64(const double* input, double* output, int64_t ndim, const int64_t* shape,
              float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms,
              void* stream) {
  return tr_impl<double>(input, output, nullptr, ndim, shape, sf, bitwidth, group_size,
                         num_keep_terms, stream);
}

int tq_tr_encode_f32(const float* input, float* output, int32_t* codes, int64_t ndim,
                     const int64_t* shape, float sf, int32_t bitwidth, int32_t group_size,
                     int32_t num_keep_terms, void* stream) {
  if (codes == nullptr) return fail(TQ_ERR_INVALID_ARGUMENT, "tr_encode: codes is null");
  return tr_impl<float>(input, output, codes, ndim, shape, sf, bitwidth, group_size,
                        num_keep_terms, stream);
}

int tq_act_encode(const float* x, int32_t in_nhwc, int64_t n, int64_t c, int64_t h, int64_t w,
                  float sf, int32_t bitwidth, int32_t num_keep_terms, void* codes, int64_t cp,
                  int32_t fmt, void* stream) {
  if (n < 0 || c < 1 || h < 0 || w < 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode: bad shape");
  if (cp < c || cp % 8 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode: cp must be >= c and a multiple of 8");
  if (fmt != TQ_CODES_I16 && fmt != TQ_CODES_F16)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode: unknown code format %d", fmt);
  if (bitwidth < 0 || bitwidth > max_code_bits(fmt))
    return fail(TQ_ERR_UNSUPPORTED, "act_encode: %s codes need bitwidth <= %d (got %d)",
                fmt == TQ_CODES_F16 ? "fp16" : "int16", max_code_bits(fmt), bitwidth);
  if (!(sf >= 0.0f)) return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode: sf must be >= 0");
  if ((uintptr_t)codes % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode: codes must be 16-byte aligned");
  if (in_nhwc && cp == c && (uintptr_t)x % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode: x must be 16-byte aligned");
  const int kk = num_keep_terms < 0 ? 0 : num_keep_terms;
  return hip_status(tq::launch_act_encode(x, in_nhwc, n, c, h, w, sf, bitwidth, kk,
                                          static_cast<int16_t*>(codes), cp, fmt,
                                          (hipStream_t)stream),
                    "act_encode launch");
}

int tq_act_encode_act(const float* x, int64_t n, int64_t c, int64_t h, int64_t w,
                      const float* ch_scale, const float* ch_shift, const float* gate,
                      int32_t act, float* out, float sf, int32_t bitwidth,
                      int32_t num_keep_terms, void* codes, int64_t cp, int32_t fmt,
                      void* stream) {
  if (n < 0 || c < 1 || h < 0 || w < 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode_act: bad shape");
  if (x == nullptr || codes == nullptr)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode_act: null buffer");
  if (act < 0 || act > tq::kActSwish)
    return fail(TQ_ERR_INVALID_ARGUMENT,
                "act_encode_act: act must be 0 (none), 1 (ReLU), 2 (ReLU6) or 3 (swish)");
  if ((ch_scale == nullptr) != (ch_shift == nullptr))
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode_act: ch_scale and ch_shift go together");
  if (cp < c || cp % 8 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode_act: cp must be >= c and a multiple of 8");
  if (fmt != TQ_CODES_I16 && fmt != TQ_CODES_F16)
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode_act: unknown code format %d", fmt);
  if (bitwidth < 0 || bitwidth > max_code_bits(fmt))
    return fail(TQ_ERR_UNSUPPORTED, "act_encode_act: codes need bitwidth <= %d (got %d)",
                max_code_bits(fmt), bitwidth);
  if (!(sf > 0.0f && sf <= 3.402823466e38f))
    return fail(TQ_ERR_INVALID_ARGUMENT, "act_encode_act: sf must be finite and > 0");
  if ((uintptr_t)codes % 16 != 0 || (uintptr_t)x % 16 != 0 || (uintptr_t)out % 16 != 0 ||
      (uintptr_t)ch_scale % 16 != 0 || (uintptr_t)ch_shift % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT,
                "act_encode_act: x, out, codes, ch_scale, ch_shift must be 16-byte aligned");
  const int kk = num_keep_terms < 0 ? 0 : num_keep_terms;
  return hip_status(tq::launch_act_encode_act(x, ch_scale, ch_shift, gate, act, out, n, c, h,
                                              w, sf, bitwidth, kk,
                                              static_cast<int16_t*>(codes), cp, fmt,
                                              (hipStream_t)stream),
                    "act_encode_act launch");
}

int tq_se_gate_f32(const float* x_sq, int64_t n, int64_t c, const int32_t* w_r, int64_t cse,
                   double scale_r, const float* b_r, float sf_r, int32_t bits_r,
                   int32_t terms_r, const int32_t* w_e_t, double scale_e, const float* b_e,
                   float sf_e, int32_t bits_e, int32_t terms_e, float* gate, void* stream) {
  if (n < 0 || c < 1 || cse < 1 || c > (1 << 20) || cse > (1 << 20))
    return fail(TQ_ERR_INVALID_ARGUMENT, "se_gate: bad shape");
  if (n > 0 && (x_sq == nullptr || w_r == nullptr || w_e_t == nullptr || gate == nullptr))
    return fail(TQ_ERR_INVALID_ARGUMENT, "se_gate: null buffer");
  if (bits_r < 0 || bits_r > 14 || bits_e < 0 || bits_e > 14)
    return fail(TQ_ERR_UNSUPPORTED, "se_gate: activation bitwidths must be <= 14");
  if (!(sf_r >= 0.0f) || !(sf_e >= 0.0f))
    return fail(TQ_ERR_INVALID_ARGUMENT, "se_gate: sf must be >= 0");
  const int64_t cpr = (c + 7) / 8 * 8;
  if ((cpr + cse) * 4 > 64 * 1024)
    return fail(TQ_ERR_UNSUPPORTED, "se_gate: channels too many for one workgroup's LDS");
  tq::SeGateArgs a;
  a.x_sq = x_sq;
  a.N = (int)n;
  a.C = (int)c;
  a.w_r = w_r;
  a.Cse = (int)cse;
  a.Cpr = (int)cpr;
  a.scale_r = scale_r;
  a.bias_r = b_r;
  a.inv_r = 1.0 / (double)sf_r;
  a.maxv_r = (float)((1u << bits_r) - 1u);
  a.k_r = terms_r < 0 ? 0 : terms_r;
  a.w_e_t = w_e_t;
  a.scale_e = scale_e;
  a.bias_e = b_e;
  a.inv_e = 1.0 / (double)sf_e;
  a.maxv_e = (float)((1u << bits_e) - 1u);
  a.k_e = terms_e < 0 ? 0 : terms_e;
  a.gate = gate;
  return hip_status(tq::launch_se_gate(a, (hipStream_t)stream), "se_gate launch");
}

int64_t tq_conv2d_cout_align(void) { return 128; }

int32_t tq_conv2d_num_configs(void) { return tq::conv_num_configs(); }

int32_t tq_conv2d_mfma_num_configs(void) { return tq::conv_mfma_num_configs(); }

int64_t tq_conv2d_workspace_bytes(int64_t pixels, int64_t cout) {
  return tq::conv_workspace_bytes(pixels, cout);
}

}  // extern "C"

namespace {

int conv_common(const int16_t* act_codes, int64_t n, int64_t h, int64_t w, int64_t cp,
                const int16_t* w_codes, int64_t cout, int64_t kh, int64_t kw, int64_t kp,
                int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                int64_t dil_h, int64_t dil_w, double scale, const float* bias, float* out,
                int64_t ho, int64_t wo, tq::ConvArgs* a) {
  if (n < 0 || h < 1 || w < 1 || cout < 1 || kh < 1 || kw < 1)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: bad shape");
  if (cp < 8 || cp % 8 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: cp must be a positive multiple of 8");
  if (kp % 32 != 0 || kp < kh * kw * cp)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: kp must be a multiple of 32 >= kh*kw*cp");
  if (stride_h < 1 || stride_w < 1 || dil_h < 1 || dil_w < 1 || pad_h < 0 || pad_w < 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: bad stride/padding/dilation");
  const int64_t eho = (h + 2 * pad_h - dil_h * (kh - 1) - 1) / stride_h + 1;
  const int64_t ewo = (w + 2 * pad_w - dil_w * (kw - 1) - 1) / stride_w + 1;
  if (ho != eho || wo != ewo || ho < 1 || wo < 1)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: output size %lldx%lld, expected %lldx%lld",
                (long long)ho, (long long)wo, (long long)eho, (long long)ewo);
  if ((uintptr_t)act_codes % 16 != 0 || (uintptr_t)w_codes % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: code buffers must be 16-byte aligned");
  if (n * h * w * cp >= (int64_t)1 << 40 || cout > (1 << 24) || kp > (1 << 24))
    return fail(TQ_ERR_UNSUPPORTED, "conv2d: problem too large");
  *a = tq::ConvArgs();
  a->x = act_codes;
  a->w = w_codes;
  a->bias = bias;
  a->out = out;
  a->P = n * ho * wo;
  a->N = (int)n;
  a->H = (int)h;
  a->W = (int)w;
  a->Cp = (int)cp;
  a->Cout = (int)cout;
  a->KH = (int)kh;
  a->KW = (int)kw;
  a->sh = (int)stride_h;
  a->sw = (int)stride_w;
  a->ph = (int)pad_h;
  a->pw = (int)pad_w;
  a->dh = (int)dil_h;
  a->dw = (int)dil_w;
  a->Ho = (int)ho;
  a->Wo = (int)wo;
  a->Kp = (int)kp;
  a->scale = scale;
  return TQ_OK;
}

int code_target(const void* codes, int64_t cp, float sf, int32_t bits, int32_t terms,
                int32_t fmt, int64_t cout, const char* which) {
  if (codes == nullptr) return TQ_OK;
  // the epilogue zeroes the pad channels [cout, cp) only up to the next multiple of 8
  // (tq_epilogue.h store_codes4), so a wider code row would keep stale pad codes
  if (cp != (cout + 7) / 8 * 8 || (uintptr_t)codes % 8 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d epilogue: codes_%s needs cp == roundup(cout, "
                "8) and 8-byte alignment", which);
  if (fmt != TQ_CODES_I16 && fmt != TQ_CODES_F16)
    return fail(TQ_ERR_INVALID_ARGUMENT, "codes_%s: unknown code format %d", which, fmt);
  if (bits < 0 || bits > max_code_bits(fmt))
    return fail(TQ_ERR_UNSUPPORTED, "conv2d epilogue: codes_%s bitwidth must be <= %d", which,
                max_code_bits(fmt));
  if (!(sf >= 0.0f))
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d epilogue: codes_%s sf must be >= 0", which);
  return TQ_OK;
}

// Fill the fused-epilogue fields of `a` from `epi` (shared by both conv engines).
// Entries of an epilogue code table (tq_device.h kLutMax) for one code target: maxv + 1 when
// 0 < sf < inf and maxv < kLutMax (and, where `relu` is required, the values are
// non-negative), else 0 (the kernels compute the codes).  The conv engines' epilogues take
// the table for signed values too (tq_device.h lut_codes); the depthwise kernel only after
// ReLU / ReLU6.  TQ_LUT=0 turns the tables off (A/B, tools only).
int lut_entries(bool codes, bool relu, double inv, float maxv) {
  const char* env = getenv("TQ_LUT");  // read per call: tests switch it
  if (env && atoi(env) == 0) return 0;
  if (!codes || !relu || !(inv > 0.0 && inv <= 1.0e308)) return 0;
  const int n = (int)maxv + 1;
  return n <= tq::kLutMax ? n : 0;
}

int apply_epilogue(const tq_conv_epilogue* epi, int64_t cout, float* out, int num_configs,
                   tq::ConvArgs* a) {
  if (cout % 4 != 0)
    return fail(TQ_ERR_UNSUPPORTED, "conv2d fused epilogue needs cout %% 4 == 0");
  if ((epi->ch_scale == nullptr) != (epi->ch_shift == nullptr))
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: ch_scale and ch_shift go together");
  if (out == nullptr && epi->codes_a == nullptr && epi->codes_b == nullptr)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: no output requested");
  if ((out && (uintptr_t)out % 16) || (epi->residual && (uintptr_t)epi->residual % 16))
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: out/residual must be 16-byte aligned");
  int rc = code_target(epi->codes_a, epi->cp_a, epi->sf_a, epi->bits_a, epi->terms_a,
                       epi->fmt_a, cout, "a");
  if (rc != TQ_OK) return rc;
  rc = code_target(epi->codes_b, epi->cp_b, epi->sf_b, epi->bits_b, epi->terms_b, epi->fmt_b,
                   cout, "b");
  if (rc != TQ_OK) return rc;
  a->ch_scale = epi->ch_scale;
  a->ch_shift = epi->ch_shift;
  a->residual = epi->residual;
  if (epi->relu < 0 || epi->relu > tq::kActSwish)
    return fail(TQ_ERR_INVALID_ARGUMENT,
                "conv2d: relu must be 0 (none), 1 (ReLU), 2 (ReLU6) or 3 (swish)");
  a->relu = epi->relu;
  a->codes_a = epi->codes_a;
  a->cp_a = (int)epi->cp_a;
  a->sf_a = epi->sf_a;
  a->inv_a = 1.0 / (double)epi->sf_a;
  a->maxv_a = (float)((1u << (epi->codes_a ? epi->bits_a : 0)) - 1u);
  a->k_a = epi->terms_a < 0 ? 0 : epi->terms_a;
  a->fmt_a = epi->fmt_a;
  a->codes_b = epi->codes_b;
  a->cp_b = (int)epi->cp_b;
  a->sf_b = epi->sf_b;
  a->inv_b = 1.0 / (double)epi->sf_b;
  a->maxv_b = (float)((1u << (epi->codes_b ? epi->bits_b : 0)) - 1u);
  a->k_b = epi->terms_b < 0 ? 0 : epi->terms_b;
  a->fmt_b = epi->fmt_b;
  a->lut_a = lut_entries(a->codes_a != nullptr, true, a->inv_a, a->maxv_a);
  a->lut_b = lut_entries(a->codes_b != nullptr, true, a->inv_b, a->maxv_b);
  if (epi->config < 0 || epi->config > num_configs || epi->split_k < -1 || epi->split_k > 64)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: bad config/split_k");
  if (epi->workspace && (uintptr_t)epi->workspace % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: workspace must be 16-byte aligned");
  if (epi->ds_codes) {
    if (epi->residual)
      return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: a fused downsample replaces the residual");
    if (epi->ds_w_codes == nullptr || epi->ds_scale == nullptr || epi->ds_shift == nullptr)
      return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: fused downsample needs weights and coefficients");
    if (epi->ds_cp < 64 || epi->ds_cp % 64 != 0 || epi->ds_stride < 1 || epi->ds_h < 1 ||
        epi->ds_w < 1)
      return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: bad fused downsample shape");
    if ((epi->ds_h - 1) / epi->ds_stride + 1 != a->Ho ||
        (epi->ds_w - 1) / epi->ds_stride + 1 != a->Wo)
      return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: fused downsample output size mismatch");
    if ((uintptr_t)epi->ds_codes % 16 || (uintptr_t)epi->ds_w_codes % 16)
      return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: fused downsample codes must be 16-byte aligned");
    if ((int64_t)a->N * epi->ds_h * epi->ds_w * epi->ds_cp >= (int64_t)1 << 40)
      return fail(TQ_ERR_UNSUPPORTED, "conv2d: fused downsample input too large");
    if (epi->split_k > 1 || epi->split_k < 0)
      return fail(TQ_ERR_UNSUPPORTED, "conv2d: a fused downsample runs data-parallel only");
    a->ds_x = reinterpret_cast<const int16_t*>(epi->ds_codes);
    a->ds_w = reinterpret_cast<const int16_t*>(epi->ds_w_codes);
    a->ds_scale = epi->ds_scale;
    a->ds_shift = epi->ds_shift;
    a->ds_H = (int)epi->ds_h;
    a->ds_W = (int)epi->ds_w;
    a->ds_Cp = (int)epi->ds_cp;
    a->ds_s = (int)epi->ds_stride;
  }
  a->config = epi->config;
  a->splits = epi->split_k;
  a->ws = epi->workspace;
  a->ws_bytes = epi->workspace ? epi->workspace_bytes : 0;
  return TQ_OK;
}

}  // namespace

extern "C" {

int tq_conv2d_termpair(const int16_t* act_codes, int64_t n, int64_t h, int64_t w, int64_t cp,
                       const int16_t* w_codes, int64_t cout, int64_t kh, int64_t kw, int64_t kp,
                       int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                       int64_t dil_h, int64_t dil_w, double scale, const float* bias,
                       float* out, int64_t ho, int64_t wo, int32_t out_nhwc, void* stream) {
  tq::ConvArgs a;
  int rc = conv_common(act_codes, n, h, w, cp, w_codes, cout, kh, kw, kp, stride_h, stride_w,
                       pad_h, pad_w, dil_h, dil_w, scale, bias, out, ho, wo, &a);
  if (rc != TQ_OK) return rc;
  if (out == nullptr) return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: out is null");
  return hip_status(tq::launch_conv2d_tp(a, out_nhwc, (hipStream_t)stream), "conv2d launch");
}

int tq_conv2d_termpair_fused(const int16_t* act_codes, int64_t n, int64_t h, int64_t w,
                             int64_t cp, const int16_t* w_codes, int64_t cout, int64_t kh,
                             int64_t kw, int64_t kp, int64_t stride_h, int64_t stride_w,
                             int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w,
                             double scale, const float* bias, float* out, int64_t ho,
                             int64_t wo, const tq_conv_epilogue* epi, void* stream) {
  tq::ConvArgs a;
  int rc = conv_common(act_codes, n, h, w, cp, w_codes, cout, kh, kw, kp, stride_h, stride_w,
                       pad_h, pad_w, dil_h, dil_w, scale, bias, out, ho, wo, &a);
  if (rc != TQ_OK) return rc;
  if (epi == nullptr) return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: epilogue is null");
  if (epi->ds_codes)
    return fail(TQ_ERR_UNSUPPORTED, "conv2d: a fused downsample needs the fp16 (MFMA) entry");
  rc = apply_epilogue(epi, cout, out, tq::conv_num_configs(), &a);
  if (rc != TQ_OK) return rc;
  if (a.relu == tq::kActSwish)
    return fail(TQ_ERR_UNSUPPORTED, "conv2d: the swish epilogue needs the fp16 (MFMA) entry");
  return hip_status(tq::launch_conv2d_tp(a, 1, (hipStream_t)stream), "conv2d launch");
}

int tq_conv2d_termpair_f16(const uint16_t* act_codes, int64_t n, int64_t h, int64_t w,
                           int64_t cp, const uint16_t* w_codes, int64_t cout, int64_t kh,
                           int64_t kw, int64_t kp, int64_t stride_h, int64_t stride_w,
                           int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w,
                           double scale, const float* bias, float* out, int64_t ho, int64_t wo,
                           int32_t out_nhwc, int32_t kc_steps, int32_t kc_chunk,
                           const tq_conv_epilogue* epi, void* stream) {
  tq::ConvArgs a;
  int rc = conv_common(reinterpret_cast<const int16_t*>(act_codes), n, h, w, cp,
                       reinterpret_cast<const int16_t*>(w_codes), cout, kh, kw, kp, stride_h,
                       stride_w, pad_h, pad_w, dil_h, dil_w, scale, bias, out, ho, wo, &a);
  if (rc != TQ_OK) return rc;
  if (kp % 64 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_f16: kp must be a multiple of 64");
  if (kc_steps < 0) return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_f16: kc_steps must be >= 0");
  a.kc_steps = kc_steps;
  // chunk-major window: n consecutive taps of one chunk span (n - 1) * (cp / 64) + 1 packed
  // K-steps, so the conservative derivation keeps them inside one kc_steps window
  const int64_t nch = cp / 64 > 0 ? cp / 64 : 1;
  a.kc_chunk = kc_chunk >= 0 ? kc_chunk : (kc_steps > 0 ? (int)((kc_steps - 1) / nch + 1) : 0);
  if (epi == nullptr) {
    if (out == nullptr) return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d: out is null");
  } else {
    if (!out_nhwc)
      return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_f16: the fused epilogue is channels_last");
    if (epi->split_k != 0 && epi->split_k != 1 && epi->split_k != -1)
      return fail(TQ_ERR_UNSUPPORTED, "conv2d_f16: split_k must be 0, 1 or -1");
    rc = apply_epilogue(epi, cout, out, tq::conv_mfma_num_configs(), &a);
    if (rc != TQ_OK) return rc;
    if (a.ds_x && (a.Cp % 64 != 0 || kh * kw > 64))
      return fail(TQ_ERR_UNSUPPORTED, "conv2d_f16: a fused downsample needs cp %% 64 == 0");
    if (a.relu == tq::kActSwish && !(a.Cp % 64 == 0 || kh * kw == 1))
      return fail(TQ_ERR_UNSUPPORTED,
                  "conv2d_f16: the swish epilogue runs on the direct engine (1x1 or cp %% 64 == 0)");
  }
  return hip_status(tq::launch_conv2d_mfma(a, out_nhwc, (hipStream_t)stream),
                    "conv2d_f16 launch");
}

static int dw_impl(const int16_t* act_codes, int64_t n, int64_t h, int64_t w, int64_t c,
                   int64_t cp, const int32_t* w_codes, int64_t kh, int64_t kw,
                   int64_t stride_h, int64_t stride_w, int64_t pad_top, int64_t pad_left,
                   int64_t dil_h, int64_t dil_w, double scale, const float* bias, float* out,
                   int64_t ho, int64_t wo, int32_t out_nhwc, const tq_dw_epilogue* epi,
                   void* stream) {
  if (n < 0 || h < 1 || w < 1 || c < 1 || kh < 1 || kw < 1 || ho < 1 || wo < 1)
    return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: bad shape");
  if (cp < c || cp % 8 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: cp must be >= c and a multiple of 8");
  if (stride_h < 1 || stride_w < 1 || dil_h < 1 || dil_w < 1 || pad_top < 0 || pad_left < 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: bad stride/padding/dilation");
  if ((uintptr_t)act_codes % 16 != 0 || (uintptr_t)w_codes % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: code buffers must be 16-byte aligned");
  if (out_nhwc && c % 8 == 0 && (uintptr_t)out % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: out must be 16-byte aligned");
  if (n * h * w * cp >= (int64_t)1 << 40 || kh * kw > 4096)
    return fail(TQ_ERR_UNSUPPORTED, "dwconv2d: problem too large");
  if (out == nullptr && (epi == nullptr || epi->codes == nullptr))
    return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: out is null");
  tq::DwConvArgs a = tq::DwConvArgs();
  a.x = act_codes;
  a.w = w_codes;
  a.bias = bias;
  a.out = out;
  a.N = (int)n;
  a.H = (int)h;
  a.W = (int)w;
  a.C = (int)c;
  a.Cp = (int)cp;
  a.KH = (int)kh;
  a.KW = (int)kw;
  a.sh = (int)stride_h;
  a.sw = (int)stride_w;
  a.ph = (int)pad_top;
  a.pw = (int)pad_left;
  a.dh = (int)dil_h;
  a.dw = (int)dil_w;
  a.Ho = (int)ho;
  a.Wo = (int)wo;
  a.out_nhwc = out_nhwc ? 1 : 0;
  a.scale = scale;
  if (epi) {
    if (!out_nhwc)
      return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: the fused epilogue is channels_last");
    if ((epi->ch_scale == nullptr) != (epi->ch_shift == nullptr))
      return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: ch_scale and ch_shift go together");
    if (epi->relu < 0 || epi->relu > tq::kActSwish)
      return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: relu must be 0, 1, 2 or 3");
    a.ch_scale = epi->ch_scale;
    a.ch_shift = epi->ch_shift;
    a.relu = epi->relu;
    if (epi->codes) {
      if (epi->cp != cp)
        return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: the codes' cp must equal the input's");
      if ((uintptr_t)epi->codes % 16 != 0)
        return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: codes must be 16-byte aligned");
      if (epi->fmt != TQ_CODES_I16 && epi->fmt != TQ_CODES_F16)
        return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: bad code format");
      if (epi->bits < 0 || epi->bits > max_code_bits(epi->fmt))
        return fail(TQ_ERR_UNSUPPORTED, "dwconv2d: codes of %d bits do not fit the format",
                    epi->bits);
      if (!(epi->sf >= 0.0f))
        return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: codes sf must be >= 0");
      a.codes = epi->codes;
      a.cp_c = (int)epi->cp;
      a.k_c = epi->terms < 0 ? 0 : epi->terms;
      a.fmt_c = epi->fmt;
      a.inv_c = 1.0 / (double)epi->sf;
      a.maxv_c = (float)((1u << epi->bits) - 1u);
      a.lut_c = lut_entries(true, tq::act_nonneg(epi->relu), a.inv_c, a.maxv_c);
    }
  }
  return hip_status(tq::launch_dwconv_tp(a, (hipStream_t)stream), "dwconv2d launch");
}

int tq_dwconv2d_termpair(const int16_t* act_codes, int64_t n, int64_t h, int64_t w, int64_t c,
                         int64_t cp, const int32_t* w_codes, int64_t kh, int64_t kw,
                         int64_t stride_h, int64_t stride_w, int64_t pad_top, int64_t pad_left,
                         int64_t dil_h, int64_t dil_w, double scale, const float* bias,
                         float* out, int64_t ho, int64_t wo, int32_t out_nhwc, void* stream) {
  return dw_impl(act_codes, n, h, w, c, cp, w_codes, kh, kw, stride_h, stride_w, pad_top,
                 pad_left, dil_h, dil_w, scale, bias, out, ho, wo, out_nhwc, nullptr, stream);
}

int tq_dwconv2d_termpair_fused(const int16_t* act_codes, int64_t n, int64_t h, int64_t w,
                               int64_t c, int64_t cp, const int32_t* w_codes, int64_t kh,
                               int64_t kw, int64_t stride_h, int64_t stride_w, int64_t pad_top,
                               int64_t pad_left, int64_t dil_h, int64_t dil_w, float* out,
                               int64_t ho, int64_t wo, const tq_dw_epilogue* epi,
                               void* stream) {
  if (epi == nullptr) return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d: epilogue is null");
  // the fused entry has no scale/bias of its own: its affine is the epilogue's per-channel
  // (ch_scale, ch_shift) -- without them every output would silently be acc * 0 + 0
  if (epi->ch_scale == nullptr || epi->ch_shift == nullptr)
    return fail(TQ_ERR_INVALID_ARGUMENT, "dwconv2d_fused: epilogue ch_scale/ch_shift are "
                "required");
  return dw_impl(act_codes, n, h, w, c, cp, w_codes, kh, kw, stride_h, stride_w, pad_top,
                 pad_left, dil_h, dil_w, 0.0, nullptr, out, ho, wo, 1, epi, stream);
}

int tq_bn_relu_maxpool_encode(const float* x, int64_t n, int64_t h, int64_t w, int64_t c,
                              const float* scale, const float* shift, int32_t k,
                              int32_t stride, int32_t pad, float* out, int64_t ho, int64_t wo,
                              void* codes_a, int64_t cp_a, float sf_a, int32_t bits_a,
                              int32_t terms_a, int32_t fmt_a, void* codes_b, int64_t cp_b,
                              float sf_b, int32_t bits_b, int32_t terms_b, int32_t fmt_b,
                              void* stream) {
  if (n < 0 || h < 1 || w < 1 || c < 8 || c % 8 != 0 || ho < 1 || wo < 1 || k < 1 ||
      stride < 1 || pad < 0 || pad >= k)
    return fail(TQ_ERR_INVALID_ARGUMENT, "bn_relu_maxpool: bad shape or pooling window");
  if ((ho - 1) * stride - pad >= h || (wo - 1) * stride - pad >= w)
    return fail(TQ_ERR_INVALID_ARGUMENT, "bn_relu_maxpool: output larger than the input");
  if (!x || !out || !scale || !shift || (uintptr_t)x % 16 || (uintptr_t)out % 16)
    return fail(TQ_ERR_INVALID_ARGUMENT, "bn_relu_maxpool: null or misaligned buffer");
  int rc = code_target(codes_a, cp_a, sf_a, bits_a, terms_a, fmt_a, c, "a");
  if (rc != TQ_OK) return rc;
  rc = code_target(codes_b, cp_b, sf_b, bits_b, terms_b, fmt_b, c, "b");
  if (rc != TQ_OK) return rc;
  if ((codes_a && (uintptr_t)codes_a % 16) || (codes_b && (uintptr_t)codes_b % 16))
    return fail(TQ_ERR_INVALID_ARGUMENT, "bn_relu_maxpool: codes must be 16-byte aligned");
  tq::PoolArgs a = tq::PoolArgs();
  a.x = x;
  a.scale = scale;
  a.shift = shift;
  a.out = out;
  a.N = (int)n;
  a.H = (int)h;
  a.W = (int)w;
  a.C = (int)c;
  a.Ho = (int)ho;
  a.Wo = (int)wo;
  a.k = k;
  a.s = stride;
  a.pad = pad;
  a.codes_a = static_cast<int16_t*>(codes_a);
  a.fmt_a = fmt_a;
  a.cp_a = (int)cp_a;
  a.sf_a = sf_a;
  a.inv_a = 1.0 / (double)sf_a;
  a.maxv_a = (float)((1u << (codes_a ? bits_a : 0)) - 1u);
  a.k_a = terms_a < 0 ? 0 : terms_a;
  a.codes_b = static_cast<int16_t*>(codes_b);
  a.fmt_b = fmt_b;
  a.cp_b = (int)cp_b;
  a.sf_b = sf_b;
  a.inv_b = 1.0 / (double)sf_b;
  a.maxv_b = (float)((1u << (codes_b ? bits_b : 0)) - 1u);
  a.k_b = terms_b < 0 ? 0 : terms_b;
  return hip_status(tq::launch_bn_relu_maxpool_encode(a, (hipStream_t)stream),
                    "bn_relu_maxpool launch");
}

int64_t tq_stem_workspace_bytes(int64_t n, int64_t h, int64_t w) {
  if (n < 0 || h < 4 || w < 4 || h > (1 << 20) || w > (1 << 20)) return -1;
  // per-workgroup counts, then one entry per (pool pixel, channel quad) of every tile (tiles
  // of up to four pool rows: at most 3 rows past Ho)
  return tq::kStemFixCountsBytes + n * (h / 4 + 3) * (w / 4) * 16 * 4;
}

int tq_stem_conv_pool_encode(const float* x, int64_t n, int64_t h, int64_t w,
                             const uint16_t* w_split, const float* scale, const float* shift,
                             float* out, int64_t ho, int64_t wo, void* codes_a, int64_t cp_a,
                             float sf_a, int32_t bits_a, int32_t terms_a, int32_t fmt_a,
                             void* codes_b, int64_t cp_b, float sf_b, int32_t bits_b,
                             int32_t terms_b, int32_t fmt_b, const double* w64,
                             const float* wbound, void* workspace, int64_t workspace_bytes,
                             void* stream) {
  if (n < 0 || h < 4 || w < 4 || h % 4 || w % 4 || ho != h / 4 || wo != w / 4 ||
      h > (1 << 20) || w > (1 << 20))
    return fail(TQ_ERR_INVALID_ARGUMENT, "stem_conv_pool: needs H, W % 4 == 0 and Ho = H/4, "
                                         "Wo = W/4 (conv 7x7/2 pad 3, pool 3x3/2 pad 1)");
  if (!x || !w_split || !out || !scale || !shift || (uintptr_t)x % 8 ||
      (uintptr_t)w_split % 16 || (uintptr_t)out % 16)
    return fail(TQ_ERR_INVALID_ARGUMENT, "stem_conv_pool: null or misaligned buffer");
  int rc = code_target(codes_a, cp_a, sf_a, bits_a, terms_a, fmt_a, 64, "a");
  if (rc != TQ_OK) return rc;
  rc = code_target(codes_b, cp_b, sf_b, bits_b, terms_b, fmt_b, 64, "b");
  if (rc != TQ_OK) return rc;
  if ((codes_a && (uintptr_t)codes_a % 16) || (codes_b && (uintptr_t)codes_b % 16))
    return fail(TQ_ERR_INVALID_ARGUMENT, "stem_conv_pool: codes must be 16-byte aligned");
  tq::PoolArgs a = tq::PoolArgs();
  a.x = x;
  a.wsplit = w_split;
  a.scale = scale;
  a.shift = shift;
  a.out = out;
  a.N = (int)n;
  a.H = (int)h;
  a.W = (int)w;
  a.C = 64;
  a.Ho = (int)ho;
  a.Wo = (int)wo;
  a.k = 3;
  a.s = 2;
  a.pad = 1;
  a.codes_a = static_cast<int16_t*>(codes_a);
  a.fmt_a = fmt_a;
  a.cp_a = (int)cp_a;
  a.sf_a = sf_a;
  a.inv_a = 1.0 / (double)sf_a;
  a.maxv_a = (float)((1u << (codes_a ? bits_a : 0)) - 1u);
  a.k_a = terms_a < 0 ? 0 : terms_a;
  a.codes_b = static_cast<int16_t*>(codes_b);
  a.fmt_b = fmt_b;
  a.cp_b = (int)cp_b;
  a.sf_b = sf_b;
  a.inv_b = 1.0 / (double)sf_b;
  a.maxv_b = (float)((1u << (codes_b ? bits_b : 0)) - 1u);
  a.k_b = terms_b < 0 ? 0 : terms_b;
  // the pooled outputs are ReLU'd: the epilogue code tables apply
  a.lut_a = lut_entries(codes_a != nullptr, true, a.inv_a, a.maxv_a);
  a.lut_b = lut_entries(codes_b != nullptr, true, a.inv_b, a.maxv_b);
  if (w64 || wbound || workspace) {  // the exact fix-up: all three or none
    if (!w64 || !wbound || !workspace || (uintptr_t)w64 % 8 || (uintptr_t)wbound % 4 ||
        (uintptr_t)workspace % 16)
      return fail(TQ_ERR_INVALID_ARGUMENT,
                  "stem_conv_pool: exact fix-up needs w64, wbound and workspace (aligned)");
    if (workspace_bytes < tq_stem_workspace_bytes(n, h, w))
      return fail(TQ_ERR_INVALID_ARGUMENT, "stem_conv_pool: workspace too small "
                                           "(tq_stem_workspace_bytes)");
    // list entries are ((pixel * 16 + quad) << 4) | mask in 32 bits
    if (n * ho * wo >= (int64_t)1 << 24)
      return fail(TQ_ERR_UNSUPPORTED, "stem_conv_pool: exact fix-up needs n*ho*wo < 2^24");
    a.w64 = w64;
    a.wbound = wbound;
    a.fix_counts = static_cast<uint32_t*>(workspace);
    a.fix_list = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) +
                                             tq::kStemFixCountsBytes);
  }
  const hipError_t e = tq::launch_stem_conv_pool(a, (hipStream_t)stream);
  if (e == hipErrorInvalidConfiguration)
    return fail(TQ_ERR_UNSUPPORTED, "stem_conv_pool: image too wide for the LDS tile");
  return hip_status(e, "stem_conv_pool launch");
}

int tq_mse_profile(const float* x, const float* hist, int64_t nbins, const float* sfs,
                   int64_t nsf, int32_t bitwidth, int32_t num_keep_terms, double* errs,
                   void* stream) {
  if (nbins < 0 || nsf < 0 || nbins > (1 << 30) || nsf > (1 << 30))
    return fail(TQ_ERR_INVALID_ARGUMENT, "mse_profile: bad sizes");
  if (bitwidth < 0 || bitwidth > tq::kMaxBitwidth)
    return fail(TQ_ERR_UNSUPPORTED, "mse_profile: bitwidth must be in [0, %d]", tq::kMaxBitwidth);
  const int kk = num_keep_terms < 0 ? 0 : num_keep_terms;
  return hip_status(tq::launch_mse_profile(x, hist, nbins, sfs, nsf, bitwidth, kk, errs,
                                           (hipStream_t)stream),
                    "mse_profile launch");
}

int tq_conv2d_termpair_wide(const int16_t* act_codes, int64_t n, int64_t h, int64_t w,
                            int64_t cp, const int32_t* w_codes, int64_t cout, int64_t kh,
                            int64_t kw, int64_t kp, int64_t stride_h, int64_t stride_w,
                            int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w,
                            double scale, const float* bias, float* out, int64_t ho, int64_t wo,
                            int32_t out_nhwc, void* stream) {
  if (n < 0 || h < 1 || w < 1 || cout < 1 || kh < 1 || kw < 1 || ho < 1 || wo < 1)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_wide: bad shape");
  if (cp < 8 || cp % 8 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_wide: cp must be a positive multiple of 8");
  if (kp != kh * kw * cp)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_wide: kp must be kh * kw * cp");
  if (stride_h < 1 || stride_w < 1 || dil_h < 1 || dil_w < 1 || pad_h < 0 || pad_w < 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_wide: bad stride/padding/dilation");
  if ((h + 2 * pad_h - dil_h * (kh - 1) - 1) / stride_h + 1 != ho ||
      (w + 2 * pad_w - dil_w * (kw - 1) - 1) / stride_w + 1 != wo)
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_wide: output size mismatch");
  if ((uintptr_t)act_codes % 16 || (uintptr_t)w_codes % 16 ||
      (out_nhwc && (uintptr_t)out % 16))
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_wide: buffers must be 16-byte aligned");
  if (out == nullptr || (n > 0 && (act_codes == nullptr || w_codes == nullptr)))
    return fail(TQ_ERR_INVALID_ARGUMENT, "conv2d_wide: null pointer");
  if (n * h * w * cp >= (int64_t)1 << 40 || n * ho * wo >= (int64_t)1 << 40 ||
      cout * kp >= (int64_t)1 << 40 || cout > (1 << 24))
    return fail(TQ_ERR_UNSUPPORTED, "conv2d_wide: problem too large");
  tq::WideConvArgs a;
  a.x = act_codes;
  a.w = w_codes;
  a.bias = bias;
  a.out = out;
  a.P = n * ho * wo;
  a.N = (int)n;
  a.H = (int)h;
  a.W = (int)w;
  a.Cp = (int)cp;
  a.Cout = (int)cout;
  a.KH = (int)kh;
  a.KW = (int)kw;
  a.sh = (int)stride_h;
  a.sw = (int)stride_w;
  a.ph = (int)pad_h;
  a.pw = (int)pad_w;
  a.dh = (int)dil_h;
  a.dw = (int)dil_w;
  a.Ho = (int)ho;
  a.Wo = (int)wo;
  a.out_nhwc = out_nhwc ? 1 : 0;
  a.Kp = kp;
  a.scale = scale;
  return hip_status(tq::launch_conv2d_wide(a, (hipStream_t)stream), "conv2d_wide launch");
}

int tq_lstm_cell_f32(const float* gx, const float* hh, float* c, float* h, int64_t batch,
                     int64_t hidden, void* stream) {
  if (batch < 0 || hidden < 0 || batch * hidden >= ((int64_t)1 << 40))
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_cell: bad sizes");
  if (batch * hidden > 0 && (!gx || !hh || !c || !h))
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_cell: null pointer");
  return hip_status(tq::launch_lstm_cell(gx, hh, c, h, batch, hidden, (hipStream_t)stream),
                    "lstm_cell launch");
}

int64_t tq_lstm_seq_workspace_bytes(int64_t batch, int64_t hidden) {
  return tq::lstm_seq_workspace_bytes(batch, hidden);
}

int tq_lstm_seq_f32(const float* gx, const float* w_hh, const float* b_hh, const float* h0,
                    const float* c0, float* out, float* c_out, int64_t steps, int64_t batch,
                    int64_t hidden, void* workspace, int64_t workspace_bytes, void* stream) {
  if (steps < 0 || batch < 0 || hidden < 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq: negative size");
  if (steps * batch * hidden == 0) return TQ_OK;
  if (tq::lstm_seq_workspace_bytes(batch, hidden) < 0)
    return fail(TQ_ERR_UNSUPPORTED, "lstm_seq: hidden <= 1024 and the batch's hidden state in "
                "one workgroup's LDS (tq_lstm_seq_workspace_bytes < 0)");
  if (!gx || !w_hh || !h0 || !c0 || !out || !c_out)
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq: null pointer");
  if (workspace_bytes < tq::lstm_seq_workspace_bytes(batch, hidden))
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq: workspace too small");
  if (c_out == c0 || c_out == out || h0 == out)
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq: c_out / out may not alias the inputs");
  return hip_status(tq::launch_lstm_seq(gx, w_hh, b_hh, h0, c0, out, c_out, steps, batch,
                                        hidden, workspace, (hipStream_t)stream),
                    "lstm_seq launch");
}

int tq_lstm_seq2_supported(int64_t batch, int64_t hidden) {
  return tq::lstm_seq2_supported(batch, hidden) ? 1 : 0;
}

int tq_lstm_seq2_f32(const float* gx0, const float* w_hh0, const float* b_hh0,
                     const float* h00, const float* c00, const float* w_ih1,
                     const float* b_ih1, const float* w_hh1, const float* b_hh1,
                     const float* h01, const float* c01, float* out0, float* out1,
                     float* c_out0, float* c_out1, int64_t steps, int64_t batch,
                     int64_t hidden, void* stream) {
  if (steps < 0 || batch < 0 || hidden < 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq2: negative size");
  if (steps * batch * hidden == 0) return TQ_OK;
  if (!tq::lstm_seq2_supported(batch, hidden))
    return fail(TQ_ERR_UNSUPPORTED, "lstm_seq2: even hidden <= 1024 and both layers' staged "
                "rows in one workgroup's LDS (tq_lstm_seq2_supported)");
  if (!gx0 || !w_hh0 || !h00 || !c00 || !w_ih1 || !w_hh1 || !h01 || !c01 || !out0 || !out1 ||
      !c_out0 || !c_out1)
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq2: null pointer");
  if (((uintptr_t)w_hh0 | (uintptr_t)w_ih1 | (uintptr_t)w_hh1) & 7)
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq2: weights must be 8-byte aligned");
  const void* ins[] = {gx0, h00, c00, h01, c01};
  const void* outs[] = {out0, out1, c_out0, c_out1};
  for (const void* o : outs) {
    for (const void* i : ins)
      if (o == i)
        return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq2: outputs may not alias the inputs");
  }
  if (out0 == out1 || c_out0 == c_out1 || (const void*)c_out0 == (const void*)out1 ||
      (const void*)c_out1 == (const void*)out0 || (const void*)c_out0 == (const void*)out0 ||
      (const void*)c_out1 == (const void*)out1)
    return fail(TQ_ERR_INVALID_ARGUMENT, "lstm_seq2: outputs may not alias each other");
  return hip_status(tq::launch_lstm_seq2(gx0, w_hh0, b_hh0, h00, c00, w_ih1, b_ih1, w_hh1,
                                         b_hh1, h01, c01, out0, out1, c_out0, c_out1, steps,
                                         batch, hidden, (hipStream_t)stream),
                    "lstm_seq2 launch");
}

int tq_histc_f32(const float* x, int64_t numel, int64_t nbins, float minv, float maxv,
                 uint64_t* counts, float* hist, void* stream) {
  if (numel < 0 || nbins < 1 || nbins > (1 << 24))
    return fail(TQ_ERR_INVALID_ARGUMENT, "histc: need numel >= 0 and 1 <= nbins <= 2^24");
  if (!(minv < maxv))
    return fail(TQ_ERR_INVALID_ARGUMENT, "histc: need min < max (got %g, %g)", (double)minv,
                (double)maxv);
  if (counts == nullptr || hist == nullptr || (numel > 0 && x == nullptr))
    return fail(TQ_ERR_INVALID_ARGUMENT, "histc: null pointer");
  if (reinterpret_cast<uintptr_t>(x) % 16 != 0)
    return fail(TQ_ERR_INVALID_ARGUMENT, "histc: x must be 16-byte aligned");
  return hip_status(tq::launch_histc(x, numel, (int)nbins, minv, maxv,
                                     reinterpret_cast<unsigned long long*>(counts), hist,
                                     (hipStream_t)stream),
                    "histc launch");
}

}  // extern "C"
