/*
 * tq.h -- C ABI of the MI355X term-quantization (TQ) library, libtq_hip.so.
 *
 * The drop-in boundary for the reference's one native op and the accumulation it leaves to
 * cuDNN.  Plain pointers and sizes only; every pointer argument except `stream` is a
 * device pointer (HIP), and work is enqueued on `stream` (a hipStream_t of the calling
 * thread's current device; NULL = the null stream).  Calls are asynchronous, keep no global
 * mutable state and are safe to issue from several host threads.
 *
 * Every entry point returns TQ_OK (0) or a TQ_ERR_* code; tq_last_error() then returns a
 * message for the calling thread.  The Python host layer (term-quantization_amd/tq_native.py)
 * raises RuntimeError with that message, as the reference's AT_ASSERTM checks do
 * (kernels/tr_cuda.cpp:12-18).  Python binding: INTEGRATION.md.
 */
#ifndef TQ_H_
#define TQ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  TQ_OK = 0,
  TQ_ERR_INVALID_ARGUMENT = 1, /* shape / parameter outside the contract */
  TQ_ERR_UNSUPPORTED = 2,      /* inside the reference's domain but not implemented */
  TQ_ERR_HIP = 3               /* a HIP runtime error (launch or memset) */
};

/*
 * Code formats of the term-pair kernels: the signed integer term sum v of an element,
 * stored in 16 bits either as int16 (VALU engine, bitwidth <= 14) or as the fp16 number v
 * (MFMA engine, exact for bitwidth <= 11).
 */
enum { TQ_CODES_I16 = 0, TQ_CODES_F16 = 1 };

/* Library version string, e.g. "tq-hip 0.1.0 gfx950". */
const char *tq_version(void);

/* Message for the last non-OK return on the calling thread ("" if none). */
const char *tq_last_error(void);

/*
 * Diagnostics: the number of bounded in-kernel waits that ran out since the previous call --
 * the row-strip conv engine's team syncs (each one means a launch went on without confirming
 * that its LDS patch was staged, so its results are suspect) -- then clears the count.
 * Synchronous (waits for the device); `count` is a host pointer.  A healthy run reads 0.
 */
int tq_sync_faults(uint32_t *count);

/*
 * Term-revealing op, float32 / float64.  Replaces the pybind entry
 *   at::Tensor tr(const at::Tensor input, const float sf, const int32_t bitwidth,
 *                 const int32_t group_size, const int32_t num_keep_terms)
 * of kernels/tr_cuda.cpp:20-24 and its launcher tr_cuda (kernels/tr_cuda_kernel.cu:128-160).
 *
 * `input` is a contiguous tensor of `ndim` >= 2 dims with sizes `shape`; `output` has the
 * same shape and receives sf * (sum of the kept HESE terms) per element.  As in the
 * reference, B = shape[0], C = shape[1], W,H = shape[2],shape[3] for 4-D inputs and 1
 * otherwise; a group is `group_size` consecutive channels at one (b, w, h); the first
 * `num_keep_terms` terms of each group in (exponent desc, channel asc) order are kept;
 * elements past B*C*W*H (3-D / 5-D inputs) are written as 0.
 * Domain: 0 <= bitwidth <= 24, 1 <= group_size <= 32, sf >= 0 (+inf allowed), ndim >= 2.
 * C % group_size != 0 uses a partial last group (the reference races there).
 */
int tq_tr_f32(const float *input, float *output, int64_t ndim, const int64_t *shape, float sf,
              int32_t bitwidth, int32_t group_size, int32_t num_keep_terms, void *stream);
int tq_tr_f64(const double *input, double *output, int64_t ndim, const int64_t *shape,
              float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms,
              void *stream);

/*
 * tq_tr_f32 that also writes the integer term sums: codes[i] = v with output[i] = v * sf
 * (|v| <= 2^bitwidth).  Used once per layer to pre-encode weights for the term-pair
 * kernels (the weight call of tr_layer.py:117-121).
 */
int tq_tr_encode_f32(const float *input, float *output, int32_t *codes, int64_t ndim,
                     const int64_t *shape, float sf, int32_t bitwidth, int32_t group_size,
                     int32_t num_keep_terms, void *stream);

/*
 * Activation TR (group_size 1, tr_layer.py:96-99) from fp32 straight into 16-bit term-sum
 * codes in NHWC with `cp` channels per pixel (cp % 8 == 0, cp >= c, pad channels = 0).
 * `in_nhwc` = 1 for a channels_last input, 0 for NCHW.  `fmt` = TQ_CODES_I16 (bitwidth
 * <= 14) or TQ_CODES_F16 (bitwidth <= 11).
 */
int tq_act_encode(const float *x, int32_t in_nhwc, int64_t n, int64_t c, int64_t h, int64_t w,
                  float sf, int32_t bitwidth, int32_t num_keep_terms, void *codes,
                  int64_t cp, int32_t fmt, void *stream);

/*
 * Affine / activation / squeeze-excite gate + activation TR of MobileNet-V2's and
 * EfficientNet-b0's stem and MBConv tensors
 * (efficientnet_pytorch MBConvBlock.forward: swish(bn0(expand_conv(x))), and
 * x = torch.sigmoid(x_sq) * x before the project conv; the consumer's input TR,
 * tr_layer.py:96-99), channels_last:
 *   v = x[p][c]; v = fp32 fma(v, ch_scale[c], ch_shift[c]) (if ch_scale: an eval BatchNorm
 *   as a per-channel affine, e.g. a stem's bn0); v = act(v): 0 none, 1 ReLU, 2 ReLU6,
 *   3 swish v * sigmoid(v)
 *   out[p][c] = v                       (if out: the fp32 activation)
 *   v = fp32(gate[img][c] * v)          (if gate: the squeeze-excite sigmoid, [n][c] fp32)
 *   codes[p][c] = TR(v; sf, bitwidth, num_keep_terms)   [n][h][w][cp] as tq_act_encode
 * x, out: [n][h][w][c] fp32, 16-byte aligned; 0 < sf < inf.
 */
int tq_act_encode_act(const float *x, int64_t n, int64_t c, int64_t h, int64_t w,
                      const float *ch_scale, const float *ch_shift, const float *gate,
                      int32_t act, float *out, float sf, int32_t bitwidth,
                      int32_t num_keep_terms, void *codes, int64_t cp, int32_t fmt,
                      void *stream);

/* Rows the weight-code matrix of tq_conv2d_termpair must be padded to (a multiple of). */
int64_t tq_conv2d_cout_align(void);

/*
 * Term-pair Conv2d (groups = 1): the exact integer sum over (kh, kw, c) of
 * act_codes * w_codes per output, scaled once: out = fp32(acc * scale) + bias.
 * With scale = double(sf_x) * double(sf_w) this is conv2d(TR(x), TR(w)) + bias -- the
 * reference's `self.conv(xq)` (tr_layer.py:124-126) on its fake-quantized tensors, to
 * within one fp32 rounding of the exact result.
 *   act_codes  [n][h][w][cp] int16 (tq_act_encode), 16-byte aligned
 *   w_codes    [cout_pad][kp] int16, k = (i*kw + j)*cp + c; cout_pad a multiple of
 *              tq_conv2d_cout_align(), kp a multiple of 32, padding zero
 *   bias       [cout] float or NULL
 *   out        float, [n][cout][ho][wo] (out_nhwc = 0) or [n][ho][wo][cout] (out_nhwc = 1)
 * The caller guarantees the int32 accumulator cannot overflow
 * (max_o sum_k |w_codes[o][k]| * max|act_code| < 2^31).
 */
int tq_conv2d_termpair(const int16_t *act_codes, int64_t n, int64_t h, int64_t w, int64_t cp,
                       const int16_t *w_codes, int64_t cout, int64_t kh, int64_t kw, int64_t kp,
                       int64_t stride_h, int64_t stride_w, int64_t pad_h, int64_t pad_w,
                       int64_t dil_h, int64_t dil_w, double scale, const float *bias,
                       float *out, int64_t ho, int64_t wo, int32_t out_nhwc, void *stream);

/*
 * Fused epilogue of tq_conv2d_termpair_fused (channels_last output only).  Per output
 * (pixel p, channel c), with acc the exact integer term-pair sum:
 *   y = fp32(acc * ch_scale[c] + ch_shift[c])          if ch_scale (conv scale, bias and an
 *                                                       eval-mode BatchNorm folded, fp64)
 *     = fp32(acc * scale + bias[c])                    otherwise (plain conv)
 *   y = y + residual[p][c]            (fp32, if residual; [P][cout] channels_last)
 *   y = max(y, 0)                     (if relu == 1; the stored out keeps a NaN, as torch.relu)
 *   y = min(max(y, 0), 6)             (if relu == 2: ReLU6, MobileNet-V2; NaN kept likewise)
 *   y = y * sigmoid(y)                (if relu == 3: swish, EfficientNet-b0; fp16 entry only,
 *                                      1x1 convs or cp % 64 == 0: the direct engine)
 *   out[p][c] = y                     (if out)
 *   codes_a[p][c] = TR(y; sf_a, bits_a, terms_a)   format fmt_a, [P][cp_a] (if codes_a)
 *   codes_b[p][c] = TR(y; sf_b, bits_b, terms_b)   format fmt_b, [P][cp_b] (if codes_b)
 * codes_a/_b are the next TR layers' activation codes (tr_layer.py:96-99 applied to y), so
 * those layers skip their own activation pass.  cp_* = roundup(cout, 8); cout % 4 == 0; the
 * pad channels [cout, cp_*) of codes_a/_b are written as zero codes.
 */
typedef struct tq_conv_epilogue {
  const double *ch_scale;
  const double *ch_shift;
  const float *residual;
  int32_t relu;
  int16_t *codes_a;
  int64_t cp_a;
  float sf_a;
  int32_t bits_a;
  int32_t terms_a;
  int16_t *codes_b;
  int64_t cp_b;
  float sf_b;
  int32_t bits_b;
  int32_t terms_b;
  /* execution choices: config 0 = built-in heuristic, 1..tq_conv2d_num_configs() = a fixed
   * tile configuration with split_k = 1 (data-parallel), > 1 (K loop split over that many
   * workgroups, int32 atomics) or -1 (stream-K: one resident round of workgroups sharing the
   * tiles x K-steps evenly).  Splitting needs `workspace` (16-byte aligned scratch of
   * `workspace_bytes` >= tq_conv2d_workspace_bytes(n*ho*wo, cout)); without one the K loop
   * is never split. */
  int32_t *workspace;
  int64_t workspace_bytes;
  int32_t split_k;
  int32_t config;
  /* code formats (TQ_CODES_*) of codes_a / codes_b: the format of the consuming kernel */
  int32_t fmt_a;
  int32_t fmt_b;
  /* Fused downsample (tq_conv2d_termpair_f16 only; NULL ds_codes = none): the identity of a
   * ResNet transition block computed as a second accumulation phase of this launch,
   *   identity[p][c] = fp32(acc2 * ds_scale[c] + ds_shift[c])
   * with acc2 the exact term-pair sum of the 1x1, stride ds_stride, pad 0 conv of ds_codes
   * [n][ds_h][ds_w][ds_cp] (fp16 codes) with ds_w_codes [cout_pad][ds_cp] -- what the
   * downsample conv with this epilogue would store -- added where `residual` would be
   * (residual must be NULL; (ds_h - 1) / ds_stride + 1 == ho, likewise w).  ds_cp % 64 == 0,
   * and every window of the whole ds_cp K range must satisfy the kc_steps bound (no flush).
   * Replaces the downsample launch and its fp32 identity round trip through HBM. */
  const uint16_t *ds_codes;
  int64_t ds_h;
  int64_t ds_w;
  int64_t ds_cp;
  int64_t ds_stride;
  const uint16_t *ds_w_codes;
  const double *ds_scale;
  const double *ds_shift;
} tq_conv_epilogue;

/* Scratch bytes that let tq_conv2d_termpair_fused use any K-split schedule for an output of
 * `pixels` (= n*ho*wo) x `cout` on the calling thread's current device. */
int64_t tq_conv2d_workspace_bytes(int64_t pixels, int64_t cout);

/* Number of tile configurations selectable through tq_conv_epilogue.config. */
int32_t tq_conv2d_num_configs(void);

int tq_conv2d_termpair_fused(const int16_t *act_codes, int64_t n, int64_t h, int64_t w,
                             int64_t cp, const int16_t *w_codes, int64_t cout, int64_t kh,
                             int64_t kw, int64_t kp, int64_t stride_h, int64_t stride_w,
                             int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w,
                             double scale, const float *bias, float *out, int64_t ho,
                             int64_t wo, const tq_conv_epilogue *epi, void *stream);

/*
 * Term-pair Conv2d (groups = 1) on the matrix cores: the same exact integer sums as
 * tq_conv2d_termpair(_fused), from fp16 codes (TQ_CODES_F16) with v_mfma_f32_32x32x16_f16.
 * fp32 accumulators are exact while every partial sum stays within 2^24 in magnitude (2^24
 * itself is an fp32 value, so every such partial sum is an exact integer); the caller passes
 * `kc_steps` >= 1 such that for every weight row m and every window of kc_steps K-steps of
 * 64 codes, max|act_code| * sum_{k in window} |w_codes[m][k]| <= 2^24 (0 = the whole K
 * range satisfies it), and max_m sum_k |w_codes[m][k]| * max|act_code| < 2^31.
 * Kernels that walk K chunk-major (the input-patch engine: for each 64-code channel chunk,
 * all filter taps) use `kc_chunk` instead: the same bound over every window of kc_chunk
 * consecutive taps of one chunk (0 = never needed; -1 = derive a conservative value from
 * kc_steps); they also flush at every chunk end.  When every act_code is >= 0 (TR of a ReLU
 * output) the window bound may use max(sum of positive w_codes, sum of |negative w_codes|)
 * in place of sum |w_codes|: every partial sum then lies between -max_act * neg and
 * max_act * pos (tq_ops.mfma_flush_steps(..., nonneg=True)).
 *   act_codes  [n][h][w][cp] fp16 codes, 16-byte aligned
 *   w_codes    [cout_pad][kp] fp16 codes, cout_pad a multiple of tq_conv2d_cout_align(),
 *              kp a multiple of 64
 * epi == NULL: out = fp32(acc * scale) + bias, NCHW (out_nhwc = 0) or NHWC (out_nhwc = 1).
 * epi != NULL: the fused epilogue of tq_conv2d_termpair_fused (out_nhwc must be 1).  Its
 * split_k: 0 = built-in choice, 1 = data-parallel tiles, -1 = stream-K where the engine has
 * it (the input-patch engine: tiles x K-steps shared evenly by one workgroup per CU, split
 * tiles finished by their last-arriving piece from int32 slabs -- bit-identical results;
 * needs `workspace` >= tq_conv2d_workspace_bytes, else data-parallel).
 */
int32_t tq_conv2d_mfma_num_configs(void);

int tq_conv2d_termpair_f16(const uint16_t *act_codes, int64_t n, int64_t h, int64_t w,
                           int64_t cp, const uint16_t *w_codes, int64_t cout, int64_t kh,
                           int64_t kw, int64_t kp, int64_t stride_h, int64_t stride_w,
                           int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w,
                           double scale, const float *bias, float *out, int64_t ho, int64_t wo,
                           int32_t out_nhwc, int32_t kc_steps, int32_t kc_chunk,
                           const tq_conv_epilogue *epi, void *stream);

/*
 * Depthwise term-pair Conv2d (groups == C_in == C_out): per output channel c,
 *   out = fp32(sum_{taps} act_codes[.., c] * w_codes[tap][c] * scale) + bias[c]
 * exactly in int32 before the one rounding -- the reference's `self.conv(xq)` for the
 * depthwise layers of MobileNet-V2 / EfficientNet-b0 (16-bit weights: int32 codes).
 *   act_codes  [n][h][w][cp] int16 (tq_act_encode), cp % 8 == 0, 16-byte aligned
 *   w_codes    [kh*kw][cp] int32, tap-major, channel fastest, pad channels 0, 16-byte aligned
 *   out        [n][ho][wo][c] (out_nhwc = 1) or [n][c][ho][wo]
 * Taps outside the input read 0, so pad_top / pad_left plus (ho, wo) express symmetric and
 * TensorFlow-style asymmetric "same" padding alike.  The caller guarantees
 * max_c sum_tap |w_codes| * max|act_code| < 2^31 and |act_code| < 2^23, |w_code| < 2^23.
 */
int tq_dwconv2d_termpair(const int16_t *act_codes, int64_t n, int64_t h, int64_t w, int64_t c,
                         int64_t cp, const int32_t *w_codes, int64_t kh, int64_t kw,
                         int64_t stride_h, int64_t stride_w, int64_t pad_top, int64_t pad_left,
                         int64_t dil_h, int64_t dil_w, double scale, const float *bias,
                         float *out, int64_t ho, int64_t wo, int32_t out_nhwc, void *stream);

/*
 * Term-pair Conv2d (groups = 1) with int32 weight codes, for weight bit widths whose term
 * sums leave int16 (the (16, 1, 16) squeeze-excite convs of EfficientNet-b0,
 * cnn_models/__init__.py:57-58; their `self.conv(xq)` at tr_layer.py:124-126):
 *   out = fp32(acc * scale + bias[c]),  acc = exact int64 sum over (kh, kw, c) of
 *   act_codes * w_codes.
 *   act_codes  [n][h][w][cp] int16 (tq_act_encode), cp % 8 == 0, 16-byte aligned
 *   w_codes    [cout][kp] int32, kp = kh * kw * cp, k = (i*kw + j)*cp + c, 16-byte aligned
 *   out        [n][cout][ho][wo] (out_nhwc = 0) or [n][ho][wo][cout] (out_nhwc = 1)
 * Every product must fit int32: |act_code| <= 2^14 and |w_code| <= 2^16 (bitwidths <= 14 /
 * 16); the int64 sum is exact.
 */
int tq_conv2d_termpair_wide(const int16_t *act_codes, int64_t n, int64_t h, int64_t w,
                            int64_t cp, const int32_t *w_codes, int64_t cout, int64_t kh,
                            int64_t kw, int64_t kp, int64_t stride_h, int64_t stride_w,
                            int64_t pad_h, int64_t pad_w, int64_t dil_h, int64_t dil_w,
                            double scale, const float *bias, float *out, int64_t ho, int64_t wo,
                            int32_t out_nhwc, void *stream);

/*
 * Squeeze-excite gate of an EfficientNet MBConv block (reference cnn_models/__init__.py:
 * 52-65: both squeeze-excite convs term-revealed at (16, 1, 16)), one launch:
 *   v   = TR(x_sq[n][c]; sf_r, bits_r, terms_r)            (int, as tq_act_encode)
 *   y1  = fp32(double(sum_c v[c] w_r[j][c]) * scale_r + b_r[j])        j < cse
 *   v2  = TR(y1 * sigmoid(y1); sf_e, bits_e, terms_e)                   (torch's fp32 swish)
 *   y2  = fp32(double(sum_j v2[j] w_e_t[j][c]) * scale_e + b_e[c])      c < c
 *   gate[n][c] = 1 / (1 + exp(-y2))                                     (torch's fp32 sigmoid)
 * x_sq [n][c] fp32 (the block's pooled activations); w_r [cse][cpr] (cpr = roundup(c, 8),
 * pad columns zero) and w_e_t [cse][c] (the expand conv's [c][cse] codes transposed) int32
 * weight codes; b_r [cse],
 * b_e [c] fp32 or NULL; scale_* = double(sf_x) * double(sf_w) of each conv; gate [n][c]
 * fp32.  Sums are exact (int64); bits <= 14 activations, <= 16-bit weight codes.
 */
int tq_se_gate_f32(const float *x_sq, int64_t n, int64_t c, const int32_t *w_r, int64_t cse,
                   double scale_r, const float *b_r, float sf_r, int32_t bits_r,
                   int32_t terms_r, const int32_t *w_e_t, double scale_e, const float *b_e,
                   float sf_e, int32_t bits_e, int32_t terms_e, float *gate, void *stream);

/*
 * Depthwise term-pair conv with a fused epilogue (MobileNet-V2's dw conv -> BN -> ReLU6 and
 * the following project conv's input TR), channels_last:
 *   y = fp32(acc * ch_scale[c] + ch_shift[c])   (folded eval BatchNorm, fp64)
 *   y = max(y, 0) (relu 1), min(max(y, 0), 6) (relu 2) or y * sigmoid(y) (relu 3, swish);
 *   out[p][c] = y (if out; NaN kept)
 *   codes[p][c] = TR(y; sf, bits, terms) in format fmt, [p][cp] with the input's cp, pad
 *   channels zero (if codes)
 * Other arguments as tq_dwconv2d_termpair.
 */
typedef struct tq_dw_epilogue {
  const double *ch_scale;
  const double *ch_shift;
  int32_t relu;
  int16_t *codes;
  int64_t cp;
  float sf;
  int32_t bits;
  int32_t terms;
  int32_t fmt;
} tq_dw_epilogue;

int tq_dwconv2d_termpair_fused(const int16_t *act_codes, int64_t n, int64_t h, int64_t w,
                               int64_t c, int64_t cp, const int32_t *w_codes, int64_t kh,
                               int64_t kw, int64_t stride_h, int64_t stride_w, int64_t pad_top,
                               int64_t pad_left, int64_t dil_h, int64_t dil_w, float *out,
                               int64_t ho, int64_t wo, const tq_dw_epilogue *epi, void *stream);

/*
 * Stem tail of a TQ ResNet in one pass (the stem conv itself stays fp32, as in the
 * reference): out = relu(maxpool_{k,s,pad}(x * scale[c] + shift[c])) with an eval-mode
 * BatchNorm as (scale, shift), plus the consuming TR layers' activation codes
 * codes_a/_b = TR(out; sf, bits, terms) ([n][ho][wo][cp] in format fmt_*, NULL to skip).
 * x, out: fp32 channels_last [n][h][w][c] / [n][ho][wo][c], c % 8 == 0, 16-byte aligned.
 */
int tq_bn_relu_maxpool_encode(const float *x, int64_t n, int64_t h, int64_t w, int64_t c,
                              const float *scale, const float *shift, int32_t k,
                              int32_t stride, int32_t pad, float *out, int64_t ho, int64_t wo,
                              void *codes_a, int64_t cp_a, float sf_a, int32_t bits_a,
                              int32_t terms_a, int32_t fmt_a, void *codes_b, int64_t cp_b,
                              float sf_b, int32_t bits_b, int32_t terms_b, int32_t fmt_b,
                              void *stream);

/*
 * The whole stem of a TQ ResNet in one pass (torchvision ResNet.forward: conv1 -> bn1 -> relu
 * -> maxpool, then the first TR layers' input TR, tr_layer.py:96-99): conv 7x7 stride 2
 * pad 3, 3 -> 64 channels, no bias, in near-fp32 arithmetic on the fp16 matrix cores
 * (two-way fp16 split of inputs, scaled per tile by a power of two, and of the weights,
 * three partial products per pair, fp32 accumulation; per-product relative error ~2^-21,
 * between the reference's fp32 cuDNN conv and cuDNN's default TF32), eval BatchNorm
 * out = conv * scale[c] + shift[c] (fp32 fma), ReLU, max-pool 3x3 stride 2 pad 1, fp32
 * output and codes as tq_bn_relu_maxpool_encode.  The 64 x (H/2) x (W/2) conv output never
 * goes to memory.
 *   x        fp32 channels_last image [n][h][w][3], 8-byte aligned; h, w multiples of 4
 *   w_split  [2][64][192] fp16 bits: the two splits of the conv weight * 2^10 (|w| <= 32) in
 *            space-to-depth
 *            K order k = ((sy*4 + sx)*2 + sub_r)*6 + sub_c*3 + c for tap (2sy+sub_r-1,
 *            2sx+sub_c-1), zero where a tap index is -1 (term-quantization_amd/tq_ops.py
 *            pack_stem_weight)
 *   out      fp32 [n][h/4][w/4][64] (ho = h/4, wo = w/4)
 * Exact fix-up (w64, wbound, workspace all non-NULL; all NULL = the split conv's result
 * stands): the split conv of output channel c at a conv position is within wbound[c] * |x|
 * of the exact sum (|x| the 2-norm of the position's 7x7x3 input window, summed by the
 * kernel beside its MFMAs; Cauchy-Schwarz).  Every pooled output whose quotient out / sf lies
 * within that error (through BN) of a rounding midpoint is listed in the workspace and
 * recomputed from the fp64 weights by the same launch (each workgroup's tail phase, after its
 * last tile) -- exact products, fp64 sum, one rounding to fp32 -- so every code equals the
 * code of the correctly rounded fp32 conv followed by the same BN / ReLU / max-pool.  The
 * workspace's first 4096 bytes hold the per-workgroup counts of listed outputs (uint32).
 *   w64      fp64 [64][7][7][3] conv weights (kernel row, column, input channel)
 *   wbound   fp32 [64], >= the split conv's relative error bound times |w[c]|_2
 *            (tq_ops.pack_stem_exact)
 *   workspace  >= tq_stem_workspace_bytes(n, h, w) bytes, 16-byte aligned; needs
 *            n * ho * wo < 2^24
 * TQ_ERR_UNSUPPORTED when the image is too wide for one LDS tile (w/4 > 84).
 */
int tq_stem_conv_pool_encode(const float *x, int64_t n, int64_t h, int64_t w,
                             const uint16_t *w_split, const float *scale, const float *shift,
                             float *out, int64_t ho, int64_t wo, void *codes_a, int64_t cp_a,
                             float sf_a, int32_t bits_a, int32_t terms_a, int32_t fmt_a,
                             void *codes_b, int64_t cp_b, float sf_b, int32_t bits_b,
                             int32_t terms_b, int32_t fmt_b, const double *w64,
                             const float *wbound, void *workspace, int64_t workspace_bytes,
                             void *stream);

/* Workspace bytes tq_stem_conv_pool_encode's exact fix-up needs for an n x 3 x h x w batch
 * (-1 for invalid sizes). */
int64_t tq_stem_workspace_bytes(int64_t n, int64_t h, int64_t w);

/*
 * Batched activation-scale calibration, replacing the 2048-launch loop of
 * tr_layer.mse_profile (tr_layer.py:43-54):
 *   errs[s] = sum_b hist[b] * (x[b] - TR(x[b]; sf = sfs[s], bitwidth, group 1, k))^2
 * for s < nsf, the per-bin term in fp32 as the reference's torch expression, the sum over
 * bins in fp64.  The caller takes the first arg-min (torch.argmin semantics).
 */
int tq_mse_profile(const float *x, const float *hist, int64_t nbins, const float *sfs,
                   int64_t nsf, int32_t bitwidth, int32_t num_keep_terms, double *errs,
                   void *stream);

/*
 * One step of an LSTM layer's point-wise update (torch.nn.LSTM gate order i, f, g, o), for the
 * term-pair LSTM path of TRLSTMLayer (tr_layer.py:162-201, whose cuDNN LSTM runs on the TR'd
 * layer-0 weights and quantized inputs): with gates = gx + hh ([b][4h], fp32),
 *   c[b][j] <- sigmoid(f) * c[b][j] + sigmoid(i) * tanh(g),  h[b][j] = sigmoid(o) * tanh(c)
 * gx = the step's input projection (TR(x) TR(W_ih)^T + b_ih, a term-pair GEMM), hh = the
 * recurrent projection (h W_hh^T + b_hh).  c is updated in place; h may not alias gx / hh.
 */
int tq_lstm_cell_f32(const float *gx, const float *hh, float *c, float *h, int64_t batch,
                     int64_t hidden, void *stream);

/*
 * A whole LSTM layer's recurrence (torch.nn.LSTM semantics, gate order i, f, g, o) in one
 * call, replacing T x (a recurrent-projection GEMM + tq_lstm_cell_f32) of TRLSTMLayer's
 * per-step loop (tr_layer.py:191-195 runs cuDNN's LSTM there): T fused step launches,
 *   gates_t = gx[t] + b_hh + h_{t-1} W_hh^T,  c_t = sigmoid(f) c_{t-1} + sigmoid(i) tanh(g),
 *   h_t = sigmoid(o) tanh(c_t),  out[t] = h_t,  for t < steps, from (h0, c0)
 * gx [steps][batch][4 hidden] (the input projection incl. b_ih), w_hh [4 hidden][hidden],
 * b_hh [4 hidden] (or NULL), h0/c0/c_out [batch][hidden], out [steps][batch][hidden], all fp32
 * device buffers; c_out = c_{steps-1} (h_{steps-1} is out[steps-1]); out and c_out may not
 * alias h0 / c0.  `workspace`: tq_lstm_seq_workspace_bytes(batch, hidden) device bytes (0 in
 * this version; < 0: the shape is outside the domain -- hidden <= 1024 and the batch's hidden
 * state staged in one workgroup's LDS, e.g. batch <= 39 at hidden 650).  fp32 arithmetic, a
 * fixed summation order.
 */
int64_t tq_lstm_seq_workspace_bytes(int64_t batch, int64_t hidden);
int tq_lstm_seq_f32(const float *gx, const float *w_hh, const float *b_hh, const float *h0,
                    const float *c0, float *out, float *c_out, int64_t steps, int64_t batch,
                    int64_t hidden, void *workspace, int64_t workspace_bytes, void *stream);

/*
 * Two stacked LSTM layers' recurrences (TRLSTMLayer's LSTM-650: layer 0 from the term-pair
 * input projection, layer 1 untouched by the reference's TR) in wavefront order: launch s
 * runs layer 0's step s and layer 1's step s - 1 in one grid, steps + 1 dependent launches
 * in all.  Layer 0 as tq_lstm_seq_f32 (gx0 [steps][batch][4 hidden] incl. b_ih0, w_hh0,
 * b_hh0, h00, c00 -> out0, c_out0); layer 1 computes its own input projection per step:
 *   gates_t = (out0[t] W_ih1^T + b_ih1) + (h_{t-1} W_hh1^T + b_hh1)
 * from (h01, c01) -> out1 [steps][batch][hidden], c_out1.  Biases may be NULL.  fp32
 * arithmetic, 16 fixed-order partial sums per dot product over interleaved column pairs (so
 * layer 0's order differs from tq_lstm_seq_f32's, and layer 1's sums are not those of a
 * separate GEMM + tq_lstm_seq_f32: both match that path to fp32 rounding, not bit for bit).
 * Returns TQ_ERR_UNSUPPORTED outside tq_lstm_seq2_supported(batch, hidden) (even hidden <=
 * 1024, both layers' staged rows in one workgroup's LDS: batch <= 23 at hidden 650); weights
 * 8-byte aligned.  Outputs may not alias the inputs.
 */
int tq_lstm_seq2_supported(int64_t batch, int64_t hidden);
int tq_lstm_seq2_f32(const float *gx0, const float *w_hh0, const float *b_hh0,
                     const float *h00, const float *c00, const float *w_ih1,
                     const float *b_ih1, const float *w_hh1, const float *b_hh1,
                     const float *h01, const float *c01, float *out0, float *out1,
                     float *c_out0, float *c_out1, int64_t steps, int64_t batch,
                     int64_t hidden, void *stream);

/*
 * Tracking histogram of the activation calibration, replacing
 *   self.hist_bins += torch.histc(x, self.num_bins, self.minv, self.maxv)
 * of LinearQuantize.forward (tr_layer.py:91-94):
 *   hist[b] += fp32(#{i < numel : x[i] in bin b})          for b < nbins
 * with torch.histc's GPU bin rule: x outside [minv, maxv] or NaN is skipped, otherwise
 * b = int(fp32(fp32(x - minv) * nbins) / (maxv - minv)) (fp32 operations), and b == nbins
 * goes to the last bin.  Counts are exact (torch.histc's fp32 atomic counts stop at 2^24 per
 * bin).  `x` is any dense fp32 buffer (16-byte aligned); `counts` is uint64 scratch [nbins]
 * that must be zero on entry and is zero again when the call's work completes.
 * Domain: 1 <= nbins <= 2^24, minv < maxv.
 */
int tq_histc_f32(const float *x, int64_t numel, int64_t nbins, float minv, float maxv,
                 uint64_t *counts, float *hist, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* TQ_H_ */
