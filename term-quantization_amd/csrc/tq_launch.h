// Internal launchers shared by the kernels and the C-ABI layer (tq_capi.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tq {

// TR op (reference tr_cuda, kernels/tr_cuda_kernel.cu:128-160).  `codes` (nullable) receives
// the signed integer term sums v with out = v * sf.
template <typename T>
hipError_t launch_tr(const T* in, T* out, int32_t* codes, int64_t B, int64_t C, int64_t WH,
                     int64_t numel, float sf, int bitwidth, int g, int k, hipStream_t stream);

struct ConvArgs {
  const int16_t* x;     // activation codes [N][H][W][Cp]
  const int16_t* w;     // weight codes [Cout_pad][Kp]
  const float* bias;    // [Cout] or nullptr
  float* out;           // [N][Cout][Ho][Wo] or [N][Ho][Wo][Cout]
  int64_t P;            // N * Ho * Wo
  int N, H, W, Cp, Cout, KH, KW, sh, sw, ph, pw, dh, dw, Ho, Wo, Kp;
  double scale;         // double(sf_x) * double(sf_w)
  // Fused epilogue (channels_last output only; all optional):
  //   y = fp32(acc * ch_scale[c] + ch_shift[c])   (per-channel: conv scale, bias, folded BN)
  //       else fp32(acc * scale + bias[c])
  //   y = y + residual[p][c] (fp32);  y = max(y, 0) if relu
  //   out[p][c] = y (if out);  codes_a/b[p][c] = TR(y; sf, bits, k) (next layers' inputs)
  const double* ch_scale;
  const double* ch_shift;
  const float* residual;
  int relu;
  int16_t* codes_a;
  int cp_a, k_a;
  float sf_a, maxv_a;
  int16_t* codes_b;
  int cp_b, k_b;
  float sf_b, maxv_b;
  int fmt_a, fmt_b;     // code formats of codes_a / codes_b (kCodesI16 / kCodesF16)
  double inv_a, inv_b;  // RN64(1 / sf_a), RN64(1 / sf_b) (set by the C-ABI layer)
  // MFMA engine only: fp32 accumulators are moved into the int32 sums every kc_steps
  // K-steps of 64 codes, a window whose |partial sums| the host has bounded by 2^24 (so
  // every fp32 partial sum is an exact integer); 0 = never needed.
  int kc_steps;
  // chunk-major engines (patch): the same bound over windows of kc_chunk consecutive taps of
  // one 64-code channel chunk (fp32 sums also flushed at every chunk end); 0 = never needed
  int kc_chunk;
  // MFMA patch engine (set by its launcher): patch slot pixels and number of patch buffers
  int patch_px, patch_bufs;
  int m_slow;  // MFMA engines: 1 = Cout tile is the slow index of the tile order
  // Execution choices: config 0 = heuristic, 1..conv_num_configs() = a fixed tile config;
  // splits: 1 data-parallel, > 1 K-split with int32 atomics into ws ([P][Cout]), -1
  // stream-K (ws holds two BM x BN int32 slabs per resident block); NHWC output only.
  // Fused downsample (second accumulation phase; direct engine): the identity of a ResNet
  // transition block, fp32(acc2 * ds_scale[c] + ds_shift[c]) with acc2 the exact term-pair
  // sum of the 1x1 stride-ds_s pad-0 conv of ds_x [N][ds_H][ds_W][ds_Cp] with weight codes
  // ds_w [Cout_pad][ds_Cp], is added where `residual` would be (which must then be null).
  // The host guarantees acc2's fp32 partial sums need no flush (one window over ds_Cp).
  const int16_t* ds_x;
  const int16_t* ds_w;
  const double* ds_scale;
  const double* ds_shift;
  int ds_H, ds_W, ds_Cp, ds_s;
  // epilogue code tables (tq_device.h kLutMax): entries of codes_a's / codes_b's table
  // (maxv + 1) when the ReLU fast path applies and it fits, else 0 (set by the C-ABI layer);
  // a kernel that places them in LDS passes the LDS pointers to the emit functions
  int lut_a, lut_b;
  int ab;  // timing-only A/B switches (TQ_AB, tools only; 0 in the product)
  int config, splits;
  int* ws;
  int64_t ws_bytes;
};

struct DwConvArgs {
  const int16_t* x;     // activation codes [N][H][W][Cp]
  const int32_t* w;     // weight codes [KH*KW][Cp] (channel fastest)
  const float* bias;    // [C] or nullptr
  float* out;           // [N][Ho][Wo][C] (out_nhwc) or [N][C][Ho][Wo]; nullptr = codes only
  int N, H, W, C, Cp, KH, KW, sh, sw, ph, pw, dh, dw, Ho, Wo, out_nhwc;
  double scale;
  // fused epilogue (NHWC only): y = fp32(acc * ch_scale[c] + ch_shift[c]) (folded BN),
  // relu 1 = ReLU, 2 = ReLU6, then the next layer's codes [P][cp_c] = TR(y)
  const double* ch_scale;
  const double* ch_shift;
  int relu;
  int16_t* codes;
  int cp_c, k_c, fmt_c, lut_c;  // lut_c: code table entries (tq_device.h kLutMax), 0 = none
  float maxv_c;
  double inv_c;
};

hipError_t launch_dwconv_tp(const DwConvArgs& a, hipStream_t stream);

struct WideConvArgs {
  const int16_t* x;     // activation codes [N][H][W][Cp] (int16), Cp % 8 == 0
  const int32_t* w;     // weight codes [Cout][Kp] (int32), k = (kh * KW + kw) * Cp + c
  const float* bias;    // [Cout] or nullptr
  float* out;           // [N][Ho][Wo][Cout] (out_nhwc) or [N][Cout][Ho][Wo]
  int64_t P;            // N * Ho * Wo
  int N, H, W, Cp, Cout, KH, KW, sh, sw, ph, pw, dh, dw, Ho, Wo, out_nhwc;
  int64_t Kp;
  double scale;
};

hipError_t launch_conv2d_wide(const WideConvArgs& a, hipStream_t stream);

// LSTM cell update (tq_lstm.hip): c, h [B][H] in place / out from gx, hh [B][4H]
hipError_t launch_lstm_cell(const float* gx, const float* hh, float* c, float* h, int64_t B,
                            int64_t H, hipStream_t stream);
// A whole LSTM layer's recurrence: T fused step launches from one call (tq_lstm.hip)
int64_t lstm_seq_workspace_bytes(int64_t B, int64_t H);
bool lstm_seq2_supported(int64_t B, int64_t H);
hipError_t launch_lstm_seq2(const float* gx0, const float* w_hh0, const float* b_hh0,
                            const float* h00, const float* c00, const float* w_ih1,
                            const float* b_ih1, const float* w_hh1, const float* b_hh1,
                            const float* h01, const float* c01, float* out0, float* out1,
                            float* cT0, float* cT1, int64_t T, int64_t B, int64_t H,
                            hipStream_t stream);
hipError_t launch_lstm_seq(const float* gx, const float* w, const float* b, const float* h0,
                           const float* c0, float* out, float* cT, int64_t T, int64_t B,
                           int64_t H, void* ws, hipStream_t stream);


struct PoolArgs {
  const float* x;        // [N][H][W][C] fp32 (channels_last), C % 8 == 0
  const float* scale;    // [C] BN scale (gamma / sqrt(var + eps))
  const float* shift;    // [C] BN shift (beta - mean * scale)
  float* out;            // [N][Ho][Wo][C]
  int N, H, W, C, Ho, Wo, k, s, pad;
  int16_t* codes_a;      // [N][Ho][Wo][cp_a] or nullptr
  int cp_a, k_a;
  float sf_a, maxv_a;
  int16_t* codes_b;
  int cp_b, k_b;
  float sf_b, maxv_b;
  int fmt_a, fmt_b;
  double inv_a, inv_b;   // RN64(1 / sf_a), RN64(1 / sf_b)
  int lut_a, lut_b;      // epilogue code table entries (as ConvArgs), 0 = none
  // fused stem (tq_stem_conv.hip): x is the [N][H][W][3] input image, H/W its size, and
  // wsplit the conv weights * 2^10 as two fp16 splits [2][64][192] (s2d K order)
  const uint16_t* wsplit;
  // fused stem, exact fix-up (nullptr fix_list: the split-fp16 result stands): w64 the conv
  // weights in fp64 [64][7][7][3] (kernel row, column, channel: the image's NHWC order),
  // wbound[c] >= err_rel * sum |w[c]| (the split conv's error per unit of the input tile's
  // max |x|), fix_list / fix_counts the per-workgroup lists of near-midpoint outputs
  const double* w64;
  const float* wbound;
  uint32_t* fix_list;
  uint32_t* fix_counts;
};

// fused stem exact fix-up workspace: per-workgroup entry counts (stem grids <= 1024), then
// the entry lists
constexpr int64_t kStemFixCountsBytes = 4096;

hipError_t launch_bn_relu_maxpool_encode(const PoolArgs& a, hipStream_t stream);
hipError_t launch_stem_conv_pool(const PoolArgs& a, hipStream_t stream);

// Squeeze-excite gate (tq_se.hip): gate = sigmoid(expand(swish(reduce(x_sq)))), both 1x1
// convs term-pair with int32 weight codes and int64 sums (as tr_conv_wide.hip).
struct SeGateArgs {
  const float* x_sq;      // [N][C] pooled activations
  int N, C;
  const int32_t* w_r;     // reduce conv weight codes [Cse][Cpr] (Cpr = roundup(C, 8), pad 0)
  int Cse, Cpr;
  double scale_r;         // double(fp32 sf_x) * double(fp32 sf_w)
  const float* bias_r;    // [Cse] or nullptr
  double inv_r;           // RN64(1 / sf) of the reduce conv's input quantizer
  float maxv_r;
  int k_r;
  const int32_t* w_e_t;   // expand conv weight codes transposed, [Cse][C]
  double scale_e;
  const float* bias_e;    // [C] or nullptr
  double inv_e;
  float maxv_e;
  int k_e;
  float* gate;            // [N][C]
};
hipError_t launch_se_gate(const SeGateArgs& a, hipStream_t stream);

hipError_t launch_act_encode_act(const float* x, const float* ch_scale, const float* ch_shift,
                                 const float* gate, int act, float* out,
                                 int64_t N, int64_t C, int64_t H, int64_t W, float sf,
                                 int bitwidth, int k, int16_t* codes, int64_t Cp, int fmt,
                                 hipStream_t stream);
hipError_t launch_act_encode(const float* x, int in_nhwc, int64_t N, int64_t C, int64_t H,
                             int64_t W, float sf, int bitwidth, int k, int16_t* codes, int64_t Cp,
                             int fmt, hipStream_t stream);

int conv_tile_m(int64_t cout);
int conv_num_configs();
int64_t conv_workspace_bytes(int64_t p, int64_t cout);
int device_cus();  // CUs of the current device (cached per thread)
// stream-K patch engine: slab + tile-counter bytes it needs in ConvArgs.ws
int64_t patch_streamk_ws_bytes(int64_t p, int64_t cout);

hipError_t launch_mse_profile(const float* x, const float* hist, int64_t nbins, const float* sfs,
                              int64_t nsf, int bitwidth, int k, double* errs, hipStream_t stream);
hipError_t launch_conv2d_tp(const ConvArgs& a, int out_nhwc, hipStream_t stream);
// tracking histogram (tq_calib.hip): hist[b] += count of x in bin b (torch.histc bin rule),
// counts = zeroed uint64 scratch [nbins], left zeroed
hipError_t launch_histc(const float* x, int64_t n, int nbins, float minv, float maxv,
                        unsigned long long* counts, float* hist, hipStream_t stream);

// MFMA engine: x, w hold fp16 codes (kCodesF16), Kp % 64 == 0, Cout_pad % 128 == 0.
hipError_t launch_conv2d_mfma(const ConvArgs& a, int out_nhwc, hipStream_t stream);
int conv_mfma_num_configs();
// MFMA input-patch engine (tr_conv_patch.hip): stride-1 convs with Cp % 64 == 0, NHWC out.
bool conv_patch_eligible(const ConvArgs& a, int out_nhwc);
hipError_t launch_conv2d_patch(const ConvArgs& a, int mb, hipStream_t stream);
// MFMA direct engine (tr_conv_direct.hip): Cp % 64 == 0, NHWC out; mb = 1 (64 x 128 tiles)
// or 2 (128 x 128 tiles).
bool conv_pw_eligible(const ConvArgs& a, int out_nhwc);
hipError_t launch_conv2d_pw(const ConvArgs& a, hipStream_t stream);
bool conv_direct_eligible(const ConvArgs& a, int out_nhwc);
hipError_t launch_conv2d_direct(const ConvArgs& a, int mb, hipStream_t stream);
// MFMA tap-ring engine (tr_conv_ring.hip): 3x3 stride-1 "same" convs, Cp % 64 == 0, NHWC out,
// persistent workgroups streaming K-steps across tiles.
bool conv_xp_eligible(const ConvArgs& a, int out_nhwc);
hipError_t launch_conv2d_xp(const ConvArgs& a, hipStream_t stream);
bool conv_ring_eligible(const ConvArgs& a, int out_nhwc);
hipError_t launch_conv2d_ring(const ConvArgs& a, hipStream_t stream);
// MFMA Cout-64 pixel-ring engine (tr_conv_c64.hip): 3x3 stride-1 pad-1 64 -> 64 convs, ReLU
// + table codes epilogue forms, NHWC out (ResNet-18 layer 1).
bool conv_c64_eligible(const ConvArgs& a, int out_nhwc);
hipError_t launch_conv2d_c64(const ConvArgs& a, hipStream_t stream);
// MFMA row-strip engine (tr_conv_strip.hip): 3x3 stride-1 pad-1 convs with 64 -> 64 channels,
// W % 8 == 0, W <= 56, kc_steps == 0, NHWC out (ResNet-18 layer 1).
bool conv_strip_eligible(const ConvArgs& a, int out_nhwc);
hipError_t launch_conv2d_strip(const ConvArgs& a, hipStream_t stream);
// reads and clears the strip engine's team-sync fault counter (synchronous)
hipError_t strip_sync_faults(uint32_t* count);

}  // namespace tq
