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
};

hipError_t launch_act_encode(const float* x, int in_nhwc, int64_t N, int64_t C, int64_t H,
                             int64_t W, float sf, int bitwidth, int k, int16_t* codes, int64_t Cp,
                             hipStream_t stream);

int conv_tile_m(int64_t cout);

hipError_t launch_mse_profile(const float* x, const float* hist, int64_t nbins, const float* sfs,
                              int64_t nsf, int bitwidth, int k, double* errs, hipStream_t stream);
hipError_t launch_conv2d_tp(const ConvArgs& a, int out_nhwc, hipStream_t stream);

}  // namespace tq
