// Stem tail of a TQ ResNet in one pass: eval-mode BatchNorm -> ReLU -> max-pool -> fp32
// output and the first TR layer's activation codes (tr_layer.py:96-99).  The reference runs
// these as four torch passes over the stem's 256x64x112x112 fp32 output (bn1, relu,
// maxpool, then the first TRConv2dLayer's input TR); the stem conv itself stays the
// reference's fp32 conv (cnn_models/__init__.py:34-36 never converts it).
//
// max-pool commutes with the monotone ReLU, and BN is applied per element before the max
// (its scale may be negative), so y = relu(max_window(x * a_c + b_c)) per channel.  Window
// positions outside the input are skipped (-inf padding, as nn.MaxPool2d).
#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

__global__ __launch_bounds__(256) void bn_relu_maxpool_encode_kernel(PoolArgs a) {
  const int chunks = a.C / 8;
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
  float sc[8], sh[8], m[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = a.scale[c0 + i];
    sh[i] = a.shift[c0 + i];
    m[i] = -INFINITY;
  }
  for (int r = 0; r < a.k; ++r) {
    const int ih = oh * a.s - a.pad + r;
    if (ih < 0 || ih >= a.H) continue;
    for (int q = 0; q < a.k; ++q) {
      const int iw = ow * a.s - a.pad + q;
      if (iw < 0 || iw >= a.W) continue;
      const float* src = a.x + ((img * a.H + ih) * a.W + iw) * a.C + c0;
      const float4 v0 = *reinterpret_cast<const float4*>(src);
      const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
      const float xv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) m[i] = fmaxf(m[i], fmaf(xv[i], sc[i], sh[i]));
    }
  }
  float y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) y[i] = m[i] > 0.0f ? m[i] : 0.0f;
  float* dst = a.out + p * a.C + c0;
  *reinterpret_cast<float4*>(dst) = make_float4(y[0], y[1], y[2], y[3]);
  *reinterpret_cast<float4*>(dst + 4) = make_float4(y[4], y[5], y[6], y[7]);
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    int16_t* codes = side ? a.codes_b : a.codes_a;
    if (!codes) continue;
    const double inv = side ? a.inv_b : a.inv_a;
    const float maxv = side ? a.maxv_b : a.maxv_a;
    const int k = side ? a.k_b : a.k_a;
    const int cp = side ? a.cp_b : a.cp_a;
    const int fmt = side ? a.fmt_b : a.fmt_a;
    uint32_t b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = code_bits(tr_value_g1_inv(y[i], inv, maxv, k), fmt);
    *reinterpret_cast<uint4*>(codes + p * cp + c0) = make_uint4(
        b[0] | (b[1] << 16), b[2] | (b[3] << 16), b[4] | (b[5] << 16), b[6] | (b[7] << 16));
  }
}

}  // namespace

hipError_t launch_bn_relu_maxpool_encode(const PoolArgs& a, hipStream_t stream) {
  const int64_t n = (int64_t)a.N * a.Ho * a.Wo * (a.C / 8);
  if (n == 0) return hipSuccess;
  bn_relu_maxpool_encode_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace tq
