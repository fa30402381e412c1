// Squeeze-excite gate of EfficientNet-b0's MBConv blocks in one launch (the fused executor,
// tq_fuse.FusedEfficientNet): given the pooled block activations x_sq = avgpool(d) [N][C],
//   gate = sigmoid(se_expand(swish(se_reduce(x_sq))))
// with both 1x1 convs term-revealed at the (16, 1, 16) settings of
// cnn_models.static_conv_layer_settings (reference cnn_models/__init__.py:52-65): each conv
// is TR(input) (tr_layer.py:96-99, the consumer's calibrated quantizer) times int32 weight
// codes, summed exactly in int64 and folded once, fp32(double(acc) * scale + bias), as
// tr_conv_wide.hip does; swish and sigmoid are torch's fp32 compositions (tq_device.h
// swish_f32: x * (1 / (1 + exp(-x)))), so the gate equals the module path's
// (TRConv2dLayer "wide" + torch swish / sigmoid) bit for bit for the same x_sq.
//
// The module path spends ~7 launches per block on [N, C, 1, 1] tensors (two act_encode
// passes, two wide-conv GEMMs of 10-40 us each, swish, sigmoid, a copy); here one workgroup
// per image holds the codes in LDS: the reduce conv's Cse outputs are wave dot products over C
// with an int64 wave reduction, the expand conv's C outputs one lane each over Cse.
#include <math.h>

#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

// 16 waves: the launch has only N workgroups (one per image, fewer than the CUs), so one
// workgroup's latency is the kernel's time -- spread each image's outputs over more waves
constexpr int kSeThreads = 1024;
constexpr int kSeU = 8;  // weight loads in flight per lane

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ __launch_bounds__(kSeThreads) void se_gate_kernel(SeGateArgs a) {
  extern __shared__ int32_t se_lds[];
  int32_t* vx = se_lds;          // [Cpr] codes of x_sq (reduce conv input)
  int32_t* v2 = se_lds + a.Cpr;  // [Cse] codes of swish(reduce) (expand conv input)
  const int n = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* xin = a.x_sq + (int64_t)n * a.C;
  for (int c = tid; c < a.Cpr; c += kSeThreads)
    vx[c] = c < a.C ? tr_value_g1_inv(xin[c], a.inv_r, a.maxv_r, a.k_r) : 0;
  __syncthreads();
  // reduce conv: output j by wave j % 16, its lanes along the input channels
  for (int j = wave; j < a.Cse; j += kSeThreads / 64) {
    const int32_t* w = a.w_r + (int64_t)j * a.Cpr;
    // kSeU independent loads in flight per lane (the loop is paced by L2 latency)
    int64_t acc = 0;
    for (int c0 = lane; c0 < a.Cpr; c0 += 64 * kSeU) {
      int32_t wv[kSeU];
#pragma unroll
      for (int u = 0; u < kSeU; ++u) wv[u] = c0 + 64 * u < a.Cpr ? w[c0 + 64 * u] : 0;
#pragma unroll
      for (int u = 0; u < kSeU; ++u)
        if (c0 + 64 * u < a.Cpr) acc += (int64_t)vx[c0 + 64 * u] * (int64_t)wv[u];
    }
    acc = wave_sum_i64(acc);
    if (lane == 0) {
      const float y = (float)((double)acc * a.scale_r + (a.bias_r ? (double)a.bias_r[j] : 0.0));
      v2[j] = tr_value_g1_inv(swish_f32(y), a.inv_e, a.maxv_e, a.k_e);
    }
  }
  __syncthreads();
  // expand conv + sigmoid: one output channel per lane (weights k-major: coalesced rows)
  float* g = a.gate + (int64_t)n * a.C;
  for (int c = tid; c < a.C; c += kSeThreads) {
    int64_t acc = 0;
    for (int j0 = 0; j0 < a.Cse; j0 += kSeU) {
      int32_t wv[kSeU];
#pragma unroll
      for (int u = 0; u < kSeU; ++u)
        wv[u] = j0 + u < a.Cse ? a.w_e_t[(int64_t)(j0 + u) * a.C + c] : 0;
#pragma unroll
      for (int u = 0; u < kSeU; ++u)
        if (j0 + u < a.Cse) acc += (int64_t)v2[j0 + u] * (int64_t)wv[u];
    }
    const float y = (float)((double)acc * a.scale_e + (a.bias_e ? (double)a.bias_e[c] : 0.0));
    g[c] = 1.0f / (1.0f + expf(-y));
  }
}

}  // namespace

hipError_t launch_se_gate(const SeGateArgs& a, hipStream_t stream) {
  if (a.N == 0) return hipSuccess;
  const size_t lds = (size_t)(a.Cpr + a.Cse) * sizeof(int32_t);
  se_gate_kernel<<<dim3((unsigned)a.N), kSeThreads, lds, stream>>>(a);
  return hipGetLastError();
}

}  // namespace tq
