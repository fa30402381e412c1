// Classifier head of the fused ResNet executor (tq_fuse.FusedResNet): global average pool
// of the last block's fp32 output and the fp32 Linear, the two torch calls that end the
// reference's forward (torchvision ResNet.forward: avgpool -> flatten -> fc; neither is a TQ
// layer -- cnn_models/__init__.py converts convolutions only).  Two short launches instead of
// torch's reduce kernel and a library GEMM of this 256 x 512 x 1000 shape (8.7 + 11.6 us in
// the round-5 layer trace, profiles/r05g_layer_times.txt).  fp32 like the reference (its
// summation orders are unpinned: a cuDNN / cuBLAS choice).
#include "tq_launch.h"

namespace tq {

namespace {

// pooled[n][c] = (sum over the HW positions of x[n][p][c]) / HW, x channels_last fp32
__global__ __launch_bounds__(128) void avgpool_kernel(const float* __restrict__ x,
                                                      float* __restrict__ pooled, int HW,
                                                      int C) {
  const int n = blockIdx.x;
  const float* xn = x + (int64_t)n * HW * C;
  for (int c = threadIdx.x * 4; c < C; c += 128 * 4) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < HW; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(xn + (int64_t)p * C + c);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    const float d = (float)HW;
    *reinterpret_cast<float4*>(pooled + (int64_t)n * C + c) =
        make_float4(s.x / d, s.y / d, s.z / d, s.w / d);
  }
}

// out[n][o] = sum_c pooled[n][c] w[o][c] + b[o]: block = 16 images x 16 outputs, one
// output per thread, both operands' rows staged in LDS 256 channels at a time
constexpr int kFcT = 16;
constexpr int kFcK = 256;
__global__ __launch_bounds__(kFcT * kFcT) void fc_kernel(const float* __restrict__ pooled,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ b,
                                                         float* __restrict__ out, int N, int C,
                                                         int O) {
  __shared__ __attribute__((aligned(16))) float ps[kFcT][kFcK + 4];
  __shared__ __attribute__((aligned(16))) float ws[kFcT][kFcK + 4];
  const int n0 = blockIdx.x * kFcT, o0 = blockIdx.y * kFcT;
  const int tid = threadIdx.x;
  const int ni = tid / kFcT, oi = tid - ni * kFcT;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int c0 = 0; c0 < C; c0 += kFcK) {
    const int kc = C - c0 < kFcK ? C - c0 : kFcK;
    __syncthreads();  // the previous chunk is no longer read
    for (int i = tid * 4; i < kFcT * kFcK; i += kFcT * kFcT * 4) {
      const int r = i / kFcK, c = i - r * kFcK;
      const bool okc = c < kc;
      const float4 pv = okc && n0 + r < N
                            ? *reinterpret_cast<const float4*>(pooled + (int64_t)(n0 + r) * C + c0 + c)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 wv = okc && o0 + r < O
                            ? *reinterpret_cast<const float4*>(w + (int64_t)(o0 + r) * C + c0 + c)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(&ps[r][c]) = pv;
      *reinterpret_cast<float4*>(&ws[r][c]) = wv;
    }
    __syncthreads();
    for (int c = 0; c < kc; c += 4) {
      const float4 pv = *reinterpret_cast<const float4*>(&ps[ni][c]);
      const float4 wv = *reinterpret_cast<const float4*>(&ws[oi][c]);
      s0 = fmaf(pv.x, wv.x, s0);
      s1 = fmaf(pv.y, wv.y, s1);
      s2 = fmaf(pv.z, wv.z, s2);
      s3 = fmaf(pv.w, wv.w, s3);
    }
  }
  if (n0 + ni < N && o0 + oi < O)
    out[(int64_t)(n0 + ni) * O + o0 + oi] = (s0 + s1) + (s2 + s3) + (b ? b[o0 + oi] : 0.0f);
}

}  // namespace

hipError_t launch_avgpool_fc(const float* x, int64_t N, int64_t HW, int64_t C, const float* w,
                             const float* b, int64_t O, float* pooled, float* out,
                             hipStream_t stream) {
  if (N == 0 || O == 0) return hipSuccess;
  avgpool_kernel<<<dim3((unsigned)N), 128, 0, stream>>>(x, pooled, (int)HW, (int)C);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  fc_kernel<<<dim3((unsigned)((N + kFcT - 1) / kFcT), (unsigned)((O + kFcT - 1) / kFcT)),
              kFcT * kFcT, 0, stream>>>(pooled, w, b, out, (int)N, (int)C, (int)O);
  return hipGetLastError();
}

}  // namespace tq
