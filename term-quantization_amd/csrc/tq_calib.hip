// Batched activation-scale calibration: tr_layer.mse_profile (tr_layer.py:43-54) in one
// launch instead of 2048 TR launches + 2048 device->host syncs per layer.
//
// errs[s] = sum_b hist[b] * (x[b] - TR(x[b]; sfs[s]))^2 for every candidate s.  The
// per-bin product is formed in fp32 exactly as the reference's torch expression
// `hist * (x - xh)**2` does; the sum over bins runs in fp64 in a fixed order (the
// reference's fp32 torch reduction order is implementation-defined), so the first arg-min
// can differ from the reference's only between candidates whose errors tie in fp32.
#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

constexpr int kCalibThreads = 256;

__global__ __launch_bounds__(kCalibThreads) void mse_profile_kernel(
    const float* __restrict__ x, const float* __restrict__ hist, int nbins,
    const float* __restrict__ sfs, float maxv, int k, double* __restrict__ errs) {
  // no fma contraction: the reference materialises xh = tr(x) as a tensor and then computes
  // x - xh, two roundings (a contracted x - v*sf would skip xh's rounding)
#pragma clang fp contract(off)
  __shared__ double part[kCalibThreads];
  const float sf = sfs[blockIdx.x];
  double acc = 0.0;
  for (int b = threadIdx.x; b < nbins; b += kCalibThreads) {
    const float xv = x[b];
    const float xh = (float)tr_value_g1(xv, sf, maxv, k) * sf;
    const float d = xv - xh;
    const float e = hist[b] * (d * d);
    acc += (double)e;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kCalibThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) errs[blockIdx.x] = part[0];
}

}  // namespace

hipError_t launch_mse_profile(const float* x, const float* hist, int64_t nbins, const float* sfs,
                              int64_t nsf, int bitwidth, int k, double* errs,
                              hipStream_t stream) {
  if (nsf == 0) return hipSuccess;
  const float maxv = (float)((1u << bitwidth) - 1u);
  mse_profile_kernel<<<dim3((unsigned)nsf), kCalibThreads, 0, stream>>>(x, hist, (int)nbins, sfs,
                                                                        maxv, k, errs);
  return hipGetLastError();
}

}  // namespace tq
