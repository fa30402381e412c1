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

// ---------------------------------------------------------------------------------------
// Tracking histogram: hist[b] += count of x in bin b, the reference's
// `hist_bins += torch.histc(x, nbins, minv, maxv)` (tr_layer.py:91-94), in two launches.
// Bin rule of torch.histc on the GPU: elements outside [minv, maxv] (and NaN) are skipped,
// b = int(fp32((x - minv) * nbins) / (maxv - minv)), b == nbins -> nbins - 1, all in fp32.
// Counts are exact integers (uint32 in LDS, uint64 in HBM); torch.histc counts in fp32
// atomics, which stop counting at 2^24 per bin (16777216 + 1 == 16777216 in fp32) -- a bin
// of a ReLU output (all the exact zeros of a 256-image layer-1 activation: ~25 M) exceeds
// that.  The final fp32 add into hist is the reference's `+=`.
constexpr int kHistThreads = 256;

__device__ __forceinline__ int hist_bin(float v, float minv, float maxv, float fbins, int nbins) {
#pragma clang fp contract(off)
  if (!(v >= minv && v <= maxv)) return -1;
  int b = (int)((v - minv) * fbins / (maxv - minv));
  return b == nbins ? nbins - 1 : b;
}

// One element per lane and call: the lanes whose bin is the hot bin (the bin of 0, where a
// ReLU output piles up) add once per wave (ballot + popcount) instead of serialising on one
// LDS address; the others take an LDS atomic.
__device__ __forceinline__ void hist_add(uint32_t* h, int b, int hot) {
  const uint64_t m = __ballot(b == hot && b >= 0);
  if (m) {
    const int lead = __ffsll((unsigned long long)m) - 1;
    if ((int)(threadIdx.x & 63) == lead) atomicAdd(h + hot, (uint32_t)__popcll(m));
  }
  if (b >= 0 && b != hot) atomicAdd(h + b, 1u);
}

template <bool LDS>
__global__ __launch_bounds__(kHistThreads) void histc_kernel(
    const float* __restrict__ x, int64_t n, int nbins, float minv, float maxv, int hot,
    unsigned long long* __restrict__ counts) {
  extern __shared__ uint32_t hs[];
  const float fbins = (float)nbins;
  if (LDS) {
    for (int b = threadIdx.x; b < nbins; b += kHistThreads) hs[b] = 0u;
    __syncthreads();
  }
  const int64_t nvec = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kHistThreads;
  const float4* xv = reinterpret_cast<const float4*>(x);
  auto add = [&](float v) {
    const int b = hist_bin(v, minv, maxv, fbins, nbins);
    if (LDS) {
      hist_add(hs, b, hot);
    } else if (b >= 0) {
      atomicAdd(counts + b, 1ull);
    }
  };
  // the loop trip count is wave-uniform (whole waves step together), so the ballots inside
  // see every lane; lanes past the end contribute bin -1
  const int64_t base = (int64_t)blockIdx.x * kHistThreads;
  for (int64_t i0 = 0; i0 * stride + base < nvec; ++i0) {
    const int64_t i = i0 * stride + base + threadIdx.x;
    float4 v = make_float4(NAN, NAN, NAN, NAN);
    if (i < nvec) v = xv[i];
    add(v.x);
    add(v.y);
    add(v.z);
    add(v.w);
  }
  if (blockIdx.x == 0) {  // tail (n % 4 elements), one full wave so the ballot is uniform
    const int64_t t = (nvec << 2) + threadIdx.x;
    if (threadIdx.x < 64) add(t < n ? x[t] : NAN);
  }
  if (LDS) {
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += kHistThreads) {
      const uint32_t c = hs[b];
      if (c) atomicAdd(counts + b, (unsigned long long)c);
    }
  }
}

// hist[b] += fp32(counts[b]); counts[b] = 0 (the scratch is left zeroed for the next call).
__global__ __launch_bounds__(kHistThreads) void histc_finish_kernel(
    unsigned long long* __restrict__ counts, float* __restrict__ hist, int nbins) {
  const int b = blockIdx.x * kHistThreads + threadIdx.x;
  if (b >= nbins) return;
  const unsigned long long c = counts[b];
  if (c) {
    hist[b] += (float)c;
    counts[b] = 0ull;
  }
}

}  // namespace

int hist_bin_host(float v, float minv, float maxv, int nbins) {
#pragma clang fp contract(off)
  if (!(v >= minv && v <= maxv)) return -1;
  int b = (int)((v - minv) * (float)nbins / (maxv - minv));
  return b == nbins ? nbins - 1 : b;
}

hipError_t launch_histc(const float* x, int64_t n, int nbins, float minv, float maxv,
                        unsigned long long* counts, float* hist, hipStream_t stream) {
  if (n > 0) {
    const int hot = hist_bin_host(0.0f, minv, maxv, nbins);
    const int64_t want = (n / 4 + kHistThreads - 1) / kHistThreads;
    const int64_t cap = 2 * (int64_t)device_cus();
    const unsigned grid = (unsigned)(want < 1 ? 1 : (want < cap ? want : cap));
    const size_t lds = (size_t)nbins * sizeof(uint32_t);
    if (lds <= 64 * 1024)
      histc_kernel<true><<<dim3(grid), kHistThreads, lds, stream>>>(x, n, nbins, minv, maxv, hot,
                                                                   counts);
    else
      histc_kernel<false><<<dim3(grid), kHistThreads, 0, stream>>>(x, n, nbins, minv, maxv, hot,
                                                                   counts);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (nbins > 0)
    histc_finish_kernel<<<dim3((unsigned)((nbins + kHistThreads - 1) / kHistThreads)),
                          kHistThreads, 0, stream>>>(counts, hist, nbins);
  return hipGetLastError();
}

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
