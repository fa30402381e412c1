// The term-revealing (TR) op -- kernels/tr_cuda_kernel.cu rebuilt for CDNA4 (gfx950).
//
// Two kernels instead of one thread-per-element kernel with (g-1)/g idle lanes:
//   tr_elem_kernel   group_size == 1 (every activation call, tr_layer.py:96-99):
//                    a pure HBM stream, 16 B per lane per load, several loads in flight.
//   tr_group_kernel  group_size > 1 (weights, tr_layer.py:117-121): one lane per group,
//                    lanes along the innermost (spatial) axis so each of the g loads is
//                    coalesced across the wave; selection by exponent threshold.
// Both produce exactly the reference's output (DESIGN.md "TR op contract").
#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

constexpr int kThreads = 256;
constexpr int kUnroll = 4;  // 16-B loads in flight per lane

template <typename T>
struct Vec16;
template <>
struct Vec16<float> {
  using type = float __attribute__((ext_vector_type(4)));
  static constexpr int n = 4;
};
template <>
struct Vec16<double> {
  using type = double __attribute__((ext_vector_type(2)));
  static constexpr int n = 2;
};

template <typename T>
__device__ __forceinline__ T tr_scale(int32_t v, float sf) {
  // kernels/tr_cuda_kernel.cu:112,122: scalar_t(sum of kept terms) * sf, one rounding.
  return (T)v * (T)sf;
}

template <typename T>
__device__ __forceinline__ void tr_vec(typename Vec16<T>::type& v, float sf, float maxv, int k) {
  T* e = reinterpret_cast<T*>(&v);
#pragma unroll
  for (int i = 0; i < Vec16<T>::n; ++i) e[i] = tr_scale<T>(tr_value_g1(e[i], sf, maxv, k), sf);
}

// group_size == 1: out[i] = TR(in[i]).  `nvec` 16-byte vectors, then a scalar tail.
template <typename T>
__global__ __launch_bounds__(kThreads) void tr_elem_kernel(const T* __restrict__ in,
                                                           T* __restrict__ out, int64_t nvec,
                                                           int64_t n, float sf, float maxv,
                                                           int k) {
  using V = typename Vec16<T>::type;
  const V* vin = reinterpret_cast<const V*>(in);
  V* vout = reinterpret_cast<V*>(out);
  const int64_t base = (int64_t)blockIdx.x * (kThreads * kUnroll) + threadIdx.x;
  V r[kUnroll];
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) {
    const int64_t i = base + u * kThreads;
    if (i < nvec) r[u] = __builtin_nontemporal_load(vin + i);
  }
#pragma unroll
  for (int u = 0; u < kUnroll; ++u) {
    const int64_t i = base + u * kThreads;
    if (i < nvec) {
      tr_vec<T>(r[u], sf, maxv, k);
      __builtin_nontemporal_store(r[u], vout + i);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = nvec * Vec16<T>::n + threadIdx.x; i < n; i += kThreads)
      out[i] = tr_scale<T>(tr_value_g1(in[i], sf, maxv, k), sf);
  }
}

// Scalar variant for misaligned views (any base address).
template <typename T>
__global__ __launch_bounds__(kThreads) void tr_elem_scalar_kernel(const T* __restrict__ in,
                                                                  T* __restrict__ out, int64_t n,
                                                                  float sf, float maxv, int k) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) out[i] = tr_scale<T>(tr_value_g1(in[i], sf, maxv, k), sf);
}

// group_size > 1.  Group (b, cg, s): channels [cg*g, min(cg*g+g, C)) of row b at spatial
// offset s (kernels/tr_cuda_kernel.cu:69-90, with the partial last group of DESIGN.md).
// Selection (kernels/tr_cuda_kernel.cu:92-116) == keep the first k terms of the group in
// (exponent desc, channel asc) order: find the threshold exponent e* with
// count(exp > e*) < k <= count(exp >= e*), keep everything above it, and at e* keep the
// lowest channels first.
template <typename T, int GMAX>
__global__ __launch_bounds__(kThreads) void tr_group_kernel(
    const T* __restrict__ in, T* __restrict__ out, int32_t* __restrict__ codes, int64_t B,
    int64_t C, int64_t WH, int g, int k, float sf, float maxv, int emax) {
  const int64_t ncg = (C + g - 1) / g;
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (t >= B * ncg * WH) return;
  const int64_t s = t % WH;
  const int64_t rest = t / WH;
  const int64_t cg = rest % ncg;
  const int64_t b = rest / ncg;
  const int gs = (int)min((int64_t)g, C - cg * g);
  const int64_t base = b * C * WH + cg * g * WH + s;

  uint32_t qv[GMAX];
  uint32_t m[GMAX];
  uint32_t negmask = 0;
  int total = 0;
#pragma unroll
  for (int j = 0; j < GMAX; ++j) {
    qv[j] = 0;
    m[j] = 0;
    if (j < gs) {
      const T x = in[base + j * WH];
      qv[j] = quantize_mag(x, sf, maxv);
      uint32_t p, n;
      hese_masks(qv[j], p, n);
      m[j] = p | n;
      negmask |= (x < (T)0 ? 1u : 0u) << j;
      total += __popc(m[j]);
    }
  }

  if (total > k) {
    // threshold exponent: q <= 2^bw - 1 puts every term at exponent <= bw = emax
    int above = 0;
    int e = emax;
    for (; e > 0; --e) {
      int c = 0;
#pragma unroll
      for (int j = 0; j < GMAX; ++j) c += (m[j] >> e) & 1u;
      if (above + c >= k) break;
      above += c;
    }
    const uint32_t hi = (e >= 31) ? 0u : (0xFFFFFFFFu << (e + 1));
    int need = k - above;
#pragma unroll
    for (int j = 0; j < GMAX; ++j) {
      const uint32_t bit = m[j] & (1u << e);
      uint32_t keep = m[j] & hi;
      if (bit && need > 0) {
        keep |= bit;
        --need;
      }
      m[j] = keep;
    }
  }

#pragma unroll
  for (int j = 0; j < GMAX; ++j) {
    if (j < gs) {
      uint32_t p, n;
      hese_masks(qv[j], p, n);
      const int32_t v = kept_value(p, n, m[j], (negmask >> j) & 1u);
      const int64_t o = base + j * WH;
      out[o] = tr_scale<T>(v, sf);
      if (codes) codes[o] = v;
    }
  }
}

template <typename T>
hipError_t launch_group(const T* in, T* out, int32_t* codes, int64_t B, int64_t C, int64_t WH,
                        int g, int k, float sf, float maxv, int emax, hipStream_t stream) {
  const int64_t n = B * ((C + g - 1) / g) * WH;
  const dim3 grid((unsigned)((n + kThreads - 1) / kThreads));
  const int bucket = g <= 2 ? 2 : g <= 4 ? 4 : g <= 8 ? 8 : g <= 16 ? 16 : 32;
  switch (bucket) {
#define TQ_GROUP_CASE(G)                                                                      \
  case G:                                                                                     \
    tr_group_kernel<T, G><<<grid, kThreads, 0, stream>>>(in, out, codes, B, C, WH, g, k, sf,  \
                                                         maxv, emax);                         \
    break;
    TQ_GROUP_CASE(2)
    TQ_GROUP_CASE(4)
    TQ_GROUP_CASE(8)
    TQ_GROUP_CASE(16)
    TQ_GROUP_CASE(32)
#undef TQ_GROUP_CASE
  }
  return hipGetLastError();
}

}  // namespace

template <typename T>
hipError_t launch_tr(const T* in, T* out, int32_t* codes, int64_t B, int64_t C, int64_t WH,
                     int64_t numel, float sf, int bitwidth, int g, int k, hipStream_t stream) {
  const float maxv = (float)((1u << bitwidth) - 1u);
  const int64_t active = B * C * WH;  // elements the reference kernel touches
  if (active < numel) {
    // 3-D / 5-D inputs: the reference treats only the first B*C elements as a (B, C)
    // matrix and leaves the rest as at::zeros_like (kernels/tr_cuda_kernel.cu:133-145).
    hipError_t e = hipMemsetAsync(out + active, 0, (numel - active) * sizeof(T), stream);
    if (e != hipSuccess) return e;
  }
  if (active == 0) return hipSuccess;
  if (g == 1 && codes == nullptr) {
    constexpr int VN = Vec16<T>::n;
    const bool aligned = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0);
    if (aligned) {
      const int64_t nvec = active / VN;
      const int64_t per_block = (int64_t)kThreads * kUnroll;
      const int64_t blocks = nvec > 0 ? (nvec + per_block - 1) / per_block : 1;
      tr_elem_kernel<T><<<dim3((unsigned)blocks), kThreads, 0, stream>>>(in, out, nvec, active,
                                                                          sf, maxv, k);
    } else {
      tr_elem_scalar_kernel<T><<<dim3((unsigned)((active + kThreads - 1) / kThreads)), kThreads,
                                 0, stream>>>(in, out, active, sf, maxv, k);
    }
    return hipGetLastError();
  }
  return launch_group<T>(in, out, codes, B, C, WH, g, k, sf, maxv, bitwidth, stream);
}

template hipError_t launch_tr<float>(const float*, float*, int32_t*, int64_t, int64_t, int64_t,
                                     int64_t, float, int, int, int, hipStream_t);
template hipError_t launch_tr<double>(const double*, double*, int32_t*, int64_t, int64_t,
                                      int64_t, int64_t, float, int, int, int, hipStream_t);

}  // namespace tq
