// Host (CPU) term-revealing op -- libtq_host.so, declared in include/tq_host.h.
//
// The product path for CPU tensors (the reference's MNIST config runs on CPU
// torch, evaluate_mlp.py:56-57).  Same design as the HIP kernels, restated for a CPU core:
//   a1 quantize   kernels/tr_cuda_kernel.cu:21-23 -- fp32 |x| / sf (IEEE division; the host
//                 has no reason to avoid it), double +0.5, saturating truncation, clamp
//   a2 encode     kernels/tr_cuda_kernel.cu:25-55 -- the closed-form HESE masks of
//                 csrc/tq_device.h (one pos and one neg bit mask per element)
//   a3 select     kernels/tr_cuda_kernel.cu:85-116 -- keep the first k terms of the group in
//                 (exponent desc, channel asc) order via the threshold exponent
//   a4 rescale    kernels/tr_cuda_kernel.cu:112,118-123 -- scalar_t(v) * sf, one rounding
// Built with -ffp-contract=off and without fast-math: every rounding step is the
// reference's.  OpenMP splits groups (or elements, g = 1) across threads; each output
// element is written by exactly one thread.
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <omp.h>

#include "../../include/tq.h"
#include "../../include/tq_host.h"

namespace {

constexpr int kMaxGroupSize = 32;  // kernels/tr_cuda_kernel.cu:9
constexpr int kMaxBitwidth = 24;   // as the HIP library (csrc/tq_device.h kMaxBitwidth)
constexpr int kCalibPartials = 256;  // csrc/tq_calib.hip kCalibThreads: same summation order

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

// cvt.rzi.s32.f64 of the reference's int32_t(double): truncate, saturate, NaN -> 0.  The
// argument is >= 0.5 or NaN here, so only the upper saturation matters.
inline uint32_t trunc_sat_clamp(double t, uint32_t maxq) {
  if (!(t == t)) return 0u;
  if (t >= 2147483647.0) return maxq;
  const uint32_t q = (uint32_t)(int32_t)t;
  return q < maxq ? q : maxq;
}

// a1 for float32: float / float, then the double literal 0.5 (tr_cuda_kernel.cu:22)
inline uint32_t quantize(float x, float sf, uint32_t maxq) {
  const float r = fabsf(x) / sf;
  return trunc_sat_clamp((double)r + 0.5, maxq);
}

// a1 for the float64 instantiation: all double
inline uint32_t quantize(double x, float sf, uint32_t maxq) {
  return trunc_sat_clamp(fabs(x) / (double)sf + 0.5, maxq);
}

// a2: HESE masks (csrc/tq_device.h hese_masks; q == pos - neg, pos & neg == 0)
inline void hese_masks(uint32_t q, uint32_t& pos, uint32_t& neg) {
  const uint32_t hi = q >> 1;
  const uint32_t lo = q << 1;
  const uint32_t a = q & ~hi;
  pos = (a & ~lo) | ((a & lo) << 1);
  neg = q & hi & ~lo;
}

// a3 for g == 1: keep the k highest set bits
inline uint32_t keep_top(uint32_t m, int k) {
  int drop = __builtin_popcount(m) - k;
  while (drop-- > 0) m &= m - 1u;
  return m;
}

inline int32_t kept_value(uint32_t pos, uint32_t neg, uint32_t keep, bool negative) {
  const int32_t v = (int32_t)(pos & keep) - (int32_t)(neg & keep);
  return negative ? -v : v;
}

template <typename T>
inline int32_t tr_value_g1(T x, float sf, uint32_t maxq, int k) {
  uint32_t p, n;
  hese_masks(quantize(x, sf, maxq), p, n);
  return kept_value(p, n, keep_top(p | n, k), x < (T)0);
}

struct Shape {
  int64_t B, C, WH, numel;
};

int check_args(int64_t ndim, const int64_t* shape, float sf, int32_t bitwidth, int32_t g,
               Shape* s) {
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
  if (bitwidth < 0 || bitwidth > kMaxBitwidth)
    return fail(TQ_ERR_UNSUPPORTED, "tr: bitwidth must be in [0, %d] (got %d)", kMaxBitwidth,
                bitwidth);
  if (g < 1 || g > kMaxGroupSize)
    return fail(TQ_ERR_INVALID_ARGUMENT, "tr: group_size must be in [1, 32] (got %d)", g);
  s->B = shape[0];
  s->C = shape[1];
  s->WH = ndim == 4 ? shape[2] * shape[3] : 1;  // kernels/tr_cuda_kernel.cu:133-141
  s->numel = n;
  return TQ_OK;
}

struct Threads {
  explicit Threads(int n) : n_(n > 0 ? n : omp_get_max_threads()) {}
  int n_;
};

template <typename T>
void tr_g1(const T* in, T* out, int32_t* codes, int64_t n, float sf, uint32_t maxq, int k,
           int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (int64_t i = 0; i < n; ++i) {
    const int32_t v = tr_value_g1(in[i], sf, maxq, k);
    out[i] = (T)v * (T)sf;
    if (codes) codes[i] = v;
  }
}

// Group (b, cg, s): channels [cg*g, min(cg*g+g, C)) of row b at spatial offset s.
template <typename T>
void tr_group(const T* in, T* out, int32_t* codes, const Shape& sh, int g, int k, float sf,
              uint32_t maxq, int emax, int nthreads) {
  const int64_t ncg = (sh.C + g - 1) / g;
  const int64_t total = sh.B * ncg;
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (int64_t r = 0; r < total; ++r) {
    const int64_t b = r / ncg, cg = r % ncg;
    const int gs = (int)(sh.C - cg * g < g ? sh.C - cg * g : g);
    const int64_t row = b * sh.C * sh.WH + cg * g * sh.WH;
    uint32_t pos[kMaxGroupSize], neg[kMaxGroupSize], m[kMaxGroupSize];
    bool negative[kMaxGroupSize];
    for (int64_t s = 0; s < sh.WH; ++s) {
      const int64_t base = row + s;
      int cnt = 0;
      for (int j = 0; j < gs; ++j) {
        const T x = in[base + j * sh.WH];
        hese_masks(quantize(x, sf, maxq), pos[j], neg[j]);
        m[j] = pos[j] | neg[j];
        negative[j] = x < (T)0;
        cnt += __builtin_popcount(m[j]);
      }
      if (cnt > k) {
        // threshold exponent e*: count(exp > e*) < k <= count(exp >= e*)
        int above = 0, e = emax;
        for (; e > 0; --e) {
          int c = 0;
          for (int j = 0; j < gs; ++j) c += (m[j] >> e) & 1u;
          if (above + c >= k) break;
          above += c;
        }
        const uint32_t hi = e >= 31 ? 0u : (0xFFFFFFFFu << (e + 1));
        int need = k - above;
        for (int j = 0; j < gs; ++j) {
          const uint32_t bit = m[j] & (1u << e);
          uint32_t keep = m[j] & hi;
          if (bit && need > 0) {
            keep |= bit;
            --need;
          }
          m[j] = keep;
        }
      }
      for (int j = 0; j < gs; ++j) {
        const int32_t v = kept_value(pos[j], neg[j], m[j], negative[j]);
        const int64_t o = base + j * sh.WH;
        out[o] = (T)v * (T)sf;
        if (codes) codes[o] = v;
      }
    }
  }
}

template <typename T>
int tr_impl(const T* in, T* out, int32_t* codes, int64_t ndim, const int64_t* shape, float sf,
            int32_t bitwidth, int32_t g, int32_t k, int32_t num_threads) {
  Shape sh;
  int rc = check_args(ndim, shape, sf, bitwidth, g, &sh);
  if (rc != TQ_OK) return rc;
  if (sh.numel == 0) return TQ_OK;
  if (in == nullptr || out == nullptr)
    return fail(TQ_ERR_INVALID_ARGUMENT, "tr: null tensor pointer");
  const int kk = k < 0 ? 0 : k;  // num_keep_terms < 0 runs no selection step: nothing kept
  const uint32_t maxq = (1u << bitwidth) - 1u;
  const int nthreads = Threads(num_threads).n_;
  const int64_t active = sh.B * sh.C * sh.WH;  // elements the reference kernel touches
  // 3-D / 5-D inputs: the rest stays at::zeros_like (kernels/tr_cuda_kernel.cu:133-145)
  for (int64_t i = active; i < sh.numel; ++i) {
    out[i] = (T)0;
    if (codes) codes[i] = 0;
  }
  if (g == 1)
    tr_g1<T>(in, out, codes, active, sf, maxq, kk, nthreads);
  else
    tr_group<T>(in, out, codes, sh, g, kk, sf, maxq, bitwidth, nthreads);
  return TQ_OK;
}

}  // namespace

extern "C" {

const char* tq_host_version(void) { return "tq-host 0.1.0"; }

const char* tq_host_last_error(void) { return g_err; }

int tq_tr_f32_host(const float* input, float* output, int64_t ndim, const int64_t* shape,
                   float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms,
                   int32_t num_threads) {
  return tr_impl<float>(input, output, nullptr, ndim, shape, sf, bitwidth, group_size,
                        num_keep_terms, num_threads);
}

int tq_tr_f64_host(const double* input, double* output, int64_t ndim, const int64_t* shape,
                   float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms,
                   int32_t num_threads) {
  return tr_impl<double>(input, output, nullptr, ndim, shape, sf, bitwidth, group_size,
                         num_keep_terms, num_threads);
}

int tq_tr_encode_f32_host(const float* input, float* output, int32_t* codes, int64_t ndim,
                          const int64_t* shape, float sf, int32_t bitwidth, int32_t group_size,
                          int32_t num_keep_terms, int32_t num_threads) {
  if (codes == nullptr) return fail(TQ_ERR_INVALID_ARGUMENT, "tr_encode: codes is null");
  return tr_impl<float>(input, output, codes, ndim, shape, sf, bitwidth, group_size,
                        num_keep_terms, num_threads);
}

int tq_mse_profile_host(const float* x, const float* hist, int64_t nbins, const float* sfs,
                        int64_t nsf, int32_t bitwidth, int32_t num_keep_terms, double* errs,
                        int32_t num_threads) {
  if (nbins < 0 || nsf < 0 || nbins > (1 << 30) || nsf > (1 << 30))
    return fail(TQ_ERR_INVALID_ARGUMENT, "mse_profile: bad sizes");
  if (bitwidth < 0 || bitwidth > kMaxBitwidth)
    return fail(TQ_ERR_UNSUPPORTED, "mse_profile: bitwidth must be in [0, %d] (got %d)",
                kMaxBitwidth, bitwidth);
  if (nsf == 0) return TQ_OK;
  if (nbins > 0 && (x == nullptr || hist == nullptr))
    return fail(TQ_ERR_INVALID_ARGUMENT, "mse_profile: null pointer");
  if (sfs == nullptr || errs == nullptr)
    return fail(TQ_ERR_INVALID_ARGUMENT, "mse_profile: null pointer");
  for (int64_t s = 0; s < nsf; ++s)
    if (!(sfs[s] >= 0.0f))
      return fail(TQ_ERR_INVALID_ARGUMENT, "mse_profile: sf must be >= 0 (got %g)",
                  (double)sfs[s]);
  const int k = num_keep_terms < 0 ? 0 : num_keep_terms;
  const uint32_t maxq = (1u << bitwidth) - 1u;
  const int nthreads = Threads(num_threads).n_;
#pragma omp parallel for schedule(dynamic, 8) num_threads(nthreads)
  for (int64_t s = 0; s < nsf; ++s) {
    const float sf = sfs[s];
    double part[kCalibPartials];
    for (int t = 0; t < kCalibPartials; ++t) {
      double acc = 0.0;
      for (int64_t b = t; b < nbins; b += kCalibPartials) {
        const float xv = x[b];
        const float xh = (float)tr_value_g1(xv, sf, maxq, k) * sf;  // the tr() tensor
        const float d = xv - xh;                                    // x - xh
        const float e = hist[b] * (d * d);                          // hist * (..)**2
        acc += (double)e;
      }
      part[t] = acc;
    }
    for (int w = kCalibPartials / 2; w > 0; w >>= 1)
      for (int t = 0; t < w; ++t) part[t] += part[t + w];
    errs[s] = part[0];
  }
  return TQ_OK;
}

}  // extern "C"
