// Probe: how v_mfma_f32_16x16x32_f16 rounds its fp32 accumulation on gfx950.
// For random fp16 A/B fragments and fp32 C, compares D = C + A*B against the exactly
// rounded value (long double-free: the 32 products of fp16 values and C are summed exactly
// in a 256-bit fixed-point accumulator on the host, then rounded to nearest-even fp32).
// Prints how many outputs equal the correctly rounded sum, and the max error in units of
// 2^-24 * (|C| + sum |a b|).  Build: hipcc --offload-arch=gfx950 -O2 -o mfma_rounding.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// one 16x16x32 MFMA per wave: lane l holds A[l%16][8(l/16)..+7], B[8(l/16)..+7][l%16],
// C/D[4(l/16)+i][l%16]
__global__ void probe(const _Float16* a, const _Float16* b, const float* c, float* d, int n) {
  const int t = blockIdx.x;
  if (t >= n) return;
  const int l = threadIdx.x;
  const int r = l & 15, kb = 8 * (l >> 4);
  f16x8 av, bv;
  for (int j = 0; j < 8; ++j) {
    av[j] = a[(int64_t)t * 512 + r * 32 + kb + j];
    bv[j] = b[(int64_t)t * 512 + (kb + j) * 16 + r];
  }
  f32x4 acc;
  for (int i = 0; i < 4; ++i) acc[i] = c[(int64_t)t * 256 + (4 * (l >> 4) + i) * 16 + r];
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) d[(int64_t)t * 256 + (4 * (l >> 4) + i) * 16 + r] = acc[i];
}

// exact sum of fp32/fp16-product terms: every term is m * 2^e with |m| < 2^48 and e >=
// -200; a __int128 pair at a fixed 2^-300 scale is enough for this probe's ranges
struct Exact {
  // value = sum of (mantissa * 2^(exp + 300)) held as a big integer in 4 x 64-bit limbs
  // (two's complement); the terms used here span < 2^(16+300), so 512 bits are plenty
  uint64_t w[8] = {0};
  void add(double v) {  // v exactly representable, |v| in [2^-200, 2^20]
    if (v == 0) return;
    int e;
    double m = frexp(v, &e);              // v = m 2^e, 0.5 <= |m| < 1
    int64_t im = (int64_t)ldexp(m, 53);   // exact
    int sh = e - 53 + 300;                // v = im * 2^(sh - 300)
    bool neg = im < 0;
    uint64_t u = neg ? (uint64_t)(-im) : (uint64_t)im;
    uint64_t limb[8] = {0};
    int q = sh / 64, s = sh % 64;
    limb[q] = u << s;
    if (s && q + 1 < 8) limb[q + 1] = u >> (64 - s);
    if (neg) {  // two's complement of limb
      unsigned carry = 1;
      for (int i = 0; i < 8; ++i) {
        uint64_t x = ~limb[i] + carry;
        carry = (carry && x == 0) ? 1 : 0;
        limb[i] = x;
      }
    }
    unsigned __int128 carry = 0;
    for (int i = 0; i < 8; ++i) {
      unsigned __int128 s2 = (unsigned __int128)w[i] + limb[i] + carry;
      w[i] = (uint64_t)s2;
      carry = s2 >> 64;
    }
  }
  // round to nearest-even fp32
  float to_float() const {
    uint64_t v[8];
    memcpy(v, w, sizeof v);
    bool neg = v[7] >> 63;
    if (neg) {
      unsigned carry = 1;
      for (int i = 0; i < 8; ++i) {
        uint64_t x = ~v[i] + carry;
        carry = (carry && x == 0) ? 1 : 0;
        v[i] = x;
      }
    }
    int top = -1;
    for (int i = 7; i >= 0 && top < 0; --i)
      if (v[i]) top = i * 64 + 63 - __builtin_clzll(v[i]);
    if (top < 0) return 0.0f;
    auto bit = [&](int p) -> int { return p < 0 ? 0 : (int)((v[p / 64] >> (p % 64)) & 1); };
    // keep 24 bits: top .. top-23
    uint64_t mant = 0;
    for (int p = top; p > top - 24; --p) mant = (mant << 1) | (uint64_t)bit(p);
    int g = bit(top - 24);
    bool sticky = false;
    for (int p = top - 25; p >= 0 && !sticky; --p) sticky = bit(p);
    if (g && (sticky || (mant & 1))) ++mant;
    double r = ldexp((double)mant, top - 23 - 300);
    return (float)(neg ? -r : r);
  }
};

int main() {
  const int n = 4096;
  std::mt19937_64 rng(1234);
  std::vector<_Float16> ha((size_t)n * 512), hb((size_t)n * 512);
  std::vector<float> hc((size_t)n * 256), hd((size_t)n * 256);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  std::uniform_int_distribution<int> ex(-14, 10);
  for (int t = 0; t < n; ++t) {
    const int mode = t % 4;  // 0: same scale; 1: wide exponents; 2: one dominant term;
                             // 3: cancellation (C = -sum)
    for (int i = 0; i < 512; ++i) {
      double va = u(rng), vb = u(rng);
      if (mode == 1) { va = ldexp(va, ex(rng) / 2); vb = ldexp(vb, ex(rng) / 2); }
      ha[(size_t)t * 512 + i] = (_Float16)va;
      hb[(size_t)t * 512 + i] = (_Float16)vb;
    }
    for (int i = 0; i < 256; ++i) hc[(size_t)t * 256 + i] = (float)(mode == 2 ? 64.0 * u(rng) : u(rng));
  }
  // mode 3: C = -(fp32 rounded sum) so the result is a cancellation residue
  for (int t = 3; t < n; t += 4)
    for (int r = 0; r < 16; ++r)
      for (int col = 0; col < 16; ++col) {
        double s = 0;
        for (int k = 0; k < 32; ++k)
          s += (double)ha[(size_t)t * 512 + r * 32 + k] * (double)hb[(size_t)t * 512 + k * 16 + col];
        hc[(size_t)t * 256 + r * 16 + col] = -(float)s;
      }
  _Float16 *da, *db;
  float *dc, *dd;
  hipMalloc(&da, ha.size() * 2);
  hipMalloc(&db, hb.size() * 2);
  hipMalloc(&dc, hc.size() * 4);
  hipMalloc(&dd, hd.size() * 4);
  hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice);
  probe<<<n, 64>>>(da, db, dc, dd, n);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  hipMemcpy(hd.data(), dd, hd.size() * 4, hipMemcpyDeviceToHost);
  long eq[4] = {0}, tot[4] = {0};
  double maxe[4] = {0}, maxulp[4] = {0};
  for (int t = 0; t < n; ++t)
    for (int r = 0; r < 16; ++r)
      for (int col = 0; col < 16; ++col) {
        Exact e;
        double mag = fabs((double)hc[(size_t)t * 256 + r * 16 + col]);
        e.add(hc[(size_t)t * 256 + r * 16 + col]);
        for (int k = 0; k < 32; ++k) {
          double p = (double)ha[(size_t)t * 512 + r * 32 + k] * (double)hb[(size_t)t * 512 + k * 16 + col];
          e.add(p);
          mag += fabs(p);
        }
        const float ref = e.to_float();
        const float got = hd[(size_t)t * 256 + r * 16 + col];
        const int m = t % 4;
        ++tot[m];
        if (ref == got) ++eq[m];
        // error vs the exact sum (ref is within half an ulp of it)
        double err = fabs((double)got - (double)ref) / (ldexp(mag, -24));
        if (err > maxe[m]) maxe[m] = err;
        double ulp = ref != 0 ? fabs((double)got - (double)ref) / ldexp(1.0, ilogb(ref) - 23) : 0;
        if (ulp > maxulp[m]) maxulp[m] = ulp;
      }
  const char* names[4] = {"same-scale", "wide-exponent", "dominant-C", "cancellation"};
  for (int m = 0; m < 4; ++m)
    printf("%-14s correctly rounded %ld / %ld   max |D - RN(exact)| = %.3f x 2^-24 (|C| + sum|ab|)"
           "   max %.2f ulp\n", names[m], eq[m], tot[m], maxe[m], maxulp[m]);
  return 0;
}
