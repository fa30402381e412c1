// Probe: alignment / truncation of v_mfma_f32_16x16x32_f16's accumulation on gfx950, on
// hand-picked fragments (every output of the 16x16 tile gets the same K vector).
//   A: C = 1, 32 products of (1 - 2^-11) 2^-24    exact 1 + 2^-19 - 2^-30   RN: 1 + 2^-19
//   B: C = 1, 32 products of (1 - 2^-11) 2^-25    exact ~1 + 2^-20          RN: 1 + 2^-20
//   C: C = 0, one product 1, 31 of (1 - 2^-11) 2^-24                         RN: 1 + 15.5 ulp -> 1 + 2^-19 - 2^-24?
//   D: C = 1, 32 products of -(1 - 2^-11) 2^-25   exact ~1 - 2^-20          RN: 1 - 2^-20
//   E: C = 1, 1 product (1 - 2^-11) 2^-24 (rest 0)  exact 1 + 2^-24 - 2^-35  RN: 1
//   F: C = 1, 1 product (1 + 2^-10) 2^-24           exact 1 + 2^-24 + 2^-34  RN: 1 + 2^-23
//   G: C = 2^20, 32 products of 1 * 2^-4 (1-2^-11)    exact 2^20 + 2 - 2^-10  RN: 2^20 + 2
// Build: hipcc --offload-arch=gfx950 -O2 -o mfma_align mfma_align.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const float* av, const float* bv, float c, float* d) {
  const int l = threadIdx.x;
  const int kb = 8 * (l >> 4);
  f16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)av[kb + j];
    b[j] = (_Float16)bv[kb + j];
  }
  f32x4 acc = {c, c, c, c};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  d[l] = acc[0];
}

static void run(const char* name, const float* a, const float* b, float c, double exact) {
  float *da, *db, *dd;
  hipMalloc(&da, 128);
  hipMalloc(&db, 128);
  hipMalloc(&dd, 256);
  hipMemcpy(da, a, 128, hipMemcpyHostToDevice);
  hipMemcpy(db, b, 128, hipMemcpyHostToDevice);
  probe<<<1, 64>>>(da, db, c, dd);
  float h[64];
  hipMemcpy(h, dd, 256, hipMemcpyDeviceToHost);
  const float rn = (float)exact;
  const double ulp = ldexp(1.0, ilogb(rn) - 23);
  printf("%s: got %.10g (1 + %.4f ulp vs RN %.10g), exact - got = %.4f ulp\n", name, h[0],
         ((double)h[0] - (double)rn) / ulp, rn, (exact - (double)h[0]) / ulp);
  hipFree(da);
  hipFree(db);
  hipFree(dd);
}

int main() {
  float a[32], b[32];
  const double m = 1.0 - ldexp(1.0, -11);
  auto fill = [&](int cnt, double va, double vb) {
    for (int k = 0; k < 32; ++k) {
      a[k] = k < cnt ? (float)va : 0.0f;
      b[k] = k < cnt ? (float)vb : 0.0f;
    }
  };
  fill(32, m * ldexp(1.0, -10), ldexp(1.0, -14));
  run("A C=1 +32x(1-2^-11)2^-24", a, b, 1.0f, 1.0 + 32 * m * ldexp(1.0, -24));
  fill(32, m * ldexp(1.0, -11), ldexp(1.0, -14));
  run("B C=1 +32x(1-2^-11)2^-25", a, b, 1.0f, 1.0 + 32 * m * ldexp(1.0, -25));
  fill(32, m * ldexp(1.0, -10), ldexp(1.0, -14));
  a[0] = 1.0f;
  b[0] = 1.0f;
  run("C C=0 1+31x(1-2^-11)2^-24", a, b, 0.0f, 1.0 + 31 * m * ldexp(1.0, -24));
  fill(32, -m * ldexp(1.0, -11), ldexp(1.0, -14));
  run("D C=1 -32x(1-2^-11)2^-25", a, b, 1.0f, 1.0 - 32 * m * ldexp(1.0, -25));
  fill(1, m * ldexp(1.0, -10), ldexp(1.0, -14));
  run("E C=1 +(1-2^-11)2^-24", a, b, 1.0f, 1.0 + m * ldexp(1.0, -24));
  fill(1, (1.0 + ldexp(1.0, -10)) * ldexp(1.0, -10), ldexp(1.0, -14));
  run("F C=1 +(1+2^-10)2^-24", a, b, 1.0f, 1.0 + (1.0 + ldexp(1.0, -10)) * ldexp(1.0, -24));
  fill(32, m * ldexp(1.0, -2), ldexp(1.0, -2));
  run("G C=2^20 +32x(1-2^-11)2^-4", a, b, 1048576.0f, 1048576.0 + 32 * m * ldexp(1.0, -4));
  fill(32, m * ldexp(1.0, -10), ldexp(1.0, -14));
  run("H C=-1 +32x(1-2^-11)2^-24", a, b, -1.0f, -1.0 + 32 * m * ldexp(1.0, -24));
  return 0;
}
