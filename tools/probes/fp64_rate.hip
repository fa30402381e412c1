// Probe: issue rate of fp64 VALU ops on gfx950 (cycles per wave64 instruction, 8 independent
// chains per lane, one wave per SIMD and four waves per SIMD).  Build: hipcc
// --offload-arch=gfx950 -O3 -o fp64_rate fp64_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(float* out, int iters) {
  double d[8];
  float f[8];
  for (int i = 0; i < 8; ++i) {
    d[i] = threadIdx.x * 1e-3 + i;
    f[i] = (float)d[i];
  }
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) d[i] = fma(d[i], 1.0000001, 1e-9);       // v_fma_f64
      if (OP == 1) d[i] = d[i] + (double)f[i];              // v_cvt_f64_f32 + v_add_f64
      if (OP == 2) f[i] = fmaf(f[i], 1.0000001f, 1e-9f);    // v_fma_f32
      if (OP == 3) f[i] = (float)(d[i] * 1.5);              // v_mul_f64 + v_cvt_f32_f64
    }
  }
  const long long t1 = clock64();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += d[i] + f[i];
  if (threadIdx.x == 0) out[blockIdx.x] = (float)(t1 - t0) / (iters * 8.0f);
  if (s == 12345.0) out[1] = 1;
}

int main() {
  float* o;
  hipMalloc(&o, 4096 * 4);
  const char* names[4] = {"v_fma_f64", "v_cvt_f64_f32 + v_add_f64", "v_fma_f32", "v_mul_f64 + v_cvt_f32_f64"};
  for (int op = 0; op < 4; ++op)
    for (int waves = 1; waves <= 16; waves *= 4) {
      auto fn = op == 0 ? k<0> : op == 1 ? k<1> : op == 2 ? k<2> : k<3>;
      fn<<<256, 64 * waves>>>(o, 4096);  // warm
      fn<<<256, 64 * waves>>>(o, 4096);
      hipDeviceSynchronize();
      float h;
      hipMemcpy(&h, o, 4, hipMemcpyDeviceToHost);
      printf("%-28s waves/CU %2d: %.2f clock64 ticks per wave instruction (per op group)\n",
             names[op], waves, h);
    }
  return 0;
}
