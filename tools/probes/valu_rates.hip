// Probe: sustained rate of the arithmetic an exact fp32 dot product can be built from, on
// gfx950, timed with HIP events over a full grid (4 waves per SIMD, 8 independent chains per
// lane): v_fma_f64, v_cvt_f64_f32 (+ v_add_f64), v_fma_f32, v_pk_fma_f32 and
// v_mfma_f64_16x16x4_f64.  Prints wave-instructions per cycle per CU at the measured clock.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rates valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));
typedef double double4v __attribute__((ext_vector_type(4)));

template <int OP>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  double d[8];
  float f[8];
  float2v p[8];
  double4v acc[4] = {};
  for (int i = 0; i < 8; ++i) {
    d[i] = threadIdx.x * 1e-3 + i;
    f[i] = (float)d[i];
    p[i] = float2v{f[i], f[i] + 1.0f};
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) d[i] = fma(d[i], 1.0000001, 1e-9);                        // v_fma_f64
      if (OP == 1) d[i] = d[i] + (double)f[i];                               // cvt + add_f64
      if (OP == 2) f[i] = fmaf(f[i], 1.0000001f, 1e-9f);                     // v_fma_f32
      if (OP == 3) p[i] = __builtin_elementwise_fma(p[i], float2v{1.0000001f, 0.9999999f},
                                                    float2v{1e-9f, 2e-9f});  // v_pk_fma_f32
      if (OP == 4 && i < 4)
        acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(d[i], d[i + 4], acc[i], 0, 0, 0);
    }
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += d[i] + f[i] + p[i].x + p[i].y;
  s += acc[0].x + acc[1].y + acc[2].z + acc[3].w;
  if (s == 12345.0) out[blockIdx.x] = 1;
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 20);
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 4;  // 4 blocks of 4 waves per CU = 4 waves per SIMD
  const int iters = 4096;
  const char* names[] = {"v_fma_f64", "v_cvt_f64_f32+v_add_f64", "v_fma_f32", "v_pk_fma_f32",
                         "v_mfma_f64_16x16x4_f64"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int op = 0; op < 5; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      switch (op) {
        case 0: k<0><<<blocks, 256>>>(out, iters); break;
        case 1: k<1><<<blocks, 256>>>(out, iters); break;
        case 2: k<2><<<blocks, 256>>>(out, iters); break;
        case 3: k<3><<<blocks, 256>>>(out, iters); break;
        case 4: k<4><<<blocks, 256>>>(out, iters); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double per = op == 4 ? 4.0 : 8.0;  // dependent-chain instructions per iteration
      const double insts = (double)blocks * 4 * iters * per;  // wave instructions
      const double ns_per = ms * 1e6 / (insts / cus);         // ns per wave instruction per CU
      if (rep == 1)
        printf("%-28s %.3f ms  %.3f ns per wave-instruction per CU  (%.2f cycles at 2.4 GHz; "
               "%.1f per SIMD)\n",
               names[op], ms, ns_per, ns_per * 2.4, ns_per * 2.4 * 4);
    }
  }
  return 0;
}
