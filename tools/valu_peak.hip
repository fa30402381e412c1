// VALU throughput probe for the term-pair conv's candidate instructions on gfx950.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o /tmp/valu_peak && /tmp/valu_peak
// Each lane runs 16 independent accumulation chains; the grid fills every SIMD with 8
// waves.  Reports lane-ops/s per instruction (78.6e12 = one lane-op per lane per clock at
// 2.4 GHz on 256 CUs x 4 SIMD32).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef short s2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kChains = 16;
constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void probe(int* out, int seed) {
  int acc[kChains];
  float facc[kChains];
  f2 pacc[kChains];
  const int a = seed + threadIdx.x, b = seed * 3 + 1;
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    acc[c] = c;
    facc[c] = (float)c;
    pacc[c] = f2{(float)c, 1.0f};
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == 0)
        acc[c] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, a + c), __builtin_bit_cast(s2, b),
                                        acc[c], false);
      else if (OP == 1)
        acc[c] = __builtin_amdgcn_sdot4(a + c, b, acc[c], false);
      else if (OP == 2)
        facc[c] = __builtin_fmaf(facc[c], 1.0001f, 0.5f);
      else if (OP == 3)
        pacc[c] = __builtin_elementwise_fma(pacc[c], f2{1.0001f, 0.9999f}, f2{0.5f, 0.25f});
      else if (OP == 4)
        acc[c] = __builtin_amdgcn_sdot8(a + c, b, acc[c], false);
      else
        acc[c] = acc[c] * (a + c) + b;  // v_mad_u32_u24 / v_mad_i32 path
    }
  }
  int s = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += acc[c] + (int)facc[c] + (int)pacc[c].x + (int)pacc[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
void run(const char* name, int* d, int macs_per_op) {
  const int blocks = 256 * 8;  // 8 WGs of 4 waves per CU -> 8 waves / SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<OP><<<blocks, 256>>>(d, 1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) probe<OP><<<blocks, 256>>>(d, r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double ops = 5.0 * blocks * 256.0 * kIters * kChains;
  printf("%-22s %7.2f T lane-op/s  (%5.1f%% of 78.6T)  %7.1f T MAC/s\n", name,
         ops / (ms * 1e-3) / 1e12, 100.0 * ops / (ms * 1e-3) / 78.6432e12,
         macs_per_op * ops / (ms * 1e-3) / 1e12);
}

int main() {
  int* d;
  hipMalloc(&d, 256 * 8 * 256 * sizeof(int));
  run<0>("v_dot2c_i32_i16", d, 2);
  run<1>("v_dot4c_i32_i8", d, 4);
  run<4>("v_dot8_i32_i4", d, 8);
  run<2>("v_fma_f32", d, 1);
  run<3>("v_pk_fma_f32", d, 2);
  run<5>("v_mad_i32", d, 1);
  hipFree(d);
  return 0;
}
