// Fused ResNet stem on the matrix cores: conv 7x7/2 (3 -> 64, pad 3, no bias) -> eval BN ->
// ReLU -> max-pool 3x3/2 (pad 1) -> fp32 output + the first TR layer's activation codes.
//
// The reference keeps the stem conv a plain fp32 conv (cnn_models/__init__.py:34-36 never
// converts it) followed by bn1 / relu / maxpool (torchvision ResNet.forward) and the first
// TRConv2dLayer's input TR (tr_layer.py:96-99).  Run as library calls that is an fp32 conv
// writing a 256x64x112x112 tensor (822 MB), a pass reading it back, and the pool output; here
// the conv output never leaves the chip: HBM sees the 154 MB input and the pooled outputs.
//
// fp32 arithmetic on bf16 matrix cores (split-bf16, "bf16x3").  Every fp32 value is split
// exactly-rounded into three bf16 parts, x = x0 + x1 + x2 + e with |x1| <= 2^-9 |x|,
// |x2| <= 2^-18 |x|, |e| <= 2^-27 |x| (each part is RN(bf16) of the exact remainder; the
// remainders are exact fp32 differences, Sterbenz).  Weights are split the same way on the
// host.  The products x0w0 + x0w1 + x1w0 + x0w2 + x1w1 + x2w0 (6 MFMAs) are exact in fp32 and
// are accumulated in fp32 by the MFMA; the dropped terms are below 2^-26 |x||w|, so each
// product carries ~2^-25 relative error -- the accuracy class of an fp32 conv, whose own
// summation order (cuDNN / MIOpen algorithm choice) the reference does not fix either.
//
// Layout.  Space-to-depth turns the stride-2 7x7 conv into a stride-1 4x4 conv over 12
// channels: the kernel padded to 8x8 (a zero tap in front), s2d pixel (R, C) = input rows
// 2R, 2R+1 x cols 2C, 2C+1 x 3 channels = 12 values; conv pixel (oy, ox) reads s2d rows
// oy-2..oy+1 and cols ox-2..ox+1, so K = 4 x 4 x 12 = 192 in the order (sy, sx, sub_r, sub_c,
// c), and any 8 consecutive K values are 8 consecutive fp32 in an s2d row ([col][12] rows).
//   LDS: weights [3 splits][64 rows of 200 bf16] (76.8 KB, staged once per workgroup) and
//        the input tile as fp32 s2d rows [2TP+4][SC][12] (46 KB for TP = 2, W = 224)
//   wave = one strip of 16 conv columns (7 pool columns) x 2TP+1 conv rows; per conv row
//        6 K-steps x (4 Cout blocks x 6 split products) v_mfma_f32_16x16x32_bf16
//   epilogue in registers: BN (fp32 fma, as the stem-tail kernel) + ReLU, vertical max over
//        the 3 conv rows of each pool row, horizontal max by lane shuffles (width 16),
//        fp32 store + TR codes for 7 pool pixels per strip.
// Max-pool pads with -inf; after ReLU every window holds a valid value >= 0, so the padded
// conv positions are read as 0 here with the same result.
#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kStemThreads = 512;
constexpr int kStemK = 192;     // s2d K
constexpr int kStemWRow = 200;  // LDS weight row (bf16): 400 B keeps the A reads spread
constexpr int kStemWBytes = 3 * 64 * kStemWRow * 2;

__device__ __forceinline__ void split3(const float (&x)[8], bf16x8& x0, bf16x8& x1,
                                       bf16x8& x2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h0 = (__bf16)x[j];
    const float r1 = x[j] - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    const float r2 = r1 - (float)h1;
    x0[j] = h0;
    x1[j] = h1;
    x2[j] = (__bf16)r2;
  }
}

template <int TP>
__global__ __launch_bounds__(kStemThreads, 1) void stem_conv_pool_kernel(PoolArgs a, int sc,
                                                                         int nb, int tiles) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds_raw[];
  uint16_t* ws = reinterpret_cast<uint16_t*>(lds_raw);
  float* xs = reinterpret_cast<float*>(reinterpret_cast<char*>(lds_raw) + kStemWBytes);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int i16 = lane & 15;
  const int g = lane >> 4;
  const int Hc = a.H / 2, Wc = a.W / 2;  // conv output
  const int tpi = (a.Ho + TP - 1) / TP;  // tiles per image

  // weights once per workgroup: [3][64][192] bf16 -> rows of kStemWRow
  for (int i = tid; i < 3 * 64 * (kStemK / 8); i += kStemThreads) {
    const int row = i / (kStemK / 8);
    const int ch = i - row * (kStemK / 8);
    *reinterpret_cast<u32x4*>(ws + row * kStemWRow + ch * 8) =
        *reinterpret_cast<const u32x4*>(a.wsplit + row * kStemK + ch * 8);
  }
  // per-lane BN coefficients of channels mb*16 + 4g + i
  float bsc[4][4], bsh[4][4];
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bsc[mb][i] = a.scale[mb * 16 + 4 * g + i];
      bsh[mb][i] = a.shift[mb * 16 + 4 * g + i];
    }

  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int n = tile / tpi;
    const int py0 = (tile - n * tpi) * TP;
    const int srow0 = 2 * py0 - 3;
    __syncthreads();  // the previous tile's s2d rows are no longer read
    // input rows -> s2d: item = (local s2d row, sub row, local s2d col), 6 floats each
    const int items = (2 * TP + 4) * 2 * sc;
    for (int it = tid; it < items; it += kStemThreads) {
      const int lr = it / (2 * sc);
      const int rem = it - lr * 2 * sc;
      const int sr = rem / sc;
      const int lc = rem - sr * sc;
      const int ir = 2 * (srow0 + lr) + sr;
      const int ic = 2 * (lc - 3);
      float2 v0 = make_float2(0.f, 0.f), v1 = v0, v2 = v0;
      if (ir >= 0 && ir < a.H && ic >= 0 && ic < a.W) {
        const float* src = a.x + (((int64_t)n * a.H + ir) * a.W + ic) * 3;
        v0 = *reinterpret_cast<const float2*>(src);
        v1 = *reinterpret_cast<const float2*>(src + 2);
        v2 = *reinterpret_cast<const float2*>(src + 4);
      }
      float* dst = xs + (lr * sc + lc) * 12 + sr * 6;
      *reinterpret_cast<float2*>(dst) = v0;
      *reinterpret_cast<float2*>(dst + 2) = v1;
      *reinterpret_cast<float2*>(dst + 4) = v2;
    }
    __syncthreads();

    for (int b = wave; b < nb; b += kStemThreads / 64) {
      const int c0 = 14 * b - 1;  // first conv column of the strip
      const int ox = c0 + i16;
      const bool colok = ox >= 0 && ox < Wc;

      // BN + ReLU of conv row (2*py0 - 1 + rr) at column ox, channels mb*16 + 4g + i.
      // The input slice of step ks+1 is read during step ks's MFMAs.
      auto load_x = [&](int rr, int ks, float (&xv)[8]) {
        const int j = 4 * ks + g;  // 8-value K slice of this lane
        const int sy = j / 6;
        const int off = (j - sy * 6) * 8;
        const float* src = xs + ((rr + sy) * sc + (ox + 1)) * 12 + off;
        const float4 xa = *reinterpret_cast<const float4*>(src);
        const float4 xb = *reinterpret_cast<const float4*>(src + 4);
        xv[0] = xa.x; xv[1] = xa.y; xv[2] = xa.z; xv[3] = xa.w;
        xv[4] = xb.x; xv[5] = xb.y; xv[6] = xb.z; xv[7] = xb.w;
      };
      auto mma_step = [&](int ks, const float (&xv)[8], f32x4 (&acc)[4]) {
        bf16x8 x0, x1, x2;
        split3(xv, x0, x1, x2);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const uint16_t* wr = ws + (mb * 16 + i16) * kStemWRow + 32 * ks + 8 * g;
          const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(wr);
          const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(wr + 64 * kStemWRow);
          const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(wr + 128 * kStemWRow);
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, x0, acc[mb], 0, 0, 0);
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, x1, acc[mb], 0, 0, 0);
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x0, acc[mb], 0, 0, 0);
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, x2, acc[mb], 0, 0, 0);
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x1, acc[mb], 0, 0, 0);
          acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, x0, acc[mb], 0, 0, 0);
        }
      };
      auto conv_row = [&](int rr, f32x4 (&y)[4]) {
        f32x4 acc[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) acc[mb] = (f32x4)0.0f;
        float xa[8], xb[8];
        load_x(rr, 0, xa);
#pragma unroll 1
        for (int ks = 0; ks < kStemK / 32; ks += 2) {
          load_x(rr, ks + 1, xb);
          mma_step(ks, xa, acc);
          if (ks + 2 < kStemK / 32) load_x(rr, ks + 2, xa);
          mma_step(ks + 1, xb, acc);
        }
        const int oy = 2 * py0 - 1 + rr;
        const bool ok = colok && oy >= 0 && oy < Hc;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = fmaf(acc[mb][i], bsc[mb][i], bsh[mb][i]);
            y[mb][i] = ok ? fmaxf(v, 0.0f) : 0.0f;
          }
      };

      // pool row j = max over conv rows rr = 2j, 2j+1, 2j+2 (rows 2j+2 are shared)
      f32x4 run[4];
#pragma unroll 1
      for (int rr = 0; rr <= 2 * TP; ++rr) {
        f32x4 y[4];
        conv_row(rr, y);
        if (rr == 0 || (rr & 1)) {
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) run[mb] = rr == 0 ? y[mb] : __builtin_elementwise_max(run[mb], y[mb]);
          continue;
        }
        const int py = py0 + rr / 2 - 1;
        float m[4][4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = fmaxf(run[mb][i], y[mb][i]);
            const float v1 = __shfl_down(v, 1, 16);
            const float v2 = __shfl_down(v, 2, 16);
            m[mb][i] = fmaxf(fmaxf(v, v1), v2);
          }
          run[mb] = y[mb];
        }
        const int px = 7 * b + (i16 >> 1);
        if (py >= a.Ho || (i16 & 1) || i16 > 12 || px >= a.Wo) continue;
        const int64_t p = ((int64_t)n * a.Ho + py) * a.Wo + px;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          const int co = mb * 16 + 4 * g;
          const float yv[4] = {m[mb][0], m[mb][1], m[mb][2], m[mb][3]};
          *reinterpret_cast<float4*>(a.out + p * 64 + co) =
              make_float4(yv[0], yv[1], yv[2], yv[3]);
#pragma unroll
          for (int side = 0; side < 2; ++side) {
            int16_t* codes = side ? a.codes_b : a.codes_a;
            if (!codes) continue;
            const double inv = side ? a.inv_b : a.inv_a;
            const float maxv = side ? a.maxv_b : a.maxv_a;
            const int k = side ? a.k_b : a.k_a;
            const int cp = side ? a.cp_b : a.cp_a;
            const int fmt = side ? a.fmt_b : a.fmt_a;
            uint32_t v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
              v[i] = code_bits(tr_value_g1_inv(yv[i], inv, maxv, k), fmt);
            *reinterpret_cast<int2*>(codes + p * cp + co) =
                make_int2((int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)));
          }
        }
      }
    }
  }
}

template <int TP>
hipError_t launch_stem_tp(const PoolArgs& a, hipStream_t stream) {
  const int nb = (a.Wo + 6) / 7;
  const int sc = (14 * nb + 5 + 3) / 4 * 4;  // s2d columns -3 .. 14 nb + 1, padded
  const int64_t bytes = kStemWBytes + (int64_t)(2 * TP + 4) * sc * 12 * 4;
  if (bytes > 160 * 1024) return hipErrorInvalidConfiguration;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_conv_pool_kernel<TP>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int tiles = a.N * ((a.Ho + TP - 1) / TP);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const int grid = tiles < cus ? tiles : cus;
  if (grid <= 0) return hipSuccess;
  stem_conv_pool_kernel<TP><<<dim3(grid), kStemThreads, (size_t)bytes, stream>>>(a, sc, nb,
                                                                                 tiles);
  return hipGetLastError();
}

}  // namespace

// Shape contract (checked by the C-ABI layer): 3 input channels, H % 4 == 0, W % 4 == 0,
// conv 7x7/2 pad 3 -> 64 channels, pool 3x3/2 pad 1 -> Ho = H/4, Wo = W/4, Wo <= 112.
hipError_t launch_stem_conv_pool(const PoolArgs& a, hipStream_t stream) {
  static const char* tp = getenv("TQ_STEM_TP");  // A/B override (tools only)
  if (tp && atoi(tp) == 4) return launch_stem_tp<4>(a, stream);
  return launch_stem_tp<2>(a, stream);
}

}  // namespace tq
