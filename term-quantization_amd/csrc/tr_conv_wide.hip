// Term-pair Conv2d (groups = 1) for weight codes wider than 16 bits: the (16, 1, 16) settings
// that cnn_models.static_conv_layer_settings gives every squeeze-excite conv of
// EfficientNet-b0 (reference cnn_models/__init__.py:57-58).  A 16-bit weight's term sum
// reaches 2^16, outside both int16 (VALU dot2 engine) and exact fp16 (MFMA engine), so the
// weight codes stay int32 and every product is one 32 x 32 -> 64-bit multiply-add into an
// int64 sum (|v_x| <= 2^14 and |v_w| <= 2^16 keep each product below 2^31; the int64 sum is
// exact for any K this library accepts).  One rounding at the end, as the other engines:
//   out = fp32(double(acc) * scale + bias[c]).
//
// These layers are small GEMMs (a squeeze-excite conv sees a 1 x 1 feature map: N x Cin x
// Cout with N the batch), so a plain LDS-tiled VALU kernel suffices:
//   workgroup = 256 lanes, tile 64 output pixels x 64 output channels, 4 x 4 outputs per lane
//   K loop    = filter taps x 32-channel chunks; int16 activation codes (NHWC, tq_act_encode)
//               and int32 weight codes ([Cout][Kp], k = tap * Cp + c) staged k-major in LDS
#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

constexpr int kWideThreads = 256;
constexpr int kWideBP = 64;  // output pixels per tile
constexpr int kWideBM = 64;  // output channels per tile
constexpr int kWideKC = 32;  // channels per K chunk
constexpr int kWidePad = 68; // LDS row stride (int32): 64 + 4 keeps 16-byte alignment

__global__ __launch_bounds__(kWideThreads) void conv2d_tp_wide_kernel(WideConvArgs a) {
  __shared__ __attribute__((aligned(16))) int32_t xs[kWideKC][kWidePad];
  __shared__ __attribute__((aligned(16))) int32_t ws[kWideKC][kWidePad];
  const int t = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kWideBP;
  const int m0 = blockIdx.y * kWideBM;
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;

  // staging roles: activation row (pixel) lp, weight row (channel) lm, 8-code slice q8
  const int lp = t >> 2, lm = t >> 2, q8 = (t & 3) * 8;
  const int64_t sp = p0 + lp;
  int64_t simg = 0;
  int ih0 = 0, iw0 = 0;
  const bool pok = sp < a.P;
  if (pok) {
    simg = sp / HoWo;
    const int rem = (int)(sp - simg * HoWo);
    const int oh = rem / a.Wo;
    const int ow = rem - oh * a.Wo;
    ih0 = oh * a.sh - a.ph;
    iw0 = ow * a.sw - a.pw;
  }
  const bool mok = m0 + lm < a.Cout;

  // compute roles: pixels 4tx..4tx+3, channels 4ty..4ty+3 of the tile
  const int tx = t & 15, ty = t >> 4;
  int64_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0;

  for (int kr = 0; kr < a.KH; ++kr) {
    const int ih = ih0 + kr * a.dh;
    for (int ks = 0; ks < a.KW; ++ks) {
      const int iw = iw0 + ks * a.dw;
      const bool inside = pok && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      const int tap = kr * a.KW + ks;
      for (int c0 = 0; c0 < a.Cp; c0 += kWideKC) {
        const bool cok = c0 + q8 < a.Cp;  // Cp % 8 == 0: a slice is all in or all out
        int4 xv = make_int4(0, 0, 0, 0);
        if (inside && cok)
          xv = *reinterpret_cast<const int4*>(a.x + ((simg * a.H + ih) * a.W + iw) * a.Cp +
                                              c0 + q8);
        int4 w0 = make_int4(0, 0, 0, 0), w1 = make_int4(0, 0, 0, 0);
        if (mok && cok) {
          const int32_t* wr = a.w + (int64_t)(m0 + lm) * a.Kp + (int64_t)tap * a.Cp + c0 + q8;
          w0 = *reinterpret_cast<const int4*>(wr);
          w1 = *reinterpret_cast<const int4*>(wr + 4);
        }
        __syncthreads();  // the previous chunk's reads are done
        const int xw[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          xs[q8 + 2 * i][lp] = (int)(short)(xw[i] & 0xFFFF);
          xs[q8 + 2 * i + 1][lp] = xw[i] >> 16;
        }
        const int wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) ws[q8 + i][lm] = wv[i];
        __syncthreads();
#pragma unroll 8
        for (int kk = 0; kk < kWideKC; ++kk) {
          const int4 xa = *reinterpret_cast<const int4*>(&xs[kk][4 * tx]);
          const int4 wb = *reinterpret_cast<const int4*>(&ws[kk][4 * ty]);
          const int xr[4] = {xa.x, xa.y, xa.z, xa.w};
          const int wr[4] = {wb.x, wb.y, wb.z, wb.w};
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] += (int64_t)xr[i] * (int64_t)wr[j];
        }
      }
    }
  }

  double sc = a.scale;
  double sh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = m0 + 4 * ty + j;
    sh[j] = (a.bias && co < a.Cout) ? (double)a.bias[co] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t p = p0 + 4 * tx + i;
    if (p >= a.P) continue;
    float y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = (float)((double)acc[i][j] * sc + sh[j]);
    const int co = m0 + 4 * ty;
    if (a.out_nhwc) {
      float* dst = a.out + p * a.Cout + co;
      if ((a.Cout & 3) == 0 && co + 3 < a.Cout) {
        *reinterpret_cast<float4*>(dst) = make_float4(y[0], y[1], y[2], y[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (co + j < a.Cout) dst[j] = y[j];
      }
    } else {
      const int64_t img = p / HoWo;
      const int64_t rem = p - img * HoWo;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (co + j < a.Cout) a.out[(img * a.Cout + co + j) * HoWo + rem] = y[j];
    }
  }
}

}  // namespace

hipError_t launch_conv2d_wide(const WideConvArgs& a, hipStream_t stream) {
  if (a.P == 0 || a.Cout == 0) return hipSuccess;
  const dim3 grid((unsigned)((a.P + kWideBP - 1) / kWideBP),
                  (unsigned)((a.Cout + kWideBM - 1) / kWideBM));
  conv2d_tp_wide_kernel<<<grid, kWideThreads, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace tq
