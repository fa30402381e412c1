// Term-pair Conv2d on the matrix cores, direct engine: activation fragments go straight from
// HBM/L2 into VGPRs (no LDS round trip, no barrier for them), weight K-steps stream through
// a small double-buffered LDS ring shared by the workgroup's 4 waves.
//
// Same arithmetic and exactness argument as tr_conv_mfma.hip: fp16 term-sum codes, exact
// products on v_mfma_f32_32x32x16_f16, fp32 partial sums exact below 2^24, moved into int32
// sums every kc_steps K-steps (windows of consecutive K-steps in packed K order, which is
// the order this kernel walks: k = tap * Cp + c).
//
// Why this shape.  The ResNet-18 TQ convs are short-K (576-4608) and their fused epilogue
// (BN fold, residual, ReLU, fp32 output, next layers' TR codes) moves more bytes than the
// main loop: a kernel that runs one workgroup per CU serialises patch load -> MFMA ->
// epilogue.  Here a workgroup needs only 16 KB of LDS and <= 256 VGPRs per lane, so two
// (or more) workgroups share a CU and one's epilogue overlaps the other's main loop.
//
//   workgroup = 4 waves, tile 64 (Cout) x 4*32*WN (output pixels)
//   wave      = 64 x 32*WN: 2 x WN MFMA blocks of 32 x 32, 8*WN MFMAs per K-step
//   K-step    = 64 codes of one filter tap (Cp % 64 == 0)
//   A (weights [Cout_pad][Kp] fp16): global_load_lds_dwordx4 into a 2-slot ring, 8 KB/slot,
//             rows swizzled chunk ^= (row >> 1) & 7 on the source side (conflict-free reads)
//   B (activation codes [N][H][W][Cp] fp16): lane (r32, hh) loads, per block column and
//             16-code substep s, the 16 bytes [16s + 8hh, +8) of its pixel at the step's tap;
//             taps in the zero padding read a zero page; next step's loads are in flight
//             during the current step's MFMAs (register double buffer)
//   epilogue: straight from the MFMA layout (lane = pixel, 4 consecutive channels per
//             register quad): every residual load of the wave tile issued first, per-channel
//             (scale, shift) from LDS, 16-byte fp32 stores, 8-byte code stores.
#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

namespace tq {

namespace {

constexpr int kDirThreads = 256;
constexpr int kDirBM = 64;

template <int WN, bool FLUSH>
__global__ __launch_bounds__(kDirThreads, 2) void conv2d_tp_direct_kernel(ConvArgs a) {
  constexpr int BN = 4 * 32 * WN;
  constexpr int SLOT = kDirBM * 8;  // u32x4 per A slot (64 rows x 128 B)
  __shared__ __attribute__((aligned(16))) u32x4 ring[2 * SLOT];
  __shared__ double coef[kDirBM][2];  // epilogue (scale, shift) of the tile's channels

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = (a.Cout + kDirBM - 1) / kDirBM;
  const int m0 = (tile % mt) * kDirBM;
  const int64_t n0 = (int64_t)(tile / mt) * BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page);

  // A staging: wave w moves rows [16w, 16w + 16) of each slot, 2 wave-instructions of 8 rows
  const uint16_t* arow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave * 2 + i) * 8 + (lane >> 3);
    arow[i] = wg + (int64_t)(m0 + r) * a.Kp + ((lane & 7) ^ ((r >> 1) & 7)) * 8;
  }

  // B pixels of this lane: element offset of the pixel's input origin + the lane's K half,
  // and the mask of filter taps inside the input (KH * KW <= 64)
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  int64_t boff[WN];
  uint64_t tmask[WN];
#pragma unroll
  for (int bn = 0; bn < WN; ++bn) {
    const int64_t p = n0 + wave * 32 * WN + 32 * bn + r32;
    boff[bn] = 0;
    tmask[bn] = 0;
    if (p < a.P) {
      const int64_t img = p / HoWo;
      const int64_t rem = p - img * HoWo;
      const int oh = (int)(rem / a.Wo);
      const int ow = (int)(rem - (int64_t)oh * a.Wo);
      const int ih0 = oh * a.sh - a.ph;
      const int iw0 = ow * a.sw - a.pw;
      boff[bn] = ((img * a.H + ih0) * a.W + iw0) * a.Cp + 8 * hh;
      for (int kr = 0; kr < a.KH; ++kr) {
        const int ih = ih0 + kr * a.dh;
        if (ih < 0 || ih >= a.H) continue;
        for (int ks = 0; ks < a.KW; ++ks) {
          const int iw = iw0 + ks * a.dw;
          if (iw >= 0 && iw < a.W) tmask[bn] |= 1ull << (kr * a.KW + ks);
        }
      }
    }
  }

  if (threadIdx.x < kDirBM) {  // visible to every wave after the main loop's barriers
    const int co = m0 + threadIdx.x;
    const bool ok = co < a.Cout;
    coef[threadIdx.x][0] = a.ch_scale ? (ok ? a.ch_scale[co] : 0.0) : a.scale;
    coef[threadIdx.x][1] = a.ch_scale ? (ok ? a.ch_shift[co] : 0.0)
                                      : ((a.bias && ok) ? (double)a.bias[co] : 0.0);
  }

  const int nch = a.Cp / kKStep;
  const int nsteps = a.Kp / kKStep;  // taps * nch, plus zero K padding steps (tap >= KH*KW)

  auto issue_a = [&](int st, int slot) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(arow[i] + (int64_t)st * kKStep, ring + slot * SLOT + (wave * 2 + i) * 64);
  };
  // B fragments of K-step st: b[bn][s] = codes [16s + 8hh, +8) of block column bn's pixel
  auto load_b = [&](int st, u32x4 (&b)[WN][4]) {
    const int tap = st / nch;
    const int cb = (st - tap * nch) * kKStep;
    const int kr = tap / a.KW;
    const int ks = tap - kr * a.KW;
    const int64_t toff = ((int64_t)kr * a.dh * a.W + (int64_t)ks * a.dw) * a.Cp + cb;
#pragma unroll
    for (int bn = 0; bn < WN; ++bn) {
      const bool ok = (tmask[bn] >> tap) & 1ull;  // tap >= KH*KW: bit clear
      const uint16_t* src = ok ? xg + (boff[bn] + toff) : zero + 8 * hh;
#pragma unroll
      for (int s = 0; s < 4; ++s) b[bn][s] = *reinterpret_cast<const u32x4*>(src + 16 * s);
    }
  };

  MfmaAcc<WN> acc;  // blocks [bn][bm]: MfmaAcc<MB> holds MB x 2, used as [WN][2]
  acc_zero(acc);
  const int kc_steps = a.kc_steps;
  int since_flush = 0;

  u32x4 b0[WN][4], b1[WN][4];
  auto step = [&](int s, u32x4 (&bc)[WN][4], u32x4 (&bnx)[WN][4]) {
    TQ_WAIT_VM(0);  // this wave's A-DMA and B loads of step s have landed
    __builtin_amdgcn_s_barrier();  // every wave's A-DMA of step s landed; slot s^1 is free
    if (s + 1 < nsteps) {
      issue_a(s + 1, (s + 1) & 1);
      load_b(s + 1, bnx);
    }
    const u32x4* img = ring + (s & 1) * SLOT;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 2 * k + hh;
      half8 af[2];
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
        af[bm] = __builtin_bit_cast(half8, img[swz(32 * bm + r32, c)]);
#pragma unroll
      for (int bn = 0; bn < WN; ++bn) {
        const half8 bf = __builtin_bit_cast(half8, bc[bn][k]);
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
          acc.f[bn][bm] =
              __builtin_amdgcn_mfma_f32_32x32x16_f16(af[bm], bf, acc.f[bn][bm], 0, 0, 0);
      }
    }
    if (FLUSH && ++since_flush == kc_steps) {
      acc_flush(acc);
      since_flush = 0;
    }
  };

  issue_a(0, 0);
  load_b(0, b0);
  int s = 0;
  for (; s + 1 < nsteps; s += 2) {
    step(s, b0, b1);
    step(s + 1, b1, b0);
  }
  if (s < nsteps) step(s, b0, b1);
  acc_flush(acc);

  // Epilogue: block (bn, bm), register quad q of lane (r32, hh) = pixel 32*bn + r32 of the
  // wave, channels 32*bm + 8q + 4hh .. +3.  Residual loads for the whole wave tile are issued
  // first (one latency), per-channel coefficients come from LDS.
  __syncthreads();  // coef[] is visible (also when the K loop was empty)
  const bool vec = (a.Cout & 3) == 0;
  if (!vec) {
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = m0 + 32 * bm + 8 * q + 4 * hh;
        if (co >= a.Cout) continue;
        double sc[4], sh[4];
        load_coef(a, co, sc, sh);
#pragma unroll
        for (int bn = 0; bn < WN; ++bn) {
          const int64_t p = n0 + wave * 32 * WN + 32 * bn + r32;
          if (p >= a.P) continue;
          const int acc4[4] = {acc.i[bn][bm][4 * q], acc.i[bn][bm][4 * q + 1],
                               acc.i[bn][bm][4 * q + 2], acc.i[bn][bm][4 * q + 3]};
          emit4_nhwc(a, p, co, acc4, sc, sh, false);
        }
      }
    return;
  }
  float4 res[2][4][WN];
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int bn = 0; bn < WN; ++bn) {
        const int co = m0 + 32 * bm + 8 * q + 4 * hh;
        const int64_t p = n0 + wave * 32 * WN + 32 * bn + r32;
        res[bm][q][bn] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.residual && co < a.Cout && p < a.P)
          res[bm][q][bn] = *reinterpret_cast<const float4*>(a.residual + p * a.Cout + co);
      }
#pragma unroll
  for (int bm = 0; bm < 2; ++bm) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int cl = 32 * bm + 8 * q + 4 * hh;  // channel within the tile
      const int co = m0 + cl;
      if (co >= a.Cout) continue;
      double sc[4], sh[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sc[i] = coef[cl + i][0];
        sh[i] = coef[cl + i][1];
      }
#pragma unroll
      for (int bn = 0; bn < WN; ++bn) {
        const int64_t p = n0 + wave * 32 * WN + 32 * bn + r32;
        if (p >= a.P) continue;
        const int acc4[4] = {acc.i[bn][bm][4 * q], acc.i[bn][bm][4 * q + 1],
                             acc.i[bn][bm][4 * q + 2], acc.i[bn][bm][4 * q + 3]};
        emit4_nhwc_res(a, p, co, acc4, sc, sh, res[bm][q][bn]);
      }
    }
  }
}

template <int WN, bool FLUSH>
hipError_t launch_direct_cfg(const ConvArgs& a, hipStream_t stream) {
  constexpr int BN = 4 * 32 * WN;
  const int64_t tiles = ((a.P + BN - 1) / BN) * ((a.Cout + kDirBM - 1) / kDirBM);
  conv2d_tp_direct_kernel<WN, FLUSH><<<dim3((unsigned)tiles), kDirThreads, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace

bool conv_direct_eligible(const ConvArgs& a, int out_nhwc) {
  return out_nhwc && a.Cp % kKStep == 0 && a.KH * a.KW <= 64 && a.Kp % kKStep == 0;
}

// wn: 1 = 128-pixel tiles, 2 = 256-pixel tiles.
hipError_t launch_conv2d_direct(const ConvArgs& a, int wn, hipStream_t stream) {
  const bool flush = a.kc_steps > 0 && a.kc_steps < a.Kp / kKStep;
  if (wn == 1)
    return flush ? launch_direct_cfg<1, true>(a, stream) : launch_direct_cfg<1, false>(a, stream);
  return flush ? launch_direct_cfg<2, true>(a, stream) : launch_direct_cfg<2, false>(a, stream);
}

}  // namespace tq
