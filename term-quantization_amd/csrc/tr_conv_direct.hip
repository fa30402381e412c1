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
// epilogue.  Here a 128-pixel workgroup needs 33 KB of LDS and ~150 VGPRs per lane, so three
// workgroups share a CU and one's epilogue overlaps the others' main loops.
//
//   workgroup = 4 waves, tile 64 (Cout) x 4*32*WN (output pixels)
//   wave      = 64 x 32*WN: 2 x WN MFMA blocks of 32 x 32, 8*WN MFMAs per K-step
//   K-step    = 64 codes of one filter tap (Cp % 64 == 0)
//   A (weights [Cout_pad][Kp] fp16): global_load_lds_dwordx4 into a 3-slot ring, 8 KB/slot,
//             rows swizzled chunk ^= (row >> 1) & 7 on the source side (conflict-free reads)
//   B (activation codes [N][H][W][Cp] fp16): lane (r32, hh) loads, per block column and
//             16-code substep s, the 16 bytes [16s + 8hh, +8) of its pixel at the step's tap;
//             taps in the zero padding read a zero page; the next two steps' loads are in
//             flight during the current step's MFMAs (register triple buffer, counted vmcnt)
//   epilogue: every residual load of the wave tile issued first, then the int32 tile is
//             transposed through LDS so 16 lanes cover one pixel's 64 channels: each store
//             instruction writes 4 whole pixel rows (fp32 out: 1 KB, codes: 512 B).
#include <utility>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

namespace tq {

namespace {

// f(integral_constant<int, J>) for J = 0 .. N-1, unrolled (constant register-array indices)
template <typename F, int... J>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>()), ...);
}

constexpr int kDirThreads = 256;
constexpr int kDirBM = 64;
// D = K-steps in flight (loads issued ahead of the step being multiplied)
template <int WN, int D>
struct DirCfg {
  static constexpr int BN = 4 * 32 * WN;
  static constexpr int NB = D + 1;                 // B register buffers = A ring slots
  static constexpr int SLOT = kDirBM * 8;          // u32x4 per A slot (64 rows x 128 B)
  static constexpr int TILE = 64 * 32 * WN / 4;    // u32x4 per wave epilogue tile (int32)
  static constexpr int LDS = NB * SLOT > 4 * TILE ? NB * SLOT : 4 * TILE;
  static constexpr int LPS = 2 + 4 * WN;           // vmem instructions per wave and K-step
};

template <int WN, bool FLUSH, int D>
__global__ __launch_bounds__(kDirThreads, WN == 1 ? 2 : 1) void conv2d_tp_direct_kernel(
    ConvArgs a) {
  using C = DirCfg<WN, D>;
  __shared__ __attribute__((aligned(16))) u32x4 lds[C::LDS];
  __shared__ double coef[kDirBM][2];  // epilogue (scale, shift) of the tile's channels

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = (a.Cout + kDirBM - 1) / kDirBM;
  const int m0 = (tile % mt) * kDirBM;
  const int64_t n0 = (int64_t)(tile / mt) * C::BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const int64_t wn0 = n0 + wave * 32 * WN;  // first pixel of this wave
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page) + 8 * hh;

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
    const int64_t p = wn0 + 32 * bn + r32;
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

  const int nsteps = a.Kp / kKStep;  // = KH * KW * Cp / 64 (Cp % 64 == 0)
  // position of the next K-step to issue, advanced incrementally (no divisions in the loop)
  int i_st = 0, i_tap = 0, i_cb = 0, i_ks = 0;
  int64_t i_toff = 0;  // ((kr * dh) * W + ks * dw) * Cp + cb
  const int64_t row_step = (int64_t)a.dh * a.W * a.Cp;
  const int64_t col_step = (int64_t)a.dw * a.Cp;
  int64_t row_off = 0;

  // Issue K-step i_st: A-DMA into `slot`, B fragments into b (lane: codes [16s + 8hh, +8)).
  auto issue = [&](int slot, u32x4 (&b)[WN][4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(arow[i] + (int64_t)i_st * kKStep, lds + slot * C::SLOT + (wave * 2 + i) * 64);
#pragma unroll
    for (int bn = 0; bn < WN; ++bn) {
      const bool ok = (tmask[bn] >> i_tap) & 1ull;
      const uint16_t* src = ok ? xg + (boff[bn] + i_toff) : zero;
#pragma unroll
      for (int s = 0; s < 4; ++s) b[bn][s] = *reinterpret_cast<const u32x4*>(src + 16 * s);
    }
    ++i_st;
    i_cb += kKStep;
    i_toff += kKStep;
    if (i_cb == a.Cp) {
      i_cb = 0;
      ++i_tap;
      if (++i_ks == a.KW) {
        i_ks = 0;
        row_off += row_step;
        i_toff = row_off;
      } else {
        i_toff = row_off + (int64_t)i_ks * col_step;
      }
    }
  };

  MfmaAcc<WN> acc;  // blocks [bn][bm]: MfmaAcc<MB> holds MB x 2, used as [WN][2]
  acc_zero(acc);
  const int kc_steps = a.kc_steps;
  int since_flush = 0;

  auto compute = [&](int slot, const u32x4 (&bc)[WN][4]) {
    const u32x4* img = lds + slot * C::SLOT;
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

  // D K-steps in flight: step t is retired by vmcnt(LPS * younger) (the loads of the
  // min(D - 1, nsteps - 1 - t) later steps stay in flight), a barrier makes every wave's
  // A-DMA of step t visible and frees the slot of step t - 1 for step t + D.
  u32x4 bufs[C::NB][WN][4];
  auto step = [&](int t, auto j_tag) {
    constexpr int j = decltype(j_tag)::value;  // t % NB
    const int younger = min(D - 1, nsteps - 1 - t);
    if (younger == D - 1)
      TQ_WAIT_VM(C::LPS * (D - 1));
    else
      wait_vm_dyn(C::LPS * younger);
    __builtin_amdgcn_s_barrier();
    if (t + D < nsteps) issue((j + D) % C::NB, bufs[(j + D) % C::NB]);
    compute(j, bufs[j]);
  };
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nsteps) issue(j, bufs[j]);
  int s = 0;
  for (; s + C::NB <= nsteps; s += C::NB)
    unroll_seq([&](auto jt) { step(s + decltype(jt)::value, jt); },
               std::make_integer_sequence<int, C::NB>());
  unroll_seq(
      [&](auto jt) {
        if (s + decltype(jt)::value < nsteps) step(s + decltype(jt)::value, jt);
      },
      std::make_integer_sequence<int, C::NB>());
  acc_flush(acc);

  // Epilogue.  Lane (slot = lane & 15) finishes channels m0 + 4*slot .. +3 of pixels
  // it*4 + (lane >> 4) of its wave: each store instruction writes 4 whole pixel rows.
  const bool vec = (a.Cout & 3) == 0;
  const int slot = lane & 15;
  const int co = m0 + 4 * slot;
  float4 res[8 * WN];  // residuals first: their latency overlaps the transpose
#pragma unroll
  for (int it = 0; it < 8 * WN; ++it) {
    const int64_t p = wn0 + it * 4 + (lane >> 4);
    res[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec && a.residual && co < a.Cout && p < a.P)
      res[it] = *reinterpret_cast<const float4*>(a.residual + p * a.Cout + co);
  }
  __syncthreads();  // every wave is done with the A ring; coef[] is visible
  u32x4* t = lds + wave * C::TILE;  // [pixel][16 slots of 4 channels], slot ^= pixel & 15
#pragma unroll
  for (int bn = 0; bn < WN; ++bn)
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int px = 32 * bn + r32;
        const int sl = 8 * bm + 2 * q + hh;  // channels 32bm + 8q + 4hh .. +3
        u32x4 v;
        v.x = (uint32_t)acc.i[bn][bm][4 * q];
        v.y = (uint32_t)acc.i[bn][bm][4 * q + 1];
        v.z = (uint32_t)acc.i[bn][bm][4 * q + 2];
        v.w = (uint32_t)acc.i[bn][bm][4 * q + 3];
        t[px * 16 + (sl ^ (px & 15))] = v;
      }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile is in LDS
  __builtin_amdgcn_wave_barrier();
  if (co >= a.Cout) return;
  double sc[4], sh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sc[i] = coef[4 * slot + i][0];
    sh[i] = coef[4 * slot + i][1];
  }
#pragma unroll
  for (int it = 0; it < 8 * WN; ++it) {
    const int px = it * 4 + (lane >> 4);
    const int64_t p = wn0 + px;
    if (p >= a.P) continue;
    const u32x4 v = t[px * 16 + (slot ^ (px & 15))];
    const int acc4[4] = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
    if (vec)
      emit4_nhwc_res(a, p, co, acc4, sc, sh, res[it]);
    else
      emit4_nhwc(a, p, co, acc4, sc, sh, false);
  }
}

template <int WN, bool FLUSH, int D>
hipError_t launch_direct_cfg(const ConvArgs& a, hipStream_t stream) {
  constexpr int BN = DirCfg<WN, D>::BN;
  const int64_t tiles = ((a.P + BN - 1) / BN) * ((a.Cout + kDirBM - 1) / kDirBM);
  conv2d_tp_direct_kernel<WN, FLUSH, D><<<dim3((unsigned)tiles), kDirThreads, 0, stream>>>(a);
  return hipGetLastError();
}

template <int WN, bool FLUSH>
hipError_t launch_direct_d(const ConvArgs& a, hipStream_t stream) {
  if (a.ab & 8) return launch_direct_cfg<WN, FLUSH, 3>(a, stream);   // A/B (tools only)
  if (a.ab & 16) return launch_direct_cfg<WN, FLUSH, 4>(a, stream);
  return launch_direct_cfg<WN, FLUSH, 2>(a, stream);
}

}  // namespace

bool conv_direct_eligible(const ConvArgs& a, int out_nhwc) {
  return out_nhwc && a.Cp % kKStep == 0 && a.KH * a.KW <= 64 && a.Kp % kKStep == 0;
}

// wn: 1 = 128-pixel tiles, 2 = 256-pixel tiles.
hipError_t launch_conv2d_direct(const ConvArgs& a, int wn, hipStream_t stream) {
  const bool flush = a.kc_steps > 0 && a.kc_steps < a.Kp / kKStep;
  if (wn == 1)
    return flush ? launch_direct_d<1, true>(a, stream) : launch_direct_d<1, false>(a, stream);
  return flush ? launch_direct_d<2, true>(a, stream) : launch_direct_d<2, false>(a, stream);
}

}  // namespace tq
