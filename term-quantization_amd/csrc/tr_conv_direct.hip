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
//   workgroup = 4 waves, tile 64*MB (Cout) x 128 (output pixels), MB = 1 or 2
//   wave      = 64*MB x 32: 2*MB MFMA blocks of 32 x 32, 8*MB MFMAs per K-step
//   K-step    = 64 codes of one filter tap (Cp % 64 == 0; 1x1 convs: any Cp, the last step
//               zero-padded)
//   A (weights [Cout_pad][Kp] fp16): global_load_lds_dwordx4 into a 3-slot ring, 8 KB/slot,
//             rows swizzled chunk ^= (row >> 1) & 7 on the source side (conflict-free reads)
//   B (activation codes [N][H][W][Cp] fp16): lane (r32, hh) loads, per block column and
//             16-code substep s, the 16 bytes [16s + 8hh, +8) of its pixel at the step's tap;
//             taps in the zero padding read a zero page; the next two steps' loads are in
//             flight during the current step's MFMAs (register triple buffer, counted vmcnt)
//   epilogue: every residual load of the wave tile issued first, then the int32 tile is
//             transposed through LDS so 16 lanes cover one pixel's 64 channels: each store
//             instruction writes 4 whole pixel rows (fp32 out: 1 KB, codes: 512 B).
#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

#ifndef TQ_ABLATE
#define TQ_ABLATE 0  // timing-only ablation builds (tools/ab/ablate.sh); 0 = the product kernel
#endif

#ifndef TQ_DIR_ASM_DMA
#define TQ_DIR_ASM_DMA 1  // 0: the weight DMA through the builtin (timing variants only)
#endif
#ifndef TQ_PHASE_TRACE
#define TQ_PHASE_TRACE 0  // timing-only builds (tools/ab/variant.sh): per-workgroup phase stamps
#endif

namespace tq {

#if TQ_PHASE_TRACE
// [workgroup][start, main loop done, epilogue done, hw id | xcc id << 32] (s_memrealtime ticks,
// 100 MHz), first kTraceMax workgroups of the last traced launch; read by tq_phase_trace_read
constexpr int kTraceMax = 1 << 16;
__device__ unsigned long long g_phase_trace[kTraceMax * 4];
#endif

namespace {

constexpr int kDirThreads = 256;
#ifndef TQ_DIR_DEPTH
#define TQ_DIR_DEPTH 2  // K-steps of activation fragments / weight images in flight
#endif
constexpr int kDirSlots = TQ_DIR_DEPTH + 1;  // A ring depth = K-steps in flight + 1

// MB = 1 or 2: Cout tile BM = 64 MB; the pixel tile is 128 (4 waves x 32 pixels)
template <int MB>
struct DirCfg {
  static constexpr int BM = 64 * MB;
  static constexpr int BN = 128;
  static constexpr int SLOT = BM * 8;                // u32x4 per A slot (BM rows x 128 B)
  static constexpr int SL = 16 * MB;                 // 4-channel slots per pixel (epilogue)
  static constexpr int TILE = 32 * SL;               // u32x4 per wave epilogue tile (int32)
  static constexpr int LDS = kDirSlots * SLOT > 4 * TILE ? kDirSlots * SLOT : 4 * TILE;
  static constexpr int AI = 2 * MB;                  // A wave-instructions per wave and step
  static constexpr int LPS = AI + 4;                 // vmem instructions per wave and K-step
};

// DS: a second accumulation phase, the fused downsample of a transition block (ConvArgs
// ds_*): its K-steps (one 1x1 tap, ds_Cp / 64 steps) run through the same pipeline after the
// main conv's, into fresh fp32 accumulators, while the main conv's sums wait in int32; the
// epilogue turns them into the identity (what the separate downsample conv would store) and
// adds it where a residual read from HBM would go.
// EPI: tq_epilogue.h epilogue_form (1 ReLU + code tables, 2 identity, 3 linear + one code
// table, 5 ReLU6 + code tables; the host picks it), 4 swish + one code table (SWISH only,
// swish_lut_form)
template <int MB, bool FLUSH, bool DS, bool SWISH, int EPI = 0>
__global__ __launch_bounds__(kDirThreads, 2) void conv2d_tp_direct_kernel(ConvArgs a) {
  using C = DirCfg<MB>;
  constexpr int NBM = 2 * MB;  // 32-row MFMA blocks per wave
  // the A ring + epilogue tile in DYNAMIC LDS (then the code tables): with a static array the
  // compiler drains every load in flight (s_waitcnt vmcnt(0)) before each ring read, as the
  // read may alias the LDS-DMA just issued -- the next K-steps' prefetch included
  extern __shared__ __attribute__((aligned(16))) u32x4 dyn_lds[];
  u32x4* lds = dyn_lds;
  __shared__ double coef[C::BM][2];  // epilogue (scale, shift) of the tile's channels
  __shared__ double coef2[DS ? C::BM : 1][2];  // the fused downsample's (scale, shift)
  uint16_t *lut_a, *lut_b;
  conv_luts(a, reinterpret_cast<uint16_t*>(dyn_lds + C::LDS), lut_a, lut_b);  // read after
                                                                              // the epilogue's barrier

#if TQ_PHASE_TRACE
  const unsigned long long tr_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = (a.Cout + C::BM - 1) / C::BM;
  const int m0 = (tile % mt) * C::BM;
  const int64_t n0 = (int64_t)(tile / mt) * C::BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const int64_t wn0 = n0 + wave * 32;  // first pixel of this wave
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page) + 8 * hh;

  // A staging: wave w moves rows [w BM/4, (w+1) BM/4) of each slot, AI instructions of 8 rows
  const uint16_t* arow[C::AI];
#pragma unroll
  for (int i = 0; i < C::AI; ++i) {
    const int r = (wave * C::AI + i) * 8 + (lane >> 3);
    arow[i] = wg + (int64_t)(m0 + r) * a.Kp + ((lane & 7) ^ ((r >> 1) & 7)) * 8;
  }

  // B pixel of this lane (MFMA column r32): element offset of its input origin + the lane's
  // K half, and the mask of filter taps inside the input (KH * KW <= 64)
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  int64_t boff = 0;
  uint64_t tmask = 0;
  int64_t boff2 = 0;      // DS: the lane's pixel in the downsample's input (1x1, pad 0)
  uint64_t tmask2 = 0;
  {
    const int64_t p = wn0 + r32;
    if (p < a.P) {
      const int64_t img = p / HoWo;
      const int64_t rem = p - img * HoWo;
      const int oh = (int)(rem / a.Wo);
      const int ow = (int)(rem - (int64_t)oh * a.Wo);
      const int ih0 = oh * a.sh - a.ph;
      const int iw0 = ow * a.sw - a.pw;
      boff = ((img * a.H + ih0) * a.W + iw0) * a.Cp + 8 * hh;
      if (DS) {
        boff2 = ((img * a.ds_H + (int64_t)oh * a.ds_s) * a.ds_W + (int64_t)ow * a.ds_s) *
                    a.ds_Cp + 8 * hh;
        tmask2 = 1ull;
      }
      for (int kr = 0; kr < a.KH; ++kr) {
        const int ih = ih0 + kr * a.dh;
        if (ih < 0 || ih >= a.H) continue;
        for (int ks = 0; ks < a.KW; ++ks) {
          const int iw = iw0 + ks * a.dw;
          if (iw >= 0 && iw < a.W) tmask |= 1ull << (kr * a.KW + ks);
        }
      }
    }
  }

  for (int i = threadIdx.x; i < C::BM; i += kDirThreads) {  // visible after the barriers
    const int co = m0 + i;
    const bool ok = co < a.Cout;
    coef[i][0] = a.ch_scale ? (ok ? a.ch_scale[co] : 0.0) : a.scale;
    coef[i][1] = a.ch_scale ? (ok ? a.ch_shift[co] : 0.0)
                            : ((a.bias && ok) ? (double)a.bias[co] : 0.0);
    if (DS) {
      coef2[i][0] = ok ? a.ds_scale[co] : 0.0;
      coef2[i][1] = ok ? a.ds_shift[co] : 0.0;
    }
  }

#if TQ_ABLATE == 6
  int nsteps = 0;  // timing only: setup + epilogue
#else
  int nsteps = a.Kp / kKStep;  // = KH * KW * Cp / 64 (Cp % 64 == 0)
#endif
  // position of the next K-step to issue, advanced incrementally (no divisions in the loop)
  int i_st = 0, i_tap = 0, i_cb = 0, i_ks = 0;
  int64_t i_toff = 0;  // ((kr * dh) * W + ks * dw) * Cp + cb
  int cur_cp = a.Cp, cur_kw = a.KW;
  const uint16_t* __restrict__ xsrc = xg;
  const int64_t row_step = (int64_t)a.dh * a.W * a.Cp;
  const int64_t col_step = (int64_t)a.dw * a.Cp;
  int64_t row_off = 0;

  // Issue K-step i_st: A-DMA into `slot`, B fragments into b (lane: codes [16s + 8hh, +8)).
  auto issue = [&](int slot, u32x4 (&b)[4]) {
#if TQ_ABLATE == 3  // timing only: no A DMA, no B loads (fragments from the zero page)
    (void)slot;
#pragma unroll
    for (int s = 0; s < 4; ++s) b[s] = (u32x4)(uint32_t)(i_st + s);
#else
#pragma unroll
    for (int i = 0; i < C::AI; ++i) {
#if TQ_DIR_ASM_DMA
      glds16_asm(arow[i] + (int64_t)i_st * kKStep,
                 lds + slot * C::SLOT + (wave * C::AI + i) * 64);
#else
      glds16(arow[i] + (int64_t)i_st * kKStep,
             lds + slot * C::SLOT + (wave * C::AI + i) * 64);
#endif
    }
    const bool ok = (tmask >> i_tap) & 1ull;
    const uint16_t* src = ok ? xsrc + (boff + i_toff) : zero;
    // codes of the lane's pixel left in this tap from its first (8-code) group: >= 56 except
    // in the partial last K-step of a 1x1 conv with Cp % 64 != 0, whose groups past Cp
    // (another pixel's channels) read the zero page instead
    const int cleft = cur_cp - i_cb - 8 * hh;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      b[s] = *reinterpret_cast<const u32x4*>((16 * s < cleft ? src : zero) + 16 * s);
#endif
    ++i_st;
    i_cb += kKStep;
    i_toff += kKStep;
    if (i_cb == cur_cp) {
      i_cb = 0;
      ++i_tap;
      if (++i_ks == cur_kw) {
        i_ks = 0;
        row_off += row_step;
        i_toff = row_off;
      } else {
        i_toff = row_off + (int64_t)i_ks * col_step;
      }
    }
  };

  float16v accf[NBM];
  int acci[(FLUSH || DS) ? NBM : 1][16];
#pragma unroll
  for (int bm = 0; bm < NBM; ++bm) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      accf[bm][r] = 0.0f;
      if (FLUSH) acci[bm][r] = 0;
    }
  }
  auto flush = [&]() {  // fp32 partial sums are exact integers below 2^24
#pragma unroll
    for (int bm = 0; bm < NBM; ++bm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acci[bm][r] += (int)accf[bm][r];
        accf[bm][r] = 0.0f;
      }
  };
  int kc_steps = a.kc_steps;
  int since_flush = 0;

  auto compute = [&](int slot, const u32x4 (&bc)[4]) {
    const u32x4* img = lds + slot * C::SLOT;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 2 * k + hh;
      const half8 bf = __builtin_bit_cast(half8, bc[k]);
#pragma unroll
      for (int bm = 0; bm < NBM; ++bm) {
        const half8 af = __builtin_bit_cast(half8, img[swz(32 * bm + r32, c)]);
#if TQ_ABLATE == 2  // timing only: no MFMA (fragments kept live)
        asm volatile("" ::"v"(af), "v"(bf));
#else
        accf[bm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, accf[bm], 0, 0, 0);
#endif
      }
    }
    if (FLUSH && ++since_flush == kc_steps) {
      flush();
      since_flush = 0;
    }
  };

  // kDirSlots - 1 K-steps in flight: step s is retired by vmcnt((kDirSlots - 2) LPS) (only
  // the steps issued after it younger), a barrier makes every wave's A-DMA of step s visible
  // and frees slot (s + kDirSlots - 1) % kDirSlots, which this step refills.
  constexpr int ND = kDirSlots;
  u32x4 bb[ND][4];
  auto step = [&](int s, int slot) {
    const int younger = nsteps - 1 - s < ND - 2 ? nsteps - 1 - s : ND - 2;
    if (younger >= 2) TQ_WAIT_VM(2 * C::LPS);
    else if (younger == 1) TQ_WAIT_VM(C::LPS);
    else TQ_WAIT_VM(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // ring reads stay behind the barrier
    if (s + ND - 1 < nsteps) issue((slot + ND - 1) % ND, bb[(slot + ND - 1) % ND]);
    compute(slot, bb[slot]);
  };
  // steady state: every wait and issue unconditional, so the compiler's own wait counts for
  // the fragment registers stay exact across the loop's back edge (with conditional issues
  // inside the loop it drained every load in flight once per iteration)
  auto step_full = [&](int slot) {
    TQ_WAIT_VM((ND - 2) * C::LPS);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // ring reads stay behind the barrier
    issue((slot + ND - 1) % ND, bb[(slot + ND - 1) % ND]);
    compute(slot, bb[slot]);
  };
  auto run = [&]() {
#pragma unroll
    for (int i = 0; i < ND - 1; ++i)
      if (i < nsteps) issue(i, bb[i]);
    int s = 0;
    for (; s + 2 * ND - 2 < nsteps; s += ND) {
#pragma unroll
      for (int j = 0; j < ND; ++j) step_full(j);
    }
    for (; s < nsteps; s += ND) {
#pragma unroll
      for (int j = 0; j < ND; ++j)
        if (s + j < nsteps) step(s + j, j);
    }
  };
  run();
  if (FLUSH) flush();
#if TQ_PHASE_TRACE
  const unsigned long long tr_t1 = __builtin_amdgcn_s_memrealtime();
#endif
  if (DS) {
    // the main conv's exact sums park in acci; the downsample accumulates from zero
#pragma unroll
    for (int bm = 0; bm < NBM; ++bm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (!FLUSH) acci[bm][r] = (int)accf[bm][r];
        accf[bm][r] = 0.0f;
      }
    __syncthreads();  // every wave is done reading the ring slots the second phase refills
#pragma unroll
    for (int i = 0; i < C::AI; ++i) {
      const int r = (wave * C::AI + i) * 8 + (lane >> 3);
      arow[i] = reinterpret_cast<const uint16_t*>(a.ds_w) + (int64_t)(m0 + r) * a.ds_Cp +
                ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    }
    nsteps = a.ds_Cp / kKStep;
    i_st = i_tap = i_cb = i_ks = 0;
    i_toff = row_off = 0;
    cur_cp = a.ds_Cp;
    cur_kw = 1;
    xsrc = reinterpret_cast<const uint16_t*>(a.ds_x);
    boff = boff2;
    tmask = tmask2;
    kc_steps = 0;  // no flush in the second phase (host-checked window)
    run();
  }

  // Epilogue.  Lane (slot = lane % SL) finishes channels m0 + 4*slot .. +3 of pixels
  // it*PXI + lane / SL of its wave: each store instruction writes PXI whole pixel rows.
  constexpr int PXI = 64 / C::SL;
  const bool vec = (a.Cout & 3) == 0;
  const int slot = lane % C::SL;
  const int co = m0 + 4 * slot;
  // A Cout tile with fewer than BM real channels (MobileNet-V2 / EfficientNet 1x1 convs: Cout
  // 16, 24, 96 ...): its epilogue packs the valid (pixel, 4-channel slot) pairs onto all 64
  // lanes instead of leaving the lanes of padding slots idle (Cout 16: 3 of 4 idle).
  const int vslots = (a.Cout - m0) < C::BM ? (a.Cout - m0 + 3) / 4 : C::SL;  // wave-uniform
  const bool packed = !DS && vec && vslots < C::SL;
  float4 res[32 / PXI];  // residuals first: their latency overlaps the transpose
#pragma unroll
  for (int it = 0; it < 32 / PXI; ++it) {
    const int64_t p = wn0 + it * PXI + lane / C::SL;
    res[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!DS && !packed && vec && a.residual && co < a.Cout && p < a.P)
      res[it] = *reinterpret_cast<const float4*>(a.residual + p * a.Cout + co);
  }
  __syncthreads();  // every wave is done with the A ring; coef[] is visible
  u32x4* t = lds + wave * C::TILE;  // [pixel][SL slots of 4 channels], slot ^= pixel & 15
  // int32 tile (MFMA layout) -> LDS, transposed so a lane reads whole 4-channel quads
  auto put_tile = [&](bool second) {
#pragma unroll
    for (int bm = 0; bm < NBM; ++bm)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int sl = 8 * bm + 2 * q + hh;  // channels 32bm + 8q + 4hh .. +3
        int v4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v4[e] = (second || !(FLUSH || DS)) ? (int)accf[bm][4 * q + e] : acci[bm][4 * q + e];
        u32x4 v;
        v.x = (uint32_t)v4[0];
        v.y = (uint32_t)v4[1];
        v.z = (uint32_t)v4[2];
        v.w = (uint32_t)v4[3];
        t[r32 * C::SL + (sl ^ (r32 & 15))] = v;
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile is in LDS
    __builtin_amdgcn_wave_barrier();
  };
  if (DS) {
    // the identity: fp32(acc2 * ds_scale + ds_shift), as the separate downsample conv stores it
    put_tile(true);
    if (co < a.Cout) {
      coef_t sc2[4], sh2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sc2[i] = (coef_t)coef2[4 * slot + i][0];
        sh2[i] = (coef_t)coef2[4 * slot + i][1];
      }
#pragma unroll
      for (int it = 0; it < 32 / PXI; ++it) {
        const int px = it * PXI + lane / C::SL;
        const u32x4 v = t[px * C::SL + (slot ^ (px & 15))];
        res[it] = make_float4(fold_acc((int)v.x, sc2[0], sh2[0]),
                              fold_acc((int)v.y, sc2[1], sh2[1]),
                              fold_acc((int)v.z, sc2[2], sh2[2]),
                              fold_acc((int)v.w, sc2[3], sh2[3]));
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // every read of the tile has returned
    __builtin_amdgcn_wave_barrier();
  }
  put_tile(false);
  if (packed) {
    // pair idx -> (pixel idx / vslots, slot idx % vslots); floor(idx * ceil(2^16 / vslots)
    // / 2^16) is the exact quotient for idx < 32 * 32 and vslots < 128
    const uint32_t inv = (65536u + vslots - 1) / vslots;
    for (int idx = lane; idx < 32 * vslots; idx += 64) {
      const int px = (int)(((uint32_t)idx * inv) >> 16);
      const int sl = idx - px * vslots;
      const int64_t p = wn0 + px;
      if (p >= a.P) continue;
      const int c4 = m0 + 4 * sl;
      coef_t psc[4], psh[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        psc[i] = (coef_t)coef[4 * sl + i][0];
        psh[i] = (coef_t)coef[4 * sl + i][1];
      }
      const float4 rv = a.residual
                            ? *reinterpret_cast<const float4*>(a.residual + p * a.Cout + c4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      const u32x4 v = t[px * C::SL + (sl ^ (px & 15))];
      const int acc4[4] = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
      if constexpr (EPI == 1)
        emit4_relu_lut(a, p, c4, acc4, psc, psh, rv, lut_a, lut_b);
      else if constexpr (EPI == 2)
        emit4_identity(a, p, c4, acc4, psc, psh);
      else if constexpr (EPI == 3)
        emit4_linear_lut(a, p, c4, acc4, psc, psh, rv, lut_a);
      else if constexpr (EPI == 4)
        emit4_swish_lut(a, p, c4, acc4, psc, psh, lut_a);
      else if constexpr (EPI == 5)
        emit4_relu_lut<true>(a, p, c4, acc4, psc, psh, rv, lut_a, lut_b);
      else
        emit4_nhwc_res<SWISH>(a, p, c4, acc4, psc, psh, rv, lut_a, lut_b);
    }
#if !TQ_PHASE_TRACE
    return;
#endif
  }
#if TQ_PHASE_TRACE
  if (!packed && co < a.Cout) {
#else
  if (co >= a.Cout) return;
#endif
  coef_t sc[4], sh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sc[i] = (coef_t)coef[4 * slot + i][0];
    sh[i] = (coef_t)coef[4 * slot + i][1];
  }
  // fully unrolled: res[] must stay in registers (a partial unroll indexes it in scratch)
#pragma clang loop unroll(full)
  for (int it = 0; it < 32 / PXI; ++it) {
    const int px = it * PXI + lane / C::SL;
    const int64_t p = wn0 + px;
    if (p >= a.P) continue;
    const u32x4 v = t[px * C::SL + (slot ^ (px & 15))];
    const int acc4[4] = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
#if TQ_ABLATE == 7  // timing only: no epilogue stores (sums kept live)
    if (acc4[0] == 0x7fffffff && a.out) a.out[p] = res[it].x + (float)(sc[0] + sh[0]);
    continue;
#endif
    if constexpr (EPI == 1)
      emit4_relu_lut(a, p, co, acc4, sc, sh, res[it], lut_a, lut_b);  // (host: vec)
    else if constexpr (EPI == 2)
      emit4_identity(a, p, co, acc4, sc, sh);
    else if constexpr (EPI == 3)
      emit4_linear_lut(a, p, co, acc4, sc, sh, res[it], lut_a);  // (host: vec)
    else if constexpr (EPI == 4)
      emit4_swish_lut(a, p, co, acc4, sc, sh, lut_a);
    else if constexpr (EPI == 5)
      emit4_relu_lut<true>(a, p, co, acc4, sc, sh, res[it], lut_a, lut_b);
    else if (vec)
      emit4_nhwc_res<SWISH>(a, p, co, acc4, sc, sh, res[it], lut_a, lut_b);
    else
      emit4_nhwc(a, p, co, acc4, sc, sh, false, lut_a, lut_b);
  }
#if TQ_PHASE_TRACE
  }
  // wave 0's stamp once its epilogue stores are issued (not completed: waiting for them
  // would hold the workgroup's slot longer than the product kernel does)
  if (threadIdx.x == 0 && blockIdx.x < kTraceMax) {
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));     // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // HW_REG_XCC_ID
    unsigned long long* r = g_phase_trace + (int64_t)blockIdx.x * 4;
    r[0] = tr_t0;
    r[1] = tr_t1;
    r[2] = t2;
    r[3] = hw | ((unsigned long long)xcc << 32);
  }
#endif
}

// ---------------------------------------------------------------------------------------
// Pointwise engine: 1x1 convs (pad 0, any stride) with K <= 3 K-steps (Cin <= 192): the
// MobileNet-V2 / EfficientNet expand and project convs and the ResNet downsamples.  Their
// tiles are mostly epilogue (1-4 K-steps of MFMA, then 8192 outputs), so one tile per
// workgroup leaves each workgroup's lifetime to fixed latencies (weight DMA, fragment loads,
// one barrier, the epilogue's stores) -- ~50k such workgroups for a 112x112 MobileNet-V2
// layer.  Here a persistent workgroup owns one 64-row Cout tile: its weights (all NKS
// K-steps), epilogue coefficients and code tables are staged once, and its 4 waves walk pixel
// tiles independently (no workgroup barrier in the loop: the weights are static and each
// wave transposes its own epilogue tile), each loading the NEXT tile's activation fragments
// into registers before running the current tile's MFMAs and epilogue.
// Same exact sums (no flush: the host window check covers K <= 4 steps or the kernel is not
// used) and the same shared epilogue as the direct engine: bit-identical outputs.
// ---------------------------------------------------------------------------------------
constexpr int kPwWaves = 4;

template <int NKS, bool SWISH>
__global__ __launch_bounds__(kDirThreads, 2) void conv2d_tp_pw_kernel(ConvArgs a, int G) {
  using C = DirCfg<1>;
  __shared__ __attribute__((aligned(16))) u32x4 wlds[NKS * C::SLOT];  // [NKS][64 rows][8]
  __shared__ __attribute__((aligned(16))) u32x4 tlds[kPwWaves * C::TILE];
  __shared__ double coef[C::BM][2];
  extern __shared__ __attribute__((aligned(16))) uint16_t dyn_lut[];
  uint16_t *lut_a, *lut_b;
  conv_luts(a, dyn_lut, lut_a, lut_b);

  const int mt = (a.Cout + C::BM - 1) / C::BM;
  const int m0 = (blockIdx.x % mt) * C::BM;
  const int g = blockIdx.x / mt;
  const int64_t ntn = (a.P + C::BN - 1) / C::BN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page) + 8 * hh;

  // the Cout tile's weights, every K-step, once (the swizzled image of the direct engine)
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int i = 0; i < C::AI; ++i) {
      const int r = (wave * C::AI + i) * 8 + (lane >> 3);
      glds16(wg + (int64_t)(m0 + r) * a.Kp + ks * kKStep + ((lane & 7) ^ ((r >> 1) & 7)) * 8,
             wlds + ks * C::SLOT + (wave * C::AI + i) * 64);
    }
  for (int i = threadIdx.x; i < C::BM; i += kDirThreads) {
    const int co = m0 + i;
    const bool ok = co < a.Cout;
    coef[i][0] = a.ch_scale ? (ok ? a.ch_scale[co] : 0.0) : a.scale;
    coef[i][1] = a.ch_scale ? (ok ? a.ch_shift[co] : 0.0)
                            : ((a.bias && ok) ? (double)a.bias[co] : 0.0);
  }
  TQ_WAIT_VM(0);
  __syncthreads();  // weights, coefficients and code tables visible; no barrier after this

  // epilogue role of this lane: channels m0 + 4 slot .. +3 of pixels it * PXI + lane / SL
  constexpr int PXI = 64 / C::SL;
  const int slot = lane % C::SL;
  const int co = m0 + 4 * slot;
  coef_t sc[4], sh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sc[i] = (coef_t)coef[4 * slot + i][0];
    sh[i] = (coef_t)coef[4 * slot + i][1];
  }
  const bool vec = (a.Cout & 3) == 0;
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  u32x4* t = tlds + wave * C::TILE;

  // activation fragments of pixel tile nt for this lane (MFMA column r32), all K-steps
  auto load_b = [&](int64_t nt, u32x4 (&b)[NKS][4]) __attribute__((always_inline)) {
    const int64_t p = nt * C::BN + wave * 32 + r32;
    const uint16_t* src = zero;
    if (p < a.P) {
      const int64_t img = p / HoWo;
      const int64_t rem = p - img * HoWo;
      const int oh = (int)(rem / a.Wo);
      const int ow = (int)(rem - (int64_t)oh * a.Wo);
      src = xg + ((img * a.H + (int64_t)oh * a.sh) * a.W + (int64_t)ow * a.sw) * a.Cp + 8 * hh;
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const int cleft = a.Cp - ks * kKStep - 8 * hh;  // codes left in this K-step's groups
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        b[ks][s4] = *reinterpret_cast<const u32x4*>(
            (p < a.P && 16 * s4 < cleft ? src + ks * kKStep : zero) + 16 * s4);
    }
  };
  auto tile = [&](int64_t nt, const u32x4 (&b)[NKS][4]) __attribute__((always_inline)) {
    const int64_t wn0 = nt * C::BN + wave * 32;
    // residuals first (their latency overlaps the MFMAs), as unconditional loads: a lane
    // without one reads the zero page (a per-lane branch around each load made the compiler
    // drain every load in flight, the next tile's fragments included)
    float4 res[32 / PXI];
    if (vec && a.residual) {
#pragma unroll
      for (int it = 0; it < 32 / PXI; ++it) {
        const int64_t p = wn0 + it * PXI + lane / C::SL;
        const bool ok = co < a.Cout && p < a.P;
        res[it] = *reinterpret_cast<const float4*>(
            ok ? a.residual + p * a.Cout + co : reinterpret_cast<const float*>(g_zero_page));
      }
    } else {
#pragma unroll
      for (int it = 0; it < 32 / PXI; ++it) res[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float16v acc[2];
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[bm][r] = 0.0f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const half8 bf = __builtin_bit_cast(half8, b[ks][k]);
#pragma unroll
        for (int bm = 0; bm < 2; ++bm) {
          const half8 af =
              __builtin_bit_cast(half8, wlds[ks * C::SLOT + swz(32 * bm + r32, 2 * k + hh)]);
          acc[bm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc[bm], 0, 0, 0);
        }
      }
    // int32 tile -> this wave's LDS region, transposed so a lane reads 4-channel quads
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int sl = 8 * bm + 2 * q + hh;
        u32x4 v;
        v.x = (uint32_t)(int)acc[bm][4 * q];
        v.y = (uint32_t)(int)acc[bm][4 * q + 1];
        v.z = (uint32_t)(int)acc[bm][4 * q + 2];
        v.w = (uint32_t)(int)acc[bm][4 * q + 3];
        t[r32 * C::SL + (sl ^ (r32 & 15))] = v;
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile is in LDS
    __builtin_amdgcn_wave_barrier();
    if (co < a.Cout) {
#pragma clang loop unroll(full)
      for (int it = 0; it < 32 / PXI; ++it) {
        const int px = it * PXI + lane / C::SL;
        const int64_t p = wn0 + px;
        if (p >= a.P) continue;
        const u32x4 v = t[px * C::SL + (slot ^ (px & 15))];
        const int acc4[4] = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
        if (vec)
          emit4_nhwc_res<SWISH>(a, p, co, acc4, sc, sh, res[it], lut_a, lut_b);
        else
          emit4_nhwc(a, p, co, acc4, sc, sh, false, lut_a, lut_b);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // every read of the tile returned before it is reused
    __builtin_amdgcn_wave_barrier();
  };
  // pixel tiles g, g + G, ...: the next tile's fragments are in flight during this one
  // (unconditional loads: past the last tile every lane reads the zero page)
  u32x4 bcur[NKS][4];
  load_b(g, bcur);
  for (int64_t nt = g; nt < ntn; nt += G) {
    u32x4 bnext[NKS][4];
    load_b(nt + G, bnext);
    tile(nt, bcur);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) bcur[ks][s4] = bnext[ks][s4];
  }
}

template <int NKS, bool SWISH>
hipError_t launch_pw_cfg(const ConvArgs& a, hipStream_t stream) {
  using C = DirCfg<1>;
  const int mt = (int)((a.Cout + C::BM - 1) / C::BM);
  const int64_t ntn = (a.P + C::BN - 1) / C::BN;
  // persistent: about 2 workgroups per CU in all (the register budget of 2 waves per SIMD)
  int64_t G = (2 * (int64_t)device_cus() + mt - 1) / mt;
  if (G > ntn) G = ntn;
  if (G < 1) G = 1;
  conv2d_tp_pw_kernel<NKS, SWISH>
      <<<dim3((unsigned)(G * mt)), kDirThreads, (size_t)conv_lut_bytes(a), stream>>>(a, (int)G);
  return hipGetLastError();
}

template <int MB, bool FLUSH, bool DS, bool SWISH = false, int EPI = 0>
hipError_t launch_direct_cfg(const ConvArgs& a, hipStream_t stream) {
  using C = DirCfg<MB>;
  const int64_t tiles = ((a.P + C::BN - 1) / C::BN) * ((a.Cout + C::BM - 1) / C::BM);
  static bool attr_set = false;  // the MB = 2 ring + code tables pass the 64 KB default
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv2d_tp_direct_kernel<MB, FLUSH, DS, SWISH, EPI>),
        hipFuncAttributeMaxDynamicSharedMemorySize,
        160 * 1024 - (C::BM + (DS ? C::BM : 1)) * 16);  // minus the static coef arrays
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  conv2d_tp_direct_kernel<MB, FLUSH, DS, SWISH, EPI>
      <<<dim3((unsigned)tiles), kDirThreads, (size_t)(C::LDS * 16 + conv_lut_bytes(a)), stream>>>(a);
  return hipGetLastError();
}

template <int MB, bool DS>
hipError_t launch_direct_mb(const ConvArgs& a, hipStream_t stream) {
  const bool flush = a.kc_steps > 0 && a.kc_steps < a.Kp / kKStep;
  const int form = MB == 1 && !DS ? epilogue_form(a) : 0;
  if (form == 1)
    return flush ? launch_direct_cfg<1, true, false, false, 1>(a, stream)
                 : launch_direct_cfg<1, false, false, false, 1>(a, stream);
  if (form == 2)
    return flush ? launch_direct_cfg<1, true, false, false, 2>(a, stream)
                 : launch_direct_cfg<1, false, false, false, 2>(a, stream);
  if (form == 3)
    return flush ? launch_direct_cfg<1, true, false, false, 3>(a, stream)
                 : launch_direct_cfg<1, false, false, false, 3>(a, stream);
  if (form == 5)
    return flush ? launch_direct_cfg<1, true, false, false, 5>(a, stream)
                 : launch_direct_cfg<1, false, false, false, 5>(a, stream);
  return flush ? launch_direct_cfg<MB, true, DS>(a, stream)
               : launch_direct_cfg<MB, false, DS>(a, stream);
}

}  // namespace

// Cp % 64 == 0, or a 1x1 conv with any Cp (% 8 == 0): its K-steps walk the zero-padded
// weight rows (Kp = roundup(Cp, 64)) and the last one reads the zero page past Cp.
bool conv_direct_eligible(const ConvArgs& a, int out_nhwc) {
  return out_nhwc && (a.Cp % kKStep == 0 || (a.KH * a.KW == 1 && a.Cp % 8 == 0)) &&
         a.KH * a.KW <= 64 && a.Kp % kKStep == 0 &&
         (a.ds_x == nullptr || a.ds_Cp % kKStep == 0);
}

// The pointwise engine's shapes: 1x1, pad 0, K <= 3 K-steps (4 spills) with no flush,
// no fused downsample.
bool conv_pw_eligible(const ConvArgs& a, int out_nhwc) {
  const int nks = a.Kp / kKStep;
  return out_nhwc && a.KH == 1 && a.KW == 1 && a.ph == 0 && a.pw == 0 && a.Cp % 8 == 0 &&
         a.Kp % kKStep == 0 && nks >= 1 && nks <= 3 &&
         (a.kc_steps == 0 || a.kc_steps >= nks) && a.ds_x == nullptr &&
         (a.relu != kActSwish || (a.Cout & 3) == 0);
}

hipError_t launch_conv2d_pw(const ConvArgs& a, hipStream_t stream) {
  const bool sw = a.relu == kActSwish;
  switch (a.Kp / kKStep) {
    case 1: return sw ? launch_pw_cfg<1, true>(a, stream) : launch_pw_cfg<1, false>(a, stream);
    case 2: return sw ? launch_pw_cfg<2, true>(a, stream) : launch_pw_cfg<2, false>(a, stream);
    case 3: return sw ? launch_pw_cfg<3, true>(a, stream) : launch_pw_cfg<3, false>(a, stream);
    default: return hipErrorInvalidValue;  // conv_pw_eligible: 1..3 K-steps only
  }
}

// mb: 1 = 64 x 128 tiles, 2 = 128 x 128 tiles.
hipError_t launch_conv2d_direct(const ConvArgs& a, int mb, hipStream_t stream) {
  if (a.relu == kActSwish) {  // swish epilogue (EfficientNet): 64-row tiles, no fused downsample
    if (a.ds_x || (a.Cout & 3)) return hipErrorInvalidValue;
    const bool flush = a.kc_steps > 0 && a.kc_steps < a.Kp / kKStep;
    if (swish_lut_form(a))  // (the expand convs' codes-only form, EPI 4)
      return flush ? launch_direct_cfg<1, true, false, true, 4>(a, stream)
                   : launch_direct_cfg<1, false, false, true, 4>(a, stream);
    return flush ? launch_direct_cfg<1, true, false, true>(a, stream)
                 : launch_direct_cfg<1, false, false, true>(a, stream);
  }
  if (a.ds_x)  // fused downsample: 64-row tiles (the second int32 tile costs registers)
    return launch_direct_mb<1, true>(a, stream);
  if (mb == 2) return launch_direct_mb<2, false>(a, stream);
  return launch_direct_mb<1, false>(a, stream);
}

#if TQ_PHASE_TRACE
extern "C" int tq_phase_trace_read(void* dst, int64_t n_wg) {
  if (n_wg > kTraceMax) n_wg = kTraceMax;
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_phase_trace), (size_t)n_wg * 32, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

}  // namespace tq
