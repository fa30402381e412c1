// Term-pair Conv2d on the matrix cores, row-strip engine: the ResNet-18 layer-1 convs
// (3x3, stride 1, pad 1, 64 -> 64 channels, W <= 56).
//
// Same arithmetic and exactness argument as tr_conv_mfma.hip (fp16 term-sum codes, exact
// products on v_mfma_f32_32x32x16_f16, fp32 partial sums exact while they stay within 2^24);
// this engine runs only when the whole K range is one exact window (kc_steps == 0), so the
// fp32 sums are converted to int32 once, and its outputs are bit-identical to the other
// engines' (same integer sums, same epilogue arithmetic).
//
// Why a separate engine.  Layer 1 is short-K (576) and wide: per output its fused epilogue
// (BN fold, residual, ReLU, fp32 store, next layer's TR codes) costs ~35 VALU, more than the
// 576 MACs cost the matrix cores, and the direct engine's activation fragments come through
// the vector L1 nine times per pixel.  Here:
//   * one persistent workgroup per CU keeps the whole 64 x 576 weight matrix in LDS (72 KB,
//     loaded once) -- no weight stream at all;
//   * the CU's 8 waves form two independent teams of 4; each team owns one LDS patch buffer
//     and works through its own tiles (4 output rows of one image), so one team's epilogue
//     VALU runs beside the other team's MFMAs on the same SIMDs (waves w and w + 4 share a
//     SIMD).  Teams synchronise through LDS counters, not the workgroup barrier;
//   * a tile's input rows (TR + 2 rows x W pixels x 64 codes) arrive by LDS-DMA
//     (global_load_lds_dwordx4) while the team runs the previous tile's epilogue, and all
//     nine taps read their A fragments from that patch;
//   * MFMA roles: A = activation codes (rows = 32 output pixels), B = weight codes (columns =
//     32 output channels).  A lane's accumulators are then 16 pixels of ONE channel, so the
//     BN coefficients are per-lane constants and every residual load / fp32 store
//     instruction covers whole 128-byte channel rows of two pixels.
//
// LDS (16-byte units): weights [64][72] (row = output channel, unit = 8 codes of K, unit
// index swizzled ^ ((row >> 1) & 7)), then per team a patch [(TR + 2) * W + 1][8] (pixel
// (j, x) of the patch = input row r0 - 1 + j, column x; units swizzled ^ ((pix >> 1) & 7);
// the extra pixel is all zeros and stands in for taps outside the image), then two team
// counters.
#include <stdlib.h>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

#ifndef TQ_ABLATE
#define TQ_ABLATE 0  // timing-only ablation builds (tools/ab/ablate.sh); 0 = the product kernel
#endif

namespace tq {

namespace {

constexpr int kStripThreads = 512;  // 2 teams x 4 waves
constexpr int kStripTR = 4;         // output rows per tile
constexpr int kStripC = 64;         // input = output channels
constexpr int kStripTaps = 9;       // 3 x 3
constexpr int kStripKU = kStripTaps * kStripC / 8;  // 72 units of 8 codes per weight row
constexpr int kStripWUnits = kStripC * kStripKU;    // 4608 units = 72 KB
constexpr int kStripMaxW = 56;

__host__ __device__ constexpr int strip_patch_px(int w) { return (kStripTR + 2) * w + 1; }

// LDS bytes of a launch before the epilogue code tables (16-byte aligned).
__host__ __device__ inline int64_t strip_lds_bytes(int64_t w) {
  return ((int64_t)kStripWUnits + 2 * strip_patch_px((int)w) * 8 + 64) * 16 + 16;
}

// Team-sync guard exhaustions since the last tq_sync_faults() (device-wide; a
// non-zero count means some launch computed with a patch whose staging was not confirmed).
__device__ uint32_t g_strip_sync_faults;

// Wave-uniform team barrier through an LDS counter: every wave of the team adds 1, then
// waits until the counter reaches `target` (4 per barrier).  The caller has already retired
// what the others must see (vmcnt for its LDS-DMA, lgkmcnt for its LDS reads).  The spin is
// bounded (a broken protocol then shows as wrong results, never as a hung GPU).
__device__ __forceinline__ void team_sync(uint32_t* ctr, uint32_t target) {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
#if TQ_ABLATE == 13  // timing only: no team synchronisation
  return;
#endif
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  int guard = 0;
  for (; guard < (1 << 22); ++guard) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
    __builtin_amdgcn_s_sleep(1);
  }
  // guard exhausted: the protocol broke and this wave goes on with a patch that may be
  // partly staged -- count it where the host can see it (tq_sync_faults)
  if (guard == (1 << 22) && (threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(&g_strip_sync_faults, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-lane epilogue constants.
struct StripEpi {
  double sc, sh;
  int npeel_a, npeel_b;
  bool fast_a, fast_b;
};

// Fixed LDS-DMA instructions per wave and patch refill (the widest patch: (TR + 2) rows x
// kStripMaxW pixels = 42 wave-instructions over 4 waves); pieces past a narrower patch land
// in a dummy slot.  A fixed count keeps the compiler's vmcnt bookkeeping exact.
constexpr int kStripDma = ((kStripTR + 2) * kStripMaxW * 8 / 64 + 3) / 4;

// The epilogue of 4 consecutive tile pixels P0 .. P0 + 3 of this lane's channel.  LUT: the
// fused executor's form only -- ReLU, every code output from its table (the host checks) --
// without the computed-code paths and the runtime activation branches.
template <bool RES, bool OUT, bool CB, bool FULL, bool LUT>
__device__ __forceinline__ void strip_emit4(const ConvArgs& a, const StripEpi& ep,
                                            const float acc4[4], const float rv[4], int P0,
                                            int nvalid, float* outp, int16_t* ca, int16_t* cbp,
                                            const uint16_t* lut_a, const uint16_t* lut_b) {
  float y[4], o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    y[e] = fold_acc((int)acc4[e], (coef_t)ep.sc, (coef_t)ep.sh);
    if (RES) y[e] += rv[e];  // (no + 0.0f without one: -0.0 stays, as in tq_epilogue.h)
    o[e] = y[e];
    if (LUT || a.relu) {
      y[e] = y[e] > 0.0f ? y[e] : 0.0f;
      if (!LUT && a.relu == 2) y[e] = y[e] < 6.0f ? y[e] : 6.0f;  // ReLU6
      o[e] = o[e] != o[e] ? o[e] : y[e];  // the stored value keeps a NaN (torch.relu)
    }
  }
  if (OUT) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (FULL || P0 + e < nvalid) outp[e * kStripC] = o[e];
  }
#pragma unroll
  for (int side = 0; side < (CB ? 2 : 1); ++side) {
    int16_t* codes = side ? cbp : ca;
    if (!codes) continue;
    const double inv = side ? a.inv_b : a.inv_a;
    const float maxv = side ? a.maxv_b : a.maxv_a;
    const uint16_t* lut = side ? lut_b : lut_a;
    const int fmt = side ? a.fmt_b : a.fmt_a;
    uint32_t bits[4];
    // the code table after a ReLU only: the signed-value variant (tq_device.h lut_codes) put
    // this engine over its register budget (scratch spills: 127 -> 177 us, r03ai); without a
    // ReLU the codes are computed
    if (LUT || (lut && act_nonneg(a.relu))) {
      uint32_t qv[4];
      relu_q_epi<4>(y, inv, maxv, qv);
#pragma unroll
      for (int e = 0; e < 4; ++e) bits[e] = lut[qv[e]];
    } else if constexpr (!LUT) {
      int32_t v[4];
      if (side ? ep.fast_b : ep.fast_a) {
        tr_values_relu4(y, inv, maxv, side ? ep.npeel_b : ep.npeel_a, v);
      } else {
        const int k = side ? a.k_b : a.k_a;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = tr_value_g1_inv(y[e], inv, maxv, k);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) bits[e] = code_bits(v[e], fmt);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (FULL || P0 + e < nvalid) codes[e * kStripC] = (int16_t)bits[e];
  }
}

// One tile of one wave: NB pixel blocks (pset, pset + 2, ...) x 32 output channels.
// RES / OUT / CB: residual input, fp32 output, second code target present (compile-time, so
// each instantiation carries only the epilogue it runs).  `refill` runs after the epilogue
// (team sync + the next patch's DMA, which then lands during the next tile's sync wait).
template <int NB, bool RES, bool OUT, bool CB, bool LUT, typename Refill>
__device__ __forceinline__ void strip_tile(const ConvArgs& a, const u32x4* patch,
                                           const u32x4* wrow_ptr, int wkey, int W, int ZP,
                                           int pset, int r32, int hh, int co, int64_t pix0,
                                           int nvalid, const StripEpi& ep, Refill refill,
                                           const uint16_t* lut_a, const uint16_t* lut_b) {
  // ---- main loop: 9 taps x 4 substeps of 16 codes; fragments one substep ahead ----
  float16v acc[NB];
  int pp0[NB];
  uint32_t edge[NB];  // bit 0: tap column -1 outside the image, bit 1: column +1 outside
#pragma unroll
  for (int i = 0; i < NB; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;
    const int P = (pset + 2 * i) * 32 + r32;
    const int ro = P / W;
    const int x = P - ro * W;
    pp0[i] = ro * W + x - 1;
    edge[i] = (x == 0 ? 1u : 0u) | (x == W - 1 ? 2u : 0u);
  }
  auto addr = [&](int t, int base[NB], int key[NB]) {
    const int kr = t / 3, ks = t - 3 * (t / 3);
    const uint32_t bad = ks == 0 ? 1u : (ks == 2 ? 2u : 0u);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int pp = (edge[i] & bad) ? ZP : pp0[i] + kr * W + ks;
      base[i] = pp * 8;
      key[i] = hh ^ ((pp >> 1) & 7);
    }
  };
  int base[NB], key[NB];
  half8 af[2][NB], bf[2];
  addr(0, base, key);
  bf[0] = __builtin_bit_cast(half8, wrow_ptr[hh ^ wkey]);
#pragma unroll
  for (int i = 0; i < NB; ++i) af[0][i] = __builtin_bit_cast(half8, patch[base[i] + key[i]]);
#pragma unroll 1
  for (int t = 0; t < (TQ_ABLATE == 15 ? 0 : kStripTaps); ++t) {
    int nbase[NB], nkey[NB];
    const int tn = t + 1 < kStripTaps ? t + 1 : t;
    addr(tn, nbase, nkey);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int cur = s & 1, nxt = cur ^ 1;
      // prefetch the next substep (the next tap's first after s == 3)
      if (s < 3) {
        bf[nxt] = __builtin_bit_cast(half8, wrow_ptr[(t * 8 + 2 * (s + 1) + hh) ^ wkey]);
#pragma unroll
        for (int i = 0; i < NB; ++i)
          af[nxt][i] = __builtin_bit_cast(half8, patch[base[i] + ((2 * (s + 1)) ^ key[i])]);
      } else {
        bf[nxt] = __builtin_bit_cast(half8, wrow_ptr[(tn * 8 + hh) ^ wkey]);
#pragma unroll
        for (int i = 0; i < NB; ++i)
          af[nxt][i] = __builtin_bit_cast(half8, patch[nbase[i] + nkey[i]]);
      }
      // keep the schedule: next substep's reads in flight during this substep's MFMAs
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NB; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[cur][i], bf[cur], acc[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      base[i] = nbase[i];
      key[i] = nkey[i];
    }
  }

#if TQ_ABLATE == 15  // timing only: the fragments feed the epilogue instead of the MFMAs
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i][0] = (float)af[0][i][0] + (float)bf[0][1];
#endif
  const bool full = nvalid == kStripTR * W;  // wave-uniform: no pixel of the tile past Ho
  // residuals of group g = 4 i + q: tile pixels pl(i) + 8 q .. + 3 (rows past a partial
  // tile re-read a valid pixel)
  auto load_res = [&](int g, float rv[4]) {
    const int lp0 = (pset + 2 * (g >> 2)) * 32 + 4 * hh + 8 * (g & 3);
    const float* rp = a.residual + (pix0 + lp0) * kStripC + co;
    // one base pointer + immediate offsets (per-element indices kept out of registers);
    // rows past a partial tile re-read the last valid pixel
    const int last = nvalid - 1 - lp0;
#pragma unroll
    for (int e = 0; e < 4; ++e) rv[e] = rp[(full || e <= last ? e : last) * kStripC];
  };
#if TQ_ABLATE == 11  // timing only: no epilogue (sums kept live)
  refill();
#pragma unroll
  for (int i = 0; i < NB; ++i)
    if (acc[i][0] == 12345.0f && a.out) a.out[pix0 + i] = acc[i][1] + acc[i][15];
  return;
#endif
  // ---- epilogue: lane = channel co, 16 pixels per block (Cout = cp = 64 per pixel) ----
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int pl = (pset + 2 * i) * 32 + 4 * hh;  // tile pixel of accumulator row 0
    const int64_t pb = pix0 + pl;
    float* outp = OUT ? a.out + pb * kStripC + co : nullptr;
    int16_t* ca = a.codes_a ? a.codes_a + pb * kStripC + co : nullptr;
    int16_t* cbp = CB ? a.codes_b + pb * kStripC + co : nullptr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int g = 4 * i + q;
      const int off = 8 * q * kStripC;
      const float acc4[4] = {acc[i][4 * q], acc[i][4 * q + 1], acc[i][4 * q + 2],
                             acc[i][4 * q + 3]};
      float rv4[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // unused without a residual
      if (RES) load_res(g, rv4);  // latency covered by the other team's waves
      __builtin_amdgcn_sched_barrier(0);  // one group's loads and values live at a time
      if (full)
        strip_emit4<RES, OUT, CB, true, LUT>(a, ep, acc4, rv4, pl + 8 * q, nvalid, outp + off,
                                   ca ? ca + off : nullptr, cbp ? cbp + off : nullptr, lut_a,
                                   lut_b);
      else
        strip_emit4<RES, OUT, CB, false, LUT>(a, ep, acc4, rv4, pl + 8 * q, nvalid, outp + off,
                                    ca ? ca + off : nullptr, cbp ? cbp + off : nullptr, lut_a,
                                    lut_b);
    }
  }
  refill();
}

template <bool RES, bool OUT, bool CB, bool LUT>
__global__ __launch_bounds__(kStripThreads, 2) void conv2d_tp_strip_kernel(ConvArgs a,
                                                                           int64_t ntiles) {
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  const int W = a.W;
  const int PX = strip_patch_px(W);            // patch pixels incl. the zero pixel
  const int ZP = PX - 1;                        // the zero pixel
  u32x4* wl = lds;                              // weights
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int team = wave >> 2;
  const int wt = wave & 3;
  u32x4* patch = lds + kStripWUnits + team * PX * 8;
  u32x4* dummy = lds + kStripWUnits + 2 * PX * 8;  // 1 KB sink for padding DMA pieces
  uint32_t* ctr = reinterpret_cast<uint32_t*>(dummy + 64) + team;
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page) + 8 * (lane & 7);

  // this workgroup's tiles: a contiguous range (neighbouring strips share halo rows; the
  // logical index keeps a run of workgroups on one XCD)
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t t_begin = g * ntiles / gridDim.x;
  const int64_t t_end = (g + 1) * ntiles / gridDim.x;
  const int rb_per_img = (a.Ho + kStripTR - 1) / kStripTR;

  // ---- weights -> LDS (all 8 waves), zero pixels, counters ----
  for (int m = wave; m < kStripWUnits / 64; m += 8) {
    const int u = m * 64 + lane;
    const int row = u / kStripKU;
    const int ph = u - row * kStripKU;
    const int ch = ph ^ ((row >> 1) & 7);
    glds16(wg + (int64_t)row * a.Kp + ch * 8, wl + m * 64);
  }
  if (threadIdx.x < 16)
    lds[kStripWUnits + (threadIdx.x >> 3) * PX * 8 + ZP * 8 + (threadIdx.x & 7)] = (u32x4)0u;
  if (threadIdx.x < 2) reinterpret_cast<uint32_t*>(dummy + 64)[threadIdx.x] = 0u;
  // epilogue code tables behind the counters (the launcher sized the LDS for them or
  // cleared lut_a / lut_b)
  uint16_t *lut_a, *lut_b;
  conv_luts(a, reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(lds) + strip_lds_bytes(W)),
            lut_a, lut_b);

  // patch DMA of tile t into this team's buffer: (TR + 2) * W pixels x 8 units, lane-linear;
  // always kStripDma instructions per wave (pieces past the patch go to the dummy slot)
  const int npieces = (kStripTR + 2) * W * 8 / 64;
  auto issue_patch = [&](int64_t t) {
    const int64_t img = t / rb_per_img;
    const int r0 = (int)(t - img * rb_per_img) * kStripTR;
#pragma unroll
    for (int k = 0; k < kStripDma; ++k) {
      const int m = wt + 4 * k;
      const int u = m * 64 + lane;
      const int pp = u >> 3;
      const int ch = (u & 7) ^ ((pp >> 1) & 7);
      const int j = pp / W;
      const int x = pp - j * W;
      const int ir = r0 - 1 + j;
      const uint16_t* src = zero;
      if (m < npieces && ir >= 0 && ir < a.H)
        src = xg + (((img * a.H + ir) * W + x) * kStripC + ch * 8);
      // as inline asm: with the builtin, the compiler waited vmcnt(0) before every residual
      // load's use in the epilogue -- draining the next tile's patch DMA (tq_mfma.h)
      glds16_asm(src, m < npieces ? patch + m * 64 : dummy);
    }
  };

  int64_t tile = t_begin + team;
  if (tile < t_end) issue_patch(tile);
  TQ_WAIT_VM(0);
  __syncthreads();  // weights, zero pixels and counters visible to every wave

  const int r32_l = lane & 31;
  const int hh_l = lane >> 5;
  const int cb = wt & 1;             // output channel block: channels 32 cb .. +31
  const int pset = wt >> 1;          // pixel blocks pset, pset + 2, ...
  const int co_l = 32 * cb + r32_l;  // this lane's output channel (epilogue)
  const int nblk = kStripTR * W / 32;
  const int nb = (nblk - pset + 1) / 2;  // this wave's blocks

  StripEpi ep;
  if (a.ch_scale) {
    ep.sc = a.ch_scale[co_l];
    ep.sh = a.ch_shift[co_l];
  } else {
    ep.sc = a.scale;
    ep.sh = a.bias ? (double)a.bias[co_l] : 0.0;
  }
  ep.npeel_a = a.codes_a ? relu_peels(a.maxv_a, a.k_a) : 0;
  ep.npeel_b = a.codes_b ? relu_peels(a.maxv_b, a.k_b) : 0;
  ep.fast_a = a.relu && a.inv_a > 0.0 && a.inv_a <= 1.0e308;
  ep.fast_b = a.relu && a.inv_b > 0.0 && a.inv_b <= 1.0e308;

  // this lane's weight row (B fragments) and its swizzle key ((32 cb + r32) >> 1) & 7
  const u32x4* wrow_ptr = wl + co_l * kStripKU;
  const int wkey = (r32_l >> 1) & 7;

  uint32_t sync_target = 0;
  for (; tile < t_end; tile += 2) {
    const int64_t img = tile / rb_per_img;
    const int r0 = (int)(tile - img * rb_per_img) * kStripTR;
    const int rows = a.Ho - r0 < kStripTR ? a.Ho - r0 : kStripTR;  // valid output rows
    const int64_t pix0 = ((int64_t)img * a.Ho + r0) * a.Wo;         // first output pixel

    // patch landed (this wave's DMA retired; the team's after the sync)
    TQ_WAIT_VM(0);
    sync_target += 4;
    team_sync(ctr, sync_target);
    asm volatile("" ::: "memory");  // patch reads stay behind the team sync
    // every wave of the team is done with the patch: refill it with the team's next tile
    auto refill = [&]() {
      sync_target += 4;
      team_sync(ctr, sync_target);
      asm volatile("" ::: "memory");  // every patch read of the team precedes the refill
      if (TQ_ABLATE != 14 && tile + 2 < t_end) issue_patch(tile + 2);
    };
#if TQ_ABLATE == 12
    refill();
    continue;  // timing only
#endif
    const int nv = rows * W;
    // opaque per-tile copies of the lane coordinates: what derives from them is recomputed
    // per tile instead of hoisted out of the tile loop into ~100 extra registers
    int r32 = r32_l, hh = hh_l;
    asm volatile("" : "+v"(r32), "+v"(hh));
    const int co = 32 * cb + r32;
    switch (nb) {  // wave-uniform
      case 4: strip_tile<4, RES, OUT, CB, LUT>(a, patch, wrow_ptr, wkey, W, ZP, pset, r32, hh, co,
                                          pix0, nv, ep, refill, lut_a, lut_b); break;
      case 3: strip_tile<3, RES, OUT, CB, LUT>(a, patch, wrow_ptr, wkey, W, ZP, pset, r32, hh, co,
                                          pix0, nv, ep, refill, lut_a, lut_b); break;
      case 2: strip_tile<2, RES, OUT, CB, LUT>(a, patch, wrow_ptr, wkey, W, ZP, pset, r32, hh, co,
                                          pix0, nv, ep, refill, lut_a, lut_b); break;
      case 1: strip_tile<1, RES, OUT, CB, LUT>(a, patch, wrow_ptr, wkey, W, ZP, pset, r32, hh, co,
                                          pix0, nv, ep, refill, lut_a, lut_b); break;
      default: refill(); break;
    }
  }
}

}  // namespace


// TQ_STRIP_RES=1 admits residual convs (A/B, tools only)
static bool strip_res_ok() {
  static const char* env = getenv("TQ_STRIP_RES");
  return env && atoi(env) == 1;
}

bool conv_strip_eligible(const ConvArgs& a, int out_nhwc) {
  return out_nhwc && a.Cp == kStripC && a.Cout == kStripC && a.KH == 3 && a.KW == 3 &&
         a.sh == 1 && a.sw == 1 && a.ph == 1 && a.pw == 1 && a.dh == 1 && a.dw == 1 &&
         a.Ho == a.H && a.Wo == a.W && a.W % 8 == 0 && a.W <= kStripMaxW &&
         a.Kp == kStripTaps * kStripC && a.kc_steps == 0 &&
         strip_lds_bytes(a.W) <= 160 * 1024 && a.Cout <= 64 &&
         (a.codes_a == nullptr || a.cp_a == kStripC) && a.codes_b == nullptr &&
         // with a residual the lane-per-channel epilogue (one dword load + store per element)
         // measured slower than the direct engine's 4-channel vectors (218.7 vs 235.8 us,
         // profiles/r02_strip.md): block conv1s only
         (a.residual == nullptr || strip_res_ok()) && a.ds_x == nullptr;
}

template <bool RES, bool OUT, bool CB, bool LUT>
hipError_t launch_strip_lut(const ConvArgs& b, int64_t grid, int64_t bytes, int64_t ntiles,
                            hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv2d_tp_strip_kernel<RES, OUT, CB, LUT>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  conv2d_tp_strip_kernel<RES, OUT, CB, LUT><<<dim3((unsigned)grid), kStripThreads,
                                               (size_t)bytes, stream>>>(b, ntiles);
  return hipGetLastError();
}

template <bool RES, bool OUT, bool CB>
hipError_t launch_strip_mode(const ConvArgs& a, hipStream_t stream) {
  const int64_t ntiles = (int64_t)a.N * ((a.Ho + kStripTR - 1) / kStripTR);
  int64_t grid = device_cus();
  if (grid > ntiles) grid = ntiles;
  ConvArgs b = a;
  int64_t bytes = strip_lds_bytes(a.W) + conv_lut_bytes(b);
  if (bytes > 160 * 1024) {  // no room for the code tables: the computed fast path
    b.lut_a = b.lut_b = 0;
    bytes = strip_lds_bytes(a.W);
  }
  // the fused executor's form (ReLU, table codes): the LUT-only epilogue (TQ_EPI_FAST=0: the
  // generic one)
  const char* env = getenv("TQ_EPI_FAST");
  const bool lut = !(env && atoi(env) == 0) && b.relu == 1 && b.codes_a != nullptr &&
                   b.lut_a > 0 && (b.codes_b == nullptr || b.lut_b > 0);
  return lut ? launch_strip_lut<RES, OUT, CB, true>(b, grid, bytes, ntiles, stream)
             : launch_strip_lut<RES, OUT, CB, false>(b, grid, bytes, ntiles, stream);
}

hipError_t strip_sync_faults(uint32_t* count) {
  uint32_t zero = 0;
  hipError_t e = hipMemcpyFromSymbol(count, HIP_SYMBOL(g_strip_sync_faults), sizeof(uint32_t));
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_strip_sync_faults), &zero, sizeof(uint32_t));
}

hipError_t launch_conv2d_strip(const ConvArgs& a, hipStream_t stream) {
  // no residual and no second code target (conv_strip_eligible); the RES instantiations
  // stay compilable for A/B work but are not launched
  if (a.residual)
    return a.out ? launch_strip_mode<true, true, false>(a, stream)
                 : launch_strip_mode<true, false, false>(a, stream);
  return a.out ? launch_strip_mode<false, true, false>(a, stream)
               : launch_strip_mode<false, false, false>(a, stream);
}

}  // namespace tq
