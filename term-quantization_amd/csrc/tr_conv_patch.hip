// Term-pair Conv2d on the matrix cores, input-patch engine (stride-1 convs with KH*KW >= 2
// and Cp % 64 == 0: every 3x3 conv of ResNet-18 but layer2/3/4.0.conv1).
//
// Same arithmetic and exactness argument as tr_conv_mfma.hip (fp16 term-sum codes,
// v_mfma_f32_32x32x16_f16, fp32 windows of kc_steps K-steps flushed into int32 sums), but
// the activation operand is not re-gathered per filter tap.  A tile is 256 consecutive
// output pixels (raster order, may span output rows and images); the input rows those
// pixels need -- one contiguous run of NHWC pixels -- are staged once per 64-channel chunk
// as an LDS "patch", and the KH*KW taps of that chunk read their B fragments straight out
// of it (pixel (oy, ox) at tap (r, q) = patch pixel (oy + r*dh, ox + q*dw) relative to the
// patch origin; taps that fall into the zero padding read a zero row).  Activation bytes
// per tile drop from KH*KW * 256 rows to ~(rows spanned + KH - 1) * W rows per chunk.
//
// K order: chunk-major, tap-minor: step (c, t) multiplies weight codes
// w[m][t*Cp + 64c .. +64] by the patch of chunk c shifted by tap t.  The weight K-step
// images stream through a 3-5 deep LDS ring; the patch of chunk c+1 is issued at the first
// tap of chunk c into the other patch buffer.  All staging is global_load_lds_dwordx4
// (lane-linear LDS image, bank swizzle on the source address), retired by counted vmcnt +
// raw s_barrier.  Layout of the dynamic LDS (16-byte units):
//   [NR][BM][8] weight ring | [NPB][PXS + 1][8] patches (row PXS of each = zeros)
// and the epilogue reuses it to transpose each wave's int32 tile (as the gather engine).
#include <stdlib.h>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

#ifndef TQ_ABLATE
#define TQ_ABLATE 0  // timing-only ablation builds (tools/ab/ablate.sh); 0 = the product kernel
#endif
#ifndef TQ_PATCH_SCHED
#define TQ_PATCH_SCHED 1  // 0: the round-2 schedule (timing variants only, tools/ab/variant.sh)
#endif

namespace tq {

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int kPatchBN = 256;       // output pixels per tile
constexpr int kPatchThreads = 512;  // 8 waves: 2 along Cout x 4 along pixels

struct PatchRows {
  int64_t base;  // first flattened input row (img * H + iy) of the patch
  int rows;
};

// Input rows needed by the tile of output pixels [n0, n0 + 256): the span from the first
// tap row of its first output row to the last tap row of its last output row (clipped to
// the images they belong to; rows of images in between are included whole).
__host__ __device__ inline PatchRows patch_rows(const ConvArgs& a, int64_t n0) {
  const int64_t n1 = (n0 + kPatchBN < a.P ? n0 + kPatchBN : a.P) - 1;
  const int64_t fr0 = n0 / a.Wo, fr1 = n1 / a.Wo;
  const int64_t img0 = fr0 / a.Ho, img1 = fr1 / a.Ho;
  const int oy0 = (int)(fr0 - img0 * a.Ho), oy1 = (int)(fr1 - img1 * a.Ho);
  int r0 = oy0 * a.sh - a.ph;
  int r1 = oy1 * a.sh - a.ph + (a.KH - 1) * a.dh;
  r0 = r0 < 0 ? 0 : (r0 > a.H - 1 ? a.H - 1 : r0);
  r1 = r1 < 0 ? 0 : (r1 > a.H - 1 ? a.H - 1 : r1);
  PatchRows pr;
  pr.base = img0 * a.H + r0;
  pr.rows = (int)(img1 * a.H + r1 - pr.base + 1);
  return pr;
}

// SK = false: one workgroup per (Cout tile, pixel tile), grid = tiles.
// SK = true (stream-K): a grid of G resident-sized workgroups; the tiles' K-steps, laid end to
// end (tile-major, chunk-major, tap-minor), are cut into G equal ranges, so every CU gets the
// same number of K-steps however the tile count falls against the CU count (ResNet-18
// layer3/4: 392 and 196 tiles on 256 CUs would run 1.53 / 0.77 rounds).  A tile split over
// several ranges ("pieces") is finished by the piece that arrives last: every partial piece
// stores its int32 sums in a slab (ws), then bumps the tile's counter; the piece that sees
// count == pieces - 1 adds the other pieces' slabs to its own sums (integer adds: the result
// is bit-identical to SK = false) and runs the epilogue.  No piece ever waits for another.
// Slab and counter accesses are agent-scope atomics (sc1 stores/loads that bypass the
// non-coherent per-XCD L2), ordered by vmcnt(0) before the counter RMW.
template <int MB, int NR, bool SK>
__global__ __launch_bounds__(kPatchThreads, TQ_PATCH_SCHED ? (MB == 1 ? 2 : 1) : (MB == 1 ? 4 : 2))
void conv2d_tp_patch_kernel(
    ConvArgs a) {
  constexpr int BM = 64 * MB;                 // 2 waves x 32*MB Cout rows
  constexpr int AI = MB;                      // weight wave-instructions per wave and step
  extern __shared__ __attribute__((aligned(16))) u32x4 lds[];
  uint16_t *lut_a_, *lut_b_;
  const int PXS = a.patch_px;                 // patch slot pixels (multiple of 64)
  const int PI = PXS / 64;                    // patch wave-instructions per wave and chunk
  const int NPB = a.patch_bufs;
  u32x4* ring = lds;
  u32x4* patch = lds + NR * BM * 8;
  // epilogue code tables behind both the K-loop images and the epilogue transpose
  {
    const int main_units = NR * BM * 8 + NPB * (PXS + 1) * 8;
    const int epi_units = 8 * 64 * 8 * MB;
    uint16_t* lt = reinterpret_cast<uint16_t*>(lds + (main_units > epi_units ? main_units
                                                                             : epi_units));
    conv_luts(a, lt, lut_a_, lut_b_);  // read only after the epilogue's barrier
  }

  const int mt = (a.Cout + BM - 1) / BM;
  const int64_t ntn = (a.P + kPatchBN - 1) / kPatchBN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = (wave >> 2) * 32 * MB;
  const int wn = (wave & 3) * 64;
  const int lrow = lane >> 3;
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page) + lane * 8;
  const int nch = a.Cp / kKStep;
  const int ntap = a.KH * a.KW;
#if TQ_ABLATE == 6
  const int nsteps = 0;  // timing only: setup + epilogue
#else
  const int nsteps = nch * ntap;
#endif
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;

  // K-steps [kb, ke) of `tile`; finish: run the epilogue with the tile's full sums.
  // sk_g: this workgroup's logical stream-K index (SK only).
  auto piece = [&](int64_t tile, int kb, int ke, int64_t sk_g) {
    const int m0 = (int)(a.m_slow ? tile / ntn : tile % mt) * BM;
    const int64_t n0 = (a.m_slow ? tile % ntn : tile / mt) * kPatchBN;
    const PatchRows pr = patch_rows(a, n0);
    const int PX = pr.rows * a.W;  // host guarantees PX <= PXS

    // zero row of every patch buffer
    if (threadIdx.x < 8 * NPB)
      patch[(threadIdx.x >> 3) * (PXS + 1) * 8 + PXS * 8 + (threadIdx.x & 7)] = (u32x4)0u;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): visible after the first barrier

    // weight rows: this lane's source chunk (swizzled), advanced per step by t*Cp + 64c
    const uint16_t* arow[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int r = (wave * AI + i) * 8 + lrow;
      arow[i] = wg + (int64_t)(m0 + r) * a.Kp + ((lane & 7) ^ ((r >> 1) & 7)) * 8;
    }
    // B fragment pixels: patch index of tap (0, 0) and the mask of in-bounds taps
    int pix[2];
    uint64_t tmask[2];
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) {
      const int64_t n = n0 + wn + 32 * bn + r32;
      pix[bn] = 0;
      tmask[bn] = 0;
      if (n < a.P) {
        const int64_t img = n / HoWo;
        const int64_t rem = n - img * HoWo;
        const int oy = (int)(rem / a.Wo);
        const int ox = (int)(rem - (int64_t)oy * a.Wo);
        const int iy0 = oy * a.sh - a.ph;
        const int ix0 = ox * a.sw - a.pw;
        pix[bn] = (int)((img * a.H + iy0 - pr.base) * a.W + ix0);
        for (int r = 0; r < a.KH; ++r) {
          const int iy = iy0 + r * a.dh;
          if (iy < 0 || iy >= a.H) continue;
          for (int q = 0; q < a.KW; ++q) {
            const int ix = ix0 + q * a.dw;
            if (ix >= 0 && ix < a.W) tmask[bn] |= 1ull << (r * a.KW + q);
          }
        }
      }
    }

    auto issue_patch = [&](int c, int buf) {
      u32x4* dst = patch + buf * (PXS + 1) * 8;
      for (int j = 0; j < PI; ++j) {
        const int pp = (wave * PI + j) * 8 + lrow;
        const uint16_t* src = zero;
        if (pp < PX)
          src = xg + ((pr.base * a.W + pp) * a.Cp + c * kKStep +
                      ((lane & 7) ^ ((pp >> 1) & 7)) * 8);
#if TQ_ABLATE != 3
        glds16(src, dst + (wave * PI + j) * 64);
#endif
      }
    };
    auto issue_w = [&](int st, int slot) {
      const int c = st / ntap;
      const int t = st - c * ntap;
      const int64_t off = (int64_t)t * a.Cp + c * kKStep;
#pragma unroll
      for (int i = 0; i < AI; ++i) {
#if TQ_ABLATE != 3
        glds16(arow[i] + off, ring + slot * BM * 8 + (wave * AI + i) * 64);
#endif
      }
    };

    MfmaAcc<MB> acc;
    acc_zero(acc);
    // Exactness windows.  This kernel walks K chunk-major (taps inner); the host bounds every
    // window of kc_chunk CONSECUTIVE taps of one 64-code chunk (ConvArgs.kc_chunk), and the
    // fp32 sums are also flushed at the end of every chunk and of the piece, so each fp32
    // window lies inside one bounded window.  kc_chunk == 0 with kc_steps > 0 means a whole
    // chunk fits one window but the full K does not: chunk-end flushes only.
    const bool flushing = a.kc_chunk > 0 || a.kc_steps > 0;
    const int kc_steps = a.kc_chunk > 0 ? a.kc_chunk : (1 << 30);
    int since_flush = 0;

    // Counted retirement: `issued` counts this wave's LDS-DMA instructions; mark[j] is its
    // value right after K-step s+j's weight image was issued, so waiting for vmcnt <=
    // issued - mark[0] retires step s's image and, issued before it, the patch of its chunk.
    // A piece that starts inside chunk c0 also stages chunk c0 + 1's patch up front (the
    // loop stages chunk c + 1 at tap 0 of chunk c, which such a piece never runs for c0).
    const int c0 = kb / ntap, t0 = kb - c0 * ntap;
    const int c_last = (ke - 1) / ntap;
    int issued = 0;
    int mark[NR - 1];
    if (kb < ke) {
      issue_patch(c0, c0 % NPB);
      issued += PI;
      if (t0 > 0 && c0 + 1 <= c_last) {
        issue_patch(c0 + 1, (c0 + 1) % NPB);
        issued += PI;
      }
    }
#pragma unroll
    for (int j = 0; j < NR - 1; ++j) {
      if (kb + j < ke) {
        issue_w(kb + j, j);
        issued += AI;
      }
      mark[j] = issued;
    }
    int c = c0, t = t0, kr = t0 / a.KW, kq = t0 - (t0 / a.KW) * a.KW;
    for (int s = kb; s < ke; ++s) {
      wait_vm_dyn(issued - mark[0]);
#if TQ_ABLATE != 4
      __builtin_amdgcn_s_barrier();
#endif
      if (t == 0 && c + 1 <= c_last) {
        issue_patch(c + 1, (c + 1) % NPB);
        issued += PI;
      }
      if (s + NR - 1 < ke) {
        issue_w(s + NR - 1, (s - kb + NR - 1) % NR);
        issued += AI;
      }
#pragma unroll
      for (int j = 0; j < NR - 2; ++j) mark[j] = mark[j + 1];
      mark[NR - 2] = issued;

      const u32x4* aimg = ring + ((s - kb) % NR) * BM * 8;
      const u32x4* pimg = patch + (c % NPB) * (PXS + 1) * 8;
      const int toff = kr * a.dh * a.W + kq * a.dw;
      int prow[2], psw[2];
#pragma unroll
      for (int bn = 0; bn < 2; ++bn) {
        const int idx = ((tmask[bn] >> t) & 1ull) ? pix[bn] + toff : PXS;
        prow[bn] = idx * 8;
        psw[bn] = (idx >> 1) & 7;
      }
      // all fragments of the step first (the reads overlap the previous step's MFMAs)
      half8 af[4][MB], bf[4][2];
#if TQ_ABLATE == 1 || TQ_ABLATE == 5  // timing only: no fragment reads
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int b = 0; b < MB; ++b) af[k][b] = (half8)(_Float16)(s + k + b);
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) bf[k][bn] = (half8)(_Float16)(prow[bn] + psw[bn] + k);
      }
#else
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ck = 2 * k + hh;
#pragma unroll
        for (int b = 0; b < MB; ++b)
          af[k][b] = __builtin_bit_cast(half8, aimg[swz(wm + 32 * b + r32, ck)]);
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
          bf[k][bn] = __builtin_bit_cast(half8, pimg[prow[bn] + (ck ^ psw[bn])]);
      }
#endif
#if TQ_ABLATE == 2 || TQ_ABLATE == 5  // timing only: no MFMA (fragments kept live)
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int bm = 0; bm < MB; ++bm)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            asm volatile("" ::"v"(af[k][bm]), "v"(bf[k][bn]));
#else
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int bm = 0; bm < MB; ++bm)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc.f[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[k][bm], bf[k][bn],
                                                                   acc.f[bm][bn], 0, 0, 0);
#if TQ_ABLATE == 0 && TQ_PATCH_SCHED
      // every fragment read of the step is issued before its first MFMA (the scheduler
      // otherwise recycles four fragment registers: read 4, wait, 4 MFMAs, ...)
      // (three K-substeps' reads, then the first substep's MFMAs under the last reads: the
      // 4-bit lgkmcnt counts at most 15 reads in flight)
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * (MB + 2), 0);  // DS reads, k = 0..2
      __builtin_amdgcn_sched_group_barrier(0x008, MB * 2, 0);        // MFMAs, k = 0
      __builtin_amdgcn_sched_group_barrier(0x100, MB + 2, 0);        // DS reads, k = 3
      __builtin_amdgcn_sched_group_barrier(0x008, 3 * MB * 2, 0);    // MFMAs, k = 1..3
#endif
#endif
      if (++since_flush == kc_steps || (flushing && t + 1 == ntap)) {
        acc_flush(acc);
        since_flush = 0;
      }
      if (++t == ntap) {
        t = 0;
        kr = 0;
        kq = 0;
        ++c;
      } else if (++kq == a.KW) {
        kq = 0;
        ++kr;
      }
    }
    acc_flush(acc);

    if constexpr (SK) {
      if (kb != 0 || ke != nsteps) {  // a partial piece: slab, count, maybe finish
        const int64_t T = (ntn * mt) * (int64_t)nsteps;
        const int64_t G = gridDim.x;
        auto wg_of = [&](int64_t st) { return ((st + 1) * G + T - 1) / T - 1; };
        // slabs [G][2][8 waves][kSlab]: slot 0 for the piece a workgroup starts with, 1 for
        // the piece it ends with (a range is at most one tile's tail + one tile's head)
        constexpr int kSlab = 32 * MB * 64;  // int32 per wave
        auto slab = [&](int64_t g, int64_t tile_start) {  // slab of g's piece of the tile
          const int64_t gb = g * T / G;
          const int which = gb >= tile_start ? 0 : 1;
          return a.ws + ((g * 2 + which) * 8 + wave) * kSlab;
        };
        const int64_t ts = tile * nsteps;
        const int64_t g_first = wg_of(ts), g_last = wg_of(ts + nsteps - 1);
        int* cnt = a.ws + G * 2 * 8 * kSlab;  // [tiles] arrival counters
        int* mine = slab(sk_g, ts);
        // slab image [MB*2*4 quads][64 lanes][4]: 16-byte sc1 (write-through) stores
#pragma unroll
        for (int bm = 0; bm < MB; ++bm)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              int* dst = mine + (((bm * 2 + bn) * 4 + q) * 64 + lane) * 4;
              const i32x4 v = {acc.i[bm][bn][4 * q], acc.i[bm][bn][4 * q + 1],
                               acc.i[bm][bn][4 * q + 2], acc.i[bm][bn][4 * q + 3]};
              asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(v)
                           : "memory");
            }
        TQ_WAIT_VM(0);  // this wave's slab stores are complete
        __syncthreads();
        // the counter value this piece saw, broadcast through the (now idle) weight ring:
        // the dynamic LDS is all in use during the K loop, so no static variable is added
        int* sk_old_p = reinterpret_cast<int*>(ring);
        if (threadIdx.x == 0)
          *sk_old_p = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int sk_old = *sk_old_p;
        // pieces of this tile: the non-empty ranges among g_first..g_last (ranges are empty
        // only when there are fewer K-steps than workgroups)
        int npieces = 0;
        for (int64_t g = g_first; g <= g_last; ++g) npieces += (g + 1) * T / G > g * T / G;
        if (sk_old != npieces - 1) return false;  // not the last piece
        for (int64_t g = g_first; g <= g_last; ++g) {
          if (g == sk_g || (g + 1) * T / G == g * T / G) continue;
          const int* other = slab(g, ts);
          // 16-byte sc1 loads (coherent across XCDs), all issued before one wait
          i32x4 v[MB * 8];
#pragma unroll
          for (int j = 0; j < MB * 8; ++j)
            asm volatile("global_load_dwordx4 %0, %1, off sc1"
                         : "=v"(v[j])
                         : "v"(other + (j * 64 + lane) * 4)
                         : "memory");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
          for (int j = 0; j < MB * 8; ++j) {
            asm volatile("" : "+v"(v[j]));  // keeps every use after the wait
            const int bm = j / 8, bn = (j / 4) % 2, q = j % 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) acc.i[bm][bn][4 * q + e] += v[j][e];
          }
        }
      }
    }

    // Epilogue: transpose each wave's (32*MB Cout) x (64 pixel) int32 tile through LDS so
    // that lanes run along channels: [pixel][8*MB slots of 4 channels], slot swizzled.
    __syncthreads();
    constexpr int SLOTS = 8 * MB;
    u32x4* tt = lds + wave * 64 * SLOTS;
    auto phys = [&](int px, int slot) {
      return px * SLOTS + (slot ^ (MB == 2 ? (px & 15) : ((px >> 1) & 7)));
    };
#pragma unroll
    for (int bm = 0; bm < MB; ++bm)
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          u32x4 v;
          v.x = (uint32_t)acc.i[bm][bn][4 * q];
          v.y = (uint32_t)acc.i[bm][bn][4 * q + 1];
          v.z = (uint32_t)acc.i[bm][bn][4 * q + 2];
          v.w = (uint32_t)acc.i[bm][bn][4 * q + 3];
          tt[phys(32 * bn + r32, 8 * bm + 2 * q + hh)] = v;
        }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    const bool vec = (a.Cout & 3) == 0;
    const int slot = lane % SLOTS;
    const int co = m0 + wm + 4 * slot;
    if (co < a.Cout) {
      coef_t sc[4], sh[4];
      load_coef(a, co, sc, sh);
      constexpr int PXI = 64 / SLOTS;  // pixels per wave-instruction
#pragma unroll 4
      for (int it = 0; it < SLOTS; ++it) {
        const int px = it * PXI + lane / SLOTS;
        const int64_t p = n0 + wn + px;
        if (p >= a.P) continue;
        const u32x4 v = tt[phys(px, slot)];
        const int acc4[4] = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
#if TQ_ABLATE == 7  // timing only: no epilogue stores (sums kept live)
        if (acc4[0] == 0x7fffffff && a.out) a.out[p] = (float)(sc[0] + sh[0]);
#else
        emit4_nhwc(a, p, co, acc4, sc, sh, vec, lut_a_, lut_b_);
#endif
      }
    }
    return true;
  };

  if constexpr (!SK) {
    piece(xcd_remap(blockIdx.x, gridDim.x), 0, nsteps, 0);
  } else {
    // logical index: consecutive ranges (which share tiles, slabs and weights) on one XCD
    const int64_t g = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t G = gridDim.x;
    const int64_t T = (ntn * mt) * (int64_t)nsteps;
    int64_t cur = g * T / G;
    const int64_t end = (g + 1) * T / G;
    while (cur < end) {
      const int64_t tile = cur / nsteps;
      const int64_t ts = tile * nsteps;
      const int kb = (int)(cur - ts);
      const int ke = (int)(end - ts < nsteps ? end - ts : nsteps);
      piece(tile, kb, ke, g);
      cur = ts + ke;
      __syncthreads();  // LDS (epilogue tile, patches, ring) is reused by the next piece
    }
  }
}

// Largest patch (pixels) over all tiles: the tile pattern repeats every
// HoWo / gcd(256, HoWo) tiles, so one period (<= HoWo tiles) is enough.
int64_t max_patch_px(const ConvArgs& a) {
  const int64_t howo = (int64_t)a.Ho * a.Wo;
  int64_t g = kPatchBN, r = howo;
  while (r) {
    const int64_t t = g % r;
    g = r;
    r = t;
  }
  const int64_t tiles = (a.P + kPatchBN - 1) / kPatchBN;
  int64_t period = howo / g;
  if (period > tiles) period = tiles;
  if (period > 4096) return -1;
  int64_t best = 0;
  for (int64_t j = 0; j < period; ++j) {
    const PatchRows pr = patch_rows(a, j * kPatchBN);
    if (pr.rows > best) best = pr.rows;
  }
  // the last (partial) tile is a prefix of a full one: never larger
  return best * a.W;
}

constexpr int kLdsBytes = 160 * 1024;

// Dynamic LDS of a (MB, NR) launch, or -1 if it does not fit.
int64_t patch_lds_bytes(int mb, int nr, int64_t px_slot, int bufs) {
  int64_t bytes = ((int64_t)nr * 64 * mb * 8 + (int64_t)bufs * (px_slot + 1) * 8) * 16;
  const int64_t epi = (int64_t)8 * 64 * 8 * mb * 16;  // epilogue transpose
  if (bytes < epi) bytes = epi;
  return bytes <= kLdsBytes ? bytes : -1;
}

template <int MB, int NR, bool SK>
hipError_t launch_patch_nr(const ConvArgs& a, int64_t bytes, int64_t grid, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv2d_tp_patch_kernel<MB, NR, SK>),
        hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  conv2d_tp_patch_kernel<MB, NR, SK>
      <<<dim3((unsigned)grid), kPatchThreads, (size_t)bytes, stream>>>(a);
  return hipGetLastError();
}

// Stream-K workspace: slabs [G][2][8][32 MB 64] int32 (G = one workgroup per CU, MB <= 2)
// then one arrival counter per tile.
int64_t patch_sk_slab_bytes(int mb) { return (int64_t)device_cus() * 2 * 8 * 32 * mb * 64 * 4; }

// Stream-K on request only (ConvArgs.splits == -1, or TQ_PATCH_SK=1 for A/B; needs the
// workspace and a shape where one workgroup fills a CU).  Measured on ResNet-18 batch 256
// (tools/layer_times.py): although the data-parallel grids leave 23 % of the CU-time idle
// on layer3/4 (392 and 196 tiles on 256 CUs), stream-K ran those convs 9-15 % SLOWER --
// the per-K-step time grows ~30 % once all 256 CUs run MFMA loops, and each range pays
// 2-3 pipeline fills plus the slab fixup -- so the default stays data-parallel.
template <int MB, int NR>
hipError_t launch_patch_sched(ConvArgs a, int64_t bytes, hipStream_t stream) {
  constexpr int BM = 64 * MB;
  const int64_t tiles = ((a.P + kPatchBN - 1) / kPatchBN) * ((a.Cout + BM - 1) / BM);
  const int64_t G = device_cus();
  const int64_t need = patch_sk_slab_bytes(MB) + tiles * 4;
  static const char* env = getenv("TQ_PATCH_SK");
  bool sk = false;
  if (a.ws && a.ws_bytes >= need && 2 * bytes > kLdsBytes) {
    sk = a.splits == -1 || (a.splits == 0 && env && atoi(env) != 0);
  }
  if (!sk) return launch_patch_nr<MB, NR, false>(a, bytes, tiles, stream);
  int* cnt = a.ws + patch_sk_slab_bytes(MB) / 4;
  hipError_t e = hipMemsetAsync(cnt, 0, (size_t)tiles * 4, stream);
  if (e != hipSuccess) return e;
  return launch_patch_nr<MB, NR, true>(a, bytes, G, stream);
}

// Deepest weight ring (5, 4 or 3 K-step images) that fits beside the patch buffers and that
// the chunk's taps cover (the patch of chunk c+1 must be issued before the weight image of
// its first step: ntap >= NR - 1).
template <int MB>
hipError_t launch_patch_mb(ConvArgs a, int64_t px, hipStream_t stream) {
  const int nch = a.Cp / kKStep;
  const int ntap = a.KH * a.KW;
  a.patch_px = (int)((px + 63) / 64 * 64);
  a.patch_bufs = nch > 1 ? 2 : 1;
  static const char* env = getenv("TQ_PATCH_RING");  // A/B override (tools only)
  const int want = env ? atoi(env) : 5;
  for (int nr = want < 5 ? want : 5; nr >= 3; --nr) {
    int64_t bytes = patch_lds_bytes(MB, nr, a.patch_px, a.patch_bufs);
    if (bytes < 0 || ntap < nr - 1) continue;
    if (bytes + conv_lut_bytes(a) <= kLdsBytes) {
      bytes += conv_lut_bytes(a);  // the epilogue code tables
    } else {
      a.lut_a = a.lut_b = 0;
    }
    if (nr == 5) return launch_patch_sched<MB, 5>(a, bytes, stream);
    if (nr == 4) return launch_patch_sched<MB, 4>(a, bytes, stream);
    return launch_patch_sched<MB, 3>(a, bytes, stream);
  }
  return hipErrorInvalidConfiguration;
}

}  // namespace

bool conv_patch_eligible(const ConvArgs& a, int out_nhwc) {
  if (!out_nhwc || a.Cp % kKStep != 0 || a.sh != 1 || a.sw != 1) return false;
  const int ntap = a.KH * a.KW;
  if (ntap < 2 || ntap > 64 || a.Kp != ntap * a.Cp) return false;
  const int64_t px = max_patch_px(a);
  if (px < 0) return false;
  const int64_t slot = (px + 63) / 64 * 64;
  return ntap >= 2 && patch_lds_bytes(2, 3, slot, a.Cp > kKStep ? 2 : 1) > 0;
}

// mb: 1 = 64-row Cout tiles, 2 = 128-row Cout tiles.
int64_t patch_streamk_ws_bytes(int64_t p, int64_t cout) {
  const int64_t tiles = ((p + kPatchBN - 1) / kPatchBN) * ((cout + 63) / 64);
  return patch_sk_slab_bytes(2) + tiles * 4;
}

hipError_t launch_conv2d_patch(const ConvArgs& a, int mb, hipStream_t stream) {
  const int64_t px = max_patch_px(a);
  if (px < 0) return hipErrorInvalidConfiguration;
  return mb == 1 ? launch_patch_mb<1>(a, px, stream) : launch_patch_mb<2>(a, px, stream);
}

}  // namespace tq
