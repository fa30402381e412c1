// Term-pair Conv2d on the matrix cores, tap-ring engine: 3x3 stride-1 convs with Cp % 64 == 0
// and Cout >= 128 (ResNet-18 layer2/3/4 3x3 convs), persistent workgroups that stream K-steps
// across tiles without refilling the pipeline.
//
// Same exact arithmetic as the other MFMA engines (tr_conv_mfma.hip): fp16 term-sum codes,
// v_mfma_f32_32x32x16_f16, fp32 partial sums that stay exact integers inside host-bounded
// windows, moved into int32 sums at every window end, one fp64 fold in the shared epilogue.
//
// Why another engine.  The input-patch engine (tr_conv_patch.hip) has the right data flow --
// activations staged once per 64-channel chunk as an LDS patch that all nine taps read, weight
// K-steps through an LDS-DMA ring -- but its K loop spends ~3500 cycles per K-step against
// 1024 of matrix-core work (r03m counters: 164 VALU, 121 SALU and 26 branches per wave and
// step: a runtime division per weight issue, a binary search for every counted wait, dynamic
// ring and patch indices), reads each step's fragments only after that step's barrier, and
// pays a pipeline fill for every tile.  Here:
//   * the nine taps of a chunk are unrolled and the ring has 3 slots, so every ring slot, LDS
//     offset and vmcnt count is a compile-time constant (9 % 3 == 0: step (c, t) uses slot t%3);
//   * the barrier at the top of step s retires step s+1's weight image (issued two steps
//     earlier), so each wave reads step s+1's first fragments during step s's last MFMAs --
//     fragment reads run one 16-code substep ahead of the MFMAs, across step boundaries;
//   * the patch rows use a 144-byte pixel pitch (128 B of codes + 16 B pad): the 16 lanes of a
//     ds_read_b128 group read 16 distinct pixels whose 16-byte chunks land in 16 distinct bank
//     quads (pitch 9 units, odd), with no XOR -- a step's four substep reads of one B block are
//     one address + immediate offsets 0/32/64/96;
//   * tiles are R whole output rows (R * Wo <= 256 pixels), so a patch is at most R + 2 input
//     rows, and the next chunk's patch -- the next tile's first chunk at a tile's end -- is
//     issued one 1 KB piece per wave and step at taps 0..PI-1 of the current chunk;
//   * workgroups are persistent (one per CU, XCD-aware tile order): the weight ring and the
//     patch stream run straight through tile boundaries; the epilogue works from the MFMA
//     register layout (no LDS transpose), so it never waits for the next tile's staging.
//
//   workgroup = 8 waves (2 along Cout x 4 along pixels), tile 128 (Cout) x 256 (pixel columns,
//               R * Wo of them real); wave tile 64 x 64 = 2 x 2 blocks of 32 x 32
//   K order   = chunk-major, tap-minor (as the patch engine: kc_chunk windows apply)
//   LDS       = [3][128 rows][128 B] weight ring (rows swizzled chunk ^= (row >> 1) & 7 on the
//               source side) | [2][8 * PI KB] patches (144 B per pixel) | one zero pixel |
//               [Cout][2] fp64 epilogue coefficients | epilogue code tables
#include <stdlib.h>

#include <mutex>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

#ifndef RING_AB
#define RING_AB 0  // timing-only ablation builds (tools/ab/variant.sh); 0 = the product kernel
#endif
#ifndef RING_DMA_LATE
#define RING_DMA_LATE 0  // 1: a step's DMA issued after its first substep (A/B builds)
#endif

#ifndef RING_TRACE
#define RING_TRACE 0  // timing-only builds: per-tile phase stamps of wave 0 (tools/ring_trace.py)
#endif

namespace tq {

#if RING_TRACE
// [workgroup][tile of its stream < 8][tile start, first barrier passed, K loop done, epilogue
// issued] (s_memrealtime ticks, 100 MHz) of the last traced launch
__device__ unsigned long long g_ring_trace[1024 * 8 * 4];
#endif

namespace {

constexpr int kRingBM = 128;            // Cout rows per tile
constexpr int kRingTaps = 9;            // 3 x 3
constexpr int kRingExtra = 160 + 8192 + 2048;  // zero pixel + Cout <= 512 coefficients + tables

// Two shapes of the engine:
//   NW = 8, KS = 64: one 512-thread workgroup per CU (160 KB of LDS), tile 128 x 256, K-steps
//                    of 64 codes (one 64-channel chunk of one tap);
//   NW = 4, KS = 32: two 256-thread workgroups per CU (80 KB of LDS each), tile 128 x 128,
//                    K-steps of 32 codes: one workgroup's epilogue, barrier waits and chunk
//                    switches run beside the other's MFMAs.
// Wave tile 64 x 64 either way (2 x 2 blocks of 32 x 32).
template <int NW, int KS>
struct RingGeom {
  static constexpr int THREADS = 64 * NW;
  static constexpr int BN = 64 * (NW / 2);   // pixel columns per tile
  static constexpr int ROWB = KS * 2;        // bytes per weight row and K-step
  static constexpr int CH = ROWB / 16;       // 16-byte chunks per row (8 or 4)
  static constexpr int SH = CH == 8 ? 1 : 2; // row swizzle shift: chunk ^= (row >> SH) & (CH-1)
  static constexpr int SLOT = kRingBM * ROWB;
  static constexpr int WI = SLOT / 1024 / NW;  // weight DMA instructions per wave and step
  static constexpr int PITCH = ROWB + 16;      // patch bytes per pixel (odd number of 16 B)
  static constexpr int SUB = KS / 16;          // MFMA substeps per K-step
  static constexpr int BUDGET = NW == 8 ? 160 * 1024 : 80 * 1024;
  static constexpr int pbuf(int pi) { return NW * pi * 1024; }
  static constexpr int pxs(int pi) { return pbuf(pi) / PITCH; }
  // weight ring depth: as deep as the LDS budget allows beside two patch buffers.  The
  // barrier of step s retires step s+1's image, issued at step s+2-NR: NR-2 steps of lead.
  static constexpr int slots(int pi) {
    const int n = (BUDGET - 2 * pbuf(pi) - kRingExtra) / SLOT;
    return n > 6 ? 6 : n;
  }
  static constexpr int patch_off(int nr) { return nr * SLOT; }
  static constexpr int zero_off(int pi, int nr) { return patch_off(nr) + 2 * pbuf(pi); }
  static constexpr int coef_off(int pi, int nr) { return zero_off(pi, nr) + 160; }
};

// The rows of one tile and the input rows its patch holds.
struct RingTile {
  int64_t p0;     // first output pixel
  int m0;         // first Cout row
  int64_t base;   // first flattened input row (img * H + iy) of the patch
  int px;         // patch pixels (rows * W)
};

__host__ __device__ inline RingTile ring_tile(const ConvArgs& a, int64_t tile, int R, int mt,
                                              int m_slow, int64_t pt_count) {
  RingTile t;
  const int64_t pt = m_slow ? tile % pt_count : tile / mt;
  const int m = (int)(m_slow ? tile / pt_count : tile % mt);
  t.m0 = m * kRingBM;
  const int64_t nrows = (int64_t)a.N * a.Ho;
  const int64_t gr0 = pt * R;
  const int64_t gr1 = (gr0 + R < nrows ? gr0 + R : nrows) - 1;
  t.p0 = gr0 * a.Wo;
  const int64_t img0 = gr0 / a.Ho, img1 = gr1 / a.Ho;
  const int oy0 = (int)(gr0 - img0 * a.Ho), oy1 = (int)(gr1 - img1 * a.Ho);
  int r0 = oy0 - a.ph;
  int r1 = oy1 - a.ph + (a.KH - 1);
  r0 = r0 < 0 ? 0 : r0;
  r1 = r1 > a.H - 1 ? a.H - 1 : r1;
  t.base = img0 * a.H + r0;
  t.px = (int)((img1 * a.H + r1 - t.base + 1) * a.W);
  return t;
}

// One LDS-DMA wave-instruction (1 KB, lane-linear destination), issued as inline asm so the
// compiler's own wait counts stay exact (tq_mfma.h glds16_asm); the LDS address is uniform.
__device__ __forceinline__ void ring_dma(const void* src, uint32_t lds_byte) {
  if (RING_AB == 3) return;  // timing only: nothing staged
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(lds_byte)
               : "memory", "m0");
}

// compile-time loop: f(ic<I>) for I in [I0, N)
template <int V>
struct ic {
  static constexpr int value = V;
};
template <int I, int N, typename F>
__host__ __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(ic<I>{});
    static_for<I + 1, N>(f);
  }
}

// Stream-K tail (SK kernels).  The q full rounds of tiles (tiles [0, q G), one per workgroup
// and round) run data-parallel as in the plain kernel; the remaining tiles -- the partial last
// round, which would leave most CUs idle -- become a chunk-granular unit stream, unit =
// (tile - q G) * nch + chunk, and workgroup g takes the units [g U / G, (g + 1) U / G).  A tile
// split over workgroups is finished by whichever contributor arrives last: every contributor
// stores its int32 partial sums write-through (sc1) into its own slab, drains, and draws a
// ticket from the tile's counter (indexed by the workgroup owning the tile's first unit); the
// last one adds the other slabs (sc1 loads) to its registers and runs the epilogue.  Integer
// partial sums add exactly in any order, so the output is the one of the unsplit tile.  The
// last arriver resets the counter (zeroed once at allocation), and nothing ever waits on
// another workgroup.
struct RingSk {
  int* cnt;     // [G] tile tickets
  int* slab;    // [G][2][64 * NW * 64] int32 partial sums: slot 0 the range's first tile,
                // slot 1 its last one
  int64_t U;    // units in the split tail
  int64_t q;    // full data-parallel rounds ahead of the tail: tiles [0, q G)
};

// workgroup owning unit u: the g with floor(g U / G) <= u < floor((g + 1) U / G)
__device__ __forceinline__ int sk_owner(int64_t u, int64_t U, int64_t G) {
  return (int)(((u + 1) * G + U - 1) / U - 1);
}

__device__ __forceinline__ half8 lds_frag(uint32_t byte_addr) {
  if (RING_AB == 7) return (half8)(_Float16)(byte_addr & 7);  // timing only: no LDS reads
  return __builtin_bit_cast(
      half8, *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(
                 (uintptr_t)byte_addr));
}

// FAST: the fused ResNet executor's epilogue forms, specialised at launch (ring_epilogue_form)
// -- 1: ReLU, fp16 codes from the code tables (every code output has one); 2: ReLU and the
// fp32 output only (the last conv) -- Cout % 4 == 0, with per-pixel base pointers and
// compile-time channel offsets; other forms (0) run the shared emit4_nhwc_res.
template <int NW, int KS, int PI, bool FLUSH, int FAST, bool SK>
__global__ __launch_bounds__(64 * NW, 2) void conv2d_tp_ring_kernel(ConvArgs a, int R,
                                                                   int64_t ptc, RingSk sk) {
  using Gm = RingGeom<NW, KS>;
  constexpr int NR = Gm::slots(PI);
  constexpr int WI = Gm::WI, CH = Gm::CH, SH = Gm::SH, SUB = Gm::SUB;
  constexpr int kRingSlot = Gm::SLOT, kPitch = Gm::PITCH;
  static_assert(NR >= 3, "the LDS budget must hold three weight images");
  // the next chunk's last patch piece (tap PI-1) must be older than the weight image the
  // barrier of that chunk's last step retires (issued at tap 10-NR)
  static_assert(PI <= 10 - NR, "patch pieces must land before the chunk switch");
  extern __shared__ __attribute__((aligned(16))) u32x4 ring_lds[];
  const uint32_t lds0 =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)ring_lds;
  constexpr uint32_t kPatchOff = Gm::patch_off(NR);
  constexpr uint32_t kZeroOff = Gm::zero_off(PI, NR);
  double* coef = reinterpret_cast<double*>(reinterpret_cast<unsigned char*>(ring_lds) +
                                           Gm::coef_off(PI, NR));
  uint16_t *lut_a, *lut_b;
  conv_luts(a, reinterpret_cast<uint16_t*>(coef + 2 * a.Cout), lut_a, lut_b);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const int wm = (wave / (NW / 2)) * 64;  // this wave's Cout rows [wm, wm + 64) of the tile
  const int wn = (wave % (NW / 2)) * 64;  // and pixel columns [wn, wn + 64)
  const int mt = (a.Cout + kRingBM - 1) / kRingBM;
  const int64_t T = ptc * mt;
  const int64_t G = gridDim.x;
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x);
  const int BNv = R * a.Wo;
  const int nch = a.Cp / KS;
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const char* __restrict__ wgb = reinterpret_cast<const char*>(a.w);
  const char* zsrc = reinterpret_cast<const char*>(g_zero_page) + lane * 16;

  // epilogue coefficients of every channel, the zero pixel
  for (int i = tid; i < a.Cout; i += Gm::THREADS) {
    coef[2 * i] = a.ch_scale ? a.ch_scale[i] : a.scale;
    coef[2 * i + 1] = a.ch_scale ? a.ch_shift[i] : (a.bias ? (double)a.bias[i] : 0.0);
  }
  if (tid < kPitch / 16)
    *reinterpret_cast<u32x4*>(reinterpret_cast<unsigned char*>(ring_lds) + kZeroOff + tid * 16) =
        (u32x4)0u;

  // ---- weight DMA: wave w moves WI instructions of 1024 / ROWB rows each of every slot
  int64_t wlane[WI];  // per-lane byte offset of its 16-byte source chunk within a K column
  uint32_t wdst[WI];  // LDS byte offset of the instruction within a slot
#pragma unroll
  for (int i = 0; i < WI; ++i) {
    const int r = (wave * WI + i) * (1024 / Gm::ROWB) + lane / CH;
    wlane[i] = (int64_t)r * a.Kp * 2 + (((lane % CH) ^ ((r >> SH) & (CH - 1))) * 16);
    wdst[i] = (uint32_t)((wave * WI + i) * 1024);
  }
  // weight image of K-step (tap t, chunk c) of the tile whose first row is m0 into `slot`
  auto issue_w = [&](int m0, int t, int c, int slot, bool live, uint32_t soff = 0)
      __attribute__((always_inline)) {
    const int64_t col = ((int64_t)m0 * a.Kp + (int64_t)t * a.Cp + (int64_t)c * KS) * 2;
#pragma unroll
    for (int i = 0; i < WI; ++i)
      ring_dma(live ? wgb + col + wlane[i] : zsrc, lds0 + slot * kRingSlot + soff + wdst[i]);
  };

  // ---- patch DMA: piece j of wave w = LDS bytes [(w PI + j) KB, +1 KB) of a patch buffer;
  // lane byte b = that + 16 lane -> pixel b / 144, 16-byte chunk (b % 144) / 16 (8 = pad)
  // per piece: the lane's pixel (or PXS + 1 for a pad chunk: never below any px) and its
  // 32-bit byte offset from the chunk's first patch pixel; no branch at issue time
  int ppix[PI];
  uint32_t poff[PI];
#pragma unroll
  for (int j = 0; j < PI; ++j) {
    const int b = (wave * PI + j) * 1024 + lane * 16;
    const int q = b / kPitch, ch = (b - q * kPitch) >> 4;
    ppix[j] = ch < CH ? q : 1 << 20;
    poff[j] = (uint32_t)((q * a.Cp + ch * 8) * 2);
  }
  // src0: byte address of the chunk's first patch pixel, channel chunk c (uniform)
  auto issue_piece = [&](int j, const char* src0, int px, int buf)
      __attribute__((always_inline)) {
    const char* src = ppix[j] < px ? src0 + poff[j] : zsrc;
    ring_dma(src, lds0 + kPatchOff + buf * Gm::pbuf(PI) + (wave * PI + j) * 1024);
  };

  // ---- B fragment pixels of the current tile: patch pixel of tap (0, 0) and in-bounds taps
  int pix[2];
  uint32_t tmask[2];
  auto setup_b = [&](const RingTile& tl) __attribute__((always_inline)) {
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) {
      const int j = wn + 32 * bn + r32;
      const int64_t p = tl.p0 + j;
      pix[bn] = 0;
      tmask[bn] = 0;
      if (j < BNv && p < a.P) {
        const int64_t img = p / HoWo;
        const int rem = (int)(p - img * HoWo);
        const int oy = rem / a.Wo;
        const int ox = rem - oy * a.Wo;
        const int iy0 = oy - a.ph, ix0 = ox - a.pw;
        pix[bn] = (int)((img * a.H + iy0 - tl.base) * a.W + ix0);
#pragma unroll
        for (int t = 0; t < kRingTaps; ++t) {
          const int iy = iy0 + t / 3, ix = ix0 + t % 3;
          if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) tmask[bn] |= 1u << t;
        }
      }
    }
  };
  // LDS byte address of B block bn's substep-0 fragment at tap t of the patch in buffer buf
  auto baddr = [&](int bn, int t, int buf) __attribute__((always_inline)) {
    const uint32_t in = lds0 + kPatchOff + buf * Gm::pbuf(PI) +
                        (uint32_t)(pix[bn] + (t / 3) * a.W + (t % 3)) * kPitch + hh * 16;
    const uint32_t zero = lds0 + kZeroOff + hh * 16;
    return ((tmask[bn] >> t) & 1u) ? in : zero;
  };
  // A fragment byte address (slot 0) of block bm, substep k: swizzled row image
  uint32_t aaddr[2][SUB];
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int k = 0; k < SUB; ++k) {
      const int row = wm + 32 * bm + r32;
      aaddr[bm][k] = lds0 + (uint32_t)(row * Gm::ROWB +
                                       (((2 * k + hh) ^ ((row >> SH) & (CH - 1))) * 16));
    }

#if RING_AB == 8  // timing only: odd workgroups start ~half a tile late (epilogue stagger)
  if (blockIdx.x & 1)
    for (int i = 0; i < a.ab; ++i) __builtin_amdgcn_s_sleep(127);
#endif
  // ---- this workgroup's tile sequence, j = 0, 1, ...: first the data-parallel tiles g + j G
  // (all of them without SK; SK: the sk.q full rounds), then (SK) the tiles its range of the
  // tail's units [u0, u1) meets -- the first one from chunk u0 % nch, the last one up to
  // chunk (u1 - 1) % nch
  const int64_t dp_n = SK ? sk.q : (T - g + G - 1) / G;
  int64_t u0 = 0, u1 = 0, sk_first = 0, n_sk = 0;
  if constexpr (SK) {
    u0 = g * sk.U / G;
    u1 = (g + 1) * sk.U / G;
    if (u1 > u0) {
      sk_first = sk.q * G + u0 / nch;
      n_sk = sk.q * G + (u1 - 1) / nch - sk_first + 1;
    }
  }
  const int64_t n_seq = dp_n + n_sk;
  if (n_seq == 0) return;  // (uniform: the whole workgroup leaves before any barrier)
  auto tile_at = [&](int64_t j) __attribute__((always_inline)) {
    return j < dp_n ? g + j * G : sk_first + (j - dp_n);
  };
  auto chunk_lo = [&](int64_t j) __attribute__((always_inline)) {
    return SK && j == dp_n ? (int)(u0 % nch) : 0;
  };
  auto chunk_hi = [&](int64_t j) __attribute__((always_inline)) {
    return SK && j >= dp_n && j == n_seq - 1 ? (int)((u1 - 1) % nch) + 1 : nch;
  };
  int64_t seq = 0;
  int64_t tile = tile_at(0);
  RingTile cur = ring_tile(a, tile, R, mt, a.m_slow, ptc);
  RingTile nxt = ring_tile(a, tile_at(seq + 1 < n_seq ? seq + 1 : seq), R, mt, a.m_slow, ptc);
  setup_b(cur);
  int c_lo = chunk_lo(0), c_hi = chunk_hi(0);
  // prologue: chunk c_lo's patch into buffer 0, weight images of steps 0 .. NR-2
#pragma unroll
  for (int j = 0; j < PI; ++j)
    issue_piece(j, reinterpret_cast<const char*>(xg + cur.base * a.W * a.Cp + (int64_t)c_lo * KS),
                cur.px, 0);
#pragma unroll
  for (int j = 0; j + 1 < NR; ++j) issue_w(cur.m0, j, c_lo, j, true);
  TQ_WAIT_VM(0);
  __syncthreads();  // coefficients, tables, zero pixel, the first images visible
  // ring slot of the current chunk's tap 0 (the stream's step index mod NR; 0 when NR | 9)
  int sbase = 0;
  auto slot_off = [&](int tt) __attribute__((always_inline)) -> uint32_t {
    if constexpr (kRingTaps % NR == 0) return (uint32_t)((tt % NR) * kRingSlot);
    else return (uint32_t)(((sbase + tt) % NR) * kRingSlot);
  };

  // residual of pixel block bn of the current tile (FAST epilogue): lane channels cl + 32 bm +
  // 8 q + [0, 4) of its pixel, zero where the pixel or channel is past the tensor
  auto load_res = [&](const RingTile& tl, int bn, float4 (&rv)[2][4])
      __attribute__((always_inline)) {
    const int cl = tl.m0 + wm + 4 * hh;
    const int j = wn + 32 * bn + r32;
    const int64_t p = tl.p0 + j;
    const bool okp = j < BNv && p < a.P;
    const int64_t pc = okp ? p * a.Cout + cl : 0;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = RING_AB != 10 && a.residual && okp && cl + 32 * bm + 8 * q < a.Cout;
        rv[bm][q] = ok ? *reinterpret_cast<const float4*>(a.residual + pc + 32 * bm + 8 * q)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
  };
  // (!FLUSH: pixel block 0's residual is loaded during the tile's last K-step, block 1's
  // before block 0's epilogue -- their HBM latency hides behind MFMAs / block 0's VALU)
  float4 rv_pre[2][4];

  float16v accf[2][2];
  int acci[FLUSH ? 2 : 1][2][16];
  half8 fa[2][2], fb[2][2];  // [buffer][block]: fragments of one 16-code substep
  int buf = 0;               // patch buffer of the current chunk

  // first fragments of the stream
#pragma unroll
  for (int bm = 0; bm < 2; ++bm) fa[0][bm] = lds_frag(aaddr[bm][0]);
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) fb[0][bn] = lds_frag(baddr(bn, 0, 0));

  for (;;) {
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 2; ++bn)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          accf[bm][bn][r] = 0.0f;
          if (FLUSH) acci[bm][bn][r] = 0;
        }
    const bool has_next = seq + 1 < n_seq;
#if RING_TRACE
    unsigned long long tr_s = __builtin_amdgcn_s_memrealtime(), tr_b = 0, tr_k = 0;
#endif
    int since = 0;
    for (int c = c_lo; c < c_hi; ++c) {
      const bool last_chunk = c + 1 == c_hi;
      // the chunk after this one in the stream: its patch rows, channel chunk and weights
      const int64_t nbase = last_chunk ? nxt.base : cur.base;
      const int nc = last_chunk ? chunk_lo(seq + 1) : c + 1;  // (a tail tile may start mid-tile)
      const int nm0 = last_chunk ? nxt.m0 : cur.m0;
      const bool nlive = !last_chunk || has_next;
      const int npx = nlive ? (last_chunk ? nxt.px : cur.px) : 0;  // 0: every lane reads zeros
      const char* nsrc0 =
          reinterpret_cast<const char*>(xg + nbase * a.W * a.Cp + (int64_t)nc * KS);
      uint32_t bcur[2];
#pragma unroll
      for (int bn = 0; bn < 2; ++bn) bcur[bn] = baddr(bn, 0, buf);
      static_for<0, kRingTaps>([&](auto tc) __attribute__((always_inline)) {
        constexpr int t = decltype(tc)::value;
        // (1) retire this wave's weight image of step s+1 (issued at step s-1; the only younger
        // vector-memory op is the patch piece step s-1 issued after it, if any), then the
        // barrier makes every wave's image visible and frees the slot of step s-1
        // younger ops: the weight images of steps s+3-NR .. s-1 (2 instructions each) and
        // the patch pieces of steps s+2-NR .. s-1 (issued after those steps' images)
        constexpr int nyoung = [] {
          int n = WI * (NR - 3);
          for (int j = 1; j <= NR - 2; ++j) n += ((t - j + 2 * kRingTaps) % kRingTaps) < PI;
          return n;
        }();
        if constexpr (RING_AB != 1) TQ_WAIT_VM(nyoung);  // (RING_AB 1: timing only, no wait)
        if constexpr (RING_AB != 5) __builtin_amdgcn_s_barrier();  // (5: timing only)
#if RING_TRACE
        if (t == 0 && c == c_lo) tr_b = __builtin_amdgcn_s_memrealtime();
#endif
        asm volatile("" ::: "memory");
        // (2) weight image of step s+NR-1 into the slot of step s-1; one patch piece of the
        // next chunk (RING_DMA_LATE: after substep 0's MFMAs, so the matrix cores restart
        // before the ~60-185 cycles per DMA issue)
        auto issue_dma = [&]() __attribute__((always_inline)) {
          if constexpr (t + NR - 1 < kRingTaps)
            issue_w(cur.m0, t + NR - 1, c, 0, true, slot_off(t + NR - 1));
          else
            issue_w(nm0, t + NR - 1 - kRingTaps, nc, 0, nlive, slot_off(t + NR - 1));
          if constexpr (t < PI) issue_piece(t, nsrc0, npx, buf ^ 1);
        };
        if constexpr (!RING_DMA_LATE) issue_dma();
        if constexpr (FAST != 0 && !FLUSH && t == kRingTaps - 1) {
          if (last_chunk) load_res(cur, 0, rv_pre);
        }
        // (3) B addresses of step s+1 (next tap, or tap 0 of the next chunk's buffer)
        uint32_t bnx[2];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
          bnx[bn] = t + 1 < kRingTaps ? baddr(bn, (t + 1) % kRingTaps, buf)
                                      : baddr(bn, 0, buf ^ 1);
        // (4) SUB substeps; the fragments of substep k+1 are read before substep k's MFMAs
        const uint32_t soff = slot_off(t), nsoff = slot_off(t + 1);
#pragma unroll
        for (int k = 0; k < SUB; ++k) {
          const int cb = k & 1, nb = cb ^ 1;
          // (at a tile's last step the k = 3 reads fetch the next tile's weights but this
          // tile's pixels: they are read again after the epilogue)
          if (k + 1 < SUB) {
#pragma unroll
            for (int bm = 0; bm < 2; ++bm) fa[nb][bm] = lds_frag(aaddr[bm][k + 1] + soff);
#pragma unroll
            for (int bn = 0; bn < 2; ++bn) fb[nb][bn] = lds_frag(bcur[bn] + 32 * (k + 1));
          } else {
#pragma unroll
            for (int bm = 0; bm < 2; ++bm) fa[nb][bm] = lds_frag(aaddr[bm][0] + nsoff);
#pragma unroll
            for (int bn = 0; bn < 2; ++bn) fb[nb][bn] = lds_frag(bnx[bn]);
          }
#pragma unroll
          for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
#if RING_AB == 2  // timing only: no MFMA (fragments kept live)
              asm volatile("" ::"v"(fa[cb][bm]), "v"(fb[cb][bn]));
#else
              accf[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[cb][bm], fb[cb][bn],
                                                                    accf[bm][bn], 0, 0, 0);
#endif
          // keep the order as written: the next substep's four reads, then this substep's four
          // MFMAs (the scheduler otherwise recycles one fragment register: read, wait, MFMA)
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // DS reads
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMAs
          if constexpr (RING_DMA_LATE != 0)
            if (k == 0) issue_dma();
        }
        // after SUB (even) substeps the next step's fragments sit in buffer 0 again
        bcur[0] = bnx[0];
        bcur[1] = bnx[1];
        if (FLUSH && RING_AB != 6 && a.kc_chunk > 0 && t + 1 < kRingTaps &&
            ++since == a.kc_chunk) {  // (RING_AB 6: timing only, chunk-end windows)
          since = 0;
#pragma unroll
          for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                acci[bm][bn][r] += (int)accf[bm][bn][r];
                accf[bm][bn][r] = 0.0f;
              }
        }
      });
      // window end at every chunk end (chunk-major K order)
      if (FLUSH) {
        since = 0;
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              acci[bm][bn][r] += (int)accf[bm][bn][r];
              accf[bm][bn][r] = 0.0f;
            }
      }
      buf ^= 1;
      sbase = (sbase + kRingTaps) % NR;
    }

    // ---- a split tile (SK): partial sums to this workgroup's slab; the last contributor adds
    // the others' and runs the epilogue (RingSk)
#if RING_TRACE
    tr_k = __builtin_amdgcn_s_memrealtime();
#endif
    bool emit = true;
    if constexpr (SK) {
      if (c_lo != 0 || c_hi != nch) {
        constexpr int kSlab = 64 * Gm::THREADS;  // int32 per slab
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            sk.slab, 0, (int)(G * 2 * kSlab * 4), 0x00020000);
        const int mine = (int)((g * 2 + (seq == dp_n ? 0 : 1)) * kSlab * 4);
#pragma unroll
        for (int i4 = 0; i4 < 16; ++i4) {
          const int bm = i4 >> 3, bn = (i4 >> 2) & 1, r0 = (i4 & 3) * 4;
          u32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = (uint32_t)(FLUSH ? acci[bm][bn][r0 + e] : (int)accf[bm][bn][r0 + e]);
          __builtin_amdgcn_raw_buffer_store_b128(v, rs, (i4 * Gm::THREADS + tid) * 16, mine, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        const int64_t ut = (tile - sk.q * G) * nch;  // the tile's first unit of the tail
        // the contributors: the distinct owners of the tile's units (a workgroup whose range
        // is empty owns none); the ticket counter is the first owner's
        const int k0 = sk_owner(ut, sk.U, G);
        int ncon = 0;
        for (int u = 0, prev = -1; u < nch; ++u) {
          const int o = sk_owner(ut + u, sk.U, G);
          ncon += o != prev;
          prev = o;
        }
        uint32_t* flag = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(ring_lds) +
                                                     kZeroOff + 144);
        if (tid == 0) {
          const int t = __hip_atomic_fetch_add(sk.cnt + k0, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
          const bool last = t == ncon - 1;
          if (last) __hip_atomic_store(sk.cnt + k0, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *flag = last ? 1u : 0u;
        }
        __syncthreads();
        emit = *flag != 0;
        if (emit) {
          for (int u = 0, prev = -1; u < nch; ++u) {
            const int g2 = sk_owner(ut + u, sk.U, G);
            if (g2 == prev) continue;
            prev = g2;
            if (g2 == g) continue;
            const int64_t first2 = sk.q * G + ((int64_t)g2 * sk.U / G) / nch;
            const int other = (int)((g2 * 2 + (tile == first2 ? 0 : 1)) * kSlab * 4);
#pragma unroll
            for (int i4 = 0; i4 < 16; ++i4) {
              const int bm = i4 >> 3, bn = (i4 >> 2) & 1, r0 = (i4 & 3) * 4;
              const u32x4 v = __builtin_bit_cast(
                  u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (i4 * Gm::THREADS + tid) * 16,
                                                               other, 16));
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                if (FLUSH) acci[bm][bn][r0 + e] += (int)v[e];
                else accf[bm][bn][r0 + e] += (float)(int)v[e];
              }
            }
          }
        }
      }
    }

    if (emit) {
      // ---- epilogue from the MFMA layout: lane (r32, hh) of block (bm, bn) holds channels
      // m0 + wm + 32 bm + 8 q + 4 hh + [0, 4) of pixel column wn + 32 bn + r32
      if constexpr (FAST != 0) {
        const int cl = cur.m0 + wm + 4 * hh;  // the lane's first channel
        const double* cf = coef + 2 * cl;
        // one pixel block's residual loads at a time (FLUSH: both blocks' would spill)
        float4 rv_next[2][4];
        static_for<0, 2>([&](auto bnc) __attribute__((always_inline)) {
          constexpr int bn = decltype(bnc)::value;
          const int j = wn + 32 * bn + r32;
          const int64_t p = cur.p0 + j;
          const bool okp = j < BNv && p < a.P;
          const int64_t pc = okp ? p * a.Cout + cl : 0;
          float4 rv[2][4];
          if constexpr (FLUSH) {
            load_res(cur, bn, rv);
          } else if constexpr (bn == 0) {
            load_res(cur, 1, rv_next);  // block 1's loads in flight during block 0
#pragma unroll
            for (int bm = 0; bm < 2; ++bm)
#pragma unroll
              for (int q = 0; q < 4; ++q) rv[bm][q] = rv_pre[bm][q];
          } else {
#pragma unroll
            for (int bm = 0; bm < 2; ++bm)
#pragma unroll
              for (int q = 0; q < 4; ++q) rv[bm][q] = rv_next[bm][q];
          }
          if (!okp || (RING_AB == 4 && a.out != (float*)p)) return;
#pragma unroll
          for (int bm = 0; bm < 2; ++bm) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int d = 32 * bm + 8 * q;
              if (cl + d >= a.Cout) continue;
              const float4 r = rv[bm][q];
              const float rr[4] = {r.x, r.y, r.z, r.w};
              float y[4], o[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int acc = FLUSH ? acci[bm][bn][4 * q + e] : (int)accf[bm][bn][4 * q + e];
                y[e] = fold_acc(acc, (coef_t)cf[2 * (d + e)], (coef_t)cf[2 * (d + e) + 1]) + rr[e];
                o[e] = y[e] != y[e] ? y[e] : fmaxf(y[e], 0.0f);  // torch.relu keeps NaN
                y[e] = fmaxf(y[e], 0.0f);                         // TR(NaN) = 0
              }
              if (RING_AB == 9) {  // timing only: no stores (values kept live)
                asm volatile("" ::"v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]));
                uint32_t qz[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) qz[e] = lut_a[relu_q(y[e], a.inv_a, a.maxv_a)];
                asm volatile("" ::"v"(qz[0]), "v"(qz[1]), "v"(qz[2]), "v"(qz[3]));
                continue;
              }
              if (FAST == 2 || a.out)
                *reinterpret_cast<float4*>(a.out + pc + d) = make_float4(o[0], o[1], o[2], o[3]);
              if constexpr (FAST == 2) continue;  // (form 2: no code outputs)
              uint32_t qa[4];
#pragma unroll
              for (int e = 0; e < 4; ++e)
                qa[e] = RING_AB == 11 ? relu_q(y[e], a.inv_a, a.maxv_a)
                                      : lut_a[relu_q(y[e], a.inv_a, a.maxv_a)];
              *reinterpret_cast<uint2*>(a.codes_a + p * a.cp_a + cl + d) =
                  make_uint2(qa[0] | (qa[1] << 16), qa[2] | (qa[3] << 16));
              if (a.codes_b) {
                uint32_t qb[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) qb[e] = lut_b[relu_q(y[e], a.inv_b, a.maxv_b)];
                *reinterpret_cast<uint2*>(a.codes_b + p * a.cp_b + cl + d) =
                    make_uint2(qb[0] | (qb[1] << 16), qb[2] | (qb[3] << 16));
              }
              if (cl + d + 4 == a.Cout) {  // the last quad zeroes the pad channels [Cout, cp)
                if (a.cp_a > a.Cout)
                  *reinterpret_cast<uint2*>(a.codes_a + p * a.cp_a + cl + d + 4) = make_uint2(0, 0);
                if (a.codes_b && a.cp_b > a.Cout)
                  *reinterpret_cast<uint2*>(a.codes_b + p * a.cp_b + cl + d + 4) = make_uint2(0, 0);
              }
            }
          }
        });
      } else {
        static_for<0, 2>([&](auto bmc) __attribute__((always_inline)) {
          constexpr int bm = decltype(bmc)::value;
          float4 rv[2][4];
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int co = cur.m0 + wm + 32 * bm + 8 * q + 4 * hh;
              const int j = wn + 32 * bn + r32;
              const int64_t p = cur.p0 + j;
              const bool ok = a.residual && co < a.Cout && j < BNv && p < a.P;
              rv[bn][q] = ok ? *reinterpret_cast<const float4*>(a.residual + p * a.Cout + co)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int co = cur.m0 + wm + 32 * bm + 8 * q + 4 * hh;
              const int j = wn + 32 * bn + r32;
              const int64_t p = cur.p0 + j;
              if (co >= a.Cout || j >= BNv || p >= a.P) continue;
              if (RING_AB == 4 && a.out != (float*)p) continue;  // timing only: no epilogue
              int acc4[4];
#pragma unroll
              for (int e = 0; e < 4; ++e)
                acc4[e] = FLUSH ? acci[bm][bn][4 * q + e] : (int)accf[bm][bn][4 * q + e];
              coef_t sc[4], sh[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                sc[e] = (coef_t)coef[2 * (co + e)];
                sh[e] = (coef_t)coef[2 * (co + e) + 1];
              }
              emit4_nhwc_res(a, p, co, acc4, sc, sh, rv[bn][q], lut_a, lut_b);
            }
        });
      }
    }

#if RING_TRACE
    if (tid == 0 && blockIdx.x < 1024 && seq < 8) {
      unsigned long long* r = g_ring_trace + ((int64_t)blockIdx.x * 8 + seq) * 4;
      r[0] = tr_s;
      r[1] = tr_b;
      r[2] = tr_k;
      r[3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if (!has_next) break;
    // ---- next tile: its patch chunk 0 and weight steps 0/1 are already staged or in flight
    ++seq;
    tile = tile_at(seq);
    cur = nxt;
    nxt = ring_tile(a, tile_at(seq + 1 < n_seq ? seq + 1 : seq), R, mt, a.m_slow, ptc);
    c_lo = chunk_lo(seq);
    c_hi = chunk_hi(seq);
    setup_b(cur);
    // its first fragments (the last step of the previous tile prefetched this tile's
    // weights but the old pixels): step 0's image and patch were retired by the barrier of
    // the previous tile's last step.  Its ring slot is the stream's step index mod NR, which
    // is not 0 when 9 * nch is not a multiple of NR.
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) fa[0][bm] = lds_frag(aaddr[bm][0] + slot_off(0));
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) fb[0][bn] = lds_frag(baddr(bn, 0, buf));
  }
}

template <int NW, int KS, int PI, bool FLUSH, int FAST, bool SK>
hipError_t launch_ring_fast(const ConvArgs& a, int R, int64_t ptc, int64_t grid, size_t lds,
                            const RingSk& sk, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv2d_tp_ring_kernel<NW, KS, PI, FLUSH, FAST, SK>),
        hipFuncAttributeMaxDynamicSharedMemorySize, RingGeom<NW, KS>::BUDGET);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  conv2d_tp_ring_kernel<NW, KS, PI, FLUSH, FAST, SK>
      <<<dim3((unsigned)grid), 64 * NW, lds, stream>>>(a, R, ptc, sk);
  return hipGetLastError();
}

// the specialised epilogue form (the kernel's FAST): 1 = ReLU + fp16 codes_a (+ codes_b) each
// served by a code table; 2 = ReLU + fp32 output, no codes; 0 = the generic emit4_nhwc_res
// (every form with TQ_EPI_FAST=0)
bool ring_codes_form(const ConvArgs& a) {
  return a.relu == 1 && a.codes_a != nullptr && a.lut_a > 0 && a.fmt_a == kCodesF16 &&
         (a.codes_b == nullptr || (a.lut_b > 0 && a.fmt_b == kCodesF16));
}
int ring_epilogue_form(const ConvArgs& a) {
  const char* v = getenv("TQ_EPI_FAST");
  if (v && atoi(v) == 0) return 0;
  if (ring_codes_form(a)) return 1;
  return a.relu == 1 && a.out != nullptr && a.codes_a == nullptr && a.codes_b == nullptr ? 2 : 0;
}

template <int NW, int KS, int PI, bool SK>
hipError_t launch_ring_sk(const ConvArgs& a, int R, int64_t ptc, int64_t grid, size_t lds,
                          const RingSk& sk, hipStream_t stream) {
  const bool flush = a.kc_steps != 0;  // 0: the whole K range is one exact window
  hipError_t e = hipErrorInvalidValue;
  static_for<0, 3>([&](auto fc) {
    constexpr int F = decltype(fc)::value;
    if (F != ring_epilogue_form(a)) return;
    e = flush ? launch_ring_fast<NW, KS, PI, true, F, SK>(a, R, ptc, grid, lds, sk, stream)
              : launch_ring_fast<NW, KS, PI, false, F, SK>(a, R, ptc, grid, lds, sk, stream);
  });
  return e;
}

// sk == nullptr: the data-parallel tile stream; else the stream-K split (8-wave shape only)
template <int NW, int KS, int PI>
hipError_t launch_ring_pi(const ConvArgs& a, int R, int64_t ptc, int64_t grid, size_t lds,
                          const RingSk* sk, hipStream_t stream) {
  if constexpr (NW == 8)
    if (sk) return launch_ring_sk<NW, KS, PI, true>(a, R, ptc, grid, lds, *sk, stream);
  return launch_ring_sk<NW, KS, PI, false>(a, R, ptc, grid, lds, RingSk{}, stream);
}

// ---- stream-K workspaces, one per (device, stream): a kernel on another stream may run
// concurrently, so no two streams share slabs or counters.  Allocated (and the counters
// zeroed) at the first split launch on a stream; a stream being captured into a graph that
// has none runs the data-parallel stream instead (same results).
struct SkWorkspace {
  int dev;
  hipStream_t stream;
  int* base;  // [1024] counters | slabs
  int64_t slab_ints;
};
constexpr int kSkMaxGrid = 1024;
constexpr int kSkMaxWorkspaces = 16;
std::mutex g_sk_mu;
SkWorkspace g_sk_ws[kSkMaxWorkspaces];
int g_sk_n = 0;

bool sk_workspace(hipStream_t stream, int64_t grid, int64_t slab_ints, RingSk* sk) {
  if (grid > kSkMaxGrid) return false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(g_sk_mu);
  SkWorkspace* w = nullptr;
  for (int i = 0; i < g_sk_n; ++i)
    if (g_sk_ws[i].dev == dev && g_sk_ws[i].stream == stream) w = &g_sk_ws[i];
  if (w && w->slab_ints < grid * slab_ints) return false;  // (grid is fixed per device)
  if (!w) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone)
      return false;
    if (g_sk_n == kSkMaxWorkspaces) return false;
    // room for the device's default grid, so later launches never outgrow it
    const int64_t ints = (grid > device_cus() ? grid : device_cus()) * slab_ints;
    int* base = nullptr;
    if (hipMalloc(&base, (size_t)(kSkMaxGrid + ints) * sizeof(int)) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    if (hipMemsetAsync(base, 0, kSkMaxGrid * sizeof(int), stream) != hipSuccess) {
      (void)hipFree(base);
      return false;
    }
    w = &g_sk_ws[g_sk_n++];
    *w = SkWorkspace{dev, stream, base, ints};
  }
  sk->cnt = w->base;
  sk->slab = w->base + kSkMaxGrid;
  return true;
}

// TQ_RING_SK: 0 (default) = data-parallel tiles only; 1 = a stream-K tail when it shortens the
// longest per-workgroup chunk list with at most one tail chunk per workgroup; 3 = whenever it
// shortens that list; 2 = a tail of about half the tiles whenever tiles are left over (tests).
// Measured (profiles/r04_ring_streamk_ab.txt): mode 1 equal-to-slower on layer 2, mode 3
// 40-45 % slower on layers 3/4 -- the SK instantiations spill more in the K loop, and an
// all-CU MFMA loop runs each step slower (the round-3 patch-engine finding)
int ring_sk_mode() {
  const char* v = getenv("TQ_RING_SK");
  return v ? atoi(v) : 0;
}

// Largest patch (pixels) over every tile: the row pattern repeats every Ho / gcd(R, Ho) tiles.
int64_t ring_max_patch_px(const ConvArgs& a, int R) {
  int64_t g = R, r = a.Ho;
  while (r) {
    const int64_t t = g % r;
    g = r;
    r = t;
  }
  const int64_t ptc = ((int64_t)a.N * a.Ho + R - 1) / R;
  int64_t period = a.Ho / g;
  if (period > ptc) period = ptc;
  int64_t best = 0;
  for (int64_t j = 0; j < period; ++j) {
    const RingTile t = ring_tile(a, j, R, 1, 0, ptc);
    if (t.px > best) best = t.px;
  }
  return best;
}

// A launch plan of one engine shape: rows per tile, patch pieces per wave, dynamic LDS.
struct RingPlan {
  int R, pi;
  int64_t lds;
};

template <int NW, int KS>
bool ring_plan(const ConvArgs& a, RingPlan* pl) {
  using Gm = RingGeom<NW, KS>;
  if (a.Cp % KS != 0 || a.Wo > Gm::BN) return false;
  pl->R = Gm::BN / a.Wo;
  const int64_t px = ring_max_patch_px(a, pl->R);
  for (int pi = 3; pi <= 6; ++pi) {
    const int nr = Gm::slots(pi);
    if (nr < 3 || pi > 10 - nr || px > Gm::pxs(pi)) continue;
    pl->pi = pi;
    pl->lds = Gm::coef_off(pi, nr) + (int64_t)a.Cout * 16 + conv_lut_bytes(a);
    return pl->lds <= Gm::BUDGET;
  }
  return false;
}

template <int NW, int KS>
hipError_t launch_ring_shape(const ConvArgs& a, const RingPlan& pl, int per_cu,
                             hipStream_t stream) {
  const int64_t ptc = ((int64_t)a.N * a.Ho + pl.R - 1) / pl.R;
  const int64_t tiles = ptc * ((a.Cout + kRingBM - 1) / kRingBM);
  int64_t grid = (int64_t)per_cu * device_cus();
  const char* genv = getenv("TQ_RING_GRID");  // tests: fewer workgroups, more tiles each
  if (genv && atoi(genv) > 0) grid = atoi(genv);
  // stream-K tail (8-wave shape, RingSk; opt-in, ring_sk_mode): after q full rounds the r
  // tiles left are split into their r * nch chunks over the whole grid, so the longest list
  // is q nch + ceil(r nch / G) chunks instead of (q + 1) nch
  RingSk sk{};
  const RingSk* skp = nullptr;
  const int skm = ring_sk_mode();
  if (NW == 8 && skm > 0) {
    const int64_t nch = a.Cp / KS;
    int64_t q = tiles / grid;
    if (skm == 2) q /= 2;  // tests: a longer tail, ranges over several tiles
    const int64_t r = tiles - q * grid;
    const int64_t U = r * nch;
    const int64_t dp_max = (tiles + grid - 1) / grid * nch;
    const int64_t sk_max = q * nch + (U + grid - 1) / grid;
    const bool want = skm == 2 ? r > 0 : r > 0 && sk_max < dp_max && (skm == 3 || U <= grid);
    if (nch > 1 && want && sk_workspace(stream, grid, 2 * 64 * RingGeom<NW, KS>::THREADS, &sk)) {
      sk.U = U;
      sk.q = q;
      skp = &sk;
    }
  }
  if (!skp && grid > tiles) grid = tiles;
  const size_t lds = (size_t)pl.lds;
  hipError_t e = hipErrorInvalidValue;
  static_for<3, 7>([&](auto pc) {
    constexpr int PI = decltype(pc)::value;
    constexpr int NR = RingGeom<NW, KS>::slots(PI);
    if constexpr (NR >= 3 && PI <= 10 - NR)  // the shapes ring_plan can choose
      if (pl.pi == PI) e = launch_ring_pi<NW, KS, PI>(a, pl.R, ptc, grid, lds, skp, stream);
  });
  return e;
}

// TQ_RING_V=1: the 8-wave shape, 2: the two-workgroups-per-CU shape (read per launch)
int ring_shape() {
  const char* v = getenv("TQ_RING_V");
  return v && atoi(v) == 2 ? 2 : 1;
}

bool ring_common(const ConvArgs& a, int out_nhwc) {
  return out_nhwc && a.KH == 3 && a.KW == 3 && a.sh == 1 && a.sw == 1 && a.dh == 1 &&
         a.dw == 1 && a.Kp == 9 * a.Cp && (a.Cout & 3) == 0 && a.Wo >= 1 &&
         a.ds_x == nullptr && a.relu != kActSwish && a.Cout <= 512 &&
         a.H == a.Ho && a.W == a.Wo;  // "same" padding: stride 1, pad 1
}

}  // namespace

bool conv_ring_eligible(const ConvArgs& a, int out_nhwc) {
  RingPlan pl;
  if (!ring_common(a, out_nhwc)) return false;
  return ring_shape() == 2 ? ring_plan<4, 32>(a, &pl) : ring_plan<8, 64>(a, &pl);
}

hipError_t launch_conv2d_ring(const ConvArgs& a, hipStream_t stream) {
  RingPlan pl;
  if (!ring_common(a, 1)) return hipErrorInvalidValue;
  if (ring_shape() == 2) {
    if (!ring_plan<4, 32>(a, &pl)) return hipErrorInvalidValue;
    return launch_ring_shape<4, 32>(a, pl, 2, stream);
  }
  if (!ring_plan<8, 64>(a, &pl)) return hipErrorInvalidValue;
  return launch_ring_shape<8, 64>(a, pl, 1, stream);
}

#if RING_TRACE
extern "C" int tq_ring_trace_read(void* dst, int64_t n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ring_trace), (size_t)n * 8, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int tq_ring_trace_clear() {
  static unsigned long long zero[1024 * 8 * 4];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ring_trace), zero, sizeof(zero), 0,
                                hipMemcpyHostToDevice);
}
#endif

}  // namespace tq
