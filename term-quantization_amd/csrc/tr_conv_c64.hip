// Term-pair Conv2d on the matrix cores, Cout-64 pixel-ring engine: 3x3 stride-1 "same" convs
// with 64 -> 64 channels (ResNet-18 layer 1: both convs of both blocks, with and without the
// block's fp32 residual and output).
//
// Same exact arithmetic as the other MFMA engines (tr_conv_mfma.hip): fp16 term-sum codes,
// v_mfma_f32_32x32x16_f16, fp32 partial sums exact inside host-bounded windows (flushed into
// int32 sums every kc_steps taps when the host asks for it), one fp64 fold per output.  Its
// outputs are bit-identical to every other engine's.
//
// Why another engine.  The layer-1 convs were the furthest below their floors (round 4:
// strip conv1s 114-118 us and direct conv2s 207 / 176 us against 24 us of MFMA work and 26 /
// 77 / 51 us of HBM traffic).  The row-strip engine splits a tile's seven 32-pixel blocks 4 : 3
// over its waves and syncs its two teams through spinning LDS counters; the direct engine
// re-reads nine taps of activation fragments through the vector L1 per 64 output channels and
// restarts its pipeline every tile.  Here:
//   * one persistent 8-wave workgroup per CU walks a contiguous run of 256-pixel tiles of the
//     flattened N*H*W pixel order (every tile full: no row alignment, no idle waves; a tile may
//     cross an image boundary, taps outside their image read a zero pixel);
//   * the whole 64 x 576 weight matrix stays in LDS (73 KB, row pitch 73 units so the B
//     fragment reads of 16 rows hit 16 distinct bank quads with no swizzle: every weight read is
//     one per-lane base plus an immediate offset);
//   * the input codes live in a RING of 640 pixel slots (80 KB): tile j reads pixels
//     [p0 - 64, p0 + 320) -- its 256 pixels and a halo of W + 1 <= 64 on either side -- while
//     the next tile's 256 new pixels [p0 + 320, p0 + 576) stream in by LDS-DMA into the slots
//     tile j - 1 used (slot = pixel mod 640, 16-byte units XOR-swizzled by (slot >> 1) & 7, so
//     a ds_read_b128 of 16 consecutive pixels hits 16 distinct bank quads).  Each input pixel
//     comes from HBM/L2 once per workgroup, as one contiguous 32 KB range per tile;
//   * one s_barrier per tile (the ring hand-off), no per-K-step synchronisation: the 36
//     substeps (9 taps x 4 x 16 codes) of a tile are unrolled with every fragment read one
//     substep ahead of the MFMAs;
//   * MFMA roles as the strip engine: A = activation codes (rows = 32 output pixels), B =
//     weight codes (columns = 32 output channels), so a lane's accumulators are 16 pixels of
//     two channels (r32 and 32 + r32): its BN coefficients are four registers for the whole
//     launch, and every residual load / fp32 store / code store instruction covers whole
//     channel rows of two pixels;
//   * the epilogues of the two waves sharing a SIMD are staggered (MI355X_MICROARCH.md "Two
//     waves per SIMD", item 9): waves 0-3 run tile j's MFMAs then its epilogue, waves 4-7 tile
//     j-1's epilogue then tile j's MFMAs, so one wave's VALU and stores run beside its
//     partner's matrix work on every SIMD.  Only waves 0-3 issue the ring DMA, so a late
//     wave's residual registers (loaded before its MFMAs, consumed after the next barrier)
//     never wait behind a DMA in its own vmcnt queue;
//   * residual loads and all epilogue stores are buffer instructions with per-lane offsets,
//     so no store is skipped by a branch and the vmcnt count a wave waits with before the
//     barrier (its DMA is older than exactly its epilogue's stores) is a compile-time
//     constant.  A pixel block past the tensor would get an offset past the buffer (loads
//     read 0, stores dropped), but under conv_c64_eligible (P % 32 == 0) no wave owns such a
//     block: a wave whose block starts at or past its workgroup's range end returns before
//     its residual loads and epilogue (the late epilogue is gated the same way), so those
//     offsets are defense in depth only (tests/test_gpu_c64.py checks a guard tail behind
//     every output buffer).
//
//   LDS = weights [64][73 x 16 B] | ring [640][128 B] | zero pixel (128 B) | code tables
#include <stdlib.h>

#include <type_traits>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

#ifndef C64_AB
#define C64_AB 0  // timing-only ablation builds (tools/ab/variant1.sh); 0 = the product kernel
#endif
#ifndef C64_PF
#define C64_PF 2  // substeps of fragment prefetch (2: conv1 77 -> 73 us; residual forms equal)
#endif
#ifndef C64_PRIO
#define C64_PRIO 0  // 1: s_setprio 1 for waves 4-7, 2: for waves 0-3 (A/B builds)
#endif
#ifndef C64_STAGGER
#define C64_STAGGER 1  // 0: every wave runs its epilogue right after its MFMAs (A/B builds)
#endif

namespace tq {

namespace {

constexpr int kC64Threads = 512;
constexpr int kC64Tile = 256;                     // output pixels per tile
constexpr int kC64Taps = 9;                       // 3 x 3
constexpr int kC64Sub = kC64Taps * 4;             // 16-code substeps per tile
constexpr int kC64WPitch = 73 * 16;               // weight row pitch (72 units + 1 pad)
constexpr int kC64WBytes = 64 * kC64WPitch;       // 74,752
constexpr int kC64Ring = 640;                     // ring slots (pixels)
constexpr int kC64Halo = 64;                      // halo pixels staged each side (>= W + 1)
constexpr int kC64RingOff = kC64WBytes;
constexpr int kC64ZeroOff = kC64RingOff + kC64Ring * 128;
constexpr int kC64LutOff = kC64ZeroOff + 128;
constexpr int kC64Budget = 160 * 1024;
constexpr int kC64ProloguePieces = (kC64Tile + 2 * kC64Halo) / 8;  // 48 (6 per wave)
constexpr int kC64TilePieces = kC64Tile / 8;                        // 32 (8 per early wave)
static_assert(kC64RingOff % 128 == 0 && kC64ZeroOff % 128 == 0, "XOR addressing");
static_assert(kC64Ring >= 2 * kC64Tile + 2 * kC64Halo, "ring: a tile's window + the next 256");
static_assert(kC64Ring % 16 == 0, "the swizzle pattern must survive the ring wrap");

// One LDS-DMA wave-instruction (1 KB, lane-linear destination) as inline asm, invisible to the
// compiler's wait-count pass (tq_mfma.h glds16_asm); the LDS address is uniform.
__device__ __forceinline__ void c64_dma(const void* src, uint32_t lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(lds_byte)
               : "memory", "m0");
}

__device__ __forceinline__ half8 c64_frag(uint32_t byte_addr) {
  return __builtin_bit_cast(
      half8, *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(
                 (uintptr_t)byte_addr));
}

template <int V>
struct c64_ic {
  static constexpr int value = V;
};
template <int I, int N, typename F>
__device__ __forceinline__ void c64_for(F&& f) {
  if constexpr (I < N) {
    f(c64_ic<I>{});
    c64_for<I + 1, N>(f);
  }
}

constexpr uint32_t kOob = 0x80000000u;  // a buffer offset past every buffer this engine uses

// RES: fp32 residual input; OUT: fp32 output; NCODES: code outputs (each from its code table,
// ReLU form); FLUSH: int32 exactness windows every kc_steps taps.
template <bool RES, bool OUT, int NCODES, bool FLUSH>
__global__ __launch_bounds__(kC64Threads) void conv2d_tp_c64_kernel(ConvArgs a, int nblk) {
  extern __shared__ __attribute__((aligned(16))) u32x4 c64_lds[];
  unsigned char* lb = reinterpret_cast<unsigned char*>(c64_lds);
  const uint32_t lds0 =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) u32x4*)c64_lds;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const bool late = C64_STAGGER && wave >= 4;  // waves 4-7: epilogue deferred by one tile

  const int G = gridDim.x;
  const int g = xcd_remap(blockIdx.x, G);
  // this workgroup's pixels [pb0, pe): an equal share of the 32-pixel blocks, walked as
  // 256-pixel tiles from pb0 (the last tile may hold fewer blocks: its idle waves skip it)
  const int pb0 = (int)((int64_t)g * nblk / G) * 32;
  const int pe = (int)((int64_t)(g + 1) * nblk / G) * 32;
  if (pb0 >= pe) return;  // (uniform: before any barrier)

  const int P = (int)a.P;  // the launcher checks P * 256 < 2^31
  const char* __restrict__ xb = reinterpret_cast<const char*>(a.x);
  const char* zsrc = reinterpret_cast<const char*>(g_zero_page) + lane * 16;

  // ring piece: 8 input pixels [q0, q0 + 8) (q0 % 8 == 0) into their slots; pixels outside
  // the tensor read zeros (no tap reads them: their taps are masked)
  auto issue_piece = [&](int q0) __attribute__((always_inline)) {
    int s0 = q0 % kC64Ring;
    s0 = s0 < 0 ? s0 + kC64Ring : s0;
    const int q = q0 + (lane >> 3);
    const int s = s0 + (lane >> 3);
    const int c = (lane & 7) ^ ((s >> 1) & 7);
    const char* src = (q >= 0 && q < P) ? xb + (int64_t)q * 128 + c * 16 : zsrc;
    c64_dma(src, lds0 + kC64RingOff + (uint32_t)s0 * 128);
  };

  // ---- prologue: the first tile's window, the weights, the zero pixel, the code tables
  const int p_first = pb0;
#pragma unroll
  for (int i = 0; i < kC64ProloguePieces / 8; ++i)
    issue_piece(p_first - kC64Halo + 8 * (wave * (kC64ProloguePieces / 8) + i));
  for (int u = tid; u < 64 * 72; u += kC64Threads) {
    const int row = u / 72, un = u - row * 72;
    const u32x4 v = *reinterpret_cast<const u32x4*>(a.w + (int64_t)row * a.Kp + un * 8);
    *reinterpret_cast<u32x4*>(lb + row * kC64WPitch + un * 16) = v;
  }
  if (tid < 8) *reinterpret_cast<u32x4*>(lb + kC64ZeroOff + tid * 16) = (u32x4)0u;
  uint16_t *lut_a, *lut_b;
  conv_luts(a, reinterpret_cast<uint16_t*>(lb + kC64LutOff), lut_a, lut_b);

  // per-lane epilogue constants: channels r32 and 32 + r32
  double sc[2], sh[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int c = 32 * nb + r32;
    sc[nb] = a.ch_scale ? a.ch_scale[c] : a.scale;
    sh[nb] = a.ch_scale ? a.ch_shift[c] : (a.bias ? (double)a.bias[c] : 0.0);
  }
  const int nf = P * 64 * 4;  // fp32 tensor bytes
  const __amdgpu_buffer_rsrc_t rs_out =
      __builtin_amdgcn_make_buffer_rsrc(a.out, 0, OUT ? nf : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_res =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.residual), 0, RES ? nf : 0,
                                        0x00020000);
  const __amdgpu_buffer_rsrc_t rs_ca =
      __builtin_amdgcn_make_buffer_rsrc(a.codes_a, 0, NCODES >= 1 ? nf / 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_cb =
      __builtin_amdgcn_make_buffer_rsrc(a.codes_b, 0, NCODES >= 2 ? nf / 2 : 0, 0x00020000);

  TQ_WAIT_VM(0);
  __syncthreads();  // weights, ring window, zero pixel, tables visible
  if (C64_PRIO == 1 && wave >= 4) __builtin_amdgcn_s_setprio(1);
  if (C64_PRIO == 2 && wave < 4) __builtin_amdgcn_s_setprio(1);

  // B (weight) fragment base: row r32 of channel block 0, unit hh; + 32 rows for block 1,
  // + (8 t + 2 k) units for tap t, substep k -- all immediate offsets
  const uint32_t wbase = lds0 + (uint32_t)(r32 * kC64WPitch + hh * 16);
  const int HW = a.H * a.W;

  float16v acc[2];
  int acci[FLUSH ? 2 : 1][16];
  float rv[RES ? 2 : 1][16];

  // residual of the wave's 32 pixels of tile pt: rv[nb][4 q + e] = pixel 8 q + 4 hh + e,
  // channel 32 nb + r32 (a block past the tensor reads zeros)
  auto load_res = [&](int pt) __attribute__((always_inline)) {
    if constexpr (RES) {
      const int pb = pt + 32 * wave;
      const uint32_t vf = pb < pe ? (uint32_t)(((pb + 4 * hh) * 64 + r32) * 4) : kOob;
      c64_for<0, 2>([&](auto nbc) __attribute__((always_inline)) {
        constexpr int nb = decltype(nbc)::value;
        c64_for<0, 16>([&](auto rc) __attribute__((always_inline)) {
          constexpr int r = decltype(rc)::value;
          constexpr uint32_t off = (8 * (r >> 2) + (r & 3)) * 256 + nb * 128;
          rv[nb][r] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rs_res, (int)(vf + off), 0, 0));
        });
      });
    }
  };

  // epilogue of the wave's 32 pixels of tile pt from acc / acci and rv
  auto epilogue = [&](int pt) __attribute__((always_inline)) {
    if (C64_AB == 1) {  // timing only: no epilogue (sums kept live)
      asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][15]));
      return;
    }
    const int pb = pt + 32 * wave;
    const bool okb = pb < pe;
    const uint32_t vf = okb ? (uint32_t)(((pb + 4 * hh) * 64 + r32) * 4) : kOob;
    const uint32_t vc = okb ? (uint32_t)(((pb + 4 * hh) * 64 + r32) * 2) : kOob;
    c64_for<0, 2>([&](auto nbc) __attribute__((always_inline)) {
      constexpr int nb = decltype(nbc)::value;
      c64_for<0, 16>([&](auto rc) __attribute__((always_inline)) {
        constexpr int r = decltype(rc)::value;
        constexpr uint32_t pix = 8 * (r >> 2) + (r & 3);
        // (without int32 windows the fp32 sum is an exact integer: converted to fp64
        // directly, the same value fold_acc gets through int32)
        float y = FLUSH || TQ_EPI_F32
                      ? fold_acc(FLUSH ? acci[nb][r] : (int)acc[nb][r], (coef_t)sc[nb],
                                 (coef_t)sh[nb])
                      : (float)((double)acc[nb][r] * sc[nb] + sh[nb]);
        if constexpr (RES) y += rv[nb][r];
        float o = y;
        y = y > 0.0f ? y : 0.0f;
        o = o != o ? o : y;  // the stored value keeps a NaN (torch.relu); its codes are 0
        if constexpr (OUT)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, o), rs_out,
                                                (int)(vf + pix * 256 + nb * 128), 0, 0);
        if constexpr (NCODES >= 1) {
          const uint32_t q = relu_q(y, a.inv_a, a.maxv_a);
          __builtin_amdgcn_raw_buffer_store_b16((unsigned short)lut_a[q], rs_ca,
                                                (int)(vc + pix * 128 + nb * 64), 0, 0);
        }
        if constexpr (NCODES >= 2) {
          const uint32_t q = relu_q(y, a.inv_b, a.maxv_b);
          __builtin_amdgcn_raw_buffer_store_b16((unsigned short)lut_b[q], rs_cb,
                                                (int)(vc + pix * 128 + nb * 64), 0, 0);
        }
      });
    });
  };
  // epilogue stores per wave and tile: what an early wave's DMA is older than at the barrier
  constexpr int kStores = 32 * ((OUT ? 1 : 0) + NCODES);
  constexpr int kWaitYoung = kStores < 63 ? kStores : 63;

  // the tile loop, compiled once per role: with one body for both, the compiler's wait-count
  // analysis merged the roles' paths (a late wave's residual loads still in flight where an
  // early wave reloads them) and drained vmcnt(0) -- the DMA just issued -- every tile
  // (and the first tile is peeled: a loop-carried "first tile?" test left a path on which a late
  // wave's residual loads were still in flight where it reloads them -- vmcnt(0) again)
  auto run = [&](auto late_c) __attribute__((always_inline)) {
    constexpr bool LATE = decltype(late_c)::value;
    auto body = [&](auto first_c, int p0) __attribute__((always_inline)) {
      constexpr bool FIRST = decltype(first_c)::value;
      const bool act = p0 + 32 * wave < pe;  // this wave's block is in the range (uniform)
      if (!FIRST) {
        // the early waves' DMA of this tile's new pixels (issued at the top of the previous
        // tile; younger than it: that tile's epilogue stores -- and its residual loads, which
        // the epilogue already waited for) has landed; the barrier publishes it and frees the
        // slots of the tile before last
        if (!LATE) TQ_WAIT_VM(kWaitYoung);
        if (C64_AB != 4) __builtin_amdgcn_s_barrier();  // (4: timing only, no barrier)
        asm volatile("" ::: "memory");
      }
      if (C64_AB != 3 && !LATE && p0 + kC64Tile < pe) {  // (3: timing only, no ring refill)
  #pragma unroll
        for (int i = 0; i < kC64TilePieces / 4; ++i)
          issue_piece(p0 + kC64Tile + kC64Halo + 8 * (wave * (kC64TilePieces / 4) + i));
      }
      if (LATE && !FIRST) epilogue(p0 - kC64Tile);  // (a wave idles in the last tile only)
      if (!act) return;  // (no barrier follows: this is the range's last tile)

      // ---- tap addresses of the lane's A row (pixel p0 + 32 wave + r32): ring slot of the tap's
      // input pixel (or the zero pixel), XOR-swizzled, unit hh applied
      uint32_t xa[kC64Taps];
      {
        const int p = p0 + 32 * wave + r32;
        const bool okp = p < P;
        const int img = okp ? p / HW : 0;
        const int rem = p - img * HW;
        const int y = rem / a.W;
        const int x = rem - y * a.W;
        int sb = (p0 % kC64Ring) + 32 * wave + r32;
        sb = sb >= kC64Ring ? sb - kC64Ring : sb;
  #pragma unroll
        for (int t = 0; t < kC64Taps; ++t) {
          const int dy = t / 3 - 1, dx = t % 3 - 1;
          const bool ok = okp && (unsigned)(y + dy) < (unsigned)a.H &&
                          (unsigned)(x + dx) < (unsigned)a.W;
          int s = sb + dy * a.W + dx;
          s = s < 0 ? s + kC64Ring : (s >= kC64Ring ? s - kC64Ring : s);
          const uint32_t in = (uint32_t)(kC64RingOff + s * 128 + ((s >> 1) & 7) * 16);
          xa[t] = (ok ? in : (uint32_t)kC64ZeroOff) ^ (uint32_t)(hh * 16);
        }
      }
      load_res(p0);

      // ---- main loop: 36 substeps, fragments one substep ahead
  #pragma unroll
      for (int nb = 0; nb < 2; ++nb)
  #pragma unroll
        for (int r = 0; r < 16; ++r) {
          acc[nb][r] = 0.0f;
          if (FLUSH) acci[nb][r] = 0;
        }
      constexpr int NF = C64_PF + 1;  // fragment buffers
      half8 fa[NF], fb[NF][2];
      auto read_frags = [&](auto sc_, int buf) __attribute__((always_inline)) {
        constexpr int s = decltype(sc_)::value;
        constexpr int t = s / 4, k = s % 4;
        // (xa ^ 32 k: the unit of substep k in the swizzled slot)
        fa[buf] = c64_frag(lds0 + (xa[t] ^ (uint32_t)(32 * k)));
        fb[buf][0] = c64_frag(wbase + (uint32_t)(128 * t + 32 * k));
        fb[buf][1] = c64_frag(wbase + (uint32_t)(32 * kC64WPitch + 128 * t + 32 * k));
      };
      c64_for<0, C64_PF>([&](auto sc_) __attribute__((always_inline)) {
        read_frags(sc_, decltype(sc_)::value);
      });
      int since = 0;
      c64_for<0, kC64Sub>([&](auto sc_) __attribute__((always_inline)) {
        constexpr int s = decltype(sc_)::value;
        constexpr int t = s / 4, k = s % 4, cb = s % NF;
        if constexpr (s + C64_PF < kC64Sub) read_frags(c64_ic<s + C64_PF>{}, (s + C64_PF) % NF);
  #if C64_AB == 2  // timing only: no MFMA (fragments kept live)
        asm volatile("" ::"v"(fa[cb]), "v"(fb[cb][0]), "v"(fb[cb][1]));
  #else
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[cb], fb[cb][0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[cb], fb[cb][1], acc[1], 0, 0, 0);
  #endif
        // keep the order: the prefetched substep's reads, then this substep's MFMAs
        if constexpr (s + C64_PF < kC64Sub) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if constexpr (FLUSH && k == 3 && t + 1 < kC64Taps) {
          if (++since == a.kc_steps) {
            since = 0;
  #pragma unroll
            for (int nb = 0; nb < 2; ++nb)
  #pragma unroll
              for (int r = 0; r < 16; ++r) {
                acci[nb][r] += (int)acc[nb][r];
                acc[nb][r] = 0.0f;
              }
          }
        }
      });
      if constexpr (FLUSH) {
  #pragma unroll
        for (int nb = 0; nb < 2; ++nb)
  #pragma unroll
          for (int r = 0; r < 16; ++r) acci[nb][r] += (int)acc[nb][r];
      }
      if (!LATE) epilogue(p0);
    };
    body(std::true_type{}, pb0);
    for (int p0 = pb0 + kC64Tile; p0 < pe; p0 += kC64Tile) body(std::false_type{}, p0);
    const int p_last = pb0 + (pe - 1 - pb0) / kC64Tile * kC64Tile;
    if (LATE && p_last + 32 * wave < pe) epilogue(p_last);
  };
  if (late)
    run(std::true_type{});
  else
    run(std::false_type{});
}

template <bool RES, bool OUT, int NCODES, bool FLUSH>
hipError_t launch_c64(const ConvArgs& a, int grid, int nblk, size_t lds, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv2d_tp_c64_kernel<RES, OUT, NCODES, FLUSH>),
        hipFuncAttributeMaxDynamicSharedMemorySize, kC64Budget);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  conv2d_tp_c64_kernel<RES, OUT, NCODES, FLUSH>
      <<<dim3((unsigned)grid), kC64Threads, lds, stream>>>(a, nblk);
  return hipGetLastError();
}

template <bool RES, bool OUT, int NCODES>
hipError_t launch_c64_flush(const ConvArgs& a, int grid, int nblk, size_t lds,
                            hipStream_t stream) {
  return a.kc_steps > 0 && a.kc_steps < kC64Taps
             ? launch_c64<RES, OUT, NCODES, true>(a, grid, nblk, lds, stream)
             : launch_c64<RES, OUT, NCODES, false>(a, grid, nblk, lds, stream);
}

template <bool RES, bool OUT>
hipError_t launch_c64_codes(const ConvArgs& a, int grid, int nblk, size_t lds,
                            hipStream_t stream) {
  if (a.codes_b) return launch_c64_flush<RES, OUT, 2>(a, grid, nblk, lds, stream);
  if (a.codes_a) return launch_c64_flush<RES, OUT, 1>(a, grid, nblk, lds, stream);
  return launch_c64_flush<RES, OUT, 0>(a, grid, nblk, lds, stream);
}

int64_t c64_lds_bytes(const ConvArgs& a) { return kC64LutOff + conv_lut_bytes(a); }

}  // namespace

// The shapes and epilogue forms the engine takes: 3x3 stride-1 pad-1 64 -> 64 convs with W <=
// 63 (halo), N*H*W % 32 == 0 (a wave's 32 pixels are all in or all past the tensor) and
// N*H*W*256 < 2^31 (32-bit buffer offsets); ReLU with every code output from its table (or no
// code output), codes channel pitch 64; fp32 output / residual optional.
bool conv_c64_eligible(const ConvArgs& a, int out_nhwc) {
  return out_nhwc && a.Cp == 64 && a.Cout == 64 && a.Kp == kC64Taps * 64 && a.KH == 3 &&
         a.KW == 3 && a.sh == 1 && a.sw == 1 && a.ph == 1 && a.pw == 1 && a.dh == 1 &&
         a.dw == 1 && a.Ho == a.H && a.Wo == a.W && a.W >= 1 && a.W + 1 <= kC64Halo &&
         a.P > 0 && a.P % 32 == 0 && a.P * 256 < ((int64_t)1 << 31) && a.ds_x == nullptr &&
         a.relu == 1 && (a.out != nullptr || a.codes_a != nullptr) &&
         (a.codes_a == nullptr || (a.lut_a > 0 && a.cp_a == 64)) &&
         (a.codes_b == nullptr || (a.codes_a != nullptr && a.lut_b > 0 && a.cp_b == 64)) &&
         a.kc_steps >= 0 && c64_lds_bytes(a) <= kC64Budget;
}

hipError_t launch_conv2d_c64(const ConvArgs& a, hipStream_t stream) {
  if (!conv_c64_eligible(a, 1)) return hipErrorInvalidValue;
  const int nblk = (int)(a.P / 32);  // 32-pixel blocks, split evenly over the workgroups
  int grid = device_cus();
  const char* genv = getenv("TQ_C64_GRID");  // tests: fewer workgroups, longer tile runs
  if (genv && atoi(genv) > 0) grid = atoi(genv);
  if (grid > (nblk + 7) / 8) grid = (nblk + 7) / 8;  // at least a full tile each
  const size_t lds = (size_t)c64_lds_bytes(a);
  if (a.residual)
    return a.out ? launch_c64_codes<true, true>(a, grid, nblk, lds, stream)
                 : launch_c64_codes<true, false>(a, grid, nblk, lds, stream);
  return a.out ? launch_c64_codes<false, true>(a, grid, nblk, lds, stream)
               : launch_c64_codes<false, false>(a, grid, nblk, lds, stream);
}

}  // namespace tq
