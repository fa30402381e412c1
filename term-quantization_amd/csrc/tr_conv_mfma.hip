// Term-pair Conv2d on the CDNA4 matrix cores -- the MFMA engine of the accumulation the
// reference leaves to a dense fp32 cuDNN conv of fake-quantized tensors (tr_layer.py:124-126).
//
// Why a matrix core can do term-pair arithmetic exactly.  A TR'd activation is sf_x * v_x
// and a TR'd weight sf_w * v_w, v the signed sum of the element's kept HESE terms; the
// term-pair sum of one output is sum_k v_x[k] * v_w[k] (tr_conv.hip).  Every v with
// |v| <= 2048 (bitwidth <= 11; ResNet-18 TQ uses 9) is an fp16 value exactly, each product
// of two is exact in fp32 (|v_x v_w| <= 2^22), and a sum of integers stays exact in fp32 as
// long as every partial sum is below 2^24 in magnitude -- in any association order, so the
// order in which v_mfma_f32_32x32x16_f16 adds its products does not matter.  The host bounds
// sum_{k in window} |v_w[m][k]| * 2^db over every window of `kc_steps` K-steps (64 codes
// each) of every weight row (tq_ops.mfma_flush_steps); the kernel moves its fp32 accumulators
// into int32 sums at least that often.  The int32 result is therefore the exact integer
// term-pair sum, bit-identical to the VALU dot2 engine, and the epilogue (tq_epilogue.h)
// rounds it once exactly as that engine does.
//
// Data layout in HBM (fp16 codes, kCodesF16):
//   activation codes  [N][H][W][Cp] fp16 (NHWC, channels padded to Cp % 8 == 0 with 0)
//   weight codes      [Cout_pad][Kp] fp16, k = (kh*KW + kw)*Cp + c, Kp % 64 == 0, zero pad
//   output            fp32, NHWC (fused epilogue) or NCHW
//
// Implicit GEMM: M = Cout, N = output pixels (N*Ho*Wo), K = KH*KW*Cp in K-steps of 64 codes.
// 256 threads = 4 waves, each wave a 64 x 64 output tile = 2 x 2 MFMA 32x32 blocks; the
// block tile is 128 x 128 (2 x 2 waves) or 64 x 256 (1 x 4 waves, Cout <= 64).  A K-step
// stages BM + BN rows x 128 B through LDS (double-buffered, one barrier per step, next
// step's 16-B global loads in flight during the current step's 16 MFMAs per wave).  LDS rows
// are 8 chunks of 16 B with chunk' = chunk ^ ((row >> 1) & 7): the MFMA fragment reads (32
// rows at one chunk per half-wave) and the staging writes (2 rows x 8 chunks per 16 lanes)
// are both bank-conflict free.
#include <stdlib.h>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

namespace tq {

namespace {

template <int BM, int BN>
struct MfmaSmem {
  u32x4 As[2][BM * 8];
  u32x4 Bs[2][BN * 8];
};

// K-steps [k_begin, k_end) of block tile (m0, n0) into acc.  Ends on a barrier.
template <int BM, int BN>
__device__ __forceinline__ void mfma_mainloop(const ConvArgs& a, int m0, int64_t n0,
                                              int k_begin, int k_end, MfmaAcc<2>& acc,
                                              MfmaSmem<BM, BN>& sm) {
  constexpr int WN = BN / 64;  // waves along N
  constexpr int A_ROWS = BM / 32;
  constexpr int B_ROWS = BN / 32;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = (wave / WN) * 64;
  const int wn = (wave % WN) * 64;
  // staging geometry: this thread moves chunk `ch` (8 codes) of rows r0 + 32 i
  const int ch = tid & 7;
  const int r0 = tid >> 3;
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;

  int64_t pbase[B_ROWS];
  int ih0[B_ROWS], iw0[B_ROWS];
#pragma unroll
  for (int r = 0; r < B_ROWS; ++r) {
    const int64_t p = n0 + r0 + 32 * r;
    if (p < a.P) {
      const int64_t img = p / HoWo;
      const int64_t rem = p - img * HoWo;
      const int oh = (int)(rem / a.Wo);
      const int ow = (int)(rem - (int64_t)oh * a.Wo);
      ih0[r] = oh * a.sh - a.ph;
      iw0[r] = ow * a.sw - a.pw;
      pbase[r] = img * a.H;
    } else {
      ih0[r] = -(1 << 28);  // never in bounds
      iw0[r] = 0;
      pbase[r] = 0;
    }
  }
  int ktap, kc, kr, ks;
  {
    const int k0 = k_begin * kKStep + ch * 8;
    ktap = k0 / a.Cp;
    kc = k0 - ktap * a.Cp;
    kr = ktap / a.KW;
    ks = ktap - kr * a.KW;
  }
  const uint16_t* __restrict__ wrow[A_ROWS];
#pragma unroll
  for (int r = 0; r < A_ROWS; ++r)
    wrow[r] = wg + (int64_t)(m0 + r0 + 32 * r) * a.Kp + (int64_t)k_begin * kKStep + ch * 8;
  const int ntaps = a.KH * a.KW;
  const int nsteps = k_end - k_begin;

  if (nsteps <= 0) return;
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const int kc_steps = a.kc_steps > 0 ? a.kc_steps : (1 << 30);
  int since_flush = 0;

  // Global -> registers of one K-step.
  // Out-of-range taps load from the (valid) tensor base and are zeroed when stored to LDS
  // (a select at load time would make the wave wait for the load right there).
  u32x4 ra[A_ROWS], rb[B_ROWS];
  uint32_t okmask = 0;
#define TQ_LOAD_STEP(step)                                                                  \
  {                                                                                         \
    _Pragma("unroll") for (int r = 0; r < A_ROWS; ++r) ra[r] =                              \
        *reinterpret_cast<const u32x4*>(wrow[r] + (int64_t)(step) * kKStep);                \
    okmask = 0;                                                                             \
    _Pragma("unroll") for (int r = 0; r < B_ROWS; ++r) {                                    \
      const int ih = ih0[r] + kr * a.dh;                                                    \
      const int iw = iw0[r] + ks * a.dw;                                                    \
      const bool ok = ktap < ntaps && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;           \
      const uint16_t* src = ok ? xg + ((pbase[r] + ih) * a.W + iw) * a.Cp + kc : xg;         \
      rb[r] = *reinterpret_cast<const u32x4*>(src);                                          \
      okmask |= (uint32_t)ok << r;                                                          \
    }                                                                                       \
    kc += kKStep;                                                                           \
    while (kc >= a.Cp) {                                                                    \
      kc -= a.Cp;                                                                           \
      ++ktap;                                                                               \
      if (++ks == a.KW) {                                                                   \
        ks = 0;                                                                             \
        ++kr;                                                                               \
      }                                                                                     \
    }                                                                                       \
  }
#define TQ_STORE_STEP(buf)                                                                  \
  {                                                                                         \
    _Pragma("unroll") for (int r = 0; r < A_ROWS; ++r) sm.As[buf][swz(r0 + 32 * r, ch)] =   \
        ra[r];                                                                              \
    _Pragma("unroll") for (int r = 0; r < B_ROWS; ++r) sm.Bs[buf][swz(r0 + 32 * r, ch)] =   \
        ((okmask >> r) & 1u) ? rb[r] : (u32x4)0u;                                           \
  }

  TQ_LOAD_STEP(0)
  TQ_STORE_STEP(0)
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    const bool more = step + 1 < nsteps;
    if (more) TQ_LOAD_STEP(step + 1)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 2 * s + hh;
      half8 af[2], bf[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        af[b] = __builtin_bit_cast(half8, sm.As[cur][swz(wm + 32 * b + r32, c)]);
        bf[b] = __builtin_bit_cast(half8, sm.Bs[cur][swz(wn + 32 * b + r32, c)]);
      }
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
          acc.f[bm][bn] =
              __builtin_amdgcn_mfma_f32_32x32x16_f16(af[bm], bf[bn], acc.f[bm][bn], 0, 0, 0);
    }
    if (++since_flush == kc_steps) {
      acc_flush(acc);
      since_flush = 0;
    }
    if (more) TQ_STORE_STEP(cur ^ 1)
    __syncthreads();
  }
#undef TQ_LOAD_STEP
#undef TQ_STORE_STEP
  acc_flush(acc);
}

// Epilogue: lane (r32, hh) of a 32x32 block holds pixel column r32 and Cout rows
// 8*(reg>>2) + 4*hh + (reg&3), i.e. 4 consecutive channels per register quad.
template <int BM, int BN, bool OUT_NHWC>
__device__ __forceinline__ void mfma_epilogue(const ConvArgs& a, int m0, int64_t n0,
                                              const MfmaAcc<2>& acc) {
  constexpr int WN = BN / 64;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave / WN) * 64;
  const int wn = (wave % WN) * 64;
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  if (OUT_NHWC) {
    const bool vec = (a.Cout & 3) == 0;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int co = m0 + wm + 32 * bm + 8 * q + 4 * hh;
        if (co >= a.Cout) continue;
        coef_t sc[4], sh[4];
        load_coef(a, co, sc, sh);
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) {
          const int64_t p = n0 + wn + 32 * bn + r32;
          if (p >= a.P) continue;
          const int acc4[4] = {acc.i[bm][bn][4 * q], acc.i[bm][bn][4 * q + 1],
                               acc.i[bm][bn][4 * q + 2], acc.i[bm][bn][4 * q + 3]};
          emit4_nhwc(a, p, co, acc4, sc, sh, vec);
        }
      }
    }
  } else {
    const int64_t HoWo = (int64_t)a.Ho * a.Wo;
#pragma unroll
    for (int bn = 0; bn < 2; ++bn) {
      const int64_t p = n0 + wn + 32 * bn + r32;
      if (p >= a.P) continue;
      const int64_t img = p / HoWo;
      const int64_t rem = p - img * HoWo;
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = m0 + wm + 32 * bm + 8 * (r >> 2) + 4 * hh + (r & 3);
          if (co >= a.Cout) continue;
          const coef_t sh = (coef_t)(a.bias ? (double)a.bias[co] : 0.0);
          a.out[(img * a.Cout + co) * HoWo + rem] =
              fold_acc(acc.i[bm][bn][r], (coef_t)a.scale, sh);
        }
    }
  }
}

template <int BM, int BN, bool OUT_NHWC>
__global__ __launch_bounds__(256, 2) void conv2d_tp_mfma_kernel(ConvArgs a) {
  static_assert((BM / 64) * (BN / 64) == 4, "4 waves of 64 x 64");
  __shared__ __attribute__((aligned(16))) MfmaSmem<BM, BN> sm;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = (a.Cout + BM - 1) / BM;
  const int m0 = (tile % mt) * BM;
  const int64_t n0 = (int64_t)(tile / mt) * BN;
  MfmaAcc<2> acc;
  acc_zero(acc);
  mfma_mainloop<BM, BN>(a, m0, n0, 0, a.Kp / kKStep, acc, sm);
  mfma_epilogue<BM, BN, OUT_NHWC>(a, m0, n0, acc);
}

// ---------------------------------------------------------------------------------------
// Pipelined engine (Cp % 64 == 0: every K-step lies inside one filter tap).  Operands go
// global -> LDS directly (global_load_lds_dwordx4, no staging registers) into an NS-deep
// ring of K-step images; stage s+NS-1 is issued while stage s is multiplied, retired by a
// counted vmcnt + raw s_barrier (never a vmcnt(0) inside the loop).  The LDS image of a
// wave-instruction is lane-linear (base + lane*16), so the bank swizzle moves to the SOURCE:
// lane l fills slot (l & 7) of row r with logical chunk (l & 7) ^ ((r >> 1) & 7), and the
// fragment reads apply the same involution (swz).  Out-of-range taps and pixels read a
// zero page.  The epilogue transposes each wave's 64 x 64 int32 tile through the freed LDS
// ring so every store instruction writes whole 256-byte pixel rows (channels_last).
constexpr int pipe_threads(int bm, int bn) { return (bm / 64) * (bn / 64) * 64; }

template <int BM, int BN, int NS>
struct PipeCfg {
  static constexpr int WAVES = (BM / 64) * (BN / 64);
  static constexpr int THREADS = WAVES * 64;
  static constexpr int WN = BN / 64;
  static constexpr int STAGE = (BM + BN) * 8;  // u32x4 per K-step image
  static constexpr int AI = BM / 8 / WAVES;    // A wave-instructions per wave and stage
  static constexpr int BI = BN / 8 / WAVES;    // B wave-instructions per wave and stage
  static constexpr int LPW = AI + BI;          // vmcnt units per wave and stage
  static constexpr int LDS = NS * STAGE > WAVES * 1024 ? NS * STAGE : WAVES * 1024;
  static_assert(AI >= 1 && BI >= 1 && AI * WAVES * 8 == BM && BI * WAVES * 8 == BN, "rows");
  static_assert(LPW * (NS - 2) <= 63, "vmcnt range");
};

template <int BM, int BN, int NS, bool OUT_NHWC, int EPI = 0>
__global__ __launch_bounds__(pipe_threads(BM, BN), 1) void conv2d_tp_mfma_pipe_kernel(
    ConvArgs a) {
  using C = PipeCfg<BM, BN, NS>;
  __shared__ __attribute__((aligned(16))) u32x4 lds[C::LDS];
  extern __shared__ __attribute__((aligned(16))) uint16_t dyn_lut[];  // epilogue code tables
  uint16_t *lut_a, *lut_b;
  conv_luts(a, dyn_lut, lut_a, lut_b);  // read only after the epilogue's barrier
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = (a.Cout + BM - 1) / BM;
  const int64_t ntn = (a.P + BN - 1) / BN;
  const int m0 = (int)(a.m_slow ? tile / ntn : tile % mt) * BM;
  const int64_t n0 = (a.m_slow ? tile % ntn : tile / mt) * BN;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave / C::WN) * 64;
  const int wn = (wave % C::WN) * 64;
  const int lrow = lane >> 3;  // row within a wave-instruction's 8 rows
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page) + lane * 8;

  // A rows (weights): fixed pointers, advanced by 64 codes per K-step.
  const uint16_t* arow[C::AI];
#pragma unroll
  for (int i = 0; i < C::AI; ++i) {
    const int r = (wave * C::AI + i) * 8 + lrow;
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    arow[i] = wg + (int64_t)(m0 + r) * a.Kp + c * 8;
  }
  // B rows (output pixels): element offset of this lane's chunk at the pixel's input
  // origin, and a bit mask of the filter taps that fall inside the input (KH*KW <= 64).
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  int64_t boff[C::BI];
  uint64_t tapmask[C::BI];
#pragma unroll
  for (int i = 0; i < C::BI; ++i) {
    const int r = (wave * C::BI + i) * 8 + lrow;  // B row = pixel n0 + r
    const int chk = ((lane & 7) ^ (((BM + r) >> 1) & 7)) * 8;
    const int64_t p = n0 + r;
    boff[i] = 0;
    tapmask[i] = 0;
    if (p < a.P) {
      const int64_t img = p / HoWo;
      const int64_t rem = p - img * HoWo;
      const int oh = (int)(rem / a.Wo);
      const int ow = (int)(rem - (int64_t)oh * a.Wo);
      const int ih0 = oh * a.sh - a.ph;
      const int iw0 = ow * a.sw - a.pw;
      boff[i] = ((img * a.H + ih0) * a.W + iw0) * a.Cp + chk;
      for (int kr = 0; kr < a.KH; ++kr) {
        const int ih = ih0 + kr * a.dh;
        if (ih < 0 || ih >= a.H) continue;
        for (int ks = 0; ks < a.KW; ++ks) {
          const int iw = iw0 + ks * a.dw;
          if (iw >= 0 && iw < a.W) tapmask[i] |= 1ull << (kr * a.KW + ks);
        }
      }
    }
  }
  const int nsteps = a.Kp / kKStep;

  // Issue K-step `st` into ring slot `slot`.  Cp % 64 == 0, so the step lies in one tap:
  // the tap and its element offset are wave-uniform (scalar) values.
  auto issue = [&](int st, int slot) {
    u32x4* img = lds + slot * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::AI; ++i)
      glds16(arow[i] + (int64_t)st * kKStep, img + (wave * C::AI + i) * 64);
    const int k0 = st * kKStep;
    const int tap = k0 / a.Cp;
    const int cb = k0 - tap * a.Cp;
    const int kr = tap / a.KW;
    const int ks = tap - kr * a.KW;
    const int64_t toff = ((int64_t)kr * a.dh * a.W + (int64_t)ks * a.dw) * a.Cp + cb;
#pragma unroll
    for (int i = 0; i < C::BI; ++i) {
      const bool ok = (tapmask[i] >> tap) & 1ull;  // tap >= KH*KW (K padding): bit clear
      const uint16_t* src = ok ? xg + (boff[i] + toff) : zero;
      glds16(src, img + BM * 8 + (wave * C::BI + i) * 64);
    }
  };

  MfmaAcc<2> acc;
  acc_zero(acc);
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const int kc_steps = a.kc_steps > 0 ? a.kc_steps : (1 << 30);
  int since_flush = 0;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nsteps) issue(s, s);
  for (int s = 0; s < nsteps; ++s) {
    // retire stage s, leaving min(nsteps - 1 - s, NS - 2) later stages in flight
    const int ahead = min(nsteps - 1 - s, NS - 2);
    if (ahead >= 2) TQ_WAIT_VM(2 * C::LPW);
    else if (ahead == 1) TQ_WAIT_VM(C::LPW);
    else TQ_WAIT_VM(0);
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < nsteps) issue(s + NS - 1, (s + NS - 1) % NS);
    const u32x4* img = lds + (s % NS) * C::STAGE;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 2 * k + hh;
      half8 af[2], bf[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        af[b] = __builtin_bit_cast(half8, img[swz(wm + 32 * b + r32, c)]);
        bf[b] = __builtin_bit_cast(half8, img[swz(BM + wn + 32 * b + r32, c)]);
      }
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
          acc.f[bm][bn] =
              __builtin_amdgcn_mfma_f32_32x32x16_f16(af[bm], bf[bn], acc.f[bm][bn], 0, 0, 0);
    }
    if (++since_flush == kc_steps) {
      acc_flush(acc);
      since_flush = 0;
    }
  }
  acc_flush(acc);

  if (!OUT_NHWC) {
    mfma_epilogue<BM, BN, false>(a, m0, n0, acc);  // NCHW: lanes along pixels already
    return;
  }
  // Transpose each wave's 64 (Cout) x 64 (pixel) int32 tile through LDS:
  // [pixel][16 slots of 4 channels], slot ^= pixel & 15 (conflict-free both ways).
  __syncthreads();  // every wave is done with the ring
  u32x4* t = lds + wave * 1024;
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int bn = 0; bn < 2; ++bn)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int px = 32 * bn + r32;
        const int slot = 8 * bm + 2 * q + hh;
        u32x4 v;
        v.x = (uint32_t)acc.i[bm][bn][4 * q];
        v.y = (uint32_t)acc.i[bm][bn][4 * q + 1];
        v.z = (uint32_t)acc.i[bm][bn][4 * q + 2];
        v.w = (uint32_t)acc.i[bm][bn][4 * q + 3];
        t[px * 16 + (slot ^ (px & 15))] = v;
      }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile is in LDS
  __builtin_amdgcn_wave_barrier();
  const bool vec = (a.Cout & 3) == 0;
  const int slot = lane & 15;
  const int co = m0 + wm + 4 * slot;
  if (co < a.Cout) {
    coef_t sc[4], sh[4];
    load_coef(a, co, sc, sh);
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int px = it * 4 + (lane >> 4);
      const int64_t p = n0 + wn + px;
      if (p >= a.P) continue;
      const u32x4 v = t[px * 16 + (slot ^ (px & 15))];
      const int acc4[4] = {(int)v.x, (int)v.y, (int)v.z, (int)v.w};
      if constexpr (EPI == 1)  // (epilogue_form 1 without a residual)
        emit4_relu_lut(a, p, co, acc4, sc, sh, make_float4(0.f, 0.f, 0.f, 0.f), lut_a, lut_b);
      else if constexpr (EPI == 2)
        emit4_identity(a, p, co, acc4, sc, sh);
      else
        emit4_nhwc(a, p, co, acc4, sc, sh, vec, lut_a, lut_b);
    }
  }
}

template <int BM, int BN, int NS, int EPI>
hipError_t launch_pipe_nhwc(const ConvArgs& b, dim3 grid, size_t dyn, hipStream_t stream) {
  using C = PipeCfg<BM, BN, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&conv2d_tp_mfma_pipe_kernel<BM, BN, NS, true, EPI>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 2 * kLutMax * 2);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  conv2d_tp_mfma_pipe_kernel<BM, BN, NS, true, EPI><<<grid, C::THREADS, dyn, stream>>>(b);
  return hipGetLastError();
}

template <int BM, int BN, int NS>
hipError_t launch_pipe_cfg(const ConvArgs& a, int out_nhwc, hipStream_t stream) {
  using C = PipeCfg<BM, BN, NS>;
  const int64_t tiles = ((a.P + BN - 1) / BN) * ((a.Cout + BM - 1) / BM);
  const dim3 grid((unsigned)tiles);
  ConvArgs b = a;
  if ((int64_t)C::LDS * 16 + conv_lut_bytes(b) > 160 * 1024) b.lut_a = b.lut_b = 0;
  if (!out_nhwc) {
    b.lut_a = b.lut_b = 0;
    conv2d_tp_mfma_pipe_kernel<BM, BN, NS, false><<<grid, C::THREADS, 0, stream>>>(b);
    return hipGetLastError();
  }
  const size_t dyn = (size_t)conv_lut_bytes(b);
  // the specialised epilogues (the ReLU one without a residual: the generic path loads it)
  const int form = epilogue_form(b);
  if (form == 1 && b.residual == nullptr)
    return launch_pipe_nhwc<BM, BN, NS, 1>(b, grid, dyn, stream);
  if (form == 2) return launch_pipe_nhwc<BM, BN, NS, 2>(b, grid, dyn, stream);
  return launch_pipe_nhwc<BM, BN, NS, 0>(b, grid, dyn, stream);
}

template <int BM, int BN>
hipError_t launch_mfma_cfg(const ConvArgs& a, int out_nhwc, hipStream_t stream) {
  const int64_t tiles = ((a.P + BN - 1) / BN) * ((a.Cout + BM - 1) / BM);
  const dim3 grid((unsigned)tiles);
  if (out_nhwc)
    conv2d_tp_mfma_kernel<BM, BN, true><<<grid, 256, 0, stream>>>(a);
  else
    conv2d_tp_mfma_kernel<BM, BN, false><<<grid, 256, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace

// Configs (1-based through ConvArgs.config): 1-2 register-staged (any Cp), 3-6 pipelined
// gather (Cp % 64 == 0 and KH*KW <= 64; else 1/2), 7-8 input patch (tr_conv_patch.hip:
// stride 1, KH*KW >= 2, NHWC out; else the gather default).
// 9-10 direct (tr_conv_direct.hip: Cp % 64 == 0, NHWC out; 128 x 128 / 64 x 128 tiles).
// 11 row strip (tr_conv_strip.hip: 3x3/1, 64 -> 64 channels, W <= 56; else the default).
// 12 persistent pointwise (tr_conv_direct.hip: 1x1, K <= 3 K-steps; else the default).
// 13 tap ring (tr_conv_ring.hip: 3x3/1 "same", Cp % 64 == 0, Wo <= 256; else the default).
// 14 expand (tr_conv_xp.hip: 1x1/1, one or two K-steps, weights <= 64 KB; else the default).
// 15 Cout-64 pixel ring (tr_conv_c64.hip: 3x3/1 "same", 64 -> 64, ReLU + table codes; else the
// default).
int conv_mfma_num_configs() { return 15; }

hipError_t launch_conv2d_mfma(const ConvArgs& a_in, int out_nhwc, hipStream_t stream) {
  if (a_in.P == 0 || a_in.Cout == 0) return hipSuccess;
  ConvArgs a = a_in;
  // Tile order: with the Cout tile as the slow index, an XCD's contiguous run of tiles
  // shares one weight slice in its L2 (speed only).  TQ_MSLOW=0/1 overrides (A/B).
  const char* ms = getenv("TQ_MSLOW");  // read per launch: tests switch it
  a.m_slow = ms ? atoi(ms) : 0;
  const bool pipe_ok = a.Cp % kKStep == 0 && a.KH * a.KW <= 64;
  int cfg = a.config > 0 ? a.config - 1 : -1;
  // TQ_CONFIG_STRICT=1 (tests): a requested engine config that cannot take the conv is an
  // error instead of a quiet fall-back to the default engine (read per launch)
  const char* strict_env = getenv("TQ_CONFIG_STRICT");
  const bool strict = strict_env && atoi(strict_env) == 1;
  static const char* ab = getenv("TQ_AB");
  a.ab = ab ? atoi(ab) : 0;
  static const char* dir = getenv("TQ_DIRECT");  // A/B override (tools only): 0 off, 1/2 MB
  if (cfg < 0 && dir && atoi(dir) > 0) cfg = atoi(dir) == 1 ? 9 : 8;
  // 1x1 convs with K <= 3 K-steps: the persistent pointwise engine on request only (config
  // 12, or TQ_PW=1): measured slower than the direct engine's one-shot tiles (fused
  // MobileNet-V2 1x1 convs 92 vs 77 us, EfficientNet-b0 142 vs 108 us: r03g), 2 persistent
  // workgroups per CU hide less latency than 4 resident one-shot ones
  const char* pw = getenv("TQ_PW");  // read per launch: tests switch it
  if ((cfg == 11 || (cfg < 0 && pw && atoi(pw) == 1)) && conv_pw_eligible(a, out_nhwc))
    return launch_conv2d_pw(a, stream);
  if (cfg == 11 && strict) return hipErrorInvalidValue;
  // expand engine: config 14, and the default for the 1x1 convs it takes (MobileNet-V2 /
  // EfficientNet-b0 expand convs: 112^2 x 16 -> 96 534 -> 408 us, tools/ab/gpu_expand_probe.sh);
  // TQ_XP=0 / 1 forces it off / on (read per launch: tests switch it)
  const char* xp = getenv("TQ_XP");
  const bool xp_on = xp ? atoi(xp) == 1 : true;
  if ((cfg == 13 || (cfg < 0 && xp_on)) && conv_xp_eligible(a, out_nhwc))
    return launch_conv2d_xp(a, stream);
  if (cfg == 13) {
    if (strict) return hipErrorInvalidValue;
    cfg = -1;
  }
  if (a.relu == kActSwish) {  // the swish epilogue exists on the direct engine only
    if (!conv_direct_eligible(a, out_nhwc)) return hipErrorInvalidValue;
    return launch_conv2d_direct(a, 1, stream);
  }
  if (a.ds_x) {  // a fused downsample phase: the direct engine only
    if (!conv_direct_eligible(a, out_nhwc)) return hipErrorInvalidValue;
    return launch_conv2d_direct(a, 1, stream);
  }
  // tap-ring engine: config 13, and the default for the 3x3 stride-1 convs with Cout >= 128
  // (ResNet-18 layer2/3/4: 1.1-1.5x the direct / input-patch engines, tools/gpu_ring_probe.sh);
  // TQ_RING=0 / 1 forces it off / on (read per launch: tests switch it)
  const char* ring = getenv("TQ_RING");
  const bool ring_on = ring ? atoi(ring) == 1 : a.Cout >= 128;
  if ((cfg == 12 || (cfg < 0 && ring_on)) && conv_ring_eligible(a, out_nhwc))
    return launch_conv2d_ring(a, stream);
  if (cfg == 12) {
    if (strict) return hipErrorInvalidValue;
    cfg = -1;
  }
  // Cout-64 pixel-ring engine: config 15, and the default for the layer-1 convs it takes
  // (TQ_C64=0 / 1 forces it off / on; read per launch: tests switch it)
  // (its epilogues are all specialised ReLU + table forms: TQ_EPI_FAST=0, the generic-epilogue
  // A/B, leaves these convs to the strip / direct engines)
  const char* c64 = getenv("TQ_C64");
  const char* epi_fast = getenv("TQ_EPI_FAST");
  const bool c64_on = c64 ? atoi(c64) == 1 : !(epi_fast && atoi(epi_fast) == 0);
  if ((cfg == 14 || (cfg < 0 && c64_on)) && conv_c64_eligible(a, out_nhwc))
    return launch_conv2d_c64(a, stream);
  if (cfg == 14) {
    if (strict) return hipErrorInvalidValue;
    cfg = -1;
  }
  static const char* strip = getenv("TQ_STRIP");  // A/B override (tools only): 0 off
  if (cfg == 10 || (cfg < 0 && !(strip && atoi(strip) == 0))) {
    if (conv_strip_eligible(a, out_nhwc)) return launch_conv2d_strip(a, stream);
    if (cfg == 10) {
      if (strict) return hipErrorInvalidValue;
      cfg = -1;
    }
  }
  // measured (tools/layer_times.py, ResNet-18 batch 256): the direct engine wins where the
  // fused epilogue dominates -- Cout <= 128 (layer1/2) and 1x1 convs
  if (cfg < 0 && !(dir && atoi(dir) == 0) && conv_direct_eligible(a, out_nhwc) &&
      (a.Cout <= 128 || a.KH * a.KW == 1))
    cfg = 9;
  if (cfg >= 8) {
    if (conv_direct_eligible(a, out_nhwc))
      return launch_conv2d_direct(a, cfg == 8 ? 2 : 1, stream);
    if (strict && a.config > 0) return hipErrorInvalidValue;
    cfg = -1;
  }
  if (cfg >= 6 || cfg < 0) {
    if (conv_patch_eligible(a, out_nhwc)) {
      const int mb = cfg == 6 ? 2 : cfg == 7 ? 1 : (a.Cout <= 64 ? 1 : 2);
      return launch_conv2d_patch(a, mb, stream);
    }
    if (strict && cfg >= 6) return hipErrorInvalidValue;
    cfg = -1;
  }
  // measured (tools/microbench.py --sweep): 64 x 512 (8 waves) for Cout <= 64, else 128 x 256
  if (cfg < 0) cfg = pipe_ok ? (a.Cout <= 64 ? 5 : 2) : (a.Cout <= 64 ? 1 : 0);
  if (cfg >= 2 && !pipe_ok) cfg = a.Cout <= 64 ? 1 : 0;
  switch (cfg) {
    case 0: return launch_mfma_cfg<128, 128>(a, out_nhwc, stream);
    case 1: return launch_mfma_cfg<64, 256>(a, out_nhwc, stream);
    case 2: return launch_pipe_cfg<128, 256, 3>(a, out_nhwc, stream);
    case 3: return launch_pipe_cfg<64, 256, 3>(a, out_nhwc, stream);
    case 4: return launch_pipe_cfg<128, 128, 3>(a, out_nhwc, stream);
    default: return launch_pipe_cfg<64, 512, 2>(a, out_nhwc, stream);
  }
}

}  // namespace tq
