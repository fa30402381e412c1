// Term-pair Conv2d on CDNA4 VALU (no MFMA) -- the accumulation the reference leaves to a
// dense fp32 cuDNN conv of fake-quantized tensors (tr_layer.py:124-126).
//
// A TR'd activation is sf_x * v_x and a TR'd weight is sf_w * v_w with v_x, v_w the signed
// sums of their kept HESE terms.  The term-pair sum of one output is
//     sum_k sum_{tx in terms(x_k)} sum_{tw in terms(w_k)} tx * tw  ==  sum_k v_x[k] * v_w[k]
// exactly (shift-adds of +-2^(ex+ew) are integer products of the term sums), so the kernel
// accumulates integer products of int16 term sums with packed v_dot2c_i32_i16 (two term-sum
// products per lane-op, exact int32 accumulation), and rounds once in the epilogue:
//     y = fp32( double(acc) * (double(sf_x) * double(sf_w)) ) + bias.
//
// Data layout in HBM:
//   activation codes  [N][H][W][Cp] int16 (NHWC, channels padded to Cp % 8 == 0 with 0)
//   weight codes      [Cout_pad][Kp] int16, k = (kh*KW + kw)*Cp + c, Kp % 32 == 0, zero pad
//   output            fp32, NCHW or NHWC (channels_last), bias optional
//
// Implicit GEMM: M = Cout, N = output pixels (N*Ho*Wo), K = KH*KW*Cp, K-step 32 (16 int16
// pairs).  256 threads, each owns an 8 (Cout) x 8 (pixel) int32 accumulator tile; operands
// are staged through LDS as [k-pair][m] / [k-pair][n] dwords (double-buffered, one barrier
// per K-step) and read with ds_read_b128; the next K-step's global loads are issued before
// the current step's 1024 dot2 per lane.
#include <cmath>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"

namespace tq {

namespace {

__device__ __forceinline__ int dot2(int a, int b, int c) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, a), __builtin_bit_cast(s2, b), c, false);
}

// LDS image of one K-step (double-buffered): [k-pair][m] and [k-pair][n] dwords.
template <int BM, int BN>
struct TileSmem {
  int32_t As[2][16][BM];
  int32_t Bs[2][16][BN];
};

// Accumulate K-steps [k_begin, k_end) of output tile (m0, n0) into acc (8 Cout x 8 pixels
// per lane).  Operands are staged through LDS, the next step's 16-B global loads are in
// flight during the current step's 1024 dot2 per lane, one barrier per step; ends on a
// barrier, so the LDS image may be reused by the next call.
template <int BM, int BN, int THREADS>
__device__ __forceinline__ void tile_mainloop(const ConvArgs& a, int m0, int64_t n0,
                                              int k_begin, int k_end, int (&acc)[8][8],
                                              TileSmem<BM, BN>& sm) {
  constexpr int TX = BN / 8;
  constexpr int ROWS = THREADS / 4;  // rows (m or n) per load slot
  constexpr int A_LOADS = BM / ROWS;
  constexpr int B_LOADS = BN / ROWS;
  const int tid = threadIdx.x;
  const int tx = tid % TX;
  const int ty = tid / TX;
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  // Load-slot geometry: a 16-B vector = 8 int16 codes = 4 k-pairs.  Lanes 0-15 of each
  // 16-lane quarter take 16 rows at the same k-vector v, so one ds_write_b32 instruction
  // puts at most 2 lanes on a bank.
  const int v = (tid >> 4) & 3;
  const int rowl = (tid & 15) + 16 * (tid >> 6);

  int64_t pbase[B_LOADS];
  int ih0[B_LOADS], iw0[B_LOADS];
#pragma unroll
  for (int r = 0; r < B_LOADS; ++r) {
    const int64_t p = n0 + rowl + ROWS * r;
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
  // this lane's k-vector position: k = (kr*KW + ks)*Cp + kc
  int ktap, kc, kr, ks;
  {
    const int k0 = k_begin * 32 + v * 8;
    ktap = k0 / a.Cp;
    kc = k0 - ktap * a.Cp;
    kr = ktap / a.KW;
    ks = ktap - kr * a.KW;
  }
  const int16_t* __restrict__ wrow[A_LOADS];
#pragma unroll
  for (int r = 0; r < A_LOADS; ++r)
    wrow[r] = a.w + (int64_t)(m0 + rowl + ROWS * r) * a.Kp + (int64_t)k_begin * 32 + v * 8;
  const int ntaps = a.KH * a.KW;
  const int nsteps = k_end - k_begin;

  int4 ra[A_LOADS], rb[B_LOADS];
  auto load_tile = [&](int step) {
#pragma unroll
    for (int r = 0; r < A_LOADS; ++r)
      ra[r] = *reinterpret_cast<const int4*>(wrow[r] + step * 32);
#pragma unroll
    for (int r = 0; r < B_LOADS; ++r) {
      rb[r] = make_int4(0, 0, 0, 0);
      if (ktap < ntaps) {
        const int ih = ih0[r] + kr * a.dh;
        const int iw = iw0[r] + ks * a.dw;
        if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
          rb[r] = *reinterpret_cast<const int4*>(a.x + ((pbase[r] + ih) * a.W + iw) * a.Cp + kc);
      }
    }
    kc += 32;  // advance this lane's k-vector by 32 codes
    while (kc >= a.Cp) {
      kc -= a.Cp;
      ++ktap;
      if (++ks == a.KW) {
        ks = 0;
        ++kr;
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int r = 0; r < A_LOADS; ++r) {
      const int m = rowl + ROWS * r;
      sm.As[buf][v * 4 + 0][m] = ra[r].x;
      sm.As[buf][v * 4 + 1][m] = ra[r].y;
      sm.As[buf][v * 4 + 2][m] = ra[r].z;
      sm.As[buf][v * 4 + 3][m] = ra[r].w;
    }
#pragma unroll
    for (int r = 0; r < B_LOADS; ++r) {
      const int n = rowl + ROWS * r;
      sm.Bs[buf][v * 4 + 0][n] = rb[r].x;
      sm.Bs[buf][v * 4 + 1][n] = rb[r].y;
      sm.Bs[buf][v * 4 + 2][n] = rb[r].z;
      sm.Bs[buf][v * 4 + 3][n] = rb[r].w;
    }
  };

  if (nsteps <= 0) return;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if (step + 1 < nsteps) load_tile(step + 1);
#pragma unroll 2
    for (int kk = 0; kk < 16; ++kk) {
      const int4 a0 = *reinterpret_cast<const int4*>(&sm.As[cur][kk][ty * 4]);
      const int4 a1 = *reinterpret_cast<const int4*>(&sm.As[cur][kk][BM / 2 + ty * 4]);
      const int4 b0 = *reinterpret_cast<const int4*>(&sm.Bs[cur][kk][tx * 4]);
      const int4 b1 = *reinterpret_cast<const int4*>(&sm.Bs[cur][kk][BN / 2 + tx * 4]);
      const int av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const int bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = dot2(av[i], bv[j], acc[i][j]);
    }
    if (step + 1 < nsteps) store_tile(cur ^ 1);
    __syncthreads();
  }
}

// Epilogue of one tile: one rounding of the exact integer sums (fp64 scale/shift), 16-byte
// stores of 4 consecutive channels (NHWC, with the fused residual/ReLU/next-layer codes) or
// 4 consecutive pixels (NCHW).
template <int BM, int BN, int THREADS, bool OUT_NHWC>
__device__ __forceinline__ void tile_epilogue(const ConvArgs& a, int m0, int64_t n0,
                                              const int (&acc)[8][8]) {
  constexpr int TX = BN / 8;
  const int tx = threadIdx.x % TX;
  const int ty = threadIdx.x / TX;
  if (OUT_NHWC) {
    const bool vec = (a.Cout & 3) == 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int co = m0 + h * (BM / 2) + ty * 4;
      if (co >= a.Cout) continue;
      coef_t sc[4], sh[4];
      load_coef(a, co, sc, sh);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t p = n0 + (j < 4 ? tx * 4 + j : BN / 2 + tx * 4 + (j - 4));
        if (p >= a.P) continue;
        const int acc4[4] = {acc[h * 4][j], acc[h * 4 + 1][j], acc[h * 4 + 2][j],
                             acc[h * 4 + 3][j]};
        emit4_nhwc(a, p, co, acc4, sc, sh, vec);
      }
    }
  } else {
    const int64_t HoWo = (int64_t)a.Ho * a.Wo;
    const bool vec = (HoWo & 3) == 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int co = m0 + (i < 4 ? ty * 4 + i : BM / 2 + ty * 4 + (i - 4));
      if (co >= a.Cout) continue;
      const coef_t sc = (coef_t)a.scale;
      const coef_t sh = (coef_t)(a.bias ? (double)a.bias[co] : 0.0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t p0 = n0 + h * (BN / 2) + tx * 4;
        float y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = fold_acc(acc[i][h * 4 + j], sc, sh);
        if (vec && p0 + 3 < a.P) {
          const int64_t img = p0 / HoWo;
          *reinterpret_cast<float4*>(a.out + (img * a.Cout + co) * HoWo + (p0 - img * HoWo)) =
              make_float4(y[0], y[1], y[2], y[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t p = p0 + j;
            if (p >= a.P) continue;
            const int64_t img = p / HoWo;
            a.out[(img * a.Cout + co) * HoWo + (p - img * HoWo)] = y[j];
          }
        }
      }
    }
  }
}

// Data-parallel schedule: one tile (or one K-split of a tile) per block.  SPLIT: the block
// adds its partial sums into the int32 workspace (exact, order-independent) and
// conv_finalize_kernel applies the epilogue.
template <int BM, int BN, int THREADS, bool OUT_NHWC, bool SPLIT, int OCC>
__global__ __launch_bounds__(THREADS, OCC) void conv2d_tp_kernel(ConvArgs a) {
  static_assert((BM / 8) * (BN / 8) == THREADS, "8x8 accumulators per thread");
  __shared__ __attribute__((aligned(16))) TileSmem<BM, BN> sm;
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int splits = SPLIT ? a.splits : 1;
  const int split = item % splits;
  const int tile = item / splits;
  const int mt = (a.Cout + BM - 1) / BM;
  const int m0 = (tile % mt) * BM;
  const int64_t n0 = (int64_t)(tile / mt) * BN;
  const int nsteps_all = a.Kp / 32;
  const int k_begin = (int)((int64_t)split * nsteps_all / splits);
  const int k_end = (int)((int64_t)(split + 1) * nsteps_all / splits);

  int acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0;
  tile_mainloop<BM, BN, THREADS>(a, m0, n0, k_begin, k_end, acc, sm);

  if (SPLIT) {
    constexpr int TX = BN / 8;
    const int tx = threadIdx.x % TX;
    const int ty = threadIdx.x / TX;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int co = m0 + h * (BM / 2) + ty * 4;
      if (co >= a.Cout) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t p = n0 + (j < 4 ? tx * 4 + j : BN / 2 + tx * 4 + (j - 4));
        if (p >= a.P) continue;
        int* dst = a.ws + p * a.Cout + co;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (co + i < a.Cout) atomicAdd(dst + i, acc[h * 4 + i][j]);
      }
    }
    return;
  }
  tile_epilogue<BM, BN, THREADS, OUT_NHWC>(a, m0, n0, acc);
}

// Stream-K schedule (NHWC outputs): exactly one resident round of G blocks; the tiles x
// K-steps work units are divided evenly, block b taking units [b*U/G, (b+1)*U/G) in tile
// order.  Whole tiles get the epilogue at once; the (at most two) partial tiles at the ends
// of a block's range park their int32 partial sums in the block's two slabs with plain
// 16-byte stores, and conv2d_tp_streamk_fixup sums a tile's slabs and runs its epilogue.
// No atomics, no inter-block synchronisation inside a launch.
__device__ __forceinline__ int64_t sk_bound(int64_t b, int64_t U, int64_t G) {
  return b * U / G;
}

template <int BM, int BN, int THREADS>
__device__ __forceinline__ int32_t* sk_slab(const ConvArgs& a, int64_t b, int slot) {
  return a.ws + (b * 2 + slot) * (int64_t)(BM * BN);
}

template <int BM, int BN, int THREADS, int OCC>
__global__ __launch_bounds__(THREADS, OCC) void conv2d_tp_streamk_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) TileSmem<BM, BN> sm;
  const int64_t G = gridDim.x;
  const int64_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = (a.Cout + BM - 1) / BM;
  const int64_t tiles = ((a.P + BN - 1) / BN) * mt;
  const int nsteps = a.Kp / 32;
  const int64_t U = tiles * nsteps;
  const int64_t u0 = sk_bound(b, U, G), u1 = sk_bound(b + 1, U, G);
  int64_t u = u0;
  while (u < u1) {
    const int64_t t = u / nsteps;
    const int k0 = (int)(u - t * nsteps);
    const int k1 = (int)min((int64_t)nsteps, (int64_t)k0 + (u1 - u));
    const int m0 = (int)(t % mt) * BM;
    const int64_t n0 = (t / mt) * BN;
    int acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0;
    tile_mainloop<BM, BN, THREADS>(a, m0, n0, k0, k1, acc, sm);
    if (k0 == 0 && k1 == nsteps) {
      tile_epilogue<BM, BN, THREADS, true>(a, m0, n0, acc);
    } else {
      int4* slab = reinterpret_cast<int4*>(sk_slab<BM, BN, THREADS>(a, b, u == u0 ? 0 : 1));
#pragma unroll
      for (int q = 0; q < 16; ++q)
        slab[q * THREADS + threadIdx.x] =
            make_int4(acc[q >> 1][(q & 1) * 4 + 0], acc[q >> 1][(q & 1) * 4 + 1],
                      acc[q >> 1][(q & 1) * 4 + 2], acc[q >> 1][(q & 1) * 4 + 3]);
    }
    u += k1 - k0;
  }
}

// One block per inner boundary b (1..G-1): if the boundary splits a tile and is the first
// boundary inside it, sum that tile's slabs from every block whose range touches it (a
// tile is slot 0 of a block iff it is the block's first tile) and apply the epilogue.
template <int BM, int BN, int THREADS>
__global__ __launch_bounds__(THREADS) void conv2d_tp_streamk_fixup(ConvArgs a, int G) {
  const int64_t b = (int64_t)blockIdx.x + 1;
  const int mt = (a.Cout + BM - 1) / BM;
  const int64_t tiles = ((a.P + BN - 1) / BN) * mt;
  const int nsteps = a.Kp / 32;
  const int64_t U = tiles * nsteps;
  const int64_t ub = sk_bound(b, U, G);
  if (ub % nsteps == 0 || ub >= U) return;           // boundary on a tile edge
  const int64_t t = ub / nsteps;
  if (sk_bound(b - 1, U, G) > t * nsteps) return;     // not the first boundary in tile t
  int acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0;
  for (int64_t bb = b - 1; bb < G && sk_bound(bb, U, G) < (t + 1) * nsteps; ++bb) {
    if (sk_bound(bb + 1, U, G) <= t * nsteps) continue;  // empty range before the tile
    const int slot = (sk_bound(bb, U, G) / nsteps == t) ? 0 : 1;
    const int4* slab = reinterpret_cast<const int4*>(sk_slab<BM, BN, THREADS>(a, bb, slot));
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int4 s = slab[q * THREADS + threadIdx.x];
      acc[q >> 1][(q & 1) * 4 + 0] += s.x;
      acc[q >> 1][(q & 1) * 4 + 1] += s.y;
      acc[q >> 1][(q & 1) * 4 + 2] += s.z;
      acc[q >> 1][(q & 1) * 4 + 3] += s.w;
    }
  }
  const int m0 = (int)(t % mt) * BM;
  const int64_t n0 = (t / mt) * BN;
  tile_epilogue<BM, BN, THREADS, true>(a, m0, n0, acc);
}

// Split-K epilogue: 4 channels of one pixel per lane from the int32 workspace.
__global__ __launch_bounds__(256) void conv_finalize_kernel(ConvArgs a) {
  const int groups = a.Cout / 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= a.P * groups) return;
  const int64_t p = t / groups;
  const int co = (int)(t - p * groups) * 4;
  const int4 s = *reinterpret_cast<const int4*>(a.ws + p * a.Cout + co);
  const int acc4[4] = {s.x, s.y, s.z, s.w};
  coef_t sc[4], sh[4];
  load_coef(a, co, sc, sh);
  emit4_nhwc(a, p, co, acc4, sc, sh, true);
}

// TR of fp32 activations straight into int16 NHWC codes (group_size 1, the reference's
// activation call, tr_layer.py:96-99).  One lane per 8 channels of one pixel.
template <bool IN_NHWC>
__global__ __launch_bounds__(256) void act_encode_kernel(const float* __restrict__ x,
                                                         int16_t* __restrict__ codes,
                                                         int64_t npix, int64_t HW, int C,
                                                         int Cp, float sf, float maxv, int k,
                                                         int fmt) {
  const int chunks = Cp / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= npix * chunks) return;
  const int64_t pix = t / chunks;
  const int c0 = (int)(t - pix * chunks) * 8;
  int32_t v[8];
  if (IN_NHWC && Cp == C) {
    const float4 x0 = *reinterpret_cast<const float4*>(x + pix * C + c0);
    const float4 x1 = *reinterpret_cast<const float4*>(x + pix * C + c0 + 4);
    const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = tr_value_g1(xs[i], sf, maxv, k);
  } else {
    const int64_t img = pix / HW;
    const int64_t s = pix - img * HW;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = c0 + i;
      v[i] = 0;
      if (c < C) {
        const float xv = IN_NHWC ? x[pix * C + c] : x[(img * C + c) * HW + s];
        v[i] = tr_value_g1(xv, sf, maxv, k);
      }
    }
  }
  uint32_t b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = code_bits(v[i], fmt);
  *reinterpret_cast<uint4*>(codes + pix * Cp + c0) =
      make_uint4(b[0] | (b[1] << 16), b[2] | (b[3] << 16), b[4] | (b[5] << 16), b[6] | (b[7] << 16));
}

// Activation / squeeze-excite gate + TR of EfficientNet-b0's MBConv tensors (channels_last,
// one lane per 8 channels of a pixel): v = act(x) (none or swish, act_apply), out = v (if
// out: the fp32 activation), v = fp32(gate[img][c] * v) (if gate: MBConvBlock.forward's
// x = sigmoid(x_sq) * x), codes[p][c] = TR(v) for the next conv (pad channels zero).
// Grid-stride: a few workgroups per CU, each building the code table once and then walking
// many chunks (a table per 2048 values cost as much as the values); IDX is the index type
// (uint32_t when npix * Cp / 8 and npix * C fit: no 64-bit divisions per chunk).
template <typename IDX>
__global__ __launch_bounds__(256) void act_encode_act_kernel(
    const float* __restrict__ x, const float* __restrict__ ch_scale,
    const float* __restrict__ ch_shift, const float* __restrict__ gate, int act,
    float* __restrict__ out,
    int16_t* __restrict__ codes, int64_t npix, int64_t HW, int C, int Cp, double inv_sf,
    float maxv, int k, int fmt, int lut_n, int fixed_chunk) {
  // the code table (lut_n = maxv + 1 entries, 0 = none): TR of a value costs its a1
  // rounding and one LDS read (tq_device.h lut_codes; signed values after swish / a gate too)
  extern __shared__ __attribute__((aligned(16))) uint16_t lut[];
  if (lut_n) {
    lut_build(lut, lut_n, k, fmt, threadIdx.x, 256);
    __syncthreads();
  }
  const IDX chunks = (IDX)(Cp / 8);
  const IDX total = (IDX)npix * chunks;
  const IDX hw = (IDX)HW;
  const double inv_hw = 1.0 / (double)HW;
  // fixed_chunk: the grid stride is a multiple of the chunks per pixel, so a lane keeps its
  // channel chunk and steps whole pixels -- no integer division per iteration; the image
  // index comes from a double reciprocal (exact after the one correction: pix < 2^32)
  const IDX t0 = (IDX)blockIdx.x * 256 + threadIdx.x;
  const IDX stride = (IDX)gridDim.x * 256;
  const IDX pstep = fixed_chunk ? stride / chunks : 0;
  IDX fpix = fixed_chunk ? t0 / chunks : 0;
  const int fc0 = fixed_chunk ? (int)(t0 - fpix * chunks) * 8 : 0;
  for (IDX t = t0; t < total; t += stride, fpix += pstep) {
    IDX pix, img;
    int c0;
    if (fixed_chunk) {
      pix = fpix;
      c0 = fc0;
      img = (IDX)((double)pix * inv_hw);
      if (pix - img * hw >= hw) ++img;
    } else {
      pix = t / chunks;
      c0 = (int)(t - pix * chunks) * 8;
      img = pix / hw;
    }
    float v[8];
    const bool vec = c0 + 8 <= C && (C & 3) == 0;
    if (vec) {
      const float4 x0 = *reinterpret_cast<const float4*>(x + pix * C + c0);
      const float4 x1 = *reinterpret_cast<const float4*>(x + pix * C + c0 + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
      v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    } else {
  #pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = c0 + i < C ? x[pix * C + c0 + i] : 0.0f;
    }
    if (ch_scale) {  // eval BatchNorm as a per-channel fp32 affine (a stem's bn before its act)
      if (vec) {  // 16-byte coefficient loads (4 per lane instead of 16 scalar ones)
        const float4 s0 = *reinterpret_cast<const float4*>(ch_scale + c0);
        const float4 s1 = *reinterpret_cast<const float4*>(ch_scale + c0 + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(ch_shift + c0);
        const float4 h1 = *reinterpret_cast<const float4*>(ch_shift + c0 + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
  #pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaf(v[i], sc[i], sh[i]);
      } else {
  #pragma unroll
        for (int i = 0; i < 8; ++i)
          v[i] = c0 + i < C ? fmaf(v[i], ch_scale[c0 + i], ch_shift[c0 + i]) : 0.0f;
      }
    }
    float o[8];
  #pragma unroll
    for (int i = 0; i < 8; ++i) act_apply(act, v[i], o[i]);
    if (out) {
      if (vec) {
        *reinterpret_cast<float4*>(out + pix * C + c0) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(out + pix * C + c0 + 4) = make_float4(o[4], o[5], o[6], o[7]);
      } else {
  #pragma unroll
        for (int i = 0; i < 8; ++i)
          if (c0 + i < C) out[pix * C + c0 + i] = o[i];
      }
    }
    if (gate) {
      if (vec) {
        const float4 g0 = *reinterpret_cast<const float4*>(gate + img * C + c0);
        const float4 g1 = *reinterpret_cast<const float4*>(gate + img * C + c0 + 4);
        const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
  #pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = g[i] * v[i];
      } else {
  #pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = c0 + i < C ? gate[img * C + c0 + i] * v[i] : 0.0f;
      }
    }
    uint32_t b[8];
    if (lut_n) {
      lut_codes<8>(v, inv_sf, maxv, fmt, act_nonneg(act) && !gate, lut, b);
  #pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = c0 + i < C ? b[i] : 0u;
    } else if (act_nonneg(act) && !gate && inv_sf > 0.0 && inv_sf <= 1.0e308) {
      // ReLU / ReLU6: v >= 0 and never NaN -- the epilogues' sign-free fast path (same codes)
      const int npeel = relu_peels(maxv, k);
  #pragma unroll
      for (int h = 0; h < 2; ++h) {
        int32_t t4[4];
        tr_values_relu4(v + 4 * h, inv_sf, maxv, npeel, t4);
  #pragma unroll
        for (int i = 0; i < 4; ++i) b[4 * h + i] = c0 + 4 * h + i < C ? code_bits(t4[i], fmt) : 0u;
      }
    } else {
  #pragma unroll
      for (int i = 0; i < 8; ++i)
        b[i] = c0 + i < C ? code_bits(tr_value_g1_inv(v[i], inv_sf, maxv, k), fmt) : 0u;
    }
    *reinterpret_cast<uint4*>(codes + (int64_t)pix * Cp + c0) =
        make_uint4(b[0] | (b[1] << 16), b[2] | (b[3] << 16), b[4] | (b[5] << 16),
                   b[6] | (b[7] << 16));
  }
}

}  // namespace

hipError_t launch_act_encode_act(const float* x, const float* ch_scale, const float* ch_shift,
                                 const float* gate, int act, float* out,
                                 int64_t N, int64_t C, int64_t H, int64_t W, float sf,
                                 int bitwidth, int k, int16_t* codes, int64_t Cp, int fmt,
                                 hipStream_t stream) {
  const float maxv = (float)((1u << bitwidth) - 1u);
  const int64_t npix = N * H * W;
  const int64_t n = npix * (Cp / 8);
  if (n == 0) return hipSuccess;
  const double inv = 1.0 / (double)sf;
  const char* lut_env = getenv("TQ_LUT");  // 0: computed codes (tests, A/B; read per launch)
  const int lut_n = (!(lut_env && atoi(lut_env) == 0) && inv > 0.0 && inv <= 1.0e308 &&
                     (int)maxv + 1 <= kLutMax) ? (int)maxv + 1 : 0;
  int64_t grid = std::min<int64_t>((n + 255) / 256, (int64_t)device_cus() * 8);
  // a grid whose stride (grid * 256 lanes) is a multiple of the chunks per pixel: every lane
  // keeps one channel chunk (TQ_AEA_FIXED=0: the per-iteration division form, A/B)
  const int64_t chunks = Cp / 8;
  int64_t g = 256, r = chunks;
  while (r) {
    const int64_t t = g % r;
    g = r;
    r = t;
  }
  const int64_t m = chunks / g;  // grid granule
  const char* fenv = getenv("TQ_AEA_FIXED");
  int fixed = !(fenv && atoi(fenv) == 0) && grid >= m;
  if (fixed) grid = grid / m * m;
  const bool small = n < (1ll << 31) && npix * Cp < (1ll << 31);
  if (small)
    act_encode_act_kernel<uint32_t><<<dim3((unsigned)grid), 256, (size_t)lut_n * 2, stream>>>(
        x, ch_scale, ch_shift, gate, act, out, codes, npix, H * W, (int)C, (int)Cp, inv, maxv,
        k, fmt, lut_n, fixed);
  else
    act_encode_act_kernel<int64_t><<<dim3((unsigned)grid), 256, (size_t)lut_n * 2, stream>>>(
        x, ch_scale, ch_shift, gate, act, out, codes, npix, H * W, (int)C, (int)Cp, inv, maxv,
        k, fmt, lut_n, fixed);
  return hipGetLastError();
}

hipError_t launch_act_encode(const float* x, int in_nhwc, int64_t N, int64_t C, int64_t H,
                             int64_t W, float sf, int bitwidth, int k, int16_t* codes, int64_t Cp,
                             int fmt, hipStream_t stream) {
  const float maxv = (float)((1u << bitwidth) - 1u);
  const int64_t npix = N * H * W;
  const int64_t n = npix * (Cp / 8);
  if (n == 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (in_nhwc)
    act_encode_kernel<true><<<grid, 256, 0, stream>>>(x, codes, npix, H * W, (int)C, (int)Cp,
                                                       sf, maxv, k, fmt);
  else
    act_encode_kernel<false><<<grid, 256, 0, stream>>>(x, codes, npix, H * W, (int)C, (int)Cp,
                                                        sf, maxv, k, fmt);
  return hipGetLastError();
}

// Tile configurations: {BM, BN, threads, waves per SIMD}.  All keep 8 x 8 accumulators per
// lane; configs 4 and 5 repeat 0 and 1 with a 4-waves-per-SIMD register budget.
struct TileCfg {
  int bm, bn, threads, occ;
};
constexpr TileCfg kTileCfgs[] = {{128, 128, 256, 3}, {64, 256, 256, 3}, {64, 128, 128, 3},
                                 {128, 64, 128, 3},  {128, 128, 256, 4}, {64, 256, 256, 4}};
constexpr int kNumTileCfgs = sizeof(kTileCfgs) / sizeof(kTileCfgs[0]);

int conv_tile_m(int64_t cout) { return cout <= 64 ? 64 : 128; }

int conv_num_configs() { return kNumTileCfgs; }

int device_cus() {
  static thread_local int cached_dev = -1, cached_cus = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev != cached_dev) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    cached_dev = dev;
    cached_cus = cus;
  }
  return cached_cus;
}

namespace {

// Resident blocks per CU of the stream-K kernel of one config (occupancy query, cached).
template <int BM, int BN, int T, int OCC>
int streamk_blocks_per_cu() {
  static thread_local int cached = 0;
  if (cached == 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &n, reinterpret_cast<const void*>(&conv2d_tp_streamk_kernel<BM, BN, T, OCC>), T,
            0) != hipSuccess || n <= 0)
      n = 1;
    cached = n;
  }
  return cached;
}

int streamk_grid(int cfg) {
  int per_cu = 1;
  switch (cfg) {
    case 0: per_cu = streamk_blocks_per_cu<128, 128, 256, 3>(); break;
    case 1: per_cu = streamk_blocks_per_cu<64, 256, 256, 3>(); break;
    case 2: per_cu = streamk_blocks_per_cu<64, 128, 128, 3>(); break;
    case 3: per_cu = streamk_blocks_per_cu<128, 64, 128, 3>(); break;
    case 4: per_cu = streamk_blocks_per_cu<128, 128, 256, 4>(); break;
    default: per_cu = streamk_blocks_per_cu<64, 256, 256, 4>(); break;
  }
  return device_cus() * per_cu;
}

// Execution plan for config 0 (heuristic), from tools/microbench.py --sweep on MI355X
// (profiles/r01_sweep2.txt): 64x256 tiles for Cout <= 64, else 128x128.  The dot2 pipe is
// saturated while 3 waves share a SIMD, so a data-parallel grid whose last round of blocks
// is partly empty loses that fraction (1568 tiles on 768 slots ran at 68 %); stream-K (one
// resident round, K-steps shared evenly, slab fixup) recovers it when the grid is under
// 2.5 rounds and K is deep enough (>= 32 steps) to amortise the fixup -- ResNet-18
// layer2-4 3x3 convs gain 2-24 %; layer1 and all 1x1 convs stay data-parallel.
// splits: 1 = data-parallel, > 1 = K-split with atomics, -1 = stream-K.
void pick_config(const ConvArgs& a, int out_nhwc, int* cfg, int* splits) {
  if (a.config > 0 && a.config <= kNumTileCfgs) {
    *cfg = a.config - 1;
    *splits = a.splits != 0 ? a.splits : 1;
  } else {
    *cfg = a.Cout <= 64 ? 1 : 0;
    *splits = 1;
    const TileCfg& t = kTileCfgs[*cfg];
    const int64_t tiles = ((a.P + t.bn - 1) / t.bn) * ((a.Cout + t.bm - 1) / t.bm);
    const int64_t slots = (int64_t)device_cus() * 3;
    const double rounds = (double)tiles / (double)slots;
    const double eff = rounds / std::ceil(rounds);
    if (eff < 0.9 && rounds < 2.5 && a.Kp / 32 >= 32) *splits = -1;
  }
  if (!out_nhwc || !a.ws || (a.Cout & 3)) *splits = 1;  // both need NHWC + a workspace
}

template <int BM, int BN, int T, int OCC>
hipError_t launch_cfg(const ConvArgs& a, int out_nhwc, int splits, hipStream_t stream) {
  const int64_t tiles = ((a.P + BN - 1) / BN) * ((a.Cout + BM - 1) / BM);
  if (splits < 0) {
    const int64_t units = tiles * (a.Kp / 32);
    int64_t g = (int64_t)device_cus() * streamk_blocks_per_cu<BM, BN, T, OCC>();
    if (g > units) g = units;
    if ((int64_t)g * 2 * BM * BN * 4 > a.ws_bytes) return hipErrorInvalidValue;
    conv2d_tp_streamk_kernel<BM, BN, T, OCC><<<dim3((unsigned)g), T, 0, stream>>>(a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || g < 2) return e;
    conv2d_tp_streamk_fixup<BM, BN, T><<<dim3((unsigned)(g - 1)), T, 0, stream>>>(a, (int)g);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)(tiles * splits));
  if (splits > 1)
    conv2d_tp_kernel<BM, BN, T, true, true, OCC><<<grid, T, 0, stream>>>(a);
  else if (out_nhwc)
    conv2d_tp_kernel<BM, BN, T, true, false, OCC><<<grid, T, 0, stream>>>(a);
  else
    conv2d_tp_kernel<BM, BN, T, false, false, OCC><<<grid, T, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace

int64_t conv_workspace_bytes(int64_t p, int64_t cout) {
  int64_t sk = 0;
  for (int c = 0; c < kNumTileCfgs; ++c) {
    const int64_t b = (int64_t)streamk_grid(c) * 2 * kTileCfgs[c].bm * kTileCfgs[c].bn * 4;
    if (b > sk) sk = b;
  }
  const int64_t split = p * cout * 4;
  const int64_t r = sk > split ? sk : split;
  const int64_t ps = patch_streamk_ws_bytes(p, cout);
  return r > ps ? r : ps;
}

hipError_t launch_conv2d_tp(const ConvArgs& a_in, int out_nhwc, hipStream_t stream) {
  if (a_in.P == 0 || a_in.Cout == 0) return hipSuccess;
  ConvArgs a = a_in;
  int cfg, splits;
  pick_config(a, out_nhwc, &cfg, &splits);
  if (splits > 1 && a.P * a.Cout * 4 > a.ws_bytes) splits = 1;
  a.splits = splits;
  if (splits > 1) {
    hipError_t e = hipMemsetAsync(a.ws, 0, (size_t)a.P * a.Cout * sizeof(int32_t), stream);
    if (e != hipSuccess) return e;
  }
  hipError_t e;
  switch (cfg) {
    case 0: e = launch_cfg<128, 128, 256, 3>(a, out_nhwc, splits, stream); break;
    case 1: e = launch_cfg<64, 256, 256, 3>(a, out_nhwc, splits, stream); break;
    case 2: e = launch_cfg<64, 128, 128, 3>(a, out_nhwc, splits, stream); break;
    case 3: e = launch_cfg<128, 64, 128, 3>(a, out_nhwc, splits, stream); break;
    case 4: e = launch_cfg<128, 128, 256, 4>(a, out_nhwc, splits, stream); break;
    default: e = launch_cfg<64, 256, 256, 4>(a, out_nhwc, splits, stream); break;
  }
  if (e != hipSuccess || splits <= 1) return e;
  const int64_t n = a.P * (a.Cout / 4);
  conv_finalize_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace tq
