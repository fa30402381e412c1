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
#include "tq_device.h"
#include "tq_launch.h"

namespace tq {

namespace {

__device__ __forceinline__ int dot2(int a, int b, int c) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, a), __builtin_bit_cast(s2, b), c, false);
}

// Per-channel epilogue coefficients of channels co..co+3: y = acc * sc + sh (fp64).
__device__ __forceinline__ void load_coef(const ConvArgs& a, int co, double sc[4],
                                          double sh[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = co + i < a.Cout;
    if (a.ch_scale) {
      sc[i] = ok ? a.ch_scale[co + i] : 0.0;
      sh[i] = ok ? a.ch_shift[co + i] : 0.0;
    } else {
      sc[i] = a.scale;
      sh[i] = (a.bias && ok) ? (double)a.bias[co + i] : 0.0;
    }
  }
}

__device__ __forceinline__ void store_codes4(int16_t* codes, int cp, int64_t p, int co,
                                             const float y[4], float sf, float maxv, int k) {
  int32_t v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = tr_value_g1(y[i], sf, maxv, k);
  *reinterpret_cast<int2*>(codes + p * cp + co) =
      make_int2((v[0] & 0xFFFF) | (v[1] << 16), (v[2] & 0xFFFF) | (v[3] << 16));
}

// Finish channels co..co+3 of output pixel p (channels_last) from exact integer sums:
// one fp64->fp32 rounding, residual add and ReLU in fp32, fp32 store, next layers' TR codes
// (tr_layer.py:96-99 applied to the stored value).
__device__ __forceinline__ void emit4_nhwc(const ConvArgs& a, int64_t p, int co,
                                           const int acc[4], const double sc[4],
                                           const double sh[4], bool vec) {
  float y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = (float)((double)acc[i] * sc[i] + sh[i]);
  if (a.residual) {
    const float* r = a.residual + p * a.Cout + co;
    if (vec) {
      const float4 rv = *reinterpret_cast<const float4*>(r);
      y[0] += rv.x;
      y[1] += rv.y;
      y[2] += rv.z;
      y[3] += rv.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (co + i < a.Cout) y[i] += r[i];
    }
  }
  if (a.relu) {
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = y[i] > 0.0f ? y[i] : 0.0f;
  }
  if (a.out) {
    float* dst = a.out + p * a.Cout + co;
    if (vec) {
      *reinterpret_cast<float4*>(dst) = make_float4(y[0], y[1], y[2], y[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (co + i < a.Cout) dst[i] = y[i];
    }
  }
  if (a.codes_a) store_codes4(a.codes_a, a.cp_a, p, co, y, a.sf_a, a.maxv_a, a.k_a);
  if (a.codes_b) store_codes4(a.codes_b, a.cp_b, p, co, y, a.sf_b, a.maxv_b, a.k_b);
}

// Implicit-GEMM term-pair conv.  BM x BN output tile (Cout x pixels), THREADS lanes with an
// 8 x 8 int32 accumulator tile each.  SPLIT: this block sums only its share of the K-steps
// and adds its partial sums into the int32 workspace (exact, order-independent);
// conv_finalize_kernel applies the epilogue afterwards.
template <int BM, int BN, int THREADS, bool OUT_NHWC, bool SPLIT, int OCC>
__global__ __launch_bounds__(THREADS, OCC) void conv2d_tp_kernel(ConvArgs a) {
  constexpr int TX = BN / 8;
  static_assert((BM / 8) * TX == THREADS, "8x8 accumulators per thread");
  constexpr int ROWS = THREADS / 4;                // rows (m or n) per load slot
  constexpr int A_LOADS = BM / ROWS;               // 16-B vectors per thread per K-step
  constexpr int B_LOADS = BN / ROWS;
  static_assert(A_LOADS >= 1 && B_LOADS >= 1, "tile too small for the thread count");

  __shared__ __attribute__((aligned(16))) int32_t As[2][16][BM];
  __shared__ __attribute__((aligned(16))) int32_t Bs[2][16][BN];

  const int tid = threadIdx.x;
  const int tx = tid % TX;
  const int ty = tid / TX;
  // XCD-aware work order: blocks are dealt round-robin to the 8 XCDs (bid % 8), so each XCD
  // gets a contiguous run of logical work items -- the K-splits and Cout tiles of one pixel
  // tile adjacent, neighbouring pixel tiles next -- and halo rows / shared activation tiles
  // hit one L2.  Bijective for any grid size (placement is a speed choice only).
  const int nblk = gridDim.x;
  const int bid = blockIdx.x;
  const int q8 = nblk >> 3, r8 = nblk & 7, xcd = bid & 7;
  const int item = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int splits = SPLIT ? a.splits : 1;
  const int split = item % splits;
  const int tile = item / splits;
  const int mt = (a.Cout + BM - 1) / BM;
  const int m0 = (tile % mt) * BM;
  const int64_t n0 = (int64_t)(tile / mt) * BN;
  const int64_t HoWo = (int64_t)a.Ho * a.Wo;
  const int nsteps_all = a.Kp / 32;
  const int ks_begin = (int)((int64_t)split * nsteps_all / splits);
  const int nsteps = (int)((int64_t)(split + 1) * nsteps_all / splits) - ks_begin;

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
    const int k0 = ks_begin * 32 + v * 8;
    ktap = k0 / a.Cp;
    kc = k0 - ktap * a.Cp;
    kr = ktap / a.KW;
    ks = ktap - kr * a.KW;
  }

  const int16_t* __restrict__ wrow[A_LOADS];
#pragma unroll
  for (int r = 0; r < A_LOADS; ++r)
    wrow[r] = a.w + (int64_t)(m0 + rowl + ROWS * r) * a.Kp + (int64_t)ks_begin * 32 + v * 8;

  const int ntaps = a.KH * a.KW;

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
    // advance this lane's k-vector by 32 codes
    kc += 32;
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
      As[buf][v * 4 + 0][m] = ra[r].x;
      As[buf][v * 4 + 1][m] = ra[r].y;
      As[buf][v * 4 + 2][m] = ra[r].z;
      As[buf][v * 4 + 3][m] = ra[r].w;
    }
#pragma unroll
    for (int r = 0; r < B_LOADS; ++r) {
      const int n = rowl + ROWS * r;
      Bs[buf][v * 4 + 0][n] = rb[r].x;
      Bs[buf][v * 4 + 1][n] = rb[r].y;
      Bs[buf][v * 4 + 2][n] = rb[r].z;
      Bs[buf][v * 4 + 3][n] = rb[r].w;
    }
  };

  int acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0;

  if (nsteps > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();

  for (int step = 0; step < nsteps; ++step) {
    const int cur = step & 1;
    if (step + 1 < nsteps) load_tile(step + 1);
#pragma unroll 2
    for (int kk = 0; kk < 16; ++kk) {
      const int4 a0 = *reinterpret_cast<const int4*>(&As[cur][kk][ty * 4]);
      const int4 a1 = *reinterpret_cast<const int4*>(&As[cur][kk][BM / 2 + ty * 4]);
      const int4 b0 = *reinterpret_cast<const int4*>(&Bs[cur][kk][tx * 4]);
      const int4 b1 = *reinterpret_cast<const int4*>(&Bs[cur][kk][BN / 2 + tx * 4]);
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

  if (SPLIT) {
    // exact int32 partial sums into the workspace ([P][Cout], zeroed by the launcher)
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

  // Epilogue: one rounding of the exact integer sum (fp64 scale/shift), 16-byte stores of 4
  // consecutive channels (NHWC) or 4 consecutive pixels (NCHW).
  if (OUT_NHWC) {
    const bool vec = (a.Cout & 3) == 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int co = m0 + h * (BM / 2) + ty * 4;
      if (co >= a.Cout) continue;
      double sc[4], sh[4];
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
    const bool vec = (HoWo & 3) == 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int co = m0 + (i < 4 ? ty * 4 + i : BM / 2 + ty * 4 + (i - 4));
      if (co >= a.Cout) continue;
      const double sc = a.scale;
      const double sh = a.bias ? (double)a.bias[co] : 0.0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t p0 = n0 + h * (BN / 2) + tx * 4;
        float y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = (float)((double)acc[i][h * 4 + j] * sc + sh);
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

// Split-K epilogue: 4 channels of one pixel per lane from the int32 workspace.
__global__ __launch_bounds__(256) void conv_finalize_kernel(ConvArgs a) {
  const int groups = a.Cout / 4;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= a.P * groups) return;
  const int64_t p = t / groups;
  const int co = (int)(t - p * groups) * 4;
  const int4 s = *reinterpret_cast<const int4*>(a.ws + p * a.Cout + co);
  const int acc4[4] = {s.x, s.y, s.z, s.w};
  double sc[4], sh[4];
  load_coef(a, co, sc, sh);
  emit4_nhwc(a, p, co, acc4, sc, sh, true);
}

// TR of fp32 activations straight into int16 NHWC codes (group_size 1, the reference's
// activation call, tr_layer.py:96-99).  One lane per 8 channels of one pixel.
template <bool IN_NHWC>
__global__ __launch_bounds__(256) void act_encode_kernel(const float* __restrict__ x,
                                                         int16_t* __restrict__ codes,
                                                         int64_t npix, int64_t HW, int C,
                                                         int Cp, float sf, float maxv, int k) {
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
  int4 packed;
  packed.x = (v[0] & 0xFFFF) | (v[1] << 16);
  packed.y = (v[2] & 0xFFFF) | (v[3] << 16);
  packed.z = (v[4] & 0xFFFF) | (v[5] << 16);
  packed.w = (v[6] & 0xFFFF) | (v[7] << 16);
  *reinterpret_cast<int4*>(codes + pix * Cp + c0) = packed;
}

}  // namespace

hipError_t launch_act_encode(const float* x, int in_nhwc, int64_t N, int64_t C, int64_t H,
                             int64_t W, float sf, int bitwidth, int k, int16_t* codes, int64_t Cp,
                             hipStream_t stream) {
  const float maxv = (float)((1u << bitwidth) - 1u);
  const int64_t npix = N * H * W;
  const int64_t n = npix * (Cp / 8);
  if (n == 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (in_nhwc)
    act_encode_kernel<true><<<grid, 256, 0, stream>>>(x, codes, npix, H * W, (int)C, (int)Cp,
                                                       sf, maxv, k);
  else
    act_encode_kernel<false><<<grid, 256, 0, stream>>>(x, codes, npix, H * W, (int)C, (int)Cp,
                                                        sf, maxv, k);
  return hipGetLastError();
}

// Tile configurations: {BM, BN, threads}.  All keep 8 x 8 accumulators per lane.
struct TileCfg {
  int bm, bn, threads;
};
constexpr TileCfg kTileCfgs[] = {{128, 128, 256}, {64, 256, 256}, {64, 128, 128},
                                 {128, 64, 128},  {128, 128, 256}, {64, 256, 256}};
// configs 4 and 5 repeat 0 and 1 with a 4-waves-per-SIMD register budget (128 VGPRs)
constexpr int kNumTileCfgs = sizeof(kTileCfgs) / sizeof(kTileCfgs[0]);

int conv_tile_m(int64_t cout) { return cout <= 64 ? 64 : 128; }

int conv_num_configs() { return kNumTileCfgs; }

namespace {

// Heuristic for config 0, from the per-layer sweep of tools/microbench.py --sweep on MI355X
// (profiles/r01_sweep.txt): 64x256 tiles for Cout <= 64, else 128x128, one K pass; only when
// the 128x128 grid leaves most CUs with < 2 tiles and K is deep (ResNet-18 layer4 3x3) does
// a 3-way K split of 128x64 tiles pay for its int32 atomics (~12 %).  Splitting any larger
// grid costs more in atomics than it gains (2-4x slower at layer1).
void pick_config(const ConvArgs& a, int out_nhwc, int* cfg, int* splits) {
  if (a.config > 0 && a.config <= kNumTileCfgs) {
    *cfg = a.config - 1;
    *splits = a.splits > 0 ? a.splits : 1;
  } else {
    *cfg = a.Cout <= 64 ? 1 : 0;
    *splits = 1;
    const int64_t tiles128 = ((a.P + 127) / 128) * ((a.Cout + 127) / 128);
    const int nsteps = a.Kp / 32;
    if (a.Cout > 64 && tiles128 < 2 * 256 && nsteps >= 96) {
      *cfg = 3;
      *splits = 3;
    }
  }
  if (!out_nhwc || !a.ws || (a.Cout & 3)) *splits = 1;  // split-K only for NHWC outputs
}

template <int BM, int BN, int T, int OCC>
hipError_t launch_cfg(const ConvArgs& a, int out_nhwc, int splits, hipStream_t stream) {
  const int64_t tiles = ((a.P + BN - 1) / BN) * ((a.Cout + BM - 1) / BM);
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

hipError_t launch_conv2d_tp(const ConvArgs& a_in, int out_nhwc, hipStream_t stream) {
  if (a_in.P == 0 || a_in.Cout == 0) return hipSuccess;
  ConvArgs a = a_in;
  int cfg, splits;
  pick_config(a, out_nhwc, &cfg, &splits);
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
  if (e != hipSuccess || splits == 1) return e;
  const int64_t n = a.P * (a.Cout / 4);
  conv_finalize_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, stream>>>(a);
  return hipGetLastError();
}

}  // namespace tq
