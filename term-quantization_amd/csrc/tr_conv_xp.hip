// Term-pair Conv2d on the matrix cores, expand engine: 1x1 stride-1 convs with a short K (one
// or two 64-code K-steps) and a wide Cout whose weights fit LDS -- the MobileNet-V2 /
// EfficientNet-b0 expand convs (16..80 -> 96..480 channels), whose launches are almost all
// epilogue: one K-step of MFMAs per 64 x 32 block, then 2048 outputs to fold, activate and
// encode for the next layer.
//
// Same arithmetic and epilogue as every other term-pair engine (fp16 term-sum codes, exact
// products and sums on v_mfma_f32_32x32x16_f16 -- the host only sends launches whose whole K
// range is one exact window, so the fp32 sums are exact integers -- then the shared
// emit4_nhwc_res): bit-identical outputs.
//
// Why a separate engine.  The direct engine gives each workgroup one 64 x 128 tile: weight
// DMA, activation loads, code tables, one K-step, epilogue; a 112^2 x 16 -> 96 tile lives ~8 us
// of which ~3.3 us is that setup, at ~3 resident workgroups per CU.  Here:
//   * a persistent workgroup stages the weights of its Cout group (NKS x MT slots of 64 rows,
//     swizzled as the direct engine's, <= 32 KB: all of Cout, or MG groups of MT 64-row tiles
//     for wider layers), the group's epilogue coefficients and the code tables once;
//   * then each wave works alone (no barrier in the loop): a work item is 32 output pixels x
//     every Cout tile of the group; its activation fragments (NKS x 4 x 16 bytes per lane)
//     come straight from HBM into registers, and the NEXT item's are loaded before this
//     item's MFMAs and epilogues run;
//   * the epilogue reads the accumulators in the MFMA layout (lane = 4 consecutive channels
//     of one pixel per quad), coefficients from LDS, no transpose: 8-byte code stores, one
//     pixel's 2 Cout bytes written by one wave within the item.
// 90 VGPRs at NKS = 1: five waves per SIMD hide the store and LDS latencies.
#include <stdlib.h>

#include "tq_device.h"
#include "tq_epilogue.h"
#include "tq_launch.h"
#include "tq_mfma.h"

namespace tq {

namespace {

constexpr int kXpThreads = 256;
constexpr int kXpSlot = 64 * 8;                 // u32x4 per weight slot: 64 rows x 64 codes
constexpr int kXpMaxWeightBytes = 32 * 1024;    // staged weights per workgroup (48 KB of
                                                // them left 2 workgroups per CU: slower than
                                                // the direct engine on 64 -> 384)
// Cout groups a launch may be split into (TQ_XP_GROUPS, read per launch; default 1 = layers
// whose weights fit one workgroup): groups re-read the activations, and measured slower than
// the direct engine on 64 -> 384, 96 -> 576 and 112 -> 672 at 14^2 (46 / 53 / 68 vs 36 / 50 /
// 59 us), faster only on 80 -> 480 (44 vs 46 us): profiles/r04_expand_probe.txt
int xp_max_groups() {
  const char* g = getenv("TQ_XP_GROUPS");
  return g && atoi(g) > 0 ? atoi(g) : 1;
}

// LDS bytes of a launch: weights, coefficients, code tables.
int64_t xp_lds_bytes(const ConvArgs& a, int nks, int mt) {
  return (int64_t)nks * mt * kXpSlot * 16 + (int64_t)mt * 64 * 16 + conv_lut_bytes(a);
}

// 64-row Cout tiles per workgroup (the weight budget) and the number of Cout groups.
void xp_groups(const ConvArgs& a, int nks, int* mt, int* mg) {
  const int tiles = (a.Cout + 63) / 64;
  const int per = kXpMaxWeightBytes / (nks * kXpSlot * 16);
  *mt = tiles < per ? tiles : per;
  *mg = (tiles + *mt - 1) / *mt;
}

// The fused executors' form of the expand convs -- ReLU / ReLU6 / swish (FAST = 1 / 2 / 3),
// one code output served by its code table, no fp32 output -- with emit4_nhwc_res's
// operations for that form only (fold, the activation the codes see, lut_codes' table path,
// the store): the generic epilogue's runtime branches and stored value cost ~36 VALU per
// output at ReLU6.
template <int FAST>
__device__ __forceinline__ void xp_emit_codes4(const ConvArgs& a, int64_t p, int co,
                                               const int acc[4], const coef_t sc[4],
                                               const coef_t sh[4], const uint16_t* lut) {
  float y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    y[i] = fold_acc(acc[i], sc[i], sh[i]);
    if (FAST == 3) {
      y[i] = swish_f32(y[i]);
    } else {
      y[i] = y[i] > 0.0f ? y[i] : 0.0f;
      if (FAST == 2) y[i] = y[i] < 6.0f ? y[i] : 6.0f;
    }
  }
  uint32_t v[4];
  if (FAST == 3) {
    lut_codes<4>(y, a.inv_a, a.maxv_a, a.fmt_a, false, lut, v);  // signed values
  } else {
    uint32_t q[4];
    relu_q_epi<4>(y, a.inv_a, a.maxv_a, q);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = lut[q[i]];
  }
  int16_t* dst = a.codes_a + p * a.cp_a + co;
  *reinterpret_cast<int2*>(dst) = make_int2((int)(v[0] | (v[1] << 16)), (int)(v[2] | (v[3] << 16)));
  if (co + 4 == a.Cout && a.cp_a > a.Cout) *reinterpret_cast<int2*>(dst + 4) = make_int2(0, 0);
}

// 5 waves per SIMD at one K-step (90 VGPRs, no spills; 6 spill), 4 at two
template <int NKS, bool SWISH, int FAST>
__global__ __launch_bounds__(kXpThreads) __attribute__((amdgpu_waves_per_eu(NKS == 1 ? 5 : 4)))
void conv2d_tp_xp_kernel(ConvArgs a, int MT, int MG) {
  extern __shared__ __attribute__((aligned(16))) u32x4 xp_lds[];
  u32x4* wl = xp_lds;                                                    // [NKS][MT][swz]
  double* coef = reinterpret_cast<double*>(wl + (int64_t)NKS * MT * kXpSlot);  // [MT 64][2]
  uint16_t *lut_a, *lut_b;
  conv_luts(a, reinterpret_cast<uint16_t*>(coef + 2 * MT * 64), lut_a, lut_b);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int r32 = lane & 31;
  const int hh = lane >> 5;
  const int cpad = MT * 64;
  const int grp = blockIdx.x % MG;  // this workgroup's Cout group: channels [mbase, + cpad)
  const int mbase = grp * cpad;
  const uint16_t* __restrict__ wg = reinterpret_cast<const uint16_t*>(a.w);
  const uint16_t* __restrict__ xg = reinterpret_cast<const uint16_t*>(a.x);

  // weights: slot (ks, mt) row r, 16-byte unit u <- w[mt 64 + r][ks 64 + 8 u .. + 8]; rows
  // past Cout are zero (their sums are never emitted)
  for (int i = tid; i < NKS * cpad * 8; i += kXpThreads) {
    const int u = i & 7;
    const int row = (i >> 3) % cpad;
    const int ks = (i >> 3) / cpad;
    const int mt = row >> 6, r = row & 63;
    u32x4 v = (u32x4)0u;
    if (mbase + row < a.Cout)
      v = *reinterpret_cast<const u32x4*>(wg + (int64_t)(mbase + row) * a.Kp + ks * kKStep +
                                          8 * u);
    wl[(ks * MT + mt) * kXpSlot + swz(r, u)] = v;
  }
  for (int i = tid; i < cpad; i += kXpThreads) {
    const int c = mbase + i;
    const bool ok = c < a.Cout;
    coef[2 * i] = ok ? (a.ch_scale ? a.ch_scale[c] : a.scale) : 0.0;
    coef[2 * i + 1] = ok ? (a.ch_scale ? a.ch_shift[c] : (a.bias ? (double)a.bias[c] : 0.0))
                         : 0.0;
  }
  __syncthreads();  // weights, coefficients, code tables: no barrier after this

  const int64_t ntile = (a.P + 31) / 32;
  // the group's workgroups (gridDim.x is a multiple of MG) walk every pixel item
  const int64_t nwave = (int64_t)(gridDim.x / MG) * (kXpThreads / 64);
  const int64_t w0 = (int64_t)(blockIdx.x / MG) * (kXpThreads / 64) + (tid >> 6);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_zero_page);

  // B fragments of pixel tile t for this lane (pixel t 32 + r32, codes 8 hh + 16 k of each
  // K-step); pixels past P and codes past Cp read the zero page (unconditional loads)
  auto load_b = [&](int64_t t, u32x4 (&b)[NKS][4]) __attribute__((always_inline)) {
    const int64_t p = t * 32 + r32;
    const bool okp = p < a.P;
    const uint16_t* src = xg + (okp ? p : 0) * a.Cp + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = okp && ks * kKStep + 16 * k + 8 * hh < a.Cp;
        b[ks][k] = *reinterpret_cast<const u32x4*>(ok ? src + ks * kKStep + 16 * k : zero);
      }
  };

  u32x4 bcur[NKS][4];
  load_b(w0, bcur);
  const float4 nores = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t t = w0; t < ntile; t += nwave) {
    u32x4 bnext[NKS][4];
    load_b(t + nwave, bnext);
    const int64_t p = t * 32 + r32;
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int bm = 0; bm < 2; ++bm) {
        const int m0 = mbase + mt * 64 + 32 * bm;
        if (m0 >= a.Cout) break;  // wave-uniform
        float16v acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const half8 af = __builtin_bit_cast(
                half8, wl[(ks * MT + mt) * kXpSlot + swz(32 * bm + r32, 2 * k + hh)]);
            const half8 bf = __builtin_bit_cast(half8, bcur[ks][k]);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf, acc, 0, 0, 0);
          }
        if (p >= a.P) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int co = m0 + 8 * q + 4 * hh;
          if (co >= a.Cout) continue;
          int acc4[4];
          coef_t sc[4], sh[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc4[e] = (int)acc[4 * q + e];
            sc[e] = (coef_t)coef[2 * (co - mbase + e)];
            sh[e] = (coef_t)coef[2 * (co - mbase + e) + 1];
          }
          if constexpr (FAST != 0)
            xp_emit_codes4<FAST>(a, p, co, acc4, sc, sh, lut_a);
          else
            emit4_nhwc_res<SWISH>(a, p, co, acc4, sc, sh, nores, lut_a, lut_b);
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int k = 0; k < 4; ++k) bcur[ks][k] = bnext[ks][k];
  }
}

template <int NKS, bool SWISH, int FAST>
hipError_t launch_xp_cfg(const ConvArgs& a, hipStream_t stream) {
  int mt, mg;
  xp_groups(a, NKS, &mt, &mg);
  const size_t lds = (size_t)xp_lds_bytes(a, NKS, mt);
  const void* fn = reinterpret_cast<const void*>(&conv2d_tp_xp_kernel<NKS, SWISH, FAST>);
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e =
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  // persistent: as many workgroups as fit at once (VGPRs / LDS), no more than the work
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kXpThreads, lds);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  // workgroups per Cout group (TQ_XP_GRID: tests, few workgroups with many items each)
  const char* genv = getenv("TQ_XP_GRID");
  int64_t per_grp = genv && atoi(genv) > 0 ? atoi(genv)
                                           : ((int64_t)per_cu * device_cus() + mg - 1) / mg;
  const int64_t items = (a.P + 31) / 32;
  const int64_t need = (items + kXpThreads / 64 - 1) / (kXpThreads / 64);
  if (per_grp > need) per_grp = need;
  if (per_grp < 1) per_grp = 1;
  conv2d_tp_xp_kernel<NKS, SWISH, FAST>
      <<<dim3((unsigned)(per_grp * mg)), kXpThreads, lds, stream>>>(a, mt, mg);
  return hipGetLastError();
}

}  // namespace

// 1x1 stride-1 pad-0 NHWC convs with one or two K-steps in one exact window, no residual and
// no fused downsample, Cout % 4 == 0, at most kXpMaxGroups Cout groups.
bool conv_xp_eligible(const ConvArgs& a, int out_nhwc) {
  const int nks = a.Kp / kKStep;
  if (!(out_nhwc && a.KH == 1 && a.KW == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 &&
        a.pw == 0 && a.Cp % 8 == 0 && a.Kp % kKStep == 0 && (nks == 1 || nks == 2) &&
        (a.kc_steps == 0 || a.kc_steps >= nks) && a.residual == nullptr &&
        a.ds_x == nullptr && (a.Cout & 3) == 0 && a.Cout > 0))
    return false;
  int mt, mg;
  xp_groups(a, nks, &mt, &mg);
  return mg <= xp_max_groups();
}

template <int NKS>
hipError_t launch_xp_nks(const ConvArgs& a, hipStream_t stream) {
  // (the two-K-step instantiations of the fast forms spill at 4 waves per SIMD)
  // (TQ_EPI_FAST=0: the generic epilogue, as every engine's specialised forms)
  const char* env = getenv("TQ_EPI_FAST");
  const bool fast = !(env && atoi(env) == 0) && NKS == 1 && a.out == nullptr &&
                    a.codes_a != nullptr && a.codes_b == nullptr && a.lut_a > 0;
  if constexpr (NKS == 1) {
    if (fast && a.relu == kActSwish) return launch_xp_cfg<NKS, true, 3>(a, stream);
    if (fast && a.relu == 2) return launch_xp_cfg<NKS, false, 2>(a, stream);
    if (fast && a.relu == 1) return launch_xp_cfg<NKS, false, 1>(a, stream);
  }
  if (a.relu == kActSwish) return launch_xp_cfg<NKS, true, 0>(a, stream);
  return launch_xp_cfg<NKS, false, 0>(a, stream);
}

hipError_t launch_conv2d_xp(const ConvArgs& a, hipStream_t stream) {
  const int nks = a.Kp / kKStep;
  if (nks == 1) return launch_xp_nks<1>(a, stream);
  if (nks == 2) return launch_xp_nks<2>(a, stream);
  return hipErrorInvalidValue;
}

}  // namespace tq
