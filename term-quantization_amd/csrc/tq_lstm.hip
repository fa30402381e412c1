// LSTM cell update of the term-pair LSTM path (tr_layer.TRLSTMLayer(termpair=True)): the
// point-wise half of one time step of torch.nn.LSTM's layer-0 recurrence (gate order i, f, g,
// o), given the step's input projection gx = TR(x) TR(W_ih)^T + b_ih (term-pair GEMM) and
// recurrent projection hh = h W_hh^T + b_hh:
//   gates = gx + hh;  c' = sigmoid(f) * c + sigmoid(i) * tanh(g);  h' = sigmoid(o) * tanh(c')
// One launch per step instead of the ~8 point-wise torch kernels; fp32 like the reference's
// cuDNN LSTM (its summation order is unpinned: DESIGN.md 3).
#include <math.h>

#include "tq_launch.h"

namespace tq {

namespace {

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ __launch_bounds__(256) void lstm_cell_kernel(const float* __restrict__ gx,
                                                        const float* __restrict__ hh,
                                                        float* __restrict__ c,
                                                        float* __restrict__ h, int64_t B,
                                                        int64_t H) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= B * H) return;
  const int64_t b = t / H;
  const int64_t j = t - b * H;
  const int64_t r = b * 4 * H + j;
  const float gi = gx[r] + hh[r];
  const float gf = gx[r + H] + hh[r + H];
  const float gg = gx[r + 2 * H] + hh[r + 2 * H];
  const float go = gx[r + 3 * H] + hh[r + 3 * H];
  const float cn = sigmoid_f(gf) * c[t] + sigmoid_f(gi) * tanhf(gg);
  c[t] = cn;
  h[t] = sigmoid_f(go) * tanhf(cn);
}

}  // namespace

hipError_t launch_lstm_cell(const float* gx, const float* hh, float* c, float* h, int64_t B,
                            int64_t H, hipStream_t stream) {
  const int64_t n = B * H;
  if (n == 0) return hipSuccess;
  lstm_cell_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, stream>>>(gx, hh, c, h, B, H);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------------------
// A whole LSTM layer's recurrence in one call (tq_lstm_seq_f32): T launches of one fused step
// kernel, enqueued from C++, instead of T x (a recurrent-projection GEMM + a cell kernel):
//   gates = gx[t] + b_hh + h_{t-1} W_hh^T;  c_t = sigmoid(f) c_{t-1} + sigmoid(i) tanh(g);
//   h_t = sigmoid(o) tanh(c_t)
// Workgroup g owns hidden units [g nu, (g + 1) nu) (nu = ceil(H / 256): 217 workgroups at
// H = 650, so the step's 6.8 MB of W_hh streams from L2 / the Infinity Cache through ~all CUs
// instead of the ~40 tiles a library GEMM of this 10-row shape gets): it stages h_{t-1} in
// LDS, 16 threads per gate row each take a 1/16 segment of the row's dot products for every
// batch row, and its cell threads finish the units.  The kernel boundary is the step's grid-
// wide hand-off.  (A persistent single-launch version exchanging h through agent-scope
// granules measured 26 us per step, and a cooperative two-layer one with W in registers and
// an agent-scope release/acquire grid barrier ~42 us per iteration -- both slower than these
// launches: DESIGN.md 7, profiles/r05_lstm_persistent_ab.txt.)
// fp32 throughout, like the reference's cuDNN LSTM; per dot product 16 partial sums of
// consecutive terms, added in a fixed order.
// ---------------------------------------------------------------------------------------
namespace {

constexpr int kStepThreads = 256;
constexpr int kStepSeg = 16;  // threads per gate row
constexpr int kStageRows = 16;  // rows per staging batch

struct LstmStepArgs {
  const float* gx;      // [B][4H] this step's input projection (incl. b_ih)
  const float* w;       // [4H][H]
  const float* b;       // [4H] or nullptr
  const float* h_prev;  // [B][H]
  const float* c_prev;  // [B][H]
  float* h;             // [B][H]
  float* c;             // [B][H] (may alias c_prev)
  int B, H, nu;
};

// L = segment length (compile time: every dot-product loop is straight-line code with no
// per-element guard); rows of h and W are staged zero-padded to HP = 16 L columns.
template <int L>
__global__ __launch_bounds__(kStepThreads) void lstm_step_kernel(LstmStepArgs a) {
  constexpr int HP = kStepSeg * L;
  extern __shared__ float step_lds[];
  const int H = a.H, B = a.B;
  const int tid = threadIdx.x;
  const int u0 = blockIdx.x * a.nu;
  const int nu = min(a.nu, H - u0);  // units of this workgroup (the last may own fewer)
  float* hprev = step_lds;                         // [B][HP]
  float* wrows = hprev + (int64_t)B * HP;          // [4 nu][HP]
  float* part = wrows + (int64_t)4 * a.nu * HP;    // [4 nu][B][kStepSeg]
  // cell-role operands first (their latency hides behind the staging below)
  const bool cell = tid < B * nu;
  const int ct = cell ? tid : 0;  // loads of non-cell threads stay in bounds (unused)
  const int cb = ct / nu, cu = ct - (ct / nu) * nu;
  const float* bsrc = a.b ? a.b : a.gx;  // no branch: the bias select happens at use
  float gpre[4], bpre[4];
#pragma unroll
  for (int gi = 0; gi < 4; ++gi) {
    const int col = gi * H + u0 + cu;
    gpre[gi] = a.gx[(int64_t)cb * 4 * H + col];
    bpre[gi] = bsrc[col];
  }
  const float cprev = a.c_prev[(int64_t)cb * H + u0 + cu];
  // this workgroup's 4 nu rows of W_hh, then the B rows of h_{t-1}, staged zero-padded with
  // coalesced loads, kStageRows rows per batch: all of a batch's loads are in flight before
  // its LDS stores (one L2 round trip per batch, not per row)
  constexpr int JC = (HP + kStepThreads - 1) / kStepThreads;
  const int nq = 4 * nu + B;
  for (int q0 = 0; q0 < nq; q0 += kStageRows) {
    float v[kStageRows][JC];
#pragma unroll
    for (int i = 0; i < kStageRows; ++i) {
      const int q = min(q0 + i, nq - 1);  // clamped: in-bounds loads, no branches
      const float* src = q < 4 * nu ? a.w + (int64_t)((q / nu) * H + u0 + q % nu) * H
                                    : a.h_prev + (int64_t)(q - 4 * nu) * H;
#pragma unroll
      for (int jj = 0; jj < JC; ++jj) {
        const int j = tid + jj * kStepThreads;
        const float x = src[min(j, H - 1)];
        v[i][jj] = j < H ? x : 0.0f;
      }
    }
#pragma unroll
    for (int i = 0; i < kStageRows; ++i) {
      const int q = q0 + i;
      if (q >= nq) break;
      float* dst = q < 4 * nu ? wrows + q * HP : hprev + (q - 4 * nu) * HP;
#pragma unroll
      for (int jj = 0; jj < JC; ++jj) {
        const int j = tid + jj * kStepThreads;
        if (j < HP) dst[j] = v[i][jj];
      }
    }
  }
  __syncthreads();
  // dot-product role: gate row r (gate r / nu, unit u0 + r % nu), segment s
  const int r = tid / kStepSeg, s = tid % kStepSeg;
  if (r < 4 * nu) {
    float wreg[L];
#pragma unroll
    for (int i = 0; i < L; ++i) wreg[i] = wrows[r * HP + s * L + i];
    for (int bb = 0; bb < B; ++bb) {
      const float* hp = hprev + bb * HP + s * L;
      float acc0 = 0.0f, acc1 = 0.0f;  // two chains; fixed order
#pragma unroll
      for (int i = 0; i + 1 < L; i += 2) {
        acc0 = fmaf(hp[i], wreg[i], acc0);
        acc1 = fmaf(hp[i + 1], wreg[i + 1], acc1);
      }
      if (L & 1) acc0 = fmaf(hp[L - 1], wreg[L - 1], acc0);
      part[((int64_t)r * B + bb) * kStepSeg + s] = acc0 + acc1;
    }
  }
  __syncthreads();
  if (cell) {  // cell role: (batch row cb, unit u0 + cu)
    float gate[4];
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      const float* pp = part + ((int64_t)(gi * nu + cu) * B + cb) * kStepSeg;
      float sum = 0.0f;
#pragma unroll
      for (int k = 0; k < kStepSeg; ++k) sum += pp[k];
      gate[gi] = gpre[gi] + (sum + (a.b ? bpre[gi] : 0.0f));
    }
    const int64_t o = (int64_t)cb * H + u0 + cu;
    const float c = sigmoid_f(gate[1]) * cprev + sigmoid_f(gate[0]) * tanhf(gate[2]);
    a.c[o] = c;
    a.h[o] = sigmoid_f(gate[3]) * tanhf(c);
  }
}

template <int L>
hipError_t launch_lstm_steps(LstmStepArgs a, const float* gx, const float* h0, const float* c0,
                             float* out, float* cT, int64_t T, hipStream_t stream) {
  constexpr int HP = kStepSeg * L;
  const int64_t B = a.B, H = a.H;
  const int grid = (int)((H + a.nu - 1) / a.nu);
  const size_t lds =
      ((size_t)B * HP + (size_t)4 * a.nu * HP + (size_t)4 * a.nu * B * kStepSeg) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_step_kernel<L>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  for (int64_t t = 0; t < T; ++t) {
    a.gx = gx + t * B * 4 * H;
    a.h_prev = t == 0 ? h0 : out + (t - 1) * B * H;
    a.c_prev = t == 0 ? c0 : cT;
    a.h = out + t * B * H;
    a.c = cT;
    lstm_step_kernel<L><<<dim3(grid), kStepThreads, lds, stream>>>(a);
  }
  return hipGetLastError();
}

}  // namespace

// Segment length of the step kernel for hidden size H (the templated L), 0 if H > 1024.
static int64_t lstm_seg_len(int64_t H) {
  const int64_t seg = (H + kStepSeg - 1) / kStepSeg;
  return seg <= 16 ? 16 : seg <= 32 ? 32 : seg <= 41 ? 41 : seg <= 48 ? 48 : seg <= 64 ? 64 : 0;
}

// 0 (no workspace) when the step kernel's LDS holds the shape, else -1 (unsupported).
int64_t lstm_seq_workspace_bytes(int64_t B, int64_t H) {
  // one cell thread per (batch row, unit) and 16 dot-product threads per gate row of a unit
  static_assert(4 * 4 * kStepSeg <= kStepThreads, "4 gate rows x nu <= 4 units of dot threads");
  const int64_t L = lstm_seg_len(H);
  if (B < 1 || H < 1 || L == 0) return -1;
  const int64_t HP = kStepSeg * L, nu = (H + 255) / 256;
  if (B * nu > kStepThreads) return -1;
  const int64_t lds = (B * HP + 4 * nu * HP + 4 * nu * B * kStepSeg) * 4;
  return lds <= 160 * 1024 ? 0 : -1;
}

hipError_t launch_lstm_seq(const float* gx, const float* w, const float* b, const float* h0,
                           const float* c0, float* out, float* cT, int64_t T, int64_t B,
                           int64_t H, void*, hipStream_t stream) {
  if (T == 0 || B == 0 || H == 0) return hipSuccess;
  LstmStepArgs a;
  a.w = w;
  a.b = b;
  a.B = (int)B;
  a.H = (int)H;
  a.nu = (int)((H + 255) / 256);  // <= 4 for H <= 1024
  switch (lstm_seg_len(H)) {
    case 16: return launch_lstm_steps<16>(a, gx, h0, c0, out, cT, T, stream);
    case 32: return launch_lstm_steps<32>(a, gx, h0, c0, out, cT, T, stream);
    case 41: return launch_lstm_steps<41>(a, gx, h0, c0, out, cT, T, stream);  // H = 650
    case 48: return launch_lstm_steps<48>(a, gx, h0, c0, out, cT, T, stream);
    case 64: return launch_lstm_steps<64>(a, gx, h0, c0, out, cT, T, stream);
    default: return hipErrorInvalidValue;
  }
}


// ---------------------------------------------------------------------------------------
// Two stacked layers in wavefront order (tq_lstm_seq2_f32): launch s runs layer 0's step s
// and layer 1's step s - 1 side by side in one grid (workgroups [0, G) and [G, 2G)), so a
// 2-layer recurrence of T steps takes T + 1 dependent launches instead of 2T plus the layer-1
// input-projection GEMM between them.  Layer 1's input projection h0_t W_ih1^T is computed
// in its step (it depends on layer 0's step t, finished by the previous launch):
//   layer 1: gates = (x_t W_ih^T + b_ih) + (h_{t-1} W_hh^T + b_hh),  x_t = layer 0's h_t
// Each dot product is 16 fixed-order partial sums; thread s of a gate row takes the column
// pairs (2 (s + 16 i), 2 (s + 16 i) + 1), i < P, so the wave's 8-byte W loads cover whole
// 64-byte runs of each row: W rows go straight from L2 into registers (no LDS staging, rows
// are 8-byte aligned for even H), and a workgroup needs only the staged h_{t-1} (and x_t) rows
// and the partial sums: <= 80 KB of LDS at LSTM-650, two workgroups per CU, both layers'
// grids resident at once.
// ---------------------------------------------------------------------------------------
namespace {

struct LstmRole {
  const float* gx;      // layer 0: [B][4H] this step's input projection (incl. b_ih)
  const float* x;       // layer 1: [B][H] this step's input (layer 0's h at the same step)
  const float* w_ih;    // layer 1: [4H][H]
  const float* b_ih;    // layer 1: [4H] or nullptr
  const float* w;       // W_hh [4H][H]
  const float* b;       // b_hh [4H] or nullptr
  const float* h_prev;  // [B][H]
  const float* c_prev;  // [B][H]
  float* h;             // [B][H]
  float* c;             // [B][H] (may alias c_prev)
};

struct LstmStep2Args {
  LstmRole r[2];
  int first;  // role of workgroups [0, G): 0, or 1 when layer 0 has no step left
  int B, H, nu, G;
};

// LDS floats of a workgroup: h_{t-1} and x rows [B][HP] each, partial sums [2][4 nu][B][16]
__host__ __device__ constexpr int64_t lstm2_lds_floats(int64_t B, int64_t HP, int64_t nu) {
  return 2 * B * HP + 2 * 4 * nu * B * kStepSeg;
}

template <int P, bool X2>
__device__ __forceinline__ void lstm2_role(const LstmRole& a, int wg, int B, int H, int nu_max,
                                           float* lds) {
  constexpr int HP = 2 * kStepSeg * P;  // staged row length (zero-padded)
  const int tid = threadIdx.x;
  const int u0 = wg * nu_max;
  const int nu = min(nu_max, H - u0);
  float* hprev = lds;                                   // [B][HP]
  float* xin = hprev + (int64_t)B * HP;                 // [B][HP] (X2)
  float* part_h = xin + (int64_t)B * HP;                // [4 nu][B][kStepSeg]
  float* part_x = part_h + (int64_t)4 * nu_max * B * kStepSeg;
  const bool cell = tid < B * nu;
  const int ct = cell ? tid : 0;
  const int cb = ct / nu, cu = ct - (ct / nu) * nu;
  float gpre[4], bpre[4], xbpre[4];
#pragma unroll
  for (int gi = 0; gi < 4; ++gi) {
    const int col = gi * H + u0 + cu;
    gpre[gi] = X2 ? 0.0f : a.gx[(int64_t)cb * 4 * H + col];
    bpre[gi] = a.b ? a.b[col] : 0.0f;
    xbpre[gi] = X2 && a.b_ih ? a.b_ih[col] : 0.0f;
  }
  const float cprev = a.c_prev[(int64_t)cb * H + u0 + cu];
  // dot-product role: gate row r (gate r / nu, unit u0 + r % nu), segment s; its W segments
  // straight into registers (L2-resident rows)
  const int r = tid / kStepSeg, s = tid % kStepSeg;
  const bool dot = r < 4 * nu;
  const int64_t wrow = dot ? (int64_t)((r / nu) * H + u0 + r % nu) * H : 0;
  float2 wh[P], wx[X2 ? P : 1];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int j = 2 * (s + kStepSeg * i);  // H even: a pair is in the row or wholly past it
    const bool ok = dot && j < H;
    wh[i] = ok ? *reinterpret_cast<const float2*>(a.w + wrow + j) : make_float2(0.f, 0.f);
    if (X2)
      wx[i] = ok ? *reinterpret_cast<const float2*>(a.w_ih + wrow + j) : make_float2(0.f, 0.f);
  }
  // stage h_{t-1} (and x_t) zero-padded to HP columns, kStageRows rows per batch of loads
  constexpr int JC = (HP + kStepThreads - 1) / kStepThreads;
  const int nrow = X2 ? 2 * B : B;
  for (int q0 = 0; q0 < nrow; q0 += kStageRows) {
    float v[kStageRows][JC];
#pragma unroll
    for (int i = 0; i < kStageRows; ++i) {
      const int q = min(q0 + i, nrow - 1);  // clamped: in-bounds loads, no branches
      const float* src = q < B ? a.h_prev + (int64_t)q * H : a.x + (int64_t)(q - B) * H;
#pragma unroll
      for (int jj = 0; jj < JC; ++jj) {
        const int j = tid + jj * kStepThreads;
        const float x = src[min(j, H - 1)];
        v[i][jj] = j < H ? x : 0.0f;
      }
    }
#pragma unroll
    for (int i = 0; i < kStageRows; ++i) {
      const int q = q0 + i;
      if (q >= nrow) break;
      float* dst = q < B ? hprev + q * HP : xin + (q - B) * HP;
#pragma unroll
      for (int jj = 0; jj < JC; ++jj) {
        const int j = tid + jj * kStepThreads;
        if (j < HP) dst[j] = v[i][jj];
      }
    }
  }
  __syncthreads();
  if (dot) {
    for (int bb = 0; bb < B; ++bb) {
      const float2* hp = reinterpret_cast<const float2*>(hprev + bb * HP) + s;
      float acc0 = 0.0f, acc1 = 0.0f;  // two chains (even / odd columns); fixed order
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const float2 hv = hp[kStepSeg * i];
        acc0 = fmaf(hv.x, wh[i].x, acc0);
        acc1 = fmaf(hv.y, wh[i].y, acc1);
      }
      part_h[((int64_t)r * B + bb) * kStepSeg + s] = acc0 + acc1;
      if (X2) {
        const float2* xp = reinterpret_cast<const float2*>(xin + bb * HP) + s;
        float x0 = 0.0f, x1 = 0.0f;
#pragma unroll
        for (int i = 0; i < P; ++i) {
          const float2 xv = xp[kStepSeg * i];
          x0 = fmaf(xv.x, wx[i].x, x0);
          x1 = fmaf(xv.y, wx[i].y, x1);
        }
        part_x[((int64_t)r * B + bb) * kStepSeg + s] = x0 + x1;
      }
    }
  }
  __syncthreads();
  if (cell) {
    float gate[4];
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      const int64_t pi = ((int64_t)(gi * nu + cu) * B + cb) * kStepSeg;
      float sum = 0.0f;
#pragma unroll
      for (int k = 0; k < kStepSeg; ++k) sum += part_h[pi + k];
      float gxv = gpre[gi];
      if (X2) {
        float xs = 0.0f;
#pragma unroll
        for (int k = 0; k < kStepSeg; ++k) xs += part_x[pi + k];
        gxv = xs + xbpre[gi];
      }
      gate[gi] = gxv + (sum + bpre[gi]);
    }
    const int64_t o = (int64_t)cb * H + u0 + cu;
    const float c = sigmoid_f(gate[1]) * cprev + sigmoid_f(gate[0]) * tanhf(gate[2]);
    a.c[o] = c;
    a.h[o] = sigmoid_f(gate[3]) * tanhf(c);
  }
}

template <int P>
__global__ __launch_bounds__(kStepThreads) void lstm_step2_kernel(LstmStep2Args a) {
  extern __shared__ float step2_lds[];
  const int role = a.first + (int)(blockIdx.x / a.G);
  const int wg = (int)(blockIdx.x % a.G);
  if (role == 0)
    lstm2_role<P, false>(a.r[0], wg, a.B, a.H, a.nu, step2_lds);
  else
    lstm2_role<P, true>(a.r[1], wg, a.B, a.H, a.nu, step2_lds);
}

// column pairs per thread of the two-layer kernel: 32 P >= H (0: H outside its domain)
static int lstm2_pairs(int64_t H) {
  if (H < 2 || (H & 1)) return 0;
  const int64_t p = (H + 31) / 32;
  return p <= 8 ? 8 : p <= 16 ? 16 : p <= 21 ? 21 : p <= 24 ? 24 : p <= 32 ? 32 : 0;
}

template <int P>
hipError_t launch_lstm_steps2(LstmStep2Args a, const float* gx0, const float* h00,
                              const float* c00, const float* h01, const float* c01, float* out0,
                              float* out1, float* cT0, float* cT1, int64_t T,
                              hipStream_t stream) {
  constexpr int HP = 2 * kStepSeg * P;
  const int64_t B = a.B, H = a.H;
  const size_t lds = (size_t)lstm2_lds_floats(B, HP, a.nu) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_step2_kernel<P>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  for (int64_t s = 0; s <= T; ++s) {
    const bool have0 = s < T, have1 = s >= 1;
    if (have0) {  // layer 0, step s
      LstmRole& r = a.r[0];
      r.gx = gx0 + s * B * 4 * H;
      r.h_prev = s == 0 ? h00 : out0 + (s - 1) * B * H;
      r.c_prev = s == 0 ? c00 : cT0;
      r.h = out0 + s * B * H;
      r.c = cT0;
    }
    if (have1) {  // layer 1, step s - 1 (its input: layer 0's step s - 1)
      const int64_t t = s - 1;
      LstmRole& r = a.r[1];
      r.x = out0 + t * B * H;
      r.h_prev = t == 0 ? h01 : out1 + (t - 1) * B * H;
      r.c_prev = t == 0 ? c01 : cT1;
      r.h = out1 + t * B * H;
      r.c = cT1;
    }
    a.first = have0 ? 0 : 1;
    const int grid = a.G * ((have0 ? 1 : 0) + (have1 ? 1 : 0));
    lstm_step2_kernel<P><<<dim3(grid), kStepThreads, lds, stream>>>(a);
  }
  return hipGetLastError();
}

}  // namespace

bool lstm_seq2_supported(int64_t B, int64_t H) {
  const int64_t P = lstm2_pairs(H);
  if (B < 1 || P == 0) return false;
  const int64_t nu = (H + 255) / 256;
  if (B * nu > kStepThreads) return false;
  return lstm2_lds_floats(B, 2 * kStepSeg * P, nu) * 4 <= 160 * 1024;
}

hipError_t launch_lstm_seq2(const float* gx0, const float* w_hh0, const float* b_hh0,
                            const float* h00, const float* c00, const float* w_ih1,
                            const float* b_ih1, const float* w_hh1, const float* b_hh1,
                            const float* h01, const float* c01, float* out0, float* out1,
                            float* cT0, float* cT1, int64_t T, int64_t B, int64_t H,
                            hipStream_t stream) {
  if (T == 0 || B == 0 || H == 0) return hipSuccess;
  LstmStep2Args a = {};
  a.r[0].w = w_hh0;
  a.r[0].b = b_hh0;
  a.r[1].w_ih = w_ih1;
  a.r[1].b_ih = b_ih1;
  a.r[1].w = w_hh1;
  a.r[1].b = b_hh1;
  a.B = (int)B;
  a.H = (int)H;
  a.nu = (int)((H + 255) / 256);
  a.G = (int)((H + a.nu - 1) / a.nu);
  switch (lstm2_pairs(H)) {
#define TQ_SEQ2(PP)                                                                         \
  case PP:                                                                                   \
    return launch_lstm_steps2<PP>(a, gx0, h00, c00, h01, c01, out0, out1, cT0, cT1, T, stream);
    TQ_SEQ2(8)
    TQ_SEQ2(16)
    TQ_SEQ2(21)  // H = 650
    TQ_SEQ2(24)
    TQ_SEQ2(32)
#undef TQ_SEQ2
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tq
