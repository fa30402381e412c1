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
// granules measured 26 us per step -- slower than these launches: DESIGN.md 7.)
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

}  // namespace tq
