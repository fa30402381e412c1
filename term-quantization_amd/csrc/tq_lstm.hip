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
// A whole LSTM layer's recurrence in one persistent launch (tq_lstm_seq_f32): T steps of
//   gates = gx[t] + b_hh + h_{t-1} W_hh^T;  c_t = sigmoid(f) c_{t-1} + sigmoid(i) tanh(g);
//   h_t = sigmoid(o) tanh(c_t)
// instead of T x (a small GEMM launch + a cell launch).  Workgroup g owns hidden units
// [g nu, (g + 1) nu): its 4 nu rows of W_hh stay in registers (16 threads per row, one
// 1/16 segment of the row each) for all T steps, and it runs those units' cell updates.
// Every step needs the whole h_{t-1}: each workgroup publishes its units' h_t as 8-byte
// {epoch, value} granules (agent-scope, write-through stores: the data is the flag, no
// fence), into one of two buffers by step parity, and every workgroup sweeps all granules
// of the previous step (agent-scope loads) into LDS.  Buffer reuse is safe: a workgroup
// overwrites a step-t granule (at step t + 2) only after it has seen every workgroup's step
// t + 1 granules, which each published after finishing its sweep of step t.  The granule
// buffers are zeroed by the launcher before every launch (tags start from 1).  Every spin is
// bounded: a wait that runs out counts in g_lstm_seq_faults (tq_sync_faults) and the kernel
// still finishes.
// fp32 throughout, like the reference's cuDNN LSTM; per dot product 16 partial sums of
// consecutive terms, added in a fixed order.
// ---------------------------------------------------------------------------------------
namespace {

constexpr int kSeqThreads = 256;
constexpr int kSeqSeg = 16;   // threads per gate row
constexpr int kSeqLMax = 64;  // weights per thread: H <= 1024
constexpr int kSeqBatch = 16; // granule loads in flight per thread during a sweep

__device__ uint32_t g_lstm_seq_faults;

struct LstmSeqArgs {
  const float* gx;  // [T][B][4H]
  const float* w;   // [4H][H]
  const float* b;   // [4H] or nullptr
  const float* h0;  // [B][H]
  const float* c0;  // [B][H]
  float* out;       // [T][B][H]
  float* cT;        // [B][H]
  uint64_t* gran;   // [2][B][H] granules, zeroed before the launch
  int T, B, H, nu;
};

__global__ __launch_bounds__(kSeqThreads) void lstm_seq_kernel(LstmSeqArgs a) {
  extern __shared__ float seq_lds[];
  const int H = a.H, B = a.B;
  float* hprev = seq_lds;                  // [B][H]
  float* part = seq_lds + (int64_t)B * H;  // [4 nu][B][kSeqSeg]
  const int tid = threadIdx.x;
  const int u0 = blockIdx.x * a.nu;
  const int nu = min(a.nu, H - u0);  // units of this workgroup (the last may own fewer)
  const int L = (H + kSeqSeg - 1) / kSeqSeg;
  // dot-product role: gate row r (gate gr = r / nu, unit u0 + r % nu), segment s
  const int r = tid / kSeqSeg, s = tid % kSeqSeg;
  const bool dot = r < 4 * nu;
  const int grow = dot ? (r / nu) * H + u0 + (r % nu) : 0;
  float wreg[kSeqLMax];
#pragma unroll
  for (int i = 0; i < kSeqLMax; ++i) {
    const int j = s * L + i;
    wreg[i] = (dot && i < L && j < H) ? a.w[(int64_t)grow * H + j] : 0.0f;
  }
  // cell role: (batch row cb, unit u0 + cu); its c stays in a register
  const int cb = tid / nu, cu = tid - (tid / nu) * nu;
  const bool cell = tid < B * nu;
  float c = cell ? a.c0[(int64_t)cb * H + u0 + cu] : 0.0f;
  uint32_t spins_left = 1u << 24;

  for (int t = 0; t < a.T; ++t) {
    // h_{t-1} into LDS: the initial state, or every workgroup's step t-1 granules
    if (t == 0) {
      for (int i = tid; i < B * H; i += kSeqThreads) hprev[i] = a.h0[i];
    } else {
      const uint64_t* g = a.gran + (int64_t)((t - 1) & 1) * B * H;
      const uint32_t epoch = (uint32_t)t;  // step t - 1 published tag t
      // kSeqBatch granules per thread in flight at once, then re-poll only those not ready
      for (int i0 = tid; i0 < B * H; i0 += kSeqBatch * kSeqThreads) {
        uint64_t v[kSeqBatch];
#pragma unroll
        for (int k = 0; k < kSeqBatch; ++k) {
          const int i = i0 + k * kSeqThreads;
          v[k] = i < B * H ? __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : ((uint64_t)epoch << 32);
        }
        // not-ready granules are re-polled together: one round trip per retry, not one per
        // granule
        uint32_t pending = 0;
#pragma unroll
        for (int k = 0; k < kSeqBatch; ++k)
          pending |= (uint32_t)((uint32_t)(v[k] >> 32) != epoch) << k;
        while (pending && spins_left) {
          __builtin_amdgcn_s_sleep(2);
          --spins_left;
#pragma unroll
          for (int k = 0; k < kSeqBatch; ++k)
            if ((pending >> k) & 1u)
              v[k] = __hip_atomic_load(g + i0 + k * kSeqThreads, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
          pending = 0;
#pragma unroll
          for (int k = 0; k < kSeqBatch; ++k)
            pending |= (uint32_t)((uint32_t)(v[k] >> 32) != epoch) << k;
        }
#pragma unroll
        for (int k = 0; k < kSeqBatch; ++k) {
          const int i = i0 + k * kSeqThreads;
          if (i < B * H) hprev[i] = __uint_as_float((uint32_t)v[k]);
        }
      }
    }
    __syncthreads();
    if (dot) {
      const int j0 = s * L;
      for (int bb = 0; bb < B; ++bb) {
        const float* hp = hprev + (int64_t)bb * H + j0;
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < kSeqLMax; ++i)
          if (i < L && j0 + i < H) acc = fmaf(hp[i], wreg[i], acc);
        part[((int64_t)r * B + bb) * kSeqSeg + s] = acc;
      }
    }
    __syncthreads();
    if (cell) {
      float gate[4];
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) {
        const int rr = gi * nu + cu;
        const float* pp = part + ((int64_t)rr * B + cb) * kSeqSeg;
        float sum = 0.0f;
#pragma unroll
        for (int k = 0; k < kSeqSeg; ++k) sum += pp[k];
        const int col = gi * H + u0 + cu;
        const float bias = a.b ? a.b[col] : 0.0f;
        gate[gi] = a.gx[((int64_t)t * B + cb) * 4 * H + col] + (sum + bias);
      }
      c = sigmoid_f(gate[1]) * c + sigmoid_f(gate[0]) * tanhf(gate[2]);
      const float h = sigmoid_f(gate[3]) * tanhf(c);
      const int64_t o = (int64_t)cb * H + u0 + cu;
      a.out[(int64_t)t * B * H + o] = h;
      if (t + 1 < a.T) {
        const uint64_t gv = ((uint64_t)(uint32_t)(t + 1) << 32) | __float_as_uint(h);
        __hip_atomic_store(a.gran + (int64_t)(t & 1) * B * H + o, gv, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      } else {
        a.cT[o] = c;
      }
    }
  }
  if (spins_left == 0u)
    __hip_atomic_fetch_add(&g_lstm_seq_faults, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

int64_t lstm_seq_workspace_bytes(int64_t B, int64_t H) { return 2 * B * H * 8; }

hipError_t launch_lstm_seq(const float* gx, const float* w, const float* b, const float* h0,
                           const float* c0, float* out, float* cT, int64_t T, int64_t B,
                           int64_t H, void* ws, hipStream_t stream) {
  if (T == 0 || B == 0 || H == 0) return hipSuccess;
  LstmSeqArgs a;
  a.gx = gx;
  a.w = w;
  a.b = b;
  a.h0 = h0;
  a.c0 = c0;
  a.out = out;
  a.cT = cT;
  a.gran = reinterpret_cast<uint64_t*>(ws);
  a.T = (int)T;
  a.B = (int)B;
  a.H = (int)H;
  a.nu = (int)((H + 255) / 256);  // <= 4 for H <= 1024
  const int grid = (int)((H + a.nu - 1) / a.nu);
  hipError_t e = hipMemsetAsync(ws, 0, (size_t)lstm_seq_workspace_bytes(B, H), stream);
  if (e != hipSuccess) return e;
  const size_t lds = ((size_t)B * H + (size_t)4 * a.nu * B * kSeqSeg) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_seq_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  lstm_seq_kernel<<<dim3(grid), kSeqThreads, lds, stream>>>(a);
  return hipGetLastError();
}

hipError_t lstm_seq_faults(uint32_t* count) {
  uint32_t zero = 0;
  hipError_t e = hipMemcpyFromSymbol(count, HIP_SYMBOL(g_lstm_seq_faults), sizeof(uint32_t));
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_lstm_seq_faults), &zero, sizeof(uint32_t));
}

}  // namespace tq
