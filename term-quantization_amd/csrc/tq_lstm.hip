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

}  // namespace tq
