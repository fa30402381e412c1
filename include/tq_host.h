/*
 * tq_host.h -- C ABI of the host (CPU) term-revealing op, libtq_host.so.
 *
 * The reference's TR extension only accepts CUDA tensors (kernels/tr_cuda.cpp:12-18), yet its
 * MNIST configuration runs on CPU torch when CUDA is off (evaluate_mlp.py:56-57,
 * train_mlp.py:90-94) -- with the TR op it could not call.  SURVEY.md 8(b) makes CPU tensors a
 * deliberate extension of the boundary: this library is that product CPU path.  It is NOT the
 * oracle (oracle/tr_oracle.c, a literal serial restatement used only by tests); it is the same
 * closed-form HESE + exponent-threshold selection design as the HIP kernels
 * (csrc/tq_device.h, csrc/tr_op.hip), multithreaded with OpenMP, and it must agree with the
 * HIP path and the oracle bit for bit.
 *
 * All pointers are host pointers.  Every entry point returns TQ_OK (0) or a TQ_ERR_* code
 * (the values of include/tq.h); tq_host_last_error() then describes it for the calling
 * thread.  Calls are synchronous, keep no global mutable state besides the per-thread error
 * message, and are safe from several host threads.
 */
#ifndef TQ_HOST_H_
#define TQ_HOST_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Library version string, e.g. "tq-host 0.1.0". */
const char *tq_host_version(void);

/* Message for the last non-OK return on the calling thread ("" if none). */
const char *tq_host_last_error(void);

/*
 * tq_tr_f32 / tq_tr_f64 / tq_tr_encode_f32 of include/tq.h on host memory: the pybind entry
 *   at::Tensor tr(const at::Tensor input, const float sf, const int32_t bitwidth,
 *                 const int32_t group_size, const int32_t num_keep_terms)
 * (kernels/tr_cuda.cpp:20-24, launcher kernels/tr_cuda_kernel.cu:128-160) for CPU tensors.
 * Same shape rules, domain (0 <= bitwidth <= 24, 1 <= group_size <= 32, sf >= 0, ndim >= 2),
 * partial last group for C % group_size != 0, and zero tail for 3-D / 5-D inputs.
 * `num_threads` <= 0 uses the OpenMP default (OMP_NUM_THREADS).
 */
int tq_tr_f32_host(const float *input, float *output, int64_t ndim, const int64_t *shape,
                   float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms,
                   int32_t num_threads);
int tq_tr_f64_host(const double *input, double *output, int64_t ndim, const int64_t *shape,
                   float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms,
                   int32_t num_threads);
int tq_tr_encode_f32_host(const float *input, float *output, int32_t *codes, int64_t ndim,
                          const int64_t *shape, float sf, int32_t bitwidth, int32_t group_size,
                          int32_t num_keep_terms, int32_t num_threads);

/*
 * tq_mse_profile of include/tq.h on host memory (tr_layer.py:43-54):
 *   errs[s] = sum_b hist[b] * (x[b] - TR(x[b]; sfs[s], bitwidth, group 1, k))^2
 * with the per-bin term in fp32 (no contraction) and the bin sum in fp64 in the same fixed
 * order as the HIP kernel (256 strided partial sums, then a pairwise tree), so host and
 * device return identical errs.
 */
int tq_mse_profile_host(const float *x, const float *hist, int64_t nbins, const float *sfs,
                        int64_t nsf, int32_t bitwidth, int32_t num_keep_terms, double *errs,
                        int32_t num_threads);

#ifdef __cplusplus
}
#endif

#endif /* TQ_HOST_H_ */
