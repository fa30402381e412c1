/*
 * oracle/tr_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, line-by-line CPU restatement of the reference term-revealing (TR) op
 * (BradMcDanel/term-quantization, kernels/tr_cuda_kernel.cu).  It exists to CHECK the
 * MI355X HIP path; nothing in the product links or calls it.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Deliberately naive: the 64-slot encode loop and the greedy k x g selection are written
 * exactly as the reference kernel does them, so the fast closed-form / threshold design in
 * term-quantization_amd/csrc/ is checked against an independent formulation.
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - HESE encode is pinned bit-for-bit against the reference's own Python encoder
 *     bit_utils.hese (tests/golden/hese_*.npz + SHA-256 of the full q < 2^17 table).
 *   - Quantize / select / rescale follow the CUDA source literally (PTX semantics for
 *     shifts and float->int conversion spelled out below).  The CUDA kernel itself cannot
 *     be built in this image (it needs ATen + CUDA headers), so those steps are pinned to
 *     this restatement only ("parity partially pinned").
 *
 * Deviations, all in territory where the reference is undefined or racy:
 *   - C % group_size != 0: the reference's last group of a row spills into the next row
 *     (and past the tensor end); here the last group is the partial group [floor(C/g)*g, C).
 *   - The spatial offset uses w*H+h (the reference's w*W+h, tr_cuda_kernel.cu:76, is only
 *     right for W == H).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_MAX_GROUP_SIZE 32 /* kernels/tr_cuda_kernel.cu:9 */
#define ORACLE_MAX_TERMS 64      /* kernels/tr_cuda_kernel.cu:10 */

/* ---- PTX semantics that the CUDA source relies on ---------------------------------- */

/* shr.s32: shift counts >= 32 are clamped, so a non-negative value shifts to 0.  x86 masks
 * the count to 5 bits instead, which is why the kernel body cannot be compiled as-is. */
static int32_t ptx_shr_s32(int32_t v, int s) {
    if (s > 31) s = 31;
    return v >> s;
}

/* shl.b32: shift counts >= 32 give 0. */
static int32_t ptx_shl_b32(int32_t v, int s) {
    if (s > 31) return 0;
    return (int32_t)((uint32_t)v << s);
}

/* cvt.rzi.s32.f64 / cvt.rzi.s32.f32: truncate, saturate, NaN -> 0. */
static int32_t cvt_rzi_s32_f64(double t) {
    if (t != t) return 0;
    if (t >= 2147483647.0) return INT32_MAX;
    if (t <= -2147483648.0) return INT32_MIN;
    return (int32_t)t;
}

static int32_t cvt_rzi_s32_f32(float t) {
    return cvt_rzi_s32_f64((double)t);
}

/* ---- a1 + a2: quantize and HESE-encode one element ---------------------------------- */

/* kernels/tr_cuda_kernel.cu:14-56 (hese_encode), with the quantize step :21-23.
 * `mag_over_sf_plus_half` is `abs(input) / sf + 0.5` evaluated in the input's precision
 * (float division then a double +0.5 for float; all-double for double). */
static void hese_encode_q(double mag_over_sf_plus_half, int32_t sign, int32_t bitwidth,
                          int32_t *terms, int32_t *num_terms) {
    float maxv = (float)(pow(2.0, (double)bitwidth) - 1.0);                 /* :21 */
    int32_t q_val = cvt_rzi_s32_f32(fminf((float)cvt_rzi_s32_f64(mag_over_sf_plus_half),
                                          maxv));                           /* :22 */
    *num_terms = 0;                                                           /* :24 */
    for (int i = 0; i < ORACLE_MAX_TERMS; i++) terms[i] = 0;                  /* :25-27 */

    for (int i = ORACLE_MAX_TERMS - 1; i >= 0; i--) {                         /* :29 */
        int32_t b0 = i == 0 ? 0 : ptx_shr_s32(q_val, i - 1) & 1;              /* :30 */
        int32_t b1 = ptx_shr_s32(q_val, i) & 1;                               /* :31 */
        int32_t b2 = i == ORACLE_MAX_TERMS - 1 ? 0 : ptx_shr_s32(q_val, i + 1) & 1; /* :32 */

        if (b2 == 0 && b1 == 0 && b0 == 0) {
            continue;
        } else if (b2 == 0 && b1 == 0 && b0 == 1) {
            continue;
        } else if (b2 == 0 && b1 == 1 && b0 == 0) {                           /* :38-41 */
            terms[*num_terms] = sign * ptx_shl_b32(1, i);
            (*num_terms)++;
            i--;
        } else if (b2 == 0 && b1 == 1 && b0 == 1) {                           /* :42-44 */
            terms[*num_terms] = sign * ptx_shl_b32(1, i + 1);
            (*num_terms)++;
        } else if (b2 == 1 && b1 == 0 && b0 == 0) {
            continue;
        } else if (b2 == 1 && b1 == 0 && b0 == 1) {
            continue;
        } else if (b2 == 1 && b1 == 1 && b0 == 0) {                           /* :49-51 */
            terms[*num_terms] = (-sign) * ptx_shl_b32(1, i);
            (*num_terms)++;
        } else {
            continue;
        }
    }
}

static void encode_f32(float x, float sf, int32_t bitwidth, int32_t *terms, int32_t *n) {
    /* float / float, then the double literal 0.5 promotes (tr_cuda_kernel.cu:22) */
    double t = (double)(fabsf(x) / sf) + 0.5;
    hese_encode_q(t, x < 0 ? -1 : 1, bitwidth, terms, n);
}

static void encode_f64(double x, float sf, int32_t bitwidth, int32_t *terms, int32_t *n) {
    double t = fabs(x) / (double)sf + 0.5;
    hese_encode_q(t, x < 0 ? -1 : 1, bitwidth, terms, n);
}

/* Exported for the HESE golden-table test: the term list of a non-negative integer q,
 * most significant first, as the reference encoder produces it (q must be < 2^31). */
int oracle_hese_terms(int32_t q, int32_t sign, int32_t *terms_out /* [64] */) {
    int32_t n = 0;
    /* q + 0.5 truncates back to q; bitwidth 31 keeps maxv >= q for every q < 2^31 */
    hese_encode_q((double)q + 0.5, sign, 31, terms_out, &n);
    return n;
}

/* ---- a3 + a4 + a5: the kernel body, run serially over groups ------------------------ */

static int32_t iabs32(int32_t v) { return v < 0 ? -v : v; }

/* Host launcher shape rules, kernels/tr_cuda_kernel.cu:133-141: B=size(0), C=size(1),
 * W,H = size(2),size(3) only for 4-D tensors, else 1. */
static int shape_bcwh(int64_t ndim, const int64_t *shape, int64_t *B, int64_t *C, int64_t *W,
                      int64_t *H) {
    if (ndim < 2) return -1;
    *B = shape[0];
    *C = shape[1];
    *W = 1;
    *H = 1;
    if (ndim == 4) {
        *W = shape[2];
        *H = shape[3];
    }
    return 0;
}

#define ORACLE_TR_BODY(SCALAR, ENCODE)                                                        \
    int64_t B, C, W, H;                                                                       \
    if (shape_bcwh(ndim, shape, &B, &C, &W, &H) != 0) return -1;                              \
    if (group_size < 1 || group_size > ORACLE_MAX_GROUP_SIZE) return -2;                      \
    int64_t numel = 1;                                                                        \
    for (int64_t d = 0; d < ndim; ++d) numel *= shape[d];                                     \
    for (int64_t i = 0; i < numel; ++i) output[i] = 0; /* at::zeros_like, :145 */             \
    const int64_t WH = W * H, CWH = C * WH;                                                   \
    const int64_t ngroups = (C + group_size - 1) / group_size; /* ceilf(C/g), :77 */          \
    int32_t term_idx[ORACLE_MAX_GROUP_SIZE];                                                  \
    int32_t num_terms[ORACLE_MAX_GROUP_SIZE];                                                 \
    static __thread int32_t terms[ORACLE_MAX_GROUP_SIZE * ORACLE_MAX_TERMS];                  \
    for (int64_t b = 0; b < B; ++b)                                                           \
        for (int64_t c = 0; c < ngroups; ++c)                                                 \
            for (int64_t s = 0; s < WH; ++s) {                                                \
                const int64_t base_offset = b * CWH + s;                                      \
                int64_t gs = C - c * group_size;                                              \
                if (gs > group_size) gs = group_size;                                         \
                for (int i = 0; i < gs; ++i) { /* :85-90 */                                   \
                    int64_t gidx = (c * group_size + i) * WH + base_offset;                   \
                    output[gidx] = 0;                                                         \
                    term_idx[i] = 0;                                                          \
                    ENCODE(input[gidx], sf, bitwidth, &terms[i * ORACLE_MAX_TERMS],           \
                           &num_terms[i]);                                                    \
                }                                                                             \
                for (int i = 0; i < num_keep_terms; ++i) { /* :92-116 */                      \
                    int32_t max_idx = 0;                                                      \
                    int32_t max_val = 0;                                                      \
                    for (int j = 0; j < gs; ++j) {                                            \
                        int32_t t = term_idx[j] < ORACLE_MAX_TERMS                            \
                                        ? terms[j * ORACLE_MAX_TERMS + term_idx[j]]           \
                                        : 0;                                                  \
                        if (iabs32(t) > iabs32(max_val)) {                                    \
                            max_val = t;                                                      \
                            max_idx = j;                                                      \
                        }                                                                     \
                    }                                                                         \
                    if (max_val == 0) break;                                                  \
                    int64_t gidx = (c * group_size + max_idx) * WH + base_offset;             \
                    output[gidx] += (SCALAR)max_val;                                          \
                    term_idx[max_idx]++;                                                      \
                }                                                                             \
                for (int i = 0; i < gs; ++i) { /* :119-123 */                                 \
                    int64_t gidx = (c * group_size + i) * WH + base_offset;                   \
                    output[gidx] *= (SCALAR)sf;                                               \
                }                                                                             \
            }                                                                                 \
    return 0;

/* tr() on a float32 tensor (kernels/tr_cuda_kernel.cu:58-125 + :128-160). */
int oracle_tr_f32(const float *input, float *output, int64_t ndim, const int64_t *shape,
                  float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms) {
    ORACLE_TR_BODY(float, encode_f32)
}

/* tr() on a float64 tensor (the AT_DISPATCH_FLOATING_TYPES double instantiation). */
int oracle_tr_f64(const double *input, double *output, int64_t ndim, const int64_t *shape,
                  float sf, int32_t bitwidth, int32_t group_size, int32_t num_keep_terms) {
    ORACLE_TR_BODY(double, encode_f64)
}
