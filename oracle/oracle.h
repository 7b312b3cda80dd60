/*
 * plssvm oracle — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference PLSSVM OpenMP hot path (the CG solver's implicit
 * kernel-matrix·vector product Q~·p), used as the parity checker for the MI355X backend.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product library (plssvm_sparse_fp22_amd/csrc) never links, calls or falls back to it.
 *
 * Pinning: the reference cannot be compiled in this container without writing stand-ins
 * for {fmt} and fast_float (absent from the image), so it is treated as unbuildable.
 * This restatement is pinned by the reference's own fixtures instead:
 *   - tests/data/libsvm/5x4.libsvm -> tests/data/models/5x4.libsvm.model (golden learn():
 *     alphas + rho, linear, fp64);
 *   - tests/data/models/500x200.libsvm.{linear,polynomial,rbf}.model +
 *     tests/data/libsvm/500x200.libsvm.test -> tests/data/predict/500x200.libsvm.predict
 *     (pins kernel_function<linear|poly|rbf> through predicted labels);
 *   - the reference's known-answer method compare::device_kernel_function / generate_q
 *     (tests/backends/compare.hpp:103-156) re-run here in numpy on the same inputs.
 * See tests/test_oracle.py.
 *
 * Functions are provided for REAL = double (_f64) and REAL = float (_f32).
 * kernel: 0 = linear, 1 = polynomial, 2 = rbf  (include/plssvm/kernel_types.hpp:27-34)
 */
#ifndef PLSSVM_ORACLE_H
#define PLSSVM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_DECLARE(REAL, SUF)                                                                                  \
    REAL orc_kernel_##SUF(int kernel, int degree, REAL gamma, REAL coef0, const REAL *a, const REAL *b,         \
                          int64_t d);                                                                           \
    void orc_q_##SUF(int kernel, int degree, REAL gamma, REAL coef0, const REAL *X, int64_t n, int64_t d,       \
                     REAL *q);                                                                                  \
    void orc_kp_##SUF(int kernel, int degree, REAL gamma, REAL coef0, const REAL *X, int64_t n, int64_t d,      \
                      const REAL *q, REAL QA_cost, REAL cost_inv, REAL add, const REAL *p, REAL *ret,           \
                      int nthreads);                                                                            \
    void orc_q_csr_##SUF(int kernel, int degree, REAL gamma, REAL coef0, const int64_t *rowptr,                 \
                         const int32_t *col, const REAL *val, int64_t n, int64_t d, REAL *q);                   \
    void orc_kp_csr_##SUF(int kernel, int degree, REAL gamma, REAL coef0, const int64_t *rowptr,                \
                          const int32_t *col, const REAL *val, int64_t n, int64_t d, const REAL *q,             \
                          REAL QA_cost, REAL cost_inv, REAL add, const REAL *p, REAL *ret, int nthreads);       \
    void orc_kp_csr_factored_##SUF(const int64_t *rowptr, const int32_t *col, const REAL *val, int64_t n, int64_t d, \
                                   const REAL *q, REAL QA_cost, REAL cost_inv, REAL add, const REAL *p, REAL *ret, \
                                   int nthreads);                                                               \
    int64_t orc_cg_##SUF(int kernel, int degree, REAL gamma, REAL coef0, const REAL *X, const int64_t *rowptr,  \
                         const int32_t *col, int64_t n, int64_t d, const REAL *b, int64_t imax, REAL eps,       \
                         const REAL *q, REAL QA_cost, REAL cost_inv, REAL *x_out, double *delta_trace,          \
                         int nthreads);                                                                         \
    int64_t orc_learn_##SUF(int kernel, int degree, REAL gamma, REAL coef0, REAL cost, REAL eps, int64_t imax,  \
                            const REAL *X, const int64_t *rowptr, const int32_t *col, const REAL *y, int64_t n, \
                            int64_t d, REAL *alpha_out, REAL *bias_out, REAL *qa_cost_out, double *delta_trace, \
                            int nthreads);                                                                      \
    void orc_predict_##SUF(int kernel, int degree, REAL gamma, REAL coef0, const REAL *SV, const REAL *alpha,   \
                           int64_t nsv, int64_t d, REAL bias, const REAL *Z, int64_t nz, REAL *out);

ORC_DECLARE(double, f64)
ORC_DECLARE(float, f32)

/* Packed FP22: binary32 truncated to its top 22 bits, round-to-nearest-even. */
uint32_t orc_fp22_encode(float v);
float orc_fp22_decode(uint32_t code);
/* 16 values per 11 little-endian uint32 words; value k of a group at bits [22k, 22k+22). */
void orc_fp22_pack(const float *v, int64_t n, uint32_t *words);
void orc_fp22_unpack(const uint32_t *words, int64_t n, float *v);
int64_t orc_fp22_words(int64_t n);

#ifdef __cplusplus
}
#endif

#endif
