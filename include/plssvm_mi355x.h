/*
 * plssvm_mi355x.h — C ABI of the MI355X-native PLSSVM CG hot path (libplssvm_mi355x.so).
 *
 * The reference exposes this path only as C++ virtuals of plssvm::csvm<T> /
 * plssvm::detail::gpu_csvm<T, device_ptr_t, queue_t>; every entry point below names the
 * reference member it replaces (paths relative to the reference repository root). The C++
 * adapter plssvm::mi355x::csvm<T> (plssvm_sparse_fp22_amd/host/csvm.hpp) maps those virtuals
 * onto these calls; ctypes/cgo/JNI bindings can call them directly.
 *
 * Conventions
 *   - Every function returns PLSSVM_MI_OK (0) or a negative PLSSVM_MI_ERR_* code; no C++
 *     exception crosses the ABI. plssvm_mi_last_error() returns the message of the last
 *     failure on that context (the text the reference would put in its backend_exception).
 *   - Host buffers are caller-owned. Calls taking host buffers are blocking: they return after
 *     results are in host memory (the reference's synchronous hipMemcpy semantics,
 *     src/plssvm/backends/HIP/detail/device_ptr.hip.cpp:40-68).
 *   - "real" buffers hold float when the context was created with real_bytes == 4 and double
 *     when real_bytes == 8 (the reference's template parameter T, include/plssvm/csvm.hpp:36).
 *   - A context owns one GPU (one HIP stream). Several contexts — one per process and GPU —
 *     form a row-block partitioned group through plssvm_mi_comm_init (RCCL over xGMI).
 *   - m = n - 1 ("dept" in the reference): the last data point is eliminated by the LS-SVM
 *     reformulation (src/plssvm/csvm.cpp:230-258).
 */
#ifndef PLSSVM_MI355X_H
#define PLSSVM_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLSSVM_MI_ABI_VERSION 1

#if defined(PLSSVM_MI_BUILDING)
#define PLSSVM_MI_API __attribute__((visibility("default")))
#else
#define PLSSVM_MI_API
#endif

/* return codes */
#define PLSSVM_MI_OK 0
#define PLSSVM_MI_ERR_ARG (-1)         /* invalid argument (plssvm::exception in the reference) */
#define PLSSVM_MI_ERR_HIP (-2)         /* HIP runtime error (plssvm::hip::backend_exception)     */
#define PLSSVM_MI_ERR_RCCL (-3)        /* RCCL error                                              */
#define PLSSVM_MI_ERR_OOM (-4)         /* device allocation failed                                */
#define PLSSVM_MI_ERR_UNSUPPORTED (-5) /* unsupported kernel/format combination                   */
#define PLSSVM_MI_ERR_STATE (-6)       /* call out of order (e.g. generate_q before setup)        */
#define PLSSVM_MI_ERR_NODEV (-7)       /* "HIP backend selected but no HIP devices were found!"   */

/* kernel types: plssvm::kernel_type (include/plssvm/kernel_types.hpp:27-34) */
#define PLSSVM_MI_KERNEL_LINEAR 0
#define PLSSVM_MI_KERNEL_POLYNOMIAL 1
#define PLSSVM_MI_KERNEL_RBF 2

/* value formats of sparse feature data (build-defined; the reference has no sparse path) */
#define PLSSVM_MI_VAL_REAL 0 /* float or double, as the context's real type */
#define PLSSVM_MI_VAL_FP22 1 /* packed FP22 words, 16 values per 11 uint32 (float contexts only) */

/* K·p algorithm selection (plssvm_mi_set_option key PLSSVM_MI_OPT_KP_MODE) */
#define PLSSVM_MI_KP_AUTO 0     /* pairwise for poly/rbf, factored for linear on sparse data      */
#define PLSSVM_MI_KP_PAIRWISE 1 /* implicit pairwise tiles (MFMA on dense data)                   */
#define PLSSVM_MI_KP_FACTORED 2 /* linear kernel only: X (X^T p) + rank-1 terms, HBM-bound         */

#define PLSSVM_MI_OPT_KP_MODE 1
/* Test hook (single GPU): value = rank | (world << 16) makes this context compute only that rank's
 * share of the implicit matrix with no collective; the rank-1 Q~ terms are added by rank 0 only,
 * so the K·p results of all simulated ranks sum to the full K·p. */
#define PLSSVM_MI_OPT_SIM_RANK 2
/* RBF pair evaluation on sparse data: 0 = auto (factored e_i e_j (exp(2 g s) - 1) when g * max |x|^2
 * keeps it in floating-point range), 1 = always direct exp(-g |x_i - x_j|^2) - e_i e_j. */
#define PLSSVM_MI_OPT_RBF_FORM 3
/* K·p algorithm of the pairwise kernels (poly, rbf) on sparse data:
 *   0 = auto: the kernel expansion when it represents the kernel to rounding (poly degree <= 16; rbf
 *       in the factored form with a Taylor degree <= 16 for the data's max |2 g x_if x_jf|), else the
 *       Gram pattern; when the chosen structure's estimated size exceeds the device-memory budget
 *       (85 % of the free memory; environment PLSSVM_MI_MEM_BUDGET = bytes overrides), or its build
 *       runs out of memory, the on-the-fly path 4 or the densified path 3, whichever the setup's
 *       estimate makes faster (the on-the-fly path below a few percent density);
 *   1 = Gram pattern: every overlapping pair (j < i) with s_ij = x_i . x_j stored at setup, the kernel
 *       function re-evaluated on each per K·p (O(sum_f c_f^2) memory and traffic);
 *   2 = kernel expansion: per-feature column moments + the stored remainder of the pairs sharing two or
 *       more features (O(nnz + #multi-feature pairs)); fails with ERR_UNSUPPORTED when not eligible;
 *   3 = densified: X densified on the device, the dense MFMA pairwise tiles (O(m d) memory, every pair
 *       recomputed from the data on each K·p as in the reference); ERR_OOM when m x d does not fit;
 *   4 = on the fly: nothing stored per pair; every K·p re-forms s_ij for the pairs sharing a feature
 *       from the CSR rows and the CSC columns (O(nnz) memory + a d x m / 2048 segment table, O(sum_f
 *       c_f^2) work per K·p, as the reference recomputes every pair). */
#define PLSSVM_MI_OPT_SPARSE_ALGO 4
#define PLSSVM_MI_SPARSE_AUTO 0
#define PLSSVM_MI_SPARSE_PATTERN 1
#define PLSSVM_MI_SPARSE_EXPANSION 2
#define PLSSVM_MI_SPARSE_DENSE 3 /* densified on the device, MFMA pairwise tiles (every pair recomputed per K·p) */
#define PLSSVM_MI_SPARSE_ONTHEFLY 4 /* s_ij re-formed from the CSR / CSC per K·p, nothing stored per pair */

/* CG recurrence of plssvm_mi_solve_cg / plssvm_mi_learn:
 *   0 = the reference's (OpenMP/csvm.cpp:82-170): two dependent inner products per iteration (d.Ad, r.r), i.e. two
 *       exposed collectives in a sharded group;
 *   1 = one-reduction CG (Chronopoulos & Gear): the same iterates in exact arithmetic, the product Q~r instead of Q~d
 *       with s = Q~d carried by a recurrence, r.r and r.Q~r summed together after ONE collective per iteration; the
 *       stop test, trace and every-50th explicit residual keep the reference's meaning (tests/test_gpu_cg1.py compares
 *       its residual curves with the oracle's over 61 iterations);
 *   2 = auto: 1 in a sharded group of several ranks, else 0. */
#define PLSSVM_MI_OPT_CG_VARIANT 5
#define PLSSVM_MI_CG_REFERENCE 0
#define PLSSVM_MI_CG_ONE_REDUCTION 1
#define PLSSVM_MI_CG_AUTO 2

typedef struct plssvm_mi_ctx plssvm_mi_ctx;

/* Number of visible HIP devices (>= 0), or a negative error code. */
PLSSVM_MI_API int plssvm_mi_device_count(void);

/* Replaces hip::csvm<T>::csvm(const parameter<T>&) (src/plssvm/backends/HIP/csvm.hip.cpp:38-81)
 * for the parameters the hot path reads (include/plssvm/csvm.hpp:242-277): real_bytes 4|8 (T),
 * kernel, degree, gamma, coef0, cost (C). device = HIP device ordinal this context drives. */
PLSSVM_MI_API int plssvm_mi_create(int real_bytes, int kernel, int degree, double gamma, double coef0, double cost, int device,
                     plssvm_mi_ctx **out);
PLSSVM_MI_API void plssvm_mi_destroy(plssvm_mi_ctx *ctx);
PLSSVM_MI_API const char *plssvm_mi_last_error(const plssvm_mi_ctx *ctx);
PLSSVM_MI_API int plssvm_mi_set_option(plssvm_mi_ctx *ctx, int key, int64_t value);

/* Test hooks mirroring mock_hip_csvm::set_cost / set_QA_cost (tests/backends/HIP/mock_hip_csvm.hpp:24-51). */
PLSSVM_MI_API int plssvm_mi_set_cost(plssvm_mi_ctx *ctx, double cost);
PLSSVM_MI_API int plssvm_mi_set_qa_cost(plssvm_mi_ctx *ctx, double qa_cost);

/* Multi-GPU row-block group: one context per process/GPU. rank 0 calls
 * plssvm_mi_get_unique_id, the id (PLSSVM_MI_UNIQUE_ID_BYTES bytes) is shared out of band (e.g.
 * torch.distributed), every rank calls plssvm_mi_comm_init. Replaces the feature-split device
 * list + host-staged device_reduction (src/plssvm/backends/gpu_csvm.cpp:136-139,366-386). */
#define PLSSVM_MI_UNIQUE_ID_BYTES 128
PLSSVM_MI_API int plssvm_mi_get_unique_id(void *id_out);
PLSSVM_MI_API int plssvm_mi_comm_init(plssvm_mi_ctx *ctx, int rank, int world_size, const void *unique_id);

/* Host-staged group exchange: the reference's own device_reduction semantics
 * (src/plssvm/backends/gpu_csvm.cpp:366-386: synchronise, copy the partial vector to the host,
 * combine there, copy the result back) with the combine step supplied by the caller, e.g. a
 * torch.distributed / MPI / gloo collective. Every rank of the group calls it with the same
 * world_size instead of plssvm_mi_comm_init; the engine then runs exactly the multi-rank work split
 * of the RCCL path (partition -> this rank's share -> exchange -> replicated CG) but moves each
 * exchange through `fn` on the host. Use: groups without RCCL, and several ranks sharing one GPU
 * (RCCL refuses two ranks on one device) — the multi-rank path's test transport on a 1-GPU box.
 *   fn(buf, count, real_bytes, op, user) must return 0 on success and be called collectively:
 *   op == PLSSVM_MI_XCHG_ALLREDUCE: buf[count] (real_bytes-wide reals) := sum over ranks, the same
 *                                   bits on every rank;
 *   op == PLSSVM_MI_XCHG_ALLGATHER: buf[world_size * count]: rank r's chunk [r*count, (r+1)*count)
 *                                   is valid on rank r; fill every other rank's chunk. */
#define PLSSVM_MI_XCHG_ALLREDUCE 0
#define PLSSVM_MI_XCHG_ALLGATHER 1
typedef int (*plssvm_mi_exchange_fn)(void *buf, int64_t count, int real_bytes, int op, void *user);
PLSSVM_MI_API int plssvm_mi_comm_init_host(plssvm_mi_ctx *ctx, int rank, int world_size, plssvm_mi_exchange_fn fn,
                                           void *user);

/* Group failure protocol of a one-process multi-GPU group (one host thread per context, e.g. the csvm<T> adapter
 * over every visible GPU, include/plssvm_mi355x_group.hpp): when one rank's call fails, the caller aborts every
 * context of the group from its own thread — an RCCL communicator is released with ncclCommAbort, so a rank waiting
 * in a collective returns — and every call of an aborted context (also the one in progress) fails with
 * PLSSVM_MI_ERR_RCCL. The reference ends its device threads the same way: a backend_exception on any device ends the
 * OpenMP region (src/plssvm/backends/gpu_csvm.cpp:366-386). May be called from any thread, concurrently with a call
 * on the same context; the context can then only be destroyed. */
PLSSVM_MI_API int plssvm_mi_comm_abort(plssvm_mi_ctx *ctx);

/* Host-only (no GPU needed): the work split of the implicit matrix for m = n - 1 rows.
 * out4 = { first super-block, end super-block, total tiles, tiles owned by `rank` } where a tile
 * is 128x128 of the lower triangle and a super-block 8x8 tiles (linear index I(I+1)/2 + J). */
PLSSVM_MI_API int plssvm_mi_partition(int64_t m, int rank, int world_size, int64_t *out4);

/* gpu_csvm::setup_data_on_device (src/plssvm/backends/gpu_csvm.cpp:130-157) for dense data:
 * X is row-major [n][d] host memory of the context's real type (all n points, the last one
 * included, exactly the reference's data_ptr_). */
PLSSVM_MI_API int plssvm_mi_setup_dense(plssvm_mi_ctx *ctx, const void *X, int64_t n, int64_t d);

/* Sparse setup (build-defined format): CSR with int64 rowptr[n+1],
 * int32 col[nnz] ascending per row, values in val_fmt (PLSSVM_MI_VAL_REAL: real[nnz];
 * PLSSVM_MI_VAL_FP22: uint32 packed words, orc/fp22 layout). Semantics == dense setup on the
 * densified matrix (the reference parser densifies, src/plssvm/parameter.cpp:66-87). */
PLSSVM_MI_API int plssvm_mi_setup_csr(plssvm_mi_ctx *ctx, const int64_t *rowptr, const int32_t *col, const void *val,
                        int val_fmt, int64_t n, int64_t d);

/* Sparse setup from COO triplets (build-defined interchange format, e.g. BASELINE configs[4]):
 * int64 row[nnz], int32 col[nnz] in any order, values in val_fmt (FP22: packed in triplet order).
 * Converted on the host to CSR (rows, then columns ascending; a duplicate (row, col) is an error) and
 * then exactly plssvm_mi_setup_csr. */
PLSSVM_MI_API int plssvm_mi_setup_coo(plssvm_mi_ctx *ctx, const int64_t *row, const int32_t *col, const void *val,
                                      int val_fmt, int64_t nnz, int64_t n, int64_t d);

/* gpu_csvm::generate_q (src/plssvm/backends/gpu_csvm.cpp:160-183) + the QA_cost line of
 * csvm::learn (src/plssvm/csvm.cpp:243): q_out[m] = k(x_i, x_last); *qa_cost_out =
 * k(x_last, x_last) + 1/C. Also stores q and QA_cost in the context for plssvm_mi_kp. */
PLSSVM_MI_API int plssvm_mi_generate_q(plssvm_mi_ctx *ctx, void *q_out, double *qa_cost_out);

/* gpu_csvm::run_device_kernel + device_reduction (src/plssvm/backends/gpu_csvm.cpp:353-386):
 * ret[m] += add * Q~ p, Q~_ij = k(x_i,x_j) + QA_cost - q_i - q_j + [i==j]/C. q may be NULL to use
 * the context's q (from generate_q); otherwise q[m] is uploaded first. All host buffers. */
PLSSVM_MI_API int plssvm_mi_kp(plssvm_mi_ctx *ctx, const void *q, const void *p, void *ret, double add);

/* Test hook (the protected-for-mock parts of run_device_kernel, tests/backends/HIP/mock_hip_csvm.hpp:
 * 24-51): out[m] = one part of Q~p for host p[m], after the group exchange:
 *   PLSSVM_MI_PART_KERNEL  : sum_{j<m} k(x_i, x_j) p_j  (Q~p without the QA_cost - q_i - q_j and 1/C
 *                            terms, which are applied analytically in O(m));
 *   PLSSVM_MI_PART_OVERLAP : sparse poly/rbf only — sum over j != i sharing a feature with i of
 *                            (k_ij - kappa_ij) p_j, kappa_ij the value non-overlapping pairs take
 *                            (e_i e_j for rbf, coef0^degree for poly): exactly the per-pair work of the
 *                            sparse K·p kernels, without the separable and diagonal terms;
 *   PLSSVM_MI_PART_REMAINDER: the sparse kernel expansion only — its stored remainder stream alone,
 *                            sum over j != i sharing >= 2 features of a_i a_j H_ij p_j (H_ij = phi(s_ij) -
 *                            sum_f phi(x_if x_jf); a = e for rbf, 1 for poly) in the stored layout (bfloat16 H
 *                            and windows where the setup chose them), without the column-moment terms. */
#define PLSSVM_MI_PART_KERNEL 0
#define PLSSVM_MI_PART_OVERLAP 1
#define PLSSVM_MI_PART_REMAINDER 2
PLSSVM_MI_API int plssvm_mi_kp_part(plssvm_mi_ctx *ctx, const void *p, void *out, int part);

/* gpu_csvm::solver_CG (src/plssvm/backends/gpu_csvm.cpp:186-324) with the OpenMP backend's
 * normative semantics (src/plssvm/backends/OpenMP/csvm.cpp:82-170; including the every-50th
 * explicit residual r = b - Q~x that the reference HIP path gets wrong on one GPU). b[m], q[m]
 * (NULL = context q); x_out[m]; delta_trace (nullable, imax+1 doubles: delta0 then delta after
 * each iteration); *iters = CG iterations run. Vectors stay device-resident throughout. */
PLSSVM_MI_API int plssvm_mi_solve_cg(plssvm_mi_ctx *ctx, const void *b, const void *q, int64_t imax, double eps, void *x_out,
                       double *delta_trace, int64_t *iters);

/* Progress of plssvm_mi_solve_cg / plssvm_mi_learn — the per-iteration output of the reference's
 * solver_CG when print_info is set (src/plssvm/backends/OpenMP/csvm.cpp:115-117,161-166;
 * gpu_csvm.cpp:233-321). The CG runs on the device and the host polls it once per batch of
 * iterations (4, 8, 16, ..., then blocks of 50); after each batch fn(first, count, deltas, target,
 * batch_ms, user) is called with the batch's iterations [first, first + count) (0-based),
 * deltas[0..count] = r^T r before iteration `first`, ..., after the batch's last iteration,
 * target = eps^2 delta0 (the stop bound) and the batch's wall time in ms. fn == NULL: no calls.
 * The callback must not call back into the context. */
typedef void (*plssvm_mi_progress_fn)(int64_t first, int64_t count, const double *deltas, double target,
                                      double batch_ms, void *user);
PLSSVM_MI_API int plssvm_mi_set_progress(plssvm_mi_ctx *ctx, plssvm_mi_progress_fn fn, void *user);

/* Stepwise CG on the same device state (used by bench.py to time single iterations):
 * begin = x0 = 1, r = b - Q~x, d = r; step runs n iterations (ignores convergence when
 * force != 0); result copies x and the trace out. */
PLSSVM_MI_API int plssvm_mi_cg_begin(plssvm_mi_ctx *ctx, const void *b, const void *q, double eps, double *delta0_out);
PLSSVM_MI_API int plssvm_mi_cg_step(plssvm_mi_ctx *ctx, int64_t n, int force, int64_t *iters_done, int *converged);
PLSSVM_MI_API int plssvm_mi_cg_result(plssvm_mi_ctx *ctx, void *x_out, double *delta_trace, int64_t trace_len, int64_t *iters);

/* csvm<T>::learn (src/plssvm/csvm.cpp:207-267) on the context's data: y[n] labels (+-1),
 * imax < 0 means num_features (the reference's imax, csvm.cpp:256). alpha_out[n] (alpha[m] =
 * -sum), *bias_out (rho = -bias), delta_trace (nullable, imax+1). */
PLSSVM_MI_API int plssvm_mi_learn(plssvm_mi_ctx *ctx, const void *y, int64_t imax, double eps, void *alpha_out, double *bias_out,
                    double *delta_trace, int64_t *iters);

/* gpu_csvm::update_w (src/plssvm/backends/gpu_csvm.cpp:327-350; OpenMP csvm.cpp:174-190):
 * w_out[d] = sum_i alpha_i x_i over all n points of the context's data (alpha[n], e.g. from
 * plssvm_mi_learn, alpha[m] included). Linear kernel model vector. */
PLSSVM_MI_API int plssvm_mi_update_w(plssvm_mi_ctx *ctx, const void *alpha, void *w_out);

/* gpu_csvm::predict (src/plssvm/backends/gpu_csvm.cpp:52-120; OpenMP csvm.cpp:193-240):
 * out[p] = bias + sum_i alpha_i k(x_i, z_p) for np points with d features (linear: w . z_p + bias),
 * the context's data being the model's support vectors. Dense points: Z row-major [np][d] of the
 * real type. Sparse points (_csr): int64 rowptr[np+1], int32 col, values in val_fmt. np == 0 is a
 * no-op; a feature-count mismatch fails with the reference's message. bias = -rho. */
PLSSVM_MI_API int plssvm_mi_predict_dense(plssvm_mi_ctx *ctx, const void *alpha, double bias, const void *Z, int64_t np,
                                          int64_t d, void *out);
PLSSVM_MI_API int plssvm_mi_predict_csr(plssvm_mi_ctx *ctx, const void *alpha, double bias, const int64_t *rowptr,
                                        const int32_t *col, const void *val, int val_fmt, int64_t np, int64_t d,
                                        void *out);

/* Timing hook (bench.py): runs `reps` K·p launches (+ reduction/collective) on resident device
 * buffers (p = a fixed device vector) and reports the average device time per K·p and per
 * dominant-kernel launch, measured with hipEvents on the context's stream. */
PLSSVM_MI_API int plssvm_mi_time_kp(plssvm_mi_ctx *ctx, int reps, double *ms_per_kp, double *ms_dominant_kernel);

/* Introspection for roofline accounting: number of pairwise tiles / work units per K·p on this
 * rank, tile edge, padded sizes, bytes of device memory held. */
typedef struct {
    int64_t n, d, m, n_pad, d_pad, nnz;
    int64_t tiles_total, tiles_local, tile_rows, tile_cols;
    int64_t device_bytes;
    int64_t pairs; /* sparse pairwise kernels: stored overlapping pairs (j < i) of this rank */
    int kp_mode, rank, world_size, real_bytes, kernel, is_sparse, val_fmt;
    int rbf_factored;   /* sparse rbf: 1 = factored pair form in use (PLSSVM_MI_OPT_RBF_FORM) */
    int64_t pair_slots; /* sparse pairwise kernels: stored pair slots incl. padding (K·p stream) */
    int64_t spmv_bytes; /* sparse factored linear: HBM bytes both SpMV passes move per K·p (padded SELL
                           stream, slot maps, panel partials) */
    int rbf_small_args; /* sparse factored rbf: 1 = every 2 g |s_ij| is below the short Taylor form's bound */
    int sparse_algo;    /* sparse poly/rbf: PLSSVM_MI_SPARSE_PATTERN | _EXPANSION | _DENSE (0 otherwise) */
    int exp_terms;      /* kernel expansion: polynomial degree K of the per-feature pair function */
    int exp_waves;      /* kernel expansion: waves of the remainder stream */
    int64_t exp_chunks; /* kernel expansion: 4-slot chunks of the remainder stream (this rank's rows); 0 = run layout */
    int exp_hbytes;     /* kernel expansion: bytes of a stored remainder value (2 = bfloat16 under the precision
                           bound of expand.hip "H storage", else sizeof(real)) */
    int exp_layout;     /* kernel expansion: remainder stream layout — 1 = 4-slot chunks with a stored row index per
                           chunk, 2 = 4-slot chunks whose rows are numbered by row-start flags (no row index),
                           4 = row-start flags per slot pair (cells padded to 2 slots); 0 = no expansion
                           (3 was round 2's run layout, removed) */
    int exp_dot2;       /* kernel expansion, bfloat16 H: 1 = the remainder's chunk products run on the v_dot2_f32_bf16
                           kernel (built with EXP_DOT2 and selected: PLSSVM_MI_EXP_DOT2 != 0), 0 = the FMA chain */
    int centered;       /* kernel expansion: 1 = the finalize forms Q~'s rank-1 terms in the centered form
                           (engine.hpp ctr_*; PLSSVM_MI_CTR=0 or a caller's own q vector: 0) */
    int exp_lt;         /* kernel expansion: 1 = the remainder's rows came from the lower-triangle join + transpose
                           (one rank holding every row; PLSSVM_MI_EXP_LT=0: the full join) */
} plssvm_mi_info;
PLSSVM_MI_API int plssvm_mi_get_info(const plssvm_mi_ctx *ctx, plssvm_mi_info *info);

#ifdef __cplusplus
}
#endif

#endif /* PLSSVM_MI355X_H */
