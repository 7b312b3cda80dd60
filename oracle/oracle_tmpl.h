/*
 * plssvm oracle — TEST INFRASTRUCTURE ONLY (see oracle.h). Included twice by oracle.c with
 * REAL/SUF defined (double/f64, float/f32). Every function cites the reference code it restates.
 */

#define ORC_CAT_(a, b) a##_##b
#define ORC_CAT(a, b) ORC_CAT_(a, b)
#define FN(name) ORC_CAT(name, SUF)

/* plssvm::operators::transposed * vector — sequential std::fma chain in index order
 * (include/plssvm/detail/operators.hpp:113-122). */
static REAL FN(orc_dot)(const REAL *a, const REAL *b, int64_t n) {
    REAL val = 0;
    for (int64_t i = 0; i < n; ++i) val = FMA(a[i], b[i], val);
    return val;
}

/* plssvm::operators::squared_euclidean_dist (operators.hpp:157-167). */
static REAL FN(orc_sqdist)(const REAL *a, const REAL *b, int64_t n) {
    REAL val = 0;
    for (int64_t i = 0; i < n; ++i) {
        const REAL diff = a[i] - b[i];
        val = FMA(diff, diff, val);
    }
    return val;
}

/* plssvm::operators::sum (operators.hpp:140-147); sequential here (reference: omp simd). */
static REAL FN(orc_sum)(const REAL *a, int64_t n) {
    REAL val = 0;
    for (int64_t i = 0; i < n; ++i) val += a[i];
    return val;
}

/* Sparse twins of the two chains above: CSR rows, columns ascending. Skipping features that are
 * zero in both rows leaves the fma chain bit-identical to the dense one on the densified rows
 * (fma(0, x, acc) == acc), which is how the reference treats LIBSVM sparse input
 * (src/plssvm/parameter.cpp:66-87 densifies, missing -> 0). */
static REAL FN(orc_dot_csr)(const int32_t *ca, const REAL *va, int64_t na, const int32_t *cb, const REAL *vb,
                            int64_t nb) {
    REAL val = 0;
    int64_t x = 0, y = 0;
    while (x < na && y < nb) {
        if (ca[x] == cb[y]) {
            val = FMA(va[x], vb[y], val);
            ++x;
            ++y;
        } else if (ca[x] < cb[y]) {
            ++x;
        } else {
            ++y;
        }
    }
    return val;
}

static REAL FN(orc_sqdist_csr)(const int32_t *ca, const REAL *va, int64_t na, const int32_t *cb, const REAL *vb,
                               int64_t nb) {
    REAL val = 0;
    int64_t x = 0, y = 0;
    while (x < na || y < nb) {
        REAL diff;
        if (y >= nb || (x < na && ca[x] < cb[y])) {
            diff = va[x++];
        } else if (x >= na || cb[y] < ca[x]) {
            diff = -vb[y++];
        } else {
            diff = va[x++] - vb[y++];
        }
        val = FMA(diff, diff, val);
    }
    return val;
}

/* plssvm::kernel_function<kernel> (include/plssvm/kernel_types.hpp:63-85):
 *   linear: x^T y;  poly: pow(fma(gamma, x^T y, coef0), (real)degree);  rbf: exp(-gamma * |x-y|^2). */
static REAL FN(orc_apply)(int kernel, int degree, REAL gamma, REAL coef0, REAL dot_or_dist) {
    switch (kernel) {
        case 0: return dot_or_dist;
        case 1: return POW(FMA(gamma, dot_or_dist, coef0), (REAL) degree);
        default: return EXP(-gamma * dot_or_dist);
    }
}

REAL FN(orc_kernel)(int kernel, int degree, REAL gamma, REAL coef0, const REAL *a, const REAL *b, int64_t d) {
    const REAL t = (kernel == 2) ? FN(orc_sqdist)(a, b, d) : FN(orc_dot)(a, b, d);
    return FN(orc_apply)(kernel, degree, gamma, coef0, t);
}

/* one view over dense row-major or CSR data */
typedef struct {
    const REAL *X;          /* dense [n][d] row-major, or CSR values when rowptr != NULL */
    const int64_t *rowptr;  /* CSR row pointer [n+1] or NULL */
    const int32_t *col;
    int64_t d;
    int kernel, degree;
    REAL gamma, coef0;
} FN(orc_view);

static REAL FN(orc_kv)(const FN(orc_view) *v, int64_t i, int64_t j) {
    REAL t;
    if (v->rowptr) {
        const int64_t a0 = v->rowptr[i], a1 = v->rowptr[i + 1], b0 = v->rowptr[j], b1 = v->rowptr[j + 1];
        t = (v->kernel == 2) ? FN(orc_sqdist_csr)(v->col + a0, v->X + a0, a1 - a0, v->col + b0, v->X + b0, b1 - b0)
                             : FN(orc_dot_csr)(v->col + a0, v->X + a0, a1 - a0, v->col + b0, v->X + b0, b1 - b0);
    } else {
        t = (v->kernel == 2) ? FN(orc_sqdist)(v->X + i * v->d, v->X + j * v->d, v->d)
                             : FN(orc_dot)(v->X + i * v->d, v->X + j * v->d, v->d);
    }
    return FN(orc_apply)(v->kernel, v->degree, v->gamma, v->coef0, t);
}

/* openmp::device_kernel_q_{linear,poly,radial} (src/plssvm/backends/OpenMP/q_kernel.cpp:18-52):
 * q[i] = k(x_i, x_last), i < n-1. */
static void FN(orc_q_view)(const FN(orc_view) *v, int64_t n, REAL *q) {
#pragma omp parallel for
    for (int64_t i = 0; i < n - 1; ++i) q[i] = FN(orc_kv)(v, i, n - 1);
}

/* openmp::detail::device_kernel<k> (src/plssvm/backends/OpenMP/svm_kernel.cpp:21-47):
 * 64x64 blocks over the lower triangle (i >= j), collapse(2) schedule(dynamic), temp computed
 * once per pair and added to both rows (omp atomic on the mirrored row). dept = m = n-1. */
#define ORC_BLOCK 64 /* plssvm::OPENMP_BLOCK_SIZE (include/plssvm/constants.hpp:38) */
static void FN(orc_kp_view)(const FN(orc_view) *v, int64_t dept, const REAL *q, REAL QA_cost, REAL cost,
                            REAL add, const REAL *d, REAL *ret, int nthreads) {
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for collapse(2) schedule(dynamic) num_threads(nthreads)
    for (int64_t i = 0; i < dept; i += ORC_BLOCK) {
        for (int64_t j = 0; j < dept; j += ORC_BLOCK) {
            for (int64_t ii = 0; ii < ORC_BLOCK && ii + i < dept; ++ii) {
                REAL ret_iii = 0;
                for (int64_t jj = 0; jj < ORC_BLOCK && jj + j < dept; ++jj) {
                    if (ii + i >= jj + j) {
                        const REAL temp = (FN(orc_kv)(v, ii + i, jj + j) + QA_cost - q[ii + i] - q[jj + j]) * add;
                        if (ii + i == jj + j) {
                            ret_iii += (temp + cost * add) * d[ii + i];
                        } else {
                            ret_iii += temp * d[jj + j];
#pragma omp atomic
                            ret[jj + j] += temp * d[ii + i];
                        }
                    }
                }
#pragma omp atomic
                ret[ii + i] += ret_iii;
            }
        }
    }
}

void FN(orc_q)(int kernel, int degree, REAL gamma, REAL coef0, const REAL *X, int64_t n, int64_t d, REAL *q) {
    FN(orc_view) v = { X, NULL, NULL, d, kernel, degree, gamma, coef0 };
    FN(orc_q_view)(&v, n, q);
}

void FN(orc_q_csr)(int kernel, int degree, REAL gamma, REAL coef0, const int64_t *rowptr, const int32_t *col,
                   const REAL *val, int64_t n, int64_t d, REAL *q) {
    FN(orc_view) v = { val, rowptr, col, d, kernel, degree, gamma, coef0 };
    FN(orc_q_view)(&v, n, q);
}

void FN(orc_kp)(int kernel, int degree, REAL gamma, REAL coef0, const REAL *X, int64_t n, int64_t d, const REAL *q,
                REAL QA_cost, REAL cost_inv, REAL add, const REAL *p, REAL *ret, int nthreads) {
    FN(orc_view) v = { X, NULL, NULL, d, kernel, degree, gamma, coef0 };
    FN(orc_kp_view)(&v, n - 1, q, QA_cost, cost_inv, add, p, ret, nthreads);
}

void FN(orc_kp_csr)(int kernel, int degree, REAL gamma, REAL coef0, const int64_t *rowptr, const int32_t *col,
                    const REAL *val, int64_t n, int64_t d, const REAL *q, REAL QA_cost, REAL cost_inv, REAL add,
                    const REAL *p, REAL *ret, int nthreads) {
    FN(orc_view) v = { val, rowptr, col, d, kernel, degree, gamma, coef0 };
    FN(orc_kp_view)(&v, n - 1, q, QA_cost, cost_inv, add, p, ret, nthreads);
}

/* CPU baseline only ("cpu_ref CSR K·p at full size, O(nnz) factored form"):
 * the linear K·p in the factored form SURVEY §8(d) verified against the reference kernel (8.7e-16),
 *   ret += add * ( X_m (X_m^T p) + (QA_cost - q_i) sum(p) - q^T p + p_i / C ),
 * on CSR rows 0..m-1, OpenMP: w = X_m^T p with per-thread column accumulators reduced in thread order,
 * then one row-parallel pass. Not a restatement of a reference function (the reference has no sparse
 * path); it is the honest O(nnz) CPU cost of the same product, timed beside the GPU. */
void FN(orc_kp_csr_factored)(const int64_t *rowptr, const int32_t *col, const REAL *val, int64_t n, int64_t d,
                             const REAL *q, REAL QA_cost, REAL cost_inv, REAL add, const REAL *p, REAL *ret,
                             int nthreads) {
    const int64_t m = n - 1;
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    REAL *wt = (REAL *) calloc((size_t) nthreads * (size_t) d, sizeof(REAL));
    REAL *w = (REAL *) calloc((size_t) d, sizeof(REAL));
    REAL sp = 0, sqp = 0;
#pragma omp parallel num_threads(nthreads)
    {
        REAL *mine = wt + (size_t) omp_get_thread_num() * (size_t) d;
#pragma omp for schedule(static)
        for (int64_t i = 0; i < m; ++i)
            for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) mine[col[k]] += val[k] * p[i];
#pragma omp for schedule(static)
        for (int64_t f = 0; f < d; ++f) {
            REAL a = 0;
            for (int t = 0; t < nthreads; ++t) a += wt[(size_t) t * (size_t) d + f];
            w[f] = a;
        }
#pragma omp for reduction(+ : sp, sqp) schedule(static)
        for (int64_t i = 0; i < m; ++i) {
            sp += p[i];
            sqp += q[i] * p[i];
        }
#pragma omp for schedule(static)
        for (int64_t i = 0; i < m; ++i) {
            REAL raw = 0;
            for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) raw += val[k] * w[col[k]];
            ret[i] += add * (raw + (QA_cost - q[i]) * sp - sqp + cost_inv * p[i]);
        }
    }
    free(wt);
    free(w);
}

/* openmp::csvm::solver_CG (src/plssvm/backends/OpenMP/csvm.cpp:82-170), the normative CG:
 * x0 = 1; r = b - Q~x; delta = r.r; loop run < imax: Ad = Q~d; a = delta/(d.Ad); x += a*d;
 * r = (run % 50 == 49) ? b - Q~x : r - a*Ad; stop if delta <= eps^2 delta0; d = beta*d + r.
 * delta_trace[0] = delta0, delta_trace[k] = delta after iteration k. Returns iterations run. */
static int64_t FN(orc_cg_view)(const FN(orc_view) *v, int64_t dept, const REAL *b, int64_t imax, REAL eps,
                               const REAL *q, REAL QA_cost, REAL cost_inv, REAL *x, double *delta_trace,
                               int nthreads) {
    REAL *r = (REAL *) malloc(sizeof(REAL) * (size_t) (dept + 1));
    REAL *Ad = (REAL *) malloc(sizeof(REAL) * (size_t) (dept + 1));
    REAL *dv = (REAL *) malloc(sizeof(REAL) * (size_t) (dept + 1));
    for (int64_t i = 0; i < dept; ++i) {
        x[i] = 1;
        r[i] = b[i];
    }
    FN(orc_kp_view)(v, dept, q, QA_cost, cost_inv, (REAL) -1, x, r, nthreads);
    REAL delta = FN(orc_dot)(r, r, dept);
    const REAL delta0 = delta;
    if (delta_trace) delta_trace[0] = (double) delta;
    for (int64_t i = 0; i < dept; ++i) dv[i] = r[i];

    int64_t run = 0;
    for (; run < imax; ++run) {
        for (int64_t i = 0; i < dept; ++i) Ad[i] = 0;
        FN(orc_kp_view)(v, dept, q, QA_cost, cost_inv, (REAL) 1, dv, Ad, nthreads);
        const REAL alpha_cd = delta / FN(orc_dot)(dv, Ad, dept);
        for (int64_t i = 0; i < dept; ++i) {
            const REAL t = alpha_cd * dv[i];
            x[i] = x[i] + t;
        }
        if (run % 50 == 49) {
            for (int64_t i = 0; i < dept; ++i) r[i] = b[i];
            FN(orc_kp_view)(v, dept, q, QA_cost, cost_inv, (REAL) -1, x, r, nthreads);
        } else {
            for (int64_t i = 0; i < dept; ++i) {
                const REAL t = alpha_cd * Ad[i];
                r[i] = r[i] - t;
            }
        }
        const REAL delta_old = delta;
        delta = FN(orc_dot)(r, r, dept);
        if (delta_trace) delta_trace[run + 1] = (double) delta;
        if (delta <= eps * eps * delta0) {
            ++run;
            break;
        }
        const REAL beta = delta / delta_old;
        for (int64_t i = 0; i < dept; ++i) {
            const REAL t = beta * dv[i];
            dv[i] = t + r[i];
        }
    }
    free(r);
    free(Ad);
    free(dv);
    return run;
}

int64_t FN(orc_cg)(int kernel, int degree, REAL gamma, REAL coef0, const REAL *X, const int64_t *rowptr,
                   const int32_t *col, int64_t n, int64_t d, const REAL *b, int64_t imax, REAL eps, const REAL *q,
                   REAL QA_cost, REAL cost_inv, REAL *x_out, double *delta_trace, int nthreads) {
    FN(orc_view) v = { X, rowptr, col, d, kernel, degree, gamma, coef0 };
    return FN(orc_cg_view)(&v, n - 1, b, imax, eps, q, QA_cost, cost_inv, x_out, delta_trace, nthreads);
}

/* csvm<T>::learn (src/plssvm/csvm.cpp:207-267): b = y[0..m) - y[m]; q; QA_cost = k(x_m,x_m) + 1/C;
 * alpha = solver_CG(b, imax = num_features, eps, q)  (csvm.cpp:256 — imax < 0 here means "d");
 * bias = y[m] + QA_cost*sum(alpha) - q.alpha; alpha[m] = -sum(alpha). rho = -bias (csvm.cpp:123). */
int64_t FN(orc_learn)(int kernel, int degree, REAL gamma, REAL coef0, REAL cost, REAL eps, int64_t imax,
                      const REAL *X, const int64_t *rowptr, const int32_t *col, const REAL *y, int64_t n, int64_t d,
                      REAL *alpha_out, REAL *bias_out, REAL *qa_cost_out, double *delta_trace, int nthreads) {
    FN(orc_view) v = { X, rowptr, col, d, kernel, degree, gamma, coef0 };
    const int64_t m = n - 1;
    REAL *q = (REAL *) malloc(sizeof(REAL) * (size_t) (m + 1));
    REAL *b = (REAL *) malloc(sizeof(REAL) * (size_t) (m + 1));
    FN(orc_q_view)(&v, n, q);
    for (int64_t i = 0; i < m; ++i) b[i] = y[i] - y[m];
    const REAL QA_cost = FN(orc_kv)(&v, m, m) + (REAL) 1 / cost;
    if (imax < 0) imax = d;
    const int64_t iters = FN(orc_cg_view)(&v, m, b, imax, eps, q, QA_cost, (REAL) 1 / cost, alpha_out, delta_trace,
                                          nthreads);
    const REAL s = FN(orc_sum)(alpha_out, m);
    *bias_out = y[m] + QA_cost * s - FN(orc_dot)(q, alpha_out, m);
    alpha_out[m] = -s;
    if (qa_cost_out) *qa_cost_out = QA_cost;
    free(q);
    free(b);
    return iters;
}

/* openmp::csvm::predict (src/plssvm/backends/OpenMP/csvm.cpp:193-240): out = bias + sum_i alpha_i k(sv_i, z);
 * linear uses w = sum_i alpha_i sv_i (update_w, :174-190). Only used to pin kernel_function against
 * the reference's predict fixtures. */
void FN(orc_predict)(int kernel, int degree, REAL gamma, REAL coef0, const REAL *SV, const REAL *alpha, int64_t nsv,
                     int64_t d, REAL bias, const REAL *Z, int64_t nz, REAL *out) {
    if (kernel == 0) {
        REAL *w = (REAL *) calloc((size_t) d, sizeof(REAL));
        for (int64_t f = 0; f < d; ++f) {
            REAL t = 0;
            for (int64_t i = 0; i < nsv; ++i) t += alpha[i] * SV[i * d + f];
            w[f] = t;
        }
        for (int64_t p = 0; p < nz; ++p) out[p] = bias + FN(orc_dot)(w, Z + p * d, d);
        free(w);
        return;
    }
#pragma omp parallel for
    for (int64_t p = 0; p < nz; ++p) {
        REAL t = 0;
        for (int64_t i = 0; i < nsv; ++i) t += alpha[i] * FN(orc_kernel)(kernel, degree, gamma, coef0, SV + i * d, Z + p * d, d);
        out[p] = bias + t;
    }
}

#undef FN
