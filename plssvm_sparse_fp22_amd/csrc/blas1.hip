// Device-resident CG vector kernels and deterministic reductions.
//
// Replaces the host BLAS-1 of gpu_csvm::solver_CG (src/plssvm/backends/gpu_csvm.cpp:262-303) and
// the per-iteration H2D/D2H copies around it: x, r, d, Ad and every CG scalar stay on the GPU.
// Operation order follows openmp::csvm::solver_CG (src/plssvm/backends/OpenMP/csvm.cpp:82-170):
// x = x + (alpha*d), r = r - (alpha*Ad), d = (beta*d) + r, each product rounded before the add
// (no contraction). Dots are two-stage tree reductions with a fixed grid: bitwise reproducible.
#include "cg_common.hpp"

#pragma clang fp contract(off)

namespace plssvm_mi {

namespace {

using namespace cgk;

// partials[blockIdx] = sum a*b (b null: sum a); second pair (c, e) into partials[RED_BLOCKS + blockIdx]
template <typename T>
__global__ __launch_bounds__(256) void dot2_kernel(const T *__restrict__ a, const T *__restrict__ b,
                                                   const T *__restrict__ c, const T *__restrict__ e, int64_t n,
                                                   T *__restrict__ partials, const cg_scalars<T> *status) {
    if (status != nullptr && status->converged) return;
    __shared__ T red[8];
    T s1 = 0, s2 = 0;
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const T av = a[i];
        s1 += b ? av * b[i] : av;
        if (c) s2 += c[i] * (e ? e[i] : T(1));
    }
    const T r1 = block_sum(s1, red);
    __syncthreads();
    const T r2 = c ? block_sum(s2, red) : T(0);
    if (threadIdx.x == 0) {
        partials[blockIdx.x] = r1;
        partials[RED_BLOCKS + blockIdx.x] = r2;
    }
}

// G > 1: a sharded group's gathered partials, G sets of 2 x RED_BLOCKS (rank-major); every thread adds its
// partials' G values in rank order (the same order, hence the same bits, on every rank)
template <typename T>
__global__ __launch_bounds__(256) void dot_final_kernel(const T *__restrict__ partials, int G, cg_scalars<T> *sc,
                                                        int op, int64_t run, double *trace, int64_t trace_cap,
                                                        T *plain_out) {
    if (op != FIN_PLAIN && sc->converged) return;
    __shared__ T red[8];
    T r1, r2;
    partials_final(partials, G, red, r1, r2);
    if (threadIdx.x != 0) return;
    switch (op) {
        case FIN_SP_SQP:
            sc->sp = r1;
            sc->sqp = r2;
            break;
        case FIN_DELTA0:  // delta = r.r after r = b - Q~x
            sc->delta = r1;
            sc->delta0 = r1;
            sc->eps2delta0 = sc->force ? T(-1) : sc->eps2delta0 * r1;  // host preset eps^2
            if (trace && trace_cap > 0) trace[0] = (double) r1;
            break;
        case FIN_ALPHA:  // alpha = delta / (d . Ad)
            sc->dAd = r1;
            sc->alpha = sc->delta / r1;
            break;
        case FIN_DELTA: {  // delta_new = r.r; convergence test; beta
            const T delta_old = sc->delta;
            sc->delta = r1;
            sc->iters = run + 1;
            if (trace && run + 1 < trace_cap) trace[run + 1] = (double) r1;
            if (r1 <= sc->eps2delta0) {
                sc->converged = 1;
            } else {
                sc->beta = r1 / delta_old;
            }
            break;
        }
        default:
            if (plain_out) {
                plain_out[0] = r1;
                plain_out[1] = r2;
            }
            break;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void cg_init_kernel(const T *__restrict__ b, int64_t m, T *__restrict__ x,
                                                      T *__restrict__ r) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    x[i] = T(1);
    r[i] = b[i];
}

template <typename T>
__global__ __launch_bounds__(256) void copy_kernel(const T *__restrict__ src, int64_t n, T *__restrict__ dst,
                                                   const cg_scalars<T> *status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

template <typename T>
__global__ __launch_bounds__(256) void cg_update_kernel(T *__restrict__ x, T *__restrict__ r, const T *__restrict__ d,
                                                        const T *__restrict__ Ad, const T *__restrict__ b, int reset,
                                                        int64_t m, const cg_scalars<T> *sc) {
    if (sc->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const T alpha = sc->alpha;
    const T t = alpha * d[i];
    x[i] = x[i] + t;
    if (reset) {
        r[i] = b[i];
    } else {
        const T u = alpha * Ad[i];
        r[i] = r[i] - u;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void cg_direction_kernel(T *__restrict__ d, const T *__restrict__ r, int64_t m,
                                                           const cg_scalars<T> *sc) {
    if (sc->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const T t = sc->beta * d[i];
    d[i] = t + r[i];
}

// The fused CG kernels are short (a few MB per launch): each thread loads its first CG_PRE grid-stride
// elements before summing the previous step's partials, so that reduction overlaps the loads; the
// per-thread element order (and every sum) is unchanged.
constexpr int CG_PRE = 2;

// slabs != null: raw_i = sum_{k < P} slabs[k * m + i], summed as panel_reduce_kernel does — from 0 in
// panel order, and for P >= 16 (its split form) as four quarter sums of ceil(P / 4) panels combined
// ((q0 + q1) + q2) + q3 — so Ad is bitwise the reduced pass output the other K·p calls see
template <typename T>
__global__ __launch_bounds__(CG_NT) void cg_fin_dad_kernel(const T *__restrict__ raw, const T *__restrict__ slabs,
                                                         int64_t P, int64_t sstride, const T *__restrict__ q,
                                                         const T *__restrict__ d, const T *__restrict__ psum, int G,
                                                         T QA_cost, T cost_inv, int raw_only, int64_t m,
                                                         T *__restrict__ Ad, T *__restrict__ pdad,
                                                         cg_scalars<T> *sc) {
    if (sc->converged) return;
    __shared__ T red[CG_NT / 64], bc[1];
    const int64_t i0 = (int64_t) blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t) gridDim.x * blockDim.x;
    auto load_raw = [&](int64_t i) {
        if (slabs == nullptr) return raw[i];
        if (P < 16) {
            T rw = 0;
            for (int64_t k = 0; k < P; ++k) rw += slabs[k * sstride + i];
            return rw;
        }
        const int64_t per = (P + 3) / 4;
        T qs[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            T a = 0;
            for (int64_t k = u * per; k < min(P, (u + 1) * per); ++k) a += slabs[k * sstride + i];
            qs[u] = a;
        }
        return ((qs[0] + qs[1]) + qs[2]) + qs[3];
    };
    T rw[CG_PRE], qv[CG_PRE], dv[CG_PRE];
#pragma unroll
    for (int e = 0; e < CG_PRE; ++e) {
        const int64_t i = i0 + e * st;
        if (i < m) rw[e] = load_raw(i), qv[e] = q[i], dv[e] = d[i];
    }
    T sp, sqp;
    partials_total(psum, G, red, bc, sp, sqp);
    if (blockIdx.x == 0 && threadIdx.x == 0) sc->sp = sp, sc->sqp = sqp;
    T s1 = 0;
    auto one = [&](int64_t i, T r_, T q_, T d_) {
        const T v = cg_fin_value(r_, q_, d_, sp, sqp, QA_cost, cost_inv, raw_only);
        Ad[i] = v;
        s1 = cg_acc(s1, d_, v);
    };
#pragma unroll
    for (int e = 0; e < CG_PRE; ++e) {
        const int64_t i = i0 + e * st;
        if (i < m) one(i, rw[e], qv[e], dv[e]);
    }
    for (int64_t i = i0 + CG_PRE * st; i < m; i += st) one(i, load_raw(i), q[i], d[i]);
    store_partial_first(s1, red, pdad);  // (consumers read the first partial of the pair only)
}

template <typename T>
__global__ __launch_bounds__(CG_NT) void cg_upd_rr_kernel(T *__restrict__ x, T *__restrict__ r, const T *__restrict__ d,
                                                        const T *__restrict__ Ad, const T *__restrict__ b, int reset,
                                                        const T *__restrict__ pdad, int G, int64_t m,
                                                        T *__restrict__ prr, cg_scalars<T> *sc) {
    if (sc->converged) return;
    __shared__ T red[CG_NT / 64], bc[1];
    const int64_t i0 = (int64_t) blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t) gridDim.x * blockDim.x;
    T xv[CG_PRE], dv[CG_PRE], av[CG_PRE], rv[CG_PRE];  // reset: av = b
#pragma unroll
    for (int e = 0; e < CG_PRE; ++e) {
        const int64_t i = i0 + e * st;
        if (i < m) xv[e] = x[i], dv[e] = d[i], av[e] = reset ? b[i] : Ad[i], rv[e] = reset ? T(0) : r[i];
    }
    const T dAd = partials_total1(pdad, G, red, bc);
    const T delta = sc->delta;
    const T alpha = delta / dAd;
    if (blockIdx.x == 0 && threadIdx.x == 0) sc->dAd = dAd, sc->alpha = alpha, sc->delta_prev = delta;
    T s1 = 0;
    auto one = [&](int64_t i, T x_, T d_, T a_, T r_) {
        const T t = alpha * d_;
        x[i] = x_ + t;
        if (reset) {
            r[i] = a_;
        } else {
            const T u = alpha * a_;
            const T rn = r_ - u;
            r[i] = rn;
            s1 += rn * rn;
        }
    };
#pragma unroll
    for (int e = 0; e < CG_PRE; ++e) {
        const int64_t i = i0 + e * st;
        if (i < m) one(i, xv[e], dv[e], av[e], rv[e]);
    }
    for (int64_t i = i0 + CG_PRE * st; i < m; i += st) one(i, x[i], d[i], reset ? b[i] : Ad[i], reset ? T(0) : r[i]);
    if (!reset) store_partial1(s1, red, prr);
}

template <typename T, bool W>
__global__ __launch_bounds__(CG_NT) void cg_dir_sums_kernel(T *__restrict__ d, const T *__restrict__ r,
                                                          const T *__restrict__ q, const T *__restrict__ prr, int G,
                                                          int init, double *trace, int64_t trace_cap, int64_t m,
                                                          T *__restrict__ psum, cg_scalars<T> *sc, dir_w_t<T> wo) {
    if (sc->converged) return;
    __shared__ T red[CG_NT / 64], bc[1];
    const int64_t i0 = (int64_t) blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t) gridDim.x * blockDim.x;
    T dv[CG_PRE], rv[CG_PRE], qv[CG_PRE], ev[CG_PRE], cv[CG_PRE];
#pragma unroll
    for (int e = 0; e < CG_PRE; ++e) {
        const int64_t i = i0 + e * st;
        if (i < m) {
            dv[e] = init ? T(0) : d[i], rv[e] = r[i], qv[e] = q[i];
            if constexpr (W) ev[e] = wo.e != nullptr ? wo.e[i] : T(1), cv[e] = wo.cw != nullptr ? wo.cw[i] : T(0);
        }
    }
    T beta = 0;
    if (!init) {
        const T rr = partials_total1(prr, G, red, bc);
        const bool conv = rr <= sc->eps2delta0;
        beta = rr / sc->delta_prev;
        if (blockIdx.x == 0 && threadIdx.x == 0) {  // FIN_DELTA of dot_final_kernel
            // the iteration index lives on the device (captured iteration blocks are position-free)
            const int64_t run = sc->iters;
            sc->delta = rr;
            sc->iters = run + 1;
            if (trace && run + 1 < trace_cap) trace[run + 1] = (double) rr;
            if (conv) sc->converged = 1;
            else sc->beta = beta;
        }
        if (conv) return;  // the same decision in every block
    }
    T s1 = 0, s2 = 0, s3 = 0;
    auto one = [&](int64_t i, T d_, T r_, T q_, T e_, T c_) {
        T dn;
        if (init) {
            dn = r_;
        } else {
            const T t = beta * d_;
            dn = t + r_;
        }
        d[i] = dn;
        s1 += dn;
        s2 += q_ * dn;
        if constexpr (W) w_elem(i, dn, e_, c_, wo.e, wo.cw, wo.w, wo.w16, s3);
    };
#pragma unroll
    for (int e = 0; e < CG_PRE; ++e) {
        const int64_t i = i0 + e * st;
        if (i < m) {
            if constexpr (W) one(i, dv[e], rv[e], qv[e], ev[e], cv[e]);
            else one(i, dv[e], rv[e], qv[e], T(1), T(0));
        }
    }
    for (int64_t i = i0 + CG_PRE * st; i < m; i += st) {
        if constexpr (W)
            one(i, init ? T(0) : d[i], r[i], q[i], wo.e != nullptr ? wo.e[i] : T(1), wo.cw != nullptr ? wo.cw[i] : T(0));
        else one(i, init ? T(0) : d[i], r[i], q[i], T(1), T(0));
    }
    store_partials(s1, s2, red, psum);
    if constexpr (W) {
        __syncthreads();
        store_partial1(s3, red, wo.spart);
    }
}

// ---- one-reduction CG (Chronopoulos & Gear 1989; a sharded group's option, plssvm_mi OPT_CG_VARIANT) ------------------
// The same iterates as openmp::csvm::solver_CG in exact arithmetic (OpenMP/csvm.cpp:82-170), with the matrix product of
// r instead of d and s = Q~d carried by a recurrence, so an iteration's inner products are summed together after one
// gather of their partials — one exposed collective per iteration instead of the reference's two (d.Ad before the
// x / r update, r.r before the direction update):
//   u_k = Q~ r_k;  gamma_k = r_k.r_k;  beta_k = gamma_k / gamma_{k-1};  d_k = r_k + beta_k d_{k-1};  s_k = u_k + beta_k s_{k-1}
//   d_k.s_k = r_k.u_k + 2 beta_k r_k.s_{k-1} + beta_k^2 d_{k-1}.s_{k-1};  alpha_k = gamma_k / d_k.s_k
//   x_{k+1} = x_k + alpha_k d_k;  r_{k+1} = r_k - alpha_k s_k   (every 50th iteration r_{k+1} = b - Q~x_{k+1} instead)
// d.s is expanded with the measured r_k.s_{k-1} (formed by the update that forms r_k, at no extra pass) rather than
// Chronopoulos-Gear's -gamma_k / alpha_{k-1}, which assumes r_k orthogonal to d_{k-1}: in fp32 the assumed form left
// the oracle's curve by up to 1.6e-3 on the long-trace expansion sets, the measured one stays with it.
// Partial sets (4 RED_BLOCKS per rank, by iteration parity): [r.u | r.r | r.s_prev | 0]; the finalize writes the first,
// the update of the previous iteration the second and third.
// The stop test delta <= eps^2 delta0 and the trace (r.r before each iteration) keep the reference's meaning; the r.r of
// r_k is known when the update of iteration k runs, so the test of r_k is made there (after u_k = Q~r_k, one matrix
// product that a converged solve does not use) or, at the end of a batch, by cg1_delta_kernel.
constexpr int CG1_SET = 4 * RED_BLOCKS;

// the first three sums of a gathered [.. | .. | .. | 0] set (G ranks, rank order in each element)
template <typename T>
__device__ __forceinline__ void cg1_totals(const T *__restrict__ pset, int G, T *red, T *bc, T &a, T &b, T &c) {
    T s1 = 0, s2 = 0, s3 = 0;
    for (int i = threadIdx.x; i < RED_BLOCKS; i += blockDim.x) {
        T x1 = pset[i], x2 = pset[RED_BLOCKS + i], x3 = pset[2 * RED_BLOCKS + i];
        for (int g = 1; g < G; ++g) {
            x1 += pset[g * CG1_SET + i];
            x2 += pset[g * CG1_SET + RED_BLOCKS + i];
            x3 += pset[g * CG1_SET + 2 * RED_BLOCKS + i];
        }
        s1 += x1;
        s2 += x2;
        s3 += x3;
    }
    a = block_sum_all(s1, red, bc);
    b = block_sum_all(s2, red, bc);
    c = block_sum_all(s3, red, bc);
}

template <typename T, bool W>
__global__ __launch_bounds__(CG_NT) void cg1_update_kernel(T *__restrict__ x, T *__restrict__ r, T *__restrict__ d,
                                                         T *__restrict__ s, const T *__restrict__ u, const T *__restrict__ b,
                                                         const T *__restrict__ q, int reset, const T *__restrict__ pset,
                                                         int G, double *trace, int64_t trace_cap, int64_t m, int par,
                                                         T *__restrict__ pnext, T *__restrict__ psum, cg_scalars<T> *sc,
                                                         dir_w_t<T> wo) {
    if (sc->converged) return;
    __shared__ T red[CG_NT / 64], bc[1];
    const int64_t i0 = (int64_t) blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t) gridDim.x * blockDim.x;
    T ru, rr, rs;
    cg1_totals(pset, G, red, bc, ru, rr, rs);  // r.u, r.r, r.s_prev, ranks in order
    const bool conv = rr <= sc->eps2delta0;
    const T gprev = sc->g1[par ^ 1], dsprev = sc->d1[par ^ 1];  // +inf / 0 before the first iteration: beta = 0
    const T beta = rr / gprev;
    const T t1 = beta * rs, bb = beta * beta;
    const T t3 = bb * dsprev;
    const T ds = (ru + (t1 + t1)) + t3;
    const T alpha = rr / ds;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t run = sc->iters;  // the iteration index lives on the device (captured blocks are position-free)
        sc->delta = rr;
        if (trace && run < trace_cap) trace[run] = (double) rr;
        if (conv) {
            sc->converged = 1;
        } else {
            sc->g1[par] = rr, sc->a1[par] = alpha, sc->d1[par] = ds;
            sc->alpha = alpha, sc->beta = beta, sc->dAd = ds, sc->delta_prev = rr;
            sc->iters = run + 1;
        }
    }
    if (conv) return;  // the same decision in every block
    T s1 = 0, s2 = 0, s3 = 0, srr = 0, srs = 0;
    for (int64_t i = i0; i < m; i += st) {
        const T ri = r[i];
        const T tb = beta * d[i];
        const T dn = ri + tb;
        d[i] = dn;
        const T ts = beta * s[i];
        const T sn = u[i] + ts;
        s[i] = sn;
        const T tx = alpha * dn;
        x[i] = x[i] + tx;
        if (reset) {
            r[i] = b[i];  // r = b - Q~x follows (engine: the matrix product of x, then cg1_rsums_kernel)
        } else {
            const T ua = alpha * sn;
            const T rn = ri - ua;
            r[i] = rn;
            srr += rn * rn;
            srs += rn * sn;
            s1 += rn;
            s2 += q[i] * rn;
            if constexpr (W) w_elem(i, rn, wo.e != nullptr ? wo.e[i] : T(1), wo.cw != nullptr ? wo.cw[i] : T(0), wo.e, wo.cw,
                                    wo.w, wo.w16, s3);
        }
    }
    if (reset) return;
    store_partial_second(srr, red, pnext);                  // r.r of r_{k+1}
    __syncthreads();
    store_partial_first(srs, red, pnext + 2 * RED_BLOCKS);  // r_{k+1}.s_k
    __syncthreads();
    store_partials(s1, s2, red, psum);  // sum r / sum q r: the rank-1 terms of the next product
    if constexpr (W) {
        __syncthreads();
        store_partial1(s3, red, wo.spart);
    }
}

// r.r, sum r, sum q r (and the expansion's w pass) of a residual formed by a matrix product (x0 = 1, every 50th
// iteration): the partials cg1_update_kernel leaves for a recurrence-formed r
template <typename T, bool W>
__global__ __launch_bounds__(CG_NT) void cg1_rsums_kernel(const T *__restrict__ r, const T *__restrict__ sv,
                                                        const T *__restrict__ q, int64_t m, T *__restrict__ pnext,
                                                        T *__restrict__ psum, const cg_scalars<T> *sc, dir_w_t<T> wo) {
    if (sc->converged) return;
    __shared__ T red[CG_NT / 64];
    const int64_t i0 = (int64_t) blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t) gridDim.x * blockDim.x;
    T s1 = 0, s2 = 0, s3 = 0, srr = 0, srs = 0;
    for (int64_t i = i0; i < m; i += st) {
        const T ri = r[i];
        srr += ri * ri;
        srs += ri * sv[i];
        s1 += ri;
        s2 += q[i] * ri;
        if constexpr (W) w_elem(i, ri, wo.e != nullptr ? wo.e[i] : T(1), wo.cw != nullptr ? wo.cw[i] : T(0), wo.e, wo.cw, wo.w,
                                wo.w16, s3);
    }
    store_partial_second(srr, red, pnext);
    __syncthreads();
    store_partial_first(srs, red, pnext + 2 * RED_BLOCKS);
    __syncthreads();
    store_partials(s1, s2, red, psum);
    if constexpr (W) {
        __syncthreads();
        store_partial1(s3, red, wo.spart);
    }
}

// the end of a batch: r.r of the current r (the second partials of pset, summed as cg1_update_kernel sums them — the
// same bits), its trace entry and the stop test, so the host's poll sees the reference's residual after each iteration
template <typename T>
__global__ __launch_bounds__(CG_NT) void cg1_delta_kernel(const T *__restrict__ pset, int G, double *trace,
                                                        int64_t trace_cap, cg_scalars<T> *sc) {
    if (sc->converged) return;
    __shared__ T red[CG_NT / 64], bc[1];
    T ru, rr, rs;
    cg1_totals(pset, G, red, bc, ru, rr, rs);
    (void) ru, (void) rs;
    if (threadIdx.x == 0) {
        const int64_t run = sc->iters;
        sc->delta = rr;
        if (trace && run < trace_cap) trace[run] = (double) rr;
        if (rr <= sc->eps2delta0) sc->converged = 1;
    }
}

}  // namespace

template <typename T>
void launch_cg1_update(T *x, T *r, T *d, T *s, const T *u, const T *b, const T *q, int reset, const T *pset, int G,
                       double *trace, int64_t trace_cap, int64_t m, int par, T *pnext, T *psum, cg_scalars<T> *sc,
                       hipStream_t st, const dir_w_t<T> *wout) {
    if (wout != nullptr && !reset)
        hipLaunchKernelGGL((cg1_update_kernel<T, true>), dim3(RED_BLOCKS), dim3(CG_NT), 0, st, x, r, d, s, u, b, q, reset,
                           pset, G, trace, trace_cap, m, par, pnext, psum, sc, *wout);
    else
        hipLaunchKernelGGL((cg1_update_kernel<T, false>), dim3(RED_BLOCKS), dim3(CG_NT), 0, st, x, r, d, s, u, b, q, reset,
                           pset, G, trace, trace_cap, m, par, pnext, psum, sc, dir_w_t<T>{});
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg1_rsums(const T *r, const T *s, const T *q, int64_t m, T *pnext, T *psum, cg_scalars<T> *sc, hipStream_t st,
                      const dir_w_t<T> *wout) {
    if (wout != nullptr)
        hipLaunchKernelGGL((cg1_rsums_kernel<T, true>), dim3(RED_BLOCKS), dim3(CG_NT), 0, st, r, s, q, m, pnext, psum, sc,
                           *wout);
    else
        hipLaunchKernelGGL((cg1_rsums_kernel<T, false>), dim3(RED_BLOCKS), dim3(CG_NT), 0, st, r, s, q, m, pnext, psum, sc,
                           dir_w_t<T>{});
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg1_delta(const T *pset, int G, double *trace, int64_t trace_cap, cg_scalars<T> *sc, hipStream_t st) {
    hipLaunchKernelGGL(cg1_delta_kernel<T>, dim3(1), dim3(CG_NT), 0, st, pset, G, trace, trace_cap, sc);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg_fin_dad(const T *raw, const T *slabs, int64_t P, int64_t sstride, const T *q, const T *d, const T *psum,
                       int G, T QA_cost, T cost_inv, int raw_only, int64_t m, T *Ad, T *pdad, cg_scalars<T> *sc,
                       hipStream_t s) {
    hipLaunchKernelGGL(cg_fin_dad_kernel<T>, dim3(RED_BLOCKS), dim3(CG_NT), 0, s, raw, slabs, P, sstride, q, d, psum, G,
                       QA_cost, cost_inv, raw_only, m, Ad, pdad, sc);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg_upd_rr(T *x, T *r, const T *d, const T *Ad, const T *b, int reset, const T *pdad, int G, int64_t m,
                      T *prr, cg_scalars<T> *sc, hipStream_t s) {
    hipLaunchKernelGGL(cg_upd_rr_kernel<T>, dim3(RED_BLOCKS), dim3(CG_NT), 0, s, x, r, d, Ad, b, reset, pdad, G, m, prr,
                       sc);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg_dir_sums(T *d, const T *r, const T *q, const T *prr, int G, int init, double *trace,
                        int64_t trace_cap, int64_t m, T *psum, cg_scalars<T> *sc, hipStream_t s, const dir_w_t<T> *wout) {
    if (wout != nullptr)
        hipLaunchKernelGGL((cg_dir_sums_kernel<T, true>), dim3(RED_BLOCKS), dim3(CG_NT), 0, s, d, r, q, prr, G, init,
                           trace, trace_cap, m, psum, sc, *wout);
    else
        hipLaunchKernelGGL((cg_dir_sums_kernel<T, false>), dim3(RED_BLOCKS), dim3(CG_NT), 0, s, d, r, q, prr, G, init,
                           trace, trace_cap, m, psum, sc, dir_w_t<T>{});
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_dot2(const T *a, const T *b, const T *c, const T *e, int64_t n, T *partials, const cg_scalars<T> *status,
                 hipStream_t s) {
    hipLaunchKernelGGL(dot2_kernel<T>, dim3(RED_BLOCKS), dim3(256), 0, s, a, b, c, e, n, partials, status);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_dot_final(const T *partials, cg_scalars<T> *sc, int op, int64_t run, double *trace, int64_t trace_cap,
                      T *plain_out, hipStream_t s, int G) {
    hipLaunchKernelGGL(dot_final_kernel<T>, dim3(1), dim3(256), 0, s, partials, G, sc, op, run, trace, trace_cap,
                       plain_out);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg_init(const T *b, int64_t m, T *x, T *r, hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(cg_init_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, b, m, x, r);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_copy(const T *src, int64_t n, T *dst, const cg_scalars<T> *status, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(copy_kernel<T>, dim3((unsigned) ceil_div(n, 256)), dim3(256), 0, s, src, n, dst, status);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg_update(T *x, T *r, const T *d, const T *Ad, const T *b, int reset, int64_t m, const cg_scalars<T> *sc,
                      hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(cg_update_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, x, r, d, Ad, b, reset,
                       m, sc);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_cg_direction(T *d, const T *r, int64_t m, const cg_scalars<T> *sc, hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(cg_direction_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, d, r, m, sc);
    MI_LAUNCH_CHECK();
}

#define INST(T)                                                                                                     \
    template void launch_dot2<T>(const T *, const T *, const T *, const T *, int64_t, T *, const cg_scalars<T> *, \
                                 hipStream_t);                                                                    \
    template void launch_dot_final<T>(const T *, cg_scalars<T> *, int, int64_t, double *, int64_t, T *,           \
                                      hipStream_t, int);                                                          \
    template void launch_cg_init<T>(const T *, int64_t, T *, T *, hipStream_t);                                   \
    template void launch_copy<T>(const T *, int64_t, T *, const cg_scalars<T> *, hipStream_t);                    \
    template void launch_cg_update<T>(T *, T *, const T *, const T *, const T *, int, int64_t,                    \
                                      const cg_scalars<T> *, hipStream_t);                                        \
    template void launch_cg_direction<T>(T *, const T *, int64_t, const cg_scalars<T> *, hipStream_t);             \
    template void launch_cg_fin_dad<T>(const T *, const T *, int64_t, int64_t, const T *, const T *, const T *,    \
                                       int, T, T, int, int64_t, T *, T *, cg_scalars<T> *, hipStream_t);           \
    template void launch_cg_upd_rr<T>(T *, T *, const T *, const T *, const T *, int, const T *, int, int64_t, T *, \
                                      cg_scalars<T> *, hipStream_t);                                                \
    template void launch_cg_dir_sums<T>(T *, const T *, const T *, const T *, int, int, double *, int64_t, int64_t, \
                                        T *, cg_scalars<T> *, hipStream_t, const dir_w_t<T> *);                     \
    template void launch_cg1_update<T>(T *, T *, T *, T *, const T *, const T *, const T *, int, const T *, int,     \
                                       double *, int64_t, int64_t, int, T *, T *, cg_scalars<T> *, hipStream_t,      \
                                       const dir_w_t<T> *);                                                         \
    template void launch_cg1_rsums<T>(const T *, const T *, const T *, int64_t, T *, T *, cg_scalars<T> *, hipStream_t, \
                                      const dir_w_t<T> *);                                                          \
    template void launch_cg1_delta<T>(const T *, int, double *, int64_t, cg_scalars<T> *, hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
