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
    store_partial1(s1, red, pdad);
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

}  // namespace

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
                                        T *, cg_scalars<T> *, hipStream_t, const dir_w_t<T> *);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
