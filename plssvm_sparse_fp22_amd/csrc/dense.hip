// Dense feature data: q vector, row norms and the implicit pairwise K·p tiles on MFMA (gfx950).
//
// Replaces the reference's device_kernel_{linear,poly,radial}
// (include/plssvm/backends/HIP/svm_kernel.hip.hpp:36-268) and device_kernel_q_*
// (q_kernel.hip.hpp:32-83). Design:
//   * X lives feature-major in HBM, XT[k][i] (k < d_pad, i < n_pad), zero padded, 64-bit offsets;
//   * one 256-thread workgroup per 128x128 lower-triangle tile (I >= J) of the implicit kernel
//     matrix; the Gram block X_I X_J^T runs on v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32
//     (exact fma chains, K = 4 per instruction) from LDS-staged [k][i] panels;
//   * the epilogue applies the kernel function in registers (RBF via ||a||^2+||b||^2-2a.b),
//     multiplies by p and reduces rows (16-lane shuffles) and columns (cross-half shuffles);
//   * no atomics: the row sums go to partial[J][i in I], the mirrored column sums to
//     partial[I][j in J]; a second kernel sums each row's nb partials in a fixed order, so
//     K·p is bitwise reproducible run to run.
#include "kernels.hpp"

namespace plssvm_mi {

namespace {

template <typename T>
__device__ __forceinline__ T kernel_apply(int kernel, int degree, T gamma, T coef0, T g, T ni, T nj) {
    if (kernel == 0) return g;
    if (kernel == 1) {
        const T base = fma(gamma, g, coef0);
        T r = T(1);
        for (int e = 0; e < degree; ++e) r *= base;
        return r;
    }
    T dist = ni + nj - T(2) * g;
    dist = dist > T(0) ? dist : T(0);
    return exp(-gamma * dist);
}

// ---------------------------------------------------------------------------------------------
// 64x64 LDS-tiled transpose of the row-major host layout into the feature-major device layout.
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T *__restrict__ X, int64_t rows, int64_t d,
                                                        T *__restrict__ XT, int64_t n_pad) {
    __shared__ T tile[64][65];
    const int64_t i0 = (int64_t) blockIdx.x * 64, k0 = (int64_t) blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int yy = ty; yy < 64; yy += 4) {
        const int64_t i = i0 + yy, k = k0 + tx;
        tile[yy][tx] = (i < rows && k < d) ? X[i * d + k] : T(0);
    }
    __syncthreads();
    for (int yy = ty; yy < 64; yy += 4) {
        const int64_t k = k0 + yy, i = i0 + tx;
        if (k < d && i < rows) XT[k * n_pad + i] = tile[tx][yy];
    }
}

template <typename T>
__global__ __launch_bounds__(256) void row_norms_kernel(const T *__restrict__ XT, int64_t n_pad, int64_t d,
                                                        T *__restrict__ norms) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    T v = 0;
    for (int64_t k = 0; k < d; ++k) {
        const T x = XT[k * n_pad + i];
        v = fma(x, x, v);
    }
    norms[i] = v;
}

template <typename T>
__global__ __launch_bounds__(256) void q_dense_kernel(kfun<T> kf, const T *__restrict__ XT, int64_t n_pad, int64_t d,
                                                      int64_t m, const T *__restrict__ xlast, T *__restrict__ q) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    T v = 0;
    if (kf.kernel == 2) {
        for (int64_t k = 0; k < d; ++k) {
            const T diff = XT[k * n_pad + i] - xlast[k];
            v = fma(diff, diff, v);
        }
        q[i] = exp(-kf.gamma * v);
    } else {
        for (int64_t k = 0; k < d; ++k) v = fma(XT[k * n_pad + i], xlast[k], v);
        if (kf.kernel == 0) {
            q[i] = v;
        } else {
            const T base = fma(kf.gamma, v, kf.coef0);
            T r = T(1);
            for (int e = 0; e < kf.degree; ++e) r *= base;
            q[i] = r;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void kp_finalize_kernel(const T *__restrict__ raw, const T *__restrict__ q,
                                                          const T *__restrict__ p, const cg_scalars<T> *sc,
                                                          T QA_cost, T cost_inv, T add, int overwrite, int64_t m,
                                                          T *__restrict__ ret,
                                                          const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const T sp = sc->sp, sqp = sc->sqp;
    // flags (overwrite): bit 0 = overwrite ret, bit 1 = raw share only (simulated rank != 0)
    const T v = (overwrite & 2) ? raw[i] : raw[i] + (QA_cost - q[i]) * sp - sqp + cost_inv * p[i];
    ret[i] = ((overwrite & 1) ? T(0) : ret[i]) + add * v;
}

// ---- factored linear: two coalesced passes over XT ----------------------------------------------
// w[k] = sum_i XT[k][i] p_i : one workgroup per feature row, 16-byte loads along i.
template <typename T>
__global__ __launch_bounds__(256) void gemv_t_kernel(const T *__restrict__ XT, int64_t n_pad, int64_t d, int64_t r0,
                                                     int64_t r1, const T *__restrict__ p, T *__restrict__ w,
                                                     const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t k = blockIdx.x;
    if (k >= d) return;
    const T *row = XT + k * n_pad;
    T s = 0;
    for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) s = fma(row[i], p[i], s);
    __shared__ T red[4];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) w[k] = (red[0] + red[1]) + (red[2] + red[3]);
}

// raw[i] = sum_k XT[k][i] w_k : thread per row, coalesced over i, w broadcast from LDS.
template <typename T>
__global__ __launch_bounds__(256) void gemv_n_kernel(const T *__restrict__ XT, int64_t n_pad, int64_t d, int64_t r0,
                                                     int64_t r1, const T *__restrict__ w, T *__restrict__ raw,
                                                     const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = r0 + (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    __shared__ T ws[1024];
    T s = 0;
    for (int64_t k0 = 0; k0 < d; k0 += 1024) {
        const int64_t kn = (d - k0) < 1024 ? (d - k0) : 1024;
        __syncthreads();
        for (int64_t u = threadIdx.x; u < kn; u += 256) ws[u] = w[k0 + u];
        __syncthreads();
        if (i < r1)
            for (int64_t u = 0; u < kn; ++u) s = fma(XT[(k0 + u) * n_pad + i], ws[u], s);
    }
    if (i < r1) raw[i] = s;
}

}  // namespace

// ---- launchers ----------------------------------------------------------------------------------
template <typename T>
void launch_transpose(const T *X, int64_t rows, int64_t d, T *XT, int64_t n_pad, hipStream_t s) {
    if (rows <= 0 || d <= 0) return;
    hipLaunchKernelGGL(transpose_kernel<T>, dim3((unsigned) ceil_div(rows, 64), (unsigned) ceil_div(d, 64)), dim3(256),
                       0, s, X, rows, d, XT, n_pad);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_row_norms(const T *XT, int64_t n_pad, int64_t d, T *norms, hipStream_t s) {
    hipLaunchKernelGGL(row_norms_kernel<T>, dim3((unsigned) ceil_div(n_pad, 256)), dim3(256), 0, s, XT, n_pad, d,
                       norms);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_q_dense(kfun<T> kf, const T *XT, int64_t n_pad, int64_t d, int64_t m, const T *xlast, T *q,
                    hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(q_dense_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, kf, XT, n_pad, d, m,
                       xlast, q);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_kp_finalize(const T *raw, const T *q, const T *p, const cg_scalars<T> *sc, T QA_cost, T cost_inv, T add,
                        int overwrite, int64_t m, T *ret, const cg_scalars<T> *status, hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(kp_finalize_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, raw, q, p, sc,
                       QA_cost, cost_inv, add, overwrite, m, ret, status);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_gemv_t(const T *XT, int64_t n_pad, int64_t d, int64_t r0, int64_t r1, const T *p, T *w,
                   const cg_scalars<T> *status, hipStream_t s) {
    if (d <= 0) return;
    hipLaunchKernelGGL(gemv_t_kernel<T>, dim3((unsigned) d), dim3(256), 0, s, XT, n_pad, d, r0, r1, p, w, status);
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_gemv_n(const T *XT, int64_t n_pad, int64_t d, int64_t r0, int64_t r1, const T *w, T *raw,
                   const cg_scalars<T> *status, hipStream_t s) {
    if (r1 <= r0) return;
    hipLaunchKernelGGL(gemv_n_kernel<T>, dim3((unsigned) ceil_div(r1 - r0, 256)), dim3(256), 0, s, XT, n_pad, d, r0,
                       r1, w, raw, status);
    MI_LAUNCH_CHECK();
}

#define INST(T)                                                                                                    \
    template void launch_transpose<T>(const T *, int64_t, int64_t, T *, int64_t, hipStream_t);                   \
    template void launch_row_norms<T>(const T *, int64_t, int64_t, T *, hipStream_t);                            \
    template void launch_q_dense<T>(kfun<T>, const T *, int64_t, int64_t, int64_t, const T *, T *, hipStream_t); \
    template void launch_kp_finalize<T>(const T *, const T *, const T *, const cg_scalars<T> *, T, T, T, int,    \
                                        int64_t, T *, const cg_scalars<T> *, hipStream_t);                       \
    template void launch_gemv_t<T>(const T *, int64_t, int64_t, int64_t, int64_t, const T *, T *,                \
                                   const cg_scalars<T> *, hipStream_t);                                          \
    template void launch_gemv_n<T>(const T *, int64_t, int64_t, int64_t, int64_t, const T *, T *,                \
                                   const cg_scalars<T> *, hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
