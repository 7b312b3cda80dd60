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

// ---------------------------------------------------------------------------------------------
// Pairwise tile kernel. 4 waves as 2x2; wave (wr, wc) owns the 64x64 sub-tile, i.e. 4x4 MFMA
// 16x16 accumulators. K loop over BK-deep feature panels staged in LDS as [k][i] with a row
// stride of 144 elements (conflict-free: k and k+1 rows land on opposite bank halves).
template <typename T, int KERNEL>
__global__ __launch_bounds__(256, 2) void kp_tile_kernel(kfun<T> kf, const T *__restrict__ XT,
                                                      const T *__restrict__ norms, const T *__restrict__ p,
                                                      T *__restrict__ partial, int64_t n_pad, int64_t d_pad,
                                                      int64_t t0, int64_t ntiles,
                                                      const cg_scalars<T> *__restrict__ status) {
    using M = mfma16<T>;
    using acc_t = typename M::acc_t;
    constexpr int BK = kp_bk<T>();
    constexpr int LDA = KP_TILE + 16;
    constexpr int VEC = 16 / (int) sizeof(T);       // elements per 16-byte load
    constexpr int VPR = KP_TILE / VEC;              // 16-byte vectors per panel row
    constexpr int NV = BK * VPR / 256;              // vectors per thread per operand
    using vec_t = typename std::conditional<sizeof(T) == 8, double2, float4>::type;

    __shared__ __attribute__((aligned(16))) T As[BK * LDA];
    __shared__ __attribute__((aligned(16))) T Bs[BK * LDA];
    __shared__ T rowbuf[2][KP_TILE];
    __shared__ T colbuf[2][KP_TILE];

    if (status != nullptr && status->converged) return;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;

    int64_t I, J;
    tri_tile(t0 + xcd_remap(blockIdx.x, ntiles), I, J);
    const int64_t I0 = I * KP_TILE, J0 = J * KP_TILE;
    const bool diag = (I == J);

    acc_t acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = acc_t{ 0, 0, 0, 0 };

    vec_t ra[NV], rb[NV];
    auto load_panel = [&](int64_t k0) {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int idx = tid + 256 * u;
            const int row = idx / VPR, cv = idx % VPR;
            const int64_t off = (k0 + row) * n_pad + cv * VEC;
            ra[u] = *reinterpret_cast<const vec_t *>(XT + off + I0);
            rb[u] = *reinterpret_cast<const vec_t *>(XT + off + J0);
        }
    };
    auto store_panel = [&]() {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int idx = tid + 256 * u;
            const int row = idx / VPR, cv = idx % VPR;
            *reinterpret_cast<vec_t *>(As + row * LDA + cv * VEC) = ra[u];
            *reinterpret_cast<vec_t *>(Bs + row * LDA + cv * VEC) = rb[u];
        }
    };

    const int64_t nk = d_pad / BK;
    load_panel(0);
    for (int64_t kc = 0; kc < nk; ++kc) {
        __syncthreads();
        store_panel();
        __syncthreads();
        if (kc + 1 < nk) load_panel((kc + 1) * BK);
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks) {
            const int kr = ks * 4 + (lane >> 4);
            T a[4], b[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) a[mt] = As[kr * LDA + wr * 64 + mt * 16 + (lane & 15)];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) b[nt] = Bs[kr * LDA + wc * 64 + nt * 16 + (lane & 15)];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = M::op(a[mt], b[nt], acc[mt][nt]);
        }
    }

    // ---- epilogue: kernel function, times p, row and column sums ----
    T pj[4], nj[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int64_t j = J0 + wc * 64 + nt * 16 + (lane & 15);
        pj[nt] = p[j];
        nj[nt] = (KERNEL == 2) ? norms[j] : T(0);
    }
    T cs[4] = { 0, 0, 0, 0 };
    T rs[4][4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = I0 + wr * 64 + mt * 16 + M::row(lane, r);
            const T pi = p[i];
            const T ni = (KERNEL == 2) ? norms[i] : T(0);
            T s = 0;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const T kv = kernel_apply<T>(KERNEL, kf.degree, kf.gamma, kf.coef0, acc[mt][nt][r], ni, nj[nt]);
                s = fma(kv, pj[nt], s);
                cs[nt] = fma(kv, pi, cs[nt]);
            }
            rs[mt][r] = s;
        }
    }
    // rows: lanes sharing (lane >> 4) hold the same row -> reduce over lane & 15
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            T v = rs[mt][r];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if ((lane & 15) == 0) rowbuf[wc][wr * 64 + mt * 16 + M::row(lane, r)] = v;
        }
    }
    if (!diag) {
        // columns: lanes sharing (lane & 15) hold the same column -> reduce over lane >> 4
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            T v = cs[nt];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane < 16) colbuf[wr][wc * 64 + nt * 16 + lane] = v;
        }
    }
    __syncthreads();
    if (tid < KP_TILE) {
        partial[J * n_pad + I0 + tid] = rowbuf[0][tid] + rowbuf[1][tid];
    } else if (!diag) {
        const int t = tid - KP_TILE;
        partial[I * n_pad + J0 + t] = colbuf[0][t] + colbuf[1][t];
    }
}

template <typename T>
__global__ __launch_bounds__(256) void kp_reduce_kernel(const T *__restrict__ partial, int64_t nb, int64_t n_pad,
                                                        int64_t m, int64_t t0, int64_t t1, T *__restrict__ raw,
                                                        const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t R = i / KP_TILE;
    T s = 0;
    if (t0 == 0 && t1 == nb * (nb + 1) / 2) {
        for (int64_t c = 0; c < nb; ++c) s += partial[c * n_pad + i];
    } else {
        for (int64_t c = 0; c < nb; ++c) {
            const int64_t t = (R >= c) ? tri_index(R, c) : tri_index(c, R);
            if (t >= t0 && t < t1) s += partial[c * n_pad + i];
        }
    }
    raw[i] = s;
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
    const T v = raw[i] + (QA_cost - q[i]) * sp - sqp + cost_inv * p[i];
    ret[i] = (overwrite ? T(0) : ret[i]) + add * v;
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
void launch_kp_tiles(kfun<T> kf, const T *XT, const T *norms, const T *p, T *partial, int64_t n_pad, int64_t d_pad,
                     int64_t t0, int64_t ntiles, const cg_scalars<T> *status, hipStream_t s) {
    if (ntiles <= 0) return;
    const dim3 grid((unsigned) ntiles), block(256);
    switch (kf.kernel) {
        case 0:
            hipLaunchKernelGGL((kp_tile_kernel<T, 0>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, t0,
                               ntiles, status);
            break;
        case 1:
            hipLaunchKernelGGL((kp_tile_kernel<T, 1>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, t0,
                               ntiles, status);
            break;
        default:
            hipLaunchKernelGGL((kp_tile_kernel<T, 2>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, t0,
                               ntiles, status);
            break;
    }
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_kp_reduce(const T *partial, int64_t nb, int64_t n_pad, int64_t m, int64_t t0, int64_t t1, T *raw,
                      const cg_scalars<T> *status, hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(kp_reduce_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, partial, nb, n_pad, m,
                       t0, t1, raw, status);
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
    template void launch_kp_tiles<T>(kfun<T>, const T *, const T *, const T *, T *, int64_t, int64_t, int64_t,   \
                                     int64_t, const cg_scalars<T> *, hipStream_t);                               \
    template void launch_kp_reduce<T>(const T *, int64_t, int64_t, int64_t, int64_t, int64_t, T *,               \
                                      const cg_scalars<T> *, hipStream_t);                                       \
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
