// update_w and predict on the context's data (the learned model's support vectors).
//
// Replaces gpu_csvm::update_w / gpu_csvm::predict (src/plssvm/backends/gpu_csvm.cpp:52-127, 327-350)
// and device_kernel_w_linear / device_kernel_predict_{poly,radial}
// (include/plssvm/backends/HIP/predict_kernel.hip.hpp:33-114):
//     out[p] = bias + sum_{i < n} alpha_i k(x_i, z_p)          (linear: w . z_p + bias, w = sum_i alpha_i x_i)
// over all n points, the last one included. The reference HIP predict kernels index the last support
// vector past the transformed data (their `data_point_index == num_data_points` branch is never
// taken); this follows the OpenMP semantics (src/plssvm/backends/OpenMP/csvm.cpp:193-240).
//
// Layouts:
//   * dense data: G = X_m Z^T for a chunk of points on rocBLAS (a plain GEMM: library territory),
//     then one workgroup per point applies the kernel function and reduces sum_i alpha_i k_ip in a
//     fixed order (no atomics: a prediction is bitwise reproducible);
//   * sparse data: one wave per CSR row and one lane per predict point (64 points per launch); the
//     chunk's points are densified feature-major (ZT[f][64]) so the per-entry gather is one
//     coalesced 64-lane read, partial sums per row block, reduced in block order.
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/plssvm_mi355x.h"
#include "engine.hpp"

namespace plssvm_mi {

namespace {

#define MI_BLAS_CHECK(expr)                                                                                  \
    do {                                                                                                     \
        rocblas_status st_ = (expr);                                                                         \
        if (st_ != rocblas_status_success)                                                                   \
            throw mi_error(-2, std::string("rocBLAS error ") + rocblas_status_to_string(st_) + " (" #expr ")"); \
    } while (0)

// k(x, z) from the dot product g = x . z and the squared norms (RBF: exp(-gamma max(0, nx + nz - 2 g)))
template <typename T>
__device__ __forceinline__ T kval(const kfun<T> &kf, T g, T nx, T nz) {
    if (kf.kernel == 0) return g;
    if (kf.kernel == 1) {
        const T base = fma(kf.gamma, g, kf.coef0);
        T r = T(1);
        for (int e = 0; e < kf.degree; ++e) r *= base;
        return r;
    }
    T dist = nx + nz - T(2) * g;
    dist = dist > T(0) ? dist : T(0);
    return exp(-kf.gamma * dist);
}

template <typename T>
__device__ __forceinline__ T block_sum256(T v, T *red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// dense data: out[p] = bias + sum_{i<m} alpha_i k(G(i,p)) + alpha_m k(x_m . z_p); one workgroup per point
template <typename T>
__global__ __launch_bounds__(256) void predict_dense_epilogue_kernel(kfun<T> kf, const T *__restrict__ G, int64_t ldg,
                                                                     int64_t m, const T *__restrict__ norms,
                                                                     const T *__restrict__ alpha,
                                                                     const T *__restrict__ Z, int64_t d,
                                                                     const T *__restrict__ xlast, T nlast, T bias,
                                                                     T *__restrict__ out) {
    __shared__ T red[4];
    const int64_t p = blockIdx.x;
    const T *z = Z + p * d;
    T nz = 0, dl = 0;
    for (int64_t k = threadIdx.x; k < d; k += 256) {
        nz = fma(z[k], z[k], nz);
        dl = fma(xlast[k], z[k], dl);
    }
    nz = block_sum256(nz, red);
    dl = block_sum256(dl, red);
    const T *g = G + p * ldg;
    T s = 0;
    for (int64_t i = threadIdx.x; i < m; i += 256) s = fma(alpha[i], kval(kf, g[i], norms ? norms[i] : T(0), nz), s);
    s = block_sum256(s, red);
    if (threadIdx.x == 0) out[p] = (s + alpha[m] * kval(kf, dl, nlast, nz)) + bias;
}

// linear: out[p] = w . z_p + bias (the reference's fast path for the linear kernel)
template <typename T>
__global__ __launch_bounds__(256) void predict_linear_kernel(const T *__restrict__ w, const T *__restrict__ Z, int64_t d,
                                                             T bias, T *__restrict__ out) {
    __shared__ T red[4];
    const int64_t p = blockIdx.x;
    const T *z = Z + p * d;
    T s = 0;
    for (int64_t k = threadIdx.x; k < d; k += 256) s = fma(w[k], z[k], s);
    s = block_sum256(s, red);
    if (threadIdx.x == 0) out[p] = s + bias;
}

// sparse data: partial[b][lane] = sum_{i in row block b} alpha_i k(x_i, z_lane); ZT = [d][64]
constexpr int PRED_ROWS = 256;  // rows per workgroup
constexpr int PRED_STEP = 8;    // CSR entries per wave step (gathers in flight)
template <typename T>
__global__ __launch_bounds__(256) void predict_csr_kernel(kfun<T> kf, const int64_t *__restrict__ rowptr,
                                                          const int32_t *__restrict__ col, const T *__restrict__ val,
                                                          int64_t m, const T *__restrict__ ZT,
                                                          const T *__restrict__ nzv, const T *__restrict__ norms,
                                                          const T *__restrict__ alpha, T *__restrict__ partial) {
    __shared__ T red[4][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t r0 = (int64_t) blockIdx.x * PRED_ROWS, r1 = min(m, r0 + PRED_ROWS);
    const T nz = nzv[lane];
    T acc = 0;
    for (int64_t i = r0 + wave; i < r1; i += 4) {
        T s = 0;
        const int64_t e0 = rowptr[i], e1 = rowptr[i + 1];
        // 8 entries per step: their (wave-uniform) column/value loads, then 8 independent ZT gathers in
        // flight, then the fma chain in entry order (a masked tail entry adds 0 * ZT = 0 exactly)
        for (int64_t k = e0; k < e1; k += PRED_STEP) {
            int32_t c[PRED_STEP];
            T v[PRED_STEP], g[PRED_STEP];
#pragma unroll
            for (int u = 0; u < PRED_STEP; ++u) {
                const int64_t kk = min(k + u, e1 - 1);
                c[u] = col[kk];
                v[u] = k + u < e1 ? val[kk] : T(0);
            }
#pragma unroll
            for (int u = 0; u < PRED_STEP; ++u) g[u] = ZT[(int64_t) c[u] * 64 + lane];
#pragma unroll
            for (int u = 0; u < PRED_STEP; ++u) s = fma(v[u], g[u], s);
        }
        acc = fma(alpha[i], kval(kf, s, norms[i], nz), acc);
    }
    red[wave][lane] = acc;
    __syncthreads();
    if (wave == 0) partial[(int64_t) blockIdx.x * 64 + lane] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// ZT[col][p] = z_p[col] and |z_p|^2 (sequential fma in column order: the densified chain with its zero
// terms dropped, exactly) for the chunk's points p < c; lanes >= c get norm 0 (ZT pre-zeroed)
template <typename T>
__global__ __launch_bounds__(64) void zt_scatter_kernel(const int64_t *__restrict__ zr, const int32_t *__restrict__ zc,
                                                       const T *__restrict__ zv, int64_t p0, int64_t c,
                                                       T *__restrict__ ZT, T *__restrict__ nz) {
    const int p = threadIdx.x;
    T v = 0;
    if (p < c) {
        for (int64_t e = zr[p0 + p]; e < zr[p0 + p + 1]; ++e) {
            const T x = zv[e];
            ZT[(int64_t) zc[e] * 64 + p] = x;
            v = fma(x, x, v);
        }
    }
    nz[p] = v;
}

// out[p] = bias + alpha_m k(x_m, z_p) + sum_b partial[b][p] (block order); one workgroup per point
template <typename T>
__global__ __launch_bounds__(256) void predict_csr_final_kernel(kfun<T> kf, const T *__restrict__ partial, int64_t nblk,
                                                                const T *__restrict__ ZT, const T *__restrict__ nzv,
                                                                int64_t d, const T *__restrict__ xlast, T nlast,
                                                                const T *__restrict__ alpha, int64_t m, T bias,
                                                                int64_t np, T *__restrict__ out) {
    __shared__ T red[4];
    const int p = blockIdx.x;
    T dl = 0;
    for (int64_t k = threadIdx.x; k < d; k += 256) dl = fma(xlast[k], ZT[k * 64 + p], dl);
    dl = block_sum256(dl, red);
    if (threadIdx.x == 0) {
        T s = 0;
        for (int64_t b = 0; b < nblk; ++b) s += partial[b * 64 + p];
        if (p < np) out[p] = (s + alpha[m] * kval(kf, dl, nlast, nzv[p])) + bias;
    }
}

// w[f] = sum_{t in column f} cval[t] alpha[crow[t]] (CSC of rows 0..m-1), one wave per column
template <typename T>
__global__ __launch_bounds__(256) void csc_w_kernel(const int64_t *__restrict__ colptr, const int32_t *__restrict__ crow,
                                                    const T *__restrict__ cval, const T *__restrict__ alpha, int64_t d,
                                                    T *__restrict__ w) {
    const int64_t f = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (f >= d) return;
    T s = 0;
    for (int64_t t = colptr[f] + lane; t < colptr[f + 1]; t += 64) s = fma(cval[t], alpha[crow[t]], s);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) w[f] = s;
}

// w[k] += a * x[k]
template <typename T>
__global__ __launch_bounds__(256) void axpy_host_scalar_kernel(T a, const T *__restrict__ x, int64_t n,
                                                               T *__restrict__ w) {
    const int64_t k = (int64_t) blockIdx.x * 256 + threadIdx.x;
    if (k < n) w[k] = fma(a, x[k], w[k]);
}

template <typename T>
rocblas_status gemm_nn(rocblas_handle h, int64_t M, int64_t N, int64_t K, const T *A, int64_t lda, const T *B,
                       int64_t ldb, T *C, int64_t ldc) {
    const T one = 1, zero = 0;
    if constexpr (sizeof(T) == 8)
        return rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int) M, (rocblas_int) N,
                             (rocblas_int) K, &one, A, (rocblas_int) lda, B, (rocblas_int) ldb, &zero, C,
                             (rocblas_int) ldc);
    else
        return rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int) M, (rocblas_int) N,
                             (rocblas_int) K, &one, A, (rocblas_int) lda, B, (rocblas_int) ldb, &zero, C,
                             (rocblas_int) ldc);
}

}  // namespace

// gpu_csvm::update_w (src/plssvm/backends/gpu_csvm.cpp:327-350): w = sum_i alpha_i x_i over all n points
template <typename T>
void engine<T>::update_w_device(const T *alpha_dev) {
    need_data();
    if (sparse) {
        if (factored()) {
            // SELL CSC pass over rows [csc_r0, csc_r1) (this rank's rows in a real group -> all-reduce)
            launch_panel_spmv<T>(csr.spmv_csc, alpha_dev + csr.csc_r0, csr.csc_r1 - csr.csc_r0, w.get(), nullptr, stream);
            if (csr.csc_r0 != 0 || csr.csc_r1 != m) allreduce(w.get(), d);
        } else if (d > 0) {
            hipLaunchKernelGGL(csc_w_kernel<T>, dim3((unsigned) ceil_div(d, 4)), dim3(256), 0, stream, csr.colptr.get(),
                               csr.crow.get(), csr.cval.get(), alpha_dev, d, w.get());
            MI_LAUNCH_CHECK();
        }
    } else {
        launch_gemv_t<T>(XT.get(), n_pad, d, 0, m, alpha_dev, w.get(), nullptr, stream);
    }
    // + alpha_m x_m (the last point is stored densely)
    std::vector<T> am(1);
    MI_HIP_CHECK(hipMemcpyAsync(am.data(), alpha_dev + m, sizeof(T), hipMemcpyDeviceToHost, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    if (d > 0)
        hipLaunchKernelGGL(axpy_host_scalar_kernel<T>, dim3((unsigned) ceil_div(d, 256)), dim3(256), 0, stream, am[0],
                           xlast.get(), d, w.get());
    MI_LAUNCH_CHECK();
}

template <typename T>
void engine<T>::update_w(const T *alpha_host, T *w_host) {
    need_data();
    if (alpha_host == nullptr) throw mi_error(-1, "No alphas provided for prediction!");
    MI_HIP_CHECK(hipSetDevice(device));
    dev_buf<T> a;
    a.alloc(std::max<int64_t>(n_pad, n), stream);
    MI_HIP_CHECK(hipMemcpyAsync(a.get(), alpha_host, sizeof(T) * (size_t) n, hipMemcpyHostToDevice, stream));
    update_w_device(a.get());
    if (w_host && d > 0) MI_HIP_CHECK(hipMemcpyAsync(w_host, w.get(), sizeof(T) * (size_t) d, hipMemcpyDeviceToHost, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
}

// gpu_csvm::predict (src/plssvm/backends/gpu_csvm.cpp:52-120). Points: dense row-major Z[np][dz] or
// CSR (zrowptr, zcol, zval in zfmt); out[np] host.
template <typename T>
void engine<T>::predict(const T *alpha_host, T bias, const T *Z, const int64_t *zrowptr, const int32_t *zcol,
                        const void *zval, int zfmt, int64_t np, int64_t dz, T *out) {
    need_data();
    if (np == 0) return;  // "return empty vector if there are no points to predict"
    if (np < 0 || (Z == nullptr && (zrowptr == nullptr || zcol == nullptr))) throw mi_error(-1, "no points to predict");
    if (dz != d)
        throw mi_error(-1, "Number of features per data point (" + std::to_string(d) +
                               ") must match the number of features per predict point (" + std::to_string(dz) + ")!");
    if (alpha_host == nullptr) throw mi_error(-1, "No alphas provided for prediction!");
    if (out == nullptr) throw mi_error(-1, "no output buffer");
    if (Z == nullptr && zfmt != PLSSVM_MI_VAL_REAL && zfmt != PLSSVM_MI_VAL_FP22) throw mi_error(-1, "unknown value format");
    if (Z == nullptr && zfmt == PLSSVM_MI_VAL_FP22 && sizeof(T) != 4) throw mi_error(-5, "FP22 values need a float context");
    MI_HIP_CHECK(hipSetDevice(device));
    dev_buf<T> a;
    a.alloc(std::max<int64_t>(n_pad, n), stream);
    MI_HIP_CHECK(hipMemcpyAsync(a.get(), alpha_host, sizeof(T) * (size_t) n, hipMemcpyHostToDevice, stream));
    // host densification of point p into dst (row-major, stride 1) — CSR input
    auto zget = [&](int64_t p, T *dst, int64_t stride) {
        if (Z) {
            for (int64_t k = 0; k < d; ++k) dst[k * stride] = Z[p * d + k];
            return;
        }
        for (int64_t k = 0; k < d; ++k) dst[k * stride] = T(0);
        for (int64_t e = zrowptr[p]; e < zrowptr[p + 1]; ++e) {
            if (zcol[e] < 0 || zcol[e] >= d) throw mi_error(-1, "CSR column index out of range");
            dst[(int64_t) zcol[e] * stride] =
                zfmt == PLSSVM_MI_VAL_FP22 ? (T) fp22_get(static_cast<const uint32_t *>(zval), e) : static_cast<const T *>(zval)[e];
        }
    };
    T nlast = 0;
    for (int64_t k = 0; k < d; ++k) nlast = std::fma(xlast_h[k], xlast_h[k], nlast);

    if (kernel == 0) {  // w . z + bias
        update_w_device(a.get());
        const int64_t pc = std::max<int64_t>(1, std::min<int64_t>(np, (int64_t) (256 << 20) / (int64_t) (sizeof(T) * std::max<int64_t>(d, 1))));
        std::vector<T> zh((size_t) (pc * d));
        dev_buf<T> zd, od;
        zd.alloc(pc * d, stream, false);
        od.alloc(pc, stream, false);
        for (int64_t p0 = 0; p0 < np; p0 += pc) {
            const int64_t c = std::min(pc, np - p0);
            for (int64_t p = 0; p < c; ++p) zget(p0 + p, zh.data() + p * d, 1);
            MI_HIP_CHECK(hipMemcpyAsync(zd.get(), zh.data(), sizeof(T) * (size_t) (c * d), hipMemcpyHostToDevice, stream));
            hipLaunchKernelGGL(predict_linear_kernel<T>, dim3((unsigned) c), dim3(256), 0, stream, w.get(), zd.get(), d, bias,
                               od.get());
            MI_LAUNCH_CHECK();
            MI_HIP_CHECK(hipMemcpyAsync(out + p0, od.get(), sizeof(T) * (size_t) c, hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
        }
        return;
    }

    if (!sparse) {
        // G = X_m Z^T on rocBLAS (column-major views: XT is (n_pad x d) with ld n_pad, a row-major
        // chunk of points is (d x c) with ld d), then the kernel-function / alpha epilogue
        if (blas == nullptr) MI_BLAS_CHECK(rocblas_create_handle(&blas));
        MI_BLAS_CHECK(rocblas_set_stream(blas, stream));
        const int64_t ldg = std::max<int64_t>(m, 1);
        const int64_t budget = (int64_t) 512 << 20;
        const int64_t pc = std::max<int64_t>(1, std::min<int64_t>(np, budget / (int64_t) (sizeof(T) * (ldg + d))));
        std::vector<T> zh((size_t) (pc * d));
        dev_buf<T> zd, gd, od;
        zd.alloc(pc * d, stream, false);
        gd.alloc(ldg * pc, stream, false);
        od.alloc(pc, stream, false);
        for (int64_t p0 = 0; p0 < np; p0 += pc) {
            const int64_t c = std::min(pc, np - p0);
            for (int64_t p = 0; p < c; ++p) zget(p0 + p, zh.data() + p * d, 1);
            MI_HIP_CHECK(hipMemcpyAsync(zd.get(), zh.data(), sizeof(T) * (size_t) (c * d), hipMemcpyHostToDevice, stream));
            if (m > 0) MI_BLAS_CHECK(gemm_nn<T>(blas, m, c, d, XT.get(), n_pad, zd.get(), d, gd.get(), ldg));
            hipLaunchKernelGGL(predict_dense_epilogue_kernel<T>, dim3((unsigned) c), dim3(256), 0, stream, kf(), gd.get(),
                               ldg, m, kernel == 2 ? norms.get() : nullptr, a.get(), zd.get(), d, xlast.get(), nlast,
                               bias, od.get());
            MI_LAUNCH_CHECK();
            MI_HIP_CHECK(hipMemcpyAsync(out + p0, od.get(), sizeof(T) * (size_t) c, hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
        }
        return;
    }

    // sparse data: the points as one device CSR (host: nonzeros in column order, FP22 decoded, range
    // checked), then per 64 points the feature-major ZT[d][64] is scattered on the device
    std::vector<int64_t> zr((size_t) np + 1, 0);
    std::vector<int32_t> zc;
    std::vector<T> zv;
    for (int64_t p = 0; p < np; ++p) {
        if (Z) {
            for (int64_t k = 0; k < d; ++k)
                if (Z[p * d + k] != T(0)) zc.push_back((int32_t) k), zv.push_back(Z[p * d + k]);
        } else {
            for (int64_t e = zrowptr[p]; e < zrowptr[p + 1]; ++e) {
                if (zcol[e] < 0 || zcol[e] >= d) throw mi_error(-1, "CSR column index out of range");
                zc.push_back(zcol[e]);
                zv.push_back(zfmt == PLSSVM_MI_VAL_FP22 ? (T) fp22_get(static_cast<const uint32_t *>(zval), e)
                                                        : static_cast<const T *>(zval)[e]);
            }
        }
        zr[(size_t) p + 1] = (int64_t) zc.size();
    }
    const int64_t znnz = (int64_t) zc.size();
    // columns ascending per point (the expansion's merge), and the points' magnitudes
    int64_t max_nnz_z = 0;
    double zabs_max = 0.0, znorm_max = 0.0;
    {
        std::vector<std::pair<int32_t, T>> tmp;
        for (int64_t p = 0; p < np; ++p) {
            const int64_t a0 = zr[(size_t) p], a1 = zr[(size_t) p + 1];
            max_nnz_z = std::max(max_nnz_z, a1 - a0);
            bool sorted = true;
            double nrm = 0.0;
            for (int64_t e = a0; e < a1; ++e) {
                if (e > a0 && zc[(size_t) e] <= zc[(size_t) e - 1]) sorted = false;
                zabs_max = std::max(zabs_max, std::fabs((double) zv[(size_t) e]));
                nrm += (double) zv[(size_t) e] * (double) zv[(size_t) e];
            }
            znorm_max = std::max(znorm_max, nrm);
            if (!sorted) {
                tmp.clear();
                for (int64_t e = a0; e < a1; ++e) tmp.emplace_back(zc[(size_t) e], zv[(size_t) e]);
                std::stable_sort(tmp.begin(), tmp.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
                for (int64_t e = a0; e < a1; ++e) zc[(size_t) e] = tmp[(size_t) (e - a0)].first, zv[(size_t) e] = tmp[(size_t) (e - a0)].second;
            }
        }
    }
    dev_buf<int64_t> zrd;
    dev_buf<int32_t> zcd;
    dev_buf<T> zvd;
    zrd.alloc(np + 1, stream, false);
    zcd.alloc(std::max<int64_t>(znnz, 1), stream, false);
    zvd.alloc(std::max<int64_t>(znnz, 1), stream, false);
    MI_HIP_CHECK(hipMemcpyAsync(zrd.get(), zr.data(), sizeof(int64_t) * (size_t) (np + 1), hipMemcpyHostToDevice, stream));
    if (znnz > 0) {
        MI_HIP_CHECK(hipMemcpyAsync(zcd.get(), zc.data(), sizeof(int32_t) * (size_t) znnz, hipMemcpyHostToDevice, stream));
        MI_HIP_CHECK(hipMemcpyAsync(zvd.get(), zv.data(), sizeof(T) * (size_t) znnz, hipMemcpyHostToDevice, stream));
    }
    if (kernel != 0 && csr.ex.on) {  // sparse poly / rbf model: through the kernel expansion (expand.hip)
        dev_buf<T> oall;
        oall.alloc(np, stream, false);
        if (expansion_predict(a.get(), alpha_host[m], bias, zrd.get(), zcd.get(), zvd.get(), np, max_nnz_z, zabs_max,
                              znorm_max, nlast, oall.get())) {
            MI_HIP_CHECK(hipMemcpyAsync(out, oall.get(), sizeof(T) * (size_t) np, hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            return;
        }
    }
    const int64_t nblk = std::max<int64_t>(1, ceil_div(m, PRED_ROWS));
    dev_buf<T> ztd, nzd, pd, od;
    ztd.alloc(d * 64, stream, false);
    nzd.alloc(64, stream, false);
    pd.alloc(nblk * 64, stream);
    od.alloc(64, stream, false);
    for (int64_t p0 = 0; p0 < np; p0 += 64) {
        const int64_t c = std::min<int64_t>(64, np - p0);
        MI_HIP_CHECK(hipMemsetAsync(ztd.get(), 0, sizeof(T) * (size_t) (d * 64), stream));
        hipLaunchKernelGGL(zt_scatter_kernel<T>, dim3(1), dim3(64), 0, stream, zrd.get(), zcd.get(), zvd.get(), p0, c,
                           ztd.get(), nzd.get());
        MI_LAUNCH_CHECK();
        if (m > 0)
            hipLaunchKernelGGL(predict_csr_kernel<T>, dim3((unsigned) ceil_div(m, PRED_ROWS)), dim3(256), 0, stream, kf(),
                               csr.rowptr.get(), csr.col.get(), csr.val.get(), m, ztd.get(), nzd.get(), norms.get(),
                               a.get(), pd.get());
        MI_LAUNCH_CHECK();
        hipLaunchKernelGGL(predict_csr_final_kernel<T>, dim3(64), dim3(256), 0, stream, kf(), pd.get(),
                           m > 0 ? ceil_div(m, PRED_ROWS) : (int64_t) 0, ztd.get(), nzd.get(), d, xlast.get(), nlast,
                           a.get(), m, bias, c, od.get());
        MI_LAUNCH_CHECK();
        MI_HIP_CHECK(hipMemcpyAsync(out + p0, od.get(), sizeof(T) * (size_t) c, hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
}

#define INST(T)                                                                                                   \
    template void engine<T>::update_w_device(const T *);                                                        \
    template void engine<T>::update_w(const T *, T *);                                                          \
    template void engine<T>::predict(const T *, T, const T *, const int64_t *, const int32_t *, const void *, int, \
                                     int64_t, int64_t, T *);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
