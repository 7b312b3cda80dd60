// Sparse (CSR / CSC / packed-FP22) data paths: setup, q, norms, factored linear K·p and the
// sparse-Gram-pattern K·p for the polynomial and RBF kernels. See DESIGN.md §4.
//
// Math (exact identities, m = n - 1, i, j < m):
//   linear (factored):  sum_j k_ij p_j = x_i . (X_m^T p)                       -> two SpMVs, HBM bound
//   rbf:  k_ij = exp(-g (n_i + n_j - 2 s_ij)),  s_ij = x_i . x_j,  e_i = exp(-g n_i)
//         pairs with no shared feature have s_ij = 0 and k_ij = e_i e_j, so
//         sum_j k_ij p_j = e_i sum_j e_j p_j + (1 - e_i^2) p_i + sum_{j in ov(i)} (k_ij - e_i e_j) p_j
//   poly: k_ij = (g s_ij + c0)^deg, kappa = c0^deg:
//         sum_j k_ij p_j = kappa sum_j p_j + (k_ii - kappa) p_i + sum_{j in ov(i)} (k_ij - kappa) p_j
// where ov(i) = { j != i : rows i and j share a feature }. The pattern ov (lower triangle, j < i)
// with s_ij is built once at setup (sort + reduce-by-key of the column-join incidences); every K·p
// re-evaluates the kernel function on each stored pair (the kernel matrix is never stored).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <numeric>

#include "../../include/plssvm_mi355x.h"
#include "engine.hpp"

namespace plssvm_mi {

namespace {

// ---- norms / e / q ----------------------------------------------------------------------------------
// 16 lanes per row, 16 rows per 256-thread block
template <typename T>
__global__ __launch_bounds__(256) void csr_norms_kernel(const int64_t *__restrict__ rowptr, vals_t<T> val, int64_t m,
                                                        T gamma, T *__restrict__ norms, T *__restrict__ e) {
    const int64_t row = (int64_t) blockIdx.x * 16 + (threadIdx.x >> 4);
    const int sl = threadIdx.x & 15;
    if (row >= m) return;
    // sequential fma chain in column order (== the dense chain: zeros add nothing) — lane 0 walks the row
    if (sl == 0) {
        T v = 0;
        for (int64_t k = rowptr[row]; k < rowptr[row + 1]; ++k) {
            const T x = val[k];
            v = fma(x, x, v);
        }
        norms[row] = v;
        if (e) e[row] = exp(-gamma * v);
    }
}

// q_i = k(x_i, x_last) with x_last dense; dot/dist via the row's non-zeros
template <typename T>
__global__ __launch_bounds__(256) void csr_q_kernel(kfun<T> kf, const int64_t *__restrict__ rowptr,
                                                    const int32_t *__restrict__ col, vals_t<T> val, int64_t m,
                                                    const T *__restrict__ xlast, T nlast, const T *__restrict__ norms,
                                                    T *__restrict__ q) {
    const int64_t row = (int64_t) blockIdx.x * 16 + (threadIdx.x >> 4);
    const int sl = threadIdx.x & 15;
    if (row >= m) return;
    T dot = 0;
    if (sl == 0) {
        for (int64_t k = rowptr[row]; k < rowptr[row + 1]; ++k) dot = fma(val[k], xlast[col[k]], dot);
        T out;
        if (kf.kernel == 0) {
            out = dot;
        } else if (kf.kernel == 1) {
            const T base = fma(kf.gamma, dot, kf.coef0);
            out = T(1);
            for (int e = 0; e < kf.degree; ++e) out *= base;
        } else {
            T dist = norms[row] + nlast - T(2) * dot;
            dist = dist > T(0) ? dist : T(0);
            out = exp(-kf.gamma * dist);
        }
        q[row] = out;
    }
}

// ---- CSC on the device (rows 0..m-1): a stable radix sort of the entries by column keeps the rows ascending
// inside every column — the host counting sort's CSC (csc_host below), bit for bit ------------------------
// entry k's row, and k itself (the sort's payload); one wave per row
__global__ __launch_bounds__(256) void csc_rowid_kernel(const int64_t *__restrict__ rowptr, int64_t m,
                                                        int32_t *__restrict__ rowid, int32_t *__restrict__ kid) {
    const int64_t i = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= m) return;
    for (int64_t k = rowptr[i] + (threadIdx.x & 63); k < rowptr[i + 1]; k += 64) {
        rowid[k] = (int32_t) i;
        kid[k] = (int32_t) k;
    }
}

// colptr[f] = #entries of a column < f, from the sorted columns: the first entry q of a column >= f writes
// it (each f exactly once: q = nnz takes the empty columns after the last entry's)
__global__ __launch_bounds__(256) void csc_colptr_kernel(const uint32_t *__restrict__ skey, int64_t nnz, int64_t d,
                                                         int64_t *__restrict__ colptr) {
    const int64_t q = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (q > nnz) return;
    const int64_t lo = q == 0 ? 0 : (int64_t) skey[q - 1] + 1, hi = q == nnz ? d : (int64_t) skey[q];
    for (int64_t f = lo; f <= hi; ++f) colptr[f] = q;
}

// CSC slot q holds entry k = sk[q]: its row, its (decoded) value; cpos[k] = q
template <typename T>
__global__ __launch_bounds__(256) void csc_gather_kernel(const int32_t *__restrict__ sk, const int32_t *__restrict__ rowid,
                                                         const T *__restrict__ val, int64_t nnz, int32_t *__restrict__ crow,
                                                         T *__restrict__ cval, int64_t *__restrict__ cpos) {
    const int64_t q = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nnz) return;
    const int32_t k = sk[q];
    crow[q] = rowid[k];
    cval[q] = val[k];
    cpos[k] = q;
}

// packed FP22 words -> the context's real type (fp22_get: the host decoding, bit for bit)
template <typename T>
__global__ __launch_bounds__(256) void fp22_unpack_kernel(const uint32_t *__restrict__ words, int64_t n, T *__restrict__ out) {
    const int64_t k = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) out[k] = (T) fp22_get(words, k);
}

// max_k x_k^2 and max_i sum_{k in row i} x_k^2 (double; each row's sum in entry order, separate multiply and add as
// on the host), as the bits of non-negative doubles (ordered like the values): mx[0], mx[1]
template <typename T>
__global__ __launch_bounds__(256) void csr_maxsq_kernel(const int64_t *__restrict__ rowptr, const T *__restrict__ val,
                                                        int64_t m, unsigned long long *__restrict__ mx) {
#pragma clang fp contract(off)
    __shared__ double red[2][4];
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    double am = 0.0, nrm = 0.0;
    if (i < m)
        for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
            const double x = (double) val[k];
            const double x2 = x * x;
            am = fmax(am, x2);
            nrm = nrm + x2;
        }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        am = fmax(am, __shfl_xor(am, o));
        nrm = fmax(nrm, __shfl_xor(nrm, o));
    }
    if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = am, red[1][threadIdx.x >> 6] = nrm;
    __syncthreads();
    if (threadIdx.x < 2) {
        double v = red[threadIdx.x][0];
        for (int w = 1; w < 4; ++w) v = fmax(v, red[threadIdx.x][w]);
        if (v > 0.0) atomicMax(mx + threadIdx.x, (unsigned long long) __double_as_longlong(v));
    }
}

// incidences of each block of rb rows: sum over its entries of #{ earlier rows in the entry's column }
// (integers: exact in any order)
__global__ __launch_bounds__(256) void csc_inc_rb_kernel(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
                                                         const int64_t *__restrict__ cpos, const int64_t *__restrict__ colptr,
                                                         int64_t m, int64_t rb, int64_t *__restrict__ inc_rb) {
    __shared__ long long part[4];
    const int64_t I = blockIdx.x;
    const int64_t k0 = rowptr[I * rb], k1 = rowptr[min(m, (I + 1) * rb)];
    long long a = 0;
    for (int64_t k = k0 + threadIdx.x; k < k1; k += 256) a += (long long) (cpos[k] - colptr[col[k]]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) inc_rb[I] = (int64_t) (part[0] + part[1] + part[2] + part[3]);
}

// ---- Gram pattern build ---------------------------------------------------------------------------------
// incidences of row i: sum over its entries e of #{ j < i in column col[e] } = cpos[e] - colptr[col[e]]
__global__ __launch_bounds__(256) void gram_count_kernel(const int64_t *__restrict__ rowptr,
                                                         const int32_t *__restrict__ col,
                                                         const int64_t *__restrict__ cpos,
                                                         const int64_t *__restrict__ colptr, int64_t i0, int64_t i1,
                                                         int64_t *__restrict__ cnt) {
    const int64_t i = i0 + (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= i1) return;
    int64_t c = 0;
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) c += cpos[k] - colptr[col[k]];
    cnt[i - i0] = c;
}

// one workgroup per row: key = (W << 32) | (i_local << 16) | (j - W*CW), val = x_if x_jf
template <typename T>
__global__ __launch_bounds__(256) void gram_gen_kernel(const int64_t *__restrict__ rowptr,
                                                       const int32_t *__restrict__ col, vals_t<T> val,
                                                       const int64_t *__restrict__ cpos,
                                                       const int64_t *__restrict__ colptr,
                                                       const int32_t *__restrict__ crow, vals_t<T> cval, int64_t i0,
                                                       const int64_t *__restrict__ off, uint64_t *__restrict__ keys,
                                                       T *__restrict__ vals) {
    const int64_t i = i0 + blockIdx.x;
    const uint64_t il = (uint64_t) blockIdx.x;
    int64_t out = off[blockIdx.x];
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const int64_t c0 = colptr[col[k]], c1 = cpos[k];
        const T xi = val[k];
        for (int64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) {
            const uint64_t j = (uint64_t) crow[t];
            constexpr uint64_t CW = GRAM_CW;
            keys[out + (t - c0)] = ((j / CW) << 32) | (il << 16) | (j % CW);
            vals[out + (t - c0)] = xi * cval[t];
        }
        out += c1 - c0;
    }
}

// pairs per group g = (window, row): the unique keys are sorted by group, so each group is one run;
// its first key writes gstart[g], its last writes rowcnt[g] = end (exclusive), no atomics (a hot
// counter per row serialised the former atomicAdd version: 3.3 ms per row block)
__device__ __forceinline__ int64_t gram_group(uint64_t k) {
    return (int64_t) (k >> 32) * GRAM_RB + (int64_t) ((k >> 16) & 0xFFFF);
}

__global__ __launch_bounds__(256) void gram_rowcount_kernel(const uint64_t *__restrict__ ukeys,
                                                            const int64_t *__restrict__ nruns,
                                                            int32_t *__restrict__ rowcnt, int32_t *__restrict__ gstart) {
    const int64_t u = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nu = *nruns;
    if (u >= nu) return;
    const int64_t g = gram_group(ukeys[u]);
    if (u == 0 || gram_group(ukeys[u - 1]) != g) gstart[g] = (int32_t) u;
    if (u == nu - 1 || gram_group(ukeys[u + 1]) != g) rowcnt[g] = (int32_t) (u + 1);
}

// rowcnt[g] = end - start for the groups written above, 0 elsewhere
__global__ __launch_bounds__(256) void gram_runlen_kernel(int32_t *__restrict__ rowcnt,
                                                          const int32_t *__restrict__ gstart, int64_t n) {
    const int64_t g = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (g < n && rowcnt[g] > 0) rowcnt[g] -= gstart[g];
}

// pads of the pattern: s = 0 (contributes exactly 0) and j = (chunk index mod 64), so the pads that the
// lanes of one wave-instruction meet hit 64 distinct LDS column accumulators (with j = 0 for every pad
// their zero-valued ds_add_u64 all went to one address and serialised)
__global__ __launch_bounds__(256) void gram_pad_index_kernel(uint16_t *__restrict__ pj, int64_t n) {
    const int64_t x = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (x < n) pj[x] = (uint16_t) ((x >> 3) & 63);
}

// rows are padded to a multiple of 8 pairs per cell (pads: s = 0, spread j), so an 8-pair chunk never
// spans two rows; pair u of group g = (W, row) goes to padded[g] + (u - uoff[g])
__global__ __launch_bounds__(256) void gram_pad_kernel(const int32_t *__restrict__ cnt, int64_t n,
                                                       int32_t *__restrict__ cnt8) {
    const int64_t g = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (g < n) cnt8[g] = (cnt[g] + 7) & ~7;
}

template <typename T>
__global__ __launch_bounds__(256) void gram_store_kernel(const uint64_t *__restrict__ ukeys,
                                                         const T *__restrict__ usum, const int64_t *__restrict__ nruns,
                                                         const int32_t *__restrict__ uoff,
                                                         const int32_t *__restrict__ padded, uint16_t *__restrict__ pj,
                                                         T *__restrict__ ps) {
    const int64_t u = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= *nruns) return;
    const uint64_t k = ukeys[u];
    const int64_t g = gram_group(k);
    const int64_t dst = (int64_t) padded[g] + (u - (int64_t) uoff[g]);
    pj[dst] = (uint16_t) (k & 0xFFFF);
    ps[dst] = usum[u];
}

// ---- Gram K·p ---------------------------------------------------------------------------------------------
__host__ __device__ inline int64_t gram_nw(int64_t I, int64_t m, int64_t cw) {
    const int64_t hi = m < (I + 1) * GRAM_RB ? m : (I + 1) * GRAM_RB;  // rows of block I are < hi, so j < hi
    return (hi + cw - 1) / cw;
}

template <typename T>
__device__ __forceinline__ void load8(const T *__restrict__ ps, int64_t e0, T (&s)[8]) {
    if constexpr (sizeof(T) == 4) {
        const float4 a = *reinterpret_cast<const float4 *>(ps + e0), b = *reinterpret_cast<const float4 *>(ps + e0 + 4);
        s[0] = a.x, s[1] = a.y, s[2] = a.z, s[3] = a.w, s[4] = b.x, s[5] = b.y, s[6] = b.z, s[7] = b.w;
    } else {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const double2 v = *reinterpret_cast<const double2 *>(ps + e0 + 2 * h);
            s[2 * h] = v.x, s[2 * h + 1] = v.y;
        }
    }
}

// One 512-thread workgroup per cell (2048 rows x 4096-row window), two resident per CU so one
// cell's prologue/epilogue overlaps another's stream. The cell's pairs are one
// contiguous, row-sorted stream cut into 8-pair chunks; each wave walks a contiguous range of
// chunks (64 per step, lane = chunk), so a lane's row only moves forward and is tracked
// incrementally. Per step and lane: 16 B of j + 32/64 B of s (prefetched one step ahead), the
// window's per-point factors from LDS, mirrored column sums into an LDS accumulator, row partials
// reduced across lanes by a segmented shuffle scan and added by segment heads.
//
// KERNEL: 0 linear, 1 poly, 2 rbf (c_ij = exp(-g max(0, n_i + n_j - 2 s)) - e_i e_j), 3 rbf factored:
// c_ij = e_i e_j (exp(2 g s) - 1), so the row sum is e_i sum_j g_ij (e_j p_j) and the column sum
// e_j sum_i g_ij (e_i p_i): one staged factor (e_j p_j) per window point and no per-pair norm. Used
// when g max(n) keeps e_i and exp(2 g s) inside the floating-point range (checked at setup).
//
// Both LDS accumulators are int64 fixed point (ds_add_u64): LDS float atomics serialise on gfx950
// (measured ~190 cycles per wave-wide ds_add_f32 vs ~10 for ds_add_u64), and integer sums are exact
// and order-independent, so the kernel is bitwise reproducible. The quantum is a per-cell power of
// two q = 2^e with (bound on |term|) < 2^(e+50) — from the cell's max |s| (setup) and the max |p|
// (or |e p|) over its rows and window — so a sum of up to 4096 terms stays below 2^62 and each term
// is rounded to 2^-51 of the cell's largest possible term. A single term is rounded with the
// 1.5*2^52 magic add in fp64 (exact for |x| < 2^51); row partials use the full fp64->int64 convert.
template <typename T>
__device__ __forceinline__ T fast_exp2(T x) {
    if constexpr (sizeof(T) == 4) return __builtin_amdgcn_exp2f(x);  // v_exp_f32
    else return exp2(x);
}

// e^y - 1 without the cancellation of exp(y) - 1 near 0 (the factored rbf pair form evaluates it at
// y = 2 g s_ij, about 1e-5 on the BASELINE sets, where exp(y) - 1 in fp32 keeps only ~2 digits).
// fp32: degree-7 Taylor polynomial for |y| < 1/4 (truncation < 2e-9 relative), v_exp_f32 - 1 above
// (relative error < 1e-6 there); both evaluated and selected, no branch. fp64: the device libm expm1.
template <typename T>
__device__ __forceinline__ T expm1_acc(T y) {
    if constexpr (sizeof(T) == 4) {
        float t = fmaf(y, 1.0f / 5040.0f, 1.0f / 720.0f);
        t = fmaf(y, t, 1.0f / 120.0f);
        t = fmaf(y, t, 1.0f / 24.0f);
        t = fmaf(y, t, 1.0f / 6.0f);
        t = fmaf(y, t, 0.5f);
        t = fmaf(y, t, 1.0f);
        const float small = y * t;
        const float big = __builtin_amdgcn_exp2f(y * 1.4426950408889634f) - 1.0f;
        return fabsf(y) < 0.25f ? small : big;
    } else {
        return expm1(y);
    }
}

// e^y - 1 for |y| < expm1_small_bound<T>(): Taylor polynomial of degree 3 (fp32) / 5 (fp64), relative
// truncation error < 2^-26 / 2^-55 — cheaper than one v_exp_f32 and exact to rounding, used when the
// setup's bound 2 g max|s_ij| is below it (every cell of the BASELINE sparse sets: 2 g |s| < 1e-4)
template <typename T>
constexpr double expm1_small_bound() { return sizeof(T) == 4 ? 0.007 : 0.0017; }

template <typename T>
__device__ __forceinline__ T expm1_small(T y) {
    if constexpr (sizeof(T) == 4) {
        return y * fmaf(y, fmaf(y, 1.0f / 6.0f, 0.5f), 1.0f);
    } else {
        double t = fma(y, 1.0 / 120.0, 1.0 / 24.0);
        t = fma(y, t, 1.0 / 6.0);
        t = fma(y, t, 0.5);
        return y * fma(y, t, 1.0);
    }
}

__device__ __forceinline__ unsigned long long fx_round(double x) {
    return (unsigned long long) (__double_as_longlong(x + 6755399441055744.0) - 0x4338000000000000LL);
}

// Workgroup size: 512 threads (two workgroups per CU) when the cell's LDS fits twice in a CU
// (fp32 linear / poly / factored rbf: 72 KB); otherwise one workgroup per CU of 1024 threads, so a CU
// still streams with 16 waves (fp64: window factors 32 KB; direct rbf: norms and e of the window too).
template <typename T, int KERNEL>
constexpr int gram_wg() { return sizeof(T) == 8 || KERNEL == 2 ? 1024 : GRAM_WG; }

template <typename T, int KERNEL, int ABL>
__global__ __launch_bounds__((gram_wg<T, KERNEL>())) void gram_kp_kernel(const gram_cell *__restrict__ cells,
                                                       const int64_t *__restrict__ rb_base,
                                                       const int32_t *__restrict__ rowoff,
                                                       const uint16_t *__restrict__ pj, const T *__restrict__ ps,
                                                       const T *__restrict__ norms, const T *__restrict__ ev,
                                                       const T *__restrict__ p, T *__restrict__ slab_row,
                                                       T *__restrict__ slab_col, int64_t m, int64_t m_pad, kfun<T> kf,
                                                       T kappa, const cg_scalars<T> *__restrict__ status) {
    constexpr int NT = gram_wg<T, KERNEL>();
    constexpr int CW = GRAM_CW, NWAVE = NT / 64;
    constexpr bool NEED_N = KERNEL == 2, NEED_E = KERNEL == 2;
    constexpr bool FACT = KERNEL == 3 || KERNEL == 4;  // factored rbf: c_ij = e_i e_j expm1(2 g s_ij)
    using acc_t = unsigned long long;
    __shared__ T wn[NEED_N ? CW : 1], we[NEED_E ? CW : 1], wp[CW];
    __shared__ acc_t colacc[CW];
    __shared__ acc_t rowacc[GRAM_RB];
    __shared__ int32_t ro[GRAM_RB + 1];
    __shared__ T wmax[NWAVE];
    if (status != nullptr && status->converged) return;
    const gram_cell cell = cells[xcd_remap(blockIdx.x, gridDim.x)];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t I0 = (int64_t) cell.I * GRAM_RB, W0 = (int64_t) cell.W * CW;
    const int rows = (int) min<int64_t>(GRAM_RB, m - I0);
    const int wlen = (int) min<int64_t>(CW, m - W0);
    const T gamma = kf.gamma;
    T pmax = 0;
    for (int t = tid; t < CW; t += NT) {
        const bool ok = t < wlen;
        if (NEED_N) wn[t] = ok ? norms[W0 + t] : T(0);
        if (NEED_E) we[t] = ok ? ev[W0 + t] : T(0);
        const T pv = ok ? (FACT ? ev[W0 + t] * p[W0 + t] : p[W0 + t]) : T(0);
        wp[t] = pv;
        pmax = max(pmax, fabs(pv));
        colacc[t] = 0;
    }
    for (int t = tid; t < GRAM_RB; t += NT) {
        rowacc[t] = 0;
        if (t < rows) pmax = max(pmax, fabs(FACT ? ev[I0 + t] * p[I0 + t] : p[I0 + t]));
    }
    for (int t = tid; t <= rows; t += NT) ro[t] = rowoff[cell.rowoff + t];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) pmax = max(pmax, __shfl_xor(pmax, o));
    if (lane == 0) wmax[wave] = pmax;
    __syncthreads();
    pmax = wmax[0];
#pragma unroll
    for (int w = 1; w < NWAVE; ++w) pmax = max(pmax, wmax[w]);
    // bound on |c| (|g| for the factored rbf) over the cell's pairs
    double cb;
    if (FACT) {
        cb = expm1(2.0 * fabs((double) gamma) * cell.smax);
    } else if (KERNEL == 2) {
        cb = 1.0;
    } else if (KERNEL == 1) {
        const double bse = fabs((double) gamma) * cell.smax + fabs((double) kf.coef0);
        double a = 1.0, b = 1.0;
        for (int q = 0; q < kf.degree; ++q) a *= bse, b *= fabs((double) kf.coef0);
        cb = a + b;
    } else {
        cb = cell.smax;
    }
    // quantum 2^qe, clamped to the smallest normal of T (terms below it are denormal anyway)
    constexpr int emin = sizeof(T) == 8 ? -1022 : -126;
    const double bound = cb * (double) pmax * 1.0000001;
    const int qe = bound > 0.0 && isfinite(bound) ? max(emin, ilogb(bound) + 1 - 50) : emin;
    const double inv_q = ldexp(1.0, -qe);
    // one pair's term (|x| < 2^50): magic-add rounding; row partials (up to 512 terms): full conversion
    auto quant = [&](T v) -> acc_t { return fx_round((double) v * inv_q); };
    auto quant_sum = [&](T v) -> acc_t { return (acc_t) __double2ll_rn((double) v * inv_q); };

    const int64_t base = rb_base[cell.I];  // 8-aligned, and every row's pair count is padded to 8
    const int64_t c0 = (base + ro[0]) >> 3, c1 = (base + ro[rows]) >> 3;
    const int64_t per_wave = ((c1 - c0 + NWAVE - 1) / NWAVE + 63) / 64 * 64;
    const int64_t wbeg = c0 + wave * per_wave;
    const int64_t wend = min<int64_t>(c1, wbeg + per_wave);

    // Software pipeline, one step deep: while step k is evaluated, step k+1's pair stream (j, s) AND
    // its lanes' row factors are already in flight. The row seek for step k+1 (LDS only) runs before
    // step k's pairs, and every load is issued unconditionally (indices clamped), so the only vmcnt
    // wait per step is at its end, covering loads that had the whole step to land. (Loading the row
    // factors after the seek of the *same* step forced a vmcnt(0) before every step: the stream
    // prefetch was waited for with them and never overlapped anything.)
    int r = 0;                      // row of the lane's chunk in the step being prefetched
    int64_t rend = base + ro[0];    // end (absolute pair index) of row r
    auto seek = [&](int64_t e) {    // move r forward to the row containing pair e (rend <= e)
        const int32_t rel = (int32_t) (e - base);
        int steps = 0;
        while (steps < 8 && ro[r + 1] <= rel) ++r, ++steps;
        if (ro[r + 1] <= rel) {  // long jump: binary search in [r, rows)
            int lo = r, hi = rows;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (ro[mid] <= rel) lo = mid;
                else hi = mid;
            }
            r = lo;
        }
        rend = base + ro[r + 1];
    };
    // row factors of row r: p (e p for the factored rbf), norm, e — plain loads, consumed one step later
    T pa_n = 0, pb_n = 0, ni_n = 0, ei_n = 0;
    auto load_row = [&]() {
        const int64_t g = I0 + min(r, rows - 1);
        if (FACT) {
            pa_n = ev[g], pb_n = p[g];
        } else {
            pa_n = p[g];
            if (NEED_N) ni_n = norms[g];
            if (NEED_E) ei_n = ev[g];
        }
    };
    // exp(-g dist) = exp2(-g log2(e) dist); exp(2 g s) = exp2(2 g log2(e) s)
    const T lg = gamma * T(1.4426950408889634);
    const T g2 = T(2) * gamma;
    const int64_t clast = wend - 1;  // clamp target for the loads of idle lanes (wend > wbeg when used)

    uint4 jv_n = make_uint4(0, 0, 0, 0);
    T s_n[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s_n[k] = T(0);
    int r_n = 0;
    if (wbeg < wend) {
        const int64_t cf = min<int64_t>(wbeg + lane, clast);
        jv_n = *reinterpret_cast<const uint4 *>(pj + (cf << 3));
        load8<T>(ps, cf << 3, s_n);
        if ((cf << 3) >= rend) seek(cf << 3);
        r_n = r;
        load_row();
    }
    for (int64_t cb = wbeg; cb < wend; cb += 64) {  // wave-uniform trip count
        const bool have = cb + lane < wend;
        // this step's operands (loaded during the previous step)
        const uint4 jv = jv_n;
        T s[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] = s_n[k];
        const int rc = r_n;
        const T pi = FACT ? pa_n * pb_n : pa_n, ni = ni_n, ei = ei_n;
        // issue the next step: stream, seek, row factors
        if (cb + 64 < wend) {  // wave-uniform
            const int64_t cn = cb + 64 + lane;
            const int64_t cl = min<int64_t>(cn, clast);
            jv_n = *reinterpret_cast<const uint4 *>(pj + (cl << 3));
            load8<T>(ps, cl << 3, s_n);
            if (cn < wend && (cn << 3) >= rend) seek(cn << 3);
            r_n = r;
            load_row();
        }
        int rl = -1;  // row of this lane's chunk (for the cross-lane reduction)
        T acc = 0;
        if (have) {
            const uint32_t jw[4] = { jv.x, jv.y, jv.z, jv.w };
            int jl[8];
            T wpj[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                jl[k] = (int) ((jw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
                wpj[k] = wp[jl[k]];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                T cv;
                if (KERNEL == 4) {  // |2 g s| below the small-argument bound of every cell (setup)
                    cv = (ABL & 2) ? lg * s[k] : expm1_small(g2 * s[k]);  // pads: s = 0 -> 0
                } else if (KERNEL == 3) {
                    cv = (ABL & 2) ? lg * s[k] : expm1_acc(g2 * s[k]);  // pads: s = 0 -> 0
                } else if (KERNEL == 2) {
                    T dist = ni + wn[jl[k]] - T(2) * s[k];
                    dist = dist > T(0) ? dist : T(0);
                    cv = (ABL & 2) ? dist - ei * we[jl[k]] : fast_exp2(-lg * dist) - ei * we[jl[k]];
                    cv = s[k] == T(0) ? T(0) : cv;  // pads (and exact-zero pairs, whose c is 0)
                } else if (KERNEL == 1) {
                    const T bse = fma(gamma, s[k], kf.coef0);
                    T kv = T(1);
                    for (int q = 0; q < kf.degree; ++q) kv *= bse;
                    cv = kv - kappa;  // pads: bse = c0 -> kv == kappa bitwise
                } else {
                    cv = s[k];
                }
                acc = fma(cv, wpj[k], acc);
                if (ABL & 1) acc += cv * pi;  // timing-only ablation: no LDS column accumulation
                else atomicAdd(&colacc[jl[k]], quant(cv * pi));
            }
            rl = rc;
        }
        // segmented reduction of (row, partial) across the wave: rows are non-decreasing in lane order
        T sacc = acc;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const T so = __shfl_down(sacc, off);
            const int rr = __shfl_down(rl, off);
            if (lane + off < 64 && rr == rl) sacc += so;
        }
        const int rprev = __shfl_up(rl, 1);
        if (rl >= 0 && (lane == 0 || rprev != rl)) atomicAdd(&rowacc[rl], quant_sum(sacc));
    }
    __syncthreads();
    for (int t = tid; t < rows; t += NT) {
        T v = (T) ldexp((double) (long long) rowacc[t], qe);
        if (FACT) v *= ev[I0 + t];
        slab_row[(int64_t) cell.W * m_pad + I0 + t] = v;
    }
    for (int t = tid; t < wlen; t += NT) {
        T v = (T) ldexp((double) (long long) colacc[t], qe);
        if (FACT) v *= ev[W0 + t];
        slab_col[(int64_t) cell.I * m_pad + W0 + t] = v;
    }
}

// per cell: max |s| over its pairs (the fixed-point bound of the K·p kernel)
template <typename T>
__global__ __launch_bounds__(256) void gram_cell_smax_kernel(gram_cell *__restrict__ cells,
                                                             const int64_t *__restrict__ rb_base,
                                                             const int32_t *__restrict__ rowoff,
                                                             const T *__restrict__ ps, int64_t m) {
    __shared__ T part[4];
    gram_cell &cell = cells[blockIdx.x];
    const int rows = (int) min<int64_t>(GRAM_RB, m - (int64_t) cell.I * GRAM_RB);
    const int64_t base = rb_base[cell.I];
    const int64_t a = base + rowoff[cell.rowoff], b = base + rowoff[cell.rowoff + rows];
    T v = 0;
    for (int64_t k = a + threadIdx.x; k < b; k += 256) v = max(v, fabs(ps[k]));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) cell.smax = (double) max(max(part[0], part[1]), max(part[2], part[3]));
}

template <typename T>
__global__ __launch_bounds__(256) void gram_reduce_kernel(const T *__restrict__ slab_row,
                                                          const T *__restrict__ slab_col, int64_t m, int64_t m_pad,
                                                          int64_t rb0, int64_t rb1, T *__restrict__ raw,
                                                          const cg_scalars<T> *__restrict__ status) {
    constexpr int64_t CW = GRAM_CW;
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t I = i / GRAM_RB, W = i / CW;
    T s = 0;
    if (I >= rb0 && I < rb1) {
        const int64_t nw = gram_nw(I, m, CW);
        for (int64_t w = 0; w < nw; ++w) s += slab_row[w * m_pad + i];
    }
    for (int64_t J = max<int64_t>(rb0, I); J < rb1; ++J) {  // blocks with rows > i may pair with j = i
        if (W < gram_nw(J, m, CW)) s += slab_col[J * m_pad + i];
    }
    raw[i] = s;
}

// raw_i += separable part + diagonal (added once, after the all-reduce)
template <typename T>
__global__ __launch_bounds__(256) void gram_base_kernel(int kernel, kfun<T> kf, T kappa, const T *__restrict__ ssc,
                                                        const T *__restrict__ norms, const T *__restrict__ ev,
                                                        const T *__restrict__ p, int64_t m, T *__restrict__ raw,
                                                        const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const T S = ssc[0];
    T add;
    if (kernel == 2) {
        const T ei = ev[i];
        add = ei * S + (T(1) - ei * ei) * p[i];
    } else if (kernel == 1) {
        const T bse = fma(kf.gamma, norms[i], kf.coef0);
        T kii = T(1);
        for (int q = 0; q < kf.degree; ++q) kii *= bse;
        add = kappa * S + (kii - kappa) * p[i];
    } else {
        add = norms[i] * p[i];
    }
    raw[i] += add;
}

// timing-only ablation switch for profiling the Gram kernel (results are wrong when non-zero):
// PLSSVM_MI_GRAM_ABLATE bit 0 = drop the LDS column accumulation, bit 1 = drop the exp
int gram_ablate() {
    static const int v = [] {
        const char *s = std::getenv("PLSSVM_MI_GRAM_ABLATE");
        return s ? std::atoi(s) : 0;
    }();
    return v;
}

template <typename T>
void host_check_csr(const int64_t *rowptr, const int32_t *col, int64_t n, int64_t d) {
    if (!rowptr || !col || n < 1 || d < 1) throw mi_error(-1, "Data set is empty!");
    if (rowptr[0] != 0) throw mi_error(-1, "CSR rowptr[0] must be 0");
    // the first failure in row order, as a sequential scan would find it: the rows before the first decreasing
    // rowptr are checked on the host threads (each thread's first error is its lowest row's, and host_parallel
    // rethrows the lowest thread's), then the rowptr error itself
    int64_t ibad = n;
    for (int64_t i = 0; i < n; ++i)
        if (rowptr[i + 1] < rowptr[i]) {
            ibad = i;
            break;
        }
    host_parallel(ibad, [&](int, int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i)
            for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
                if (col[k] < 0 || col[k] >= d) throw mi_error(-1, "CSR column index out of range");
                if (k > rowptr[i] && col[k] <= col[k - 1]) throw mi_error(-1, "CSR columns must be strictly ascending");
            }
    });
    if (ibad < n) throw mi_error(-1, "CSR rowptr must be non-decreasing");
}

}  // namespace

// FP22 input: the SELL streams hold the packed values (2.75 B per value; their exact fp32 decoding, 4 B, measured
// equal to 1 % slower on config 5, round 4)
inline bool sell_fp22_stream() { return true; }

// ---- engine members ----------------------------------------------------------------------------------
// the CSC of rows 0..m-1 from the device CSR (0 < nnz < 2^31): entries sorted by column with a stable radix sort
// (rows stay ascending inside a column), colptr from the sorted columns, crow / cval / cpos by a gather
template <typename T>
void engine<T>::csc_device(int64_t nnz, dev_buf<int64_t> &cpos_d) {
    const int n32 = (int) nnz;
    int end_bit = 1;
    while (end_bit < 32 && (int64_t(1) << end_bit) < d) ++end_bit;
    dev_buf<int32_t> rowid, kid, kid_s;
    dev_buf<uint32_t> key_s;
    rowid.alloc(nnz, stream, false);
    kid.alloc(nnz, stream, false);
    kid_s.alloc(nnz, stream, false);
    key_s.alloc(nnz, stream, false);
    hipLaunchKernelGGL(csc_rowid_kernel, dim3((unsigned) ceil_div(m, 4)), dim3(256), 0, stream, csr.rowptr.get(), m,
                       rowid.get(), kid.get());
    MI_LAUNCH_CHECK();
    {  // test hook: the device sort running out of memory after its first temporaries (the host fallback, setup_csr)
        const char *e = std::getenv("PLSSVM_MI_CSC");
        if (e != nullptr && std::strcmp(e, "oom") == 0) throw mi_error(-4, "device CSC: out of memory (test hook)");
    }
    const uint32_t *keys = reinterpret_cast<const uint32_t *>(csr.col.get());  // columns >= 0: the same order unsigned
    size_t tb = 0;
    MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, key_s.get(), kid.get(), kid_s.get(), n32, 0, end_bit,
                                                    stream));
    {
        dev_buf<unsigned char> tmp;
        tmp.alloc((int64_t) std::max<size_t>(tb, 16), stream, false);
        MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.get(), tb, keys, key_s.get(), kid.get(), kid_s.get(), n32, 0,
                                                        end_bit, stream));
        csr.colptr.alloc(d + 1, stream, false);
        hipLaunchKernelGGL(csc_colptr_kernel, dim3((unsigned) ceil_div(nnz + 1, 256)), dim3(256), 0, stream, key_s.get(),
                           nnz, d, csr.colptr.get());
        MI_LAUNCH_CHECK();
        csr.crow.alloc(nnz, stream, false);
        csr.cval.alloc(nnz, stream, false);
        cpos_d.alloc(nnz, stream, false);
        hipLaunchKernelGGL(csc_gather_kernel<T>, dim3((unsigned) ceil_div(nnz, 256)), dim3(256), 0, stream, kid_s.get(),
                           rowid.get(), csr.val.get(), nnz, csr.crow.get(), csr.cval.get(), cpos_d.get());
        MI_LAUNCH_CHECK();
        MI_HIP_CHECK(hipStreamSynchronize(stream));  // the temporaries are freed on return
    }
}

template <typename T>
void engine<T>::setup_csr(const int64_t *rowptr, const int32_t *col, const void *val, int val_fmt, int64_t n_,
                          int64_t d_) {
    phase_timer pt;
    host_check_csr<T>(rowptr, col, n_, d_);
    if (!val && rowptr[n_] > 0) throw mi_error(-1, "CSR values missing");
    if (val_fmt != PLSSVM_MI_VAL_REAL && val_fmt != PLSSVM_MI_VAL_FP22) throw mi_error(-1, "unknown value format");
    if (val_fmt == PLSSVM_MI_VAL_FP22 && sizeof(T) != 4) throw mi_error(-5, "FP22 values need a float context");
    // HIP loads expand.hip's code object (11 MB of device code) at the first launch of one of its kernels, ~0.1 s into
    // the expansion's build on the critical path of a process's first sparse setup: for the kernels that can use the
    // expansion (poly, rbf) a host thread loads it now, once per process, beside the uploads and the CSC sort
    // (sparse.hip kernels); it is joined before the expansion is built (and at the latest when setup_csr returns)
    struct loader_t {
        std::thread t;
        void join() {
            if (t.joinable()) t.join();
        }
        ~loader_t() { join(); }
    } exp_loader;
    {
        static std::atomic<bool> loaded{ false };
        if ((kernel == 1 || kernel == 2) && n_ > 1 && rowptr[n_ - 1] > 0 && !loaded.exchange(true)) {
            try {
                const int dev = device;
                exp_loader.t = std::thread([dev] {
                    if (hipSetDevice(dev) == hipSuccess) exp_load_code_object();
                });
            } catch (...) {  // no thread: the kernels load at their first launch
            }
        }
    }
    MI_HIP_CHECK(hipSetDevice(device));
    sparse = true;
    n = n_;
    d = d_;
    m = n - 1;
    nb = ceil_div(m, KP_TILE);
    n_pad = std::max<int64_t>(nb, 1) * KP_TILE;
    d_pad = d;
    csr = csr_data<T>{};
    csr.val_fmt = val_fmt;
    const int64_t nnz = rowptr[m];  // rows 0..m-1
    csr.nnz = nnz;
    auto hval = [&](int64_t k) -> T {
        return val_fmt == PLSSVM_MI_VAL_FP22 ? (T) fp22_get(static_cast<const uint32_t *>(val), k)
                                             : static_cast<const T *>(val)[k];
    };
    // last point, densified (the reference's data_last_d_)
    xlast_h.assign(d, T(0));
    for (int64_t k = rowptr[m]; k < rowptr[n]; ++k) xlast_h[col[k]] = hval(k);
    xlast.alloc(d, stream);
    MI_HIP_CHECK(hipMemcpyAsync(xlast.get(), xlast_h.data(), sizeof(T) * (size_t) d, hipMemcpyHostToDevice, stream));

    // CSR of rows 0..m-1
    csr.rowptr.alloc(m + 1, stream);
    MI_HIP_CHECK(hipMemcpyAsync(csr.rowptr.get(), rowptr, sizeof(int64_t) * (size_t) (m + 1), hipMemcpyHostToDevice,
                                stream));
    csr.col.alloc(std::max<int64_t>(nnz, 1), stream);
    if (nnz) MI_HIP_CHECK(hipMemcpyAsync(csr.col.get(), col, sizeof(int32_t) * (size_t) nnz, hipMemcpyHostToDevice, stream));
    // device CSR values in the context's real type: q, norms and the Gram-pattern build read them at
    // setup only (the Gram K·p streams the products s_ij); packed FP22 input is decoded here once and
    // stays packed only where the K·p streams feature values (the factored-linear SELL stream)
    csr.val.alloc(std::max<int64_t>(nnz, 1), stream);
    if (nnz && val_fmt == PLSSVM_MI_VAL_FP22) {
        // the packed words cross PCIe (2.75 B per value) and are decoded on the device (fp22_get, as on the host)
        const int64_t nw = fp22_words(nnz);
        dev_buf<uint32_t> w22;
        w22.alloc(nw, stream, false);
        MI_HIP_CHECK(hipMemcpyAsync(w22.get(), val, sizeof(uint32_t) * (size_t) nw, hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(fp22_unpack_kernel<T>, dim3((unsigned) ceil_div(nnz, 256)), dim3(256), 0, stream, w22.get(), nnz,
                           csr.val.get());
        MI_LAUNCH_CHECK();
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    } else if (nnz) {
        MI_HIP_CHECK(hipMemcpyAsync(csr.val.get(), val, sizeof(T) * (size_t) nnz, hipMemcpyHostToDevice, stream));
    }
    norms.alloc(std::max<int64_t>(n_pad, 1), stream);
    csr.e.alloc(std::max<int64_t>(n_pad, 1), stream);
    if (m > 0)
        hipLaunchKernelGGL(csr_norms_kernel<T>, dim3((unsigned) ceil_div(m, 16)), dim3(256), 0, stream,
                           csr.rowptr.get(), csr.rvals(), m, gamma, norms.get(), csr.e.get());
    MI_LAUNCH_CHECK();
    finish_setup();  // row split r0, r1
    pt.mark("setup_csr: check + upload + norms");

    // CSC of rows 0..m-1 (rows ascending inside each column) and, per CSR entry, its CSC position cpos (the
    // Gram pattern's column join needs "rows < i in this column" = cpos - colptr). On the device by default
    // (csc_device: a radix sort, the host keeps colptr and crow for its estimates and fetches the values only
    // for the SELL plans); on the host threads (csc_host: a counting sort) when nnz reaches 2^31 or with
    // PLSSVM_MI_CSC=host. Both give the same arrays.
    std::vector<int64_t> colptr(d + 1, 0), cpos;
    std::vector<int32_t> crow;
    // values in CSC order, decoded (FP22 input included: the Gram build multiplies them once at setup,
    // the K·p stream holds the products s_ij, so FP22 changes only the input format)
    std::vector<T> cval_real;
    dev_buf<int64_t> cpos_d;
    double amax = 0.0, nmax = 0.0;  // max x^2 and max |x_i|^2 (kernel expansion eligibility)
    bool dev_csc = [&] {
        const char *e = std::getenv("PLSSVM_MI_CSC");
        return nnz > 0 && nnz < (int64_t) INT32_MAX && !(e != nullptr && std::strcmp(e, "host") == 0);
    }();
    if (dev_csc) {
        // the device sort's temporaries (~16 B per entry + the radix-sort scratch) may not fit where the CSR
        // does: out of device memory, the host counting sort builds the same arrays, so a rank never
        // leaves setup here while its peers wait in the next group exchange
        try {
            csc_device(nnz, cpos_d);
        } catch (const std::exception &ex) {
            if (exception_code(ex) != -4) throw;
            dev_csc = false;
            csr.colptr.reset();
            csr.crow.reset();
            csr.cval.reset();
            cpos_d.reset();
            (void) hipGetLastError();
            MI_HIP_CHECK(hipStreamSynchronize(stream));
        }
    }
    if (dev_csc) {
        crow.resize((size_t) nnz);
        MI_HIP_CHECK(hipMemcpyAsync(colptr.data(), csr.colptr.get(), sizeof(int64_t) * (size_t) (d + 1),
                                    hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipMemcpyAsync(crow.data(), csr.crow.get(), sizeof(int32_t) * (size_t) nnz, hipMemcpyDeviceToHost,
                                    stream));
        // amax / nmax on the device, each row's sum of squares in the host sort's order (entries in order, no fma)
        {
            dev_buf<unsigned long long> mx;
            mx.alloc(2, stream);
            hipLaunchKernelGGL(csr_maxsq_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, csr.rowptr.get(),
                               csr.val.get(), m, mx.get());
            MI_LAUNCH_CHECK();
            unsigned long long h[2] = { 0ull, 0ull };
            MI_HIP_CHECK(hipMemcpyAsync(h, mx.get(), sizeof(h), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            std::memcpy(&amax, &h[0], sizeof(double));
            std::memcpy(&nmax, &h[1], sizeof(double));
        }
    } else {
        cpos.assign((size_t) std::max<int64_t>(nnz, 1), 0);
        crow.assign((size_t) std::max<int64_t>(nnz, 1), 0);
        cval_real.assign((size_t) std::max<int64_t>(nnz, 1), T(0));
        {
            const int NT = (int) std::max<int64_t>(1, std::min<int64_t>(host_threads(), nnz / 65536 + 1));
            std::vector<int64_t> rb(NT + 1, 0);  // row ranges balanced by entries
            for (int t = 1; t < NT; ++t)
                rb[t] = std::upper_bound(rowptr, rowptr + m + 1, (nnz * t) / NT) - rowptr - 1;
            rb[NT] = m;
            for (int t = 1; t <= NT; ++t) rb[t] = std::max(rb[t], rb[t - 1]);
            std::vector<std::vector<int64_t>> cnt((size_t) NT);
            std::vector<double> amax_t(NT, 0.0), nmax_t(NT, 0.0);
            host_parallel(NT, [&](int, int64_t t0, int64_t t1) {
                for (int64_t t = t0; t < t1; ++t) {
                    auto &c = cnt[(size_t) t];
                    c.assign((size_t) d, 0);
                    for (int64_t k = rowptr[rb[t]]; k < rowptr[rb[t + 1]]; ++k) ++c[(size_t) col[k]];
                }
            }, NT);
            for (int64_t f = 0; f < d; ++f) {  // colptr and each thread's first slot per column
                int64_t a = colptr[f];
                for (int t = 0; t < NT; ++t) {
                    const int64_t v = cnt[(size_t) t][(size_t) f];
                    cnt[(size_t) t][(size_t) f] = a;
                    a += v;
                }
                colptr[f + 1] = a;
            }
            host_parallel(NT, [&](int, int64_t t0, int64_t t1) {
                for (int64_t t = t0; t < t1; ++t) {
                    auto &fill = cnt[(size_t) t];
                    double am = 0.0, nm = 0.0;
                    for (int64_t i = rb[t]; i < rb[t + 1]; ++i) {
                        double nrm = 0.0;
                        for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
                            const int64_t q = fill[(size_t) col[k]]++;
                            crow[q] = (int32_t) i;
                            cpos[k] = q;
                            cval_real[q] = hval(k);
                            const double x = (double) cval_real[q];
                            am = std::max(am, x * x);
                            nrm += x * x;
                        }
                        nm = std::max(nm, nrm);
                    }
                    amax_t[(size_t) t] = am;
                    nmax_t[(size_t) t] = nm;
                }
            }, NT);
            for (int t = 0; t < NT; ++t) amax = std::max(amax, amax_t[(size_t) t]), nmax = std::max(nmax, nmax_t[(size_t) t]);
        }
    }
    // the CSC values on the host (the SELL plans' CSC generator): fetched on first use after a device sort
    auto need_cval_h = [&](hipStream_t s) {
        if (!dev_csc || !cval_real.empty()) return;
        cval_real.resize((size_t) nnz);
        MI_HIP_CHECK(hipMemcpyAsync(cval_real.data(), csr.cval.get(), sizeof(T) * (size_t) nnz, hipMemcpyDeviceToHost, s));
        MI_HIP_CHECK(hipStreamSynchronize(s));
    };
    // CSC segments of rows [c0, c1) (rows ascending in each column: a contiguous part of the column)
    auto csc_gen = [&](int64_t c0, int64_t c1) {
        return [&, c0, c1](auto emit, int64_t f0, int64_t f1) {
            for (int64_t f = f0; f < f1; ++f) {
                const int32_t *b0 = crow.data() + colptr[f], *b1 = crow.data() + colptr[f + 1];
                const int32_t *lo = c0 > 0 ? std::lower_bound(b0, b1, (int32_t) c0) : b0;
                const int32_t *hi = c1 < m ? std::lower_bound(lo, b1, (int32_t) c1) : b1;
                for (const int32_t *t = lo; t < hi; ++t) emit(f, (int64_t) *t - c0, (double) cval_real[(size_t) (t - crow.data())]);
            }
        };
    };
    // CSR segments = rows [base + s0, base + s1)
    auto csr_gen = [&](int64_t base) {
        return [&, base](auto emit, int64_t s0, int64_t s1) {
            for (int64_t s = s0; s < s1; ++s)
                for (int64_t k = rowptr[base + s]; k < rowptr[base + s + 1]; ++k) emit(s, (int64_t) col[k], (double) hval(k));
        };
    };
    if (factored()) {
        // factored linear: w = X_rows^T p over rows [csc_r0, csc_r1) — all rows for
        // a single or simulated rank, this rank's rows in a real group (w is then all-reduced) — and
        // raw[r0, r1) = X w, both as panelled SELL-64 SpMVs (spmv.hpp)
        const bool local = (world > 1 && sim_world == 0) || (sim_world > 0 && shard);
        csr.csc_r0 = local ? r0 : 0;
        csr.csc_r1 = local ? r1 : m;
        const bool f22 = val_fmt == PLSSVM_MI_VAL_FP22 && sell_fp22_stream();
        const int64_t blocks = sell_target_blocks();
        // the CSR-side plans need no CSC values: a host thread builds them (uploads on a stream of its own) while this
        // thread fetches the CSC values and builds the CSC plan (round 5)
        std::exception_ptr rfail;
        hipStream_t rs = nullptr;
        std::thread rplans([&] {
            try {
                MI_HIP_CHECK(hipSetDevice(device));
                MI_HIP_CHECK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
                build_spmv_plan<T>(csr.spmv_csr, r1 - r0, d, rowptr[r1] - rowptr[r0], f22, csr_gen(r0), blocks, rs);
                if (world == 1 && sim_world == 0)  // CG: CSR pass + finalize in one launch
                    build_rowblock_plan<T>(csr.rb_csr, m, d, f22, csr_gen(0), blocks, rs);
                MI_HIP_CHECK(hipStreamSynchronize(rs));
            } catch (...) {
                rfail = std::current_exception();
            }
        });
        std::exception_ptr cfail;
        try {
            need_cval_h(stream);
            // the K·p reads only the SELL streams: no device CSC
            cpos_d.reset(), csr.colptr.reset(), csr.crow.reset(), csr.cval.reset();
            build_spmv_plan<T>(csr.spmv_csc, d, csr.csc_r1 - csr.csc_r0, rowptr[csr.csc_r1] - rowptr[csr.csc_r0], f22,
                               csc_gen(csr.csc_r0, csr.csc_r1), blocks, stream);
        } catch (...) {
            cfail = std::current_exception();
        }
        rplans.join();
        if (rs != nullptr) (void) hipStreamDestroy(rs);
        if (cfail) std::rethrow_exception(cfail);
        if (rfail) std::rethrow_exception(rfail);
        pt.mark("setup_csr: SELL plans");
        return;
    }
    csr.csc_r0 = 0;
    csr.csc_r1 = m;
    if (!dev_csc) {  // the host sort's CSC to the device
        csr.colptr.alloc(d + 1, stream);
        MI_HIP_CHECK(hipMemcpyAsync(csr.colptr.get(), colptr.data(), sizeof(int64_t) * (size_t) (d + 1),
                                    hipMemcpyHostToDevice, stream));
        csr.crow.alloc(std::max<int64_t>(nnz, 1), stream);
        if (nnz)
            MI_HIP_CHECK(hipMemcpyAsync(csr.crow.get(), crow.data(), sizeof(int32_t) * (size_t) nnz, hipMemcpyHostToDevice,
                                        stream));
        csr.cval.alloc(std::max<int64_t>(nnz, 1), stream);
        if (nnz)
            MI_HIP_CHECK(hipMemcpyAsync(csr.cval.get(), cval_real.data(), sizeof(T) * (size_t) nnz, hipMemcpyHostToDevice,
                                        stream));
        cpos_d.alloc(std::max<int64_t>(nnz, 1), stream);
        if (nnz)
            MI_HIP_CHECK(hipMemcpyAsync(cpos_d.get(), cpos.data(), sizeof(int64_t) * (size_t) nnz, hipMemcpyHostToDevice,
                                        stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
    pt.mark(dev_csc ? "setup_csr: device CSC" : "setup_csr: host CSC");

    {
        // Gram pattern: row blocks owned by this rank, balanced by column-join incidences
        const int64_t nRB = ceil_div(std::max<int64_t>(m, 1), GRAM_RB);
        std::vector<int64_t> inc_rb(nRB, 0);
        if (dev_csc) {
            dev_buf<int64_t> irb;
            irb.alloc(nRB, stream);
            if (m > 0) {
                hipLaunchKernelGGL(csc_inc_rb_kernel, dim3((unsigned) nRB), dim3(256), 0, stream, csr.rowptr.get(),
                                   csr.col.get(), cpos_d.get(), csr.colptr.get(), m, (int64_t) GRAM_RB, irb.get());
                MI_LAUNCH_CHECK();
            }
            MI_HIP_CHECK(hipMemcpyAsync(inc_rb.data(), irb.get(), sizeof(int64_t) * (size_t) nRB, hipMemcpyDeviceToHost,
                                        stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
        } else {
            host_parallel(nRB, [&](int, int64_t I0, int64_t I1) {
                for (int64_t I = I0; I < I1; ++I) {
                    int64_t a = 0;
                    for (int64_t k = rowptr[I * GRAM_RB]; k < rowptr[std::min<int64_t>(m, (I + 1) * GRAM_RB)]; ++k)
                        a += cpos[k] - colptr[col[k]];
                    inc_rb[(size_t) I] = a;
                }
            });
        }
        const int eff_world = sim_world > 0 ? sim_world : world, eff_rank = sim_world > 0 ? sim_rank : rank;
        std::vector<int64_t> cum(nRB + 1, 0);
        for (int64_t I = 0; I < nRB; ++I) cum[I + 1] = cum[I] + inc_rb[I];
        auto split = [&](int r) {
            if (r <= 0) return (int64_t) 0;
            if (r >= eff_world) return nRB;
            return (int64_t) (std::lower_bound(cum.begin(), cum.end(), (cum[nRB] * r) / eff_world) - cum.begin());
        };
        csr.nRB = nRB;
        csr.nW = ceil_div(std::max<int64_t>(m, 1), (int64_t) GRAM_CW);
        csr.rb0 = std::min(split(eff_rank), nRB);
        csr.rb1 = std::max(csr.rb0, std::min(split(eff_rank + 1), nRB));
        csr.pair_bound = cum[csr.rb1] - cum[csr.rb0];
        int64_t max_inc = 0;
        for (int64_t I = csr.rb0; I < csr.rb1; ++I) max_inc = std::max(max_inc, inc_rb[I]);
        // kernel expansion (expand.hip) when it represents the kernel to rounding, else the Gram pattern;
        // either only within the device-memory budget, else the densified MFMA path
        csr.ex.umax = 2.0 * std::fabs((double) gamma) * amax;
        const bool fact_ok = kernel != 2 || std::fabs((double) gamma) * nmax <= (sizeof(T) == 8 ? 300.0 : 40.0);
        const bool elig = sparse_algo != 3 && fact_ok && expansion_eligible();
        if (sparse_algo == 2 && !elig)
            throw mi_error(-5, "the kernel expansion cannot represent this kernel on this data (Taylor degree > 16 or "
                               "the factored rbf form out of range): use the Gram pattern");
        int64_t budget = sparse_mem_budget();
        const bool use_exp = elig && sparse_algo != 1;
        const bool unstored = sparse_algo == 3 || sparse_algo == 4;  // forced densified / on the fly
        if (!unstored) {
            int64_t inc_total = 0;
            for (int64_t I = csr.rb0; I < csr.rb1; ++I) inc_total += inc_rb[I];
            double rs[2] = { 0.0, 0.0 };
            csr.est_bytes = use_exp ? estimate_expansion_bytes(rowptr, col, colptr, crow, inc_total, rs)
                                    : csr.pair_bound * (int64_t) (2 * (2 + sizeof(T))) + max_inc * 48;
            csr.ex.rj_mean = rs[0], csr.ex.rj_max = rs[1];  // the one-pass row join's slots per row
        }
        // A real group takes every choice below once, identically on all ranks (the paths run different
        // collectives on different partitions): the largest estimate against the smallest budget, the
        // slowest on-the-fly estimate, and a fallback only when the ranks agree a build failed.
        // (eligibility, the forced options and t_dense depend only on data and parameters every rank holds)
        if (in_group()) {
            const auto g = group_gather({ (double) csr.est_bytes, (double) budget });
            double est = 0.0, bud = 0.0;
            for (int r = 0; r < world; ++r) {
                est = std::max(est, g[(size_t) (2 * r)]);
                bud = r == 0 ? g[1] : std::min(bud, g[(size_t) (2 * r + 1)]);
            }
            csr.est_bytes = (int64_t) est;
            budget = (int64_t) bud;
        }
        csr.budget_b = budget;  // read before the SELL plans' host thread allocates (the row join's pool)
        // a failed step of the group: the same error on every rank (the worst code; ERR_OOM = fall back)
        auto agree = [&](int code, const std::string &why) -> int {
            if (!in_group()) return code;
            const auto g = group_gather({ (double) code });
            int worst = 0;
            for (int r = 0; r < world; ++r) {
                const int c = (int) g[(size_t) r];
                if (c != 0 && (worst == 0 || worst == -4)) worst = c;
            }
            if (worst != 0 && worst != -4)
                throw mi_error(worst, code != 0 ? why : std::string("sparse setup failed on another rank of the group"));
            return worst;
        };
        pt.mark("setup_csr: incidences + size estimate");
        const bool forced = sparse_algo == 1 || sparse_algo == 2;
        bool stored = false;
        if (!unstored && (forced || csr.est_bytes <= budget)) {
            int fail = 0;
            std::string why;
            try {
                if (use_exp) {
                    // the two SELL passes of the kernel expansion (the factored linear path's plans, with K channels):
                    // column moments over the CSC of this rank's rows in a real group (all-reduced, d x K values)
                    // or of all rows, the Horner pass over this rank's CSR rows
                    const bool f22 = val_fmt == PLSSVM_MI_VAL_FP22 && sell_fp22_stream();
                    const int64_t blocks = sell_target_blocks();
                    const bool local = (world > 1 && sim_world == 0) || (sim_world > 0 && shard);
                    csr.csc_r0 = local ? r0 : 0;
                    csr.csc_r1 = local ? r1 : m;
                    // the two SELL plans (host work + uploads on a stream of their own) run on a host thread while
                    // the GPU builds the remainder's rows; build_expansion joins it before the group agreement
                    // (round 5: the CSR plan needs no CSC values, so it runs on a thread of its own from the start; the
                    // CSC plan's thread first fetches the CSC values — the two plans' host work overlaps)
                    std::exception_ptr plan_fail, plan_fail2;
                    hipStream_t ps = nullptr, ps2 = nullptr;
                    std::thread plans([&] {
                        try {
                            phase_timer tp;
                            MI_HIP_CHECK(hipSetDevice(device));
                            MI_HIP_CHECK(hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
                            need_cval_h(ps);
                            tp.mark("setup_csr: (plans thread) CSC values to the host");
                            build_spmv_plan<T>(csr.spmv_csc, d, csr.csc_r1 - csr.csc_r0,
                                               rowptr[csr.csc_r1] - rowptr[csr.csc_r0], f22, csc_gen(csr.csc_r0, csr.csc_r1),
                                               blocks, ps, 0, 1, csr.ex.KM);
                            MI_HIP_CHECK(hipStreamSynchronize(ps));
                            tp.mark("setup_csr: SELL plan CSC (host thread, beside the row join)");
                        } catch (...) {
                            plan_fail = std::current_exception();
                        }
                    });
                    std::thread plans2([&] {
                        try {
                            phase_timer tp;
                            MI_HIP_CHECK(hipSetDevice(device));
                            MI_HIP_CHECK(hipStreamCreateWithFlags(&ps2, hipStreamNonBlocking));
                            build_spmv_plan<T>(csr.spmv_csr, r1 - r0, d, rowptr[r1] - rowptr[r0], f22, csr_gen(r0), blocks,
                                               ps2, 0, csr.ex.KM, 1);
                            MI_HIP_CHECK(hipStreamSynchronize(ps2));
                            tp.mark("setup_csr: SELL plan CSR (host thread, beside the row join)");
                        } catch (...) {
                            plan_fail2 = std::current_exception();
                        }
                    });
                    bool joined = false;
                    auto join_plans = [&]() -> std::exception_ptr {
                        if (!joined) {
                            plans.join();
                            plans2.join();
                            joined = true;
                            if (ps != nullptr) (void) hipStreamDestroy(ps);
                            if (ps2 != nullptr) (void) hipStreamDestroy(ps2);
                        }
                        return plan_fail ? plan_fail : plan_fail2;
                    };
                    exp_loader.join();  // expand.hip's code object is in place before its first kernel
                    try {
                        build_expansion(cpos_d.get(), max_inc, join_plans);
                    } catch (...) {
                        join_plans();
                        throw;
                    }
                    join_plans();
                    pt.mark("setup_csr: expansion");
                } else {
                    build_gram_blocks(cpos_d.get(), max_inc);
                }
                stored = true;
            } catch (const std::exception &e) {
                // any failure (also a host table's bad_alloc or length_error, or one rethrown from host_parallel):
                // in a group every rank must still reach agree() below, with a code
                const int c = exception_code(e);
                if (!in_group() && (c != -4 || forced)) throw;
                fail = c;
                why = c == -4 && dynamic_cast<const mi_error *>(&e) == nullptr ? "host allocation failed" : e.what();
            }
            fail = agree(fail, why);
            if (fail != 0 && forced) throw mi_error(fail, why.empty() ? "the forced sparse structure did not fit on another rank" : why);
            if (fail != 0) {
                MI_HIP_CHECK(hipStreamSynchronize(stream));
                const int64_t keep = csr.est_bytes;  // the stored structure did not fit after all: drop it
                release_sparse_structures();
                csr.est_bytes = keep;
                stored = false;
            }
        }
        if (!stored) {
            // no stored structure: the on-the-fly path or the densified MFMA tiles, whichever the estimate
            // makes faster (auto), unless one is forced
            cpos_d.reset();
            bool otf = sparse_algo == 4;
            if (sparse_algo == 0) {
                const double peak = sizeof(T) == 8 ? 78.6e12 : 157.3e12;
                const double dp = (double) round_up(std::max<int64_t>(d, 1), kp_dpad<T>());
                const int eff_world = sim_world > 0 ? sim_world : world;
                const double t_dense = (double) m * (double) m * dp / (double) eff_world / (0.85 * peak);
                double t_otf = otf_estimate_s(rowptr, col, colptr);
                if (in_group()) {  // the slowest rank's share decides
                    const auto g = group_gather({ t_otf });
                    t_otf = *std::max_element(g.begin(), g.end());
                }
                otf = t_otf < t_dense;
                if (std::getenv("PLSSVM_MI_TIMING") != nullptr)
                    std::fprintf(stderr, "[plssvm_mi] unstored sparse K·p: on the fly ~%.3g s, densified ~%.3g s\n", t_otf,
                                 t_dense);
            }
            if (otf) {
                int fail = 0;
                std::string why;
                try {
                    setup_otf(fact_ok ? 1 : 0);
                } catch (const std::exception &e) {  // its tables did not fit either: the densified path decides
                    const int c = exception_code(e);
                    if (!in_group() && (c != -4 || sparse_algo == 4)) throw;
                    fail = c;
                    why = e.what();
                }
                fail = agree(fail, why);
                if (fail != 0 && sparse_algo == 4) throw mi_error(fail, why.empty() ? "on-the-fly setup failed on another rank" : why);
                if (fail != 0) {
                    MI_HIP_CHECK(hipStreamSynchronize(stream));
                    csr.seg.reset(), csr.ecb.reset(), csr.pne.reset(), csr.cjv.reset(), csr.otf_part.reset();
                    csr.otf_on = false;
                    otf = false;
                }
            }
            if (!otf) {
                int fail = 0;
                std::string why;
                try {
                    setup_sparse_dense();
                } catch (const std::exception &e) {
                    if (!in_group()) throw;
                    fail = exception_code(e);
                    why = e.what();
                }
                fail = agree(fail, why);
                if (fail != 0) throw mi_error(fail, why.empty() ? "densified setup failed on another rank of the group" : why);
            }
        }
    }
}

// device bytes the stored sparse structures may use: 85 % of the free memory (PLSSVM_MI_MEM_BUDGET =
// bytes overrides it, tests force the densified path with it)
template <typename T>
int64_t engine<T>::sparse_mem_budget() const {
    if (const char *e = std::getenv("PLSSVM_MI_MEM_BUDGET")) {
        const long long v = std::atoll(e);
        if (v > 0) return (int64_t) v;
    }
    size_t free_b = 0, total_b = 0;
    MI_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    return (int64_t) ((double) free_b * 0.85);
}

// peak device bytes of build_expansion: the remainder's symmetric entries (sampled: partners sharing two
// or more features of up to 64 rows of this rank, capped at ~2^28 column-join incidences) times the
// bytes its build holds per entry (lower list, symmetric rows, cells, sort keys), plus one sub-block of
// sort temporaries
template <typename T>
int64_t engine<T>::estimate_expansion_bytes(const int64_t *rowptr, const int32_t *col, const std::vector<int64_t> &colptr,
                                            const std::vector<int32_t> &crow, int64_t inc_total, double *row_stats) const {
    const int64_t R = r1 - r0;
    if (R <= 0 || m <= 0) return 0;
    std::vector<int32_t> cnt((size_t) m, 0);
    std::vector<int32_t> touched;
    const int64_t S = std::min<int64_t>(R, 64);
    int64_t sampled = 0, entries = 0, inc = 0, row_max = 0;
    for (int64_t s = 0; s < S && inc < (int64_t(1) << 28); ++s) {
        const int64_t i = r0 + (s * R) / S;
        touched.clear();
        for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
            const int32_t f = col[k];
            for (int64_t t = colptr[f]; t < colptr[f + 1]; ++t) {
                const int32_t j = crow[t];
                if (cnt[j]++ == 0) touched.push_back(j);
            }
            inc += colptr[f + 1] - colptr[f];
        }
        int64_t row_entries = 0;
        for (const int32_t j : touched) {
            if (j != i && cnt[j] >= 2) ++row_entries;
            cnt[j] = 0;
        }
        entries += row_entries;
        row_max = std::max(row_max, row_entries);
        ++sampled;
    }
    const double per_row = sampled ? (double) entries / (double) sampled : 0.0;
    if (row_stats != nullptr) row_stats[0] = per_row, row_stats[1] = (double) row_max;
    const double est_entries = per_row * (double) R;
    const int64_t per_entry = 2 * (4 + 4 + (int64_t) sizeof(T)) + 4 * (4 + (int64_t) sizeof(T)) + 16;
    const int64_t blk = std::min<int64_t>(inc_total, int64_t(1) << 27);
    return (int64_t) (est_entries * (double) per_entry) + blk * 80;
}

// drop every stored sparse K·p structure (a build that ran out of memory)
template <typename T>
void engine<T>::release_sparse_structures() {
    csr.ex = exp_data<T>{};
    csr.spmv_csc = spmv_plan<T>{};
    csr.spmv_csr = spmv_plan<T>{};
    csr.pj.reset(), csr.ps.reset(), csr.rb_base.reset(), csr.rowoff.reset(), csr.cells.reset();
    csr.slab_row.reset(), csr.slab_col.reset();
    csr.have_gram = false;
    csr.pairs = csr.slots = 0;
}

template <typename T>
__global__ __launch_bounds__(256) void csr_densify_kernel(const int64_t *__restrict__ rowptr,
                                                          const int32_t *__restrict__ col, const T *__restrict__ val,
                                                          int64_t m, int64_t n_pad, T *__restrict__ XT) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) XT[(int64_t) col[k] * n_pad + i] = val[k];
}

// the densified path: XT[d_pad][n_pad] from the device CSR, the dense pairwise partial slab; K·p then
// runs the MFMA tiles of the dense path (every pair recomputed from the data, as the reference does on
// its densified arrays)
template <typename T>
void engine<T>::setup_sparse_dense() {
    const int64_t dp = round_up(std::max<int64_t>(d, 1), kp_dpad<T>());
    const int64_t need = (dp * n_pad + std::max<int64_t>(kp_wgs, 1) * KP_REC) * (int64_t) sizeof(T);
    size_t free_b = 0, total_b = 0;
    MI_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    if ((double) need > 0.95 * (double) free_b)
        throw mi_error(-4, "sparse data: the stored K·p structures exceed the device budget (estimated " +
                               std::to_string(csr.est_bytes >> 20) + " MiB) and the densified matrix needs " +
                               std::to_string(need >> 20) + " MiB of " + std::to_string(free_b >> 20) +
                               " MiB free: use more GPUs or a smaller data set");
    d_pad = dp;
    XT.alloc(d_pad * n_pad, stream);
    partial.alloc(std::max<int64_t>(kp_wgs, 1) * KP_REC, stream, false);
    if (m > 0)
        hipLaunchKernelGGL(csr_densify_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream,
                           csr.rowptr.get(), csr.col.get(), csr.val.get(), m, n_pad, XT.get());
    MI_LAUNCH_CHECK();
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    csr.dense_on = true;
}

template <typename T>
void engine<T>::build_gram_blocks(const int64_t *cpos, int64_t max_inc) {
    csr.m_pad = round_up(std::max<int64_t>(m, 1), 256);
    // host cell table
    std::vector<gram_cell> cells;
    std::vector<int64_t> rowoff_base(csr.nRB, 0);
    int64_t ro_total = 0;
    const int64_t CW = GRAM_CW;
    for (int64_t I = csr.rb0; I < csr.rb1; ++I) {
        const int64_t nw = gram_nw(I, m, CW);
        rowoff_base[I] = ro_total;
        for (int64_t W = 0; W < nw; ++W) cells.push_back(gram_cell{ (int32_t) I, (int32_t) W, ro_total + W * GRAM_RB, 0.0 });
        ro_total += nw * GRAM_RB + 1;
    }
    csr.ncells = (int64_t) cells.size();
    csr.cells.alloc(std::max<int64_t>(csr.ncells, 1), stream);
    if (csr.ncells)
        MI_HIP_CHECK(hipMemcpyAsync(csr.cells.get(), cells.data(), sizeof(gram_cell) * cells.size(),
                                    hipMemcpyHostToDevice, stream));
    csr.rowoff.alloc(std::max<int64_t>(ro_total, 1), stream);
    csr.rb_base.alloc(std::max<int64_t>(csr.nRB, 1), stream);
    // each row block's pairs start 8-aligned (the K·p kernel reads 8 pairs per lane with 16-byte loads)
    // unique pairs <= incidences (pair_bound); padding adds < 8 per non-empty (row, window) group
    int64_t groups = 0;
    for (int64_t I = csr.rb0; I < csr.rb1; ++I)
        groups += (std::min<int64_t>(m, (I + 1) * GRAM_RB) - I * GRAM_RB) * gram_nw(I, m, CW);
    const int64_t pcap = csr.pair_bound + 7 * std::min(csr.pair_bound, groups) + 16;
    csr.pj.alloc(pcap, stream, false);
    hipLaunchKernelGGL(gram_pad_index_kernel, dim3((unsigned) ceil_div(pcap, 256)), dim3(256), 0, stream, csr.pj.get(),
                       pcap);
    MI_LAUNCH_CHECK();
    csr.ps.alloc(pcap, stream);
    csr.slab_row.alloc(std::max<int64_t>(csr.nW, 1) * csr.m_pad, stream);
    csr.slab_col.alloc(std::max<int64_t>(csr.nRB, 1) * csr.m_pad, stream);
    csr.ssc.alloc(2, stream);

    // temporaries for one row block
    const int64_t cap = std::max<int64_t>(max_inc, 1);
    dev_buf<uint64_t> keys, keys_s;
    dev_buf<T> vals, vals_s;
    dev_buf<int64_t> cnt, off, nruns;
    dev_buf<int32_t> rowcnt, uoff, cnt8;
    keys.alloc(cap, stream, false);
    keys_s.alloc(cap, stream, false);
    vals.alloc(cap, stream, false);
    vals_s.alloc(cap, stream, false);
    cnt.alloc(GRAM_RB + 1, stream);
    off.alloc(GRAM_RB + 1, stream);
    nruns.alloc(1, stream);
    rowcnt.alloc(csr.nW * GRAM_RB + 1, stream);
    uoff.alloc(csr.nW * GRAM_RB + 1, stream);
    cnt8.alloc(csr.nW * GRAM_RB + 1, stream);
    size_t tmp_sort = 0, tmp_scan = 0, tmp_red = 0, tmp_scan32 = 0;
    MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_sort, keys.get(), keys_s.get(), vals.get(),
                                                    vals_s.get(), (int) std::min<int64_t>(cap, INT32_MAX), 0, 64,
                                                    stream));
    MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_scan, cnt.get(), off.get(), GRAM_RB + 1, stream));
    MI_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(nullptr, tmp_red, keys_s.get(), keys.get(), vals_s.get(),
                                                   vals.get(), nruns.get(), hipcub::Sum(),
                                                   (int) std::min<int64_t>(cap, INT32_MAX), stream));
    MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_scan32, rowcnt.get(), rowcnt.get(),
                                                  (int) (csr.nW * GRAM_RB + 1), stream));
    dev_buf<unsigned char> tmp;
    tmp.alloc((int64_t) std::max({ tmp_sort, tmp_scan, tmp_red, tmp_scan32, (size_t) 16 }), stream, false);
    if (cap > INT32_MAX) throw mi_error(-5, "a Gram row block exceeds 2^31 incidences");

    std::vector<int64_t> rb_base(csr.nRB, 0);
    int64_t pos = 0;
    csr.pairs = 0;
    const int end_bit = 32 + std::max(1, (int) std::ceil(std::log2((double) csr.nW + 1.0)));
    for (int64_t I = csr.rb0; I < csr.rb1; ++I) {
        const int64_t i0 = I * GRAM_RB, i1 = std::min<int64_t>(m, i0 + GRAM_RB), rows = i1 - i0;
        const int64_t nw = gram_nw(I, m, CW);
        pos = round_up(pos, 8);
        rb_base[I] = pos;
        MI_HIP_CHECK(hipMemsetAsync(cnt.get(), 0, sizeof(int64_t) * (GRAM_RB + 1), stream));
        hipLaunchKernelGGL(gram_count_kernel, dim3((unsigned) ceil_div(rows, 256)), dim3(256), 0, stream,
                           csr.rowptr.get(), csr.col.get(), cpos, csr.colptr.get(), i0, i1, cnt.get());
        MI_LAUNCH_CHECK();
        size_t ts = tmp_scan;
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.get(), ts, cnt.get(), off.get(), (int) (rows + 1), stream));
        int64_t total = 0;
        MI_HIP_CHECK(hipMemcpyAsync(&total, off.get() + rows, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        MI_HIP_CHECK(hipMemsetAsync(rowcnt.get(), 0, sizeof(int32_t) * (size_t) (nw * GRAM_RB + 1), stream));
        int64_t nu = 0;
        if (total > 0) {
            hipLaunchKernelGGL(gram_gen_kernel<T>, dim3((unsigned) rows), dim3(256), 0, stream, csr.rowptr.get(),
                               csr.col.get(), csr.rvals(), cpos, csr.colptr.get(), csr.crow.get(), csr.cvals(), i0,
                               off.get(), keys.get(), vals.get());
            MI_LAUNCH_CHECK();
            size_t t1s = tmp_sort;
            MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.get(), t1s, keys.get(), keys_s.get(), vals.get(),
                                                            vals_s.get(), (int) total, 0, end_bit, stream));
            size_t t2s = tmp_red;
            MI_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(tmp.get(), t2s, keys_s.get(), keys.get(), vals_s.get(),
                                                           vals.get(), nruns.get(), hipcub::Sum(), (int) total,
                                                           stream));
            MI_HIP_CHECK(hipMemcpyAsync(&nu, nruns.get(), sizeof(int64_t), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            // cnt8 holds the group starts here (gram_pad_kernel rewrites it below)
            hipLaunchKernelGGL(gram_rowcount_kernel, dim3((unsigned) ceil_div(nu, 256)), dim3(256), 0, stream,
                               keys.get(), nruns.get(), rowcnt.get(), cnt8.get());
            MI_LAUNCH_CHECK();
            const int64_t ngr = nw * GRAM_RB;
            hipLaunchKernelGGL(gram_runlen_kernel, dim3((unsigned) ceil_div(ngr, 256)), dim3(256), 0, stream,
                               rowcnt.get(), cnt8.get(), ngr);
            MI_LAUNCH_CHECK();
        }
        const int ng = (int) (nw * GRAM_RB + 1);
        int32_t *padded = csr.rowoff.get() + rowoff_base[I];
        size_t t3s = tmp_scan32;
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.get(), t3s, rowcnt.get(), uoff.get(), ng, stream));
        hipLaunchKernelGGL(gram_pad_kernel, dim3((unsigned) ceil_div(ng, 256)), dim3(256), 0, stream, rowcnt.get(),
                           (int64_t) ng, cnt8.get());
        MI_LAUNCH_CHECK();
        t3s = tmp_scan32;
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.get(), t3s, cnt8.get(), padded, ng, stream));
        int32_t slots = 0;
        MI_HIP_CHECK(hipMemcpyAsync(&slots, padded + ng - 1, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        if (slots < 0 || pos + slots > pcap) throw mi_error(-5, "Gram pattern exceeds its capacity bound");
        if (nu > 0) {
            hipLaunchKernelGGL(gram_store_kernel<T>, dim3((unsigned) ceil_div(nu, 256)), dim3(256), 0, stream,
                               keys.get(), vals.get(), nruns.get(), uoff.get(), padded, csr.pj.get() + pos,
                               csr.ps.get() + pos);
            MI_LAUNCH_CHECK();
        }
        csr.pairs += nu;
        pos += slots;
    }
    csr.slots = pos;
    MI_HIP_CHECK(hipMemcpyAsync(csr.rb_base.get(), rb_base.data(), sizeof(int64_t) * (size_t) csr.nRB,
                                hipMemcpyHostToDevice, stream));
    if (csr.ncells > 0) {
        hipLaunchKernelGGL(gram_cell_smax_kernel<T>, dim3((unsigned) csr.ncells), dim3(256), 0, stream, csr.cells.get(),
                           csr.rb_base.get(), csr.rowoff.get(), csr.ps.get(), m);
        MI_LAUNCH_CHECK();
    }
    // factored rbf c_ij = e_i e_j expm1(2 g s_ij): only while 2 g max|s_ij| <= 1. The fixed-point quantum
    // of the K·p accumulators is set by the cell's bound expm1(2 g smax) max|e p|, which overestimates the
    // actual terms (|e_i e_j expm1(2 g s)| <= 1) by up to expm1(2 g smax) e_i: above 1 the factored
    // terms would lose digits to it, and the direct form exp(-g |x_i - x_j|^2) - e_i e_j (bound 1) is used
    csr.rbf_factored = false;
    if (kernel == 2) {
        std::vector<gram_cell> hc((size_t) csr.ncells);
        if (csr.ncells)
            MI_HIP_CHECK(hipMemcpyAsync(hc.data(), csr.cells.get(), sizeof(gram_cell) * hc.size(), hipMemcpyDeviceToHost,
                                        stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        double smax = 0.0;
        for (const auto &c : hc) smax = std::max(smax, c.smax);
        const double u = 2.0 * std::fabs((double) gamma) * smax;
        csr.rbf_factored = rbf_form != 1 && u <= 1.0;
        // every pair's 2 g |s_ij| below the small-argument polynomial's bound -> KERNEL 4
        csr.rbf_small = u < expm1_small_bound<T>();
    }
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    csr.have_gram = true;
}

// factored linear passes: w = X_rows^T p, raw[r0..r1) = X w (panelled SELL SpMVs, spmv.hpp)
template <typename T>
void engine<T>::spmv_pass_csc(const T *p, const cg_scalars<T> *status) {
    launch_panel_spmv<T>(csr.spmv_csc, p + csr.csc_r0, csr.csc_r1 - csr.csc_r0, w.get(), status, stream);
}

template <typename T>
void engine<T>::spmv_pass_csr(const cg_scalars<T> *status) {
    launch_panel_spmv<T>(csr.spmv_csr, w.get(), d, raw.get() + r0, status, stream);
}

template <typename T>
void engine<T>::sparse_q() {
    if (m <= 0) return;
    T nlast = 0;
    for (int64_t k = 0; k < d; ++k) nlast = std::fma(xlast_h[k], xlast_h[k], nlast);
    hipLaunchKernelGGL(csr_q_kernel<T>, dim3((unsigned) ceil_div(m, 16)), dim3(256), 0, stream, kf(),
                       csr.rowptr.get(), csr.col.get(), csr.rvals(), m, xlast.get(), nlast, norms.get(), q.get());
    MI_LAUNCH_CHECK();
}

template <typename T>
void engine<T>::sparse_kp_raw(const T *p, const cg_scalars<T> *status, bool with_base) {
    if (factored()) {
        spmv_pass_csc(p, status);
        allreduce(w.get(), d);
        spmv_pass_csr(status);
        if (!shard) allgather_rows(raw.get());
        return;
    }
    if (csr.otf_on) {
        otf_kp_raw(p, status, with_base);
        return;
    }
    if (csr.ex.on) {
        expansion_kp_raw(p, status, with_base);
        return;
    }
    // separable sum: sum(e p) (rbf) or sum(p) (poly)
    gather_input(p);
    launch_dot2<T>(p, kernel == 2 ? csr.e.get() : nullptr, nullptr, nullptr, m, red.get(), status, stream);
    launch_dot_final<T>(red.get(), sc.get(), FIN_PLAIN, 0, nullptr, 0, csr.ssc.get(), stream);
    sparse_dominant(p, status);
    hipLaunchKernelGGL(gram_reduce_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream,
                       csr.slab_row.get(), csr.slab_col.get(), m, csr.m_pad, csr.rb0, csr.rb1, raw.get(), status);
    MI_LAUNCH_CHECK();
    if (shard) reduce_scatter_rows(raw.get());
    else allreduce(raw.get(), m);
    if (with_base && !(sim_world > 0 && sim_rank != 0)) {
        T kappa = 0;
        if (kernel == 1) {
            kappa = 1;
            for (int q2 = 0; q2 < degree; ++q2) kappa *= coef0;
        }
        hipLaunchKernelGGL(gram_base_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, kernel, kf(),
                           kappa, csr.ssc.get(), norms.get(), csr.e.get(), p, m, raw.get(), status);
        MI_LAUNCH_CHECK();
    }
}

template <typename T>
void engine<T>::sparse_dominant(const T *p, const cg_scalars<T> *status) {
    if (factored()) {  // both SpMV passes (the factored K·p without its collectives)
        spmv_pass_csc(p, status);
        spmv_pass_csr(status);
        return;
    }
    if (csr.otf_on) {  // the on-the-fly pair kernel (rows of this rank)
        otf_dominant(p, status);
        return;
    }
    if (csr.ex.on) {  // timing: the remainder stream (p stands in for w)
        expansion_dominant(p, status);
        return;
    }
    if (csr.ncells == 0) return;
    T kappa = 0;
    if (kernel == 1) {
        kappa = 1;
        for (int q2 = 0; q2 < degree; ++q2) kappa *= coef0;
    }
    const dim3 grid((unsigned) csr.ncells);
    auto launch = [&](auto kern, int nt) {
        hipLaunchKernelGGL(kern, grid, dim3(nt), 0, stream, csr.cells.get(), csr.rb_base.get(), csr.rowoff.get(),
                           csr.pj.get(), csr.ps.get(), norms.get(), csr.e.get(), p, csr.slab_row.get(),
                           csr.slab_col.get(), m, csr.m_pad, kf(), kappa, status);
    };
    auto pick = [&](auto abl) {
        constexpr int A = decltype(abl)::value;
        if (kernel == 0) launch(gram_kp_kernel<T, 0, A>, gram_wg<T, 0>());
        else if (kernel == 1) launch(gram_kp_kernel<T, 1, A>, gram_wg<T, 1>());
        else if (csr.rbf_factored && csr.rbf_small) launch(gram_kp_kernel<T, 4, A>, gram_wg<T, 4>());
        else if (csr.rbf_factored) launch(gram_kp_kernel<T, 3, A>, gram_wg<T, 3>());
        else launch(gram_kp_kernel<T, 2, A>, gram_wg<T, 2>());
    };
    switch (gram_ablate() & 3) {  // ablations are timing-only variants (wrong results)
    case 1: pick(std::integral_constant<int, 1>{}); break;
    case 2: pick(std::integral_constant<int, 2>{}); break;
    case 3: pick(std::integral_constant<int, 3>{}); break;
    default: pick(std::integral_constant<int, 0>{});
    }
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_gram_base(int kernel, kfun<T> kf, T kappa, const T *ssc, const T *norms, const T *ev, const T *p, int64_t m,
                      T *raw, const cg_scalars<T> *status, hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(gram_base_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, kernel, kf, kappa, ssc,
                       norms, ev, p, m, raw, status);
    MI_LAUNCH_CHECK();
}

#define INST(T)                                                                                                 \
    template void launch_gram_base<T>(int, kfun<T>, T, const T *, const T *, const T *, const T *, int64_t, T *, \
                                      const cg_scalars<T> *, hipStream_t);                                      \
    template void engine<T>::setup_csr(const int64_t *, const int32_t *, const void *, int, int64_t, int64_t); \
    template void engine<T>::build_gram_blocks(const int64_t *, int64_t);                                     \
    template void engine<T>::sparse_q();                                                                      \
    template void engine<T>::sparse_kp_raw(const T *, const cg_scalars<T> *, bool);                           \
    template void engine<T>::sparse_dominant(const T *, const cg_scalars<T> *);                               \
    template void engine<T>::spmv_pass_csc(const T *, const cg_scalars<T> *);                                 \
    template void engine<T>::spmv_pass_csr(const cg_scalars<T> *);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
