// Sparse polynomial / RBF K·p recomputed on the fly from the CSR rows: nothing per pair
// is stored, every call re-forms s_ij = x_i . x_j for the pairs that share a feature, as the reference
// recomputes every k(x_i, x_j) per call (include/plssvm/backends/HIP/svm_kernel.hip.hpp:206-268;
// src/plssvm/backends/OpenMP/svm_kernel.cpp:21-47). The fallback when neither stored structure (the kernel
// expansion's remainder, the Gram pattern) fits the device, below the density where the densified MFMA
// tiles win.
//
// One wave owns one row i and an LDS row of CW partner accumulators. For each window of CW partners it
// walks the CSC segments of row i's features restricted to that window (segment table seg[f][W]),
// lanes over the segment's entries (a column holds distinct rows, so the lanes of one feature never
// collide): s[j] = fma(x_if, x_jf, s[j]) feature by feature in ascending order — the same fma chain as
// the dense dot product over the densified rows. Then the window is scanned once: every non-zero s_ij,
// j != i, contributes the pair part c_ij p_j (c_ij = k_ij - kappa_ij, the separable part kappa_ij is
// added in O(m) by gram_base_kernel, with the diagonal). Waves are independent (no barriers, no atomics),
// all sums in fixed orders: bitwise reproducible.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "../../include/plssvm_mi355x.h"
#include "engine.hpp"

namespace plssvm_mi {

namespace {

constexpr int OTF_NT = 256;   // 4 waves (rows) per workgroup; 5 workgroups per CU by LDS
#ifndef OTF_U_DEF
#define OTF_U_DEF 4  // measured (1 % density): U = 2 / 4 / 8 / 16: 0.73 / 0.59 / 0.61 / 0.82 s
#endif
#ifndef OTF_ATOMIC
#define OTF_ATOMIC 0
#endif
constexpr int OTF_U = OTF_U_DEF;  // features whose segment loads are in flight together
constexpr int OTF_BINMAX = 16;
constexpr int OTF_SCAN = 8;  // scan steps (64 partners each) whose partner loads are in flight together

// a CSC entry (row j, value) as one aligned vector load: a short column segment touches one contiguous
// range instead of two (the row and value arrays)
template <typename T>
struct alignas(2 * sizeof(T)) otf_jv {
    int32_t j;
    T v;
};

template <typename T>
__global__ __launch_bounds__(256) void otf_jv_kernel(const int32_t *__restrict__ crow, const T *__restrict__ cval,
                                                     int64_t nnz, otf_jv<T> *__restrict__ cjv) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nnz) cjv[t] = otf_jv<T>{ crow[t], cval[t] };
}

// a partner's p_j, |x_j|^2 and e_j packed for one vector load in the window scan (rebuilt per K·p)
template <typename T>
struct alignas(4 * sizeof(T)) pne_t {
    T p, n, e, pad;
};

template <typename T>
__global__ __launch_bounds__(256) void otf_pack_kernel(const T *__restrict__ p, const T *__restrict__ norms,
                                                       const T *__restrict__ ev, int64_t m, pne_t<T> *__restrict__ pne,
                                                       const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t j = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) pne[j] = pne_t<T>{ p[j], norms[j], ev != nullptr ? ev[j] : T(1), T(0) };
}

// partner accumulators per wave: CWB bytes (8 KiB; 16 / 32 KiB measured 1.06x / 2.3x slower — fewer waves —, 4 KiB
// 1.9x slower)
template <typename T, int CWB>
constexpr int otf_cw() { return CWB / (int) sizeof(T); }
constexpr int OTF_CWB = 8192;
inline int otf_cwb() { return OTF_CWB; }

// pair part c_ij = k_ij - kappa_ij for s_ij != 0 (the Gram pattern's forms, sparse.hip)
template <typename T>
struct otf_pair {
    int kernel;  // 0 linear (pairwise mode), 1 poly, 2 rbf
    int form;    // rbf: 0 factored e_i e_j expm1(2 g s), 1 direct; poly: 0 binomial, 1 direct
    int deg;
    T g, c0, kappa;
    T bin[OTF_BINMAX + 1];  // poly binomial form: c = sum_k bin[k] s^k, bin[k] = C(deg,k) c0^(deg-k) g^k
};

template <typename T>
__device__ __forceinline__ T otf_c(const otf_pair<T> &pf, T s, T ni, T nj, T ei, T ej) {
    if (pf.kernel == 0) return s;
    if (pf.kernel == 2) {
        if (pf.form == 0) return ei * ej * expm1(T(2) * pf.g * s);
        T dist = ni + nj - T(2) * s;
        dist = dist > T(0) ? dist : T(0);
        return exp(-pf.g * dist) - ei * ej;
    }
    if (pf.form == 0) {
        T h = T(0);
        for (int k = pf.deg; k >= 1; --k) h = (h + pf.bin[k]) * s;
        return h;
    }
    const T base = fma(pf.g, s, pf.c0);
    T r = T(1);
    for (int e = 0; e < pf.deg; ++e) r *= base;
    return r - pf.kappa;
}

__device__ __forceinline__ int rl32(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ int64_t rl64(int64_t x, int l) {
    const int lo = __builtin_amdgcn_readlane((int) (uint32_t) x, l);
    const int hi = __builtin_amdgcn_readlane((int) (x >> 32), l);
    return (int64_t) (((uint64_t) (uint32_t) hi << 32) | (uint32_t) lo);
}
__device__ __forceinline__ float rlT(float x, int l) { return __int_as_float(rl32(__float_as_int(x), l)); }
__device__ __forceinline__ double rlT(double x, int l) { return __longlong_as_double(rl64(__double_as_longlong(x), l)); }

// seg[f][W] = (first entry of column f with row >= W CW, column-local; #entries with row in window W), so one
// aligned 8-byte load gives a feature's segment of a window (CSC rows ascending inside a column)
__global__ __launch_bounds__(256) void otf_seg_kernel(const int64_t *__restrict__ colptr,
                                                      const int32_t *__restrict__ crow, int64_t d, int64_t nW,
                                                      int64_t CW, int2 *__restrict__ seg) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nW * d) return;
    const int64_t f = t / nW, W = t - f * nW;
    const int64_t a = colptr[f], b = colptr[f + 1];
    auto first_at_least = [&](int64_t key) {
        int64_t lo = a, hi = b;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t) crow[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const int64_t lo = first_at_least(W * CW), hi = first_at_least((W + 1) * CW);
    seg[t] = make_int2((int) (lo - a), (int) (hi - lo));
}

// ecb[k] = colptr[col[k]]: the CSC start of each CSR entry's column (read coalesced with the row)
__global__ __launch_bounds__(256) void otf_ecb_kernel(const int64_t *__restrict__ colptr, const int32_t *__restrict__ col,
                                                      int64_t nnz, int64_t *__restrict__ ecb) {
    const int64_t k = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nnz) ecb[k] = colptr[col[k]];
}

// s += a in LDS: read-add-write (the lanes of one feature never share a j; one wave's LDS operations
// complete in issue order). OTF_ATOMIC = 1 uses no-return LDS atomic adds instead: measured 1.4x (1 %
// density) to 2.7x (5 %) slower on gfx950.
template <typename T>
__device__ __forceinline__ void otf_add(T *a, T v) {
#if OTF_ATOMIC
    __hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
#else
    *a += v;
#endif
}

// One batch of up to 64 features of row i against the partner window [j0, j0 + CW): lane k holds feature
// k's segment (absolute CSC start lo, length len) and value v. Groups of OTF_U features; the next group's
// loads (first 64 entries of each segment) are issued before the current group's updates, so one memory
// latency per group is overlapped with the previous group's LDS work (straight-line: a past-the-end group
// loads entry 0 with length 0). A longer segment's further entries follow right after its first 64, so
// every s_ij accumulates its features in ascending order.
template <typename T>
__device__ __forceinline__ void otf_batch(T *__restrict__ s, const otf_jv<T> *__restrict__ cjv, int j0, int nk,
                                          int64_t lo, int len, T v,
                                          int lane) {
    int64_t lo_c[OTF_U], lo_n[OTF_U];
    int len_c[OTF_U], len_n[OTF_U], jj_c[OTF_U], jj_n[OTF_U];
    T v_c[OTF_U], v_n[OTF_U], vv_c[OTF_U], vv_n[OTF_U];
    auto fetch = [&](int u, int64_t *lo_x, int *len_x, T *v_x, int *jj_x, T *vv_x) {
#pragma unroll
        for (int x = 0; x < OTF_U; ++x) {
            const int src = u + x < nk ? u + x : 0;
            lo_x[x] = rl64(lo, src);
            len_x[x] = u + x < nk ? rl32(len, src) : 0;
            v_x[x] = rlT(v, src);
            const int64_t t = lane < len_x[x] ? lo_x[x] + lane : 0;
            const otf_jv<T> e = cjv[t];  // raw load: validity is tested at the update, not here (keeps it in flight)
            jj_x[x] = e.j;
            vv_x[x] = e.v;
        }
    };
    fetch(0, lo_c, len_c, v_c, jj_c, vv_c);
    for (int u = 0; u < nk; u += OTF_U) {
        fetch(u + OTF_U, lo_n, len_n, v_n, jj_n, vv_n);
#pragma unroll
        for (int x = 0; x < OTF_U; ++x) {
            if (lane < len_c[x]) otf_add(s + (jj_c[x] - j0), v_c[x] * vv_c[x]);
            for (int o = 64; o < len_c[x]; o += 64) {  // segments longer than a wave (dense columns)
                if (o + lane < len_c[x]) {
                    const int64_t t = lo_c[x] + o + lane;
                    const otf_jv<T> e = cjv[t];
                    otf_add(s + (e.j - j0), v_c[x] * e.v);
                }
            }
        }
#pragma unroll
        for (int x = 0; x < OTF_U; ++x) {
            lo_c[x] = lo_n[x], len_c[x] = len_n[x], v_c[x] = v_n[x], jj_c[x] = jj_n[x], vv_c[x] = vv_n[x];
        }
    }
}

#ifndef OTF_V2
#define OTF_V2 1  // segment loads through per-feature buffer descriptors (0: per-lane 64-bit addresses)
#endif

// A feature's segment through a buffer descriptor whose base is the segment's first entry and whose size
// is its byte length: lane l reads entry o + l at the constant offset (o + l) * sizeof(entry), lanes past
// the end read zeros without touching memory, and the descriptor is built from wave-uniform values with
// scalar instructions — no per-lane address arithmetic or past-the-end clamping per feature.
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t otf_seg_rsrc(const otf_jv<T> *cjv, int64_t lo, int len) {
    return __builtin_amdgcn_make_buffer_rsrc((void *) (cjv + lo), (short) 0, len * (int) sizeof(otf_jv<T>), 0x00020000);
}
template <typename T>
__device__ __forceinline__ otf_jv<T> otf_seg_load(__amdgpu_buffer_rsrc_t rs, int k) {
    if constexpr (sizeof(T) == 4) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b64(rs, k * 8, 0, 0);
        return otf_jv<T>{ (int32_t) r[0], __uint_as_float(r[1]) };
    } else {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, k * 16, 0, 0);
        return otf_jv<T>{ (int32_t) r[0], __longlong_as_double((long long) (((uint64_t) r[3] << 32) | r[2])) };
    }
}

// otf_batch with the segments read through otf_seg_rsrc and the prefetch ping-ponged between two register
// sets (no loop-carried copies that wait for the loads): the same entries, updates and update order
template <typename T>
__device__ __forceinline__ void otf_batch2(T *__restrict__ s, const otf_jv<T> *__restrict__ cjv, int j0, int nk,
                                           int64_t lo, int len, T v, int lane) {
    struct grp {
        __amdgpu_buffer_rsrc_t rs[OTF_U];
        int len[OTF_U];
        T v[OTF_U];
        otf_jv<T> e[OTF_U];
    };
    T *sb = s - j0;  // s[j - j0]
    nk = __builtin_amdgcn_readfirstlane(nk);
    auto fetch = [&](grp &g, int u) {
#pragma unroll
        for (int x = 0; x < OTF_U; ++x) {
            const int k = (u + x) & 63;  // past the batch: a zero-length segment (nothing is read)
            const int n = u + x < nk ? rl32(len, k) : 0;
            g.len[x] = n;
            g.v[x] = rlT(v, k);
            g.rs[x] = otf_seg_rsrc<T>(cjv, rl64(lo, k), n);
            g.e[x] = otf_seg_load<T>(g.rs[x], lane);
        }
    };
    auto process = [&](const grp &g) {
#pragma unroll
        for (int x = 0; x < OTF_U; ++x) {
            if (lane < g.len[x]) otf_add(sb + g.e[x].j, g.v[x] * g.e[x].v);
            for (int o = 64; o < g.len[x]; o += 64) {  // segments longer than a wave (dense columns)
                const otf_jv<T> e = otf_seg_load<T>(g.rs[x], o + lane);
                if (o + lane < g.len[x]) otf_add(sb + e.j, g.v[x] * e.v);
            }
        }
    };
    grp A, B;
    fetch(A, 0);
    for (int u = 0; u < nk; u += 2 * OTF_U) {
        fetch(B, u + OTF_U);
        process(A);
        if (u + OTF_U >= nk) break;  // wave-uniform
        fetch(A, u + 2 * OTF_U);
        process(B);
    }
}

// raw[i] = sum_{j != i, s_ij != 0} c_ij p_j for this rank's rows i in [r0, r1)
template <typename T, int CWB>
__global__ __launch_bounds__(OTF_NT) void otf_kp_kernel(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
                                                        const T *__restrict__ val, const int64_t *__restrict__ ecb,
                                                        const otf_jv<T> *__restrict__ cjv, const int2 *__restrict__ seg, const T *__restrict__ norms,
                                                        const T *__restrict__ ev, const pne_t<T> *__restrict__ pne, int64_t m,
                                                        int64_t nW, int64_t r0, int64_t r1, otf_pair<T> pf,
                                                        int64_t Wa, int64_t Wb, double *__restrict__ part,
                                                        T *__restrict__ raw, const cg_scalars<T> *__restrict__ status) {
    constexpr int CW = otf_cw<T, CWB>();
    __shared__ T S[OTF_NT / 64][CW];
    if (status != nullptr && status->converged) return;
    // wave-uniform row (scalar loads of its row pointers, counts and segment descriptors)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int64_t i = r0 + (int64_t) blockIdx.x * (OTF_NT / 64) + wave;
    if (i >= r1) return;  // waves never synchronise: each owns its accumulator row
    T *s = S[wave];
    for (int t = lane; t < CW; t += 64) s[t] = T(0);
    const int64_t b0 = rowptr[i], nz = rowptr[i + 1] - b0;
    const T ni = norms[i], ei = ev != nullptr ? ev[i] : T(1);
    // the row's first 64 features stay in registers across the windows (feature, value, column start), and
    // their next window's segments are loaded one window ahead
    const bool h0 = lane < nz;
    const int32_t f0 = h0 ? col[b0 + lane] : 0;
    const T v0 = h0 ? val[b0 + lane] : T(0);
    const int64_t c0 = h0 ? ecb[b0 + lane] : 0;
    int2 sg0 = h0 ? seg[(int64_t) f0 * nW + Wa] : make_int2(0, 0);
    double acc = 0.0;
    for (int64_t W = Wa; W < Wb; ++W) {
        const int j0 = (int) (W * CW);
        if (nz > 0) {
            const int2 sg = sg0;
            sg0 = h0 && W + 1 < Wb ? seg[(int64_t) f0 * nW + W + 1] : make_int2(0, 0);
            if constexpr (OTF_V2) otf_batch2<T>(s, cjv, j0, (int) (nz < 64 ? nz : 64), c0 + sg.x, sg.y, v0, lane);
            else otf_batch<T>(s, cjv, j0, (int) (nz < 64 ? nz : 64), c0 + sg.x, sg.y, v0, lane);
        }
        for (int64_t q0 = 64; q0 < nz; q0 += 64) {  // further features: reloaded per window
            const int64_t k = q0 + lane;
            int64_t lo = 0;
            int len = 0;
            T v = T(0);
            if (k < nz) {
                const int32_t f = col[b0 + k];
                v = val[b0 + k];
                const int2 sg = seg[(int64_t) f * nW + W];
                lo = ecb[b0 + k] + sg.x;
                len = sg.y;
            }
            if constexpr (OTF_V2) otf_batch2<T>(s, cjv, j0, (int) (nz - q0 < 64 ? nz - q0 : 64), lo, len, v, lane);
            else otf_batch<T>(s, cjv, j0, (int) (nz - q0 < 64 ? nz - q0 : 64), lo, len, v, lane);
        }
        // the window's pair terms, lane-strided (fixed order); the accumulators are left zeroed. The partners'
        // (p_j, |x_j|^2, e_j) come as one packed load per lane, OTF_SCAN steps issued before their use (the
        // loads do not depend on s_ij: one memory latency per OTF_SCAN steps, not per step)
        for (int t0 = 0; t0 < CW; t0 += 64 * OTF_SCAN) {
            T sv[OTF_SCAN];
            pne_t<T> q[OTF_SCAN];
#pragma unroll
            for (int u = 0; u < OTF_SCAN; ++u) {
                const int t = t0 + 64 * u + lane;
                sv[u] = s[t];
                const int64_t j = j0 + t;
                q[u] = pne[j < m ? j : m - 1];
            }
#pragma unroll
            for (int u = 0; u < OTF_SCAN; ++u) {
                if (sv[u] != T(0)) {
                    const int t = t0 + 64 * u + lane;
                    s[t] = T(0);
                    if (j0 + t != i) acc += (double) otf_c<T>(pf, sv[u], ni, q[u].n, ei, q[u].e) * (double) q[u].p;
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) {  // windows [Wa, Wb) of a K·p split over launches: partial sums in window order
        if (Wa > 0) acc += part[i];
        if (Wb == nW) raw[i] = (T) acc;
        else part[i] = acc;
    }
}

}  // namespace

// device bytes and an estimated time (s) of one on-the-fly K·p share, from the host CSR / CSC counts
template <typename T>
double engine<T>::otf_estimate_s(const int64_t *rowptr, const int32_t *col, const std::vector<int64_t> &colptr) const {
    const int64_t CW = otf_cwb() / (int64_t) sizeof(T), nW = ceil_div(std::max<int64_t>(m, 1), CW);
    double fill = 0.0;  // column-segment entries walked: sum over the rank's entries of their column length
    for (int64_t k = rowptr[r0]; k < rowptr[r1]; ++k) fill += (double) (colptr[col[k] + 1] - colptr[col[k]]);
    const double nnz_r = (double) (rowptr[r1] - rowptr[r0]), R = (double) (r1 - r0);
    // fitted on the box (fp32 RBF, 0.1-5 % density): segment entries, per-(entry, window)
    // segment set-up, and the LDS scan of every (row, window) partner
    const double es = (double) sizeof(T) / 4.0;
    return es * (fill * 4.0e-13 + nnz_r * (double) nW * 5.0e-11 + R * (double) m * 1.33e-12);
}

template <typename T>
void engine<T>::setup_otf(int rbf_fact_ok) {
    const int64_t CW = otf_cwb() / (int64_t) sizeof(T);
    csr.otf_cw = (int) CW;
    csr.otf_nw = ceil_div(std::max<int64_t>(m, 1), CW);
    const int64_t tot = csr.otf_nw * d;
    csr.seg.alloc(std::max<int64_t>(tot, 1), stream, false);
    if (tot > 0)
        hipLaunchKernelGGL(otf_seg_kernel, dim3((unsigned) ceil_div(tot, 256)), dim3(256), 0, stream, csr.colptr.get(),
                           csr.crow.get(), d, csr.otf_nw, CW, csr.seg.get());
    MI_LAUNCH_CHECK();
    csr.pne.alloc(4 * std::max<int64_t>(m, 1), stream, false);
    csr.otf_part.alloc(std::max<int64_t>(m, 1), stream, false);
    csr.cjv.alloc(2 * std::max<int64_t>(csr.nnz, 1), stream, false);
    if (csr.nnz > 0)
        hipLaunchKernelGGL(otf_jv_kernel<T>, dim3((unsigned) ceil_div(csr.nnz, 256)), dim3(256), 0, stream,
                           csr.crow.get(), csr.cval.get(), csr.nnz, reinterpret_cast<otf_jv<T> *>(csr.cjv.get()));
    MI_LAUNCH_CHECK();
    csr.ecb.alloc(std::max<int64_t>(csr.nnz, 1), stream, false);
    if (csr.nnz > 0)
        hipLaunchKernelGGL(otf_ecb_kernel, dim3((unsigned) ceil_div(csr.nnz, 256)), dim3(256), 0, stream,
                           csr.colptr.get(), csr.col.get(), csr.nnz, csr.ecb.get());
    MI_LAUNCH_CHECK();
    if (csr.ssc.get() == nullptr) csr.ssc.alloc(1, stream);
    csr.rbf_factored = kernel == 2 && rbf_form != 1 && rbf_fact_ok;
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    csr.otf_on = true;
}

template <typename T>
void engine<T>::otf_dominant(const T *p, const cg_scalars<T> *status) {
    if (r1 <= r0) return;
    otf_pair<T> pf{};
    pf.kernel = kernel;
    pf.deg = degree;
    pf.g = gamma;
    pf.c0 = coef0;
    T kappa = 0;
    if (kernel == 1) {
        kappa = 1;
        for (int q2 = 0; q2 < degree; ++q2) kappa *= coef0;
        pf.form = (degree >= 1 && degree <= OTF_BINMAX) ? 0 : 1;
        if (pf.form == 0) {  // C(deg, k) c0^(deg - k) g^k in double, rounded once
            for (int k = 1; k <= degree; ++k) {
                double c = 1.0;
                for (int t = 0; t < k; ++t) c = c * (double) (degree - t) / (double) (t + 1);
                pf.bin[k] = (T) (c * std::pow((double) coef0, degree - k) * std::pow((double) gamma, k));
            }
        }
    } else {
        pf.form = csr.rbf_factored ? 0 : 1;
    }
    pf.kappa = kappa;
    pne_t<T> *pne = reinterpret_cast<pne_t<T> *>(csr.pne.get());
    hipLaunchKernelGGL(otf_pack_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, p, norms.get(),
                       kernel == 2 ? csr.e.get() : nullptr, m, pne, status);
    MI_LAUNCH_CHECK();
    // all partner windows in one launch (round 3: splitting them over launches, so that every wave of the GPU works on
    // one window whose CSC segments are shared in the L2s / Infinity Cache, measured no gain at 1 % density — 1 / 4 /
    // all windows per launch 0.626 / 0.605 / 0.610 s: the segment walk is bound by its scattered L2 misses either way)
    const int64_t nW = csr.otf_nw;
    hipLaunchKernelGGL((otf_kp_kernel<T, OTF_CWB>), dim3((unsigned) ceil_div(r1 - r0, OTF_NT / 64)), dim3(OTF_NT), 0, stream,
                       csr.rowptr.get(), csr.col.get(), csr.val.get(), csr.ecb.get(),
                       reinterpret_cast<const otf_jv<T> *>(csr.cjv.get()), csr.seg.get(), norms.get(),
                       kernel == 2 ? csr.e.get() : nullptr, pne, m, nW, r0, r1, pf, (int64_t) 0, nW, csr.otf_part.get(),
                       raw.get(), status);
    MI_LAUNCH_CHECK();
}

// raw = sum_j k_ij p_j (with_base: + the separable part and the diagonal, as the Gram pattern's)
template <typename T>
void engine<T>::otf_kp_raw(const T *p, const cg_scalars<T> *status, bool with_base) {
    MI_HIP_CHECK(hipMemsetAsync(raw.get(), 0, sizeof(T) * (size_t) m, stream));
    gather_input(p);  // sharded group: the partners' p from every rank
    otf_dominant(p, status);
    if (!shard) allgather_rows(raw.get());
    if (with_base && !(sim_world > 0 && sim_rank != 0)) {
        launch_dot2<T>(p, kernel == 2 ? csr.e.get() : nullptr, nullptr, nullptr, m, red.get(), status, stream);
        launch_dot_final<T>(red.get(), sc.get(), FIN_PLAIN, 0, nullptr, 0, csr.ssc.get(), stream);
        T kappa = 0;
        if (kernel == 1) {
            kappa = 1;
            for (int q2 = 0; q2 < degree; ++q2) kappa *= coef0;
        }
        launch_gram_base<T>(kernel, kf(), kappa, csr.ssc.get(), norms.get(), csr.e.get(), p, m, raw.get(), status, stream);
    }
}

#define INST(T)                                                                                                        \
    template double engine<T>::otf_estimate_s(const int64_t *, const int32_t *, const std::vector<int64_t> &) const;   \
    template void engine<T>::setup_otf(int);                                                                           \
    template void engine<T>::otf_dominant(const T *, const cg_scalars<T> *);                                           \
    template void engine<T>::otf_kp_raw(const T *, const cg_scalars<T> *, bool);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
