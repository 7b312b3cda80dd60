// Sparse polynomial / RBF K·p by kernel expansion.
//
// For sparse data most pairs share no feature, and a pair that shares exactly one feature f has
// s_ij = x_if x_jf. Write the pair part of the kernel as a function of s:
//   rbf  (factored):  k_ij = e_i e_j (1 + E(s_ij)),   E(s) = expm1(2 g s),  e_i = exp(-g |x_i|^2)
//   poly:             k_ij = kappa + c(s_ij),          c(s) = (g s + c0)^deg - c0^deg,  kappa = c0^deg
// and let phi be E or c. Then, exactly,
//   phi(s_ij) = sum_{f shared by i, j} phi(x_if x_jf) + H_ij,
// where the remainder H_ij is non-zero only for pairs sharing two or more features (and i == j).
// phi is a polynomial (c exactly, of degree deg; E as its Taylor series, truncated at the degree K
// whose remainder is below the real type's rounding for every |2 g x_if x_jf| of the data), so the
// per-feature part of a row is separable through the column moments:
//   sum_j sum_{f shared} phi(x_if x_jf) w_j = sum_{f in x_i} sum_{k=1..K} coef_k x_if^k M_k(f),
//   M_k(f) = sum_{j in column f} x_jf^k w_j,   w_j = e_j p_j (rbf) | p_j (poly).
// One K·p = the moments (one CSC pass), a CSR pass (Horner per entry), and the stored remainder H of
// the multi-feature pairs (symmetric rows, padded to 8 slots): O(nnz K + #multi pairs) instead of the
// O(sum_f c_f^2) pairs of the Gram pattern, and O(nnz + #multi pairs) memory.
//   rbf : sum_j k_ij p_j = e_i [ S + J_i + H_ii w_i + sum_j H_ij w_j ],  S = sum_j e_j p_j
//   poly: sum_j k_ij p_j = kappa S + J_i + H_ii p_i + sum_j H_ij p_j,     S = sum_j p_j
// (J_i = the moment sum, including j = i). The reference evaluates k(x_i, x_j) for every pair from the
// dense rows (include/plssvm/backends/HIP/svm_kernel.hip.hpp:206-268); the results agree to rounding.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../../include/plssvm_mi355x.h"
#include "engine.hpp"

namespace plssvm_mi {

namespace {

// phi in double: the exact per-pair function (rbf: expm1(2 g a); poly: sum_k bin_k a^k, no cancellation)
struct phi_fn {
    int rbf = 0, deg = 0;
    double g2 = 0.0;                   // rbf: 2 g
    double bin[EXP_KMAX + 1] = {};     // poly: C(deg, k) c0^(deg - k) g^k
    __host__ __device__ double operator()(double a) const {
        if (rbf) return expm1(g2 * a);
        double h = 0.0;
        for (int k = deg; k >= 1; --k) h = (h + bin[k]) * a;
        return h;
    }
};

struct coefs {
    double c[EXP_KMAX + 1];
};

struct d2sum {
    __host__ __device__ double2 operator()(const double2 &a, const double2 &b) const {
        return make_double2(a.x + b.x, a.y + b.y);
    }
};

struct hpair {
    uint64_t key;  // (row - i0) << 32 | j
    double h;
};

// keep pairs with a non-zero remainder (in the real type) that touch this rank's rows
struct h_keep {
    int64_t i0, r0, r1;
    int f32;
    __host__ __device__ bool operator()(const hpair &p) const {
        if (f32 ? ((float) p.h == 0.0f) : (p.h == 0.0)) return false;
        const int64_t i = i0 + (int64_t) (p.key >> 32), j = (int64_t) (p.key & 0xFFFFFFFFull);
        return (i >= r0 && i < r1) || (j >= r0 && j < r1);
    }
};

// incidences of row i: sum over its entries e of #{ j < i in column col[e] }
__global__ __launch_bounds__(256) void exp_count_kernel(const int64_t *__restrict__ rowptr,
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

// one workgroup per row i: every incidence (i, j < i, f) -> key (i - i0, j), value (a, phi(a)), a = x_if x_jf
template <typename T>
__global__ __launch_bounds__(256) void exp_gen_kernel(const int64_t *__restrict__ rowptr,
                                                      const int32_t *__restrict__ col, const T *__restrict__ val,
                                                      const int64_t *__restrict__ cpos,
                                                      const int64_t *__restrict__ colptr,
                                                      const int32_t *__restrict__ crow, const T *__restrict__ cval,
                                                      int64_t i0, const int64_t *__restrict__ off,
                                                      uint64_t *__restrict__ keys, double2 *__restrict__ vals,
                                                      phi_fn phi) {
    const int64_t i = i0 + blockIdx.x;
    const uint64_t il = (uint64_t) blockIdx.x;
    int64_t out = off[blockIdx.x];
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const int64_t c0 = colptr[col[k]], c1 = cpos[k];
        const double xi = (double) val[k];
        for (int64_t t = c0 + threadIdx.x; t < c1; t += blockDim.x) {
            const double a = xi * (double) cval[t];
            keys[out + (t - c0)] = (il << 32) | (uint64_t) (uint32_t) crow[t];
            vals[out + (t - c0)] = make_double2(a, phi(a));
        }
        out += c1 - c0;
    }
}

// remainder of every unique pair: H = phi(s) - sum_f phi(a_f)  (0 for single-feature pairs)
__global__ __launch_bounds__(256) void exp_h_kernel(const uint64_t *__restrict__ ukeys, const double2 *__restrict__ agg,
                                                    const int64_t *__restrict__ nruns, phi_fn phi,
                                                    hpair *__restrict__ out) {
    const int64_t u = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= *nruns) return;
    const double2 v = agg[u];
    out[u] = hpair{ ukeys[u], phi(v.x) - v.y };
}

template <typename T>
__global__ __launch_bounds__(256) void exp_append_kernel(const hpair *__restrict__ sel, const int64_t *__restrict__ nsel,
                                                         int64_t i0, int32_t *__restrict__ li, int32_t *__restrict__ lj,
                                                         T *__restrict__ lh) {
    const int64_t u = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= *nsel) return;
    const hpair p = sel[u];
    li[u] = (int32_t) (i0 + (int64_t) (p.key >> 32));
    lj[u] = (int32_t) (p.key & 0xFFFFFFFFull);
    lh[u] = (T) p.h;
}

// row histograms of the kept pairs: lower part (i in [r0, r1)) and upper part (j in [r0, r1))
__global__ __launch_bounds__(256) void exp_hist_kernel(const int32_t *__restrict__ li, const int32_t *__restrict__ lj,
                                                       int64_t P, int64_t r0, int64_t r1,
                                                       unsigned long long *__restrict__ clo,
                                                       unsigned long long *__restrict__ cup,
                                                       uint32_t *__restrict__ upflag) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P) return;
    const int64_t i = li[t], j = lj[t];
    if (i >= r0 && i < r1) atomicAdd(&clo[i - r0], 1ull);
    const bool up = j >= r0 && j < r1;
    if (up) atomicAdd(&cup[j - r0], 1ull);
    upflag[t] = up ? (uint32_t) (j - r0) : 0xFFFFFFFFu;  // sort key of the upper part (others sort last)
}

__global__ __launch_bounds__(256) void exp_pad8_kernel(const unsigned long long *__restrict__ clo,
                                                       const unsigned long long *__restrict__ cup, int64_t R,
                                                       int64_t *__restrict__ cnt8) {
    const int64_t r = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (r < R) cnt8[r] = (int64_t) ((clo[r] + cup[r] + 7ull) & ~7ull);
}

// slots of row r: j = r (pads), H = 0; chunk rows
template <typename T>
__global__ __launch_bounds__(256) void exp_init_rows_kernel(const int64_t *__restrict__ off8, int64_t R, int64_t r0,
                                                            int32_t *__restrict__ hj, T *__restrict__ hv,
                                                            int32_t *__restrict__ hcrow) {
    const int64_t r = (int64_t) blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (r >= R) return;
    const int lane = threadIdx.x & 63;
    for (int64_t s = off8[r] + lane; s < off8[r + 1]; s += 64) {
        hj[s] = (int32_t) (r0 + r);
        hv[s] = T(0);
        if ((s & 7) == 0) hcrow[s >> 3] = (int32_t) (r0 + r);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void exp_place_lower_kernel(const int32_t *__restrict__ li,
                                                              const int32_t *__restrict__ lj, const T *__restrict__ lh,
                                                              int64_t P, int64_t r0, int64_t r1,
                                                              const int64_t *__restrict__ lo_start,
                                                              const int64_t *__restrict__ off8, int32_t *__restrict__ hj,
                                                              T *__restrict__ hv) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P) return;
    const int64_t i = li[t];
    if (i < r0 || i >= r1) return;
    const int64_t r = i - r0, pos = off8[r] + (t - lo_start[r]);
    hj[pos] = lj[t];
    hv[pos] = lh[t];
}

template <typename T>
__global__ __launch_bounds__(256) void exp_place_upper_kernel(const uint32_t *__restrict__ skey,
                                                              const uint32_t *__restrict__ sidx, int64_t nup,
                                                              const int32_t *__restrict__ li, const T *__restrict__ lh,
                                                              const unsigned long long *__restrict__ clo,
                                                              const int64_t *__restrict__ up_start,
                                                              const int64_t *__restrict__ off8, int32_t *__restrict__ hj,
                                                              T *__restrict__ hv) {
    const int64_t u = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nup) return;
    const int64_t r = skey[u], t = sidx[u];
    const int64_t pos = off8[r] + (int64_t) clo[r] + (u - up_start[r]);
    hj[pos] = li[t];
    hv[pos] = lh[t];
}

// H_ii = phi(|x_i|^2) - sum_f phi(x_if^2) and phi(|x_i|^2), rows 0..m-1
template <typename T>
__global__ __launch_bounds__(256) void exp_diag_kernel(const int64_t *__restrict__ rowptr, const T *__restrict__ val,
                                                       int64_t m, phi_fn phi, T *__restrict__ hdiag,
                                                       T *__restrict__ phin) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double n = 0.0, s = 0.0;
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const double x = (double) val[k], a = x * x;
        n += a;
        s += phi(a);
    }
    const double pn = phi(n);
    hdiag[i] = (T) (pn - s);
    phin[i] = (T) pn;
}

__global__ __launch_bounds__(256) void exp_iota_kernel(uint32_t *__restrict__ v, int64_t n) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) v[t] = (uint32_t) t;
}

// ---- per K·p ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void exp_w_kernel(const T *__restrict__ e, const T *__restrict__ p, int64_t m,
                                                    T *__restrict__ w, const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) w[i] = e[i] * p[i];
}

// M[f][k] = coef_{k+1} sum_{j in col f} x_jf^(k+1) w_j: one wave per column, fp64, fixed order
template <typename T, int KM>
__global__ __launch_bounds__(256) void exp_moments_kernel(const int64_t *__restrict__ colptr,
                                                          const int32_t *__restrict__ crow, const T *__restrict__ cval,
                                                          const T *__restrict__ w, int64_t d, coefs cf,
                                                          double *__restrict__ M,
                                                          const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t f = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (f >= d) return;
    const int lane = threadIdx.x & 63;
    double acc[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) acc[k] = 0.0;
    const int64_t t1 = colptr[f + 1];
    for (int64_t t = colptr[f] + lane; t < t1; t += 64) {
        const double x = (double) cval[t];
        double xp = x * (double) w[crow[t]];
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            acc[k] += xp;
            xp *= x;
        }
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        double v = acc[k];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
        acc[k] = v;
    }
    if (lane < KM) {
        double v = acc[0];
#pragma unroll
        for (int k = 1; k < KM; ++k) v = lane == k ? acc[k] : v;
        M[f * KM + lane] = cf.c[lane + 1] * v;
    }
}

// hs[i] = sum_j H_ij w_j over the stored remainder rows: each wave owns a row-aligned chunk range;
// lanes take 8-slot chunks (64 per step, coalesced), gather w_j, and the rows' partial sums are
// combined by a segmented shuffle reduction, the last row of a step carried into the next. Fixed
// order, no atomics.
template <typename T>
__global__ __launch_bounds__(256) void exp_hstream_kernel(const int64_t *__restrict__ wave_chunk, int64_t nwaves,
                                                          const int32_t *__restrict__ hcrow,
                                                          const int32_t *__restrict__ hj, const T *__restrict__ hv,
                                                          const T *__restrict__ w, T *__restrict__ hs,
                                                          const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (gw >= nwaves) return;
    const int64_t c0 = wave_chunk[gw], c1 = wave_chunk[gw + 1];
    T carry = 0;
    int carry_row = -1;
    for (int64_t cb = c0; cb < c1; cb += 64) {  // wave-uniform trip count
        const int64_t c = cb + lane;
        const bool have = c < c1;
        int rl = -1;
        T acc = 0;
        if (have) {
            rl = hcrow[c];
            const int4 ja = *reinterpret_cast<const int4 *>(hj + 8 * c);
            const int4 jb = *reinterpret_cast<const int4 *>(hj + 8 * c + 4);
            T h[8];
            if constexpr (sizeof(T) == 4) {
                const float4 a = *reinterpret_cast<const float4 *>(hv + 8 * c), b = *reinterpret_cast<const float4 *>(hv + 8 * c + 4);
                h[0] = a.x, h[1] = a.y, h[2] = a.z, h[3] = a.w, h[4] = b.x, h[5] = b.y, h[6] = b.z, h[7] = b.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const double2 v = *reinterpret_cast<const double2 *>(hv + 8 * c + 2 * q);
                    h[2 * q] = v.x, h[2 * q + 1] = v.y;
                }
            }
            const int js[8] = { ja.x, ja.y, ja.z, ja.w, jb.x, jb.y, jb.z, jb.w };
            T wj[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) wj[k] = w[js[k]];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc = fma(h[k], wj[k], acc);
        }
        // segmented suffix sums: rows are non-decreasing in lane order
        T sacc = acc;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const T so = __shfl_down(sacc, off);
            const int rr = __shfl_down(rl, off);
            if (lane + off < 64 && rr == rl) sacc += so;
        }
        const int rprev = __shfl_up(rl, 1);
        const bool head = rl >= 0 && (lane == 0 || rprev != rl);
        const int row0 = __shfl(rl, 0);
        if (carry_row >= 0 && row0 != carry_row) {  // the carried row ended at the step boundary
            if (lane == 0) hs[carry_row] = carry;
            carry_row = -1;
        }
        if (lane == 0 && carry_row >= 0) sacc += carry;
        const bool more = cb + 64 < c1;
        const int lastlane = more ? 63 : (int) (c1 - 1 - cb);
        const int rowL = __shfl(rl, lastlane);
        const unsigned long long mk = __ballot(rl == rowL);
        const int hl = __ffsll((long long) mk) - 1;
        const T segL = __shfl(sacc, hl);
        if (head && !(more && rl == rowL)) hs[rl] = sacc;
        if (more) {
            carry = segL;
            carry_row = rowL;
        } else {
            carry_row = -1;
        }
    }
}

// raw_i for rows [r0, r1) (0 elsewhere): base + scale (J_i + H_ii w_i + hs_i) [- the diagonal term when
// only the overlap part is asked for], 8 lanes per row walking the CSR entries (Horner on the moments)
template <typename T, int KM>
__global__ __launch_bounds__(256) void exp_rows_kernel(const int64_t *__restrict__ rowptr,
                                                       const int32_t *__restrict__ col, const T *__restrict__ val,
                                                       const double *__restrict__ M, const T *__restrict__ e,
                                                       const T *__restrict__ w, const T *__restrict__ hdiag,
                                                       const T *__restrict__ phin, const T *__restrict__ hs,
                                                       const T *__restrict__ ssc, T kappa, int64_t m, int64_t r0,
                                                       int64_t r1, int overlap_only, T *__restrict__ raw,
                                                       const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * 32 + (threadIdx.x >> 3);
    const int sl = threadIdx.x & 7;
    if (i >= m) return;
    if (i < r0 || i >= r1) {
        if (sl == 0) raw[i] = T(0);
        return;
    }
    double J = 0.0;
    const int64_t k1 = rowptr[i + 1];
    for (int64_t k = rowptr[i] + sl; k < k1; k += 8) {
        const double x = (double) val[k];
        const double *Mf = M + (int64_t) col[k] * KM;
        double h = Mf[KM - 1];
#pragma unroll
        for (int q = KM - 2; q >= 0; --q) h = fma(h, x, Mf[q]);
        J = fma(h, x, J);
    }
    J += __shfl_xor(J, 4);
    J += __shfl_xor(J, 2);
    J += __shfl_xor(J, 1);
    if (sl == 0) {
        const double wi = (double) w[i];
        double t = J + (double) hdiag[i] * wi + (double) hs[i];
        const double sc = e != nullptr ? (double) e[i] : 1.0;
        double v;
        if (overlap_only) {
            v = sc * (t - (double) phin[i] * wi);
        } else {
            const double base = (e != nullptr ? (double) e[i] : (double) kappa) * (double) ssc[0];
            v = base + sc * t;
        }
        raw[i] = (T) v;
    }
}

template <typename T>
phi_fn make_phi(int kernel, int degree, T gamma, T coef0) {
    phi_fn phi;
    if (kernel == 2) {
        phi.rbf = 1;
        phi.g2 = 2.0 * (double) gamma;
    } else {
        phi.deg = degree;
        double binom = 1.0;
        for (int k = 1; k <= degree && k <= EXP_KMAX; ++k) {
            binom = binom * (double) (degree - k + 1) / (double) k;
            phi.bin[k] = binom * std::pow((double) coef0, (double) (degree - k)) * std::pow((double) gamma, (double) k);
        }
    }
    return phi;
}

}  // namespace

// Can the expansion represent this kernel to rounding? rbf (factored form): the Taylor degree K of
// E(a) = expm1(2 g a) whose remainder |u|^K e^{2|u|} / (K+1)! is below 2^-27 (fp32) / 2^-56 (fp64)
// relative for every |u| = |2 g x_if x_jf| <= umax; poly: K = degree (exact). K <= EXP_KMAX.
template <typename T>
bool engine<T>::expansion_eligible() {
    auto &ex = csr.ex;
    std::fill(std::begin(ex.coef), std::end(ex.coef), 0.0);
    if (kernel == 1) {
        if (degree < 0 || degree > EXP_KMAX) return false;
        const phi_fn phi = make_phi<T>(kernel, degree, gamma, coef0);
        ex.K = degree;
        for (int k = 1; k <= degree; ++k) ex.coef[k] = phi.bin[k];
    } else if (kernel == 2) {
        if (rbf_form == 1) return false;
        const double umax = ex.umax;
        const double tol = sizeof(T) == 4 ? std::ldexp(1.0, -27) : std::ldexp(1.0, -56);
        int K = 1;
        double fact = 2.0;  // (K + 1)!
        while (K <= EXP_KMAX && std::pow(umax, K) * std::exp(2.0 * umax) / fact > tol) {
            ++K;
            fact *= (double) (K + 1);
        }
        if (K > EXP_KMAX) return false;
        ex.K = K;
        double c = 1.0;  // (2 g)^k / k!
        for (int k = 1; k <= K; ++k) {
            c = c * 2.0 * (double) gamma / (double) k;
            ex.coef[k] = c;
        }
    } else {
        return false;
    }
    ex.KM = ex.K <= 4 ? 4 : (ex.K <= 8 ? 8 : 16);
    return true;
}

// Setup: the remainder H of the pairs sharing >= 2 features, from the column join (sort +
// reduce-by-key of (a, phi(a)) per pair), as symmetric rows [r0, r1); H_ii; the moment buffers.
template <typename T>
void engine<T>::build_expansion(const int64_t *cpos, int64_t /*max_inc*/) {
    auto &ex = csr.ex;
    const phi_fn phi = make_phi<T>(kernel, degree, gamma, coef0);
    ex.M.alloc(std::max<int64_t>(d, 1) * ex.KM, stream);
    csr.ssc.alloc(2, stream);  // device scalar S = sum_j w_j
    ex.hdiag.alloc(n_pad, stream);
    ex.hs.alloc(n_pad, stream);
    ex.wv.alloc(kernel == 2 ? n_pad : 1, stream);
    ex.phin.alloc(n_pad, stream);
    if (m > 0)
        hipLaunchKernelGGL(exp_diag_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, csr.rowptr.get(),
                           csr.val.get(), m, phi, ex.hdiag.get(), ex.phin.get());
    MI_LAUNCH_CHECK();

    // ---- incidences per row (host) -> row sub-blocks of at most CAP incidences ----
    std::vector<int64_t> inc(std::max<int64_t>(m, 1), 0);
    {
        dev_buf<int64_t> cnt;
        cnt.alloc(std::max<int64_t>(m, 1), stream);
        if (m > 0)
            hipLaunchKernelGGL(exp_count_kernel, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream,
                               csr.rowptr.get(), csr.col.get(), cpos, csr.colptr.get(), (int64_t) 0, m, cnt.get());
        MI_LAUNCH_CHECK();
        if (m > 0)
            MI_HIP_CHECK(hipMemcpyAsync(inc.data(), cnt.get(), sizeof(int64_t) * (size_t) m, hipMemcpyDeviceToHost,
                                        stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
    constexpr int64_t CAP = int64_t(1) << 27;      // incidences per sub-block (48 B each in flight)
    constexpr int64_t ROWS_MAX = 65536;            // rows per sub-block (one workgroup per row)
    std::vector<std::pair<int64_t, int64_t>> blocks;
    {
        int64_t a = r0, acc = 0;  // pairs (i, j < i) touch rows [r0, r1) only if i >= r0
        for (int64_t i = r0; i < m; ++i) {
            if (inc[i] > CAP) throw mi_error(-4, "a data point shares features with more than 2^27 others (dense row)");
            if (i > a && (acc + inc[i] > CAP || i - a >= ROWS_MAX)) {
                blocks.emplace_back(a, i);
                a = i;
                acc = 0;
            }
            acc += inc[i];
        }
        if (a < m) blocks.emplace_back(a, m);
    }
    int64_t max_blk = 1;
    for (auto &b : blocks) {
        int64_t s = 0;
        for (int64_t i = b.first; i < b.second; ++i) s += inc[i];
        max_blk = std::max(max_blk, s);
    }

    // ---- temporaries ----
    dev_buf<uint64_t> keys, keys_s;
    dev_buf<double2> vals, vals_s;
    dev_buf<hpair> hp, hsel;
    dev_buf<int64_t> cntb, off, nruns, nsel;
    keys.alloc(max_blk, stream, false);
    keys_s.alloc(max_blk, stream, false);
    vals.alloc(max_blk, stream, false);
    vals_s.alloc(max_blk, stream, false);
    cntb.alloc(ROWS_MAX + 1, stream);
    off.alloc(ROWS_MAX + 1, stream);
    nruns.alloc(1, stream);
    nsel.alloc(1, stream);
    size_t tmp_sort = 0, tmp_scan = 0, tmp_red = 0, tmp_sel = 0;
    const int nmax = (int) max_blk;
    MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_sort, keys.get(), keys_s.get(), vals.get(),
                                                    vals_s.get(), nmax, 0, 64, stream));
    MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_scan, cntb.get(), off.get(), (int) (ROWS_MAX + 1), stream));
    MI_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(nullptr, tmp_red, keys_s.get(), keys.get(), vals_s.get(), vals.get(),
                                                   nruns.get(), d2sum(), nmax, stream));
    hp.alloc(max_blk, stream, false);
    hsel.alloc(max_blk, stream, false);
    MI_HIP_CHECK(hipcub::DeviceSelect::If(nullptr, tmp_sel, hp.get(), hsel.get(), nsel.get(), nmax,
                                          h_keep{ 0, r0, r1, sizeof(T) == 4 }, stream));
    dev_buf<unsigned char> tmp;
    tmp.alloc((int64_t) std::max({ tmp_sort, tmp_scan, tmp_red, tmp_sel, (size_t) 16 }), stream, false);

    // growable list of kept lower pairs (li > lj), in (li, lj) order
    dev_buf<int32_t> Li, Lj;
    dev_buf<T> Lh;
    int64_t P = 0, cap = 0;
    auto grow = [&](int64_t need) {
        if (need <= cap) return;
        const int64_t nc = std::max<int64_t>(need, cap + cap / 2 + 1024);
        dev_buf<int32_t> ni, nj;
        dev_buf<T> nh;
        ni.alloc(nc, stream, false);
        nj.alloc(nc, stream, false);
        nh.alloc(nc, stream, false);
        if (P > 0) {
            MI_HIP_CHECK(hipMemcpyAsync(ni.get(), Li.get(), sizeof(int32_t) * (size_t) P, hipMemcpyDeviceToDevice, stream));
            MI_HIP_CHECK(hipMemcpyAsync(nj.get(), Lj.get(), sizeof(int32_t) * (size_t) P, hipMemcpyDeviceToDevice, stream));
            MI_HIP_CHECK(hipMemcpyAsync(nh.get(), Lh.get(), sizeof(T) * (size_t) P, hipMemcpyDeviceToDevice, stream));
        }
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        Li = std::move(ni);
        Lj = std::move(nj);
        Lh = std::move(nh);
        cap = nc;
    };
    for (auto &b : blocks) {
        const int64_t i0 = b.first, rows = b.second - b.first;
        int64_t total = 0;
        for (int64_t i = b.first; i < b.second; ++i) total += inc[i];
        if (total == 0) continue;
        hipLaunchKernelGGL(exp_count_kernel, dim3((unsigned) ceil_div(rows, 256)), dim3(256), 0, stream,
                           csr.rowptr.get(), csr.col.get(), cpos, csr.colptr.get(), i0, b.second, cntb.get());
        MI_LAUNCH_CHECK();
        size_t ts = tmp_scan;
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.get(), ts, cntb.get(), off.get(), (int) (rows + 1), stream));
        hipLaunchKernelGGL(exp_gen_kernel<T>, dim3((unsigned) rows), dim3(256), 0, stream, csr.rowptr.get(), csr.col.get(),
                           csr.val.get(), cpos, csr.colptr.get(), csr.crow.get(), csr.cval.get(), i0, off.get(),
                           keys.get(), vals.get(), phi);
        MI_LAUNCH_CHECK();
        const int end_bit = 32 + std::max(1, (int) std::ceil(std::log2((double) rows + 1.0)));
        size_t t1s = tmp_sort;
        MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.get(), t1s, keys.get(), keys_s.get(), vals.get(),
                                                        vals_s.get(), (int) total, 0, end_bit, stream));
        size_t t2s = tmp_red;
        MI_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(tmp.get(), t2s, keys_s.get(), keys.get(), vals_s.get(),
                                                       vals.get(), nruns.get(), d2sum(), (int) total, stream));
        hipLaunchKernelGGL(exp_h_kernel, dim3((unsigned) ceil_div(total, 256)), dim3(256), 0, stream, keys.get(),
                           vals.get(), nruns.get(), phi, hp.get());
        MI_LAUNCH_CHECK();
        int64_t nu = 0;
        MI_HIP_CHECK(hipMemcpyAsync(&nu, nruns.get(), sizeof(int64_t), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        size_t t3s = tmp_sel;
        MI_HIP_CHECK(hipcub::DeviceSelect::If(tmp.get(), t3s, hp.get(), hsel.get(), nsel.get(), (int) nu,
                                              h_keep{ i0, r0, r1, sizeof(T) == 4 }, stream));
        int64_t ns = 0;
        MI_HIP_CHECK(hipMemcpyAsync(&ns, nsel.get(), sizeof(int64_t), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        if (ns == 0) continue;
        grow(P + ns);
        hipLaunchKernelGGL(exp_append_kernel<T>, dim3((unsigned) ceil_div(ns, 256)), dim3(256), 0, stream, hsel.get(),
                           nsel.get(), i0, Li.get() + P, Lj.get() + P, Lh.get() + P);
        MI_LAUNCH_CHECK();
        P += ns;
    }
    keys.reset(), keys_s.reset(), vals.reset(), vals_s.reset(), hp.reset(), hsel.reset(), tmp.reset();
    if (P > INT32_MAX) throw mi_error(-5, "more than 2^31 multi-feature pairs on one rank: use more GPUs");

    // ---- symmetric rows [r0, r1), padded to 8 slots ----
    const int64_t R = r1 - r0;
    dev_buf<unsigned long long> clo, cup;
    dev_buf<int64_t> cnt8, off8, lo_start, up_start;
    dev_buf<uint32_t> ukey, ukey_s, uidx, uidx_s;
    clo.alloc(std::max<int64_t>(R, 1), stream);
    cup.alloc(std::max<int64_t>(R, 1), stream);
    cnt8.alloc(R + 1, stream);
    off8.alloc(R + 1, stream);
    lo_start.alloc(R + 1, stream);
    up_start.alloc(R + 1, stream);
    ukey.alloc(std::max<int64_t>(P, 1), stream, false);
    if (P > 0) {
        hipLaunchKernelGGL(exp_hist_kernel, dim3((unsigned) ceil_div(P, 256)), dim3(256), 0, stream, Li.get(), Lj.get(), P,
                           r0, r1, clo.get(), cup.get(), ukey.get());
        MI_LAUNCH_CHECK();
    }
    if (R > 0) {
        hipLaunchKernelGGL(exp_pad8_kernel, dim3((unsigned) ceil_div(R, 256)), dim3(256), 0, stream, clo.get(), cup.get(),
                           R, cnt8.get());
        MI_LAUNCH_CHECK();
    }
    {
        size_t ta = 0, tb = 0, tc = 0;  // each scan queries its own temporary size (types differ)
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, ta, cnt8.get(), off8.get(), (int) (R + 1), stream));
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, clo.get(), lo_start.get(), (int) R, stream));
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tc, cup.get(), up_start.get(), (int) R, stream));
        dev_buf<unsigned char> t;
        t.alloc((int64_t) std::max({ ta, tb, tc, (size_t) 16 }), stream, false);
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(t.get(), ta, cnt8.get(), off8.get(), (int) (R + 1), stream));
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(t.get(), tb, clo.get(), lo_start.get(), (int) R, stream));
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(t.get(), tc, cup.get(), up_start.get(), (int) R, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
    ex.pairs = 0;
    {
        // rows' lower pairs are the list's prefix (sorted by li); count them
        std::vector<unsigned long long> hlo(std::max<int64_t>(R, 1), 0);
        if (R > 0)
            MI_HIP_CHECK(hipMemcpyAsync(hlo.data(), clo.get(), sizeof(unsigned long long) * (size_t) R,
                                        hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        for (int64_t r = 0; r < R; ++r) ex.pairs += (int64_t) hlo[r];
    }
    std::vector<int64_t> hoff(R + 1, 0);
    MI_HIP_CHECK(hipMemcpyAsync(hoff.data(), off8.get(), sizeof(int64_t) * (size_t) (R + 1), hipMemcpyDeviceToHost, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    ex.slots = hoff[R];
    ex.nchunks = ex.slots / 8;
    ex.hj.alloc(std::max<int64_t>(ex.slots, 8), stream, false);
    ex.hv.alloc(std::max<int64_t>(ex.slots, 8), stream);
    ex.hcrow.alloc(std::max<int64_t>(ex.nchunks, 1), stream, false);
    if (R > 0) {
        hipLaunchKernelGGL(exp_init_rows_kernel<T>, dim3((unsigned) ceil_div(R, 4)), dim3(256), 0, stream, off8.get(), R,
                           r0, ex.hj.get(), ex.hv.get(), ex.hcrow.get());
        MI_LAUNCH_CHECK();
    }
    if (P > 0) {
        hipLaunchKernelGGL(exp_place_lower_kernel<T>, dim3((unsigned) ceil_div(P, 256)), dim3(256), 0, stream, Li.get(),
                           Lj.get(), Lh.get(), P, r0, r1, lo_start.get(), off8.get(), ex.hj.get(), ex.hv.get());
        MI_LAUNCH_CHECK();
        // upper part: entries with j in [r0, r1), stably sorted by j (their li order is kept)
        uidx.alloc(P, stream, false);
        ukey_s.alloc(P, stream, false);
        uidx_s.alloc(P, stream, false);
        {
            hipLaunchKernelGGL(exp_iota_kernel, dim3((unsigned) ceil_div(P, 256)), dim3(256), 0, stream, uidx.get(), P);
            MI_LAUNCH_CHECK();
            size_t tb = 0;
            MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ukey.get(), ukey_s.get(), uidx.get(),
                                                            uidx_s.get(), (int) P, 0, 32, stream));
            dev_buf<unsigned char> t;
            t.alloc((int64_t) std::max<size_t>(tb, 16), stream, false);
            MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(t.get(), tb, ukey.get(), ukey_s.get(), uidx.get(),
                                                            uidx_s.get(), (int) P, 0, 32, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
        }
        int64_t nup = 0;
        {
            std::vector<unsigned long long> hup(std::max<int64_t>(R, 1), 0);
            if (R > 0)
                MI_HIP_CHECK(hipMemcpyAsync(hup.data(), cup.get(), sizeof(unsigned long long) * (size_t) R,
                                            hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            for (int64_t r = 0; r < R; ++r) nup += (int64_t) hup[r];
        }
        if (nup > 0) {
            hipLaunchKernelGGL(exp_place_upper_kernel<T>, dim3((unsigned) ceil_div(nup, 256)), dim3(256), 0, stream,
                               ukey_s.get(), uidx_s.get(), nup, Li.get(), Lh.get(), clo.get(), up_start.get(), off8.get(),
                               ex.hj.get(), ex.hv.get());
            MI_LAUNCH_CHECK();
        }
    }
    // waves: row-aligned chunk ranges of about equal size
    {
        const int64_t target_waves = std::max<int64_t>(1, std::min<int64_t>(R, 8192));
        const int64_t per = std::max<int64_t>(1, ceil_div(ex.nchunks, target_waves));
        std::vector<int64_t> wc{ 0 };
        int64_t next = per;
        for (int64_t r = 0; r < R; ++r) {
            const int64_t ce = hoff[r + 1] / 8;
            if (ce >= next && ce < ex.nchunks) {
                wc.push_back(ce);
                next = ce + per;
            }
        }
        wc.push_back(ex.nchunks);
        ex.nwaves = (int64_t) wc.size() - 1;
        ex.wave_chunk.alloc((int64_t) wc.size(), stream);
        MI_HIP_CHECK(hipMemcpyAsync(ex.wave_chunk.get(), wc.data(), sizeof(int64_t) * wc.size(), hipMemcpyHostToDevice,
                                    stream));
    }
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    csr.pairs = ex.pairs;
    csr.slots = ex.slots;
    csr.rbf_factored = kernel == 2;
    ex.on = true;
}

// timing/test-only ablations (results are wrong when non-zero): PLSSVM_MI_EXP_ABLATE bit 0 = drop the
// stored remainder H of the multi-feature pairs, bit 1 = keep only the first term of phi's polynomial
int exp_ablate() {
    static const int v = [] {
        const char *s = std::getenv("PLSSVM_MI_EXP_ABLATE");
        return s ? std::atoi(s) : 0;
    }();
    return v;
}

template <typename T>
void engine<T>::expansion_dominant(const T *w, const cg_scalars<T> *status) {
    auto &ex = csr.ex;
    if (d > 0) {
        coefs cf;
        std::memcpy(cf.c, ex.coef, sizeof(cf.c));
        if (exp_ablate() & 2)
            for (int k = 2; k <= EXP_KMAX; ++k) cf.c[k] = 0.0;
        auto mom = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned) ceil_div(d, 4)), dim3(256), 0, stream, csr.colptr.get(),
                               csr.crow.get(), csr.cval.get(), w, d, cf, ex.M.get(), status);
        };
        if (ex.KM == 4) mom(exp_moments_kernel<T, 4>);
        else if (ex.KM == 8) mom(exp_moments_kernel<T, 8>);
        else mom(exp_moments_kernel<T, 16>);
        MI_LAUNCH_CHECK();
    }
    if (r1 > r0) MI_HIP_CHECK(hipMemsetAsync(ex.hs.get() + r0, 0, sizeof(T) * (size_t) (r1 - r0), stream));
    if (ex.nwaves > 0 && !(exp_ablate() & 1)) {
        hipLaunchKernelGGL(exp_hstream_kernel<T>, dim3((unsigned) ceil_div(ex.nwaves, 4)), dim3(256), 0, stream,
                           ex.wave_chunk.get(), ex.nwaves, ex.hcrow.get(), ex.hj.get(), ex.hv.get(), w, ex.hs.get(),
                           status);
        MI_LAUNCH_CHECK();
    }
}

template <typename T>
void engine<T>::expansion_kp_raw(const T *p, const cg_scalars<T> *status, bool with_base) {
    auto &ex = csr.ex;
    const T *w = p;
    if (kernel == 2) {
        hipLaunchKernelGGL(exp_w_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, csr.e.get(), p, m,
                           ex.wv.get(), status);
        MI_LAUNCH_CHECK();
        w = ex.wv.get();
    }
    launch_dot2<T>(w, nullptr, nullptr, nullptr, m, red.get(), status, stream);  // S = sum_j w_j
    launch_dot_final<T>(red.get(), sc.get(), FIN_PLAIN, 0, nullptr, 0, csr.ssc.get(), stream);
    expansion_dominant(w, status);
    T kappa = 0;
    if (kernel == 1) {
        kappa = 1;
        for (int q2 = 0; q2 < degree; ++q2) kappa *= coef0;
    }
    auto rows = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned) ceil_div(m, 32)), dim3(256), 0, stream, csr.rowptr.get(), csr.col.get(),
                           csr.val.get(), ex.M.get(), kernel == 2 ? csr.e.get() : nullptr, w, ex.hdiag.get(),
                           ex.phin.get(), ex.hs.get(), csr.ssc.get(), kappa, m, r0, r1, with_base ? 0 : 1,
                           raw.get(), status);
    };
    if (ex.KM == 4) rows(exp_rows_kernel<T, 4>);
    else if (ex.KM == 8) rows(exp_rows_kernel<T, 8>);
    else rows(exp_rows_kernel<T, 16>);
    MI_LAUNCH_CHECK();
    allgather_rows(raw.get());
}

#define INST(T)                                                                              \
    template bool engine<T>::expansion_eligible();                                           \
    template void engine<T>::build_expansion(const int64_t *, int64_t);                      \
    template void engine<T>::expansion_dominant(const T *, const cg_scalars<T> *);           \
    template void engine<T>::expansion_kp_raw(const T *, const cg_scalars<T> *, bool);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
