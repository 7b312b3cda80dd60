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
#include <type_traits>

#include "../../include/plssvm_mi355x.h"
#include "cg_common.hpp"
#include "engine.hpp"

namespace plssvm_mi {

namespace {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// phi in double: the exact per-pair function (rbf: expm1(2 g a); poly: sum_k bin_k a^k, no cancellation).
// rbf with |u| = |2 g a| < 2^-7 (every pair of the BASELINE sets: u <= 2 g max x^2 ~ 1e-4): the Taylor
// polynomial of degree 7, whose remainder u^8 / 8! is below 2^-54 |u| there — fp64 accuracy in 8 fma instead of
// the library expm1's range reduction (the setup's remainder kernels evaluate phi once per wave step)
struct phi_fn {
    int rbf = 0, deg = 0;
    double g2 = 0.0;                   // rbf: 2 g
    double bin[EXP_KMAX + 1] = {};     // poly: C(deg, k) c0^(deg - k) g^k
    __host__ __device__ double operator()(double a) const {
        if (rbf) {
            const double u = g2 * a;
            if (fabs(u) < 0x1p-7) {
                double p = 1.0 / 5040.0;
                p = fma(p, u, 1.0 / 720.0);
                p = fma(p, u, 1.0 / 120.0);
                p = fma(p, u, 1.0 / 24.0);
                p = fma(p, u, 1.0 / 6.0);
                p = fma(p, u, 0.5);
                p = fma(p, u, 1.0);
                return p * u;
            }
            return expm1(u);
        }
        double h = 0.0;
        for (int k = deg; k >= 1; --k) h = (h + bin[k]) * a;
        return h;
    }
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

// lower-triangle join (build_expansion): a lower pair's row and H travel together through the transpose's sort
template <typename T>
struct lt_val {
    T h;
    int32_t i;
};

// row r's lower list (slots r cap .. r cap + cnt[r]) to the compact arrays at loff[r]: partner keys and (row, H);
// one wave per row, coalesced
template <typename T>
__global__ __launch_bounds__(256) void exp_lt_compact_kernel(const int32_t *__restrict__ sj, const T *__restrict__ sv,
                                                             const int64_t *__restrict__ cnt, const int64_t *__restrict__ loff,
                                                             int64_t R, int64_t cap, uint32_t *__restrict__ lk,
                                                             lt_val<T> *__restrict__ lv) {
    const int64_t r = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int lane = threadIdx.x & 63;
    const int64_t b = loff[r];
    for (int64_t k = lane; k < cnt[r]; k += 64) {
        lk[b + k] = (uint32_t) sj[r * cap + k];
        lv[b + k] = lt_val<T>{ sv[r * cap + k], (int32_t) r };
    }
}

// per row j: its upper pairs are the run of key j in the sorted keys: ustart[j] = first, tot[j] = lower + upper count
// (R + 1 entries: tot[R] = 0 for the scan's total)
__global__ __launch_bounds__(256) void exp_lt_runs_kernel(const uint32_t *__restrict__ ks, int64_t NL,
                                                          const int64_t *__restrict__ lcnt, int64_t R,
                                                          int64_t *__restrict__ ustart, int64_t *__restrict__ tot) {
    const int64_t j = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (j > R) return;
    if (j == R) {
        tot[R] = 0;
        return;
    }
    auto lb = [&](uint32_t key) {
        int64_t lo = 0, hi = NL;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (ks[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const int64_t a = lb((uint32_t) j), b = lb((uint32_t) j + 1u);
    ustart[j] = a;
    tot[j] = lcnt[j] + (b - a);
}

// the symmetric rows: lower pair q (compact order) at off8[i] + (q - loff[i]); sorted pair p (partner j) at
// off8[j] + lcnt[j] + (p - ustart[j]) — both coalesced
template <typename T>
__global__ __launch_bounds__(256) void exp_lt_place_kernel(const uint32_t *__restrict__ lk, const lt_val<T> *__restrict__ lv,
                                                           const uint32_t *__restrict__ ks, const lt_val<T> *__restrict__ vs,
                                                           int64_t NL, const int64_t *__restrict__ loff,
                                                           const int64_t *__restrict__ lcnt,
                                                           const int64_t *__restrict__ ustart,
                                                           const int64_t *__restrict__ off8, int32_t *__restrict__ hj,
                                                           T *__restrict__ hv) {
    const int64_t q = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= NL) return;
    const lt_val<T> a = lv[q];
    const int64_t pl = off8[a.i] + (q - loff[a.i]);
    hj[pl] = (int32_t) lk[q];
    hv[pl] = a.h;
    const uint32_t j = ks[q];
    const lt_val<T> b = vs[q];
    const int64_t pu = off8[j] + lcnt[j] + (q - ustart[j]);
    hj[pu] = b.i;
    hv[pu] = b.h;
}

// ---- row join: the remainder's symmetric rows built per row (default; PLSSVM_MI_EXP_JOIN=sort keeps the
// column-join sort below) ------------------------------------------------------------------------------
// 512-thread workgroups with a 32 KiB bitmap (round 5): 47 KiB of LDS and 75 VGPRs each, so three rows are joined
// per CU at once (their incidence reads in flight together, one row's barriers and scans under the others' reads).
// The rounds-3/4 form (1024 threads, 128 KiB bitmap: `-DRJ_NT_OPT=1024 -DRJ_BMW_OPT=32768`) held one row per CU;
// same-box A/Bs (profiles/r05_join_ab.json): the 3-RBF / config-5 join 0.18–0.21 / 0.29 s there, 0.14–0.17 / 0.24–0.25 s
// with two rows per CU (512 threads, 64 KiB), 0.12 / 0.21 s with three — more passes per row (262 144 partner rows each)
// cost less than the parallelism gains
#ifndef RJ_NT_OPT
#define RJ_NT_OPT 512
#endif
#ifndef RJ_BMW_OPT
#define RJ_BMW_OPT 8192
#endif
constexpr int RJ_NT = RJ_NT_OPT;
constexpr int RJ_BMW = RJ_BMW_OPT;  // bitmap words: 262 144 partner rows per pass (32 KiB of LDS)
constexpr int RJ_LCAP = 2048;  // repeat sightings held per pass (more: the pass range is halved)
constexpr int RJ_ECAP = 256;   // entries of row i held in LDS (longer rows: the sort join)
constexpr int RJ_WPT = RJ_BMW / RJ_NT;
// bitmap word L of the join (partner rows 32 L .. 32 L + 31 of the pass) lives at LDS word (L % WPT) NT + L / WPT:
// thread t owns the contiguous words t WPT .. t WPT + WPT - 1 (its count and its ascending enumeration), and at
// each step of those loops the 64 lanes read consecutive LDS words — one bank each (word t WPT + w of a plain
// layout put every lane of a wave on the same bank: 64-way conflicts)
template <int WPT, int NT>
__device__ __forceinline__ int bm_addr(int64_t L) {
    return (int) (L % WPT) * NT + (int) (L / WPT);
}
#ifndef RJ_U
#define RJ_U 4  // incidence reads in flight per thread in the join's walk
#endif
constexpr int RJ_PMAX = 256;   // passes per row at most (more: the rank takes the sort join; PLSSVM_MI_EXP_RJ_PMAX: tests)

// Rows [r0, r0 + gridDim.x) of the rank, one workgroup per row i: its partners j != i sharing two or more
// features, ascending, in both triangles. Per pass over a range of partner rows, the column entries of
// row i's features (the incidences, read coalesced from the CSC) mark an LDS bitmap; a second sighting of
// a row appends it to a list, the list becomes a set in the bitmap and is enumerated in ascending order
// (a block scan of per-thread popcounts). Count mode (sj == nullptr): cnt[r] = #partners. Write mode:
// partner k of row r at sj[off8[r] + k], pads up to off8[r + 1] marked -1 (exp_rowjoin_h_kernel then
// forms H). Both modes take the same passes (the halving decisions depend on the data only): deterministic.
// A halved span grows back (doubles) after every completed range, so one dense cluster of partners does not
// cut the rest of the row into small passes; a row needing more than RJ_PMAX passes (every pass rescans its
// incidences) sets *ovf in count mode and the host builds the rank's rows by the sort join instead.
// Slot mode (off8 == nullptr, sj != nullptr; the default one-pass join): partner k of row r at sj[r cap + k]
// for k < cap, cnt[r] = the row's count (also beyond cap: *cnt_max lets the host redo such rows by the two
// passes), no pads — the count pass is not needed.
// Lower mode (cposl != nullptr, round 5): only the partners j < i — the passes cover rows [0, i) and each column's
// range ends at row i's own entry (cposl: the CSR entry's CSC position), so a row reads on average half of its
// incidences; the other triangle is the transpose of these lists (build_expansion).
#if defined(RJ_WPE_OPT) && RJ_WPE_OPT > 0  // compile the join for this many waves per SIMD (a register cap)
#define RJ_WPE_ATTR __attribute__((amdgpu_waves_per_eu(RJ_WPE_OPT)))
#else
#define RJ_WPE_ATTR
#endif
__global__ __launch_bounds__(RJ_NT) RJ_WPE_ATTR void exp_rowjoin_kernel(const int64_t *__restrict__ rowptr,
                                                            const int32_t *__restrict__ col,
                                                            const int64_t *__restrict__ colptr,
                                                            const int32_t *__restrict__ crow, int64_t m, int64_t r0,
                                                            int64_t *__restrict__ cnt, const int64_t *__restrict__ off8,
                                                            int32_t *__restrict__ sj, unsigned int *__restrict__ ovf,
                                                            int pmax, int64_t cap, unsigned long long *__restrict__ cnt_max,
                                                            const int64_t *__restrict__ csplit, int nsplit,
                                                            const int64_t *__restrict__ cposl = nullptr) {
    __shared__ uint32_t bm[RJ_BMW];
    __shared__ int32_t rep[RJ_LCAP];
    __shared__ int32_t zcol[RJ_ECAP];
    __shared__ int32_t zoff[RJ_ECAP + 1];
    __shared__ int64_t cst[RJ_ECAP];
    __shared__ int64_t pst[RJ_ECAP];    // a partial pass: each column's first entry with a row in [R0, R1)
    __shared__ int32_t pzoff[RJ_ECAP + 1];
    __shared__ int32_t wtot[RJ_NT / 64];
    __shared__ int nrep_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t r = blockIdx.x, i = r0 + r;
    const int64_t e0 = rowptr[i];
    const int ne = (int) (rowptr[i + 1] - e0);  // <= RJ_ECAP (host-checked)
    for (int e = tid; e < ne; e += RJ_NT) {  // column starts and lengths in parallel (one global read each)
        const int32_t f = col[e0 + e];
        zcol[e] = f;
        const int64_t c0 = colptr[f];
        cst[e] = c0;
        zoff[e + 1] = (int32_t) (colptr[f + 1] - c0);
    }
    __syncthreads();
    if (tid == 0) {  // prefix over LDS only
        zoff[0] = 0;
        for (int e = 0; e < ne; ++e) zoff[e + 1] += zoff[e];
    }
    __syncthreads();
    const bool wr = sj != nullptr, slots = wr && off8 == nullptr;
    int64_t written = 0;
    constexpr int64_t SPAN_MAX = (int64_t) RJ_BMW * 32;
    int64_t span = SPAN_MAX;
    int passes = 0;
    const bool lower = cposl != nullptr;
    const int64_t Rend = lower ? i : m;  // partner rows [0, Rend)
    for (int64_t R0 = 0; R0 < Rend;) {
        if (++passes > pmax) {  // uniform
            if ((!wr || slots) && tid == 0) {
                cnt[r] = 0;
                atomicOr(ovf, 1u);
            }
            return;
        }
        const int64_t R1 = min(Rend, R0 + span);
        // the bitmap words of this pass's range only (words L < nw, owned by threads < tcnt): a short range — every
        // lower-triangle row's first pass is [0, i) — clears, counts and enumerates only its part of the bitmap
        const int64_t nw = (R1 - R0 + 31) >> 5;
        const int tcnt = (int) min((int64_t) RJ_NT, (nw + RJ_WPT - 1) / RJ_WPT);
        if (tid < tcnt)
            for (int w = 0; w < RJ_WPT; ++w) bm[w * RJ_NT + tid] = 0u;
        if (tid == 0) nrep_s = 0;
        // a pass over part of the partner rows reads only that part of each column (rows ascend within a
        // column: two binary searches per feature), not every incidence of the row once per pass
        const bool whole = !lower && R0 == 0 && R1 >= m;
        if (lower) {
            // lower mode: each bound from the column's start (R0 = 0), the setup's table (a full-span boundary), row
            // i's own position (R1 = i) or a binary search
            for (int e = tid; e < ne; e += RJ_NT) {
                const int64_t a = cst[e], b = a + (zoff[e + 1] - zoff[e]);
                const int32_t f = zcol[e];
                auto first_ge = [&](int64_t Rb) -> int64_t {
                    if (csplit != nullptr && Rb % SPAN_MAX == 0) return csplit[(int64_t) f * nsplit + Rb / SPAN_MAX];
                    int64_t lo = a, hi = b;
                    while (lo < hi) {
                        const int64_t mid = (lo + hi) >> 1;
                        if (crow[mid] < Rb) lo = mid + 1;
                        else hi = mid;
                    }
                    return lo;
                };
                const int64_t lo = R0 == 0 ? a : first_ge(R0);
                const int64_t lo2 = R1 == i ? cposl[e0 + e] : first_ge(R1);
                pst[e] = lo;
                pzoff[e + 1] = (int32_t) (lo2 - lo);
            }
            __syncthreads();
            if (tid == 0) {
                pzoff[0] = 0;
                for (int e = 0; e < ne; ++e) pzoff[e + 1] += pzoff[e];
            }
        } else if (!whole) {
            // a pass of the full span starts and ends where every row's passes do: the column positions come from the
            // setup's table (one load per feature) instead of two binary searches (a chain of dependent loads)
            const bool tab = csplit != nullptr && R0 % SPAN_MAX == 0 && (R1 >= m || R1 % SPAN_MAX == 0);
            for (int e = tid; e < ne; e += RJ_NT) {
                const int64_t a = cst[e], b = a + (zoff[e + 1] - zoff[e]);
                int64_t lo = a, lo2 = b;
                if (tab) {
                    const int64_t *cs = csplit + (int64_t) zcol[e] * nsplit;
                    lo = cs[R0 / SPAN_MAX];
                    lo2 = R1 >= m ? b : cs[R1 / SPAN_MAX];
                } else {
                    int64_t hi = b;
                    while (lo < hi) {  // first row >= R0
                        const int64_t mid = (lo + hi) >> 1;
                        if (crow[mid] < R0) lo = mid + 1;
                        else hi = mid;
                    }
                    lo2 = lo;
                    int64_t hi2 = b;
                    while (lo2 < hi2) {  // first row >= R1
                        const int64_t mid = (lo2 + hi2) >> 1;
                        if (crow[mid] < R1) lo2 = mid + 1;
                        else hi2 = mid;
                    }
                }
                pst[e] = lo;
                pzoff[e + 1] = (int32_t) (lo2 - lo);
            }
            __syncthreads();
            if (tid == 0) {
                pzoff[0] = 0;
                for (int e = 0; e < ne; ++e) pzoff[e + 1] += pzoff[e];
            }
        }
        __syncthreads();
        const int64_t *S = whole ? cst : pst;
        const int32_t *Z = whole ? zoff : pzoff;
        const int32_t pinc = Z[ne];
        // RJ_U incidences per thread in flight (the walk is bound by the latency of these scattered reads)
        int e = 0;
        for (int32_t t0 = tid; t0 < pinc; t0 += RJ_U * RJ_NT) {
            int64_t jv[RJ_U];
#pragma unroll
            for (int u = 0; u < RJ_U; ++u) {
                const int32_t t = t0 + u * RJ_NT;
                jv[u] = -1;
                if (t < pinc) {
                    while (Z[e + 1] <= t) ++e;
                    jv[u] = crow[S[e] + (t - Z[e])];
                }
            }
#pragma unroll
            for (int u = 0; u < RJ_U; ++u) {
                const int64_t j = jv[u];
                if (j < 0 || j == i || j < R0 || j >= R1) continue;
                const uint32_t bit = 1u << ((j - R0) & 31);
                const uint32_t old = atomicOr(&bm[bm_addr<RJ_WPT, RJ_NT>((j - R0) >> 5)], bit);
                if (old & bit) {
                    const int q = atomicAdd(&nrep_s, 1);
                    if (q < RJ_LCAP) rep[q] = (int32_t) j;
                }
            }
        }
        __syncthreads();
        const int nr = nrep_s;
        if (nr > RJ_LCAP) {  // uniform: this range again in halves
            span = (span + 1) / 2;
            __syncthreads();
            continue;
        }
        if (tid < tcnt)
            for (int w = 0; w < RJ_WPT; ++w) bm[w * RJ_NT + tid] = 0u;
        __syncthreads();
        for (int q = tid; q < nr; q += RJ_NT) {
            const int64_t j = rep[q] - R0;
            atomicOr(&bm[bm_addr<RJ_WPT, RJ_NT>(j >> 5)], 1u << (j & 31));
        }
        __syncthreads();
        int c = 0;
        if (tid < tcnt) {
#pragma unroll 8
            for (int w = 0; w < RJ_WPT; ++w) c += __popc(bm[w * RJ_NT + tid]);
        }
        // exclusive block scan of c (wave scans + wave totals)
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wtot[wave] = incl;
        __syncthreads();
        int before = 0, U = 0;
        for (int w = 0; w < RJ_NT / 64; ++w) {
            const int v = wtot[w];
            if (w < wave) before += v;
            U += v;
        }
        if (wr) {
            int pos = before + incl - c;
            for (int w = 0; w < (tid < tcnt ? RJ_WPT : 0); ++w) {
                uint32_t word = bm[w * RJ_NT + tid];
                while (word) {
                    const int b = __ffs(word) - 1;
                    word &= word - 1;
                    rep[pos++] = (int32_t) (R0 + (int64_t) (tid * RJ_WPT + w) * 32 + b);
                }
            }
            __syncthreads();
            if (slots) {
                const int64_t base = r * cap + written;
                for (int q = tid; q < U && written + q < cap; q += RJ_NT) sj[base + q] = rep[q];
            } else {
                const int64_t base = off8[r] + written;
                for (int q = tid; q < U; q += RJ_NT) sj[base + q] = rep[q];
            }
        }
        written += U;
        __syncthreads();  // bm / rep are reused by the next pass
        R0 = R1;
        span = min(span * 2, SPAN_MAX);
    }
    if (!wr || slots) {
        if (tid == 0) {
            cnt[r] = written;
            if (slots) atomicMax(cnt_max, (unsigned long long) written);
        }
        return;
    }
    const int64_t b0 = off8[r], b1 = off8[r + 1];
    for (int64_t k = b0 + written + tid; k < b1; k += RJ_NT) sj[k] = -1;  // pads (exp_rowjoin_h_kernel)
}

// csplit[f][p] = the first position of column f whose row is >= p x (the join's full pass span), p < nsplit
__global__ __launch_bounds__(256) void exp_colsplit_kernel(const int64_t *__restrict__ colptr, const int32_t *__restrict__ crow,
                                                           int64_t d, int nsplit, int64_t span, int64_t *__restrict__ csplit) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= d * nsplit) return;
    const int64_t f = t / nsplit, R = (t % nsplit) * span;
    int64_t lo = colptr[f], hi = colptr[f + 1];
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (crow[mid] < R) lo = mid + 1;
        else hi = mid;
    }
    csplit[t] = lo;
}

// H of the row join's partners (sj from exp_rowjoin_kernel's write / slot pass; row r's entries in
// [rbeg[r], rend[r])): one 256-thread workgroup per row i, row i's features in an LDS hash (open addressing,
// <= 1/8 full: one probe per lookup instead of a binary search), one partner per wave at a time: the lanes take
// row j's entries (coalesced, 64 per step), look each up in row i, and the matches — ascending features — are
// summed in that order from a ballot: H_ij = phi(s_ij) - sum_f phi(x_if x_jf) in fp64, rounded to T (the
// sequential sum of the sort join; rbf: a product recurrence without the expm1 of s_ij, in the body). The next
// partner's row bounds are loaded one step ahead. Pads (sj < 0): j = i, H = 0. lower_nz += #(j < i, H != 0 in T).
constexpr int RJH_NT = 256;
// a wave-uniform 64-bit value into scalar registers
__device__ __forceinline__ int64_t rj_uni64(int64_t v) {
    const uint32_t lo = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) v);
    const uint32_t hi = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) ((uint64_t) v >> 32));
    return (int64_t) (((uint64_t) hi << 32) | lo);
}
constexpr int RJ_HS = 2048;  // hash slots for row i's features (<= RJ_ECAP keys)
__device__ __forceinline__ int rj_hash(int32_t f) { return (int) (((uint32_t) f * 2654435761u) >> (32 - 11)); }
#ifndef RJH_WPE
#define RJH_WPE 8  // waves per SIMD the H kernel is compiled for (<= 64 VGPRs: 8 resident 256-thread workgroups per CU)
#endif
// rbf phi in float (exp_rowjoin_h_kernel<float, true>): expm1(2 g a), a degree-5 Taylor polynomial where |2 g a| < 2^-7
// (truncation < 2^-35 / 720 relative), expm1f otherwise
__device__ __forceinline__ float rj_phi32(float g2, float a) {
    const float u = g2 * a;
    if (fabsf(u) < 0x1p-7f) {
        float p = 1.0f / 120.0f;
        p = fmaf(p, u, 1.0f / 24.0f);
        p = fmaf(p, u, 1.0f / 6.0f);
        p = fmaf(p, u, 0.5f);
        p = fmaf(p, u, 1.0f);
        return p * u;
    }
    return expm1f(u);
}
// F32 (round 5; float contexts, rbf): the shared features' products, their phi and the product recurrence in float.
// The recurrence has no cancellation (two shared features: H = E_a E_b), so H keeps float's relative accuracy, which
// is what the float (or bfloat16) stream stores anyway; the fp64 evaluation cost twice the VALU cycles per partner of
// this VALU-bound kernel. Poly (H = c(s) - sum c(a_f) cancels) and fp64 contexts keep fp64.
template <typename T, bool F32 = false>
__global__ __launch_bounds__(RJH_NT) __attribute__((amdgpu_waves_per_eu(RJH_WPE, RJH_WPE))) void exp_rowjoin_h_kernel(const int64_t *__restrict__ rowptr,
                                                               const int32_t *__restrict__ col,
                                                               const T *__restrict__ val, int64_t r0, phi_fn phi,
                                                               double kbase, const int64_t *__restrict__ rbeg,
                                                               const int64_t *__restrict__ rend,
                                                               int32_t *__restrict__ sj, T *__restrict__ sv,
                                                               unsigned long long *__restrict__ lower_nz,
                                                               unsigned long long *__restrict__ ratio_bits) {
    __shared__ int32_t hkey[RJ_HS];
    __shared__ uint8_t hidx[RJ_HS];
    __shared__ T zval[RJ_ECAP];
    __shared__ unsigned long long lnz_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t r = blockIdx.x, i = r0 + r;
    const int64_t e0 = rowptr[i];
    const int ne = (int) (rowptr[i + 1] - e0);  // <= RJ_ECAP (host-checked)
    for (int q = tid; q < RJ_HS; q += RJH_NT) hkey[q] = -1;
    if (tid == 0) lnz_s = 0ull;
    __syncthreads();
    for (int e = tid; e < ne; e += RJH_NT) {
        const int32_t f = col[e0 + e];
        zval[e] = val[e0 + e];
        int h = rj_hash(f);
        while (atomicCAS(&hkey[h], -1, f) != -1) h = (h + 1) & (RJ_HS - 1);  // distinct features: no duplicates
        hidx[h] = (uint8_t) e;
    }
    __syncthreads();
    unsigned long long lnz = 0ull;
    double rmax = 0.0;
    // The partner bookkeeping is wave-uniform and kept in scalar registers (readfirstlane): the partner loop, the step
    // loop and the entry addresses (scalar base + 32-bit lane offset) cost no VALU. The prefetches stay vector loads
    // (an opaque zero offset): a scalar load would share lgkmcnt with the LDS probes and be waited for at once. A
    // partner's row bounds are loaded one partner ahead, its index two ahead.
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int64_t q0 = rj_uni64(rbeg[r]), q1 = rj_uni64(rend[r]);
    constexpr int NW = RJH_NT / 64;
    // buffer loads (always vector memory instructions) through descriptors built in scalar registers: the row's
    // partner list from its start (offsets < 2^31 B), a partner's two row bounds as one 16-byte load
    const __amdgpu_buffer_rsrc_t rs_sj = __builtin_amdgcn_make_buffer_rsrc((void *) (sj + q0), (short) 0, 0x7FFFFFFF, 0x00020000);
    auto load_j = [&](int64_t qq) -> uint32_t {
        return qq < q1 ? __builtin_amdgcn_raw_buffer_load_b32(rs_sj, 0, (int) ((qq - q0) * 4), 0) : 0xFFFFFFFFu;
    };
    using u32x4 = decltype(__builtin_amdgcn_raw_buffer_load_b128(rs_sj, 0, 0, 0));
    auto load_bounds = [&](int64_t jj) -> u32x4 {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *) (rowptr + jj), (short) 0, 16, 0x00020000);
        return __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, 0);
    };
    auto uni_lo = [](u32x4 v) {
        return (int64_t) (((uint64_t) (uint32_t) __builtin_amdgcn_readfirstlane((int) v[1]) << 32) |
                          (uint32_t) __builtin_amdgcn_readfirstlane((int) v[0]));
    };
    auto uni_hi = [](u32x4 v) {
        return (int64_t) (((uint64_t) (uint32_t) __builtin_amdgcn_readfirstlane((int) v[3]) << 32) |
                          (uint32_t) __builtin_amdgcn_readfirstlane((int) v[2]));
    };
    int64_t q = q0 + wv;
    int64_t jn = (int32_t) __builtin_amdgcn_readfirstlane((int) load_j(q));
    u32x4 bn = {};
    if (jn >= 0) bn = load_bounds(jn);
    uint32_t jnn = load_j(q + NW);
    for (; q < q1; q += NW) {
        const int64_t j = jn;
        const int64_t kb = j >= 0 ? uni_lo(bn) : 0, ke = j >= 0 ? uni_hi(bn) : 0;
        jn = (int32_t) __builtin_amdgcn_readfirstlane((int) jnn);  // the next partner: its bounds now, the one after's index
        if (jn >= 0) bn = load_bounds(jn);
        jnn = load_j(q + 2 * NW);
        if (j < 0) {  // pad
            if (lane == 0) {
                sj[q] = (int32_t) i;
                sv[q] = T(0);
            }
            continue;
        }
        // rbf: with E_f = expm1(2 g x_if x_jf), 1 + E(s_ij) = prod_f (1 + E_f), so H = prod (1 + E_f) - 1 - sum E_f
        // accumulates over the shared features (ascending) as Q += P E_f, P += E_f + P E_f (P = prod - 1): no
        // expm1 of s_ij and no cancellation (two shared features: H = E_a E_b exactly). poly: H = c(s) - sum c(a_f).
        using A = typename std::conditional<F32, float, double>::type;
        const bool rbf = F32 || phi.rbf != 0;
        A sd = 0, sphi = 0, P = 0;
        for (int64_t k0 = kb; k0 < ke; k0 += 64) {
            const int32_t *ck = col + k0;
            const T *vkp = val + k0;
            A a = 0, pa = 0;
            bool hit = false;
            if (lane < ke - k0) {
                // the value is loaded with the feature (one latency per partner, not a second one after the probe)
                const int32_t f = ck[lane];
                const T vk = vkp[lane];
                int h = rj_hash(f);
                int32_t key;
                while ((key = hkey[h]) >= 0 && key != f) h = (h + 1) & (RJ_HS - 1);
                if (key == f) {
                    a = (A) zval[hidx[h]] * (A) vk;
                    if constexpr (F32) pa = rj_phi32((float) phi.g2, a);
                    else pa = phi(a);
                    hit = true;
                }
            }
            uint64_t mask = __ballot(hit);
            while (mask) {  // wave-uniform: the shared features in ascending order
                const int b = __ffsll((long long) mask) - 1;
                mask &= mask - 1;
                const A pb = __shfl(pa, b);
                if (rbf) {
                    const A t = P * pb;
                    sphi += t;  // Q
                    P += pb + t;
                } else {
                    sd += __shfl(a, b);
                    sphi += pb;
                }
            }
        }
        const double ps = rbf ? (double) P : phi((double) sd);  // E(s) or c(s)
        const T h = (T) (rbf ? sphi : (A) (ps - (double) sphi));
        // |H| relative to the pair's kernel value without the e_i e_j factor (rbf 1 + E(s), poly kappa + c(s));
        // the division only when it can raise the maximum (wave-uniform values)
        const double kv = fabs(kbase + ps), ah = fabs((double) h);
        if (h != T(0) && ah > rmax * kv) rmax = kv > 0.0 ? ah / kv : 1e300;
        if (lane == 0) {
            sv[q] = h;
            if (j < i && h != T(0)) ++lnz;
        }
    }
    if (lane == 0 && lnz) atomicAdd(&lnz_s, lnz);
    if (lane == 0 && rmax > 0.0) atomicMax(ratio_bits, (unsigned long long) __double_as_longlong(rmax));  // >= 0: bit order
    __syncthreads();
    if (tid == 0 && lnz_s) atomicAdd(lower_nz, lnz_s);
}

// the one-pass join's row ranges: beg[r] = r cap, end[r] = r cap + cnt[r] (every count <= cap, host-checked)
__global__ __launch_bounds__(256) void exp_pool_range_kernel(const int64_t *__restrict__ cnt, int64_t R, int64_t cap,
                                                             int64_t *__restrict__ beg, int64_t *__restrict__ end) {
    const int64_t r = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (r < R) beg[r] = r * cap, end[r] = r * cap + cnt[r];
}

__global__ __launch_bounds__(256) void exp_pad8_cnt_kernel(const int64_t *__restrict__ cnt, int64_t R,
                                                           int64_t *__restrict__ cnt8) {
    const int64_t r = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (r < R) cnt8[r] = (cnt[r] + 7) & ~int64_t(7);
}

// ---- per K·p ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void exp_w_kernel(const T *__restrict__ e, const T *__restrict__ p, int64_t m,
                                                    T *__restrict__ w, const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) w[i] = e[i] * p[i];
}

// M[f][k] = coef_{k+1} mom[k][f] (the CSR pass gathers the KC channels of a feature together)
template <typename T>
__global__ __launch_bounds__(256) void exp_mscale_kernel(const T *__restrict__ mom, int64_t d, int kc, coefs cf,
                                                         T *__restrict__ M, const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= d * kc) return;
    const int64_t f = t / kc;
    const int k = (int) (t % kc);
    M[t] = (T) (cf.c[k + 1] * (double) mom[(int64_t) k * d + f]);
}

// the moment pass's P panel slabs reduced straight into the Horner coefficients: M[f][k] = coef_{k+1} sum_q
// partial[q][k d + f], the sum in panel_reduce_kernel's order (quarters combined in order when split), so M is
// bitwise that of panel_reduce + exp_mscale_kernel — one launch fewer per K·p
template <typename T>
__global__ __launch_bounds__(256) void exp_mom_reduce_kernel(const T *__restrict__ partial, int64_t P, int64_t d, int kc,
                                                             int split, coefs cf, T *__restrict__ M,
                                                             const T *__restrict__ spart, int sG, T *__restrict__ sout,
                                                             const cg_scalars<T> *__restrict__ status) {
    if (spart != nullptr && blockIdx.x == gridDim.x - 1) {
        // the extra last block: S = sum_j w_j from w's RED_BLOCKS partials, dot_final_kernel's sum (FIN_PLAIN, which
        // also runs after convergence) — one launch fewer
        __shared__ T red[8];
        T r1, r2;
        cgk::partials_final(spart, sG, red, r1, r2);
        if (threadIdx.x == 0) sout[0] = r1, sout[1] = r2;
        return;
    }
    if (status != nullptr && status->converged) return;
    __shared__ T part[3][64];
    const int64_t ns = d * kc;
    const int lane = split ? (threadIdx.x & 63) : threadIdx.x, quarter = split ? (threadIdx.x >> 6) : 0;
    const int64_t s = (int64_t) blockIdx.x * (split ? 64 : 256) + lane;
    const int64_t per = split ? (P + 3) / 4 : P, q0 = quarter * per, q1 = min(P, q0 + per);
    T a = 0;
    if (s < ns) {
        int64_t q = q0;
        for (; q + 8 <= q1; q += 8) {
            T v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = partial[(q + u) * ns + s];
#pragma unroll
            for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; q < q1; ++q) a += partial[q * ns + s];
    }
    if (split) {
        if (quarter > 0) part[quarter - 1][lane] = a;
        __syncthreads();
        if (quarter != 0) return;
        a = ((a + part[0][lane]) + part[1][lane]) + part[2][lane];
    }
    if (s >= ns) return;
    const int64_t k = s / d, f = s % d;
    M[f * kc + k] = (T) (cf.c[k + 1] * (double) a);
}

// ---- remainder stream layout (built from the padded symmetric rows) ---------------------------------------
// count index of (row r, window W): ((I NWV + v) nW + W) RPW + rr,  r = I RB + v RPW + rr
__device__ __forceinline__ int64_t exp_cidx(int64_t r, int64_t W, int64_t nW, int64_t RB) {
    const int64_t RPW = RB / EXP_NWV;
    const int64_t I = r / RB, v = (r % RB) / RPW, rr = r % RPW;
    return ((I * EXP_NWV + v) * nW + W) * RPW + rr;
}

// The cell kernels below walk one row per wave: a row's entries (sorted by j; H == 0 entries — pads, or a
// remainder that rounded to 0 — skipped) are read 64 at a time, coalesced (one row per thread read a row's
// range serially: uncoalesced, 3-4x slower at setup). The valid entries of a step form runs of equal windows
// (j ascending); per run: on_open(prev window, window) when a window starts (wave-uniform), on_entry for each
// of its entries with its rank k among the row's valid entries of that window (lane-parallel), and
// on_close(window, count) when the window's last entry has been seen (wave-uniform). Same order, same values
// as the sequential walk.
template <typename T, typename FO, typename FE, typename FC>
__device__ __forceinline__ void exp_row_windows(const int32_t *__restrict__ sj, const T *__restrict__ sv, int64_t b,
                                                int64_t e, int64_t CW, FO on_open, FE on_entry, FC on_close) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    int curW = -1;
    int64_t kcur = 0;
    for (int64_t s0 = b; s0 < e; s0 += 64) {
        const int64_t s = s0 + lane;
        bool valid = false;
        int W = 0;
        int32_t jj = 0;
        T h = T(0);
        if (s < e) {
            h = sv[s];
            jj = sj[s];
            valid = h != T(0);
            W = valid ? (int) (jj / CW) : 0;
        }
        uint64_t rem = __ballot(valid);
        while (rem) {  // wave-uniform: one run of equal windows at a time
            const int W0 = __shfl(W, __ffsll((long long) rem) - 1);
            const uint64_t m0 = __ballot(valid && W == W0) & rem;
            if (W0 != curW) {
                if (curW >= 0) on_close(curW, kcur);
                on_open(curW, W0);
                curW = W0;
                kcur = 0;
            }
            if ((m0 >> lane) & 1ull) on_entry(jj, h, W0, kcur + __popcll(m0 & below));
            kcur += __popcll(m0);
            rem &= ~m0;
        }
    }
    if (curW >= 0) on_close(curW, kcur);
}

// per row r (rank-local), window W: count of its non-zero entries with j in W, rounded up to gran (4: chunks, 2: pair
// flags) slots; the cells without entries are left as they are (0, or a dummy written before)
template <typename T>
__global__ __launch_bounds__(256) void exp_cell_count_kernel(const int64_t *__restrict__ rbeg, const int64_t *__restrict__ rend,
                                                             const int32_t *__restrict__ sj, const T *__restrict__ sv,
                                                             int64_t R, int64_t nW, int64_t CW, int64_t RB, int64_t gran,
                                                             int64_t *__restrict__ cnt) {
    const int64_t r = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int lane = threadIdx.x & 63;
    exp_row_windows<T>(sj, sv, rbeg[r], rend[r], CW, [](int, int) {}, [](int32_t, T, int, int64_t) {},
                       [&](int W, int64_t k) {
                           if (lane == 0) cnt[exp_cidx(r, W, nW, RB)] = (k + gran - 1) & ~(gran - 1);
                       });
}

// pair flags: a wave's stream of a window (RPW consecutive cells, exp_cidx) padded to a multiple of 4 slots, the
// 2 padding slots (H = 0, no flag: they add 0 to the row open at the end) given to the group's last cell — so every
// (block, wave, window) range starts on a chunk (woff = coff / 4)
__global__ __launch_bounds__(256) void exp_cell_pad_groups_kernel(int64_t ngroups, int64_t RPW, int64_t *__restrict__ cnt) {
    const int64_t gi = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= ngroups) return;
    int64_t *c = cnt + gi * RPW;
    int64_t s = 0;
    for (int64_t k = 0; k < RPW; ++k) s += c[k];
    if (s & 2) c[RPW - 1] += 2;
}

using cgk::bf16_rne;

// S = sum_j w_j (cw non-null: the centered S_c = sum_j cw_j w_j, engine.hpp ctr_*) as RED_BLOCKS block partials
// in dot2_kernel's grid, order and block reduction (bitwise the same partials), writing the remainder stream's
// bfloat16 copy of w on the way (w16 non-null: hbf16 layouts)
template <typename T>
__global__ __launch_bounds__(256) void exp_wsum_kernel(const T *__restrict__ w, int64_t n, uint16_t *__restrict__ w16,
                                                       const T *__restrict__ cw, T *__restrict__ partials,
                                                       const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    __shared__ T red[4];
    T s1 = 0;
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const T v = w[i];
        s1 += cw != nullptr ? cw[i] * v : v;
        if (w16 != nullptr) w16[i] = bf16_rne((float) v);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s1 += __shfl_xor(s1, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s1;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = 0;
        for (int v = 0; v < 4; ++v) t += red[v];
        partials[blockIdx.x] = t;
        partials[RED_BLOCKS + blockIdx.x] = T(0);
    }
}

// sharded groups with bfloat16 windows: the rank's rows only — w_i = e_i p_i (rbf; e null: w = p, nothing
// written), its bfloat16 copy, and the rows' share of S = sum_j w_j as RED_BLOCKS block partials (gathered
// with the group's other partials and summed in rank order: the same S on every rank)
// (cw non-null: the rows' share of the centered S_c = sum_j cw_j w_j instead, engine.hpp ctr_*)
template <typename T>
__global__ __launch_bounds__(cgk::CG_NT) void exp_wown_kernel(const T *__restrict__ e, const T *__restrict__ p,
                                                             int64_t ib, int64_t ie, T *__restrict__ w,
                                                             uint16_t *__restrict__ w16, const T *__restrict__ cw,
                                                             T *__restrict__ partials,
                                                             const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    __shared__ T red[cgk::CG_NT / 64];
    T s1 = 0;
    // the fused CG kernels' grid and element order (cg_dir_sums_kernel carries this pass in a CG iteration: the
    // same partials bit for bit); four elements' loads in flight per thread, summed in the thread's element order
    const int64_t n = ie - ib, st = (int64_t) gridDim.x * blockDim.x;
    const T *pp = p + ib, *ep = e != nullptr ? e + ib : nullptr, *cp = cw != nullptr ? cw + ib : nullptr;
    T *wp = w + ib;
    uint16_t *w16p = w16 + ib;
    int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * st < n; i += 4 * st) {
        T pv[4], ev[4], cv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pv[u] = pp[i + u * st];
            ev[u] = ep != nullptr ? ep[i + u * st] : T(1);
            cv[u] = cp != nullptr ? cp[i + u * st] : T(0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) cgk::w_elem(i + u * st, pv[u], ev[u], cv[u], ep, cp, wp, w16p, s1);
    }
    for (; i < n; i += st)
        cgk::w_elem(i, pp[i], ep != nullptr ? ep[i] : T(1), cp != nullptr ? cp[i] : T(0), ep, cp, wp, w16p, s1);
    cgk::store_partial1(s1, red, partials);
}

template <typename T>
__global__ __launch_bounds__(256) void exp_cell_scatter_kernel(const int64_t *__restrict__ rbeg, const int64_t *__restrict__ rend,
                                                               const int32_t *__restrict__ sj, const T *__restrict__ sv,
                                                               int64_t R, int64_t nW, int64_t CW, int64_t RB,
                                                               const int64_t *__restrict__ coff,
                                                               uint16_t *__restrict__ hjl, T *__restrict__ hv,
                                                               uint16_t *__restrict__ hv16, uint16_t *__restrict__ hrow) {
    const int64_t r = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int lane = threadIdx.x & 63;
    const uint16_t rl = (uint16_t) (r % RB);
    int64_t base = 0;
    exp_row_windows<T>(sj, sv, rbeg[r], rend[r], CW, [&](int, int W) { base = coff[exp_cidx(r, W, nW, RB)]; },
                       [&](int32_t j, T h, int W, int64_t k) {
                           hjl[base + k] = (uint16_t) (j - (int64_t) W * CW);
                           if (hv16 != nullptr) hv16[base + k] = bf16_rne((float) h);
                           else hv[base + k] = h;
                       },
                       [&](int, int64_t k) {
                           for (int64_t q = lane; q < ((k + 3) >> 2); q += 64) hrow[(base >> 2) + q] = rl;
                       });
}

// ---- flagged chunks (hbf16 layouts): no per-chunk row index ------------------------------------------------
// A stored bfloat16 H with |H| < 2 has bit 14 (the exponent's top bit) clear, so the first H of a chunk can
// carry a flag instead: set on the first chunk of each (row, window) cell. Every row of the rank gets at least
// one chunk per window (a dummy: j = 0, H = 0, when it has no partners there), so inside a wave's stream of a
// window the rows follow each other without gaps and a chunk's row is the wave's first row + (the number of
// flags up to it) - 1: a ballot and a lane count per 64 chunks instead of 2 bytes per chunk.

// stats[0] += windows without entries (the dummies the layout would add), stats[1] |= 1 when a stored H's
// bfloat16 has bit 14 set (|H| >= 2: the bit is not free)
template <typename T>
__global__ __launch_bounds__(256) void exp_cell_stats_kernel(const int64_t *__restrict__ rbeg, const int64_t *__restrict__ rend,
                                                             const int32_t *__restrict__ sj, const T *__restrict__ sv,
                                                             int64_t R, int64_t nW, int64_t CW,
                                                             unsigned long long *__restrict__ stats) {
    const int64_t r = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    int64_t nwin = 0;
    unsigned long long big = 0;
    exp_row_windows<T>(sj, sv, rbeg[r], rend[r], CW, [&](int, int) { ++nwin; },
                       [&](int32_t, T h, int, int64_t) {
                           if (bf16_rne((float) h) & 0x4000u) big = 1;
                       },
                       [](int, int64_t) {});
    big = __ballot(big != 0) ? 1ull : 0ull;
    if ((threadIdx.x & 63) == 0) {
        if (nW - nwin) atomicAdd(stats, (unsigned long long) (nW - nwin));
        if (big) atomicOr(stats + 1, big);
    }
}

// the dummies: a (row, window) cell without entries takes one 4-slot chunk (pair flags: one 2-slot pair)
__global__ __launch_bounds__(256) void exp_cell_fill_empty_kernel(int64_t R, int64_t nW, int64_t RB, int64_t dsz,
                                                                  int64_t *__restrict__ cnt) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= R * nW) return;
    const int64_t idx = exp_cidx(t / nW, t % nW, nW, RB);
    if (cnt[idx] == 0) cnt[idx] = dsz;
}

#ifndef EXP_JH
#define EXP_JH 1  // flagged layout: a chunk's 4 indices and 4 bfloat16 H side by side (one 16-byte load per lane)
#endif
// flagged layout, EXP_JH: slot t of chunk c = t / 4 keeps its index at 8 c + t % 4 and its H at 8 c + 4 + t % 4
// of the one array (0: two arrays, index and H at t)
__device__ __forceinline__ int64_t exp_jh_j(int64_t t) { return EXP_JH ? ((t & ~int64_t(3)) << 1) + (t & 3) : t; }
__device__ __forceinline__ int64_t exp_jh_h(int64_t t) { return EXP_JH ? ((t & ~int64_t(3)) << 1) + 4 + (t & 3) : t; }

// exp_cell_scatter_kernel for the flagged layout (bfloat16 H, buffers zeroed): every window of the row in
// order, its entries with bit 14 set on the cell's first H, or a dummy (j = 0, H = 0 with the bit) for a window
// without entries
template <typename T>
__global__ __launch_bounds__(256) void exp_cell_scatter_flag_kernel(const int64_t *__restrict__ rbeg, const int64_t *__restrict__ rend,
                                                                    const int32_t *__restrict__ sj, const T *__restrict__ sv,
                                                                    int64_t R, int64_t nW, int64_t CW, int64_t RB,
                                                                    const int64_t *__restrict__ coff,
                                                                    uint16_t *__restrict__ hjl, uint16_t *__restrict__ hv16) {
    const int64_t r = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const int lane = threadIdx.x & 63;
    auto dummies = [&](int64_t w0, int64_t w1) {  // windows [w0, w1) without entries
        for (int64_t w = w0 + lane; w < w1; w += 64) hv16[exp_jh_h(coff[exp_cidx(r, w, nW, RB)])] = (uint16_t) 0x4000u;
    };
    int64_t base = 0, last = -1;
    exp_row_windows<T>(sj, sv, rbeg[r], rend[r], CW,
                       [&](int prev, int W) {
                           dummies(prev + 1, W);
                           base = coff[exp_cidx(r, W, nW, RB)];
                           last = W;
                       },
                       [&](int32_t j, T h, int W, int64_t k) {
                           hjl[exp_jh_j(base + k)] = (uint16_t) (j - (int64_t) W * CW);
                           hv16[exp_jh_h(base + k)] = (uint16_t) (bf16_rne((float) h) | (k == 0 ? 0x4000u : 0u));
                       },
                       [](int, int64_t) {});
    dummies(last + 1, nW);
}

// first chunk of (block I, wave v, window W), W = 0..nW (W = nW: the end of the wave's stream)
__global__ __launch_bounds__(256) void exp_cell_woff_kernel(const int64_t *__restrict__ coff, int64_t nbv, int64_t nW,
                                                            int64_t RB, int64_t *__restrict__ woff) {
    const int64_t RPW = RB / EXP_NWV;
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nbv * (nW + 1)) return;
    const int64_t bv = t / (nW + 1), W = t % (nW + 1);
    woff[t] = coff[(bv * nW + W) * RPW] >> 2;
}

#ifndef EXP_DPP
#define EXP_DPP 1  // remainder stream: segmented row sums by DPP row shifts / broadcasts (0: ds_bpermute shuffles)
#endif
#ifndef EXP_NH
#define EXP_NH 2  // remainder stream: groups of 64 chunks per lane step (bytes in flight per wave)
#endif
#ifndef EXP_PSCAN
#define EXP_PSCAN 1  // bfloat16 remainder: row sums as differences of one unsegmented lane prefix (0: segmented scan)
#endif
#ifndef EXP_COLPROBE
// cost probe of the one-triangle stream (built only as a variant, -DEXP_COLPROBE=1): every bfloat16
// slot also adds H_ij times a stand-in for w_i into an LDS float at its partner's index with ds_add_f32 — the column
// scatter that design needs — into the row accumulator's LDS (the window already takes the rest), so the results
// are wrong by construction; the timing bounds the design from below
#define EXP_COLPROBE 0
#endif
#ifndef EXP_DOT2
// bfloat16 remainder: a chunk's 4 products as two v_dot2_f32_bf16 (the stream is VALU-bound). The instruction
// pair is inline assembly whose hazard padding (the s_nop in exp_hcell_kernel) was verified on the GPU with the
// ROCm 7.2 compiler (clang 22, tests/test_gpu_sparse.py::test_expansion_dot2_equals_fma_path); any other
// compiler builds the FMA chain until the sequence is re-verified there.
#if HIP_VERSION_MAJOR == 7 && HIP_VERSION_MINOR == 2 && __clang_major__ == 22
#define EXP_DOT2 1
#else
#define EXP_DOT2 0
#endif
#endif

// v added to a row accumulator in LDS (read-add-write; each wave owns its rows). LDS float atomics (ds_add_f32, no
// wait for the read) measured slower in round 6: config 5's pair-flag stream 0.842 -> 1.045 ms, 3-RBF unchanged
template <typename T>
__device__ __forceinline__ void racc_add(T *p, T v) {
    *p += v;
}

// one step of a segmented inclusive lane scan keyed by k (keys non-decreasing in lane order): v += the DPP
// source lane's v when that lane holds the same key. A lane without a source (or in a masked DPP row) reads
// value 0 and key 0 (bound_ctrl / old = 0: no initialising moves) — a false key match then adds +0, which
// changes no sum
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_step(float &v, int k) {
    const float vs = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, true));
    const int ks = __builtin_amdgcn_update_dpp(0, k, CTRL, ROWS, 0xF, true);
    if (ks == k) v += vs;
}
template <int CTRL, int ROWS>
__device__ __forceinline__ void seg_step(double &v, int k) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int) (uint32_t) b, CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int) (b >> 32), CTRL, ROWS, 0xF, false);
    const double vs = __longlong_as_double((long long) (((uint64_t) (uint32_t) hi << 32) | (uint32_t) lo));
    const int ks = __builtin_amdgcn_update_dpp(-2, k, CTRL, ROWS, 0xF, false);
    if (ks == k) v += vs;
}

// hs[i] = sum_j H_ij w_j. One 1024-thread workgroup per block of RB rows walks the windows of
// partners: the window of w (CW values) is staged in LDS (the next window is loaded into registers
// while the current one is used, then stored between two barriers), each wave streams its rows' 4-slot chunks (one
// contiguous range across all windows, coalesced, nontemporal so the stream does not evict w from L2,
// software-pipelined one step ahead, also across window boundaries), gathers w_j from LDS and adds its
// rows' partial sums (segmented shuffle reduction) into an LDS row accumulator only it writes.
// Fixed order, no atomics: bitwise reproducible.
// D2 (bfloat16 H only): the dot instructions (EXP_DOT2) or the FMA chain (PLSSVM_MI_EXP_DOT2=0: tests, A/B)
// RF: 0 = a stored row index per chunk, 1 = row-start flags per chunk, 2 = row-start flags per slot pair (cells
// padded to 2 slots instead of 4, see "pair flags" below)
template <typename T, int RBB, bool HB, int RF = 0, bool D2 = true>
__global__ __launch_bounds__(EXP_NWV * 64) void exp_hcell_kernel(const int64_t *__restrict__ woff,
                                                                 const uint16_t *__restrict__ hrow,
                                                                 const uint16_t *__restrict__ hjl,
                                                                 const T *__restrict__ hv,
                                                                 const uint16_t *__restrict__ hv16, const T *__restrict__ w,
                                                                 const uint16_t *__restrict__ w16,
                                                                 int64_t m, int64_t r0, int64_t R, int64_t nW,
                                                                 int64_t RB, int64_t nI, int G, T *__restrict__ hs,
                                                                 T *__restrict__ hslab,
                                                                 const cg_scalars<T> *__restrict__ status, int wdrop = 0) {
    // wdrop = 1: test-only ablation (PLSSVM_MI_EXP_ABLATE bit 2), the last window of every row block is skipped
    // RB (rows per block, a multiple of 16) <= RBC, the accumulator's capacity. G > 1 window groups:
    // block (I, g) streams only windows [g nW / G, (g + 1) nW / G) of its rows and writes its row sums
    // to hslab[g][rows] (summed in g order by exp_combine_kernel); the blocks of one XCD share g,
    // so they share w's windows in L2
    // HB: H and the window of w in bfloat16 (twice the partners per window; expand.hip "H storage")
    using WT = std::conditional_t<HB, uint16_t, T>;
    constexpr int CW = HB ? exp_cw16_of<RBB>() : exp_cw_of<T, RBB>(), RBC = exp_rb_of<T, RBB>(), NT = EXP_NWV * 64;
    static_assert(CW <= 65536, "window-local partner indices are 16-bit");
    __shared__ __attribute__((aligned(16))) WT wl[CW];
    __shared__ T racc[RBC];
    const WT *wsrc;
    if constexpr (HB) wsrc = w16;
    else wsrc = w;
    if (status != nullptr && status->converged) return;
    const int64_t bx = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t I = bx % nI, g = bx / nI;
    const int64_t W0 = g * nW / G, W1 = (g + 1) * nW / G - (wdrop && g == G - 1 && nW > 0 ? 1 : 0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: the wave's offsets are scalar loads
    for (int t = tid; t < RB; t += NT) racc[t] = T(0);
    // the window of w moves as 16-byte vectors: thread tid takes vectors tid, tid + NT, ... (PV of them)
    constexpr int VE = 16 / (int) sizeof(WT), NV = CW / VE, PV = (NV + NT - 1) / NT;
    using wvec = __attribute__((ext_vector_type(VE))) WT;
    wvec reg[PV];
    auto load_win = [&](int64_t W) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < PV; ++q) {
            const int v = q * NT + tid;
            if (NV % NT == 0 || v < NV) {
                const int64_t idx = W * CW + (int64_t) v * VE;
                if (idx + VE <= m) {
                    reg[q] = *reinterpret_cast<const wvec *>(wsrc + idx);
                } else {
#pragma unroll
                    for (int e = 0; e < VE; ++e) reg[q][e] = idx + e < m ? wsrc[idx + e] : WT(0);
                }
            }
        }
    };
    auto wat = [&](uint32_t j) __attribute__((always_inline)) -> T {  // w_j from the staged window
        if constexpr (HB) return (T) __uint_as_float((uint32_t) wl[j] << 16);
        else return wl[j];
    };
    auto store_win = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < PV; ++q) {
            const int v = q * NT + tid;
            if (NV % NT == 0 || v < NV) reinterpret_cast<wvec *>(wl)[v] = reg[q];
        }
    };
    const int64_t *wo = woff + (I * EXP_NWV + wave) * (nW + 1);
    const int64_t s_end = wo[W1];
    // one step of the stream in registers: EXP_NH groups of 64 chunks (group h: chunk step start + 64 h +
    // lane), loads clamped to the stream; prefetched one step ahead
    struct group_regs {
        int rl = 0;
        u32x2 jj = { 0u, 0u };
        T h[4] = { T(0), T(0), T(0), T(0) };
        u32x2 hb = { 0u, 0u };  // bfloat16 H, kept raw until the step uses it (a conversion here would wait for the load)
    };
    group_regs nx[EXP_NH];
    const bool empty = s_end == wo[W0];
    auto fetch = [&](int64_t c) __attribute__((always_inline)) {
        if (empty) return;  // empty stream (wave-uniform)
#pragma unroll
        for (int hh = 0; hh < EXP_NH; ++hh) {
            const int64_t cl = c + 64 * hh;  // past s_end: the stream's zeroed padding (masked by have)
            group_regs &g = nx[hh];
            if constexpr (!RF) g.rl = (int) __builtin_nontemporal_load(hrow + cl);
            if constexpr (RF && EXP_JH) {  // indices and H of the chunk in one 16-byte load
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(hjl + 8 * cl));
                g.jj = u32x2{ v.x, v.y };
                g.hb = u32x2{ v.z, v.w };
                continue;
            }
            g.jj = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(hjl + 4 * cl));
            if constexpr (HB) {
                g.hb = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(hv16 + 4 * cl));
            } else if constexpr (sizeof(T) == 4) {
                const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(hv + 4 * cl));
                g.h[0] = v.x, g.h[1] = v.y, g.h[2] = v.z, g.h[3] = v.w;
            } else {
                const f64x2 v0 = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(hv + 4 * cl));
                const f64x2 v1 = __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(hv + 4 * cl + 2));
                g.h[0] = v0.x, g.h[1] = v0.y, g.h[2] = v1.x, g.h[3] = v1.y;
            }
        }
    };
    // one group of 64 chunks: the 4 slots times w from the window, then the rows' sums into racc
    // RF: the rows of a window's chunks from their row-start flags (carry = the row before the step's first chunk + 1)
    int carry = 0;
#if EXP_COLPROBE
    auto col_probe = [&](u32x2 jj, uint32_t hx, uint32_t hy, float wi) __attribute__((always_inline)) {
        if constexpr (HB && sizeof(T) == 4) {
            constexpr uint32_t MSK = (uint32_t) RBC - 1u;  // RBC: a power of two
            atomicAdd(&racc[(jj.x & 0xFFFFu) & MSK], __uint_as_float(hx << 16) * wi);
            atomicAdd(&racc[(jj.x >> 16) & MSK], __uint_as_float(hx & 0xFFFF0000u) * wi);
            atomicAdd(&racc[(jj.y & 0xFFFFu) & MSK], __uint_as_float(hy << 16) * wi);
            atomicAdd(&racc[(jj.y >> 16) & MSK], __uint_as_float(hy & 0xFFFF0000u) * wi);
        }
    };
#endif
    auto group = [&](const group_regs &g, bool have) __attribute__((always_inline)) {
        if constexpr (RF == 2) {
            static_assert(HB && EXP_JH && sizeof(T) == 4, "pair flags: bfloat16 H, side-by-side chunks");
            // pair flags: bit 14 of the chunk's H0 / H2 marks a row starting at slot 0 / 2. A lane's two pairs give
            // a01 (slots 0, 1) and a23 (slots 2, 3); t = a01 + a23. With P the inclusive lane prefix of t and E the
            // exclusive one, a row that starts in lane A (its tail there) and ends in lane B (its head there) sums to
            // tail_A - P_A + E_B + head_B: lanes with a flag add tail - P to the row they leave open and E + head to
            // the row their first flag closes; a row inside one lane (pair 0 flagged and pair 1 flagged) adds a01;
            // lane 63 adds P_63 to the row open at the group's end. Each phase writes distinct rows (one instruction
            // never updates a row twice); fixed order: bitwise reproducible. The cancellation bound of the prefix
            // differences is the one of the chunk-flag layout below (bfloat16 H: <= 2^-24 of the group's |H w|).
            const bool f0 = have && (g.hb.x & 0x4000u) != 0u, f1 = have && (g.hb.y & 0x4000u) != 0u;
            const uint32_t hx = g.hb.x & ~0x4000u, hy = g.hb.y & ~0x4000u;
            float a01 = 0.f, a23 = 0.f;
            if (have) {
                const u32x2 jj = g.jj;
                const uint32_t w01 = (uint32_t) wl[jj.x & 0xFFFFu] | ((uint32_t) wl[jj.x >> 16] << 16);
                const uint32_t w23 = (uint32_t) wl[jj.y & 0xFFFFu] | ((uint32_t) wl[jj.y >> 16] << 16);
                if constexpr (D2 && EXP_DOT2) {
                    asm("v_dot2_f32_bf16 %0, %2, %3, 0\n\tv_dot2_f32_bf16 %1, %4, %5, 0\n\ts_nop 1"
                        : "=&v"(a01), "=&v"(a23)
                        : "v"(hx), "v"(w01), "v"(hy), "v"(w23));
                } else {
                    a01 = __uint_as_float(hx << 16) * __uint_as_float(w01 << 16);
                    a01 = fmaf(__uint_as_float(hx & 0xFFFF0000u), __uint_as_float(w01 & 0xFFFF0000u), a01);
                    a23 = __uint_as_float(hy << 16) * __uint_as_float(w23 << 16);
                    a23 = fmaf(__uint_as_float(hy & 0xFFFF0000u), __uint_as_float(w23 & 0xFFFF0000u), a23);
                }
#if EXP_COLPROBE
                col_probe(jj, hx, hy, a01);
#endif
            }
            const float t = a01 + a23;
            float P = t;
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x111, 0xF, 0xF, true));  // row_shr:1
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x112, 0xF, 0xF, true));  // row_shr:2
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x114, 0xF, 0xF, true));  // row_shr:4
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x118, 0xF, 0xF, true));  // row_shr:8
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x142, 0xA, 0xF, true));  // row_bcast:15
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x143, 0xC, 0xF, true));  // row_bcast:31
            const float E = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x138, 0xF, 0xF, true));  // wave_shr:1
            const unsigned long long b0 = __ballot(f0), b1 = __ballot(f1), bh = __ballot(have);
            const int below = (int) __builtin_amdgcn_mbcnt_hi((uint32_t) (b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) b0, 0u)) +
                              (int) __builtin_amdgcn_mbcnt_hi((uint32_t) (b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) b1, 0u));
            const int row0 = carry + below + (f0 ? 1 : 0) - 1, row1 = row0 + (f1 ? 1 : 0);
            carry += __popcll(b0) + __popcll(b1);
            if (bh == 0ull) return;  // a group wholly past the window's end
            if (f0 || f1) racc_add(&racc[f1 ? row1 : row0], (f1 ? a23 : t) - P);  // tail: the row left open in this lane
            if (f0 && f1) racc_add(&racc[row0], a01);                             // a row inside this lane
            // head: not for a row that starts at the group's first valid lane (its predecessor is no row of this pass)
            const int lead = __builtin_ctzll(bh);
            if ((f0 || f1) && !(lane == lead && f0)) racc_add(&racc[(f0 ? row0 : row1) - 1], E + (f0 ? 0.f : a01));
            if (lane == 63) racc_add(&racc[row1], P);                             // the row open at the group's end
            return;
        }
        int rl = have ? g.rl : -1;
        uint32_t hx = g.hb.x;
        if constexpr (RF) {
            const uint32_t fb = (hx >> 14) & 1u;  // the row-start flag as 0 / 1
            const unsigned long long bal = __ballot((hx & 0x4000u) != 0u) & __ballot(have);
            const int below = (int) __builtin_amdgcn_mbcnt_hi((uint32_t) (bal >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t) bal, 0u));
            rl = have ? carry + below + (int) fb - 1 : -1;
            carry += __popcll(bal);
            hx &= ~0x4000u;
        }
        const u32x2 jj = g.jj;
        T h0 = g.h[0], h1 = g.h[1], h2 = g.h[2], h3 = g.h[3];
        if constexpr (HB) {  // bfloat16 H: the float's top 16 bits
            h0 = (T) __uint_as_float(hx << 16), h1 = (T) __uint_as_float(hx & 0xFFFF0000u);
            h2 = (T) __uint_as_float(g.hb.y << 16), h3 = (T) __uint_as_float(g.hb.y & 0xFFFF0000u);
        }
        T acc = T(0);
        if constexpr (HB && D2 && EXP_DOT2 && sizeof(T) == 4) {
            // bfloat16 H and w: the pairs' products (exact in fp32) summed by two bf16 dot instructions, H and w
            // packed as they are stored (the window holds w's bfloat16 bits)
            (void) h0, (void) h1, (void) h2, (void) h3;
            if (have) {
                const uint32_t w01 = (uint32_t) wl[jj.x & 0xFFFFu] | ((uint32_t) wl[jj.x >> 16] << 16);
                const uint32_t w23 = (uint32_t) wl[jj.y & 0xFFFFu] | ((uint32_t) wl[jj.y >> 16] << 16);
                // VOP3P form in inline assembly: the compiler's v_dot2c lowering of two chained
                // __builtin_amdgcn_fdot2_f32_bf16 calls read the same H register twice here (ROCm 7.2 clang);
                // the s_nop covers the DPP read of acc that follows (2 wait states after a VALU write)
                asm("v_dot2_f32_bf16 %0, %1, %2, 0\n\tv_dot2_f32_bf16 %0, %3, %4, %0\n\ts_nop 1"
                    : "=&v"(acc)
                    : "v"(hx), "v"(w01), "v"(g.hb.y), "v"(w23));
#if EXP_COLPROBE
                col_probe(jj, hx, g.hb.y, acc);
#endif
            }
        } else if (have) {
            acc = h0 * wat(jj.x & 0xFFFFu);
            acc = fma(h1, wat(jj.x >> 16), acc);
            acc = fma(h2, wat(jj.y & 0xFFFFu), acc);
            acc = fma(h3, wat(jj.y >> 16), acc);
        }
#if EXP_DPP
        if constexpr (HB && EXP_PSCAN && sizeof(T) == 4) {
            // bfloat16 H (|H w| <= 2^-16 |k w| per pair): an unsegmented inclusive prefix P of the 64 chunk sums (six
            // DPP adds, no keys); a row ending at lane e adds P_e to its accumulator and the row that starts at
            // e + 1 subtracts it — the row's sum as a difference of prefixes. The cancellation costs at most
            // 2^-24 of the group's |H w| (<= 256 pair terms of <= 2^-16 |k w| each), far below the float rounding
            // of the row's K·p; fixed order, bitwise reproducible.
            float P = acc;
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x111, 0xF, 0xF, true));  // row_shr:1
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x112, 0xF, 0xF, true));  // row_shr:2
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x114, 0xF, 0xF, true));  // row_shr:4
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x118, 0xF, 0xF, true));  // row_shr:8
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x142, 0xA, 0xF, true));  // row_bcast:15
            P += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(P), 0x143, 0xC, 0xF, true));  // row_bcast:31
            const int rnext = __builtin_amdgcn_update_dpp(-1, rl, 0x130, 0xF, 0xF, false);  // wave_shl:1 (lane 63: -1)
            const bool end = rl >= 0 && (lane == 63 || rnext != rl);
            if (end) racc_add(&racc[rl], (T) P);  // rows of this wave only
            if (end && lane != 63 && rnext >= 0) racc_add(&racc[rnext], -(T) P);
            return;
        }
        // segmented inclusive prefix sums over the lanes by DPP (rows are non-decreasing in lane order):
        // row_shr 1/2/4/8 inside each 16-lane row, then row_bcast 15 / 31 across rows; the total of a
        // row's run lands on its last lane, which adds it to the row accumulator
        T sacc = acc;
        seg_step<0x111, 0xF>(sacc, rl);  // row_shr:1
        seg_step<0x112, 0xF>(sacc, rl);  // row_shr:2
        seg_step<0x114, 0xF>(sacc, rl);  // row_shr:4
        seg_step<0x118, 0xF>(sacc, rl);  // row_shr:8
        seg_step<0x142, 0xA>(sacc, rl);  // row_bcast:15 (rows 1, 3)
        seg_step<0x143, 0xC>(sacc, rl);  // row_bcast:31 (rows 2, 3)
        const int rnext = __builtin_amdgcn_update_dpp(0, rl, 0x130, 0xF, 0xF, true);  // wave_shl:1 (lane 63: tested apart)
        if (rl >= 0 && (lane == 63 || rnext != rl)) racc_add(&racc[rl], sacc);  // rows of this wave only
#else
        // segmented suffix sums: rows are non-decreasing in lane order
        T sacc = acc;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const T so = __shfl_down(sacc, off);
            const int rr = __shfl_down(rl, off);
            if (lane + off < 64 && rr == rl) sacc += so;
        }
        const int rprev = __shfl_up(rl, 1);
        if (rl >= 0 && (lane == 0 || rprev != rl)) racc[rl] += sacc;  // rows of this wave only
#endif
    };
    if (W0 < W1) {
        load_win(W0);
        store_win();
        fetch(wo[W0] + lane);
    }
    __syncthreads();
    constexpr int STEP = 64 * EXP_NH;
    // Steps restart at every window: the part of a window's last step past its end is masked and loaded again as the
    // next window's first step (mostly from L2). Round 6 measured a walk that ignores the window boundaries (a
    // straddling step processed for both windows, nothing loaded twice): 3-RBF 0.766 vs 0.770 ms over three same-box
    // pairs and FETCH 4.915 vs 4.93 GB — nothing to show for it; with pair flags 4.5 % slower (registers, a spill).
    for (int64_t W = W0; W < W1; ++W) {
        if (W + 1 < W1) load_win(W + 1);  // lands in registers while this window is processed
        const int64_t c_end = wo[W + 1];
        carry = wave * (int) (RB / EXP_NWV);  // RF: the wave's first row starts every window
        for (int64_t cb = wo[W]; cb < c_end; cb += STEP) {  // wave-uniform trip count
            group_regs cur[EXP_NH];
#pragma unroll
            for (int hh = 0; hh < EXP_NH; ++hh) cur[hh] = nx[hh];
            // next step (next window's first at c_end; groups past a window's end are loaded, masked, and
            // loaded again as the next window's)
            fetch((cb + STEP < c_end ? cb + STEP : c_end) + lane);
#pragma unroll
            for (int hh = 0; hh < EXP_NH; ++hh) group(cur[hh], cb + 64 * hh + lane < c_end);  // groups in order
        }
        if (W + 1 < W1) {
            __syncthreads();  // every wave is done with window W
            store_win();
        }
        __syncthreads();
    }
    const int64_t rb0 = I * RB;
    const int rows = (int) min<int64_t>(RB, R - rb0);
    if (G == 1) {
        for (int t = tid; t < rows; t += NT) hs[r0 + rb0 + t] = racc[t];
    } else {
        for (int t = tid; t < rows; t += NT) hslab[g * R + rb0 + t] = racc[t];
    }
}

// raw_i for rows [r0, r1) (0 elsewhere), raw holding J_i there (the CSR pass): base + scale (J_i +
// H_ii w_i + hs_i, hs_i = the remainder stream's row sum) [- the diagonal's pair part when only the overlap part is asked for], in fp64.
// jslab != null: the CSR pass left its P < 16 panel slabs (jslab[q][i - r0]) and J_i is their sum from 0 in
// panel order — panel_reduce_kernel's sum, bit for bit, without its launch
// one row of the combine (rows [r0, r1)): the body of exp_combine_kernel, shared with the fused combine +
// CG finalize so both compile the same arithmetic
// cb non-null: the centered base cb_i S (engine.hpp ctr_*) in place of e_i S / kappa S
template <typename T>
__device__ __forceinline__ T exp_combine_row(const T *__restrict__ e, const T *__restrict__ cb, const T *__restrict__ w,
                                             const T *__restrict__ hdiag,
                                             const T *__restrict__ phin, const T *__restrict__ hs,
                                             const T *__restrict__ hslab, int G, const T *__restrict__ jslab, int P,
                                             const T *__restrict__ raw, const T *__restrict__ ssc, T kappa, int64_t i,
                                             int64_t r0, int64_t r1, int overlap_only) {
    const double wi = (double) w[i];
    T h = 0;  // the remainder stream's row sum (G window groups: their slabs in g order)
    if (G > 1) {
        for (int g = 0; g < G; ++g) h += hslab[(int64_t) g * (r1 - r0) + (i - r0)];
    } else {
        h = hs[i];
    }
    T J;
    if (jslab != nullptr) {
        J = T(0);
        for (int q = 0; q < P; ++q) J += jslab[(int64_t) q * (r1 - r0) + (i - r0)];
    } else {
        J = raw[i];
    }
    const double t = (double) J + (double) hdiag[i] * wi + (double) h;
    const double sc = e != nullptr ? (double) e[i] : 1.0;
    double v;
    if (overlap_only == 2) {  // PLSSVM_MI_PART_REMAINDER: the remainder stream's row sum alone
        v = sc * (double) h;
    } else if (overlap_only) {
        v = sc * (t - (double) phin[i] * wi);
    } else {
        const double base =
            (cb != nullptr ? (double) cb[i] : e != nullptr ? (double) e[i] : (double) kappa) * (double) ssc[0];
        v = base + sc * t;
    }
    return (T) v;
}

template <typename T>
__global__ __launch_bounds__(256) void exp_combine_kernel(const T *__restrict__ e, const T *__restrict__ cb,
                                                          const T *__restrict__ w,
                                                          const T *__restrict__ hdiag, const T *__restrict__ phin,
                                                          const T *__restrict__ hs, const T *__restrict__ hslab, int G,
                                                          const T *__restrict__ jslab, int P,
                                                          const T *__restrict__ ssc, T kappa,
                                                          int64_t ib, int64_t ie, int64_t r0, int64_t r1, int overlap_only,
                                                          T *__restrict__ raw, const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = ib + (int64_t) blockIdx.x * blockDim.x + threadIdx.x;  // rows [ib, ie)
    if (i >= ie) return;
    if (i < r0 || i >= r1) {
        raw[i] = T(0);
        return;
    }
    raw[i] = exp_combine_row<T>(e, cb, w, hdiag, phin, hs, hslab, G, jslab, P, raw, ssc, kappa, i, r0, r1, overlap_only);
}

// the combine of a CG iteration's K·p fused with the iteration's finalize (cg_fin_dad_kernel): rows [r0, r1) =
// the CG's own rows, in cg_fin_dad_kernel's grid (RED_BLOCKS x CG_NT), element order and partials — Ad and the
// d.Ad partials bit for bit those of the two launches, raw is not written
template <typename T>
__global__ __launch_bounds__(cgk::CG_NT) void exp_combine_fin_kernel(
    const T *__restrict__ e, const T *__restrict__ cb, const T *__restrict__ w, const T *__restrict__ hdiag, const T *__restrict__ hs,
    const T *__restrict__ hslab, int G, const T *__restrict__ jslab, int P, const T *__restrict__ raw,
    const T *__restrict__ ssc, T kappa, int64_t r0, int64_t r1, const T *__restrict__ q, const T *__restrict__ d,
    const T *__restrict__ psum, int GP, T QA_cost, T cost_inv, T *__restrict__ Ad, T *__restrict__ pdad,
    cg_scalars<T> *sc) {
    if (sc->converged) return;
    __shared__ T red[cgk::CG_NT / 64], bc[1];
    T sp, sqp;
    cgk::partials_total(psum, GP, red, bc, sp, sqp);
    if (blockIdx.x == 0 && threadIdx.x == 0) sc->sp = sp, sc->sqp = sqp;
    const int64_t st = (int64_t) gridDim.x * blockDim.x;
    T s1 = 0;
    for (int64_t k = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; k < r1 - r0; k += st) {
        const int64_t i = r0 + k;
        const T rw = exp_combine_row<T>(e, cb, w, hdiag, nullptr, hs, hslab, G, jslab, P, raw, ssc, kappa, i, r0, r1, 0);
        const T di = d[i];
        const T v = cgk::cg_fin_value(rw, q[i], di, sp, sqp, QA_cost, cost_inv, 0);
        Ad[i] = v;
        s1 = cgk::cg_acc(s1, di, v);
    }
    cgk::store_partial_first(s1, red, pdad);  // (consumers read the first partial of the pair only)
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
    ex.KM = ex.K <= 2 ? 2 : (ex.K <= 4 ? 4 : (ex.K <= 8 ? 8 : 16));
    return true;
}

// Setup: the remainder H of the pairs sharing >= 2 features as symmetric rows [r0, r1) — by the row join
// (exp_rowjoin_kernel: per row, an LDS bitmap of the rows met in its features' columns; count pass, scan,
// write pass with H from a merge of the two rows), or by the column-join sort (every incidence (i, j < i,
// a, phi(a)) generated, radix-sorted and reduced by key; PLSSVM_MI_EXP_JOIN=sort); H_ii; the moment buffers.
template <typename T>
void engine<T>::build_expansion(const int64_t *cpos, int64_t /*max_inc*/,
                                const std::function<std::exception_ptr()> &before_agree) {
    auto &ex = csr.ex;
    phase_timer pt;
    const phi_fn phi = make_phi<T>(kernel, degree, gamma, coef0);
    const int64_t R = r1 - r0;
    dev_buf<int64_t> off8;
    dev_buf<int32_t> sj;
    dev_buf<T> sv;
    int64_t nslot8 = 0;
    dev_buf<int64_t> pbeg, pend;
    const int64_t *rbeg = nullptr, *rend = nullptr;  // row r's symmetric entries: [rbeg[r], rend[r]) of (sj, sv)
    ex.hratio = -1.0;
    {
        const char *e = std::getenv("PLSSVM_MI_EXP_DOT2");
        ex.dot2 = !(e != nullptr && std::strcmp(e, "0") == 0);
    }
    // phase 1 (the symmetric rows) may fail on one rank only (memory, a dense row): in a real group every rank
    // still reaches the agreement after it, which raises the same error everywhere
    std::exception_ptr fail1;
    try {
    ex.M.alloc(std::max<int64_t>(d, 1) * ex.KM, stream);
    ex.mom.alloc(std::max<int64_t>(d, 1) * ex.KM, stream);
    csr.ssc.alloc(2, stream);  // device scalar S = sum_j w_j
    ex.hdiag.alloc(n_pad, stream);
    ex.hs.alloc(n_pad, stream);
    ex.wv.alloc(kernel == 2 ? n_pad : 1, stream);
    ex.phin.alloc(n_pad, stream);
    if (m > 0)
        hipLaunchKernelGGL(exp_diag_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, csr.rowptr.get(),
                           csr.val.get(), m, phi, ex.hdiag.get(), ex.phin.get());
    MI_LAUNCH_CHECK();

    // ---- the remainder's symmetric rows [r0, r1), padded to 8 slots: off8[R + 1], (sj, sv)[nslot8] ----
    // the column-join sort (PLSSVM_MI_EXP_JOIN=sort, and rows longer than the row join's LDS copy)
    auto sort_join = [&]() {
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
        constexpr int64_t CAP = int64_t(1) << 27;  // incidences per sub-block (≈ 80 B each in flight)
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
        double st_gen = 0, st_sort = 0, st_red = 0, st_sel = 0;  // PLSSVM_MI_TIMING: stage seconds
        auto stage = [&](double &acc) {
            if (!pt.on) return;
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            const auto now = std::chrono::steady_clock::now();
            acc += std::chrono::duration<double>(now - pt.t).count();
            pt.t = now;
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
            stage(st_gen);
            const int end_bit = 32 + std::max(1, (int) std::ceil(std::log2((double) rows + 1.0)));
            size_t t1s = tmp_sort;
            MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp.get(), t1s, keys.get(), keys_s.get(), vals.get(),
                                                            vals_s.get(), (int) total, 0, end_bit, stream));
            stage(st_sort);
            size_t t2s = tmp_red;
            MI_HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(tmp.get(), t2s, keys_s.get(), keys.get(), vals_s.get(),
                                                           vals.get(), nruns.get(), d2sum(), (int) total, stream));
            hipLaunchKernelGGL(exp_h_kernel, dim3((unsigned) ceil_div(total, 256)), dim3(256), 0, stream, keys.get(),
                               vals.get(), nruns.get(), phi, hp.get());
            MI_LAUNCH_CHECK();
            stage(st_red);
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
            stage(st_sel);
        }
        if (pt.on)
            std::fprintf(stderr, "[plssvm_mi] column join: %zu blocks, gen %.3f sort %.3f reduce %.3f select+append %.3f\n",
                         blocks.size(), st_gen, st_sort, st_red, st_sel);
        keys.reset(), keys_s.reset(), vals.reset(), vals_s.reset(), hp.reset(), hsel.reset(), tmp.reset();
        pt.mark("expansion: column join (blocks)");
        if (P > INT32_MAX) throw mi_error(-5, "more than 2^31 multi-feature pairs on one rank: use more GPUs");

        // ---- symmetric rows [r0, r1), padded to 8 slots ----
        dev_buf<unsigned long long> clo, cup;
        dev_buf<int64_t> cnt8, lo_start, up_start;
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
        // padded symmetric rows (temporary): row r's entries in [off8[r], off8[r + 1]), sorted by j
        MI_HIP_CHECK(hipMemcpyAsync(&nslot8, off8.get() + R, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        dev_buf<int32_t> scrow;
        sj.alloc(std::max<int64_t>(nslot8, 8), stream, false);
        sv.alloc(std::max<int64_t>(nslot8, 8), stream);
        scrow.alloc(std::max<int64_t>(nslot8 / 8, 1), stream, false);
        if (R > 0) {
            hipLaunchKernelGGL(exp_init_rows_kernel<T>, dim3((unsigned) ceil_div(R, 4)), dim3(256), 0, stream, off8.get(), R,
                               r0, sj.get(), sv.get(), scrow.get());
            MI_LAUNCH_CHECK();
        }
        scrow.reset();
        if (P > 0) {
            hipLaunchKernelGGL(exp_place_lower_kernel<T>, dim3((unsigned) ceil_div(P, 256)), dim3(256), 0, stream, Li.get(),
                               Lj.get(), Lh.get(), P, r0, r1, lo_start.get(), off8.get(), sj.get(), sv.get());
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
                                   sj.get(), sv.get());
                MI_LAUNCH_CHECK();
            }
        }
        Li.reset(), Lj.reset(), Lh.reset(), uidx.reset(), ukey.reset(), ukey_s.reset(), uidx_s.reset();
    };
    const char *je = std::getenv("PLSSVM_MI_EXP_JOIN");
    bool row_join = !(je != nullptr && std::strcmp(je, "sort") == 0);
    if (row_join && R > 0) {
        // host checks: every row of the rank within the row join's LDS copy, incidences within int32
        std::vector<int64_t> rp((size_t) (R + 1));
        MI_HIP_CHECK(hipMemcpyAsync(rp.data(), csr.rowptr.get() + r0, sizeof(int64_t) * (size_t) (R + 1),
                                    hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        for (int64_t r = 0; r < R && row_join; ++r) row_join = rp[(size_t) r + 1] - rp[(size_t) r] <= RJ_ECAP;
        if (row_join && csr.nnz >= (int64_t) INT32_MAX) row_join = false;  // a row's incidences <= nnz
    }
    // the join's pass boundaries in every column (more rows than one bitmap pass: each row's full passes start at the
    // same partner rows, p x RJ_BMW x 32, so each column's positions there are found once here)
    dev_buf<int64_t> csplit;
    int nsplit = 0;
    const char *cse = std::getenv("PLSSVM_MI_EXP_COLSPLIT");  // "0": binary searches only (tests)
    if (row_join && R > 0 && d > 0 && m > (int64_t) RJ_BMW * 32 && !(cse != nullptr && std::strcmp(cse, "0") == 0)) {
        nsplit = (int) ceil_div(m, (int64_t) RJ_BMW * 32);
        csplit.alloc(d * nsplit, stream, false);
        hipLaunchKernelGGL(exp_colsplit_kernel, dim3((unsigned) ceil_div(d * nsplit, 256)), dim3(256), 0, stream,
                           csr.colptr.get(), csr.crow.get(), d, nsplit, (int64_t) RJ_BMW * 32, csplit.get());
        MI_LAUNCH_CHECK();
    }
    dev_buf<int64_t> cnt, cnt8;
    dev_buf<unsigned long long> lnz;
    unsigned int ovf_h = 0u;
    const int rj_pmax = [] {
        const char *e = std::getenv("PLSSVM_MI_EXP_RJ_PMAX");
        const int v = e ? std::atoi(e) : 0;
        return v >= 1 ? v : RJ_PMAX;
    }();
    double kbase = 1.0;  // rbf: 1 + E(s); poly: kappa + c(s)
    if (kernel == 1)
        for (int q2 = 0; q2 < degree; ++q2) kbase *= (double) coef0;
    auto read_lnz = [&]() {
        unsigned long long np[2] = { 0ull, 0ull };
        MI_HIP_CHECK(hipMemcpyAsync(np, lnz.get(), sizeof(np), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        ex.pairs = (int64_t) np[0];
        double rm = 0.0;
        std::memcpy(&rm, &np[1], sizeof(rm));
        ex.hratio = rm;
    };
    // one pass of the join into fixed per-row slot ranges of cap partners (exp_rowjoin_kernel's slot mode, no
    // count pass), cap from the setup's sample of the rank's rows (estimate_expansion_bytes); a row beyond its
    // slots: the two passes with the counts this pass took. PLSSVM_MI_EXP_RJ=twopass: count pass + write pass.
    bool have_cnt = false;  // cnt[] holds every row's exact partner count (a slot pass whose cap was too small)
    // the H kernel: float evaluation for rbf in a float context (exp_rowjoin_h_kernel's F32; PLSSVM_MI_EXP_H64=1: fp64)
    const bool h64 = [] {
        const char *e = std::getenv("PLSSVM_MI_EXP_H64");
        return e != nullptr && std::atoi(e) != 0;
    }();
    auto launch_h = [&](const int64_t *hb, const int64_t *he, int32_t *hj, T *hv) {
        if (sizeof(T) == 4 && phi.rbf != 0 && !h64)
            hipLaunchKernelGGL((exp_rowjoin_h_kernel<T, true>), dim3((unsigned) R), dim3(RJH_NT), 0, stream,
                               csr.rowptr.get(), csr.col.get(), csr.val.get(), r0, phi, kbase, hb, he, hj, hv, lnz.get(),
                               lnz.get() + 1);
        else
            hipLaunchKernelGGL((exp_rowjoin_h_kernel<T, false>), dim3((unsigned) R), dim3(RJH_NT), 0, stream,
                               csr.rowptr.get(), csr.col.get(), csr.val.get(), r0, phi, kbase, hb, he, hj, hv, lnz.get(),
                               lnz.get() + 1);
        MI_LAUNCH_CHECK();
    };
    auto h_pass = [&]() {  // H of every listed partner, then the pairs count and the H bound
        if (R > 0) launch_h(rbeg, rend, sj.get(), sv.get());
        read_lnz();
    };
    // Lower-triangle join (round 5; one rank holding every row): each row joins only its partners j < i (half the
    // incidences), H is formed once per unordered pair, and the upper lists are the transpose — a stable radix sort
    // of the lower pairs by partner (rows stay ascending within a partner). The symmetric rows, their partners and
    // their H are bit for bit those of the full join (H_ij = H_ji: commutative products, features in ascending
    // order). PLSSVM_MI_EXP_LT=0 keeps the full join. Anything unusual (a row beyond its slots, a dense cluster,
    // out of memory) falls back to the full join below.
    auto lt_join = [&]() -> bool {
        const char *lte = std::getenv("PLSSVM_MI_EXP_LT");
        const char *rj = std::getenv("PLSSVM_MI_EXP_RJ");
        if ((lte != nullptr && std::strcmp(lte, "0") == 0) || (rj != nullptr && std::strcmp(rj, "twopass") == 0)) return false;
        if (!(row_join && R > 0 && R == m && r0 == 0 && !shard && world == 1 && sim_world == 0 && cpos != nullptr &&
              ex.rj_mean > 0.0 && m < (int64_t) INT32_MAX))
            return false;
        int64_t cap = round_up(std::max<int64_t>({ (int64_t) (2.0 * ex.rj_mean), (int64_t) (1.5 * ex.rj_max), 64 }), 8);
        if (const char *e = std::getenv("PLSSVM_MI_EXP_RJ_CAP")) {
            const long long v = std::atoll(e);
            if (v > 0) cap = v;
        }
        const double room = csr.budget_b > 0 ? (double) (csr.budget_b - csr.est_bytes) : 0.0;
        if ((double) R * (double) cap * (double) (4 + sizeof(T)) > room) return false;
        try {
            dev_buf<int32_t> ls;
            dev_buf<T> lv;
            dev_buf<int64_t> lcnt, lb, le;
            ls.alloc(R * cap, stream, false);
            lcnt.alloc(R + 1, stream);
            lnz.alloc(3, stream);
            dev_buf<unsigned int> ovf;
            ovf.alloc(1, stream);
            hipLaunchKernelGGL(exp_rowjoin_kernel, dim3((unsigned) R), dim3(RJ_NT), 0, stream, csr.rowptr.get(),
                               csr.col.get(), csr.colptr.get(), csr.crow.get(), m, r0, lcnt.get(), (const int64_t *) nullptr,
                               ls.get(), ovf.get(), rj_pmax, cap, lnz.get() + 2, csplit.get(), nsplit, cpos);
            MI_LAUNCH_CHECK();
            // the H buffers are mapped while the join runs (a multi-GB hipMalloc is tens of ms of host time)
            lv.alloc(R * cap, stream, false);
            lb.alloc(R, stream, false);
            le.alloc(R, stream, false);
            unsigned long long cmax = 0ull;
            unsigned int ov = 0u;
            MI_HIP_CHECK(hipMemcpyAsync(&ov, ovf.get(), sizeof(ov), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipMemcpyAsync(&cmax, lnz.get() + 2, sizeof(cmax), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            if (ov != 0u || (int64_t) cmax > cap) return false;
            pt.mark("expansion: row join, lower triangle");
            hipLaunchKernelGGL(exp_pool_range_kernel, dim3((unsigned) ceil_div(R, 256)), dim3(256), 0, stream, lcnt.get(),
                               R, cap, lb.get(), le.get());
            MI_LAUNCH_CHECK();
            launch_h(lb.get(), le.get(), ls.get(), lv.get());
            read_lnz();  // pairs with H != 0 and the H bound: the lower pairs are every unordered pair
            pt.mark("expansion: row join, lower triangle (H)");
            // compact lower pairs, in row order (rows ascending, partners ascending)
            dev_buf<int64_t> loff;
            loff.alloc(R + 1, stream, false);
            auto excl = [&](const int64_t *in, int64_t *out, int64_t n1) {
                size_t tb = 0;
                MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int) n1, stream));
                dev_buf<unsigned char> t;
                t.alloc((int64_t) std::max<size_t>(tb, 16), stream, false);
                MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(t.get(), tb, in, out, (int) n1, stream));
            };
            excl(lcnt.get(), loff.get(), R + 1);  // lcnt[R] = 0 (allocated zeroed)
            int64_t NL = 0;
            MI_HIP_CHECK(hipMemcpyAsync(&NL, loff.get() + R, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            if (NL >= (int64_t) INT32_MAX) return false;
            // the transpose's peak: the packed pairs, their sorted copy and the symmetric rows (both
            // triangles) live together once the slot pool is freed — gated on the same room as the pool
            const double tr_b = (double) NL * (double) (2 * (sizeof(uint32_t) + sizeof(lt_val<T>)) + 2 * (4 + sizeof(T))) +
                                4.0 * 8.0 * (double) (R + 1);
            if (tr_b > room) return false;
            const int64_t NLa = std::max<int64_t>(NL, 1);
            dev_buf<uint32_t> lk, ks;
            dev_buf<lt_val<T>> lvv, vs;
            lk.alloc(NLa, stream, false);
            lvv.alloc(NLa, stream, false);
            hipLaunchKernelGGL(exp_lt_compact_kernel<T>, dim3((unsigned) ceil_div(R, 4)), dim3(256), 0, stream, ls.get(),
                               lv.get(), lcnt.get(), loff.get(), R, cap, lk.get(), lvv.get());
            MI_LAUNCH_CHECK();
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            ls.reset(), lv.reset(), lb.reset(), le.reset();
            // the transpose: a stable sort of the pairs by partner (their row order kept within a partner)
            ks.alloc(NLa, stream, false);
            vs.alloc(NLa, stream, false);
            if (NL > 0) {
                int end_bit = 1;
                while (end_bit < 32 && (int64_t(1) << end_bit) < m) ++end_bit;
                size_t tb = 0;
                MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, lk.get(), ks.get(), lvv.get(), vs.get(), (int) NL,
                                                                0, end_bit, stream));
                dev_buf<unsigned char> t;
                t.alloc((int64_t) std::max<size_t>(tb, 16), stream, false);
                MI_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(t.get(), tb, lk.get(), ks.get(), lvv.get(), vs.get(), (int) NL,
                                                                0, end_bit, stream));
            }
            // the symmetric rows: row r = its lower list, then its upper list (ascending partners throughout)
            dev_buf<int64_t> tot, ustart;
            tot.alloc(R + 1, stream, false);
            ustart.alloc(R + 1, stream, false);
            hipLaunchKernelGGL(exp_lt_runs_kernel, dim3((unsigned) ceil_div(R + 1, 256)), dim3(256), 0, stream, ks.get(), NL,
                               lcnt.get(), R, ustart.get(), tot.get());
            MI_LAUNCH_CHECK();
            off8.alloc(R + 1, stream, false);
            excl(tot.get(), off8.get(), R + 1);
            MI_HIP_CHECK(hipMemcpyAsync(&nslot8, off8.get() + R, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            sj.alloc(std::max<int64_t>(nslot8, 8), stream, false);
            sv.alloc(std::max<int64_t>(nslot8, 8), stream, false);
            if (NL > 0) {
                hipLaunchKernelGGL(exp_lt_place_kernel<T>, dim3((unsigned) ceil_div(NL, 256)), dim3(256), 0, stream, lk.get(),
                                   lvv.get(), ks.get(), vs.get(), NL, loff.get(), lcnt.get(), ustart.get(), off8.get(),
                                   sj.get(), sv.get());
                MI_LAUNCH_CHECK();
            }
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            rbeg = off8.get();
            rend = off8.get() + 1;
            pt.mark("expansion: row join, transpose");
            return true;
        } catch (const std::exception &e) {
            if (exception_code(e) != -4) throw;
            (void) hipGetLastError();
            sj.reset(), sv.reset(), off8.reset();
            rbeg = rend = nullptr;
            return false;
        }
    };
    if (lt_join()) {
        ex.lt = true;
    } else {  // the full join recounts the pairs and the H bound; nothing the lower join read may survive it
        ex.pairs = 0;
        ex.hratio = -1.0;
    }
    if (row_join && R > 0 && rbeg == nullptr) {
        const char *rj = std::getenv("PLSSVM_MI_EXP_RJ");
        const bool want = !(rj != nullptr && std::strcmp(rj, "twopass") == 0);
        int64_t cap = round_up(std::max<int64_t>({ (int64_t) (2.0 * ex.rj_mean), (int64_t) (1.5 * ex.rj_max), 64 }), 8);
        if (const char *e = std::getenv("PLSSVM_MI_EXP_RJ_CAP")) {  // tests: force the overflow redo
            const long long v = std::atoll(e);
            if (v > 0) cap = v;
        }
        // the one-pass join's slot pool beside the structures the estimate counts: gated on the budget left over by the
        // estimate, both taken before the SELL plans' host thread allocates — the same choice on every run
        double room = (double) (csr.budget_b - csr.est_bytes);
        if (csr.budget_b <= 0) {
            size_t free_b = 0, total_b = 0;
            MI_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
            room = 0.4 * (double) free_b;
        }
        const double pool_b = (double) R * (double) cap * (double) (4 + sizeof(T));
        if (want && ex.rj_mean > 0.0 && pool_b <= room) {
            sj.alloc(R * cap, stream, false);
            cnt.alloc(R, stream);
            lnz.alloc(3, stream);  // [0] lower pairs with H != 0, [1] max |H| / kernel value (double bits), [2] max count
            dev_buf<unsigned int> ovf;
            ovf.alloc(1, stream);
            hipLaunchKernelGGL(exp_rowjoin_kernel, dim3((unsigned) R), dim3(RJ_NT), 0, stream, csr.rowptr.get(),
                               csr.col.get(), csr.colptr.get(), csr.crow.get(), m, r0, cnt.get(), (const int64_t *) nullptr,
                               sj.get(), ovf.get(), rj_pmax, cap, lnz.get() + 2, csplit.get(), nsplit);
            MI_LAUNCH_CHECK();
            unsigned long long cmax = 0ull;
            MI_HIP_CHECK(hipMemcpyAsync(&ovf_h, ovf.get(), sizeof(ovf_h), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipMemcpyAsync(&cmax, lnz.get() + 2, sizeof(cmax), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
            pt.mark("expansion: row join (one pass)");
            if (ovf_h != 0u) {  // a row whose partner clusters need more than RJ_PMAX passes: the sort join
                sj.reset(), cnt.reset();
                row_join = false;
            } else if ((int64_t) cmax > cap) {  // a row beyond its slots: the two-pass join with these exact counts
                sj.reset();
                have_cnt = true;
            } else {
                sv.alloc(R * cap, stream, false);
                pbeg.alloc(R, stream, false);
                pend.alloc(R, stream, false);
                hipLaunchKernelGGL(exp_pool_range_kernel, dim3((unsigned) ceil_div(R, 256)), dim3(256), 0, stream, cnt.get(),
                                   R, cap, pbeg.get(), pend.get());
                MI_LAUNCH_CHECK();
                rbeg = pbeg.get();
                rend = pend.get();
                h_pass();
                pt.mark("expansion: row join (H)");
            }
        }
    }
    if (row_join && rbeg == nullptr) {
        // two passes: count (unless the slot pass counted), padded offsets, then the write pass and H
        off8.alloc(R + 1, stream);
        if (!have_cnt) cnt.alloc(std::max<int64_t>(R, 1), stream);
        cnt8.alloc(R + 1, stream);
        lnz.alloc(3, stream);
        dev_buf<unsigned int> ovf;
        ovf.alloc(1, stream);
        if (R > 0 && !have_cnt) {
            hipLaunchKernelGGL(exp_rowjoin_kernel, dim3((unsigned) R), dim3(RJ_NT), 0, stream, csr.rowptr.get(),
                               csr.col.get(), csr.colptr.get(), csr.crow.get(), m, r0, cnt.get(),
                               (const int64_t *) nullptr, (int32_t *) nullptr, ovf.get(), rj_pmax, (int64_t) 0,
                               (unsigned long long *) nullptr, csplit.get(), nsplit);
            MI_LAUNCH_CHECK();
        }
        if (R > 0) {
            hipLaunchKernelGGL(exp_pad8_cnt_kernel, dim3((unsigned) ceil_div(R, 256)), dim3(256), 0, stream, cnt.get(),
                               R, cnt8.get());
            MI_LAUNCH_CHECK();
        }
        size_t tb = 0;
        MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt8.get(), off8.get(), (int) (R + 1), stream));
        {
            dev_buf<unsigned char> t;
            t.alloc((int64_t) std::max<size_t>(tb, 16), stream, false);
            MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(t.get(), tb, cnt8.get(), off8.get(), (int) (R + 1), stream));
            MI_HIP_CHECK(hipMemcpyAsync(&nslot8, off8.get() + R, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipMemcpyAsync(&ovf_h, ovf.get(), sizeof(ovf_h), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
        }
        pt.mark("expansion: row join (count)");
        if (ovf_h != 0u) {  // a row whose partner clusters need more than RJ_PMAX passes: the sort join
            off8.reset();
            row_join = false;
        } else {
            sj.alloc(std::max<int64_t>(nslot8, 8), stream, false);
            sv.alloc(std::max<int64_t>(nslot8, 8), stream, false);
            if (R > 0) {
                hipLaunchKernelGGL(exp_rowjoin_kernel, dim3((unsigned) R), dim3(RJ_NT), 0, stream, csr.rowptr.get(),
                                   csr.col.get(), csr.colptr.get(), csr.crow.get(), m, r0, cnt.get(), off8.get(), sj.get(),
                                   (unsigned int *) nullptr, rj_pmax, (int64_t) 0, (unsigned long long *) nullptr,
                                   csplit.get(), nsplit);
                MI_LAUNCH_CHECK();
            }
            rbeg = off8.get();
            rend = off8.get() + 1;
            h_pass();
            pt.mark("expansion: row join (rows)");
        }
    }
    if (!row_join) {
        sort_join();
        rbeg = off8.get();
        rend = off8.get() + 1;
    }
    pt.mark("expansion: symmetric rows");
    } catch (...) {
        fail1 = std::current_exception();
    }
    if (before_agree) {  // the caller's concurrent step (the SELL plans): joined here, its failure counts as ours
        std::exception_ptr e = before_agree();
        if (e && !fail1) fail1 = e;
    }
    // H storage (float contexts): bfloat16 when every stored |H_ij| is at most 2^-16 of its pair's kernel value
    // (the row join's hratio; see "H storage" below). A sharded group gathers bfloat16 w or real w by this flag
    // (expansion_kp_raw), so a real group takes it once: the AND over the ranks, after every rank's join.
    const char *hf = std::getenv("PLSSVM_MI_EXP_HFMT");
    bool hb_ok = !fail1 && sizeof(T) == 4 && ex.hratio >= 0.0 && ex.hratio <= std::ldexp(1.0, -16) &&
                 !(hf != nullptr && std::strcmp(hf, "full") == 0);
    if (in_group()) {
        int code = 0;
        std::string why;
        if (fail1) {
            try {
                std::rethrow_exception(fail1);
            } catch (const std::exception &e) {
                code = exception_code(e);
                why = e.what();
            } catch (...) {
                code = -1;
                why = "unknown exception in the expansion setup";
            }
        }
        const auto g = group_step(code, why, { hb_ok ? 1.0 : 0.0 });  // throws on every rank if any failed
        for (double v : g) hb_ok = hb_ok && v != 0.0;
    } else if (fail1) {
        std::rethrow_exception(fail1);
    }

    // ---- cells: blocks of RB rows x windows of CW partners, rows padded to 4 slots per cell ----
    // geometry: rows per block RB = the rank's rows spread evenly over the CUs (a multiple of 16: one
    // round of blocks, every CU busy), in the smallest accumulator class that holds it (the rest of the
    // LDS is the window). Few rows (an 8-GPU rank's share: blocks of less than half the largest class):
    // the largest class instead, and G window groups per row block to fill the CUs — every row block
    // restages all of w once, so fewer, bigger row blocks restage less. PLSSVM_MI_EXP_RBB forces a class.
    {
        int cus = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            cus = prop.multiProcessorCount;
        const int es = (int) sizeof(T);
        const int64_t Rr = std::max<int64_t>(R, 1), cap_max = 32768 / es;
        const int64_t want = round_up(ceil_div(Rr, (int64_t) cus), (int64_t) EXP_NWV);
        ex.G = 1;
        if (want * 2 > cap_max) {
            ex.RBB = 32768;
            for (int rbb : { 4096, 8192, 16384, 32768 }) {
                if (want * es <= rbb) {
                    ex.RBB = rbb;
                    break;
                }
            }
            ex.RB = (int) std::min<int64_t>(want, ex.RBB / es);
        } else {
            ex.RBB = 32768;
            int64_t nI = ceil_div(Rr, cap_max);
            ex.G = (int) std::max<int64_t>(1, cus / nI);
            // as many row blocks as the G window groups leave CUs (3-RBF: 128 x 2 = 256 workgroups, not 123 x 2)
            nI = std::max<int64_t>(nI, cus / ex.G);
            ex.RB = (int) round_up(ceil_div(Rr, nI), (int64_t) EXP_NWV);
        }
        if (const char *e = std::getenv("PLSSVM_MI_EXP_RBB")) {
            const int v = std::atoi(e);
            if (v == 4096 || v == 8192 || v == 16384 || v == 32768) ex.RBB = v, ex.RB = v / es, ex.G = 1;
        }
        if (const char *e = std::getenv("PLSSVM_MI_EXP_G")) {  // window groups (tests)
            const int v = std::atoi(e);
            if (v >= 1) ex.G = v;
        }
        ex.CW = exp_cw_host(ex.RBB, es);
    }
    const int64_t RB = ex.RB;
    ex.nblk = ceil_div(R, RB);
    const int64_t nbv = ex.nblk * EXP_NWV;
    {
        dev_buf<int64_t> cnt, coff;
        dev_buf<unsigned char> t;
        auto scan = [&](int64_t ncnt) {
            size_t tb = 0;
            MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt.get(), coff.get(), ncnt + 1, stream));
            t.alloc((int64_t) std::max<size_t>(tb, 16), stream, false);
            MI_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(t.get(), tb, cnt.get(), coff.get(), ncnt + 1, stream));
            MI_HIP_CHECK(hipMemcpyAsync(&ex.slots, coff.get() + ncnt, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
            MI_HIP_CHECK(hipStreamSynchronize(stream));
        };
        {
            // H storage (float contexts): bfloat16 H and bfloat16 windows of w when every stored |H_ij| is at most
            // 2^-16 of its pair's kernel value (row join's hratio). H_ij w_j is then formed from two values with
            // relative error <= 2^-9 each, so each pair's term moves by at most ~2^-8 |H_ij w_j| <= 2^-24 of
            // the pair's k_ij w_j — the float rounding of that term itself. PLSSVM_MI_EXP_HFMT=full keeps the
            // real type. The bfloat16 window holds twice the partners (fewer windows, fewer padded cells).
            // hb_ok: agreed by the whole group (above).
            ex.hbf16 = hb_ok;
            ex.CW = ex.hbf16 ? exp_cw16_host(ex.RBB) : exp_cw_host(ex.RBB, (int) sizeof(T));
            ex.nW = ceil_div(std::max<int64_t>(m, 1), (int64_t) ex.CW);
            const int64_t CW = ex.CW, ncnt = ex.nblk * RB * ex.nW;
            cnt.alloc(ncnt + 1, stream);
            coff.alloc(ncnt + 1, stream, false);
            auto count_cells = [&](int64_t gran) {
                if (R <= 0) return;
                hipLaunchKernelGGL(exp_cell_count_kernel<T>, dim3((unsigned) ceil_div(R, 4)), dim3(256), 0, stream,
                                   rbeg, rend, sj.get(), sv.get(), R, ex.nW, CW, RB, gran, cnt.get());
                MI_LAUNCH_CHECK();
            };
            count_cells(4);
            // flagged chunks (bfloat16 H only): when every |H| < 2 and the dummies of empty cells (16 B each) cost
            // at most half of the row indices they replace (2 B per chunk). PLSSVM_MI_EXP_ROWS=index keeps the
            // row index, =flags forces the flags (when the bit is free)
            ex.rflags = false;
            ex.rpairs = false;
            if (ex.hbf16 && R > 0) {
                const char *rs = std::getenv("PLSSVM_MI_EXP_ROWS");
                const int ropt = rs == nullptr ? 0
                                 : std::strcmp(rs, "index") == 0 ? -1
                                 : std::strcmp(rs, "flags") == 0 ? 1
                                 : std::strcmp(rs, "pairs") == 0 ? 2 : 0;
                if (ropt >= 0) {
                    dev_buf<unsigned long long> st;
                    st.alloc(2, stream);
                    hipLaunchKernelGGL(exp_cell_stats_kernel<T>, dim3((unsigned) ceil_div(R, 4)), dim3(256), 0, stream,
                                       rbeg, rend, sj.get(), sv.get(), R, ex.nW, CW, st.get());
                    MI_LAUNCH_CHECK();
                    unsigned long long hs2[2] = { 0ull, 0ull };
                    MI_HIP_CHECK(hipMemcpyAsync(hs2, st.get(), sizeof(hs2), hipMemcpyDeviceToHost, stream));
                    scan(ncnt);  // synchronises; ex.slots = the indexed layout's slots
                    const double chunks = (double) ex.slots / 4.0;
                    ex.rflags = hs2[1] == 0 && (ropt >= 1 || 16.0 * (double) hs2[0] <= 0.5 * 2.0 * chunks);
                    if (ex.rflags) {
                        hipLaunchKernelGGL(exp_cell_fill_empty_kernel, dim3((unsigned) ceil_div(R * ex.nW, 256)), dim3(256),
                                           0, stream, R, ex.nW, RB, (int64_t) 4, cnt.get());
                        MI_LAUNCH_CHECK();
                    }
                    // pair flags (round 5): the flags on slot pairs, cells padded to 2 slots instead of 4 (the 4-slot
                    // padding is ~15 % of the stream on config 5's 2M geometry). Taken when it saves >= 3 % of the
                    // chunk-flag layout's slots (PLSSVM_MI_EXP_ROWS=pairs forces it, =flags keeps the chunk flags)
                    if (ex.rflags && ropt != 1) {
                        scan(ncnt);
                        const int64_t slots4 = ex.slots;
                        MI_HIP_CHECK(hipMemsetAsync(cnt.get(), 0, sizeof(int64_t) * (size_t) (ncnt + 1), stream));
                        count_cells(2);
                        hipLaunchKernelGGL(exp_cell_fill_empty_kernel, dim3((unsigned) ceil_div(R * ex.nW, 256)), dim3(256),
                                           0, stream, R, ex.nW, RB, (int64_t) 2, cnt.get());
                        MI_LAUNCH_CHECK();
                        const int64_t ngroups = nbv * ex.nW, RPW = RB / EXP_NWV;
                        hipLaunchKernelGGL(exp_cell_pad_groups_kernel, dim3((unsigned) ceil_div(ngroups, 256)), dim3(256), 0,
                                           stream, ngroups, RPW, cnt.get());
                        MI_LAUNCH_CHECK();
                        scan(ncnt);
                        ex.rpairs = ropt == 2 || (double) ex.slots <= 0.97 * (double) slots4;
                        if (!ex.rpairs) {  // back to the chunk-flag counts
                            MI_HIP_CHECK(hipMemsetAsync(cnt.get(), 0, sizeof(int64_t) * (size_t) (ncnt + 1), stream));
                            count_cells(4);
                            hipLaunchKernelGGL(exp_cell_fill_empty_kernel, dim3((unsigned) ceil_div(R * ex.nW, 256)),
                                               dim3(256), 0, stream, R, ex.nW, RB, (int64_t) 4, cnt.get());
                            MI_LAUNCH_CHECK();
                        }
                    }
                }
            }
            scan(ncnt);
            ex.nchunks = ex.slots / 4;
            // EXP_NH x 64 chunks of zeroed padding past the stream's end: the remainder stream's loads of a step
            // past the end read padding (masked) instead of clamping each lane's 64-bit address
            const int64_t spad = std::max<int64_t>(ex.slots, 4) + (int64_t) EXP_NH * 64 * 4;
            ex.hjl.alloc(spad * (ex.rflags && EXP_JH ? 2 : 1), stream);
            if (ex.hbf16) {
                if (ex.rflags && EXP_JH) ex.hv16.reset();
                else ex.hv16.alloc(spad, stream);
                ex.wv16.alloc(round_up(std::max<int64_t>({ m, chunk * G, 8 }), (int64_t) 8), stream);
            }
            else ex.hv.alloc(spad, stream);
            if (ex.rflags) {
                ex.hrow.reset();
                hipLaunchKernelGGL(exp_cell_scatter_flag_kernel<T>, dim3((unsigned) ceil_div(R, 4)), dim3(256), 0, stream,
                                   rbeg, rend, sj.get(), sv.get(), R, ex.nW, CW, RB, coff.get(), ex.hjl.get(),
                                   EXP_JH ? ex.hjl.get() : ex.hv16.get());
                MI_LAUNCH_CHECK();
            } else {
                ex.hrow.alloc(std::max<int64_t>(ex.nchunks, 1) + (int64_t) EXP_NH * 64, stream);
                if (R > 0) {
                    hipLaunchKernelGGL(exp_cell_scatter_kernel<T>, dim3((unsigned) ceil_div(R, 4)), dim3(256), 0, stream,
                                       rbeg, rend, sj.get(), sv.get(), R, ex.nW, CW, RB, coff.get(), ex.hjl.get(),
                                       ex.hv.get(), ex.hv16.get(), ex.hrow.get());
                    MI_LAUNCH_CHECK();
                }
            }
            ex.woff.alloc(std::max<int64_t>(nbv * (ex.nW + 1), 1), stream);
            if (nbv > 0) {
                hipLaunchKernelGGL(exp_cell_woff_kernel, dim3((unsigned) ceil_div(nbv * (ex.nW + 1), 256)), dim3(256),
                                   0, stream, coff.get(), nbv, ex.nW, RB, ex.woff.get());
                MI_LAUNCH_CHECK();
            }
        }
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
    ex.G = (int) std::max<int64_t>(1, std::min<int64_t>(ex.G, ex.nW));
    if (ex.G > 1) ex.hslab.alloc((int64_t) ex.G * R, stream, false);
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    pt.mark("expansion: cells");
    csr.pairs = ex.pairs;
    csr.slots = ex.slots;
    csr.rbf_factored = kernel == 2;
    ex.on = true;
}

// timing/test-only ablations (results are wrong when non-zero): PLSSVM_MI_EXP_ABLATE bit 0 = drop the
// stored remainder H of the multi-feature pairs, bit 1 = keep only the first term of phi's polynomial, bit 2 =
// the remainder stream skips the last partner window of every row block (chunk layouts)
int exp_ablate() {
    static const int v = [] {
        const char *s = std::getenv("PLSSVM_MI_EXP_ABLATE");
        return s ? std::atoi(s) : 0;
    }();
    return v;
}

// the remainder stream alone (the dominant kernel of the expansion's K·p; time_kp / bench roofline)
template <typename T>
void engine<T>::expansion_dominant(const T *w, const cg_scalars<T> *status) {
    auto &ex = csr.ex;
    if (ex.nblk > 0 && !(exp_ablate() & 1)) {
        auto launch = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned) (ex.nblk * ex.G)), dim3(EXP_NWV * 64), 0, stream, ex.woff.get(),
                               ex.hrow.get(), ex.hjl.get(), ex.hv.get(), ex.hv16.get(), w, ex.wv16.get(), m, r0, r1 - r0, ex.nW,
                               (int64_t) ex.RB, ex.nblk, ex.G, ex.hs.get(), ex.hslab.get(), status, (exp_ablate() & 4) ? 1 : 0);
        };
        {
            auto pick = [&](auto hb, auto rf, auto d2) {
                constexpr bool HB = decltype(hb)::value, D2 = decltype(d2)::value;
                constexpr int RF = decltype(rf)::value;
                switch (ex.RBB) {
                    case 4096: launch(exp_hcell_kernel<T, 4096, HB, RF, D2>); break;
                    case 8192: launch(exp_hcell_kernel<T, 8192, HB, RF, D2>); break;
                    case 32768: launch(exp_hcell_kernel<T, 32768, HB, RF, D2>); break;
                    default: launch(exp_hcell_kernel<T, 16384, HB, RF, D2>);
                }
            };
            const bool dot2 = ex.dot2;
            using R0 = std::integral_constant<int, 0>;
            using R1 = std::integral_constant<int, 1>;
            using R2 = std::integral_constant<int, 2>;
            if constexpr (sizeof(T) == 4) {
                if (ex.hbf16 && ex.rpairs && dot2) pick(std::true_type{}, R2{}, std::true_type{});
                else if (ex.hbf16 && ex.rpairs) pick(std::true_type{}, R2{}, std::false_type{});
                else if (ex.hbf16 && ex.rflags && dot2) pick(std::true_type{}, R1{}, std::true_type{});
                else if (ex.hbf16 && ex.rflags) pick(std::true_type{}, R1{}, std::false_type{});
                else if (ex.hbf16 && dot2) pick(std::true_type{}, R0{}, std::true_type{});
                else if (ex.hbf16) pick(std::true_type{}, R0{}, std::false_type{});
                else pick(std::false_type{}, R0{}, std::true_type{});
            } else {
                pick(std::false_type{}, R0{}, std::true_type{});
            }
        }
        MI_LAUNCH_CHECK();  // G > 1: the row sums stay in hslab, summed in g order by exp_combine_kernel
    } else if (r1 > r0) {
        MI_HIP_CHECK(hipMemsetAsync(ex.hs.get() + r0, 0, sizeof(T) * (size_t) (r1 - r0), stream));
        if (ex.G > 1) MI_HIP_CHECK(hipMemsetAsync(ex.hslab.get(), 0, sizeof(T) * (size_t) (ex.G * (r1 - r0)), stream));
    }
}

// the column-moment pass (SELL CSC pass, mode 1) over rows [csc_r0, csc_r1); several panels: their slabs are
// reduced straight into the scaled Horner coefficients M (returns true), one panel: the pass wrote the raw
// moments mom, scaled by expansion_mscale after the group's all-reduce (returns false)
template <typename T>
bool engine<T>::expansion_moments_fused() const {
    const auto &pl = csr.spmv_csc;
    return pl.P > 1 && pl.nseg == d && pl.nblocks > 0;
}

// spart != null (fused passes only): the moment reduce also forms S = csr.ssc from w's partials (sG sets)
template <typename T>
bool engine<T>::expansion_moment_pass(const T *w, const cg_scalars<T> *status, const T *spart, int sG) {
    auto &ex = csr.ex;
    const auto &pl = csr.spmv_csc;
    const bool fused = expansion_moments_fused();
    launch_panel_spmv<T>(pl, w + csr.csc_r0, csr.csc_r1 - csr.csc_r0, ex.mom.get(), status, stream, ex.KM, 1, !fused);
    if (fused) {
        const int split = pl.P >= 16 ? 1 : 0;
        const unsigned nb = (unsigned) ceil_div(d * ex.KM, split ? 64 : 256) + (spart != nullptr ? 1u : 0u);
        hipLaunchKernelGGL(exp_mom_reduce_kernel<T>, dim3(nb), dim3(256), 0, stream, pl.partial.get(), pl.P, d, ex.KM, split,
                           expansion_coefs(), ex.M.get(), spart, sG, csr.ssc.get(), status);
        MI_LAUNCH_CHECK();
    }
    return fused;
}

template <typename T>
void engine<T>::expansion_moments(const T *w, const cg_scalars<T> *status, const T *spart, int sG) {
    auto &ex = csr.ex;
    if (d > 0) {  // column moments, then the coefficients (a real group: each rank's rows, then one
        // all-reduce of the d x K values — linear, so the scaled coefficients are all-reduced when fused)
        const bool fused = expansion_moment_pass(w, status, spart, sG);
        if (csr.csc_r1 - csr.csc_r0 < m) allreduce(fused ? ex.M.get() : ex.mom.get(), d * ex.KM);
        if (!fused) expansion_mscale(status);
    }
}

template <typename T>
coefs engine<T>::expansion_coefs() const {
    coefs cf;
    std::memcpy(cf.c, csr.ex.coef, sizeof(cf.c));
    if (exp_ablate() & 2)
        for (int k = 2; k <= EXP_KMAX; ++k) cf.c[k] = 0.0;
    return cf;
}

// M[f][k] = coef_{k+1} mom[k][f] (after the group's all-reduce of the moments)
template <typename T>
void engine<T>::expansion_mscale(const cg_scalars<T> *status) {
    auto &ex = csr.ex;
    if (d <= 0) return;
    hipLaunchKernelGGL(exp_mscale_kernel<T>, dim3((unsigned) ceil_div(d * ex.KM, 256)), dim3(256), 0, stream,
                       ex.mom.get(), d, ex.KM, expansion_coefs(), ex.M.get(), status);
    MI_LAUNCH_CHECK();
}

// The CG direction update carries the next K·p's w pass (round 5): with bfloat16 windows the K·p of d starts with
// exp_wown_kernel over the rows the direction update has just written (w = e d, its bfloat16 copy, S partials); the
// update forms them in its own element loop (cgk::w_elem, the same grid and order: the same bits) and the K·p skips
// the launch. Sharded: the rank's rows, whose w the group then gathers as before. (Measured neutral, round 5.)
template <typename T>
bool engine<T>::dir_w_fill(dir_w_t<T> &o) {
    if (!sparse_stored() || factored() || csr.otf_on || !csr.ex.on || !csr.ex.hbf16) return false;
    if (shard) {  // expansion_kp_raw's g16 over [r0, r1)
        const bool rgrp = comm != nullptr && cstream != nullptr;
        if (d <= 0 || !(rgrp || sim_world > 0) || v0 != r0 || vn != r1 - r0) return false;
    } else if (v0 != 0 || vn != m) {  // wown_all over [0, m)
        return false;
    }
    o.e = kernel == 2 ? csr.e.get() + v0 : nullptr;
    o.w = kernel == 2 ? csr.ex.wv.get() + v0 : nullptr;
    o.w16 = csr.ex.wv16.get() + v0;
    o.cw = ctr_active() && kernel == 2 ? ctr_cw.get() + v0 : nullptr;
    o.spart = wsp.get();
    return true;
}

template <typename T>
void engine<T>::expansion_kp_raw(const T *p, const cg_scalars<T> *status, bool with_base) {
    auto &ex = csr.ex;
    // sharded: w of this rank's rows, then gathered from every rank (the remainder stream reads partners of
    // all rows); the raw of this rank's rows stays local (no row gather)
    const int64_t ib = shard ? r0 : 0, ie = shard ? r1 : m;
    const T *w = p;
    // sharded RCCL group with bfloat16 windows: the bfloat16 w (2 B per row) is what the group gathers
    // (a simulated rank of such a group runs the same kernels without the collectives: timing only)
    const bool rgrp = shard && comm != nullptr && cstream != nullptr && d > 0;
    const bool g16 = shard && d > 0 && ex.hbf16 && (rgrp || sim_world > 0);
    // unsharded with bfloat16 windows: w, its bfloat16 copy and the S partials in one pass (exp_wown_kernel over
    // all rows: exp_w_kernel's w and exp_wsum_kernel's partials, bit for bit)
    const bool wown_all = !shard && ex.hbf16;
    // centered finalize (engine.hpp ctr_*): S becomes S_c = sum_j cw_j w_j, the combine's base c_i S_c (rbf) / 0 (poly)
    const T *cw = ctr_now && kernel == 2 ? ctr_cw.get() : nullptr;
    // the w pass's S partials (spt): wsp for exp_wown_kernel and the direction update that carries it (w_pre == p:
    // done, dir_w_fill), red for exp_wsum_kernel
    T *spt = (g16 || wown_all) ? wsp.get() : red.get();
    const bool pre = (g16 || wown_all) && w_pre != nullptr && w_pre == p;
    w_pre = nullptr;  // any other w pass below overwrites w, its copy and the partials
    if (g16 || wown_all) {
        if (!pre) {
            hipLaunchKernelGGL(exp_wown_kernel<T>, dim3(RED_BLOCKS), dim3(cgk::CG_NT), 0, stream,
                               kernel == 2 ? csr.e.get() : nullptr, p, ib, ie, ex.wv.get(), ex.wv16.get(), cw, spt, status);
            MI_LAUNCH_CHECK();
        }
        if (kernel == 2) w = ex.wv.get();
    } else if (kernel == 2) {
        if (ie > ib)
            hipLaunchKernelGGL(exp_w_kernel<T>, dim3((unsigned) ceil_div(ie - ib, 256)), dim3(256), 0, stream,
                               csr.e.get() + ib, p + ib, ie - ib, ex.wv.get() + ib, status);
        MI_LAUNCH_CHECK();
        w = ex.wv.get();
    }
    if (rgrp) {
        // sharded RCCL group: the all-gather of w (with the pending CG partials) and the all-reduce of the
        // moments run on the collective stream, overlapping the moments pass and the remainder stream
        MI_HIP_CHECK(hipEventRecord(cev[0], stream));
        MI_HIP_CHECK(hipStreamWaitEvent(cstream, cev[0], 0));
        MI_NCCL_CHECK(ncclGroupStart());
        if (psum_pending) {  // the previous CG step's direction partials ride along
            MI_NCCL_CHECK(ncclAllGather(cgp.get(), cgp_g.get(), (size_t) (2 * RED_BLOCKS), nccl_type<T>(), comm, cstream));
            psum_pending = false;
        }
        T *sg = cgp_g.get() + (int64_t) 4 * G * 2 * RED_BLOCKS;  // slot 4: the ranks' S partials
        if (g16) {
            MI_NCCL_CHECK(ncclAllGather(ex.wv16.get() + (int64_t) rank * chunk, ex.wv16.get(), (size_t) chunk, ncclBfloat16,
                                        comm, cstream));
            MI_NCCL_CHECK(ncclAllGather(spt, sg, (size_t) (2 * RED_BLOCKS), nccl_type<T>(), comm, cstream));
        } else {
            MI_NCCL_CHECK(ncclAllGather(const_cast<T *>(w) + (int64_t) rank * chunk, const_cast<T *>(w), (size_t) chunk,
                                        nccl_type<T>(), comm, cstream));
        }
        MI_NCCL_CHECK(ncclGroupEnd());
        MI_HIP_CHECK(hipEventRecord(cev[1], cstream));
        const bool fused = expansion_moment_pass(w, status);
        T *mt = fused ? ex.M.get() : ex.mom.get();
        MI_HIP_CHECK(hipEventRecord(cev[2], stream));
        MI_HIP_CHECK(hipStreamWaitEvent(cstream, cev[2], 0));
        MI_NCCL_CHECK(ncclAllReduce(mt, mt, (size_t) (d * ex.KM), nccl_type<T>(), ncclSum, comm, cstream));
        MI_HIP_CHECK(hipEventRecord(cev[3], cstream));
        MI_HIP_CHECK(hipStreamWaitEvent(stream, cev[1], 0));  // w of every rank
        if (g16) {  // S from the ranks' partials, in rank order
            launch_dot_final<T>(sg, sc.get(), FIN_PLAIN, 0, nullptr, 0, csr.ssc.get(), stream, G);
        } else {
            hipLaunchKernelGGL(exp_wsum_kernel<T>, dim3(RED_BLOCKS), dim3(256), 0, stream, w, m,
                               ex.hbf16 ? ex.wv16.get() : nullptr, cw, red.get(), status);  // S = sum_j w_j (+ bf16 w)
            MI_LAUNCH_CHECK();
            launch_dot_final<T>(red.get(), sc.get(), FIN_PLAIN, 0, nullptr, 0, csr.ssc.get(), stream);
        }
        expansion_dominant(w, status);
        MI_HIP_CHECK(hipStreamWaitEvent(stream, cev[3], 0));  // the group's moments
        if (!fused) expansion_mscale(status);
    } else if (g16) {
        // S from w's partials: inside the moment reduce when the moment pass has one (one launch fewer)
        const bool sfold = d > 0 && expansion_moments_fused();
        if (!sfold) launch_dot_final<T>(spt, sc.get(), FIN_PLAIN, 0, nullptr, 0, csr.ssc.get(), stream);
        expansion_moments(w, status, sfold ? spt : nullptr, 1);
        expansion_dominant(w, status);
    } else {
        gather_input(w);
        if (!wown_all) {
            hipLaunchKernelGGL(exp_wsum_kernel<T>, dim3(RED_BLOCKS), dim3(256), 0, stream, w, m,
                               ex.hbf16 ? ex.wv16.get() : nullptr, cw, red.get(), status);  // S = sum_j w_j (+ bf16 w)
            MI_LAUNCH_CHECK();
        }
        const bool sfold = d > 0 && expansion_moments_fused();
        if (!sfold) launch_dot_final<T>(spt, sc.get(), FIN_PLAIN, 0, nullptr, 0, csr.ssc.get(), stream);
        expansion_moments(w, status, sfold ? spt : nullptr, 1);
        expansion_dominant(w, status);
    }
    T kappa = 0;
    if (kernel == 1 && !ctr_now) {
        kappa = 1;
        for (int q2 = 0; q2 < degree; ++q2) kappa *= coef0;
    }
    const T *cb = ctr_now && kernel == 2 ? ctr_c.get() : nullptr;
    // J_i = sum_{f in x_i} sum_k x_if^(k+1) M[f][k]: one SELL pass over this rank's CSR rows (mode 2)
    // (few panels: the combine sums the pass's panel slabs itself, one launch fewer)
    const auto &pc = csr.spmv_csr;
    const bool jfuse = pc.P > 1 && pc.P < 16 && pc.nseg == r1 - r0 && pc.nblocks > 0;
    if (r1 > r0) launch_panel_spmv<T>(pc, ex.M.get(), d, raw.get() + r0, status, stream, ex.KM, 2, !jfuse);
    // a CG iteration on its own rows (one GPU, or a sharded rank): the combine and the iteration's finalize in
    // one launch (the gathered partials it needs are in place: carried by the K·p's collective or flushed here)
    if (kp_fin_req != nullptr && with_base && r1 > r0 && ib == r0 && ie == r1 && ib == v0 && ie - ib == vn &&
        (shard || (world == 1 && sim_world == 0))) {
        flush_psum();
        const kp_fin_t &f = *kp_fin_req;
        hipLaunchKernelGGL(exp_combine_fin_kernel<T>, dim3(RED_BLOCKS), dim3(cgk::CG_NT), 0, stream,
                           kernel == 2 ? csr.e.get() : nullptr, cb, w, ex.hdiag.get(), ex.hs.get(),
                           ex.G > 1 ? ex.hslab.get() : nullptr, ex.G, jfuse ? pc.partial.get() : nullptr, (int) pc.P,
                           raw.get(), csr.ssc.get(), kappa, r0, r1, f.q, f.d, f.psum, f.G, f.QA_cost, f.cost_inv, f.Ad,
                           f.pdad, sc.get());
        MI_LAUNCH_CHECK();
        kp_fin_done = true;
        return;  // sharded (or one rank): nothing to gather
    }
    if (ie > ib)
        hipLaunchKernelGGL(exp_combine_kernel<T>, dim3((unsigned) ceil_div(ie - ib, 256)), dim3(256), 0, stream,
                           kernel == 2 ? csr.e.get() : nullptr, cb, w, ex.hdiag.get(), ex.phin.get(), ex.hs.get(),
                           ex.G > 1 ? ex.hslab.get() : nullptr, ex.G, jfuse ? pc.partial.get() : nullptr, (int) pc.P,
                           csr.ssc.get(), kappa, ib, ie, r0, r1, with_base ? 0 : (part_mode == 2 ? 2 : 1), raw.get(), status);
    MI_LAUNCH_CHECK();
    if (!shard) allgather_rows(raw.get());
}

// ---- centered rank-1 terms of the finalize (engine.hpp ctr_*) -------------------------------------------------
// per row i < m, in fp64 from the row's entries and the last point x_m (dense, xlast):
//   rbf:  c_i = e_i - e_m = e_m expm1(gamma (|x_m|^2 - |x_i|^2)),  cw_i = c_i / e_i = -expm1(gamma (|x_i|^2 - |x_m|^2)),
//         h_i = e_i e_m expm1(2 gamma x_i.x_m)
//   poly: h_i = (gamma x_i.x_m + c0)^deg - c0^deg as its binomial sum (no cancellation)
// bad = 1 when a value does not fit the real type (then the plain finalize is used)
template <typename T>
__global__ __launch_bounds__(256) void exp_ctr_kernel(int kernel, int degree, double gamma, double coef0,
                                                      const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
                                                      vals_t<T> val, int64_t m, const T *__restrict__ xlast, double nlast,
                                                      const T *__restrict__ norms, double em, T *__restrict__ c,
                                                      T *__restrict__ cw, T *__restrict__ h, int *__restrict__ bad) {
    const int64_t row = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= m) return;
    double s = 0;
    for (int64_t k = rowptr[row]; k < rowptr[row + 1]; ++k) s = fma((double) val[k], (double) xlast[col[k]], s);
    const double lim = sizeof(T) == 4 ? 1e37 : 1e307;
    if (kernel == 2) {
        const double ni = (double) norms[row];
        const double ei = exp(-gamma * ni);
        const double ci = em * expm1(gamma * (nlast - ni)), cwi = -expm1(gamma * (ni - nlast));
        const double hi = ei * em * expm1(2.0 * gamma * s);
        if (!(fabs(cwi) < lim) || !(fabs(hi) < lim)) *bad = 1;
        c[row] = (T) ci;
        cw[row] = (T) cwi;
        h[row] = (T) hi;
    } else {
        const double u = gamma * s;
        double hi = 0, binom = 1, uk = 1;
        for (int k = 1; k <= degree; ++k) {
            binom = binom * (double) (degree - k + 1) / (double) k;
            uk *= u;
            double c0p = 1;
            for (int t = 0; t < degree - k; ++t) c0p *= coef0;
            hi += binom * c0p * uk;
        }
        if (!(fabs(hi) < lim)) *bad = 1;
        h[row] = (T) hi;
    }
}

template <typename T>
bool engine<T>::ctr_active() const {
    return ctr_ok && q_gen && sparse && !csr.dense_on && csr.ex.on && !csr.otf_on && (kernel == 1 || kernel == 2);
}

template <typename T>
T engine<T>::QAf() const {
    if (!ctr_active()) return QA_cost;
    // a caller's QA_cost (plssvm_mi_set_qa_cost) that differs from k_mm + 1/C keeps its difference
    return (T) (ctr_hm + (double) cost_inv()) + (QA_cost - (ctr_kmm + T(1) / cost));
}

template <typename T>
void engine<T>::ctr_setup() {
    ctr_ok = false;
    const char *cv = std::getenv("PLSSVM_MI_CTR");  // read per setup: tests compare both finalizes in one process
    const int mode = cv == nullptr ? 1 : std::atoi(cv);
    if (mode == 0 || !sparse || csr.dense_on || !csr.ex.on || csr.otf_on || (kernel != 1 && kernel != 2) || m <= 0) return;
    double nlast = 0;
    for (int64_t k = 0; k < d; ++k) nlast = std::fma((double) xlast_h[k], (double) xlast_h[k], nlast);
    const double g = (double) gamma, em = std::exp(-g * nlast);
    if (kernel == 2) {
        ctr_hm = -std::expm1(-2.0 * g * nlast);  // e_m^2 expm1(2 gamma |x_m|^2) = 1 - e_m^2
    } else {
        double hm = 0, binom = 1, uk = 1;
        for (int k = 1; k <= degree; ++k) {
            binom = binom * (double) (degree - k + 1) / (double) k;
            uk *= g * nlast;
            double c0p = 1;
            for (int t = 0; t < degree - k; ++t) c0p *= (double) coef0;
            hm += binom * c0p * uk;
        }
        ctr_hm = hm;
    }
    const int64_t len = q.size();
    ctr_h.alloc(len, stream);
    if (kernel == 2) {
        ctr_c.alloc(len, stream);
        ctr_cw.alloc(len, stream);
    }
    dev_buf<int> bad;
    bad.alloc(1, stream);
    hipLaunchKernelGGL(exp_ctr_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, kernel, degree, g,
                       (double) coef0, csr.rowptr.get(), csr.col.get(), csr.rvals(), m, xlast.get(), nlast, norms.get(),
                       em, ctr_c.get(), ctr_cw.get(), ctr_h.get(), bad.get());
    MI_LAUNCH_CHECK();
    int hb = 0;
    MI_HIP_CHECK(hipMemcpyAsync(&hb, bad.get(), sizeof(int), hipMemcpyDeviceToHost, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    ctr_ok = hb == 0;
}

// ---- predict through the expansion (csvm::predict on sparse poly / rbf models) -----------------------
// sum_{i<m} alpha_i k(x_i, z) = base_z (S + J_z + sum_{i sharing >= 2 features with z} w_i H_iz), with
// w = alpha e (rbf) / alpha (poly), S = sum w, J_z = sum_{f in z} sum_k coef_k z_f^k M_k(f) from the
// model's column moments M_k(f) = sum_{i in col f} x_if^k w_i (once per call), and H_iz = phi(s_iz) -
// sum_{f shared} phi(x_if z_f) for the support vectors sharing two or more features with z: per point,
// the CSC columns of z's features are walked with an LDS bitmap of rows (seen once / twice), the repeat
// rows are enumerated in ascending order and their exact s_iz and phi sums formed by merging row i with
// z. Fixed orders throughout: deterministic. O(nnz_z K + sum_{f in z} c_f) per point instead of O(nnz_X).
constexpr int PRED_NT = 1024;
constexpr int PRED_BMW = 24576;             // bitmap words (96 KiB): rows per pass = 786 432
constexpr int PRED_ZCAP = 2048;             // entries of one point held in LDS
constexpr int PRED_MCAP = 4096;             // repeat rows per pass

template <typename T>
__global__ __launch_bounds__(256) void exp_pred_w_kernel(const T *__restrict__ alpha, const T *__restrict__ e, int64_t m,
                                                         T *__restrict__ w) {
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) w[i] = e != nullptr ? alpha[i] * e[i] : alpha[i];
}

// M[f][k] = coef_{k+1} sum_{t in col f} cval[t]^(k+1) w[crow[t]], one wave per column (lane-strided,
// then a butterfly: fixed order)
template <typename T>
__global__ __launch_bounds__(256) void exp_pred_moments_kernel(const int64_t *__restrict__ colptr,
                                                               const int32_t *__restrict__ crow,
                                                               const T *__restrict__ cval, const T *__restrict__ w,
                                                               int64_t d, int K, int KM, coefs cf, T *__restrict__ M) {
    const int64_t f = (int64_t) blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (f >= d) return;
    double acc[EXP_KMAX];
#pragma unroll
    for (int k = 0; k < EXP_KMAX; ++k) acc[k] = 0.0;
    for (int64_t t = colptr[f] + lane; t < colptr[f + 1]; t += 64) {
        const double v = (double) cval[t];
        double pw = v * (double) w[crow[t]];
#pragma unroll
        for (int k = 0; k < EXP_KMAX; ++k) {
            if (k < K) acc[k] += pw;
            pw *= v;
        }
    }
#pragma unroll
    for (int k = 0; k < EXP_KMAX; ++k) {
        if (k < K) {  // K is uniform
            double a = acc[k];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o);
            if (lane == 0) M[f * KM + k] = (T) (cf.c[k + 1] * a);
        }
    }
    if (lane == 0)
        for (int k = K; k < KM; ++k) M[f * KM + k] = T(0);
}

template <typename T>
__device__ __forceinline__ double pred_block_sum(double v, double *red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
    for (int w2 = 0; w2 < PRED_NT / 64; ++w2) s += red[w2];
    return s;
}

// one point per workgroup; zr/zc/zv: the points' CSR (columns ascending); S: sum w (device scalar);
// flag[0] set when a pass held more than PRED_MCAP repeat rows (the caller then recomputes brute force)
template <typename T>
__global__ __launch_bounds__(PRED_NT) void exp_pred_point_kernel(
    const int64_t *__restrict__ zr, const int32_t *__restrict__ zc, const T *__restrict__ zv, const int64_t *__restrict__ colptr,
    const int32_t *__restrict__ crow, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const T *__restrict__ val, const T *__restrict__ w, const T *__restrict__ M, int KM, phi_fn phi, int64_t m,
    const T *__restrict__ S, const T *__restrict__ xlast, T nlast, T alpha_m, kfun<T> kf, T kappa, T bias,
    T *__restrict__ out, int *__restrict__ flag) {
    __shared__ uint32_t bm[PRED_BMW];
    __shared__ int32_t zcol_s[PRED_ZCAP];
    __shared__ T zval_s[PRED_ZCAP];
    __shared__ int32_t multi[PRED_MCAP];
    __shared__ int64_t zoff[PRED_ZCAP + 1];
    __shared__ double red[PRED_NT / 64];
    __shared__ int nmulti, wcnt[PRED_NT];
    const int tid = threadIdx.x;
    const int64_t p = blockIdx.x;
    const int64_t e0 = zr[p];
    const int nz = (int) (zr[p + 1] - e0);
    // the point's entries, x_m at its columns and its columns' CSC lengths: one parallel read each (a serial
    // loop of dependent global reads in one thread cost ~1 us per entry); x_m's values borrow the bitmap's LDS,
    // which every pass below clears before use
    static_assert(PRED_ZCAP * sizeof(T) <= PRED_BMW * sizeof(uint32_t), "x_m staging must fit the bitmap");
    T *xl_s = reinterpret_cast<T *>(bm);
    for (int e = tid; e < nz; e += PRED_NT) {
        const int32_t f = zc[e0 + e];
        zcol_s[e] = f;
        zval_s[e] = zv[e0 + e];
        xl_s[e] = xlast[f];
        zoff[e + 1] = colptr[f + 1] - colptr[f];
    }
    __syncthreads();
    // |z|^2 (column order) and x_m . z (entry order), thread 0, from LDS
    if (tid == 0) {
        T nzz = 0, dl = 0;
        for (int e = 0; e < nz; ++e) {
            nzz = fma(zval_s[e], zval_s[e], nzz);
            dl = fma(xl_s[e], zval_s[e], dl);
        }
        red[0] = (double) nzz;
        red[1] = (double) dl;
        // CSC offsets of z's columns (flattened incidences)
        zoff[0] = 0;
        for (int e = 0; e < nz; ++e) zoff[e + 1] += zoff[e];
    }
    __syncthreads();
    const T nzz = (T) red[0], dl = (T) red[1];
    const int64_t inc = zoff[nz];
    // J_z = sum_e z_e (M0 + z_e (M1 + ...)) in the real type's Horner order
    double js = 0.0;
    for (int e = tid; e < nz; e += PRED_NT) {
        const T z = zval_s[e];
        const T *Mf = M + (int64_t) zcol_s[e] * KM;
        T h = Mf[KM - 1];
        for (int k = KM - 2; k >= 0; --k) h = fma(h, z, Mf[k]);
        js += (double) (h * z);
    }
    const double J = pred_block_sum<T>(js, red);
    double hs = 0.0;
    const int64_t BMBITS = (int64_t) PRED_BMW * 32;
    for (int64_t R0 = 0; R0 < m; R0 += BMBITS) {
        const int64_t R1 = min(m, R0 + BMBITS);
        for (int q = tid; q < PRED_BMW; q += PRED_NT) bm[q] = 0u;
        if (tid == 0) nmulti = 0;
        __syncthreads();
        // rows seen once -> bit set; seen again -> appended (duplicates for 3+ shared features)
        for (int64_t t = tid; t < inc; t += PRED_NT) {
            int lo = 0, hi = nz - 1;  // entry e with zoff[e] <= t < zoff[e + 1]
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (zoff[mid] <= t) lo = mid;
                else hi = mid - 1;
            }
            const int64_t i = crow[colptr[zcol_s[lo]] + (t - zoff[lo])];
            if (i < R0 || i >= R1) continue;
            const uint32_t bit = 1u << ((i - R0) & 31);
            const uint32_t old = atomicOr(&bm[bm_addr<PRED_BMW / PRED_NT, PRED_NT>((i - R0) >> 5)], bit);
            if (old & bit) {
                const int q = atomicAdd(&nmulti, 1);
                if (q < PRED_MCAP) multi[q] = (int32_t) i;
            }
        }
        __syncthreads();
        const int nm = nmulti;
        if (nm > PRED_MCAP) {
            if (tid == 0) flag[0] = 1;
            return;  // uniform: every thread read the same nmulti
        }
        // the repeat rows as a set in the bitmap, then enumerated in ascending row order
        for (int q = tid; q < PRED_BMW; q += PRED_NT) bm[q] = 0u;
        __syncthreads();
        for (int q = tid; q < nm; q += PRED_NT) {
            const int64_t i = multi[q] - R0;
            atomicOr(&bm[bm_addr<PRED_BMW / PRED_NT, PRED_NT>(i >> 5)], 1u << (i & 31));
        }
        __syncthreads();
        constexpr int WPT = PRED_BMW / PRED_NT;
        int c = 0;
        for (int q = 0; q < WPT; ++q) c += __popc(bm[q * PRED_NT + tid]);
        // exclusive block scan of the counts (wave scans, then the wave totals), not a serial loop over 1024
        const int lane = tid & 63, wave = tid >> 6;
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        if (lane == 63) wcnt[wave] = incl;
        __syncthreads();
        int before = 0, tot = 0;
        for (int w2 = 0; w2 < PRED_NT / 64; ++w2) {
            const int v = wcnt[w2];
            if (w2 < wave) before += v;
            tot += v;
        }
        if (tid == 0) nmulti = tot;
        {
            int pos = before + incl - c;
            for (int q = 0; q < WPT; ++q) {
                uint32_t word = bm[q * PRED_NT + tid];
                while (word) {
                    const int b = __ffs(word) - 1;
                    word &= word - 1;
                    multi[pos++] = (int32_t) (R0 + (int64_t) (tid * WPT + q) * 32 + b);
                }
            }
        }
        __syncthreads();
        const int U = nmulti;
        // H_iz = phi(s) - sum phi(x_if z_f) over the shared features (fp64), times w_i
        for (int q = tid; q < U; q += PRED_NT) {
            const int64_t i = multi[q];
            double sdot = 0.0, sphi = 0.0;
            for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
                const int32_t f = col[k];
                int lo = 0, hi = nz - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (zcol_s[mid] < f) lo = mid + 1;
                    else hi = mid;
                }
                if (nz > 0 && zcol_s[lo] == f) {
                    const double a = (double) val[k] * (double) zval_s[lo];
                    sdot += a;
                    sphi += phi(a);
                }
            }
            hs += (double) w[i] * (phi(sdot) - sphi);
        }
        __syncthreads();
    }
    const double H = pred_block_sum<T>(hs, red);
    if (tid == 0) {
        double v;
        if (phi.rbf) {
            const double ez = exp(-(double) kf.gamma * (double) nzz);
            v = ez * ((double) S[0] + J + H);
        } else {
            v = (double) kappa * (double) S[0] + J + H;
        }
        // the last training point (kept apart, as the reference's data_last)
        T kl;
        if (kf.kernel == 1) {
            const T base = fma(kf.gamma, dl, kf.coef0);
            kl = T(1);
            for (int e = 0; e < kf.degree; ++e) kl *= base;
        } else {
            T dist = nlast + nzz - T(2) * dl;
            dist = dist > T(0) ? dist : T(0);
            kl = exp(-kf.gamma * dist);
        }
        out[p] = (T) (v + (double) (alpha_m * kl)) + bias;
    }
}

// predict through the expansion; false when it does not apply (the caller predicts brute force)
template <typename T>
bool engine<T>::expansion_predict(const T *alpha_dev, T alpha_m, T bias, const int64_t *zr_dev, const int32_t *zc_dev,
                                  const T *zv_dev, int64_t np, int64_t max_nnz_z, double zabs_max, double znorm_max,
                                  T nlast, T *out_dev) {
    auto &ex = csr.ex;
    if (!ex.on || kernel == 0 || m <= 0 || max_nnz_z > PRED_ZCAP) return false;
    if (std::getenv("PLSSVM_MI_PRED_BRUTE") != nullptr) return false;
    // the model's Taylor degree covers |2 g x z| up to umax; the factored rbf form |z|^2 in range
    const double xabs = std::sqrt(ex.umax / std::max(2.0 * std::fabs((double) gamma), 1e-300));
    if (kernel == 2 && 2.0 * std::fabs((double) gamma) * xabs * zabs_max > ex.umax) return false;
    if (kernel == 2 && std::fabs((double) gamma) * znorm_max > (sizeof(T) == 8 ? 300.0 : 40.0)) return false;
    const phi_fn phi = make_phi<T>(kernel, degree, gamma, coef0);
    dev_buf<T> wv, Md, Sd;
    wv.alloc(std::max<int64_t>(m, 1), stream, false);
    Md.alloc(std::max<int64_t>(d, 1) * ex.KM, stream, false);
    Sd.alloc(2, stream);
    hipLaunchKernelGGL(exp_pred_w_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, stream, alpha_dev,
                       kernel == 2 ? csr.e.get() : nullptr, m, wv.get());
    MI_LAUNCH_CHECK();
    launch_dot2<T>(wv.get(), nullptr, nullptr, nullptr, m, red.get(), nullptr, stream);
    launch_dot_final<T>(red.get(), sc.get(), FIN_PLAIN, 0, nullptr, 0, Sd.get(), stream);
    coefs cf;
    std::memcpy(cf.c, ex.coef, sizeof(cf.c));
    if (d > 0)
        hipLaunchKernelGGL(exp_pred_moments_kernel<T>, dim3((unsigned) ceil_div(d, 4)), dim3(256), 0, stream,
                           csr.colptr.get(), csr.crow.get(), csr.cval.get(), wv.get(), d, ex.K, ex.KM, cf, Md.get());
    MI_LAUNCH_CHECK();
    T kappa = 0;
    if (kernel == 1) {
        kappa = 1;
        for (int q2 = 0; q2 < degree; ++q2) kappa *= coef0;
    }
    dev_buf<int> flag;
    flag.alloc(1, stream);
    hipLaunchKernelGGL(exp_pred_point_kernel<T>, dim3((unsigned) np), dim3(PRED_NT), 0, stream, zr_dev, zc_dev, zv_dev,
                       csr.colptr.get(), csr.crow.get(), csr.rowptr.get(), csr.col.get(), csr.val.get(), wv.get(),
                       Md.get(), ex.KM, phi, m, Sd.get(), xlast.get(), nlast, alpha_m, kf(), kappa, bias, out_dev,
                       flag.get());
    MI_LAUNCH_CHECK();
    int hf = 0;
    MI_HIP_CHECK(hipMemcpyAsync(&hf, flag.get(), sizeof(int), hipMemcpyDeviceToHost, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    return hf == 0;
}

int exp_dot2_built() { return EXP_DOT2 ? 1 : 0; }

void exp_load_code_object() {
    hipFuncAttributes a;
    (void) hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&exp_rowjoin_kernel));
}

#define INST(T)                                                                              \
    template bool engine<T>::expansion_eligible();                                           \
    template void engine<T>::build_expansion(const int64_t *, int64_t, const std::function<std::exception_ptr()> &);                      \
    template void engine<T>::expansion_dominant(const T *, const cg_scalars<T> *);           \
    template void engine<T>::expansion_moments(const T *, const cg_scalars<T> *, const T *, int);            \
    template void engine<T>::expansion_mscale(const cg_scalars<T> *);                        \
    template bool engine<T>::expansion_moment_pass(const T *, const cg_scalars<T> *, const T *, int);         \
    template bool engine<T>::expansion_moments_fused() const;        \
    template coefs engine<T>::expansion_coefs() const;                                       \
    template void engine<T>::expansion_kp_raw(const T *, const cg_scalars<T> *, bool);      \
    template bool engine<T>::dir_w_fill(dir_w_t<T> &);                                        \
    template bool engine<T>::ctr_active() const;                                              \
    template T engine<T>::QAf() const;                                                        \
    template void engine<T>::ctr_setup();                                                     \
    template bool engine<T>::expansion_predict(const T *, T, T, const int64_t *, const int32_t *, const T *, int64_t, \
                                               int64_t, double, double, T, T *);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
