// Sparse (CSR / CSC / packed-FP22) device data for the MI355X PLSSVM backend.
// Build-defined formats: the reference has no sparse device path; its
// LIBSVM parser densifies (src/plssvm/parameter.cpp:66-87). Semantics here == the dense path on
// the densified matrix.
#pragma once

#include "buffer.hpp"
#include "fp22.hpp"
#include "kernels.hpp"
#include "spmv.hpp"

namespace plssvm_mi {

// ---- sparse Gram pattern (pairwise kernels on sparse data), see DESIGN.md §4 ------------------------
// rows are grouped in row blocks of GRAM_RB rows, candidate partners j < i in windows of GRAM_CW rows;
// a cell (I, W) holds, row by row (i ascending) then j ascending, every j in window W with
// s_ij = x_i . x_j structurally non-zero (some shared feature), stored as (uint16 j - W*CW, s).
constexpr int GRAM_RB = 2048;
// window edge: the K·p kernel stages n_j, e_j, p_j of the window plus int64 column and row
// accumulators in LDS (fp64: 3 x 32 + 32 + 16 KiB + row offsets = 152 KiB; fp32: 96 KiB)
constexpr int GRAM_CW = 4096;
constexpr int GRAM_WG = 512;  // K·p workgroup size when two fit a CU (else 1024: gram_wg in sparse.hip)

struct gram_cell {
    int32_t I, W;
    int64_t rowoff;  // index in rowoff[] of the cell's row 0 (rowoff holds GRAM_RB + 1 entries per cell)
    double smax;     // max |s_ij| over the cell's pairs (fixed-point bound of the K·p accumulators)
};

// ---- kernel expansion path (sparse poly / rbf), see DESIGN.md §5 and expand.hip ----------------------
// sum_j k_ij p_j = base_i + scale_i * sum_j [ sum_{f shared by i, j} phi(x_if x_jf) + H_ij ] w_j
// with phi a polynomial of degree K (exact for poly, Taylor for the factored rbf), evaluated per
// feature through the column moments M_k(f) = sum_{j in col f} x_jf^k w_j, and H_ij the remainder of
// the pairs sharing two or more features (stored, symmetric, rows padded to 8 slots).
constexpr int EXP_KMAX = 16;
constexpr int EXP_NWV = 16;  // waves per remainder-stream workgroup (one workgroup per CU)
// Remainder-stream geometry: one 1024-thread workgroup per block of RB rows (RB / EXP_NWV rows per
// wave) holds an LDS row accumulator (RB values) and one LDS window of CW partners (the next window is
// prefetched into registers), together the CU's 160 KiB. RBB = accumulator bytes in {4, 8, 16, 32} KiB;
// setup picks the largest whose block count still fills the CUs (bigger blocks = w restaged fewer
// times; a bigger window = fewer (row, window) groups = less 4-slot padding).
constexpr int EXP_LDS = 163840;
template <typename T, int RBB>
constexpr int exp_rb_of() { return RBB / (int) sizeof(T); }
template <typename T, int RBB>
constexpr int exp_cw_of() { return (EXP_LDS - RBB) / (int) sizeof(T) / 1024 * 1024; }
inline int exp_cw_host(int rbb, int es) { return (EXP_LDS - rbb) / es / 1024 * 1024; }
// bfloat16 windows (hbf16, expand.hip "H storage"): twice the partners in the same LDS, at most 65536
// (16-bit window-local j)
template <int RBB>
constexpr int exp_cw16_of() { return (EXP_LDS - RBB) / 2 / 1024 * 1024 < 65536 ? (EXP_LDS - RBB) / 2 / 1024 * 1024 : 65536; }
inline int exp_cw16_host(int rbb) { return std::min((EXP_LDS - rbb) / 2 / 1024 * 1024, 65536); }

// phi's polynomial coefficients (kernel argument of the moment / Horner kernels)
struct coefs {
    double c[EXP_KMAX + 1];
};

template <typename T>
struct exp_data {
    bool on = false;
    int K = 0, KM = 2;                // polynomial degree of phi; moment channels (2, 4, 8, 16 >= K)
    double coef[EXP_KMAX + 1] = {};   // phi(a) = sum_{k=1..K} coef[k] a^k
    double umax = 0.0;                // rbf: 2 |g| max x^2 (Taylor bound)
    dev_buf<T> mom;                   // [KM][d]: M_k(f) = sum_{j in col f} x_jf^(k+1) w_j (SELL pass, mode 1)
    dev_buf<T> M;                     // [d][KM]: coef[k+1] M_k(f), gathered by the CSR pass (mode 2)
    dev_buf<T> hdiag;                 // [n_pad]: H_ii
    dev_buf<T> phin;                  // [n_pad]: phi(|x_i|^2) (the diagonal's pair part, for the overlap hook)
    dev_buf<T> wv;                    // [n_pad]: w = e p (rbf)
    dev_buf<T> hs;                    // [n_pad]: sum_j H_ij w_j
    int64_t pairs = 0;                // unordered pairs sharing >= 2 features with H != 0 (this rank's rows)
    // remainder stream: per row block I (RB rows), per wave v (its RB / EXP_NWV rows), per
    // window W of CW partners j, row by row: the row's entries with j in W, padded to a multiple of 4
    // slots (pads: j = 0, H = 0); each wave's stream is one contiguous range across the windows
    int64_t slots = 0, nchunks = 0, nblk = 0, nW = 0;
    int RBB = 16384, RB = 0, CW = 0;  // geometry (see above): accumulator bytes, rows per block, window
    int G = 1;                         // window groups per row block (G > 1: row sums via hslab)
    dev_buf<T> hslab;                  // [G][rows] partial row sums of the window groups
    dev_buf<uint16_t> hjl;            // [slots] j - W * CW
    dev_buf<T> hv;                    // [slots] H_ij (the real type)
    dev_buf<uint16_t> hv16;           // [slots] H_ij as bfloat16 (hbf16: see expand.hip, "H storage")
    dev_buf<uint16_t> wv16;           // [m] the stream's partner weights w_j as bfloat16 (hbf16)
    bool hbf16 = false;
    bool dot2 = true;                 // bfloat16 H: the dot-instruction kernel (PLSSVM_MI_EXP_DOT2=0: the FMA chain)
    bool rflags = false;              // hbf16 chunks without hrow: bit 14 of a chunk's first H marks a row's first chunk
    bool rpairs = false;              // with rflags: the flags mark slot pairs (cells padded to 2 slots, not 4; layout 4)
    bool lt = false;                  // the symmetric rows came from the lower-triangle join + transpose
    double rj_mean = 0.0, rj_max = 0.0;  // setup's sample of the rank's rows: partners sharing >= 2 features (mean, max)
    double hratio = -1.0;             // row join: max |H_ij| / |kernel value of the pair| (< 0: unknown)
    dev_buf<uint16_t> hrow;           // [nchunks] block-local row of each 4-slot chunk
    dev_buf<int64_t> woff;            // [nblk][EXP_NWV][nW + 1] first chunk of each (block, wave, window)
    int64_t bytes() const {
        return mom.bytes() + M.bytes() + hdiag.bytes() + phin.bytes() + wv.bytes() + hs.bytes() + hjl.bytes() + hv.bytes() + hv16.bytes() + wv16.bytes() +
               hrow.bytes() + woff.bytes() + hslab.bytes();
    }
};

template <typename T>
struct csr_data {
    int64_t nnz = 0;  // entries of rows 0..m-1
    int val_fmt = 0;  // PLSSVM_MI_VAL_REAL | PLSSVM_MI_VAL_FP22
    dev_buf<int64_t> rowptr;
    dev_buf<int32_t> col;
    dev_buf<T> val;  // decoded values (setup-time kernels: q, norms, Gram build)
    dev_buf<int64_t> colptr;  // CSC of rows 0..m-1
    dev_buf<int32_t> crow;
    dev_buf<T> cval;  // CSC values (decoded; Gram pattern build only)
    // factored linear: w = X_rows^T p (rows [csc_r0, csc_r1): all rows for one / simulated ranks,
    // this rank's rows in a real group) and raw[r0, r1) = X w, both as panelled SELL SpMVs
    int64_t csc_r0 = 0, csc_r1 = 0;
    spmv_plan<T> spmv_csc, spmv_csr;
    rb_plan<T> rb_csr;  // one GPU: the CSR pass as row blocks with the CG finalize fused (spmv.hpp)
    dev_buf<T> e;                     // rbf separable factor exp(-gamma n_i)

    // Gram pattern
    bool have_gram = false;
    int64_t pairs = 0, pair_bound = 0;  // unique overlapping pairs; incidence bound
    int64_t slots = 0;                   // stored pair slots (rows padded to 8 per cell)
    bool rbf_factored = false;  // rbf pairs as e_i e_j (exp(2 g s) - 1), see sparse.hip
    bool rbf_small = false;     // ... with 2 g |s_ij| small enough for the short Taylor form (expm1_small)
    int64_t nRB = 0, nW = 0, rb0 = 0, rb1 = 0, m_pad = 0, ncells = 0;
    dev_buf<uint16_t> pj;
    dev_buf<T> ps;
    dev_buf<int64_t> rb_base;  // [nRB]
    dev_buf<int32_t> rowoff;
    dev_buf<gram_cell> cells;
    dev_buf<T> slab_row;  // [nW][m_pad]
    dev_buf<T> slab_col;  // [nRB][m_pad]
    dev_buf<T> ssc;       // device scalars: [0] = sum(e p) or sum(p)

    exp_data<T> ex;       // kernel expansion path (instead of the Gram pattern)
    // densified fallback (PLSSVM_MI_SPARSE_DENSE): neither stored structure fits the device budget, so
    // X is densified into the engine's XT and every K·p recomputes all pairs on the MFMA tiles
    bool dense_on = false;
    int64_t budget_b = 0;   // the (group's smallest) device budget of the stored structures, taken before the build
    int64_t est_bytes = 0;  // estimated device bytes of the chosen stored structure (0: not estimated)
    // on-the-fly path (PLSSVM_MI_SPARSE_ONTHEFLY, otf.hip): nothing stored per pair; seg[f][W] = (first
    // entry of CSC column f whose row lies in partner window W (CW rows), column-local; their count)
    bool otf_on = false;
    int otf_cw = 0;
    int64_t otf_nw = 0;
    dev_buf<int2> seg;      // [d][otf_nw]
    dev_buf<int64_t> ecb;   // [nnz]: colptr[col[k]] per CSR entry
    dev_buf<T> pne;         // [m][4]: p_j, |x_j|^2, e_j, 0 of the current K·p
    dev_buf<T> cjv;         // [nnz][2]: CSC (row, value) pairs (the row as int32 bits in the first slot)
    dev_buf<double> otf_part;  // [m]: row sums of the windows done so far (K·p split over launches)

    vals_t<T> rvals() const { return vals_t<T>{ val.get(), nullptr }; }
    vals_t<T> cvals() const { return vals_t<T>{ cval.get(), nullptr }; }
    int64_t bytes() const {
        return rowptr.bytes() + col.bytes() + val.bytes() + colptr.bytes() + crow.bytes() +
               cval.bytes() + spmv_csc.bytes() + spmv_csr.bytes() + rb_csr.bytes() + e.bytes() + pj.bytes() + ps.bytes() +
               rb_base.bytes() + rowoff.bytes() + cells.bytes() + slab_row.bytes() + slab_col.bytes() + ex.bytes() +
               seg.bytes() + ecb.bytes() + pne.bytes() + cjv.bytes() + otf_part.bytes();
    }
};

// raw_i += the separable part of sum_j k_ij p_j and the diagonal pair (sparse.hip; Gram pattern and
// on-the-fly paths, after the group exchange)
template <typename T>
void launch_gram_base(int kernel, kfun<T> kf, T kappa, const T *ssc, const T *norms, const T *ev, const T *p, int64_t m,
                      T *raw, const cg_scalars<T> *status, hipStream_t s);

}  // namespace plssvm_mi
