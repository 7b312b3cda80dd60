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

    vals_t<T> rvals() const { return vals_t<T>{ val.get(), nullptr }; }
    vals_t<T> cvals() const { return vals_t<T>{ cval.get(), nullptr }; }
    int64_t bytes() const {
        return rowptr.bytes() + col.bytes() + val.bytes() + colptr.bytes() + crow.bytes() +
               cval.bytes() + spmv_csc.bytes() + spmv_csr.bytes() + e.bytes() + pj.bytes() + ps.bytes() +
               rb_base.bytes() + rowoff.bytes() + cells.bytes() + slab_row.bytes() + slab_col.bytes();
    }
};

}  // namespace plssvm_mi
