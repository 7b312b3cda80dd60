// Sparse (CSR / CSC / packed-FP22) device data for the MI355X PLSSVM backend.
// Build-defined formats: the reference has no sparse device path; its
// LIBSVM parser densifies (src/plssvm/parameter.cpp:66-87). Semantics here == the dense path on
// the densified matrix.
#pragma once

#include "buffer.hpp"
#include "kernels.hpp"

namespace plssvm_mi {

// ---- packed FP22: binary32 truncated to its top 22 bits (RNE), 16 values per 11 uint32 words ----
__host__ __device__ inline float fp22_decode(uint32_t code) {
    union {
        uint32_t u;
        float f;
    } v;
    v.u = (code & 0x3FFFFFu) << 10;
    return v.f;
}

inline uint32_t fp22_encode_host(float x) {
    union {
        float f;
        uint32_t u;
    } v;
    v.f = x;
    const uint32_t u = v.u;
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return ((u >> 10) | 0x1000u) & 0x3FFFFFu;
    return ((u + 0x1FFu + ((u >> 10) & 1u)) >> 10) & 0x3FFFFFu;
}

inline int64_t fp22_words(int64_t n) { return ((n + 15) / 16) * 11; }

__host__ __device__ inline float fp22_get(const uint32_t *words, int64_t e) {
    const int64_t g = e >> 4;
    const int bit = 22 * (int) (e & 15);
    const uint32_t *w = words + g * 11 + (bit >> 5);
    const int s = bit & 31;
    uint64_t x = (uint64_t) w[0] >> s;
    if (s > 10) x |= (uint64_t) w[1] << (32 - s);
    return fp22_decode((uint32_t) x);
}

// value accessor: real array or packed FP22 words
template <typename T>
struct vals_t {
    const T *v;
    const uint32_t *v22;
    __device__ __forceinline__ T operator[](int64_t e) const { return v22 ? (T) fp22_get(v22, e) : v[e]; }
};

// ---- sparse Gram pattern (pairwise kernels on sparse data), see DESIGN.md §4 ------------------------
// rows are grouped in row blocks of GRAM_RB rows, candidate partners j < i in windows of GRAM_CW rows;
// a cell (I, W) holds, row by row (i ascending) then j ascending, every j in window W with
// s_ij = x_i . x_j structurally non-zero (some shared feature), stored as (uint16 j - W*CW, s).
constexpr int GRAM_RB = 2048;
// window edge: the K·p kernel stages n_j, e_j, p_j of the window plus int64 column and row
// accumulators in LDS (fp64: 3 x 32 + 32 + 16 KiB + row offsets = 152 KiB; fp32: 96 KiB)
constexpr int GRAM_CW = 4096;
constexpr int GRAM_WG = 512;  // K·p workgroup size

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
    dev_buf<T> val;
    dev_buf<uint32_t> val22;
    dev_buf<int64_t> colptr;  // CSC of rows 0..m-1
    dev_buf<int32_t> crow;
    dev_buf<T> cval;
    dev_buf<uint32_t> cval22;
    dev_buf<int64_t> col_lo, col_hi;  // per column: CSC range of this rank's rows (factored multi-rank)
    dev_buf<T> e;                     // rbf separable factor exp(-gamma n_i)

    // Gram pattern
    bool have_gram = false;
    int64_t pairs = 0, pair_bound = 0;  // unique overlapping pairs; incidence bound
    int64_t slots = 0;                   // stored pair slots (rows padded to 8 per cell)
    bool rbf_factored = false;  // rbf pairs as e_i e_j (exp(2 g s) - 1), see sparse.hip
    int64_t nRB = 0, nW = 0, rb0 = 0, rb1 = 0, m_pad = 0, ncells = 0;
    dev_buf<uint16_t> pj;
    dev_buf<T> ps;
    dev_buf<int64_t> rb_base;  // [nRB]
    dev_buf<int32_t> rowoff;
    dev_buf<gram_cell> cells;
    dev_buf<T> slab_row;  // [nW][m_pad]
    dev_buf<T> slab_col;  // [nRB][m_pad]
    dev_buf<T> ssc;       // device scalars: [0] = sum(e p) or sum(p)

    vals_t<T> rvals() const { return vals_t<T>{ val.get(), val22.get() }; }
    vals_t<T> cvals() const { return vals_t<T>{ cval.get(), cval22.get() }; }
    int64_t bytes() const {
        return rowptr.bytes() + col.bytes() + val.bytes() + val22.bytes() + colptr.bytes() + crow.bytes() +
               cval.bytes() + cval22.bytes() + col_lo.bytes() + col_hi.bytes() + e.bytes() + pj.bytes() + ps.bytes() +
               rb_base.bytes() + rowoff.bytes() + cells.bytes() + slab_row.bytes() + slab_col.bytes();
    }
};

}  // namespace plssvm_mi
