// Launcher declarations for the MI355X PLSSVM hot-path kernels (implemented in *.hip).
#pragma once

#include <vector>

#include "common.hpp"

namespace plssvm_mi {

// kernel parameters of the LS-SVM kernel function (include/plssvm/kernel_types.hpp:63-85)
template <typename T>
struct kfun {
    int kernel;  // 0 linear, 1 polynomial, 2 rbf
    int degree;
    T gamma;
    T coef0;
};

// device-resident CG scalars (all CG scalars live on the GPU; the host only polls `converged`)
template <typename T>
struct cg_scalars {
    T delta, delta0, alpha, beta, sp, sqp, eps2delta0, dAd;
    T delta_prev;  // delta of the previous iteration (fused CG kernels: read while delta is rewritten)
    T g1[2], a1[2], d1[2];  // one-reduction CG, by iteration parity: r.r (+inf before the first), alpha, d.Q~d (0)
    int converged;
    int force;  // bench mode: never converge (same work per iteration)
    int64_t iters;
};

// ---- dense pairwise tiles -----------------------------------------------------------------------
// tile edge of the implicit Q~ tiles (rows and columns); n_pad is a multiple of this.
constexpr int KP_TILE = 128;
// K-chunk depth of the pairwise tile kernel: 8 (fp64) / 16 (fp32) keeps LDS at <= 49 KB for 3
// workgroups per CU
template <typename T, int KERNEL>
constexpr int kp_bk() { return sizeof(T) == 8 ? 8 : 16; }
// feature padding of the device layout: a multiple of every chunk depth
template <typename T>
constexpr int kp_dpad() { return 16; }

// XT[k][i] = X[i][k] for i < rows, k < d (X row-major [rows][d]); XT is [>=d][n_pad], pre-zeroed
template <typename T>
void launch_transpose(const T *X, int64_t rows, int64_t d, T *XT, int64_t n_pad, hipStream_t s);

// row norms ||x_i||^2 (sequential fma chain in feature order) for the RBF norm trick
template <typename T>
void launch_row_norms(const T *XT, int64_t n_pad, int64_t d, T *norms, hipStream_t s);

// q_i = k(x_i, x_last), i < m (device_kernel_q_*, include/plssvm/backends/HIP/q_kernel.hip.hpp:32-83)
template <typename T>
void launch_q_dense(kfun<T> kf, const T *XT, int64_t n_pad, int64_t d, int64_t m, const T *xlast, T *q,
                    hipStream_t s);

// Tiles are scheduled in KP_SUPER x KP_SUPER super-blocks of the lower triangle (super-block
// (SI, SJ), SI >= SJ, linear index tri_index(SI, SJ)); a rank owns a contiguous super-block range.
constexpr int KP_SUPER = 8;

// slab record of one tile: its 128 row sums, then its 128 column sums (the rank's slab: wgs records)
constexpr int KP_REC = 2 * KP_TILE;
// partial[wg][KP_REC]: per tile wg of super-blocks [s0, s0+nsuper), sum_{j in J} k(x_i,x_j) p_j for i in I
// and sum_{i in I} k(x_i,x_j) p_i for j in J
// wg_off[k] (k = 0..nsuper): first workgroup of super-block s0 + k (one workgroup per real tile: 64 for a
// full super-block, 36 for a diagonal one, fewer in the ragged last row); wgs = wg_off[nsuper]
void kp_tile_offsets(int64_t nb, int64_t s0, int64_t nsuper, std::vector<int32_t> &wg_off);
template <typename T>
void launch_kp_tiles(kfun<T> kf, const T *XT, const T *norms, const T *p, T *partial, int64_t n_pad, int64_t d_pad,
                     int64_t nb, int64_t s0, int64_t nsuper, const int32_t *wg_off, int64_t wgs,
                     const cg_scalars<T> *status, hipStream_t s);

// raw[i] = sum over the column blocks c in order of row i's slab values of the tiles whose super-block lies
// in [s0, s1) (tile (Ib, c) row sums for c <= Ib, tile (c, Ib) column sums for c > Ib); i < m
template <typename T>
void launch_kp_reduce(const T *partial, int64_t nb, int64_t m, int64_t s0, int64_t s1, const int32_t *wg_off, T *raw,
                      const cg_scalars<T> *status, hipStream_t s);

// ret[i] = (overwrite ? 0 : ret[i]) + add * (raw[i] + (QA - q_i) * sum(p) - sum(q p) + p_i / C)
// raw may alias ret only when overwrite is false and ... (never aliased by callers).
template <typename T>
void launch_kp_finalize(const T *raw, const T *q, const T *p, const cg_scalars<T> *sc, T QA_cost, T cost_inv, T add,
                        int overwrite, int64_t m, T *ret, const cg_scalars<T> *status, hipStream_t s);

// ---- linear factored path: Q~p = X_m (X_m^T p) + rank-1 terms --------------------------------------
template <typename T>
void launch_gemv_t(const T *XT, int64_t n_pad, int64_t d, int64_t r0, int64_t r1, const T *p, T *w,
                   const cg_scalars<T> *status, hipStream_t s);  // w[k] = sum_{r0<=i<r1} XT[k][i] p_i
template <typename T>
void launch_gemv_n(const T *XT, int64_t n_pad, int64_t d, int64_t r0, int64_t r1, const T *w, T *raw,
                   const cg_scalars<T> *status, hipStream_t s);  // raw[i] = sum_k XT[k][i] w_k, r0<=i<r1

// ---- BLAS-1 / CG --------------------------------------------------------------------------------
constexpr int RED_BLOCKS = 512;
// partials[b] for b < RED_BLOCKS; out = sum(a*b) (b == nullptr: sum(a)); second pair optional
template <typename T>
void launch_dot2(const T *a, const T *b, const T *c, const T *e, int64_t n, T *partials, const cg_scalars<T> *status,
                 hipStream_t s);
// final reductions with CG scalar updates; `what` selects the update (see blas1.hip)
enum final_op { FIN_SP_SQP = 0, FIN_DELTA0 = 1, FIN_ALPHA = 2, FIN_DELTA = 3, FIN_PLAIN = 4 };
// G > 1: G gathered partial sets of a sharded group (rank-major, summed in rank order per partial)
template <typename T>
void launch_dot_final(const T *partials, cg_scalars<T> *sc, int op, int64_t run, double *trace, int64_t trace_cap,
                      T *plain_out, hipStream_t s, int G = 1);
template <typename T>
void launch_cg_init(const T *b, int64_t m, T *x, T *r, hipStream_t s);
template <typename T>
void launch_copy(const T *src, int64_t n, T *dst, const cg_scalars<T> *status, hipStream_t s);
// x += alpha d; if !reset: r -= alpha Ad  else r = b
template <typename T>
void launch_cg_update(T *x, T *r, const T *d, const T *Ad, const T *b, int reset, int64_t m, const cg_scalars<T> *sc,
                      hipStream_t s);
// d = beta d + r
template <typename T>
void launch_cg_direction(T *d, const T *r, int64_t m, const cg_scalars<T> *sc, hipStream_t s);
// Fused CG steps. Each block first sums the previous step's RED_BLOCKS partial pairs itself (in
// dot_final_kernel's order: every block gets the same value), so no final-reduction launch sits
// between them; dots keep dot2_kernel's grid and order, so the results are bitwise those of the
// unfused sequence.
// The input partials (psum, pdad, prr) are G gathered sets in a sharded group (G = 1 otherwise); the
// vectors are the caller's element range (pointers offset to it, m = its length).
// Ad = Q~ d from raw (kp_finalize arithmetic, add = 1, overwrite), sum d / sum q d from psum;
// d.Ad partials -> pdad. slabs != null: raw = the P panel slabs [P][sstride] of an unreduced SpMV pass.
template <typename T>
void launch_cg_fin_dad(const T *raw, const T *slabs, int64_t P, int64_t sstride, const T *q, const T *d, const T *psum,
                       int G, T QA_cost, T cost_inv, int raw_only, int64_t m, T *Ad, T *pdad, cg_scalars<T> *sc,
                       hipStream_t s);
// alpha = delta / d.Ad (pdad); x += alpha d; r -= alpha Ad and r.r partials -> prr (reset: r = b)
template <typename T>
void launch_cg_upd_rr(T *x, T *r, const T *d, const T *Ad, const T *b, int reset, const T *pdad, int G, int64_t m,
                      T *prr, cg_scalars<T> *sc, hipStream_t s);
// delta = r.r (prr), stop test, beta; d = beta d + r (init: d = r, scalars untouched);
// sum d / sum q d partials -> psum. The iteration index is sc->iters (trace[iters + 1] = delta, iters += 1).
// wout non-null (kernel expansion with bfloat16 windows, round 5): the next K·p's first kernel rides along — w = e d
// (e null: w = d, not written), its bfloat16 copy and the S partials (cw non-null: the centered S_c), in
// exp_wown_kernel's grid, element order and block reduction (bitwise its partials)
template <typename T>
struct dir_w_t {
    const T *e;
    T *w;
    uint16_t *w16;
    const T *cw;
    T *spart;
};
// one-reduction CG (Chronopoulos-Gear, blas1.hip): the update of iteration k from the gathered [r.u | r.r] partials
// (pset, G sets), the residual sums of a new r, the r.r of a batch's last r (poll)
template <typename T>
void launch_cg1_update(T *x, T *r, T *d, T *s, const T *u, const T *b, const T *q, int reset, const T *pset, int G,
                       double *trace, int64_t trace_cap, int64_t m, int par, T *pnext, T *psum, cg_scalars<T> *sc,
                       hipStream_t st, const dir_w_t<T> *wout);
template <typename T>
void launch_cg1_rsums(const T *r, const T *s, const T *q, int64_t m, T *pnext, T *psum, cg_scalars<T> *sc, hipStream_t st,
                      const dir_w_t<T> *wout);
template <typename T>
void launch_cg1_delta(const T *pset, int G, double *trace, int64_t trace_cap, cg_scalars<T> *sc, hipStream_t st);
template <typename T>
void launch_cg_dir_sums(T *d, const T *r, const T *q, const T *prr, int G, int init, double *trace, int64_t trace_cap,
                        int64_t m, T *psum, cg_scalars<T> *sc, hipStream_t s, const dir_w_t<T> *wout = nullptr);

// ---- sparse (CSR / FP22) ------------------------------------------------------------------------
// declared in sparse.hpp

}  // namespace plssvm_mi
