// Per-GPU engine behind the C ABI: device memory, one HIP stream, optional RCCL communicator,
// device-resident CG. One engine<T> per context; T = float | double (the reference's real_type).
#pragma once

#include <rccl/rccl.h>
#include <rocblas/rocblas.h>

#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "buffer.hpp"
#include "kernels.hpp"
#include "sparse.hpp"

namespace plssvm_mi {

template <typename T>
inline ncclDataType_t nccl_type() {
    return sizeof(T) == 8 ? ncclFloat64 : ncclFloat32;
}

// an RCCL call of an engine member: under comm_mu, refused once plssvm_mi_comm_abort has released the communicator
#define MI_NCCL_CHECK(expr)                                                                                          \
    do {                                                                                                             \
        ncclResult_t r_;                                                                                             \
        {                                                                                                            \
            std::lock_guard<std::mutex> lk_(this->comm_mu);                                                         \
            if (this->comm_aborted) throw ::plssvm_mi::mi_error(-3, "the group was aborted by another rank");      \
            r_ = (expr);                                                                                             \
        }                                                                                                            \
        if (r_ != ncclSuccess) {                                                                                     \
            throw ::plssvm_mi::mi_error(-3, std::string("RCCL error '") + ncclGetErrorString(r_) + "' (" #expr ")"); \
        }                                                                                                            \
    } while (0)

int exp_dot2_built();  // expand.hip: 1 if the bfloat16 remainder's dot-instruction kernel was compiled (EXP_DOT2)
void exp_load_code_object();  // expand.hip: its code object loaded (one kernel's attributes queried)
void partition_superblocks(int64_t nb, int rank, int world, int64_t &s0, int64_t &s1, int64_t &s_total,
                           int64_t &tiles_total, int64_t &tiles_local);

struct engine_base {
    virtual ~engine_base() = default;
    // plssvm_mi_comm_abort (another thread of a one-process multi-GPU group, after a peer failed): the communicator
    // is aborted (ncclCommAbort releases a rank waiting in a collective) and every later RCCL call of the engine
    // fails (MI_NCCL_CHECK); the C ABI reports any call that ran into the abort as failed
    std::mutex comm_mu;
    std::atomic<bool> comm_aborted{ false };
    virtual void comm_abort() = 0;
};

template <typename T>
struct engine : engine_base {
    // ---- parameters (csvm<T> protected state, include/plssvm/csvm.hpp:242-277) ----
    int kernel = 0, degree = 3;
    T gamma = 1, coef0 = 0, cost = 1;
    int device = 0;
    hipStream_t stream = nullptr;
    int kp_mode = 0;  // PLSSVM_MI_KP_*
    int rbf_form = 0;  // PLSSVM_MI_OPT_RBF_FORM
    int sparse_algo = 0;  // PLSSVM_MI_OPT_SPARSE_ALGO (0 auto, 1 Gram pattern, 2 kernel expansion, 3 dense, 4 on the fly)

    // ---- multi-GPU row-block group ----
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    void comm_abort() override;
    // host-staged exchange (plssvm_mi_comm_init_host): the reference's device_reduction transport
    int (*xchg)(void *, int64_t, int, int, void *) = nullptr;
    void *xchg_user = nullptr;
    std::vector<T> xbuf;
    // test hook: compute only rank sim_rank's share of a sim_world group, no collective, rank-1
    // terms only on sim rank 0 (so the shares of all sim ranks sum to the full K·p)
    int sim_rank = 0, sim_world = 0;

    // ---- data ----
    bool have_data = false, sparse = false;
    int64_t n = 0, d = 0, m = 0, n_pad = 0, d_pad = 0, nb = 0;
    std::vector<T> xlast_h;
    dev_buf<T> XT, norms, xlast;  // dense: XT[d_pad][n_pad]
    csr_data<T> csr;              // sparse

    // work split
    int64_t t_total = 0, t0 = 0, t1 = 0;  // pairwise tile super-blocks owned by this rank: [t0, t1) of t_total
    int64_t tiles_total = 0, tiles_local = 0;
    dev_buf<int32_t> kp_wgoff;  // tile kernel workgroup table (kp_tile_offsets), kp_wgs workgroups
    int64_t kp_wgs = 0;
    void tiles_upload();
    int64_t r0 = 0, r1 = 0, chunk = 0;    // rows owned by this rank (factored / sparse row paths)

    // sharded CG (a real group on sparse data by default; PLSSVM_MI_SHARD = 0 / 1 overrides, 1 also for dense
    // data and simulated ranks): each rank updates only its rows [v0, v0 + vn) of x, r, d, Ad; every dot is
    // summed from the G ranks' gathered partials in rank order (the same bits everywhere); a K·p input the
    // path needs whole is gathered first, a path's full-length partial result reduce-scattered
    bool shard = false;
    bool gathered = false;  // sharded in a real group (any size, also a one-rank RCCL group): partials and
                            // inputs move through the group's transport
    int64_t v0 = 0, vn = 0;
    int G = 1;
    dev_buf<T> cgp_g;      // gathered partials, slots [5][G][2 RED_BLOCKS]: sum d / sum q d, d.Ad, r.r, kp sums, S
    std::vector<T> xpart;  // host staging of the host exchange's partial gathers
    const T *gather_partials(T *local, int slot, int64_t K = 2 * RED_BLOCKS);  // K values per rank
    // RCCL group: the sum d / sum q d partials of a CG step ride with the next collective of the K·p
    // (one launch, one latency) instead of a collective of their own
    bool psum_pending = false;
    void psum_group_begin(hipStream_t s);
    void psum_group_end();
    void flush_psum();
    // second stream for collectives that overlap kernels of the same K·p (kernel expansion, sharded RCCL group)
    hipStream_t cstream = nullptr;
    hipEvent_t cev[4] = { nullptr, nullptr, nullptr, nullptr };
    void gather_input(const T *p);   // sharded group: p's rows of every rank, in place
    void reduce_scatter_rows(T *buf);  // sharded group: own rows of the sum over ranks

    // ---- vectors (n_pad, zero padded) ----
    dev_buf<T> partial, q, pv, ret, x, r, dv, Ad, b, raw, w, red;
    // kernel expansion with bfloat16 windows (round 5): the S partials of the w pass (exp_wown_kernel, or the direction
    // update that carries it: dir_w_fill); w_pre = the vector whose w, bfloat16 copy and S partials are in place
    // (set after a carrying direction update of dv, cleared by any other w pass), graph_w_end = w_pre after a
    // captured iteration block
    dev_buf<T> wsp;
    const T *w_pre = nullptr, *graph_w_end = nullptr;
    bool dir_w_fill(dir_w_t<T> &o);
    dev_buf<T> cgp;  // fused CG partials: [0, 2R) sum d / sum q d, [2R, 4R) d.Ad, [4R, 6R) r.r
    // one-reduction CG (blas1.hip cg1_*; PLSSVM_MI_OPT_CG_VARIANT): s = Q~d by recurrence (sv), u = Q~r in Ad, and two
    // partial sets [r.u | r.r] by iteration parity (cg1p), gathered by one collective per iteration
    int cg_variant = 2;  // PLSSVM_MI_CG_REFERENCE / _ONE_REDUCTION / _AUTO (default: one-reduction in sharded groups)
    bool cg1 = false;    // the running solve uses it (cg_begin)
    int cg_par = 0;      // parity of the iteration cg_iter forms
    dev_buf<T> sv, cg1p;
    bool cg1_wanted() const;
    void cg1_iter(int reset);
    dev_buf<cg_scalars<T>> sc;
    dev_buf<double> trace;
    int64_t trace_cap = 0;
    T QA_cost = 0;
    bool have_q = false;
    int64_t run = 0;
    bool cg_active = false;
    static constexpr int CG_RESET = 50;  // r = b - Q~x every 50th iteration (csvm.cpp:119-132)
    hipGraphExec_t cg_graph = nullptr;   // one captured block of CG_RESET iterations (graph_block)
    // a CG iteration's finalize (Ad, d.Ad partials) offered to the K·p: a path that can form it in its own last
    // kernel (the kernel expansion's combine) does so and sets kp_fin_done; cg_iter launches it otherwise
    struct kp_fin_t {
        const T *q, *d, *psum;
        int G;
        T QA_cost, cost_inv;
        T *Ad, *pdad;
    };
    const kp_fin_t *kp_fin_req = nullptr;
    bool kp_fin_done = false;
    // Centered rank-1 terms (round 5, kernel expansion): with k_ij = a_i a_j (kappa' + phi_ij) (rbf: a = e, kappa' = 1;
    // poly: a = 1, phi = c, the kappa terms cancel exactly) the finalize's QA_cost - q_i - q_j + the separable part
    // is (a_i - a_m)(a_j - a_m) kappa' - h_i - h_j + h_m with h_i = a_i a_m phi(x_i . x_m): the same Q~, but formed
    // from small quantities instead of O(1) kernel values that cancel to O(gamma |x|^2) — in fp32 the naive sum loses
    // ~log10(1 / (gamma |x|^2)) digits per K·p (tests/long_trace_cases.py). Inside a finalize-bound K·p the combine's
    // base is c_i S_c (c = a - a_m, S_c = sum_j cw_j w_j, cw = c / e) and the finalize runs with q -> h,
    // QA_cost -> h_m + 1/C (+ any difference of a caller's QA_cost from k_mm + 1/C).
    dev_buf<T> ctr_c, ctr_cw, ctr_h;
    double ctr_hm = 0;
    T ctr_kmm = 0;         // k(x_m, x_m) as generate_q's QA_cost has it
    bool ctr_ok = false;   // the vectors are built and finite (PLSSVM_MI_CTR=0: never)
    bool q_gen = false;    // the device q is the engine's own k(x_i, x_m)
    bool ctr_now = false;  // set by kp_device / cg_iter around their K·p: the expansion drops its separable base
    std::vector<T> q_gen_h;
    bool ctr_active() const;
    const T *qf() const { return ctr_active() ? ctr_h.get() : q.get(); }
    T QAf() const;
    void ctr_setup();
    cg_scalars<T> polled{};               // the CG scalars read by the last cg_step poll
    // plssvm_mi_set_progress: called by solve_cg after each polled batch of iterations
    void (*progress)(int64_t, int64_t, const double *, double, double, void *) = nullptr;
    void *progress_user = nullptr;

    engine(int kernel_, int degree_, double gamma_, double coef0_, double cost_, int device_);
    ~engine() override;

    kfun<T> kf() const { return kfun<T>{ kernel, degree, gamma, coef0 }; }
    T cost_inv() const { return T(1) / cost; }
    bool factored() const;
    void need_data() const;
    void need_q() const;

    void comm_init(int rank_, int world_, const void *uid);
    void comm_init_host(int rank_, int world_, int (*fn)(void *, int64_t, int, int, void *), void *user);
    void kp_part(const T *p_host, T *out_host, int part);  // test hook, PLSSVM_MI_PART_*
    int part_mode = 0;  // kp_part in progress: PLSSVM_MI_PART_* (the expansion's combine writes that part)
    void setup_dense(const T *X, int64_t n_, int64_t d_);
    void setup_csr(const int64_t *rowptr, const int32_t *col, const void *val, int val_fmt, int64_t n_, int64_t d_);
    void finish_setup();
    void generate_q(T *q_out, double *qa_out);
    void set_q(const T *q_host);

    // out = (overwrite ? 0 : out) + add * Q~ p  (device vectors, length >= m)
    void kp_device(const T *p, T *out, T add, bool overwrite, const cg_scalars<T> *status);
    void kp_raw(const T *p, const cg_scalars<T> *status);  // raw = the pairwise / sparse part of Q~ p
    void kp_host(const T *q_host, const T *p, T *ret_host, T add);

    void cg_begin(const T *b_host, const T *q_host, T eps, bool force, double *delta0_out, int64_t trace_len);
    void cg_iter(int reset);
    bool graph_usable() const;
    void graph_capture();
    void graph_block();
    void graph_reset();
    void cg_step(int64_t nsteps, bool &converged, int64_t &iters);
    void cg_result(T *x_out, double *trace_out, int64_t trace_len, int64_t *iters);
    void solve_cg(const T *b, const T *q_host, int64_t imax, T eps, T *x_out, double *trace_out, int64_t *iters);
    void learn(const T *y, int64_t imax, T eps, T *alpha_out, double *bias_out, double *trace_out, int64_t *iters);
    void time_kp(int reps, double *ms_kp, double *ms_dom);

    // sparse paths (sparse.hip)
    void sparse_q();                                              // q, norms, e on CSR data
    void build_gram_blocks(const int64_t *cpos, int64_t max_inc);  // sparse Gram pattern (pairwise kernels)
    int64_t sparse_mem_budget() const;                             // device bytes for stored sparse structures
    // row_stats (optional): the sampled rows' partners sharing >= 2 features, mean and max
    int64_t estimate_expansion_bytes(const int64_t *rowptr, const int32_t *col, const std::vector<int64_t> &colptr,
                                     const std::vector<int32_t> &crow, int64_t inc_total, double *row_stats = nullptr) const;
    void release_sparse_structures();
    void csc_device(int64_t nnz, dev_buf<int64_t> &cpos_d);  // csr.colptr / crow / cval and cpos on the device
    void setup_sparse_dense();                                     // densified fallback (PLSSVM_MI_SPARSE_DENSE)
    // on-the-fly path (otf.hip, PLSSVM_MI_SPARSE_ONTHEFLY): estimated seconds per K·p share, setup, K·p
    double otf_estimate_s(const int64_t *rowptr, const int32_t *col, const std::vector<int64_t> &colptr) const;
    void setup_otf(int rbf_fact_ok);
    void otf_dominant(const T *p, const cg_scalars<T> *status);
    void otf_kp_raw(const T *p, const cg_scalars<T> *status, bool with_base);
    bool sparse_stored() const { return sparse && !csr.dense_on; } // K·p through the CSR structures
    bool expansion_eligible();                                    // expand.hip: K, coefficients; true if usable
    // multi-overlap remainder H, diagonal; before_agree (optional): waits for a step the caller runs concurrently
    // (the SELL plans, on a host thread) and returns its failure, which joins the group's agreement and is rethrown
    void build_expansion(const int64_t *cpos, int64_t max_inc,
                         const std::function<std::exception_ptr()> &before_agree = {});
    void expansion_kp_raw(const T *p, const cg_scalars<T> *status, bool with_base);
    void expansion_dominant(const T *p, const cg_scalars<T> *status);  // the remainder stream
    // column moments (SELL CSC pass); spart: the moment reduce also forms S from w's partials (sG sets)
    void expansion_moments(const T *w, const cg_scalars<T> *status, const T *spart = nullptr, int sG = 1);
    void expansion_mscale(const cg_scalars<T> *status);                 // moments -> Horner coefficients
    bool expansion_moment_pass(const T *w, const cg_scalars<T> *status, const T *spart = nullptr,
                               int sG = 1);  // true: reduced straight into M
    bool expansion_moments_fused() const;  // the moment pass has panel slabs (then its reduce can form S)
    coefs expansion_coefs() const;
    // predict through the expansion (expand.hip); false: not applicable, predict brute force
    bool expansion_predict(const T *alpha_dev, T alpha_m, T bias, const int64_t *zr_dev, const int32_t *zc_dev,
                           const T *zv_dev, int64_t np, int64_t max_nnz_z, double zabs_max, double znorm_max, T nlast,
                           T *out_dev);
    // raw[i] = sum_j k_ij p_j, i < m (with_base = false: only the overlap terms, PLSSVM_MI_PART_OVERLAP)
    void sparse_kp_raw(const T *p, const cg_scalars<T> *status, bool with_base = true);
    void sparse_dominant(const T *p, const cg_scalars<T> *status);  // the dominant sparse kernel
    void spmv_pass_csc(const T *p, const cg_scalars<T> *status);    // factored linear: w = X^T p
    void spmv_pass_csr(const cg_scalars<T> *status);                // factored linear: raw = X w
    int64_t csr_bytes() const { return csr.bytes(); }

    // model use (predict.hip): gpu_csvm::update_w / predict
    rocblas_handle blas = nullptr;
    void update_w_device(const T *alpha_dev);  // w = sum_i alpha_i x_i (device alpha[n])
    void update_w(const T *alpha_host, T *w_host);
    void predict(const T *alpha_host, T bias, const T *Z, const int64_t *zrowptr, const int32_t *zcol, const void *zval,
                 int zfmt, int64_t np, int64_t dz, T *out);

    void allreduce(T *buf, int64_t count);
    // setup decisions of a real group: every rank's K values, rank-major (world == 1: the local ones)
    std::vector<double> group_gather(const std::vector<double> &v);
    // one step of a group setup: every rank reports its failure (0 = none, else a PLSSVM_MI_ERR_* code) with
    // K values; a failure anywhere throws the same error on every rank (no rank is left waiting in a later
    // exchange), else every rank gets the world x K values, rank-major
    std::vector<double> group_step(int code, const std::string &why, const std::vector<double> &v);
    bool in_group() const { return world > 1 && sim_world == 0 && (comm != nullptr || xchg != nullptr); }
    void allgather_rows(T *buf);
    int64_t device_bytes() const;
};

}  // namespace plssvm_mi
