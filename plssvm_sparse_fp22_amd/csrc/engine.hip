// engine<T>: setup, q, K·p and the device-resident CG (host orchestration on one HIP stream).
//
// Reference call stack replaced: csvm::learn -> gpu_csvm::setup_data_on_device
// (src/plssvm/backends/gpu_csvm.cpp:130-157) -> generate_q (:160-183) -> solver_CG (:186-324) ->
// run_device_kernel (:353-363) -> device_reduction (:366-386).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include <limits>

#include "engine.hpp"

namespace plssvm_mi {

namespace {


// host kernel_function<k> (include/plssvm/kernel_types.hpp:63-85) for QA_cost = k(x_m, x_m) + 1/C
template <typename T>
T host_kernel(int kernel, int degree, T gamma, T coef0, const T *a, const T *b, int64_t d) {
    T v = 0;
    if (kernel == 2) {
        for (int64_t k = 0; k < d; ++k) {
            const T diff = a[k] - b[k];
            v = std::fma(diff, diff, v);
        }
        return std::exp(-gamma * v);
    }
    for (int64_t k = 0; k < d; ++k) v = std::fma(a[k], b[k], v);
    if (kernel == 0) return v;
    return std::pow(std::fma(gamma, v, coef0), (T) degree);
}

}  // namespace

// The tile kernel's workgroup table: wg_off[k] = the first workgroup of super-block s0 + k (one
// workgroup per real tile: 64 in a full super-block, 36 in a diagonal one, fewer in the ragged last
// row), wg_off[nsuper] = the grid size. Workgroup ids are 32-bit: a share of more than 2^31 - 1 tiles
// (m beyond ~8.4M rows on one rank) is rejected.
void kp_tile_offsets(int64_t nb, int64_t s0, int64_t nsuper, std::vector<int32_t> &wg_off) {
    wg_off.assign((size_t) nsuper + 1, 0);
    int64_t acc = 0;
    for (int64_t k = 0; k < nsuper; ++k) {
        int64_t SI, SJ;
        tri_tile(s0 + k, SI, SJ);
        const int64_t rows = std::min<int64_t>(KP_SUPER, nb - SI * KP_SUPER), cols = std::min<int64_t>(KP_SUPER, nb - SJ * KP_SUPER);
        acc += SI == SJ ? rows * (rows + 1) / 2 : rows * cols;
        if (acc > (int64_t) INT32_MAX)
            throw mi_error(-5, "the dense pairwise share of this rank exceeds 2^31 tiles: use more GPUs");
        wg_off[(size_t) k + 1] = (int32_t) acc;
    }
}

// Balanced contiguous ranges of 8x8-tile super-blocks of the lower triangle (each holds 64 tiles,
// diagonal ones 36, edge ones fewer): rank r gets the super-blocks whose cumulative tile count
// crosses [r, r+1) * total / world. Host-only (plssvm_mi_partition exposes it for CPU tests).
void partition_superblocks(int64_t nb, int rank, int world, int64_t &s0, int64_t &s1, int64_t &s_total,
                           int64_t &tiles_total, int64_t &tiles_local) {
    const int64_t ns = ceil_div(nb, KP_SUPER);
    s_total = ns * (ns + 1) / 2;
    tiles_total = nb * (nb + 1) / 2;
    std::vector<int64_t> cum(s_total + 1, 0);  // tiles before super-block s
    for (int64_t s = 0; s < s_total; ++s) {
        int64_t SI, SJ;
        tri_tile(s, SI, SJ);
        const int64_t rows = std::min<int64_t>(KP_SUPER, nb - SI * KP_SUPER);
        int64_t cnt = 0;
        for (int64_t a = 0; a < rows; ++a) {
            const int64_t I = SI * KP_SUPER + a;
            cnt += std::max<int64_t>(0, std::min<int64_t>(KP_SUPER, I - SJ * KP_SUPER + 1));
        }
        cum[s + 1] = cum[s] + cnt;
    }
    auto split = [&](int r) {
        return (int64_t) (std::lower_bound(cum.begin(), cum.end(), (tiles_total * r) / world) - cum.begin());
    };
    s0 = rank == 0 ? 0 : split(rank);
    s1 = rank == world - 1 ? s_total : split(rank + 1);
    if (s1 < s0) s1 = s0;
    tiles_local = cum[s1] - cum[s0];
}

template <typename T>
engine<T>::engine(int kernel_, int degree_, double gamma_, double coef0_, double cost_, int device_) :
    kernel(kernel_), degree(degree_), gamma((T) gamma_), coef0((T) coef0_), cost((T) cost_), device(device_) {
    MI_HIP_CHECK(hipSetDevice(device));
    MI_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    sc.alloc(1, stream);
    red.alloc(2 * RED_BLOCKS, stream);
    wsp.alloc(2 * RED_BLOCKS, stream);
    cgp.alloc(6 * RED_BLOCKS, stream);
}

template <typename T>
engine<T>::~engine() {
    (void) hipSetDevice(device);
    if (stream) (void) hipStreamSynchronize(stream);
    graph_reset();
    if (comm) (void) ncclCommDestroy(comm);
    for (auto &e : cev)
        if (e) (void) hipEventDestroy(e);
    if (cstream) (void) hipStreamDestroy(cstream);
    if (blas) (void) rocblas_destroy_handle(blas);
    XT.reset();
    partial.reset();
    if (stream) (void) hipStreamDestroy(stream);
}

template <typename T>
bool engine<T>::factored() const {
    if (kernel != 0) return false;
    if (kp_mode == 2) return true;
    if (kp_mode == 1) return false;
    return sparse;  // AUTO: dense linear runs the MFMA pairwise tiles, sparse linear the factored SpMVs
}

template <typename T>
void engine<T>::need_data() const {
    if (!have_data) throw mi_error(-6, "No data on the device! Maybe a call to setup_data_on_device() is missing?");
}

template <typename T>
void engine<T>::need_q() const {
    if (!have_q) throw mi_error(-6, "No q vector! Maybe a call to generate_q() is missing?");
}

template <typename T>
void engine<T>::comm_init(int rank_, int world_, const void *uid) {
    if (world_ < 1 || rank_ < 0 || rank_ >= world_) throw mi_error(-1, "invalid rank/world_size");
    if (have_data) throw mi_error(-6, "plssvm_mi_comm_init must be called before setup");
    MI_HIP_CHECK(hipSetDevice(device));
    if (comm) {
        (void) ncclCommDestroy(comm);
        comm = nullptr;
    }
    rank = rank_;
    world = world_;
    // a single-rank group still gets a communicator (every collective then runs through RCCL on
    // one GPU: the test path for the collective code on a one-GPU box)
    if (uid == nullptr) {
        if (world > 1) throw mi_error(-1, "a multi-rank group needs a unique id");
        return;
    }
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    // an aborted context stays aborted: a peer that failed before this rank got here will never join the rendezvous
    // below, and resetting the flag would leave this thread blocked in ncclCommInitRank (device_group's failure protocol)
    if (comm_aborted) throw mi_error(-3, "the group was aborted by another rank");
    {
        ncclComm_t c = nullptr;
        const ncclResult_t rc = ncclCommInitRank(&c, world, id, rank);  // blocks until every rank joined
        if (rc != ncclSuccess)
            throw mi_error(-3, std::string("RCCL error '") + ncclGetErrorString(rc) + "' (ncclCommInitRank)");
        std::lock_guard<std::mutex> lk(comm_mu);
        comm = c;
    }
    if (cstream == nullptr) {
        MI_HIP_CHECK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
        for (auto &e : cev) MI_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
}

// called from another host thread while this engine's own thread may be inside a collective: ncclCommAbort makes the
// pending RCCL kernels return; the engine's later RCCL calls throw (MI_NCCL_CHECK), its destructor skips the destroy
template <typename T>
void engine<T>::comm_abort() {
    std::lock_guard<std::mutex> lk(comm_mu);
    comm_aborted = true;
    if (comm != nullptr) {
        (void) ncclCommAbort(comm);
        comm = nullptr;
    }
}

template <typename T>
void engine<T>::comm_init_host(int rank_, int world_, int (*fn)(void *, int64_t, int, int, void *), void *user) {
    if (world_ < 1 || rank_ < 0 || rank_ >= world_) throw mi_error(-1, "invalid rank/world_size");
    if (fn == nullptr) throw mi_error(-1, "a host-staged group needs an exchange function");
    if (have_data) throw mi_error(-6, "plssvm_mi_comm_init_host must be called before setup");
    if (sim_world > 0) throw mi_error(-1, "a simulated rank cannot join a group");
    MI_HIP_CHECK(hipSetDevice(device));
    if (comm) {
        (void) ncclCommDestroy(comm);
        comm = nullptr;
    }
    comm_aborted = false;
    rank = rank_;
    world = world_;
    xchg = fn;
    xchg_user = user;
}

// Exchange step of one K·p. RCCL: in-stream collective. Host-staged: the reference's
// device_reduction (gpu_csvm.cpp:366-386) — synchronise, D2H, combine on the host (caller's
// collective), H2D — so the device work before and after is exactly the RCCL path's.
template <typename T>
void engine<T>::allreduce(T *buf, int64_t count) {
    if (count <= 0) return;
    if (comm != nullptr) {
        psum_group_begin(stream);
        MI_NCCL_CHECK(ncclAllReduce(buf, buf, (size_t) count, nccl_type<T>(), ncclSum, comm, stream));
        psum_group_end();
    } else if (xchg != nullptr) {
        xbuf.resize((size_t) count);
        MI_HIP_CHECK(hipMemcpyAsync(xbuf.data(), buf, sizeof(T) * (size_t) count, hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        if (xchg(xbuf.data(), count, (int) sizeof(T), 0, xchg_user) != 0) throw mi_error(-3, "host exchange failed");
        MI_HIP_CHECK(hipMemcpyAsync(buf, xbuf.data(), sizeof(T) * (size_t) count, hipMemcpyHostToDevice, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));  // xbuf is reused by the next exchange
    }
}

// sharded CG: the 2 x RED_BLOCKS partials of every rank (rank-major, into slot `slot` of cgp_g); the
// consumers sum them in rank order. Unsharded or a single rank: the local partials.
template <typename T>
const T *engine<T>::gather_partials(T *local, int slot, int64_t K) {
    if (!gathered) return local;
    T *out = cgp_g.get() + (int64_t) slot * G * 2 * RED_BLOCKS;  // K = 4 R: slots slot and slot + 1
    if (comm != nullptr) {
        MI_NCCL_CHECK(ncclAllGather(local, out, (size_t) K, nccl_type<T>(), comm, stream));
    } else {
        xpart.resize((size_t) (G * K));
        MI_HIP_CHECK(hipMemcpyAsync(xpart.data() + rank * K, local, sizeof(T) * (size_t) K, hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        if (xchg(xpart.data(), K, (int) sizeof(T), 1, xchg_user) != 0) throw mi_error(-3, "host exchange failed");
        MI_HIP_CHECK(hipMemcpyAsync(out, xpart.data(), sizeof(T) * xpart.size(), hipMemcpyHostToDevice, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
    return out;
}

template <typename T>
void engine<T>::psum_group_begin(hipStream_t s) {
    if (!psum_pending || comm == nullptr) return;
    MI_NCCL_CHECK(ncclGroupStart());
    MI_NCCL_CHECK(ncclAllGather(cgp.get(), cgp_g.get(), (size_t) (2 * RED_BLOCKS), nccl_type<T>(), comm, s));
}

template <typename T>
void engine<T>::psum_group_end() {
    if (!psum_pending || comm == nullptr) return;
    MI_NCCL_CHECK(ncclGroupEnd());
    psum_pending = false;
}

template <typename T>
void engine<T>::flush_psum() {
    if (!psum_pending) return;
    psum_pending = false;
    gather_partials(cgp.get(), 0);
}

template <typename T>
void engine<T>::gather_input(const T *p) {
    if (gathered) allgather_rows(const_cast<T *>(p));
}

template <typename T>
void engine<T>::reduce_scatter_rows(T *buf) {
    if (comm != nullptr) {
        psum_group_begin(stream);
        MI_NCCL_CHECK(ncclReduceScatter(buf, buf + (int64_t) rank * chunk, (size_t) chunk, nccl_type<T>(), ncclSum, comm,
                                        stream));
        psum_group_end();
    } else if (xchg != nullptr) {
        allreduce(buf, chunk * world);  // the host transport sums everything; the own rows are used
    }
}

template <typename T>
void engine<T>::allgather_rows(T *buf) {
    if (comm != nullptr) {
        psum_group_begin(stream);
        MI_NCCL_CHECK(ncclAllGather(buf + (int64_t) rank * chunk, buf, (size_t) chunk, nccl_type<T>(), comm, stream));
        psum_group_end();
    } else if (xchg != nullptr) {
        const int64_t total = chunk * world;
        xbuf.resize((size_t) total);
        MI_HIP_CHECK(hipMemcpyAsync(xbuf.data(), buf, sizeof(T) * (size_t) total, hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        if (xchg(xbuf.data(), chunk, (int) sizeof(T), 1, xchg_user) != 0) throw mi_error(-3, "host exchange failed");
        MI_HIP_CHECK(hipMemcpyAsync(buf, xbuf.data(), sizeof(T) * (size_t) total, hipMemcpyHostToDevice, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
}

// Small all-gather for setup decisions that every rank of a group must take identically (the sparse
// algorithm, its fallbacks): each rank contributes K values and gets all world x K, rank-major, through
// RCCL or the host exchange. The values pass through the real type T, so every rank compares the same
// rounded numbers. No group (or a simulated rank): the local values.
template <typename T>
std::vector<double> engine<T>::group_gather(const std::vector<double> &v) {
    const int64_t K = (int64_t) v.size();
    if (!in_group() || K == 0) return v;
    std::vector<T> h((size_t) (K * world), T(0));
    for (int64_t k = 0; k < K; ++k) h[(size_t) (rank * K + k)] = (T) v[(size_t) k];
    if (comm != nullptr) {
        dev_buf<T> buf;
        buf.alloc(K * world, stream);
        MI_HIP_CHECK(hipMemcpyAsync(buf.get(), h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice, stream));
        MI_NCCL_CHECK(ncclAllGather(buf.get() + rank * K, buf.get(), (size_t) K, nccl_type<T>(), comm, stream));
        MI_HIP_CHECK(hipMemcpyAsync(h.data(), buf.get(), sizeof(T) * h.size(), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    } else if (xchg(h.data(), K, (int) sizeof(T), 1, xchg_user) != 0) {
        throw mi_error(-3, "host exchange failed");
    }
    return std::vector<double>(h.begin(), h.end());
}

template <typename T>
std::vector<double> engine<T>::group_step(int code, const std::string &why, const std::vector<double> &v) {
    std::vector<double> mine{ (double) code };
    mine.insert(mine.end(), v.begin(), v.end());
    const auto g = group_gather(mine);
    const size_t K1 = mine.size();
    const int nr = (int) (g.size() / K1);
    int worst = 0;  // the first rank's failure, a non-OOM one over ERR_OOM (OOM alone: the caller's fallback)
    for (int r = 0; r < nr; ++r) {
        const int c = (int) g[(size_t) r * K1];
        if (c != 0 && (worst == 0 || worst == -4)) worst = c;
    }
    if (worst != 0)
        throw mi_error(worst, code != 0 ? why : std::string("sparse setup failed on another rank of the group"));
    std::vector<double> out;
    out.reserve((size_t) nr * v.size());
    for (int r = 0; r < nr; ++r)
        out.insert(out.end(), g.begin() + (std::ptrdiff_t) ((size_t) r * K1 + 1), g.begin() + (std::ptrdiff_t) ((size_t) (r + 1) * K1));
    return out;
}

template <typename T>
void engine<T>::setup_dense(const T *X, int64_t n_, int64_t d_) {
    if (X == nullptr || n_ < 1 || d_ < 1) throw mi_error(-1, "Data set is empty!");
    MI_HIP_CHECK(hipSetDevice(device));
    sparse = false;
    n = n_;
    d = d_;
    m = n - 1;
    nb = ceil_div(m, KP_TILE);
    n_pad = std::max<int64_t>(nb, 1) * KP_TILE;
    d_pad = round_up(d, kp_dpad<T>());
    // device layout: feature-major XT[d_pad][n_pad] of the first m points; the last point separately
    // (the reference's data_d_ / data_last_d_, gpu_csvm.cpp:142-155, with 64-bit offsets and tile padding)
    XT.alloc(d_pad * n_pad, stream);
    {
        dev_buf<T> tmp;
        tmp.alloc(std::max<int64_t>(m, 1) * d, stream, false);
        if (m > 0) {
            MI_HIP_CHECK(hipMemcpyAsync(tmp.get(), X, sizeof(T) * (size_t) (m * d), hipMemcpyHostToDevice, stream));
            launch_transpose<T>(tmp.get(), m, d, XT.get(), n_pad, stream);
        }
        MI_HIP_CHECK(hipStreamSynchronize(stream));
    }
    xlast_h.assign(X + m * d, X + m * d + d);
    xlast.alloc(d_pad, stream);
    MI_HIP_CHECK(hipMemcpyAsync(xlast.get(), xlast_h.data(), sizeof(T) * (size_t) d, hipMemcpyHostToDevice, stream));
    norms.alloc(n_pad, stream);
    if (kernel == 2) launch_row_norms<T>(XT.get(), n_pad, d, norms.get(), stream);
    finish_setup();
}

template <typename T>
void engine<T>::finish_setup() {
    // work split of the implicit matrix over the group (replaces feature_ranges_, gpu_csvm.cpp:136-139)
    partition_superblocks(nb, sim_world > 0 ? sim_rank : rank, sim_world > 0 ? sim_world : world, t0, t1, t_total,
                          tiles_total, tiles_local);
    const int eff_world = sim_world > 0 ? sim_world : world, eff_rank = sim_world > 0 ? sim_rank : rank;
    chunk = ceil_div(std::max<int64_t>(m, 1), eff_world);
    r0 = std::min<int64_t>(m, eff_rank * chunk);
    r1 = std::min<int64_t>(m, r0 + chunk);
    const int64_t vec_len = std::max<int64_t>(n_pad, chunk * eff_world);
    {
        const char *se = std::getenv("PLSSVM_MI_SHARD");
        const int opt = se != nullptr ? std::atoi(se) : -1;
        // a one-rank RCCL group with PLSSVM_MI_SHARD=1 runs every sharded collective through RCCL on one GPU
        // (the test path of the sharded RCCL code on a one-GPU box)
        const bool grp = (comm != nullptr || xchg != nullptr) && sim_world == 0;
        shard = (grp && (opt == 1 || (opt < 0 && sparse && world > 1))) || (sim_world > 0 && opt == 1);
        gathered = shard && grp;
        v0 = shard ? r0 : 0;
        vn = shard ? r1 - r0 : m;
        G = gathered ? world : 1;
        if (gathered) cgp_g.alloc(5 * (int64_t) G * 2 * RED_BLOCKS, stream);
    }
    tiles_upload();
    if (!sparse && !factored()) {
        // the rank's tile slab: one record of row and column sums per own tile (scales with 1 / world)
        partial.alloc(std::max<int64_t>(kp_wgs, 1) * KP_REC, stream, false);
    } else {
        partial.reset();
    }
    q.alloc(vec_len, stream);
    pv.alloc(vec_len, stream);
    ret.alloc(vec_len, stream);
    x.alloc(vec_len, stream);
    r.alloc(vec_len, stream);
    dv.alloc(vec_len, stream);
    Ad.alloc(vec_len, stream);
    b.alloc(vec_len, stream);
    raw.alloc(vec_len, stream);
    w.alloc(std::max<int64_t>(d_pad, 1), stream);
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    have_data = true;
    have_q = false;
    q_gen = false;
    ctr_ok = false;
    cg_active = false;
    graph_reset();
}

// the tile kernel's workgroup table for this rank's super-blocks [t0, t1) (also the densified sparse path)
template <typename T>
void engine<T>::tiles_upload() {
    std::vector<int32_t> off;
    kp_tile_offsets(nb, t0, t1 - t0, off);
    kp_wgs = off.back();
    kp_wgoff.alloc((int64_t) off.size(), stream, false);
    MI_HIP_CHECK(hipMemcpyAsync(kp_wgoff.get(), off.data(), sizeof(int32_t) * off.size(), hipMemcpyHostToDevice, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
}

template <typename T>
void engine<T>::generate_q(T *q_out, double *qa_out) {
    need_data();
    MI_HIP_CHECK(hipSetDevice(device));
    if (sparse) {
        sparse_q();
    } else {
        launch_q_dense<T>(kf(), XT.get(), n_pad, d, m, xlast.get(), q.get(), stream);
    }
    ctr_kmm = host_kernel<T>(kernel, degree, gamma, coef0, xlast_h.data(), xlast_h.data(), d);
    QA_cost = ctr_kmm + T(1) / cost;
    q_gen_h.resize((size_t) std::max<int64_t>(m, 0));
    if (m > 0) MI_HIP_CHECK(hipMemcpyAsync(q_gen_h.data(), q.get(), sizeof(T) * (size_t) m, hipMemcpyDeviceToHost, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    if (q_out && m > 0) std::memcpy(q_out, q_gen_h.data(), sizeof(T) * (size_t) m);
    if (qa_out) *qa_out = (double) QA_cost;
    have_q = true;
    q_gen = true;
    if (sparse) ctr_setup();
    graph_reset();
}

template <typename T>
void engine<T>::set_q(const T *q_host) {
    need_data();
    if (q_host == nullptr) {
        need_q();
        return;
    }
    if (m > 0) MI_HIP_CHECK(hipMemcpyAsync(q.get(), q_host, sizeof(T) * (size_t) m, hipMemcpyHostToDevice, stream));
    // a caller's q equal to the generated one keeps the centered finalize; any other q is used as given
    q_gen = (int64_t) q_gen_h.size() == m && (m == 0 || std::memcmp(q_host, q_gen_h.data(), sizeof(T) * (size_t) m) == 0);
    if (!have_q) {
        QA_cost = host_kernel<T>(kernel, degree, gamma, coef0, xlast_h.data(), xlast_h.data(), d) + T(1) / cost;
        have_q = true;
    }
}

// out = (overwrite ? 0 : out) + add * Q~ p   — run_device_kernel + device_reduction
template <typename T>
void engine<T>::kp_device(const T *p, T *out, T add, bool overwrite, const cg_scalars<T> *status) {
    if (m <= 0) return;
    cg_scalars<T> *scp = sc.get();
    // sum(p) and sum(q p): the rank-1 parts of Q~ (QA_cost - q_i - q_j) never enter the tiles (sharded: this
    // rank's rows, then the gathered partials of all ranks)
    launch_dot2<T>(p + v0, nullptr, qf() + v0, p + v0, vn, red.get(), status, stream);
    launch_dot_final<T>(gather_partials(red.get(), 3), scp, FIN_SP_SQP, 0, nullptr, 0, nullptr, stream, G);
    ctr_now = ctr_active();
    kp_raw(p, status);
    ctr_now = false;
    const int flags = (overwrite ? 1 : 0) | ((sim_world > 0 && sim_rank != 0 && !shard) ? 2 : 0);
    launch_kp_finalize<T>(raw.get() + v0, qf() + v0, p + v0, scp, QAf(), cost_inv(), add, flags, vn, out + v0,
                          status, stream);
}

template <typename T>
void engine<T>::kp_raw(const T *p, const cg_scalars<T> *status) {
    if (m <= 0) return;
    if (sparse_stored()) {
        sparse_kp_raw(p, status);
    } else if (factored()) {
        const bool all_rows = sim_world > 0 && !shard;
        launch_gemv_t<T>(XT.get(), n_pad, d, all_rows ? 0 : r0, all_rows ? m : r1, p, w.get(), status, stream);
        allreduce(w.get(), d);
        launch_gemv_n<T>(XT.get(), n_pad, d, r0, r1, w.get(), raw.get(), status, stream);
        if (!shard) allgather_rows(raw.get());
    } else {
        gather_input(p);
        launch_kp_tiles<T>(kf(), XT.get(), norms.get(), p, partial.get(), n_pad, d_pad, nb, t0, t1 - t0, kp_wgoff.get(), kp_wgs, status,
                           stream);
        launch_kp_reduce<T>(partial.get(), nb, m, t0, t1, kp_wgoff.get(), raw.get(), status, stream);
        if (shard) reduce_scatter_rows(raw.get());
        else allreduce(raw.get(), m);
    }
}

template <typename T>
void engine<T>::kp_host(const T *q_host, const T *p, T *ret_host, T add) {
    need_data();
    MI_HIP_CHECK(hipSetDevice(device));
    set_q(q_host);
    cg_active = false;
    MI_HIP_CHECK(hipMemsetAsync(sc.get(), 0, sizeof(cg_scalars<T>), stream));
    if (m > 0) {
        MI_HIP_CHECK(hipMemcpyAsync(pv.get(), p, sizeof(T) * (size_t) m, hipMemcpyHostToDevice, stream));
        MI_HIP_CHECK(hipMemcpyAsync(ret.get(), ret_host, sizeof(T) * (size_t) m, hipMemcpyHostToDevice, stream));
        kp_device(pv.get(), ret.get(), add, false, nullptr);
        if (gathered) allgather_rows(ret.get());  // device_reduction's result on every rank
        MI_HIP_CHECK(hipMemcpyAsync(ret_host, ret.get(), sizeof(T) * (size_t) m, hipMemcpyDeviceToHost, stream));
    }
    MI_HIP_CHECK(hipStreamSynchronize(stream));
}

// test hook: one part of Q~p (PLSSVM_MI_PART_KERNEL: sum_j k_ij p_j; PLSSVM_MI_PART_OVERLAP: the
// sparse overlap sum only; PLSSVM_MI_PART_REMAINDER: the kernel expansion's stored remainder stream only), after the
// group exchange
template <typename T>
void engine<T>::kp_part(const T *p_host, T *out_host, int part) {
    need_data();
    if (part < 0 || part > 2) throw mi_error(-1, "unknown K·p part");
    if (part == 1 && !(sparse_stored() && !factored()))
        throw mi_error(-5, "the overlap part exists for the stored sparse poly/rbf paths only");
    if (part == 2 && !(sparse_stored() && !factored() && csr.ex.on && !csr.otf_on))
        throw mi_error(-5, "the remainder part exists for the sparse kernel expansion only");
    MI_HIP_CHECK(hipSetDevice(device));
    cg_active = false;
    MI_HIP_CHECK(hipMemsetAsync(sc.get(), 0, sizeof(cg_scalars<T>), stream));
    if (m > 0) {
        MI_HIP_CHECK(hipMemcpyAsync(pv.get(), p_host, sizeof(T) * (size_t) m, hipMemcpyHostToDevice, stream));
        part_mode = part;
        try {
            if (part != 0) sparse_kp_raw(pv.get(), nullptr, false);
            else kp_raw(pv.get(), nullptr);
        } catch (...) {
            part_mode = 0;
            throw;
        }
        part_mode = 0;
        if (gathered) allgather_rows(raw.get());
        MI_HIP_CHECK(hipMemcpyAsync(out_host, raw.get(), sizeof(T) * (size_t) m, hipMemcpyDeviceToHost, stream));
    }
    MI_HIP_CHECK(hipStreamSynchronize(stream));
}

// ---- CG: openmp::csvm::solver_CG semantics (src/plssvm/backends/OpenMP/csvm.cpp:82-170) -------------
template <typename T>
void engine<T>::cg_begin(const T *b_host, const T *q_host, T eps, bool force, double *delta0_out, int64_t trace_len) {
    need_data();
    MI_HIP_CHECK(hipSetDevice(device));
    set_q(q_host);
    cg_scalars<T> init{};
    init.eps2delta0 = eps * eps;
    init.force = force ? 1 : 0;
    cg1 = cg1_wanted();
    init.g1[0] = init.g1[1] = init.a1[0] = init.a1[1] = std::numeric_limits<T>::infinity();
    MI_HIP_CHECK(hipMemcpyAsync(sc.get(), &init, sizeof(init), hipMemcpyHostToDevice, stream));
    trace_cap = std::max<int64_t>(trace_len, 1);
    if (trace.size() < trace_cap) trace.alloc(trace_cap, stream);
    graph_reset();  // QA_cost, trace and the vectors' contents may differ from the captured solve
    if (m > 0) MI_HIP_CHECK(hipMemcpyAsync(b.get(), b_host, sizeof(T) * (size_t) m, hipMemcpyHostToDevice, stream));
    // x = 1; r = b; r -= Q~x   (csvm.cpp:85-90)
    launch_cg_init<T>(b.get(), m, x.get(), r.get(), stream);
    kp_device(x.get(), r.get(), T(-1), false, nullptr);
    // delta = r.r ; delta0 ; d = r   (:92-97)   (sharded: this rank's rows, the ranks' partials gathered)
    launch_dot2<T>(r.get() + v0, r.get() + v0, nullptr, nullptr, vn, red.get(), nullptr, stream);
    launch_dot_final<T>(gather_partials(red.get(), 3), sc.get(), FIN_DELTA0, 0, trace.get(), trace_cap, nullptr, stream, G);
    dir_w_t<T> wo{};
    const bool fw = dir_w_fill(wo);
    if (cg1) {
        // one-reduction CG: d = s = 0, the r.r / sum r / sum q r partials of r0 (set 0) for the first product Q~r
        if (sv.size() < q.size()) sv.alloc(q.size(), stream);
        if (cg1p.size() < 8 * RED_BLOCKS) cg1p.alloc(8 * RED_BLOCKS, stream);  // two [r.u | r.r | r.s | 0] sets
        MI_HIP_CHECK(hipMemsetAsync(dv.get(), 0, sizeof(T) * (size_t) q.size(), stream));
        MI_HIP_CHECK(hipMemsetAsync(sv.get(), 0, sizeof(T) * (size_t) q.size(), stream));
        launch_cg1_rsums<T>(r.get() + v0, sv.get() + v0, qf() + v0, vn, cg1p.get(), cgp.get(), sc.get(), stream, fw ? &wo : nullptr);
        w_pre = fw ? r.get() : nullptr;
    } else {
        // d = r, with sum d / sum q d for the first Q~d
        launch_cg_dir_sums<T>(dv.get() + v0, r.get() + v0, qf() + v0, nullptr, 1, 1, nullptr, 0, vn, cgp.get(), sc.get(),
                              stream, fw ? &wo : nullptr);
        w_pre = fw ? dv.get() : nullptr;
    }
    if (gathered && comm != nullptr) psum_pending = true;  // gathered with the first K·p's collective
    else gather_partials(cgp.get(), 0);
    run = 0;
    cg_active = true;
    // a solve that can reach a whole block captures it now (capture launches nothing; the
    // instantiation stays out of the iterations' time)
    if (trace_len > CG_RESET && graph_usable()) graph_capture();
    if (delta0_out) {
        cg_scalars<T> h{};
        MI_HIP_CHECK(hipMemcpyAsync(&h, sc.get(), sizeof(h), hipMemcpyDeviceToHost, stream));
        MI_HIP_CHECK(hipStreamSynchronize(stream));
        *delta0_out = (double) h.delta0;
    }
}

// one CG iteration (reset: the every-50th recomputation r = b - Q~x), all launches on the engine stream
// the one-reduction recurrence: forced (PLSSVM_MI_CG_ONE_REDUCTION), or auto for a sharded group of several ranks
template <typename T>
bool engine<T>::cg1_wanted() const {
    return cg_variant == 1 || (cg_variant == 2 && gathered && G > 1);
}

// one iteration of the one-reduction CG (blas1.hip cg1_update_kernel): u = Q~r with the finalize forming the r.u
// partials beside the r.r ones of set `par`, ONE gather of that set, then d, s, x, r and the next partials in one kernel
template <typename T>
void engine<T>::cg1_iter(int reset) {
    const cg_scalars<T> *st = sc.get();
    T *psum = cgp.get();
    T *cur = cg1p.get() + (int64_t) cg_par * 4 * RED_BLOCKS, *nxt = cg1p.get() + (int64_t) (cg_par ^ 1) * 4 * RED_BLOCKS;
    const T *psum_in = gathered ? cgp_g.get() : psum;
    const int raw_only = (sim_world > 0 && sim_rank != 0 && !shard) ? 1 : 0;
    const T *slabs = nullptr;
    int64_t P = 0;
    bool fin = false;
    if (sparse_stored() && factored() && world == 1 && sim_world == 0 && csr.rb_csr.nblk > 0) {
        spmv_pass_csc(r.get(), st);
        launch_rowblock_fin<T>(csr.rb_csr, w.get(), d, q.get(), r.get(), psum, QA_cost, cost_inv(), Ad.get(), cur, st, stream);
        fin = true;
    } else if (sparse && factored() && world == 1 && sim_world == 0 && csr.spmv_csr.P > 1) {
        spmv_pass_csc(r.get(), st);
        launch_panel_spmv<T>(csr.spmv_csr, w.get(), d, raw.get(), st, stream, 1, 0, false);
        slabs = csr.spmv_csr.partial.get();
        P = csr.spmv_csr.P;
    } else {
        const kp_fin_t f{ qf(), r.get(), psum_in, G, QAf(), cost_inv(), Ad.get(), cur };
        kp_fin_req = raw_only ? nullptr : &f;
        kp_fin_done = false;
        ctr_now = ctr_active();
        kp_raw(r.get(), st);
        ctr_now = false;
        kp_fin_req = nullptr;
        fin = kp_fin_done;
        kp_fin_done = false;
    }
    flush_psum();
    if (!fin)
        launch_cg_fin_dad<T>(raw.get() + v0, slabs, P, m, qf() + v0, r.get() + v0, psum_in, G, QAf(), cost_inv(), raw_only, vn,
                             Ad.get() + v0, cur, sc.get(), stream);
    // the one collective of the iteration: [r.u | r.r] partials of every rank
    const T *pset = gather_partials(cur, 1, 4 * RED_BLOCKS);
    dir_w_t<T> wo{};
    const bool fw = !reset && dir_w_fill(wo);
    launch_cg1_update<T>(x.get() + v0, r.get() + v0, dv.get() + v0, sv.get() + v0, Ad.get() + v0, b.get() + v0, qf() + v0,
                         reset, pset, G, trace.get(), trace_cap, vn, cg_par, nxt, psum, sc.get(), stream, fw ? &wo : nullptr);
    w_pre = fw ? r.get() : nullptr;
    if (reset) {  // r = b - Q~x, then its partials (csvm.cpp:119-132)
        kp_device(x.get(), r.get(), T(-1), false, st);
        dir_w_t<T> wr{};
        const bool fr = dir_w_fill(wr);
        launch_cg1_rsums<T>(r.get() + v0, sv.get() + v0, qf() + v0, vn, nxt, psum, sc.get(), stream, fr ? &wr : nullptr);
        w_pre = fr ? r.get() : nullptr;
    }
    if (gathered && comm != nullptr) psum_pending = true;  // gathered with the next product's first collective
    else gather_partials(psum, 0);
}

template <typename T>
void engine<T>::cg_iter(int reset) {
    if (cg1) {
        cg1_iter(reset);
        return;
    }
    const cg_scalars<T> *st = sc.get();
    T *psum = cgp.get(), *pdad = psum + 2 * RED_BLOCKS, *prr = psum + 4 * RED_BLOCKS;
    // sharded: the partials the previous step gathered (slot 0: sum d / sum q d)
    const T *psum_in = gathered ? cgp_g.get() : psum;
    const int raw_only = (sim_world > 0 && sim_rank != 0 && !shard) ? 1 : 0;
    // Ad = Q~ d (:111-113); alpha = delta / (d . Ad) (:116) in the next kernel
    const T *slabs = nullptr;
    int64_t P = 0;
    if (sparse_stored() && factored() && world == 1 && sim_world == 0 && csr.rb_csr.nblk > 0) {
        // one GPU, factored sparse linear: CSC pass, then the row-block CSR pass with the finalize and
        // the d.Ad partials fused (spmv.hpp)
        spmv_pass_csc(dv.get(), st);
        launch_rowblock_fin<T>(csr.rb_csr, w.get(), d, q.get(), dv.get(), psum, QA_cost, cost_inv(), Ad.get(), pdad, st,
                               stream);
    } else if (sparse && factored() && world == 1 && sim_world == 0 && csr.spmv_csr.P > 1) {
        // one GPU, factored sparse linear: the CSR pass's panel slabs are summed by cg_fin_dad
        spmv_pass_csc(dv.get(), st);
        launch_panel_spmv<T>(csr.spmv_csr, w.get(), d, raw.get(), st, stream, 1, 0, false);
        slabs = csr.spmv_csr.partial.get();
        P = csr.spmv_csr.P;
    } else {
        const kp_fin_t fin{ qf(), dv.get(), psum_in, G, QAf(), cost_inv(), Ad.get(), pdad };
        kp_fin_req = raw_only ? nullptr : &fin;
        kp_fin_done = false;
        ctr_now = ctr_active();
        kp_raw(dv.get(), st);
        ctr_now = false;
        kp_fin_req = nullptr;
    }
    flush_psum();  // no collective of the K·p carried it
    if (kp_fin_done) {
        kp_fin_done = false;  // the K·p's last kernel formed Ad and the d.Ad partials
    } else if (!(sparse_stored() && factored() && world == 1 && sim_world == 0 && csr.rb_csr.nblk > 0)) {
        launch_cg_fin_dad<T>(raw.get() + v0, slabs, P, m, qf() + v0, dv.get() + v0, psum_in, G, QAf(), cost_inv(),
                             raw_only, vn, Ad.get() + v0, pdad, sc.get(), stream);
    }
    // x += alpha d; r = b - Q~x every 50th iteration, else r -= alpha Ad   (:119-132)
    launch_cg_upd_rr<T>(x.get() + v0, r.get() + v0, dv.get() + v0, Ad.get() + v0, b.get() + v0, reset,
                        gather_partials(pdad, 1), G, vn, prr, sc.get(), stream);
    if (reset) {
        kp_device(x.get(), r.get(), T(-1), false, st);
        launch_dot2<T>(r.get() + v0, r.get() + v0, nullptr, nullptr, vn, prr, st, stream);
    }
    // delta = r.r ; stop test ; beta (:135-146); d = beta d + r (:149-151), with sum d / sum q d
    // (kernel expansion, bfloat16 windows: with the next K·p's w pass, dir_w_fill)
    dir_w_t<T> wo{};
    const bool fw = dir_w_fill(wo);
    launch_cg_dir_sums<T>(dv.get() + v0, r.get() + v0, qf() + v0, gather_partials(prr, 2), G, 0, trace.get(), trace_cap,
                          vn, psum, sc.get(), stream, fw ? &wo : nullptr);
    w_pre = fw ? dv.get() : nullptr;
    if (gathered && comm != nullptr) psum_pending = true;  // gathered with the next K·p's first collective
    else gather_partials(psum, 0);
}

// Iteration blocks of CG_RESET (the reset period) starting at a multiple of it are replayed from one
// captured hipGraph: the launches of a block depend only on the engine's buffers (the iteration
// index lives on the device), so one capture serves every block of a solve. Host-staged groups
// synchronise inside the exchange and are never captured; RCCL groups are captured only with
// PLSSVM_MI_GRAPH=2 (the collectives then run as graph nodes); PLSSVM_MI_GRAPH=0 disables graphs.
template <typename T>
bool engine<T>::graph_usable() const {
    const char *ge = std::getenv("PLSSVM_MI_GRAPH");  // read per call (tests compare graphs off / on in one process)
    const int mode = ge == nullptr ? 1 : std::atoi(ge);
    if (mode == 0 || xchg != nullptr || m <= 0) return false;
    return comm == nullptr || mode == 2;
}

template <typename T>
void engine<T>::graph_reset() {
    if (cg_graph != nullptr) {
        (void) hipGraphExecDestroy(cg_graph);
        cg_graph = nullptr;
    }
}

template <typename T>
void engine<T>::graph_capture() {
    if (cg_graph == nullptr) {
        hipGraph_t g = nullptr;
        // a block forms its first w itself (the replay may follow any other K·p); w_pre stays what the launched
        // work left, graph_w_end is what a replay leaves
        const T *keep = w_pre;
        w_pre = nullptr;
        MI_HIP_CHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
        try {
            for (int k = 0; k < CG_RESET; ++k) {
                cg_par = k & 1;  // blocks start at multiples of CG_RESET (even)
                cg_iter(k == CG_RESET - 1 ? 1 : 0);
            }
        } catch (...) {
            (void) hipStreamEndCapture(stream, &g);
            if (g) (void) hipGraphDestroy(g);
            w_pre = keep;
            throw;
        }
        graph_w_end = w_pre;
        w_pre = keep;
        MI_HIP_CHECK(hipStreamEndCapture(stream, &g));
        const hipError_t e = hipGraphInstantiate(&cg_graph, g, nullptr, nullptr, 0);
        (void) hipGraphDestroy(g);
        MI_HIP_CHECK(e);
    }
}

template <typename T>
void engine<T>::graph_block() {
    graph_capture();
    MI_HIP_CHECK(hipGraphLaunch(cg_graph, stream));
    w_pre = graph_w_end;
}

template <typename T>
void engine<T>::cg_step(int64_t nsteps, bool &converged, int64_t &iters) {
    if (!cg_active) throw mi_error(-6, "cg_step without cg_begin");
    MI_HIP_CHECK(hipSetDevice(device));
    // m == 0: the kernels see no elements, converge at once
    for (int64_t s = 0; s < nsteps;) {
        if (run % CG_RESET == 0 && nsteps - s >= CG_RESET && graph_usable()) {
            graph_block();
            s += CG_RESET;
            run += CG_RESET;
        } else {
            cg_par = (int) (run & 1);
            cg_iter(run % CG_RESET == CG_RESET - 1 ? 1 : 0);
            ++s;
            ++run;
        }
    }
    if (cg1 && nsteps > 0) {  // the residual after the batch's last iteration: trace, stop test (cg1_delta_kernel)
        const T *cur = cg1p.get() + (int64_t) (run & 1) * 4 * RED_BLOCKS;
        flush_psum();
        launch_cg1_delta<T>(gather_partials(const_cast<T *>(cur), 1, 4 * RED_BLOCKS), G, trace.get(), trace_cap, sc.get(), stream);
    }
    cg_scalars<T> h{};
    MI_HIP_CHECK(hipMemcpyAsync(&h, sc.get(), sizeof(h), hipMemcpyDeviceToHost, stream));
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    polled = h;
    converged = h.converged != 0;
    iters = h.iters;
}

template <typename T>
void engine<T>::cg_result(T *x_out, double *trace_out, int64_t trace_len, int64_t *iters) {
    if (!cg_active) throw mi_error(-6, "cg_result without cg_begin");
    MI_HIP_CHECK(hipSetDevice(device));
    cg_scalars<T> h{};
    MI_HIP_CHECK(hipMemcpyAsync(&h, sc.get(), sizeof(h), hipMemcpyDeviceToHost, stream));
    if (x_out && m > 0) {
        if (gathered) allgather_rows(x.get());  // every rank's rows of the solution
        MI_HIP_CHECK(hipMemcpyAsync(x_out, x.get(), sizeof(T) * (size_t) m, hipMemcpyDeviceToHost, stream));
    }
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    const int64_t it = h.iters;
    if (iters) *iters = it;
    if (trace_out && trace_len > 0) {
        const int64_t cnt = std::min<int64_t>(std::min<int64_t>(trace_len, it + 1), trace_cap);
        MI_HIP_CHECK(hipMemcpy(trace_out, trace.get(), sizeof(double) * (size_t) cnt, hipMemcpyDeviceToHost));
    }
}

template <typename T>
void engine<T>::solve_cg(const T *b_host, const T *q_host, int64_t imax, T eps, T *x_out, double *trace_out,
                         int64_t *iters) {
    if (imax < 0) throw mi_error(-1, "imax must be >= 0");
    cg_begin(b_host, q_host, eps, false, nullptr, imax + 1);
    bool conv = false;
    int64_t it = 0;
    // batches of iterations between host polls (kernels after convergence exit at entry): 4, 8, 16,
    // then up to the first reset, then whole CG_RESET blocks (one captured graph each)
    int64_t batch = 4;
    std::vector<double> seg;
    while (!conv && run < imax) {
        const int64_t ns = std::min<int64_t>(run < CG_RESET ? std::min<int64_t>(batch, CG_RESET - run) : CG_RESET,
                                             imax - run);
        const int64_t first = it;
        const auto t0 = std::chrono::steady_clock::now();
        cg_step(ns, conv, it);
        batch *= 2;
        if (progress != nullptr && it > first) {
            // the batch's residuals delta_first .. delta_it (the iterations' "Start Iteration" lines,
            // OpenMP/csvm.cpp:115-117), the stop target and the batch's wall time
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            seg.resize((size_t) (it - first + 1));
            MI_HIP_CHECK(hipMemcpy(seg.data(), trace.get() + first, sizeof(double) * seg.size(), hipMemcpyDeviceToHost));
            progress(first, it - first, seg.data(), (double) polled.eps2delta0, ms, progress_user);
        }
    }
    cg_result(x_out, trace_out, imax + 1, iters);
}

// csvm<T>::learn (src/plssvm/csvm.cpp:207-267)
template <typename T>
void engine<T>::learn(const T *y, int64_t imax, T eps, T *alpha_out, double *bias_out, double *trace_out,
                      int64_t *iters) {
    need_data();
    if (y == nullptr) throw mi_error(-1, "No labels given for training! Maybe the data is only usable for prediction?");
    std::vector<T> qh(std::max<int64_t>(m, 1)), bh(std::max<int64_t>(m, 1));
    generate_q(qh.data(), nullptr);
    for (int64_t i = 0; i < m; ++i) bh[i] = y[i] - y[m];  // b = y[0..m) - y[m]   (:238-239)
    if (imax < 0) imax = d;                                // solver_CG(b, num_features_, ...)  (:256)
    solve_cg(bh.data(), nullptr, imax, eps, alpha_out, trace_out, iters);
    T s = 0, qa = 0;
    for (int64_t i = 0; i < m; ++i) s += alpha_out[i];
    for (int64_t i = 0; i < m; ++i) qa = std::fma(qh[i], alpha_out[i], qa);
    const T bias = y[m] + QA_cost * s - qa;  // (:257)
    alpha_out[m] = -s;                       // (:258)
    if (bias_out) *bias_out = (double) bias;
}

// time_kp's cache eviction: reads n 16-byte words (their contents are never used; the sink is written only
// for a value no sweep produces in practice, which keeps the loads)
__global__ __launch_bounds__(256) void flush_read_kernel(const uint4 *__restrict__ a, int64_t n, unsigned *__restrict__ sink) {
    unsigned s = 0;
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x9E3779B9u) sink[0] = s;
}

template <typename T>
void engine<T>::time_kp(int reps, double *ms_kp, double *ms_dom) {
    need_data();
    need_q();
    MI_HIP_CHECK(hipSetDevice(device));
    if (reps < 1) reps = 1;
    std::vector<T> ph(std::max<int64_t>(m, 1));
    for (int64_t i = 0; i < m; ++i) ph[i] = T(1) + T((i * 2654435761ull) % 1000) / T(1000);
    if (m > 0) MI_HIP_CHECK(hipMemcpyAsync(pv.get(), ph.data(), sizeof(T) * (size_t) m, hipMemcpyHostToDevice, stream));
    MI_HIP_CHECK(hipMemsetAsync(sc.get(), 0, sizeof(cg_scalars<T>), stream));
    hipEvent_t e0, e1, d0, d1;
    MI_HIP_CHECK(hipEventCreate(&e0));
    MI_HIP_CHECK(hipEventCreate(&e1));
    MI_HIP_CHECK(hipEventCreate(&d0));
    MI_HIP_CHECK(hipEventCreate(&d1));
    kp_device(pv.get(), ret.get(), T(1), true, nullptr);  // warm-up
    double dom = 0;
    MI_HIP_CHECK(hipEventRecord(e0, stream));
    for (int it = 0; it < reps; ++it) kp_device(pv.get(), ret.get(), T(1), true, nullptr);
    MI_HIP_CHECK(hipEventRecord(e1, stream));
    MI_HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    MI_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    // dominant kernel alone, same stream, same launches; before each launch a 512 MiB read sweep evicts what
    // the previous launch left in the L2s and the Infinity Cache (256 MiB), as the other kernels of a CG
    // iteration do between two launches — back-to-back launches would otherwise re-read part of their stream
    // from there (a read, not a memset: dirty lines would be written back during the timed launch)
    dev_buf<uint4> flush;
    try {
        flush.alloc(((int64_t) 512 << 20) / 16 + 1, stream, false);
    } catch (const mi_error &) {
        flush.reset();  // no room: time without the eviction
        (void) hipGetLastError();
    }
    for (int it = 0; it < reps; ++it) {
        if (flush.get() != nullptr) {
            hipLaunchKernelGGL(flush_read_kernel, dim3(4096), dim3(256), 0, stream, flush.get(), flush.size() - 1,
                               reinterpret_cast<unsigned *>(flush.get() + flush.size() - 1));
            MI_LAUNCH_CHECK();
        }
        MI_HIP_CHECK(hipEventRecord(d0, stream));
        if (sparse_stored()) {
            sparse_dominant(pv.get(), nullptr);
        } else if (factored()) {
            launch_gemv_n<T>(XT.get(), n_pad, d, r0, r1, w.get(), raw.get(), nullptr, stream);
        } else {
            launch_kp_tiles<T>(kf(), XT.get(), norms.get(), pv.get(), partial.get(), n_pad, d_pad, nb, t0, t1 - t0, kp_wgoff.get(), kp_wgs,
                               nullptr, stream);
        }
        MI_HIP_CHECK(hipEventRecord(d1, stream));
        MI_HIP_CHECK(hipEventSynchronize(d1));
        float t = 0;
        MI_HIP_CHECK(hipEventElapsedTime(&t, d0, d1));
        dom += t;
    }
    (void) hipEventDestroy(e0);
    (void) hipEventDestroy(e1);
    (void) hipEventDestroy(d0);
    (void) hipEventDestroy(d1);
    if (ms_kp) *ms_kp = ms / reps;
    if (ms_dom) *ms_dom = dom / reps;
}

template <typename T>
int64_t engine<T>::device_bytes() const {
    return XT.bytes() + norms.bytes() + xlast.bytes() + partial.bytes() + q.bytes() * 10 + w.bytes() + csr_bytes();
}

template struct engine<float>;
template struct engine<double>;

}  // namespace plssvm_mi
