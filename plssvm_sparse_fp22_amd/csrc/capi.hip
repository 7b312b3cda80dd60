// C ABI (include/plssvm_mi355x.h): exception-free wrappers around engine<float|double>.
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>

#include "../../include/plssvm_mi355x.h"
#include "engine.hpp"

using plssvm_mi::engine;
using plssvm_mi::mi_error;
constexpr int EXP_NWV_C = plssvm_mi::EXP_NWV;

struct plssvm_mi_ctx {
    int real_bytes = 8;
    int kernel = 0;
    std::unique_ptr<plssvm_mi::engine_base> eng;
    std::string err;

    template <typename F>
    int call(F &&f) {
        try {
            if (real_bytes == 4) {
                f(*static_cast<engine<float> *>(eng.get()));
            } else {
                f(*static_cast<engine<double> *>(eng.get()));
            }
            if (eng->comm_aborted) {  // the group was aborted while (or before) this call ran: its results are void
                err = "the group was aborted by another rank";
                return PLSSVM_MI_ERR_RCCL;
            }
            err.clear();
            return PLSSVM_MI_OK;
        } catch (const mi_error &e) {
            err = e.what();
            return e.code;
        } catch (const std::bad_alloc &) {
            err = "host allocation failed";
            return PLSSVM_MI_ERR_OOM;
        } catch (const std::exception &e) {
            err = e.what();
            return PLSSVM_MI_ERR_ARG;
        }
    }
};

namespace {
thread_local std::string g_create_error;
}

extern "C" {

int plssvm_mi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int plssvm_mi_create(int real_bytes, int kernel, int degree, double gamma, double coef0, double cost, int device,
                     plssvm_mi_ctx **out) {
    if (out == nullptr) return PLSSVM_MI_ERR_ARG;
    *out = nullptr;
    if (real_bytes != 4 && real_bytes != 8) return PLSSVM_MI_ERR_ARG;
    if (kernel < 0 || kernel > 2) return PLSSVM_MI_ERR_UNSUPPORTED;  // unsupported_kernel_type_exception
    if (kernel == 1 && degree < 0) return PLSSVM_MI_ERR_ARG;
    if (!(cost > 0)) return PLSSVM_MI_ERR_ARG;
    const int ndev = plssvm_mi_device_count();
    if (ndev <= 0) {
        g_create_error = "HIP backend selected but no HIP devices were found!";
        return PLSSVM_MI_ERR_NODEV;
    }
    if (device < 0 || device >= ndev) return PLSSVM_MI_ERR_ARG;
    try {
        auto ctx = std::make_unique<plssvm_mi_ctx>();
        ctx->real_bytes = real_bytes;
        ctx->kernel = kernel;
        if (real_bytes == 4) {
            ctx->eng = std::make_unique<engine<float>>(kernel, degree, gamma, coef0, cost, device);
        } else {
            ctx->eng = std::make_unique<engine<double>>(kernel, degree, gamma, coef0, cost, device);
        }
        *out = ctx.release();
        return PLSSVM_MI_OK;
    } catch (const mi_error &e) {
        g_create_error = e.what();
        return e.code;
    } catch (const std::exception &e) {
        g_create_error = e.what();
        return PLSSVM_MI_ERR_HIP;
    }
}

void plssvm_mi_destroy(plssvm_mi_ctx *ctx) { delete ctx; }

const char *plssvm_mi_last_error(const plssvm_mi_ctx *ctx) {
    return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

int plssvm_mi_set_option(plssvm_mi_ctx *ctx, int key, int64_t value) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        if (e.have_data) throw mi_error(PLSSVM_MI_ERR_STATE, "set options before setup");
        if (key == PLSSVM_MI_OPT_KP_MODE && value >= 0 && value <= 2) {
            e.kp_mode = (int) value;
        } else if (key == PLSSVM_MI_OPT_SIM_RANK && value >= 0) {
            const int r = (int) (value & 0xFFFF), w = (int) (value >> 16);
            if (w < 0 || (w > 0 && r >= w) || e.world > 1) throw mi_error(PLSSVM_MI_ERR_ARG, "bad simulated rank");
            e.sim_rank = r;
            e.sim_world = w;
        } else if (key == PLSSVM_MI_OPT_RBF_FORM && value >= 0 && value <= 1) {
            e.rbf_form = (int) value;
        } else if (key == PLSSVM_MI_OPT_SPARSE_ALGO && value >= 0 && value <= 4) {
            e.sparse_algo = (int) value;
        } else if (key == PLSSVM_MI_OPT_CG_VARIANT && value >= 0 && value <= 2) {
            e.cg_variant = (int) value;
        } else {
            throw mi_error(PLSSVM_MI_ERR_ARG, "bad option");
        }
    });
}

int plssvm_mi_partition(int64_t m, int rank, int world_size, int64_t *out4) {
    if (m < 0 || world_size < 1 || rank < 0 || rank >= world_size || !out4) return PLSSVM_MI_ERR_ARG;
    int64_t s0, s1, st, tt, tl;
    plssvm_mi::partition_superblocks(plssvm_mi::ceil_div(m, plssvm_mi::KP_TILE), rank, world_size, s0, s1, st, tt, tl);
    out4[0] = s0;
    out4[1] = s1;
    out4[2] = tt;
    out4[3] = tl;
    return PLSSVM_MI_OK;
}

int plssvm_mi_set_cost(plssvm_mi_ctx *ctx, double cost) {
    if (!ctx || !(cost > 0)) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        e.cost = (decltype(e.cost)) cost;
        e.graph_reset();  // a captured CG block holds 1/C
    });
}

int plssvm_mi_set_qa_cost(plssvm_mi_ctx *ctx, double qa) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        e.need_data();
        e.QA_cost = (decltype(e.QA_cost)) qa;
        e.have_q = true;
        e.graph_reset();
    });
}

int plssvm_mi_get_unique_id(void *id_out) {
    if (!id_out) return PLSSVM_MI_ERR_ARG;
    static_assert(sizeof(ncclUniqueId) == PLSSVM_MI_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return PLSSVM_MI_ERR_RCCL;
    std::memcpy(id_out, &id, sizeof(id));
    return PLSSVM_MI_OK;
}

int plssvm_mi_comm_init(plssvm_mi_ctx *ctx, int rank, int world_size, const void *unique_id) {
    if (!ctx || (world_size > 1 && !unique_id)) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) { e.comm_init(rank, world_size, unique_id); });
}

int plssvm_mi_comm_abort(plssvm_mi_ctx *ctx) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    ctx->eng->comm_abort();  // no ctx->call: this runs beside the context's own thread, which may be inside a call
    return PLSSVM_MI_OK;
}

int plssvm_mi_comm_init_host(plssvm_mi_ctx *ctx, int rank, int world_size, plssvm_mi_exchange_fn fn, void *user) {
    if (!ctx || !fn) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) { e.comm_init_host(rank, world_size, fn, user); });
}

int plssvm_mi_setup_dense(plssvm_mi_ctx *ctx, const void *X, int64_t n, int64_t d) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.setup_dense(static_cast<const T *>(X), n, d);
    });
}

int plssvm_mi_setup_csr(plssvm_mi_ctx *ctx, const int64_t *rowptr, const int32_t *col, const void *val, int val_fmt,
                        int64_t n, int64_t d) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) { e.setup_csr(rowptr, col, val, val_fmt, n, d); });
}

int plssvm_mi_setup_coo(plssvm_mi_ctx *ctx, const int64_t *row, const int32_t *col, const void *val, int val_fmt,
                        int64_t nnz, int64_t n, int64_t d) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        using plssvm_mi::mi_error;
        if (n < 1 || d < 1) throw mi_error(PLSSVM_MI_ERR_ARG, "Data set is empty!");
        if (nnz < 0 || (nnz > 0 && (!row || !col || !val))) throw mi_error(PLSSVM_MI_ERR_ARG, "COO arrays missing");
        if (val_fmt != PLSSVM_MI_VAL_REAL && val_fmt != PLSSVM_MI_VAL_FP22) throw mi_error(PLSSVM_MI_ERR_ARG, "unknown value format");
        // counting sort by row (stable), then columns ascending inside each row
        std::vector<int64_t> rowptr((size_t) n + 1, 0);
        for (int64_t k = 0; k < nnz; ++k) {
            if (row[k] < 0 || row[k] >= n) throw mi_error(PLSSVM_MI_ERR_ARG, "COO row index out of range");
            if (col[k] < 0 || col[k] >= d) throw mi_error(PLSSVM_MI_ERR_ARG, "COO column index out of range");
            ++rowptr[(size_t) row[k] + 1];
        }
        for (int64_t i = 0; i < n; ++i) rowptr[(size_t) i + 1] += rowptr[(size_t) i];
        std::vector<int64_t> perm((size_t) std::max<int64_t>(nnz, 1)), fill(rowptr.begin(), rowptr.end() - 1);
        for (int64_t k = 0; k < nnz; ++k) perm[(size_t) fill[(size_t) row[k]]++] = k;
        std::vector<int32_t> ccol((size_t) std::max<int64_t>(nnz, 1));
        for (int64_t i = 0; i < n; ++i) {
            auto b = perm.begin() + rowptr[(size_t) i], en = perm.begin() + rowptr[(size_t) i + 1];
            std::sort(b, en, [&](int64_t a, int64_t c) { return col[a] < col[c]; });
            for (auto it = b; it != en; ++it) {
                if (it != b && col[*it] == col[*(it - 1)])
                    throw mi_error(PLSSVM_MI_ERR_ARG, "duplicate COO entry (row " + std::to_string(i) + ", column " +
                                                          std::to_string(col[*it]) + ")");
                ccol[(size_t) (it - perm.begin())] = col[*it];
            }
        }
        if (val_fmt == PLSSVM_MI_VAL_FP22) {  // re-pack the words in CSR order (decode(encode(x)) is exact)
            const auto *w = static_cast<const uint32_t *>(val);
            std::vector<uint32_t> words((size_t) plssvm_mi::fp22_words(std::max<int64_t>(nnz, 1)) + 1, 0u);
            for (int64_t t = 0; t < nnz; ++t) {
                const uint64_t code = plssvm_mi::fp22_encode_host(plssvm_mi::fp22_get(w, perm[(size_t) t]));
                const int64_t g = t >> 4;
                const int bit = 22 * (int) (t & 15);
                const int64_t wi = g * 11 + (bit >> 5);
                const int sh = bit & 31;
                words[(size_t) wi] |= (uint32_t) (code << sh);
                if (sh > 10) words[(size_t) wi + 1] |= (uint32_t) (code >> (32 - sh));
            }
            e.setup_csr(rowptr.data(), ccol.data(), words.data(), val_fmt, n, d);
        } else {
            const auto *v = static_cast<const T *>(val);
            std::vector<T> cval((size_t) std::max<int64_t>(nnz, 1));
            for (int64_t t = 0; t < nnz; ++t) cval[(size_t) t] = v[perm[(size_t) t]];
            e.setup_csr(rowptr.data(), ccol.data(), cval.data(), val_fmt, n, d);
        }
    });
}

int plssvm_mi_generate_q(plssvm_mi_ctx *ctx, void *q_out, double *qa_cost_out) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.generate_q(static_cast<T *>(q_out), qa_cost_out);
    });
}

int plssvm_mi_kp(plssvm_mi_ctx *ctx, const void *q, const void *p, void *ret, double add) {
    if (!ctx || !p || !ret) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.kp_host(static_cast<const T *>(q), static_cast<const T *>(p), static_cast<T *>(ret), (T) add);
    });
}

int plssvm_mi_kp_part(plssvm_mi_ctx *ctx, const void *p, void *out, int part) {
    if (!ctx || !p || !out) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.kp_part(static_cast<const T *>(p), static_cast<T *>(out), part);
    });
}

int plssvm_mi_solve_cg(plssvm_mi_ctx *ctx, const void *b, const void *q, int64_t imax, double eps, void *x_out,
                       double *delta_trace, int64_t *iters) {
    if (!ctx || !b || !x_out) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.solve_cg(static_cast<const T *>(b), static_cast<const T *>(q), imax, (T) eps, static_cast<T *>(x_out),
                   delta_trace, iters);
    });
}

int plssvm_mi_set_progress(plssvm_mi_ctx *ctx, plssvm_mi_progress_fn fn, void *user) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        e.progress = fn;
        e.progress_user = user;
    });
}

int plssvm_mi_cg_begin(plssvm_mi_ctx *ctx, const void *b, const void *q, double eps, double *delta0_out) {
    if (!ctx || !b) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.cg_begin(static_cast<const T *>(b), static_cast<const T *>(q), (T) eps, false, delta0_out, 4096);
    });
}

int plssvm_mi_cg_step(plssvm_mi_ctx *ctx, int64_t n, int force, int64_t *iters_done, int *converged) {
    if (!ctx || n < 0) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        if (force) {
            // bench mode: keep iterating past convergence with identical work per iteration
            using T = std::remove_reference_t<decltype(e.gamma)>;
            plssvm_mi::cg_scalars<T> h{};
            MI_HIP_CHECK(hipMemcpyAsync(&h, e.sc.get(), sizeof(h), hipMemcpyDeviceToHost, e.stream));
            MI_HIP_CHECK(hipStreamSynchronize(e.stream));
            if (!h.force) {
                h.force = 1;
                h.eps2delta0 = T(-1);
                h.converged = 0;
                MI_HIP_CHECK(hipMemcpyAsync(e.sc.get(), &h, sizeof(h), hipMemcpyHostToDevice, e.stream));
            }
        }
        bool conv = false;
        int64_t it = 0;
        e.cg_step(n, conv, it);
        if (iters_done) *iters_done = it;
        if (converged) *converged = conv ? 1 : 0;
    });
}

int plssvm_mi_cg_result(plssvm_mi_ctx *ctx, void *x_out, double *delta_trace, int64_t trace_len, int64_t *iters) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.cg_result(static_cast<T *>(x_out), delta_trace, trace_len, iters);
    });
}

int plssvm_mi_learn(plssvm_mi_ctx *ctx, const void *y, int64_t imax, double eps, void *alpha_out, double *bias_out,
                    double *delta_trace, int64_t *iters) {
    if (!ctx || !alpha_out) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.learn(static_cast<const T *>(y), imax, (T) eps, static_cast<T *>(alpha_out), bias_out, delta_trace, iters);
    });
}

int plssvm_mi_time_kp(plssvm_mi_ctx *ctx, int reps, double *ms_per_kp, double *ms_dominant_kernel) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) { e.time_kp(reps, ms_per_kp, ms_dominant_kernel); });
}

int plssvm_mi_update_w(plssvm_mi_ctx *ctx, const void *alpha, void *w_out) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        e.update_w(static_cast<const T *>(alpha), static_cast<T *>(w_out));
    });
}

int plssvm_mi_predict_dense(plssvm_mi_ctx *ctx, const void *alpha, double bias, const void *Z, int64_t np, int64_t d,
                            void *out) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        if (np > 0 && Z == nullptr) throw plssvm_mi::mi_error(PLSSVM_MI_ERR_ARG, "no points to predict");
        e.predict(static_cast<const T *>(alpha), (T) bias, static_cast<const T *>(Z), nullptr, nullptr, nullptr,
                  PLSSVM_MI_VAL_REAL, np, d, static_cast<T *>(out));
    });
}

int plssvm_mi_predict_csr(plssvm_mi_ctx *ctx, const void *alpha, double bias, const int64_t *rowptr, const int32_t *col,
                          const void *val, int val_fmt, int64_t np, int64_t d, void *out) {
    if (!ctx) return PLSSVM_MI_ERR_ARG;
    return ctx->call([&](auto &e) {
        using T = std::remove_reference_t<decltype(e.gamma)>;
        if (np > 0 && (rowptr == nullptr || col == nullptr || (val == nullptr && rowptr[np] > 0)))
            throw plssvm_mi::mi_error(PLSSVM_MI_ERR_ARG, "no points to predict");
        e.predict(static_cast<const T *>(alpha), (T) bias, nullptr, rowptr, col, val, val_fmt, np, d,
                  static_cast<T *>(out));
    });
}

int plssvm_mi_get_info(const plssvm_mi_ctx *cctx, plssvm_mi_info *info) {
    if (!cctx || !info) return PLSSVM_MI_ERR_ARG;
    auto *ctx = const_cast<plssvm_mi_ctx *>(cctx);
    return ctx->call([&](auto &e) {
        std::memset(info, 0, sizeof(*info));
        info->n = e.n;
        info->d = e.d;
        info->m = e.m;
        info->n_pad = e.n_pad;
        info->d_pad = e.d_pad;
        info->nnz = e.csr.nnz;
        info->tiles_total = e.tiles_total;
        info->tiles_local = e.tiles_local;
        info->tile_rows = plssvm_mi::KP_TILE;
        info->tile_cols = plssvm_mi::KP_TILE;
        info->device_bytes = e.device_bytes();
        info->pairs = e.csr.pairs;
        info->kp_mode = e.factored() ? PLSSVM_MI_KP_FACTORED : PLSSVM_MI_KP_PAIRWISE;
        info->rank = e.rank;
        info->world_size = e.world;
        info->real_bytes = (int) sizeof(e.gamma);
        info->kernel = e.kernel;
        info->is_sparse = e.sparse ? 1 : 0;
        info->val_fmt = e.csr.val_fmt;
        info->rbf_factored = e.csr.rbf_factored ? 1 : 0;
        info->pair_slots = e.csr.slots;
        info->spmv_bytes = e.csr.spmv_csc.stream_bytes() + e.csr.spmv_csr.stream_bytes();
        info->rbf_small_args = e.csr.rbf_small ? 1 : 0;
        info->sparse_algo = e.csr.dense_on ? PLSSVM_MI_SPARSE_DENSE
                            : e.csr.otf_on ? PLSSVM_MI_SPARSE_ONTHEFLY
                            : e.csr.ex.on  ? PLSSVM_MI_SPARSE_EXPANSION
                                           : (e.csr.have_gram ? PLSSVM_MI_SPARSE_PATTERN : 0);
        info->exp_terms = e.csr.ex.on ? e.csr.ex.K : 0;
        info->exp_waves = (int) (e.csr.ex.nblk * EXP_NWV_C);
        info->exp_chunks = e.csr.ex.nchunks;
        info->exp_hbytes = e.csr.ex.on ? (e.csr.ex.hbf16 ? 2 : (int) sizeof(e.gamma)) : 0;
        info->exp_layout = !e.csr.ex.on ? 0 : e.csr.ex.rpairs ? 4 : e.csr.ex.rflags ? 2 : 1;
        info->exp_dot2 = e.csr.ex.on && e.csr.ex.hbf16 && e.csr.ex.dot2 && sizeof(e.gamma) == 4 && plssvm_mi::exp_dot2_built() ? 1 : 0;
        info->centered = e.ctr_active() ? 1 : 0;
        info->exp_lt = e.csr.ex.on && e.csr.ex.lt ? 1 : 0;
    });
}

}  // extern "C"
