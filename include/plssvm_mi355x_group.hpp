/*
 * plssvm_mi355x_group.hpp — one process driving several GPUs through the C ABI (header-only, C++17).
 *
 * The reference's hip::csvm<T>(params) takes every visible GPU in one process: its device list is
 * min(#GPUs, ...) (src/plssvm/backends/HIP/csvm.hip.cpp:53-55) and gpu_csvm runs one OpenMP thread per device
 * (src/plssvm/backends/gpu_csvm.cpp:136-155,366-386). device_group is that arrangement on the row-block
 * partitioned C ABI: one host thread and one plssvm_mi_ctx per GPU, the contexts joined into one group, every
 * call issued on all threads at once (the contexts' collectives meet inside the library), rank 0's outputs handed
 * back. The transport:
 *   - RCCL (distinct devices): rank 0 creates the unique id, every thread calls plssvm_mi_comm_init with it;
 *   - the in-process host exchange (a device listed twice, e.g. two contexts on one GPU, which RCCL refuses, or on
 *     request): thread_exchange below is the plssvm_mi_exchange_fn of every rank — the reference's own
 *     device_reduction semantics (host-staged, summed in rank order, the same bits on every rank).
 * Failure protocol: the first rank whose call fails aborts the group (plssvm_mi_comm_abort on every context, and
 * the host exchange wakes every rank waiting in it), so no thread is left waiting in a collective; run() then
 * throws group_error with that rank's code and message on the calling thread. The group is unusable afterwards
 * (like the reference after a backend_exception).
 */
#ifndef PLSSVM_MI355X_GROUP_HPP
#define PLSSVM_MI355X_GROUP_HPP

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "plssvm_mi355x.h"

namespace plssvm::mi355x {

struct group_error : std::runtime_error {
    int code, rank;
    group_error(int c, int r, const std::string &m) : std::runtime_error(m), code(c), rank(r) {}
};

// In-process host exchange between the world threads of one group (plssvm_mi_exchange_fn semantics,
// include/plssvm_mi355x.h): all-reduce = the rank-order sum b_0 + b_1 + ... computed by every rank for itself
// (identical bits), all-gather = rank r's chunk copied from rank r's buffer. Two barriers per exchange: every
// buffer is posted before any is read, and read before any is changed again.
class thread_exchange {
  public:
    explicit thread_exchange(int world) :
        world_(world), bufs_((size_t) world, nullptr), sums_((size_t) world), users_((size_t) world) {
        for (int r = 0; r < world; ++r) users_[(size_t) r] = { this, r };
    }
    void *user(int rank) { return &users_[(size_t) rank]; }
    void abort() {
        std::lock_guard<std::mutex> lk(mu_);
        aborted_ = true;
        cv_.notify_all();
    }
    static int fn(void *buf, int64_t count, int real_bytes, int op, void *user) {
        const auto *u = static_cast<const rank_user *>(user);
        return u->x->exchange(u->rank, buf, count, real_bytes, op);
    }

  private:
    struct rank_user {
        thread_exchange *x;
        int rank;
    };
    int barrier() {
        std::unique_lock<std::mutex> lk(mu_);
        if (aborted_) return -1;
        const long long gen = gen_;
        if (++arrived_ == world_) {
            arrived_ = 0;
            ++gen_;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen_ != gen || aborted_; });
        }
        return aborted_ ? -1 : 0;
    }
    template <typename T>
    void sum_into(int rank, int64_t count) {
        std::vector<T> acc(static_cast<const T *>(bufs_[0]), static_cast<const T *>(bufs_[0]) + count);
        for (int r = 1; r < world_; ++r) {
            const T *b = static_cast<const T *>(bufs_[(size_t) r]);
            for (int64_t k = 0; k < count; ++k) acc[(size_t) k] += b[k];
        }
        auto &s = sums_[(size_t) rank];
        s.resize(sizeof(T) * (size_t) count);
        if (count > 0) std::memcpy(s.data(), acc.data(), s.size());
    }
    int exchange(int rank, void *buf, int64_t count, int real_bytes, int op) {
        if (count < 0 || (real_bytes != 4 && real_bytes != 8)) return -1;
        {
            std::lock_guard<std::mutex> lk(mu_);
            bufs_[(size_t) rank] = buf;
        }
        if (barrier() != 0) return -1;  // every rank's buffer is posted
        if (op == PLSSVM_MI_XCHG_ALLREDUCE) {
            if (real_bytes == 4) sum_into<float>(rank, count);
            else sum_into<double>(rank, count);
        } else if (op == PLSSVM_MI_XCHG_ALLGATHER) {
            const size_t chunk = (size_t) count * (size_t) real_bytes;
            for (int r = 0; r < world_; ++r)
                if (r != rank)
                    std::memcpy(static_cast<unsigned char *>(buf) + chunk * (size_t) r,
                                static_cast<const unsigned char *>(bufs_[(size_t) r]) + chunk * (size_t) r, chunk);
        } else {
            abort();
            return -1;
        }
        if (barrier() != 0) return -1;  // every buffer has been read
        if (op == PLSSVM_MI_XCHG_ALLREDUCE) {
            auto &s = sums_[(size_t) rank];
            if (!s.empty()) std::memcpy(buf, s.data(), s.size());
        }
        return 0;
    }

    int world_;
    std::mutex mu_;
    std::condition_variable cv_;
    int arrived_ = 0;
    long long gen_ = 0;
    bool aborted_ = false;
    std::vector<void *> bufs_;
    std::vector<std::vector<unsigned char>> sums_;
    std::vector<rank_user> users_;
};

// One host thread + one context per listed device; run(f) executes f(rank, ctx) on every rank's thread
// concurrently and returns when all are done.
class device_group {
  public:
    enum class transport { automatic, rccl, host };

    device_group(const std::vector<int> &devices, int real_bytes, int kernel, int degree, double gamma, double coef0,
                 double cost, transport tr = transport::automatic) :
        devices_(devices) {
        const int world = (int) devices_.size();
        if (world < 1) throw group_error(PLSSVM_MI_ERR_ARG, 0, "a device group needs at least one device");
        ctx_.assign((size_t) world, nullptr);
        create_err_.assign((size_t) world, std::string());
        bool repeated = false;
        for (int a = 0; a < world; ++a)
            for (int b = 0; b < a; ++b) repeated = repeated || devices_[(size_t) a] == devices_[(size_t) b];
        host_ = world > 1 && (tr == transport::host || (tr == transport::automatic && repeated));
        if (world > 1 && !host_ && repeated)
            throw group_error(PLSSVM_MI_ERR_ARG, 0, "RCCL needs distinct devices (two ranks on one GPU: the host exchange)");
        workers_.reserve((size_t) world);
        for (int r = 0; r < world; ++r) workers_.emplace_back(new worker);
        for (int r = 0; r < world; ++r) workers_[(size_t) r]->t = std::thread([this, r] { loop(r); });
        try {
            run([&](int r, plssvm_mi_ctx *&c) {
                const int rc = plssvm_mi_create(real_bytes, kernel, degree, gamma, coef0, cost, devices_[(size_t) r], &c);
                if (rc != PLSSVM_MI_OK) create_err_[(size_t) r] = plssvm_mi_last_error(nullptr);
                return rc;
            });
            created_ = true;
            if (world > 1) {
                if (host_) {
                    xchg_.reset(new thread_exchange(world));
                    run([&](int r, plssvm_mi_ctx *&c) {
                        return plssvm_mi_comm_init_host(c, r, world, &thread_exchange::fn, xchg_->user(r));
                    });
                } else {
                    char id[PLSSVM_MI_UNIQUE_ID_BYTES];
                    const int rc = plssvm_mi_get_unique_id(id);
                    if (rc != PLSSVM_MI_OK) throw group_error(rc, 0, "RCCL unique id");
                    run([&](int r, plssvm_mi_ctx *&c) { return plssvm_mi_comm_init(c, r, world, id); });
                }
            }
        } catch (...) {
            shutdown();
            throw;
        }
    }
    ~device_group() { shutdown(); }
    device_group(const device_group &) = delete;
    device_group &operator=(const device_group &) = delete;

    int size() const { return (int) devices_.size(); }
    bool host_exchange() const { return host_; }
    const std::vector<int> &devices() const { return devices_; }

    // f(rank, ctx) -> PLSSVM_MI_* code, on every rank's thread at once. The first failure aborts the group and
    // is rethrown here as group_error (code, rank, that context's message).
    void run(const std::function<int(int, plssvm_mi_ctx *&)> &f) {
        if (dead_) throw group_error(PLSSVM_MI_ERR_STATE, 0, "the device group was aborted by an earlier failure");
        const int world = size();
        first_fail_.store(-1);
        fail_msg_.clear();
        fail_code_ = 0;
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            ++job_gen_;
            pending_ = world;
        }
        cv_job_.notify_all();
        std::unique_lock<std::mutex> lk(mu_);
        cv_done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
        const int fr = first_fail_.load();
        if (fr >= 0) {
            dead_ = true;
            throw group_error(fail_code_, fr, fail_msg_);
        }
    }

  private:
    struct worker {
        std::thread t;
    };
    void loop(int r) {
        long long seen = 0;
        for (;;) {
            const std::function<int(int, plssvm_mi_ctx *&)> *job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_job_.wait(lk, [&] { return stop_ || job_gen_ != seen; });
                if (stop_) return;
                seen = job_gen_;
                job = job_;
            }
            try {
                const int rc = (*job)(r, ctx_[(size_t) r]);
                if (rc != PLSSVM_MI_OK) {
                    const char *m = ctx_[(size_t) r] != nullptr ? plssvm_mi_last_error(ctx_[(size_t) r])
                                                                : create_err_[(size_t) r].c_str();
                    record_failure(r, rc, m != nullptr ? m : "");
                }
            } catch (const std::exception &e) {  // a caller's job that throws counts as a failure of its rank
                record_failure(r, PLSSVM_MI_ERR_ARG, e.what());
            }
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) cv_done_.notify_all();
        }
    }
    void record_failure(int r, int rc, const std::string &msg) {
        int expect = -1;
        if (first_fail_.compare_exchange_strong(expect, r)) {
            {
                std::lock_guard<std::mutex> lk(fail_mu_);
                fail_code_ = rc;
                fail_msg_ = msg;
            }
            // release every rank that waits (or will wait) for this one in a collective
            if (xchg_) xchg_->abort();
            if (created_)
                for (plssvm_mi_ctx *c : ctx_)
                    if (c != nullptr) (void) plssvm_mi_comm_abort(c);
        }
    }
    void shutdown() {
        if (!workers_.empty() && !stop_) {
            // contexts are destroyed on their own threads (each has its device current there)
            try {
                dead_ = false;
                run([](int, plssvm_mi_ctx *&c) {
                    plssvm_mi_destroy(c);
                    c = nullptr;
                    return PLSSVM_MI_OK;
                });
            } catch (...) {
            }
            {
                std::lock_guard<std::mutex> lk(mu_);
                stop_ = true;
            }
            cv_job_.notify_all();
            for (auto &w : workers_)
                if (w->t.joinable()) w->t.join();
        }
        for (auto &w : workers_) delete w;
        workers_.clear();
    }

    std::vector<int> devices_;
    std::vector<plssvm_mi_ctx *> ctx_;
    std::vector<std::string> create_err_;
    std::vector<worker *> workers_;
    std::unique_ptr<thread_exchange> xchg_;
    bool host_ = false, dead_ = false, stop_ = false, created_ = false;
    std::mutex mu_, fail_mu_;
    std::condition_variable cv_job_, cv_done_;
    const std::function<int(int, plssvm_mi_ctx *&)> *job_ = nullptr;
    long long job_gen_ = 0;
    int pending_ = 0;
    std::atomic<int> first_fail_{ -1 };
    int fail_code_ = 0;
    std::string fail_msg_;
};

}  // namespace plssvm::mi355x

#endif /* PLSSVM_MI355X_GROUP_HPP */
