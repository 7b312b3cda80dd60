// plssvm::mi355x::csvm<T> — the reference's plssvm::csvm<T> / hip::csvm<T> surface over the C ABI
// (include/plssvm_mi355x.h). Host-only C++17; all compute runs in libplssvm_mi355x.so on the GPU.
//
// Derives from csvm_interface<T> (csvm_interface.hpp: the reference's abstract plssvm::csvm<T>, restated:
// same pure virtuals, state, constructor checks and learn()) and implements its five pure virtuals on the
// C ABI — exactly what a maintainer's hip::csvm<T> replacement does. The hooks
// mock_hip_csvm exposes (tests/backends/HIP/mock_hip_csvm.hpp:24-51) are public here; write_model()
// writes the LIBSVM model format of csvm.cpp:60-204.
#pragma once

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/plssvm_mi355x.h"
#include "../../include/plssvm_mi355x_group.hpp"
#include "csvm_interface.hpp"
#include "parameter.hpp"

namespace plssvm::mi355x {

struct backend_exception : std::runtime_error {  // plssvm::hip::backend_exception
    int code;
    backend_exception(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

template <typename T>
class csvm : public csvm_interface<T> {
    using base = csvm_interface<T>;

  public:
    using real_type = T;
    using base::learn;  // learn() (imax = num_features) and learn(imax)

    // hip::csvm<T>(params) (src/plssvm/backends/HIP/csvm.hip.cpp:38-81): every visible GPU of the node, one host
    // thread and one context per GPU in a row-block group (RCCL), at most one GPU per row of the m = N - 1 rows
    explicit csvm(const parameter<T> &params) : csvm(params, all_devices(params)) {}
    // one GPU (plssvm-train --device N)
    csvm(const parameter<T> &params, int device) : csvm(params, std::vector<int>{ device }) {}
    // an explicit device list; a device listed twice forms the group over the in-process host exchange
    // (device_group: two contexts on one GPU, which RCCL refuses — the multi-rank path's test transport)
    csvm(const parameter<T> &params, const std::vector<int> &devices,
         device_group::transport tr = device_group::transport::automatic) :
        base(params) {
        try {
            grp_ = std::make_unique<device_group>(devices, (int) sizeof(T), (int) this->kernel_, this->degree_,
                                                  (double) this->gamma_, (double) this->coef0_, (double) this->cost_, tr);
        } catch (const group_error &e) {
            throw backend_exception(e.code, e.what());
        }
    }

    // the visible GPUs the default constructor takes: min(#GPUs, m), like the reference's min(#GPUs, #features)
    // feature split (csvm.hip.cpp:53-55), here over rows
    static std::vector<int> all_devices(const parameter<T> &params) {
        const int n = plssvm_mi_device_count();
        if (n <= 0) throw backend_exception(PLSSVM_MI_ERR_NODEV, "HIP backend selected but no HIP devices were found!");
        const int64_t m = std::max<int64_t>(params.num_data_points - 1, 1);
        std::vector<int> d((size_t) std::min<int64_t>(n, m));
        for (size_t k = 0; k < d.size(); ++k) d[k] = (int) k;
        return d;
    }
    int num_devices() const { return grp_->size(); }
    const std::vector<int> &devices() const { return grp_->devices(); }

    // one process per GPU instead (MPI / torch launchers): a one-device csvm joins a row-block group before setup
    // (rank 0 creates the id)
    void join_group(int rank, int world, const void *unique_id) {
        if (grp_->size() != 1) throw exception{ "join_group needs a one-device csvm" };
        on_all([&](int, plssvm_mi_ctx *c) { return plssvm_mi_comm_init(c, rank, world, unique_id); });
    }

    // ---- the reference's pure virtuals (csvm.hpp:188-214), public here like mock_hip_csvm's hooks ----
    // every call runs on all ranks at once (their collectives meet inside the library); outputs come from rank 0
    void setup_data_on_device() override {
        const auto &p = this->params_;
        on_all([&](int, plssvm_mi_ctx *c) {
            if (p.sparse) {
                const bool f22 = !p.val22.empty() && sizeof(T) == 4;  // packed FP22 input stays packed
                return plssvm_mi_setup_csr(c, p.rowptr.data(), p.col.data(), f22 ? (const void *) p.val22.data() : p.val.data(),
                                           f22 ? PLSSVM_MI_VAL_FP22 : PLSSVM_MI_VAL_REAL, p.num_data_points, p.num_features);
            }
            return plssvm_mi_setup_dense(c, p.dense.data(), p.num_data_points, p.num_features);
        });
        on_device_ = true;
    }
    [[nodiscard]] std::vector<T> generate_q() override {
        const size_t len = std::max<std::size_t>(this->num_data_points_ - 1, 1);
        std::vector<T> q(len);
        auto sc = scratch(len);
        on_all([&](int r, plssvm_mi_ctx *c) {
            double qa = 0;
            return plssvm_mi_generate_q(c, r == 0 ? q.data() : sc[(size_t) r].data(), &qa);
        });
        q.resize(this->num_data_points_ - 1);
        return q;
    }
    // with print_info, the reference's per-iteration lines (OpenMP/csvm.cpp:115-117,161-166): the residual
    // before each iteration and the stop target, streamed per polled batch of device iterations; the
    // "Done in" time of an iteration is its batch's wall time / iterations (the device runs a batch
    // without host round trips), truncated to ms like the reference's duration_cast
    std::vector<T> solver_CG(const std::vector<T> &b, std::size_t imax, T eps, const std::vector<T> &q) override {
        const size_t len = std::max<std::size_t>(b.size(), 1);
        std::vector<T> x(len);
        auto sc = scratch(len);
        std::vector<std::vector<double>> tr((size_t) grp_->size(), std::vector<double>(imax + 1, 0.0));
        std::vector<int64_t> its((size_t) grp_->size(), 0);
        progress_state ps{ (int64_t) imax, 0.0, 0.0, 0 };
        on_all([&](int r, plssvm_mi_ctx *c) {
            int rc = plssvm_mi_set_qa_cost(c, (double) this->QA_cost_);  // learn() computed it on the host
            if (rc != PLSSVM_MI_OK) return rc;
            if (this->print_info_ && r == 0) {
                rc = plssvm_mi_set_progress(c, &csvm::print_progress, &ps);
                if (rc != PLSSVM_MI_OK) return rc;
            }
            rc = plssvm_mi_solve_cg(c, b.data(), q.data(), (int64_t) imax, (double) eps, r == 0 ? x.data() : sc[(size_t) r].data(),
                                    tr[(size_t) r].data(), &its[(size_t) r]);
            if (this->print_info_ && r == 0) (void) plssvm_mi_set_progress(c, nullptr, nullptr);
            return rc;
        });
        const int64_t it = its[0];
        iterations_ = it;
        trace_ = std::move(tr[0]);
        trace_.resize((std::size_t) it + 1);
        x.resize(b.size());
        if (this->print_info_) {
            const int64_t shown = std::min<int64_t>(it, (int64_t) imax);  // min(run + 1, imax)
            std::printf("Finished after %lld iterations with a residuum of %s (target: %s) and an average iteration time of %lldms.\n",
                        (long long) shown, shortest((T) trace_.back()).c_str(), shortest((T) ps.target).c_str(),
                        (long long) (shown > 0 ? ps.ms_total / (double) shown : 0.0));
            std::fflush(stdout);
        }
        return x;
    }
    // gpu_csvm::update_w (gpu_csvm.cpp:327-350): w_ = sum_i alpha_i x_i (linear model vector)
    void update_w() override {
        need_model();
        const size_t len = std::max<std::size_t>(this->num_features_, 1);
        this->w_.assign(len, T(0));
        auto sc = scratch(len);
        const T *alpha = this->alpha_ptr_->data();
        on_all([&](int r, plssvm_mi_ctx *c) {
            return plssvm_mi_update_w(c, alpha, r == 0 ? this->w_.data() : sc[(size_t) r].data());
        });
        this->w_.resize(this->num_features_);
    }
    // gpu_csvm::predict (gpu_csvm.cpp:52-127): decision values bias + sum_i alpha_i k(x_i, z) of dense points
    [[nodiscard]] std::vector<T> predict(const std::vector<std::vector<T>> &points) override {
        need_model();
        if (points.empty()) return {};
        std::vector<T> Z;
        Z.reserve(points.size() * points[0].size());
        for (const auto &z : points) {
            if (z.size() != points[0].size()) throw exception{ "All points in the data vector must have the same number of features!" };
            Z.insert(Z.end(), z.begin(), z.end());
        }
        std::vector<T> out(points.size());
        auto sc = scratch(points.size());
        const T *alpha = this->alpha_ptr_->data();
        on_all([&](int r, plssvm_mi_ctx *c) {
            return plssvm_mi_predict_dense(c, alpha, (double) this->bias_, Z.data(), (int64_t) points.size(),
                                           (int64_t) points[0].size(), r == 0 ? out.data() : sc[(size_t) r].data());
        });
        return out;
    }

    // ---- run_device_kernel + the mock_hip_csvm setters (tests/backends/HIP/mock_hip_csvm.hpp:24-51) ----
    void run_device_kernel(const std::vector<T> &q, std::vector<T> &ret, const std::vector<T> &d, T add) {
        std::vector<std::vector<T>> rets((size_t) grp_->size(), ret);  // every rank adds into its own copy
        on_all([&](int r, plssvm_mi_ctx *c) {
            return plssvm_mi_kp(c, q.data(), d.data(), r == 0 ? ret.data() : rets[(size_t) r].data(), (double) add);
        });
    }
    void set_cost(T c) {
        on_all([&](int, plssvm_mi_ctx *x) { return plssvm_mi_set_cost(x, (double) c); });
        this->cost_ = c;
    }
    void set_QA_cost(T qa) {
        on_all([&](int, plssvm_mi_ctx *x) { return plssvm_mi_set_qa_cost(x, (double) qa); });
        this->QA_cost_ = qa;
    }

    // csvm<T>::write_model (src/plssvm/csvm.cpp:60-204): positive-label support vectors first
    void write_model(const std::string &filename) const {
        if (this->alpha_ptr_ == nullptr) throw exception{ "No alphas given! Maybe a call to 'learn()' is missing?" };
        const auto &p = this->params_;
        const auto &alpha_ = *this->alpha_ptr_;
        const T bias_ = this->bias_;
        std::size_t npos = 0, nneg = 0;
        for (const T v : p.labels) (v > 0 ? npos : nneg) += 1;
        std::string out = "svm_type c_svc\nkernel_type ";
        out += kernel_name(p.kernel);
        out += "\n";
        if (p.kernel == kernel_type::polynomial) {
            out += "degree " + std::to_string(p.degree) + "\ngamma " + shortest(p.gamma) + "\ncoef0 " + shortest(p.coef0) + "\n";
        } else if (p.kernel == kernel_type::rbf) {
            out += "gamma " + shortest(p.gamma) + "\n";
        }
        out += "nr_class 2\ntotal_sv " + std::to_string(npos + nneg) + "\nrho " + shortest(-bias_) +
               "\nlabel 1 -1\nnr_sv " + std::to_string(npos) + " " + std::to_string(nneg) + "\nSV\n";
        for (int pass = 0; pass < 2; ++pass) {
            for (int64_t i = 0; i < p.num_data_points; ++i) {
                if ((p.labels[(std::size_t) i] > 0) != (pass == 0)) continue;
                out += shortest(alpha_[(std::size_t) i]) + " ";
                char buf[64];
                auto feat = [&](int64_t f, T v) {
                    std::snprintf(buf, sizeof buf, "%lld:%e ", (long long) f, (double) v);  // "{}:{:e} "
                    out += buf;
                };
                if (p.sparse) {
                    for (int64_t k = p.rowptr[i]; k < p.rowptr[i + 1]; ++k)
                        if (p.val[(std::size_t) k] != T(0)) feat(p.col[(std::size_t) k], p.val[(std::size_t) k]);
                } else {
                    for (int64_t f = 0; f < p.num_features; ++f)
                        if (p.dense[(std::size_t) (i * p.num_features + f)] != T(0)) feat(f, p.dense[(std::size_t) (i * p.num_features + f)]);
                }
                out += "\n";
            }
        }
        std::FILE *fp = std::fopen(filename.c_str(), "w");
        if (!fp) throw std::runtime_error("Can't open model file '" + filename + "'!");
        std::fwrite(out.data(), 1, out.size(), fp);
        std::fclose(fp);
    }

    // model use (csvm.hpp:123-178; gpu_csvm::update_w / predict, gpu_csvm.cpp:52-127,327-350). Without a
    // preceding learn(), set_model() supplies the alphas and rho of a model file.
    void set_model(std::vector<T> alpha, T rho) {
        if (alpha.size() != this->num_data_points_)
            throw exception{ "Number of weights (" + std::to_string(alpha.size()) + ") must match the number of data points (" +
                             std::to_string(this->num_data_points_) + ")!" };
        this->alpha_ptr_ = std::make_shared<const std::vector<T>>(std::move(alpha));
        this->bias_ = -rho;
        this->w_.clear();
    }
    // decision values bias + sum_i alpha_i k(sv_i, z) of the points held by `points` (dense or CSR)
    std::vector<T> predict(const parameter<T> &points) {
        need_model();
        const size_t len = (std::size_t) std::max<int64_t>(points.num_data_points, 1);
        std::vector<T> out(len);
        auto sc = scratch(len);
        const T *alpha = this->alpha_ptr_->data();
        on_all([&](int r, plssvm_mi_ctx *c) {
            T *o = r == 0 ? out.data() : sc[(size_t) r].data();
            if (points.sparse)
                return plssvm_mi_predict_csr(c, alpha, (double) this->bias_, points.rowptr.data(), points.col.data(),
                                             points.val.data(), PLSSVM_MI_VAL_REAL, points.num_data_points,
                                             points.num_features, o);
            return plssvm_mi_predict_dense(c, alpha, (double) this->bias_, points.dense.data(), points.num_data_points,
                                           points.num_features, o);
        });
        out.resize((std::size_t) points.num_data_points);
        return out;
    }
    // csvm::predict_label: sign of the decision values (operators.hpp:174-177)
    std::vector<T> predict_label(const parameter<T> &points) {
        std::vector<T> v = predict(points);
        for (T &x : v) x = x > T(0) ? T(1) : T(-1);
        return v;
    }
    // csvm::accuracy(points, correct_labels)
    T accuracy(const parameter<T> &points) {
        if (points.labels.empty()) throw exception{ "No labels given for the accuracy calculation!" };
        const std::vector<T> l = predict_label(points);
        if (l.size() != points.labels.size())
            throw exception{ "Number of data points to predict and correct labels mismatch!" };
        std::size_t ok = 0;
        for (std::size_t i = 0; i < l.size(); ++i) ok += l[i] * points.labels[i] > T(0);
        return (T) ok / (T) l.size();
    }

    const std::vector<T> &alpha() const { return *this->alpha_ptr_; }
    const std::vector<T> &w() const { return this->w_; }
    T bias() const { return this->bias_; }
    T rho() const { return -this->bias_; }
    T QA_cost() const { return this->QA_cost_; }
    int64_t iterations() const { return iterations_; }
    const std::vector<double> &residual_trace() const { return trace_; }

    static std::string shortest(T v) {  // fmt "{}" of a floating point value: shortest round-trip form
        char buf[64];
        const auto r = std::to_chars(buf, buf + sizeof buf, v);
        return std::string(buf, r.ptr);
    }

  private:
    struct progress_state {
        int64_t imax;
        double target, ms_total;
        int64_t printed;
    };
    static void print_progress(int64_t first, int64_t count, const double *deltas, double target, double batch_ms, void *user) {
        auto &ps = *static_cast<progress_state *>(user);
        ps.target = target;
        const double per = batch_ms / (double) count;
        for (int64_t k = 0; k < count; ++k) {
            std::printf("Start Iteration %lld (max: %lld) with current residuum %s (target: %s). Done in %lldms.\n",
                        (long long) (first + k + 1), (long long) ps.imax, shortest((T) deltas[k]).c_str(),
                        shortest((T) target).c_str(), (long long) per);
        }
        ps.ms_total += (double) (long long) per * (double) count;
        ps.printed += count;
        std::fflush(stdout);
    }
    void need_model() {
        if (this->alpha_ptr_ == nullptr) throw exception{ "No alphas provided for prediction!" };
        if (!on_device_) setup_data_on_device();
    }
    // f(rank, ctx) -> PLSSVM_MI_* code on every rank at once; the first failing rank's message is thrown
    template <typename F>
    void on_all(F &&f) {
        try {
            grp_->run([&](int r, plssvm_mi_ctx *&c) { return f(r, c); });
        } catch (const group_error &e) {
            throw backend_exception(e.code, e.what());
        }
    }
    // host output buffers of the ranks other than 0 (their results equal rank 0's)
    std::vector<std::vector<T>> scratch(size_t len) const {
        std::vector<std::vector<T>> v((size_t) grp_->size());
        for (size_t r = 1; r < v.size(); ++r) v[r].assign(len, T(0));
        return v;
    }
    std::unique_ptr<device_group> grp_;
    std::vector<double> trace_;
    int64_t iterations_ = 0;
    bool on_device_ = false;
};

}  // namespace plssvm::mi355x
