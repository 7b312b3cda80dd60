// plssvm::mi355x::csvm<T> — the reference's plssvm::csvm<T> / hip::csvm<T> surface over the C ABI
// (include/plssvm_mi355x.h). Host-only C++17; all compute runs in libplssvm_mi355x.so on the GPU.
//
// Mirrors include/plssvm/csvm.hpp:33-278 for the training path: the constructor validates the data
// like csvm.cpp:43-53, learn() is csvm.cpp:207-267 calling setup_data_on_device / generate_q /
// solver_CG (the hooks mock_hip_csvm exposes, tests/backends/HIP/mock_hip_csvm.hpp:24-51, are public
// here too), write_model() writes the LIBSVM model format of csvm.cpp:60-204.
#pragma once

#include <charconv>
#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/plssvm_mi355x.h"
#include "parameter.hpp"

namespace plssvm::mi355x {

struct backend_exception : std::runtime_error {  // plssvm::hip::backend_exception
    int code;
    backend_exception(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

template <typename T>
class csvm {
  public:
    using real_type = T;

    explicit csvm(const parameter<T> &params, int device = 0) : params_(params) {
        if (params.num_data_points == 0) throw std::invalid_argument("Data set is empty!");
        if (params.num_features == 0) throw std::invalid_argument("No features provided for the data points!");
        const int rc = plssvm_mi_create((int) sizeof(T), (int) params.kernel, params.degree, (double) params.gamma,
                                        (double) params.coef0, (double) params.cost, device, &ctx_);
        if (rc != PLSSVM_MI_OK) throw backend_exception(rc, plssvm_mi_last_error(nullptr));
    }
    ~csvm() { plssvm_mi_destroy(ctx_); }
    csvm(const csvm &) = delete;
    csvm &operator=(const csvm &) = delete;

    // one process per GPU: join a row-block group before setup (rank 0 creates the id)
    void join_group(int rank, int world, const void *unique_id) { check(plssvm_mi_comm_init(ctx_, rank, world, unique_id)); }

    // ---- gpu_csvm hot-path surface ----
    void setup_data_on_device() {
        const auto &p = params_;
        if (p.sparse) {
            const bool f22 = !p.val22.empty() && sizeof(T) == 4;  // packed FP22 input stays packed
            check(plssvm_mi_setup_csr(ctx_, p.rowptr.data(), p.col.data(), f22 ? (const void *) p.val22.data() : p.val.data(),
                                      f22 ? PLSSVM_MI_VAL_FP22 : PLSSVM_MI_VAL_REAL, p.num_data_points, p.num_features));
        } else {
            check(plssvm_mi_setup_dense(ctx_, p.dense.data(), p.num_data_points, p.num_features));
        }
    }
    std::vector<T> generate_q() {
        std::vector<T> q((std::size_t) std::max<int64_t>(params_.num_data_points - 1, 1));
        double qa = 0;
        check(plssvm_mi_generate_q(ctx_, q.data(), &qa));
        QA_cost_ = (T) qa;
        q.resize((std::size_t) (params_.num_data_points - 1));
        return q;
    }
    std::vector<T> solver_CG(const std::vector<T> &b, std::size_t imax, T eps, const std::vector<T> &q) {
        std::vector<T> x(std::max<std::size_t>(b.size(), 1));
        trace_.assign(imax + 1, 0.0);
        int64_t it = 0;
        check(plssvm_mi_solve_cg(ctx_, b.data(), q.data(), (int64_t) imax, (double) eps, x.data(), trace_.data(), &it));
        iterations_ = it;
        trace_.resize((std::size_t) it + 1);
        x.resize(b.size());
        return x;
    }
    void run_device_kernel(const std::vector<T> &q, std::vector<T> &ret, const std::vector<T> &d, T add) {
        check(plssvm_mi_kp(ctx_, q.data(), d.data(), ret.data(), (double) add));
    }
    void set_cost(T c) { check(plssvm_mi_set_cost(ctx_, (double) c)); }
    void set_QA_cost(T qa) {
        check(plssvm_mi_set_qa_cost(ctx_, (double) qa));
        QA_cost_ = qa;
    }

    // csvm<T>::learn (src/plssvm/csvm.cpp:207-267); imax < 0 = num_features (csvm.cpp:256)
    void learn(int64_t imax = -1) {
        const auto &y = params_.labels;
        if (y.empty()) throw std::invalid_argument("No labels given for training! Maybe the data is only usable for prediction?");
        if ((int64_t) y.size() != params_.num_data_points)
            throw std::invalid_argument("Number of labels must match the number of data points!");
        setup_data_on_device();
        on_device_ = true;
        const std::vector<T> q = generate_q();
        const std::size_t m = (std::size_t) params_.num_data_points - 1;
        std::vector<T> b(y.begin(), y.begin() + (std::ptrdiff_t) m);
        for (T &v : b) v -= y.back();
        std::vector<T> alpha = solver_CG(b, (std::size_t) (imax < 0 ? params_.num_features : imax), params_.epsilon, q);
        T s = 0, qa = 0;
        for (std::size_t i = 0; i < m; ++i) s += alpha[i];
        for (std::size_t i = 0; i < m; ++i) qa = std::fma(q[i], alpha[i], qa);
        bias_ = y.back() + QA_cost_ * s - qa;
        alpha.push_back(-s);
        alpha_ = std::move(alpha);
    }

    // csvm<T>::write_model (src/plssvm/csvm.cpp:60-204): positive-label support vectors first
    void write_model(const std::string &filename) const {
        if (alpha_.empty()) throw std::invalid_argument("No alphas given! Maybe a call to 'learn()' is missing?");
        const auto &p = params_;
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
        if ((int64_t) alpha.size() != params_.num_data_points)
            throw std::invalid_argument("Number of alphas must match the number of support vectors!");
        alpha_ = std::move(alpha);
        bias_ = -rho;
        on_device_ = false;
    }
    std::vector<T> update_w() {
        need_model();
        std::vector<T> w((std::size_t) std::max<int64_t>(params_.num_features, 1));
        check(plssvm_mi_update_w(ctx_, alpha_.data(), w.data()));
        w.resize((std::size_t) params_.num_features);
        return w;
    }
    // decision values bias + sum_i alpha_i k(sv_i, z) of the points held by `points`
    std::vector<T> predict(const parameter<T> &points) {
        need_model();
        std::vector<T> out((std::size_t) std::max<int64_t>(points.num_data_points, 1));
        if (points.sparse)
            check(plssvm_mi_predict_csr(ctx_, alpha_.data(), (double) bias_, points.rowptr.data(), points.col.data(),
                                        points.val.data(), PLSSVM_MI_VAL_REAL, points.num_data_points,
                                        points.num_features, out.data()));
        else
            check(plssvm_mi_predict_dense(ctx_, alpha_.data(), (double) bias_, points.dense.data(), points.num_data_points,
                                          points.num_features, out.data()));
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
        if (points.labels.empty()) throw std::invalid_argument("No labels given for the accuracy calculation!");
        const std::vector<T> l = predict_label(points);
        if (l.size() != points.labels.size())
            throw std::invalid_argument("Number of data points to predict and correct labels mismatch!");
        std::size_t ok = 0;
        for (std::size_t i = 0; i < l.size(); ++i) ok += l[i] * points.labels[i] > T(0);
        return (T) ok / (T) l.size();
    }

    const std::vector<T> &alpha() const { return alpha_; }
    T bias() const { return bias_; }
    T rho() const { return -bias_; }
    T QA_cost() const { return QA_cost_; }
    int64_t iterations() const { return iterations_; }
    const std::vector<double> &residual_trace() const { return trace_; }

    static std::string shortest(T v) {  // fmt "{}" of a floating point value: shortest round-trip form
        char buf[64];
        const auto r = std::to_chars(buf, buf + sizeof buf, v);
        return std::string(buf, r.ptr);
    }

  private:
    void need_model() {
        if (alpha_.empty()) throw std::invalid_argument("No alphas provided for prediction!");
        if (!on_device_) {
            setup_data_on_device();
            on_device_ = true;
        }
    }
    void check(int rc) const {
        if (rc != PLSSVM_MI_OK) throw backend_exception(rc, plssvm_mi_last_error(ctx_));
    }
    parameter<T> params_;
    plssvm_mi_ctx *ctx_ = nullptr;
    T QA_cost_ = 0, bias_ = 0;
    std::vector<T> alpha_;
    std::vector<double> trace_;
    int64_t iterations_ = 0;
    bool on_device_ = false;
};

}  // namespace plssvm::mi355x
