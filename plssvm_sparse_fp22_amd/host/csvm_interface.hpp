// plssvm::mi355x::csvm_interface<T> — the reference's abstract C-SVM surface, restated (host only, C++17).
//
// Same protected pure virtuals with the same signatures as plssvm::csvm<T> (include/plssvm/csvm.hpp:188-214):
//   setup_data_on_device(), generate_q(), solver_CG(b, imax, eps, q), update_w(), predict(points),
// the same protected state a backend reads (csvm.hpp:242-277: kernel_, degree_, gamma_, coef0_, cost_,
// epsilon_, print_info_, data_ptr_, value_ptr_, alpha_ptr_, num_data_points_, num_features_, bias_,
// QA_cost_, w_), the constructor checks of csvm.cpp:42-56 and learn() of csvm.cpp:207-267, which calls
// the three hot-path virtuals in the reference's order. A backend written against the reference's
// base compiles against this one unchanged (tests/test_boundary.py), and the
// MI355X adapter (csvm.hpp) derives from it.
//
// Build-defined difference: a parameter set holding CSR data (parameter<T>::sparse) is never densified;
// data_ptr_ is then null and the backend reads the CSR arrays from params_ (the reference has no sparse
// path, its parser densifies).
#pragma once

#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "parameter.hpp"

namespace plssvm::mi355x {

// plssvm::exception (include/plssvm/exceptions/exceptions.hpp)
struct exception : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <typename T>
class csvm_interface {
    static_assert(std::is_same_v<T, float> || std::is_same_v<T, double>, "The template type can only be 'float' or 'double'!");

  public:
    using real_type = T;

    explicit csvm_interface(const parameter<T> &params) :
        kernel_{ params.kernel }, degree_{ params.degree }, gamma_{ params.gamma }, coef0_{ params.coef0 },
        cost_{ params.cost }, epsilon_{ params.epsilon }, print_info_{ params.print_info }, params_{ params } {
        if (params.num_data_points == 0) throw exception{ "Data set is empty!" };
        if (params.num_features == 0) throw exception{ "No features provided for the data points!" };
        if (!params.sparse) {  // the reference's shared AoS rows
            auto rows = std::make_shared<std::vector<std::vector<T>>>((std::size_t) params.num_data_points);
            for (int64_t i = 0; i < params.num_data_points; ++i)
                (*rows)[(std::size_t) i].assign(params.dense.begin() + i * params.num_features,
                                                params.dense.begin() + (i + 1) * params.num_features);
            data_ptr_ = std::move(rows);
        }
        if (!params.labels.empty()) value_ptr_ = std::make_shared<const std::vector<T>>(params.labels);
        num_data_points_ = (std::size_t) params.num_data_points;
        num_features_ = (std::size_t) params.num_features;
    }
    virtual ~csvm_interface() = default;
    csvm_interface(const csvm_interface &) = delete;
    csvm_interface &operator=(const csvm_interface &) = delete;

    // csvm<T>::learn (src/plssvm/csvm.cpp:207-267): setup, q, b = y[0..m) - y[m], QA_cost = k(x_m, x_m) + 1/C,
    // solver_CG with imax = num_features, bias = y[m] + QA_cost sum(alpha) - q^T alpha, alpha[m] = -sum(alpha)
    void learn() { learn(num_features_); }
    // the same with an explicit CG iteration limit (plssvm-train --max_iter; the reference fixes imax = d)
    void learn(std::size_t imax) {
        if (value_ptr_ == nullptr) throw exception{ "No labels given for training! Maybe the data is only usable for prediction?" };
        if (value_ptr_->size() != num_data_points_)
            throw exception{ "Number of labels (" + std::to_string(value_ptr_->size()) +
                             ") must match the number of data points (" + std::to_string(num_data_points_) + ")!" };
        setup_data_on_device();
        auto start = std::chrono::steady_clock::now();
        const std::vector<T> q = generate_q();
        std::vector<T> b(value_ptr_->begin(), value_ptr_->end() - 1);
        for (T &v : b) v -= value_ptr_->back();
        const std::vector<T> last = point(num_data_points_ - 1);
        QA_cost_ = kernel_function(last, last) + T(1) / cost_;
        if (print_info_) {
            std::printf("Setup for solving the optimization problem done in %lldms.\n", (long long) ms_since(start));
            start = std::chrono::steady_clock::now();
        }
        std::vector<T> alpha = solver_CG(b, imax, epsilon_, q);
        T s = 0, qa = 0;
        for (const T a : alpha) s += a;
        for (std::size_t i = 0; i < alpha.size(); ++i) qa = std::fma(q[i], alpha[i], qa);  // transposed{ q } * alpha
        bias_ = value_ptr_->back() + QA_cost_ * s - qa;
        alpha.push_back(-s);
        alpha_ptr_ = std::make_shared<const std::vector<T>>(std::move(alpha));
        w_.clear();
        if (print_info_) {
            std::printf("Solved minimization problem (r = b - Ax) using CG in %lldms.\n", (long long) ms_since(start));
            std::fflush(stdout);
        }
    }

  protected:
    static long long ms_since(std::chrono::steady_clock::time_point t) {
        return (long long) std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t).count();
    }

    // ---- pure virtual, implemented by every backend (include/plssvm/csvm.hpp:188-214) ----
    virtual void setup_data_on_device() = 0;
    [[nodiscard]] virtual std::vector<real_type> generate_q() = 0;
    virtual std::vector<real_type> solver_CG(const std::vector<real_type> &b, std::size_t imax, real_type eps,
                                             const std::vector<real_type> &q) = 0;
    virtual void update_w() = 0;
    [[nodiscard]] virtual std::vector<real_type> predict(const std::vector<std::vector<real_type>> &points) = 0;

    // kernel_function<k> (include/plssvm/kernel_types.hpp:63-85): sequential fma chains
    [[nodiscard]] real_type kernel_function(const std::vector<real_type> &xi, const std::vector<real_type> &xj) const {
        T v = 0;
        if (kernel_ == kernel_type::rbf) {
            for (std::size_t k = 0; k < xi.size(); ++k) {
                const T diff = xi[k] - xj[k];
                v = std::fma(diff, diff, v);
            }
            return std::exp(-gamma_ * v);
        }
        for (std::size_t k = 0; k < xi.size(); ++k) v = std::fma(xi[k], xj[k], v);
        if (kernel_ == kernel_type::linear) return v;
        return std::pow(std::fma(gamma_, v, coef0_), static_cast<T>(degree_));
    }

    // point i as a dense row (from data_ptr_ or, for CSR parameter sets, from the CSR row)
    [[nodiscard]] std::vector<T> point(std::size_t i) const {
        if (data_ptr_) return (*data_ptr_)[i];
        std::vector<T> row(num_features_, T(0));
        for (int64_t k = params_.rowptr[i]; k < params_.rowptr[i + 1]; ++k) row[(std::size_t) params_.col[(std::size_t) k]] = params_.val[(std::size_t) k];
        return row;
    }

    // ---- state read by the backends (include/plssvm/csvm.hpp:242-277) ----
    const kernel_type kernel_;
    const int degree_;
    real_type gamma_;
    const real_type coef0_;
    real_type cost_;
    const real_type epsilon_;
    const bool print_info_;
    std::shared_ptr<const std::vector<std::vector<real_type>>> data_ptr_{};  // null for CSR parameter sets
    std::shared_ptr<const std::vector<real_type>> value_ptr_{};
    std::shared_ptr<const std::vector<real_type>> alpha_ptr_{};
    std::size_t num_data_points_{};
    std::size_t num_features_{};
    real_type bias_{};
    real_type QA_cost_{};
    std::vector<real_type> w_{};
    parameter<T> params_;  // the parameter set itself (CSR arrays of sparse sets)
};

}  // namespace plssvm::mi355x
