// csvm_interface<T>::learn() calls the backend's hot-path virtuals once each, in the reference's order
// (tests/csvm_test.cpp:215-231: EXPECT_CALL(setup_data_on_device / generate_q / solver_CG).Times(1)),
// with imax = num_features, b = y[0..m) - y[m] and eps = epsilon; the constructor and learn() fail with
// the reference's messages. A recording mock stands in for GMock (tests/mock_csvm.hpp:28-69).
// usage: learn_call_order <5x4.libsvm>     exit 0 = pass, 1 = fail (the reason on stderr)
#include <cstdio>
#include <string>
#include <vector>

#include "csvm_interface.hpp"

using namespace plssvm::mi355x;

template <typename T>
struct mock_csvm : csvm_interface<T> {
    using csvm_interface<T>::csvm_interface;
    std::vector<std::string> calls;
    std::size_t imax_seen = 0;
    T eps_seen = 0;
    std::vector<T> b_seen;
    void setup_data_on_device() override { calls.push_back("setup_data_on_device"); }
    std::vector<T> generate_q() override {
        calls.push_back("generate_q");
        return std::vector<T>(this->num_data_points_ - 1, T(0.5));
    }
    std::vector<T> solver_CG(const std::vector<T> &b, std::size_t imax, T eps, const std::vector<T> &q) override {
        calls.push_back("solver_CG");
        imax_seen = imax;
        eps_seen = eps;
        b_seen = b;
        return std::vector<T>(q.size(), T(1));
    }
    void update_w() override { calls.push_back("update_w"); }
    std::vector<T> predict(const std::vector<std::vector<T>> &p) override {
        calls.push_back("predict");
        return std::vector<T>(p.size(), T(0));
    }
    T bias() const { return this->bias_; }
    const std::vector<T> &alpha() const { return *this->alpha_ptr_; }
};

static int fails = 0;
#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                       \
        }                                                                  \
    } while (0)

template <typename T>
void run(const std::string &path) {
    parameter<T> p;
    p.parse_train_file(path);
    mock_csvm<T> svm{ p };
    svm.learn();
    CHECK((svm.calls == std::vector<std::string>{ "setup_data_on_device", "generate_q", "solver_CG" }));
    CHECK(svm.imax_seen == 4);  // solver_CG(b, num_features_, epsilon_, q)  (csvm.cpp:256)
    CHECK(svm.eps_seen == T(0.001));
    CHECK((svm.b_seen == std::vector<T>{ 2, 2, 0, 0 }));  // y = 1 1 -1 -1 -1: b_i = y_i - y_m
    CHECK(svm.alpha().size() == 5 && svm.alpha().back() == T(-4));  // alpha_m = -sum(alpha)
    // bias = y_m + QA_cost sum(alpha) - q^T alpha with QA_cost = k(x_m, x_m) + 1/C (linear: |x_m|^2 + 1)
    std::vector<T> xm(p.dense.end() - 4, p.dense.end());
    T nm = 0;
    for (T v : xm) nm = std::fma(v, v, nm);
    const T want = T(-1) + (nm + T(1)) * T(4) - T(2);
    CHECK(std::fabs(svm.bias() - want) <= T(1e-5) * std::fabs(want));

    // exceptions (csvm.cpp:42-56, 211-216)
    parameter<T> nolabel = p;
    nolabel.labels.clear();
    mock_csvm<T> s2{ nolabel };
    try {
        s2.learn();
        CHECK(false);
    } catch (const exception &e) {
        CHECK(std::string(e.what()) == "No labels given for training! Maybe the data is only usable for prediction?");
    }
    CHECK(s2.calls.empty());
    parameter<T> empty;
    try {
        mock_csvm<T> s3{ empty };
        CHECK(false);
    } catch (const exception &e) {
        CHECK(std::string(e.what()) == "Data set is empty!");
    }
}

int main(int argc, char **argv) {
    if (argc != 2) return 2;
    run<float>(argv[1]);
    run<double>(argv[1]);
    if (fails == 0) std::printf("ok\n");
    return fails == 0 ? 0 : 1;
}
