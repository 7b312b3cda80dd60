// Test driver for the C++ host readers (plssvm_sparse_fp22_amd/host/parameter.hpp): parses one file
// and prints what it read, or the exception's type and message (tests/test_parsers.py).
//   parse_driver libsvm|model float|double <path>
// output: "OK <n> <d> <has_labels>" then one line per point "[label|alpha] v0 v1 ... v(d-1)" (%.17g),
//         model files add "RHO <rho>", "KERNEL <k> <degree> <gamma> <coef0>", "NRSV <a> <b>";
//         or "ERROR <invalid_file_format|file_not_found|other>: <message>"
#include <cstdio>
#include <string>

#include "parameter.hpp"

template <typename T>
int run(const std::string &kind, const std::string &path) {
    using namespace plssvm::mi355x;
    parameter<T> p;
    try {
        if (kind == "libsvm") p.parse_train_file(path);
        else p.parse_model_file(path);
    } catch (const invalid_file_format_exception &e) {
        std::printf("ERROR invalid_file_format: %s\n", e.what());
        return 0;
    } catch (const file_not_found_exception &e) {
        std::printf("ERROR file_not_found: %s\n", e.what());
        return 0;
    } catch (const std::exception &e) {
        std::printf("ERROR other: %s\n", e.what());
        return 0;
    }
    const bool model = kind == "model";
    const bool has = model || !p.labels.empty();
    std::printf("OK %lld %lld %d\n", (long long) p.num_data_points, (long long) p.num_features, has ? 1 : 0);
    for (int64_t i = 0; i < p.num_data_points; ++i) {
        if (model) std::printf("%.17g", (double) p.alpha[(std::size_t) i]);
        else if (has) std::printf("%.17g", (double) p.labels[(std::size_t) i]);
        for (int64_t f = 0; f < p.num_features; ++f) std::printf(" %.17g", (double) p.value(i, f));
        std::printf("\n");
    }
    if (model) {
        std::printf("RHO %.17g\n", (double) p.rho);
        std::printf("KERNEL %s %d %.17g %.17g\n", kernel_name(p.kernel), p.degree, (double) p.gamma, (double) p.coef0);
        std::printf("NRSV %lld %lld\n", (long long) p.nr_sv[0], (long long) p.nr_sv[1]);
    } else {
        std::printf("GAMMA %.17g\n", (double) p.gamma);
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: parse_driver libsvm|model float|double <path>\n");
        return 2;
    }
    const std::string kind = argv[1], type = argv[2], path = argv[3];
    return type == "float" ? run<float>(kind, path) : run<double>(kind, path);
}
