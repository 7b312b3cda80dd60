// plssvm-train for the MI355X backend: same flags, defaults and output as the reference executable
// (src/main_train.cpp:27-91, src/plssvm/parameter_train.cpp:38-142), training through
// plssvm::mi355x::csvm<T> (host/csvm.hpp) on libplssvm_mi355x.so.
//
// Additions (not in the reference): --sparse keeps LIBSVM input as CSR (the reference densifies),
// --max_iter overrides the CG limit (default: num_features, csvm.cpp:256), --single trains in fp32
// (the reference selects that at compile time, main_train.cpp:21-25), --device picks the GPU.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "cli.hpp"
#include "csvm.hpp"

namespace {

const char *kHelp =
    "LS-SVM with multiple (GPU-)backends\n"
    "Usage:\n"
    "  plssvm-train [OPTION...] training_set_file [model_file]\n\n"
    "  -t, --kernel_type arg      set type of kernel function.\n"
    "                                  0 -- linear: u'*v\n"
    "                                  1 -- polynomial: (gamma*u'*v + coef0)^degree\n"
    "                                  2 -- radial basis function: exp(-gamma*|u-v|^2) (default: 0)\n"
    "  -d, --degree arg           set degree in kernel function (default: 3)\n"
    "  -g, --gamma arg            set gamma in kernel function (default: 1 / num_features)\n"
    "  -r, --coef0 arg            set coef0 in kernel function (default: 0)\n"
    "  -c, --cost arg             set the parameter C (default: 1)\n"
    "  -e, --epsilon arg          set the tolerance of termination criterion (default: 0.001)\n"
    "  -b, --backend arg          choose the backend: automatic|hip (default: automatic)\n"
    "  -p, --target_platform arg  choose the target platform: automatic|gpu_amd (default: automatic)\n"
    "  -q, --quiet                quiet mode (no outputs)\n"
    "  -h, --help                 print this helper message\n"
    "      --sparse               keep the data as CSR on the device (MI355X backend addition)\n"
    "      --max_iter arg         maximum CG iterations (default: num_features)\n"
    "      --single               train in single precision (float)\n"
    "      --device arg           train on this one HIP device (default: every visible device)\n"
    "      --devices arg          comma-separated device list, one rank per entry (a device listed twice:\n"
    "                             in-process host exchange instead of RCCL)\n";

template <typename T>
int train(const cli &c) {
    using namespace plssvm::mi355x;
    parameter<T> params;
    if (c.opt.count("kernel_type")) params.kernel = parse_kernel(c.opt.at("kernel_type"));
    if (c.opt.count("degree")) params.degree = std::stoi(c.opt.at("degree"));
    if (c.opt.count("gamma")) {
        params.gamma = to_real<T>(c.opt.at("gamma"));
        if (params.gamma == T(0)) {
            std::fprintf(stderr, "gamma = 0.0 is not allowed, it doesnt make any sense!\n");
            std::printf("%s", kHelp);
            return EXIT_FAILURE;
        }
    }
    if (c.opt.count("coef0")) params.coef0 = to_real<T>(c.opt.at("coef0"));
    if (c.opt.count("cost")) params.cost = to_real<T>(c.opt.at("cost"));
    if (c.opt.count("epsilon")) params.epsilon = to_real<T>(c.opt.at("epsilon"));
    const std::string backend = c.opt.count("backend") ? c.opt.at("backend") : "automatic";
    if (backend != "automatic" && backend != "hip" && backend != "mi355x")
        throw std::invalid_argument("Unavailable backend: '" + backend + "' (this build provides hip = MI355X)");
    const std::string target = c.opt.count("target_platform") ? c.opt.at("target_platform") : "automatic";
    if (target != "automatic" && target != "gpu_amd")
        throw std::invalid_argument("Invalid target platform '" + target + "' for the HIP backend!");
    params.print_info = !c.opt.count("quiet");
    if (c.pos.empty()) {
        std::fprintf(stderr, "Error missing input file!");
        std::printf("%s", kHelp);
        return EXIT_FAILURE;
    }
    params.input_filename = c.pos[0];
    if (c.pos.size() > 1) params.model_filename = c.pos[1];
    const auto t0 = std::chrono::steady_clock::now();
    params.parse_train_file(c.pos[0], c.opt.count("sparse") > 0);
    if (c.pos.size() > 1) params.model_filename = c.pos[1];
    if (params.print_info) {
        std::printf("Read %lld data points with %lld features in %lldms using the libsvm parser from file '%s'.\n\n",
                    (long long) params.num_data_points, (long long) params.num_features,
                    (long long) std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count(),
                    params.input_filename.c_str());
        std::printf("task: training\nkernel type: %s -> ", kernel_name(params.kernel));
        switch (params.kernel) {
            case kernel_type::linear: std::printf("u'*v\n"); break;
            case kernel_type::polynomial:
                std::printf("(gamma*u'*v + coef0)^degree\ngamma: %s\ncoef0: %s\ndegree: %d\n",
                            csvm<T>::shortest(params.gamma).c_str(), csvm<T>::shortest(params.coef0).c_str(), params.degree);
                break;
            default: std::printf("exp(-gamma*|u-v|^2)\ngamma: %s\n", csvm<T>::shortest(params.gamma).c_str()); break;
        }
        std::printf("cost: %s\nepsilon: %s\ninput file (data set): '%s'\noutput file (model): '%s'\n\n",
                    csvm<T>::shortest(params.cost).c_str(), csvm<T>::shortest(params.epsilon).c_str(),
                    params.input_filename.c_str(), params.model_filename.c_str());
        std::printf("Using HIP (MI355X, gfx950) as backend.\n");
    }
    // hip::csvm<T>(params) takes every visible device (csvm.hip.cpp:53-55): here one rank of a row-block group per
    // device; --device keeps one, --devices lists them
    std::vector<int> devs;
    if (c.opt.count("devices")) {
        const std::string &l = c.opt.at("devices");
        for (size_t a = 0; a <= l.size();) {
            const size_t b = std::min(l.find(',', a), l.size());
            devs.push_back(std::stoi(l.substr(a, b - a)));
            a = b + 1;
        }
    } else if (c.opt.count("device")) {
        devs.push_back(std::stoi(c.opt.at("device")));
    } else {
        devs = csvm<T>::all_devices(params);
    }
    csvm<T> svm(params, devs);
    if (params.print_info) {
        std::printf("Found %d HIP device(s):\n", svm.num_devices());
        for (const int d : svm.devices()) std::printf("  [%d, gfx950]\n", d);
        std::printf("\n");
    }
    // learn() prints the reference's setup line, one line per CG iteration and the solve summary
    // (csvm.cpp:226-266, OpenMP/csvm.cpp:115-117,161-166)
    if (c.opt.count("max_iter")) svm.learn((std::size_t) std::stoll(c.opt.at("max_iter")));
    else svm.learn();
    svm.write_model(params.model_filename);
    if (params.print_info) std::printf("Wrote model file ('%s').\n", params.model_filename.c_str());
    return EXIT_SUCCESS;
}

}  // namespace

int main(int argc, char **argv) {
    try {
        const cli c = parse_cli(argc, argv, { { "t", "kernel_type" }, { "d", "degree" }, { "g", "gamma" }, { "r", "coef0" },
                                              { "c", "cost" }, { "e", "epsilon" }, { "b", "backend" },
                                              { "p", "target_platform" }, { "q", "quiet" }, { "h", "help" } },
                                { "quiet", "help", "sparse", "single" });
        if (c.opt.count("help")) {
            std::printf("%s", kHelp);
            return EXIT_SUCCESS;
        }
        return c.opt.count("single") ? train<float>(c) : train<double>(c);
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return EXIT_FAILURE;
    }
}
