// plssvm-predict for the MI355X backend: same usage, output file and accuracy line as the reference
// executable (src/main_predict.cpp:27-115, src/plssvm/parameter_predict.cpp:38-116), predicting through
// plssvm::mi355x::csvm<T> (host/csvm.hpp) on libplssvm_mi355x.so.
//
// Additions (not in the reference): --sparse keeps model and test data as CSR (the reference
// densifies), --single predicts in fp32, --device picks the GPU.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "cli.hpp"
#include "csvm.hpp"

namespace {

const char *kHelp =
    "LS-SVM with multiple (GPU-)backends\n"
    "Usage:\n"
    "  plssvm-predict [OPTION...] test_file model_file [output_file]\n\n"
    "  -b, --backend arg          choose the backend: automatic|hip (default: automatic)\n"
    "  -p, --target_platform arg  choose the target platform: automatic|gpu_amd (default: automatic)\n"
    "  -q, --quiet                quiet mode (no outputs)\n"
    "  -h, --help                 print this helper message\n"
    "      --sparse               keep the data as CSR on the device (MI355X backend addition)\n"
    "      --single               predict in single precision (float)\n"
    "      --device arg           HIP device ordinal (default: 0)\n";

template <typename T>
int predict(const cli &c) {
    using namespace plssvm::mi355x;
    const std::string backend = c.opt.count("backend") ? c.opt.at("backend") : "automatic";
    if (backend != "automatic" && backend != "hip" && backend != "mi355x")
        throw std::invalid_argument("Unavailable backend: '" + backend + "' (this build provides hip = MI355X)");
    const std::string target = c.opt.count("target_platform") ? c.opt.at("target_platform") : "automatic";
    if (target != "automatic" && target != "gpu_amd")
        throw std::invalid_argument("Invalid target platform '" + target + "' for the HIP backend!");
    const bool print_info = !c.opt.count("quiet");
    if (c.pos.empty()) {
        std::fprintf(stderr, "Error missing test file!");
        std::printf("%s", kHelp);
        return EXIT_FAILURE;
    }
    if (c.pos.size() < 2) {
        std::fprintf(stderr, "Error missing model file!");
        std::printf("%s", kHelp);
        return EXIT_FAILURE;
    }
    const bool sparse = c.opt.count("sparse") > 0;
    parameter<T> model, test;
    model.input_filename = c.pos[0];
    const std::string predict_filename = c.pos.size() > 2 ? c.pos[2] : model.predict_name_from_input();
    test.parse_test_file(c.pos[0], sparse);
    model.parse_model_file(c.pos[1], sparse, test.num_features);
    if (test.num_features < model.num_features) test.parse_test_file(c.pos[0], sparse, model.num_features);
    if (print_info) {
        std::printf("\ntask: prediction\nkernel type: %s -> ", kernel_name(model.kernel));
        switch (model.kernel) {
            case kernel_type::linear: std::printf("u'*v\n"); break;
            case kernel_type::polynomial:
                std::printf("(gamma*u'*v + coef0)^degree\ngamma: %s\ncoef0: %s\ndegree: %d\n",
                            csvm<T>::shortest(model.gamma).c_str(), csvm<T>::shortest(model.coef0).c_str(), model.degree);
                break;
            default: std::printf("exp(-gamma*|u-v|^2)\ngamma: %s\n", csvm<T>::shortest(model.gamma).c_str()); break;
        }
        std::printf("rho: %s\ninput file (data set): '%s'\ninput file (model): '%s'\noutput file (prediction): '%s'\n\n",
                    csvm<T>::shortest(model.rho).c_str(), c.pos[0].c_str(), c.pos[1].c_str(), predict_filename.c_str());
    }
    const int device = c.opt.count("device") ? std::stoi(c.opt.at("device")) : 0;
    csvm<T> svm(model, device);
    svm.set_model(model.alpha, model.rho);
    const std::vector<T> labels = svm.predict_label(test);

    const auto t0 = std::chrono::steady_clock::now();
    {
        std::FILE *fp = std::fopen(predict_filename.c_str(), "w");
        if (!fp) throw std::runtime_error("Can't open prediction file '" + predict_filename + "'!");
        for (std::size_t i = 0; i < labels.size(); ++i)  // fmt::join(labels, "\n"): no trailing newline
            std::fprintf(fp, i + 1 < labels.size() ? "%s\n" : "%s", csvm<T>::shortest(labels[i]).c_str());
        std::fclose(fp);
    }
    if (print_info)
        std::printf("Wrote prediction file ('%s') with %zu labels in %lldms.\n", predict_filename.c_str(), labels.size(),
                    (long long) std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count());
    if (!test.labels.empty()) {
        std::size_t correct = 0;
        for (std::size_t i = 0; i < labels.size(); ++i) correct += test.labels[i] * labels[i] > T(0);
        std::printf("Accuracy = %s%% (%zu/%zu) (classification)\n",
                    csvm<T>::shortest((T) correct / (T) labels.size() * T(100)).c_str(), correct, labels.size());
    }
    return EXIT_SUCCESS;
}

}  // namespace

int main(int argc, char **argv) {
    try {
        const cli c = parse_cli(argc, argv, { { "b", "backend" }, { "p", "target_platform" }, { "q", "quiet" }, { "h", "help" } },
                                { "quiet", "help", "sparse", "single" });
        if (c.opt.count("help")) {
            std::printf("%s", kHelp);
            return EXIT_SUCCESS;
        }
        return c.opt.count("single") ? predict<float>(c) : predict<double>(c);
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return EXIT_FAILURE;
    }
}
