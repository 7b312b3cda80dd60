// Test driver of the one-process multi-GPU group (include/plssvm_mi355x_group.hpp), run by
// tests/test_gpu_group.py on the GPU box. Two ranks on device 0 over the in-process host exchange (RCCL refuses two
// ranks on one GPU): the group's failure protocol — a rank failing while its peer waits in a collective must end
// every rank's call, with the failing rank's code and message, without a hang; the group refuses further calls and
// is destroyed cleanly. Prints one JSON line.
//
// usage: plssvm-group-check {early|library|none} [devices, default 0,0]
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/plssvm_mi355x_group.hpp"

using plssvm::mi355x::device_group;
using plssvm::mi355x::group_error;

int main(int argc, char **argv) {
    const std::string mode = argc > 1 ? argv[1] : "early";
    std::vector<int> devs{ 0, 0 };
    if (argc > 2) {
        devs.clear();
        const std::string l = argv[2];
        for (size_t a = 0; a <= l.size();) {
            const size_t b = std::min(l.find(',', a), l.size());
            devs.push_back(std::stoi(l.substr(a, b - a)));
            a = b + 1;
        }
    }
    const int64_t n = 600, d = 16, m = n - 1;
    std::vector<double> X((size_t) (n * d)), p((size_t) m), ret0((size_t) m, 0.0);
    for (int64_t i = 0; i < n * d; ++i) X[(size_t) i] = std::sin(0.37 * (double) i) + 0.1 * (double) (i % 7);
    for (int64_t i = 0; i < m; ++i) p[(size_t) i] = 1.0 + 0.5 * std::cos(0.11 * (double) i);
    const auto t0 = std::chrono::steady_clock::now();
    int world = 0, host = 0, fail_rank = -1, fail_code = 0, refused = 0;
    std::vector<int> rcs(devs.size(), 0);
    std::string msg;
    try {
        device_group g(devs, 8, PLSSVM_MI_KERNEL_RBF, 3, 1.0 / (double) d, 0.0, 1.0);
        world = g.size();
        host = g.host_exchange() ? 1 : 0;
        g.run([&](int, plssvm_mi_ctx *&c) {
            int rc = plssvm_mi_setup_dense(c, X.data(), n, d);
            if (rc == PLSSVM_MI_OK) rc = plssvm_mi_generate_q(c, nullptr, nullptr);
            return rc;
        });
        std::vector<std::vector<double>> rets(devs.size(), ret0);
        try {
            g.run([&](int r, plssvm_mi_ctx *&c) {
                int rc;
                if (r == 1 && mode == "early") {
                    rc = PLSSVM_MI_ERR_STATE;  // fails before its collective (its peer waits in the exchange)
                } else if (r == 1 && mode == "library") {
                    rc = plssvm_mi_kp_part(c, p.data(), rets[(size_t) r].data(), 7);  // "unknown K·p part"
                } else {
                    rc = plssvm_mi_kp(c, nullptr, p.data(), rets[(size_t) r].data(), 1.0);  // all-reduce of the tiles
                }
                rcs[(size_t) r] = rc;
                return rc;
            });
        } catch (const group_error &e) {
            fail_rank = e.rank;
            fail_code = e.code;
            msg = e.what();
            try {
                g.run([](int, plssvm_mi_ctx *&) { return PLSSVM_MI_OK; });
            } catch (const group_error &e2) {
                refused = e2.code == PLSSVM_MI_ERR_STATE ? 1 : 0;
            }
        }
        if (mode == "none") {  // both ranks' K·p must be the same bits
            bool same = true;
            for (size_t r = 1; r < rets.size(); ++r) same = same && std::memcmp(rets[r].data(), rets[0].data(), sizeof(double) * (size_t) m) == 0;
            msg = same ? "equal" : "differ";
            double s = 0;
            for (double v : rets[0]) s += v;
            std::printf("{\"mode\": \"%s\", \"world\": %d, \"host\": %d, \"ranks\": \"%s\", \"sum\": %.17g, \"rc0\": %d, \"rc1\": %d}\n",
                        mode.c_str(), world, host, msg.c_str(), s, rcs[0], rcs.size() > 1 ? rcs[1] : 0);
            return 0;
        }
    } catch (const group_error &e) {
        std::printf("{\"mode\": \"%s\", \"setup_error\": \"%s\", \"code\": %d}\n", mode.c_str(), e.what(), e.code);
        return 2;
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::string esc;
    for (char ch : msg) esc += (ch == '"' || ch == '\\') ? '\'' : ch;
    std::printf("{\"mode\": \"%s\", \"world\": %d, \"host\": %d, \"fail_rank\": %d, \"fail_code\": %d, \"msg\": \"%s\", "
                "\"rc0\": %d, \"rc1\": %d, \"refused\": %d, \"seconds\": %.3f}\n",
                mode.c_str(), world, host, fail_rank, fail_code, esc.c_str(), rcs[0], rcs.size() > 1 ? rcs[1] : 0, refused,
                secs);
    return 0;
}
