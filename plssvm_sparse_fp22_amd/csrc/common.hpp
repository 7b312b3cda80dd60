// Shared device/host helpers for the MI355X PLSSVM backend (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <exception>
#include <thread>
#include <vector>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace plssvm_mi {

// Error carrier turned into a PLSSVM_MI_ERR_* code at the C ABI (the reference throws
// plssvm::hip::backend_exception from PLSSVM_HIP_ERROR_CHECK, src/plssvm/backends/HIP/detail/utility.hip.cpp:19-23).
struct mi_error : std::runtime_error {
    int code;
    mi_error(int c, const std::string &msg) : std::runtime_error(msg), code(c) {}
};

// the PLSSVM_MI_ERR_* code of any exception a setup step may raise (mi_error: its code; host or device
// allocation: ERR_OOM; anything else, e.g. std::length_error from a host table: ERR_ARG — the C ABI's mapping)
inline int exception_code(const std::exception &e) {
    if (const auto *m = dynamic_cast<const mi_error *>(&e)) return m->code;
    if (dynamic_cast<const std::bad_alloc *>(&e) != nullptr) return -4;
    return -1;
}

#define MI_HIP_CHECK(expr)                                                                                        \
    do {                                                                                                          \
        hipError_t e_ = (expr);                                                                                   \
        if (e_ != hipSuccess) {                                                                                   \
            throw ::plssvm_mi::mi_error(e_ == hipErrorOutOfMemory ? -4 : -2,                                      \
                                        std::string("HIP error '") + hipGetErrorString(e_) + "' at " __FILE__ ":" + \
                                            std::to_string(__LINE__) + " (" #expr ")");                           \
        }                                                                                                         \
    } while (0)

#define MI_LAUNCH_CHECK() MI_HIP_CHECK(hipGetLastError())

// setup phase timer: PLSSVM_MI_TIMING=1 prints "[plssvm_mi] <phase> <seconds>" to stderr (measurements)
struct phase_timer {
    bool on;
    std::chrono::steady_clock::time_point t;
    phase_timer() : on(std::getenv("PLSSVM_MI_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
    void mark(const char *what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[plssvm_mi] %s %.3f\n", what, std::chrono::duration<double>(now - t).count());
        t = now;
    }
};

// host worker threads for setup-time loops: OMP_NUM_THREADS when set (the GPU box sets it to its CPU
// share), else the hardware threads, at most 64
inline int host_threads() {
    static const int n = [] {
        int v = 0;
        if (const char *e = std::getenv("OMP_NUM_THREADS")) v = std::atoi(e);
        if (v <= 0) v = (int) std::thread::hardware_concurrency();
        return v < 1 ? 1 : (v > 64 ? 64 : v);
    }();
    return n;
}

// f(t, begin, end) on host_threads() threads over contiguous parts of [0, n) (part t = [t n / T, (t+1) n / T)),
// joined before returning; the first exception is rethrown
template <typename F>
void host_parallel(int64_t n, F f, int nthreads = 0) {
    const int T = (int) std::max<int64_t>(1, std::min<int64_t>(nthreads > 0 ? nthreads : host_threads(), std::max<int64_t>(n, 1)));
    if (T == 1) {
        f(0, (int64_t) 0, n);
        return;
    }
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err((size_t) T);
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            try {
                f(t, n * t / T, n * (t + 1) / T);
            } catch (...) {
                err[(size_t) t] = std::current_exception();
            }
        });
    for (auto &x : th) x.join();
    for (auto &e : err)
        if (e) std::rethrow_exception(e);
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// ---- MFMA tile traits ---------------------------------------------------------------------------
// 16x16 output tiles, K = 4 per instruction. A operand: lane l holds A[i = l&15][k = l>>4];
// B operand: lane l holds B[k = l>>4][j = l&15]. C/D maps differ between f32 and f64
// (cdna_hip_programming.md §3 "Fragment layout"): f32 row = (l>>4)*4 + r, f64 row = (l>>4) + 4*r,
// col = l&15 for both. Both layouts are checked on the GPU by tests/test_gpu_parity.py.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct mfma16;

template <>
struct mfma16<float> {
    using acc_t = f32x4;
    __device__ static __forceinline__ acc_t op(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static __forceinline__ int row(int lane, int r) { return ((lane >> 4) << 2) + r; }
};

template <>
struct mfma16<double> {
    using acc_t = f64x4;
    __device__ static __forceinline__ acc_t op(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    __device__ static __forceinline__ int row(int lane, int r) { return (lane >> 4) + (r << 2); }
};

// XCD-aware bijective remap of a 1-D grid: blocks are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md §Workgroup dispatch), so give every XCD one contiguous range of work
// items, keeping tiles that share an operand panel in one L2. Speed only, never correctness.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nblocks) {
    const int64_t q = nblocks >> 3, r = nblocks & 7, xcd = b & 7, pos = b >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

// lower-triangle tile index t -> (I, J), I >= J, t = I(I+1)/2 + J
__device__ __host__ __forceinline__ void tri_tile(int64_t t, int64_t &I, int64_t &J) {
    int64_t i = (int64_t) ((sqrt(8.0 * (double) t + 1.0) - 1.0) * 0.5);
    while (i * (i + 1) / 2 > t) --i;
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    I = i;
    J = t - i * (i + 1) / 2;
}

__device__ __host__ __forceinline__ int64_t tri_index(int64_t I, int64_t J) { return I * (I + 1) / 2 + J; }

}  // namespace plssvm_mi
