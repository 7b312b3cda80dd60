// Development microbenchmark (not product code): the two SpMV passes of the factored sparse-linear
// K·p on a config-3-shaped matrix (1M rows x 50k cols, 50 nnz/row, fp32), with ablations that
// isolate the index/value stream, the gather and the LDS reduction.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/spmv_microbench.hip -o build/spmv_microbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../plssvm_sparse_fp22_amd/csrc/spmv.hpp"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);         \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

constexpr int NT = 256;

// MODE 0: full (idx, val, gather); 1: no gather (x[0]); 2: val only; 3: gather with idx but no LDS reduce
template <int CHUNK, int MODE, bool NTL>
__global__ __launch_bounds__(NT) void seg_spmv(const int64_t *__restrict__ ptr, const int32_t *__restrict__ idx,
                                               const float *__restrict__ val, const float *__restrict__ x,
                                               const int64_t *__restrict__ bseg, float *__restrict__ out) {
    constexpr int PER = CHUNK / NT;
    __shared__ float prod[CHUNK];
    const int tid = threadIdx.x;
    const int64_t s0 = bseg[blockIdx.x], s1 = bseg[blockIdx.x + 1];
    const int64_t e0 = ptr[s0], e1 = ptr[s1];
    const int cnt = (int) (e1 - e0);
    {
        int c[PER];
        float v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = tid + u * NT;
            if (k < cnt) {
                if (MODE != 2) c[u] = NTL ? __builtin_nontemporal_load(idx + e0 + k) : idx[e0 + k];
                v[u] = NTL ? __builtin_nontemporal_load(val + e0 + k) : val[e0 + k];
            }
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = tid + u * NT;
            if (k < cnt) {
                if (MODE == 0 || MODE == 3) prod[k] = v[u] * x[c[u]];
                else if (MODE == 1) prod[k] = v[u] * x[c[u] & 63];
                else prod[k] = v[u];
            }
        }
    }
    __syncthreads();
    if (MODE == 3) {
        if (tid == 0) out[s0] = prod[0];
        return;
    }
    const int nseg = (int) (s1 - s0);
    int L = 64;
    while (L > 1 && L * nseg > NT) L >>= 1;
    const int lane = tid & (L - 1), ngrp = NT / L;
    for (int g = tid / L; g < nseg; g += ngrp) {
        const int a = (int) (ptr[s0 + g] - e0), b = (int) (ptr[s0 + g + 1] - e0);
        float s = 0;
        for (int k = a + lane; k < b; k += L) s += prod[k];
        for (int o = L >> 1; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if (lane == 0) out[s0 + g] = s;
    }
}

// old kernels (for comparison)
__global__ __launch_bounds__(256) void csr_gemv_old(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
                                                    const float *__restrict__ val, int64_t r1, const float *__restrict__ w,
                                                    float *__restrict__ raw) {
    const int64_t row = (int64_t) blockIdx.x * 16 + (threadIdx.x >> 4);
    const int sl = threadIdx.x & 15;
    float s = 0;
    if (row < r1) {
        const int64_t b = rowptr[row + 1];
        for (int64_t k = rowptr[row] + sl; k < b; k += 16) s = fmaf(val[k], w[col[k]], s);
    }
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    s += __shfl_xor(s, 8);
    if (row < r1 && sl == 0) raw[row] = s;
}

__global__ void stream_copy(const float4 *__restrict__ a, float4 *__restrict__ b, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x)
        b[i] = a[i];
}

std::vector<int64_t> blocks(const std::vector<int64_t> &ptr, int64_t ns, int64_t chunk) {
    std::vector<int64_t> bs{ 0 };
    int64_t s = 0;
    while (s < ns) {
        int64_t t = s;
        while (t < ns && t - s < 4096 && ptr[t + 1] - ptr[s] <= chunk) ++t;
        if (t == s) t = s + 1;
        bs.push_back(t);
        s = t;
    }
    return bs;
}

template <typename F>
float timeit(F f, int reps = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int only_tb = argc > 1 ? atoi(argv[1]) : 0;  // run only this target block count (PMC runs)
    const int64_t n = 1000000, d = 50000, k = 50, nnz = n * k;
    std::mt19937_64 rng(3);
    std::vector<int64_t> rowptr(n + 1);
    std::vector<int32_t> col(nnz);
    std::vector<float> val(nnz);
    std::uniform_real_distribution<float> U(-1, 1);
    for (int64_t i = 0; i < n; ++i) {
        rowptr[i] = i * k;
        std::vector<int32_t> c(k);
        for (auto &x : c) x = (int32_t) (rng() % d);
        std::sort(c.begin(), c.end());
        for (int j = 0; j < k; ++j) col[i * k + j] = c[j], val[i * k + j] = U(rng);
    }
    rowptr[n] = nnz;
    std::vector<int64_t> colptr(d + 1, 0);
    for (auto c : col) ++colptr[c + 1];
    for (int64_t f = 0; f < d; ++f) colptr[f + 1] += colptr[f];
    std::vector<int64_t> fill(colptr.begin(), colptr.end() - 1);
    std::vector<int32_t> crow(nnz);
    std::vector<float> cval(nnz);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t e = rowptr[i]; e < rowptr[i + 1]; ++e) {
            const int64_t t = fill[col[e]]++;
            crow[t] = (int32_t) i;
            cval[t] = val[e];
        }
    auto up = [](auto &v) {
        using E = typename std::decay_t<decltype(v)>::value_type;
        E *p;
        CK(hipMalloc(&p, sizeof(E) * v.size()));
        CK(hipMemcpy(p, v.data(), sizeof(E) * v.size(), hipMemcpyHostToDevice));
        return p;
    };
    int64_t *d_rowptr = up(rowptr);
    int32_t *d_col = up(col);
    float *d_val = up(val);
    std::vector<float> p(n, 1.0f), w(d, 1.0f);
    float *d_p = up(p), *d_w = up(w), *d_out;
    CK(hipMalloc(&d_out, sizeof(float) * n));
    const double bytes = nnz * 8.0;
    auto rep = [&](const char *name, float ms, double b) { printf("%-48s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, b / ms / 1e6); };
    {
        float4 *a, *b;
        const int64_t n4 = nnz * 2 / 4;
        CK(hipMalloc(&a, n4 * 16));
        CK(hipMalloc(&b, n4 * 16));
        rep("stream copy float4 (read+write 400MB each)", timeit([&] { stream_copy<<<4096, 256>>>(a, b, n4); }), 2.0 * n4 * 16);
    }
    rep("old csr_gemv", timeit([&] { csr_gemv_old<<<(unsigned) ((n + 15) / 16), 256>>>(d_rowptr, d_col, d_val, n, d_w, d_out); }), bytes);
    using namespace plssvm_mi;
    auto gen_csr = [&](auto emit) {
        for (int64_t i = 0; i < n; ++i)
            for (int64_t e = rowptr[i]; e < rowptr[i + 1]; ++e) emit(i, (int64_t) col[e], (double) val[e]);
    };
    auto gen_csc = [&](auto emit) {
        for (int64_t i = 0; i < n; ++i)
            for (int64_t e = rowptr[i]; e < rowptr[i + 1]; ++e) emit((int64_t) col[e], i, (double) val[e]);
    };
    for (int mode : { 2, 1 }) {
        for (int64_t tb : { 256, 512, 1024 }) {
            if (mode == 2 && tb != 512) continue;
            if (only_tb && (mode != 1 || tb != only_tb)) continue;
            spmv_plan<float> pr, pc;
            build_spmv_plan<float>(pr, n, d, nnz, false, gen_csr, tb, nullptr, mode);
            build_spmv_plan<float>(pc, d, n, nnz, false, gen_csc, tb, nullptr, mode);
            char name[128];
            snprintf(name, sizeof name, "CSR pass %s P=%ld blocks=%ld pad=%.3f", mode == 1 ? "lds" : "glb", (long) pr.P, (long) pr.nblocks, (double) pr.entries / nnz);
            rep(name, timeit([&] { launch_panel_spmv<float>(pr, d_w, d, d_out, nullptr, nullptr); }), (double) pr.stream_bytes());
            snprintf(name, sizeof name, "CSC pass %s P=%ld blocks=%ld pad=%.3f", mode == 1 ? "lds" : "glb", (long) pc.P, (long) pc.nblocks, (double) pc.entries / nnz);
            rep(name, timeit([&] { launch_panel_spmv<float>(pc, d_p, n, d_out, nullptr, nullptr); }), (double) pc.stream_bytes());
        }
    }
    return 0;
}
