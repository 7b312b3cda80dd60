// Development probe (not product code): achievable fp64 / fp32 MFMA rate on this MI355X
// (back-to-back v_mfma_f64_16x16x4f64 / v_mfma_f32_16x16x4f32 with independent accumulators on
// every SIMD) and rocBLAS dgemm / sgemm at 8192^3 — the practical ceilings that the dense K·p tile
// kernel's roofline fraction is read against.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_peak.hip -lrocblas -o mfma_peak
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <vector>

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int ITERS>
__global__ __launch_bounds__(256) void mfma_f64(double *out, double a0) {
    f64x4 acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = f64x4{ 0, 0, 0, 0 };
    double a = a0 + threadIdx.x, b = a0 - threadIdx.x;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    if (s == 12345.678) out[0] = s;
}

template <int ITERS>
__global__ __launch_bounds__(256) void mfma_f32(float *out, float a0) {
    f32x4 acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = f32x4{ 0, 0, 0, 0 };
    float a = a0 + threadIdx.x, b = a0 - threadIdx.x;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[k], 0, 0, 0);
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    if (s == 12345.678f) out[0] = s;
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    constexpr int IT = 4096;
    const int blocks = 256 * 8;  // 8 workgroups of 4 waves per CU
    double *od;
    float *of;
    hipMalloc(&od, 8);
    hipMalloc(&of, 4);
    const double flop = 2.0 * 16 * 16 * 4 * 8 * IT * (double) blocks * 4;  // per wave: 8 MFMA per iter
    float ms = timeit([&] { mfma_f64<IT><<<blocks, 256>>>(od, 1.0); }, 5);
    printf("mfma f64 16x16x4 back-to-back: %.1f TFLOP/s\n", flop / ms / 1e9);
    ms = timeit([&] { mfma_f32<IT><<<blocks, 256>>>(of, 1.0f); }, 5);
    printf("mfma f32 16x16x4 back-to-back: %.1f TFLOP/s\n", flop / ms / 1e9);

    rocblas_handle h;
    rocblas_create_handle(&h);
    for (int n : { 4096, 8192 }) {
        double *A, *B, *C;
        hipMalloc(&A, sizeof(double) * n * n);
        hipMalloc(&B, sizeof(double) * n * n);
        hipMalloc(&C, sizeof(double) * n * n);
        std::vector<double> init((size_t) n * n);
        for (size_t i = 0; i < init.size(); ++i) init[i] = (double) ((i * 2654435761u) % 1000) / 1000.0 - 0.5;
        hipMemcpy(A, init.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
        hipMemcpy(B, init.data(), sizeof(double) * n * n, hipMemcpyHostToDevice);
        const double one = 1, zero = 0;
        ms = timeit([&] { rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, n, n, n, &one, A, n, B, n, &zero, C, n); }, 5);
        printf("rocblas dgemm NT n=%d: %.1f TFLOP/s (%.2f ms)\n", n, 2.0 * n * (double) n * n / ms / 1e9, ms);
        float *Af = (float *) A, *Bf = (float *) B, *Cf = (float *) C;
        const float onef = 1, zerof = 0;
        ms = timeit([&] { rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_transpose, n, n, n, &onef, Af, n, Bf, n, &zerof, Cf, n); }, 5);
        printf("rocblas sgemm NT n=%d: %.1f TFLOP/s (%.2f ms)\n", n, 2.0 * n * (double) n * n / ms / 1e9, ms);
        hipFree(A);
        hipFree(B);
        hipFree(C);
    }
    return 0;
}
