// Development probe (not product code): can fp64 VALU work overlap fp64 MFMA on gfx950?
// Each 512-thread workgroup (2 waves per SIMD) runs ITERS steps of 8 independent
// v_mfma_f64_16x16x4f64; variants add fp64 / fp32 / int VALU work either in the same waves or in
// separate "VALU-only" waves (waves 4-7). If the MFMA time does not grow when VALU work is added in
// other waves, the pipes overlap; if it grows by the VALU issue time, they share the DP units.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/coexec_probe.hip -o coexec_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

// MODE 0: MFMA only (all 8 waves)      1: MFMA + NV fp64 FMAs per step in the same wave
// MODE 2: waves 0-3 MFMA, waves 4-7 fp64 FMA only (NV per step)
// MODE 3: waves 0-3 MFMA only, waves 4-7 idle     4: waves 0-3 MFMA, waves 4-7 fp32 FMA only
// MODE 5: waves 0-3 MFMA, waves 4-7 int32 ops only   6 / 7: fp64 / fp32 FMA only in all waves
template <int MODE, int NV>
__global__ __launch_bounds__(512) void probe(double *out, int iters, double a0) {
    const int wave = threadIdx.x >> 6;
    f64x4 acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = f64x4{ 0, 0, 0, 0 };
    double a = a0 + threadIdx.x, b = a0 - threadIdx.x;
    double v[8];
    float vf[8];
    int vi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = a0 * (k + 1), vf[k] = (float) v[k], vi[k] = k + threadIdx.x;
    const bool mfma_wave = MODE < 6 && ((MODE == 0 || MODE == 1) || wave < 4);
    if (mfma_wave) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
            if (MODE == 1) {
#pragma unroll
                for (int j = 0; j < NV; ++j) v[j & 7] = fma(v[j & 7], 1.0000001, 1e-9);
            }
        }
    } else if (MODE == 2) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < NV; ++j) v[j & 7] = fma(v[j & 7], 1.0000001, 1e-9);
        }
    } else if (MODE == 4) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < NV; ++j) vf[j & 7] = fmaf(vf[j & 7], 1.0000001f, 1e-9f);
        }
    } else if (MODE == 6 || MODE == 7) {  // no MFMA anywhere: fp64 (6) / fp32 (7) FMA throughput alone
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                if (MODE == 6) v[j & 7] = fma(v[j & 7], 1.0000001, 1e-9);
                else vf[j & 7] = fmaf(vf[j & 7], 1.0000001f, 1e-9f);
            }
        }
    } else if (MODE == 5) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < NV; ++j) vi[j & 7] = vi[j & 7] * 3 + 7;
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + v[k] + vf[k] + vi[k];
    if (s == 12345.678) out[0] = s;
}

template <int MODE, int NV>
float run(double *out, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    probe<MODE, NV><<<256 * 2, 512>>>(out, iters, 1.0);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) probe<MODE, NV><<<256 * 2, 512>>>(out, iters, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 3;
}

int main() {
    double *out;
    hipMalloc(&out, 8);
    const int iters = 2048;
    printf("MODE0 mfma only (8 waves/CU-SIMD pair)      %.3f ms\n", run<0, 0>(out, iters));
    printf("MODE3 mfma waves 0-3, 4-7 idle              %.3f ms\n", run<3, 0>(out, iters));
    printf("MODE1 mfma + 8 f64 fma same wave            %.3f ms\n", run<1, 8>(out, iters));
    printf("MODE1 mfma + 32 f64 fma same wave           %.3f ms\n", run<1, 32>(out, iters));
    printf("MODE2 mfma 0-3 / 32 f64 fma in waves 4-7    %.3f ms\n", run<2, 32>(out, iters));
    printf("MODE2 mfma 0-3 / 64 f64 fma in waves 4-7    %.3f ms\n", run<2, 64>(out, iters));
    printf("MODE4 mfma 0-3 / 64 f32 fma in waves 4-7    %.3f ms\n", run<4, 64>(out, iters));
    printf("MODE5 mfma 0-3 / 64 int ops in waves 4-7    %.3f ms\n", run<5, 64>(out, iters));
    printf("MODE6 no mfma, 64 f64 fma per step, 8 waves %.3f ms\n", run<6, 64>(out, iters));
    printf("MODE7 no mfma, 64 f32 fma per step, 8 waves %.3f ms\n", run<7, 64>(out, iters));
    return 0;
}
