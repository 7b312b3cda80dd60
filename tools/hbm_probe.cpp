// HBM bandwidth probe ("verify on the box with a STREAM-copy probe and report both the
// datasheet and the measured denominator"). Read-only sweep (16-B nontemporal loads summed into one value
// per thread, the access shape of the remainder stream and the SELL passes) and a float4 copy, at the
// stream sizes of the bench's dominant kernels, timed with hipEvents over repeated launches.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.cpp ; run on the GPU box:
//   tools/hbm_probe > profiles/<round>_hbm_probe.json
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_kernel(const f4 *__restrict__ a, int64_t n, float *__restrict__ sink) {
    float s = 0.f;
    const int64_t st = (int64_t) gridDim.x * blockDim.x;
    int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * st < n; i += 4 * st) {  // four 16-B loads in flight per thread
        const f4 v0 = __builtin_nontemporal_load(a + i), v1 = __builtin_nontemporal_load(a + i + st);
        const f4 v2 = __builtin_nontemporal_load(a + i + 2 * st), v3 = __builtin_nontemporal_load(a + i + 3 * st);
        s += (v0.x + v1.y) + (v2.z + v3.w);
    }
    for (; i < n; i += st) s += __builtin_nontemporal_load(a + i).x;
    if (s == 12345.f) sink[0] = s;  // keeps the loads; never true for the zero-filled buffer
}

__global__ __launch_bounds__(256) void copy_kernel(const f4 *__restrict__ a, f4 *__restrict__ b, int64_t n) {
    const int64_t st = (int64_t) gridDim.x * blockDim.x;
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += st) b[i] = a[i];
}

int main() {
    const double sizes_gb[] = { 0.3, 0.65, 1.0, 5.4, 8.0 };
    const int64_t max_bytes = (int64_t) (8.0e9);
    f4 *a = nullptr, *b = nullptr;
    float *sink = nullptr;
    CHECK(hipMalloc(&a, max_bytes));
    CHECK(hipMalloc(&b, (int64_t) 2.0e9));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(a, 0, max_bytes));
    CHECK(hipMemset(b, 0, (int64_t) 2.0e9));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grid = 256 * 16;
    std::printf("{\"probe\": \"tools/hbm_probe.cpp\", \"grid\": %d, \"block\": 256, \"read\": [", grid);
    bool first = true;
    for (double gb : sizes_gb) {
        const int64_t n = (int64_t) (gb * 1e9) / 16;
        const int reps = gb < 2.0 ? 50 : 10;
        hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, a, n, sink);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, 0, a, n, sink);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double s = ms * 1e-3 / reps;
        std::printf("%s{\"GB\": %.2f, \"us_per_launch\": %.2f, \"TBps\": %.3f}", first ? "" : ", ", gb, s * 1e6,
                    (double) n * 16 / s / 1e12);
        first = false;
    }
    std::printf("], \"copy\": [");
    first = true;
    for (double gb : { 0.4, 1.0 }) {  // bytes read (the same again written)
        const int64_t n = (int64_t) (gb * 1e9) / 16;
        hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, 0, a, b, n);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, 0, a, b, n);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double s = ms * 1e-3 / 20;
        std::printf("%s{\"GB_read\": %.2f, \"us_per_launch\": %.2f, \"TBps_read_plus_write\": %.3f}", first ? "" : ", ", gb,
                    s * 1e6, 2.0 * (double) n * 16 / s / 1e12);
        first = false;
    }
    std::printf("], \"datasheet_TBps\": 8.0}\n");
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(sink));
    return 0;
}
