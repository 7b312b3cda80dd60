// Debug probe (not product code): decode packed FP22 words on the device with the product's
// fp22_get / vals_t and compare with the host decode. Input: raw files written by the caller:
// words.bin (uint32 packed), ref.bin (float32 decoded).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../plssvm_sparse_fp22_amd/csrc/fp22.hpp"

__global__ void decode_all(plssvm_mi::vals_t<float> v, int64_t n, float *out) {
    for (int64_t e = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; e < n; e += (int64_t) gridDim.x * blockDim.x)
        out[e] = v[e];
}

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    std::vector<uint32_t> w;
    uint32_t x;
    while (fread(&x, 4, 1, f) == 1) w.push_back(x);
    fclose(f);
    f = fopen(argv[2], "rb");
    std::vector<float> ref;
    float y;
    while (fread(&y, 4, 1, f) == 1) ref.push_back(y);
    fclose(f);
    const int64_t n = (int64_t) ref.size();
    uint32_t *dw;
    float *dout;
    hipMalloc(&dw, (w.size() + 1) * 4);
    hipMemset(dw, 0, (w.size() + 1) * 4);
    hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice);
    hipMalloc(&dout, n * 4);
    decode_all<<<1024, 256>>>(plssvm_mi::vals_t<float>{ nullptr, dw }, n, dout);
    std::vector<float> got(n);
    hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost);
    int64_t bad = 0, first = -1, hostbad = 0;
    for (int64_t e = 0; e < n; ++e) {
        if (got[e] != ref[e]) {
            if (first < 0) first = e;
            ++bad;
        }
        if (plssvm_mi::fp22_get(w.data(), e) != ref[e]) ++hostbad;
    }
    printf("n=%ld words=%zu device mismatches=%ld first=%ld host mismatches=%ld\n", (long) n, w.size(), (long) bad,
           (long) first, (long) hostbad);
    if (first >= 0) printf("e=%ld got %g want %g\n", (long) first, got[first], ref[first]);
    return 0;
}
