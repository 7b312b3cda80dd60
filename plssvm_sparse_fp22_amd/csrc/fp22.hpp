// Packed FP22 codec and the sparse value accessor (build-defined format).
#pragma once

#include <cstdint>

#include <hip/hip_runtime.h>

namespace plssvm_mi {

// ---- packed FP22: binary32 truncated to its top 22 bits (RNE), 16 values per 11 uint32 words ----
__host__ __device__ inline float fp22_decode(uint32_t code) {
    union {
        uint32_t u;
        float f;
    } v;
    v.u = (code & 0x3FFFFFu) << 10;
    return v.f;
}

inline uint32_t fp22_encode_host(float x) {
    union {
        float f;
        uint32_t u;
    } v;
    v.f = x;
    const uint32_t u = v.u;
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return ((u >> 10) | 0x1000u) & 0x3FFFFFu;
    return ((u + 0x1FFu + ((u >> 10) & 1u)) >> 10) & 0x3FFFFFu;
}

inline int64_t fp22_words(int64_t n) { return ((n + 15) / 16) * 11; }

__host__ __device__ inline float fp22_get(const uint32_t *words, int64_t e) {
    const int64_t g = e >> 4;
    const int bit = 22 * (int) (e & 15);
    const uint32_t *w = words + g * 11 + (bit >> 5);
    const int s = bit & 31;
    uint64_t x = (uint64_t) w[0] >> s;
    if (s > 10) x |= (uint64_t) w[1] << (32 - s);
    return fp22_decode((uint32_t) x);
}

// value accessor: real array or packed FP22 words
template <typename T>
struct vals_t {
    const T *v;
    const uint32_t *v22;
    __device__ __forceinline__ T operator[](int64_t e) const { return v22 ? (T) fp22_get(v22, e) : v[e]; }
};

}  // namespace plssvm_mi
