// Device helpers shared by the fused CG kernels (blas1.hip) and the kernels that fuse a CG step into the
// producer of its input (expand.hip: the expansion's combine + finalize): one definition, so the fused and
// unfused sequences compile the same arithmetic and give the same bits.
#pragma once

#include "kernels.hpp"

namespace plssvm_mi {
namespace cgk {

// fused CG kernels: RED_BLOCKS blocks of CG_NT threads (16 waves per block: memory parallelism for
// the vector streams; one partial per block as for dot2_kernel)
constexpr int CG_NT = 1024;

template <typename T>
__device__ __forceinline__ T block_sum(T v, T *red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    T s = 0;
    if (threadIdx.x == 0) {
        for (int w = 0; w < (int) (blockDim.x >> 6); ++w) s += red[w];
    }
    return s;
}

// block_sum with the total broadcast to every thread
template <typename T>
__device__ __forceinline__ T block_sum_all(T v, T *red, T *bc) {
    const T s = block_sum(v, red);
    if (threadIdx.x == 0) *bc = s;
    __syncthreads();
    const T out = *bc;
    __syncthreads();
    return out;
}

// the RED_BLOCKS partial pairs of a dot2_kernel-shaped producer (G gathered sets of a sharded group),
// summed as dot_final_kernel does
template <typename T>
__device__ __forceinline__ void partials_total(const T *__restrict__ partials, int G, T *red, T *bc, T &r1, T &r2) {
    T s1 = 0, s2 = 0;
    for (int i = threadIdx.x; i < RED_BLOCKS; i += blockDim.x) {
        T a = partials[i], b = partials[RED_BLOCKS + i];
        for (int g = 1; g < G; ++g) {
            a += partials[g * 2 * RED_BLOCKS + i];
            b += partials[g * 2 * RED_BLOCKS + RED_BLOCKS + i];
        }
        s1 += a;
        s2 += b;
    }
    r1 = block_sum_all(s1, red, bc);
    r2 = block_sum_all(s2, red, bc);
}

// partials_total's first sum only (producers whose second partial is zero: d.Ad, r.r) — the same bits for r1,
// one block reduction fewer
template <typename T>
__device__ __forceinline__ T partials_total1(const T *__restrict__ partials, int G, T *red, T *bc) {
    T s1 = 0;
    for (int i = threadIdx.x; i < RED_BLOCKS; i += blockDim.x) {
        T a = partials[i];
        for (int g = 1; g < G; ++g) a += partials[g * 2 * RED_BLOCKS + i];
        s1 += a;
    }
    return block_sum_all(s1, red, bc);
}

// store_partials(v1, 0): the second partial of the pair is zero
template <typename T>
__device__ __forceinline__ void store_partial1(T v1, T *red, T *__restrict__ partials) {
    const T r1 = block_sum(v1, red);
    if (threadIdx.x == 0) {
        partials[blockIdx.x] = r1;
        partials[RED_BLOCKS + blockIdx.x] = T(0);
    }
}

// the first partial of the pair only: the second slot keeps what another kernel put there (the one-reduction CG keeps
// its r.r partials beside the r.u partials of the finalize, so that one collective gathers both)
template <typename T>
__device__ __forceinline__ void store_partial_first(T v1, T *red, T *__restrict__ partials) {
    const T r1 = block_sum(v1, red);
    if (threadIdx.x == 0) partials[blockIdx.x] = r1;
}

// the second partial of the pair only
template <typename T>
__device__ __forceinline__ void store_partial_second(T v2, T *red, T *__restrict__ partials) {
    const T r2 = block_sum(v2, red);
    if (threadIdx.x == 0) partials[RED_BLOCKS + blockIdx.x] = r2;
}

template <typename T>
__device__ __forceinline__ void store_partials(T v1, T v2, T *red, T *__restrict__ partials) {
    const T r1 = block_sum(v1, red);
    __syncthreads();
    const T r2 = block_sum(v2, red);
    if (threadIdx.x == 0) {
        partials[blockIdx.x] = r1;
        partials[RED_BLOCKS + blockIdx.x] = r2;
    }
}

// dot_final_kernel's sum of the RED_BLOCKS partial pairs (G gathered sets, rank order), for a 256-thread block:
// every thread its partials, then block_sum — the same bits wherever it runs (thread 0 holds r1, r2)
template <typename T>
__device__ __forceinline__ void partials_final(const T *__restrict__ partials, int G, T *red, T &r1, T &r2) {
    T s1 = 0, s2 = 0;
    for (int i = threadIdx.x; i < RED_BLOCKS; i += blockDim.x) {
        T a = partials[i], b = partials[RED_BLOCKS + i];
        for (int g = 1; g < G; ++g) {
            a += partials[g * 2 * RED_BLOCKS + i];
            b += partials[g * 2 * RED_BLOCKS + RED_BLOCKS + i];
        }
        s1 += a;
        s2 += b;
    }
    r1 = block_sum(s1, red);
    __syncthreads();
    r2 = block_sum(s2, red);
}

// Ad_i of the CG finalize: raw_i + (QA - q_i) sum(d) - sum(q d) + d_i / C (kp_finalize_kernel's
// expression, contracted as in dense.hip)
template <typename T>
__device__ __forceinline__ T cg_fin_value(T r_, T q_, T d_, T sp, T sqp, T QA_cost, T cost_inv, int raw_only) {
#pragma clang fp contract(fast)
    T v = raw_only ? r_ : r_ + (QA_cost - q_) * sp - sqp + cost_inv * d_;
    v = T(0) + T(1) * v;
    return v;
}

// s + a * b with the product rounded before the add (the dot partials of the CG kernels)
template <typename T>
__device__ __forceinline__ T cg_acc(T s, T a, T b) {
#pragma clang fp contract(off)
    return s + a * b;
}

// bfloat16 of a float, round to nearest even (finite values)
__device__ __forceinline__ uint16_t bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t) (u >> 16);
}

// element i of the kernel expansion's w pass: w_i = e_i p_i (e null: w = p, not written), its bfloat16 copy, and
// the S term (cw non-null: the centered cw_i w_i) added to s — one definition for exp_wown_kernel and the
// direction update that carries it (blas1.hip), so both give the same bits
template <typename T>
__device__ __forceinline__ void w_elem(int64_t i, T v, T ev, T cv, const T *e, const T *cw, T *__restrict__ w,
                                       uint16_t *__restrict__ w16, T &s) {
    if (e != nullptr) {
        v = ev * v;
        w[i] = v;
    }
    s += cw != nullptr ? cv * v : v;
    w16[i] = bf16_rne((float) v);
}

}  // namespace cgk
}  // namespace plssvm_mi
