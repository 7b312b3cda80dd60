// Implicit pairwise K·p tiles on MFMA (gfx950) — the dense hot kernel.
//
// Replaces device_kernel_{linear,poly,radial} (include/plssvm/backends/HIP/svm_kernel.hip.hpp:36-268)
// and its OpenMP twin (src/plssvm/backends/OpenMP/svm_kernel.cpp:21-47). Per 128x128 lower-triangle
// tile (I >= J) of k(x_i, x_j):
//   * X is feature-major in HBM (XT[k][i]); each BK-deep K chunk of the two 128-column panels is
//     streamed global -> LDS with global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPR
//     staging), double-buffered so chunk kc+1 lands while chunk kc feeds the MFMAs: one barrier
//     per chunk;
//   * 4 waves as 2x2, each a 64x64 sub-tile = 4x4 accumulators of v_mfma_f64_16x16x4_f64 /
//     v_mfma_f32_16x16x4_f32 (exact fma chains in k order);
//   * epilogue in registers: kernel function (RBF via ||a||^2 + ||b||^2 - 2 a.b, clamped at 0),
//     times p_j -> row sums (16-lane shuffles) and times p_i -> mirrored column sums (cross-half
//     shuffles); results go to partial[J][i in I] and partial[I][j in J] — no atomics, so a
//     fixed-order second pass makes K·p bitwise reproducible;
//   * tiles are visited in 8x8 super-blocks (16 panels = 4 MiB in fp64: one XCD's L2) and the
//     workgroup ids are remapped so each XCD walks a contiguous range of super-blocks.
#include "kernels.hpp"

namespace plssvm_mi {

namespace {

template <typename T>
__device__ __forceinline__ T kernel_apply(int kernel, int degree, T gamma, T coef0, T g, T ni, T nj) {
    if (kernel == 0) return g;
    if (kernel == 1) {
        const T base = fma(gamma, g, coef0);
        T r = T(1);
        for (int e = 0; e < degree; ++e) r *= base;
        return r;
    }
    T dist = ni + nj - T(2) * g;
    dist = dist > T(0) ? dist : T(0);
    return exp(-gamma * dist);
}

__device__ __forceinline__ void glds16(const void *src, void *lds_dst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *) src,
                                     (__attribute__((address_space(3))) void *) lds_dst, 16, 0, 0);
}

template <typename T, int KERNEL>
__global__ __launch_bounds__(256, 2) void kp_tile_kernel(kfun<T> kf, const T *__restrict__ XT,
                                                         const T *__restrict__ norms, const T *__restrict__ p,
                                                         T *__restrict__ partial, int64_t n_pad, int64_t d_pad,
                                                         int64_t nb, int64_t s0,
                                                         const cg_scalars<T> *__restrict__ status) {
    using M = mfma16<T>;
    using acc_t = typename M::acc_t;
    constexpr int BK = kp_bk<T>();
    constexpr int PANEL = BK * KP_TILE;            // elements of one [BK][128] panel
    constexpr int EPP = 1024 / (int) sizeof(T);    // elements per 1 KiB wave-instruction
    constexpr int PIECES = PANEL / EPP / 4;        // wave-instructions per wave per panel
    constexpr int VEC = 16 / (int) sizeof(T);
    constexpr int OFF_PN = 4 * PANEL;              // p_I, p_J, n_I, n_J
    constexpr int OFF_RED = OFF_PN + 4 * KP_TILE;  // rowbuf[2][128], colbuf[2][128]
    __shared__ __attribute__((aligned(16))) T smem[OFF_RED + 4 * KP_TILE];

    if (status != nullptr && status->converged) return;

    const int64_t wg = xcd_remap(blockIdx.x, gridDim.x);
    int64_t SI, SJ;
    tri_tile(s0 + wg / (KP_SUPER * KP_SUPER), SI, SJ);
    const int slot = (int) (wg % (KP_SUPER * KP_SUPER));
    const int64_t I = SI * KP_SUPER + slot / KP_SUPER, J = SJ * KP_SUPER + slot % KP_SUPER;
    if (I >= nb || J > I) return;  // uniform per workgroup
    const int64_t I0 = I * KP_TILE, J0 = J * KP_TILE;
    const bool diag = (I == J);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;

    // p and norms of the tile's rows/cols -> LDS (issued first: their wait must not drain the DMA)
    const int64_t pidx = (tid < KP_TILE) ? I0 + tid : J0 + (tid - KP_TILE);
    const T pin = p[pidx];
    const T nin = (KERNEL == 2) ? norms[pidx] : T(0);

    auto issue = [&](int64_t kc, int buf) {
        const int64_t k0 = kc * BK;
        T *pa = smem + (2 * buf) * PANEL;
        T *pb = pa + PANEL;
#pragma unroll
        for (int j = 0; j < PIECES; ++j) {
            const int u = w * PIECES + j;
            const int elem = u * EPP + lane * VEC;
            const int row = elem / KP_TILE, col = elem % KP_TILE;
            const T *src = XT + (k0 + row) * n_pad + col;
            glds16(src + I0, pa + u * EPP);
            glds16(src + J0, pb + u * EPP);
        }
    };

    acc_t acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = acc_t{ 0, 0, 0, 0 };

    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    smem[OFF_PN + tid] = pin;
    smem[OFF_PN + 2 * KP_TILE + tid] = nin;

    const int64_t nk = d_pad / BK;
    for (int64_t kc = 0; kc < nk; ++kc) {
        if (kc > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // chunk kc visible to all waves; every wave is done reading chunk kc-1
        if (kc + 1 < nk) issue(kc + 1, (int) ((kc + 1) & 1));
        const T *A = smem + (2 * (kc & 1)) * PANEL;
        const T *B = A + PANEL;
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks) {
            const int kr = ks * 4 + (lane >> 4);
            T a[4], b[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) a[mt] = A[kr * KP_TILE + wr * 64 + mt * 16 + (lane & 15)];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) b[nt] = B[kr * KP_TILE + wc * 64 + nt * 16 + (lane & 15)];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = M::op(a[mt], b[nt], acc[mt][nt]);
        }
    }

    // ---- epilogue: kernel function, times p, row and column sums ----
    const T *pI = smem + OFF_PN, *pJ = pI + KP_TILE, *nI = pI + 2 * KP_TILE, *nJ = pI + 3 * KP_TILE;
    T *rowbuf = smem + OFF_RED, *colbuf = rowbuf + 2 * KP_TILE;
    T pj[4], nj[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int jl = wc * 64 + nt * 16 + (lane & 15);
        pj[nt] = pJ[jl];
        nj[nt] = nJ[jl];
    }
    T cs[4] = { 0, 0, 0, 0 };
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int il = wr * 64 + mt * 16 + M::row(lane, r);
            const T pi = pI[il];
            const T ni = nI[il];
            T s = 0;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const T kv = kernel_apply<T>(KERNEL, kf.degree, kf.gamma, kf.coef0, acc[mt][nt][r], ni, nj[nt]);
                s = fma(kv, pj[nt], s);
                cs[nt] = fma(kv, pi, cs[nt]);
            }
            // lanes sharing (lane >> 4) hold the same row: reduce over lane & 15
            s += __shfl_xor(s, 1);
            s += __shfl_xor(s, 2);
            s += __shfl_xor(s, 4);
            s += __shfl_xor(s, 8);
            if ((lane & 15) == 0) rowbuf[wc * KP_TILE + il] = s;
        }
    }
    if (!diag) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {  // lanes sharing (lane & 15) hold the same column
            T v = cs[nt];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane < 16) colbuf[wr * KP_TILE + wc * 64 + nt * 16 + lane] = v;
        }
    }
    __syncthreads();
    if (tid < KP_TILE) {
        partial[J * n_pad + I0 + tid] = rowbuf[tid] + rowbuf[KP_TILE + tid];
    } else if (!diag) {
        const int t = tid - KP_TILE;
        partial[I * n_pad + J0 + t] = colbuf[t] + colbuf[KP_TILE + t];
    }
}

template <typename T>
__global__ __launch_bounds__(256) void kp_reduce_kernel(const T *__restrict__ partial, int64_t nb, int64_t n_pad,
                                                        int64_t m, int64_t s0, int64_t s1, int64_t s_total,
                                                        T *__restrict__ raw,
                                                        const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    T s = 0;
    if (s0 == 0 && s1 == s_total) {
        for (int64_t c = 0; c < nb; ++c) s += partial[c * n_pad + i];
    } else {
        const int64_t RS = (i / KP_TILE) / KP_SUPER;
        for (int64_t c = 0; c < nb; ++c) {
            const int64_t CS = c / KP_SUPER;
            const int64_t sb = (RS >= CS) ? tri_index(RS, CS) : tri_index(CS, RS);
            if (sb >= s0 && sb < s1) s += partial[c * n_pad + i];
        }
    }
    raw[i] = s;
}

}  // namespace

template <typename T>
void launch_kp_tiles(kfun<T> kf, const T *XT, const T *norms, const T *p, T *partial, int64_t n_pad, int64_t d_pad,
                     int64_t nb, int64_t s0, int64_t nsuper, const cg_scalars<T> *status, hipStream_t s) {
    if (nsuper <= 0 || nb <= 0) return;
    const dim3 grid((unsigned) (nsuper * KP_SUPER * KP_SUPER)), block(256);
    switch (kf.kernel) {
        case 0:
            hipLaunchKernelGGL((kp_tile_kernel<T, 0>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, nb,
                               s0, status);
            break;
        case 1:
            hipLaunchKernelGGL((kp_tile_kernel<T, 1>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, nb,
                               s0, status);
            break;
        default:
            hipLaunchKernelGGL((kp_tile_kernel<T, 2>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, nb,
                               s0, status);
            break;
    }
    MI_LAUNCH_CHECK();
}

template <typename T>
void launch_kp_reduce(const T *partial, int64_t nb, int64_t n_pad, int64_t m, int64_t s0, int64_t s1, T *raw,
                      const cg_scalars<T> *status, hipStream_t s) {
    if (m <= 0) return;
    const int64_t ns = ceil_div(nb, KP_SUPER);
    hipLaunchKernelGGL(kp_reduce_kernel<T>, dim3((unsigned) ceil_div(m, 256)), dim3(256), 0, s, partial, nb, n_pad, m,
                       s0, s1, ns * (ns + 1) / 2, raw, status);
    MI_LAUNCH_CHECK();
}

#define INST(T)                                                                                                  \
    template void launch_kp_tiles<T>(kfun<T>, const T *, const T *, const T *, T *, int64_t, int64_t, int64_t, \
                                     int64_t, int64_t, const cg_scalars<T> *, hipStream_t);                    \
    template void launch_kp_reduce<T>(const T *, int64_t, int64_t, int64_t, int64_t, int64_t, T *,             \
                                      const cg_scalars<T> *, hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
