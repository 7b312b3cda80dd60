// Panelled SELL-64-σ SpMV for the factored sparse-linear K·p.
//
//   out[s] = sum_{entries e of segment s} val[e] * x[index(e)]
//
// used twice per K·p: CSC pass w = X^T p (segments = columns, gathered vector = p) and CSR pass
// raw = X w (segments = rows, gathered vector = w).
//
// Why this layout (measured, tools/spmv_microbench.hip, config 3 = 1M x 50k @ 50 nnz/row, fp32):
//  * a dword gather from global memory costs about one cache-line request per lane: a CSR-vector
//    kernel gathering w / p from global memory runs at 1.2-1.5 TB/s whatever the stream layout, so
//    the gathered vector is cut into panels of W elements (64 KiB) held in LDS. The matrix is stored
//    panel-major and every entry carries a 16-bit panel-local index (6 B per fp32 entry, not 8);
//  * segments of a panel are dealt to lanes: 64 segments form a chunk whose entries are stored
//    lane-interleaved (entry j of the chunk's slot l at chunk_off + 64 j + l), so every load of a
//    wave is one contiguous, coalesced 128 / 256 B line and each lane accumulates its own segment
//    in a register, in entry order — no product buffer, no segment reduction, no atomics.
//    Chunks are padded to their longest segment with (index 0, value 0) entries; segments are
//    sorted by length (descending, stable) inside windows of SELL_SIGMA segments so that padding
//    stays small and a chunk's output stays inside one window (slot -> segment map `perm`);
//  * a workgroup takes a contiguous chunk range of one panel, loads the panel of x into LDS once,
//    and its 16 waves walk the chunks; panel results are partial sums partial[q][s], reduced in
//    panel order (deterministic).
// When the panels would cost more than the stream (P * nseg > nnz / 2: very wide, very sparse
// matrices) the plan uses one panel with 32-bit global indices gathered from global memory.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "buffer.hpp"
#include "fp22.hpp"
#include "kernels.hpp"
#include "cg_common.hpp"

namespace plssvm_mi {

constexpr int SELL_NT = 1024;  // 16 waves per workgroup
constexpr int SELL_WAVES = SELL_NT / 64;
#ifndef SELL_LDS_KB
#define SELL_LDS_KB 160  // LDS panel of the gathered vector (KiB); variants only (tools/variants.sh): 80 = two workgroups per CU
#endif
constexpr int SELL_XBYTES = SELL_LDS_KB * 1024;  // LDS panel of the gathered vector (default: all of a CU's LDS)
constexpr int SELL_WG_PER_CU = 160 / SELL_LDS_KB;
static_assert(SELL_WG_PER_CU * SELL_LDS_KB == 160, "the panel divides the CU's LDS");
constexpr int SELL_SIGMA = 4096;     // sorting window (segments)
// entries per lane in flight per step: the passes are bound by the bytes in flight per CU (one 1024-thread
// workgroup per CU, every step's loads issued together). Measured on one box (round 3, CG it/s): real-typed
// values 4 / 6 / 8 entries: config 3 6 777 / 7 011 / 7 203, 3-RBF 958 / 961 / 969; packed FP22 (8-byte loads
// per value) config 5 778 / 771 / 761 — so 8 for real values, 4 for FP22 (round 2, before the row-block pass
// and the 16-bit pair loads, measured 4 best for both)
#ifndef SELL_SU_REAL
#define SELL_SU_REAL 8  // A/B variants only (tools/variants.sh)
#endif
template <bool F22>
constexpr int sell_unroll() { return F22 ? 4 : SELL_SU_REAL; }
// LDS-panel passes: the 16-bit panel indices of entries 2t, 2t+1 of a slot are adjacent, so one 32-bit load per lane
// (256 B per wave-instruction) fetches two (chunk widths padded to even); packed FP22 values likewise, one 12-byte
// load per lane (3 words at 4-byte alignment) decodes two. (Pairing real values too measured no gain, round 2.)
// storage position of the entry at value position t = off + 64 j + l (off % 128 == 0 when paired)
inline int64_t sell_pair_pos(int64_t t) { return (t & ~int64_t(127)) + 2 * (t & 63) + ((t >> 6) & 1); }
static_assert(sell_unroll<false>() % 2 == 0 && sell_unroll<true>() % 2 == 0, "paired indices need an even step");
template <typename T>
constexpr int sell_width() { return SELL_XBYTES / (int) sizeof(T); }
// workgroups per pass: equal-cost chunk ranges, one per CU (one resident workgroup per CU with a full-LDS panel;
// 512 / 768 / 1024 measured 8 / 14 / 18 % slower on config 3, round 4)
inline int64_t sell_target_blocks() { return 256 * SELL_WG_PER_CU; }

struct sell_chunk {
    int64_t off;    // first entry (entry j of slot l at off + 64 j + l)
    int32_t width;  // entries per slot (longest segment of the chunk)
    int32_t q;      // panel
};

template <bool LDSX>
struct sell_idx {
    using type = int32_t;
};
template <>
struct sell_idx<true> {
    using type = uint16_t;
};

template <typename T>
struct spmv_plan {
    bool ldsx = false;
    int64_t P = 0, nseg = 0, W = 0, nnz = 0, slots_total = 0, entries = 0, nchunks = 0, nblocks = 0;
    int64_t nchp = 0;  // chunks per panel (panel q's chunks are [q nchp, (q + 1) nchp))
    dev_buf<sell_chunk> chunks;
    dev_buf<int32_t> perm;    // [nchunks * 64] slot -> segment (-1: padding slot)
    dev_buf<uint16_t> idx16;  // ldsx: panel-local index
    dev_buf<int32_t> idx32;   // !ldsx: global index
    dev_buf<T> val;
    dev_buf<uint32_t> val22;
    dev_buf<int32_t> bchunk;  // [nblocks + 1]: chunk range of block b (all of one panel)
    dev_buf<T> partial;       // [P][nseg] (P > 1)

    vals_t<T> vals() const { return vals_t<T>{ val.get(), val22.get() }; }
    int64_t bytes() const {
        return chunks.bytes() + perm.bytes() + idx16.bytes() + idx32.bytes() + val.bytes() + val22.bytes() +
               bchunk.bytes() + partial.bytes();
    }
    // bytes one pass moves through HBM: padded index/value stream, slot map, partial slab write + read
    int64_t stream_bytes() const {
        const int64_t vb = val22.get() ? fp22_words(entries) * 4 : entries * (int64_t) sizeof(T);
        return entries * (ldsx ? 2 : 4) + vb + perm.bytes() + chunks.bytes() + (P > 1 ? 2 * partial.bytes() : 0);
    }
};

// FP22: the two words holding the value come as one 8-byte load at 4-byte alignment (gfx950 global
// loads take dword-aligned dwordx2; the packed array carries one word of padding)
typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x3_a4 __attribute__((ext_vector_type(3), aligned(4)));
template <typename T, bool F22>
__device__ __forceinline__ T sell_val(const vals_t<T> &val, int64_t k) {
    if constexpr (F22) {
        const int64_t g = k >> 4;
        const int bit = 22 * (int) (k & 15);
        const uint32_t *w = val.v22 + g * 11 + (bit >> 5);
        const int sh = bit & 31;
        const u32x2_a4 ww = __builtin_nontemporal_load(reinterpret_cast<const u32x2_a4 *>(w));
        return (T) fp22_decode((uint32_t) ((((uint64_t) ww.y << 32) | ww.x) >> sh));
    } else {
        return __builtin_nontemporal_load(val.v + k);
    }
}

// MODE 0: out[s] = sum_e v_e x[i_e]                                   (plain SpMV, KC = 1)
// MODE 1: out[k][s] = sum_e v_e^(k+1) x[i_e], k < KC                  (power moments, KC outputs per segment)
// MODE 2: out[s] = sum_e sum_{k<KC} v_e^(k+1) x[i_e][k]               (KC-channel gathered vector, Horner)
// (the kernel expansion of the sparse poly / rbf K·p, expand.hip, runs MODE 1 over the CSC and MODE 2
// over the CSR of the same data as the factored linear path's two MODE 0 passes)
template <typename T, bool LDSX, bool F22, int KC = 1, int MODE = 0>
__global__ __launch_bounds__(SELL_NT, 4 * SELL_WG_PER_CU) void sell_spmv_kernel(const sell_chunk *__restrict__ chunks,
                                                            const int32_t *__restrict__ perm,
                                                            const typename sell_idx<LDSX>::type *__restrict__ idx,
                                                            vals_t<T> val, const int32_t *__restrict__ bchunk,
                                                            const T *__restrict__ x, int64_t xn, int64_t W,
                                                            int64_t nseg, int nchp, T *__restrict__ out,
                                                            const cg_scalars<T> *__restrict__ status) {
    constexpr int XC = MODE == 2 ? KC : 1;   // channels of the gathered vector
    constexpr int OC = MODE == 1 ? KC : 1;   // outputs per segment
    constexpr int XW = LDSX ? sell_width<T>() : 1;
    constexpr int SU = sell_unroll<F22>();
    using idx_t = typename sell_idx<LDSX>::type;
    __shared__ T xs[XW];
    if (status != nullptr && status->converged) return;
    const int tid = threadIdx.x, lane = tid & 63;
    // XCD-aware: consecutive chunk ranges (the blocks of one panel) share an XCD, so a panel of x is
    // fetched into that XCD's L2 once and the other blocks' fills hit it
    const int blk = (int) xcd_remap(blockIdx.x, gridDim.x);
    const int c0 = bchunk[blk], c1 = bchunk[blk + 1];
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    auto gx = [&](const T *xg, int64_t c) -> T {
        if constexpr (LDSX) return xs[c];
        else return xg[c];
    };
    // the block's chunk range may cross panels (blocks are cut by cost over the whole panel-major chunk
    // sequence): one LDS fill per panel, all waves done with the previous panel first
    for (int cb = c0; cb < c1;) {
        const int q = chunks[cb].q;
        const int ce = min(c1, (q + 1) * nchp);  // chunks of panel q are [q nchp, (q + 1) nchp)
        T *o = out + (int64_t) q * nseg * OC;
        const T *xg = x + (int64_t) q * W * XC;  // LDSX: panel q gathers x[q W + local]; otherwise W = 0
        if constexpr (LDSX) {
            if (cb != c0) __syncthreads();
            const int xl = (int) min((int64_t) W, xn - (int64_t) q * W) * XC;
            // 16-byte loads and LDS stores (XW is a multiple of 16 B per thread); a misaligned panel
            // start (the CSC pass of a group rank gathers p + r0) or the ragged last panel go per element
            using V = __attribute__((ext_vector_type(4))) float;
            constexpr int EV = 16 / (int) sizeof(T);  // elements per vector
            constexpr int VPER = XW / EV / SELL_NT;
            static_assert(VPER * EV * SELL_NT == XW, "panel width must be a multiple of 16 B per thread");
            if (xl == XW && (reinterpret_cast<uintptr_t>(xg) & 15) == 0) {
                V t[VPER];
#pragma unroll
                for (int u = 0; u < VPER; ++u) t[u] = reinterpret_cast<const V *>(xg)[tid + u * SELL_NT];
#pragma unroll
                for (int u = 0; u < VPER; ++u) reinterpret_cast<V *>(xs)[tid + u * SELL_NT] = t[u];
            } else {
                constexpr int XPER = XW / SELL_NT;
                for (int u = 0; u < XPER; ++u) {
                    const int k = tid + u * SELL_NT;
                    xs[k] = k < xl ? xg[k] : T(0);
                }
            }
            __syncthreads();
        }
        for (int c = cb + wave; c < ce; c += SELL_WAVES) {
            const sell_chunk ch = chunks[c];
            const int seg = perm[(int64_t) c * 64 + lane];
            const int64_t base = ch.off + lane;
            // steps of SU entries; a step past the width re-reads the slot's last entry (same
            // cache line) and masks it, so every step issues all of its loads at once
            const int last = max(ch.width - 1, 0);
            T acc[OC];
#pragma unroll
            for (int k = 0; k < OC; ++k) acc[k] = T(0);
            for (int j = 0; j < ch.width; j += SU) {
                idx_t ci[SU];
                T vi[SU];
#pragma unroll
                for (int u = 0; u < SU; ++u) {
                    const int64_t k = base + (int64_t) min(j + u, last) * 64;
                    if constexpr (!LDSX) ci[u] = __builtin_nontemporal_load(idx + k);
                    if constexpr (!(LDSX && F22)) vi[u] = sell_val<T, F22>(val, k);
                }
                if constexpr (LDSX && F22) {
                    // entries jj, jj + 1 (jj even) of this slot at stream positions p, p + 1, p = off + 128 (jj / 2) + 2 lane:
                    // bits 22 p .. 22 p + 43 lie in the 3 words from (22 p) / 32 (shift 22 p % 32 <= 28)
                    const int lastp = max((ch.width >> 1) - 1, 0);
#pragma unroll
                    for (int u2 = 0; u2 < SU / 2; ++u2) {
                        const int64_t pp = ch.off + 128 * (int64_t) min((j >> 1) + u2, lastp) + 2 * lane;
                        const int64_t bit = 22 * pp;
                        const u32x3_a4 ww = __builtin_nontemporal_load(reinterpret_cast<const u32x3_a4 *>(val.v22 + (bit >> 5)));
                        const int sh = (int) (bit & 31);
                        const uint64_t lo = ((uint64_t) ww.y << 32) | ww.x;
                        const uint32_t c0 = (uint32_t) (lo >> sh) & 0x3FFFFFu;
                        const int sh1 = sh + 22;  // 22..50: the second value straddles words 1 and 2 when sh1 > 32
                        const uint64_t hi = ((uint64_t) ww.z << 32) | ww.y;
                        const uint32_t c1 = (uint32_t) (sh1 >= 32 ? hi >> (sh1 - 32) : lo >> sh1) & 0x3FFFFFu;
                        vi[2 * u2] = (T) fp22_decode(c0);
                        vi[2 * u2 + 1] = (T) fp22_decode(c1);
                    }
                }
                if constexpr (LDSX) {
                    const uint32_t *ip = reinterpret_cast<const uint32_t *>(idx) + (ch.off >> 1) + lane;
                    const int lastp = max((ch.width >> 1) - 1, 0);
#pragma unroll
                    for (int u2 = 0; u2 < SU / 2; ++u2) {
                        const uint32_t pr = __builtin_nontemporal_load(ip + (int64_t) min((j >> 1) + u2, lastp) * 64);
                        ci[2 * u2] = (idx_t) (pr & 0xFFFFu);
                        ci[2 * u2 + 1] = (idx_t) (pr >> 16);
                    }
                }
#pragma unroll
                for (int u = 0; u < SU; ++u) {
                    const T v = j + u < ch.width ? vi[u] : T(0);
                    if constexpr (MODE == 0) {
                        acc[0] = fma(v, gx(xg, (int64_t) ci[u]), acc[0]);
                    } else if constexpr (MODE == 1) {
                        T t = v * gx(xg, (int64_t) ci[u]);
#pragma unroll
                        for (int k = 0; k < KC; ++k) {
                            acc[k] += t;
                            t *= v;
                        }
                    } else {
                        const int64_t cx = (int64_t) ci[u] * KC;
                        T h = gx(xg, cx + KC - 1);
#pragma unroll
                        for (int k = KC - 2; k >= 0; --k) h = fma(h, v, gx(xg, cx + k));
                        acc[0] = fma(h, v, acc[0]);
                    }
                }
            }
            if (seg >= 0) {
#pragma unroll
                for (int k = 0; k < OC; ++k) o[(int64_t) k * nseg + seg] = acc[k];
            }
        }
        cb = ce;
    }
}

// out[s] = sum_q partial[q][s]. Many panels (split): a block of 256 threads takes 64 segments and its
// 4 waves each sum one quarter of the panels (coalesced 64-segment rows, 8 loads in flight); the
// quarters are added in order through LDS — a fixed order, so deterministic. The CSC pass has few
// segments and many panels: splitting its panel loop gives it 4x the memory parallelism of one
// thread per segment. Few panels: one thread per segment (256 segments per block).
template <typename T>
__global__ __launch_bounds__(256) void panel_reduce_kernel(const T *__restrict__ partial, int64_t P, int64_t nseg,
                                                           int split, T *__restrict__ out,
                                                           const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    __shared__ T part[3][64];
    const int lane = split ? (threadIdx.x & 63) : threadIdx.x, quarter = split ? (threadIdx.x >> 6) : 0;
    const int64_t s = (int64_t) blockIdx.x * (split ? 64 : 256) + lane;
    const int64_t per = split ? (P + 3) / 4 : P, q0 = quarter * per, q1 = min(P, q0 + per);
    T a = 0;
    if (s < nseg) {
        int64_t q = q0;
        for (; q + 8 <= q1; q += 8) {
            T v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = partial[(q + u) * nseg + s];
#pragma unroll
            for (int u = 0; u < 8; ++u) a += v[u];
        }
        for (; q < q1; ++q) a += partial[q * nseg + s];
    }
    if (!split) {
        if (s < nseg) out[s] = a;
        return;
    }
    if (quarter > 0) part[quarter - 1][lane] = a;
    __syncthreads();
    if (quarter == 0 && s < nseg) out[s] = ((a + part[0][lane]) + part[1][lane]) + part[2][lane];
}

// out[0..nseg) = the pass result (partial slabs + reduction when P > 1). kc / mode: see sell_spmv_kernel
// (mode 1 writes kc outputs per segment, out[k * nseg + s]; mode 2 gathers kc channels x[i * kc + k]);
// the plan must have been built with the same channel counts.
template <typename T, int KC, int MODE>
inline void launch_panel_spmv_t(const spmv_plan<T> &pl, const T *x, int64_t xn, T *out, const cg_scalars<T> *status,
                                hipStream_t stream) {
    const bool f22 = pl.val22.get() != nullptr;
    T *dst = pl.P > 1 ? pl.partial.get() : out;
    const dim3 grid((unsigned) pl.nblocks), block(SELL_NT);
    if (pl.ldsx) {
        auto k = f22 ? sell_spmv_kernel<T, true, true, KC, MODE> : sell_spmv_kernel<T, true, false, KC, MODE>;
        hipLaunchKernelGGL(k, grid, block, 0, stream, pl.chunks.get(), pl.perm.get(), pl.idx16.get(), pl.vals(),
                           pl.bchunk.get(), x, xn, pl.W, pl.nseg, (int) pl.nchp, dst, status);
    } else {
        auto k = f22 ? sell_spmv_kernel<T, false, true, KC, MODE> : sell_spmv_kernel<T, false, false, KC, MODE>;
        hipLaunchKernelGGL(k, grid, block, 0, stream, pl.chunks.get(), pl.perm.get(), pl.idx32.get(), pl.vals(),
                           pl.bchunk.get(), x, xn, (int64_t) 0, pl.nseg, (int) pl.nchp, dst, status);
    }
    MI_LAUNCH_CHECK();
}

// reduce = false (mode 0 only): a multi-panel pass leaves its P partial slabs in pl.partial for the
// consumer to sum in panel order (cg_fin_dad_kernel), out is not written
template <typename T>
inline void launch_panel_spmv(const spmv_plan<T> &pl, const T *x, int64_t xn, T *out, const cg_scalars<T> *status,
                              hipStream_t stream, int kc = 1, int mode = 0, bool reduce = true) {
    if (pl.nseg <= 0 || pl.nblocks <= 0) return;
    if (mode == 0) {
        launch_panel_spmv_t<T, 1, 0>(pl, x, xn, out, status, stream);
    } else if (mode == 1) {
        switch (kc) {
            case 2: launch_panel_spmv_t<T, 2, 1>(pl, x, xn, out, status, stream); break;
            case 4: launch_panel_spmv_t<T, 4, 1>(pl, x, xn, out, status, stream); break;
            case 8: launch_panel_spmv_t<T, 8, 1>(pl, x, xn, out, status, stream); break;
            default: launch_panel_spmv_t<T, 16, 1>(pl, x, xn, out, status, stream);
        }
    } else {
        switch (kc) {
            case 2: launch_panel_spmv_t<T, 2, 2>(pl, x, xn, out, status, stream); break;
            case 4: launch_panel_spmv_t<T, 4, 2>(pl, x, xn, out, status, stream); break;
            case 8: launch_panel_spmv_t<T, 8, 2>(pl, x, xn, out, status, stream); break;
            default: launch_panel_spmv_t<T, 16, 2>(pl, x, xn, out, status, stream);
        }
    }
    if (pl.P > 1 && reduce) {
        const int64_t ns = pl.nseg * (mode == 1 ? kc : 1);
        const int split = pl.P >= 16 ? 1 : 0;
        hipLaunchKernelGGL(panel_reduce_kernel<T>, dim3((unsigned) ceil_div(ns, split ? 64 : 256)), dim3(256), 0,
                           stream, pl.partial.get(), pl.P, ns, split, out, status);
        MI_LAUNCH_CHECK();
    }
}

// packed FP22 words of v (16 values per 11 words, fp22_words(n) + 2 words: the paired 3-word loads may read 2 past
// the last), groups on the host threads
inline std::vector<uint32_t> fp22_pack_host(const std::vector<float> &v) {
    const int64_t n = (int64_t) v.size(), groups = (n + 15) / 16;
    std::vector<uint32_t> words((size_t) (fp22_words(n) + 2), 0u);
    host_parallel(groups, [&](int, int64_t g0, int64_t g1) {
        for (int64_t g = g0; g < g1; ++g)
            for (int k = 0; k < 16 && g * 16 + k < n; ++k) {
                const uint64_t code = fp22_encode_host(v[(size_t) (g * 16 + k)]);
                const int bit = 22 * k;
                const int64_t wi = g * 11 + (bit >> 5);
                const int sh = bit & 31;
                words[(size_t) wi] |= (uint32_t) (code << sh);
                if (sh > 10) words[(size_t) wi + 1] |= (uint32_t) (code >> (32 - sh));
            }
    });
    return words;
}

// Host construction. gen(emit, s0, s1) must call emit(s, global_index, value) for every entry of the
// segments s in [s0, s1), the entries of one segment in their summation order (for each panel); it is
// called from several host threads on disjoint segment ranges. xn = length of the gathered vector.
// target_blocks: workgroups per pass (each loads its panel of x once). force_mode: 0 auto,
// 1 LDS panels, 2 one panel gathered from global memory.
// xch: channels of the gathered vector (mode 2 passes: the LDS panel holds sell_width / xch indices);
// och: outputs per segment (mode 1 passes: the partial slab holds och values per segment).
template <typename T, typename Gen>
void build_spmv_plan(spmv_plan<T> &pl, int64_t nseg, int64_t xn, int64_t nnz, bool fp22, Gen gen, int64_t target_blocks,
                     hipStream_t stream, int force_mode = 0, int xch = 1, int och = 1) {
    pl = spmv_plan<T>{};
    pl.nseg = nseg;
    pl.nnz = nnz;
    if (nseg <= 0) return;
    phase_timer pt;
    const int64_t Wmax = sell_width<T>() / xch;
    const int64_t P_lds = std::max<int64_t>(1, ceil_div(std::max<int64_t>(xn, 1), Wmax));
    bool ldsx = P_lds * (nseg + 1) * 2 <= std::max<int64_t>(nnz, 1);
    if (force_mode == 1) ldsx = true;
    if (force_mode == 2) ldsx = false;
    pl.ldsx = ldsx;
    pl.P = ldsx ? P_lds : 1;
    pl.W = ldsx ? Wmax : std::max<int64_t>(xn, 1);
    const int64_t P = pl.P, W = pl.W;
    // segment lengths per panel (segment ranges on the host threads: each length has one writer)
    std::vector<int32_t> len((size_t) (P * nseg), 0);
    host_parallel(nseg, [&](int, int64_t s0, int64_t s1) {
        gen([&](int64_t s, int64_t g, double) { ++len[(size_t) ((g / W) * nseg + s)]; }, s0, s1);
    });
    pt.mark("  SELL plan: segment lengths");
    // per panel: sort windows by length (descending, stable), deal 64 slots per chunk
    const int64_t slots_per_panel = round_up(nseg, 64);
    const int64_t nch_per_panel = slots_per_panel / 64;
    std::vector<sell_chunk> chunks((size_t) (P * nch_per_panel));
    std::vector<int32_t> perm((size_t) (P * slots_per_panel), -1);
    std::vector<int64_t> pos((size_t) (P * nseg));  // next storage position of segment (q, s)
    const int64_t nwin = ceil_div(nseg, (int64_t) SELL_SIGMA);
    host_parallel(P * nwin, [&](int, int64_t a, int64_t b) {
        std::vector<int32_t> order;
        for (int64_t task = a; task < b; ++task) {
            const int64_t q = task / nwin, w0 = (task % nwin) * SELL_SIGMA;
            const int32_t *lq = len.data() + q * nseg;
            const int64_t w1 = std::min(nseg, w0 + (int64_t) SELL_SIGMA);
            order.resize((size_t) (w1 - w0));
            std::iota(order.begin(), order.end(), (int32_t) w0);
            std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return lq[x] > lq[y]; });
            // the slots of this window are [w0, w1) (SELL_SIGMA is a multiple of 64)
            for (int64_t k = 0; k < (int64_t) order.size(); ++k) perm[(size_t) (q * slots_per_panel + w0 + k)] = order[k];
        }
    });
    int64_t off = 0;
    for (int64_t q = 0; q < P; ++q) {
        const int32_t *lq = len.data() + q * nseg;
        for (int64_t c = 0; c < nch_per_panel; ++c) {
            int32_t width = 0;
            for (int l = 0; l < 64; ++l) {
                const int32_t sgm = perm[(size_t) (q * slots_per_panel + c * 64 + l)];
                if (sgm >= 0) width = std::max(width, lq[sgm]);
            }
            if (ldsx) width = (width + 1) & ~1;  // paired indices: even widths, off % 128 == 0
            chunks[(size_t) (q * nch_per_panel + c)] = sell_chunk{ off, width, (int32_t) q };
            for (int l = 0; l < 64; ++l) {
                const int32_t sgm = perm[(size_t) (q * slots_per_panel + c * 64 + l)];
                if (sgm >= 0) pos[(size_t) (q * nseg + sgm)] = off + l;
            }
            off += (int64_t) width * 64;
        }
    }
    pt.mark("  SELL plan: order + chunks");
    pl.entries = off;
    pl.nchunks = (int64_t) chunks.size();
    pl.nchp = nch_per_panel;
    pl.slots_total = P * slots_per_panel;
    // fill (zero padding: index 0, value 0 contributes exactly 0) plus a 64-entry zero tail; segment ranges
    // on the host threads (disjoint slots; FP22 words hold several segments' values, so they are packed
    // afterwards from a float copy, 16-value groups per thread)
    const int64_t cap = off + 64;
    std::vector<uint16_t> i16(ldsx ? cap : 0, 0);
    std::vector<int32_t> i32(ldsx ? 0 : cap, 0);
    std::vector<T> vr(fp22 ? 0 : cap, T(0));
    std::vector<float> vf(fp22 ? cap : 0, 0.0f);
    host_parallel(nseg, [&](int, int64_t s0, int64_t s1) {
        gen([&](int64_t s, int64_t g, double v) {
            const int64_t q = g / W;
            int64_t &p = pos[(size_t) (q * nseg + s)];
            const int64_t t = p;
            p += 64;
            if (ldsx) {
                // IDX2: entry j of slot l (value position t = off + 64 j + l) keeps its index at
                // off + 128 (j >> 1) + 2 l + (j & 1)
                i16[sell_pair_pos(t)] = (uint16_t) (g - q * W);
            }
            else i32[t] = (int32_t) g;
            const int64_t tv = (fp22 && ldsx) ? sell_pair_pos(t) : t;  // value position
            if (fp22) vf[tv] = (float) v;
            else vr[tv] = (T) v;
        }, s0, s1);
    });
    pt.mark("  SELL plan: fill");
    const std::vector<uint32_t> v22 = fp22 ? fp22_pack_host(vf) : std::vector<uint32_t>{};
    pt.mark("  SELL plan: FP22 pack");
    // blocks: target_blocks contiguous chunk ranges of equal cost (entries + a per-chunk charge for its
    // descriptor, slot map and output) over the panel-major chunk sequence; a range may cross panels
    constexpr int64_t CHUNK_COST = 8 * 64;
    auto cost = [&](const sell_chunk &c) { return (int64_t) c.width * 64 + CHUNK_COST; };
    int64_t total_cost = 0;
    for (const auto &c : chunks) total_cost += cost(c);
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(target_blocks, (int64_t) chunks.size()));
    std::vector<int32_t> bchunk{ 0 };
    {
        int64_t acc = 0, k = 1;
        for (int64_t i = 0; i < (int64_t) chunks.size(); ++i) {
            acc += cost(chunks[(size_t) i]);
            if (i + 1 < (int64_t) chunks.size() && k < nb && acc * nb >= k * total_cost) {
                bchunk.push_back((int32_t) (i + 1));
                ++k;
            }
        }
        bchunk.push_back((int32_t) chunks.size());
    }
    pl.nblocks = (int64_t) bchunk.size() - 1;
    auto up = [&](auto &buf, const auto &vec) {
        using E = typename std::decay_t<decltype(vec)>::value_type;
        if (vec.empty()) return;
        buf.alloc((int64_t) vec.size(), stream, false);
        MI_HIP_CHECK(hipMemcpyAsync(buf.get(), vec.data(), sizeof(E) * vec.size(), hipMemcpyHostToDevice, stream));
    };
    up(pl.chunks, chunks);
    up(pl.perm, perm);
    up(pl.idx16, i16);
    up(pl.idx32, i32);
    up(pl.val, vr);
    up(pl.val22, v22);
    up(pl.bchunk, bchunk);
    if (P > 1) pl.partial.alloc(P * nseg * och, stream, false);
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    pt.mark("  SELL plan: blocks + upload");
}

// ---- row-block CSR pass with the CG finalize fused (factored sparse linear, one GPU) ------------------
// raw = X w for a block of RBK rows owned by one 1024-thread workgroup: for each panel q of w (LDS), the
// block's rows sorted by their panel-q length (descending) are dealt 64 per chunk to the waves, and each
// lane adds its row's panel-q sum into an LDS row accumulator (every row once per panel, panels in
// order: bitwise the (0 + slab0) + slab1 + ... of the panelled pass). The epilogue is cg_fin_dad's:
// Ad_i = raw_i + (QA - q_i) sum(d) - sum(q d) + d_i / C, one d.Ad partial per block — no panel slabs,
// no separate finalize launch.
template <typename T>
constexpr int rb_rows() { return 16384 / (int) sizeof(T); }  // row accumulator: 16 KiB
template <typename T>
constexpr int rb_width() { return (163840 - 16384) / (int) sizeof(T) / 1024 * 1024; }  // panel: the rest

template <typename T>
struct rb_plan {
    int64_t P = 0, W = 0, RBK = 0, nblk = 0, nrows = 0, entries = 0;
    dev_buf<sell_chunk> chunks;  // ordered (block, panel, chunk)
    dev_buf<int32_t> perm;       // [nchunks * 64] slot -> block-local row (-1: padding)
    dev_buf<uint16_t> idx16;     // panel-local index, IDX2 pair layout
    dev_buf<T> val;
    dev_buf<uint32_t> val22;
    dev_buf<int32_t> bpc;        // [nblk * P + 1]: chunk range of (block, panel)
    vals_t<T> vals() const { return vals_t<T>{ val.get(), val22.get() }; }
    int64_t bytes() const {
        return chunks.bytes() + perm.bytes() + idx16.bytes() + val.bytes() + val22.bytes() + bpc.bytes();
    }
    int64_t stream_bytes() const {
        const int64_t vb = val22.get() ? fp22_words(entries) * 4 : entries * (int64_t) sizeof(T);
        return entries * 2 + vb + perm.bytes() + chunks.bytes();
    }
};

template <typename T, bool F22>
__global__ __launch_bounds__(SELL_NT) void sell_rowblock_fin_kernel(
    const sell_chunk *__restrict__ chunks, const int32_t *__restrict__ perm, const uint16_t *__restrict__ idx,
    vals_t<T> val, const int32_t *__restrict__ bpc, int64_t P, int64_t W, int64_t RBK, const T *__restrict__ x,
    int64_t xn, int64_t nrows, const T *__restrict__ q, const T *__restrict__ d, const T *__restrict__ psum,
    T QA_cost, T cost_inv, T *__restrict__ Ad, T *__restrict__ pdad, const cg_scalars<T> *__restrict__ status) {
    constexpr int XW = rb_width<T>(), RB = rb_rows<T>();
    constexpr int SU = sell_unroll<F22>();
    constexpr int RPT = (RB + SELL_NT - 1) / SELL_NT;  // rows per thread
    __shared__ T xs[XW];
    __shared__ T racc[RB];
    T *red = racc, *bc = racc + SELL_WAVES;  // block-reduction scratch (before / after the accumulator's use)
    if (status != nullptr && status->converged) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int blk = (int) blockIdx.x;
    const int64_t row0 = (int64_t) blk * RBK;
    const int rows = (int) min<int64_t>(RBK, nrows - row0);
    // sum(d), sum(q d) from the previous step's RED_BLOCKS partial pairs, in dot_final_kernel's order
    T sp, sqp;
    {
        T s1 = 0, s2 = 0;
        for (int i = tid; i < RED_BLOCKS; i += SELL_NT) {
            s1 += psum[i];
            s2 += psum[RED_BLOCKS + i];
        }
        auto bsum = [&](T v) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            if (lane == 0) red[wave] = v;
            __syncthreads();
            if (tid == 0) {
                T t = 0;
                for (int w2 = 0; w2 < SELL_WAVES; ++w2) t += red[w2];
                bc[0] = t;
            }
            __syncthreads();
            const T out = bc[0];
            __syncthreads();
            return out;
        };
        sp = bsum(s1);
        sqp = bsum(s2);
    }
    for (int t = tid; t < RB; t += SELL_NT) racc[t] = T(0);  // visible after the first panel fill's barrier
    for (int64_t qq = 0; qq < P; ++qq) {
        const T *xg = x + qq * W;
        {
            if (qq > 0) __syncthreads();  // every wave is done with panel qq - 1
            const int xl = (int) min((int64_t) W, xn - qq * W);
            using V = __attribute__((ext_vector_type(4))) float;
            constexpr int EV = 16 / (int) sizeof(T);
            constexpr int VPER = XW / EV / SELL_NT;
            static_assert(VPER * EV * SELL_NT == XW, "panel width must be a multiple of 16 B per thread");
            if (xl == XW && (reinterpret_cast<uintptr_t>(xg) & 15) == 0) {
                V t[VPER];
#pragma unroll
                for (int u = 0; u < VPER; ++u) t[u] = reinterpret_cast<const V *>(xg)[tid + u * SELL_NT];
#pragma unroll
                for (int u = 0; u < VPER; ++u) reinterpret_cast<V *>(xs)[tid + u * SELL_NT] = t[u];
            } else {
                for (int k = tid; k < XW; k += SELL_NT) xs[k] = k < xl ? xg[k] : T(0);
            }
            __syncthreads();
        }
        const int cb = bpc[blk * P + qq], ce = bpc[blk * P + qq + 1];
        for (int c = cb + wave; c < ce; c += SELL_WAVES) {
            const sell_chunk ch = chunks[c];
            const int seg = perm[(int64_t) c * 64 + lane];
            const int64_t base = ch.off + lane;
            const int last = max(ch.width - 1, 0);
            const int lastp = max((ch.width >> 1) - 1, 0);
            const uint32_t *ip = reinterpret_cast<const uint32_t *>(idx) + (ch.off >> 1) + lane;
            T acc = T(0);
            for (int j = 0; j < ch.width; j += SU) {
                uint16_t ci[SU];
                T vi[SU];
#pragma unroll
                for (int u = 0; u < SU; ++u) vi[u] = sell_val<T, F22>(val, base + (int64_t) min(j + u, last) * 64);
#pragma unroll
                for (int u2 = 0; u2 < SU / 2; ++u2) {
                    const uint32_t pr = __builtin_nontemporal_load(ip + (int64_t) min((j >> 1) + u2, lastp) * 64);
                    ci[2 * u2] = (uint16_t) (pr & 0xFFFFu);
                    ci[2 * u2 + 1] = (uint16_t) (pr >> 16);
                }
#pragma unroll
                for (int u = 0; u < SU; ++u) {
                    const T v = j + u < ch.width ? vi[u] : T(0);
                    acc = fma(v, xs[ci[u]], acc);
                }
            }
            if (seg >= 0) racc[seg] += acc;  // each row once per panel
        }
    }
    __syncthreads();
    T s1 = 0;
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int t = tid + u * SELL_NT;
        if (t >= rows) break;
        const int64_t i = row0 + t;
        const T rw = racc[t], qi = q[i], di = d[i];
        T v;
        {
#pragma clang fp contract(fast)  // cg_fin_dad_kernel's expression
            v = rw + (QA_cost - qi) * sp - sqp + cost_inv * di;
            v = T(0) + T(1) * v;
        }
        Ad[i] = v;
        s1 += di * v;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s1 += __shfl_xor(s1, o);
    __syncthreads();  // every row of the accumulator has been read: reuse it as scratch
    if (lane == 0) red[wave] = s1;
    __syncthreads();
    if (tid == 0) {
        T t = 0;
        for (int w2 = 0; w2 < SELL_WAVES; ++w2) t += red[w2];
        pdad[blk] = t;
    }
    // the consumer sums RED_BLOCKS partials: the slots past this launch's blocks are zero
    if (blk == 0)
        for (int b = (int) gridDim.x + tid; b < RED_BLOCKS; b += SELL_NT) pdad[b] = T(0);
}

template <typename T>
inline void launch_rowblock_fin(const rb_plan<T> &pl, const T *w, int64_t xn, const T *q, const T *d, const T *psum,
                                T QA_cost, T cost_inv, T *Ad, T *pdad, const cg_scalars<T> *status,
                                hipStream_t stream) {
    if (pl.nblk <= 0) return;
    auto k = pl.val22.get() ? sell_rowblock_fin_kernel<T, true> : sell_rowblock_fin_kernel<T, false>;
    hipLaunchKernelGGL(k, dim3((unsigned) pl.nblk), dim3(SELL_NT), 0, stream, pl.chunks.get(), pl.perm.get(),
                       pl.idx16.get(), pl.vals(), pl.bpc.get(), pl.P, pl.W, pl.RBK, w, xn, pl.nrows, q, d, psum,
                       QA_cost, cost_inv, Ad, pdad, status);
    MI_LAUNCH_CHECK();
}

// Host construction (rows = segments s in [0, nrows), gathered vector of length xn); gen as for
// build_spmv_plan. Returns false (plan left empty) when the rows need more than RED_BLOCKS blocks.
template <typename T, typename Gen>
bool build_rowblock_plan(rb_plan<T> &pl, int64_t nrows, int64_t xn, bool fp22, Gen gen, int64_t target_blocks,
                         hipStream_t stream) {
    pl = rb_plan<T>{};
    if (nrows <= 0) return false;
    const int64_t W = rb_width<T>(), P = std::max<int64_t>(1, ceil_div(std::max<int64_t>(xn, 1), W));
    const int64_t RBK = std::min<int64_t>(rb_rows<T>(), round_up(ceil_div(nrows, target_blocks), 64));
    const int64_t nblk = ceil_div(nrows, RBK);
    if (nblk > RED_BLOCKS) return false;
    pl.P = P, pl.W = W, pl.RBK = RBK, pl.nblk = nblk, pl.nrows = nrows;
    std::vector<int32_t> len((size_t) (P * nrows), 0);
    host_parallel(nrows, [&](int, int64_t s0, int64_t s1) {
        gen([&](int64_t s, int64_t g, double) { ++len[(size_t) ((g / W) * nrows + s)]; }, s0, s1);
    });
    const int64_t cpb = RBK / 64;  // chunks per (block, panel)
    std::vector<sell_chunk> chunks((size_t) (nblk * P * cpb));
    std::vector<int32_t> perm(chunks.size() * 64, -1);
    std::vector<int64_t> pos((size_t) (P * nrows));
    std::vector<int32_t> bpc{ 0 };
    // each (block, panel)'s rows sorted by their panel length (descending, stable), on the host threads
    std::vector<std::vector<int32_t>> orders((size_t) (nblk * P));
    host_parallel(nblk * P, [&](int, int64_t a, int64_t b) {
        for (int64_t task = a; task < b; ++task) {
            const int64_t blk = task / P, qq = task % P;
            const int64_t r0 = blk * RBK, r1 = std::min(nrows, r0 + RBK);
            const int32_t *lq = len.data() + qq * nrows;
            auto &order = orders[(size_t) task];
            order.resize((size_t) (r1 - r0));
            std::iota(order.begin(), order.end(), (int32_t) r0);
            std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return lq[x] > lq[y]; });
        }
    });
    int64_t off = 0, c = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        const int64_t r0 = b * RBK;
        for (int64_t qq = 0; qq < P; ++qq) {
            const int32_t *lq = len.data() + qq * nrows;
            const auto &order = orders[(size_t) (b * P + qq)];
            for (int64_t k = 0; k < cpb; ++k, ++c) {
                int32_t width = 0;
                for (int l = 0; l < 64; ++l) {
                    const int64_t t = k * 64 + l;
                    if (t < (int64_t) order.size()) width = std::max(width, lq[order[(size_t) t]]);
                }
                width = (width + 1) & ~1;  // IDX2 pairs
                chunks[(size_t) c] = sell_chunk{ off, width, (int32_t) qq };
                for (int l = 0; l < 64; ++l) {
                    const int64_t t = k * 64 + l;
                    if (t < (int64_t) order.size()) {
                        const int32_t row = order[(size_t) t];
                        perm[(size_t) (c * 64 + l)] = (int32_t) (row - r0);
                        pos[(size_t) (qq * nrows + row)] = off + l;
                    }
                }
                off += (int64_t) width * 64;
            }
            bpc.push_back((int32_t) c);
        }
    }
    pl.entries = off;
    const int64_t cap = off + 128;
    std::vector<uint16_t> i16((size_t) cap, 0);
    std::vector<T> vr(fp22 ? 0 : (size_t) cap, T(0));
    std::vector<float> vf(fp22 ? (size_t) cap : 0, 0.0f);
    host_parallel(nrows, [&](int, int64_t s0, int64_t s1) {
        gen([&](int64_t s, int64_t g, double v) {
            const int64_t qq = g / W;
            int64_t &p = pos[(size_t) (qq * nrows + s)];
            const int64_t t = p;
            p += 64;
            i16[(size_t) sell_pair_pos(t)] = (uint16_t) (g - qq * W);
            if (fp22) vf[(size_t) t] = (float) v;
            else vr[(size_t) t] = (T) v;
        }, s0, s1);
    });
    const std::vector<uint32_t> v22 = fp22 ? fp22_pack_host(vf) : std::vector<uint32_t>{};
    auto up = [&](auto &buf, const auto &vec) {
        using E = typename std::decay_t<decltype(vec)>::value_type;
        if (vec.empty()) return;
        buf.alloc((int64_t) vec.size(), stream, false);
        MI_HIP_CHECK(hipMemcpyAsync(buf.get(), vec.data(), sizeof(E) * vec.size(), hipMemcpyHostToDevice, stream));
    };
    up(pl.chunks, chunks);
    up(pl.perm, perm);
    up(pl.idx16, i16);
    up(pl.val, vr);
    up(pl.val22, v22);
    up(pl.bpc, bpc);
    MI_HIP_CHECK(hipStreamSynchronize(stream));
    return true;
}

}  // namespace plssvm_mi
