// Implicit pairwise K·p tiles on MFMA (gfx950) — the dense hot kernel.
//
// Replaces device_kernel_{linear,poly,radial} (include/plssvm/backends/HIP/svm_kernel.hip.hpp:36-268)
// and its OpenMP twin (src/plssvm/backends/OpenMP/svm_kernel.cpp:21-47). Per 128x128 lower-triangle
// tile (I >= J) of k(x_i, x_j):
//   * X is feature-major in HBM (XT[k][i]); each BK-deep K chunk of the two 128-column panels is
//     streamed global -> LDS with buffer_load_dwordx4 ... lds (1 KiB per wave-instruction, no VGPR
//     staging; scalar descriptor base + constant per-lane offset, so no VALU address math in the K
//     loop), double-buffered so chunk kc+1 lands while chunk kc feeds the MFMAs: one barrier per
//     chunk;
//   * 4 waves as 2x2, each a 64x64 sub-tile = 4x4 accumulators of v_mfma_f64_16x16x4_f64 /
//     v_mfma_f32_16x16x4_f32 (exact fma chains in k order);
//   * epilogue in registers: kernel function (RBF via ||a||^2 + ||b||^2 - 2 a.b, clamped at 0),
//     times p_j -> row sums (16-lane shuffles) and times p_i -> mirrored column sums (cross-half
//     shuffles); results go to the tile's own 256-value record of the rank's slab (row sums, then
//     column sums: the slab holds only this rank's tiles, so it shrinks with the group) — no atomics,
//     so a fixed-order second pass makes K·p bitwise reproducible;
//   * tiles are visited in 8x8 super-blocks (16 panels = 4 MiB in fp64: one XCD's L2) and the
//     workgroup ids are remapped so each XCD walks a contiguous range of super-blocks.
#include <cstdlib>

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

// exp for the fp64 RBF epilogue, in the scaled domain y = x * 256 / ln2 (x = -gamma * dist <= 0):
// exp(x) = 2^(j >> 8) * 2^((j & 255) / 256) * e^(r ln2 / 256), j = rint(y), r = y - j in [-1/2, 1/2];
// 2^(i/256) from a 256-entry LDS table (correctly rounded), e^(r ln2/256) by a degree-4 polynomial
// (truncation < 4e-17 relative). 9 fp64 VALU + 3 integer + 1 LDS read per element instead of ~26
// for dist + libm exp: on gfx950 every VALU cycle of the epilogue is a cycle of the fp64 MFMA pipe
// (DESIGN.md §3.1), so the instruction count is what matters. No clamp of y at 0: the norm trick can
// round dist to -1e-16 relative, giving exp of a tiny positive number (as harmless as the clamp).
// The rounding of y (|y| < ~1500 on the BASELINE data) adds < 2e-15 relative error.
__constant__ double c_exp2_256[256] = {
    1.0, 1.0027112750502025, 1.0054299011128027, 1.0081558981184175,
    1.0108892860517005, 1.0136300849514894, 1.016378314910953, 1.019133996077738,
    1.0218971486541166, 1.0246677928971357, 1.0274459491187637, 1.030231637686041,
    1.0330248790212284, 1.0358256936019572, 1.0386341019613787, 1.041450124688316,
    1.0442737824274138, 1.0471050958792898, 1.0499440858006872, 1.0527907730046264,
    1.0556451783605572, 1.0585073227945128, 1.061377227289262, 1.0642549128844645,
    1.0671404006768237, 1.0700337118202419, 1.0729348675259756, 1.075843889062791,
    1.0787607977571199, 1.0816856149932152, 1.0846183622133092, 1.0875590609177697,
    1.0905077326652577, 1.0934643990728858, 1.0964290818163769, 1.099401802630222,
    1.102382583307841, 1.1053714457017412, 1.1083684117236787, 1.1113735033448175,
    1.1143867425958924, 1.1174081515673693, 1.1204377524096067, 1.12347556733302,
    1.1265216186082418, 1.129575928566288, 1.1326385195987192, 1.1357094141578055,
    1.1387886347566916, 1.1418762039695616, 1.1449721444318042, 1.148076478840179,
    1.1511892299529827, 1.154310420590216, 1.1574400736337511, 1.1605782120274988,
    1.1637248587775775, 1.1668800369524817, 1.1700437696832502, 1.1732160801636373,
    1.1763969916502812, 1.1795865274628758, 1.182784710984341, 1.1859915656609938,
    1.189207115002721, 1.1924313825831512, 1.1956643920398273, 1.1989061670743806,
    1.202156731452703, 1.2054161090051239, 1.2086843236265816, 1.2119613992768012,
    1.215247359980469, 1.2185422298274085, 1.2218460329727576, 1.2251587936371455,
    1.22848053610687, 1.2318112847340759, 1.2351510639369334, 1.2384998981998165,
    1.241857812073484, 1.245224830175258, 1.2486009771892048, 1.2519862778663162,
    1.255380757024691, 1.2587844395497165, 1.2621973503942507, 1.2656195145788063,
    1.2690509571917332, 1.2724917033894028, 1.275941778396392, 1.2794012075056693,
    1.2828700160787783, 1.2863482295460256, 1.2898358734066657, 1.2933329732290895,
    1.2968395546510096, 1.3003556433796506, 1.3038812651919358, 1.3074164459346773,
    1.3109612115247644, 1.3145155879493546, 1.318079601266064, 1.3216532776031575,
    1.3252366431597413, 1.3288297242059544, 1.3324325470831615, 1.3360451382041458,
    1.339667524053303, 1.3432997311868353, 1.3469417862329458, 1.3505937158920345,
    1.3542555469368927, 1.3579273062129011, 1.3616090206382248, 1.365300717204012,
    1.3690024229745905, 1.3727141650876684, 1.3764359707545302, 1.380167867260238,
    1.383909881963832, 1.387662042298529, 1.3914243757719262, 1.3951969099662003,
    1.3989796725383112, 1.4027726912202048, 1.4065759938190154, 1.4103896082172707,
    1.4142135623730951, 1.4180478843204152, 1.4218926021691656, 1.4257477441054942,
    1.42961333839197, 1.433489413367789, 1.4373759974489824, 1.4412731191286257,
    1.4451808069770467, 1.449099089642035, 1.4530279958490526, 1.4569675544014438,
    1.460917794180647, 1.4648787441464057, 1.4688504333369818, 1.4728328908693675,
    1.4768261459394993, 1.4808302278224719, 1.4848451658727524, 1.488870989524397,
    1.4929077282912648, 1.4969554117672355, 1.5010140696264256, 1.5050837316234065,
    1.5091644275934228, 1.5132561874526098, 1.5173590411982147, 1.5214730189088146,
    1.5255981507445384, 1.529734466947287, 1.533881997840956, 1.5380407738316568,
    1.5422108254079407, 1.5463921831410214, 1.550584877685, 1.5547889397770887,
    1.559004400237837, 1.5632312899713576, 1.567469639965553, 1.5717194812923414,
    1.5759808451078865, 1.5802537626528246, 1.5845382652524937, 1.588834384317164,
    1.593142151342267, 1.597461597908627, 1.6017927556826934, 1.606135656416771,
    1.6104903319492543, 1.6148568142048607, 1.6192351351948637, 1.6236253270173289,
    1.6280274218573478, 1.632441451987275, 1.6368674497669644, 1.6413054476440063,
    1.645755478153965, 1.6502175739206177, 1.6546917676561943, 1.6591780921616162,
    1.6636765803267364, 1.6681872651305825, 1.6727101796415966, 1.6772453570178785,
    1.681792830507429, 1.6863526334483934, 1.6909247992693053, 1.6955093614893326,
    1.7001063537185235, 1.7047158096580513, 1.709337763100463, 1.713972247929926,
    1.718619298122478, 1.723278947746274, 1.7279512309618377, 1.732636182022311,
    1.7373338352737062, 1.7420442251551564, 1.746767386199169, 1.7515033530318782,
    1.7562521603732995, 1.761013843037584, 1.7657884359332727, 1.7705759740635547,
    1.7753764925265212, 1.7801900265154245, 1.785016611318935, 1.789856282321401,
    1.7947090750031072, 1.7995750249405351, 1.804454167806624, 1.809346539371032,
    1.8142521755003989, 1.8191711121586085, 1.8241033854070534, 1.8290490314048973,
    1.8340080864093424, 1.8389805867758937, 1.843966568958626, 1.8489660695104508,
    1.8539791250833855, 1.8590057724288205, 1.864046048397789, 1.8690999899412386,
    1.8741676341103, 1.8792490180565602, 1.8843441790323345, 1.8894531543909392,
    1.8945759815869656, 1.8997126981765553, 1.9048633418176741, 1.9100279502703899,
    1.9152065613971474, 1.9203992131630474, 1.925605943636125, 1.930826790987627,
    1.9360617934922943, 1.9413109895286405, 1.9465744175792332, 1.9518521162309783,
    1.9571441241754002, 1.9624504802089273, 1.9677712232331759, 1.9731063922552343,
    1.978456026387951, 1.9838201648502194, 1.9891988469672663, 1.9945921121709402
};

// (A 32-entry table — one 256-B LDS bank row, conflict-free for any index pattern — with a degree-5 / 6 Chebyshev
// polynomial measured 39.36 / 39.57 ms against 39.07 ms for this 256-entry table on config 2, DESIGN.md §3.1: the
// table read costs its issue and latency, not bank conflicts.)
constexpr int EXP_TAB = 256;
constexpr double KEXP = 369.3299304675746;  // EXP_TAB / ln 2

__device__ __forceinline__ double exp_scaled_f64(double y, const double *tab) {
    const double jn = rint(y);
    const double r = y - jn;  // exact
    double t = fma(2.239395190875157e-12, r, 3.3083026805413713e-09);  // (ln2/256)^k / k!, k = 4..1
    t = fma(t, r, 3.6655655969101062e-06);
    t = fma(t, r, 0.0027076061740622863);
    const double pr = fma(t, r, 1.0);
    const int j = (int) jn;  // saturates for huge |y|: the ldexp below then returns 0
    return ldexp(tab[j & (EXP_TAB - 1)] * pr, j >> 8);
}

// 16 B per lane global -> LDS through a buffer descriptor on a wave-uniform base: the per-lane part is
// voff, a wave-uniform offset goes in soff (SGPR), so no VALU address math is needed per load
__device__ __forceinline__ void glds16_buf(const void *base, void *lds_dst, uint32_t voff, uint32_t soff) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *) base, (short) 0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *) lds_dst, 16, voff, soff, 0, 0);
}


// occupancy: 3 workgroups per CU (<= 49 KB LDS, <= 168 VGPRs) hide the chunk barriers / DMA waits
// best; the fp64 RBF variant spills a few epilogue values at that budget (outside the K loop), and
// still runs as fast as with 2 workgroups and 16-deep chunks
template <typename T, int KERNEL>
constexpr int kp_waves_per_eu() { return 3; }

// fp64 RBF: chunk kc+1's DMA is issued after chunk kc's LDS reads; every other instance: right after the barrier.
// Same box, round 6 (profiles/r06_kp_dma_order_ab.json): config 2 (fp64 RBF) 39.51 / 39.58 ms against 39.62 / 39.67 ms
// with the DMA first; fp64 linear 37.18 / 37.23 against 36.67 / 36.67 ms, fp64 poly 38.72 / 38.76 against 38.58 /
// 38.58 ms, configs[3] (fp32 linear) 1 913 against 1 782 ms. KP_DMA_AFTER_READS=0 / 1 forces one order (A/B only)
#ifndef KP_DMA_AFTER_READS
#define KP_DMA_AFTER_READS 2
#endif
template <typename T, int KERNEL>
constexpr bool kp_dma_after_reads() {
    return KP_DMA_AFTER_READS == 2 ? (sizeof(T) == 8 && KERNEL == 2) : KP_DMA_AFTER_READS == 1;
}

template <typename T, int KERNEL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kp_waves_per_eu<T, KERNEL>(), kp_waves_per_eu<T, KERNEL>()))) void kp_tile_kernel(kfun<T> kf, const T *__restrict__ XT,
                                                         const T *__restrict__ norms, const T *__restrict__ p,
                                                         T *__restrict__ partial, int64_t n_pad, int64_t d_pad,
                                                         int64_t nb, int64_t s0, int64_t nsuper,
                                                         const int32_t *__restrict__ wg_off,
                                                         const cg_scalars<T> *__restrict__ status) {
    using M = mfma16<T>;
    using acc_t = typename M::acc_t;
    constexpr int BK = kp_bk<T, KERNEL>();
    constexpr int PANEL = BK * KP_TILE;            // elements of one [BK][128] panel
    constexpr int EPP = 1024 / (int) sizeof(T);    // elements per 1 KiB wave-instruction
    constexpr int PIECES = PANEL / EPP / 4;        // wave-instructions per wave per panel
    constexpr int VEC = 16 / (int) sizeof(T);
    // LDS: p_I, p_J, n_I, n_J, then the two double-buffered panel pairs; once the K loop is done the
    // epilogue's reduction buffers overlay the panels: row partials [wc][128 rows][16 (+1 pad)],
    // column partials [wr][128 cols][4 (+1 pad)]
    constexpr int OFF_PAN = 4 * KP_TILE;
    constexpr int RSTR = 17, RHALF = KP_TILE * RSTR + 1, CSTR = 5;
    constexpr int RED = 2 * RHALF + 2 * KP_TILE * CSTR;
    constexpr int SMEM = OFF_PAN + (4 * PANEL > RED ? 4 * PANEL : RED);
    __shared__ __attribute__((aligned(16))) T smem[SMEM];
    constexpr bool FAST_EXP = (KERNEL == 2) && sizeof(T) == 8;
    __shared__ double exp_tab[FAST_EXP ? EXP_TAB : 1];

    if (status != nullptr && status->converged) return;

    // workgroups: one per real tile. wg_off[k] = first workgroup of the rank's super-block s0 + k (a full
    // super-block has 64 tiles, a diagonal one 36, the ragged last super-block row fewer): no empty
    // workgroups, so the XCDs' contiguous ranges carry equal work (empty ones bunched at the end of a
    // range made the last rank of 8 3.9 % slower than the others)
    const int64_t wg = xcd_remap(blockIdx.x, gridDim.x);
    int lo = 0, hi = (int) nsuper;  // largest k with wg_off[k] <= wg
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t) wg_off[mid] <= wg) lo = mid;
        else hi = mid;
    }
    const int64_t sb = s0 + lo, local = wg - wg_off[lo];
    int64_t SI, SJ;
    tri_tile(sb, SI, SJ);
    int64_t ta, tb;  // tile row / column inside the super-block
    if (SI == SJ) {
        tri_tile(local, ta, tb);  // lower triangle, tb <= ta
    } else {
        const int64_t cols = min<int64_t>(KP_SUPER, nb - SJ * KP_SUPER);
        ta = local / cols;
        tb = local % cols;
    }
    const int64_t I = SI * KP_SUPER + ta, J = SJ * KP_SUPER + tb;
    if (I >= nb || J > I) return;  // uniform per workgroup
    const int64_t I0 = I * KP_TILE, J0 = J * KP_TILE;
    const bool diag = (I == J);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform, provably (scalar LDS bases)
    const int wr = w >> 1, wc = w & 1;

    // p and norms of the tile's rows/cols -> LDS (issued first: their wait must not drain the DMA)
    const int64_t pidx = (tid < KP_TILE) ? I0 + tid : J0 + (tid - KP_TILE);
    const T pin = p[pidx];
    const T nin = (KERNEL == 2) ? norms[pidx] : T(0);
    // fast fp64 RBF: the accumulators start at -n_j / 2 (column j = lane & 15 of every block), so they
    // end at g_ij - n_j / 2 and y_ij = 2 g KEXP (g_ij - n_j / 2) - g KEXP n_i is one fma per element
    T acc0[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
        acc0[nt] = FAST_EXP ? T(-0.5) * norms[J0 + wc * 64 + nt * 16 + (lane & 15)] : T(0);

    // per-lane byte offsets of this wave's DMA pieces inside a chunk (32-bit, reused for every chunk
    // and both panels: the chunk base and the panel offset are wave-uniform, see glds16_buf)
    uint32_t doff[PIECES];
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
        const int elem = (w * PIECES + j) * EPP + lane * VEC;
        doff[j] = (uint32_t) (((int64_t) (elem / KP_TILE) * n_pad + elem % KP_TILE) * (int64_t) sizeof(T));
    }
    // LDS-DMA through a buffer descriptor: the chunk base is a scalar pointer (SALU), the per-lane part
    // is the constant doff and the panel offset goes in soffset — no VALU address math per chunk
    const uint32_t offI = __builtin_amdgcn_readfirstlane((uint32_t) (I0 * (int64_t) sizeof(T)));
    const uint32_t offJ = __builtin_amdgcn_readfirstlane((uint32_t) (J0 * (int64_t) sizeof(T)));
    auto issue = [&](int64_t kc, int buf) {
        const T *cb = XT + kc * BK * n_pad;
        T *pa = smem + OFF_PAN + (2 * buf) * PANEL;
        T *pb = pa + PANEL;
#pragma unroll
        for (int j = 0; j < PIECES; ++j) {
            const int u = w * PIECES + j;
            glds16_buf(cb, pa + u * EPP, doff[j], offI);
            glds16_buf(cb, pb + u * EPP, doff[j], offJ);
        }
    };

    acc_t acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = acc_t{ acc0[b], acc0[b], acc0[b], acc0[b] };

    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    smem[tid] = pin;
    smem[2 * KP_TILE + tid] = nin;
    if constexpr (FAST_EXP) {
        if (tid < EXP_TAB) exp_tab[tid] = c_exp2_256[tid];  // visible after the first K-loop barrier
    }

    const int64_t nk = d_pad / BK;
    for (int64_t kc = 0; kc < nk; ++kc) {
        if (kc > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // chunk kc visible to all waves; every wave is done reading chunk kc-1
        if (!kp_dma_after_reads<T, KERNEL>() && kc + 1 < nk) issue(kc + 1, (int) ((kc + 1) & 1));
        const T *A = smem + OFF_PAN + (2 * (kc & 1)) * PANEL;
        const T *B = A + PANEL;
        // fp64 RBF: the whole chunk's operands come out of LDS before chunk kc+1's DMA is issued — the compiler cannot
        // tell the DMA's LDS target from the buffer being read, so an LDS read issued after the DMA waits for it
        // (vmcnt(0)) and the prefetch sits on each wave's critical path instead of under its MFMAs (the other instances
        // measured faster with the DMA first, see kp_dma_after_reads)
        T a[BK / 4][4], b[BK / 4][4];
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks) {
            const int kr = ks * 4 + (lane >> 4);
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) a[ks][mt] = A[kr * KP_TILE + wr * 64 + mt * 16 + (lane & 15)];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) b[ks][nt] = B[kr * KP_TILE + wc * 64 + nt * 16 + (lane & 15)];
        }
        if (kp_dma_after_reads<T, KERNEL>() && kc + 1 < nk) issue(kc + 1, (int) ((kc + 1) & 1));
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = M::op(a[ks][mt], b[ks][nt], acc[mt][nt]);
    }

    // ---- epilogue: kernel function, times p, row and column partial sums ----
    const T *pI = smem, *pJ = smem + KP_TILE, *nI = smem + 2 * KP_TILE, *nJ = smem + 3 * KP_TILE;
    T pj[4], nj[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int jl = wc * 64 + nt * 16 + (lane & 15);
        pj[nt] = pJ[jl];
        nj[nt] = (KERNEL == 2 && !FAST_EXP) ? nJ[jl] : T(0);
    }
    T cs[4] = { 0, 0, 0, 0 };
    const T c2 = FAST_EXP ? T(2) * kf.gamma * T(KEXP) : T(0);
    // Each row has 32 partials (16 lanes x 2 column-half waves), each column 8 (4 lane groups x 2
    // row-half waves). They are parked in LDS and every thread then sums one half-row and one
    // half-column: ~20 adds per lane instead of a 4-level shuffle tree per row (64 adds + 128
    // ds_bpermute); the fixed summation order keeps K·p bitwise reproducible.
    __syncthreads();  // every wave is done with the last K chunk: the panels become reduction buffers
    T *rowp = smem + OFF_PAN + wc * RHALF;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int il = wr * 64 + mt * 16 + M::row(lane, r);
            const T pi = pI[il];
            const T ni = nI[il];
            const T ai = FAST_EXP ? -kf.gamma * T(KEXP) * ni : T(0);
            T s = 0;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                T kv;
                if constexpr (FAST_EXP)
                    kv = (T) exp_scaled_f64(fma(c2, acc[mt][nt][r], ai), exp_tab);
                else
                    kv = kernel_apply<T>(KERNEL, kf.degree, kf.gamma, kf.coef0, acc[mt][nt][r], ni, nj[nt]);
                s = fma(kv, pj[nt], s);
                cs[nt] = fma(kv, pi, cs[nt]);
            }
            rowp[il * RSTR + (lane & 15)] = s;
        }
    }
    if (!diag) {
        T *colp = smem + OFF_PAN + 2 * RHALF + wr * KP_TILE * CSTR;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) colp[(wc * 64 + nt * 16 + (lane & 15)) * CSTR + (lane >> 4)] = cs[nt];
    }
    __syncthreads();
    const int q = tid >> 1, h = tid & 1;  // row / column q of the tile, half h
    const T *rp = smem + OFF_PAN + h * RHALF + q * RSTR;
    T a = rp[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) a += rp[k];
    a += __shfl_xor(a, 1);
    if (!diag) {
        const T *cp = smem + OFF_PAN + 2 * RHALF + (h * KP_TILE + q) * CSTR;
        T c = (cp[0] + cp[1]) + (cp[2] + cp[3]);
        c += __shfl_xor(c, 1);
        if (h == 1) partial[wg * KP_REC + KP_TILE + q] = c;  // column sums of the J rows
    }
    if (h == 0) partial[wg * KP_REC + q] = a;  // row sums of the I rows
}

// Slab values of row i (row block Ib, offset q) for the column blocks c of column super-block CS, in c
// order: tile (Ib, c)'s row sums when c <= Ib, tile (c, Ib)'s column sums when c > Ib. base = the first
// record of the super-block holding those tiles (kp_tile_offsets' table); tiles inside a super-block are
// numbered row-major (a diagonal one: its lower triangle, ta (ta + 1) / 2 + tb).
template <typename T>
__device__ __forceinline__ void kp_sb_values(const T *__restrict__ partial, int64_t Ib, int64_t q, int64_t CS,
                                             int64_t nb, int64_t base, T *v, int cnt) {
    const int64_t RS = Ib / KP_SUPER;
    for (int u = 0; u < cnt; ++u) {
        const int64_t c = CS * KP_SUPER + u;
        const int64_t I = c <= Ib ? Ib : c, J = c <= Ib ? c : Ib;
        const int64_t SI = c <= Ib ? RS : CS, SJ = c <= Ib ? CS : RS;
        const int64_t ta = I - SI * KP_SUPER, tb = J - SJ * KP_SUPER;
        const int64_t local = SI == SJ ? ta * (ta + 1) / 2 + tb : ta * min<int64_t>(KP_SUPER, nb - SJ * KP_SUPER) + tb;
        v[u] = partial[(base + local) * KP_REC + (c <= Ib ? 0 : KP_TILE) + q];
    }
}


// raw[i] = sum of the slab values of the super-blocks [s0, s1) (a rank's share, or the whole triangle): the
// column super-blocks of a row are dealt to the 16 waves of a block (64 rows per block, lanes = rows:
// coalesced) and the 16 partial sums are added in wave order — a fixed order, deterministic; the critical
// path per thread is 1/16 of the row (one thread per row is latency-bound)
constexpr int KP_RED_G = 16;
template <typename T>
__global__ __launch_bounds__(64 * KP_RED_G) void kp_reduce_share_kernel(const T *__restrict__ partial, int64_t nb,
                                                                        int64_t m, int64_t s0, int64_t s1,
                                                                        const int32_t *__restrict__ wg_off,
                                                                        T *__restrict__ raw,
                                                                        const cg_scalars<T> *__restrict__ status) {
    if (status != nullptr && status->converged) return;
    __shared__ T red[KP_RED_G][64];
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t i = (int64_t) blockIdx.x * 64 + lane;
    const int64_t ns = (nb + KP_SUPER - 1) / KP_SUPER;
    const int64_t Ib = __builtin_amdgcn_readfirstlane((int) (((int64_t) blockIdx.x * 64) / KP_TILE));
    T s = 0;
    if (i < m) {
        const int64_t q = i % KP_TILE, RS = Ib / KP_SUPER;
        // column super-blocks dealt round-robin to the waves: a rank's owned super-blocks of a row (often a
        // short run of CS) spread over the waves instead of landing in one
        for (int64_t CS = g; CS < ns; CS += KP_RED_G) {
            const int64_t sb = (RS >= CS) ? tri_index(RS, CS) : tri_index(CS, RS);
            if (sb < s0 || sb >= s1) continue;
            const int64_t base = wg_off[sb - s0];
            const int cnt = (int) min<int64_t>(KP_SUPER, nb - CS * KP_SUPER);
            T v[KP_SUPER];
            if (cnt == KP_SUPER) {
                kp_sb_values(partial, Ib, q, CS, nb, base, v, KP_SUPER);
#pragma unroll
                for (int u = 0; u < KP_SUPER; ++u) s += v[u];
            } else {
                kp_sb_values(partial, Ib, q, CS, nb, base, v, cnt);
                for (int u = 0; u < cnt; ++u) s += v[u];
            }
        }
    }
    red[g][lane] = s;
    __syncthreads();
    if (g == 0 && i < m) {
        T a = red[0][lane];
#pragma unroll
        for (int h = 1; h < KP_RED_G; ++h) a += red[h][lane];
        raw[i] = a;
    }
}

}  // namespace

template <typename T>
void launch_kp_tiles(kfun<T> kf, const T *XT, const T *norms, const T *p, T *partial, int64_t n_pad, int64_t d_pad,
                     int64_t nb, int64_t s0, int64_t nsuper, const int32_t *wg_off, int64_t wgs,
                     const cg_scalars<T> *status, hipStream_t s) {
    if (nsuper <= 0 || nb <= 0 || wgs <= 0) return;
    // 32-bit DMA offsets inside a chunk (kp_tile_kernel): (BK - 1) rows of n_pad plus a tile row
    if ((int64_t) kp_dpad<T>() * n_pad * (int64_t) sizeof(T) >= ((int64_t) 1 << 31))
        throw mi_error(-5, "too many points for the pairwise tile kernel's 32-bit chunk offsets");
    const dim3 grid((unsigned) wgs), block(256);
    switch (kf.kernel) {
        case 0:
            hipLaunchKernelGGL((kp_tile_kernel<T, 0>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, nb,
                               s0, nsuper, wg_off, status);
            break;
        case 1:
            hipLaunchKernelGGL((kp_tile_kernel<T, 1>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, nb,
                               s0, nsuper, wg_off, status);
            break;
        default:
            hipLaunchKernelGGL((kp_tile_kernel<T, 2>), grid, block, 0, s, kf, XT, norms, p, partial, n_pad, d_pad, nb,
                               s0, nsuper, wg_off, status);
            break;
    }
    MI_LAUNCH_CHECK();
}

// Both the whole triangle and a rank's share use the wave-split reduction (16 waves per 64 rows, each a
// range of column super-blocks, partial sums added in wave order): one thread per row walking all nb
// records (round 1's kp_reduce_kernel) was latency-bound — 0.43 ms for config 2's 627 MB slab.
template <typename T>
void launch_kp_reduce(const T *partial, int64_t nb, int64_t m, int64_t s0, int64_t s1, const int32_t *wg_off, T *raw,
                      const cg_scalars<T> *status, hipStream_t s) {
    if (m <= 0) return;
    hipLaunchKernelGGL(kp_reduce_share_kernel<T>, dim3((unsigned) ceil_div(m, 64)), dim3(64 * KP_RED_G), 0, s,
                       partial, nb, m, s0, s1, wg_off, raw, status);
    MI_LAUNCH_CHECK();
}

#define INST(T)                                                                                                  \
    template void launch_kp_tiles<T>(kfun<T>, const T *, const T *, const T *, T *, int64_t, int64_t, int64_t, \
                                     int64_t, int64_t, const int32_t *, int64_t, const cg_scalars<T> *,        \
                                     hipStream_t);                                                              \
    template void launch_kp_reduce<T>(const T *, int64_t, int64_t, int64_t, int64_t, const int32_t *, T *,     \
                                      const cg_scalars<T> *, hipStream_t);
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
