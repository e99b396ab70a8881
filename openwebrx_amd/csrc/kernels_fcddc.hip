// kernels_fcddc.hip -- exact fast-convolution form of the fused Selector front end:
// Shift(rate_c) (csdr/chain/selector.py:95,132-140) followed by FirDecimate(D, transition,
// cutoff) (selector.py:11-35), for every chain of one (D, taps) group.
//
//   y_c[k] = sum_{t<T} h[t] x[kD + t] exp(j 2 pi phase_c(kD + t))
//          = rot_c(k) * sum_{r<D} sum_{p<P} u_r[k + p] g_{c,r}[p]
// with rot_c(k) = exp(j 2 pi phase_c(kD)) (64-bit fixed-point phase, as ddc_lds seeds it),
// u_r[i] = x[iD + r] (polyphase branch r of the wideband input, shared by all chains) and
// g_{c,r}[p] = h[pD + r] exp(j 2 pi rate_c (pD + r)) (the chain's modulated branch taps).
//
// Each branch correlation runs on frames of M branch samples through M-point DFTs
// (overlap-save: V = M - P + 1 valid outputs per frame).  For frame f, k0 = k_begin + f V:
//   U[kappa][f][r]  = sum_{i<M} u_r[k0 + i] e^{-j 2 pi i kappa / M}            (fc_fwd)
//   Y_c[f][kappa]   = sum_r U[kappa][f][r] W_c[kappa][r]                       (fc_mac: per kappa
//                                                         one complex GEMM frames x chains x D)
//   y_c[k0 + m]     = rot_c(k0 + m) IDFT_M(Y_c[f])[m],   m < V                 (fc_out)
// with W_c[kappa][r] = sum_p g_{c,r}[p] e^{+j 2 pi p kappa / M} built once per chain and
// rebuilt on retune (fc_make_w, fp64).  Exact up to fp32 rounding: a numpy float32 model of
// these steps is 1.8e-7 rel-RMS from the float64 oracle at D = 833 (tests/test_gpu_parity.py
// holds the GPU to <= 1e-5).
//
// Work per output and chain: 8 M Dp / V flop (7.5k at D = 833, M = 256) against 4T + 6D =
// 94k for the direct form (ddc_lds) -- and it is a real matrix product, so it runs on the
// f32 MFMA (v_mfma_f32_16x16x4_f32, exact f32 products and sums; the complex product is the
// real GEMM [Ur Ui] x [[Wr Wi] [-Wi Wr]]).  Its operands stream once per block: W (C M Dp 8 B,
// unique per chain) from HBM, U from L2, so fc_mac sits between the HBM and the f32 MFMA roof.
#include <vector>
#include <stdlib.h>
#include <string.h>

#include "owrx_types.h"
#include "fft_lds.h"

namespace owrx {

typedef float fc_f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const fc_f4 gf4;  // global (not flat) loads

#define HIPCHK_RET(expr)                 \
    do {                                 \
        hipError_t _e = (expr);          \
        if (_e != hipSuccess) return _e; \
    } while (0)

constexpr int kFcRT = 16;   // branches (r) per fc_fwd / fc_make_w workgroup
// W's layout per bin kappa: [chain / T][K-block of 8 branches][chain % T][8 branches] (cf32),
// T = kFcTile chains: fc_mac's load instruction for 8 chains and one K-block reads 512
// contiguous bytes, the CTT loads of a wave tile are adjacent when T >= 8 CTT, and the K-blocks
// follow each other (its load pattern alone, T = 8: 54 -> 48 us per C3 launch from HBM,
// tools/micro/fc_floor.hip).  Element (kappa, chain c, branch r) at
// kappa w_ks + fc_w_chain(c, Dp) + fc_w_branch(r).  Capacities are multiples of T.  T = 32 (a
// wave's four tiles of 8 chains in 2 KB runs): fc_mac 0.467-0.468 of HBM at C3 vs 0.443-0.460
// for T = 8 and 0.467-0.471 for T = 64, same box (profiles/r03aj_ab_w_tile_c3.txt); 32 is
// already the smallest capacity, so small engines allocate nothing extra.
#ifndef OWRX_FC_TILE
#define OWRX_FC_TILE 32
#endif
constexpr int kFcTile = OWRX_FC_TILE;
static_assert(kFcTile >= 8 && (kFcTile & (kFcTile - 1)) == 0, "W tile: a power of two >= 8 chains");
#define OWRX_DEV_HOST_INLINE __host__ __device__ __forceinline__
OWRX_DEV_HOST_INLINE int64_t fc_w_chain(int c, int Dp) {
    return (int64_t)(c / kFcTile) * kFcTile * Dp + (c % kFcTile) * 8;
}
OWRX_DEV_HOST_INLINE int64_t fc_w_branch(int r) { return (int64_t)(r >> 3) * kFcTile * 8 + (r & 7); }
constexpr int kFcDpAlign = 96;  // Dp: a multiple of kFcRT and of 4 (K split) x 3 K-blocks of 8

// Frame lengths: powers of two (64, 128, 256) and three times one (192, 384).  A row of
// M = 3 L is kept as three sub-rows of L (stride SRS), x[L n1 + n2] at sub-row n1, so the
// M-point DFT is a radix-3 pass over n1 (twiddled by W_M^(n2 k1)) then L-point DFTs of the
// sub-rows; bin k = k1 + 3 k2 lands in sub-row k1 at k2.  (M = 192 fits the C2 / C3 block:
// 31 frames of V = 166 in two 16-frame MFMA tiles, where M = 256 needs 22 of 32.)
template <int M>
struct FcM {
    static constexpr bool R3 = (M % 3) == 0;
    static constexpr int L = R3 ? M / 3 : M;
    static constexpr int LOGL = L == 32 ? 5 : L == 64 ? 6 : L == 128 ? 7 : 8;
    static_assert((1 << LOGL) == L, "frame length");
    static constexpr int SRS = L + 1;                 // sub-row stride (float2), R3 only
    static constexpr int RS = R3 ? 3 * SRS : M + 1;   // row stride
    // LDS position of time sample i / of bin k within a row
    OWRX_DEV static int tpos(int i) { return R3 ? (i / L) * SRS + i % L : i; }
    OWRX_DEV static int kpos(int k) { return R3 ? (k % 3) * SRS + k / 3 : k; }
};

// forward M-point DFT of R rows (row stride FcM<M>::RS) in place; tw: the M-point table
template <int M, int R, int NT>
OWRX_DEV void fc_fft_rows(float2* sm, const float2* __restrict__ tw) {
    using F = FcM<M>;
    if constexpr (!F::R3) {
        lds_fft_rows<F::LOGL, R, NT>(sm, F::RS, tw, 1);
    } else {
        constexpr int L = F::L, SRS = F::SRS;
        const float c3 = -0.5f, s3 = -0.86602540378443865f;  // W_3 = e^{-j 2 pi / 3}
        for (int e = threadIdx.x; e < R * L; e += NT) {
            const int row = e / L, n2 = e % L;
            float2* b = sm + row * F::RS + n2;
            const float2 a0 = b[0], a1 = b[SRS], a2 = b[2 * SRS];
            const float2 sp = make_float2(a1.x + a2.x, a1.y + a2.y);
            const float2 sm_ = make_float2(a1.x - a2.x, a1.y - a2.y);
            const float2 y0 = make_float2(a0.x + sp.x, a0.y + sp.y);
            const float2 t = make_float2(a0.x + c3 * sp.x, a0.y + c3 * sp.y);
            // y1 = t + j s3 sm_, y2 = t - j s3 sm_
            const float2 y1 = make_float2(t.x - s3 * sm_.y, t.y + s3 * sm_.x);
            const float2 y2 = make_float2(t.x + s3 * sm_.y, t.y - s3 * sm_.x);
            b[0] = y0;
            b[SRS] = n2 ? cmul(y1, tw[n2]) : y1;
            b[2 * SRS] = n2 ? cmul(y2, tw[2 * n2]) : y2;
        }
        __syncthreads();
        lds_fft_rows<F::LOGL, 3 * R, NT>(sm, SRS, tw, 3);  // W_L^m = W_M^(3 m)
    }
}

// ---- W_c[kappa][r], fp64 ----------------------------------------------------------------------
// One workgroup: kFcRT branches of one chain.  h: the group's linear taps (T floats); the chain's
// row kappa is written at W + kappa * w_ks.  fc_make_w: one chain per launch (grid Dp / kFcRT;
// retunes); fc_make_w_jobs: every chain that joined since the last flush (grid (Dp / kFcRT,
// jobs)), so a burst of joins fills the chip instead of 54 workgroups per launch.
template <int M>
__device__ void fc_make_w_rows(const float* __restrict__ h, int T, int D, int P, uint64_t rate_fx,
                               float2* __restrict__ W, int64_t w_ks) {
    __shared__ double2 g[kFcRT][64];   // P <= 64
    __shared__ double2 tw[M];          // e^{+j 2 pi m / M}
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * kFcRT;
    for (int m = tid; m < M; m += 256) {
        double s, c;
        sincospi(2.0 * (double)m / (double)M, &s, &c);
        tw[m] = make_double2(c, s);
    }
    for (int e = tid; e < kFcRT * P; e += 256) {
        const int j = e / P, p = e % P;
        const int r = r0 + j;
        const int64_t t = (int64_t)p * D + r;
        double2 v = make_double2(0.0, 0.0);
        if (r < D && t < T) {
            // phase of tap t in 2^-64 turns, exact; signed turns in [-0.5, 0.5)
            const int64_t ph = (int64_t)((uint64_t)t * rate_fx);
            const double turns = (double)ph * 5.421010862427522e-20;  // 2^-64
            double s, c;
            sincospi(2.0 * turns, &s, &c);
            const double hv = (double)h[t];
            v = make_double2(hv * c, hv * s);
        }
        g[j][p] = v;
    }
    __syncthreads();
    const int j = tid % kFcRT;
    for (int kap = tid / kFcRT; kap < M; kap += 256 / kFcRT) {
        double re = 0.0, im = 0.0;
        for (int p = 0; p < P; ++p) {
            const double2 a = g[j][p];
            const double2 b = tw[(p * kap) % M];
            re += a.x * b.x - a.y * b.y;
            im += a.x * b.y + a.y * b.x;
        }
        const int r = r0 + j;  // tiled: the chain's K-block of 8 branches every 64 entries
        W[(int64_t)kap * w_ks + (r >> 3) * kFcTile * 8 + (r & 7)] = make_float2((float)re, (float)im);  // zero for r >= D
    }
}

template <int M>
__global__ void __launch_bounds__(256)
fc_make_w(const float* __restrict__ h, int T, int D, int Dp, int P, uint64_t rate_fx,
          float2* __restrict__ W, int64_t w_ks) {
    fc_make_w_rows<M>(h, T, D, P, rate_fx, W, w_ks);
}

template <int M>
__global__ void __launch_bounds__(256)
fc_make_w_jobs(const float* __restrict__ h, int T, int D, int P, const FcWJob* __restrict__ jobs,
               float2* __restrict__ W, int64_t w_ks) {
    const FcWJob j = jobs[blockIdx.y];
    fc_make_w_rows<M>(h, T, D, P, j.rate_fx, W + j.off, w_ks);
}

// Frame f of an engine block of caller blocks (FcSubs): its sub-block s, the sub-block's first
// output nk0 and first frame f0.
struct FcFrame {
    int s, nk0, f0;
};
OWRX_DEV FcFrame fc_frame_sub(const FcSubs& sb, int f, int V) {
    FcFrame r{0, 0, 0};
    for (int s = 0; s + 1 < sb.n; ++s) {
        const int fe = r.f0 + (sb.nk[s] - r.nk0 + V - 1) / V;
        if (f < fe) break;
        r.s = s + 1;
        r.nk0 = sb.nk[s];
        r.f0 = fe;
    }
    return r;
}

// ---- U[kappa][f][r]: M-point DFT of every branch frame --------------------------------------
// grid: (Dp / kFcRT, F); block 256.  tw: M-point table e^{-j 2 pi m / M}.
// Caller blocks grouped into one engine block (owrx_set_block_group): each sub-block's frames
// start at its first output and are zero past its own input end (FcSubs) -- the frames and zero
// padding each block's own launch would have had, so U is bit-identical to separate launches.
template <int M>
__global__ void __launch_bounds__(256)
fc_fwd(const float2* __restrict__ blk, int64_t blk_start, FcSubs sb, int64_t k_begin, int V, int D,
       int Dp, int Fs, const float2* __restrict__ tw, float2* __restrict__ U) {
    using FM = FcM<M>;
    constexpr int RS = FM::RS;         // LDS row stride (float2): column writes hit distinct banks
    __shared__ float2 sm[kFcRT * RS];
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * kFcRT;
    const int f = blockIdx.y;
    const FcFrame fr = fc_frame_sub(sb, f, V);
    const int64_t k0 = k_begin + fr.nk0 + (int64_t)(f - fr.f0) * V;
    const int64_t blk_end = sb.end[fr.s];
    const int j = tid % kFcRT;
    const int r = r0 + j;
    // rows i of the frame: 16 consecutive branches = one 128-B run per row
#pragma unroll 4
    for (int i = tid / kFcRT; i < M; i += 256 / kFcRT) {
        const int64_t n = (k0 + i) * (int64_t)D + r;
        float2 x = make_float2(0.0f, 0.0f);
        if (r < D && n < blk_end) x = blk[n - blk_start];
        sm[j * RS + FM::tpos(i)] = x;
    }
    __syncthreads();
    fc_fft_rows<M, kFcRT, 256>(sm, tw);
    float2* out = U + (int64_t)f * Dp + r0 + j;
#pragma unroll 4
    for (int kap = tid / kFcRT; kap < M; kap += 256 / kFcRT)
        out[(int64_t)kap * Fs * Dp] = sm[j * RS + FM::kpos(kap)];
}

// ---- Y_c[f][kappa] = sum_r U[kappa][f][r] W_c[kappa][r] on the f32 MFMA ---------------------
// One workgroup: one kappa, FTT tiles of 16 frames x CTT tiles of 8 chains; its four waves
// split the branch range four ways (K split) and are summed through LDS in a fixed order.
// v_mfma_f32_16x16x4_f32 lane layout: A[i][k] and B[k][j] at lane i|j + 16 k, D[4 (l/16) + v][l%16].
// Rows = frames, columns = (chain, re|im), K = (r, re|im).  The K order inside a block of 8
// branches is permuted (lane group g takes branches 2g, 2g+1 of the block, MFMA s takes
// component s of that float4), the same permutation on both operands.  W of chain slot c at
// W + c * w_cs + kappa * w_ks.
constexpr int kFcKSplit = 4;
constexpr int kFcMaxKSlices = 16;  // K slices across workgroups (fc_kslices): Y holds this many
// Three waves per SIMD (<= 168 registers): C3's 2^20-sample blocks launch M x 4 = 512
// workgroups, one more round than stream A's 240 CUs hold at two (480)
template <int FTT, int CTT, bool NT>
__global__ void __launch_bounds__(64 * kFcKSplit) __attribute__((amdgpu_waves_per_eu(3)))
fc_mac(const float2* __restrict__ U, const float2* __restrict__ W, int64_t w_cs, int64_t w_ks,
       int nchains, int Fs, int F, int Dp, int M, int ncg, int chain_fastest,
       float2* __restrict__ Y) {
    // XCD-aware decode: consecutive workgroup ids land on different XCDs (round robin), so the
    // ids one XCD receives are mapped to one contiguous kappa range (the 8-B Y stores of
    // neighbouring kappas -- one Y line -- meet in that XCD's L2).  Within an XCD the chain
    // groups of one (kappa, frame group) come consecutively, so the workgroups that read the
    // same U tile run together and fetch it from HBM once (the kappa-fastest order re-read it
    // per chain group: 770 MB of HBM reads per C3 launch against 510 MB of W + U)
    const int w = blockIdx.x;
    const int xcd = w & 7;
    const int q = w >> 3;
    const int mper = M >> 3;
    int kap, cg, fg;
    const int nfg = (F + 16 * FTT - 1) / (16 * FTT);
    if (chain_fastest && nfg > 1) {
        // several frame tiles (grouped blocks, F > 16 FTT): a (kappa, chain group)'s frame tiles
        // come back to back on one XCD, so the second reads its W tile from L2 and W streams
        // from HBM once per launch (frame tiles outermost re-read all of W per tile)
        fg = q % nfg;
        const int r1 = q / nfg;
        cg = r1 % ncg;
        kap = xcd * mper + r1 / ncg;
    } else if (chain_fastest) {
        cg = q % ncg;
        const int r1 = q / ncg;
        kap = xcd * mper + r1 % mper;
        fg = r1 / mper;
    } else {
        kap = xcd * mper + q % mper;
        const int rest = q / mper;
        cg = rest % ncg;
        fg = rest / ncg;
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    const int col = lane & 15;
    const int cc = col >> 1;
    const bool bim = col & 1;
    // this wave's K range: a quarter of the K-blocks of 8 branches (Dp is a multiple of 96,
    // so a multiple of 3 blocks each)
    const int nkb = (Dp >> 3) / kFcKSplit;
    const int kb0 = wave * nkb;

    // rows of frames >= F and columns of chains >= nchains read frame 0 / chain 0 instead:
    // an MFMA row (column) of D depends only on its A row (B column), and those outputs are
    // never stored, so the loads need no guard (and the loop no branches)
    const gf4* up[FTT];
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft) {
        const int f = fg * 16 * FTT + ft * 16 + col;
        up[ft] = (const gf4*)(U + ((int64_t)kap * Fs + (f < F ? f : 0)) * Dp + 8 * kb0 + 2 * g);
    }
    const gf4* wp[CTT];
#pragma unroll
    for (int t = 0; t < CTT; ++t) {
        const int c = cg * 8 * CTT + t * 8 + cc;
        wp[t] = (const gf4*)(W + (int64_t)kap * w_ks + fc_w_chain(c < nchains ? c : 0, (int)w_cs) +
                             fc_w_branch(8 * kb0 + 2 * g));
    }
    fc_f4 acc[FTT][CTT];
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
        for (int t = 0; t < CTT; ++t) acc[ft][t] = fc_f4{0.0f, 0.0f, 0.0f, 0.0f};

    // operands of K-blocks kb (ready), kb + 1 and kb + 2 (in flight) in three register sets
    // with fixed roles (a 3-way unrolled loop): two blocks of MFMA work cover the load latency
    fc_f4 ua0[FTT], ua1[FTT], ua2[FTT], wa0[CTT], wa1[CTT], wa2[CTT];
    auto load = [&](fc_f4* ua, fc_f4* wa, int kb) {
        const int o = (kb < nkb ? kb : nkb - 1) * 4;
#pragma unroll
        for (int ft = 0; ft < FTT; ++ft) ua[ft] = up[ft][o];
#pragma unroll
        for (int t = 0; t < CTT; ++t) {  // tiled W: K-blocks kFcTile * 8 cf32 = 4 kFcTile float4 apart
            if constexpr (NT) wa[t] = __builtin_nontemporal_load(wp[t] + o * kFcTile);
            else wa[t] = wp[t][o * kFcTile];
        }
    };
    auto block = [&](const fc_f4* ua, const fc_f4* wa) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            float bsel[CTT];
#pragma unroll
            for (int t = 0; t < CTT; ++t) {
                // B[(r, a)][(c, b)]: a = 0 -> (Wr | Wi), a = 1 -> (-Wi | Wr)
                const float wr = (s < 2) ? wa[t].x : wa[t].z;
                const float wi = (s < 2) ? wa[t].y : wa[t].w;
                bsel[t] = (s & 1) ? (bim ? wr : -wi) : (bim ? wi : wr);
            }
#pragma unroll
            for (int ft = 0; ft < FTT; ++ft) {
                const float a = ua[ft][s];
#pragma unroll
                for (int t = 0; t < CTT; ++t)
                    acc[ft][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bsel[t], acc[ft][t], 0, 0, 0);
            }
        }
    };
    // the prologue issues the two groups in the loop's order (ua0's loads the older): the
    // wait-count pass merges the loop header's entry and back-edge states, and with ua1's
    // loads scheduled first here it made every block wait for the next block's operands too
    load(ua0, wa0, 0);
    __builtin_amdgcn_sched_barrier(0);
    load(ua1, wa1, 1);
    __builtin_amdgcn_sched_barrier(0);
    for (int kb = 0; kb < nkb; kb += 3) {
        load(ua2, wa2, kb + 2);
        __builtin_amdgcn_sched_barrier(0);  // issue the loads before this block's MFMAs
        block(ua0, wa0);
        load(ua0, wa0, kb + 3);
        __builtin_amdgcn_sched_barrier(0);
        block(ua1, wa1);
        load(ua1, wa1, kb + 4);
        __builtin_amdgcn_sched_barrier(0);
        block(ua2, wa2);
    }
    // K-split sum, fixed order ((w0 + w1) + (w2 + w3))
    __shared__ fc_f4 red[kFcKSplit - 1][FTT * CTT][64];
    if (wave > 0) {
#pragma unroll
        for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
            for (int t = 0; t < CTT; ++t) red[wave - 1][ft * CTT + t][lane] = acc[ft][t];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
        for (int t = 0; t < CTT; ++t) {
            const int i = ft * CTT + t;
            acc[ft][t] = (acc[ft][t] + red[0][i][lane]) + (red[1][i][lane] + red[2][i][lane]);
        }
    // lanes col = 2cc (re) and 2cc + 1 (im) hold one chain's 4 frames: swap halves, each lane
    // stores two complex outputs
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
        for (int t = 0; t < CTT; ++t) {
            const fc_f4 o = acc[ft][t];
            fc_f4 p;
            p.x = __shfl_xor(o.x, 1);
            p.y = __shfl_xor(o.y, 1);
            p.z = __shfl_xor(o.z, 1);
            p.w = __shfl_xor(o.w, 1);
            const int c = cg * 8 * CTT + t * 8 + cc;
            if (c >= nchains) continue;
            const int fb = fg * 16 * FTT + ft * 16 + 4 * g + (bim ? 2 : 0);
            const float2 y0 = bim ? make_float2(p.z, o.z) : make_float2(o.x, p.x);
            const float2 y1 = bim ? make_float2(p.w, o.w) : make_float2(o.y, p.y);
            float2* yc = Y + ((int64_t)c * Fs) * M + kap;
            if (fb < F) yc[(int64_t)fb * M] = y0;
            if (fb + 1 < F) yc[(int64_t)(fb + 1) * M] = y1;
        }
}

// ---- fc_mac with the operand stream through an LDS ring (LDS-DMA; the default form) ---------
// Same workgroup decode, K split, MFMA order and epilogue as fc_mac (bit-identical Y).  Each wave
// streams its own K-blocks into a private ring of NR slots with global_load_lds_dwordx4 (1 KiB per
// instruction, no VGPR destination, no duplicate lanes): per K-block CTT/2 instructions of W
// (two 8-chain runs of 512 B each) and FTT of U (16 frames x 64 B), NR - 1 blocks in flight.
// Only the issuing wave reads a slot, so its counted vmcnt orders the reads (no barrier).
// Slot image: [t][chain % 8][branch pair] then [ft][frame][branch pair], 16 B entries.
template <int FTT, int CTT, int NR>
__global__ void __launch_bounds__(64 * kFcKSplit)
fc_mac_lds(const float2* __restrict__ U, const float2* __restrict__ W, int64_t w_cs, int64_t w_ks,
           int nchains, int Fs, int F, int Dp, int M, int ncg, int chain_fastest,
           float2* __restrict__ Y, int ks, int64_t y_slice) {
    constexpr int P = CTT / 2 + FTT;  // DMA instructions per K-block
    constexpr int kSlot = P * 1024;
    constexpr int kRing = NR * kSlot;
    constexpr int kRed = (kFcKSplit - 1) * FTT * CTT * 64 * 16;
    constexpr int kLds = kFcKSplit * kRing > kRed ? kFcKSplit * kRing : kRed;
    static_assert((NR - 1) * P <= 63, "vmcnt holds 6 bits");
    __shared__ __attribute__((aligned(1024))) char lds[kLds];
    // K slices across workgroups (ks > 1: grids too small to fill the chip, e.g. C4's per-GPU
    // share of 128 chains): slice sl of tile w holds K-blocks [sl KB / ks, (sl + 1) KB / ks) and
    // writes its partial Y to Y + sl y_slice; fc_out sums the slices in slice order.  The tile
    // count is a multiple of 8, so a tile's slices share its XCD (and its U tile in L2).
    const int tiles = M * ncg * (int)(gridDim.x / (unsigned)(M * ncg * ks));
    const int sl = blockIdx.x / tiles;
    const int w = blockIdx.x - sl * tiles;
    Y += sl * y_slice;
    const int xcd = w & 7;
    const int q = w >> 3;
    const int mper = M >> 3;
    int kap, cg, fg;
    const int nfg = (F + 16 * FTT - 1) / (16 * FTT);
    if (chain_fastest && nfg > 1) {
        // several frame tiles (grouped blocks, F > 16 FTT): a (kappa, chain group)'s frame tiles
        // come back to back on one XCD, so the second reads its W tile from L2 and W streams
        // from HBM once per launch (frame tiles outermost re-read all of W per tile)
        fg = q % nfg;
        const int r1 = q / nfg;
        cg = r1 % ncg;
        kap = xcd * mper + r1 / ncg;
    } else if (chain_fastest) {
        cg = q % ncg;
        const int r1 = q / ncg;
        kap = xcd * mper + r1 % mper;
        fg = r1 / mper;
    } else {
        kap = xcd * mper + q % mper;
        const int rest = q / mper;
        cg = rest % ncg;
        fg = rest / ncg;
    }
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4;
    const int col = lane & 15;
    const int cc = col >> 1;
    const bool bim = col & 1;
    const int nkb = (Dp >> 3) / (kFcKSplit * ks);
    const int kb0 = (sl * kFcKSplit + wave) * nkb;
    char* ring = lds + wave * kRing;

    // DMA sources (per lane): W instruction i covers tiles 2i, 2i + 1 (lanes 0-31, 32-63), lane
    // (l & 31) = chain (l & 31) >> 2, branch pair l & 3; U instruction ft: frame l >> 2, pair l & 3
    const float2* ws[CTT / 2];
#pragma unroll
    for (int i = 0; i < CTT / 2; ++i) {
        const int c = cg * 8 * CTT + (2 * i + (lane >> 5)) * 8 + ((lane & 31) >> 2);
        ws[i] = W + (int64_t)kap * w_ks + fc_w_chain(c < nchains ? c : 0, (int)w_cs) +
                fc_w_branch(8 * kb0 + 2 * (lane & 3));
    }
    const float2* us[FTT];
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft) {
        const int f = fg * 16 * FTT + ft * 16 + (lane >> 2);
        us[ft] = U + ((int64_t)kap * Fs + (f < F ? f : 0)) * Dp + 8 * kb0 + 2 * (lane & 3);
    }
    auto issue = [&](int kb) {
        const int k = kb < nkb ? kb : nkb - 1;
        char* s = ring + (kb % NR) * kSlot;
#pragma unroll
        for (int i = 0; i < CTT / 2; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(ws[i] + (int64_t)k * kFcTile * 8),
                                             (__attribute__((address_space(3))) void*)(s + i * 1024), 16, 0, 0);
#pragma unroll
        for (int ft = 0; ft < FTT; ++ft)
            __builtin_amdgcn_global_load_lds((const void*)(us[ft] + 8 * k),
                                             (__attribute__((address_space(3))) void*)(s + (CTT / 2 + ft) * 1024), 16, 0, 0);
    };
    fc_f4 acc[FTT][CTT];
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
        for (int t = 0; t < CTT; ++t) acc[ft][t] = fc_f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < NR - 1; ++j) issue(j);
    constexpr int kWait = (NR - 1) * P;  // vmcnt once block kb has landed
    constexpr int kEnc = (kWait & 15) | ((kWait >> 4) << 14) | (7 << 4) | (15 << 8);
    for (int kb = 0; kb < nkb; ++kb) {
        issue(kb + NR - 1);  // into the slot block kb - 1 left (its reads retired before its MFMAs)
        __builtin_amdgcn_s_waitcnt(kEnc);
        __builtin_amdgcn_sched_barrier(0);
        const char* s = ring + (kb % NR) * kSlot;
        fc_f4 ua[FTT], wa[CTT];
#pragma unroll
        for (int t = 0; t < CTT; ++t) wa[t] = *(const fc_f4*)(s + t * 512 + cc * 64 + g * 16);
#pragma unroll
        for (int ft = 0; ft < FTT; ++ft) ua[ft] = *(const fc_f4*)(s + (CTT / 2 + ft) * 1024 + col * 64 + g * 16);
        __builtin_amdgcn_sched_barrier(0);  // all reads of the slot issued back to back
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            float bsel[CTT];
#pragma unroll
            for (int t = 0; t < CTT; ++t) {
                const float wr = (st < 2) ? wa[t].x : wa[t].z;
                const float wi = (st < 2) ? wa[t].y : wa[t].w;
                bsel[t] = (st & 1) ? (bim ? wr : -wi) : (bim ? wi : wr);
            }
#pragma unroll
            for (int ft = 0; ft < FTT; ++ft) {
                const float a = ua[ft][st];
#pragma unroll
                for (int t = 0; t < CTT; ++t)
                    acc[ft][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bsel[t], acc[ft][t], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // the clamped tail blocks land before the ring is reused
    __syncthreads();
    fc_f4* red = (fc_f4*)lds;  // [kFcKSplit - 1][FTT * CTT][64]
    if (wave > 0) {
#pragma unroll
        for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
            for (int t = 0; t < CTT; ++t) red[((wave - 1) * FTT * CTT + ft * CTT + t) * 64 + lane] = acc[ft][t];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
        for (int t = 0; t < CTT; ++t) {
            const int i = ft * CTT + t;
            acc[ft][t] = (acc[ft][t] + red[i * 64 + lane]) +
                         (red[(FTT * CTT + i) * 64 + lane] + red[(2 * FTT * CTT + i) * 64 + lane]);
        }
#pragma unroll
    for (int ft = 0; ft < FTT; ++ft)
#pragma unroll
        for (int t = 0; t < CTT; ++t) {
            const fc_f4 o = acc[ft][t];
            fc_f4 p;
            p.x = __shfl_xor(o.x, 1);
            p.y = __shfl_xor(o.y, 1);
            p.z = __shfl_xor(o.z, 1);
            p.w = __shfl_xor(o.w, 1);
            const int c = cg * 8 * CTT + t * 8 + cc;
            if (c >= nchains) continue;
            const int fb = fg * 16 * FTT + ft * 16 + 4 * g + (bim ? 2 : 0);
            const float2 y0 = bim ? make_float2(p.z, o.z) : make_float2(o.x, p.x);
            const float2 y1 = bim ? make_float2(p.w, o.w) : make_float2(o.y, p.y);
            float2* yc = Y + ((int64_t)c * Fs) * M + kap;
            if (fb < F) yc[(int64_t)fb * M] = y0;
            if (fb + 1 < F) yc[(int64_t)(fb + 1) * M] = y1;
        }
}

// ---- a member's spectra to another slot of the tiled W (swap-remove on a chain's leave) ------
// grid M (one bin each), block 256
__global__ void __launch_bounds__(256)
fc_move_w(float2* __restrict__ W, int64_t w_ks, int Dp, int src, int dst) {
    float2* row = W + (int64_t)blockIdx.x * w_ks;
    for (int r = threadIdx.x; r < Dp; r += 256)
        row[fc_w_chain(dst, Dp) + fc_w_branch(r)] = row[fc_w_chain(src, Dp) + fc_w_branch(r)];
}

hipError_t launch_fc_move_w(int M, float2* W, int64_t w_ks, int Dp, int src, int dst, hipStream_t st) {
    hipLaunchKernelGGL(fc_move_w, dim3(M), dim3(256), 0, st, W, w_ks, Dp, src, dst);
    return hipGetLastError();
}

int64_t fc_w_chain_offset(int c, int Dp) { return fc_w_chain(c, Dp); }

// Host self-test of the tiled W layout (owrx_selftest_w_layout): for a group of `cap` member
// slots and Dp branches, every (slot, branch) entry that fc_make_w / fc_move_w write and fc_mac /
// fc_mac_lds read lies inside the bin's row of cap * Dp entries, and no two share one.  0 if so;
// -1 for a geometry the engine never allocates (cap not a multiple of the tile, Dp not of 8);
// -2 for an entry outside the row; -3 for two entries on one element.
int fc_w_layout_check(int Dp, int cap) {
    if (Dp <= 0 || cap <= 0 || Dp % 8 || cap % kFcTile) return -1;
    const int64_t row = (int64_t)cap * Dp;
    std::vector<uint8_t> seen((size_t)row, 0);
    for (int c = 0; c < cap; ++c)
        for (int r = 0; r < Dp; ++r) {
            const int64_t o = fc_w_chain(c, Dp) + fc_w_branch(r);
            if (o < 0 || o >= row) return -2;
            if (seen[(size_t)o]++) return -3;
        }
    return 0;
}
int fc_w_tile() { return kFcTile; }

// ---- y_c[k0 + m] = rot_c(k0 + m) IDFT_M(Y_c[f])[m] into the group's output rows ------------
// grid: ceil(nchains F / RW) workgroups of RW = 1024 / M rows; block 256.
OWRX_DEV float2 fc_rotator(const DdcChain& ch, int64_t n) {
    const uint64_t ph = ch.P0 + (uint64_t)(n - ch.n0 + 1) * ch.rate_fx;
    const int32_t hi = (int32_t)(uint32_t)(ph >> 32);
    const float t = (float)hi * 2.3283064365386963e-10f;  // 2^-32
    float s, c;
    sincospif(2.0f * t, &s, &c);
    return make_float2(c, s);
}

template <int M>
__global__ void __launch_bounds__(256)
fc_out(const float2* __restrict__ Y, const DdcChain* __restrict__ chains, int nchains, int Fs,
       int F, int V, int D, int64_t k_begin, int nk, FcSubs sb,
       const float2* __restrict__ tw, float2* __restrict__ out, int ks, int64_t y_slice) {
    using FM = FcM<M>;
    constexpr int RW = FM::R3 ? 3072 / M : 1024 / M;
    constexpr int RS = FM::RS;
    __shared__ float2 sm[RW * RS];
    const int tid = threadIdx.x;
    const int row0 = blockIdx.x * RW;
    const int nrows = nchains * F;
    // conj(Y) in, forward DFT, conj out = M * IDFT(Y)
    for (int e = tid; e < RW * M; e += 256) {
        const int rr = e / M, kap = e % M;
        const int row = row0 + rr;
        float2 v = make_float2(0.0f, 0.0f);
        if (row < nrows) {
            const int c = row / F, f = row % F;
            const float2* y = Y + ((int64_t)c * Fs + f) * M + kap;
            v = y[0];
            for (int sl = 1; sl < ks; ++sl) {  // K slices in slice order (fixed)
                const float2 u = y[sl * y_slice];
                v = make_float2(v.x + u.x, v.y + u.y);
            }
        }
        sm[rr * RS + FM::tpos(kap)] = make_float2(v.x, -v.y);
    }
    __syncthreads();
    fc_fft_rows<M, RW, 256>(sm, tw);
    const float inv = 1.0f / (float)M;
    for (int e = tid; e < RW * M; e += 256) {
        const int rr = e / M, m = e % M;
        const int row = row0 + rr;
        if (row >= nrows || m >= V) continue;
        const int c = row / F, f = row % F;
        // the frame's sub-block (fc_fwd): its outputs [nk[s - 1], nk[s])
        const FcFrame fr = fc_frame_sub(sb, f, V);
        const int kk = fr.nk0 + (f - fr.f0) * V + m;
        if (kk >= sb.nk[fr.s]) continue;
        const float2 z = sm[rr * RS + FM::kpos(m)];
        const float2 y = make_float2(z.x * inv, -z.y * inv);
        const float2 rot = fc_rotator(chains[c], (k_begin + kk) * (int64_t)D);
        out[(int64_t)c * nk + kk] = cmul(y, rot);
    }
}

// ---- host launchers ----------------------------------------------------------------------

// K slices across workgroups for a tile grid of `tiles` workgroups: 1 when the tiles alone give
// every CU of the chip three or more workgroups; otherwise the smallest count that does (each
// wave of a slice must keep a whole number of the Dp / 8 K-blocks), at most kFcMaxKSlices.
// OWRX_FC_KSLICES=n forces n (A/B; 1 = the unsliced form).
int fc_kslices(int tiles, int Dp, int ncu) {
    static const int forced = [] {
        const char* v = getenv("OWRX_FC_KSLICES");
        return v ? atoi(v) : 0;
    }();
    const int per_wave = (Dp >> 3) / kFcKSplit;  // K-blocks per wave, unsliced
    auto ok = [&](int k) { return k >= 1 && k <= kFcMaxKSlices && per_wave % k == 0; };
    if (forced > 0) return ok(forced) ? forced : 1;
    // a grid of 1.5 or more workgroups per CU keeps whole K: C3's unpaired 384 tiles on 228 CUs
    // (1.7 per CU; the push path, ranks run with --no-pairing) ran 0.53 of HBM unsliced vs 0.51
    // with 3 slices (profiles/r04_fc_kslices_c3.txt, profiles/r05_c5_kslices.txt), and paired C3
    // grids are twice that; C4's 128 and C5's 64 tiles gain 0.32 -> 0.48 and 0.25 -> 0.36 from
    // slicing, and a paired C5 GEMM's 256 tiles (1.1 per CU) 0.26 -> 0.33 with 3 slices
    // (round 5 moved the bound to 2 per CU, which sliced unpaired C3 too: ADVICE r05)
    if (2 * tiles >= 3 * ncu) return 1;
    int best = 1;
    for (int k = 2; k <= kFcMaxKSlices; ++k) {
        if (!ok(k)) continue;
        best = k;
        if (tiles * k >= 3 * ncu) break;
    }
    return best;
}

// the most slices a group of nchains may use: its smallest tile grid (64-chain tiles, one frame
// tile) against the CU count of its stream
int fc_kslices_max(int M, int nchains, int Dp, int ncu) {
    return fc_kslices(M * ((nchains + 63) / 64), Dp, ncu);
}

#define OWRX_FC_SWITCH(m, CALL)          \
    switch (m) {                         \
        case 64: CALL(64); break;        \
        case 128: CALL(128); break;      \
        case 192: CALL(192); break;      \
        case 256: CALL(256); break;      \
        case 384: CALL(384); break;      \
        default: return hipErrorInvalidValue; \
    }

int fc_frame_supported(int m) { return m == 64 || m == 128 || m == 192 || m == 256 || m == 384; }

hipError_t launch_fc_make_w_jobs(int m, const float* h, int T, int D, int Dp, int P,
                                 const FcWJob* jobs, int njobs, float2* W, int64_t w_ks,
                                 hipStream_t st) {
    if (njobs <= 0) return hipSuccess;
    if (njobs > 65535) return hipErrorInvalidValue;
    const dim3 grid(Dp / kFcRT, njobs);
#define OWRX_FC_WJ(MM) hipLaunchKernelGGL(fc_make_w_jobs<MM>, grid, dim3(256), 0, st, h, T, D, P, jobs, W, w_ks)
    OWRX_FC_SWITCH(m, OWRX_FC_WJ)
#undef OWRX_FC_WJ
    return hipGetLastError();
}

hipError_t launch_fc_make_w(int m, const float* h, int T, int D, int Dp, int P,
                            uint64_t rate_fx, float2* W, int64_t w_ks, hipStream_t st) {
    const dim3 grid(Dp / kFcRT);
#define OWRX_FC_W(MM) hipLaunchKernelGGL(fc_make_w<MM>, grid, dim3(256), 0, st, h, T, D, Dp, P, rate_fx, W, w_ks)
    OWRX_FC_SWITCH(m, OWRX_FC_W)
#undef OWRX_FC_W
    return hipGetLastError();
}

// frames per block F = ceil(nk / V); U: [M][Fs][Dp], Y: [nchains][Fs][M], out: [nchains][nk].
// Grouped caller blocks (FcSubs): each sub-block's outputs in frames of their own; one GEMM over
// all of them (W read once for the group's blocks).
int fc_frames(const FcSubs& sb, int V) {
    int F = 0, k0 = 0;
    for (int s = 0; s < sb.n; ++s) {
        F += (sb.nk[s] - k0 + V - 1) / V;
        k0 = sb.nk[s];
    }
    return F;
}

hipError_t launch_fc_ddc(int M, const float2* blk, int64_t blk_start, const FcSubs& sb,
                         const DdcChain* chains, const float2* W, int64_t w_cs, int64_t w_ks,
                         int nchains, int D, int Dp, int V, int Fs, int64_t k_begin, int nk,
                         const float2* tw, float2* U, float2* Y, int64_t y_cap, float2* out,
                         int ncu, hipStream_t st, hipEvent_t mac0, hipEvent_t mac1, int* form) {
    if (sb.n < 1 || sb.n > kMaxSubBlocks || sb.nk[sb.n - 1] != nk) return hipErrorInvalidValue;
    for (int s = 0; s < sb.n; ++s)
        if (sb.nk[s] < (s ? sb.nk[s - 1] : 0) || sb.end[s] < (s ? sb.end[s - 1] : blk_start))
            return hipErrorInvalidValue;
    const int F = fc_frames(sb, V);
    if (F > Fs || nk <= 0 || nchains <= 0) return hipErrorInvalidValue;
    const dim3 gf(Dp / kFcRT, F);
#define OWRX_FC_F(MM) hipLaunchKernelGGL(fc_fwd<MM>, gf, dim3(256), 0, st, blk, blk_start, sb, k_begin, V, D, Dp, Fs, tw, U)
    OWRX_FC_SWITCH(M, OWRX_FC_F)
#undef OWRX_FC_F
    HIPCHK_RET(hipGetLastError());
    // the LDS-DMA ring form by default: C3 fc_mac 0.469-0.495 of HBM vs 0.455-0.465 with register
    // operands, 5 815-5 899 vs 5 712-5 788 Msps, same box (profiles/r03al_ab_fc_mac_lds_c3.txt);
    // OWRX_FC_MAC=reg: the register form (A/B)
    static const bool lds_ring = [] {
        const char* v = getenv("OWRX_FC_MAC");
        return !(v && strcmp(v, "reg") == 0);
    }();
    // wave tiles: 32 frames x 32 chains, or 16 frames x 64 chains when a block has <= 16 frames.
    // OWRX_FC_TALL=1 (A/B): 64 frames x 32 chains past 32 frames (grouped blocks: C3 quads,
    // F = 52), one frame tile and twice the MFMAs per K-block's loads -- but 320 registers, one
    // wave per SIMD: C3 quads 0.40 of the MFMA peak vs 0.43 with the 32-frame tiles, whose W tile
    // the frame-tile-fastest decode serves from L2 to the second tile (profiles/r06_fc_tall_ab.txt)
    static const bool tall_ok = [] {
        const char* v = getenv("OWRX_FC_TALL");
        return v && strcmp(v, "1") == 0;
    }();
    bool tall = tall_ok && F > 32 && lds_ring;
    const bool wide = F > 16;
    int ctt = 0, ftt = 0, ncg = 0, nfg = 0;
    dim3 gm;
    auto shape = [&]() {
        ctt = tall ? 4 : wide ? 4 : 8;
        ftt = tall ? 4 : wide ? 2 : 1;
        ncg = (nchains + 8 * ctt - 1) / (8 * ctt);
        nfg = (F + 16 * ftt - 1) / (16 * ftt);
        gm = dim3(M * ncg * nfg);
    };
    shape();
    // the tall tiles only in the ring form (below): a grid of one round keeps the register form
    if (tall && (int)gm.x <= (ncu > 0 ? ncu : 256)) {
        tall = false;
        shape();
    }
    if (Dp % kFcDpAlign) return hipErrorInvalidValue;
    static const int chain_fastest = [] {  // OWRX_FC_ORDER=kappa: the previous order (A/B)
        const char* v = getenv("OWRX_FC_ORDER");
        return (v && strcmp(v, "kappa") == 0) ? 0 : 1;
    }();
    // the ring where the grid needs two or more workgroups per CU (C3: 512); a grid one round of
    // single workgroups holds (C4's per-GPU share: 128, long K) keeps register operands, which
    // measured 6 % faster there than the ring at 2 or 4 slots (profiles/r03ap_ab_fc_mac_c4.txt).
    // ncu: the CUs of the launching stream (stream A's mask, not the device's 256: a paired C5
    // GEMM's 256 workgroups took the register form and two rounds on A's 228 CUs)
    ncu = ncu > 0 ? ncu : 256;
    // K slices across workgroups where the tile grid leaves CUs idle (fc_kslices)
    const int64_t y_slice = (int64_t)nchains * Fs * M;
    int ks = lds_ring ? fc_kslices((int)gm.x, Dp, ncu) : 1;
    while (ks > 1 && ks * y_slice > y_cap) --ks;  // within the group's Y (fc_kslices_max)
    while (ks > 1 && ((Dp >> 3) / kFcKSplit) % ks) --ks;
    const dim3 gk(gm.x * ks);
    const bool ring = lds_ring && (int)gk.x > ncu;
    if (form) *form = ring ? ks : 0;  // 0: register form; k >= 1: the ring with k K slices
    if (mac0) HIPCHK_RET(hipEventRecord(mac0, st));
    if (ring && tall)
        hipLaunchKernelGGL((fc_mac_lds<4, 4, 2>), gk, dim3(64 * kFcKSplit), 0, st, U, W, w_cs, w_ks, nchains, Fs, F, Dp, M, ncg, chain_fastest, Y, ks, y_slice);
    else if (ring && wide)
        hipLaunchKernelGGL((fc_mac_lds<2, 4, 2>), gk, dim3(64 * kFcKSplit), 0, st, U, W, w_cs, w_ks, nchains, Fs, F, Dp, M, ncg, chain_fastest, Y, ks, y_slice);
    else if (ring)
        hipLaunchKernelGGL((fc_mac_lds<1, 8, 2>), gk, dim3(64 * kFcKSplit), 0, st, U, W, w_cs, w_ks, nchains, Fs, F, Dp, M, ncg, chain_fastest, Y, ks, y_slice);
    else if (wide)  // (the register form keeps 32-frame tiles: at 64 it spills)
        hipLaunchKernelGGL((fc_mac<2, 4, false>), gm, dim3(64 * kFcKSplit), 0, st, U, W, w_cs, w_ks, nchains, Fs, F, Dp, M, ncg, chain_fastest, Y);
    else
        hipLaunchKernelGGL((fc_mac<1, 8, false>), gm, dim3(64 * kFcKSplit), 0, st, U, W, w_cs, w_ks, nchains, Fs, F, Dp, M, ncg, chain_fastest, Y);
    HIPCHK_RET(hipGetLastError());
    if (mac1) HIPCHK_RET(hipEventRecord(mac1, st));
    const int rw = (M % 3 == 0) ? 3072 / M : 1024 / M;
    const dim3 go((nchains * F + rw - 1) / rw);
#define OWRX_FC_O(MM) hipLaunchKernelGGL(fc_out<MM>, go, dim3(256), 0, st, Y, chains, nchains, Fs, F, V, D, k_begin, nk, sb, tw, out, ring ? ks : 1, y_slice)
    OWRX_FC_SWITCH(M, OWRX_FC_O)
#undef OWRX_FC_O
    return hipGetLastError();
}

#undef OWRX_FC_SWITCH

}  // namespace owrx
