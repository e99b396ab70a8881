// kernels_ddc.hip -- Selector front end fused for every client chain that shares one
// FirDecimate design: Shift(rate_c) (csdr/chain/selector.py:95,132-140) followed by
// FirDecimate(D, transition, cutoff) (selector.py:11-35).
//
//   y_c[m] = sum_{t<T} h[t] * x[s0_c + mD + t] * exp(j 2 pi (mD + t + 1) rate_c)
//
// Polyphase form t = pD + r (r < D, p < P = ceil(T/D) ~ 27 for this chain family):
//   y_c[m] = sum_r sum_p h[pD + r] * s_c[(m + p) D + r].
// A lane owns one (chain, tile of R consecutive outputs); a wave's lanes share the phase r
// being processed, so the P taps of phase r are wave-uniform (scalar loads, SGPR operands)
// and the sample loads x[(m0 + q) D + r] are wave-uniform per tile (1-2 distinct addresses
// per wave-load, served by L1/L2).  Each loaded sample is rotated once (complex multiply by
// a per-lane rotator, seeded exactly from 64-bit fixed-point phase once per phase and advanced
// by exp(j 2 pi D rate) per sample) and then feeds up to P accumulators: ~27 complex x real
// MACs (54 FMAs) per load, so the kernel is FP32-VALU bound, not HBM bound.
// Phases are split into `nseg` segments across workgroups to fill the chip; the post kernel
// adds the segment partials in a fixed order (deterministic).
#include <type_traits>

#include "owrx_types.h"

namespace owrx {

template <int I, int N, typename F>
OWRX_DEV void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

OWRX_DEV float2 seed_rotator(const DdcChain& ch, int64_t n) {
    // exp(j 2 pi (P0 + (n - n0 + 1) * rate)), phase exact in 2^-64 turns
    const uint64_t ph = ch.P0 + (uint64_t)(n - ch.n0 + 1) * ch.rate_fx;
    // top 32 bits -> signed turns in [-0.5, 0.5)
    const int32_t hi = (int32_t)(uint32_t)(ph >> 32);
    const float t = (float)hi * 2.3283064365386963e-10f;  // 2^-32
    float s, c;
    sincospif(2.0f * t, &s, &c);
    return make_float2(c, s);
}

template <int P, int R>
__global__ void __launch_bounds__(256)
ddc_polyphase(const float2* __restrict__ blk, int64_t blk_start, int64_t blk_end,
              const float* __restrict__ taps_poly,  // [D][P]: taps_poly[r*P + p] = h[pD + r]
              const DdcChain* __restrict__ chains, int nchains, int D, int64_t k_begin,
              int nk, int cpw, int tpw, int ntg, int pps, float2* __restrict__ partial) {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int tg = blockIdx.x * 4 + wave;  // tile group handled by this wave
    if (tg >= ntg) return;                 // wave-uniform
    const int seg = blockIdx.y;
    const int ci = lane % cpw;
    const int ti = lane / cpw;
    const int chain_raw = blockIdx.z * cpw + ci;
    const int tile = tg * tpw + ti;
    const bool active = (ti < tpw) && (chain_raw < nchains) && (tile * R < nk);
    const int chain = chain_raw < nchains ? chain_raw : nchains - 1;
    const int tile_c = (tile * R < nk) ? tile : (nk - 1) / R;
    const DdcChain ch = chains[chain];
    const int64_t k0 = k_begin + (int64_t)tile_c * R;

    const int r_begin = seg * pps;
    const int r_end = min(D, r_begin + pps);

    float2 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = make_float2(0.0f, 0.0f);

    for (int r = r_begin; r < r_end; ++r) {
        float h[P];
#pragma unroll
        for (int p = 0; p < P; ++p) h[p] = taps_poly[r * P + p];
        const int64_t n0 = k0 * D + r;  // absolute index of q = 0
        float2 rot = seed_rotator(ch, n0);
        const float2 wD = ch.wD;
        // last q whose sample is inside the block (samples past it only feed discarded outputs)
        const int64_t qmax = (blk_end - 1 - n0) / D;
        const float2* xp = blk + (n0 - blk_start);
        const int qmax32 = (int)(qmax < (int64_t)(R + P) ? qmax : (int64_t)(R + P));
        // fully unrolled at compile time: every acc index is a constant (registers, no scratch)
        static_for<0, R + P - 1>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const int qq = q < qmax32 ? q : qmax32;
            const float2 x = xp[qq * D];
            const float2 s = cmul(x, rot);
            rot = cmul(rot, wD);
            constexpr int plo = q - R + 1 > 0 ? q - R + 1 : 0;
            constexpr int phi = q < P - 1 ? q : P - 1;
            static_for<plo, phi + 1>([&](auto pc) {
                constexpr int p = decltype(pc)::value;
                acc[q - p].x = fmaf(h[p], s.x, acc[q - p].x);
                acc[q - p].y = fmaf(h[p], s.y, acc[q - p].y);
            });
            // bound the scheduler's load hoisting (keeps ~8 samples in flight per wave instead of
            // the whole window, which would cost 1 wave/SIMD of occupancy)
            if constexpr ((q % 8) == 7) __builtin_amdgcn_sched_barrier(0);
        });
    }
    if (!active) return;
    float2* out = partial + ((int64_t)seg * nchains + chain) * nk;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int kk = tile * R + i;
        if (kk < nk) out[kk] = acc[i];
    }
}

template <int P>
static hipError_t launch_ddc_p(const float2* blk, int64_t blk_start, int64_t blk_end,
                               const float* taps_poly, const DdcChain* chains, int nchains,
                               int D, int64_t k_begin, int nk, int nseg, float2* partial,
                               hipStream_t st) {
    constexpr int R = 32;
    int cpw = 1;
    while (cpw < nchains && cpw < 64) cpw <<= 1;
    const int tpw = 64 / cpw;
    const int ntiles = (nk + R - 1) / R;
    const int ntg = (ntiles + tpw - 1) / tpw;
    const int ncg = (nchains + cpw - 1) / cpw;
    const int pps = (D + nseg - 1) / nseg;
    const int segs = (D + pps - 1) / pps;
    dim3 grid((ntg + 3) / 4, segs, ncg);
    hipLaunchKernelGGL((ddc_polyphase<P, R>), grid, dim3(256), 0, st, blk, blk_start, blk_end,
                       taps_poly, chains, nchains, D, k_begin, nk, cpw, tpw, ntg, pps, partial);
    return hipGetLastError();
}

// Supported polyphase depths; taps are zero padded up to the instantiated P.
int ddc_padded_p(int p) {
    static const int ps[] = {8, 16, 27, 28, 30, 32, 36, 40, 48, 64};
    for (int v : ps)
        if (p <= v) return v;
    return -1;
}

// Number of phase segments actually launched for a requested split.
int ddc_segments(int D, int nseg) {
    const int pps = (D + nseg - 1) / nseg;
    return (D + pps - 1) / pps;
}

hipError_t launch_ddc(int P, const float2* blk, int64_t blk_start, int64_t blk_end,
                      const float* taps_poly, const DdcChain* chains, int nchains, int D,
                      int64_t k_begin, int nk, int nseg, float2* partial, hipStream_t st) {
#define OWRX_DDC_CASE(v)                                                                    \
    case v:                                                                                 \
        return launch_ddc_p<v>(blk, blk_start, blk_end, taps_poly, chains, nchains, D,     \
                               k_begin, nk, nseg, partial, st);
    switch (P) {
        OWRX_DDC_CASE(8)
        OWRX_DDC_CASE(16)
        OWRX_DDC_CASE(27)
        OWRX_DDC_CASE(28)
        OWRX_DDC_CASE(30)
        OWRX_DDC_CASE(32)
        OWRX_DDC_CASE(36)
        OWRX_DDC_CASE(40)
        OWRX_DDC_CASE(48)
        OWRX_DDC_CASE(64)
        default:
            return hipErrorInvalidValue;
    }
#undef OWRX_DDC_CASE
}

}  // namespace owrx
