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
// Phases are split into `nseg` segments across workgroups to fill the chip, each segment four
// ways across the waves of its workgroup (reduced through LDS); the post kernel adds the
// segment partials in a fixed order (deterministic).
#include <type_traits>

#include "owrx_types.h"

namespace owrx {

typedef float f2v __attribute__((ext_vector_type(2)));  // packed FP32 (v_pk_fma_f32) pair

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

constexpr int kDdcWaves = 4;  // phase sub-segments per workgroup, reduced through LDS

// Tuning knobs (defaults = the production configuration, launch_ddc_p):
//   R    outputs per lane (register tile)          WPE  waves-per-SIMD target (VGPR budget)
//   SB   scheduling barrier every SB samples (bounds load hoisting), 0 = none
// Measured on MI355X (tools/micro/ddc_bench.cpp, D = 833, 27 phases x 32 outputs): R = 32,
// WPE = 2, SB = 16 -> 58 TFLOP/s at 32 chains, 65 TFLOP/s at 256 (buffer-load addressing was
// 2x slower than the flat loads; WPE >= 3 spills).
template <int P, int R, int WPE, int SB>
__global__ void __launch_bounds__(64 * kDdcWaves) __attribute__((amdgpu_waves_per_eu(WPE)))
ddc_polyphase(const float2* __restrict__ blk, int64_t blk_start, int64_t blk_end,
              const float* __restrict__ taps_poly,  // [D][P]: taps_poly[r*P + p] = h[pD + r]
              const DdcChain* __restrict__ chains, int nchains, int D, int64_t k_begin,
              int nk, int cpw, int tpw, int pps, float2* __restrict__ partial) {
    // the workgroup's waves share one tile group and split its phase segment four ways
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int tg = blockIdx.x;
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

    const int sub = seg * kDdcWaves + wave;
    const int r_begin = min(D, sub * pps);
    const int r_end = min(D, r_begin + pps);

    // (re, im) accumulator pairs: one v_pk_fma_f32 per tap and output (2 FMAs per instruction,
    // the form the FP32 vector peak assumes)
    f2v acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = f2v{0.0f, 0.0f};

    // lane offset (in samples) from the wave's first tile: the per-q sample address is then a
    // wave-uniform base (SGPR arithmetic) plus this fixed per-lane offset
    const int ti_c = tile_c - tg * tpw;
    const int lane_off = ti_c * R * D;
    const int64_t k0_wave = k_begin + (int64_t)tg * tpw * R;
    const f2v wv = f2v{ch.wD.x, ch.wD.y};
    const f2v wp = f2v{-ch.wD.y, ch.wD.x};  // j * wD

    for (int r = r_begin; r < r_end; ++r) {
        float h[P];
#pragma unroll
        for (int p = 0; p < P; ++p) h[p] = taps_poly[r * P + p];
        const int64_t n0 = k0 * D + r;  // absolute index of q = 0
        const float2 rot0 = seed_rotator(ch, n0);
        f2v rv = f2v{rot0.x, rot0.y};
        const float2* wbase = blk + (k0_wave * D + r - blk_start);  // wave-uniform
        // fast path: every lane's window [n0, n0 + (R+P-2) D] lies inside the block
        const bool inside = n0 + (int64_t)(R + P - 2) * D < blk_end;
        auto body = [&](auto clamp) {
            constexpr bool CLAMP = decltype(clamp)::value;
            int qmax32 = R + P;
            if (CLAMP) {  // last q whose sample is inside the block (later ones feed discarded outputs)
                const int64_t qmax = (blk_end - 1 - n0) / D;
                qmax32 = (int)(qmax < (int64_t)(R + P) ? qmax : (int64_t)(R + P));
            }
            // fully unrolled at compile time: every acc index is a constant (registers, no scratch)
            static_for<0, R + P - 1>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                float2 x;
                if (CLAMP) {
                    const int qq = q < qmax32 ? q : qmax32;
                    x = wbase[qq * D + lane_off];
                } else {
                    const float2* wq = wbase + q * D;  // uniform
                    x = wq[lane_off];
                }
                // s = x * rot, rot *= wD, as packed pairs: x.re * rot + x.im * (j rot)
                const f2v rp = f2v{-rv.y, rv.x};
                const f2v sv = __builtin_elementwise_fma(f2v{x.y, x.y}, rp, f2v{x.x, x.x} * rv);
                rv = __builtin_elementwise_fma(f2v{rv.y, rv.y}, wp, f2v{rv.x, rv.x} * wv);
                constexpr int plo = q - R + 1 > 0 ? q - R + 1 : 0;
                constexpr int phi = q < P - 1 ? q : P - 1;
                static_for<plo, phi + 1>([&](auto pc) {
                    constexpr int p = decltype(pc)::value;
                    acc[q - p] = __builtin_elementwise_fma(f2v{h[p], h[p]}, sv, acc[q - p]);
                });
                // bound the scheduler's load hoisting (keeps ~8 samples in flight per wave
                // instead of the whole window, which would cost occupancy)
                if constexpr (SB > 0 && (q % SB) == SB - 1) __builtin_amdgcn_sched_barrier(0);
            });
        };
        if (__all(inside)) body(std::false_type{});
        else body(std::true_type{});
    }
    // fixed-order tree over the four waves: ((w0 + w2) + (w1 + w3))
    __shared__ float2 red[2][R][64];
    if (wave >= 2) {
#pragma unroll
        for (int i = 0; i < R; ++i) red[wave - 2][i][lane] = make_float2(acc[i].x, acc[i].y);
    }
    __syncthreads();
    if (wave < 2) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const float2 v = red[wave][i][lane];
            acc[i] += f2v{v.x, v.y};
        }
    }
    __syncthreads();
    if (wave == 1) {
#pragma unroll
        for (int i = 0; i < R; ++i) red[0][i][lane] = make_float2(acc[i].x, acc[i].y);
    }
    __syncthreads();
    if (wave != 0 || !active) return;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const float2 v = red[0][i][lane];
        acc[i] += f2v{v.x, v.y};
    }
    float2* out = partial + ((int64_t)seg * nchains + chain) * nk;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int kk = tile * R + i;
        if (kk < nk) out[kk] = make_float2(acc[i].x, acc[i].y);
    }
}

template <int P, int R = 32, int WPE = 2, int SB = 16>
static hipError_t launch_ddc_p(const float2* blk, int64_t blk_start, int64_t blk_end,
                               const float* taps_poly, const DdcChain* chains, int nchains,
                               int D, int64_t k_begin, int nk, int nseg, float2* partial,
                               hipStream_t st) {
    int cpw = 1;
    while (cpw < nchains && cpw < 64) cpw <<= 1;
    const int tpw = 64 / cpw;
    const int ntiles = (nk + R - 1) / R;
    const int ntg = (ntiles + tpw - 1) / tpw;
    const int ncg = (nchains + cpw - 1) / cpw;
    const int pps = (D + kDdcWaves * nseg - 1) / (kDdcWaves * nseg);
    dim3 grid(ntg, nseg, ncg);  // nseg comes from ddc_segments (no empty segment)
    hipLaunchKernelGGL((ddc_polyphase<P, R, WPE, SB>), grid, dim3(64 * kDdcWaves), 0, st, blk, blk_start,
                       blk_end, taps_poly, chains, nchains, D, k_begin, nk, cpw, tpw, pps,
                       partial);
    return hipGetLastError();
}

// Supported polyphase depths; taps are zero padded up to the instantiated P.
int ddc_padded_p(int p) {
    static const int ps[] = {8, 16, 27, 28, 30, 32, 36, 40, 48, 64};
    for (int v : ps)
        if (p <= v) return v;
    return -1;
}

// Number of phase segments (= partial sums written per output) actually launched for a
// requested split; each segment is kDdcWaves sub-segments of pps phases, one per wave.
int ddc_segments(int D, int nseg) {
    const int pps = (D + kDdcWaves * nseg - 1) / (kDdcWaves * nseg);
    const int subs = (D + pps - 1) / pps;
    return (subs + kDdcWaves - 1) / kDdcWaves;
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
