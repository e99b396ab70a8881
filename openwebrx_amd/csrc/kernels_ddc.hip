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
//
// Production kernel: ddc_lds (ddc_kernels.h) stages each chunk of 16 phases x (tiles + P - 1)
// sample rows in LDS with coalesced loads, double-buffered, so the inner loop is ds_read_b64
// at immediate offsets + packed FMAs.  Measured on MI355X (tools/micro/ddc_bench.cpp, D = 833,
// P = 27): 67-74 TFLOP/s at 32 chains and 80-87 at 256, against 50-56 / 60-66 for the
// register-direct ddc_polyphase (OWRX_DDC_KERNEL=flat, kept for A/B at P = 27).
#include <atomic>
#include <stdlib.h>
#include <string.h>

#include "ddc_kernels.h"

namespace owrx {

// Kernel selection: ddc_lds (production) or the register-direct ddc_polyphase
// (OWRX_DDC_KERNEL=flat, kept for A/B measurements).
static bool ddc_flat() {
    static const bool flat = [] {
        const char* v = getenv("OWRX_DDC_KERNEL");
        return v && strcmp(v, "flat") == 0;
    }();
    return flat;
}

static int ddc_tiles_per_wave(int nchains) {
    int cpw = 1;
    while (cpw < nchains && cpw < 64) cpw <<= 1;
    return 64 / cpw;
}

static bool ddc_uses_flat(int P, int nchains) {
    return (P == 27 && ddc_flat()) || ddc_tiles_per_wave(nchains) > kLdsMaxTiles;
}

OWRX_DDC_DEPTHS(OWRX_DDC_INSTANTIATE, extern)

// Resident workgroups per CU of the kernel a group of nchains runs (launch-shape choice in
// engine.hip).
int ddc_blocks_per_cu(int P, int nchains) {
    const bool flat = ddc_uses_flat(P, nchains);
    const int tpw = ddc_tiles_per_wave(nchains);
    // memoised per (depth, form, tiles per wave): the occupancy query cost ~10 us per chain
    // create (group_refresh_device runs on every join)
    static std::atomic<int> memo[7][2][7];
    const int pi = P == 8 ? 0 : P == 16 ? 1 : P == 27 ? 2 : P == 28 ? 3 : P == 32 ? 4 : P == 48 ? 5 : 6;
    int ti = 0;
    while (ti < 6 && (1 << ti) < tpw) ++ti;
    std::atomic<int>& m = memo[pi][flat ? 1 : 0][ti];
    const int known = m.load(std::memory_order_relaxed);
    if (known > 0) return known;
    int nb = 2;
    switch (P) {
        case 8: nb = ddc_occ<8>(flat, tpw); break;
        case 16: nb = ddc_occ<16>(flat, tpw); break;
        case 27: nb = ddc_occ<27>(flat, tpw); break;
        case 28: nb = ddc_occ<28>(flat, tpw); break;
        case 32: nb = ddc_occ<32>(flat, tpw); break;
        case 48: nb = ddc_occ<48>(flat, tpw); break;
        case 64: nb = ddc_occ<64>(flat, tpw); break;
        default: return 2;
    }
    m.store(nb, std::memory_order_relaxed);
    return nb;
}

// Supported polyphase depths; taps are zero padded up to the instantiated P.
int ddc_padded_p(int p) {
    static const int ps[] = {8, 16, 27, 28, 32, 48, 64};
    for (int v : ps)
        if (p <= v) return v;
    return -1;
}

// Number of phase segments (= partial sums written per output) actually launched for a
// requested split; each segment is kDdcWaves sub-segments of pps phases, one per wave.
int ddc_segments(int D, int nseg, int P, int nchains) {
    if (!ddc_uses_flat(P, nchains)) {
        const int len = ddc_seg_len(D, nseg);
        return (D + len - 1) / len;
    }
    const int pps = (D + kDdcWaves * nseg - 1) / (kDdcWaves * nseg);
    const int subs = (D + pps - 1) / pps;
    return (subs + kDdcWaves - 1) / kDdcWaves;
}

hipError_t launch_ddc(int P, const float2* blk, int64_t blk_start, int64_t blk_end,
                      const float* taps_poly, const DdcChain* chains, int nchains, int D,
                      int64_t k_begin, int nk, int nseg, float2* partial, hipStream_t st) {
    // ddc_lds stages (tiles per wave x R + P - 1) sample rows and is built for at most
    // kLdsMaxTiles tiles per wave (32+ chains); smaller groups, where the DDC is cheap anyway,
    // run the register-direct kernel
    const bool flat = ddc_uses_flat(P, nchains);
#define OWRX_DDC_CASE(v)                                                                    \
    case v:                                                                                 \
        if (flat)                                                                           \
            return launch_ddc_p<v>(blk, blk_start, blk_end, taps_poly, chains, nchains, D,  \
                                   k_begin, nk, nseg, partial, st);                         \
        return launch_ddc_lds_p<v>(blk, blk_start, blk_end, taps_poly, chains, nchains, D,   \
                                   k_begin, nk, nseg, partial, st);
    switch (P) {
        OWRX_DDC_CASE(8)
        OWRX_DDC_CASE(16)
        OWRX_DDC_CASE(27)
        OWRX_DDC_CASE(28)
        OWRX_DDC_CASE(32)
        OWRX_DDC_CASE(48)
        OWRX_DDC_CASE(64)
        default:
            return hipErrorInvalidValue;
    }
#undef OWRX_DDC_CASE
}

}  // namespace owrx
