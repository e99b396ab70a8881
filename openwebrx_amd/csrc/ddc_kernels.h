// ddc_kernels.h -- the DDC kernel templates (see kernels_ddc.hip for the design notes).
#pragma once
#include <stdlib.h>
#include <string.h>

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

// ---- LDS-staged variant (production) ------------------------------------------------------
// Same arithmetic and lane mapping as ddc_polyphase, but the workgroup's samples are staged
// through LDS: the phase range of a segment is walked in chunks of kChunk phases (kPhW per
// wave), and for each chunk the workgroup copies the (tpw*R + P - 1) x kChunk sample window
// from HBM/L2 with coalesced loads (rows of kChunk consecutive samples) into one of two LDS
// buffers while the waves compute the previous chunk.  Each lane then reads its samples with
// ds_read_b64 at compile-time offsets (every lane of a tile broadcasts one address), so the
// inner loop has no address arithmetic and no vector-memory waits; samples past the block end
// are staged as zeros (they only meet the zero padding of the last polyphase row or feed
// outputs beyond nk).  The complex rotations use v_pk_* operand modifiers (op_sel / neg) so
// a sample costs two packed instructions to rotate and two to advance the rotator, bit-identical
// to ddc_polyphase's fma(x.im, j*rot, x.re * rot) order.
constexpr int kPhW = 4;                       // phases per wave per chunk
constexpr int kChunk = kPhW * kDdcWaves;      // phases per chunk (LDS row length)
constexpr int kLdsMaxTiles = 2;               // tiles per wave the staging registers cover

// (re, im) * (re, im): two packed instructions
OWRX_DEV f2v cmul_pk(f2v x, f2v r) {
    f2v t, s;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(x), "v"(r));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(s)
        : "v"(x), "v"(r), "v"(t));
    return s;
}

template <int P, int R, int WPE>
__global__ void __launch_bounds__(64 * kDdcWaves) __attribute__((amdgpu_waves_per_eu(WPE)))
ddc_lds(const float2* __restrict__ blk, int64_t blk_start, int64_t blk_end,
        const float* __restrict__ taps_poly, const DdcChain* __restrict__ chains, int nchains,
        int D, int64_t k_begin, int nk, int cpw, int tpw, int seg_len,
        float2* __restrict__ partial) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: SGPR taps
    const int lane = threadIdx.x & 63;
    const int tg = blockIdx.x;
    const int seg = blockIdx.y;
    const int ci = lane % cpw;
    const int ti = lane / cpw;
    const int chain_raw = blockIdx.z * cpw + ci;
    const int tile = tg * tpw + ti;
    const bool active = (ti < tpw) && (chain_raw < nchains) && (tile * R < nk);
    const int chain = chain_raw < nchains ? chain_raw : nchains - 1;
    const DdcChain ch = chains[chain];
    const int64_t k0 = k_begin + (int64_t)tile * R;  // lane's first output
    const int64_t k0_wave = k_begin + (int64_t)tg * tpw * R;
    const int Q = tpw * R + P - 1;                   // window rows
    const int rb = seg * seg_len;
    const int re = min(D, rb + seg_len);
    const int nchunks = (re - rb + kChunk - 1) / kChunk;
    const int lane_row = (ti < tpw ? ti : 0) * R;    // lane's first window row
    const int buf_elems = Q * kChunk;                // one chunk buffer (two, alternating)

    // staging: element e -> (row q = e / kChunk, column c = e % kChunk); per thread at most
    // kFill elements per chunk, held in registers while the previous chunk is computed
    constexpr int kFill =
        ((kLdsMaxTiles * R + P - 1) * kChunk + 64 * kDdcWaves - 1) / (64 * kDdcWaves);
    const int nel = Q * kChunk;
    float2 st[kFill];
    auto fetch = [&](int c) {
        const int r0 = rb + c * kChunk;
#pragma unroll
        for (int u = 0; u < kFill; ++u) {
            const int e = threadIdx.x + u * 64 * kDdcWaves;
            const int q = e / kChunk, col = e % kChunk;
            const int64_t n = (k0_wave + q) * (int64_t)D + r0 + col;
            st[u] = (e < nel && r0 + col < re && n < blk_end) ? blk[n - blk_start]
                                                                : make_float2(0.0f, 0.0f);
        }
    };
    auto stash = [&](int c) {
        float2* b = lds + (c & 1) * buf_elems;
#pragma unroll
        for (int u = 0; u < kFill; ++u) {
            const int e = threadIdx.x + u * 64 * kDdcWaves;
            if (e < nel) b[e] = st[u];
        }
    };

    f2v acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = f2v{0.0f, 0.0f};
    const f2v wv = f2v{ch.wD.x, ch.wD.y};

    fetch(0);
    stash(0);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        if (c + 1 < nchunks) fetch(c + 1);  // in flight while this chunk is computed
        const int r0 = rb + c * kChunk;
        const float2* col_base = lds + (c & 1) * buf_elems + lane_row * kChunk;
        for (int j = 0; j < kPhW; ++j) {
            const int rc = wave * kPhW + j;  // column in the chunk
            const int r = r0 + rc;
            if (r >= re) break;              // wave-uniform
            float h[P];
#pragma unroll
            for (int p = 0; p < P; ++p) h[p] = taps_poly[r * P + p];
            const float2 rot0 = seed_rotator(ch, k0 * D + r);
            f2v rv = f2v{rot0.x, rot0.y};
            const float2* xs = col_base + rc;
            static_for<0, R + P - 1>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const float2 x = xs[q * kChunk];
                const f2v sv = cmul_pk(f2v{x.x, x.y}, rv);
                rv = cmul_pk(rv, wv);
                constexpr int plo = q - R + 1 > 0 ? q - R + 1 : 0;
                constexpr int phi = q < P - 1 ? q : P - 1;
                static_for<plo, phi + 1>([&](auto pc) {
                    constexpr int p = decltype(pc)::value;
                    acc[q - p] = __builtin_elementwise_fma(f2v{h[p], h[p]}, sv, acc[q - p]);
                });
            });
        }
        if (c + 1 < nchunks) stash(c + 1);
        __syncthreads();
    }
    // fixed-order tree over the four waves: ((w0 + w2) + (w1 + w3)), through the same LDS
    float2* red = lds;  // [2][R][64]
    if (wave >= 2) {
#pragma unroll
        for (int i = 0; i < R; ++i) red[((wave - 2) * R + i) * 64 + lane] = make_float2(acc[i].x, acc[i].y);
    }
    __syncthreads();
    if (wave < 2) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const float2 v = red[(wave * R + i) * 64 + lane];
            acc[i] += f2v{v.x, v.y};
        }
    }
    __syncthreads();
    if (wave == 1) {
#pragma unroll
        for (int i = 0; i < R; ++i) red[i * 64 + lane] = make_float2(acc[i].x, acc[i].y);
    }
    __syncthreads();
    if (wave != 0 || !active) return;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const float2 v = red[i * 64 + lane];
        acc[i] += f2v{v.x, v.y};
    }
    float2* out = partial + ((int64_t)seg * nchains + chain) * nk;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int kk = tile * R + i;
        if (kk < nk) out[kk] = make_float2(acc[i].x, acc[i].y);
    }
}

constexpr int kLdsR = 32;
#ifndef OWRX_DDC_LDS_WPE
#define OWRX_DDC_LDS_WPE 4
#endif
// waves-per-EU target of ddc_lds: 4 caps it at 128 VGPRs (132 at 2, i.e. 3 waves per SIMD);
// the compiler then spills 8 VGPRs, all outside the chunk loop (prologue and the final wave
// reduction).  Same-box A/B on MI355X: +4 % DDC TFLOP/s at 32 chains, +6 % at 256.
constexpr int kLdsWpe = OWRX_DDC_LDS_WPE;



// Phases per segment for a requested split: whole chunks, so only the last segment has a
// partial chunk.  The number of segments actually launched is ceil(D / seg_len).
inline int ddc_seg_len(int D, int nseg) {
    const int chunks = (D + kChunk - 1) / kChunk;
    const int per = (chunks + nseg - 1) / nseg;
    return per * kChunk;
}


// LDS bytes of ddc_lds for a window of tpw tiles (max of the two chunk buffers and the
// 4-wave reduction buffer)
inline size_t ddc_lds_bytes(int P, int tpw, int R = kLdsR) {
    const size_t win = (size_t)2 * (tpw * R + P - 1) * kChunk * sizeof(float2);
    const size_t red = (size_t)2 * R * 64 * sizeof(float2);
    return win > red ? win : red;
}

template <int P, int WPE = kLdsWpe, int R = kLdsR>
hipError_t launch_ddc_lds_p(const float2* blk, int64_t blk_start, int64_t blk_end,
                                   const float* taps_poly, const DdcChain* chains, int nchains,
                                   int D, int64_t k_begin, int nk, int nseg, float2* partial,
                                   hipStream_t st) {
    int cpw = 1;
    while (cpw < nchains && cpw < 64) cpw <<= 1;
    const int tpw = 64 / cpw;
    const int ntiles = (nk + R - 1) / R;
    const int ntg = (ntiles + tpw - 1) / tpw;
    const int ncg = (nchains + cpw - 1) / cpw;
    const int seg_len = ddc_seg_len(D, nseg);
    const int segs = (D + seg_len - 1) / seg_len;
    dim3 grid(ntg, segs, ncg);
    hipLaunchKernelGGL((ddc_lds<P, R, WPE>), grid, dim3(64 * kDdcWaves), ddc_lds_bytes(P, tpw, R), st,
                       blk, blk_start, blk_end, taps_poly, chains, nchains, D, k_begin, nk, cpw,
                       tpw, seg_len, partial);
    return hipGetLastError();
}

template <int P, int R = 32, int WPE = 2, int SB = 16>
hipError_t launch_ddc_p(const float2* blk, int64_t blk_start, int64_t blk_end,
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

// Resident workgroups per CU of one instantiation (registers / LDS bound).
template <int P>
int ddc_occ(bool flat, int tpw) {
    int nb = 0;
    hipError_t e = flat
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &nb, reinterpret_cast<const void*>(&ddc_polyphase<P, 32, 2, 16>), 64 * kDdcWaves, 0)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &nb, reinterpret_cast<const void*>(&ddc_lds<P, kLdsR, kLdsWpe>), 64 * kDdcWaves,
              ddc_lds_bytes(P, tpw));
    if (e != hipSuccess) return 2;
    return nb > 0 ? nb : 1;
}

// Explicit instantiation, one translation unit per group of depths (kernels_ddc_p*.hip) so
// the fully unrolled kernels compile in parallel; kernels_ddc.hip only dispatches.
#define OWRX_DDC_SIG                                                                         \
    (const float2*, int64_t, int64_t, const float*, const DdcChain*, int, int, int64_t, int, \
     int, float2*, hipStream_t)
#define OWRX_DDC_INSTANTIATE(EXT, P)                                                         \
    EXT template hipError_t launch_ddc_p<P, 32, 2, 16> OWRX_DDC_SIG;                         \
    EXT template hipError_t launch_ddc_lds_p<P, kLdsWpe, kLdsR> OWRX_DDC_SIG;                      \
    EXT template int ddc_occ<P>(bool, int);
#define OWRX_DDC_DEPTHS(X, EXT) X(EXT, 8) X(EXT, 16) X(EXT, 27) X(EXT, 28) X(EXT, 32) X(EXT, 48) X(EXT, 64)

}  // namespace owrx
