// fft_lds.h -- batched in-LDS complex FFT used by the four-step waterfall FFT
// (kernels_waterfall.hip) and the per-chain secondary FFT (kernels_sfft.hip).
#pragma once
#include "owrx_dev.h"

namespace owrx {

// R rows of length 2^LOGL in LDS (row stride RS float2), in-place Stockham radix-4 (+ one
// radix-2 pass for odd LOGL); W_L^m = tw[m * twstep] (tw: the N-point table).
template <int LOGL, int R, int NT>
OWRX_DEV void lds_fft_rows(float2* sm, int RS, const float2* __restrict__ tw, int twstep) {
    constexpr int L = 1 << LOGL;
    constexpr int NB = R * (L / 4) / NT;
    static_assert(NB >= 1 && NB * NT == R * (L / 4), "rows x butterflies must tile the threads");
    const int tid = threadIdx.x;
    int lns = 0;
#pragma unroll
    for (int pass = 0; pass < LOGL / 2; ++pass) {
        float2 a[NB][4];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int idx = tid + b * NT;
            const int base = (idx / (L / 4)) * RS;
            const int j = idx % (L / 4);
#pragma unroll
            for (int r = 0; r < 4; ++r) a[b][r] = sm[base + j + r * (L / 4)];
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int idx = tid + b * NT;
            const int base = (idx / (L / 4)) * RS;
            const int j = idx % (L / 4);
            const int k = j & ((1 << lns) - 1);
            const int ts = (k << (LOGL - 2 - lns)) * twstep;
            const float2 a0 = a[b][0];
            const float2 a1 = cmul(a[b][1], tw[ts]);
            const float2 a2 = cmul(a[b][2], tw[2 * ts]);
            const float2 a3 = cmul(a[b][3], tw[3 * ts]);
            const float2 t0 = make_float2(a0.x + a2.x, a0.y + a2.y);
            const float2 t1 = make_float2(a0.x - a2.x, a0.y - a2.y);
            const float2 t2 = make_float2(a1.x + a3.x, a1.y + a3.y);
            const float2 t3 = make_float2(a1.y - a3.y, a3.x - a1.x);  // -i (a1 - a3)
            const int d = base + ((j >> lns) << (lns + 2)) + k;
            const int ns = 1 << lns;
            sm[d] = make_float2(t0.x + t2.x, t0.y + t2.y);
            sm[d + ns] = make_float2(t1.x + t3.x, t1.y + t3.y);
            sm[d + 2 * ns] = make_float2(t0.x - t2.x, t0.y - t2.y);
            sm[d + 3 * ns] = make_float2(t1.x - t3.x, t1.y - t3.y);
        }
        __syncthreads();
        lns += 2;
    }
    if constexpr (LOGL & 1) {
        constexpr int NB2 = R * (L / 2) / NT;
        float2 a[NB2][2];
#pragma unroll
        for (int b = 0; b < NB2; ++b) {
            const int idx = tid + b * NT;
            const int base = (idx / (L / 2)) * RS;
            const int j = idx % (L / 2);
            a[b][0] = sm[base + j];
            a[b][1] = sm[base + j + L / 2];
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < NB2; ++b) {
            const int idx = tid + b * NT;
            const int base = (idx / (L / 2)) * RS;
            const int j = idx % (L / 2);
            const int k = j & ((1 << lns) - 1);
            const float2 a1 = cmul(a[b][1], tw[(k << (LOGL - 1 - lns)) * twstep]);
            const int d = base + ((j >> lns) << (lns + 1)) + k;
            sm[d] = make_float2(a[b][0].x + a1.x, a[b][0].y + a1.y);
            sm[d + (1 << lns)] = make_float2(a[b][0].x - a1.x, a[b][0].y - a1.y);
        }
        __syncthreads();
    }
}

}  // namespace owrx
