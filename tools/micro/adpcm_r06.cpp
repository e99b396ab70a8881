// IMA-ADPCM serial encoder microbenchmark, round 6 (diagnostic; not part of the product):
// cycles per sample of one 64-lane wave (one lane per stream, 64 streams x 5000 samples) for the
// production encoder adpcm_encode_rem (owrx_dev.h) and adpcm_encode_rem_o: the same remainder form
// with the predictor kept offset by 32768 (|d| as one v_sad_u32 of the offset sample and
// predictor) and its update split so that only (a3 ^ sgn), a subtraction and the clamp (v_med3)
// follow the last magnitude bit: pred' = (pred + sgn (s3 + a0) + sgn) - (a3 ^ sgn), the first part
// computed beside the compares.  Every code byte is compared with adpcm_encode_rem's.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 adpcm_r06.cpp -o adpcm_r06
#include "../../openwebrx_amd/csrc/owrx_dev.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

template <int V>
__global__ void __launch_bounds__(64) kern(const int16_t* __restrict__ x, int n, uint8_t* __restrict__ out,
                                           long long* cyc) {
    __shared__ __align__(16) uint2 NSR[kAdpcmRemEntries];
    adpcm_rem_fill(NSR, threadIdx.x, 64);
    __shared__ __align__(16) uint4 NSR4[V == 2 ? kAdpcmRemEntries : 1];
    if constexpr (V == 2) adpcm_rem4_fill(NSR4, threadIdx.x, 64);
    __syncthreads();
    const int lane = threadIdx.x;
    const int16_t* src = x + (size_t)lane * (n + 16);
    uint8_t* o = out + (size_t)lane * n;
    AdpcmRem rem = adpcm_rem_state(AdpcmState{0, 0});
    AdpcmRemO remo = adpcm_rem_o_state(AdpcmState{0, 0});
    AdpcmRem4 rem4 = adpcm_rem4_state(AdpcmState{0, 0});
    int cur[8], nxt[8];
    for (int q = 0; q < 8; ++q) cur[q] = src[q];
    const long long t0 = clock64();
    const long long r0 = wall_clock64();
    for (int j = 0; j < n; j += 8) {
        for (int q = 0; q < 8; ++q) nxt[q] = src[j + 8 + q];
        uint32_t w = 0;
        if constexpr (V == 0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) w |= (adpcm_encode_rem(rem, cur[u], NSR) & 15u) << (4 * u);
        } else if constexpr (V == 2) {
#pragma unroll
            for (int u = 0; u < 8; ++u) w |= (adpcm_encode_rem4(rem4, cur[u], NSR4) & 15u) << (4 * u);
        } else {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                w |= (adpcm_encode_rem_o(remo, (uint32_t)(cur[u] + 32768), NSR) & 15u) << (4 * u);
        }
        w ^= 0x77777777u;
        *reinterpret_cast<uint32_t*>(o + (j >> 1)) = w;
        for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
    }
    const long long t1 = clock64();
    const long long r1 = wall_clock64();
    if (lane == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = r1 - r0;
    }
}

int main() {
    const int S = 64, n = 5000;
    std::vector<int16_t> h((size_t)S * (n + 16));
    srand(3);
    for (int c = 0; c < S; ++c) {
        double y = 0, amp = 2000 + 15000.0 * (c % 7) / 6.0;
        for (int i = 0; i < n + 16; ++i) {
            y = 0.9 * y + (rand() / (double)RAND_MAX - 0.5);
            double v = amp * (0.6 * sin(0.05 * i * (1 + c % 11) + c) + 0.25 * y);
            if (c % 3 == 0) v = (rand() % 65536) - 32768;  // full-scale noise: large steps
            v = v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
            h[(size_t)c * (n + 16) + i] = (int16_t)v;
        }
    }
    int16_t* dx;
    uint8_t *d0, *d1;
    long long* dc;
    hipMalloc(&dx, h.size() * 2);
    hipMemcpy(dx, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&d0, (size_t)S * n);
    hipMalloc(&d1, (size_t)S * n);
    hipMalloc(&dc, 16);
    auto run = [&](const char* name, void (*k)(const int16_t*, int, uint8_t*, long long*), uint8_t* o) {
        long long cyc[2] = {0, 0};
        for (int rep = 0; rep < 5; ++rep) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, n, o, dc);
            hipDeviceSynchronize();
        }
        hipMemcpy(cyc, dc, 16, hipMemcpyDeviceToHost);
        int wrate = 0;
        hipDeviceGetAttribute(&wrate, hipDeviceAttributeWallClockRate, 0);  // kHz
        const double ns = cyc[1] * 1e6 / (double)wrate / n;
        printf("%-52s %7.1f cycles/sample, %6.1f ns/sample (%.2f GHz) (%s)\n", name, cyc[0] / (double)n, ns,
               cyc[0] / (double)n / ns, hipGetErrorString(hipGetLastError()));
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("adpcm_encode_rem (round-5 production)", kern<0>, d0);
        run("adpcm_encode_rem_o (offset predictor, short update)", kern<1>, d1);
    }
    uint8_t* d2;
    hipMalloc(&d2, (size_t)S * n);
    run("adpcm_encode_rem4 (16-B records, s3 in the record)", kern<2>, d2);
    run("adpcm_encode_rem (round-5 production)", kern<0>, d0);
    run("adpcm_encode_rem4 (16-B records, s3 in the record)", kern<2>, d2);
    std::vector<uint8_t> a((size_t)S * n), b(a.size());
    hipMemcpy(a.data(), d0, a.size(), hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), d1, b.size(), hipMemcpyDeviceToHost);
    size_t diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("adpcm_encode_rem_o codes differing: %zu of %d bytes\n", diff, S * n / 2);
    hipMemcpy(b.data(), d2, b.size(), hipMemcpyDeviceToHost);
    diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("adpcm_encode_rem4 codes differing: %zu of %d bytes\n", diff, S * n / 2);
    return 0;
}
