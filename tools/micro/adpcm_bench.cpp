// IMA-ADPCM serial encoder microbenchmark (diagnostic; not part of the product): cycles per
// sample of encoder formulations, one lane per stream, 32 streams x 5000 samples.
#include "../../openwebrx_amd/csrc/owrx_dev.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

template <int V>
__global__ void __launch_bounds__(64) kern(const int16_t* __restrict__ x, int n, int nstreams,
                                           uint8_t* __restrict__ out, long long* cyc) {
    __shared__ __align__(16) uint32_t NS[kAdpcmTabEntries];
    adpcm_tab_fill(NS, threadIdx.x, 64);
    __syncthreads();
    const int lane = threadIdx.x;
    const int c = lane < nstreams ? lane : 0;
    const int16_t* src = x + (size_t)c * (n + 16);
    uint8_t* o = out + (size_t)c * n;
    AdpcmTab ad = adpcm_tab_state(AdpcmState{0, 0});
    AdpcmTab ad2 = ad;
    const int16_t* src2 = x + (size_t)(c + 32) * (n + 16);
    long long t0 = clock64();
    int cur[8], nxt[8];
    for (int q = 0; q < 8; ++q) cur[q] = src[q];
    int acc = 0;
    for (int j = 0; j < n; j += 8) {
        for (int q = 0; q < 8; ++q) nxt[q] = src[j + 8 + q];
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            int c0, c1;
            if (V == 3) {
                c0 = adpcm_encode_tab(ad, cur[u], NS);
                c1 = adpcm_encode_tab(ad, cur[u + 1], NS);
            } else if (V == 4) {
                const int e0 = adpcm_encode_tab(ad, cur[u], NS);
                const int f0 = adpcm_encode_tab(ad2, src2[j + u], NS);
                const int e1 = adpcm_encode_tab(ad, cur[u + 1], NS);
                const int f1 = adpcm_encode_tab(ad2, src2[j + u + 1], NS);
                c0 = e0 ^ f0;
                c1 = e1 ^ f1;
            } else if (V == 0 || V == 2) {
                c0 = adpcm_encode_tab(ad, cur[u], NS);
                c1 = adpcm_encode_tab(ad, cur[u + 1], NS);
            } else {  // two streams per lane, interleaved
                const int e0 = adpcm_encode_tab(ad, cur[u], NS);
                const int f0 = adpcm_encode_tab(ad2, src2[j + u], NS);
                const int e1 = adpcm_encode_tab(ad, cur[u + 1], NS);
                const int f1 = adpcm_encode_tab(ad2, src2[j + u + 1], NS);
                c0 = e0 ^ f0;
                c1 = e1 ^ f1;
            }
            if (V != 2) o[(j + u) >> 1] = (uint8_t)(c0 | (c1 << 4));
            else acc += c0 + c1;
        }
        for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
    }
    long long t1 = clock64();
    if (V == 2) o[0] = (uint8_t)acc;
    if (lane == 0) *cyc = t1 - t0;
}

int main(int argc, char** argv) {
    const int S = 64, n = 5000;
    std::vector<int16_t> h((size_t)S * (n + 16));
    srand(3);
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    for (int c = 0; c < S; ++c) {
        double y = 0, amp = 2000 + 15000.0 * (c % 7) / 6.0;
        for (int i = 0; i < n + 16; ++i) {
            if (mode == 0) {
                h[(size_t)c * (n + 16) + i] = (int16_t)(20000 * sin(0.07 * i * (1 + c % 5)) +
                                                        (rand() % 2000) - 1000);
            } else {  // independent noisy audio-like streams of different loudness
                y = 0.9 * y + (rand() / (double)RAND_MAX - 0.5);
                double v = amp * (0.6 * sin(0.05 * i * (1 + c % 11) + c) + 0.25 * y);
                v = v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
                h[(size_t)c * (n + 16) + i] = (int16_t)v;
            }
        }
    }
    int16_t* dx;
    uint8_t* dout;
    long long* dc;
    hipMalloc(&dx, h.size() * 2);
    hipMemcpy(dx, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&dout, (size_t)S * n);
    hipMalloc(&dc, 8);
    auto run = [&](const char* name, void (*k)(const int16_t*, int, int, uint8_t*, long long*),
                   double per) {
        long long cyc = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, n, 32, dout, dc);
            hipDeviceSynchronize();
        }
        hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
        printf("%-34s %7.1f cycles/sample (%s)\n", name, cyc / (n * per),
               hipGetErrorString(hipGetLastError()));
    };
    run("table encoder + byte stores", kern<0>, 1.0);
    run("x2 streams/lane (per stream)", kern<1>, 2.0);
    run("table encoder, no stores", kern<2>, 1.0);
    run("single dependent read + stores", kern<3>, 1.0);
    run("single read x2 streams/lane (per stream)", kern<4>, 2.0);
    return 0;
}
