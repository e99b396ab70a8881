// IMA-ADPCM serial encoder, scalar formulation (diagnostic microbenchmark, not the product):
// one WAVE per stream, every state value wave-uniform so the recurrence runs on the scalar
// ALU, the step table spread over the lanes of one VGPR and read with v_readlane (SGPR index).
// Compares cycles per sample with the one-lane-per-stream LDS-table encoder and checks the
// codes are identical.
#include "../../openwebrx_amd/csrc/owrx_dev.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

// One encoder step on the scalar ALU.  State: pred, idx (clamped index), st (step).
// Critical path: compare/select pairs for the three magnitude bits, index update + clamp,
// v_readlane of the packed step table (lane L = step[2L] | step[2L+1] << 16).
__device__ __forceinline__ int enc_scalar(int sample, int& pred, int& idx, int& st,
                                          uint32_t tab) {
    int code;
    int a, t0, t1, t2, dq, m, inc, li, sh, w;
    asm volatile(
        "s_sub_i32 %[t0], %[x], %[p]\n\t"          // d
        "s_abs_i32 %[a], %[t0]\n\t"                // a = |d|
        "s_ashr_i32 %[t0], %[t0], 31\n\t"          // sgn
        "s_lshr_b32 %[dq], %[st], 3\n\t"
        "s_sub_i32 %[t1], %[a], %[st]\n\t"         // a - step
        "s_cmp_ge_i32 %[a], %[st]\n\t"             // b4
        "s_cselect_b32 %[a], %[t1], %[a]\n\t"
        "s_cselect_b32 %[t2], %[st], 0\n\t"
        "s_cselect_b32 %[m], 4, 0\n\t"
        "s_cselect_b32 %[inc], 2, -1\n\t"          // b4 ? 2 : -1 (+4 b2 + 2 b1 below)
        "s_add_i32 %[dq], %[dq], %[t2]\n\t"
        "s_lshr_b32 %[t2], %[st], 1\n\t"           // h
        "s_sub_i32 %[t1], %[a], %[t2]\n\t"
        "s_cmp_ge_i32 %[a], %[t2]\n\t"             // b2
        "s_cselect_b32 %[a], %[t1], %[a]\n\t"
        "s_cselect_b32 %[t2], %[t2], 0\n\t"
        "s_cselect_b32 %[w], 2, 0\n\t"
        "s_or_b32 %[m], %[m], %[w]\n\t"
        "s_add_i32 %[dq], %[dq], %[t2]\n\t"
        "s_lshr_b32 %[t2], %[st], 2\n\t"           // q
        "s_cmp_ge_i32 %[a], %[t2]\n\t"             // b1
        "s_cselect_b32 %[t2], %[t2], 0\n\t"
        "s_cselect_b32 %[w], 1, 0\n\t"
        "s_or_b32 %[m], %[m], %[w]\n\t"
        "s_add_i32 %[dq], %[dq], %[t2]\n\t"
        // inc = b4 ? 2 + 2 * (m & 3) : -1
        "s_and_b32 %[w], %[m], 3\n\t"
        "s_lshl_b32 %[w], %[w], 1\n\t"
        "s_cmp_ge_u32 %[m], 4\n\t"
        "s_cselect_b32 %[w], %[w], 0\n\t"
        "s_add_i32 %[inc], %[inc], %[w]\n\t"
        "s_add_i32 %[inc], %[inc], %[i]\n\t"
        "s_max_i32 %[inc], %[inc], 0\n\t"
        "s_min_i32 %[i], %[inc], 88\n\t"
        "s_lshr_b32 %[li], %[i], 1\n\t"
        "s_and_b32 %[sh], %[i], 1\n\t"
        "s_lshl_b32 %[sh], %[sh], 4\n\t"
        "v_readlane_b32 %[w], %[tab], %[li]\n\t"
        // pred update overlaps the table read
        "s_xor_b32 %[dq], %[dq], %[t0]\n\t"
        "s_sub_i32 %[dq], %[dq], %[t0]\n\t"
        "s_add_i32 %[p], %[p], %[dq]\n\t"
        "s_max_i32 %[p], %[p], 0xffff8000\n\t"
        "s_min_i32 %[p], %[p], 0x7fff\n\t"
        "s_and_b32 %[t0], %[t0], 8\n\t"
        "s_or_b32 %[code], %[m], %[t0]\n\t"
        "s_nop 1\n\t"
        "s_lshr_b32 %[w], %[w], %[sh]\n\t"
        "s_and_b32 %[st], %[w], 0xffff\n\t"
        : [a] "=&s"(a), [t0] "=&s"(t0), [t1] "=&s"(t1), [t2] "=&s"(t2), [dq] "=&s"(dq),
          [m] "=&s"(m), [inc] "=&s"(inc), [li] "=&s"(li), [sh] "=&s"(sh), [w] "=&s"(w),
          [code] "=&s"(code), [p] "+s"(pred), [i] "+s"(idx), [st] "+s"(st)
        : [x] "s"(sample), [tab] "v"(tab)
        : "scc");
    return code;
}

__global__ void __launch_bounds__(1024) kscalar(const int16_t* __restrict__ x, int n,
                                                uint8_t* __restrict__ out, long long* cyc) {
    const int c = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    uint32_t tab = 0;
    if (lane < 45)
        tab = (uint32_t)kAdpcmStep[2 * lane] |
              ((2 * lane + 1 < 89 ? (uint32_t)kAdpcmStep[2 * lane + 1] : 0u) << 16);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(x + (size_t)c * (n + 16));
    uint32_t* o = reinterpret_cast<uint32_t*>(out + (size_t)c * n);
    int idx = 0, pred = 0, step = 7;
    long long t0 = clock64();
    uint32_t cur[8], nxt[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) cur[q] = src[q];
    for (int j = 0; j < n; j += 16) {
#pragma unroll
        for (int q = 0; q < 8; ++q) nxt[q] = src[(j >> 1) + 8 + q];
        uint32_t w0 = 0, w1 = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int s0 = (int)(int16_t)(cur[q] & 0xffffu);
            const int s1 = (int)(int16_t)(cur[q] >> 16);
            const int c0 = enc_scalar(s0, pred, idx, step, tab);
            const int c1 = enc_scalar(s1, pred, idx, step, tab);
            const uint32_t b = (uint32_t)(c0 | (c1 << 4));
            if (q < 4) w0 |= b << (8 * q);
            else w1 |= b << (8 * (q - 4));
        }
        if (lane == 0) {
            o[(j >> 3)] = w0;
            o[(j >> 3) + 1] = w1;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
    }
    long long t1 = clock64();
    if (lane == 0 && c == 0) *cyc = t1 - t0;
}

__global__ void __launch_bounds__(64) klds(const int16_t* __restrict__ x, int n, int nstreams,
                                           uint8_t* __restrict__ out, long long* cyc) {
    __shared__ __align__(16) uint32_t NS[kAdpcmTabEntries];
    adpcm_tab_fill(NS, threadIdx.x, 64);
    __syncthreads();
    const int lane = threadIdx.x;
    const int c = lane < nstreams ? lane : 0;
    const int16_t* src = x + (size_t)c * (n + 16);
    uint8_t* o = out + (size_t)c * n;
    AdpcmTab ad = adpcm_tab_state(AdpcmState{0, 0});
    long long t0 = clock64();
    int cur[8], nxt[8];
    for (int q = 0; q < 8; ++q) cur[q] = src[q];
    for (int j = 0; j < n; j += 8) {
        for (int q = 0; q < 8; ++q) nxt[q] = src[j + 8 + q];
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            const int c0 = adpcm_encode_tab(ad, cur[u], NS);
            const int c1 = adpcm_encode_tab(ad, cur[u + 1], NS);
            if (lane < nstreams) o[(j + u) >> 1] = (uint8_t)(c0 | (c1 << 4));
        }
        for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
    }
    long long t1 = clock64();
    if (lane == 0) *cyc = t1 - t0;
}

int main(int argc, char** argv) {
    const int S = 32, n = 4992;
    std::vector<int16_t> h((size_t)S * (n + 16));
    srand(3);
    for (int c = 0; c < S; ++c) {
        double y = 0, amp = 2000 + 15000.0 * (c % 7) / 6.0;
        for (int i = 0; i < n + 16; ++i) {
            y = 0.9 * y + (rand() / (double)RAND_MAX - 0.5);
            double v = amp * (0.6 * sin(0.05 * i * (1 + c % 11) + c) + 0.25 * y);
            v = v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
            h[(size_t)c * (n + 16) + i] = (int16_t)v;
        }
    }
    int16_t* dx;
    uint8_t *d1, *d2;
    long long* dc;
    hipMalloc(&dx, h.size() * 2);
    hipMemcpy(dx, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&d1, (size_t)S * n);
    hipMalloc(&d2, (size_t)S * n);
    hipMalloc(&dc, 8);
    long long cyc = 0;
    std::vector<uint8_t> o1((size_t)S * n / 2), o2((size_t)S * n / 2);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(klds, dim3(1), dim3(64), 0, 0, dx, n, S, d1, dc);
        hipDeviceSynchronize();
    }
    hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
    printf("LDS table, lane per stream     %7.1f cycles/sample\n", cyc / (double)n);
    for (int wpb : {1, 2, 4, 8}) {  // streams (waves) per workgroup: SALU is shared per CU
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a, 0);
            hipLaunchKernelGGL(kscalar, dim3(S / wpb), dim3(64 * wpb), 0, 0, dx, n, d2, dc);
            hipEventRecord(b, 0);
            hipDeviceSynchronize();
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 2) {
                hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
                printf("scalar, wave per stream, %d/WG  %7.1f cycles/sample, %.3f ms wall (%s)\n", wpb,
                       cyc / (double)n, ms, hipGetErrorString(hipGetLastError()));
            }
        }
    }
    // codes: LDS version writes bytes per stream at o[c*n + i/2]; scalar likewise
    std::vector<uint8_t> a1((size_t)S * n), a2((size_t)S * n);
    hipMemcpy(a1.data(), d1, a1.size(), hipMemcpyDeviceToHost);
    hipMemcpy(a2.data(), d2, a2.size(), hipMemcpyDeviceToHost);
    long bad = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) bad += a1[(size_t)c * n + i] != a2[(size_t)c * n + i];
    printf("mismatching bytes: %ld of %d\n", bad, S * n / 2);
    return bad != 0;
}
