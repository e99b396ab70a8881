// IMA-ADPCM encoder formulations (diagnostic; not part of the product): cycles per sample and
// lane of the table encoder in owrx_dev.h (adpcm_encode_tab) against a leaner formulation with
// biased (unsigned) samples and predictor, borrow-chain magnitude bits and 32-B successor
// records; checks that both produce the codes of the reference encoder (adpcm_encode).
// Build: hipcc -O3 --offload-arch=gfx950 adpcm_lean.cpp -o adpcm_lean
#include "../../openwebrx_amd/csrc/owrx_dev.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

struct LeanRec {  // successor record of (index, magnitude): the next state's step terms
    uint32_t step, h, q, s3;
    uint32_t row, code, code8, pad;  // row = next index; code = magnitude of this transition
};
constexpr int kLeanEntries = 89 * 8;

__device__ void lean_fill(LeanRec* T, int tid, int nt) {
    for (int e = tid; e < kLeanEntries; e += nt) {
        const int i = e >> 3, inv = e & 7, mag = 7 - inv;
        int ni = i + kAdpcmIndex[mag];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        const uint32_t st = (uint32_t)kAdpcmStep[ni];
        T[e] = LeanRec{st, st >> 1, st >> 2, st >> 3, (uint32_t)ni, (uint32_t)mag, (uint32_t)(mag | 8), 0};
    }
}

struct LeanState {
    uint32_t step, h, q, s3, row;
    int pb;  // predictor + 32768
};

__device__ LeanState lean_state(int index, int pred) {
    const uint32_t st = (uint32_t)kAdpcmStep[index];
    return LeanState{st, st >> 1, st >> 2, st >> 3, (uint32_t)index, pred + 32768};
}

// xb = sample + 32768 (0 .. 65535); returns the 4-bit code
__device__ __forceinline__ int lean_encode(LeanState& s, uint32_t xb, const LeanRec* __restrict__ T) {
    const uint32_t pb = (uint32_t)s.pb;
    const bool neg = xb < pb;
    const uint32_t a = __builtin_amdgcn_sad_u16(xb, pb, 0u);  // |xb - pb| (both < 2^16)
    uint32_t a1, a2, t;
    const bool b4 = __builtin_sub_overflow(a, s.step, &a1);
    if (b4) a1 = a;
    const bool b2 = __builtin_sub_overflow(a1, s.h, &a2);
    if (b2) a2 = a1;
    const bool b1 = __builtin_sub_overflow(a2, s.q, &t);
    const uint32_t t1 = b1 ? 0u : s.q;
    const uint32_t dq = s.s3 + a + t1 - a2;
    int p = neg ? (int)pb - (int)dq : (int)pb + (int)dq;
    s.pb = min(max(p, 0), 65535);
    const uint32_t idx = ((s.row * 2 + b4) * 2 + b2) * 2 + b1;
    const LeanRec& r = T[idx];
    s.step = r.step;
    s.h = r.h;
    s.q = r.q;
    s.s3 = r.s3;
    s.row = r.row;
    return (int)(neg ? r.code8 : r.code);
}

template <int V>
__global__ void __launch_bounds__(64) kern(const int16_t* __restrict__ x, int n, uint8_t* __restrict__ out,
                                           long long* cyc) {
    __shared__ __align__(16) uint32_t NS[kAdpcmTabEntries];
    __shared__ __align__(16) LeanRec T[kLeanEntries];
    adpcm_tab_fill(NS, threadIdx.x, 64);
    lean_fill(T, threadIdx.x, 64);
    __syncthreads();
    const int lane = threadIdx.x;
    const int16_t* src = x + (size_t)lane * (n + 16);
    uint8_t* o = out + (size_t)lane * n;
    AdpcmTab ad = adpcm_tab_state(AdpcmState{0, 0});
    LeanState ls = lean_state(0, 0);
    long long t0 = clock64();
    for (int j = 0; j < n; j += 8) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + j);
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
        uint32_t w = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            int code;
            if (V == 0) {
                const int xs = (int)(int16_t)(wv[t >> 1] >> (16 * (t & 1)));
                code = adpcm_encode_tab(ad, xs, NS);
            } else {
                const uint32_t xb = ((wv[t >> 1] >> (16 * (t & 1))) & 0xffffu) ^ 0x8000u;
                code = lean_encode(ls, xb, T);
            }
            w |= (uint32_t)code << (4 * t);
        }
        *reinterpret_cast<uint32_t*>(o + (j >> 1)) = w;
    }
    long long t1 = clock64();
    if (lane == 0) *cyc = t1 - t0;
}

static int ref_encode(AdpcmState& s, int sample) {
    static const int ix[16] = {-1, -1, -1, -1, 2, 4, 6, 8, -1, -1, -1, -1, 2, 4, 6, 8};
    static const int st[89] = {
        7,     8,     9,     10,    11,    12,    13,    14,    16,    17,    19,    21,    23,
        25,    28,    31,    34,    37,    41,    45,    50,    55,    60,    66,    73,    80,
        88,    97,    107,   118,   130,   143,   157,   173,   190,   209,   230,   253,   279,
        307,   337,   371,   408,   449,   494,   544,   598,   658,   724,   796,   876,   963,
        1060,  1166,  1282,  1411,  1552,  1707,  1878,  2066,  2272,  2499,  2749,  3024,  3327,
        3660,  4026,  4428,  4871,  5358,  5894,  6484,  7132,  7845,  8630,  9493,  10442, 11487,
        12635, 13899, 15289, 16818, 18500, 20350, 22385, 24623, 27086, 29794, 32767};
    int step = st[s.index], diff = sample - s.pred, code = 0;
    if (diff < 0) {
        code = 8;
        diff = -diff;
    }
    int ts = step;
    if (diff >= ts) { code |= 4; diff -= ts; }
    ts >>= 1;
    if (diff >= ts) { code |= 2; diff -= ts; }
    ts >>= 1;
    if (diff >= ts) code |= 1;
    int dq = step >> 3;
    if (code & 4) dq += step;
    if (code & 2) dq += step >> 1;
    if (code & 1) dq += step >> 2;
    int p = s.pred + ((code & 8) ? -dq : dq);
    s.pred = p > 32767 ? 32767 : (p < -32768 ? -32768 : p);
    int i = s.index + ix[code];
    s.index = i < 0 ? 0 : (i > 88 ? 88 : i);
    return code;
}

int main() {
    const int S = 64, n = 8000;
    std::vector<int16_t> h((size_t)S * (n + 16));
    srand(3);
    for (int c = 0; c < S; ++c) {
        double y = 0, amp = 500 + 32000.0 * (c % 9) / 8.0;
        for (int i = 0; i < n + 16; ++i) {
            y = 0.9 * y + (rand() / (double)RAND_MAX - 0.5);
            double v = amp * (0.6 * sin(0.05 * i * (1 + c % 11) + c) + 0.5 * y);
            if (c % 13 == 5) v = (rand() % 65536) - 32768;  // full-range noise
            v = v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
            h[(size_t)c * (n + 16) + i] = (int16_t)v;
        }
    }
    std::vector<uint8_t> ref((size_t)S * n / 2);
    for (int c = 0; c < S; ++c) {
        AdpcmState s{0, 0};
        for (int i = 0; i < n; i += 2) {
            const int c0 = ref_encode(s, h[(size_t)c * (n + 16) + i]);
            const int c1 = ref_encode(s, h[(size_t)c * (n + 16) + i + 1]);
            ref[(size_t)c * n / 2 + i / 2] = (uint8_t)(c0 | (c1 << 4));
        }
    }
    int16_t* dx;
    uint8_t* dout;
    long long* dc;
    hipMalloc(&dx, h.size() * 2);
    hipMemcpy(dx, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&dout, (size_t)S * n);
    hipMalloc(&dc, 8);
    auto run = [&](const char* name, void (*k)(const int16_t*, int, uint8_t*, long long*)) {
        long long cyc = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, n, dout, dc);
            hipDeviceSynchronize();
        }
        hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
        std::vector<uint8_t> got((size_t)S * n);
        hipMemcpy(got.data(), dout, got.size(), hipMemcpyDeviceToHost);
        long bad = 0;
        for (int c = 0; c < S; ++c)
            for (int b = 0; b < n / 2; ++b) bad += got[(size_t)c * n + b] != ref[(size_t)c * n / 2 + b];
        printf("%-28s %7.1f cycles/sample, %ld mismatching bytes (%s)\n", name, cyc / (double)n, bad,
               hipGetErrorString(hipGetLastError()));
    };
    run("adpcm_encode_tab", kern<0>);
    run("lean (biased, borrows)", kern<1>);
    return 0;
}
