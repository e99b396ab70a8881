// Waterfall FFT kernels in isolation (diagnostic, not part of the product), round 5: C3's
// geometry (10 Msps, N = 16384, hop 11454), FT frames per launch in groups of F, frames read from
// HBM (512 MiB streamed between launches, as the DDC's operand streams evict them in the engine).
// Variants: l32 (round-4 production), q16 (1024 threads x 16 points), r16 (reference for the
// partial rows), and the load patterns alone.  Prints us per launch, the rate on the algorithmic
// bytes (the frames' span of cf32 IQ, 8 B per sample read once) and each kernel's difference
// from wf_fft_r16<14> (positions mapped back to bins).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-slp-vectorize wf_r05.hip -o wf_r05
// Run:   ./wf_r05 [FT ...]
#include "../../openwebrx_amd/csrc/kernels_waterfall.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

using namespace owrx;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                                   \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

constexpr int N = 16384;

// the frame loads alone, NT threads of N/NT points, 8 B per lane per load, the next frame in
// flight while the current one is summed
template <int NT>
__global__ void __launch_bounds__(NT)
wf_mem8(const float2* __restrict__ blk, const WfGroup* __restrict__ groups, float* __restrict__ partial) {
    constexpr int P = N / NT;
    const WfGroup g = groups[blockIdx.x];
    const int t = threadIdx.x;
    const int nfr = g.nframes;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(blk + g.start), 0,
                                                      (int)(8 * ((int64_t)(nfr - 1) * g.hop + N)), 0x00020000);
    float acc[P] = {};
    float2 nx[P];
    auto ld = [&](int f, float2* v) {
        const int fo = f < nfr ? f * g.hop * 8 : (1 << 30);
#pragma unroll
        for (int m = 0; m < P; ++m)
            v[m] = make_float2(
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, t * 8 + fo, m * NT * 8, 0)),
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, t * 8 + fo + 4, m * NT * 8, 0)));
    };
    ld(0, nx);
    for (int f = 0; f < nfr; ++f) {
        float2 x[P];
#pragma unroll
        for (int m = 0; m < P; ++m) x[m] = nx[m];
        ld(f + 1, nx);
#pragma unroll
        for (int m = 0; m < P; ++m) acc[m] = fmaf(x[m].x, x[m].x, fmaf(x[m].y, x[m].y, acc[m]));
    }
#pragma unroll
    for (int m = 0; m < P; ++m) partial[(int64_t)blockIdx.x * N + t + NT * m] = acc[m];
}

// 16-B loads (two adjacent samples per lane), NT threads, DEPTH frames in flight, AUX cache policy
template <int NT, int DEPTH, int AUX>
__global__ void __launch_bounds__(NT)
wf_mem16(const float2* __restrict__ blk, const WfGroup* __restrict__ groups, float* __restrict__ partial) {
    constexpr int P = N / NT / 2;  // 16-B loads per thread per frame
    const WfGroup g = groups[blockIdx.x];
    const int t = threadIdx.x;
    const int nfr = g.nframes;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(blk + g.start), 0,
                                                      (int)(8 * ((int64_t)(nfr - 1) * g.hop + N)), 0x00020000);
    float acc[P] = {};
    float4 nx[DEPTH][P];
    auto ld = [&](int f, float4* v) {
        const int fo = f < nfr ? f * g.hop * 8 : (1 << 30);
#pragma unroll
        for (int m = 0; m < P; ++m) {
            const int o = t * 16 + fo;
            v[m] = make_float4(
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o, m * NT * 16, AUX)),
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o + 4, m * NT * 16, AUX)),
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o + 8, m * NT * 16, AUX)),
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, o + 12, m * NT * 16, AUX)));
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) ld(d, nx[d]);
    for (int f = 0; f < nfr; f += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            float4 x[P];
#pragma unroll
            for (int m = 0; m < P; ++m) x[m] = nx[d][m];
            ld(f + d + DEPTH, nx[d]);
#pragma unroll
            for (int m = 0; m < P; ++m)
                acc[m] = fmaf(x[m].x, x[m].x, fmaf(x[m].y, x[m].y, fmaf(x[m].z, x[m].z, fmaf(x[m].w, x[m].w, acc[m]))));
        }
    }
#pragma unroll
    for (int m = 0; m < P; ++m) partial[(int64_t)blockIdx.x * N + t + NT * m] = acc[m];
}

// calibration: a grid-stride 16-B streaming read of n float4
__global__ void __launch_bounds__(256) stream_read(const float4* __restrict__ p, size_t n, float* sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        acc = fmaf(v.x, v.y, acc) + fmaf(v.z, v.w, acc);
    }
    if (acc == 12345.f) sink[0] = acc;
}
// calibration: each workgroup streams one contiguous chunk of `chunk` float4 (16-B loads, 8 in
// flight per lane)
__global__ void __launch_bounds__(256) chunk_read(const float4* __restrict__ p, size_t chunk, float* sink) {
    float acc = 0.f;
    const float4* q = p + blockIdx.x * chunk;
    for (size_t i = threadIdx.x; i < chunk; i += 256 * 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = i + u * 256 < chunk ? q[i + u * 256] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = fmaf(v[u].x, v[u].y, acc) + fmaf(v[u].z, v[u].w, acc);
    }
    if (acc == 12345.f) sink[0] = acc;
}

__global__ void flush_read(const float4* __restrict__ p, size_t n, float* sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;
}

static void* g_flush = nullptr;

static double time_us(const std::function<void()>& launch, hipStream_t stream) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t fb = (size_t)512 << 20;
    if (!g_flush) {
        CK(hipMalloc(&g_flush, fb));
        CK(hipMemset(g_flush, 0, fb));
    }
    const int iters = 30;
    std::vector<float> t;
    for (int i = 0; i < iters + 5; ++i) {
        hipLaunchKernelGGL(flush_read, dim3(4096), dim3(256), 0, stream, (const float4*)g_flush, fb / 16,
                           (float*)g_flush);
        CK(hipEventRecord(e0, stream));
        launch();
        CK(hipEventRecord(e1, stream));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (i >= 5) t.push_back(ms * 1e3f);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv) {
    const int hop = 11454;
    std::vector<int> fts;
    for (int i = 1; i < argc; ++i) fts.push_back(atoi(argv[i]));
    if (fts.empty()) fts = {1920, 3840};
    const int FTmax = *std::max_element(fts.begin(), fts.end());
    const int64_t S = (int64_t)FTmax * hop + N;
    std::vector<float2> x(S);
    srand(1);
    for (auto& v : x) v = float2{rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f};
    std::vector<float> win(N);
    for (int i = 0; i < N; ++i) win[i] = (float)(0.54 - 0.46 * cos(2 * M_PI * i / (N - 1)));
    std::vector<float2> tw(N);
    for (int k = 0; k < N; ++k) tw[k] = float2{(float)cos(2 * M_PI * k / N), (float)-sin(2 * M_PI * k / N)};
    float2 *dx, *dtw;
    float *dwin, *dref, *dpart;
    WfGroup* dg;
    CK(hipMalloc(&dx, sizeof(float2) * S));
    CK(hipMalloc(&dtw, sizeof(float2) * N));
    CK(hipMalloc(&dwin, sizeof(float) * N));
    CK(hipMalloc(&dref, sizeof(float) * (size_t)FTmax * N));
    CK(hipMalloc(&dpart, sizeof(float) * (size_t)2 * FTmax * N));
    CK(hipMalloc(&dg, sizeof(WfGroup) * 2 * FTmax));
    int* dwork;
    CK(hipMalloc(&dwork, 64));
    CK(hipMemset(dwork, 0, 64));
    CK(hipMemcpy(dx, x.data(), sizeof(float2) * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtw, tw.data(), sizeof(float2) * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwin, win.data(), sizeof(float) * N, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void*)wf_fft_r16<14>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfR16<14>::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_l32, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfL32::kLds));
#define SETQ(v) CK(hipFuncSetAttribute((const void*)wf_fft_q16<v>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WfQ16::kLds))
    SETQ(0); SETQ(1); SETQ(2); SETQ(3); SETQ(4); SETQ(6); SETQ(7); SETQ(8); SETQ(32); SETQ(1); SETQ(160); SETQ(40); SETQ(64); SETQ(96); SETQ(72); SETQ(104);
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    // the engine's stream A: CU-masked to 228 CUs (bits [0, 228))
    hipStream_t s_a = nullptr;
    {
        const int words = (ncu + 31) / 32;
        std::vector<uint32_t> lo(words, 0);
        for (int c = 0; c < ncu; ++c)
            if (c < 228) lo[c / 32] |= 1u << (c % 32);
        CK(hipExtStreamCreateWithCUMask(&s_a, words, lo.data()));
    }
    const int cus = 228;
    printf("N=%d hop=%d CUs %d, stream masked to %d, frames from HBM\n", N, hop, ncu, cus);
    for (int FT : fts) {
        const double alg = 8.0 * (double)FT * hop;  // frames x hop x 8 B (the engine's figure)
        for (int F : {4, 8, 16}) {
            const int G = (FT + F - 1) / F;
            std::vector<WfGroup> grp(G);
            for (int g = 0; g < G; ++g) grp[g] = WfGroup{(int64_t)g * F * hop, std::min(F, FT - g * F), hop};
            const int Sk = wf_tail_split(14, G, cus);
            int T = 0;
            for (int g = G - Sk; g < G; ++g)
                for (int j = 0; j < grp[g].nframes; ++j, ++T)
                    grp.push_back(WfGroup{grp[g].start + (int64_t)j * hop, 1, hop});
            CK(hipMemcpy(dg, grp.data(), sizeof(WfGroup) * grp.size(), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(wf_fft_r16<14>, dim3(G), dim3(WfR16<14>::NT), WfR16<14>::kLds, 0, dx, (int64_t)0,
                               dg, dwin, dtw, dref);
            CK(hipDeviceSynchronize());
            std::vector<float> a((size_t)G * N), b((size_t)G * N);
            CK(hipMemcpy(a.data(), dref, sizeof(float) * a.size(), hipMemcpyDeviceToHost));
            struct V {
                const char* name;
                std::function<void()> run;
                int map;  // 0: none (not checked), 1: bin order, 2: q16 positions
            };
            auto l32 = [&](int skip, int tail) {
                const int items = G - skip + tail;
                hipLaunchKernelGGL(wf_fft_l32, dim3(std::min(items, cus)), dim3(WfL32::NT), WfL32::kLds, s_a, dx,
                                   (int64_t)0, dg, dwin, dtw, dpart, 0, 0, items, dwork, G - skip, skip);
            };
            auto q16 = [&](int skip, int tail, int abl = 0) {
                const int items = G - skip + tail;
                decltype(&wf_fft_q16<0>) k = wf_fft_q16<0>;
                switch (abl) {
                    case 1: k = wf_fft_q16<1>; break;
                    case 2: k = wf_fft_q16<2>; break;
                    case 3: k = wf_fft_q16<3>; break;
                    case 4: k = wf_fft_q16<4>; break;
                    case 6: k = wf_fft_q16<6>; break;
                    case 7: k = wf_fft_q16<7>; break;
                    case 8: k = wf_fft_q16<8>; break;
                    case 32: k = wf_fft_q16<32>; break;
                    case 160: k = wf_fft_q16<160>; break;
                    case 40: k = wf_fft_q16<40>; break;
                    case 64: k = wf_fft_q16<64>; break;
                    case 96: k = wf_fft_q16<96>; break;
                    case 72: k = wf_fft_q16<72>; break;
                    case 104: k = wf_fft_q16<104>; break;
                }
                hipLaunchKernelGGL(k, dim3(std::min(items, cus)), dim3(WfQ16::NT), WfQ16::kLds, s_a, dx,
                                   (int64_t)0, dg, dwin, dtw, dpart, items, dwork, G - skip, skip, 0, 0);
            };
            std::vector<V> vs = {
                {"l32", [&] { l32(0, 0); }, 1},
                {"l32 tail", [&] { l32(Sk, T); }, 0},
                {"q16", [&] { q16(0, 0); }, 1},
                {"q16 tail", [&] { q16(Sk, T); }, 0},
                {"q16 spread", [&] { q16(0, 0, 8); }, 1},
                {"q16 spread tail", [&] { q16(Sk, T, 8); }, 0},
                {"q16 w16", [&] { q16(0, 0, 32); }, 1},
                {"q16 late spread", [&] { q16(0, 0, 72); }, 1},
                {"q16 w16 tail", [&] { q16(Sk, T, 32); }, 0},
                {"q16 w16 spread tail", [&] { q16(Sk, T, 40); }, 0},
                {"q16 late tail", [&] { q16(Sk, T, 64); }, 0},
                {"q16 w16 late", [&] { q16(0, 0, 96); }, 1},
                {"q16 w16 late tail", [&] { q16(Sk, T, 96); }, 0},
                {"q16 late spread tail", [&] { q16(Sk, T, 72); }, 0},
                {"q16 w16 late spread tail", [&] { q16(Sk, T, 104); }, 0},
                {"q16 -ld", [&] { q16(0, 0, 1); }, 0},
                {"q16 -lds", [&] { q16(0, 0, 2); }, 0},
                {"q16 -ld-lds", [&] { q16(0, 0, 3); }, 0},
                {"q16 -bar", [&] { q16(0, 0, 4); }, 0},
                {"q16 -lds-bar", [&] { q16(0, 0, 6); }, 0},
                {"q16 valu", [&] { q16(0, 0, 7); }, 0},
                {"mem8 512", [&] { hipLaunchKernelGGL(wf_mem8<512>, dim3(G), dim3(512), 0, s_a, dx, dg, dpart); }, 0},
                {"mem8 1024", [&] { hipLaunchKernelGGL(wf_mem8<1024>, dim3(G), dim3(1024), 0, s_a, dx, dg, dpart); }, 0},
                {"mem16 1024 d1", [&] { hipLaunchKernelGGL((wf_mem16<1024, 1, 0>), dim3(G), dim3(1024), 0, s_a, dx, dg, dpart); }, 0},
                {"mem16 1024 d2", [&] { hipLaunchKernelGGL((wf_mem16<1024, 2, 0>), dim3(G), dim3(1024), 0, s_a, dx, dg, dpart); }, 0},
                {"mem16 1024 d1 nt", [&] { hipLaunchKernelGGL((wf_mem16<1024, 1, 2>), dim3(G), dim3(1024), 0, s_a, dx, dg, dpart); }, 0},
                {"mem16 512 d1", [&] { hipLaunchKernelGGL((wf_mem16<512, 1, 0>), dim3(G), dim3(512), 0, s_a, dx, dg, dpart); }, 0},
                {"mem16 512 d2", [&] { hipLaunchKernelGGL((wf_mem16<512, 2, 0>), dim3(G), dim3(512), 0, s_a, dx, dg, dpart); }, 0},
                {"mem16 256 d2", [&] { hipLaunchKernelGGL((wf_mem16<256, 2, 0>), dim3(G), dim3(256), 0, s_a, dx, dg, dpart); }, 0},
            };
            {
                const size_t nf4 = (size_t)FT * hop * 8 / 16;
                vs.push_back({"stream 228x8", [&, nf4] { hipLaunchKernelGGL(stream_read, dim3(228 * 8), dim3(256), 0, s_a, (const float4*)dx, nf4, dpart); }, 0});
                vs.push_back({"stream 228x2", [&, nf4] { hipLaunchKernelGGL(stream_read, dim3(228 * 2), dim3(256), 0, s_a, (const float4*)dx, nf4, dpart); }, 0});
                vs.push_back({"chunk 228x4", [&, nf4] { hipLaunchKernelGGL(chunk_read, dim3(228 * 4), dim3(256), 0, s_a, (const float4*)dx, nf4 / (228 * 4), dpart); }, 0});
                vs.push_back({"chunk 2048", [&, nf4] { hipLaunchKernelGGL(chunk_read, dim3(2048), dim3(256), 0, s_a, (const float4*)dx, nf4 / 2048, dpart); }, 0});
            }
            if (getenv("MEMONLY")) vs.erase(vs.begin(), vs.begin() + 4 + 17);
            for (auto& v : vs) {
                const double us = time_us(v.run, s_a);
                printf("FT=%5d F=%d G=%4d S=%3d %-10s %8.2f us  %7.1f GB/s  %5.3f of 8 TB/s", FT, F, G, Sk, v.name, us,
                       alg / us * 1e-3, alg / us * 1e-3 / 8000.0);
                if (v.map) {
                    CK(hipMemset(dpart, 0, sizeof(float) * (size_t)G * N));
                    v.run();
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(b.data(), dpart, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
                    if (v.map == 2) {
                        std::vector<float> nb(b.size());
                        for (int g = 0; g < G; ++g)
                            for (int p = 0; p < N; ++p) nb[(size_t)g * N + q16_bin(p)] = b[(size_t)g * N + p];
                        b.swap(nb);
                    }
                    double d2 = 0, a2 = 0, worst = 0;
                    for (size_t i = 0; i < a.size(); ++i) {
                        const double d = fabs((double)a[i] - b[i]);
                        d2 += d * d;
                        a2 += (double)a[i] * a[i];
                        worst = std::max(worst, d / std::max((double)fabs(a[i]), 1e-30));
                    }
                    printf("  vs r16: rel-RMS %.2e max rel %.2e", sqrt(d2 / a2), worst);
                }
                printf("\n");
                fflush(stdout);
            }
#ifdef OWRX_WF_WSTAMPS
            for (int abl : {72, 0}) {
                time_us([&] { q16(0, 0, abl); }, s_a);
                std::vector<unsigned long long> st((size_t)256 * 16 * 12);
                CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wf_wstamp), sizeof(unsigned long long) * st.size()));
                const int nwg = std::min(G, cus);
                auto at = [&](int g, int w, int i) { return (long long)st[((size_t)g * 16 + w) * 12 + i]; };
                std::vector<long long> mn[12], mx[12];
                for (int g = 0; g < nwg; ++g) {
                    long long t0 = at(g, 0, 0);
                    for (int w = 0; w < 16; ++w) t0 = std::min(t0, at(g, w, 0));
                    for (int i = 0; i < 11; ++i) {
                        long long a = 1LL << 60, b = 0;
                        for (int w = 0; w < 16; ++w) {
                            a = std::min(a, at(g, w, i) - t0);
                            b = std::max(b, at(g, w, i) - t0);
                        }
                        mn[i].push_back(a);
                        mx[i].push_back(b);
                    }
                }
                const char* nm[] = {"frame start", "data arrived", "loads issued(early)", "P1 done", "barrier 1 out",
                                    "ex1 writes issued", "barrier 2 out", "barrier 4 out", "loads issued(late)",
                                    "P2 done", "P3 done"};
                printf("   q16<%d> per-wave stamps, frame 2 (cycles from the first wave's frame start; median over workgroups of first / last wave):\n", abl);
                for (int i = 0; i < 11; ++i) {
                    std::sort(mn[i].begin(), mn[i].end());
                    std::sort(mx[i].begin(), mx[i].end());
                    printf("     %-14s %7lld %7lld\n", nm[i], mn[i][mn[i].size() / 2], mx[i][mx[i].size() / 2]);
                }
            }
#endif
#ifdef OWRX_WF_STAMPS
            {
                time_us([&] { q16(0, 0); }, s_a);
                std::vector<unsigned long long> st((size_t)1024 * 16);
                CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wf_stamp), sizeof(unsigned long long) * st.size()));
                const int nwg = std::min(G, cus);
                auto med = [&](int a0, int b0) {
                    std::vector<long long> d;
                    for (int q = 0; q < nwg; ++q) d.push_back((long long)(st[q * 16 + b0] - st[q * 16 + a0]));
                    std::sort(d.begin(), d.end());
                    return d[d.size() / 2];
                };
                printf("   q16 stamps (median cycles, wave 0, frame 1): clock %.2f GHz, kernel %lld;"
                       " wait+window %lld P1 %lld bar+wr+bar %lld P2 %lld bar+wr+bar %lld P3 %lld = frame %lld\n",
                       (double)med(12, 13) / (double)med(14, 15) * 0.1, med(12, 13), med(0, 1), med(1, 2), med(2, 3),
                       med(3, 4), med(4, 5), med(5, 6), med(0, 6));
            }
#endif
        }
    }
    return 0;
}
