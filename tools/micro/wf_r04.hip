// Waterfall FFT kernels in isolation (diagnostic, not part of the product), round 4: C3's
// geometry (10 Msps, N = 16384, hop 11454), FT frames per launch in groups of F, frames read
// from HBM (OWRX_WF_FLUSH=1, default: 512 MiB streamed between launches, as the DDC's operand
// streams evict them in the engine) or from the Infinity Cache (OWRX_WF_FLUSH=0).
// Prints us per launch and the rate on the algorithmic bytes (the frames' span of cf32 IQ,
// 8 B per sample read once), for the production kernel(s) and the load pattern alone, and the
// relative difference of each kernel's partial rows from wf_fft_r16<14> (the radix-16 kernel).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-slp-vectorize wf_r04.hip -o wf_r04
// Run:   ./wf_r04 [FT ...]
#include "../../openwebrx_amd/csrc/kernels_waterfall.hip"
#include "wf_l32x.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
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

// the frame loads (16 B per lane, 512 threads) and partial-row stores alone, the next frame in
// flight while the current one is summed: the memory floor of the access pattern
__global__ void __launch_bounds__(512)
wf_mem_pf(const float2* __restrict__ blk, const WfGroup* __restrict__ groups, float* __restrict__ partial) {
    const WfGroup g = groups[blockIdx.x];
    const int t = threadIdx.x;
    const int nfr = g.nframes;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(blk + g.start), 0,
                                                      (int)(8 * ((int64_t)(nfr - 1) * g.hop + N)), 0x00020000);
    float acc[16] = {};
    float4 nx[16];
    auto ld = [&](int f, float4* v) {
        const int fo = f < nfr ? f * g.hop * 8 : (1 << 30);
#pragma unroll
        for (int m = 0; m < 16; ++m)
            v[m] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, t * 16 + fo, m * 8192, 0));
    };
    ld(0, nx);
    for (int f = 0; f < nfr; ++f) {
        float4 x[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) x[m] = nx[m];
        ld(f + 1, nx);
#pragma unroll
        for (int m = 0; m < 16; ++m)
            acc[m] = fmaf(x[m].x, x[m].x, fmaf(x[m].y, x[m].y, fmaf(x[m].z, x[m].z, fmaf(x[m].w, x[m].w, acc[m]))));
    }
#pragma unroll
    for (int m = 0; m < 16; ++m)
        for (int u = 0; u < 2; ++u) partial[(int64_t)blockIdx.x * N + 2 * (t + 512 * m) + u] = acc[m];
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
static bool flush_on() {
    static const bool v = !getenv("OWRX_WF_FLUSH") || atoi(getenv("OWRX_WF_FLUSH"));
    return v;
}
#ifdef OWRX_WF_STAMPS
__global__ void mark_rt(unsigned long long* out, int i) {
    if (threadIdx.x == 0) out[i] = __builtin_amdgcn_s_memrealtime();
}
#endif

static double time_us(const std::function<void()>& launch, hipStream_t stream = 0) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t fb = (size_t)512 << 20;
    if (!g_flush) {
        CK(hipMalloc(&g_flush, fb));
        CK(hipMemset(g_flush, 0, fb));
    }
    const int iters = 40;
    std::vector<float> t;
    for (int i = 0; i < iters + 5; ++i) {
        if (flush_on())
            hipLaunchKernelGGL(flush_read, dim3(4096), dim3(256), 0, 0, (const float4*)g_flush, fb / 16,
                               (float*)g_flush);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, stream));
        launch();
        CK(hipEventRecord(e1, stream));
        CK(hipDeviceSynchronize());
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
    if (fts.empty()) fts = {960, 1920};
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
#define SETX(v) CK(hipFuncSetAttribute((const void*)wf_fft_l32x<v>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WfL32::kLds))
    SETX(0); SETX(1); SETX(2); SETX(3); SETX(4); SETX(5); SETX(6);
    printf("N=%d hop=%d, frames from %s\n", N, hop, flush_on() ? "HBM (512 MiB flushed between launches)" : "cache");
    // CU-masked streams (the engine's stream A masks 16 CUs off for the serial streams):
    // bits [0, 240) as create_streams does, and 240 CUs with every 16th bit off instead
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t s_lo = nullptr, s_even = nullptr, s_hi = nullptr, s_all = nullptr, s_plain = nullptr;
    CK(hipStreamCreateWithFlags(&s_plain, hipStreamNonBlocking));
    {
        const int words = (ncu + 31) / 32;
        std::vector<uint32_t> lo(words, 0), even(words, 0), hi(words, 0);
        for (int c = 0; c < ncu; ++c) {
            if (c < ncu - 16) lo[c / 32] |= 1u << (c % 32);
            if (c % 16 != 15) even[c / 32] |= 1u << (c % 32);
            if (c >= 16) hi[c / 32] |= 1u << (c % 32);
        }
        CK(hipExtStreamCreateWithCUMask(&s_lo, words, lo.data()));
        CK(hipExtStreamCreateWithCUMask(&s_even, words, even.data()));
        CK(hipExtStreamCreateWithCUMask(&s_hi, words, hi.data()));
        std::vector<uint32_t> all(words, 0xffffffffu);
        CK(hipExtStreamCreateWithCUMask(&s_all, words, all.data()));
    }
    auto l32 = [&](int G, hipStream_t st, int skip = 0, int tail = 0) {
        const int items = G - skip + tail;  // (the counters are left zeroed by each launch)
        hipLaunchKernelGGL(wf_fft_l32, dim3(std::min(items, st == 0 || st == s_plain || st == s_all ? 256 : 240)), dim3(WfL32::NT), WfL32::kLds, st, dx, (int64_t)0,
                           dg, dwin, dtw, dpart, 0, 0, items, dwork, G - skip, skip);
    };
    printf("CUs %d\n", ncu);
    for (int FT : fts) {
        const double alg = 8.0 * ((double)(FT - 1) * hop + N);
        for (int F : {2, 4, 8}) {
            const int G = (FT + F - 1) / F;
            std::vector<WfGroup> grp(G);
            for (int g = 0; g < G; ++g) grp[g] = WfGroup{(int64_t)g * F * hop, std::min(F, FT - g * F), hop};
            // the engine's tail split for a 240-CU stream: the last S groups also frame by frame
            const int S = wf_tail_split(14, G, 240);
            int T = 0;
            for (int g = G - S; g < G; ++g)
                for (int j = 0; j < grp[g].nframes; ++j, ++T)
                    grp.push_back(WfGroup{grp[g].start + (int64_t)j * hop, 1, hop});
            CK(hipMemcpy(dg, grp.data(), sizeof(WfGroup) * grp.size(), hipMemcpyHostToDevice));
            {
                // bit identity: a split group's frames folded in order == the group's own sum
                l32(G, 0);
                CK(hipDeviceSynchronize());
                std::vector<float> A((size_t)G * N), B((size_t)(G + T) * N);
                CK(hipMemcpy(A.data(), dpart, sizeof(float) * A.size(), hipMemcpyDeviceToHost));
                l32(G, 0, S, T);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(B.data(), dpart, sizeof(float) * B.size(), hipMemcpyDeviceToHost));
                size_t bad = 0;
                int f0 = G;
                for (int g = 0; g < G; ++g) {
                    for (int k = 0; k < N; ++k) {
                        float v;
                        if (g < G - S) {
                            v = B[(size_t)g * N + k];
                        } else {
                            v = B[(size_t)f0 * N + k];
                            for (int j = 1; j < grp[g].nframes; ++j) v = v + B[(size_t)(f0 + j) * N + k];
                        }
                        bad += memcmp(&v, &A[(size_t)g * N + k], 4) != 0;
                    }
                    if (g >= G - S) f0 += grp[g].nframes;
                }
                printf("FT=%5d F=%d G=%4d tail split S=%d groups (%d frames): %zu of %zu partial bins differ from the unsplit launch\n",
                       FT, F, G, S, T, bad, (size_t)G * N);
            }
            hipLaunchKernelGGL(wf_fft_r16<14>, dim3(G), dim3(WfR16<14>::NT), WfR16<14>::kLds, 0, dx, (int64_t)0,
                               dg, dwin, dtw, dref);
            CK(hipDeviceSynchronize());
            std::vector<float> a((size_t)G * N), b((size_t)G * N);
            CK(hipMemcpy(a.data(), dref, sizeof(float) * a.size(), hipMemcpyDeviceToHost));
            struct V {
                const char* name;
                std::function<void()> run;
                bool check;
                bool half_major = false;  // partial rows bin 2k + h at h N/2 + k
                hipStream_t stream = 0;
            };
            std::vector<V> vs = {
                {"l32", [&] {
                     l32(G, 0);
                 }, true},
                {"r16", [&] {
                     hipLaunchKernelGGL(wf_fft_r16<14>, dim3(G), dim3(WfR16<14>::NT), WfR16<14>::kLds, 0, dx,
                                        (int64_t)0, dg, dwin, dtw, dpart);
                 }, true},
                {"l32 mask[0,240)", [&] {
                     l32(G, s_lo);
                 }, false, false, s_lo},
                {"l32 tail mask[0,240)", [&] {
                     l32(G, s_lo, S, T);
                 }, false, false, s_lo},

                {"l32 tail plain", [&] {
                     l32(G, s_plain, S, T);
                 }, false, false, s_plain},
                {"l32 mask[16,256)", [&] {
                     l32(G, s_hi);
                 }, false, false, s_hi},
                {"l32 mask-all", [&] {
                     l32(G, s_all);
                 }, false, false, s_all},
                {"l32 stream", [&] {
                     l32(G, s_plain);
                 }, false, false, s_plain},
                {"mem mask[0,240)", [&] {
                     hipLaunchKernelGGL(wf_mem_pf, dim3(G), dim3(512), 0, s_lo, dx, dg, dpart);
                 }, false, false, s_lo},
                {"l32 mask-every16", [&] {
                     l32(G, s_even);
                 }, false, false, s_even},
#define XV(v, nm) {nm, [&] { hipLaunchKernelGGL(wf_fft_l32x<v>, dim3(G), dim3(WfL32::NT), WfL32::kLds, 0, dx, dg, dwin, dtw, dpart); }, v == 0}
                XV(0, "x0"), XV(1, "x-load"), XV(2, "x-lds"), XV(3, "x-ld-lds"), XV(4, "x-math"), XV(5, "x-ld-mth"), XV(6, "x-lds-mth"),
                {"mem", [&] {
                     hipLaunchKernelGGL(wf_mem_pf, dim3(G), dim3(512), 0, 0, dx, dg, dpart);
                 }, false},
            };
            for (auto& v : vs) {
                const double us = time_us(v.run, v.stream);
                printf("FT=%5d F=%d G=%4d %-8s %8.2f us  %7.1f GB/s  %5.1f %% of 8 TB/s", FT, F, G, v.name, us,
                       alg / us * 1e-3, alg / us * 1e-3 / 80.0);
                if (v.check) {
                    v.run();
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(b.data(), dpart, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
                    double d2 = 0, a2 = 0, worst = 0;
                    if (v.half_major) {  // back to bin order
                        std::vector<float> nb(b.size());
                        for (int q = 0; q < G; ++q)
                            for (int k = 0; k < N; ++k)
                                nb[(size_t)q * N + k] = b[(size_t)q * N + (k & 1) * (N / 2) + (k >> 1)];
                        b.swap(nb);
                    }
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
#ifdef OWRX_WF_STAMPS
            if (F == 4) {
                auto stamps = [&](const char* nmk, int nwg, const std::function<void()>& run) {
                    time_us(run);
                    std::vector<unsigned long long> st((size_t)1024 * 16);
                    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wf_stamp), sizeof(unsigned long long) * st.size()));
                    auto med = [&](int a0, int b0) {
                        std::vector<long long> d;
                        for (int q = 0; q < std::min(nwg, 1024); ++q) d.push_back((long long)(st[q * 16 + b0] - st[q * 16 + a0]));
                        std::sort(d.begin(), d.end());
                        return d[d.size() / 2];
                    };
                    const double clk = (double)med(0, 13) / (double)med(14, 15) * 0.1;
                    printf("   stamps %s (median cycles, wave 0): clock %.2f GHz, total %lld\n", nmk, clk, med(0, 13));
                    const char* nm[] = {"load+dft32", "P1 bar+store", "bar+P2", "bar+P3 reads", "P3 math"};
                    for (int f = 0; f < 2; ++f) {
                        const int b0 = 1 + 6 * f;
                        printf("   frame %d starts at %lld:", f, med(0, b0));
                        for (int p = 0; p < 5; ++p) printf("  %s %lld", nm[p], med(b0 + p, b0 + p + 1));
                        printf("\n");
                    }
                    printf("   frame 2.. to end: %lld\n", med(12, 13));
                };
                // l32 on a plain and on a CU-masked stream: per-workgroup start and end (realtime)
                unsigned long long* dmark = nullptr;
                CK(hipMalloc(&dmark, 64));
                for (hipStream_t sq : {s_plain, s_lo}) {
                    time_us([&] {
                        hipLaunchKernelGGL(mark_rt, dim3(1), dim3(64), 0, sq, dmark, 0);
                        l32(G, sq);
                        hipLaunchKernelGGL(mark_rt, dim3(1), dim3(64), 0, sq, dmark, 1);
                    }, sq);
                    unsigned long long mk[2];
                    CK(hipMemcpy(mk, dmark, 16, hipMemcpyDeviceToHost));
                    std::vector<unsigned long long> st((size_t)1024 * 16);
                    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wf_stamp), sizeof(unsigned long long) * st.size()));
                    const int nwg = std::min(G, sq == s_plain ? 256 : 240);
                    unsigned long long t0m = ~0ull;
                    for (int q = 0; q < nwg; ++q) t0m = std::min(t0m, st[q * 16 + 14]);
                    std::vector<double> a0, a1, du;
                    for (int q = 0; q < nwg; ++q) {
                        a0.push_back((st[q * 16 + 14] - t0m) / 100.0);
                        a1.push_back((st[q * 16 + 15] - t0m) / 100.0);
                        du.push_back((st[q * 16 + 15] - st[q * 16 + 14]) / 100.0);
                    }
                    auto pr = [&](const char* nm, std::vector<double> v) {
                        std::sort(v.begin(), v.end());
                        printf("  %s p0 %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f", nm, v[0], v[v.size() / 10],
                               v[v.size() / 2], v[v.size() * 9 / 10], v.back());
                    };
                    printf("   l32 %s: first workgroup %.1f us after the marker before, marker after at %.1f us\n",
                           sq == s_plain ? "plain" : "mask[0,240)", ((long long)t0m - (long long)mk[0]) / 100.0,
                           ((long long)mk[1] - (long long)mk[0]) / 100.0);
                    printf("   l32 %s wg us:", sq == s_plain ? "plain" : "mask[0,240)");
                    pr("start", a0);
                    pr("end", a1);
                    pr("dur", du);
                    printf("\n");
                }
                stamps("x0", G, [&] { hipLaunchKernelGGL(wf_fft_l32x<0>, dim3(G), dim3(WfL32::NT), WfL32::kLds, 0, dx, dg, dwin, dtw, dpart); });
            }
#endif
        }
    }
    return 0;
}
