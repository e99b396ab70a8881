// Waterfall FFT kernels in isolation (diagnostic; not part of the product): C3's geometry
// (10 Msps, N = 16384, hop 11454) over FT frames, launched back to back so the chip holds its
// loaded clock.  Prints µs per launch and the HBM rate on the algorithmic bytes (the frames'
// span of cf32 IQ, read once) for:
//   r16 G x F     the production radix-16 kernel, G groups of F frames
//   lean G x F    wf_fft_lean (table twiddles, swizzled image)
//   mem G x F     the same loads and partial-row stores with no FFT (the memory floor)
//   fin           wf_finalize of those partial rows (4 rows)
//   rocfft        a batched out-of-place C2C rocFFT of FT contiguous 16384-point frames (yardstick)
// and the largest relative difference of the lean partial rows from the production ones.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-slp-vectorize -I../../openwebrx_amd/csrc wf_bench.hip -lrocfft -o wf_bench
// Run:   ./wf_bench [FT]
#include "../../openwebrx_amd/csrc/kernels_waterfall.hip"
#include "wf_variants.hip"

#include <rocfft/rocfft.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <map>

using namespace owrx;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                                   \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

// the production kernel's loads and partial-row stores, no transform
template <int LOGN>
__global__ void __launch_bounds__(1024)
wf_mem_only(const float2* __restrict__ blk, const WfGroup* __restrict__ groups,
            const float* __restrict__ window, float* __restrict__ partial) {
    constexpr int N = 1 << LOGN, NT = N / 16;
    const WfGroup g = groups[blockIdx.x];
    const int t = threadIdx.x;
    float acc[16] = {};
    for (int f = 0; f < g.nframes; ++f) {
        const float2* x = blk + g.start + (int64_t)f * g.hop;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float2 v = x[t + NT * r];
            const float w = window[t + NT * r];
            acc[r] = fmaf(v.x * w, v.x * w, fmaf(v.y * w, v.y * w, acc[r]));
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) partial[(int64_t)blockIdx.x * N + t + NT * r] = acc[r];
}

constexpr int LOGN = 14, N = 1 << LOGN;

__global__ void flush_read(const float4* __restrict__ p, size_t n, float* sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;  // never true for the zeroed buffer: keeps the reads
}
// the b2/l32 load pattern alone: 512 threads, 16-B per lane per m1, |x|^2 kept so the loads stay;
// PF = 1 prefetches the next frame into registers
template <int PF>
__global__ void __launch_bounds__(512)
wf_mem_b2(const float2* __restrict__ blk, const WfGroup* __restrict__ groups, float* __restrict__ partial) {
    const WfGroup g = groups[blockIdx.x];
    const int t = threadIdx.x;
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(blk + g.start), 0,
                                                      (int)(8 * ((int64_t)(g.nframes - 1) * g.hop + 16384)), 0x00020000);
    float acc[16] = {};
    float4 nx[16];
    auto ld = [&](int f, float4* v) {
#pragma unroll
        for (int m = 0; m < 16; ++m)
            v[m] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, (t * 2 + f * g.hop) * 8, m * 8192, 0));
    };
    if (PF) ld(0, nx);
    for (int f = 0; f < g.nframes; ++f) {
        float4 x[16];
        if (PF) {
#pragma unroll
            for (int m = 0; m < 16; ++m) x[m] = nx[m];
            if (f + 1 < g.nframes) ld(f + 1, nx);
        } else {
            ld(f, x);
        }
#pragma unroll
        for (int m = 0; m < 16; ++m)
            acc[m] = fmaf(x[m].x, x[m].x, fmaf(x[m].y, x[m].y, fmaf(x[m].z, x[m].z, fmaf(x[m].w, x[m].w, acc[m]))));
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) partial[(int64_t)blockIdx.x * 16384 + t + 512 * m] = acc[m];
}
// OWRX_WF_FLUSH=1: before every timed launch, write 512 MiB elsewhere so the frames come from HBM
// (as in the engine, where the DDC's operand streams evict them) instead of the Infinity Cache
static void* g_flush = nullptr;
static bool flush_on() {
    static const bool v = getenv("OWRX_WF_FLUSH") && atoi(getenv("OWRX_WF_FLUSH"));
    return v;
}
template <typename F>
static double time_us_flushed(F&& launch, int iters = 30) {
    const size_t fb = (size_t)512 << 20;
    if (!g_flush) CK(hipMalloc(&g_flush, fb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double tot = 0;
    for (int i = 0; i < iters + 3; ++i) {
        hipLaunchKernelGGL(flush_read, dim3(4096), dim3(256), 0, 0, (const float4*)g_flush, fb / 16,
                           (float*)g_flush);
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (i >= 3) tot += ms;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return tot * 1e3 / iters;
}
template <typename F>
static double time_us(F&& launch, int warm = 50, int iters = 200) {
    if (flush_on()) return time_us_flushed(launch);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < warm; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
    const int hop = 11454;
    const int FT = argc > 1 ? atoi(argv[1]) : 366;
    const int64_t S = (int64_t)FT * hop + N;
    const double alg_bytes = 8.0 * ((double)(FT - 1) * hop + N);
    std::vector<float2> x(S);
    srand(1);
    for (auto& v : x) v = float2{rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f};
    std::vector<float> win(N);
    for (int i = 0; i < N; ++i) win[i] = (float)(0.54 - 0.46 * cos(2 * M_PI * i / (N - 1)));
    std::vector<float2> tw(N);
    for (int k = 0; k < N; ++k) tw[k] = float2{(float)cos(2 * M_PI * k / N), (float)-sin(2 * M_PI * k / N)};
    float2 *dx, *dtw;
    float *dwin, *dpart, *dpart2;
    WfGroup* dg;
    CK(hipMalloc(&dx, sizeof(float2) * S));
    CK(hipMalloc(&dtw, sizeof(float2) * N));
    CK(hipMalloc(&dwin, sizeof(float) * N));
    CK(hipMalloc(&dpart, sizeof(float) * (size_t)FT * N));
    CK(hipMalloc(&dpart2, sizeof(float) * (size_t)FT * N));
    CK(hipMalloc(&dg, sizeof(WfGroup) * FT));
    CK(hipMemcpy(dx, x.data(), sizeof(float2) * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtw, tw.data(), sizeof(float2) * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwin, win.data(), sizeof(float) * N, hipMemcpyHostToDevice));
    std::vector<float2> tw2(WfB2::kTw2);
    for (int j = 0; j < 64; ++j)
        for (int k = 0; k < 16; ++k)
            tw2[16 * j + k] = float2{(float)cos(2 * M_PI * j * k / 1024), (float)-sin(2 * M_PI * j * k / 1024)};
    float2* dtw2;
    CK(hipMalloc(&dtw2, sizeof(float2) * tw2.size()));
    CK(hipMemcpy(dtw2, tw2.data(), sizeof(float2) * tw2.size(), hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void*)wf_fft_b2<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfB2::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_b2<0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfB2::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_b2<0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfB2::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_b2<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfB2::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_b2<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfB2::kLds));
    using KL = WfLean<LOGN>;
    using KR = WfR16<LOGN>;
    CK(hipFuncSetAttribute((const void*)wf_fft_lean<LOGN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)KL::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_r16<LOGN>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)KR::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_l32, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfL32::kLds));
    CK(hipFuncSetAttribute((const void*)wf_fft_h32, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfH32::kLds));
    WfFrame* dfr;
    float* dmember;
    int* dtick;
    CK(hipMalloc(&dfr, sizeof(WfFrame) * (FT + 64)));
    CK(hipMalloc(&dmember, sizeof(float) * (size_t)(FT + 64) * N));
    CK(hipMalloc(&dtick, sizeof(int) * FT));
    CK(hipMemset(dtick, 0, sizeof(int) * FT));
    // frames of groups of F, members of a group on one XCD (workgroup ids w, w + 8, ...)
    auto frame_table = [&](int F) {
        const int G = (FT + F - 1) / F;
        std::vector<std::vector<WfFrame>> col(8);
        for (int g = 0; g < G; ++g) {
            const int nm = std::min(F, FT - g * F);
            auto& c = col[g % 8];
            for (int m = 0; m < nm; ++m)
                c.push_back(WfFrame{(int64_t)(g * F + m) * hop, g, (int16_t)m, (int16_t)nm});
        }
        size_t rows = 0;
        for (auto& c : col) rows = std::max(rows, c.size());
        std::vector<WfFrame> tab(rows * 8, WfFrame{0, 0, 0, 0});
        for (int x = 0; x < 8; ++x)
            for (size_t i = 0; i < col[x].size(); ++i) tab[x + 8 * i] = col[x][i];
        CK(hipMemcpy(dfr, tab.data(), sizeof(WfFrame) * tab.size(), hipMemcpyHostToDevice));
        return (int)tab.size();
    };
    auto groups = [&](int F) {
        const int G = (FT + F - 1) / F;
        std::vector<WfGroup> grp(G);
        for (int g = 0; g < G; ++g) grp[g] = WfGroup{(int64_t)g * F * hop, std::min(F, FT - g * F), hop};
        CK(hipMemcpy(dg, grp.data(), sizeof(WfGroup) * G, hipMemcpyHostToDevice));
        return G;
    };
    auto report = [&](const char* name, int G, int F, double us) {
        printf("%-6s G=%4d F=%d  %8.2f us  %7.1f GB/s  (%.1f %% of 8 TB/s)\n", name, G, F, us,
               alg_bytes / us * 1e-3, alg_bytes / us * 1e-3 / 80.0);
        fflush(stdout);
    };
    printf("FT=%d frames, N=%d, hop=%d, algorithmic %.2f MB; lean LDS %zu B, r16 LDS %zu B\n", FT, N,
           hop, alg_bytes * 1e-6, KL::kLds, KR::kLds);
    for (int F : {1, 2, 3, 4}) {
        const int G = groups(F);
        report("r16", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_fft_r16<LOGN>, dim3(G), dim3(KR::NT), KR::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dpart);
               }));
        report("lean", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_fft_lean<LOGN>, dim3(G), dim3(KL::NT), KL::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dpart2);
               }));
        report("l32", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_fft_l32, dim3(G), dim3(WfL32::NT), WfL32::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dpart2, 0, 0);
               }));
        report("b2", G, F, time_us([&] {
                   hipLaunchKernelGGL((wf_fft_b2<0, 0>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dtw2, dpart2);
               }));
        report("b2pf", G, F, time_us([&] {
                   hipLaunchKernelGGL((wf_fft_b2<1, 0>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dtw2, dpart2);
               }));
        report("b2pfnl", G, F, time_us([&] {
                   hipLaunchKernelGGL((wf_fft_b2<1, 1>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dtw2, dpart2);
               }));
        report("b2nold", G, F, time_us([&] {
                   hipLaunchKernelGGL((wf_fft_b2<0, 1>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dtw2, dpart2);
               }));
        report("b2nobar", G, F, time_us([&] {
                   hipLaunchKernelGGL((wf_fft_b2<0, 2>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg,
                                      dwin, dtw, dtw2, dpart2);
               }));
        const int nwg = frame_table(F);
        report("h32", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_fft_h32, dim3(nwg), dim3(WfH32::NT), WfH32::kLds, 0, dx, (int64_t)0, dfr,
                                      dwin, dtw, dmember, dtick, dpart2);
               }));
        report("mem", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_mem_only<LOGN>, dim3(G), dim3(1024), 0, 0, dx, dg, dwin, dpart2);
               }));
        report("memb2", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_mem_b2<0>, dim3(G), dim3(512), 0, 0, dx, dg, dpart2);
               }));
        report("mempf", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_mem_b2<1>, dim3(G), dim3(512), 0, 0, dx, dg, dpart2);
               }));
        // parity of lean vs r16 on the same groups
        hipLaunchKernelGGL(wf_fft_r16<LOGN>, dim3(G), dim3(KR::NT), KR::kLds, 0, dx, (int64_t)0, dg, dwin, dtw,
                           dpart);
        hipLaunchKernelGGL(wf_fft_lean<LOGN>, dim3(G), dim3(KL::NT), KL::kLds, 0, dx, (int64_t)0, dg, dwin, dtw,
                           dpart2);
        CK(hipDeviceSynchronize());
        std::vector<float> a((size_t)G * N), b((size_t)G * N);
        CK(hipMemcpy(a.data(), dpart, sizeof(float) * a.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), dpart2, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
        double worst = 0, mx = 0;
        for (size_t i = 0; i < a.size(); ++i) mx = std::max(mx, (double)fabs(a[i]));
        double rms_d = 0, rms_a = 0;
        for (size_t i = 0; i < a.size(); ++i) {
            const double d = fabs((double)a[i] - b[i]);
            worst = std::max(worst, d / std::max((double)fabs(a[i]), 1e-30));
            rms_d += d * d;
            rms_a += (double)a[i] * a[i];
        }
        printf("       lean vs r16: max rel %.3e, rel-RMS %.3e\n", worst, sqrt(rms_d / rms_a));
        hipLaunchKernelGGL(wf_fft_l32, dim3(G), dim3(WfL32::NT), WfL32::kLds, 0, dx, (int64_t)0, dg, dwin, dtw,
                           dpart2, 0, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), dpart2, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
        worst = 0; rms_d = 0;
        for (size_t i = 0; i < a.size(); ++i) {
            const double d = fabs((double)a[i] - b[i]);
            worst = std::max(worst, d / std::max((double)fabs(a[i]), 1e-30));
            rms_d += d * d;
        }
        printf("       l32  vs r16: max rel %.3e, rel-RMS %.3e\n", worst, sqrt(rms_d / rms_a));
        hipLaunchKernelGGL((wf_fft_b2<0, 0>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg, dwin, dtw,
                           dtw2, dpart2);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), dpart2, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
        worst = 0; rms_d = 0;
        for (size_t i = 0; i < a.size(); ++i) {
            const double d = fabs((double)a[i] - b[i]);
            worst = std::max(worst, d / std::max((double)fabs(a[i]), 1e-30));
            rms_d += d * d;
        }
        printf("       b2   vs r16: max rel %.3e, rel-RMS %.3e\n", worst, sqrt(rms_d / rms_a));
        hipLaunchKernelGGL((wf_fft_b2<1, 0>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg, dwin, dtw,
                           dtw2, dpart2);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), dpart2, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
        worst = 0; rms_d = 0;
        for (size_t i = 0; i < a.size(); ++i) {
            const double d = fabs((double)a[i] - b[i]);
            worst = std::max(worst, d / std::max((double)fabs(a[i]), 1e-30));
            rms_d += d * d;
        }
        printf("       b2pf vs r16: max rel %.3e, rel-RMS %.3e\n", worst, sqrt(rms_d / rms_a));
        hipLaunchKernelGGL(wf_fft_h32, dim3(nwg), dim3(WfH32::NT), WfH32::kLds, 0, dx, (int64_t)0, dfr, dwin, dtw,
                           dmember, dtick, dpart2);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), dpart2, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
        worst = 0; rms_d = 0;
        for (size_t i = 0; i < a.size(); ++i) {
            const double d = fabs((double)a[i] - b[i]);
            worst = std::max(worst, d / std::max((double)fabs(a[i]), 1e-30));
            rms_d += d * d;
        }
        printf("       h32  vs r16: max rel %.3e, rel-RMS %.3e\n", worst, sqrt(rms_d / rms_a));
        {  // determinism: a second run bit-identical
            std::vector<float> c2v(b.size());
            hipLaunchKernelGGL(wf_fft_h32, dim3(nwg), dim3(WfH32::NT), WfH32::kLds, 0, dx, (int64_t)0, dfr, dwin,
                               dtw, dmember, dtick, dpart2);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(c2v.data(), dpart2, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
            printf("       h32 rerun bit-identical: %s\n", memcmp(c2v.data(), b.data(), 4 * b.size()) ? "NO" : "yes");
        }
#ifdef OWRX_WF_STAMPS
        for (int abl = 0; abl < 2; ++abl) {
            // b2 phase stamps of wave 0, frame 1: medians over workgroups
            if (F < 2) break;
            time_us([&] {
                if (abl)
                    hipLaunchKernelGGL((wf_fft_b2<0, 1>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg,
                                       dwin, dtw, dtw2, dpart2);
                else
                    hipLaunchKernelGGL((wf_fft_b2<0, 0>), dim3(G), dim3(WfB2::NT), WfB2::kLds, 0, dx, (int64_t)0, dg,
                                       dwin, dtw, dtw2, dpart2);
            });
            std::vector<unsigned long long> st((size_t)1024 * 16);
            CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wf_stamp), sizeof(unsigned long long) * st.size()));
            auto med = [&](int a, int b) {
                std::vector<long long> d;
                for (int g = 0; g < std::min(G, 1024); ++g) d.push_back((long long)(st[g * 16 + b] - st[g * 16 + a]));
                std::sort(d.begin(), d.end());
                return d[d.size() / 2];
            };
            const double clk = (double)med(0, 13) / (double)med(14, 15) * 0.1;
            {
                // co-residency: the most workgroups alive at once on one CU (HW_ID: CU, SH, SE; XCC_ID)
                std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev;
                for (int g = 0; g < std::min(G, 1024); ++g) {
                    const unsigned long long id = st[g * 16 + 12];
                    const unsigned lo = (unsigned)id, xcc = (unsigned)(id >> 32) & 15;
                    const unsigned long long cu = ((unsigned long long)xcc << 16) | (lo & 0xff00) | ((lo >> 12) & 0xf) << 20;
                    ev[cu].push_back({st[g * 16 + 0], +1});
                    ev[cu].push_back({st[g * 16 + 13], -1});
                }
                int best = 0;
                for (auto& kv : ev) {
                    std::sort(kv.second.begin(), kv.second.end());
                    int c = 0;
                    for (auto& e : kv.second) best = std::max(best, c += e.second);
                }
                printf("       b2 CUs used %zu, max workgroups resident on one CU %d\n", ev.size(), best);
            }
            printf("       b2%s stamps (median cycles, wave 0): clock %.2f GHz, total %lld, frame0 %lld;"
                   " frame 1: S1+X1 %lld S2+X2 %lld S3+X3 %lld S4 %lld\n",
                   abl ? "nold" : "", clk, med(0, 13), med(0, 1), med(1, 2), med(2, 3), med(3, 4), med(4, 5));
        }
        {
            // l32 phase stamps of wave 0: medians over workgroups
            time_us([&] {
                hipLaunchKernelGGL(wf_fft_l32, dim3(G), dim3(WfL32::NT), WfL32::kLds, 0, dx, (int64_t)0, dg,
                                   dwin, dtw, dpart2, 0, 0);
            });
            std::vector<unsigned long long> st((size_t)1024 * 16);
            CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wf_stamp), sizeof(unsigned long long) * st.size()));
            auto med = [&](int a, int b) {
                std::vector<long long> d;
                for (int g = 0; g < std::min(G, 1024); ++g) d.push_back((long long)(st[g * 16 + b] - st[g * 16 + a]));
                std::sort(d.begin(), d.end());
                return d[d.size() / 2];
            };
            const double clk = (double)med(0, 13) / (double)med(14, 15) * 0.1;  // GHz (realtime: 100 MHz)
            printf("       stamps (median cycles, wave 0): clock %.2f GHz, total %lld\n", clk, med(0, 13));
            const char* nm[] = {"dft32", "P1 barrier+store", "P2", "P3 reads", "P3 dft16x2"};
            for (int f = 0; f < std::min(F, 2); ++f) {
                const int b = 1 + 6 * f;
                printf("       frame %d starts at %lld:", f, med(0, b));
                for (int p = 0; p < 5; ++p) printf("  %s %lld", nm[p], med(b + p, b + p + 1));
                printf("\n");
            }
        }
#endif
        if (F == 2) {
            // finalize of 4 rows of ~G/4 groups each
            std::vector<WfRow> rows(4);
            const int per = G / 4;
            for (int r = 0; r < 4; ++r) rows[r] = WfRow{r * per, per, 0, 1, r, 0};
            WfRow* drows;
            float *dcar, *df32;
            int16_t* ds16;
            CK(hipMalloc(&drows, sizeof(WfRow) * 4));
            CK(hipMalloc(&dcar, sizeof(float) * 2 * N));
            CK(hipMalloc(&df32, sizeof(float) * 4 * N));
            CK(hipMalloc(&ds16, sizeof(int16_t) * 4 * N));
            CK(hipMemcpy(drows, rows.data(), sizeof(WfRow) * 4, hipMemcpyHostToDevice));
            const double us = time_us([&] {
                CK(launch_wf_finalize(dpart, drows, 4, dcar, dcar + N, N, -90.0f, 1, ds16, df32, 0));
            });
            printf("fin    G=%4d      %8.2f us  (reads %.1f MB of partial rows)\n", G, us,
                   4.0 * per * N * 4 * 1e-6);
        }
    }
    // rocFFT yardstick: FT contiguous frames, out of place
    {
        rocfft_setup();
        rocfft_plan plan;
        size_t len = N;
        if (rocfft_plan_create(&plan, rocfft_placement_notinplace, rocfft_transform_type_complex_forward,
                               rocfft_precision_single, 1, &len, (size_t)FT, nullptr) != rocfft_status_success) {
            printf("rocfft plan failed\n");
            return 1;
        }
        size_t wsz = 0;
        rocfft_plan_get_work_buffer_size(plan, &wsz);
        void* wbuf = nullptr;
        rocfft_execution_info info;
        rocfft_execution_info_create(&info);
        if (wsz) {
            CK(hipMalloc(&wbuf, wsz));
            rocfft_execution_info_set_work_buffer(info, wbuf, wsz);
        }
        float2 *din, *dout;
        CK(hipMalloc(&din, sizeof(float2) * (size_t)FT * N));
        CK(hipMalloc(&dout, sizeof(float2) * (size_t)FT * N));
        CK(hipMemcpy(din, dx, sizeof(float2) * (size_t)FT * N < sizeof(float2) * S ? sizeof(float2) * (size_t)FT * N
                                                                                   : sizeof(float2) * S,
                     hipMemcpyDeviceToDevice));
        void* ib[1] = {din};
        void* ob[1] = {dout};
        const double us = time_us([&] { rocfft_execute(plan, ib, ob, info); }, 20, 100);
        const double bytes = 8.0 * FT * N;
        printf("rocfft batch=%d   %8.2f us  reads %.1f MB + writes %.1f MB: %.1f GB/s in+out; on the "
               "waterfall's algorithmic bytes %.1f %% of 8 TB/s (work buffer %zu B)\n",
               FT, us, bytes * 1e-6, bytes * 1e-6, 2 * bytes / us * 1e-3, alg_bytes / us * 1e-3 / 80.0, wsz);
        rocfft_plan_destroy(plan);
        rocfft_execution_info_destroy(info);
        rocfft_cleanup();
    }
    return 0;
}
