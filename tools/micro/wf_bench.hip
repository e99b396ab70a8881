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

template <typename F>
static double time_us(F&& launch, int warm = 50, int iters = 200) {
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
        const int nwg = frame_table(F);
        report("h32", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_fft_h32, dim3(nwg), dim3(WfH32::NT), WfH32::kLds, 0, dx, (int64_t)0, dfr,
                                      dwin, dtw, dmember, dtick, dpart2);
               }));
        report("mem", G, F, time_us([&] {
                   hipLaunchKernelGGL(wf_mem_only<LOGN>, dim3(G), dim3(1024), 0, 0, dx, dg, dwin, dpart2);
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
