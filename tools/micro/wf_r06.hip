// Waterfall FFT in isolation, round 6 (diagnostic, not product): wf_fft_q16 variants at C3's
// production launch (10 Msps, N = 16384, hop 11454, groups of 8 frames, FT frames per launch on
// 228 CU-masked CUs, frames from HBM), the packed-FP32 (ABL 256) and wave-uniform-twiddle (512)
// forms against the production one (72), each also as a VALU-only ablation (| 7).  Prints us per
// launch, the rate on the algorithmic bytes (frames x hop x 8 B) and the partial rows' difference
// from wf_fft_r16<14>.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-slp-vectorize wf_r06.hip -o wf_r06
// Run:   ./wf_r06 [FT ...]
#include "../../openwebrx_amd/csrc/kernels_waterfall.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
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
    const int iters = 20;
    std::vector<float> t;
    for (int i = 0; i < iters + 3; ++i) {
        hipLaunchKernelGGL(flush_read, dim3(4096), dim3(256), 0, stream, (const float4*)g_flush, fb / 16,
                           (float*)g_flush);
        CK(hipEventRecord(e0, stream));
        launch();
        CK(hipEventRecord(e1, stream));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (i >= 3) t.push_back(ms * 1e3f);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

#define Q16_VARIANTS(X) X(72) X(79) X(328) X(335) X(584) X(591) X(840) X(847)

int main(int argc, char** argv) {
    const int hop = 11454;
    std::vector<int> fts;
    for (int i = 1; i < argc; ++i) fts.push_back(atoi(argv[i]));
    if (fts.empty()) fts = {3480};
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
    CK(hipMalloc(&dpart, sizeof(float) * (size_t)FTmax * N));
    CK(hipMalloc(&dg, sizeof(WfGroup) * FTmax));
    int* dwork;
    CK(hipMalloc(&dwork, 64));
    CK(hipMemset(dwork, 0, 64));
    CK(hipMemcpy(dx, x.data(), sizeof(float2) * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtw, tw.data(), sizeof(float2) * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwin, win.data(), sizeof(float) * N, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void*)wf_fft_r16<14>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)WfR16<14>::kLds));
#define SETQ(v) CK(hipFuncSetAttribute((const void*)wf_fft_q16<v>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WfQ16::kLds));
    Q16_VARIANTS(SETQ)
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
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
        const double alg = 8.0 * (double)FT * hop;
        const int F = 8;
        const int G = (FT + F - 1) / F;
        std::vector<WfGroup> grp(G);
        for (int g = 0; g < G; ++g) grp[g] = WfGroup{(int64_t)g * F * hop, std::min(F, FT - g * F), hop};
        CK(hipMemcpy(dg, grp.data(), sizeof(WfGroup) * grp.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(wf_fft_r16<14>, dim3(G), dim3(WfR16<14>::NT), WfR16<14>::kLds, 0, dx, (int64_t)0, dg,
                           dwin, dtw, dref);
        CK(hipDeviceSynchronize());
        std::vector<float> a((size_t)G * N), b((size_t)G * N);
        CK(hipMemcpy(a.data(), dref, sizeof(float) * a.size(), hipMemcpyDeviceToHost));
        auto q16 = [&](int abl) {
            decltype(&wf_fft_q16<0>) k = nullptr;
#define CASEQ(v) \
    if (abl == v) k = wf_fft_q16<v>;
            Q16_VARIANTS(CASEQ)
            hipLaunchKernelGGL(k, dim3(std::min(G, cus)), dim3(WfQ16::NT), WfQ16::kLds, s_a, dx, (int64_t)0, dg,
                               dwin, dtw, dpart, G, dwork, G, 0, 0, 0);
        };
        for (int abl : {72, 328, 584, 840, 79, 335, 591, 847}) {
            const double us = time_us([&] { q16(abl); }, s_a);
            printf("FT=%5d F=%d G=%4d q16<%3d>%s%s%s %8.2f us  %7.1f GB/s  %5.3f of 8 TB/s", FT, F, G, abl,
                   (abl & 256) ? " packed" : "       ", (abl & 512) ? " tbS" : "    ", (abl & 7) == 7 ? " valu" : "     ",
                   us, alg / us * 1e-3, alg / us * 1e-3 / 8000.0);
            if ((abl & 7) == 0) {
                CK(hipMemset(dpart, 0, sizeof(float) * (size_t)G * N));
                q16(abl);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(b.data(), dpart, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
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
    }
    return 0;
}
