// Phase timing of the production waterfall FFT (diagnostic; not part of the product): builds the
// N = 16384 kernel launch_wf_fft selects (OWRX_WF_KERNEL) with OWRX_WF_STAMPS, runs it alone on C3's block geometry (10 Msps, N = 16384,
// hop 11454: 366 frames, G groups of F frames) and prints, over the workgroups, the median
// cycles (s_memtime) of each phase of wave 0: loads, the three radix-16 passes, the radix-4
// pass, and the kernel time from HIP events.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-slp-vectorize -I../../openwebrx_amd/csrc wf_stamp.hip -o wf_stamp
// Run:   ./wf_stamp [groups] [frames_per_group]
#define OWRX_WF_STAMPS
#include "../../openwebrx_amd/csrc/kernels_waterfall.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                                   \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

int main(int argc, char** argv) {
    constexpr int LOGN = 14, N = 1 << LOGN;
    const int hop = 11454;
    const int G = argc > 1 ? atoi(argv[1]) : 183;
    const int F = argc > 2 ? atoi(argv[2]) : 2;
    if (G < 1 || G > 1024 || F < 1 || F > 16) return 2;
    const int64_t S = (int64_t)G * F * hop + N;
    std::vector<float2> x(S);
    srand(1);
    for (auto& v : x) v = float2{rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f};
    std::vector<float> win(N);
    for (int i = 0; i < N; ++i) win[i] = (float)(0.54 - 0.46 * cos(2 * M_PI * i / (N - 1)));
    std::vector<float2> tw(N);
    for (int k = 0; k < N; ++k) tw[k] = float2{(float)cos(2 * M_PI * k / N), (float)-sin(2 * M_PI * k / N)};
    std::vector<WfGroup> grp(G);
    for (int g = 0; g < G; ++g) grp[g] = WfGroup{(int64_t)g * F * hop, F, hop};
    float2 *dx, *dtw;
    float *dwin, *dpart;
    WfGroup* dg;
    CK(hipMalloc(&dx, sizeof(float2) * S));
    CK(hipMalloc(&dtw, sizeof(float2) * N));
    CK(hipMalloc(&dwin, sizeof(float) * N));
    CK(hipMalloc(&dpart, sizeof(float) * (size_t)G * N));
    CK(hipMalloc(&dg, sizeof(WfGroup) * G));
    CK(hipMemcpy(dx, x.data(), sizeof(float2) * S, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtw, tw.data(), sizeof(float2) * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwin, win.data(), sizeof(float) * N, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, grp.data(), sizeof(WfGroup) * G, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int it = 0; it < 25; ++it) {
        CK(hipEventRecord(e0, 0));
        CK(launch_fft_sel<LOGN>(dx, 0, dg, G, dwin, dtw, dpart, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (it >= 5) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::vector<unsigned long long> st((size_t)1024 * 16);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_wf_stamp), sizeof(unsigned long long) * st.size()));
    printf("G=%d F=%d: kernel median %.2f us (min %.2f)\n", G, F, ms[ms.size() / 2] * 1e3, ms[0] * 1e3);
    const char* names[] = {"loads+window", "pass0 (dft16+store)", "pass1", "pass2", "pass3 (radix-4)"};
    auto med = [&](int a, int b) {
        std::vector<long long> d;
        for (int g = 0; g < G; ++g) d.push_back((long long)(st[g * 16 + b] - st[g * 16 + a]));
        std::sort(d.begin(), d.end());
        return d[d.size() / 2];
    };
    for (int f = 0; f < std::min(F, 2); ++f) {
        const int b = 1 + 6 * f;
        printf(" frame %d: start at %lld cycles\n", f, med(0, b));
        for (int p = 0; p < 5; ++p) printf("   %-22s %7lld cycles\n", names[p], med(b + p, b + p + 1));
    }
    printf(" total (start -> partial written) %lld cycles\n", med(0, 13));
    return 0;
}
