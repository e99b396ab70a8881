// Serial chain-tail kernels in isolation (diagnostic; not part of the product): times
// post_serial_front<ADPCM> and chain_adpcm from kernels_post.hip on C2-shaped inputs
// (32 chains x ~5000 samples, two demodulator runs padded to 64 lanes each).
#include "../../openwebrx_amd/csrc/kernels_post.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace owrx;

int main(int argc, char** argv) {
    const int C = argc > 1 ? atoi(argv[1]) : 32;
    const int n = argc > 2 ? atoi(argv[2]) : 5033;
    const int cap = n + 512;
    std::vector<ChainPost> hp(C);
    std::vector<int> sel;
    for (int dm = 0; dm < 2; ++dm) {
        int run = 0;
        for (int c = 0; c < C; ++c)
            if (c % 2 == dm) {
                sel.push_back(c);
                run++;
            }
        while (run % 64) {
            sel.push_back(-1);
            run++;
        }
    }
    std::vector<float> dem(cap);
    std::vector<ChainCounts> hc(C);
    ChainStateS* d_ss;
    hipMalloc(&d_ss, sizeof(ChainStateS) * C);
    std::vector<ChainStateS> hss(C);
    for (auto& s : hss) {
        memset(&s, 0, sizeof(s));
        s.agc.env = 0.8f / 1000.0f;
    }
    hipMemcpy(d_ss, hss.data(), sizeof(ChainStateS) * C, hipMemcpyHostToDevice);
    for (int c = 0; c < C; ++c) {
        ChainPost& p = hp[c];
        memset(&p, 0, sizeof(p));
        p.demod = c % 2;
        p.output = 1;
        p.deemph_alpha = 0.145f;
        p.deemph_beta = 1.0f - p.deemph_alpha;
        p.agc = AgcParams{0.8f, 0.1f, 0.001f, 65535.0f, 1000.0f, 0};
        p.sstate = d_ss + c;
        for (int i = 0; i < cap; ++i)
            dem[i] = 0.3f * sinf(0.05f * i * (1 + c % 7)) + 0.05f * ((rand() % 1000) / 1000.0f - 0.5f);
        hipMalloc(&p.dem, sizeof(float) * cap);
        hipMemcpy(p.dem, dem.data(), sizeof(float) * cap, hipMemcpyHostToDevice);
        hipMalloc(&p.s16, sizeof(int16_t) * cap);
        hipMemset(p.s16, 0, sizeof(int16_t) * cap);
        p.out_cap = 4 * cap;
        hipMalloc(&p.out, p.out_cap);
        hc[c].n_sq = n;
    }
    ChainPost* d_posts;
    ChainCounts* d_counts;
    int* d_sel;
    hipMalloc(&d_posts, sizeof(ChainPost) * C);
    hipMemcpy(d_posts, hp.data(), sizeof(ChainPost) * C, hipMemcpyHostToDevice);
    hipMalloc(&d_counts, sizeof(ChainCounts) * C);
    hipMemcpy(d_counts, hc.data(), sizeof(ChainCounts) * C, hipMemcpyHostToDevice);
    hipMalloc(&d_sel, sizeof(int) * sel.size());
    hipMemcpy(d_sel, sel.data(), sizeof(int) * sel.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    auto timeit = [&](const char* name, auto fn) {
        fn();
        hipDeviceSynchronize();
        const int iters = 10;
        hipEventRecord(e0);
        for (int i = 0; i < iters; ++i) fn();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= iters;
        printf("%-28s %8.1f us  %6.1f cycles/sample @%.1f GHz (%s)\n", name, ms * 1e3,
               ms * 1e-3 * clk * 1e3 / n, clk / 1e6, hipGetErrorString(hipGetLastError()));
    };
    const int nsel = (int)sel.size();
    timeit("post_serial_front<ADPCM>", [&] {
        launch_post_serial(d_posts, d_counts, d_sel, nsel, 1, 0, 0);
    });
    timeit("chain_adpcm", [&] { launch_chain_adpcm(d_posts, d_counts, d_sel, nsel, 0); });
    return 0;
}
