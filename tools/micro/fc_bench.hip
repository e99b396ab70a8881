// fc_mac microbenchmark (diagnostic; not part of the product): times the fast-convolution
// DDC's per-bin complex GEMM (kernels_fcddc.hip) on a C3-sized block for W layouts and load
// hints.  Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 fc_bench.hip -o fc_bench
#include "../../openwebrx_amd/csrc/kernels_fcddc.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

int main(int argc, char** argv) {
    const int C = argc > 1 ? atoi(argv[1]) : 256;
    const int M = argc > 2 ? atoi(argv[2]) : 256;
    const int F = argc > 3 ? atoi(argv[3]) : 22;
    const int D = argc > 4 ? atoi(argv[4]) : 833;
    const int Dp = (D + kFcDpAlign - 1) / kFcDpAlign * kFcDpAlign;
    const int Fs = (F + 15) & ~15;
    const size_t nu = (size_t)M * Fs * Dp, nw = (size_t)C * M * Dp, ny = (size_t)C * Fs * M;
    float2 *U, *W, *Y;
    hipMalloc(&U, nu * 8);
    hipMalloc(&W, nw * 8);
    hipMalloc(&Y, ny * 8);
    std::vector<float2> h(std::max(nu, nw));
    for (auto& v : h) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
    hipMemcpy(U, h.data(), nu * 8, hipMemcpyHostToDevice);
    hipMemcpy(W, h.data(), nw * 8, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const bool wide = F > 16;
    const int ctt = wide ? 4 : 8, ftt = wide ? 2 : 1;
    const int ncg = (C + 8 * ctt - 1) / (8 * ctt);
    const int nfg = (F + 16 * ftt - 1) / (16 * ftt);
    const dim3 gm(M * ncg * nfg);
    struct L {
        const char* name;
        int64_t cs, ks;
        bool nt;
    } ls[] = {{"[c][kap][r]      ", (int64_t)M * Dp, Dp, false},
              {"[c][kap][r]  nt  ", (int64_t)M * Dp, Dp, true},
              {"[kap][c][r]      ", Dp, (int64_t)C * Dp, false},
              {"[kap][c][r]  nt  ", Dp, (int64_t)C * Dp, true}};
    const double flop = 8.0 * M * Dp * C * ((F + 15) / 16 * 16);
    const double useful = 8.0 * M * Dp * C * F;
    for (int rep = 0; rep < 2; ++rep)
        for (const L& l : ls) {
            auto run = [&]() {
                if (wide) {
                    if (l.nt) hipLaunchKernelGGL((fc_mac<2, 4, true>), gm, dim3(64 * kFcKSplit), 0, 0, U, W, l.cs, l.ks, C, Fs, F, Dp, M, ncg, 1, Y);
                    else hipLaunchKernelGGL((fc_mac<2, 4, false>), gm, dim3(64 * kFcKSplit), 0, 0, U, W, l.cs, l.ks, C, Fs, F, Dp, M, ncg, 1, Y);
                } else {
                    if (l.nt) hipLaunchKernelGGL((fc_mac<1, 8, true>), gm, dim3(64 * kFcKSplit), 0, 0, U, W, l.cs, l.ks, C, Fs, F, Dp, M, ncg, 1, Y);
                    else hipLaunchKernelGGL((fc_mac<1, 8, false>), gm, dim3(64 * kFcKSplit), 0, 0, U, W, l.cs, l.ks, C, Fs, F, Dp, M, ncg, 1, Y);
                }
            };
            run();
            hipEventRecord(a);
            const int it = 20;
            for (int i = 0; i < it; ++i) run();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double us = ms * 1e3 / it;
            printf("C=%d M=%d F=%d D=%d %s %8.1f us  %6.1f TF (padded) %6.1f TF useful  W %6.0f GB/s\n", C, M,
                   F, D, l.name, us, flop / us / 1e6, useful / us / 1e6, nw * 8.0 / us / 1e3);
        }
    return 0;
}
