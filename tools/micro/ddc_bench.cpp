// DDC kernel variant microbenchmark (diagnostic; not part of the product).  Builds the real
// kernel template from kernels_ddc.hip and times tuning variants on a C2-sized block.
#include "../../openwebrx_amd/csrc/ddc_kernels.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

typedef hipError_t (*LaunchFn)(const float2*, int64_t, int64_t, const float*, const DdcChain*, int,
                               int, int64_t, int, int, float2*, hipStream_t);

struct Variant {
    const char* name;
    LaunchFn fn;
    int R;
    bool lds;
};

int main(int argc, char** argv) {
    const int C = argc > 1 ? atoi(argv[1]) : 32;
    const int D = 833, P = 27;
    const int64_t hist = 1 << 18, block = 1 << 22;
    std::vector<float2> h_in(hist + block);
    srand(1);
    for (auto& v : h_in)
        v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
    std::vector<float> taps((size_t)D * P);
    for (auto& t : taps) t = (rand() / (float)RAND_MAX - 0.5f) * 1e-3f;
    std::vector<DdcChain> ch(C);
    for (int c = 0; c < C; ++c) {
        const double rate = -0.4 + 0.8 * c / C;
        ch[c].rate_fx = (uint64_t)(int64_t)(rate * 9223372036854775808.0) * 2;
        const double a = 2 * M_PI * rate * D;
        ch[c].wD = make_float2((float)cos(a), (float)sin(a));
        ch[c].n0 = 0;
        ch[c].P0 = 0;
    }
    float2 *d_in, *d_part;
    float* d_taps;
    DdcChain* d_ch;
    hipMalloc(&d_in, sizeof(float2) * h_in.size());
    hipMemcpy(d_in, h_in.data(), sizeof(float2) * h_in.size(), hipMemcpyHostToDevice);
    hipMalloc(&d_taps, sizeof(float) * taps.size());
    hipMemcpy(d_taps, taps.data(), sizeof(float) * taps.size(), hipMemcpyHostToDevice);
    hipMalloc(&d_ch, sizeof(DdcChain) * C);
    hipMemcpy(d_ch, ch.data(), sizeof(DdcChain) * C, hipMemcpyHostToDevice);
    const int64_t blk_start = hist, blk_end = hist + block;
    const int T = D * (P - 1) + 1;
    const int64_t k_begin = 0;
    const int nk = (int)((blk_end - T) / D + 1);
    const size_t part_elems = (size_t)64 * C * nk;
    hipMalloc(&d_part, sizeof(float2) * part_elems);

    Variant vs[] = {
        {"flat R32 W2 SB16", launch_ddc_p<27, 32, 2, 16>, 32, false},
        {"lds R32 W2", launch_ddc_lds_p<27, 2>, 32, true},
        {"lds R32 W3", launch_ddc_lds_p<27, 3>, 32, true},
        {"lds R48 W2", launch_ddc_lds_p<27, 2, 48>, 48, true},
        {"lds R40 W3", launch_ddc_lds_p<27, 3, 40>, 40, true},
        {"lds R64 W2", launch_ddc_lds_p<27, 2, 64>, 64, true},
    };
    std::vector<float2> ref, out;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& v : vs) {
        int cpw = 1;
        while (cpw < C && cpw < 64) cpw <<= 1;
        const int tpw = 64 / cpw;
        const int ntg = ((nk + v.R - 1) / v.R + tpw - 1) / tpw;
        const int ncg = (C + cpw - 1) / cpw;
        const int base = ntg * ncg;
        int nseg = std::min(std::max(1, (1024 + base - 1) / base), std::max(1, D / 32));
        if (argc > 2) nseg = atoi(argv[2]);
        if (v.lds) {  // segments actually launched for the request
            const int len = ddc_seg_len(D, nseg);
            nseg = (D + len - 1) / len;
        } else {
            const int pps = (D + kDdcWaves * nseg - 1) / (kDdcWaves * nseg);
            nseg = ((D + pps - 1) / pps + kDdcWaves - 1) / kDdcWaves;
        }
        hipMemset(d_part, 0, sizeof(float2) * part_elems);
        v.fn(d_in + hist, blk_start, blk_end, d_taps, d_ch, C, D, k_begin, nk, nseg, d_part, 0);
        hipDeviceSynchronize();
        // reduce partials on the host for a cross-check against the first variant
        std::vector<float2> pp((size_t)nseg * C * nk);
        hipMemcpy(pp.data(), d_part, sizeof(float2) * pp.size(), hipMemcpyDeviceToHost);
        out.assign((size_t)C * nk, make_float2(0, 0));
        for (int sgi = 0; sgi < nseg; ++sgi)
            for (size_t i = 0; i < out.size(); ++i) {
                out[i].x += pp[(size_t)sgi * C * nk + i].x;
                out[i].y += pp[(size_t)sgi * C * nk + i].y;
            }
        double err = 0, nrm = 0;
        if (ref.empty()) ref = out;
        {   // where do the variants differ (diagnostic)
            double worst = 0;
            size_t wi = 0;
            long nbad = 0;
            for (size_t i = 0; i < out.size(); ++i) {
                const double d = hypot(out[i].x - ref[i].x, out[i].y - ref[i].y);
                const double m = hypot(ref[i].x, ref[i].y) + 1e-6;
                if (d > 1e-4 * m) nbad++;
                if (d > worst) { worst = d; wi = i; }
            }
            printf("   worst |diff| %.3e at chain %zu k %zu of %d (ref %.3e), %ld outputs off\n", worst,
                   wi / nk, wi % nk, nk, hypot(ref[wi].x, ref[wi].y), nbad);
        }
        for (size_t i = 0; i < out.size(); ++i) {
            err += pow(out[i].x - ref[i].x, 2) + pow(out[i].y - ref[i].y, 2);
            nrm += pow(ref[i].x, 2) + pow(ref[i].y, 2);
        }
        const int iters = 20;
        hipEventRecord(e0);
        for (int it = 0; it < iters; ++it)
            v.fn(d_in + hist, blk_start, blk_end, d_taps, d_ch, C, D, k_begin, nk, nseg, d_part, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= iters;
        const double flops = (double)C * nk * (4.0 * T + 6.0 * D);
        printf("%-18s nseg %3d  %8.1f us  %6.1f TFLOP/s  rel.err %.2e  (%s)\n", v.name, nseg,
               ms * 1e3, flops / (ms * 1e-3) / 1e12, sqrt(err / (nrm + 1e-30)),
               hipGetErrorString(hipGetLastError()));
    }
    return 0;
}
