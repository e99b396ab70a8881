// wf_finalize in isolation, round 6 (diagnostic, not product): C3's batched launch (3 424 frames
// in 428 groups of 8, 35 rows of ~12 groups, 16384 bins, ADPCM rows), the partial rows written by
// a kernel just before (as the FFT leaves them).  Prints us per launch.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt
//        -fno-slp-vectorize wf_fin_r06.cpp.hip -o wf_fin_r06
#include "../../openwebrx_amd/csrc/kernels_waterfall.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace owrx;

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

__global__ void fill_partials(float* p, size_t n, float seed) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = 1e-6f + (float)((i * 2654435761u) & 1023) * seed;
}

int main() {
    const int N = 16384, G = 428, R = 35;
    float *partial, *cin, *cout;
    int16_t* s16;
    WfRow* rows;
    WfGroup* groups;
    CK(hipMalloc(&partial, sizeof(float) * (size_t)G * N));
    CK(hipMalloc(&cin, sizeof(float) * N));
    CK(hipMalloc(&cout, sizeof(float) * N));
    CK(hipMalloc(&s16, sizeof(int16_t) * (size_t)R * N));
    CK(hipMemset(cin, 0, sizeof(float) * N));
    std::vector<WfRow> hr(R);
    int g = 0;
    for (int r = 0; r < R; ++r) {
        const int ng = (r % 4 == 0) ? 13 : 12;
        hr[r] = WfRow{g, std::min(ng, G - g), r == 0, r + 1 < R, r, 0};
        g += hr[r].ngroups;
    }
    std::vector<WfGroup> hg(G);
    for (int i = 0; i < G; ++i) hg[i] = WfGroup{};
    for (int i = 0; i < G; ++i) hg[i].nframes = 8;
    CK(hipMalloc(&rows, sizeof(WfRow) * R));
    CK(hipMalloc(&groups, sizeof(WfGroup) * G));
    CK(hipMemcpy(rows, hr.data(), sizeof(WfRow) * R, hipMemcpyHostToDevice));
    CK(hipMemcpy(groups, hg.data(), sizeof(WfGroup) * G, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int pass = 0; pass < 2; ++pass) {
        double tot = 0;
        const int reps = 20;
        for (int it = 0; it < reps; ++it) {
            hipLaunchKernelGGL(fill_partials, dim3(2048), dim3(256), 0, 0, partial, (size_t)G * N, 1e-3f);
            CK(hipEventRecord(a, 0));
            CK(launch_wf_finalize(partial, rows, R, cin, cout, N, -70.f, 1, s16, nullptr, 0, groups, G, 0));
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            tot += ms;
        }
        printf("wf_finalize: %d rows, %d groups: %.2f us per launch (%.2f GB/s on the partials)\n", R, G,
               1e3 * tot / reps, (double)G * N * 4 / (tot / reps * 1e-3) / 1e9);
    }
    return 0;
}
