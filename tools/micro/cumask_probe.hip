// Workgroup placement on CU-masked queues (diagnostic, not part of the product).
// Each workgroup records its hardware location (XCC, SE, CU) and its wall-clock start and end;
// the host reports how many workgroups ran at once and on how many distinct CUs, for a
// one-workgroup-per-CU shape (512 threads, 128 KiB LDS: wf_fft_l32's) and lighter ones, on an
// unmasked stream and on masked ones (240 of 256 CUs, as the engine's stream A).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 cumask_probe.hip -o cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <functional>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                                   \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

// per wave: the SIMD it runs on, and the clocks a fixed amount of VALU work took
__global__ void simds(unsigned* rec, float* sink, int iters) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const long long c0 = clock64();
    const unsigned long long w0 = wall_clock64();
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
#pragma unroll 1
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 32; ++k) a = fmaf(a, b, 1e-7f);
    }
    const long long c1 = clock64();
    const unsigned long long w1 = wall_clock64();
    if (a == 12345.f) sink[threadIdx.x] = a;
    const int wave = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) {
        rec[(blockIdx.x * 16 + wave) * 2 + 0] = (hw >> 4) & 3;
        rec[(blockIdx.x * 16 + wave) * 2 + 1] = (unsigned)(c1 - c0);
        rec[2 * 16 * 256 + blockIdx.x * 16 + wave] = (unsigned)(w1 - w0);
    }
}

// each workgroup streams its own `per` bytes (16 B loads) and records its wall time
__global__ void stream_rd(const float4* __restrict__ src, size_t per, unsigned* rec, float* sink) {
    const unsigned long long w0 = wall_clock64();
    const float4* p = src + blockIdx.x * (per / 16);
    float acc = 0.f;
    for (size_t i = threadIdx.x; i < per / 16; i += blockDim.x * 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i + u * blockDim.x < per / 16 ? p[i + u * blockDim.x] : float4{};
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    __syncthreads();
    if (acc == 1234.5f) sink[threadIdx.x] = acc;
    if (threadIdx.x == 0) rec[blockIdx.x] = (unsigned)(wall_clock64() - w0);
}

// rec[4 b + 0..3] = start, end (100 MHz ticks), HW_ID, XCC_ID
__global__ void probe(unsigned long long* rec, int spin_ticks) {
    extern __shared__ float lds[];
    lds[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    const unsigned long long t0 = wall_clock64();
    while ((long long)(wall_clock64() - t0) < spin_ticks) __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        rec[4 * blockIdx.x + 0] = t0;
        rec[4 * blockIdx.x + 1] = wall_clock64();
        rec[4 * blockIdx.x + 2] = hw + lds[1];
        rec[4 * blockIdx.x + 3] = xcc;
    }
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int words = (ncu + 31) / 32;
    std::vector<uint32_t> all(words, 0), lo(words, 0), hi(words, 0), every(words, 0), half(words, 0);
    for (int c = 0; c < ncu; ++c) {
        all[c / 32] |= 1u << (c % 32);
        if (c < ncu - 16) lo[c / 32] |= 1u << (c % 32);
        if (c >= 16) hi[c / 32] |= 1u << (c % 32);
        if (c % 16 != 15) every[c / 32] |= 1u << (c % 32);
        if (c < ncu / 2) half[c / 32] |= 1u << (c % 32);
    }
    struct S {
        const char* name;
        hipStream_t s;
    };
    std::vector<S> streams(6);
    streams[0].name = "plain";
    CK(hipStreamCreateWithFlags(&streams[0].s, hipStreamNonBlocking));
    streams[1].name = "mask-all";
    CK(hipExtStreamCreateWithCUMask(&streams[1].s, words, all.data()));
    streams[2].name = "mask[0,240)";
    CK(hipExtStreamCreateWithCUMask(&streams[2].s, words, lo.data()));
    streams[3].name = "mask[16,256)";
    CK(hipExtStreamCreateWithCUMask(&streams[3].s, words, hi.data()));
    streams[4].name = "mask-every16";
    CK(hipExtStreamCreateWithCUMask(&streams[4].s, words, every.data()));
    streams[5].name = "mask[0,128)";
    CK(hipExtStreamCreateWithCUMask(&streams[5].s, words, half.data()));
    CK(hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int maxg = 1024;
    unsigned long long* d = nullptr;
    CK(hipMalloc(&d, sizeof(unsigned long long) * 4 * maxg));
    std::vector<unsigned long long> h(4 * maxg);
    struct Shape {
        int threads, lds_kb, grid;
    };
    const Shape shapes[] = {{512, 128, 240}, {512, 128, 256}, {512, 64, 480}, {256, 16, 240},
                            {64, 0, 240}, {1024, 0, 240}};
    printf("CUs %d; spin 20 us per workgroup\n", ncu);
    for (const Shape& sh : shapes) {
        for (const S& st : streams) {
            // one warm launch, then the recorded one
            for (int it = 0; it < 2; ++it) {
                hipLaunchKernelGGL(probe, dim3(sh.grid), dim3(sh.threads), (size_t)sh.lds_kb * 1024 + 4096, st.s, d, 2000);
                CK(hipGetLastError());
                CK(hipStreamSynchronize(st.s));
            }
            CK(hipMemcpy(h.data(), d, sizeof(unsigned long long) * 4 * sh.grid, hipMemcpyDeviceToHost));
            unsigned long long t_min = ~0ull, t_max = 0;
            std::vector<std::pair<unsigned long long, int>> ev;
            std::set<std::tuple<int, int, int>> cus;
            std::set<int> xccs, ses;
            for (int b = 0; b < sh.grid; ++b) {
                const unsigned long long s0 = h[4 * b], s1 = h[4 * b + 1];
                const unsigned hw = (unsigned)h[4 * b + 2];
                const int xcc = (int)(h[4 * b + 3] & 0xf), se = (hw >> 13) & 7, cu = (hw >> 8) & 31;
                cus.insert({xcc, se, cu});
                xccs.insert(xcc);
                ses.insert(xcc * 8 + se);
                t_min = std::min(t_min, s0);
                t_max = std::max(t_max, s1);
                ev.push_back({s0, +1});
                ev.push_back({s1, -1});
            }
            std::sort(ev.begin(), ev.end(), [](auto& a, auto& b) {
                return a.first != b.first ? a.first < b.first : a.second < b.second;
            });
            int cur = 0, peak = 0;
            for (auto& e : ev) peak = std::max(peak, cur += e.second);
            // start-time spread: how many waves of workgroups the dispatch took
            std::vector<unsigned long long> st0;
            for (int b = 0; b < sh.grid; ++b) st0.push_back(h[4 * b] - t_min);
            std::sort(st0.begin(), st0.end());
            printf("%4d thr %3d KiB grid %3d %-13s span %6.1f us  peak concurrent %3d  distinct CUs %3d"
                   "  XCDs %d SEs %2d  start p50 %5.1f p90 %5.1f max %5.1f us\n",
                   sh.threads, sh.lds_kb, sh.grid, st.name, (t_max - t_min) / 100.0, peak,
                   (int)cus.size(), (int)xccs.size(), (int)ses.size(), st0[st0.size() / 2] / 100.0,
                   st0[st0.size() * 9 / 10] / 100.0, st0.back() / 100.0);
        }
    }
    // waves per SIMD within a 512-thread workgroup (128 KiB LDS), and a fixed VALU loop's clocks
    {
        CK(hipFuncSetAttribute((const void*)simds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        unsigned* dr = nullptr;
        float* sink = nullptr;
        CK(hipMalloc(&dr, sizeof(unsigned) * 3 * 16 * 256));
        CK(hipMalloc(&sink, 4096));
        std::vector<unsigned> hr(3 * 16 * 256);
        for (const S& st : streams) {
            for (int it = 0; it < 2; ++it) {
                hipLaunchKernelGGL(simds, dim3(240), dim3(512), (size_t)128 * 1024, st.s, dr, sink, 2000);
                CK(hipGetLastError());
                CK(hipStreamSynchronize(st.s));
            }
            CK(hipMemcpy(hr.data(), dr, sizeof(unsigned) * 3 * 16 * 256, hipMemcpyDeviceToHost));
            int hist[9] = {0};  // workgroups by their busiest SIMD's wave count
            double clk = 0, wall = 0;
            unsigned clk_max = 0;
            for (int b = 0; b < 240; ++b) {
                int per[4] = {0};
                for (int w = 0; w < 8; ++w) {
                    per[hr[(b * 16 + w) * 2] & 3]++;
                    clk += hr[(b * 16 + w) * 2 + 1];
                    wall += hr[2 * 16 * 256 + b * 16 + w];
                    clk_max = std::max(clk_max, hr[(b * 16 + w) * 2 + 1]);
                }
                hist[*std::max_element(per, per + 4)]++;
            }
            printf("simds %-13s workgroups by max waves on one SIMD: 2:%d 3:%d 4:%d 5+:%d  "
                   "VALU loop clocks mean %.0f max %u, wall %.1f us -> %.0f MHz\n", st.name, hist[2], hist[3], hist[4],
                   hist[5] + hist[6] + hist[7] + hist[8], clk / (240 * 8), clk_max, wall / (240 * 8) / 100.0,
                   clk / wall * 100.0);
        }
    }
    // event-timed launches: an empty kernel, a 4-byte memset, and the 20 us probe at grids that
    // fit one round (200) or not (240), with 128 KiB LDS
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        int* dw = nullptr;
        CK(hipMalloc(&dw, 64));
        for (const S& st : streams) {
            auto timed = [&](const std::function<void()>& f) {
                float best = 1e9, sum = 0;
                for (int it = 0; it < 12; ++it) {
                    (void)hipEventRecord(e0, st.s);
                    f();
                    (void)hipEventRecord(e1, st.s);
                    (void)hipStreamSynchronize(st.s);
                    float ms = 0;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    if (it >= 2) {
                        best = std::min(best, ms);
                        sum += ms;
                    }
                }
                return std::make_pair(best * 1e3, sum / 10 * 1e3);
            };
            auto a = timed([&] { hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, st.s, d, 0); });
            auto b = timed([&] { (void)hipMemsetAsync(dw, 0, 4, st.s); });
            auto c = timed([&] { hipLaunchKernelGGL(probe, dim3(200), dim3(512), (size_t)132 * 1024, st.s, d, 2000); });
            auto e = timed([&] { hipLaunchKernelGGL(probe, dim3(240), dim3(512), (size_t)132 * 1024, st.s, d, 2000); });
            auto g = timed([&] { hipLaunchKernelGGL(probe, dim3(240), dim3(512), (size_t)16 * 1024, st.s, d, 2000); });
            printf("events %-13s empty %.1f/%.1f  memset4 %.1f/%.1f  probe200x132K %.1f/%.1f  probe240x132K %.1f/%.1f  probe240x16K %.1f/%.1f us (best/mean)\n",
                   st.name, a.first, a.second, b.first, b.second, c.first, c.second, e.first, e.second, g.first, g.second);
        }
    }
    // HBM streaming: 240 workgroups x 2 MiB each, per queue
    {
        const size_t per = 2u << 20;
        float4* src = nullptr;
        float* sink = nullptr;
        unsigned* dr = nullptr;
        CK(hipMalloc(&src, per * 256));
        CK(hipMemset(src, 0, per * 256));
        CK(hipMalloc(&sink, 4096));
        CK(hipMalloc(&dr, 4 * 256));
        void* flush = nullptr;
        CK(hipMalloc(&flush, 512u << 20));
        std::vector<unsigned> hr(256);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (const S& st : streams) {
            float best = 1e9;
            double wsum = 0;
            for (int it = 0; it < 4; ++it) {
                CK(hipMemsetAsync(flush, it, 512u << 20, st.s));
                CK(hipEventRecord(e0, st.s));
                hipLaunchKernelGGL(stream_rd, dim3(240), dim3(512), 0, st.s, src, per, dr, sink);
                CK(hipEventRecord(e1, st.s));
                CK(hipStreamSynchronize(st.s));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it && ms < best) {
                    best = ms;
                    CK(hipMemcpy(hr.data(), dr, 4 * 240, hipMemcpyDeviceToHost));
                    wsum = 0;
                    for (int b = 0; b < 240; ++b) wsum += hr[b];
                }
            }
            printf("stream %-13s 240 x 2 MiB: %7.1f us  %6.0f GB/s  per-workgroup mean %.1f us\n",
                   st.name, best * 1e3, 240.0 * per / (best * 1e-3) / 1e9, wsum / 240 / 100.0);
        }
    }
    return 0;
}
