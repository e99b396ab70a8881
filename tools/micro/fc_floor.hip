// fc_mac against the memory floor of its own access pattern, HBM-resident (diagnostic; not part
// of the product).  C3's geometry at 2^20-sample blocks (C = 256, M = 128, F = 13, D = 833), W in
// the engine's layout W[kappa][slot][Dp]; a 512 MiB read kernel between launches so W comes
// from HBM, as in the engine.  Times: fc_mac<1, 8> (production), the same grid and per-lane loads
// with the MFMAs replaced by adds (its load floor), and a fully coalesced stream of W's bytes.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 fc_floor.hip -o fc_floor
#include "../../openwebrx_amd/csrc/kernels_fcddc.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace owrx;

__global__ void flush_read(const float4* __restrict__ p, size_t n, float* sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;
}

// fc_mac<1, 8>'s workgroup decode and per-lane loads (U: one float4, W: 8 float4 per K-block,
// three K-blocks in flight per wave), summed instead of multiplied
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
fc_loads(const float2* __restrict__ U, const float2* __restrict__ W, int64_t w_cs, int64_t w_ks,
         int nchains, int Fs, int F, int Dp, int M, int ncg, float* __restrict__ out) {
    const int w = blockIdx.x, xcd = w & 7, q = w >> 3, mper = M >> 3;
    const int cg = q % ncg, r1 = q / ncg, kap = xcd * mper + r1 % mper;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15, cc = col >> 1;
    const int nkb = (Dp >> 3) / kFcKSplit, kb0 = wave * nkb;
    const int f = col;
    const gf4* up = (const gf4*)(U + ((int64_t)kap * Fs + (f < F ? f : 0)) * Dp + 8 * kb0 + 2 * g);
    const gf4* wp[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const int c = cg * 64 + t * 8 + cc;
        wp[t] = (const gf4*)(W + (c < nchains ? c : 0) * w_cs + (int64_t)kap * w_ks + 8 * kb0 + 2 * g);
    }
    fc_f4 acc = {0, 0, 0, 0};
    for (int kb = 0; kb < nkb; kb += 3) {
        fc_f4 v[3][9];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int o = (kb + j < nkb ? kb + j : nkb - 1) * 4;
            v[j][8] = up[o];
#pragma unroll
            for (int t = 0; t < 8; ++t) v[j][t] = wp[t][o];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) acc += v[j][t];
    }
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

// the same loads from W tiled as [kappa][chain / 8][K-block][chain % 8][8 branches]: a wave's
// load instruction reads 512 contiguous bytes, K-blocks follow each other
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
fc_loads_tiled(const float2* __restrict__ U, const float2* __restrict__ W, int64_t w_ks,
               int nchains, int Fs, int F, int Dp, int M, int ncg, float* __restrict__ out) {
    const int w = blockIdx.x, xcd = w & 7, q = w >> 3, mper = M >> 3;
    const int cg = q % ncg, r1 = q / ncg, kap = xcd * mper + r1 % mper;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, g = lane >> 4, col = lane & 15, cc = col >> 1;
    const int nkb = (Dp >> 3) / kFcKSplit, kb0 = wave * nkb;
    const int f = col;
    const gf4* up = (const gf4*)(U + ((int64_t)kap * Fs + (f < F ? f : 0)) * Dp + 8 * kb0 + 2 * g);
    const gf4* wp[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        int c = cg * 64 + t * 8 + cc;
        c = c < nchains ? c : 0;
        wp[t] = (const gf4*)(W + (int64_t)kap * w_ks + (int64_t)(c >> 3) * 8 * Dp + kb0 * 64 + (c & 7) * 8 + 2 * g);
    }
    fc_f4 acc = {0, 0, 0, 0};
    for (int kb = 0; kb < nkb; kb += 3) {
        fc_f4 v[3][9];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int kk = kb + j < nkb ? kb + j : nkb - 1;
            v[j][8] = up[kk * 4];
#pragma unroll
            for (int t = 0; t < 8; ++t) v[j][t] = wp[t][kk * 32];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) acc += v[j][t];
    }
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

__global__ void stream_read(const float4* __restrict__ p, size_t n, float* out) {
    float4 a = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = a.x + a.y + a.z + a.w;
}

int main() {
    const int C = 256, M = 128, F = 13, D = 833;
    const int Dp = (D + kFcDpAlign - 1) / kFcDpAlign * kFcDpAlign, Fs = 16;
    const size_t nu = (size_t)M * Fs * Dp, nw = (size_t)C * M * Dp, ny = (size_t)C * Fs * M;
    float2 *U, *W, *Y;
    float* out;
    void* fl;
    const size_t fb = (size_t)512 << 20;
    hipMalloc(&U, nu * 8);
    hipMalloc(&W, nw * 8);
    hipMalloc(&Y, ny * 8);
    hipMalloc(&out, (size_t)M * 4 * 256 * 4 + (1 << 22));
    hipMalloc(&fl, fb);
    hipMemset(fl, 0, fb);
    std::vector<float2> h(std::max(nu, nw));
    for (auto& v : h) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
    hipMemcpy(U, h.data(), nu * 8, hipMemcpyHostToDevice);
    hipMemcpy(W, h.data(), nw * 8, hipMemcpyHostToDevice);
    const int ncg = C / 64;
    const dim3 gm(M * ncg);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timed = [&](auto&& launch) {
        double tot = 0;
        for (int i = 0; i < 23; ++i) {
            hipLaunchKernelGGL(flush_read, dim3(4096), dim3(256), 0, 0, (const float4*)fl, fb / 16, out);
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (i >= 3) tot += ms;
        }
        return tot * 1e3 / 20;
    };
    const double wb = nw * 8.0;
    {  // LDS-ring variants: Y identical to fc_mac<1, 8>
        std::vector<float2> y0(ny), y1(ny);
        hipMemset(Y, 0, ny * 8);
        hipLaunchKernelGGL((fc_mac<1, 8, false>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        hipMemcpy(y0.data(), Y, ny * 8, hipMemcpyDeviceToHost);
        auto cmp = [&](const char* name) {
            hipMemcpy(y1.data(), Y, ny * 8, hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (int c = 0; c < C; ++c)
                for (int f = 0; f < F; ++f)
                    for (int k = 0; k < M; ++k) {
                        const size_t i = ((size_t)c * Fs + f) * M + k;
                        bad += memcmp(&y0[i], &y1[i], 8) != 0;
                    }
            printf("%s: %zu of %d outputs differ from fc_mac<1,8>\n", name, bad, C * F * M);
        };
        hipMemset(Y, 0, ny * 8);
        hipLaunchKernelGGL((fc_mac_lds<1, 8, 2>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        cmp("fc_mac_lds<1,8,2>");
        hipMemset(Y, 0, ny * 8);
        hipLaunchKernelGGL((fc_mac_lds<1, 8, 3>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        cmp("fc_mac_lds<1,8,3>");
        hipMemset(Y, 0, ny * 8);
        hipLaunchKernelGGL((fc_mac_lds<1, 8, 4>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        cmp("fc_mac_lds<1,8,4>");
    }
    for (int rep = 0; rep < 2; ++rep) {
        double us;
        us = timed([&] {
            hipLaunchKernelGGL((fc_mac_lds<1, 8, 2>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        });
        printf("fc_mac_lds NR=2  %7.1f us  W %6.0f GB/s (%.3f of 8 TB/s)\n", us, wb / us / 1e3, wb / us / 8e6);
        us = timed([&] {
            hipLaunchKernelGGL((fc_mac_lds<1, 8, 3>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        });
        printf("fc_mac_lds NR=3  %7.1f us  W %6.0f GB/s (%.3f of 8 TB/s)\n", us, wb / us / 1e3, wb / us / 8e6);
        us = timed([&] {
            hipLaunchKernelGGL((fc_mac_lds<1, 8, 4>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        });
        printf("fc_mac_lds NR=4  %7.1f us  W %6.0f GB/s (%.3f of 8 TB/s)\n", us, wb / us / 1e3, wb / us / 8e6);

        us = timed([&] {
            hipLaunchKernelGGL((fc_mac<1, 8, false>), gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, 1, Y);
        });
        printf("fc_mac<1,8>      %7.1f us  W %6.0f GB/s (%.3f of 8 TB/s)\n", us, wb / us / 1e3, wb / us / 8e6);
        us = timed([&] {
            hipLaunchKernelGGL(fc_loads, gm, dim3(256), 0, 0, U, W, (int64_t)Dp, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, out);
        });
        printf("its loads alone  %7.1f us  W %6.0f GB/s (%.3f of 8 TB/s)\n", us, wb / us / 1e3, wb / us / 8e6);
        us = timed([&] {
            hipLaunchKernelGGL(fc_loads_tiled, gm, dim3(256), 0, 0, U, W, (int64_t)C * Dp, C, Fs, F, Dp, M, ncg, out);
        });
        printf("loads, W tiled   %7.1f us  W %6.0f GB/s (%.3f of 8 TB/s)\n", us, wb / us / 1e3, wb / us / 8e6);
        us = timed([&] {
            hipLaunchKernelGGL(stream_read, dim3(4096), dim3(256), 0, 0, (const float4*)W, nw / 2, out);
        });
        printf("W streamed       %7.1f us  W %6.0f GB/s (%.3f of 8 TB/s)\n", us, wb / us / 1e3, wb / us / 8e6);
    }
    return 0;
}
