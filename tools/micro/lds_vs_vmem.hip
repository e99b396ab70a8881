// Probe (diagnostic): how long do LDS stores / loads take to issue while the wave has global
// loads in flight?  Every CU runs one 1024-thread workgroup; each wave issues K 8-B (or 16-B)
// buffer loads of a large HBM buffer (distinct addresses per workgroup), then 16 ds_write_b64
// (or ds_read_b64) of registers unrelated to the loads, then waits for the loads.  Stamps (s_memtime)
// before the LDS ops, after them (issue) and after lgkmcnt(0) (done), per wave; median printed.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 lds_vs_vmem.hip -o lds_vs_vmem
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__device__ unsigned long long g_st[512][16][4];

// MODE 0: ds_write_b64; 1: ds_read_b64; 2: VALU only (16 x 8 FMAs); 3: ds_write, loads via LDS-DMA
template <int K, int W16, int MODE>
__global__ void __launch_bounds__(1024) probe(const float* __restrict__ src, float* __restrict__ sink, int stride) {
    extern __shared__ float2 lds[];
    const int t = threadIdx.x;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src + (size_t)blockIdx.x * stride), 0,
                                                      0x7fffffff, 0x00020000);
    float2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = make_float2((float)(t + i), (float)(t - i));
    float acc = 0.f;
    float2 ld[K > 0 ? K : 1];
    __syncthreads();
    const unsigned long long t0 = clock64();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (W16)
            ld[k].x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, t * 16, k * 16384, 0)) +
                      __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, t * 16 + 4, k * 16384, 0)) +
                      __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, t * 16 + 8, k * 16384, 0)) +
                      __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, t * 16 + 12, k * 16384, 0));
        else
            ld[k].x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, t * 8, k * 8192, 0)) +
                      __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, t * 8 + 4, k * 8192, 0));
    }
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = clock64();
    __builtin_amdgcn_sched_barrier(0);
    if (MODE == 0) {
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[i * 1024 + t] = v[i];
    } else if (MODE == 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = lds[i * 1024 + (t ^ i)];
    } else {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i].x = fmaf(v[i].x, v[i].y, v[i].x);
    }
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t2 = clock64();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t3 = clock64();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t4 = clock64();
#pragma unroll
    for (int k = 0; k < K; ++k) acc += ld[k].x;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += v[i].x + v[i].y;
    if ((t & 63) == 0 && blockIdx.x < 512) {
        g_st[blockIdx.x][t >> 6][0] = t1 - t0;
        g_st[blockIdx.x][t >> 6][1] = t2 - t1;
        g_st[blockIdx.x][t >> 6][2] = t3 - t1;
        g_st[blockIdx.x][t >> 6][3] = t4 - t1;
    }
    if (acc == 1234.5f) sink[t] = acc;
}

template <int K, int W16, int MODE>
static int run(const char* nm, const float* src, float* sink, int ncu) {
    CK(hipFuncSetAttribute((const void*)probe<K, W16, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    for (int it = 0; it < 3; ++it) {
        hipLaunchKernelGGL((probe<K, W16, MODE>), dim3(ncu), dim3(1024), 131072, 0, src, sink, 1 << 20);
        CK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> st((size_t)512 * 16 * 4);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_st), sizeof(unsigned long long) * st.size()));
    printf("%-34s", nm);
    const char* col[] = {"load issue", "op issue", "op done", "loads done"};
    for (int c = 0; c < 4; ++c) {
        std::vector<unsigned long long> v;
        for (int b = 0; b < ncu; ++b)
            for (int w = 0; w < 16; ++w) v.push_back(st[((size_t)b * 16 + w) * 4 + c]);
        std::sort(v.begin(), v.end());
        printf("  %s p50 %6llu p90 %6llu", col[c], v[v.size() / 2], v[v.size() * 9 / 10]);
    }
    printf("\n");
    return 0;
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    float *src, *sink;
    CK(hipMalloc(&src, (size_t)ncu * (4 << 20) + (64 << 20)));
    CK(hipMemset(src, 0, (size_t)ncu * (4 << 20) + (64 << 20)));
    CK(hipMalloc(&sink, 4096 * 4));
    printf("%d CUs, one 1024-thread workgroup each; cycles per wave (median / p90 over waves)\n", ncu);
    run<0, 0, 0>("ds_write x16, no loads", src, sink, ncu);
    run<4, 0, 0>("ds_write x16 after 4 8-B loads", src, sink, ncu);
    run<16, 0, 0>("ds_write x16 after 16 8-B loads", src, sink, ncu);
    run<8, 1, 0>("ds_write x16 after 8 16-B loads", src, sink, ncu);
    run<0, 0, 1>("ds_read x16, no loads", src, sink, ncu);
    run<16, 0, 1>("ds_read x16 after 16 8-B loads", src, sink, ncu);
    run<0, 0, 2>("VALU 128, no loads", src, sink, ncu);
    run<16, 0, 2>("VALU 128 after 16 8-B loads", src, sink, ncu);
    return 0;
}
