// Single-wave issue / latency microbenchmark (diagnostic; not part of the product): cycles per
// instruction for one 64-lane wave alone on a CU -- a dependent v_add chain, four independent
// v_add chains interleaved, a v_cmp -> v_cndmask chain, an LDS pointer chase (ds_read_b32),
// and an LDS chase through ds_read_b128.  Sizes the IMA-ADPCM encoder's per-sample budget.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 issue_r05.cpp -o issue_r05
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIt = 4096;

template <int V>
__global__ void __launch_bounds__(64) kern(int seed, int* out, long long* cyc) {
    __shared__ __align__(16) int L[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) L[i] = ((i * 97 + 13) & 1023) * 4;  // chase links
    __syncthreads();
    int a = seed + threadIdx.x, b = a * 3, c = a * 5, d = a * 7;
    const long long t0 = clock64();
    if constexpr (V == 0) {  // dependent v_add_u32 chain: 8 per iteration
        for (int i = 0; i < kIt; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
        }
    } else if constexpr (V == 1) {  // four independent chains interleaved: 8 per iteration
        for (int i = 0; i < kIt; ++i) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(c) : "v"(b));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(d) : "v"(b));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(b) : "v"(a));
            }
        }
    } else if constexpr (V == 2) {  // v_cmp -> v_cndmask dependent pairs: 8 instructions per it
        for (int i = 0; i < kIt; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                asm volatile(
                    "v_cmp_lt_i32 vcc, %0, %1\n\t"
                    "v_cndmask_b32 %0, %1, %0, vcc"
                    : "+v"(a)
                    : "v"(b)
                    : "vcc");
        }
    } else if constexpr (V == 3) {  // LDS chase, ds_read_b32 (address = loaded value)
        int p = (threadIdx.x * 4) & 4095;
        for (int i = 0; i < kIt; ++i) p = *reinterpret_cast<const int*>(reinterpret_cast<const char*>(L) + p);
        a = p;
    } else if constexpr (V == 4) {  // LDS chase through ds_read_b128 (first word = next address)
        int p = (threadIdx.x * 16) & 4095;
        for (int i = 0; i < kIt; ++i) {
            const int4 v = *reinterpret_cast<const int4*>(reinterpret_cast<const char*>(L) + (p & ~15));
            p = v.x ^ (v.y & 0) ^ (v.z & 0) ^ (v.w & 0);
        }
        a = p;
    } else if constexpr (V == 5) {  // LDS chase + one dependent v_add per step (b32)
        int p = (threadIdx.x * 4) & 4095;
        for (int i = 0; i < kIt; ++i) {
            p = *reinterpret_cast<const int*>(reinterpret_cast<const char*>(L) + p);
            asm volatile("v_add_u32 %0, %0, 0" : "+v"(p));
        }
        a = p;
    }
    const long long t1 = clock64();
    out[threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    int* d;
    long long* c;
    hipMalloc(&d, 256 * sizeof(int));
    hipMalloc(&c, sizeof(long long));
    auto run = [&](const char* name, void (*k)(int, int*, long long*), double per) {
        long long cyc = 0;
        for (int r = 0; r < 3; ++r) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, 1, d, c);
            hipDeviceSynchronize();
        }
        hipMemcpy(&cyc, c, sizeof(cyc), hipMemcpyDeviceToHost);
        printf("%-46s %6.2f cycles per unit (%s)\n", name, cyc / (double)kIt / per,
               hipGetErrorString(hipGetLastError()));
    };
    run("dependent v_add_u32", kern<0>, 8);
    run("4 independent v_add_u32 chains", kern<1>, 8);
    run("v_cmp -> v_cndmask (per instruction)", kern<2>, 8);
    run("LDS chase ds_read_b32 (per load)", kern<3>, 1);
    run("LDS chase ds_read_b128 (per load)", kern<4>, 1);
    run("LDS chase b32 + dependent v_add (per step)", kern<5>, 1);
    return 0;
}
