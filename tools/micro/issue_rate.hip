// Single-wave VALU issue/latency microbenchmark (diagnostic, not part of the product).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void dep_chain(int* out, int iters, long long* cyc) {
    int a = threadIdx.x, b = threadIdx.x * 3 + 1;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
        }
    }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void indep(int* out, int iters, long long* cyc) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, b = threadIdx.x * 3 + 1;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b));
        }
    }
    long long t1 = clock64();
    out[threadIdx.x] = a0 + a1 + a2 + a3;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void fdep(float* out, int iters, long long* cyc) {
    float a = threadIdx.x, b = 1.0001f;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 64; ++k) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lds_dep(int* out, int iters, long long* cyc) {
    __shared__ int t[128];
    t[threadIdx.x] = (threadIdx.x + 1) & 63;
    __syncthreads();
    int a = threadIdx.x;
    long long t0 = clock64();
    for (int i = 0; i < iters * 64; ++i) a = t[a];
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    int* d; long long* c; long long h;
    hipMalloc(&d, 4096); hipMalloc(&c, 64);
    const int iters = 1000;
    auto run = [&](const char* name, void (*k)(int*, int, long long*), int per_iter) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, iters, c);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, iters, c);
        hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("%-10s %.2f clock64 ticks per instruction\n", name, (double)h / (iters * (double)per_iter));
    };
    run("dep_add", dep_chain, 64);
    run("indep_add", indep, 64);
    run("lds_chain", lds_dep, 64);
    hipLaunchKernelGGL(fdep, dim3(1), dim3(64), 0, 0, (float*)d, iters, c);
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("%-10s %.2f clock64 ticks per instruction\n", "dep_fmul", (double)h / (iters * 64.0));
    // wall clock reference for clock64 frequency
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(dep_chain, dim3(1), dim3(64), 0, 0, d, 100000, c);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("dep_add 6.4M instr: %.3f ms wall, %lld ticks -> %.1f ns/instr, clock64 %.2f GHz\n", ms, h,
           ms * 1e6 / 6.4e6, h / (ms * 1e6));
    int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("device clock rate attr %d kHz\n", clk);
    return 0;
}
