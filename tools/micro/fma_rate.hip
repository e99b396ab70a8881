// FP32 VALU peak check (diagnostic): independent v_fma_f32 vs v_pk_fma_f32 streams, full chip.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) k_fma(float* out, int iters, float s) {
    float a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = __builtin_fmaf(a[i], s, 1.0f);
    }
    float r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_pk(float* out, int iters, float s) {
    f2 a[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = f2{(float)threadIdx.x + i, (float)i};
    const f2 sv = f2{s, s}, one = f2{1.0f, 1.0f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = __builtin_elementwise_fma(a[i], sv, one);
    }
    float r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += a[i].x + a[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
    const int blocks = 256 * 8, iters = 4096;
    float* d;
    hipMalloc(&d, sizeof(float) * blocks * 256);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int v = 0; v < 2; ++v) {
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a, 0);
            if (v == 0) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f);
            else hipLaunchKernelGGL(k_pk, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        const double flops = 2.0 * 16 * iters * (double)blocks * 256 * (v ? 2 : 1);
        printf("%s: %.2f ms, %.1f TFLOP/s\n", v ? "v_pk_fma_f32" : "v_fma_f32", ms, flops / ms / 1e9);
    }
    return 0;
}
