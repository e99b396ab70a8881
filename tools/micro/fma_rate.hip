// FP32 VALU rate check (diagnostic): independent v_fma_f32 / v_add_f32 vs v_pk_fma_f32 /
// v_pk_add_f32 / v_pk_mul_f32 streams at 1, 2, 4 and 8 waves per SIMD, full chip.  Reports the
// cycles one SIMD spends per wave-instruction (2.4 GHz assumed; the clock is also printed from
// s_memrealtime vs s_memtime) and the FLOP rate.  Settles whether packed FP32 raises the VALU
// throughput of the waterfall FFT's butterflies on gfx950 or only cuts the instruction count.
// Build: hipcc -O3 --offload-arch=gfx950 fma_rate.hip -o fma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kAcc = 16;  // independent chains per lane

template <int OP>
__global__ void __launch_bounds__(256) k_rate(float* out, int iters, float s, long long* clk) {
    f2 a[kAcc];
#pragma unroll
    for (int i = 0; i < kAcc; ++i) a[i] = f2{(float)threadIdx.x + i, (float)i};
    const f2 sv = f2{s, s};
    const long long t0 = __builtin_amdgcn_s_memtime();
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < kAcc; ++i) {
            if constexpr (OP == 0) {
                asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i].x) : "v"(sv.x));
            } else if constexpr (OP == 1) {
                asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(sv));
            } else if constexpr (OP == 2) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i].x) : "v"(sv.x));
            } else if constexpr (OP == 3) {
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(sv));
            } else if constexpr (OP == 4) {
                asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(sv));
            } else {
                // the waterfall's complex product: v_pk_mul + v_pk_fma (op_sel / neg forms)
                f2 t;
                asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a[i]), "v"(sv));
                asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
                             : "+v"(a[i]) : "v"(sv), "v"(t));
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    float r = 0;
#pragma unroll
    for (int i = 0; i < kAcc; ++i) r += a[i].x + a[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 2048;
    float* d;
    long long* clk;
    hipMalloc(&d, sizeof(float) * ncu * 8 * 256);
    hipMalloc(&clk, 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_add_f32", "v_pk_add_f32", "v_pk_mul_f32", "cmul pk_mul+pk_fma"};
    const int flops_per[] = {2, 4, 1, 2, 2, 6};     // per lane per instruction (cmul: per pair)
    const int insts_per[] = {1, 1, 1, 1, 1, 2};
    for (int op = 0; op < 6; ++op) {
        for (int wps : {1, 2, 4, 8}) {
            const int blocks = ncu * wps;  // 256 threads = one wave per SIMD per block
            float ms = 0;
            for (int rep = 0; rep < 4; ++rep) {
                hipEventRecord(a, 0);
                switch (op) {
                    case 0: hipLaunchKernelGGL(k_rate<0>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f, clk); break;
                    case 1: hipLaunchKernelGGL(k_rate<1>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f, clk); break;
                    case 2: hipLaunchKernelGGL(k_rate<2>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f, clk); break;
                    case 3: hipLaunchKernelGGL(k_rate<3>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f, clk); break;
                    case 4: hipLaunchKernelGGL(k_rate<4>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f, clk); break;
                    default: hipLaunchKernelGGL(k_rate<5>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999f, clk); break;
                }
                hipEventRecord(b, 0);
                hipEventSynchronize(b);
                hipEventElapsedTime(&ms, a, b);
            }
            long long c[2];
            hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
            const double wave_insts = (double)iters * kAcc * insts_per[op];  // per wave
            const double cyc_per = (double)c[0] / wave_insts;                 // one wave's view
            const double simd_cyc = cyc_per / wps;                            // per wave-instruction per SIMD
            const double flops = (double)flops_per[op] * kAcc * iters * (double)blocks * 256;
            printf("%-20s waves/SIMD %d: %.3f ms  %.1f TFLOP/s  wave cyc/inst %.2f  SIMD cyc/inst %.2f  clock %.2f GHz\n",
                   names[op], wps, ms, flops / ms / 1e9, cyc_per, simd_cyc,
                   (double)c[0] / ((double)c[1] / 100e6) / 1e9);
        }
    }
    return 0;
}
