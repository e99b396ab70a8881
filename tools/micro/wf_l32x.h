// Ablations of wf_fft_l32 (diagnostic, not part of the product): the production kernel's code
// with parts switched off, to see which resource bounds a frame.  V bits:
//   1  no frame loads after the first frame (the transform reruns on the first frame's samples)
//   2  no LDS exchange (each pass transforms the previous pass's registers; no barriers)
//   4  no FFT arithmetic (the loads, the window product, the exchanges and |X|^2 only)
// Results are meaningless for V != 0; only the time is.
#pragma once
namespace owrx {
template <int V>
__global__ void __launch_bounds__(WfL32::NT)
wf_fft_l32x(const float2* __restrict__ blk, const WfGroup* __restrict__ groups,
            const float* __restrict__ window, const float2* __restrict__ tw, float* __restrict__ partial) {
    using K = WfL32;
    constexpr int N = K::N, NT = K::NT;
    constexpr bool kLoads = !(V & 1), kLds = !(V & 2), kMath = !(V & 4);
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int t0 = threadIdx.x;
    WF_RSTAMP(14);
    WF_STAMP(0);
    const int gi = blockIdx.x;
    const WfGroup g = groups[gi];
    const int64_t g0 = __builtin_amdgcn_readfirstlane((int)g.start);
    const int hop = __builtin_amdgcn_readfirstlane(g.hop);
    const int nfr = __builtin_amdgcn_readfirstlane(g.nframes);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(blk + g0), 0, (int)(sizeof(float2) * ((int64_t)(nfr - 1) * hop + N)), 0x00020000);
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0, (int)(sizeof(float) * N),
                                                      0x00020000);
    auto load_x = [&](int f, float2* v) {
        const int fo = f < nfr ? f * hop * 8 : kWfOob;
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            const int vo = t0 * 8 + fo;
            v[r] = make_float2(
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo, r * NT * 8, 0)),
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4, r * NT * 8, 0)));
        }
    };
    auto load_w = [&](float* v) {
#pragma unroll
        for (int r = 0; r < 32; ++r)
            v[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, t0 * 4, r * NT * 4, 0));
    };
    float2 tp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) tp[i] = tw[(t0 << i) & (N - 1)];
    float2 t2v[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = t0 + NT * i;
        t2v[i] = e < 31 * 32 ? tw[(((e >> 5) + 1) * (e & 31)) << 4] : make_float2(0.f, 0.f);
    }
    float2 nx[32];
    load_x(0, nx);
#pragma unroll
    for (int i = 0; i < 2; ++i)
        if (t0 + NT * i < 31 * 32) sm[K::TW2 + t0 + NT * i] = t2v[i];
    float acc[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) acc[m] = 0.0f;
    const int sw = wf_swz32(t0);
    float wv[32];
    load_w(wv);
#pragma unroll 1
    for (int f = 0; f < nfr; ++f) {
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        const int sb = 1 + 6 * f;
        if (f < 2) WF_STAMP(sb);
        float2 a[32];
        {
            if (kLoads) load_w(wv);
#pragma unroll
            for (int r = 0; r < 32; ++r) a[r] = make_float2(nx[r].x * wv[r], nx[r].y * wv[r]);
        }
        if (kLoads) load_x(f + 1, nx);
        if (kMath) f2dft32(a);
        if (f < 2) WF_STAMP(sb + 1);
        if (kLds) {
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 32; ++k) sm[32 * t + (k ^ (t & 15))] = a[l32_at(k)];
        }
        if (f < 2) WF_STAMP(sb + 2);
        if (kLds) __syncthreads();
        {
            const int ts = wf_swz32(t);
            if (kLds) {
#pragma unroll
                for (int r = 0; r < 32; ++r) a[r] = sm[ts + NT * r];
            }
            const int k = t & 31;
            const float2* T = sm + K::TW2 + k;
            if (kMath) {
#pragma unroll
                for (int r = 1; r < 32; ++r) {
                    a[r] = f2mul(a[r], kLds ? T[(r - 1) * 32] : tp[r & 3]);
                    if ((r & 7) == 7) __builtin_amdgcn_sched_barrier(0);
                }
                f2dft32(a);
            }
            if (kLds) {
                __syncthreads();
                const int base = (t >> 5) * 1024 + k;
#pragma unroll
                for (int r = 0; r < 32; ++r) sm[wf_swz32(base + 32 * r)] = a[l32_at(r)];
            }
        }
        if (f < 2) WF_STAMP(sb + 3);
        if (kLds) {
            __syncthreads();
#pragma unroll
            for (int m = 0; m < 32; ++m) a[m] = sm[sw + NT * m];
        }
        if (f < 2) WF_STAMP(sb + 4);
        if (kMath) {
            float2 tb[16];
            tb[1] = tp[0];
            tb[2] = tp[1];
            tb[4] = tp[2];
            tb[8] = tp[3];
            tb[3] = f2mul(tp[0], tp[1]);
            tb[5] = f2mul(tp[0], tp[2]);
            tb[6] = f2mul(tp[1], tp[2]);
            tb[7] = f2mul(tb[3], tp[2]);
#pragma unroll
            for (int r = 9; r < 16; ++r) tb[r] = f2mul(tb[r - 8], tp[3]);
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                float2 c[16];
                c[0] = a[b];
#pragma unroll
                for (int r = 1; r < 16; ++r) {
                    const float2 w = b ? f2mul32(tb[r], r) : tb[r];
                    c[r] = f2mul(a[b + 2 * r], w);
                }
                f2dft<16>(c);
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    acc[b + 2 * r] = fmaf(c[r].y, c[r].y, fmaf(c[r].x, c[r].x, acc[b + 2 * r]));
            }
        } else {
#pragma unroll
            for (int m = 0; m < 32; ++m) acc[m] = fmaf(a[m].y, a[m].y, fmaf(a[m].x, a[m].x, acc[m]));
        }
        if (f < 2) WF_STAMP(sb + 5);
    }
    float* out = partial + (int64_t)blockIdx.x * N;
#pragma unroll
    for (int m = 0; m < 32; ++m) out[t0 + NT * m] = acc[m];
    WF_STAMP(13);
    WF_RSTAMP(15);
}
}  // namespace owrx
