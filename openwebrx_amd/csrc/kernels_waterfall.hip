// kernels_waterfall.hip -- FftChain on CDNA4 (csdr/chain/fft.py:25-96, driven by
// owrx/fft.py:36-59): Fft(size=N, every_n_samples=hop) -> LogAveragePower(add_db, N, avg)
// -> FftSwap -> FftAdpcm.
//
// wf_fft_l32 (N = 16384, production for C2/C3/C5): 32 x 32 x 16 with two LDS exchanges, 512
//   threads of 32 points, one workgroup per group of consecutive frames (see its comment).
// wf_fft_r16 (1024 <= N <= 8192; N = 16384 with OWRX_WF_KERNEL=r16): one workgroup (N/16 threads) per group of
//   consecutive frames of one waterfall row.  Each frame: cf32 samples * Hamming window in
//   registers (16 per thread, the next frame prefetched during the passes), radix-16 register
//   DFTs with Stockham exchanges through LDS (N complex + 1-in-16 padding: 136 KiB at
//   N = 16384, one workgroup per CU), twiddle bases from LDS tables; |X|^2 summed in registers
//   over the group's frames and written once per group.  wf_fft_power (radix 4): N = 256, 512.
//   Variants that lost their same-box A/B live in tools/micro/wf_variants.hip.
// wf_fft4_cols / wf_fft4_rows (N = 32768, 65536): four-step FFT through a cf32 scratch frame.
// wf_finalize: sums each row's group partials in a fixed order onto the carried accumulator
//   (rows span blocks), 10*log10 + add_db correction, fftshift, quantise (short)(dB*100).
// wf_adpcm_rows_spec: FftAdpcm (IMA-ADPCM of each padded row), one workgroup per row at a
//   time, segment-parallel and exact (adpcm_spec.h).
#include <algorithm>
#include <stdlib.h>
#include <string.h>

#include "adpcm_spec.h"
#include "fft_lds.h"
#include "owrx_types.h"

namespace owrx {

OWRX_DEV float2 ld2(const float2* p) { return *p; }

// A buffer-load offset past every waterfall descriptor's range (num_records < 2^30 bytes): such
// loads return zeros and never touch memory, so a prefetch can be issued unconditionally.
constexpr int kWfOob = 1 << 30;

template <int LOGN>
__global__ void __launch_bounds__(1024)
wf_fft_power(const float2* __restrict__ blk, int64_t blk_start,
             const WfGroup* __restrict__ groups, const float* __restrict__ window,
             const float2* __restrict__ tw, float* __restrict__ partial) {
    constexpr int N = 1 << LOGN;
    constexpr int NT = (N / 4 < 1024) ? N / 4 : 1024;
    constexpr int BPT = (N / 4) / NT;   // radix-4 butterflies per thread
    constexpr int PPT = N / NT;         // points per thread
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int tid0 = threadIdx.x;
    const WfGroup g = groups[blockIdx.x];
    // |X|^2 accumulated in registers across the group's frames (<= 16 per thread)
    constexpr bool kRegAcc = PPT <= 16;
    float acc[kRegAcc ? PPT : 1];
#pragma unroll
    for (int m = 0; m < (kRegAcc ? PPT : 1); ++m) acc[m] = 0.0f;
    float* gacc = partial + (int64_t)blockIdx.x * N;

    for (int f = 0; f < g.nframes; ++f) {
        // opaque copy of the thread id: stops the compiler hoisting every pass's LDS/twiddle
        // address arithmetic out of the frame loop (which spills at N = 16384)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const float2* x = blk + (g.start + (int64_t)f * g.hop - blk_start);
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int i = tid + m * NT;
            const float2 v = x[i];
            const float w = window[i];
            sm[i] = make_float2(v.x * w, v.y * w);
        }
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
        int lns = 0;  // log2(Ns)
#pragma unroll
        for (int pass = 0; pass < LOGN / 2; ++pass) {
            float2 a[BPT][4];
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int j = tid + b * NT;
#pragma unroll
                for (int r = 0; r < 4; ++r) a[b][r] = sm[j + r * (N / 4)];
            }
            __syncthreads();
#pragma unroll
            for (int b = 0; b < BPT; ++b) {
                const int j = tid + b * NT;
                const int k = j & ((1 << lns) - 1);
                const int ts = k << (LOGN - 2 - lns);  // k * N / (4 Ns)
                float2 a0 = a[b][0];
                float2 a1 = cmul(a[b][1], tw[ts]);
                float2 a2 = cmul(a[b][2], tw[2 * ts]);
                float2 a3 = cmul(a[b][3], tw[3 * ts]);
                const float2 t0 = make_float2(a0.x + a2.x, a0.y + a2.y);
                const float2 t1 = make_float2(a0.x - a2.x, a0.y - a2.y);
                const float2 t2 = make_float2(a1.x + a3.x, a1.y + a3.y);
                const float2 t3 = make_float2(a1.y - a3.y, a3.x - a1.x);  // -i (a1 - a3)
                const int d = ((j >> lns) << (lns + 2)) + k;
                const int ns = 1 << lns;
                sm[d] = make_float2(t0.x + t2.x, t0.y + t2.y);
                sm[d + ns] = make_float2(t1.x + t3.x, t1.y + t3.y);
                sm[d + 2 * ns] = make_float2(t0.x - t2.x, t0.y - t2.y);
                sm[d + 3 * ns] = make_float2(t1.x - t3.x, t1.y - t3.y);
                if (BPT > 2) __builtin_amdgcn_sched_barrier(0);  // <= 3 twiddles in flight
            }
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);  // keep next pass's twiddle loads out of this one
            lns += 2;
        }
        if constexpr (LOGN & 1) {
            constexpr int B2 = (N / 2) / NT;
            float2 a[B2][2];
#pragma unroll
            for (int b = 0; b < B2; ++b) {
                const int j = tid + b * NT;
                a[b][0] = sm[j];
                a[b][1] = sm[j + N / 2];
            }
            __syncthreads();
#pragma unroll
            for (int b = 0; b < B2; ++b) {
                const int j = tid + b * NT;
                const int k = j & ((1 << lns) - 1);
                const float2 a1 = cmul(a[b][1], tw[k << (LOGN - 1 - lns)]);
                const int d = ((j >> lns) << (lns + 1)) + k;
                sm[d] = make_float2(a[b][0].x + a1.x, a[b][0].y + a1.y);
                sm[d + (1 << lns)] = make_float2(a[b][0].x - a1.x, a[b][0].y - a1.y);
            }
            __syncthreads();
        }
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const float2 X = sm[tid + m * NT];
            const float pw = X.x * X.x + X.y * X.y;
            if constexpr (kRegAcc)
                acc[m] += pw;
            else
                gacc[tid + m * NT] = (f == 0) ? pw : gacc[tid + m * NT] + pw;
            if (!kRegAcc && (m % 4) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (kRegAcc) {
#pragma unroll
        for (int m = 0; m < PPT; ++m) gacc[tid0 + m * NT] = acc[m];
    }
}

// ---- wf_fft_r16: the same product with radix-16 passes in registers (N = 1024 .. 16384) ----
// N/16 threads, 16 points each.  Stockham passes of radix 16 (and one final radix 2/4/8 pass
// for log2 N not a multiple of 4): pass 1 takes its 16 points straight from HBM (coalesced, times
// the window), every pass but the last writes LDS, the last one squares its outputs into
// per-thread |X|^2 accumulators -- the bins a thread finishes are the same in every frame, so a
// group of frames is summed in registers and written once.  Three LDS round trips per frame at
// N = 16384 (seven for the radix-4 kernel), twiddles W^k from the N-point table once per pass
// and their powers by complex products; the LDS image is padded one element in 16 so that the
// stride-16 stores of the first pass spread over the banks.
OWRX_DEV int wf_pad(int i) { return i + (i >> 4); }



// Complex arithmetic on packed FP32 pairs: a complex add is one v_pk_add_f32, a complex product
// two packed instructions, so a radix-4 butterfly is 8 instructions instead of 16 (the FFT is
// VALU-bound per CU at these sizes: ~1.5k scalar instructions per thread and 16384-point frame).
typedef float c2 __attribute__((ext_vector_type(2)));
OWRX_DEV c2 c2_of(float2 v) { return c2{v.x, v.y}; }
OWRX_DEV float2 f2_of(c2 v) { return make_float2(v.x, v.y); }
OWRX_DEV c2 pk_mul(c2 a, c2 w) {  // complex a * w
    c2 t, s;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(s) : "v"(a), "v"(w), "v"(t));
    return s;
}
OWRX_DEV c2 pk_add_mi(c2 t, c2 d) {  // t + (-i) d
    c2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(t), "v"(d));
    return r;
}
OWRX_DEV c2 pk_sub_mi(c2 t, c2 d) {  // t - (-i) d
    c2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(t), "v"(d));
    return r;
}

// W_L^k = exp(-2 pi i k / L), L a power of two
OWRX_DEV c2 wf_twiddle(int k, int L) {
    float s, c;
    sincospif(-2.0f * (float)k / (float)L, &s, &c);
    return c2{c, s};
}

// in-register DFT of size R (forward), natural order in and out
OWRX_DEV void dft4(c2& a0, c2& a1, c2& a2, c2& a3) {
    const c2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = a1 - a3;
    a0 = t0 + t2;
    a2 = t0 - t2;
    a1 = pk_add_mi(t1, d);
    a3 = pk_sub_mi(t1, d);
}

// W_32^m = exp(-2 pi i m / 32), m < 32 (compile-time after unrolling)
OWRX_DEV c2 w32(int m) {
    const float c[8] = {1.0f, 0.98078528040323043f, 0.92387953251128676f, 0.83146961230254524f,
                        0.70710678118654752f, 0.55557023301960218f, 0.38268343236508977f,
                        0.19509032201612827f};
    // cos / sin of 2 pi m / 32 from the first octant
    const int q = (m >> 3) & 3, r = m & 7;
    const float cr = c[r], sr = r ? c[8 - r] : 0.0f;
    float cs, sn;
    if (q == 0) { cs = cr; sn = sr; }
    else if (q == 1) { cs = -sr; sn = cr; }
    else if (q == 2) { cs = -cr; sn = -sr; }
    else { cs = sr; sn = -cr; }
    return c2{cs, -sn};
}

template <int R>
OWRX_DEV void dft_r(c2* a) {
    if constexpr (R == 2) {
        const c2 t = a[1];
        a[1] = a[0] - t;
        a[0] = a[0] + t;
    } else if constexpr (R == 4) {
        dft4(a[0], a[1], a[2], a[3]);
    } else if constexpr (R == 8) {
        // n = 2 n1 + n2 (n1 < 4, n2 < 2), k = k1 + 4 k2
        c2 b0[4] = {a[0], a[2], a[4], a[6]}, b1[4] = {a[1], a[3], a[5], a[7]};
        dft4(b0[0], b0[1], b0[2], b0[3]);
        dft4(b1[0], b1[1], b1[2], b1[3]);
        const float h = 0.70710678118654752f;
        const c2 w[4] = {c2{1.f, 0.f}, c2{h, -h}, c2{0.f, -1.f}, c2{-h, -h}};  // W8^k1
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) {
            const c2 t = k1 ? pk_mul(b1[k1], w[k1]) : b1[k1];
            a[k1] = b0[k1] + t;
            a[k1 + 4] = b0[k1] - t;
        }
    } else if constexpr (R == 32) {
        // n = 4 n1 + n2 (n1 < 8, n2 < 4), k = k1 + 8 k2: DFT8 over n1, twiddle W32^(n2 k1),
        // DFT4 over n2
        c2 b[4][8];
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) {
#pragma unroll
            for (int n1 = 0; n1 < 8; ++n1) b[n2][n1] = a[4 * n1 + n2];
            dft_r<8>(b[n2]);
        }
#pragma unroll
        for (int n2 = 1; n2 < 4; ++n2)
#pragma unroll
            for (int k1 = 1; k1 < 8; ++k1) b[n2][k1] = pk_mul(b[n2][k1], w32(n2 * k1));
#pragma unroll
        for (int k1 = 0; k1 < 8; ++k1) {
            dft4(b[0][k1], b[1][k1], b[2][k1], b[3][k1]);
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) a[k1 + 8 * k2] = b[k2][k1];
        }
    } else {
        static_assert(R == 16, "radix");
        // n = 4 n1 + n2, k = k1 + 4 k2: DFT4 over n1, twiddle W16^(n2 k1), DFT4 over n2
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) dft4(a[n2], a[4 + n2], a[8 + n2], a[12 + n2]);
        const float c1 = 0.92387953251128676f, s1 = 0.38268343236508977f, h = 0.70710678118654752f;
        // B[n2][k1] sits at a[4 k1 + n2]; multiply by W16^(n2 k1)
        a[4 * 1 + 1] = pk_mul(a[4 * 1 + 1], c2{c1, -s1});   // W^1
        a[4 * 2 + 1] = pk_mul(a[4 * 2 + 1], c2{h, -h});     // W^2
        a[4 * 3 + 1] = pk_mul(a[4 * 3 + 1], c2{s1, -c1});   // W^3
        a[4 * 1 + 2] = pk_mul(a[4 * 1 + 2], c2{h, -h});     // W^2
        a[4 * 2 + 2] = c2{a[4 * 2 + 2].y, -a[4 * 2 + 2].x}; // W^4 = -i
        a[4 * 3 + 2] = pk_mul(a[4 * 3 + 2], c2{-h, -h});    // W^6
        a[4 * 1 + 3] = pk_mul(a[4 * 1 + 3], c2{s1, -c1});   // W^3
        a[4 * 2 + 3] = pk_mul(a[4 * 2 + 3], c2{-h, -h});    // W^6
        a[4 * 3 + 3] = pk_mul(a[4 * 3 + 3], c2{-c1, s1});   // W^9
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) dft4(a[4 * k1], a[4 * k1 + 1], a[4 * k1 + 2], a[4 * k1 + 3]);
        // X[k1 + 4 k2] is at a[4 k1 + k2]: transpose the 4 x 4 register block
        c2 t[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i] = a[i];
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) a[k1 + 4 * k2] = t[4 * k1 + k2];
    }
}

// a[r] *= W^(r k) for r < R given w1 = W^k (successive powers: two live twiddles; the
// rounding of 15 products stays ~1e-6 relative)
template <int R>
OWRX_DEV void twiddle_r(c2* a, c2 w1) {
    c2 w = w1;
#pragma unroll
    for (int r = 1; r < R; ++r) {
        a[r] = pk_mul(a[r], w);
        if (r + 1 < R) w = pk_mul(w, w1);
    }
}

template <int LOGN>
struct WfR16 {
    static constexpr int N = 1 << LOGN;
    static constexpr int NT = N / 16;
    static constexpr int P16 = LOGN / 4;                          // radix-16 passes
    static constexpr int RL = 1 << (LOGN - 4 * P16);              // last radix (1: none)
    static constexpr int BL = RL > 1 ? N / RL / NT : 1;           // butterflies / thread, last
    static constexpr int NACC = RL > 1 ? BL * RL : 16;            // bins per thread
    // twiddle tables behind the padded frame image: passes 1 .. P16-1 (16, 256, ... entries,
    // W_(16 Ns)^k at (Ns - 16) / 15 + k), then the last pass's bases W_N^tid (NT entries)
    static constexpr int TW0 = N + N / 16;
    static constexpr int NTP = P16 > 1 ? ((1 << (4 * P16)) - 16) / 15 : 0;
    static constexpr int NTL = RL > 1 ? NT : 0;
    static constexpr size_t kLds = sizeof(float2) * (TW0 + NTP + NTL);
};

// Phase stamps of wave 0 (diagnostic builds only: tools/micro/wf_stamp.hip defines
// OWRX_WF_STAMPS): kernel start, per frame (first two) its start, loads arrived, each pass done,
// and the partial row written.
#ifdef OWRX_WF_STAMPS
__device__ unsigned long long g_wf_stamp[1024][16];
#define WF_STAMP(i)                                                                           \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 1024 && (i) < 16) g_wf_stamp[blockIdx.x][i] = clock64(); \
    } while (0)
#define WF_RSTAMP(i)                                                                          \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 1024 && (i) < 16)                                \
            g_wf_stamp[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();                     \
    } while (0)
#ifdef OWRX_WF_WSTAMPS
// per-wave stamps (wf_fft_q16, frame 2 of the first item): [workgroup][wave][slot]
__device__ unsigned long long g_wf_wstamp[256][16][12];
// (held in registers during the frame -- a global store per stamp queues behind the frame's
// loads and would itself delay the wave -- and stored after the frame loop)
#define WF_WSTAMP(i)                                                                          \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        wst_[i] = __builtin_readcyclecounter();                                               \
        __builtin_amdgcn_sched_barrier(0);                                                    \
    } while (0)
#endif
#else
#define WF_STAMP(i) \
    do {            \
    } while (0)
#define WF_RSTAMP(i) \
    do {             \
    } while (0)
#endif
#ifndef OWRX_WF_WSTAMPS
#define WF_WSTAMP(i) \
    do {             \
    } while (0)
#endif

template <int LOGN>
__global__ void __launch_bounds__(WfR16<LOGN>::NT)
wf_fft_r16(const float2* __restrict__ blk, int64_t blk_start,
           const WfGroup* __restrict__ groups, const float* __restrict__ window,
           const float2* __restrict__ tw, float* __restrict__ partial) {
    using K = WfR16<LOGN>;
    constexpr int N = K::N, NT = K::NT, P16 = K::P16, RL = K::RL, BL = K::BL;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int tid0 = threadIdx.x;
    const WfGroup g = groups[blockIdx.x];
    WF_STAMP(0);
    // The twiddles come from LDS tables filled once per workgroup, so the frame loop's only
    // global loads are the next frame's samples (issued in pass 0, in flight across the passes)
    // and the window taps at the frame's start.  vmcnt retires loads in order, so a twiddle load
    // between the prefetch and its use would have waited for the whole prefetch.  Both go through
    // buffer descriptors: one VGPR of per-lane offset, the frame / tap offsets in SGPRs (64-bit
    // addresses per load take 32 VGPRs).
    const int64_t g0 = __builtin_amdgcn_readfirstlane((int)(g.start - blk_start));
    const int hop = __builtin_amdgcn_readfirstlane(g.hop);
    const int nfr = __builtin_amdgcn_readfirstlane(g.nframes);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(blk + g0), 0, (int)(sizeof(float2) * ((int64_t)(nfr - 1) * hop + N)),
        0x00020000);
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0,
                                                      (int)(sizeof(float) * N), 0x00020000);
    auto load_x = [&](int f, c2* v) {
        const int fo = f < nfr ? f * hop * 8 : kWfOob;  // f == nfr: zeros (see wf_fft_l32)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // two dword loads the compiler pairs into one dwordx2 (this hipcc's vector-returning
            // raw_buffer_load_b64 / _b128 builtins load one dword and splat it); the frame offset
            // in the one VGPR, the tap offset r NT in the SGPR soffset
            const int vo = tid0 * 8 + fo;
            v[r] = c2{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo, r * NT * 8, 0)),
                      __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4, r * NT * 8, 0))};
        }
    };
    auto load_w = [&](float* v) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
            v[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, tid0 * 4, r * NT * 4, 0));
    };

    // the first frame's samples are requested before the twiddle tables: the table fill waits
    // for its own loads (vmcnt is in order), by then the frame has arrived as well
    c2 nx[16];
    load_x(0, nx);
    for (int i = tid0; i < K::NTP; i += NT) {
        int base = 0, ns = 16;
        while (i >= base + ns) {
            base += ns;
            ns *= 16;
        }
        sm[K::TW0 + i] = tw[(i - base) * (N / (ns * 16))];
    }
    if constexpr (RL > 1) sm[K::TW0 + K::NTP + tid0] = tw[tid0];
    float acc[K::NACC];  // sum over the group's frames of |X|^2 per bin
#pragma unroll
    for (int m = 0; m < K::NACC; ++m) acc[m] = 0.0f;
#pragma unroll 1
    for (int f = 0; f < nfr; ++f) {
        // opaque copy of the thread id: keeps every pass's address arithmetic inside the frame
        // loop (hoisted, the addresses of all passes stay live and spill)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        c2 a[16];
        const int st0 = 1 + 6 * f;
        WF_STAMP(st0);
        // pass 1 (Ns = 1, no twiddles): j = tid, inputs j + r N/16
        {
            float wv[16];  // L2-resident taps; the wait for them also covers the prefetch
            load_w(wv);
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = nx[r] * wv[r];
        }
        WF_STAMP(st0 + 1);
        int ns = 1;
#pragma unroll
        for (int pass = 0; pass < P16; ++pass) {
            if (pass > 0) {
                __syncthreads();  // the previous pass's stores
#pragma unroll
                for (int r = 0; r < 16; ++r) a[r] = c2_of(sm[wf_pad(tid + r * NT)]);
                const int k = tid & (ns - 1);
                if (k) twiddle_r<16>(a, c2_of(sm[K::TW0 + (ns - 16) / 15 + k]));  // W_(16 Ns)^k
            }
            __builtin_amdgcn_sched_barrier(0);
            dft_r<16>(a);
            __builtin_amdgcn_sched_barrier(0);
            const bool last = (pass == P16 - 1) && RL == 1;
            if (last) {
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = fmaf(a[r].y, a[r].y, fmaf(a[r].x, a[r].x, acc[r]));
            } else {
                if (pass > 0) __syncthreads();  // every load of this pass before any store
                const int k = tid & (ns - 1);
                const int d = ((tid / ns) * ns * 16) + k;
#pragma unroll
                for (int r = 0; r < 16; ++r) sm[wf_pad(d + r * ns)] = f2_of(a[r]);
                if (pass == 0) load_x(f + 1, nx);
            }
            ns *= 16;
            WF_STAMP(st0 + 2 + pass);
        }
        if constexpr (RL > 1) {
            // last pass: radix RL, Ns = N / RL, butterflies j = tid + b NT, outputs j + r N/RL
            __syncthreads();
            const c2 tl = c2_of(sm[K::TW0 + K::NTP + tid]);  // W_N^tid
#pragma unroll
            for (int b = 0; b < BL; ++b) {
                const int j = tid + b * NT;
                c2 c[RL];
#pragma unroll
                for (int r = 0; r < RL; ++r) c[r] = c2_of(sm[wf_pad(j + r * (N / RL))]);
                // W_N^j = W_N^tid W_16^b (NT = N / 16)
                if (b == 0) {
                    if (j) twiddle_r<RL>(c, tl);
                } else {
                    twiddle_r<RL>(c, pk_mul(tl, w32(2 * b)));
                }
                dft_r<RL>(c);
#pragma unroll
                for (int r = 0; r < RL; ++r)
                    acc[b * RL + r] = fmaf(c[r].y, c[r].y, fmaf(c[r].x, c[r].x, acc[b * RL + r]));
                __builtin_amdgcn_sched_barrier(0);
            }
            WF_STAMP(st0 + 5);
        }
        __syncthreads();  // LDS reused by the next frame
    }
    float* out = partial + (int64_t)blockIdx.x * N;
    if constexpr (RL > 1) {
#pragma unroll
        for (int b = 0; b < BL; ++b)
#pragma unroll
            for (int r = 0; r < RL; ++r) out[tid0 + b * NT + r * (N / RL)] = acc[b * RL + r];
    } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) out[tid0 + r * NT] = acc[r];
    }
    WF_STAMP(13);
}

// ---- plain-FP32 complex helpers (wf_fft_l32) ------------------------------------------------
// A packed FP32 instruction issues in twice the cycles of a scalar one on CDNA4's 32-lane SIMDs,
// so these are scalar float2 butterflies (FMA-contracted complex products, 4 VALU each).

// W_16^m = exp(-2 pi i m / 16), m a compile-time constant after unrolling
OWRX_DEV float2 w16c(int m) {
    constexpr float c[16] = {1.0f, 0.92387953251128676f, 0.70710678118654752f, 0.38268343236508977f,
                             0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128676f,
                             -1.0f, -0.92387953251128676f, -0.70710678118654752f, -0.38268343236508977f,
                             0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128676f};
    return make_float2(c[m & 15], -c[(m + 12) & 15]);  // sin(2 pi m / 16) = cos(2 pi (m - 4) / 16)
}

OWRX_DEV float2 f2add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
OWRX_DEV float2 f2sub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
OWRX_DEV float2 f2mi(float2 a) { return make_float2(a.y, -a.x); }  // -i a
// complex product, FMA form (4 VALU instructions)
OWRX_DEV float2 f2mul(float2 a, float2 w) {
    return make_float2(fmaf(a.x, w.x, -(a.y * w.y)), fmaf(a.x, w.y, a.y * w.x));
}

OWRX_DEV void f2dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = f2add(a0, a2), t1 = f2sub(a0, a2), t2 = f2add(a1, a3), d = f2mi(f2sub(a1, a3));
    a0 = f2add(t0, t2);
    a2 = f2sub(t0, t2);
    a1 = f2add(t1, d);
    a3 = f2sub(t1, d);
}

// in-register forward DFT of size R in natural order (R = 2, 4, 8, 16)
template <int R>
OWRX_DEV void f2dft(float2* a) {
    if constexpr (R == 2) {
        const float2 t = a[1];
        a[1] = f2sub(a[0], t);
        a[0] = f2add(a[0], t);
    } else if constexpr (R == 4) {
        f2dft4(a[0], a[1], a[2], a[3]);
    } else if constexpr (R == 8) {
        float2 b0[4] = {a[0], a[2], a[4], a[6]}, b1[4] = {a[1], a[3], a[5], a[7]};
        f2dft4(b0[0], b0[1], b0[2], b0[3]);
        f2dft4(b1[0], b1[1], b1[2], b1[3]);
        const float h = 0.70710678118654752f;
        b1[1] = make_float2(h * (b1[1].x + b1[1].y), h * (b1[1].y - b1[1].x));    // W8^1
        b1[2] = f2mi(b1[2]);                                                      // W8^2
        b1[3] = make_float2(h * (b1[3].y - b1[3].x), -h * (b1[3].x + b1[3].y));   // W8^3
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a[k] = f2add(b0[k], b1[k]);
            a[k + 4] = f2sub(b0[k], b1[k]);
        }
    } else {
        static_assert(R == 16, "radix");
        // n = 4 n1 + n2, k = k1 + 4 k2: DFT4 over n1, twiddle W16^(n2 k1), DFT4 over n2
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) f2dft4(a[n2], a[4 + n2], a[8 + n2], a[12 + n2]);
        const float c1 = 0.92387953251128676f, s1 = 0.38268343236508977f, h = 0.70710678118654752f;
        a[5] = f2mul(a[5], make_float2(c1, -s1));                                      // W^1
        a[9] = make_float2(h * (a[9].x + a[9].y), h * (a[9].y - a[9].x));              // W^2
        a[13] = f2mul(a[13], make_float2(s1, -c1));                                    // W^3
        a[6] = make_float2(h * (a[6].x + a[6].y), h * (a[6].y - a[6].x));              // W^2
        a[10] = f2mi(a[10]);                                                           // W^4
        a[14] = make_float2(h * (a[14].y - a[14].x), -h * (a[14].x + a[14].y));        // W^6
        a[7] = f2mul(a[7], make_float2(s1, -c1));                                      // W^3
        a[11] = make_float2(h * (a[11].y - a[11].x), -h * (a[11].x + a[11].y));        // W^6
        a[15] = f2mul(a[15], make_float2(-c1, s1));                                    // W^9
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) f2dft4(a[4 * k1], a[4 * k1 + 1], a[4 * k1 + 2], a[4 * k1 + 3]);
        float2 t[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i] = a[i];
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) a[k1 + 4 * k2] = t[4 * k1 + k2];
    }
}

// W_32^m = exp(-2 pi i m / 32), m a compile-time constant after unrolling
OWRX_DEV float2 w32c(int m) {
    constexpr float c[32] = {
        1.0f, 0.98078528040323043f, 0.92387953251128676f, 0.83146961230254524f,
        0.70710678118654752f, 0.55557023301960218f, 0.38268343236508977f, 0.19509032201612827f,
        0.0f, -0.19509032201612827f, -0.38268343236508977f, -0.55557023301960218f,
        -0.70710678118654752f, -0.83146961230254524f, -0.92387953251128676f, -0.98078528040323043f,
        -1.0f, -0.98078528040323043f, -0.92387953251128676f, -0.83146961230254524f,
        -0.70710678118654752f, -0.55557023301960218f, -0.38268343236508977f, -0.19509032201612827f,
        0.0f, 0.19509032201612827f, 0.38268343236508977f, 0.55557023301960218f,
        0.70710678118654752f, 0.83146961230254524f, 0.92387953251128676f, 0.98078528040323043f};
    return make_float2(c[m & 31], -c[(m + 24) & 31]);
}

// a * W_32^m for a compile-time m: the eighth turns as adds and a multiply, -i as a swap
OWRX_DEV float2 f2mul32(float2 a, int m) {
    const float h = 0.70710678118654752f;
    switch (m & 31) {
        case 0: return a;
        case 4: return make_float2(h * (a.x + a.y), h * (a.y - a.x));
        case 8: return f2mi(a);
        case 12: return make_float2(h * (a.y - a.x), -h * (a.x + a.y));
        case 16: return make_float2(-a.x, -a.y);
        case 20: return make_float2(-h * (a.x + a.y), h * (a.x - a.y));
        case 24: return make_float2(-a.y, a.x);
        case 28: return make_float2(h * (a.x - a.y), h * (a.x + a.y));
        default: return f2mul(a, w32c(m));
    }
}

// in-register forward DFT-32 in place: n = 4 n1 + n2 (n1 < 8, n2 < 4), k = k1 + 8 k2; X[k] is
// left at a[4 k1 + k2] (l32_at(k)), so no register array is copied
OWRX_DEV constexpr int l32_at(int k) { return 4 * (k & 7) + (k >> 3); }
OWRX_DEV void f2dft32(float2* a) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
        float2 v[8];
#pragma unroll
        for (int n1 = 0; n1 < 8; ++n1) v[n1] = a[4 * n1 + n2];
        f2dft<8>(v);
#pragma unroll
        for (int k1 = 0; k1 < 8; ++k1) a[4 * k1 + n2] = k1 && n2 ? f2mul32(v[k1], n2 * k1) : v[k1];
    }
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) f2dft4(a[4 * k1], a[4 * k1 + 1], a[4 * k1 + 2], a[4 * k1 + 3]);
}


// ---- wf_fft_l32: N = 16384 as 32 x 32 x 16, two LDS exchanges ------------------------------
// 512 threads of 32 points (two waves per SIMD, up to 256 VGPRs each), one workgroup per CU.
// LDS stores are the scarcest resource of the exchange (~85 B/clk/CU for any store width), so
// radix 32 cuts them from three 128 KiB exchanges per frame to two:
//  P1 (Ns = 1):    x[t + 512 r] * window -> DFT32 -> image[32 t + k]
//  P2 (Ns = 32):   image[t + 512 r] * W_1024^(r k), k = t & 31 (LDS table [31][32]) -> DFT32
//                  -> image[(t >> 5) 1024 + k + 32 r]
//  P3 (Ns = 1024): two radix-16 butterflies j = t + 512 b: image[j + 1024 r] * W_N^(r j), the
//                  bases W_N^(r t) in registers for the whole group (W_N^(r j) = W_N^(r t) W_32^(r b))
//                  -> DFT16 -> |X|^2 of bins j + 1024 r, summed in registers over the group.
// The image is XOR-swizzled (e ^ ((e >> 5) & 15)): the stride-32 stores of P1 and every read
// are bank-conflict-free.  The next frame's samples are loaded in P1 (in flight across P2 and
// P3) and the window taps in P3, so a frame starts on data already in registers.
struct WfL32 {
    static constexpr int LOGN = 14, N = 1 << LOGN, NT = 512;
    static constexpr int TW2 = N;  // [31][32]: W_1024^(r k), r = 1..31
    static constexpr size_t kLds = sizeof(float2) * (N + 31 * 32);
};
OWRX_DEV int wf_swz32(int e) { return e ^ ((e >> 5) & 15); }

// qlog > 0 (N = 16384 << qlog, wf_dif_split first): workgroup blockIdx.x = (group << qlog) + j
// transforms sub-frame j of its group's frames from the split scratch (blk; sub-frames of one
// group `fstride` frames apart), its partial row landing at partial + group * (N << qlog) +
// j * N; tw then is the (N << qlog)-point table, read at stride 1 << qlog.
//
// Tail split (qlog = 0): the launch's last `skip` groups also come as single-frame descriptors
// after the `whole` + `skip` groups (host-built), and item i is descriptor i < whole ? i :
// i + skip.  Every frame's |X|^2 is added to its accumulator as one rounded value (acc + p, p =
// fma(y, y, x x)), so a group summed in a workgroup's registers and the same group's frames
// folded in order by wf_finalize from their own partial rows give the same bits: the split
// changes no result, only how finely the last round of work is dealt.
//
// FUS (N = 16384 << qlog without the split's scratch): item w = (group << qlog) + j reads its
// group's frames from the stream itself and forms sub-frame j on load, y_j[n] = W_N^(nj) sum_q
// w[n + 16384 q] x[n + 16384 q] W_Q^(qj) with the split kernel's operations in its order (rows
// bit-identical to the split path); the Q workgroups of a frame group read it through L2 / the
// Infinity Cache instead of the split writing and re-reading 2 x 8 N bytes per frame.  No
// next-frame prefetch (the Q quarters do not fit the registers): the frame's loads go in chunks.
template <bool FUS>
__global__ void __launch_bounds__(WfL32::NT)
wf_fft_l32(const float2* __restrict__ blk, int64_t blk_start, const WfGroup* __restrict__ groups,
           const float* __restrict__ window, const float2* __restrict__ tw,
           float* __restrict__ partial, int qlog, int fstride, int items, int* __restrict__ work,
           int whole, int skip) {
    using K = WfL32;
    constexpr int N = K::N, NT = K::NT;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ int s_next;
    const int t0 = threadIdx.x;
    WF_RSTAMP(14);
    WF_STAMP(0);
    // Work items (a group's frames, or one sub-frame j of a group after the DIF split) are dealt
    // dynamically: every workgroup, its first item included, takes the next unclaimed one from
    // `work` (zeroed before the launch) until none is left.  With one workgroup per CU a static
    // first item (workgroup b on item b) doubled a launch's time whenever some workgroups were
    // placed late: on a CU-masked queue part of the grid only starts when the first wave of
    // workgroups retires, and each of those then still ran its own item at the end (measured 88
    // vs 52 us per 960 C3 frames, and the same with the first items alone static).  A late
    // workgroup now finds the items taken and exits.  An item's rows are still summed by one
    // workgroup in frame order, so the results do not depend on which workgroup took it.
    struct Item {
        __amdgpu_buffer_rsrc_t xr;
        int hop, nfr;
    };
    auto desc = [&](int i) { return i < whole ? i : i + skip; };  // item -> descriptor
    auto item = [&](int w) {
        const int gi = w >> qlog;
        const WfGroup g = groups[gi];
        const int64_t g0 = __builtin_amdgcn_readfirstlane(
            qlog && !FUS ? (int)((((int64_t)gi * fstride << qlog) + (w & ((1 << qlog) - 1))) * N)
                         : (int)(g.start - blk_start));
        Item it;
        it.hop = __builtin_amdgcn_readfirstlane(qlog && !FUS ? N << qlog : g.hop);
        it.nfr = __builtin_amdgcn_readfirstlane(g.nframes);
        it.xr = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float2*>(blk + g0), 0,
            (int)(sizeof(float2) * ((int64_t)(it.nfr - 1) * it.hop + (FUS ? N << qlog : N))), 0x00020000);
        return it;
    };
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0,
                                                      (int)(sizeof(float) * N), 0x00020000);
    // the samples of the frame at byte offset fo of descriptor xr (fo = kWfOob: zeros, no memory
    // access).  The prefetch of the next frame is unconditional: behind an `if` the wait-count
    // pass merged the two paths at vmcnt(0) before the window products, so every frame waited
    // for its successor's samples.
    auto load_x = [&](__amdgpu_buffer_rsrc_t xr, int fo, float2* v) {
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
    // FUS: the frame at byte offset fo of xr as sub-frame j (the split's y_j), in chunks of
    // kFusPts points: every quarter's samples, window taps and the point's twiddle in flight
    // together
    constexpr int kFusPts = 2;
    // (tt: the thread index made opaque per frame, so the frame-invariant window and twiddle
    // loads are not hoisted out of the frame loop: 64 + 128 values held across it spilled)
    auto fused_frame = [&](__amdgpu_buffer_rsrc_t xr, int fo, int j, int tt, float2* a) {
#pragma clang fp contract(off)  // the split kernel's roundings exactly (it is uncontracted too)
        const int NQ = N << qlog;
        const auto wq = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0,
                                                          (int)(sizeof(float) * NQ), 0x00020000);
        // (the twiddles through a buffer resource too: 32-bit offsets; per-lane 64-bit addresses
        // for every point were the kernel's spills)
        const auto tq = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(tw), 0,
                                                          (int)(sizeof(float2) * NQ), 0x00020000);
        // unrolled (a[] keeps constant indices: registers), a scheduling barrier per chunk (with
        // 8-point chunks and no barrier the kernel spilled 186 registers)
#pragma unroll
        for (int c = 0; c < 32 / kFusPts; ++c) {
            __builtin_amdgcn_sched_barrier(0);
            float2 v[4][kFusPts];
            float wv8[4][kFusPts];
            float2 tj[kFusPts];
#pragma unroll
            for (int u = 0; u < kFusPts; ++u) {
                const int n = tt + NT * (kFusPts * c + u);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q >= (1 << qlog)) break;
                    const int vo = (n + N * q) * 8 + fo;
                    v[q][u] = make_float2(
                        __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo, 0, 0)),
                        __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4, 0, 0)));
                    wv8[q][u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wq, (n + N * q) * 4, 0, 0));
                }
                const int to = ((n * j) & (NQ - 1)) * 8;
                tj[u] = make_float2(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(tq, to, 0, 0)),
                                    __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(tq, to + 4, 0, 0)));
            }
#pragma unroll
            for (int u = 0; u < kFusPts; ++u) {
                float2 vq[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q < (1 << qlog)) vq[q] = make_float2(v[q][u].x * wv8[q][u], v[q][u].y * wv8[q][u]);
                float2 y;
                if (qlog == 1) {
                    y = j ? f2sub(vq[0], vq[1]) : f2add(vq[0], vq[1]);
                } else {  // the split's DFT4 over q, output j
                    const float2 e0 = f2add(vq[0], vq[2]), e1 = f2sub(vq[0], vq[2]);
                    const float2 e2 = f2add(vq[1], vq[3]), d = f2mi(f2sub(vq[1], vq[3]));
                    y = j == 0 ? f2add(e0, e2) : j == 2 ? f2sub(e0, e2) : j == 1 ? f2add(e1, d) : f2sub(e1, d);
                }
                a[kFusPts * c + u] = j ? f2mul(y, tj[u]) : y;
            }
        }
    };
    // L2-resident tables first (vmcnt retires in order: the frame's HBM loads queue behind them)
    float2 tp[4];  // W_N^(2^i t), i < 4: P3's bases W_N^(r t) are products of at most four
#pragma unroll
    for (int i = 0; i < 4; ++i) tp[i] = tw[((t0 << i) & (N - 1)) << qlog];
    float2 t2v[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = t0 + NT * i;  // 992 entries: (r - 1) * 32 + k
        t2v[i] = e < 31 * 32 ? tw[(((e >> 5) + 1) * (e & 31)) << (4 + qlog)] : make_float2(0.f, 0.f);
    }
    // work[0] counts claims, work[1] exits: the last workgroup out zeroes both, so the next
    // launch on the stream finds them zero without a memset in between
    auto finish = [&]() {
        __syncthreads();
        if (t0 == 0 && atomicAdd(work + 1, 1) == (int)gridDim.x - 1) {
            atomicExch(work, 0);
            atomicExch(work + 1, 0);
        }
    };
    if (t0 == 0) s_next = atomicAdd(work, 1);
    __syncthreads();
    int w = __builtin_amdgcn_readfirstlane(s_next);
    if (w >= items) {  // uniform: every item is taken
        finish();
        return;
    }
    w = desc(w);
    Item cur = item(w);
    float2 nx[FUS ? 1 : 32];
    if constexpr (!FUS) load_x(cur.xr, 0, nx);
#pragma unroll
    for (int i = 0; i < 2; ++i)
        if (t0 + NT * i < 31 * 32) sm[K::TW2 + t0 + NT * i] = t2v[i];
    const int sw = wf_swz32(t0);  // swz(t + 512 m) = swz(t) + 512 m
#pragma unroll 1
    while (true) {
        // claim the item after this one now: its first frame is prefetched during this one's last
        __syncthreads();  // every wave has read s_next (the item it holds) before it changes
        if (t0 == 0) s_next = atomicAdd(work, 1);
        __syncthreads();
        const int wi = __builtin_amdgcn_readfirstlane(s_next);
        const bool has_next = wi < items;
        const int wn = has_next ? desc(wi) : w;
        const Item nxt = item(wn);
        float acc[32];
#pragma unroll
        for (int m = 0; m < 32; ++m) acc[m] = 0.0f;
#pragma unroll 1
        for (int f = 0; f < cur.nfr; ++f) {
            int t = threadIdx.x;
            asm volatile("" : "+v"(t));
            const int sb = 1 + 6 * f;
            if (f < 2) WF_STAMP(sb);
            float2 a[32];
            if constexpr (FUS) {
                fused_frame(cur.xr, f * cur.hop * 8, __builtin_amdgcn_readfirstlane(w & ((1 << qlog) - 1)), t, a);
            } else {
                {
                    float wv[32];
                    load_w(wv);
#pragma unroll
                    for (int r = 0; r < 32; ++r) a[r] = make_float2(nx[r].x * wv[r], nx[r].y * wv[r]);
                }
                // next frame: this item's, else the next item's first, else nothing (zeros)
                const bool last = f + 1 == cur.nfr;
                load_x(last ? nxt.xr : cur.xr,
                       !last ? (f + 1) * cur.hop * 8 : has_next ? 0 : kWfOob, nx);
            }
            f2dft32(a);
            if (f < 2) WF_STAMP(sb + 1);
            __syncthreads();  // the previous frame's P3 reads (and, at f = 0, the table stores)
#pragma unroll
            for (int k = 0; k < 32; ++k) sm[32 * t + (k ^ (t & 15))] = a[l32_at(k)];
            if (f < 2) WF_STAMP(sb + 2);
            __syncthreads();
            // P2
            {
                const int ts = wf_swz32(t);
#pragma unroll
                for (int r = 0; r < 32; ++r) a[r] = sm[ts + NT * r];
                const int k = t & 31;
                const float2* T = sm + K::TW2 + k;
#pragma unroll
                for (int r = 1; r < 32; ++r) {
                    a[r] = f2mul(a[r], T[(r - 1) * 32]);
                    if ((r & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // <= 8 twiddles live
                }
                f2dft32(a);
                __syncthreads();  // every P2 read before any P2 store
                const int base = (t >> 5) * 1024 + k;
#pragma unroll
                for (int r = 0; r < 32; ++r) sm[wf_swz32(base + 32 * r)] = a[l32_at(r)];
            }
            if (f < 2) WF_STAMP(sb + 3);
            __syncthreads();
            // P3
#pragma unroll
            for (int m = 0; m < 32; ++m) a[m] = sm[sw + NT * m];
            if (f < 2) WF_STAMP(sb + 4);
            float2 tb[16];  // W_N^(r t) from the exact powers of two, at most three products each
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
                    const float2 wt = b ? f2mul32(tb[r], r) : tb[r];
                    c[r] = f2mul(a[b + 2 * r], wt);
                }
                f2dft<16>(c);
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    acc[b + 2 * r] = acc[b + 2 * r] + fmaf(c[r].y, c[r].y, c[r].x * c[r].x);
            }
            if (f < 2) WF_STAMP(sb + 5);
        }
        float* out = partial + (int64_t)w * N;  // = group * (N << qlog) + j * N, or descriptor w
#pragma unroll
        for (int m = 0; m < 32; ++m) out[t0 + NT * m] = acc[m];
        if (!has_next) break;
        w = wn;
        cur = nxt;
    }
    WF_STAMP(13);
    WF_RSTAMP(15);
    finish();
}

// ---- wf_fft_q16: N = 16384 as 16 x 16 x 64, 1024 threads of 16 points -------------------------
// Four waves per SIMD (the LDS exchanges reach their full rate there; at two per SIMD the 8-B
// stores ran at about half of it) and the window taps resident in registers.
//   n = n1 + 1024 n2, n1 = n1a + 64 n1b, n1a = q + 4 m;   k = k2 + 16 (k1b + 16 (c + 16 d)).
//  P1 (thread n1 = t):  x[t + 1024 n2] w -> DFT16 over n2 -> * W_N^(t k2) -> image[k2 1024 + t]
//  P2 (t = n1a + 64 k2): image[k2 1024 + n1a + 64 n1b] -> DFT16 over n1b -> * W_1024^(n1a k1b)
//                       -> image[k2 S2 + k1b R2 + n1a]
//  P3 (t = q + 4 k1b + 64 k2): image[k2 S2 + k1b R2 + q + 4 m] -> DFT16 over m
//                       -> * W_64^(q c) -> DFT4 over q across the lane quad (DPP) -> |X|^2.
// Every image access is one conflict-free 8-B LDS instruction per point.  The quad's DFT4 leaves
// lane q with bin d = {0, 2, 3, 1}[q] up to a sign, which |X|^2 does not see (q16_bin(c 1024 + t)
// is thread t's bin c).  At a group's end the sums are transposed to bin order through the LDS,
// so partial rows are natural-order rows like every kernel's.  Frames, groups, the dynamic
// dealing and the tail split are wf_fft_l32's.
struct WfQ16 {
    static constexpr int LOGN = 14, N = 1 << LOGN, NT = 1024;
    // P2 -> P3 image: rows of 64 padded to R2 = 68 (k1b rows 4 banks apart: P3's reads, a quad
    // per k1b row, are conflict-free with immediate offsets), k2 blocks of S2
    // The tables come first: their reads then take immediate offsets from one base register
    // (the DS offset field is 16 bits).
    // P1's twiddle W_N^(n1 k2) = TA[k2][n1 & 63] * TB[k2][n1 >> 6] (W_N^(n1a k2) W_256^(n1b k2);
    // in registers its bases spilled, and a scratch reload's vmcnt wait drains the prefetch)
    static constexpr int R2 = 68, S2 = 16 * R2;
    static constexpr int TW3 = 0;          // [16][4]:  W_64^(q c)
    static constexpr int TW2 = 64;         // [16][64]: W_1024^(n1a k1b)
    static constexpr int TA = 1088;        // [16][64]: W_N^(n1a k2)
    static constexpr int TB = 2112;        // [16][16]: W_256^(n1b k2)
    static constexpr int IMG = 2368;       // the image: 16 S2 entries
    static constexpr size_t kLds = sizeof(float2) * (IMG + 16 * S2);
};
__host__ __device__ constexpr inline int q16_bin(int p) {
    const int c = p >> 10, t = p & 1023;
    const int q = t & 3, k1b = (t >> 2) & 15, k2 = t >> 6;
    const int d = (0x78 >> (2 * q)) & 3;  // {0, 2, 3, 1}
    return k2 + 16 * k1b + 256 * c + 4096 * d;
}

// LDS position of bin b in wf_fft_q16's group-end transpose: b with bits 0-4 XORed by bits
// 4-6 and 12-13 (the lanes of one store differ in those), a bijection
OWRX_DEV int wf_q16_lswz(int b) { return b ^ (((b >> 4) & 7) | (((b >> 12) & 3) << 3)); }

// wf_fft_q16's butterflies and twiddle products: scalar FP32 (f2dft / f2mul) or packed (dft_r /
// pk_mul: half the instructions, each issuing over twice the cycles; ABL 256, tools/micro A/B)
template <bool PK>
OWRX_DEV void q16_dft16(float2* a) {
    if constexpr (PK) {
        c2 t[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i] = c2_of(a[i]);
        dft_r<16>(t);
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = f2_of(t[i]);
    } else {
        f2dft<16>(a);
    }
}
template <bool PK>
OWRX_DEV float2 q16_mul(float2 a, float2 w) {
    if constexpr (PK)
        return f2_of(pk_mul(c2_of(a), c2_of(w)));
    else
        return f2mul(a, w);
}

template <int CTRL>
OWRX_DEV float dppq(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

// ABL: variant and diagnostic bits (tools/micro; the product picks one).  Ablations: 1 no frame
// loads (the first frame's samples reused), 2 no LDS exchanges, 4 no barriers inside the frame.
// Variants: 8 the next frame's loads spread over the four phases; 32 16-B loads (two adjacent
// samples per lane, regrouped across the wave's halves with v_permlane32_swap, so lane L holds
// n1 = 64 w + 2 (L & 31) + (L >> 5)); 64 the loads issued after the first exchange's LDS stores
// (LDS stores queued behind a wave's just-issued loads waited ~11k cycles, tools/micro/wf_r05.hip
// stamps); 128 the swap's operands reversed (semantics check).
template <int ABL = 0>
__global__ void __launch_bounds__(WfQ16::NT)
wf_fft_q16(const float2* __restrict__ blk, int64_t blk_start, const WfGroup* __restrict__ groups,
           const float* __restrict__ window, const float2* __restrict__ tw,
           float* __restrict__ partial, int items, int* __restrict__ work, int whole, int skip,
           int qlog, int fstride) {
    using K = WfQ16;
    WF_RSTAMP(14);
    WF_STAMP(12);
    constexpr int N = K::N, NT = K::NT;
    constexpr bool kSpread = (ABL & 8) != 0, kW16 = (ABL & 32) != 0, kLate = (ABL & 64) != 0;
    constexpr bool kSwapRev = (ABL & 128) != 0;
    constexpr bool kPk = (ABL & 256) != 0;   // packed FP32 butterflies and twiddle products
    constexpr bool kTbS = (ABL & 512) != 0;  // P1's W_256^(n1b k2) factor wave-uniform (SGPRs), not LDS
    constexpr int kUnits = kW16 ? 8 : 16;  // load instructions per thread per frame
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ int s_next;
    const int t0 = threadIdx.x;
    // P1's point n1 of this thread, and its place in the first image (a swizzle keeps the 16-B
    // variant's stores conflict-free: its 16-lane store groups hold even or odd n1 only)
    const int n1 = kW16 ? (t0 & ~63) + 2 * (t0 & 31) + ((t0 >> 5) & 1) : t0;
    auto swz1 = [](int e) { return kW16 ? e ^ ((e >> 4) & 1) : e; };
    struct Item {
        __amdgpu_buffer_rsrc_t xr;
        int hop, nfr;
    };
    auto desc = [&](int i) { return i < whole ? i : i + skip; };
    // qlog > 0 (N = 16384 << qlog, wf_dif_split first): item w = (group << qlog) + j transforms
    // sub-frame j of its group's frames from the split scratch (as wf_fft_l32 does), tw is the
    // (N << qlog)-point table read at stride 1 << qlog, the window is ones
    auto item = [&](int w) {
        const WfGroup g = groups[w >> qlog];
        Item it;
        it.hop = __builtin_amdgcn_readfirstlane(qlog ? N << qlog : g.hop);
        it.nfr = __builtin_amdgcn_readfirstlane(g.nframes);
        const int g0 = __builtin_amdgcn_readfirstlane(
            qlog ? (int)(((((int64_t)(w >> qlog) * fstride) << qlog) + (w & ((1 << qlog) - 1))) * N)
                 : (int)(g.start - blk_start));
        it.xr = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float2*>(blk + g0), 0,
            (int)(sizeof(float2) * ((int64_t)(it.nfr - 1) * it.hop + N)), 0x00020000);
        return it;
    };
    // raw[2 r], raw[2 r + 1]: point r (n = n1 + 1024 r) once regrouped
    auto load_units = [&](__amdgpu_buffer_rsrc_t xr, int fo, float* raw, int lo, int hi) {
#pragma unroll
        for (int u = lo; u < hi; ++u) {
            if constexpr (kW16) {
                // 16 B at n = 64 w + 2 (L & 31) + 1024 (2 u + (L >> 5))
                const int vo = ((t0 & ~63) + 2 * (t0 & 31) + 1024 * ((t0 >> 5) & 1)) * 8 + fo;
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    raw[4 * u + c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4 * c, u * 2048 * 8, 0));
            } else {
                const int vo = t0 * 8 + fo;
#pragma unroll
                for (int c = 0; c < 2; ++c)
                    raw[2 * u + c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4 * c, u * NT * 8, 0));
            }
        }
    };
    // L2-resident constants first (vmcnt retires in order)
    float wv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) wv[r] = window[n1 + NT * r];
    const float2 t2v = tw[(((t0 & 63) * (t0 >> 6) * 16) & (N - 1)) << qlog];          // [k1b][n1a]
    const float2 t3v = tw[(((t0 & 3) * ((t0 >> 2) & 15) * 256) & (N - 1)) << qlog];   // [c][q], t0 < 64
    const float2 tav = tw[(((t0 & 63) * (t0 >> 6)) & (N - 1)) << qlog];               // [k2][n1a]
    const float2 tbv = tw[(((t0 & 15) * ((t0 >> 4) & 15) * 64) & (N - 1)) << qlog];   // [k2][n1b], t0 < 256
    // kTbS: n1b = t >> 6 is the wave's index, so W_256^(n1b k2) is uniform over the wave
    float2 tbs[16];
    if constexpr (kTbS && !kW16) {
        const int wv6 = __builtin_amdgcn_readfirstlane(t0 >> 6);
#pragma unroll
        for (int r = 1; r < 16; ++r) tbs[r] = tw[((64 * r * wv6) & (N - 1)) << qlog];
    }
    auto finish = [&]() {
        __syncthreads();
        if (t0 == 0 && atomicAdd(work + 1, 1) == (int)gridDim.x - 1) {
            atomicExch(work, 0);
            atomicExch(work + 1, 0);
        }
    };
    if (t0 == 0) s_next = atomicAdd(work, 1);
    __syncthreads();
    int w = __builtin_amdgcn_readfirstlane(s_next);
    if (w >= items) {
        finish();
        return;
    }
    w = desc(w);
    Item cur = item(w);
    float nx[32];
#ifdef OWRX_WF_WSTAMPS
    unsigned long long wst_[12] = {};
#endif
    load_units(cur.xr, 0, nx, 0, kUnits);
    sm[K::TW2 + t0] = t2v;
    sm[K::TA + t0] = tav;
    if (t0 < 256) sm[K::TB + t0] = tbv;
    if (t0 < 64) sm[K::TW3 + t0] = t3v;
    float2* const img = sm + K::IMG;
#pragma unroll 1
    while (true) {
        __syncthreads();
        if (t0 == 0) s_next = atomicAdd(work, 1);
        __syncthreads();
        const int wi = __builtin_amdgcn_readfirstlane(s_next);
        const bool has_next = wi < items;
        const int wn = has_next ? desc(wi) : w;
        const Item nxt = item(wn);
        float acc[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) acc[m] = 0.0f;
#pragma unroll 1
        for (int f = 0; f < cur.nfr; ++f) {
            int t = threadIdx.x;
            asm volatile("" : "+v"(t));
            float2 a[16];
            if (f == 1) WF_STAMP(0);
#define WF_WS(i)                     \
    do {                             \
        if (f == 2) WF_WSTAMP(i);    \
    } while (0)
// (diagnostic builds: the values computed so far are forced before a stamp, or the compiler
// sinks the arithmetic past it)
#ifdef OWRX_WF_WSTAMPS
#define WF_PIN(arr)                                                          \
    do {                                                                     \
        if (f == 2)                                                          \
            for (int pr_ = 0; pr_ < 16; ++pr_)                               \
                asm volatile("" : "+v"(arr[pr_].x), "+v"(arr[pr_].y));        \
    } while (0)
#else
#define WF_PIN(arr) \
    do {            \
    } while (0)
#endif
            WF_WS(0);
#ifdef OWRX_WF_WSTAMPS
            if (f == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            WF_WS(1);
            if constexpr (kW16) {
#pragma unroll
                for (int u = 0; u < 8; ++u)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        // X = raw[4u + c] (lanes < 32: n1 even, j = 2u; lanes >= 32: n1 even,
                        // j = 2u + 1), Y = raw[4u + 2 + c]: swap X's upper half with Y's lower
                        const unsigned xo = __builtin_bit_cast(unsigned, nx[4 * u + c]);
                        const unsigned yo = __builtin_bit_cast(unsigned, nx[4 * u + 2 + c]);
                        if constexpr (!kSwapRev) {
                            const auto r = __builtin_amdgcn_permlane32_swap(xo, yo, false, false);
                            nx[4 * u + c] = __builtin_bit_cast(float, (unsigned)r[0]);
                            nx[4 * u + 2 + c] = __builtin_bit_cast(float, (unsigned)r[1]);
                        } else {
                            const auto r = __builtin_amdgcn_permlane32_swap(yo, xo, false, false);
                            nx[4 * u + 2 + c] = __builtin_bit_cast(float, (unsigned)r[0]);
                            nx[4 * u + c] = __builtin_bit_cast(float, (unsigned)r[1]);
                        }
                    }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = make_float2(nx[2 * r] * wv[r], nx[2 * r + 1] * wv[r]);
            const bool last = f + 1 == cur.nfr;
            const auto lxr = last ? nxt.xr : cur.xr;
            const int lfo = !last ? (f + 1) * cur.hop * 8 : has_next ? 0 : kWfOob;
            constexpr int kQ = kUnits / 4;  // units per spread phase
            if (!(ABL & 1) && !kLate) load_units(lxr, lfo, nx, 0, kSpread ? kQ : kUnits);
            WF_WS(2);
            if (f == 1) WF_STAMP(1);
            // P1
            q16_dft16<kPk>(a);
            {
                int tn = threadIdx.x;
                asm volatile("" : "+v"(tn));
                const int m1 = kW16 ? (tn & ~63) + 2 * (tn & 31) + ((tn >> 5) & 1) : tn;
                const float2* TA = sm + K::TA + (m1 & 63);
                const float2* TB = sm + K::TB + (m1 >> 6);
                if constexpr (kTbS && !kW16) {
#pragma unroll
                    for (int r = 1; r < 16; ++r) a[r] = q16_mul<kPk>(a[r], q16_mul<kPk>(TA[64 * r], tbs[r]));
                } else {
#pragma unroll
                    for (int r = 1; r < 16; ++r) a[r] = q16_mul<kPk>(a[r], q16_mul<kPk>(TA[64 * r], TB[16 * r]));
                }
            }
            if (f == 1) WF_STAMP(2);
            WF_PIN(a);
            WF_WS(3);
            if (!(ABL & 4)) __syncthreads();  // the previous frame's P3 reads (and, at f = 0, the table stores)
            WF_WS(4);
            if (!(ABL & 2)) {
                const int p1 = swz1(n1);
#pragma unroll
                for (int r = 0; r < 16; ++r) img[r * 1024 + p1] = a[r];
            }
            WF_WS(5);
            if (!(ABL & 1) && kLate) load_units(lxr, lfo, nx, 0, kSpread ? kQ : kUnits);
            WF_WS(8);
            if (!(ABL & 4)) __syncthreads();
            if (f == 1) WF_STAMP(3);
            WF_WS(6);
            if (kSpread && !(ABL & 1)) load_units(lxr, lfo, nx, kQ, 2 * kQ);
            // P2
            {
                const int n1a = t & 63, k2 = t >> 6;
                if (!(ABL & 2)) {
                    const int p = k2 * 1024 + swz1(n1a);
#pragma unroll
                    for (int r = 0; r < 16; ++r) a[r] = img[p + 64 * r];
                }
                q16_dft16<kPk>(a);
#pragma unroll
                for (int r = 1; r < 16; ++r) a[r] = q16_mul<kPk>(a[r], sm[K::TW2 + r * 64 + n1a]);
                if (f == 1) WF_STAMP(4);
                WF_PIN(a);
                WF_WS(9);
                if (kSpread && !(ABL & 1)) load_units(lxr, lfo, nx, 2 * kQ, 3 * kQ);
                if (!(ABL & 4)) __syncthreads();  // every P2 read before any P2 store
                if (!(ABL & 2)) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) img[k2 * K::S2 + r * K::R2 + n1a] = a[r];
                }
            }
            if (!(ABL & 4)) __syncthreads();
            if (f == 1) WF_STAMP(5);
            WF_WS(7);
            if (kSpread && !(ABL & 1)) load_units(lxr, lfo, nx, 3 * kQ, 4 * kQ);
            // P3
            {
                const int q = t & 3;
                const int k1b = (t >> 2) & 15, k2 = t >> 6;
                const int base = k2 * K::S2 + k1b * K::R2 + q;
                if (!(ABL & 2)) {
#pragma unroll
                    for (int m = 0; m < 16; ++m) a[m] = img[base + 4 * m];
                }
                q16_dft16<kPk>(a);
#pragma unroll
                for (int c = 1; c < 16; ++c) a[c] = q16_mul<kPk>(a[c], sm[K::TW3 + c * 4 + q]);
                const float s1 = q < 2 ? 1.0f : -1.0f;
                const float s2 = (q == 0 || q == 3) ? 1.0f : -1.0f;
                const bool q3 = q == 3;
                // four bins at a time, each step over all four: the cross-lane moves of one bin
                // fill the others' DPP hazard slots (one bin at a time was a dependent chain of
                // ~10 instructions with s_nops between)
#pragma unroll
                for (int c0 = 0; c0 < 16; c0 += 4) {
                    float vx[4], vy[4], px[4], py[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {  // stage 1: partner q ^ 2
                        px[u] = dppq<0x4E>(a[c0 + u].x);
                        py[u] = dppq<0x4E>(a[c0 + u].y);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float x = fmaf(px[u], s1, a[c0 + u].x);
                        const float y = fmaf(py[u], s1, a[c0 + u].y);
                        vx[u] = q3 ? y : x;  // lane 3: * -i
                        vy[u] = q3 ? -x : y;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {  // stage 2: partner q ^ 1
                        px[u] = dppq<0xB1>(vx[u]);
                        py[u] = dppq<0xB1>(vy[u]);
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float x = fmaf(px[u], s2, vx[u]);
                        const float y = fmaf(py[u], s2, vy[u]);
                        acc[c0 + u] = acc[c0 + u] + fmaf(y, y, x * x);
                    }
                }
            }
            if (f == 1) WF_STAMP(6);
#ifdef OWRX_WF_WSTAMPS
            if (f == 2)
                for (int pr_ = 0; pr_ < 16; ++pr_) asm volatile("" : "+v"(acc[pr_]));
#endif
            WF_WS(10);
#undef WF_WS
        }
        // group end: the |X|^2 sums go back to bin order through the (now free) image, so the
        // partial row is stored coalesced and in natural order (wf_finalize and the tail split
        // as for every kernel); the swizzle keeps both LDS passes conflict-free
        __syncthreads();  // every P3 read of the image done
        {
            // (an opaque thread index: hoisted out of the frame loop, these addresses spilled)
            int tt = threadIdx.x;
            asm volatile("" : "+v"(tt));
            float* const limg = reinterpret_cast<float*>(img);
            const int k1b = (tt >> 2) & 15, k2 = tt >> 6;
            const int d = (0x78 >> (2 * (tt & 3))) & 3;
#pragma unroll
            for (int c = 0; c < 16; ++c) limg[wf_q16_lswz(k2 + 16 * k1b + 256 * c + 4096 * d)] = acc[c];
            __syncthreads();
            float* out = partial + (int64_t)w * N;
#pragma unroll
            for (int j = 0; j < 16; ++j) out[tt + NT * j] = limg[wf_q16_lswz(tt + NT * j)];
        }
        if (!has_next) break;
        w = wn;
        cur = nxt;
    }
    WF_STAMP(13);
    WF_RSTAMP(15);
#ifdef OWRX_WF_WSTAMPS
    if ((t0 & 63) == 0 && blockIdx.x < 256)
        for (int i = 0; i < 12; ++i) g_wf_wstamp[blockIdx.x][t0 >> 6][i] = wst_[i];
#endif
    finish();
}

// the product's variant: the next frame's loads after the first exchange's stores, spread
// over the phases (tools/micro/wf_r05.hip: 0.29 vs 0.25 of HBM for wf_fft_l32 at 3840 C3 frames),
// and P1's W_256^(n1b k2) factor from SGPRs (round 6, +512: half of P1's LDS table reads gone,
// the same products, bit-identical rows; tools/micro/wf_r06.hip 0.258 vs 0.256 at 3480 frames,
// 0.249 vs 0.244 at 1740).  The packed-FP32 butterflies (+256) measured no faster: 0.260 / 0.248,
// and slower as VALU alone (0.405 vs 0.427; profiles/r06_wf_micro_a.txt, profiles/r06_fma_rate.txt)
constexpr int kWfQ16 = 584;

// ---- FFT sizes above one CU's LDS (32768, 65536): decimation-in-frequency split ------------
// N = Q * 16384 (Q = 2, 4): X[Q k + j] = sum_n y_j[n] W_16384^(n k) with
//   y_j[n] = W_N^(n j) * sum_q w[n + 16384 q] x[n + 16384 q] W_Q^(q j),   n < 16384,
// so one frame becomes Q independent 16384-point sub-frames that wf_fft_l32 transforms (the
// |X|^2 of bins Q k + j lands j-major in the partial row; wf_finalize reads it back in bin
// order).  wf_dif_split: one thread per (frame, n) -- reads the frame once (Q loads), writes the
// Q sub-frames to the scratch (frame f of group g at ((g fstride + f) Q + j) 16384).
template <int QLOG>
__global__ void __launch_bounds__(256)
wf_dif_split(const float2* __restrict__ blk, int64_t blk_start, const WfGroup* __restrict__ groups,
             const float* __restrict__ window, const float2* __restrict__ tw, int fstride,
             float2* __restrict__ y) {
#pragma clang fp contract(off)  // (wf_fft_l32<true> forms the same values on load: same roundings)
    constexpr int M = 16384, Q = 1 << QLOG, N = M << QLOG;
    const int n = blockIdx.x * 256 + threadIdx.x;
    const int f = blockIdx.y;
    const WfGroup g = groups[blockIdx.z];
    if (f >= g.nframes) return;
    const float2* x = blk + (g.start - blk_start) + (int64_t)f * g.hop;
    float2 v[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const float2 a = x[n + q * M];
        const float w = window[n + q * M];
        v[q] = make_float2(a.x * w, a.y * w);
    }
    float2 s[Q];
    if constexpr (Q == 2) {
        s[0] = f2add(v[0], v[1]);
        s[1] = f2sub(v[0], v[1]);
    } else {
        static_assert(Q == 4, "split");
        // DFT4 over q: s_j = sum_q v_q (-i)^(q j)
        const float2 t0 = f2add(v[0], v[2]), t1 = f2sub(v[0], v[2]);
        const float2 t2 = f2add(v[1], v[3]), d = f2mi(f2sub(v[1], v[3]));
        s[0] = f2add(t0, t2);
        s[2] = f2sub(t0, t2);
        s[1] = f2add(t1, d);
        s[3] = f2sub(t1, d);
    }
    float2* o = y + ((int64_t)blockIdx.z * fstride + f) * N + n;
    o[0] = s[0];
#pragma unroll
    for (int j = 1; j < Q; ++j) o[j * M] = f2mul(s[j], tw[(n * j) & (N - 1)]);
}

// ---- the four-step form (N = 32768, 65536; OWRX_WF_KERNEL=fourstep, A/B) ------------------
// N = N1 * N2, n = N2*n1 + n2, k = k1 + N1*k2:
//   X[k1 + N1 k2] = sum_n2 W_N2^(n2 k2) * W_N^(n2 k1) * sum_n1 x[N2 n1 + n2] W_N1^(n1 k1).
// wf_fft4_cols: 32 columns n2 of one frame per workgroup -- windowed loads (32 consecutive
//   samples = 256 B per n1), N1-point FFTs in LDS, twiddle W_N^(n2 k1), store Y[k1][n2]
//   (256 B runs).  wf_fft4_rows: 32 rows k1 per workgroup -- contiguous loads of Y, N2-point
//   FFTs in LDS, |X|^2 stored in natural bin order (32 consecutive bins = 128 B runs).  Y is a
//   per-frame scratch of N cf32 (L2/HBM); the frame is read once from HBM like the LDS kernel.
constexpr int kF4Rows = 32;    // columns (pass 1) / rows (pass 2) per workgroup
constexpr int kF4Threads = 256;

template <int LOG1, int LOG2>
__global__ void __launch_bounds__(kF4Threads)
wf_fft4_cols(const float2* __restrict__ blk, int64_t blk_start, const WfGroup* __restrict__ groups,
             const float* __restrict__ window, const float2* __restrict__ tw,
             float2* __restrict__ Y) {
    constexpr int N1 = 1 << LOG1, N2 = 1 << LOG2, N = N1 * N2, C = kF4Rows, RS = N1 + 1;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int tid = threadIdx.x;
    const int c0 = blockIdx.x * C;
    const WfGroup g = groups[blockIdx.y];
    const float2* x = blk + (g.start - blk_start);
    for (int i = tid; i < N1 * C; i += kF4Threads) {
        const int n1 = i / C, cc = i % C;
        const int n = N2 * n1 + c0 + cc;
        const float2 v = x[n];
        const float w = window[n];
        sm[cc * RS + n1] = make_float2(v.x * w, v.y * w);
    }
    __syncthreads();
    lds_fft_rows<LOG1, C, kF4Threads>(sm, RS, tw, N2);
    float2* y = Y + (int64_t)blockIdx.y * N;
    for (int i = tid; i < N1 * C; i += kF4Threads) {
        const int k1 = i / C, cc = i % C;
        const int n2 = c0 + cc;
        y[k1 * N2 + n2] = cmul(sm[cc * RS + k1], tw[(n2 * k1) & (N - 1)]);
    }
}

template <int LOG1, int LOG2>
__global__ void __launch_bounds__(kF4Threads)
wf_fft4_rows(const float2* __restrict__ Y, const float2* __restrict__ tw,
             float* __restrict__ partial) {
    constexpr int N1 = 1 << LOG1, N2 = 1 << LOG2, N = N1 * N2, R = kF4Rows, RS = N2 + 1;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * R;
    const float2* y = Y + (int64_t)blockIdx.y * N;
    for (int i = tid; i < R * N2; i += kF4Threads) {
        const int r = i / N2, n2 = i % N2;
        sm[r * RS + n2] = y[(r0 + r) * N2 + n2];
    }
    __syncthreads();
    lds_fft_rows<LOG2, R, kF4Threads>(sm, RS, tw, N1);
    float* out = partial + (int64_t)blockIdx.y * N;
    for (int i = tid; i < R * N2; i += kF4Threads) {
        const int r = i % R, k2 = i / R;
        const float2 X = sm[r * RS + k2];
        out[r0 + r + N1 * k2] = X.x * X.x + X.y * X.y;
    }
}

// Each thread sums four consecutive positions of the partial rows (16-B loads; a position is
// bin i's place in a partial row: natural, or j-major after the DIF split, bin Q k + j at
// j (N / Q) + k).  The carried accumulator is kept in position
// order too.
OWRX_DEV float4 f4add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__global__ void __launch_bounds__(256)
wf_finalize(const float* __restrict__ partial, const WfRow* __restrict__ rows,
            const float* __restrict__ carry_in, float* __restrict__ carry_out, int N,
            float add_corr, int adpcm, int16_t* __restrict__ s16_out,
            float* __restrict__ f32_out, int qlog, const WfGroup* __restrict__ groups,
            int ngroups, int skip) {
#pragma clang fp contract(off)
    const int p0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
    if (p0 >= N) return;
    const WfRow r = rows[blockIdx.y];
    float4 s = r.use_carry ? *reinterpret_cast<const float4*>(carry_in + p0)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
    auto at = [&](const float* base, int64_t row) {
        return *reinterpret_cast<const float4*>(base + row * N);
    };
    // the groups' partials in order (the row's summation order); loads batched 16 deep
    const float* pp = partial + (int64_t)r.first_group * N + p0;
    // groups [ngroups - skip, ngroups) were transformed frame by frame (wf_fft_l32's tail
    // split): their frames' partial rows follow the groups', folded here in frame order into the
    // group's sum first, as the workgroup would have
    const int g_split = ngroups - skip;
    const int n_whole = max(0, min(r.ngroups, g_split - r.first_group));
    int gi = 0;
    for (; gi + 16 <= n_whole; gi += 16) {
        float4 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = at(pp, gi + u);
#pragma unroll
        for (int u = 0; u < 16; ++u) s = f4add(s, v[u]);
    }
    if (gi + 8 <= n_whole) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = at(pp, gi + u);
#pragma unroll
        for (int u = 0; u < 8; ++u) s = f4add(s, v[u]);
        gi += 8;
    }
    for (; gi < n_whole; ++gi) s = f4add(s, at(pp, gi));
    if (gi < r.ngroups) {
        // (loads issued eight groups' frame counts and up to four frames at a time: a serial
        // chain of dependent L2 reads per group cost tens of us per launch)
        int f0 = r.pad;  // the row's first split frame's descriptor (host-computed)
        for (; gi < r.ngroups; gi += 8) {
            int nfv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                nfv[u] = gi + u < r.ngroups ? groups[r.first_group + gi + u].nframes : 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int nf = nfv[u];
                if (nf == 0) break;
                const float* fp = partial + (int64_t)f0 * N + p0;
                float4 v[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = q < nf ? at(fp, q) : make_float4(0.f, 0.f, 0.f, 0.f);
                float4 g = v[0];
#pragma unroll
                for (int q = 1; q < 4; ++q)
                    if (q < nf) g = f4add(g, v[q]);
                for (int q = 4; q < nf; ++q) g = f4add(g, at(fp, q));
                s = f4add(s, g);
                f0 += nf;
            }
        }
    }
    if (!r.complete) {
        *reinterpret_cast<float4*>(carry_out + p0) = s;
        return;
    }
    const float sv[4] = {s.x, s.y, s.z, s.w};
    const int nq = N >> qlog;  // positions per sub-row
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int p = p0 + c;
        const int i = qlog ? ((p % nq) << qlog) + p / nq : p;  // the position's bin
        const float lg = log10f(sv[c]);
        const float t = 10.0f * lg;
        const float db = t + add_corr;
        const int o = (i + N / 2) & (N - 1);  // FftSwap
        if (adpcm)
            s16_out[(int64_t)r.out_index * N + o] = db_to_s16(db);
        else
            f32_out[(int64_t)r.out_index * N + o] = db;
    }
}

// FftAdpcm: 10 copies of the first value (COMPRESS_FFT_PAD_N, htdocs/openwebrx.js:845), then
// the row; fresh codec state per row; low nibble first.  Row-parallel exact encoder: one
// workgroup per row, the row (10 pad samples +
// N bins) staged in LDS and encoded by the speculative segment-parallel encoder of
// adpcm_spec.h (bit-identical to the sequential FftAdpcm restatement, oracle
// orc_fft_adpcm_row); rows longer than kRowWin samples go window by window.  Waterfall rows
// re-merge after ~100-900 samples from a guessed start (index 30 measured fastest), so the
// Jacobi repair converges in a few rounds.
constexpr int kRowWin = 16400;

__global__ void __launch_bounds__(kSpecThreads)
wf_adpcm_rows_spec(const int16_t* __restrict__ s16, int N, int nrows, uint8_t* __restrict__ out,
                   int row_bytes) {
    extern __shared__ __align__(16) uint8_t smem[];
    SpecLds<kRowWin>& L = *reinterpret_cast<SpecLds<kRowWin>*>(smem);
    const int tid = threadIdx.x;
    for (int i = tid; i < 89; i += kSpecThreads) L.T[i] = kAdpcmStep[i];
    adpcm_rem_fill(L.NSR, tid, kSpecThreads);
    const int M = N + 10;
    // rows dealt round-robin over a grid that fits its CUs at once (launch_wf_adpcm)
    for (int row = blockIdx.x; row < nrows; row += gridDim.x) {
    const int16_t* x = s16 + (int64_t)row * N;
    uint8_t* o = out + (int64_t)row * row_bytes;
    uint32_t state = 0;  // FftAdpcm restarts every row at (index 0, predictor 0)
    for (int w0 = 0; w0 < M; w0 += kRowWin) {
        const int nw = min(kRowWin, M - w0);
        const SpecGeom gm = spec_geom(nw, 64);
        __syncthreads();
        for (int i = tid; i < nw; i += kSpecThreads) {
            const int t = w0 + i;
            L.x[spec_at(gm, i)] = t < 10 ? x[0] : x[t - 10];
        }
        __syncthreads();
        adpcm_spec_window(L, nw, gm, state, 30);
        __syncthreads();
        for (int i = tid; i < nw / 2; i += kSpecThreads)
            o[w0 / 2 + i] = (uint8_t)((L.code[spec_at(gm, 2 * i)] & 15) |
                                      (L.code[spec_at(gm, 2 * i + 1)] << 4));
        state = L.traj[spec_at(gm, nw - 1)];
    }
    }
}

// host launch helpers -------------------------------------------------------------------
template <int LOGN>
static hipError_t launch_fft_r16(const float2* blk, int64_t blk_start, const WfGroup* groups,
                                 int ngroups, const float* window, const float2* tw,
                                 float* partial, hipStream_t st) {
    using K = WfR16<LOGN>;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)wf_fft_r16<LOGN>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)K::kLds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(wf_fft_r16<LOGN>, dim3(ngroups), dim3(K::NT), K::kLds, st, blk, blk_start,
                       groups, window, tw, partial);
    return hipGetLastError();
}

template <int LOGN>
static hipError_t launch_fft_t(const float2* blk, int64_t blk_start, const WfGroup* groups,
                               int ngroups, const float* window, const float2* tw,
                               float* partial, hipStream_t st) {
    constexpr int N = 1 << LOGN;
    constexpr int NT = (N / 4 < 1024) ? N / 4 : 1024;
    const size_t lds = sizeof(float2) * N;
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)wf_fft_power<LOGN>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(wf_fft_power<LOGN>, dim3(ngroups), dim3(NT), lds, st, blk, blk_start,
                       groups, window, tw, partial);
    return hipGetLastError();
}

template <int LOG1, int LOG2>
static hipError_t launch_fft4_t(const float2* blk, int64_t blk_start, const WfGroup* groups,
                                int ngroups, const float* window, const float2* tw,
                                float* partial, float2* scratch, hipStream_t st) {
    constexpr int N1 = 1 << LOG1, N2 = 1 << LOG2;
    const size_t lds1 = sizeof(float2) * kF4Rows * (N1 + 1);
    const size_t lds2 = sizeof(float2) * kF4Rows * (N2 + 1);
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)wf_fft4_cols<LOG1, LOG2>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)wf_fft4_rows<LOG1, LOG2>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (!scratch) return hipErrorInvalidValue;
    hipLaunchKernelGGL((wf_fft4_cols<LOG1, LOG2>), dim3(N2 / kF4Rows, ngroups), dim3(kF4Threads),
                       lds1, st, blk, blk_start, groups, window, tw, scratch);
    hipLaunchKernelGGL((wf_fft4_rows<LOG1, LOG2>), dim3(N1 / kF4Rows, ngroups), dim3(kF4Threads),
                       lds2, st, scratch, tw, partial);
    return hipGetLastError();
}

// N = 16384: wf_fft_q16 (OWRX_WF_KERNEL=l32: the round-4 radix-32 kernel, =r16 the radix-16 one)
// (A/B); 1024 <= N <= 8192: radix 16.  (A half-frame kernel with two workgroups per CU,
// wf_fft_h2, measured 68 vs 50 us per 960 C3 frames, its loads exposed: removed, in the history
// before this file's round-4 cleanup.)
static int wf_n16k_kernel() {  // 0: q16 (default), 1: l32, 2: r16
    static const int v = [] {
        const char* s = getenv("OWRX_WF_KERNEL");
        return s && strcmp(s, "r16") == 0 ? 2 : s && strcmp(s, "l32") == 0 ? 1 : 0;
    }();
    return v;
}
static bool wf_force_r16() { return wf_n16k_kernel() == 2; }

// N = 16384 on a dealt whole-frame kernel (q16 or l32: groups, tail split)
bool wf_uses_l32(int logn) { return logn == 14 && wf_n16k_kernel() != 2; }
// frames per group of the N = 16384 dealt kernels: 8 for q16 (its group-end transpose and partial
// row amortise over twice the frames; 0.291 vs 0.275 of HBM at 3840 C3 frames in the micro), 4
// for l32
int wf_default_fpg(int logn) { return logn == 14 && wf_n16k_kernel() == 0 ? 8 : 4; }

// N = 32768, 65536: the DIF split onto wf_fft_l32 (OWRX_WF_KERNEL=fourstep: the four-step, A/B)
bool wf_uses_split(int logn) {
    static const bool fourstep = [] {
        const char* s = getenv("OWRX_WF_KERNEL");
        return s && strcmp(s, "fourstep") == 0;
    }();
    return (logn == 15 || logn == 16) && !fourstep;
}

static hipError_t launch_fft_l32(const float2* blk, int64_t blk_start, const WfGroup* groups,
                                 int ngroups, const float* window, const float2* tw,
                                 float* partial, int* work, int cus, hipStream_t st, int qlog = 0,
                                 int fstride = 0, int skip = 0, int tail = 0, bool fus = false) {
    static bool attr = false;
    if (!attr) {
        for (const void* k : {(const void*)wf_fft_l32<false>, (const void*)wf_fft_l32<true>}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)WfL32::kLds);
            if (e != hipSuccess) return e;
        }
        attr = true;
    }
    if (fus && !qlog) return hipErrorInvalidValue;
    if (!work || skip < 0 || skip > ngroups || (qlog && (skip || tail))) return hipErrorInvalidValue;
    // items: the whole groups, then the split groups' frames (descriptors ngroups ..)
    const int whole = (ngroups - skip) << qlog;
    const int items = whole + tail;
    // one workgroup per CU (the 136 KiB image), at most one per item
    const int grid = std::max(1, std::min(items, cus));
    if (fus)
        hipLaunchKernelGGL(wf_fft_l32<true>, dim3(grid), dim3(WfL32::NT), WfL32::kLds, st, blk,
                           blk_start, groups, window, tw, partial, qlog, fstride, items, work, whole,
                           skip);
    else
        hipLaunchKernelGGL(wf_fft_l32<false>, dim3(grid), dim3(WfL32::NT), WfL32::kLds, st, blk,
                           blk_start, groups, window, tw, partial, qlog, fstride, items, work, whole,
                           skip);
    return hipGetLastError();
}

// the tail split of a wf_fft_l32 launch of `ngroups` groups on `cus` CUs: how many of the last
// groups go frame by frame.  The workgroups placed at once on a CU-masked queue are fewer than
// its CUs (measured 227-230 of 240 for the engine's stream-A mask: the dispatcher's per-engine
// share), so a launch of one item per CU ran its last items in a second round, doubling its time
// (89 vs 52 us per 960 C3 frames); the groups that would start a partial last round, plus a
// 16th of a round, are dealt as single frames instead.  0 for the other kernels.
// the workgroups a masked queue holds at once: ~15/16 of its CUs (measured 227-230 of 240)
static int wf_held(int cus) { return cus - cus / 16; }

int wf_round_frames(int logn, int cus, int fpg) {
    return logn == 14 && wf_n16k_kernel() != 2 ? wf_held(cus) * std::max(1, fpg) : 0;
}

int wf_tail_split(int logn, int ngroups, int cus, int64_t frames, int fpg) {
    if (logn != 14 || wf_n16k_kernel() == 2 || cus < 8 || ngroups < 2) return 0;
    static const int mode = [] {
        const char* s = getenv("OWRX_WF_TAIL");
        return s ? atoi(s) : -1;
    }();
    if (mode == 0) return 0;
    // the groups past the last full round of the held workgroups, plus a 16th of a round, go
    // frame by frame.  A launch whose frames end within an eighth of a round of a whole number of
    // rounds keeps its groups whole: its last round is nearly full, and the split's per-frame
    // partial rows (wf_finalize reads them all back) cost more than the idle tail (3 480 frames
    // in situ at C3: 0.245 of HBM whole vs 0.22 split; 3 848 frames: 0.206 whole vs 0.233 split,
    // profiles/r05_wf_tail_batch_ab.txt)
    const int held = wf_held(cus);
    if (mode < 0 && frames > 0 && fpg > 0) {
        const double r = (double)frames / ((double)held * fpg);
        if (r >= 1.0 && r - std::floor(r) < 0.125) return 0;
    }
    const int lo = held - cus / 16;
    if (ngroups <= lo) return 0;
    const int s = ngroups <= held ? ngroups - lo : ngroups % held + cus / 16;
    return std::min(s, ngroups);
}

static hipError_t launch_fft_q16(const float2* blk, int64_t blk_start, const WfGroup* groups,
                                 int ngroups, const float* window, const float2* tw,
                                 float* partial, int* work, int cus, hipStream_t st, int skip,
                                 int tail, int qlog, int fstride);
// N = 16384 << QLOG: the split into sub-frames, then wf_fft_l32 on them (window of ones: the
// split applied the frame's window); or, OWRX_WF_FUSED=1 (A/B, read at every launch),
// wf_fft_l32<true> forming the sub-frames on load without the scratch.  Rows bit-identical; the
// fused form measured slower at C4 (0.068 vs 0.091-0.094 of HBM, profiles/r06_wf_fused_split_ab.txt):
// a frame's four quarters, window taps and twiddles do not fit the registers beside the FFT's, so
// its loads go two points at a time with their latency exposed, where the split streams them.
bool wf_split_fused() {
    const char* s = getenv("OWRX_WF_FUSED");
    return s && strcmp(s, "1") == 0;
}
template <int QLOG>
static hipError_t launch_fft_split(const float2* blk, int64_t blk_start, const WfGroup* groups,
                                   int ngroups, int fpg, const float* window, const float* ones,
                                   const float2* tw, float* partial, float2* scratch, int* work,
                                   int cus, hipStream_t st) {
    if (fpg < 1) return hipErrorInvalidValue;
    if (wf_split_fused())
        return launch_fft_l32(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st,
                              QLOG, fpg, 0, 0, true);
    if (!scratch || !ones) return hipErrorInvalidValue;
    // the sub-frames on wf_fft_q16 (its qlog form), or wf_fft_l32 with OWRX_WF_SUB=l32 (A/B):
    // C4 0.0965-0.0968 vs 0.0928-0.0935 of HBM (profiles/r06_wf_sub_q16_ab.txt)
    // (read at every launch, as OWRX_WF_FUSED: the fused form's rows test compares against l32)
    const char* sv = getenv("OWRX_WF_SUB");
    const bool sub_q16 = !(sv && strcmp(sv, "l32") == 0);
    hipLaunchKernelGGL(wf_dif_split<QLOG>, dim3(16384 / 256, fpg, ngroups), dim3(256), 0, st, blk,
                       blk_start, groups, window, tw, fpg, scratch);
    if (sub_q16)
        return launch_fft_q16(scratch, 0, groups, ngroups, ones, tw, partial, work, cus, st, 0, 0,
                              QLOG, fpg);
    return launch_fft_l32(scratch, 0, groups, ngroups, ones, tw, partial, work, cus, st, QLOG, fpg);
}


static hipError_t launch_fft_q16(const float2* blk, int64_t blk_start, const WfGroup* groups,
                                 int ngroups, const float* window, const float2* tw,
                                 float* partial, int* work, int cus, hipStream_t st, int skip,
                                 int tail, int qlog, int fstride) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)wf_fft_q16<kWfQ16>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)WfQ16::kLds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (!work || skip < 0 || skip > ngroups || tail < 0 || (qlog && (skip || tail)))
        return hipErrorInvalidValue;
    const int whole = (ngroups - skip) << qlog;
    const int items = whole + tail;
    // one 1024-thread workgroup per CU (the 147 KiB LDS image), at most one per item
    const int grid = std::max(1, std::min(items, cus));
    hipLaunchKernelGGL(wf_fft_q16<kWfQ16>, dim3(grid), dim3(WfQ16::NT), WfQ16::kLds, st, blk,
                       blk_start, groups, window, tw, partial, items, work, whole, skip, qlog,
                       fstride);
    return hipGetLastError();
}

template <int LOGN>
static hipError_t launch_fft_sel(const float2* blk, int64_t blk_start, const WfGroup* groups,
                                 int ngroups, const float* window, const float2* tw, float* partial,
                                 int* work, int cus, hipStream_t st, int skip, int tail) {
    if constexpr (LOGN == 14) {
        if (wf_n16k_kernel() == 0)
            return launch_fft_q16(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st,
                                  skip, tail, 0, 0);
        if (!wf_force_r16())
            return launch_fft_l32(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st,
                                  0, 0, skip, tail);
    }
    return launch_fft_r16<LOGN>(blk, blk_start, groups, ngroups, window, tw, partial, st);
}


hipError_t launch_wf_fft(int logn, const float2* blk, int64_t blk_start, const WfGroup* groups,
                         int ngroups, int fpg, const float* window, const float* ones,
                         const float2* tw, float* partial, float2* scratch, int* work, int cus,
                         hipStream_t st, int skip, int tail) {
    if ((skip || tail) && logn != 14) return hipErrorInvalidValue;
    if (logn == 14) return launch_fft_sel<14>(blk, blk_start, groups, ngroups, window, tw, partial,
                                              work, cus, st, skip, tail);
    if (wf_uses_split(logn))
        return logn == 15 ? launch_fft_split<1>(blk, blk_start, groups, ngroups, fpg, window, ones, tw,
                                                partial, scratch, work, cus, st)
                          : launch_fft_split<2>(blk, blk_start, groups, ngroups, fpg, window, ones, tw,
                                                partial, scratch, work, cus, st);
    switch (logn) {
        case 8: return launch_fft_t<8>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 9: return launch_fft_t<9>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 10: return launch_fft_sel<10>(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st, 0, 0);
        case 11: return launch_fft_sel<11>(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st, 0, 0);
        case 12: return launch_fft_sel<12>(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st, 0, 0);
        case 13: return launch_fft_sel<13>(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st, 0, 0);
        case 14: return launch_fft_sel<14>(blk, blk_start, groups, ngroups, window, tw, partial, work, cus, st, 0, 0);
        case 15: return launch_fft4_t<7, 8>(blk, blk_start, groups, ngroups, window, tw, partial,
                                            scratch, st);
        case 16: return launch_fft4_t<8, 8>(blk, blk_start, groups, ngroups, window, tw, partial,
                                            scratch, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_wf_finalize(const float* partial, const WfRow* rows, int nrows,
                              const float* carry_in, float* carry_out, int N, float add_corr,
                              int adpcm, int16_t* s16_out, float* f32_out, hipStream_t st,
                              const WfGroup* groups, int ngroups, int skip) {
    int logn = 0;
    while ((1 << logn) < N) ++logn;
    // partial rows sub-frame-major after the DIF split (Q = N / 16384)
    const int qlog = wf_uses_split(logn) ? logn - 14 : 0;
    if (N % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wf_finalize, dim3((N / 4 + 255) / 256, nrows), dim3(256), 0, st, partial,
                       rows, carry_in, carry_out, N, add_corr, adpcm, s16_out, f32_out, qlog,
                       groups, ngroups, skip);
    return hipGetLastError();
}

// grid: at most `wgs` workgroups (2 x the row queue's CUs), rows looped inside.  A grid of one
// workgroup per row kept workgroups waiting for CUs, and while they waited the command
// processor's pipe dispatched nothing else: stream R's output gathers, which share that pipe
// (engine.hip create_streams), stalled 0.4-0.85 ms once per waterfall batch
// (profiles/r04_rows_grid_ab.txt).
hipError_t launch_wf_adpcm(const int16_t* s16, int N, int nrows, uint8_t* out, int row_bytes,
                           int wgs, hipStream_t st) {
    const size_t lds = sizeof(SpecLds<kRowWin>);
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)wf_adpcm_rows_spec,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    if (nrows <= 0) return hipSuccess;
    const int grid = wgs > 0 ? std::min(nrows, wgs) : nrows;
    hipLaunchKernelGGL(wf_adpcm_rows_spec, dim3(grid), dim3(kSpecThreads), lds, st, s16, N,
                       nrows, out, row_bytes);
    return hipGetLastError();
}

}  // namespace owrx
