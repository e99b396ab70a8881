// kernels_waterfall.hip -- FftChain on CDNA4 (csdr/chain/fft.py:25-96, driven by
// owrx/fft.py:36-59): Fft(size=N, every_n_samples=hop) -> LogAveragePower(add_db, N, avg)
// -> FftSwap -> FftAdpcm.
//
// wf_fft_power: one workgroup (N/4 threads, <= 1024) per group of consecutive frames of one
//   waterfall row.  Each frame: coalesced cf32 load * Hamming window -> LDS (N complex,
//   128 KiB at N = 16384, one workgroup per CU), Stockham radix-4 passes (plus one radix-2
//   pass for odd log2 N) in place through registers, twiddles from an L2-resident table;
//   |X|^2 accumulated in registers across the group's frames, written once per group.
//   Bound: HBM (8 B of IQ per input sample; frames overlap by N - hop and the overlap is
//   re-read from L2).
// wf_finalize: sums each row's group partials in a fixed order onto the carried accumulator
//   (rows span blocks), 10*log10 + add_db correction, fftshift, quantise (short)(dB*100).
// wf_adpcm_rows_spec: FftAdpcm (IMA-ADPCM of each padded row), one workgroup per row,
//   segment-parallel and exact (adpcm_spec.h).
#include "adpcm_spec.h"
#include "fft_lds.h"
#include "owrx_types.h"

namespace owrx {

OWRX_DEV float2 ld2(const float2* p) { return *p; }

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

// ---- FFT sizes above one CU's LDS (32768, 65536): four-step, two launches ------------------
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

__global__ void __launch_bounds__(256)
wf_finalize(const float* __restrict__ partial, const WfRow* __restrict__ rows,
            const float* __restrict__ carry_in, float* __restrict__ carry_out, int N,
            float add_corr, int adpcm, int16_t* __restrict__ s16_out,
            float* __restrict__ f32_out) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const WfRow r = rows[blockIdx.y];
    float s = r.use_carry ? carry_in[i] : 0.0f;
    for (int gi = 0; gi < r.ngroups; ++gi) s += partial[(int64_t)(r.first_group + gi) * N + i];
    if (!r.complete) {
        carry_out[i] = s;
        return;
    }
    const float lg = log10f(s);
    const float t = 10.0f * lg;
    const float db = t + add_corr;
    const int o = (i + N / 2) & (N - 1);   // FftSwap
    if (adpcm)
        s16_out[(int64_t)r.out_index * N + o] = db_to_s16(db);
    else
        f32_out[(int64_t)r.out_index * N + o] = db;
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
    const int row = blockIdx.x;
    for (int i = tid; i < 89; i += kSpecThreads) L.T[i] = kAdpcmStep[i];
    adpcm_tab_fill(L.NS, tid, kSpecThreads);
    const int M = N + 10;
    const int16_t* x = s16 + (int64_t)row * N;
    uint8_t* o = out + (int64_t)row * row_bytes;
    uint32_t state = 0;  // FftAdpcm restarts every row at (index 0, predictor 0)
    for (int w0 = 0; w0 < M; w0 += kRowWin) {
        const int nw = min(kRowWin, M - w0);
        __syncthreads();
        for (int i = tid; i < nw; i += kSpecThreads) {
            const int t = w0 + i;
            L.x[i] = t < 10 ? x[0] : x[t - 10];
        }
        __syncthreads();
        adpcm_spec_window(L, nw, state, 30, 64);
        __syncthreads();
        for (int i = tid; i < nw / 2; i += kSpecThreads)
            o[w0 / 2 + i] = (uint8_t)((L.code[2 * i] & 15) | (L.code[2 * i + 1] << 4));
        state = L.traj[nw - 1];
    }
}

// host launch helpers -------------------------------------------------------------------
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

// scratch: ngroups * N cf32, used for N > 16384 (groups hold one frame each there)
hipError_t launch_wf_fft(int logn, const float2* blk, int64_t blk_start, const WfGroup* groups,
                         int ngroups, const float* window, const float2* tw, float* partial,
                         float2* scratch, hipStream_t st) {
    switch (logn) {
        case 8: return launch_fft_t<8>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 9: return launch_fft_t<9>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 10: return launch_fft_t<10>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 11: return launch_fft_t<11>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 12: return launch_fft_t<12>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 13: return launch_fft_t<13>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 14: return launch_fft_t<14>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 15: return launch_fft4_t<7, 8>(blk, blk_start, groups, ngroups, window, tw, partial,
                                            scratch, st);
        case 16: return launch_fft4_t<8, 8>(blk, blk_start, groups, ngroups, window, tw, partial,
                                            scratch, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_wf_finalize(const float* partial, const WfRow* rows, int nrows,
                              const float* carry_in, float* carry_out, int N, float add_corr,
                              int adpcm, int16_t* s16_out, float* f32_out, hipStream_t st) {
    hipLaunchKernelGGL(wf_finalize, dim3((N + 255) / 256, nrows), dim3(256), 0, st, partial,
                       rows, carry_in, carry_out, N, add_corr, adpcm, s16_out, f32_out);
    return hipGetLastError();
}

hipError_t launch_wf_adpcm(const int16_t* s16, int N, int nrows, uint8_t* out, int row_bytes,
                           hipStream_t st) {
    const size_t lds = sizeof(SpecLds<kRowWin>);
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)wf_adpcm_rows_spec,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(wf_adpcm_rows_spec, dim3(nrows), dim3(kSpecThreads), lds, st, s16, N,
                       nrows, out, row_bytes);
    return hipGetLastError();
}

}  // namespace owrx
