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
// wf_adpcm_rows: IMA-ADPCM of each padded row (serial per row, one lane per row).
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
// the row; fresh codec state per row; low nibble first.  One lane per row (rows of one launch
// have the same length, so the wave runs them in lockstep); 8 input samples per 16-B load,
// prefetched one load ahead; step table in LDS, lookup off the dependency chain.
__global__ void __launch_bounds__(64)
wf_adpcm_rows(const int16_t* __restrict__ s16, int N, int nrows, uint8_t* __restrict__ out,
              int row_bytes) {
    __shared__ int16_t T[96];
    for (int i = threadIdx.x; i < 89; i += 64) T[i] = kAdpcmStep[i];
    __syncthreads();
    const int r = blockIdx.x * 64 + threadIdx.x;
    if (r >= nrows) return;
    const int16_t* s = s16 + (int64_t)r * N;
    uint8_t* o = out + (int64_t)r * row_bytes;
    AdpcmFast st{0, 0, (int)T[0]};
    const int first = s[0];
    for (int t = 0; t < 10; t += 2) {
        const int lo = adpcm_encode_fast(st, first, T);
        const int hi = adpcm_encode_fast(st, first, T);
        o[t >> 1] = (uint8_t)(lo | (hi << 4));
    }
    const int4* v4 = reinterpret_cast<const int4*>(s);
    int4 nxt = v4[0];
    for (int i = 0; i < N; i += 8) {
        const int4 cur = nxt;
        if (i + 8 < N) nxt = v4[(i >> 3) + 1];
        const int w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int a = (int)(int16_t)(w[j] & 0xffff);
            const int b = (int)(int16_t)((uint32_t)w[j] >> 16);
            const int lo = adpcm_encode_fast(st, a, T);
            const int hi = adpcm_encode_fast(st, b, T);
            o[5 + ((i >> 1) + j)] = (uint8_t)(lo | (hi << 4));
        }
    }
}

// FftAdpcm, row-parallel exact encoder.  IMA-ADPCM is a serial recurrence, but two encoders
// started from different states on the same input reach the same (index, predictor) state
// after ~100-900 samples on waterfall data and are identical from then on.  Each row is split
// into kSeg segments, one lane each:
//   pass 1: every segment encodes from a guessed state (segment 0 from the true state),
//           storing its codes and its state trajectory;
//   pass 2: a segment whose start differs from its predecessor's final state re-encodes from
//           that state until its state equals the stored trajectory (then the stored codes are
//           exact from there on) or to its end (then its trajectory / final state are
//           replaced).  Jacobi iterations until no segment re-runs (<= kSeg, typically 1-2);
//   pass 3: nibble packing.
// The result is bit-identical to the sequential encoder (oracle orc_fft_adpcm_row).
constexpr int kSeg = 16;

OWRX_DEV uint32_t pack_state(const AdpcmFast& s) {
    return ((uint32_t)s.index << 16) | ((uint32_t)s.pred & 0xffffu);
}
OWRX_DEV AdpcmFast unpack_state(uint32_t v, const int16_t* T) {
    AdpcmFast s;
    s.index = (int)(v >> 16);
    s.pred = (int)(int16_t)(v & 0xffffu);
    s.step = T[s.index];
    return s;
}

__global__ void __launch_bounds__(64)
wf_adpcm_rows_spec(const int16_t* __restrict__ s16, int N, int nrows, uint8_t* __restrict__ out,
                   int row_bytes, uint8_t* __restrict__ codes, uint32_t* __restrict__ traj) {
    __shared__ int16_t T[96];
    __shared__ uint32_t seg_start[4][kSeg], seg_final[4][kSeg];
    __shared__ int any_rerun;
    const int lane = threadIdx.x;
    for (int i = lane; i < 89; i += 64) T[i] = kAdpcmStep[i];
    const int rl = lane / kSeg, j = lane % kSeg;
    const int row_raw = blockIdx.x * 4 + rl;
    const bool active = row_raw < nrows;
    const int row = active ? row_raw : nrows - 1;
    const int M = N + 10;
    const int L = ((M + kSeg - 1) / kSeg + 1) & ~1;
    const int b0 = min(j * L, M), b1 = min(b0 + L, M);
    const int16_t* x = s16 + (int64_t)row * N;
    uint8_t* cd = codes + (int64_t)row * M;
    uint32_t* tr = traj + (int64_t)row * M;
    auto sample = [&](int t) -> int { return t < 10 ? (int)x[0] : (int)x[t - 10]; };
    __syncthreads();

    // pass 1: speculative encode of every segment
    AdpcmFast st;
    if (j == 0) {
        st = AdpcmFast{0, 0, (int)T[0]};
    } else {
        st.index = 30;  // measured to merge fastest on waterfall rows
        st.pred = sample(b0 - 1);
        st.step = T[30];
    }
    const uint32_t start0 = pack_state(st);
    for (int t = b0; t < b1; ++t) {
        cd[t] = (uint8_t)adpcm_encode_fast(st, sample(t), T);
        tr[t] = pack_state(st);
    }
    seg_start[rl][j] = start0;
    seg_final[rl][j] = pack_state(st);
    __syncthreads();

    // pass 2: repair from the predecessor's final state until consistent
    for (int it = 0; it < kSeg; ++it) {
        if (lane == 0) any_rerun = 0;
        __syncthreads();
        const uint32_t want = j > 0 ? seg_final[rl][j - 1] : seg_start[rl][0];
        const bool rerun = active && j > 0 && want != seg_start[rl][j] && b0 < b1;
        uint32_t fin = seg_final[rl][j];
        __syncthreads();  // everyone has read the finals of this iteration
        if (rerun) {
            AdpcmFast r = unpack_state(want, T);
            bool merged = false;
            for (int t = b0; t < b1; ++t) {
                cd[t] = (uint8_t)adpcm_encode_fast(r, sample(t), T);
                const uint32_t ps = pack_state(r);
                if (ps == tr[t]) {
                    merged = true;
                    break;
                }
                tr[t] = ps;
            }
            if (!merged) fin = pack_state(r);
            seg_start[rl][j] = want;
            seg_final[rl][j] = fin;
            any_rerun = 1;
        }
        __syncthreads();
        if (!any_rerun) break;
    }

    // pass 3: nibbles -> bytes (low nibble first)
    __syncthreads();
    if (active) {
        uint8_t* o = out + (int64_t)row * row_bytes;
        for (int i = j; i < M / 2; i += kSeg) o[i] = (uint8_t)((cd[2 * i] & 15) | (cd[2 * i + 1] << 4));
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

hipError_t launch_wf_fft(int logn, const float2* blk, int64_t blk_start, const WfGroup* groups,
                         int ngroups, const float* window, const float2* tw, float* partial,
                         hipStream_t st) {
    switch (logn) {
        case 8: return launch_fft_t<8>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 9: return launch_fft_t<9>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 10: return launch_fft_t<10>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 11: return launch_fft_t<11>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 12: return launch_fft_t<12>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 13: return launch_fft_t<13>(blk, blk_start, groups, ngroups, window, tw, partial, st);
        case 14: return launch_fft_t<14>(blk, blk_start, groups, ngroups, window, tw, partial, st);
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
                           uint8_t* codes, uint32_t* traj, hipStream_t st) {
    if (codes && traj) {
        hipLaunchKernelGGL(wf_adpcm_rows_spec, dim3((nrows + 3) / 4), dim3(64), 0, st, s16, N,
                           nrows, out, row_bytes, codes, traj);
    } else {
        hipLaunchKernelGGL(wf_adpcm_rows, dim3((nrows + 63) / 64), dim3(64), 0, st, s16, N,
                           nrows, out, row_bytes);
    }
    return hipGetLastError();
}

}  // namespace owrx
