// kernels_sfft.hip -- the per-client secondary FFT.
//
// Reference: ClientDemodulatorChain._createSecondaryFftChain (owrx/dsp.py:220-225) builds
// FftChain(selectorOutputRate, digimodes_fft_size, 0.3, 9, "adpcm") (sizes owrx/dsp.py:60-63)
// on a reader of the Selector output buffer, i.e. the same Fft -> LogAveragePower/LogPower ->
// FftSwap -> FftAdpcm modules as the main waterfall (csdr/chain/fft.py:25-96), at the 12 kHz
// client rate.  Frames go to the browser as type 0x03 (owrx/connection.py:500-501).
//
// chain_sfft<LOGN>: one workgroup per chain (256 threads), launched on stream A right after
// post_parallel, which appended this step's squelch-gated Selector output to the chain's
// sf_buf.  Every whole frame is windowed into LDS, transformed by the batched LDS FFT
// (fft_lds.h), and |X|^2 summed in registers; a completed row is finalised exactly like
// wf_finalize (fixed summation order, 10 log10 + correction, fftshift, (short)(dB*100)) and
// IMA-ADPCM-encoded by the segment-parallel exact encoder of the waterfall rows (adpcm_spec.h).
// An open row's sum is carried in sf_acc.  At ~4 frames of 2048 points per chain per 2^22-sample
// block this is latency work next to the DDC; chains run in parallel across CUs.
#include "adpcm_spec.h"
#include "fft_lds.h"
#include "owrx_types.h"

namespace owrx {

constexpr int kSfThreads = 256;
static_assert(kSfThreads == kSpecThreads, "the row encoder assumes its own block size");

template <int LOGN>
struct SfLds {
    float2 x[1 << LOGN];
    SpecLds<(1 << LOGN) + 16> enc;
};

template <int LOGN>
__global__ void __launch_bounds__(kSfThreads)
chain_sfft(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts) {
    constexpr int N = 1 << LOGN;
    constexpr int PPT = N / kSfThreads;
    const ChainPost& P = posts[blockIdx.x];
    if (P.sf_n != N) return;  // chains without (or with another size of) secondary FFT
    if (P.sf_hop <= 0 || P.sf_avg <= 0) return;  // never a frame loop that does not advance
    extern __shared__ __align__(16) uint8_t smem[];
    SfLds<LOGN>& S = *reinterpret_cast<SfLds<LOGN>*>(smem);
    const int tid = threadIdx.x;
    const int hop = P.sf_hop, avg = P.sf_avg, adpcm = P.sf_adpcm;
    const float corr = P.sf_corr;
    const auto buf = gp(P.sf_buf);
    const auto win = gp(P.sf_window);
    ChainStateP* ps = P.pstate;
    const int fill = ps->sf_fill;
    int next = ps->sf_next;
    int rf = ps->sf_row_frame;
    if (adpcm) {
        for (int i = tid; i < 89; i += kSfThreads) S.enc.T[i] = kAdpcmStep[i];
        adpcm_rem_fill(S.enc.NSR, tid, kSfThreads);
    }
    float acc[PPT];
#pragma unroll
    for (int m = 0; m < PPT; ++m) acc[m] = rf > 0 ? P.sf_acc[tid + m * kSfThreads] : 0.0f;
    const int64_t rb = adpcm ? (N + 10) / 2 : 4 * (int64_t)N;
    const SpecGeom gm = spec_geom(N + 10, 64);  // the FftAdpcm window's transposed layout
    int rows = 0;
    while (next + N <= fill) {
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const int i = tid + m * kSfThreads;
            const float2 v = buf[next + i];
            const float w = win[i];
            S.x[i] = make_float2(v.x * w, v.y * w);
        }
        __syncthreads();
        lds_fft_rows<LOGN, 1, kSfThreads>(S.x, N, P.sf_tw, 1);
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
            const float2 X = S.x[tid + m * kSfThreads];
            acc[m] += X.x * X.x + X.y * X.y;
        }
        __syncthreads();
        next += hop;
        if (++rf < avg) continue;
        // row complete: LogAveragePower -> FftSwap -> (FftAdpcm)
        const bool room = (int64_t)(rows + 1) * rb <= P.sf_out_cap;
        uint8_t* row = P.sf_out + (int64_t)rows * rb;
#pragma unroll
        for (int m = 0; m < PPT; ++m) {
#pragma clang fp contract(off)
            const int i = tid + m * kSfThreads;
            const float lg = log10f(acc[m]);
            const float t = 10.0f * lg;
            const float db = t + corr;
            const int o = (i + N / 2) & (N - 1);
            if (adpcm) {
                const int16_t q = db_to_s16(db);
                S.enc.x[spec_at(gm, 10 + o)] = q;
                if (o == 0) {
#pragma unroll
                    for (int k = 0; k < 10; ++k) S.enc.x[spec_at(gm, k)] = q;  // COMPRESS_FFT_PAD_N copies
                }
            } else if (room) {
                reinterpret_cast<float*>(row)[o] = db;
            }
            acc[m] = 0.0f;
        }
        if (adpcm) {
            __syncthreads();
            adpcm_spec_window(S.enc, N + 10, gm, 0u, 30);  // FftAdpcm: fresh state per row
            __syncthreads();
            if (room)
                for (int i = tid; i < (N + 10) / 2; i += kSfThreads)
                    row[i] = (uint8_t)((S.enc.code[spec_at(gm, 2 * i)] & 15) |
                                       (S.enc.code[spec_at(gm, 2 * i + 1)] << 4));
            __syncthreads();
        }
        rf = 0;
        rows++;
    }
    if (rf > 0) {
#pragma unroll
        for (int m = 0; m < PPT; ++m) P.sf_acc[tid + m * kSfThreads] = acc[m];
    }
    if (tid == 0) {
        ps->sf_next = next;
        ps->sf_row_frame = rf;
        counts[blockIdx.x].sf_bytes = (int32_t)((int64_t)rows * rb);
    }
}

template <int LOGN>
static hipError_t launch_sfft_t(const ChainPost* posts, int nposts, ChainCounts* counts,
                                hipStream_t st) {
    const size_t lds = sizeof(SfLds<LOGN>);
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)chain_sfft<LOGN>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(chain_sfft<LOGN>, dim3(nposts), dim3(kSfThreads), lds, st, posts, counts);
    return hipGetLastError();
}

// one launch per secondary FFT size in use; workgroups of chains with another size return
hipError_t launch_chain_sfft(int logn, const ChainPost* posts, int nposts, ChainCounts* counts,
                             hipStream_t st) {
    if (nposts <= 0) return hipSuccess;
    switch (logn) {
        case 10: return launch_sfft_t<10>(posts, nposts, counts, st);
        case 11: return launch_sfft_t<11>(posts, nposts, counts, st);
        case 12: return launch_sfft_t<12>(posts, nposts, counts, st);
        case 13: return launch_sfft_t<13>(posts, nposts, counts, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace owrx
