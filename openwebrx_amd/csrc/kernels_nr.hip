// kernels_nr.hip -- NoiseFilter(nr_threshold) of ClientAudioChain (csdr/chain/clientaudio.py:
// 12-13, enabled by nr_enabled / nr_threshold, owrx/dsp.py:496-509, 559-560; BASELINE config 5).
//
// The reference's filter is csdr's NoiseFilter ("spectral subtraction", CHANGELOG.md:852); its
// source is not in /root/reference, so the algorithm is the build's documented choice, restated
// identically in oracle/csdr_oracle.c orc_noise_filter (parity unpinned against csdr):
//   frames of kNrN = 512 samples at hop kNrHop = 256 (50 % overlap), analysis and synthesis
//   window sqrt(periodic Hann) (w^2 overlap-adds to 1, so gain 1 reconstructs exactly);
//   per bin k: P = |X_k|^2, smoothed S = 0.7 S + 0.3 P (first frame S = P); noise floor
//   Nf = geometric mean of S over the 257 bins (signals occupy few bins), smoothed 0.9 / 0.1
//   across frames; gain G = S / (S + t Nf + 1e-30), t = 10^(threshold/10);
//   y = w * IFFT(G X), overlap-added; output lags the input by one hop.
// Every step is continuous in its inputs (no decisions), so fp32 GPU rounding stays at the
// rounding level against the double-precision oracle.
//
// chain_nr: one workgroup (128 threads) per chain on stream B after post_serial_front, which
// appended this step's AGC output to nr_in.  Frames run in order (the smoothing is a recurrence
// across frames); the FFTs are the batched LDS FFT of fft_lds.h.  Output: Convert(FLOAT, SHORT)
// into the ADPCM encoder's input (or the S16 / F32 output).
#include "fft_lds.h"
#include "owrx_types.h"
#include "../../include/owrx_amd.h"

namespace owrx {

constexpr int kNrThreads = 128;
constexpr int kNrBins = kNrN / 2 + 1;

__global__ void __launch_bounds__(kNrThreads)
chain_nr(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts) {
    const ChainPost& P = posts[blockIdx.x];
    if (!P.nr_enabled || P.output == OWRX_OUT_IQ) return;
    __shared__ float2 X[kNrN];
    __shared__ float G[kNrBins];
    __shared__ float sh_lsum[kNrThreads / 64];
    // tables in LDS and the per-bin / overlap state in registers: each frame is a handful of
    // LDS passes instead of a chain of dependent global round trips (measured 95 us per frame
    // with the tables and state in global memory)
    __shared__ float2 sh_tw[kNrN];
    __shared__ float sh_win[kNrN];
    const int tid = threadIdx.x;
    const auto in = gp(P.nr_in);
    const auto pw = gp(P.nr_pow);  // [0, kNrBins): smoothed power per bin, [kNrBins]: floor
    const auto ola = gp(P.nr_ola);
    const auto win = gp(P.nr_win);
    NrState st = *P.nr_state;
    for (int i = tid; i < kNrN; i += kNrThreads) {
        sh_tw[i] = P.nr_tw[i];
        sh_win[i] = win[i];
    }
    constexpr int kBinsPT = (kNrBins + kNrThreads - 1) / kNrThreads;  // bins per thread
    constexpr int kOlaPT = kNrHop / kNrThreads;
    float Sreg[kBinsPT], olar[kOlaPT];
#pragma unroll
    for (int m = 0; m < kBinsPT; ++m) {
        const int k = tid + m * kNrThreads;
        Sreg[m] = k < kNrBins ? pw[k] : 0.0f;
    }
#pragma unroll
    for (int m = 0; m < kOlaPT; ++m) olar[m] = ola[tid + m * kNrThreads];
    __syncthreads();
    const int n_in = (int)counts[blockIdx.x].n_sq;
    const int fill = kNrHop + st.pend + n_in;
    const float t = P.nr_t;
    float nf = pw[kNrBins];  // smoothed noise floor (uniform)
    int base = 0, nout = 0;
    while (fill - base >= kNrN) {
        for (int i = tid; i < kNrN; i += kNrThreads)
            X[i] = make_float2(in[base + i] * sh_win[i], 0.0f);
        __syncthreads();
        lds_fft_rows<9, 1, kNrThreads>(X, kNrN, sh_tw, 1);
        float lsum = 0.0f;
#pragma unroll
        for (int m = 0; m < kBinsPT; ++m) {
#pragma clang fp contract(off)
            const int k = tid + m * kNrThreads;
            if (k >= kNrBins) break;
            const float2 v = X[k];
            const float p = v.x * v.x + v.y * v.y;
            float S = p;
            if (st.frames > 0) {
                const float s0 = 0.7f * Sreg[m];
                const float s1 = 0.3f * p;
                S = s0 + s1;
            }
            Sreg[m] = S;
            G[k] = S;
            lsum += logf(S + 1e-30f);
        }
        for (int o = 32; o > 0; o >>= 1) lsum += __shfl_xor(lsum, o);
        if ((tid & 63) == 0) sh_lsum[tid >> 6] = lsum;
        __syncthreads();
        float Nf;
        {
#pragma clang fp contract(off)
            float ls = 0.0f;
#pragma unroll
            for (int w = 0; w < kNrThreads / 64; ++w) ls += sh_lsum[w];
            const float geo = expf(ls / (float)kNrBins);
            Nf = geo;
            if (st.frames > 0) {
                const float n0 = 0.9f * nf;
                const float n1 = 0.1f * geo;
                Nf = n0 + n1;
            }
        }
        const float tn = t * Nf;
        for (int k = tid; k < kNrBins; k += kNrThreads) {
#pragma clang fp contract(off)
            const float S = G[k];
            const float den = (S + tn) + 1e-30f;
            G[k] = S / den;
        }
        __syncthreads();
        nf = Nf;
        // Y = G X (G symmetric in k <-> N - k); IFFT(Y) = conj(FFT(conj(Y))) / N
        for (int i = tid; i < kNrN; i += kNrThreads) {
            const float g = G[i <= kNrN / 2 ? i : kNrN - i];
            const float2 v = X[i];
            X[i] = make_float2(g * v.x, -(g * v.y));
        }
        __syncthreads();
        lds_fft_rows<9, 1, kNrThreads>(X, kNrN, sh_tw, 1);
#pragma unroll
        for (int m = 0; m < kOlaPT; ++m) {
#pragma clang fp contract(off)
            const int i = tid + m * kNrThreads;
            const float y0 = (X[i].x * (1.0f / kNrN)) * sh_win[i];
            const float y1 = (X[kNrHop + i].x * (1.0f / kNrN)) * sh_win[kNrHop + i];
            const float o = olar[m] + y0;
            olar[m] = y1;
            if (st.frames > 0) {  // frame 0's first half is the zero history before sample 0
                const int q = nout + i;
                if (P.output == OWRX_OUT_F32)
                    gp(reinterpret_cast<float*>(P.out))[q] = o;
                else if (P.output == OWRX_OUT_S16)
                    gp(reinterpret_cast<int16_t*>(P.out))[q] = convert_s16(o);
                else
                    gp(P.s16)[q] = convert_s16(o);
            }
        }
        if (st.frames > 0) nout += kNrHop;
        st.frames++;
        base += kNrHop;
        __syncthreads();
    }
    // keep [base, fill): the last hop of the last frame plus pending input
    const int keep = fill - base;
    for (int b0 = 0; b0 < keep; b0 += kNrThreads) {
        const int i = b0 + tid;
        float v = 0.0f;
        if (i < keep) v = in[base + i];
        __syncthreads();
        if (i < keep) in[i] = v;
    }
#pragma unroll
    for (int m = 0; m < kBinsPT; ++m) {
        const int k = tid + m * kNrThreads;
        if (k < kNrBins) pw[k] = Sreg[m];
    }
#pragma unroll
    for (int m = 0; m < kOlaPT; ++m) ola[tid + m * kNrThreads] = olar[m];
    if (tid == 0) {
        pw[kNrBins] = nf;
        st.pend = keep - kNrHop;  // keep >= kNrHop: the last frame's second half stays
        *P.nr_state = st;
        ChainCounts& c = counts[blockIdx.x];
        c.n_sq = nout;  // what the ADPCM encoder reads
        if (P.output == OWRX_OUT_F32) c.out_bytes = 4 * (int64_t)nout;
        if (P.output == OWRX_OUT_S16) c.out_bytes = 2 * (int64_t)nout;
    }
}

hipError_t launch_chain_nr(const ChainPost* posts, int nposts, ChainCounts* counts,
                           hipStream_t st) {
    if (nposts <= 0) return hipSuccess;
    hipLaunchKernelGGL(chain_nr, dim3(nposts), dim3(kNrThreads), 0, st, posts, counts);
    return hipGetLastError();
}

}  // namespace owrx
