// kernels_post.hip -- everything after the fused DDC, one workgroup per client chain:
//   segment-partial reduce (FirDecimate output, csdr/chain/selector.py:29)
//   -> FractionalDecimator (12-point Lagrange, selector.py:32-33)
//   -> Bandpass (complex FIR, selector.py:115-117, 159-166; csdr uses FFT overlap-add, the
//      causal convolution here is the same linear operator)
//   -> Squelch (block power, gate, s-meter writer; selector.py:119-130)
//   -> NFm [FmDemod, Limit, NfmDeemphasis, Agc] | Am [AmDemod, DcBlock, Agc] | Ssb
//      [RealPart, Agc] (csdr/chain/analog.py)
//   -> Convert(FLOAT, SHORT) -> AdpcmEncoder(sync=True) (csdr/chain/clientaudio.py).
// Rate here is ~12 kHz per chain, so the work is tiny; the stages that are per-sample
// independent run across the workgroup, the recurrences (deemphasis, DC block, AGC, ADPCM)
// run on one lane per chain from an LDS-staged chunk.
#include "owrx_types.h"

namespace owrx {

constexpr int kPostThreads = 256;
constexpr int kMaxSqBlocks = 1024;
constexpr int kSerialChunk = 1024;
constexpr int kMaxSqLen = 3072;  // longest squelch block kept in registers while compacting

// Lagrange basis denominators for nodes j - 5.5, j = 0..11: 1 / prod_{j != i} (n_i - n_j)
OWRX_DEV float lagrange_den(int i) {
    // prod_{j != i} (i - j) = (-1)^(11-i) * i! * (11-i)!
    const float fact[12] = {1.0f, 1.0f, 2.0f, 6.0f, 24.0f, 120.0f, 720.0f, 5040.0f,
                            40320.0f, 362880.0f, 3628800.0f, 39916800.0f};
    const float d = fact[i] * fact[11 - i];
    return ((11 - i) & 1) ? -1.0f / d : 1.0f / d;
}

__global__ void __launch_bounds__(kPostThreads)
post_chains(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts) {
    const ChainPost P = posts[blockIdx.x];
    const int tid = threadIdx.x;
    constexpr int NT = kPostThreads;

    __shared__ ChainState S;
    __shared__ int sh_n_fd;
    __shared__ float sh_power[kMaxSqBlocks];
    __shared__ uint8_t sh_pass[kMaxSqBlocks];
    __shared__ float sh_chunk[kSerialChunk];
    __shared__ int16_t sh_step[89];
    __shared__ int8_t sh_idx[16];

    if (tid == 0) S = *P.state;
    if (tid < 89) sh_step[tid] = kAdpcmStep[tid];
    if (tid < 16) sh_idx[tid] = kAdpcmIndex[tid];
    __syncthreads();

    // ---- 0. FirDecimate output: fixed-order sum of the phase-segment partials ----------
    const int64_t kb = P.k_begin > P.k_first ? P.k_begin : P.k_first;
    const int64_t nn = P.k_begin + P.nk - kb;
    const int n_new = nn > 0 ? (int)nn : 0;
    const int col0 = (int)(kb - P.k_begin);
    for (int i = tid; i < n_new; i += NT) {
        float2 y = make_float2(0.0f, 0.0f);
        for (int s = 0; s < P.nseg; ++s) {
            const float2 v =
                P.partial[((int64_t)s * P.group_chains + P.chain_in_group) * P.nk + col0 + i];
            y.x += v.x;
            y.y += v.y;
        }
        P.ddc_buf[kFdHist + i] = y;
        if (P.debug && i < P.dbg_cap) P.dbg_ddc[i] = y;
    }
    __syncthreads();
    const int64_t ddc_base = S.ddc_count - kFdHist;  // local index of ddc_buf[0]
    const int64_t ddc_total = S.ddc_count + n_new;

    // ---- 1. FractionalDecimator ------------------------------------------------------------
    if (P.frac_enabled) {
        if (tid == 0) {
            const double r = P.frac_rate;
            auto valid = [&](int64_t k) {
                const double w = 6.0 + (double)k * r;
                return (int64_t)ceil(w) + 5 < ddc_total;
            };
            int64_t ke = (int64_t)floor(((double)ddc_total - 12.0) / r);
            if (ke < S.fd_next) ke = S.fd_next;
            while (valid(ke)) ++ke;
            while (ke > S.fd_next && !valid(ke - 1)) --ke;
            sh_n_fd = (int)(ke - S.fd_next);
        }
        __syncthreads();
        const int n_fd = sh_n_fd;
        for (int j = tid; j < n_fd; j += NT) {
            const int64_t k = S.fd_next + j;
            const double w = 6.0 + (double)k * P.frac_rate;
            const int64_t hi = (int64_t)ceil(w);
            const int64_t lo = hi - 6;
            const float u = (float)((w - (double)lo) - 5.5);
            float d[kFdPoints];
#pragma unroll
            for (int i = 0; i < kFdPoints; ++i) d[i] = u - ((float)i - 5.5f);
            float pre[kFdPoints], suf[kFdPoints];
            pre[0] = 1.0f;
#pragma unroll
            for (int i = 1; i < kFdPoints; ++i) pre[i] = pre[i - 1] * d[i - 1];
            suf[kFdPoints - 1] = 1.0f;
#pragma unroll
            for (int i = kFdPoints - 2; i >= 0; --i) suf[i] = suf[i + 1] * d[i + 1];
            const float2* x = P.ddc_buf + (lo - ddc_base);
            float2 acc = make_float2(0.0f, 0.0f);
#pragma unroll
            for (int i = 0; i < kFdPoints; ++i) {
                const float L = pre[i] * suf[i] * lagrange_den(i);
                acc.x = fmaf(L, x[i].x, acc.x);
                acc.y = fmaf(L, x[i].y, acc.y);
            }
            P.fd_buf[kBpHist + j] = acc;
        }
    } else {
        if (tid == 0) sh_n_fd = n_new;
        for (int j = tid; j < n_new; j += NT) P.fd_buf[kBpHist + j] = P.ddc_buf[kFdHist + j];
    }
    __syncthreads();
    const int n_fd = sh_n_fd;
    {   // keep the last kFdHist DDC outputs as interpolator history
        float2 t = make_float2(0.0f, 0.0f);
        if (tid < kFdHist) t = P.ddc_buf[n_new + tid];
        __syncthreads();
        if (tid < kFdHist) P.ddc_buf[tid] = t;
    }

    // ---- 2. Bandpass -------------------------------------------------------------------------
    const int pend = S.sq_pending;
    for (int j = tid; j < n_fd; j += NT) {
        const float2* x = P.fd_buf + kBpHist + j;
        float2 y;
        if (P.bp_ntaps > 0) {
            float ar = 0.0f, ai = 0.0f;
            for (int t = 0; t < P.bp_ntaps; ++t) {
                const float2 g = P.bp_taps[t];
                const float2 v = x[-t];
                ar = fmaf(g.x, v.x, ar);
                ar = fmaf(-g.y, v.y, ar);
                ai = fmaf(g.x, v.y, ai);
                ai = fmaf(g.y, v.x, ai);
            }
            y = make_float2(ar, ai);
        } else {
            y = x[0];
        }
        P.sq_buf[pend + j] = y;
        if (P.debug && j < P.dbg_cap) {
            P.dbg_fd[j] = x[0];
            P.dbg_bp[j] = y;
        }
    }
    __syncthreads();
    {   // keep the last kBpHist bandpass inputs
        const float2 t = P.fd_buf[n_fd + tid];  // kBpHist == NT
        __syncthreads();
        P.fd_buf[tid] = t;
    }

    // ---- 3. Squelch: block powers, gate, s-meter ---------------------------------------
    const int L = P.sq_len;
    const int total = pend + n_fd;
    const int nb = total / L;
    for (int b = tid; b < nb; b += NT) {
        float p = 0.0f;
        int cnt = 0;
        for (int i = 0; i < L; i += P.sq_dec) {
            const float2 v = P.sq_buf[b * L + i];
            p = fmaf(v.x, v.x, p);
            p = fmaf(v.y, v.y, p);
            cnt++;
        }
        sh_power[b] = p / (float)cnt;
    }
    __syncthreads();
    if (tid == 0) {
        int ns = 0;
        for (int b = 0; b < nb; ++b) {
            const float power = sh_power[b];
            const int64_t bi = S.sq_blocks + b;
            if (P.sq_report > 0 && ((bi + 1) % P.sq_report) == 0) {
                if (ns < P.smeter_cap) P.smeter[ns] = power;
                ns++;
            }
            int pass;
            if (P.sq_level == 0.0f || power >= P.sq_level) {
                S.hang_ctr = P.sq_hang;
                S.flush_ctr = P.sq_flush;
                pass = 1;
            } else if (S.hang_ctr > 0) {
                S.hang_ctr -= L;
                pass = 1;
            } else {
                if (S.flush_ctr > 0) S.flush_ctr -= L;
                pass = 0;
            }
            sh_pass[b] = (uint8_t)pass;
        }
        counts[blockIdx.x].smeter = ns < P.smeter_cap ? ns : P.smeter_cap;
    }
    __syncthreads();

    // ---- 4. demodulator front (per-sample independent) ------------------------------------
    const int nsq = nb * L;
    const float2 fm_prev0 = S.fm_last;
    for (int i = tid; i < nsq; i += NT) {
        const float2 x = sh_pass[i / L] ? P.sq_buf[i] : make_float2(0.0f, 0.0f);
        if (P.debug && i < P.dbg_cap) P.dbg_sq[i] = x;
        float v;
        if (P.demod == 0) {
            float2 prev = fm_prev0;
            if (i > 0) prev = sh_pass[(i - 1) / L] ? P.sq_buf[i - 1] : make_float2(0.0f, 0.0f);
            v = limit_step(fm_step(x, prev), 1.0f);
        } else if (P.demod == 1) {
            v = am_step(x);
        } else {
            v = x.x;
        }
        P.dem_buf[i] = v;
    }
    __syncthreads();
    {   // move the incomplete squelch block to the front
        const int rem = total - nsq;
        float2 last = S.fm_last;
        if (nsq > 0) last = sh_pass[nb - 1] ? P.sq_buf[nsq - 1] : make_float2(0.0f, 0.0f);
        float2 t[kMaxSqLen / NT];
#pragma unroll
        for (int m = 0; m < kMaxSqLen / NT; ++m) {
            const int i = tid + m * NT;
            if (i < rem) t[m] = P.sq_buf[nsq + i];
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < kMaxSqLen / NT; ++m) {
            const int i = tid + m * NT;
            if (i < rem) P.sq_buf[i] = t[m];
        }
        if (tid == 0) {
            S.fm_last = last;
            S.sq_pending = rem;
        }
    }

    // ---- 5. recurrences: deemphasis / DC block, AGC, Convert, ADPCM --------------------
    int64_t ob = 0;
    for (int c0 = 0; c0 < nsq; c0 += kSerialChunk) {
        const int cn = min(kSerialChunk, nsq - c0);
        __syncthreads();
        for (int i = tid; i < cn; i += NT) sh_chunk[i] = P.dem_buf[c0 + i];
        __syncthreads();
        if (tid == 0) {
            for (int i = 0; i < cn; ++i) {
                float v = sh_chunk[i];
                if (P.demod == 0)
                    v = deemph_step(v, P.deemph_alpha, P.deemph_beta, S.deemph_y);
                else if (P.demod == 1)
                    v = dcblock_step(v, S.dc_xp, S.dc_yp);
                if (P.debug && c0 + i < P.dbg_cap) P.dbg_dem[c0 + i] = v;
                const float a = agc_step(v, P.agc, S.agc);
                if (P.debug && c0 + i < P.dbg_cap) P.dbg_agc[c0 + i] = a;
                if (P.output == 2) {  // OWRX_OUT_F32
                    if (ob + 4 <= P.out_cap) *(float*)(P.out + ob) = a;
                    ob += 4;
                } else {
                    const int16_t s16 = convert_s16(a);
                    if (P.output == 0) {  // OWRX_OUT_S16
                        if (ob + 2 <= P.out_cap) {
                            P.out[ob] = (uint8_t)(s16 & 0xff);
                            P.out[ob + 1] = (uint8_t)((s16 >> 8) & 0xff);
                        }
                        ob += 2;
                    } else {  // ADPCM with sync
                        if (!S.has_left) {
                            S.left_sample = s16;
                            S.has_left = 1;
                        } else {
                            if ((S.adpcm_bytes % kAdpcmSyncPeriod) == 0) {
                                if (ob + 8 <= P.out_cap) {
                                    P.out[ob] = 'S';
                                    P.out[ob + 1] = 'Y';
                                    P.out[ob + 2] = 'N';
                                    P.out[ob + 3] = 'C';
                                    const int16_t ix = (int16_t)S.adpcm.index;
                                    const int16_t pr = (int16_t)S.adpcm.pred;
                                    P.out[ob + 4] = (uint8_t)(ix & 0xff);
                                    P.out[ob + 5] = (uint8_t)((ix >> 8) & 0xff);
                                    P.out[ob + 6] = (uint8_t)(pr & 0xff);
                                    P.out[ob + 7] = (uint8_t)((pr >> 8) & 0xff);
                                }
                                ob += 8;
                            }
                            const int lo = adpcm_encode(S.adpcm, S.left_sample);
                            const int hi = adpcm_encode(S.adpcm, s16);
                            if (ob + 1 <= P.out_cap) P.out[ob] = (uint8_t)(lo | (hi << 4));
                            ob += 1;
                            S.adpcm_bytes++;
                            S.has_left = 0;
                        }
                    }
                }
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        S.ddc_count = ddc_total;
        if (P.frac_enabled) S.fd_next += n_fd;
        S.fd_count += n_fd;
        S.sq_blocks += nb;
        *P.state = S;
        ChainCounts& c = counts[blockIdx.x];
        c.out_bytes = ob;
        c.n_ddc = n_new;
        c.n_fd = n_fd;
        c.n_bp = n_fd;
        c.n_sq = nsq;
    }
}

hipError_t launch_post(const ChainPost* posts, int nchains, ChainCounts* counts,
                       hipStream_t st) {
    if (nchains <= 0) return hipSuccess;
    hipLaunchKernelGGL(post_chains, dim3(nchains), dim3(kPostThreads), 0, st, posts, counts);
    return hipGetLastError();
}

}  // namespace owrx
