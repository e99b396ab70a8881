// kernels_post.hip -- everything after the fused DDC.
//
// post_parallel (stream A, one 256-thread workgroup per client chain): the per-sample
// independent stages at the ~12 kHz chain rate
//   segment-partial reduce (FirDecimate output, csdr/chain/selector.py:29)
//   -> FractionalDecimator (12-point Lagrange, selector.py:32-33)
//   -> Bandpass (complex FIR; csdr applies it by FFT overlap-add, the causal convolution here
//      is the same linear operator; selector.py:115-117, 159-166)
//   -> Squelch (block power, gate, s-meter writer; selector.py:119-130)
//   -> demodulator front: FmDemod + Limit | AmDemod | RealPart (csdr/chain/analog.py)
// post_serial (stream B, one LANE per chain, 64 chains per wave): the recurrences
//   NfmDeemphasis | DcBlock -> Agc -> Convert(FLOAT, SHORT) -> AdpcmEncoder(sync=True)
//   (analog.py, clientaudio.py).  All lanes walk their streams in lockstep, so 32-256 chains
//   cost about one chain; inputs are prefetched 16 samples ahead, the ADPCM step table lives in
//   LDS and its lookup is off the dependency chain (adpcm_encode_fast).  Runs concurrently
//   with the next block's stream-A work.
#include <type_traits>

#include "owrx_types.h"

namespace owrx {

constexpr int kPostThreads = 256;
constexpr int kMaxSqBlocks = 1024;
constexpr int kMaxSqLen = 3072;  // longest squelch block kept in registers while compacting
constexpr int kBpLds = 6144;     // bandpass input window staged in LDS (48 KiB)

// 1 / prod_{j != i} (i - j) for the 12 Lagrange nodes
OWRX_DEV float lagrange_den(int i) {
    const float fact[12] = {1.0f, 1.0f, 2.0f, 6.0f, 24.0f, 120.0f, 720.0f, 5040.0f,
                            40320.0f, 362880.0f, 3628800.0f, 39916800.0f};
    const float d = fact[i] * fact[11 - i];
    return ((11 - i) & 1) ? -1.0f / d : 1.0f / d;
}

__global__ void __launch_bounds__(kPostThreads)
post_parallel(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts) {
    const ChainPost P = posts[blockIdx.x];
    const int tid = threadIdx.x;
    constexpr int NT = kPostThreads;

    __shared__ ChainStateP S;
    __shared__ int sh_n_fd;
    __shared__ float2 sh_taps[kBpHist + 1];
    __shared__ float2 sh_x[kBpLds];
    __shared__ float sh_power[kMaxSqBlocks];
    __shared__ uint8_t sh_pass[kMaxSqBlocks];

    if (tid == 0) S = *P.pstate;
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

    // ---- 2. Bandpass (inputs + taps staged in LDS when they fit) ------------------------
    const int pend = S.sq_pending;
    const int nbt = P.bp_ntaps;
    const bool lds_bp = nbt > 0 && (kBpHist + n_fd) <= kBpLds;
    if (lds_bp) {
        for (int j = tid; j < kBpHist + n_fd; j += NT) sh_x[j] = P.fd_buf[j];
        for (int t = tid; t < nbt; t += NT) sh_taps[t] = P.bp_taps[t];
        __syncthreads();
    }
    for (int j = tid; j < n_fd; j += NT) {
        const float2* x = P.fd_buf + kBpHist + j;
        float2 y;
        if (lds_bp) {
            const float2* xs = sh_x + kBpHist + j;
            float ar = 0.0f, ai = 0.0f, br = 0.0f, bi = 0.0f;
            int t = 0;
#pragma unroll 4
            for (; t + 1 < nbt; t += 2) {
                const float2 g0 = sh_taps[t], g1 = sh_taps[t + 1];
                const float2 v0 = xs[-t], v1 = xs[-t - 1];
                ar = fmaf(g0.x, v0.x, ar);
                ar = fmaf(-g0.y, v0.y, ar);
                ai = fmaf(g0.x, v0.y, ai);
                ai = fmaf(g0.y, v0.x, ai);
                br = fmaf(g1.x, v1.x, br);
                br = fmaf(-g1.y, v1.y, br);
                bi = fmaf(g1.x, v1.y, bi);
                bi = fmaf(g1.y, v1.x, bi);
            }
            if (t < nbt) {
                const float2 g0 = sh_taps[t];
                const float2 v0 = xs[-t];
                ar = fmaf(g0.x, v0.x, ar);
                ar = fmaf(-g0.y, v0.y, ar);
                ai = fmaf(g0.x, v0.y, ai);
                ai = fmaf(g0.y, v0.x, ai);
            }
            y = make_float2(ar + br, ai + bi);
        } else if (nbt > 0) {
            float ar = 0.0f, ai = 0.0f;
            for (int t = 0; t < nbt; ++t) {
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
    {   // block power: one wave per block, lanes stride the decimated samples
        const int wave = tid >> 6, lane = tid & 63;
        const int nper = (L + P.sq_dec - 1) / P.sq_dec;
        for (int b = wave; b < nb; b += NT / 64) {
            float p = 0.0f;
            for (int m = lane; m < nper; m += 64) {
                const float2 v = P.sq_buf[b * L + m * P.sq_dec];
                p = fmaf(v.x, v.x, p);
                p = fmaf(v.y, v.y, p);
            }
            for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o);
            if (lane == 0) sh_power[b] = p / (float)nper;
        }
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
        P.dem[i] = v;
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
            S.ddc_count = ddc_total;
            if (P.frac_enabled) S.fd_next += n_fd;
            S.fd_count += n_fd;
            S.sq_blocks += nb;
            *P.pstate = S;
            ChainCounts& c = counts[blockIdx.x];
            c.n_ddc = n_new;
            c.n_fd = n_fd;
            c.n_bp = n_fd;
            c.n_sq = nsq;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// post_serial: one lane per chain.  Branch-free hot loop (mode selects instead of exec-mask
// regions), 8 samples per iteration loaded one block ahead, lanes that run out of samples keep
// computing on padding but their state updates / stores are masked by selects.
struct SerState {
    float deemph_y, dc_xp, dc_yp;
    AgcState agc;
    AdpcmFast ad;
};

OWRX_DEV float serial_front(float v, int demod, float alpha, float beta, const AgcParams& agcp,
                            SerState& s, float* dem_out) {
    // NfmDeemphasis and DcBlock both advance (only the chain's own one is ever output)
    const float vd = deemph_step(v, alpha, beta, s.deemph_y);
    const float vc = dcblock_step(v, s.dc_xp, s.dc_yp);
    const float u = demod == 0 ? vd : (demod == 1 ? vc : v);
    *dem_out = u;
    return agc_step(u, agcp, s.agc);
}

template <int OUT, bool DEBUG>
__global__ void __launch_bounds__(64)
post_serial(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts,
            const int* __restrict__ sel, int nsel) {
    __shared__ int16_t T[96];
    const int lane = threadIdx.x;
    for (int i = lane; i < 89; i += 64) T[i] = kAdpcmStep[i];
    __syncthreads();
    const int k = blockIdx.x * 64 + lane;
    const bool active = k < nsel;
    const int c = sel[active ? k : nsel - 1];
    const ChainPost* Pp = posts + c;
    const int n = active ? (int)counts[c].n_sq : 0;
    const int demod = Pp->demod;
    const AgcParams agcp = Pp->agc;
    const float alpha = Pp->deemph_alpha, beta = Pp->deemph_beta;
    uint8_t* __restrict__ out = Pp->out;
    const int64_t cap = Pp->out_cap;
    float* __restrict__ dbg_dem = Pp->dbg_dem;
    float* __restrict__ dbg_agc = Pp->dbg_agc;
    const int64_t dcap = Pp->dbg_cap;
    const float* __restrict__ dem = Pp->dem;
    ChainStateS* sp = Pp->sstate;
    const ChainStateS st0 = *sp;

    SerState S;
    S.deemph_y = st0.deemph_y;
    S.dc_xp = st0.dc_xp;
    S.dc_yp = st0.dc_yp;
    S.agc = st0.agc;
    S.ad = adpcm_fast_init(st0.adpcm, T);
    int has_left = st0.has_left;
    int left_code = st0.left_code;
    int64_t bytes = st0.adpcm_bytes;
    int64_t ob = 0;

    // ADPCM: a pending nibble first pairs with sample 0 (per-lane, once)
    int i0 = 0;
    if (OUT == 1 && has_left && n > 0) {
        float dv;
        const float a = serial_front(dem[0], demod, alpha, beta, agcp, S, &dv);
        if (DEBUG && dcap > 0) {
            dbg_dem[0] = dv;
            dbg_agc[0] = a;
        }
        const int code = adpcm_encode_fast(S.ad, convert_s16(a), T);
        if (ob < cap) out[ob] = (uint8_t)(left_code | (code << 4));
        ob++;
        bytes++;
        has_left = 0;
        i0 = 1;
    }
    const int nrem = n - i0;  // samples in the main loop
    int nmax = nrem;
    for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o));
    const float* __restrict__ src = dem + i0;
    // countdown to the next "SYNC" header (before data byte bytes % 1001 == 0)
    int until_sync = (int)((kAdpcmSyncPeriod - (bytes % kAdpcmSyncPeriod)) % kAdpcmSyncPeriod);

    float cur[8], nxt[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cur[j] = j < nrem ? src[j] : 0.0f;
    int nmin = nrem;
    for (int o = 32; o > 0; o >>= 1) nmin = min(nmin, __shfl_xor(nmin, o));
    auto block8 = [&](int i, auto guard) {
        constexpr bool G = decltype(guard)::value;
            if (OUT == 1) {
    #pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const bool valid = !G || (i + j + 1 < nrem);  // whole pair present
                    const SerState keep = S;
                    float d0, d1;
                    const float a0 = serial_front(cur[j], demod, alpha, beta, agcp, S, &d0);
                    const float a1 = serial_front(cur[j + 1], demod, alpha, beta, agcp, S, &d1);
                    if (valid && until_sync == 0) {  // rare: header carries the state before the pair
                        if (ob + 8 <= cap) {
                            const uint32_t w0 = 0x434e5953u;  // "SYNC"
                            const uint32_t w1 = (uint32_t)(uint16_t)S.ad.index |
                                                ((uint32_t)(uint16_t)S.ad.pred << 16);
                            for (int b = 0; b < 4; ++b) out[ob + b] = (uint8_t)(w0 >> (8 * b));
                            for (int b = 0; b < 4; ++b) out[ob + 4 + b] = (uint8_t)(w1 >> (8 * b));
                        }
                        ob += 8;
                        until_sync = kAdpcmSyncPeriod;
                    }
                    const int lo = adpcm_encode_fast(S.ad, convert_s16(a0), T);
                    const int hi = adpcm_encode_fast(S.ad, convert_s16(a1), T);
                    if (DEBUG) {
                        const int64_t q = i0 + i + j;
                        if (valid && q + 1 < dcap) {
                            dbg_dem[q] = d0;
                            dbg_agc[q] = a0;
                            dbg_dem[q + 1] = d1;
                            dbg_agc[q + 1] = a1;
                        }
                    }
                    if (valid && ob < cap) out[ob] = (uint8_t)(lo | (hi << 4));
                    ob += valid ? 1 : 0;
                    bytes += valid ? 1 : 0;
                    until_sync -= valid ? 1 : 0;
                    if (G && !valid) S = keep;
                }
            } else {
    #pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool valid = !G || (i + j < nrem);
                    const SerState keep = S;
                    float d;
                    const float a = serial_front(cur[j], demod, alpha, beta, agcp, S, &d);
                    if (DEBUG) {
                        const int64_t q = i0 + i + j;
                        if (valid && q < dcap) {
                            dbg_dem[q] = d;
                            dbg_agc[q] = a;
                        }
                    }
                    if (OUT == 2) {
                        if (valid && ob + 4 <= cap) *reinterpret_cast<float*>(out + ob) = a;
                        ob += valid ? 4 : 0;
                    } else {
                        const int16_t s16 = convert_s16(a);
                        if (valid && ob + 2 <= cap) *reinterpret_cast<int16_t*>(out + ob) = s16;
                        ob += valid ? 2 : 0;
                    }
                    if (G && !valid) S = keep;
                }
            }
    };
    for (int i = 0; i < nmax; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) nxt[j] = (i + 8 + j < nrem) ? src[i + 8 + j] : 0.0f;
        if (i + 8 <= nmin)
            block8(i, std::integral_constant<bool, false>{});
        else
            block8(i, std::integral_constant<bool, true>{});
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
    }
    // ADPCM: an odd trailing sample waits for its pair
    if (OUT == 1 && (nrem & 1)) {
        float dv;
        const float a = serial_front(src[nrem - 1], demod, alpha, beta, agcp, S, &dv);
        if (DEBUG && i0 + nrem - 1 < dcap) {
            dbg_dem[i0 + nrem - 1] = dv;
            dbg_agc[i0 + nrem - 1] = a;
        }
        if (until_sync == 0) {
            if (ob + 8 <= cap) {
                const uint32_t w0 = 0x434e5953u;
                const uint32_t w1 = (uint32_t)(uint16_t)S.ad.index |
                                    ((uint32_t)(uint16_t)S.ad.pred << 16);
                for (int b = 0; b < 4; ++b) out[ob + b] = (uint8_t)(w0 >> (8 * b));
                for (int b = 0; b < 4; ++b) out[ob + 4 + b] = (uint8_t)(w1 >> (8 * b));
            }
            ob += 8;
        }
        left_code = adpcm_encode_fast(S.ad, convert_s16(a), T);
        has_left = 1;
    }
    if (!active) return;
    ChainStateS st = st0;
    st.deemph_y = S.deemph_y;
    st.dc_xp = S.dc_xp;
    st.dc_yp = S.dc_yp;
    st.agc = S.agc;
    st.adpcm.index = S.ad.index;
    st.adpcm.pred = S.ad.pred;
    st.has_left = has_left;
    st.left_code = left_code;
    st.adpcm_bytes = bytes;
    *sp = st;
    counts[c].out_bytes = ob;
}

// ADPCM output: the recurrence is split over two waves of one workgroup, pipelined by chunk:
// wave 0 runs deemphasis / DC block + AGC + Convert for chunk c of 64 chains into an LDS ring
// while wave 1 IMA-encodes chunk c-1 (pairs, "SYNC" headers, byte stores).  Per sample each wave
// issues about half of the single-wave instruction stream, so a block of samples costs about
// the longer of the two halves instead of their sum.
constexpr int kSerChunk = 256;

template <bool DEBUG>
__global__ void __launch_bounds__(128)
post_serial_adpcm(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts,
                  const int* __restrict__ sel, int nsel) {
    __shared__ int16_t T[96];
    __shared__ int16_t ring[2][kSerChunk][64];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 89; i += 128) T[i] = kAdpcmStep[i];
    const int k = blockIdx.x * 64 + lane;
    const bool active = k < nsel;
    const int c = sel[active ? k : nsel - 1];
    const ChainPost* Pp = posts + c;
    const int n = active ? (int)counts[c].n_sq : 0;
    int nmax = n;
    for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o));
    const int nchunks = (nmax + kSerChunk - 1) / kSerChunk;
    ChainStateS* sp = Pp->sstate;
    const ChainStateS st0 = *sp;
    __syncthreads();

    if (wave == 0) {
        // ---- front: deemphasis / DC block, AGC, Convert -> LDS ring
        const int demod = Pp->demod;
        const AgcParams agcp = Pp->agc;
        const float alpha = Pp->deemph_alpha, beta = Pp->deemph_beta;
        float* __restrict__ dbg_dem = Pp->dbg_dem;
        float* __restrict__ dbg_agc = Pp->dbg_agc;
        const int64_t dcap = Pp->dbg_cap;
        const float* __restrict__ dem = Pp->dem;
        SerState S;
        S.deemph_y = st0.deemph_y;
        S.dc_xp = st0.dc_xp;
        S.dc_yp = st0.dc_yp;
        S.agc = st0.agc;
        for (int ch = 0; ch <= nchunks; ++ch) {
            if (ch < nchunks) {
                const int base = ch * kSerChunk;
                int16_t(*dst)[64] = ring[ch & 1];
                float nxt[8], cur[8];
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) cur[jj] = base + jj < n ? dem[base + jj] : 0.0f;
                for (int i = 0; i < kSerChunk; i += 8) {
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj)
                        nxt[jj] = (base + i + 8 + jj < n && i + 8 < kSerChunk) ? dem[base + i + 8 + jj] : 0.0f;
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const int q = base + i + jj;
                        const bool valid = q < n;
                        const SerState keep = S;
                        float d;
                        const float a = serial_front(cur[jj], demod, alpha, beta, agcp, S, &d);
                        if (DEBUG && valid && q < dcap) {
                            dbg_dem[q] = d;
                            dbg_agc[q] = a;
                        }
                        dst[i + jj][lane] = convert_s16(a);
                        if (!valid) S = keep;
                    }
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) cur[jj] = nxt[jj];
                }
            }
            __syncthreads();
        }
        if (active) {
            ChainStateS st = st0;
            st.deemph_y = S.deemph_y;
            st.dc_xp = S.dc_xp;
            st.dc_yp = S.dc_yp;
            st.agc = S.agc;
            // adpcm fields are written by wave 1 (separate words of the same struct)
            sp->deemph_y = st.deemph_y;
            sp->dc_xp = st.dc_xp;
            sp->dc_yp = st.dc_yp;
            sp->agc = st.agc;
        }
    } else {
        // ---- IMA-ADPCM with sync frames from the LDS ring (one chunk behind)
        uint8_t* __restrict__ out = Pp->out;
        const int64_t cap = Pp->out_cap;
        AdpcmFast ad = adpcm_fast_init(st0.adpcm, T);
        int has_left = st0.has_left;
        int left = st0.left_code;
        int64_t bytes = st0.adpcm_bytes;
        int until_sync = (int)((kAdpcmSyncPeriod - (bytes % kAdpcmSyncPeriod)) % kAdpcmSyncPeriod);
        int64_t ob = 0;
        for (int ch = 0; ch <= nchunks; ++ch) {
            if (ch > 0) {
                const int base = (ch - 1) * kSerChunk;
                const int16_t(*srcr)[64] = ring[(ch - 1) & 1];
                for (int i = 0; i < kSerChunk; ++i) {
                    const bool valid = base + i < n;
                    const int v = srcr[i][lane];
                    if (valid && !has_left && until_sync == 0) {  // rare: "SYNC" + state
                        if (ob + 8 <= cap) {
                            const uint32_t w1 = (uint32_t)(uint16_t)ad.index |
                                                ((uint32_t)(uint16_t)ad.pred << 16);
                            out[ob] = 'S';
                            out[ob + 1] = 'Y';
                            out[ob + 2] = 'N';
                            out[ob + 3] = 'C';
                            for (int b = 0; b < 4; ++b) out[ob + 4 + b] = (uint8_t)(w1 >> (8 * b));
                        }
                        ob += 8;
                        until_sync = kAdpcmSyncPeriod;
                    }
                    const AdpcmFast keep = ad;
                    const int code = adpcm_encode_fast(ad, v, T);
                    const bool emit = valid && has_left;
                    if (emit && ob < cap) out[ob] = (uint8_t)(left | (code << 4));
                    ob += emit ? 1 : 0;
                    bytes += emit ? 1 : 0;
                    until_sync -= emit ? 1 : 0;
                    left = (valid && !has_left) ? code : left;
                    has_left = valid ? (has_left ^ 1) : has_left;
                    if (!valid) ad = keep;
                }
            }
            __syncthreads();
        }
        if (active) {
            sp->adpcm.index = ad.index;
            sp->adpcm.pred = ad.pred;
            sp->has_left = has_left;
            sp->left_code = left;
            sp->adpcm_bytes = bytes;
            counts[c].out_bytes = ob;
        }
    }
}

hipError_t launch_post_parallel(const ChainPost* posts, int nchains, ChainCounts* counts,
                                hipStream_t st) {
    if (nchains <= 0) return hipSuccess;
    hipLaunchKernelGGL(post_parallel, dim3(nchains), dim3(kPostThreads), 0, st, posts, counts);
    return hipGetLastError();
}

hipError_t launch_post_serial(const ChainPost* posts, ChainCounts* counts, const int* sel,
                              int nsel, int output, int debug, hipStream_t st) {
    if (nsel <= 0) return hipSuccess;
    const dim3 g((nsel + 63) / 64), b(64);
    switch (output * 2 + (debug ? 1 : 0)) {
        case 0: hipLaunchKernelGGL((post_serial<0, false>), g, b, 0, st, posts, counts, sel, nsel); break;
        case 1: hipLaunchKernelGGL((post_serial<0, true>), g, b, 0, st, posts, counts, sel, nsel); break;
        case 2: hipLaunchKernelGGL((post_serial_adpcm<false>), g, dim3(128), 0, st, posts, counts, sel, nsel); break;
        case 3: hipLaunchKernelGGL((post_serial_adpcm<true>), g, dim3(128), 0, st, posts, counts, sel, nsel); break;
        case 4: hipLaunchKernelGGL((post_serial<2, false>), g, b, 0, st, posts, counts, sel, nsel); break;
        case 5: hipLaunchKernelGGL((post_serial<2, true>), g, b, 0, st, posts, counts, sel, nsel); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace owrx
