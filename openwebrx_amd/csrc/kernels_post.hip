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
// post_serial_front (stream B, one LANE per chain, 64 chains per workgroup): the recurrences
//   NfmDeemphasis | DcBlock -> Agc -> Convert(FLOAT, SHORT)  (analog.py, clientaudio.py),
//   pipelined over three waves; all lanes walk their streams in lockstep, so 32-256 chains
//   cost about one chain.
// chain_adpcm (stream C, one LANE per chain): AdpcmEncoder(sync=True).  Streams B and C run
//   concurrently with the next blocks' stream-A work.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "../../include/owrx_amd.h"
#include "owrx_types.h"

namespace owrx {

constexpr int kPostThreads = 256;
constexpr int kMaxSqBlocks = 1024;
constexpr int kMaxSqLen = 3072;  // longest squelch block kept in registers while compacting
constexpr int kBpLds = 6400;     // bandpass input window staged in LDS (50 KiB)
// the staged bandpass on the f32 MFMA (bp_mfma_tiles, round 6); false keeps round 5's packed-FMA
// direct form (A/B builds: -DOWRX_BP_FMA)
#ifdef OWRX_BP_FMA
constexpr bool kBpMfma = false;
#else
constexpr bool kBpMfma = true;
#endif
// Timing ablations of post_parallel's sections (diagnostic builds only, wrong outputs):
// -DOWRX_PP_ABL=1 no bandpass arithmetic, 2 no FractionalDecimator interpolation, 4 no demodulator
// front, 8 no squelch block powers
#ifndef OWRX_PP_ABL
#define OWRX_PP_ABL 0
#endif
// LDS position of bandpass-window sample i: one float2 of padding per 16 with the MFMA tiles,
// whose 16 lanes of one A-operand read are 16 samples apart (a 16-way bank conflict unpadded,
// 17 apart = conflict-free)
OWRX_DEV int bpw(int i) { return kBpMfma ? i + (i >> 4) : i; }

// 1 / prod_{j != i} (i - j) for the 12 Lagrange nodes
OWRX_DEV float lagrange_den(int i) {
    const float fact[12] = {1.0f, 1.0f, 2.0f, 6.0f, 24.0f, 120.0f, 720.0f, 5040.0f,
                            40320.0f, 362880.0f, 3628800.0f, 39916800.0f};
    const float d = fact[i] * fact[11 - i];
    return ((11 - i) & 1) ? -1.0f / d : 1.0f / d;
}

// chunked in-place move dst[0, n) = src[0, n) with src = dst + off, off >= 0: every chunk's
// reads precede its writes, and later chunks read at or beyond off + base + NT, past every index
// written before them
template <typename T, typename PTR>
OWRX_DEV void move_front(PTR buf, int64_t off, int n) {
    const int tid = threadIdx.x;
    for (int base = 0; base < n; base += kPostThreads) {
        const int i = base + tid;
        T v{};
        if (i < n) v = buf[off + i];
        __syncthreads();
        if (i < n) buf[i] = v;
    }
    __syncthreads();
}

// Output-count searches step at most this far from their estimate (normally 0-2 steps).
constexpr int kSearchMax = 64;

// WFM audio: FractionalDecimator(FLOAT, IF/audio, prefilter=True) (csdr/chain/analog.py:69)
// on the FmDemod + Limit output the block appended at wf_buf[kWfHist, +nsq): a causal lowpass
// prefilter, then the 12-point Lagrange interpolator of the Selector's FractionalDecimator at
// positions 6 + k * rate.  Writes the audio-rate samples to `dem` (the serial kernels' input)
// and returns their count.
OWRX_DEV int wfm_audio(const ChainPost& P, ChainStateP& S, int nsq) {
    const int tid = threadIdx.x;
    constexpr int NT = kPostThreads;
    static_assert(kWfHist == NT, "history moves assume one sample per thread");
    __shared__ float sh_pf[kWfHist];
    __shared__ int sh_n;
    const auto wf = gp(P.wf_buf);
    const auto pf = gp(P.pf_buf);
    const auto dem = gp(P.dem);
    const int nt = P.pf_ntaps;
    for (int t = tid; t < nt; t += NT) sh_pf[t] = P.pf_taps[t];
    __syncthreads();
    for (int i = tid; i < nsq; i += NT) {
        const auto x = wf + (kWfHist + i);
        float acc = 0.0f;
        for (int t = 0; t < nt; ++t) acc = fmaf(sh_pf[t], x[-t], acc);
        pf[kWfHist + i] = acc;
    }
    const int64_t total = S.wf_count + nsq;
    const double r = P.wfm_rate;
    if (tid == 0) {
        auto valid = [&](int64_t k) { return (int64_t)ceil(6.0 + (double)k * r) + 5 < total; };
        int64_t ke = (int64_t)floor(((double)total - 12.0) / r);
        if (ke < S.wf_next) ke = S.wf_next;
        // the estimate is within a sample or two; a bounded search (a descriptor with a
        // non-positive or non-finite rate must not spin stream A forever)
        for (int it = 0; it < kSearchMax && valid(ke); ++it) ++ke;
        for (int it = 0; it < kSearchMax && ke > S.wf_next && !valid(ke - 1); ++it) --ke;
        if (!(r > 0.0) || valid(ke) || (ke > S.wf_next && !valid(ke - 1))) ke = S.wf_next;
        sh_n = (int)(ke - S.wf_next);
    }
    __syncthreads();
    const int n = sh_n;
    const int64_t base = S.wf_count - kWfHist;  // absolute IF index of pf[0]
    for (int j = tid; j < n; j += NT) {
        const int64_t k = S.wf_next + j;
        const double w = 6.0 + (double)k * r;
        const int64_t hi = (int64_t)ceil(w);
        const int64_t lo = hi - 6;
        const float u = (float)((w - (double)lo) - 5.5);
        float d[kFdPoints], pre[kFdPoints], suf[kFdPoints];
#pragma unroll
        for (int i = 0; i < kFdPoints; ++i) d[i] = u - ((float)i - 5.5f);
        pre[0] = 1.0f;
#pragma unroll
        for (int i = 1; i < kFdPoints; ++i) pre[i] = pre[i - 1] * d[i - 1];
        suf[kFdPoints - 1] = 1.0f;
#pragma unroll
        for (int i = kFdPoints - 2; i >= 0; --i) suf[i] = suf[i + 1] * d[i + 1];
        const auto x = pf + (lo - base);
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < kFdPoints; ++i) acc = fmaf(pre[i] * suf[i] * lagrange_den(i), x[i], acc);
        dem[j] = acc;
    }
    __syncthreads();
    {   // keep the last kWfHist IF samples of both streams
        const float a = wf[nsq + tid], b = pf[nsq + tid];
        __syncthreads();
        wf[tid] = a;
        pf[tid] = b;
    }
    __syncthreads();
    if (tid == 0) {
        S.wf_count = total;
        S.wf_next += n;
    }
    __syncthreads();
    return n;
}

// One chain-block after the DDC: sections 0-1 (segment reduce, FractionalDecimator), 2
// (Bandpass), 3 (Squelch), 4 (demodulator front; WFM: prefilter + Lagrange to the audio rate).
// PHASE 0 runs a chain whole, except that a chain with a long bandpass (bp_long: WFM's
// 3125-tap complex FIR at 250 kHz) stops after section 1; bp_long then filters it across many
// workgroups and PHASE 2 (post_tail) runs sections 3-4.
// The workgroup's LDS, declared by each kernel (post_body has two instantiations in post_parallel)
constexpr int kBpPad = 272 + 32;  // the bandpass taps zero-padded for the MFMA tiles (>= Kp + 18)
struct PostLds {
    ChainStateP S;
    int n_fd;
    float2 taps[kBpHist + 1];
    float2 hp[kBpPad];  // hp[k] = taps[k - p], zero outside [0, nbt) (bp_mfma_tiles)
    float2 x[kBpLds];  // the bandpass window; with FUSED the chain-block's whole working set
    float power[kMaxSqBlocks];
    uint8_t pass[kMaxSqBlocks];
};

// One tile shape KP (bp_mfma_tiles below picks it).
template <int KP, typename OUT, typename DBG>
OWRX_DEV void bp_mfma_tiles_k(const float2* __restrict__ win, const float2* __restrict__ hp, int nbt,
                              int n_fd, int64_t abs0, OUT out, DBG dbg) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int p = KP - nbt;
    const int a0 = (int)(abs0 & 15);
    const int ntile = (n_fd + a0 + 255) >> 8;
    const int xmax = kBpHist + n_fd - 1;
    const float2* hq = hp + (lane & 15) + (lane >> 4);
    for (int tl = wv; tl < ntile; tl += kPostThreads / 64) {
        const int j0 = 256 * tl - a0;
        const int xi = kBpHist + j0 + 16 * (lane & 15) + p - (lane >> 4);
        f4 ar = {0.0f, 0.0f, 0.0f, 0.0f}, ai = {0.0f, 0.0f, 0.0f, 0.0f};
        // fully unrolled (KP a compile-time constant): the compiler issues the k-steps' LDS reads
        // ahead of the MFMAs that use them (as a runtime loop every k-step waited for its own
        // reads, lgkmcnt(0): post_parallel 39 us per C3 pair)
        float2 xv[KP / 4], hv[KP / 4];
#pragma unroll
        for (int k = 0; k < KP / 4; ++k) {
            xv[k] = win[bpw(min(max(xi - 4 * k, 0), xmax))];
            hv[k] = hq[4 * k];
        }
#pragma unroll
        for (int k = 0; k < KP / 4; ++k) {
            ar = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[k].x, hv[k].x, ar, 0, 0, 0);
            ai = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[k].y, hv[k].x, ai, 0, 0, 0);
            ar = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[k].y, -hv[k].y, ar, 0, 0, 0);
            ai = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[k].x, hv[k].y, ai, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int j = j0 + 16 * (4 * (lane >> 4) + r) + (lane & 15);
            if (j >= 0 && j < n_fd) {
                const float2 y = make_float2(ar[r], ai[r]);
                out(j, y);
                dbg(j, win[bpw(kBpHist + j)], y);
            }
        }
    }
}

// Bandpass (complex FIR, nbt taps) on the f32 MFMA: y[j] = sum_t h[t] x[j - t] for the n_fd
// outputs of the window x[j] = win[bpw(kBpHist + j)] (history below), written to out[j].  Tiles of
// 256 outputs j = j0 + 16 c + a are one 16 x 16 product D[c][a] = sum_s X[c][s] H[s][a] over
// s < Kp (nbt + 15 rounded up to an instantiated 64 / 168 / 272): X[c][s] = x[j0 + 16 c + p - s],
// H[s][a] = h[a - p + s] (p = Kp - nbt), so s runs over the taps t = a - p + s in ascending order
// and the zero taps outside [0, nbt) are exact no-ops; complex as four real products per k-step
// (re: h.x x.x then -h.y x.y; im: h.x x.y then h.y x.x).  v_mfma_f32_16x16x4_f32 is a k-ordered
// f32 fmaf chain (cdna_hip_programming.md, FP32-input MFMA), and each output's row a is its
// absolute index mod 16 (abs0 = that of j = 0), so every output's arithmetic is the same whatever
// the block cut: paired / unpaired and sharded runs stay byte-identical.  One tile is Kp MFMAs of
// 32 cycles on one wave; the FMA form it replaces issued ~600 dependent VALU ops per output at one
// wave per SIMD (30-40 of post_parallel's ~50 us per C3 pair, profiles/r05_post_parallel_phases.txt).
// The window reads are clamped into [0, kBpHist + n_fd): only zero-tap products and outputs past
// n_fd (not stored) see a clamped value, and it is a finite sample of the window.  nbt <= 257.
template <typename OUT, typename DBG>
OWRX_DEV void bp_mfma_tiles(const float2* __restrict__ win, const float2* __restrict__ hp, int nbt,
                            int n_fd, int64_t abs0, OUT out, DBG dbg) {
    if (nbt + 15 <= 64)
        bp_mfma_tiles_k<64>(win, hp, nbt, n_fd, abs0, out, dbg);
    else if (nbt + 15 <= 168)
        bp_mfma_tiles_k<168>(win, hp, nbt, n_fd, abs0, out, dbg);
    else
        bp_mfma_tiles_k<272>(win, hp, nbt, n_fd, abs0, out, dbg);
}
// the tile depth bp_mfma_tiles uses for nbt taps (hp is filled for it)
OWRX_DEV int bp_mfma_kp(int nbt) { return nbt + 15 <= 64 ? 64 : nbt + 15 <= 168 ? 168 : 272; }

// FUSED (PHASE 0): the block's DDC outputs, FractionalDecimator output (the bandpass window) and
// bandpass output stay in LDS -- stages 0-4 read and write the chain's global buffers only for
// the carried histories and the demodulator output -- when its working set fits x[]
// (post_fits): x[0, kBpHist + n_fd) = bandpass window, the DDC outputs (+ history) at the top
// of x[] until the FractionalDecimator consumed them, then the squelch input (pending + this
// block's) at the top.
OWRX_DEV bool post_fits(const ChainPost& P, const StepTable* steps) {
    if (P.bp_long || P.output == OWRX_OUT_IQ || P.bp_hist != kBpHist || P.bp_ntaps > kBpHist + 1)
        return false;
    const int64_t nk = P.step_idx >= 0 ? steps->g[P.step_idx].nk : P.nk;
    const double r = P.frac_enabled ? P.frac_rate : 1.0;
    if (!(r >= 0.5)) return false;
    const int64_t nfd = (int64_t)((double)nk / r) + 2;
    const int64_t win = kBpHist + nfd + (kBpMfma ? (kBpHist + nfd) / 16 + 1 : 0);  // bpw padding
    return win + kFdHist + nk <= kBpLds && win + P.sq_len + nfd <= kBpLds;
}

template <int PHASE, bool FUSED = false>
OWRX_DEV void post_body(const ChainPost& Pin, ChainCounts& cnt, PostLds& Ls,
                        const StepTable* steps = nullptr) {
    ChainPost P = Pin;
    if (PHASE == 0 && P.step_idx >= 0) {  // this block's group fields (StepTable argument)
        const GroupStep g = steps->g[P.step_idx];
        P.k_begin = g.k_begin;
        P.nk = g.nk;
        P.nseg = g.nseg;
    }
    const int tid = threadIdx.x;
    constexpr int NT = kPostThreads;
    const int H = P.bp_hist;  // fd_buf[0, H) = bandpass history

    static_assert(!FUSED || PHASE == 0, "fused: post_parallel only");
    ChainStateP& S = Ls.S;
    int& sh_n_fd = Ls.n_fd;
    float2* const sh_taps = Ls.taps;
    float2* const sh_x = Ls.x;
    float* const sh_power = Ls.power;
    uint8_t* const sh_pass = Ls.pass;

    const auto partial = gp(P.partial);
    const auto ddc_g = gp(P.ddc_buf);
    const auto fd_buf = gp(P.fd_buf);
    const auto sq_g = gp(P.sq_buf);
    const auto dem = gp(P.dem);
    const auto bp_taps = gp(P.bp_taps);
    const auto smeter = gp(P.smeter);
    if (tid == 0) S = *P.pstate;
    __syncthreads();
    int n_new, n_fd;
    int64_t ddc_total;
    if constexpr (PHASE == 0) {

    // ---- 0. FirDecimate output: fixed-order sum of the phase-segment partials ----------
    const int64_t kb = P.k_begin > P.k_first ? P.k_begin : P.k_first;
    const int64_t nn = P.k_begin + P.nk - kb;
    n_new = nn > 0 ? (int)nn : 0;
    const int col0 = (int)(kb - P.k_begin);
    // FUSED: the DDC outputs (with their kFdHist history) at the top of x[], the bandpass
    // window's history at its bottom
    float2* const ddc_l = sh_x + (kBpLds - kFdHist - (n_new > 0 ? n_new : 0));
    const auto ddc_buf = [&]() {
        if constexpr (FUSED) return ddc_l;
        else return ddc_g;
    }();
    if constexpr (FUSED) {
        if (tid < kFdHist) ddc_l[tid] = ddc_g[tid];
        sh_x[bpw(tid)] = fd_buf[tid];  // kBpHist == NT
    }
    if (P.nseg == 1 && P.output != OWRX_OUT_IQ) {
        // one segment (the fast-convolution DDC): eight outputs' loads in flight per thread (the
        // index clamped, not branched on, so the compiler issues them together) -- a load per
        // loop iteration left ~10 full L2 / HBM round trips per thread back to back
        const auto src = partial + (int64_t)P.chain_in_group * P.nk + col0;
        for (int i0 = 0; i0 < n_new; i0 += 8 * NT) {
            float2 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = src[min(i0 + u * NT + tid, n_new - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * NT + tid;
                if (i >= n_new) break;
                const float2 y = make_float2(0.0f + v[u].x, 0.0f + v[u].y);  // as the sum below
                if (P.debug && i < P.dbg_cap) P.dbg_ddc[i] = y;
                ddc_buf[kFdHist + i] = y;
            }
        }
    } else {   // segment partials: 8 independent loads in flight per thread, summed in segment order
        const int64_t sstride = (int64_t)P.group_chains * P.nk;
        const int nseg = P.nseg;
        for (int i = tid; i < n_new; i += NT) {
            const auto src = partial + (int64_t)P.chain_in_group * P.nk + col0 + i;
            float2 y = make_float2(0.0f, 0.0f);
            int s = 0;
            for (; s + 8 <= nseg; s += 8) {
                float2 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = src[(s + u) * sstride];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    y.x += v[u].x;
                    y.y += v[u].y;
                }
            }
            for (; s < nseg; ++s) {
                const float2 v = src[s * sstride];
                y.x += v.x;
                y.y += v.y;
            }
            if (P.debug && i < P.dbg_cap) P.dbg_ddc[i] = y;
            if (P.output == OWRX_OUT_IQ) {  // service Resampler: the DDC output is the product
                reinterpret_cast<float2*>(P.out)[i] = y;
                continue;
            }
            ddc_buf[kFdHist + i] = y;
        }
    }
    if (P.output == OWRX_OUT_IQ) {
        if (tid == 0) {
            S.ddc_count += n_new;
            *P.pstate = S;
            ChainCounts& c = cnt;
            c.out_bytes = (int64_t)n_new * 8;
            c.smeter = 0;
            c.n_ddc = n_new;
            c.n_fd = c.n_bp = c.n_sq = c.n_gate = c.n_front = 0;
        }
        return;
    }
    __syncthreads();
    const int64_t ddc_base = S.ddc_count - kFdHist;  // local index of ddc_buf[0]
    ddc_total = S.ddc_count + n_new;

    // ---- 1. FractionalDecimator ------------------------------------------------------------
    if (P.frac_enabled && !(OWRX_PP_ABL & 2)) {
        if (tid == 0) {
            const double r = P.frac_rate;
            auto valid = [&](int64_t k) {
                const double w = 6.0 + (double)k * r;
                return (int64_t)ceil(w) + 5 < ddc_total;
            };
            int64_t ke = (int64_t)floor(((double)ddc_total - 12.0) / r);
            if (ke < S.fd_next) ke = S.fd_next;
            for (int it = 0; it < kSearchMax && valid(ke); ++it) ++ke;  // bounded (see wfm_audio)
            for (int it = 0; it < kSearchMax && ke > S.fd_next && !valid(ke - 1); ++it) --ke;
            if (!(r > 0.0) || valid(ke) || (ke > S.fd_next && !valid(ke - 1))) ke = S.fd_next;
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
            const auto x = ddc_buf + (lo - ddc_base);
            float2 acc = make_float2(0.0f, 0.0f);
#pragma unroll
            for (int i = 0; i < kFdPoints; ++i) {
                const float L = pre[i] * suf[i] * lagrange_den(i);
                const float2 xi = x[i];
                acc.x = fmaf(L, xi.x, acc.x);
                acc.y = fmaf(L, xi.y, acc.y);
            }
            if constexpr (FUSED) sh_x[bpw(kBpHist + j)] = acc;
            else fd_buf[H + j] = acc;
        }
    } else {
        if (tid == 0) sh_n_fd = n_new;
        for (int j = tid; j < n_new; j += NT) {
            if constexpr (FUSED) sh_x[bpw(kBpHist + j)] = ddc_buf[kFdHist + j];
            else fd_buf[H + j] = ddc_buf[kFdHist + j];
        }
    }
    __syncthreads();
    n_fd = sh_n_fd;
    {   // keep the last kFdHist DDC outputs as interpolator history
        float2 t = make_float2(0.0f, 0.0f);
        if (tid < kFdHist) t = ddc_buf[n_new + tid];
        if constexpr (!FUSED) __syncthreads();
        if (tid < kFdHist) ddc_g[tid] = t;
    }
    if (P.bp_long) {  // the bandpass and everything after it run in bp_long / post_tail
        if (tid == 0) {
            S.ddc_count = ddc_total;
            if (P.frac_enabled) S.fd_next += n_fd;
            S.fd_count += n_fd;
            *P.pstate = S;
            cnt.n_ddc = n_new;
            cnt.n_fd = n_fd;
            cnt.n_bp = n_fd;
        }
        return;
    }
    } else {  // PHASE 2: sections 0-1 ran in post_parallel, section 2 in bp_long
        n_new = (int)cnt.n_ddc;
        n_fd = (int)cnt.n_fd;
        ddc_total = S.ddc_count;
    }
    // secondary FFT input: drop the samples chain_sfft has consumed (keep [sf_next, sf_fill))
    int sf_fill = 0;
    if (P.sf_n > 0) {
        const int next = P.sf_reset ? 0 : S.sf_next;
        const int keep = P.sf_reset ? 0 : S.sf_fill - next;
        __syncthreads();
        move_front<float2>(gp(P.sf_buf), next, keep);
        sf_fill = keep > 0 ? keep : 0;
        if (tid == 0) {
            S.sf_fill = sf_fill;
            S.sf_next = keep > 0 ? 0 : -keep;  // hop > N: the next frame starts past the data
            if (P.sf_reset) S.sf_row_frame = 0;
        }
    }

    // ---- 2. Bandpass (inputs + taps staged in LDS when they fit) ------------------------
    const int pend = S.sq_pending;
    const int nbt = (OWRX_PP_ABL & 1) ? 0 : P.bp_ntaps;
    // (the MFMA form's window is padded, bpw: its last entry must lie inside x[] too)
    const bool lds_bp = !P.bp_long && nbt > 0 && bpw(kBpHist + n_fd - 1) < kBpLds;
    // FUSED: the squelch input (the pending samples, then this block's bandpass output) at the
    // top of x[], where the DDC outputs were
    float2* const sq_l = sh_x + (kBpLds - pend - n_fd);
    const auto sq_buf = [&]() {
        if constexpr (FUSED) return sq_l;
        else return sq_g;
    }();
    if constexpr (FUSED) {
        __syncthreads();  // every read of the DDC outputs (interpolator history) is done
        // the pending squelch samples: four loads in flight per thread (clamped index)
        for (int j0 = 0; j0 < pend; j0 += 4 * NT) {
            float2 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = sq_g[min(j0 + u * NT + tid, pend - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j0 + u * NT + tid < pend) sq_l[j0 + u * NT + tid] = v[u];
        }
        if (lds_bp && kBpMfma) {
            const int Kp = bp_mfma_kp(nbt);
            for (int k = tid; k < kBpPad; k += NT) {
                const int t = k - (Kp - nbt);
                Ls.hp[k] = (t >= 0 && t < nbt) ? bp_taps[t] : make_float2(0.0f, 0.0f);
            }
        } else {
            for (int t = tid; t < nbt; t += NT) sh_taps[t] = bp_taps[t];
        }
        __syncthreads();
    } else if (lds_bp) {
        for (int j = tid; j < kBpHist + n_fd; j += NT) sh_x[bpw(j)] = fd_buf[j];
        if (kBpMfma) {
            const int Kp = bp_mfma_kp(nbt);
            for (int k = tid; k < kBpPad; k += NT) {
                const int t = k - (Kp - nbt);
                Ls.hp[k] = (t >= 0 && t < nbt) ? bp_taps[t] : make_float2(0.0f, 0.0f);
            }
        } else {
            for (int t = tid; t < nbt; t += NT) sh_taps[t] = bp_taps[t];
        }
        __syncthreads();
    }
    const auto fd_win = [&]() {
        if constexpr (FUSED) return sh_x;
        else return fd_buf;
    }();
    typedef float bp_f2 __attribute__((ext_vector_type(2)));
    int j = tid;
    if (lds_bp && kBpMfma) {
        bp_mfma_tiles(
            sh_x, Ls.hp, nbt, n_fd, S.fd_count, [&](int jj, float2 y) { sq_buf[pend + jj] = y; },
            [&](int jj, float2 x0, float2 y) {
                if (P.debug && jj < P.dbg_cap) {
                    P.dbg_fd[jj] = x0;
                    P.dbg_bp[jj] = y;
                }
            });
        j = n_fd;
    } else if (lds_bp) {
        // four outputs per thread in flight (j, j + NT, j + 2 NT, j + 3 NT): each output is two
        // dependent FMA chains of ~nbt steps, so one output at a time left the loop latency-bound
        // (~55 cycles per tap and output; phase stamps: 30-40 of post_parallel's ~50 us per C3
        // pair).  Per output the FMA order is unchanged (bit-identical); the block's x reads sit
        // at constant offsets (r NT) from one address.  Whole blocks only; the rest below.
        constexpr int kBpR = 4;
        for (; j + (kBpR - 1) * NT < n_fd; j += kBpR * NT) {
            const float2* xs = sh_x + kBpHist + j;
            bp_f2 a[kBpR], b[kBpR];
#pragma unroll
            for (int r = 0; r < kBpR; ++r) a[r] = b[r] = bp_f2{0.0f, 0.0f};
            int t = 0;
#pragma unroll 2
            for (; t + 1 < nbt; t += 2) {
                const float2 g0 = sh_taps[t], g1 = sh_taps[t + 1];
#pragma unroll
                for (int r = 0; r < kBpR; ++r) {
                    const float2 v0 = xs[r * NT - t], v1 = xs[r * NT - t - 1];
                    a[r] = __builtin_elementwise_fma(bp_f2{g0.x, g0.x}, bp_f2{v0.x, v0.y}, a[r]);
                    a[r] = __builtin_elementwise_fma(bp_f2{-g0.y, g0.y}, bp_f2{v0.y, v0.x}, a[r]);
                    b[r] = __builtin_elementwise_fma(bp_f2{g1.x, g1.x}, bp_f2{v1.x, v1.y}, b[r]);
                    b[r] = __builtin_elementwise_fma(bp_f2{-g1.y, g1.y}, bp_f2{v1.y, v1.x}, b[r]);
                }
            }
            if (t < nbt) {
                const float2 g0 = sh_taps[t];
#pragma unroll
                for (int r = 0; r < kBpR; ++r) {
                    const float2 v0 = xs[r * NT - t];
                    a[r] = __builtin_elementwise_fma(bp_f2{g0.x, g0.x}, bp_f2{v0.x, v0.y}, a[r]);
                    a[r] = __builtin_elementwise_fma(bp_f2{-g0.y, g0.y}, bp_f2{v0.y, v0.x}, a[r]);
                }
            }
#pragma unroll
            for (int r = 0; r < kBpR; ++r) {
                const int jr = j + r * NT;
                const float2 y = make_float2(a[r].x + b[r].x, a[r].y + b[r].y);
                sq_buf[pend + jr] = y;
                if (P.debug && jr < P.dbg_cap) {
                    P.dbg_fd[jr] = xs[r * NT];
                    P.dbg_bp[jr] = y;
                }
            }
        }
    }
    for (; j < (P.bp_long ? 0 : n_fd); j += NT) {
        const auto x = fd_win + kBpHist + j;
        float2 y;
        if (lds_bp) {
            // packed FP32 (v_pk_fma_f32): each complex MAC is two packed FMAs -- (re, im) +=
            // (g.x, g.x) (v.x, v.y), then += (-g.y, g.y) (v.y, v.x) -- the same FMA sequence per
            // accumulator as four scalar FMAs (bit-identical) at half the instructions; even taps
            // in a, odd in b
            const float2* xs = sh_x + kBpHist + j;
            bp_f2 a = bp_f2{0.0f, 0.0f}, b = bp_f2{0.0f, 0.0f};
            int t = 0;
#pragma unroll 4
            for (; t + 1 < nbt; t += 2) {
                const float2 g0 = sh_taps[t], g1 = sh_taps[t + 1];
                const float2 v0 = xs[-t], v1 = xs[-t - 1];
                a = __builtin_elementwise_fma(bp_f2{g0.x, g0.x}, bp_f2{v0.x, v0.y}, a);
                a = __builtin_elementwise_fma(bp_f2{-g0.y, g0.y}, bp_f2{v0.y, v0.x}, a);
                b = __builtin_elementwise_fma(bp_f2{g1.x, g1.x}, bp_f2{v1.x, v1.y}, b);
                b = __builtin_elementwise_fma(bp_f2{-g1.y, g1.y}, bp_f2{v1.y, v1.x}, b);
            }
            if (t < nbt) {
                const float2 g0 = sh_taps[t];
                const float2 v0 = xs[-t];
                a = __builtin_elementwise_fma(bp_f2{g0.x, g0.x}, bp_f2{v0.x, v0.y}, a);
                a = __builtin_elementwise_fma(bp_f2{-g0.y, g0.y}, bp_f2{v0.y, v0.x}, a);
            }
            y = make_float2(a.x + b.x, a.y + b.y);
        } else if (nbt > 0) {
            float ar = 0.0f, ai = 0.0f;
            for (int t = 0; t < nbt; ++t) {
                const float2 g = bp_taps[t];
                const float2 v = x[-t];
                ar = fmaf(g.x, v.x, ar);
                ar = fmaf(-g.y, v.y, ar);
                ai = fmaf(g.x, v.y, ai);
                ai = fmaf(g.y, v.x, ai);
            }
            y = make_float2(ar, ai);
        } else if constexpr (FUSED) {
            y = sh_x[bpw(kBpHist + j)];  // (the LDS window is padded: bpw)
        } else {
            y = x[0];
        }
        sq_buf[pend + j] = y;
        if (P.debug && j < P.dbg_cap) {
            P.dbg_fd[j] = FUSED ? y : x[0];
            P.dbg_bp[j] = y;
        }
    }
    __syncthreads();
    if constexpr (FUSED) {
        fd_buf[tid] = sh_x[bpw(n_fd + tid)];  // keep the last kBpHist bandpass inputs
    } else if (P.bp_long) {  // keep the last H bandpass inputs
        move_front<float2>(fd_buf, n_fd, H);
    } else {  // keep the last kBpHist bandpass inputs
        const float2 t = fd_buf[n_fd + tid];  // kBpHist == NT
        __syncthreads();
        fd_buf[tid] = t;
    }

    // ---- 3. Squelch: block powers, gate, s-meter ---------------------------------------
    const int L = P.sq_len;
    const int total = pend + n_fd;
    const int nb = total / L;
    {   // block power: one wave per block, lanes stride the decimated samples
        const int wave = tid >> 6, lane = tid & 63;
        const int nper = (L + P.sq_dec - 1) / P.sq_dec;
        for (int b = wave; b < ((OWRX_PP_ABL & 8) ? 0 : nb); b += NT / 64) {
            float p = 0.0f;
            for (int m = lane; m < nper; m += 64) {
                const float2 v = sq_buf[b * L + m * P.sq_dec];
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
                if (ns < P.smeter_cap) smeter[ns] = power;
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
        cnt.smeter = ns < P.smeter_cap ? ns : P.smeter_cap;
    }
    __syncthreads();

    // ---- 4. demodulator front (per-sample independent) ------------------------------------
    const int nsq = nb * L;
    const float2 fm_prev0 = S.fm_last;
    const bool sel_out = P.output == OWRX_OUT_SEL;  // the Selector output is the product
    for (int i = tid; i < ((OWRX_PP_ABL & 4) ? 0 : nsq); i += NT) {
        const float2 x = sh_pass[i / L] ? sq_buf[i] : make_float2(0.0f, 0.0f);
        if (sel_out) {
            if (P.debug && i < P.dbg_cap) P.dbg_sq[i] = x;
            if ((int64_t)(i + 1) * 8 <= P.out_cap) reinterpret_cast<float2*>(P.out)[i] = x;
            continue;
        }
        if (P.debug && i < P.dbg_cap) P.dbg_sq[i] = x;
        if (P.tap_sq && i < P.tap_sq_cap) P.tap_sq[i] = x;  // selectorBuffer readers
        if (P.sf_n > 0) P.sf_buf[sf_fill + i] = x;  // Selector output -> secondary FFT
        if (P.demod == OWRX_DEMOD_SAM) {  // SAm: the Selector output for chain_afc (cf32)
            gp(reinterpret_cast<float2*>(P.dem))[i] = x;
            continue;
        }
        float v;
        if (P.demod == 0 || P.demod == 3) {
            float2 prev = fm_prev0;
            if (i > 0) prev = sh_pass[(i - 1) / L] ? sq_buf[i - 1] : make_float2(0.0f, 0.0f);
            v = limit_step(fm_step(x, prev), 1.0f);
        } else if (P.demod == 1) {
            v = am_step(x);
        } else {
            v = x.x;
        }
        if (P.demod == 3)
            P.wf_buf[kWfHist + i] = v;  // WFM: FmDemod + Limit at the IF rate
        else
            dem[i] = v;
    }
    __syncthreads();
    int n_audio = nsq;
    if (P.demod == 3 && !sel_out) n_audio = wfm_audio(P, S, nsq);
    {   // move the incomplete squelch block to the front
        const int rem = total - nsq;
        float2 last = S.fm_last;
        if (nsq > 0) last = sh_pass[nb - 1] ? sq_buf[nsq - 1] : make_float2(0.0f, 0.0f);
        if constexpr (FUSED) {
            for (int i = tid; i < rem; i += NT) sq_g[i] = sq_buf[nsq + i];
        } else if (P.sq_len > kMaxSqLen) {  // WFM: 15625-sample squelch blocks
            __syncthreads();
            move_front<float2>(sq_buf, nsq, rem);
        } else {
            float2 t[kMaxSqLen / NT];
#pragma unroll
            for (int m = 0; m < kMaxSqLen / NT; ++m) {
                const int i = tid + m * NT;
                if (i < rem) t[m] = sq_buf[nsq + i];
            }
            __syncthreads();
#pragma unroll
            for (int m = 0; m < kMaxSqLen / NT; ++m) {
                const int i = tid + m * NT;
                if (i < rem) sq_buf[i] = t[m];
            }
        }
        if (tid == 0) {
            S.fm_last = last;
            S.sq_pending = rem;
            if (PHASE == 0) {
                S.ddc_count = ddc_total;
                if (P.frac_enabled) S.fd_next += n_fd;
                S.fd_count += n_fd;
            }
            S.sq_blocks += nb;
            if (P.sf_n > 0) S.sf_fill = sf_fill + nsq;
            *P.pstate = S;
            ChainCounts& c = cnt;
            c.n_ddc = n_new;
            c.n_fd = n_fd;
            c.n_bp = n_fd;
            c.n_sq = n_audio;
            c.n_front = n_audio;
            c.n_gate = nsq;
            if (sel_out) c.out_bytes = min((int64_t)nsq * 8, P.out_cap & ~(int64_t)7);
        }
    }
}

__global__ void __launch_bounds__(kPostThreads)
post_parallel(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts, StepTable steps) {
    __shared__ PostLds Ls;
    const ChainPost& P = posts[blockIdx.x];
    if (post_fits(P, &steps))
        post_body<0, true>(P, counts[blockIdx.x], Ls, &steps);
    else
        post_body<0, false>(P, counts[blockIdx.x], Ls, &steps);
}

// sections 3-4 of the long-bandpass chains listed in idx (after bp_long)
__global__ void __launch_bounds__(kPostThreads)
post_tail(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts,
          const int* __restrict__ idx) {
    __shared__ PostLds Ls;
    const int i = idx[blockIdx.x];
    post_body<2>(posts[i], counts[i], Ls);
}

// Bandpass(transition=320/IF, use_fft=True) (csdr/chain/selector.py:115-117) for chains whose
// FIR is too long for the in-kernel path (WFM: 3125 complex taps at 250 kHz): grid (tiles,
// chains); each workgroup stages the taps and its input window in LDS and computes kBlTile
// outputs (two per thread) of y[j] = sum_t g[t] x[j - t] into the squelch input.
constexpr int kBlTile = 512;
constexpr int kBlMaxTaps = 4095;

__global__ void __launch_bounds__(kPostThreads)
bp_long(const ChainPost* __restrict__ posts, const ChainCounts* __restrict__ counts,
        const int* __restrict__ idx) {
    const int c = idx[blockIdx.y];
    const ChainPost& P = posts[c];
    const int n_fd = (int)counts[c].n_fd;
    const int j0 = blockIdx.x * kBlTile;
    if (j0 >= n_fd) return;
    const int nt = P.bp_ntaps;
    const int H = P.bp_hist;
    const int tid = threadIdx.x;
    const auto fd = gp(P.fd_buf);
    const int pend = P.pstate->sq_pending;
    const auto sq = gp(P.sq_buf);
    if (nt == 0) {  // bandpass switched off (setBandpass(None, None)): pass through
        for (int jl = tid; jl < kBlTile && j0 + jl < n_fd; jl += kPostThreads) {
            const int j = j0 + jl;
            const float2 y = fd[H + j];
            sq[pend + j] = y;
            if (P.debug && j < P.dbg_cap) {
                P.dbg_fd[j] = y;
                P.dbg_bp[j] = y;
            }
        }
        return;
    }
    extern __shared__ __align__(16) float2 bl_sm[];
    float2* taps = bl_sm;
    float2* xs = bl_sm + ((nt + 3) & ~3);
    const int nw = min(kBlTile, n_fd - j0) + nt - 1;
    for (int t = tid; t < nt; t += kPostThreads) taps[t] = P.bp_taps[t];
    const int64_t x0 = (int64_t)H + j0 - (nt - 1);  // >= 0: H >= nt - 1
    for (int m = tid; m < nw; m += kPostThreads) xs[m] = fd[x0 + m];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int jl = tid + h * kPostThreads;
        if (j0 + jl >= n_fd) break;
        const float2* x = xs + jl + (nt - 1);
        float ar = 0.0f, ai = 0.0f, br = 0.0f, bi = 0.0f;
        int t = 0;
#pragma unroll 4
        for (; t + 1 < nt; t += 2) {
            const float2 g0 = taps[t], g1 = taps[t + 1];
            const float2 v0 = x[-t], v1 = x[-t - 1];
            ar = fmaf(g0.x, v0.x, ar);
            ar = fmaf(-g0.y, v0.y, ar);
            ai = fmaf(g0.x, v0.y, ai);
            ai = fmaf(g0.y, v0.x, ai);
            br = fmaf(g1.x, v1.x, br);
            br = fmaf(-g1.y, v1.y, br);
            bi = fmaf(g1.x, v1.y, bi);
            bi = fmaf(g1.y, v1.x, bi);
        }
        if (t < nt) {
            const float2 g0 = taps[t];
            const float2 v0 = x[-t];
            ar = fmaf(g0.x, v0.x, ar);
            ar = fmaf(-g0.y, v0.y, ar);
            ai = fmaf(g0.x, v0.y, ai);
            ai = fmaf(g0.y, v0.x, ai);
        }
        const float2 y = make_float2(ar + br, ai + bi);
        const int j = j0 + jl;
        sq[pend + j] = y;
        if (P.debug && j < P.dbg_cap) {
            P.dbg_fd[j] = x[0];
            P.dbg_bp[j] = y;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// post_serial_front: the per-chain recurrences after the demodulator, one LANE per chain
// (64 chains per workgroup), four waves pipelined by chunks of kSerChunk samples through LDS:
//   wave 0    NfmDeemphasis | DcBlock and the AGC envelope (chunk c) -> (u, env) in LDS
//   wave 1    loads chunk c + 1 of every chain into LDS (the only wave with global loads, so
//             its waits never cover outstanding stores), and a quarter of the gain work
//   wave 1-3  gain = reference / env (clamped), a = u * gain (chunk c - 1; the IEEE division
//             makes this the heavier half)
//   wave 2-3  Convert + store (chunk c - 2): int16 to the output slot (S16), float (F32), or
//             the chain's int16 scratch for the ADPCM encoder (chain_adpcm below)
// The arithmetic is exactly deemph_step / dcblock_step / agc_step / convert_s16 split at the
// AGC gain, so the result is bit-identical to the sequential order (oracle orc_agc etc.).
constexpr int kSerChunk = 64;
constexpr int kFrontThreads = 256;  // wave 0: recurrences, waves 1-3: gain + Convert

// Lane -> chain for the serial kernels.  The host orders `sel` by demodulator and pads every
// demodulator's run to whole workgroups with -1 (inactive lanes), so the demodulator is
// uniform per workgroup; sel[first lane of the workgroup] is always a real chain.
struct SerLane {
    int c;        // chain (a real one even for inactive lanes)
    bool active;
};
OWRX_DEV SerLane ser_lane(const int* __restrict__ sel, int nsel) {
    const int k = blockIdx.x * 64 + (threadIdx.x & 63);
    const int c0 = sel[blockIdx.x * 64];
    const int cs = k < nsel ? sel[k] : -1;
    return SerLane{cs >= 0 ? cs : c0, cs >= 0};
}

template <int OUT, bool DEBUG, bool NR>
__global__ void __launch_bounds__(kFrontThreads)
post_serial_front(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts,
                  const int* __restrict__ sel, int nsel) {
    __shared__ float2 ue[2][kSerChunk][64];  // wave 0 -> waves 1, 2: (u, envelope)
    __shared__ float as_[2][kSerChunk][65];  // waves 1-3: AGC output, [sample][chain], padded
    __shared__ float in_[2][kSerChunk][65];  // waves 1-3 -> wave 0: demodulator output, staged
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const SerLane sl = ser_lane(sel, nsel);
    const int c = sl.c;
    const ChainPost* Pp = posts + c;
    const int n = sl.active ? (int)counts[c].n_sq : 0;
    // idle lanes compute along on their workgroup's first chain and never store
    int nmax = n, nmin = sl.active ? n : INT_MAX;
    for (int o = 32; o > 0; o >>= 1) {
        nmax = max(nmax, __shfl_xor(nmax, o));
        nmin = min(nmin, __shfl_xor(nmin, o));
    }
    const int nchunks = (nmax + kSerChunk - 1) / kSerChunk;
    const int nfull = nmin / kSerChunk;  // chunks in which every active lane has kSerChunk samples
    const AgcParams agcp = Pp->agc;
    ChainStateS* sp = Pp->sstate;
    // uniform (see ser_lane); SAm continues as AM after chain_afc (DcBlock -> Agc / Gain)
    int demod = __builtin_amdgcn_readfirstlane(Pp->demod);
    if (demod == OWRX_DEMOD_SAM) demod = OWRX_DEMOD_AM;
    // Gain(agc.max_gain) instead of the Agc (RawAm / RawSAm): envelope 0 selects the clamp
    const bool fixed_gain = Pp->fixed_gain != 0;

    // Data movement is lane = chain, in quads of samples (samples 4q .. 4q+3 of a chunk).
    // Input staging: the recurrences are a few dependent VALU ops per sample, so a global load
    // per sample (an L2 / MALL round trip: the demodulator output was written by other CUs)
    // would set the pace; wave 1 loads chunk c + 1 (16-B loads from each chain's own buffer)
    // while wave 0 walks chunk c out of LDS.
    constexpr int kQuads = kSerChunk / 4;
    const auto dem_in = gp(reinterpret_cast<const float4*>(Pp->dem));
    float4 pre[kQuads];
    // unconditional loads (the quad index clamped to the lane's last quad), zeroed past n when
    // stored to LDS (after wave 1's gain work, which the loads' latency hides behind): a per-lane
    // `i < n ?` load is a branch the compiler may close with a full wait before the next one (it
    // did for the first chunk: 16 memory latencies per launch)
    const int last_q = n > 0 ? (n - 1) >> 2 : 0;
    auto stage_load = [&](int ch) {
#pragma unroll
        for (int q = 0; q < kQuads; ++q) pre[q] = dem_in[min(ch * kQuads + q, last_q)];
    };
    auto stage_store = [&](int ch) {
#pragma unroll
        for (int q = 0; q < kQuads; ++q) {
            if (ch * kSerChunk + 4 * q >= n) pre[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            in_[ch & 1][4 * q][lane] = pre[q].x;
            in_[ch & 1][4 * q + 1][lane] = pre[q].y;
            in_[ch & 1][4 * q + 2][lane] = pre[q].z;
            in_[ch & 1][4 * q + 3][lane] = pre[q].w;
        }
    };
    if (wave == 1 && nchunks > 0) {
        stage_load(0);
        stage_store(0);
    }
    __syncthreads();

    if (wave == 0) {
        // ---- recurrences: NfmDeemphasis | DcBlock, AGC envelope -> (u, env)
        float deemph_y = sp->deemph_y, dc_xp = sp->dc_xp, dc_yp = sp->dc_yp;
        AgcState agc = sp->agc;
        const float alpha = Pp->deemph_alpha, beta = Pp->deemph_beta;
        auto run = [&](auto dm, auto fl, int ch) {
            constexpr int DM = decltype(dm)::value;
            constexpr bool FULL = decltype(fl)::value;
            const int base = ch * kSerChunk;
            float2(*dst)[64] = ue[ch & 1];
            const float(*src)[65] = in_[ch & 1];
            for (int i = 0; i < kSerChunk; i += 8) {
                float cur[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) cur[j] = src[i + j][lane];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float v = cur[j];
                    const float ky = deemph_y, kx = dc_xp, kyy = dc_yp, ke = agc.env;
                    float u;
                    if (DM == 0 || DM == 3) u = deemph_step(v, alpha, beta, deemph_y);
                    else if (DM == 1) u = dcblock_step(v, dc_xp, dc_yp);
                    else u = v;
                    {
#pragma clang fp contract(off)
                        const float a = fabsf(u);
                        const float d = a - agc.env;
                        // rate * d, rate = attack if d > 0 else decay: attack > decay > 0 in
                        // every profile (design.cpp agc_params), so it is max(attack d, decay d)
                        // exactly (rounding is monotonic; d = +-0 gives +-0 either way) -- no
                        // compare / select and its lane-mask wait states on the recurrence
                        const float t = fmaxf(agcp.attack * d, agcp.decay * d);
                        agc.env = agc.env + t;
                    }
                    // WFm has no Agc (csdr/chain/analog.py:66-71): envelope = reference makes
                    // the gain exactly 1 (correctly rounded x / x; the host keeps max_gain >= 1)
                    dst[i + j][lane] = make_float2(u, DM == 3 ? agcp.reference
                                                          : fixed_gain ? 0.0f : agc.env);
                    if (!FULL && base + i + j >= n) {  // past this lane's end: keep state
                        deemph_y = ky;
                        dc_xp = kx;
                        dc_yp = kyy;
                        agc.env = ke;
                    }
                }
            }
        };
        auto run_dm = [&](auto dm, int ch) {
            if (ch < nfull) run(dm, std::true_type{}, ch);
            else run(dm, std::false_type{}, ch);
        };
        for (int it = 0; it < nchunks + 2; ++it) {
            if (it < nchunks) {
                if (demod == 0) run_dm(std::integral_constant<int, 0>{}, it);
                else if (demod == 1) run_dm(std::integral_constant<int, 1>{}, it);
                else if (demod == 3) run_dm(std::integral_constant<int, 3>{}, it);  // WfmDeemphasis
                else run_dm(std::integral_constant<int, 2>{}, it);
            }
            __syncthreads();
        }
        if (sl.active) {
            sp->deemph_y = deemph_y;
            sp->dc_xp = dc_xp;
            sp->dc_yp = dc_yp;
            sp->agc = agc;
            if (OUT == 2) counts[c].out_bytes = 4 * (int64_t)n;
            if (OUT == 0) counts[c].out_bytes = 2 * (int64_t)n;
        }
    } else {
        // ---- gain + Convert (waves 1..3 take every third sample), one chunk behind; a chain
        // with a NoiseFilter stores the AGC output for chain_nr instead (Convert follows it).
        // The results go through LDS (as_) and are written out one more chunk behind, lane =
        // chain, a quad of samples per store (8-B int16 / 16-B float vectors where aligned).
        const bool nr = NR && sl.active;
        const int64_t nr_fill = nr ? kNrHop + Pp->nr_state->pend : 0;
        int64_t lim = 0;
        void* dptr = nullptr;
        if (sl.active) {
            if (NR) {
                lim = n;
                dptr = Pp->nr_in + nr_fill;
            } else if (OUT == 2) {
                lim = min((int64_t)n, Pp->out_cap / 4);
                dptr = Pp->out;
            } else if (OUT == 0) {
                lim = min((int64_t)n, Pp->out_cap / 2);
                dptr = Pp->out;
            } else {
                lim = n;  // the chain's int16 scratch (read by chain_adpcm)
                dptr = Pp->s16;
            }
        }
        constexpr bool kF32 = NR || OUT == 2;
        const bool vec = ((uintptr_t)dptr & (kF32 ? 15 : 7)) == 0;
        float* const tap = sl.active ? Pp->tap_agc : nullptr;
        int tap_lim = tap ? (int)min<int64_t>(Pp->tap_agc_cap, INT_MAX) : 0;
        float g_ref = agcp.reference, g_max = agcp.max_gain;
        // materialise the descriptor loads here: a first use inside the loop would wait for
        // every load in flight there (vmcnt(0)), including wave 1's staging loads
        asm volatile("" : "+v"(tap_lim), "+v"(g_ref), "+v"(g_max), "+v"(lim), "+v"(dptr));
        // gain samples of a chunk: j % 8 in {0, 1} (wave 1), {2, 3, 4} (wave 2), {5, 6, 7} (3);
        // fully unrolled per wave (no inner loop: a loop header would make the compiler wait
        // for wave 1's in-flight loads before the gain work instead of after it)
        // the audioBuffer tap is rare: its per-sample store test only in the instantiation
        // that has one (wave-uniform choice)
        const bool any_tap = __any(tap_lim > 0);
        auto gain = [&](auto lo_c, auto cnt_c, auto tap_c, int ch) {
            constexpr int LO = decltype(lo_c)::value, CNT = decltype(cnt_c)::value;
            constexpr bool TAP = decltype(tap_c)::value;
            const int base = ch * kSerChunk;
            const float2(*srcu)[64] = ue[ch & 1];
            const bool full = ch < nfull;
#pragma unroll
            for (int g8 = 0; g8 < kSerChunk / 8; ++g8) {
#pragma unroll
                for (int r = 0; r < CNT; ++r) {
                    const int j = g8 * 8 + LO + r;
                    const float2 q = srcu[j][lane];
                    float a;
                    {
#pragma clang fp contract(off)
                        // (q.y > 0 ? reference / q.y : max_gain) clamped to max_gain: the envelope
                        // is never negative or -0, and reference / +0 = +inf clamps to max_gain,
                        // so one min (no compare / select pairs and their wait states)
                        const float g = fminf(g_ref / q.y, g_max);
                        a = g * q.x;
                    }
                    as_[ch & 1][j][lane] = a;
                    if (TAP) {  // audioBuffer readers (a secondary demodulator on the audio)
                        const int qi = base + j;
                        if ((full || qi < n) && qi < tap_lim) gp(tap)[qi] = a;
                    }
                    if (DEBUG) {
                        const int64_t qi = base + j;
                        const bool valid = sl.active && (full || qi < n);
                        if (valid && qi < Pp->dbg_cap) {
                            gp(Pp->dbg_dem)[qi] = q.x;
                            gp(Pp->dbg_agc)[qi] = a;
                        }
                    }
                }
            }
        };
        using I0 = std::integral_constant<int, 0>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        using I5 = std::integral_constant<int, 5>;
        for (int it = 0; it < nchunks + 2; ++it) {
            const bool ld = wave == 1 && it + 1 < nchunks;  // stage chunk it + 1 for wave 0
            if (ld) stage_load(it + 1);
            const int ch = it - 1;
            if (ch >= 0 && ch < nchunks) {
                if (any_tap) {
                    if (wave == 1) gain(I0{}, I2{}, std::true_type{}, ch);
                    else if (wave == 2) gain(I2{}, I3{}, std::true_type{}, ch);
                    else gain(I5{}, I3{}, std::true_type{}, ch);
                } else {
                    if (wave == 1) gain(I0{}, I2{}, std::false_type{}, ch);
                    else if (wave == 2) gain(I2{}, I3{}, std::false_type{}, ch);
                    else gain(I5{}, I3{}, std::false_type{}, ch);
                }
            }
            const int w = it - 2;  // chunk written out this iteration (as_ complete since the
            if (w >= 0 && wave >= 2) {  // previous barrier); quads alternate waves 2, 3
                const float(*src)[65] = as_[w & 1];
#pragma unroll
                for (int k = 0; k < kQuads / 2; ++k) {
                    const int q = wave - 2 + 2 * k;
                    const int64_t i0 = (int64_t)w * kSerChunk + 4 * q;
                    if (i0 >= lim) continue;
                    const float v0 = src[4 * q][lane], v1 = src[4 * q + 1][lane];
                    const float v2 = src[4 * q + 2][lane], v3 = src[4 * q + 3][lane];
                    if (kF32) {
                        float* d = reinterpret_cast<float*>(dptr) + i0;
                        if (vec && i0 + 4 <= lim) {
                            *gp(reinterpret_cast<float4*>(d)) = make_float4(v0, v1, v2, v3);
                        } else {
                            gp(d)[0] = v0;
                            if (i0 + 1 < lim) gp(d)[1] = v1;
                            if (i0 + 2 < lim) gp(d)[2] = v2;
                            if (i0 + 3 < lim) gp(d)[3] = v3;
                        }
                    } else {
                        int16_t* d = reinterpret_cast<int16_t*>(dptr) + i0;
                        const int16_t s0 = convert_s16(v0), s1 = convert_s16(v1);
                        const int16_t s2 = convert_s16(v2), s3 = convert_s16(v3);
                        if (vec && i0 + 4 <= lim) {
                            const uint2 pk = make_uint2((uint32_t)(uint16_t)s0 | ((uint32_t)(uint16_t)s1 << 16),
                                                        (uint32_t)(uint16_t)s2 | ((uint32_t)(uint16_t)s3 << 16));
                            *gp(reinterpret_cast<uint2*>(d)) = pk;
                        } else {
                            gp(d)[0] = s0;
                            if (i0 + 1 < lim) gp(d)[1] = s1;
                            if (i0 + 2 < lim) gp(d)[2] = s2;
                            if (i0 + 3 < lim) gp(d)[3] = s3;
                        }
                    }
                }
            }
            if (ld) stage_store(it + 1);
            __syncthreads();
        }
    }
}

// Afc -> RealPart of the SAm / RawSAm chains (csdr/chain/analog.py:141-167), one LANE per chain
// (64 per workgroup) on the serial stream ahead of post_serial_front: the front left the
// Selector output (cf32) in the chain's dem slot; the corrected real part goes back in place
// (sample i's float lands at float index i, below the cf32 still to be read at 2 (i + 1)).
// Loads run 8 samples ahead of the AFC recurrence (double sincos per sample).
__global__ void __launch_bounds__(64)
chain_afc(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts,
          const int* __restrict__ sel, int nsel) {
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nsel) return;
    const int c = sel[k];
    const ChainPost& P = posts[c];
    const int n = (int)counts[c].n_sq;
    const int U = P.afc_update, S = P.afc_sample;
    AfcState st = P.sstate->afc;
    const float2* in = reinterpret_cast<const float2*>(P.dem);
    float* out = P.dem;
    int i = 0;
    for (; i + 8 <= n; i += 8) {
        float2 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = in[i + u];
        float y[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) y[u] = afc_step(st, x[u], U, S).x;  // RealPart
#pragma unroll
        for (int u = 0; u < 8; ++u) out[i + u] = y[u];
    }
    for (; i < n; ++i) {
        const float2 x = in[i];
        out[i] = afc_step(st, x, U, S).x;
    }
    P.sstate->afc = st;
}

hipError_t launch_chain_afc(const ChainPost* posts, ChainCounts* counts, const int* sel, int nsel,
                            hipStream_t st) {
    if (nsel <= 0) return hipSuccess;
    hipLaunchKernelGGL(chain_afc, dim3((nsel + 63) / 64), dim3(64), 0, st, posts, counts, sel, nsel);
    return hipGetLastError();
}

// AdpcmEncoder(sync=True), one LANE per chain (64 chains per workgroup).  IMA-ADPCM's
// predictor carries offsets indefinitely (two encoders started apart on the same audio do not
// re-merge), so unlike the waterfall rows the chain audio cannot be encoded speculatively in
// segments; this kernel is the serial recurrence with everything else moved off its path:
//   wave 1  stages the int16 input (16-B loads, lane = chain) into an LDS ring one chunk of
//           kAdChunk samples ahead, so the encoder never waits on memory;
//   wave 0  encodes groups of 32 samples out of LDS (four ds_read_b128 per group) with the
//           remainder form (adpcm_encode_rem: no lane masks, the successor record in one LDS
//           read; the encoder is issue-bound, so its instruction count is its speed) and emits
//           the group's 16 completed bytes as one store.  32-sample groups: the per-group
//           conditions (a wave vote, exec-mask plumbing, the store) cost ~70 instructions, a
//           third of an 8-sample group's encoding (profiles/r05_adpcm_group32.txt).
// Byte stream: low nibble first; a byte started by the last sample of a block completes with
// the next block's first sample (has_left).  Frames: "SYNC" + (index, predictor) before every
// byte whose index in the chain's byte stream is a multiple of 1001 (AudioEngine.js:449-491),
// written with the state before that byte's first sample.  A group in which a lane starts such a
// byte, or in which a lane's samples end, runs a variant of the same unrolled encoder (below).
// Runs on stream C behind post_serial_front, so block k's encoding overlaps block k+1's front
// and block k+2's DDC.
#ifndef OWRX_AD_G
#define OWRX_AD_G 64
#endif
constexpr int kAdG = OWRX_AD_G;         // samples per encoder group (kAdG / 2 byte starts)
constexpr int kAdChunk = 4 * kAdG;      // samples per staged chunk
constexpr int kAdQ = kAdChunk / 8;      // 16-B quads (8 samples) per lane and chunk
constexpr int kAdGQ = kAdG / 8;         // quads per encoder group
constexpr int kAdGroups = kAdChunk / kAdG;

typedef uint32_t __attribute__((aligned(1))) u32_unaligned;
struct __attribute__((packed, aligned(1))) U128Unaligned {
    uint32_t x, y, z, w;
};

__global__ void __launch_bounds__(128)
chain_adpcm(const ChainPost* __restrict__ posts, ChainCounts* __restrict__ counts,
            const int* __restrict__ sel, int nsel) {
    __shared__ __align__(16) uint2 NS[kAdpcmRemEntries];
    __shared__ uint4 ring[2][kAdQ][64];  // [slot][quad][lane]: 8 int16 samples
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    adpcm_rem_fill(NS, threadIdx.x, 128);  // (array reference: the extent is checked)
    const SerLane sl = ser_lane(sel, nsel);
    const int c = sl.c;
    const ChainPost* Pp = posts + c;
    const int n = sl.active ? (int)counts[c].n_sq : 0;
    int nmax = n;
    for (int o = 32; o > 0; o >>= 1) nmax = max(nmax, __shfl_xor(nmax, o));
    const int nchunks = (nmax + kAdChunk - 1) / kAdChunk;
    const auto src = gp(reinterpret_cast<const uint4*>(Pp->s16));  // 16-B aligned slot

    // wave 1: chunk ch -> ring slot ch & 1.  The loads are unconditional (the quad index clamped
    // to the lane's last quad; quads past n are never encoded), so all 16 are in flight at once
    const int last_q = n > 0 ? (n - 1) >> 3 : 0;
    auto stage = [&](int ch) {
        uint4 v[kAdQ];
#pragma unroll
        for (int q = 0; q < kAdQ; ++q) v[q] = src[min(ch * kAdQ + q, last_q)];
#pragma unroll
        for (int q = 0; q < kAdQ; ++q) ring[ch & 1][q][lane] = v[q];
    };
    if (wave == 1 && nchunks > 0) stage(0);
    __syncthreads();

    if (wave == 1) {
        for (int ch = 0; ch < nchunks; ++ch) {
            if (ch + 1 < nchunks) stage(ch + 1);
            __syncthreads();
        }
        return;
    }

    // ---- wave 0: the encoder
    ChainStateS* sp = Pp->sstate;
    const ChainStateS st0 = *sp;
    AdpcmRem ad = adpcm_rem_state(st0.adpcm);
    const int pend = st0.has_left;  // 1: bytes start at odd samples of this block
    int left = st0.left_code;       // the started byte's low nibble (pend == 1)
    int64_t K = st0.adpcm_bytes + pend;  // index of the next byte to start
    int kmod = (int)(K % kAdpcmSyncPeriod);
    const auto out = gp(Pp->out);
    const int64_t cap = Pp->out_cap;
    int ob = 0;  // bytes staged this block (< 2^31)
    for (int ch = 0; ch < nchunks; ++ch) {
        const uint4(*rg)[64] = ring[ch & 1];
        uint4 vn[kAdGQ];
#pragma unroll
        for (int k = 0; k < kAdGQ; ++k) vn[k] = rg[k][lane];
        for (int g = 0; g < kAdGroups; ++g) {
            const int i0 = ch * kAdChunk + kAdG * g;
            if (i0 >= nmax) break;
            uint4 v[kAdGQ];  // the next group's reads are in flight while this one encodes
#pragma unroll
            for (int k = 0; k < kAdGQ; ++k) v[k] = vn[k];
            if (g + 1 < kAdGroups) {
#pragma unroll
                for (int k = 0; k < kAdGQ; ++k) vn[k] = rg[kAdGQ * (g + 1) + k][lane];
            }
            // kAdG / 2 byte starts in the group: bytes K .. K + kAdG / 2 - 1; a frame precedes byte k when
            // k % 1001 == 0, here the group's start fb (< 0: none), whose first sample is sf.  Every
            // group runs the unrolled encoder; two conditions take variants of it instead of the
            // per-sample path rounds 2-5 used:
            //  - a lane with a frame (chains that joined at different blocks have their frames at
            //    different starts: nearly every group has such a lane in a server, 1 - (1 -
            //    32 / 1001)^64 = 87 %): the state before sample sf is captured in passing and the
            //    frame goes into the lane's stores;
            //  - a lane whose samples end in the group (the chains of a wave release different
            //    squelch-block counts, so their ends differ by up to a squelch block): its state
            //    is held past its m samples and only its complete bytes are stored.
            // With both on the per-sample path, chains created a few blocks apart encoded 2.2x
            // slower than chains created together (tools/dbg/adpcm_phase.py).
            const int m = sl.active ? min(max(n - i0, 0), kAdG) : 0;  // the lane's samples here
            const int fb = kmod == 0 ? 0 : kmod > kAdpcmSyncPeriod - kAdG / 2 ? kAdpcmSyncPeriod - kmod : -1;
            const int sf = fb >= 0 ? 2 * fb + pend : kAdG;
            const bool framed = sf < m;
            const bool any_part = __any(sl.active && m < kAdG);
            const bool any_frame = __any(framed);
            uint32_t w[kAdGQ];  // the codes ^ 7 (adpcm_encode_rem), fixed below
            uint32_t cw0 = 0;   // the state before sample sf
            int cpred = 0;
            auto encode_group = [&](auto capture, auto hold) {
                constexpr bool kCap = decltype(capture)::value, kHold = decltype(hold)::value;
                int rem = m;  // kHold: samples left to the lane's end (opaque per step: the 64
                              // compares against m hoisted were 128 SGPRs)
#pragma unroll
                for (int k = 0; k < kAdGQ; ++k) {
                    const uint32_t wv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
                    // each code enters at the top nibble and the word shifts down by one
                    // (alignbit: one instruction; the record index's high bits fall off)
                    uint32_t acc = 0;
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        const int x = (int)(int16_t)(wv[t >> 1] >> (16 * (t & 1)));
                        if constexpr (kCap) {
                            const bool hit = 8 * k + t == sf;
                            cw0 = hit ? ad.w0 : cw0;
                            cpred = hit ? ad.pred : cpred;
                        }
                        if constexpr (kHold) {
                            asm volatile("" : "+v"(rem));
                            const AdpcmRem keep = ad;
                            acc = __builtin_amdgcn_alignbit(adpcm_encode_rem(ad, x, NS), acc, 4);
                            if (rem <= 0) ad = keep;  // past the lane's end: the state holds
                            --rem;
                        } else {
                            acc = __builtin_amdgcn_alignbit(adpcm_encode_rem(ad, x, NS), acc, 4);
                        }
                    }
                    w[k] = acc ^ 0x77777777u;
                }
            };
            if (any_part) {
                if (any_frame) encode_group(std::true_type{}, std::true_type{});
                else encode_group(std::false_type{}, std::true_type{});
            } else {
                if (any_frame) encode_group(std::true_type{}, std::false_type{});
                else encode_group(std::false_type{}, std::false_type{});
            }
            uint32_t prev = (uint32_t)left;
            if (pend) {  // bytes start at odd samples: shift the nibble stream by one
#pragma unroll
                for (int k = 0; k < kAdGQ; ++k) {
                    const uint32_t wk = w[k];
                    w[k] = (wk << 4) | prev;
                    prev = wk >> 28;
                }
            }
            // the lane's complete bytes: nibble 0 the pending start's code (pend), then its m codes
            const int nb = (pend + m) >> 1;
            if (m == kAdG) {
                if (pend) left = (int)prev;
            } else if (any_part && m > 0 && ((pend + m) & 1)) {
                uint32_t wn = w[0];  // w[nb >> 2] (a select chain: no indexed registers)
#pragma unroll
                for (int k = 1; k < kAdGQ; ++k) wn = (nb >> 2) == k ? w[k] : wn;
                left = (int)((wn >> (8 * (nb & 3))) & 15u);  // the start left open
            }
            if (m > 0) {
                if (m == kAdG && !framed) {
#pragma unroll
                    for (int q = 0; q < kAdGQ / 4; ++q) {
                        auto* d = reinterpret_cast<__attribute__((address_space(1))) U128Unaligned*>(&out.p[ob + 16 * q]);
                        d->x = w[4 * q];
                        d->y = w[4 * q + 1];
                        d->z = w[4 * q + 2];
                        d->w = w[4 * q + 3];
                    }
                } else if ((any_part || any_frame) && ob + nb + (framed ? 8 : 0) <= cap) {
                    // bytes [0, nb), the 8-B frame before byte pf when framed (the pending byte's
                    // completion comes first when pend): whole words in place or 8 bytes on, a
                    // word that pf or nb splits byte by byte
                    const int pf = framed ? fb + pend : kAdG;
                    auto st32 = [&](int off, uint32_t val) {
                        *reinterpret_cast<__attribute__((address_space(1))) u32_unaligned*>(&out.p[off]) = val;
                    };
#pragma unroll
                    for (int k = 0; k < kAdGQ; ++k) {
                        const int lo = 4 * k;
                        if (lo + 4 <= nb && (lo + 4 <= pf || lo >= pf)) {
                            st32(ob + lo + (lo >= pf ? 8 : 0), w[k]);
                        } else if (lo < nb) {
                            for (int b = 0; b < 4; ++b)
                                if (lo + b < nb) out[ob + lo + b + (lo + b >= pf ? 8 : 0)] = (uint8_t)(w[k] >> (8 * b));
                        }
                    }
                    if (framed) {
                        st32(ob + pf, 0x434E5953u);  // "SYNC"
                        st32(ob + pf + 4, (uint32_t)(uint16_t)(cw0 >> 17) | ((uint32_t)(uint16_t)cpred << 16));
                    }
                }
                ob += nb + (framed ? 8 : 0);
                kmod += pend ? m >> 1 : (m + 1) >> 1;  // the starts among its m samples
                if (kmod >= kAdpcmSyncPeriod) kmod -= kAdpcmSyncPeriod;
            }
        }
        __syncthreads();  // chunk ch + 1 staged; slot ch & 1 free for chunk ch + 2
    }
    if (!sl.active) return;
    // bytes completed this block: ob minus frame bytes; the state carries the parity
    const int pend_out = (pend + n) & 1;
    int64_t K_end = st0.adpcm_bytes + pend;
    {
        // starts this block = samples at start positions: (n + (1 - pend)) / 2 for pend = 0
        const int starts = pend ? n / 2 : (n + 1) / 2;
        K_end += starts;
    }
    sp->adpcm.index = ad.index();
    sp->adpcm.pred = ad.pred;
    sp->has_left = pend_out;
    sp->left_code = left;
    sp->adpcm_bytes = K_end - pend_out;
    counts[c].out_bytes = ob;
}

hipError_t launch_post_parallel(const ChainPost* posts, int nchains, ChainCounts* counts,
                                const StepTable& steps, hipStream_t st) {
    if (nchains <= 0) return hipSuccess;
    hipLaunchKernelGGL(post_parallel, dim3(nchains), dim3(kPostThreads), 0, st, posts, counts, steps);
    return hipGetLastError();
}

hipError_t launch_post_long(const ChainPost* posts, ChainCounts* counts, const int* idx,
                            int nlong, int64_t max_fd, int max_taps, hipStream_t st) {
    if (nlong <= 0) return hipSuccess;
    if (max_taps > kBlMaxTaps) return hipErrorInvalidValue;
    const size_t lds = sizeof(float2) * (((max_taps + 3) & ~3) + kBlTile + max_taps);
    static bool attr = false;
    if (!attr) {
        const size_t most = sizeof(float2) * (kBlMaxTaps + 1 + kBlTile + kBlMaxTaps);
        hipError_t e = hipFuncSetAttribute((const void*)bp_long,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)most);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int tiles = (int)((max_fd + kBlTile - 1) / kBlTile);
    hipLaunchKernelGGL(bp_long, dim3(std::max(1, tiles), nlong), dim3(kPostThreads), lds, st,
                       posts, counts, idx);
    hipLaunchKernelGGL(post_tail, dim3(nlong), dim3(kPostThreads), 0, st, posts, counts, idx);
    return hipGetLastError();
}

hipError_t launch_post_serial(const ChainPost* posts, ChainCounts* counts, const int* sel,
                              int nsel, int output, int debug, int nr, hipStream_t st) {
    if (nsel <= 0) return hipSuccess;
    const dim3 g((nsel + 63) / 64), b(kFrontThreads);
#define OWRX_FRONT(O, D, N)                                                                  \
    if (output == O && (debug != 0) == D && (nr != 0) == N) {                                \
        hipLaunchKernelGGL((post_serial_front<O, D, N>), g, b, 0, st, posts, counts, sel, nsel); \
        return hipGetLastError();                                                            \
    }
#define OWRX_FRONT_O(O) \
    OWRX_FRONT(O, false, false) OWRX_FRONT(O, true, false) OWRX_FRONT(O, false, true) OWRX_FRONT(O, true, true)
    OWRX_FRONT_O(0)
    OWRX_FRONT_O(1)
    OWRX_FRONT_O(2)
#undef OWRX_FRONT_O
#undef OWRX_FRONT
    return hipErrorInvalidValue;
}

hipError_t launch_chain_adpcm(const ChainPost* posts, ChainCounts* counts, const int* sel,
                              int nsel, hipStream_t st) {
    if (nsel <= 0) return hipSuccess;
    hipLaunchKernelGGL(chain_adpcm, dim3((nsel + 63) / 64), dim3(128), 0, st, posts, counts, sel,
                       nsel);
    return hipGetLastError();
}

}  // namespace owrx
