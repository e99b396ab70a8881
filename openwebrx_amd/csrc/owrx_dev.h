// owrx_dev.h -- device-side types and per-sample DSP steps shared by the fused kernels
// (kernels_*.hip) and the single-module runners (modules.hip).
//
// Semantics follow the csdr modules named in each comment (call sites in the reference's
// csdr/chain/*.py); the fp32 operation order of every serial step is identical to
// oracle/csdr_oracle.c, with FP contraction disabled, so identical inputs give identical bits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define OWRX_DEV __device__ __forceinline__

namespace owrx {

constexpr int kWave = 64;
constexpr int kFdPoints = 12;     // FractionalDecimator Lagrange points
constexpr int kFdHist = 16;       // DDC outputs kept for the interpolator window
constexpr int kBpHist = 256;      // Bandpass history (taps - 1 <= 255) of the in-kernel FIR
constexpr int kNrN = 512;         // NoiseFilter frame (42.7 ms at 12 kHz), 50 % overlap
constexpr int kNrHop = kNrN / 2;
constexpr int kWfHist = 256;      // WFM: IF-rate demod / prefilter history (prefilter <= 255 taps)
constexpr int kAdpcmSyncPeriod = 1001;  // data bytes per "SYNC" frame (AudioEngine.js:449-491)
constexpr float kFmK = 0.340447f; // fmdemod_quadri_K

struct AgcParams {
    float reference, attack, decay, max_gain, initial_gain;
    int hang_time;  // unused by the continuous follower, kept for ABI stability
};
struct AgcState {
    float env;
    int pad;
};
struct AdpcmState {
    int index;
    int pred;
};

// Global-address-space view of a pointer read from a descriptor.  Generic (flat) accesses
// count against the LDS wait counter too, so a kernel mixing them with LDS traffic waits on
// HBM latency at every LDS use; global_* accesses only wait where their data is consumed.
// (HIP vector classes cannot be address-space qualified, so float2 goes through the native
// ext_vector type.)
template <typename T> struct GNative { using type = T; };
template <> struct GNative<float2> { using type = float __attribute__((ext_vector_type(2))); };
template <> struct GNative<float4> { using type = float __attribute__((ext_vector_type(4))); };
template <> struct GNative<uint2> { using type = unsigned int __attribute__((ext_vector_type(2))); };

template <typename T>
struct GRef {
    using N = typename GNative<T>::type;
    __attribute__((address_space(1))) N* p;
    OWRX_DEV operator T() const { return __builtin_bit_cast(T, *p); }
    OWRX_DEV T get() const { return __builtin_bit_cast(T, *p); }
    OWRX_DEV const GRef& operator=(T v) const {
        *p = __builtin_bit_cast(N, v);
        return *this;
    }
    // element copy (a[i] = b[i]), never a rebinding of the reference
    OWRX_DEV const GRef& operator=(const GRef& o) const { return *this = o.get(); }
};

template <typename T>
struct GPtr {
    using N = typename GNative<T>::type;
    __attribute__((address_space(1))) N* p;
    OWRX_DEV GRef<T> operator[](int64_t i) const { return GRef<T>{p + i}; }
    OWRX_DEV GRef<T> operator*() const { return GRef<T>{p}; }
    OWRX_DEV GPtr operator+(int64_t i) const { return GPtr{p + i}; }
    OWRX_DEV GPtr operator-(int64_t i) const { return GPtr{p - i}; }
};

template <typename T>
OWRX_DEV GPtr<T> gp(const T* q) {
    using N = typename GNative<T>::type;
    return GPtr<T>{(__attribute__((address_space(1))) N*)(const_cast<T*>(q))};
}

OWRX_DEV float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// ---- serial / per-sample steps (bit-exact with the oracle) --------------------------------

// FmDemod (csdr/chain/analog.py:43), quadri-correlator.
OWRX_DEV float fm_step(float2 x, float2 last) {
#pragma clang fp contract(off)
    float dq = x.y - last.y;
    float di = x.x - last.x;
    float a = x.x * dq;
    float b = x.y * di;
    float num = a - b;
    float ii = x.x * x.x;
    float qq = x.y * x.y;
    float den = ii + qq;
    float kn = kFmK * num;
    return (den != 0.0f) ? kn / den : 0.0f;
}

// AmDemod (analog.py:16)
OWRX_DEV float am_step(float2 x) {
#pragma clang fp contract(off)
    float ii = x.x * x.x;
    float qq = x.y * x.y;
    return sqrtf(ii + qq);
}

// Limit (analog.py:44)
OWRX_DEV float limit_step(float v, float m) {
    if (v > m) v = m;
    if (v < -m) v = -m;
    return v;
}

// NfmDeemphasis (analog.py:45): y = alpha*x + (1-alpha)*y_prev
OWRX_DEV float deemph_step(float x, float alpha, float beta, float& yp) {
#pragma clang fp contract(off)
    float a = alpha * x;
    float b = beta * yp;
    float y = a + b;
    yp = y;
    return y;
}

// DcBlock (analog.py:17): y = x - x_prev + 0.999*y_prev
OWRX_DEV float dcblock_step(float x, float& xp, float& yp) {
#pragma clang fp contract(off)
    const float a = 0.999f;
    float d = x - xp;
    float f = a * yp;
    float y = d + f;
    xp = x;
    yp = y;
    return y;
}

// Afc(updatePeriod U, samplePeriod S) of SAm / RawSAm (csdr/chain/analog.py:141-167), the build's
// choice (csdr's algorithm is not in the reference; oracle afc): y = x e^{-j ph}, ph += w (ph
// wrapped to [-pi, pi]); every S samples the pair product y[n] conj(y[n - S]) is summed, and
// after U pairs w += arg(sum) / (2 S).  Phase and frequency in double, the rotation in float.
struct AfcState {
    double ph, w, re, im;
    float2 prev;
    int64_t n;
    int32_t pairs;
    int32_t pad;
};
OWRX_DEV float2 afc_step(AfcState& s, float2 x, int U, int S) {
    double sn, cs;
    sincos(s.ph, &sn, &cs);
    const float c = (float)cs, si = (float)sn;
    float2 y;
    {
#pragma clang fp contract(off)
        y = make_float2(x.x * c + x.y * si, x.y * c - x.x * si);
    }
    s.ph += s.w;
    if (s.ph > M_PI) s.ph -= 2.0 * M_PI;
    else if (s.ph < -M_PI) s.ph += 2.0 * M_PI;
    if (s.n % S == 0) {
        if (s.n >= S) {
            const double pr = s.prev.x, pi = s.prev.y;
            s.re += (double)y.x * pr + (double)y.y * pi;
            s.im += (double)y.y * pr - (double)y.x * pi;
            if (++s.pairs == U) {
                s.w += atan2(s.im, s.re) / (2.0 * S);
                s.re = s.im = 0.0;
                s.pairs = 0;
            }
        }
        s.prev = y;
    }
    s.n++;
    return y;
}

// Agc(FLOAT) (analog.py:13-15, 38-40, 121-122): continuous attack/decay envelope follower,
// gain = reference / envelope clamped to max_gain (see oracle/csdr_oracle.c orc_agc).
OWRX_DEV float agc_step(float x, const AgcParams& p, AgcState& s) {
#pragma clang fp contract(off)
    float a = fabsf(x);
    float d = a - s.env;
    float rate = (d > 0.0f) ? p.attack : p.decay;
    float t = rate * d;
    s.env = s.env + t;
    float g = (s.env > 0.0f) ? p.reference / s.env : p.max_gain;
    if (g > p.max_gain) g = p.max_gain;
    return g * x;
}

OWRX_DEV int16_t f_to_s16(float v) {
    if (v != v) return 0;
    if (v > 32767.0f) v = 32767.0f;
    if (v < -32768.0f) v = -32768.0f;
    return (int16_t)v;
}

// Convert(FLOAT, SHORT) (clientaudio.py:18)
OWRX_DEV int16_t convert_s16(float x) {
#pragma clang fp contract(off)
    float v = x * 32767.0f;
    return f_to_s16(v);
}

// Convert(COMPLEX_SHORT, COMPLEX_FLOAT) then Gain(COMPLEX_FLOAT, g) per component
// (owrx/source/direct.py:51-71): x / 32767 (csdr's short -> float scale, the inverse of
// convert_s16), then * g, two roundings as the two modules apply them.
OWRX_DEV float s16_to_f32(int16_t x) {
#pragma clang fp contract(off)
    return (float)x / 32767.0f;
}
OWRX_DEV float gain_step(float x, float g) {
#pragma clang fp contract(off)
    return x * g;
}

// FftAdpcm quantiser: (short)(dB*100) (csdr/chain/fft.py:43-45, htdocs/openwebrx.js:1118-1126)
OWRX_DEV int16_t db_to_s16(float db) {
#pragma clang fp contract(off)
    float t = db * 100.0f;
    return f_to_s16(t);
}

__constant__ static const int8_t kAdpcmIndex[16] = {-1, -1, -1, -1, 2, 4, 6, 8,
                                                     -1, -1, -1, -1, 2, 4, 6, 8};
__constant__ static const int16_t kAdpcmStep[89] = {
    7,     8,     9,     10,    11,    12,    13,    14,    16,    17,    19,    21,    23,
    25,    28,    31,    34,    37,    41,    45,    50,    55,    60,    66,    73,    80,
    88,    97,    107,   118,   130,   143,   157,   173,   190,   209,   230,   253,   279,
    307,   337,   371,   408,   449,   494,   544,   598,   658,   724,   796,   876,   963,
    1060,  1166,  1282,  1411,  1552,  1707,  1878,  2066,  2272,  2499,  2749,  3024,  3327,
    3660,  4026,  4428,  4871,  5358,  5894,  6484,  7132,  7845,  8630,  9493,  10442, 11487,
    12635, 13899, 15289, 16818, 18500, 20350, 22385, 24623, 27086, 29794, 32767};

// IMA ADPCM encode of one sample (AdpcmEncoder / FftAdpcm); decoder in
// htdocs/lib/AudioEngine.js:493-509.
OWRX_DEV int adpcm_encode(AdpcmState& s, int sample) {
    int step = kAdpcmStep[s.index];
    int diff = sample - s.pred;
    int code = 0;
    if (diff < 0) {
        code = 8;
        diff = -diff;
    }
    int ts = step;
    if (diff >= ts) {
        code |= 4;
        diff -= ts;
    }
    ts >>= 1;
    if (diff >= ts) {
        code |= 2;
        diff -= ts;
    }
    ts >>= 1;
    if (diff >= ts) code |= 1;
    int dq = step >> 3;
    if (code & 4) dq += step;
    if (code & 2) dq += step >> 1;
    if (code & 1) dq += step >> 2;
    int p = s.pred + ((code & 8) ? -dq : dq);
    p = p > 32767 ? 32767 : (p < -32768 ? -32768 : p);
    s.pred = p;
    int idx = s.index + kAdpcmIndex[code];
    s.index = idx < 0 ? 0 : (idx > 88 ? 88 : idx);
    return code;
}

// Table-driven variant.  NS[index * 8 + magnitude] = next step | (next index * 8) << 16, i.e.
// the successor record for every (index, code magnitude), so the index update (+ table step,
// clamp to [0, 88]) and the step-table lookup become one dependent LDS read at row + magnitude.
// Measured on MI355X (tools/micro/adpcm_bench.cpp): 177 cycles per sample and lane against 194
// for prefetching the 8 successors of the row and selecting by the magnitude bits, and 243 for
// the 5-candidate step prefetch.  State: AdpcmTab{rec, pred}.  Bit-identical to adpcm_encode.
constexpr int kAdpcmTabEntries = 89 * 8;

OWRX_DEV uint32_t adpcm_tab_rec(int index) {
    return (uint32_t)kAdpcmStep[index] | ((uint32_t)(index * 8) << 16);
}

// The tables are filled through references to arrays, so a table declared smaller than the
// fill cannot compile (commits dd5bbb0..dfdd34f had an 89 x 8 LDS array under the 89 x 16 fill).
template <int EXT>
OWRX_DEV void adpcm_tab_fill(uint32_t (&NS)[EXT], int tid, int nthreads) {
    static_assert(EXT >= kAdpcmTabEntries, "successor table too small");
    for (int e = tid; e < kAdpcmTabEntries; e += nthreads) {
        const int i = e >> 3, m = e & 7;
        int ni = i + kAdpcmIndex[m];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        NS[e] = adpcm_tab_rec(ni);
    }
}

struct AdpcmTab {
    uint32_t rec;  // step | (index * 8) << 16
    int pred;
    OWRX_DEV int index() const { return (int)(rec >> 19); }
};

OWRX_DEV AdpcmTab adpcm_tab_state(AdpcmState s) { return AdpcmTab{adpcm_tab_rec(s.index), s.pred}; }

OWRX_DEV int adpcm_encode_tab(AdpcmTab& s, int sample, const uint32_t* __restrict__ NS) {
    const uint32_t row = s.rec >> 16;  // index * 8
    const int step = (int)(s.rec & 0xffffu);
    const int h = step >> 1, q = step >> 2, s3 = step >> 3;
    const int d = sample - s.pred;
    const int sgn = d >> 31;
    int a = max(d, -d);
    const bool m4 = a >= step;
    const int t4 = m4 ? step : 0;
    a -= t4;
    const bool m2 = a >= h;
    const int t2 = m2 ? h : 0;
    a -= t2;
    const bool m1 = a >= q;
    const int dq = s3 + t4 + t2 + (m1 ? q : 0);
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    const int mag = (m4 ? 4 : 0) | (m2 ? 2 : 0) | (m1 ? 1 : 0);
    s.rec = NS[row + mag];
    return mag | (sgn & 8);
}

// Remainder form (chain_adpcm): no lane masks on the recurrence.  One wave issues about one
// instruction per 4.5-5 cycles and the serial encoder is issue-bound
// (profiles/r05_issue_latency_micro.txt), so this form minimises instructions, not depth:
//   - 8-B successor records {step | (2 index) << 16, h | q << 16} (h = step >> 1, q = step >> 2)
//     whose 16-bit fields the subtractions read in place (SDWA): nothing is unpacked per sample;
//   - per magnitude bit t in (step, h, q): u = a - t; the sign of u is the INVERTED bit (a < t), an
//     alignbit shifts it into the record index; a = min_u32(a, u) is the remainder (u wraps above
//     a when a < t);
//   - rows of 8 records in reverse magnitude order, one row per (index, sign):
//     NSR[(2 index + sign) * 8 + (7 - mag)], so the index built from (2 index + sign) and the
//     three inverted bits addresses the successor directly and its low nibble is the code ^ 7;
//   - dq = (step >> 3) + a0 - a3 (the subtracted thresholds; step >> 3 = h >> 2).
// 136 vs 199 cycles per sample for the masked byte-addressed table it replaced
// (tools/micro/adpcm_r05.cpp, profiles/r05_adpcm_encoder_variants.txt); bit-identical to
// adpcm_encode.
constexpr int kAdpcmRemEntries = 89 * 16;

template <int EXT>
OWRX_DEV void adpcm_rem_fill(uint2 (&NSR)[EXT], int tid, int nthreads) {
    static_assert(EXT >= kAdpcmRemEntries, "remainder-form successor table too small");
    for (int e = tid; e < kAdpcmRemEntries; e += nthreads) {
        const int i = e >> 4, m = 7 - (e & 7);
        int ni = i + kAdpcmIndex[m];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        const uint32_t st = (uint32_t)kAdpcmStep[ni];
        NSR[e] = make_uint2(st | ((uint32_t)(ni * 2) << 16), (st >> 1) | ((st >> 2) << 16));
    }
}

struct AdpcmRem {
    uint32_t w0, w1;  // step | (2 index) << 16, h | q << 16
    int pred;
    OWRX_DEV int index() const { return (int)(w0 >> 17); }
};

OWRX_DEV AdpcmRem adpcm_rem_state(AdpcmState s) {
    const uint32_t st = (uint32_t)kAdpcmStep[s.index];
    return AdpcmRem{st | ((uint32_t)(s.index * 2) << 16), (st >> 1) | ((st >> 2) << 16), s.pred};
}

// Returns the successor's record index; its low nibble is the 4-bit code ^ 7.
OWRX_DEV uint32_t adpcm_encode_rem(AdpcmRem& s, int sample, const uint2* __restrict__ NSR) {
    const int d = sample - s.pred;
    const int sgn = d >> 31;
    const uint32_t a0 = (uint32_t)max(d, -d);
    const uint32_t w0 = s.w0, w1 = s.w1;
    uint32_t acc = ((uint32_t)d >> 31) + (w0 >> 16);
    const uint32_t u4 = a0 - (w0 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u4, 31);
    const uint32_t a1 = min(a0, u4);
    const uint32_t u2 = a1 - (w1 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u2, 31);
    const uint32_t a2 = min(a1, u2);
    const uint32_t u1 = a2 - (w1 >> 16);
    acc = __builtin_amdgcn_alignbit(acc, u1, 31);
    const uint32_t a3 = min(a2, u1);
    const uint2 r = NSR[acc];
    // dq = (step >> 3) + a0 - a3 with a0 >= a3: the |a0 - a3| + s3 form is one v_sad_u32
    const uint32_t s3 = (w1 & 0xffffu) >> 2;
    const int dq = (int)((a0 > a3 ? a0 - a3 : a3 - a0) + s3);
    s.w0 = r.x;
    s.w1 = r.y;
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    return acc;
}

// The remainder form with a shorter predictor recurrence (round 6).  The encoder is bound by its
// two loop-carried chains as much as by issue: the predictor (pred -> d -> |d| -> three magnitude
// bits -> dq -> pred') and the successor record (record -> magnitude bits -> index -> LDS read ->
// record).  Here the predictor is kept offset by 32768 (predo = pred + 32768 in [0, 65535]) and the
// sample comes offset too, so |d| is one v_sad_u32 (no negate / max pair), and the update
//   pred' = pred + sgn (s3 + a0 - a3) = (predo + sgn (s3 + a0) + sgn) - (a3 ^ sgn)
// (sgn (v) = (v ^ sgn) - sgn, sgn = 0 or -1) has its first part computed beside the magnitude
// compares: after the last bit only the xor, the subtraction and the clamp (v_med3) remain.
// Bit-identical to adpcm_encode_rem; same records and return value.
struct AdpcmRemO {
    uint32_t w0, w1;  // as AdpcmRem
    int predo;        // pred + 32768
    OWRX_DEV int index() const { return (int)(w0 >> 17); }
    OWRX_DEV int pred() const { return predo - 32768; }
};

OWRX_DEV AdpcmRemO adpcm_rem_o_state(AdpcmState s) {
    const AdpcmRem r = adpcm_rem_state(s);
    return AdpcmRemO{r.w0, r.w1, s.pred + 32768};
}

// xo = sample + 32768
OWRX_DEV uint32_t adpcm_encode_rem_o(AdpcmRemO& s, uint32_t xo, const uint2* __restrict__ NSR) {
    const int d = (int)xo - s.predo;
    const int sgn = d >> 31;
    const uint32_t po = (uint32_t)s.predo;
    const uint32_t a0 = xo > po ? xo - po : po - xo;  // one v_sad_u32 (as dq in adpcm_encode_rem)
    const uint32_t w0 = s.w0, w1 = s.w1;
    const uint32_t s3 = (w1 & 0xffffu) >> 2;
    const int e = (int)(s3 + a0);
    const int q = s.predo + ((e ^ sgn) - sgn) + sgn;  // beside the compares
    uint32_t acc = ((uint32_t)d >> 31) + (w0 >> 16);
    const uint32_t u4 = a0 - (w0 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u4, 31);
    const uint32_t a1 = min(a0, u4);
    const uint32_t u2 = a1 - (w1 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u2, 31);
    const uint32_t a2 = min(a1, u2);
    const uint32_t u1 = a2 - (w1 >> 16);
    acc = __builtin_amdgcn_alignbit(acc, u1, 31);
    const uint32_t a3 = min(a2, u1);
    const uint2 r = NSR[acc];
    s.w0 = r.x;
    s.w1 = r.y;
    const int p = q - (int)(a3 ^ (uint32_t)sgn);
    s.predo = min(max(p, 0), 65535);
    return acc;
}

// The remainder form with 16-B successor records (round 6): {step | (2 index) << 16, h | q << 16,
// step >> 3, 0}, read with one ds_read_b128, so dq's s3 term comes with the record instead of a
// v_bfe_u32 per sample (the encoder is issue-bound: one instruction fewer of ~25 per sample).
// Same record order, index and return value as adpcm_encode_rem; bit-identical.
template <int EXT>
OWRX_DEV void adpcm_rem4_fill(uint4 (&NSR)[EXT], int tid, int nthreads) {
    static_assert(EXT >= kAdpcmRemEntries, "16-B successor table too small");
    for (int e = tid; e < kAdpcmRemEntries; e += nthreads) {
        const int i = e >> 4, m = 7 - (e & 7);
        int ni = i + kAdpcmIndex[m];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        const uint32_t st = (uint32_t)kAdpcmStep[ni];
        NSR[e] = make_uint4(st | ((uint32_t)(ni * 2) << 16), (st >> 1) | ((st >> 2) << 16), st >> 3, 0u);
    }
}

struct AdpcmRem4 {
    uint32_t w0, w1, s3;
    int pred;
    OWRX_DEV int index() const { return (int)(w0 >> 17); }
};

OWRX_DEV AdpcmRem4 adpcm_rem4_state(AdpcmState s) {
    const uint32_t st = (uint32_t)kAdpcmStep[s.index];
    return AdpcmRem4{st | ((uint32_t)(s.index * 2) << 16), (st >> 1) | ((st >> 2) << 16), st >> 3, s.pred};
}

OWRX_DEV uint32_t adpcm_encode_rem4(AdpcmRem4& s, int sample, const uint4* __restrict__ NSR) {
    const int d = sample - s.pred;
    const int sgn = d >> 31;
    const uint32_t a0 = (uint32_t)max(d, -d);
    const uint32_t w0 = s.w0, w1 = s.w1;
    uint32_t acc = ((uint32_t)d >> 31) + (w0 >> 16);
    const uint32_t u4 = a0 - (w0 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u4, 31);
    const uint32_t a1 = min(a0, u4);
    const uint32_t u2 = a1 - (w1 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u2, 31);
    const uint32_t a2 = min(a1, u2);
    const uint32_t u1 = a2 - (w1 >> 16);
    acc = __builtin_amdgcn_alignbit(acc, u1, 31);
    const uint32_t a3 = min(a2, u1);
    const uint4 r = NSR[acc];
    const int dq = (int)((a0 > a3 ? a0 - a3 : a3 - a0) + s.s3);
    s.w0 = r.x;
    s.w1 = r.y;
    s.s3 = r.z;
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    return acc;
}

}  // namespace owrx
