/*
 * oracle/csdr_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * CPU restatement of the csdr modules on the OpenWebRX IQ hot path.  Header comment in
 * csdr_oracle.h explains provenance.  Every function names the reference call site whose
 * parameters it consumes; the algorithm bodies restate upstream csdr (absent from
 * /root/reference, parity "unpinned" unless a golden vector in tests/golden/ pins it).
 *
 * Precision contract (DESIGN.md "Parity"):
 *   - filters (FirDecimate, FractionalDecimator, Bandpass, FFT, Shift) are evaluated in
 *     double: they approximate the exact real-number result the fp32 GPU kernels are
 *     compared against with a relative tolerance;
 *   - per-sample post-decimation stages (demods, limit, deemphasis, dcblock, AGC, convert,
 *     ADPCM, waterfall quantisation) are written as an explicit fp32 operation sequence
 *     with contraction disabled (-ffp-contract=off), so the GPU kernels, which use the
 *     same sequence, must match them bit for bit on identical inputs.
 */
#include "csdr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------ */
/* filter design                                                                        */
/* ------------------------------------------------------------------------------------ */

/* csdr firdes_filter_len(): int(4.0/tbw), forced odd.  tbw arrives as float (pycsdr takes
 * float args); selector.py:22 computes it as 0.15*out/in. */
int orc_firdes_filter_len(float transition_bw) {
    int result = (int)(4.0 / (double)transition_bw);
    if (result % 2 == 0) result++;
    return result;
}

static double hamming_kernel(double r) {
    /* csdr firdes_wkernel_hamming, also htdocs/lib/AudioEngine.js:548-551 */
    double rate = 0.5 + r / 2.0;
    return 0.54 - 0.46 * cos(2.0 * M_PI * rate);
}

static void lowpass_d(double* out, int length, double cutoff) {
    int middle = length / 2;
    out[middle] = 2.0 * M_PI * cutoff * hamming_kernel(0.0);
    for (int i = 1; i <= middle; i++) {
        double v = (sin(2.0 * M_PI * cutoff * i) / i) * hamming_kernel((double)i / middle);
        out[middle - i] = v;
        out[middle + i] = v;
    }
    double sum = 0.0;
    for (int i = 0; i < length; i++) sum += out[i];
    for (int i = 0; i < length; i++) out[i] /= sum;
}

/* csdr firdes_lowpass_f: Hamming windowed sinc, normalised to unit DC gain.  Golden:
 * htdocs/lib/AudioEngine.js:544-565 (evaluated in double, rounded to float here). */
void orc_firdes_lowpass_f(float* out, int length, float cutoff_rate) {
    double* t = (double*)malloc(sizeof(double) * length);
    lowpass_d(t, length, (double)cutoff_rate);
    for (int i = 0; i < length; i++) out[i] = (float)t[i];
    free(t);
}

/* csdr firdes_bandpass_c: lowpass of half-width (hi-lo)/2 modulated to (hi+lo)/2.
 * Called through Bandpass.setBandpass (csdr/chain/selector.py:159-166). */
void orc_firdes_bandpass_c(float* out_cf, int length, float lowcut, float highcut) {
    double* t = (double*)malloc(sizeof(double) * length);
    lowpass_d(t, length, ((double)highcut - (double)lowcut) / 2.0);
    double fc = ((double)highcut + (double)lowcut) / 2.0;
    for (int i = 0; i < length; i++) {
        double turns = fmod(fc * (double)i, 1.0);
        double ph = 2.0 * M_PI * turns;
        out_cf[2 * i] = (float)(cos(ph) * t[i]);
        out_cf[2 * i + 1] = (float)(sin(ph) * t[i]);
    }
    free(t);
}

/* csdr HammingWindow as applied by Fft (csdr/chain/fft.py:34): w[i] over i/(N-1). */
void orc_hamming_window(float* out, int n) {
    for (int i = 0; i < n; i++) {
        double r = (n > 1) ? 2.0 * (double)i / (double)(n - 1) - 1.0 : 0.0;
        out[i] = (float)hamming_kernel(r);
    }
}

/* ------------------------------------------------------------------------------------ */
/* Selector: Shift -> FirDecimate -> FractionalDecimator -> Bandpass -> Squelch          */
/* ------------------------------------------------------------------------------------ */

static uint64_t rate_to_fx(float rate) {
    double r = (double)rate;
    r -= floor(r);                          /* turns per sample in [0,1) */
    double s = r * 18446744073709551616.0;  /* 2^64 */
    if (s >= 18446744073709551615.0) return 0;
    return (uint64_t)s;
}

/* Shift(rate) (csdr/chain/selector.py:95,132-140; rate = -offset/inRate).  Sample n of the
 * chain is multiplied by exp(j*2*pi*(n+1)*rate) -- ShiftAddfast's (n+1) convention -- with
 * the phase accumulated exactly (64-bit fixed-point turns) instead of csdr's per-call float
 * re-seed, which is chunk-size dependent upstream. */
void orc_shift(const float* in_cf, float* out_cf, int64_t n, float rate) {
    uint64_t fx = rate_to_fx(rate);
    for (int64_t i = 0; i < n; i++) {
        uint64_t ph = (uint64_t)(i + 1) * fx;
        double turns = (double)ph * (1.0 / 18446744073709551616.0);
        double a = 2.0 * M_PI * turns;
        double c = cos(a), s = sin(a);
        double re = in_cf[2 * i], im = in_cf[2 * i + 1];
        out_cf[2 * i] = (float)(re * c - im * s);
        out_cf[2 * i + 1] = (float)(re * s + im * c);
    }
}

/* FirDecimate(D, tbw, cutoff) (csdr/chain/selector.py:29): y[m] = sum_t h[t] x[mD+t],
 * no zero history (first output once ntaps inputs are present). */
int64_t orc_fir_decimate(const float* in_cf, int64_t n, const float* taps, int ntaps,
                         int decimation, float* out_cf) {
    if (n < ntaps) return 0;
    int64_t m_out = (n - ntaps) / decimation + 1;
    double* h = (double*)malloc(sizeof(double) * ntaps);
    for (int t = 0; t < ntaps; t++) h[t] = taps[t];
    for (int64_t m = 0; m < m_out; m++) {
        const float* x = in_cf + 2 * (m * decimation);
        double ar = 0.0, ai = 0.0;
        for (int t = 0; t < ntaps; t++) {
            ar += h[t] * (double)x[2 * t];
            ai += h[t] * (double)x[2 * t + 1];
        }
        out_cf[2 * m] = (float)ar;
        out_cf[2 * m + 1] = (float)ai;
    }
    free(h);
    return m_out;
}

/* FractionalDecimator(COMPLEX_FLOAT, rate) (csdr/chain/selector.py:32-33), no prefilter.
 * 12-point Lagrange interpolation at positions w_k = 6 + k*rate; input window
 * [ceil(w)-6, ceil(w)+5]; nodes expressed as u = w - (ceil(w)-6) - 5.5. */
#define FD_POINTS 12
int64_t orc_fractional_decimator(const float* in_cf, int64_t n, double rate, float* out_cf) {
    int64_t k = 0;
    for (;; k++) {
        double w = 6.0 + (double)k * rate;
        int64_t hi = (int64_t)ceil(w);
        int64_t lo = hi - FD_POINTS / 2;
        if (hi + (FD_POINTS / 2 - 1) >= n) break;
        double u = (w - (double)lo) - 5.5;
        double ar = 0.0, ai = 0.0;
        for (int i = 0; i < FD_POINTS; i++) {
            double L = 1.0;
            double ni = (double)i - 5.5;
            for (int j = 0; j < FD_POINTS; j++) {
                if (j == i) continue;
                double nj = (double)j - 5.5;
                L *= (u - nj) / (ni - nj);
            }
            ar += L * (double)in_cf[2 * (lo + i)];
            ai += L * (double)in_cf[2 * (lo + i) + 1];
        }
        out_cf[2 * k] = (float)ar;
        out_cf[2 * k + 1] = (float)ai;
    }
    return k;
}

/* WFm's FractionalDecimator(FLOAT, 250000/hd_rate, prefilter=True) (csdr/chain/analog.py:69):
 * causal lowpass prefilter (taps from orc_firdes_lowpass_f(firdes_filter_len(0.03), 0.5/rate),
 * the build's recalled csdr default, unpinned), then the same 12-point Lagrange positions as
 * orc_fractional_decimator on the real stream. */
void orc_fir_real(const float* in, int64_t n, const float* taps, int ntaps, float* out) {
    for (int64_t i = 0; i < n; i++) {
        double a = 0.0;
        int tmax = (i + 1 < ntaps) ? (int)(i + 1) : ntaps;
        for (int t = 0; t < tmax; t++) a += (double)taps[t] * (double)in[i - t];
        out[i] = (float)a;
    }
}

int64_t orc_fractional_decimator_f(const float* in, int64_t n, double rate, float* out) {
    int64_t k = 0;
    for (;; k++) {
        double w = 6.0 + (double)k * rate;
        int64_t hi = (int64_t)ceil(w);
        int64_t lo = hi - FD_POINTS / 2;
        if (hi + (FD_POINTS / 2 - 1) >= n) break;
        double u = (w - (double)lo) - 5.5;
        double a = 0.0;
        for (int i = 0; i < FD_POINTS; i++) {
            double L = 1.0;
            double ni = (double)i - 5.5;
            for (int j = 0; j < FD_POINTS; j++) {
                if (j == i) continue;
                double nj = (double)j - 5.5;
                L *= (u - nj) / (ni - nj);
            }
            a += L * (double)in[lo + i];
        }
        out[k] = (float)a;
    }
    return k;
}

/* WfmDeemphasis(rate, tau) (csdr/chain/analog.py:70): csdr deemphasis_wfm_ff,
 * alpha = dt/(tau+dt), dt = 1/rate; the recurrence is orc_deemphasis. */
float orc_wfm_deemphasis_alpha(int sample_rate, float tau) {
    double dt = 1.0 / (double)sample_rate;
    return (float)(dt / ((double)tau + dt));
}

/* Bandpass(transition, use_fft=True).setBandpass(lo, hi) (csdr/chain/selector.py:115-117,
 * 159-166).  csdr applies it by FFT overlap-add; the result is the causal convolution
 * y[n] = sum_t g[t] x[n-t] with zero history, which is what is computed here. */
void orc_fir_complex(const float* in_cf, int64_t n, const float* taps_cf, int ntaps,
                     float* out_cf) {
    for (int64_t i = 0; i < n; i++) {
        double ar = 0.0, ai = 0.0;
        int tmax = (i + 1 < ntaps) ? (int)(i + 1) : ntaps;
        for (int t = 0; t < tmax; t++) {
            double gr = taps_cf[2 * t], gi = taps_cf[2 * t + 1];
            double xr = in_cf[2 * (i - t)], xi = in_cf[2 * (i - t) + 1];
            ar += gr * xr - gi * xi;
            ai += gr * xi + gi * xr;
        }
        out_cf[2 * i] = (float)ar;
        out_cf[2 * i + 1] = (float)ai;
    }
}

/* Squelch(COMPLEX_FLOAT, length=L, decimation=d, hangLength, flushLength, reportInterval)
 * (csdr/chain/selector.py:119-130), setSquelchLevel(10^(dB/10)) (:145-147).
 * Block power = mean |x|^2 over every d-th sample of each L-sample block; every
 * reportInterval blocks that power goes to the s-meter writer (owrx/connection.py:483-489).
 * Gate: open (copy) when level==0 or power>=level (re-arms hang/flush); otherwise copy
 * while hang lasts, then zeros.  Only whole blocks are emitted. */
int64_t orc_squelch(const float* in_cf, int64_t n, int length, int decimation, int hang,
                    int flush, int report_interval, float level, float* out_cf,
                    float* power_out, int64_t* n_power) {
    int64_t nb = n / length;
    int64_t hang_ctr = 0, flush_ctr = 0, np = 0;
    for (int64_t b = 0; b < nb; b++) {
        const float* x = in_cf + 2 * b * length;
        double p = 0.0;
        int cnt = 0;
        for (int i = 0; i < length; i += decimation) {
            p += (double)x[2 * i] * x[2 * i] + (double)x[2 * i + 1] * x[2 * i + 1];
            cnt++;
        }
        float power = (float)(p / cnt);
        if (report_interval > 0 && ((b + 1) % report_interval) == 0) {
            if (power_out) power_out[np] = power;
            np++;
        }
        int pass;
        if (level == 0.0f || power >= level) {
            hang_ctr = hang;
            flush_ctr = flush;
            pass = 1;
        } else if (hang_ctr > 0) {
            hang_ctr -= length;
            pass = 1;
        } else {
            if (flush_ctr > 0) flush_ctr -= length;
            pass = 0;
        }
        float* y = out_cf + 2 * b * length;
        if (pass)
            memcpy(y, x, sizeof(float) * 2 * length);
        else
            memset(y, 0, sizeof(float) * 2 * length);
    }
    if (n_power) *n_power = np;
    return nb * length;
}

/* ------------------------------------------------------------------------------------ */
/* demodulators and audio path (fp32 sequences mirrored by the GPU serial kernels)       */
/* ------------------------------------------------------------------------------------ */

#define FMDEMOD_QUADRI_K 0.340447f

/* FmDemod() (csdr/chain/analog.py:43): quadri-correlator discriminator. */
void orc_fmdemod(const float* in_cf, int64_t n, float* out) {
    float li = 0.0f, lq = 0.0f;
    for (int64_t k = 0; k < n; k++) {
        float i = in_cf[2 * k], q = in_cf[2 * k + 1];
        float dq = q - lq;
        float di = i - li;
        float a = i * dq;
        float b = q * di;
        float num = a - b;
        float ii = i * i;
        float qq = q * q;
        float den = ii + qq;
        float kn = FMDEMOD_QUADRI_K * num;
        out[k] = (den != 0.0f) ? kn / den : 0.0f;
        li = i;
        lq = q;
    }
}

/* AmDemod() (csdr/chain/analog.py:16). */
void orc_amdemod(const float* in_cf, int64_t n, float* out) {
    for (int64_t k = 0; k < n; k++) {
        float i = in_cf[2 * k], q = in_cf[2 * k + 1];
        float ii = i * i;
        float qq = q * q;
        out[k] = sqrtf(ii + qq);
    }
}

/* RealPart() (csdr/chain/analog.py:124, Ssb). */
void orc_realpart(const float* in_cf, int64_t n, float* out) {
    for (int64_t k = 0; k < n; k++) out[k] = in_cf[2 * k];
}

/* Limit() (csdr/chain/analog.py:44), max amplitude 1.0. */
void orc_limit(const float* in, int64_t n, float maxv, float* out) {
    for (int64_t k = 0; k < n; k++) {
        float v = in[k];
        if (v > maxv) v = maxv;
        if (v < -maxv) v = -maxv;
        out[k] = v;
    }
}

/* DcBlock() (csdr/chain/analog.py:17): y[n] = x[n] - x[n-1] + a*y[n-1], a = 0.999. */
void orc_dcblock(const float* in, int64_t n, float* out) {
    const float a = 0.999f;
    float xp = 0.0f, yp = 0.0f;
    for (int64_t k = 0; k < n; k++) {
        float x = in[k];
        float d = x - xp;
        float f = a * yp;
        float y = d + f;
        out[k] = y;
        xp = x;
        yp = y;
    }
}

/* NfmDeemphasis(rate) (csdr/chain/analog.py:45): one-pole de-emphasis
 * y = alpha*x + (1-alpha)*y_prev with alpha = dt/(tau+dt), tau = 1/(2*pi*300 Hz). */
float orc_nfm_deemphasis_alpha(int sample_rate) {
    double dt = 1.0 / (double)sample_rate;
    double tau = 1.0 / (2.0 * M_PI * 300.0);
    return (float)(dt / (tau + dt));
}

void orc_deemphasis(const float* in, int64_t n, float alpha, float* out) {
    float beta = 1.0f - alpha;
    float yp = 0.0f;
    for (int64_t k = 0; k < n; k++) {
        float a = alpha * in[k];
        float b = beta * yp;
        float y = a + b;
        out[k] = y;
        yp = y;
    }
}

/* Agc(FLOAT) + AgcProfile (csdr/chain/analog.py:13-15, 38-40, 121-122; owrx/dsp.py:619).
 * Upstream's AGC internals and profile constants are not recoverable; the build uses a
 * continuous attack/decay envelope follower (gain = reference/envelope, clamped to max_gain).
 * It is continuous in its input, so fp32 rounding differences upstream of it cannot be
 * amplified by branch flips.  Constants are the build's documented choice. */
void orc_agc_profile(int profile, orc_agc_params* p) {
    p->reference = 0.8f;
    p->max_gain = 65535.0f;
    p->initial_gain = 1.0f;
    p->hang_time = 0;
    switch (profile) {
        case 0: /* FAST */ p->attack_rate = 0.1f;  p->decay_rate = 0.001f;  break;
        case 1: /* SLOW */ p->attack_rate = 0.05f; p->decay_rate = 0.0001f; break;
        case 2: /* MID */  p->attack_rate = 0.1f;  p->decay_rate = 0.0005f; break;
        default: /* LAGGY */ p->attack_rate = 0.01f; p->decay_rate = 0.0001f; break;
    }
}

void orc_agc(const float* in, int64_t n, const orc_agc_params* p, float* out) {
    float env = p->reference / p->initial_gain;
    for (int64_t k = 0; k < n; k++) {
        float x = in[k];
        float a = fabsf(x);
        float d = a - env;
        float rate = (d > 0.0f) ? p->attack_rate : p->decay_rate;
        float t = rate * d;
        env = env + t;
        float g = (env > 0.0f) ? p->reference / env : p->max_gain;
        if (g > p->max_gain) g = p->max_gain;
        out[k] = g * x;
    }
}

static inline int16_t f_to_s16(float v) {
    if (v != v) return 0;
    if (v > 32767.0f) v = 32767.0f;
    if (v < -32768.0f) v = -32768.0f;
    return (int16_t)v; /* C conversion: truncation toward zero */
}

/* Convert(FLOAT, SHORT) (csdr/chain/clientaudio.py:18). */
void orc_convert_f_s16(const float* in, int64_t n, int16_t* out) {
    for (int64_t k = 0; k < n; k++) {
        float v = in[k] * 32767.0f;
        out[k] = f_to_s16(v);
    }
}

/* Ingest conversion Chain([Convert(COMPLEX_SHORT, COMPLEX_FLOAT), Gain(COMPLEX_FLOAT, g)])
 * (owrx/source/direct.py:51-71, fifi_sdr.py:27-28).  csdr scales short -> float by 1/SHRT_MAX
 * (the inverse of convert_f_s16 above; recalled, parity unpinned), then Gain multiplies. */
void orc_convert_s16_f(const int16_t* in, int64_t n, float* out) {
    for (int64_t k = 0; k < n; k++) out[k] = (float)in[k] / 32767.0f;
}

void orc_gain(const float* in, int64_t n, float gain, float* out) {
    for (int64_t k = 0; k < n; k++) out[k] = in[k] * gain;
}

/* ---- IMA ADPCM (AdpcmEncoder(sync=True) csdr/chain/clientaudio.py:34, FftAdpcm) ---- */
static const int adpcm_index_table[16] = {-1, -1, -1, -1, 2, 4, 6, 8,
                                          -1, -1, -1, -1, 2, 4, 6, 8};
static const int adpcm_step_table[89] = {
    7,     8,     9,     10,    11,    12,    13,    14,    16,    17,    19,    21,    23,
    25,    28,    31,    34,    37,    41,    45,    50,    55,    60,    66,    73,    80,
    88,    97,    107,   118,   130,   143,   157,   173,   190,   209,   230,   253,   279,
    307,   337,   371,   408,   449,   494,   544,   598,   658,   724,   796,   876,   963,
    1060,  1166,  1282,  1411,  1552,  1707,  1878,  2066,  2272,  2499,  2749,  3024,  3327,
    3660,  4026,  4428,  4871,  5358,  5894,  6484,  7132,  7845,  8630,  9493,  10442, 11487,
    12635, 13899, 15289, 16818, 18500, 20350, 22385, 24623, 27086, 29794, 32767};

typedef struct { int index; int pred; } adpcm_state;

static int adpcm_encode_sample(adpcm_state* s, int sample) {
    int step = adpcm_step_table[s->index];
    int diff = sample - s->pred;
    int code = 0;
    if (diff < 0) { code = 8; diff = -diff; }
    int ts = step;
    if (diff >= ts) { code |= 4; diff -= ts; }
    ts >>= 1;
    if (diff >= ts) { code |= 2; diff -= ts; }
    ts >>= 1;
    if (diff >= ts) { code |= 1; }
    int dq = step >> 3;
    if (code & 4) dq += step;
    if (code & 2) dq += step >> 1;
    if (code & 1) dq += step >> 2;
    s->pred += (code & 8) ? -dq : dq;
    if (s->pred > 32767) s->pred = 32767;
    if (s->pred < -32768) s->pred = -32768;
    s->index += adpcm_index_table[code];
    if (s->index < 0) s->index = 0;
    if (s->index > 88) s->index = 88;
    return code;
}

#define ADPCM_SYNC_PERIOD 1001
int64_t orc_adpcm_encode(const int16_t* in, int64_t n, int sync, uint8_t* out) {
    adpcm_state s = {0, 0};
    int64_t o = 0, data_bytes = 0;
    for (int64_t k = 0; k + 1 < n; k += 2) {
        if (sync && (data_bytes % ADPCM_SYNC_PERIOD) == 0) {
            out[o++] = 'S'; out[o++] = 'Y'; out[o++] = 'N'; out[o++] = 'C';
            int16_t idx = (int16_t)s.index, pr = (int16_t)s.pred;
            out[o++] = (uint8_t)(idx & 0xff); out[o++] = (uint8_t)((idx >> 8) & 0xff);
            out[o++] = (uint8_t)(pr & 0xff);  out[o++] = (uint8_t)((pr >> 8) & 0xff);
        }
        int lo = adpcm_encode_sample(&s, in[k]);
        int hi = adpcm_encode_sample(&s, in[k + 1]);
        out[o++] = (uint8_t)(lo | (hi << 4));
        data_bytes++;
    }
    return o;
}

/* Canonical IMA decoder (state starts at step_table[0]); used by tests only. */
int64_t orc_adpcm_decode(const uint8_t* in, int64_t nbytes, int16_t* out) {
    int index = 0, pred = 0;
    int64_t o = 0;
    for (int64_t b = 0; b < nbytes; b++) {
        for (int h = 0; h < 2; h++) {
            int code = h ? (in[b] >> 4) & 15 : in[b] & 15;
            int step = adpcm_step_table[index];
            int dq = step >> 3;
            if (code & 4) dq += step;
            if (code & 2) dq += step >> 1;
            if (code & 1) dq += step >> 2;
            pred += (code & 8) ? -dq : dq;
            if (pred > 32767) pred = 32767;
            if (pred < -32768) pred = -32768;
            index += adpcm_index_table[code];
            if (index < 0) index = 0;
            if (index > 88) index = 88;
            out[o++] = (int16_t)pred;
        }
    }
    return o;
}

/* ------------------------------------------------------------------------------------ */
/* waterfall: Fft -> LogAveragePower/LogPower -> FftSwap -> FftAdpcm (csdr/chain/fft.py)  */
/* ------------------------------------------------------------------------------------ */

void orc_fft(const double* in_cf, int N, double* out) {
    int lg = 0;
    while ((1 << lg) < N) lg++;
    for (int i = 0; i < N; i++) {
        int r = 0;
        for (int b = 0; b < lg; b++)
            if (i & (1 << b)) r |= 1 << (lg - 1 - b);
        out[2 * r] = in_cf[2 * i];
        out[2 * r + 1] = in_cf[2 * i + 1];
    }
    for (int len = 2; len <= N; len <<= 1) {
        int half = len / 2;
        for (int j = 0; j < half; j++) {
            double a = -2.0 * M_PI * (double)j / (double)len;
            double wr = cos(a), wi = sin(a);
            for (int i = j; i < N; i += len) {
                double ur = out[2 * i], ui = out[2 * i + 1];
                double vr = out[2 * (i + half)], vi = out[2 * (i + half) + 1];
                double tr = vr * wr - vi * wi, ti = vr * wi + vi * wr;
                out[2 * i] = ur + tr;
                out[2 * i + 1] = ui + ti;
                out[2 * (i + half)] = ur - tr;
                out[2 * (i + half) + 1] = ui - ti;
            }
        }
    }
}

/* Fft(size=N, every_n_samples=hop) (csdr/chain/fft.py:34,55) + LogAveragePower(add_db=-70,
 * fft_size=N, avg_number=avg) (fft.py:18-22).  avg row power is the sum over avg frames;
 * dB = 10*log10(sum) + add_db - 10*log10(avg)  (avg=1 reproduces LogPower). */
int64_t orc_waterfall_rows(const float* in_cf, int64_t n, int N, int hop, int avg,
                           float add_db, float* rows_db) {
    float* w = (float*)malloc(sizeof(float) * N);
    orc_hamming_window(w, N);
    double* buf = (double*)malloc(sizeof(double) * 2 * N);
    double* X = (double*)malloc(sizeof(double) * 2 * N);
    double* acc = (double*)malloc(sizeof(double) * N);
    int64_t nframes = (n >= N) ? (n - N) / hop + 1 : 0;
    int64_t nrows = nframes / avg;
    double corr = (double)add_db - 10.0 * log10((double)avg);
    for (int64_t r = 0; r < nrows; r++) {
        memset(acc, 0, sizeof(double) * N);
        for (int f = 0; f < avg; f++) {
            const float* x = in_cf + 2 * ((r * avg + f) * (int64_t)hop);
            for (int i = 0; i < N; i++) {
                buf[2 * i] = (double)x[2 * i] * (double)w[i];
                buf[2 * i + 1] = (double)x[2 * i + 1] * (double)w[i];
            }
            orc_fft(buf, N, X);
            for (int i = 0; i < N; i++) acc[i] += X[2 * i] * X[2 * i] + X[2 * i + 1] * X[2 * i + 1];
        }
        for (int i = 0; i < N; i++) rows_db[r * N + i] = (float)(10.0 * log10(acc[i]) + corr);
    }
    free(w); free(buf); free(X); free(acc);
    return nrows;
}

/* FftSwap(fft_size=N) (csdr/chain/fft.py:36). */
void orc_fftswap(const float* in, int N, float* out) {
    for (int i = 0; i < N; i++) out[i] = in[(i + N / 2) % N];
}

static inline int16_t db_to_s16(float v) {
    float t = v * 100.0f;
    return f_to_s16(t);
}

/* FftAdpcm(fft_size=N) (csdr/chain/fft.py:43-45); pad COMPRESS_FFT_PAD_N=10
 * (htdocs/openwebrx.js:845,1118-1126). */
int64_t orc_fft_adpcm_row(const float* row_db, int N, uint8_t* out) {
    int16_t* s = (int16_t*)malloc(sizeof(int16_t) * (N + 10));
    int16_t first = db_to_s16(row_db[0]);
    for (int i = 0; i < 10; i++) s[i] = first;
    for (int i = 0; i < N; i++) s[10 + i] = db_to_s16(row_db[i]);
    int64_t nb = orc_adpcm_encode(s, N + 10, 0, out);
    free(s);
    return nb;
}

/* ------------------------------------------------------------------------------------ */
/* whole client chain: owrx/dsp.py:72 [Selector, demod, ClientAudioChain]                */
/* ------------------------------------------------------------------------------------ */

int64_t orc_run_chain(const float* iq, int64_t n, const orc_chain_params* p, uint8_t* out,
                      int64_t out_cap, float* smeter, int64_t* n_smeter) {
    float* a = (float*)malloc(sizeof(float) * 2 * (size_t)n);
    orc_shift(iq, a, n, p->shift_rate);
    int64_t m_cap = n / p->decimation + 2;
    float* b = (float*)malloc(sizeof(float) * 2 * (size_t)m_cap);
    int64_t m = orc_fir_decimate(a, n, p->taps, p->ntaps, p->decimation, b);
    free(a);
    float* c = b;
    if (p->frac_rate != 1.0) {
        float* t = (float*)malloc(sizeof(float) * 2 * (size_t)(m + 2));
        m = orc_fractional_decimator(b, m, p->frac_rate, t);
        free(b);
        c = t;
    }
    if (p->bp_ntaps > 0) {
        float* t = (float*)malloc(sizeof(float) * 2 * (size_t)(m + 1));
        orc_fir_complex(c, m, p->bp_taps, p->bp_ntaps, t);
        free(c);
        c = t;
    }
    float* sq = (float*)malloc(sizeof(float) * 2 * (size_t)(m + 1));
    m = orc_squelch(c, m, p->sq_length, p->sq_decimation, p->sq_hang, p->sq_flush,
                    p->sq_report, p->sq_level, sq, smeter, n_smeter);
    free(c);
    float* d = (float*)malloc(sizeof(float) * (size_t)(m + 1));
    float* e = (float*)malloc(sizeof(float) * (size_t)(m + 1));
    if (p->mode == 0) {
        orc_fmdemod(sq, m, d);
        orc_limit(d, m, 1.0f, e);
        orc_deemphasis(e, m, p->deemph_alpha, d);
    } else if (p->mode == 1) {
        orc_amdemod(sq, m, e);
        orc_dcblock(e, m, d);
    } else {
        orc_realpart(sq, m, d);
    }
    free(sq);
    orc_agc(d, m, &p->agc, e);
    int16_t* s = (int16_t*)malloc(sizeof(int16_t) * (size_t)(m + 1));
    orc_convert_f_s16(e, m, s);
    free(d);
    free(e);
    int64_t nb;
    if (p->compression) {
        int64_t need = m / 2 + 8 * (m / 2 / ADPCM_SYNC_PERIOD + 1);
        if (need > out_cap) { free(s); return -1; }
        nb = orc_adpcm_encode(s, m, 1, out);
    } else {
        if (2 * m > out_cap) { free(s); return -1; }
        memcpy(out, s, 2 * (size_t)m);
        nb = 2 * m;
    }
    free(s);
    return nb;
}

int64_t orc_run_chains_parallel(const float* iq, int64_t n, const orc_chain_params* p,
                                int nchains, int nthreads) {
    int64_t total = 0;
    int64_t cap = n / 8 + 4096;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
#endif
    for (int c = 0; c < nchains; c++) {
        uint8_t* out = (uint8_t*)malloc((size_t)cap);
        int64_t ns = 0;
        float* sm = (float*)malloc(sizeof(float) * (size_t)(n / 64 + 16));
        int64_t r = orc_run_chain(iq, n, &p[c], out, cap, sm, &ns);
        total += r;
        free(out);
        free(sm);
    }
    return total;
}

int64_t orc_run_workload(const float* iq, int64_t n, int N, int hop, int avg, float add_db,
                         const orc_chain_params* p, int nchains, int nthreads) {
    int64_t total = 0;
    int64_t cap = n / 8 + 4096;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
#endif
    for (int c = 0; c <= nchains; c++) {
        if (c == nchains) {
            int64_t nrows = ((n >= N) ? (n - N) / hop + 1 : 0) / avg + 1;
            float* rows = (float*)malloc(sizeof(float) * (size_t)N * (size_t)nrows);
            float* sw = (float*)malloc(sizeof(float) * (size_t)N);
            uint8_t* ob = (uint8_t*)malloc((size_t)N + 16);
            int64_t r = orc_waterfall_rows(iq, n, N, hop, avg, add_db, rows);
            for (int64_t i = 0; i < r; i++) {
                orc_fftswap(rows + i * N, N, sw);
                total += orc_fft_adpcm_row(sw, N, ob);
            }
            free(rows); free(sw); free(ob);
            continue;
        }
        uint8_t* out = (uint8_t*)malloc((size_t)cap);
        int64_t ns = 0;
        float* sm = (float*)malloc(sizeof(float) * (size_t)(n / 64 + 16));
        int64_t r = orc_run_chain(iq, n, &p[c], out, cap, sm, &ns);
        total += r;
        free(out);
        free(sm);
    }
    return total;
}


/* NoiseFilter(nr_threshold) (csdr/chain/clientaudio.py:12-13; "spectral subtraction",
 * CHANGELOG.md:852).  csdr's source is not available: this is the build's documented choice,
 * mirrored by kernels_nr.hip (parity unpinned against csdr).  Frames of 512 at hop 256,
 * sqrt(periodic Hann) analysis + synthesis; per bin S = 0.7 S + 0.3 |X|^2 (first frame
 * S = |X|^2); noise floor Nf = geometric mean of S over the 257 bins (a tone or voice occupies
 * few bins, so the log-average stays at the noise), smoothed 0.9 / 0.1 across frames; gain
 * S / (S + t Nf + 1e-30) with t = 10^(threshold/10); overlap-add, one hop of latency (zero
 * history before sample 0).
 * Returns the samples emitted: whole hops after the first frame. */
#define NR_N 512
#define NR_H 256
int64_t orc_noise_filter(const float* in, int64_t n, float threshold_db, float* out) {
    double w[NR_N], S[NR_N / 2 + 1], Nf = 0.0, ola[NR_H];
    double buf[2 * NR_N], X[2 * NR_N];
    double t = pow(10.0, (double)threshold_db / 10.0);
    for (int i = 0; i < NR_N; i++) w[i] = sqrt(0.5 - 0.5 * cos(2.0 * M_PI * i / NR_N));
    memset(ola, 0, sizeof(ola));
    int64_t nout = 0;
    /* frame f covers input [f*H - H, f*H + H) */
    for (int64_t f = 0; f * NR_H + NR_H <= n; f++) {
        for (int i = 0; i < NR_N; i++) {
            int64_t s = f * NR_H - NR_H + i;
            buf[2 * i] = (s >= 0 ? (double)in[s] : 0.0) * w[i];
            buf[2 * i + 1] = 0.0;
        }
        orc_fft(buf, NR_N, X);
        double G[NR_N / 2 + 1], lsum = 0.0;
        for (int k = 0; k <= NR_N / 2; k++) {
            double p = X[2 * k] * X[2 * k] + X[2 * k + 1] * X[2 * k + 1];
            S[k] = f == 0 ? p : 0.7 * S[k] + 0.3 * p;
            lsum += log(S[k] + 1e-30);
        }
        double geo = exp(lsum / (NR_N / 2 + 1));
        Nf = f == 0 ? geo : 0.9 * Nf + 0.1 * geo;
        for (int k = 0; k <= NR_N / 2; k++) G[k] = S[k] / (S[k] + t * Nf + 1e-30);
        for (int i = 0; i < NR_N; i++) {
            double g = G[i <= NR_N / 2 ? i : NR_N - i];
            buf[2 * i] = g * X[2 * i];
            buf[2 * i + 1] = -g * X[2 * i + 1];
        }
        orc_fft(buf, NR_N, X);
        for (int i = 0; i < NR_H; i++) {
            double y0 = X[2 * i] / NR_N * w[i];
            double y1 = X[2 * (NR_H + i)] / NR_N * w[NR_H + i];
            double o = ola[i] + y0;
            ola[i] = y1;
            if (f > 0) out[nout + i] = (float)o;
        }
        if (f > 0) nout += NR_H;
    }
    return nout;
}
