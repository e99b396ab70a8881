/* cpu_baseline.c -- the timed CPU baseline of bench.py (SURVEY.md 8d "CPU baseline"; test
 * infrastructure: only bench.py's cpu_baseline leg calls it, never the product path).
 *
 * The same workload as orc_run_workload (waterfall + client chains on one stream), with the
 * stages that dominate csdr's cost computed the way csdr computes them -- fp32, SIMD-friendly --
 * instead of the oracle's double-precision checker form:
 *   - Shift (csdr/chain/selector.py:95): fp32 rotator re-seeded every 1024 samples from the
 *     exact phase (shift_addfast's per-call re-seed),
 *   - FirDecimate (selector.py:29): y[m] = sum_t h[t] s[mD + t] over de-interleaved fp32 re / im
 *     arrays, vectorised dot products (AVX2 FMA, -ffast-math),
 *   - the waterfall FFT (csdr/chain/fft.py:34, FFTW in csdr): iterative fp32 radix-2 with a
 *     twiddle table, |X|^2 averaged in fp32.
 * The 12 kHz tail (FractionalDecimator ... AdpcmEncoder) reuses the oracle's functions; it is
 * < 0.1 % of the work.  csdr runs one thread per module per chain; this runs one task per chain
 * (and one for the waterfall) on an OpenMP pool. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "csdr_oracle.h"

#define CPB_CHUNK 262144   /* input samples per DDC chunk (plus the FIR history) */
#define CPB_RESEED 1024    /* shift_addfast re-seeds its rotator every call */

/* Shift + FirDecimate of one chain, fp32: out gets floor((n - T) / D) + 1 outputs. */
static int64_t cpb_ddc(const float* iq, int64_t n, float rate, const float* h, int T, int D,
                       float* out) {
    if (n < T) return 0;
    const int64_t m_out = (n - T) / D + 1;
    const int64_t per = CPB_CHUNK / D;                 /* outputs per chunk */
    const int64_t span = per * D + T;                  /* samples a chunk reads */
    float* re = (float*)aligned_alloc(64, sizeof(float) * ((size_t)span + 64));
    float* im = (float*)aligned_alloc(64, sizeof(float) * ((size_t)span + 64));
    const double drate = (double)rate;
    for (int64_t m0 = 0; m0 < m_out; m0 += per) {
        const int64_t mc = (m0 + per <= m_out) ? per : m_out - m0;
        const int64_t s0 = m0 * D;
        const int64_t len = (mc - 1) * D + T;
        /* shifted samples s[s0 .. s0 + len) */
        for (int64_t b = 0; b < len; b += CPB_RESEED) {
            const int64_t e = (b + CPB_RESEED < len) ? b + CPB_RESEED : len;
            const double ph = 2.0 * M_PI * fmod((double)(s0 + b + 1) * drate, 1.0);
            float cr = (float)cos(ph), ci = (float)sin(ph);
            const float wr = (float)cos(2.0 * M_PI * drate), wi = (float)sin(2.0 * M_PI * drate);
            for (int64_t k = b; k < e; k++) {
                const float xr = iq[2 * (s0 + k)], xi = iq[2 * (s0 + k) + 1];
                re[k] = xr * cr - xi * ci;
                im[k] = xr * ci + xi * cr;
                const float nr = cr * wr - ci * wi;
                ci = cr * wi + ci * wr;
                cr = nr;
            }
        }
        for (int64_t m = 0; m < mc; m++) {
            const float* xr = re + m * D;
            const float* xi = im + m * D;
            float sr = 0.f, si = 0.f;
            /* a plain dot product: -ffast-math lets the compiler split it into AVX2 FMA lanes
               (csdr's FIR loops are built the same way) */
            for (int t = 0; t < T; t++) {
                sr += h[t] * xr[t];
                si += h[t] * xi[t];
            }
            out[2 * (m0 + m)] = sr;
            out[2 * (m0 + m) + 1] = si;
        }
    }
    free(re);
    free(im);
    return m_out;
}

/* in-place iterative radix-2 FFT (forward), fp32; tw: N/2 twiddles exp(-2 pi i k / N) */
static void cpb_fft(float* x, int N, const float* tw) {
    for (int i = 1, j = 0; i < N; i++) {
        int bit = N >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) {
            float t0 = x[2 * i], t1 = x[2 * i + 1];
            x[2 * i] = x[2 * j];
            x[2 * i + 1] = x[2 * j + 1];
            x[2 * j] = t0;
            x[2 * j + 1] = t1;
        }
    }
    for (int len = 2; len <= N; len <<= 1) {
        const int half = len >> 1, step = N / len;
        for (int i = 0; i < N; i += len)
            for (int k = 0; k < half; k++) {
                const float wr = tw[2 * k * step], wi = tw[2 * k * step + 1];
                float* a = x + 2 * (i + k);
                float* b = x + 2 * (i + k + half);
                const float br = b[0] * wr - b[1] * wi, bi = b[0] * wi + b[1] * wr;
                b[0] = a[0] - br;
                b[1] = a[1] - bi;
                a[0] += br;
                a[1] += bi;
            }
    }
}

static int64_t cpb_waterfall(const float* iq, int64_t n, int N, int hop, int avg, float add_db,
                             float* rows) {
    float* w = (float*)malloc(sizeof(float) * N);
    orc_hamming_window(w, N);
    float* tw = (float*)malloc(sizeof(float) * N);
    for (int k = 0; k < N / 2; k++) {
        tw[2 * k] = (float)cos(-2.0 * M_PI * k / N);
        tw[2 * k + 1] = (float)sin(-2.0 * M_PI * k / N);
    }
    float* x = (float*)malloc(sizeof(float) * 2 * N);
    float* acc = (float*)malloc(sizeof(float) * N);
    const int64_t nframes = (n >= N) ? (n - N) / hop + 1 : 0;
    const int64_t nrows = nframes / avg;
    const float corr = (float)(add_db - 10.0 * log10((double)avg));
    for (int64_t r = 0; r < nrows; r++) {
        memset(acc, 0, sizeof(float) * N);
        for (int f = 0; f < avg; f++) {
            const float* s = iq + 2 * ((r * avg + f) * (int64_t)hop);
            for (int i = 0; i < N; i++) {
                x[2 * i] = s[2 * i] * w[i];
                x[2 * i + 1] = s[2 * i + 1] * w[i];
            }
            cpb_fft(x, N, tw);
            for (int i = 0; i < N; i++) acc[i] += x[2 * i] * x[2 * i] + x[2 * i + 1] * x[2 * i + 1];
        }
        for (int i = 0; i < N; i++) rows[r * N + i] = 10.0f * log10f(acc[i]) + corr;
    }
    free(w);
    free(tw);
    free(x);
    free(acc);
    return nrows;
}

/* one client chain: fp32 Shift + FirDecimate, then the oracle's 12 kHz tail */
static int64_t cpb_run_chain(const float* iq, int64_t n, const orc_chain_params* p, uint8_t* out,
                             int64_t out_cap) {
    const int64_t m_cap = n / p->decimation + 2;
    float* b = (float*)malloc(sizeof(float) * 2 * (size_t)m_cap);
    int64_t m = cpb_ddc(iq, n, p->shift_rate, p->taps, p->ntaps, p->decimation, b);
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
    float* sm = (float*)malloc(sizeof(float) * (size_t)(m / 4 + 16));
    int64_t nsm = 0;
    m = orc_squelch(c, m, p->sq_length, p->sq_decimation, p->sq_hang, p->sq_flush, p->sq_report,
                    p->sq_level, sq, sm, &nsm);
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
    orc_agc(d, m, &p->agc, e);
    int16_t* s = (int16_t*)malloc(sizeof(int16_t) * (size_t)(m + 1));
    orc_convert_f_s16(e, m, s);
    int64_t nb = -1;
    if (m / 2 + 8 * (m / 2 / 1001 + 1) <= out_cap) nb = orc_adpcm_encode(s, m, 1, out);
    free(sq);
    free(sm);
    free(d);
    free(e);
    free(s);
    return nb;
}

int64_t cpb_run_workload(const float* iq, int64_t n, int N, int hop, int avg, float add_db,
                         const orc_chain_params* p, int nchains, int nthreads) {
    int64_t total = 0;
    const int64_t cap = n / 8 + 4096;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
#endif
    for (int c = 0; c <= nchains; c++) {
        if (c == nchains) {  /* the waterfall: FftChain -> FftSwap -> FftAdpcm */
            const int64_t nrows = ((n >= N) ? (n - N) / hop + 1 : 0) / avg + 1;
            float* rows = (float*)malloc(sizeof(float) * (size_t)N * (size_t)nrows);
            float* sw = (float*)malloc(sizeof(float) * (size_t)N);
            uint8_t* ob = (uint8_t*)malloc((size_t)N + 16);
            const int64_t r = cpb_waterfall(iq, n, N, hop, avg, add_db, rows);
            for (int64_t i = 0; i < r; i++) {
                orc_fftswap(rows + i * N, N, sw);
                total += orc_fft_adpcm_row(sw, N, ob);
            }
            free(rows);
            free(sw);
            free(ob);
            continue;
        }
        uint8_t* out = (uint8_t*)malloc((size_t)cap);
        total += cpb_run_chain(iq, n, &p[c], out, cap);
        free(out);
    }
    return total;
}

/* ---- the csdr-shaped baseline (round 6) -------------------------------------
 * csdr runs every module of a chain in a thread of its own, modules connected by ring buffers
 * (csdr/module/__init__.py:36-53 pump threads; pycsdr Buffer / Reader between modules).  This
 * leg reproduces that structure: per chain one thread per module -- Shift + FirDecimate (one
 * module pair reading the shared wideband buffer), FractionalDecimator, Bandpass, Squelch, the
 * demodulator (FmDemod + Limit + NfmDeemphasis | AmDemod + DcBlock | RealPart), Agc, Convert,
 * AdpcmEncoder -- and for the waterfall Fft + LogAveragePower, FftSwap, FftAdpcm, every pair of
 * threads joined by a bounded queue of chunks (mutex + condition variables, as pycsdr's Buffer
 * wakes its readers).  The work per chunk is the same code as the OpenMP leg (fp32 DDC and FFT,
 * the oracle's 12 kHz tail), each module applied to each chunk on its own (a timing model: a
 * module's state is not carried from one chunk to the next, so its output is not the exact
 * stream).  The OS schedules the threads on the cores the process may use. */
#include <pthread.h>

#define CPB_QCAP 4
#define CPB_PIPE_CHUNK (1 << 20)

typedef struct {
    float* data;   /* NULL: end of stream */
    int64_t n;     /* samples (complex or real) or bytes */
} cpb_chunk;

typedef struct {
    cpb_chunk slot[CPB_QCAP];
    int head, count;
    pthread_mutex_t mu;
    pthread_cond_t not_empty, not_full;
} cpb_queue;

static void q_init(cpb_queue* q) {
    q->head = q->count = 0;
    pthread_mutex_init(&q->mu, NULL);
    pthread_cond_init(&q->not_empty, NULL);
    pthread_cond_init(&q->not_full, NULL);
}
static void q_free(cpb_queue* q) {
    pthread_mutex_destroy(&q->mu);
    pthread_cond_destroy(&q->not_empty);
    pthread_cond_destroy(&q->not_full);
}
static void q_push(cpb_queue* q, cpb_chunk c) {
    pthread_mutex_lock(&q->mu);
    while (q->count == CPB_QCAP) pthread_cond_wait(&q->not_full, &q->mu);
    q->slot[(q->head + q->count) % CPB_QCAP] = c;
    q->count++;
    pthread_cond_signal(&q->not_empty);
    pthread_mutex_unlock(&q->mu);
}
static cpb_chunk q_pop(cpb_queue* q) {
    pthread_mutex_lock(&q->mu);
    while (q->count == 0) pthread_cond_wait(&q->not_empty, &q->mu);
    cpb_chunk c = q->slot[q->head];
    q->head = (q->head + 1) % CPB_QCAP;
    q->count--;
    pthread_cond_signal(&q->not_full);
    pthread_mutex_unlock(&q->mu);
    return c;
}

enum { ST_DDC, ST_FD, ST_BP, ST_SQ, ST_DEMOD, ST_AGC, ST_CONV, ST_ADPCM, ST_N,
       ST_WF_FFT = 100, ST_WF_SWAP, ST_WF_ADPCM };

typedef struct {
    int kind;
    cpb_queue* in;   /* NULL for the first stage (reads the wideband buffer) */
    cpb_queue* out;  /* NULL for the last stage */
    const float* iq;
    int64_t n;
    const orc_chain_params* p;
    int N, hop, avg;
    float add_db;
    int64_t produced;
} cpb_stage;

static void* cpb_stage_run(void* arg) {
    cpb_stage* s = (cpb_stage*)arg;
    const orc_chain_params* p = s->p;
    if (s->kind == ST_DDC || s->kind == ST_WF_FFT) {
        /* the wideband source in chunks (with the filter / FFT history): 2^20 samples for a chain
         * (~1 260 outputs at 12 kHz: a whole squelch block, as the chunk-local modules need), one
         * waterfall row's frames (avg x hop) for the waterfall */
        const int64_t hist = s->kind == ST_DDC ? p->ntaps : s->N;
        const int64_t step = s->kind == ST_DDC ? CPB_PIPE_CHUNK : (int64_t)s->avg * s->hop;
        for (int64_t s0 = 0; s0 + hist < s->n; s0 += step) {
            const int64_t len = (s0 + step + hist <= s->n) ? step + hist : s->n - s0;
            cpb_chunk c;
            if (s->kind == ST_DDC) {
                float* o = (float*)malloc(sizeof(float) * 2 * (size_t)(len / p->decimation + 2));
                c.n = cpb_ddc(s->iq + 2 * s0, len, p->shift_rate, p->taps, p->ntaps, p->decimation, o);
                c.data = o;
            } else {
                const int64_t nfr = (len - s->N) / s->hop + 1;
                const int64_t nr = nfr / s->avg + 1;
                float* o = (float*)malloc(sizeof(float) * (size_t)s->N * (size_t)nr);
                c.n = cpb_waterfall(s->iq + 2 * s0, len, s->N, s->hop, s->avg, s->add_db, o);
                c.data = o;
            }
            q_push(s->out, c);
        }
        q_push(s->out, (cpb_chunk){NULL, 0});
        return NULL;
    }
    for (;;) {
        cpb_chunk c = q_pop(s->in);
        if (!c.data) {
            if (s->out) q_push(s->out, c);
            return NULL;
        }
        const int64_t m = c.n;
        cpb_chunk o = {NULL, 0};
        switch (s->kind) {
            case ST_FD:
                if (p->frac_rate != 1.0) {
                    o.data = (float*)malloc(sizeof(float) * 2 * (size_t)(m + 2));
                    o.n = orc_fractional_decimator(c.data, m, p->frac_rate, o.data);
                } else {
                    o.data = (float*)malloc(sizeof(float) * 2 * (size_t)(m + 1));
                    memcpy(o.data, c.data, sizeof(float) * 2 * (size_t)m);
                    o.n = m;
                }
                break;
            case ST_BP:
                o.data = (float*)malloc(sizeof(float) * 2 * (size_t)(m + 1));
                if (p->bp_ntaps > 0) orc_fir_complex(c.data, m, p->bp_taps, p->bp_ntaps, o.data);
                else memcpy(o.data, c.data, sizeof(float) * 2 * (size_t)m);
                o.n = m;
                break;
            case ST_SQ: {
                float* sm = (float*)malloc(sizeof(float) * (size_t)(m / 4 + 16));
                int64_t nsm = 0;
                o.data = (float*)malloc(sizeof(float) * 2 * (size_t)(m + 1));
                o.n = orc_squelch(c.data, m, p->sq_length, p->sq_decimation, p->sq_hang, p->sq_flush,
                                  p->sq_report, p->sq_level, o.data, sm, &nsm);
                free(sm);
                break;
            }
            case ST_DEMOD: {
                o.data = (float*)malloc(sizeof(float) * (size_t)(m + 1));
                if (p->mode == 0) {
                    float* t = (float*)malloc(sizeof(float) * (size_t)(m + 1));
                    orc_fmdemod(c.data, m, o.data);
                    orc_limit(o.data, m, 1.0f, t);
                    orc_deemphasis(t, m, p->deemph_alpha, o.data);
                    free(t);
                } else if (p->mode == 1) {
                    float* t = (float*)malloc(sizeof(float) * (size_t)(m + 1));
                    orc_amdemod(c.data, m, t);
                    orc_dcblock(t, m, o.data);
                    free(t);
                } else {
                    orc_realpart(c.data, m, o.data);
                }
                o.n = m;
                break;
            }
            case ST_AGC:
                o.data = (float*)malloc(sizeof(float) * (size_t)(m + 1));
                orc_agc(c.data, m, &p->agc, o.data);
                o.n = m;
                break;
            case ST_CONV:
                o.data = (float*)malloc(sizeof(int16_t) * (size_t)(m + 1));
                orc_convert_f_s16(c.data, m, (int16_t*)o.data);
                o.n = m;
                break;
            case ST_ADPCM: {
                uint8_t* b = (uint8_t*)malloc((size_t)(m / 2 + 8 * (m / 2 / 1001 + 1) + 16));
                s->produced += orc_adpcm_encode((const int16_t*)c.data, m, 1, b);
                free(b);
                break;
            }
            case ST_WF_SWAP: {
                o.data = (float*)malloc(sizeof(float) * (size_t)s->N * (size_t)(m + 1));
                for (int64_t r = 0; r < m; r++) orc_fftswap(c.data + r * s->N, s->N, o.data + r * s->N);
                o.n = m;
                break;
            }
            case ST_WF_ADPCM: {
                uint8_t* b = (uint8_t*)malloc((size_t)s->N + 16);
                for (int64_t r = 0; r < m; r++) s->produced += orc_fft_adpcm_row(c.data + r * s->N, s->N, b);
                free(b);
                break;
            }
        }
        free(c.data);
        if (s->out) q_push(s->out, o);
    }
}

/* One thread per module per chain (and per waterfall module), bounded queues between them; the
 * threads run on whatever cores the process may use.  Returns the output bytes (audio + rows);
 * *nthreads_out = the module threads started. */
int64_t cpb_run_pipeline(const float* iq, int64_t n, int N, int hop, int avg, float add_db,
                         const orc_chain_params* p, int nchains, int* nthreads_out) {
    const int nst = nchains * ST_N + 3;
    cpb_stage* st = (cpb_stage*)calloc((size_t)nst, sizeof(cpb_stage));
    cpb_queue* qs = (cpb_queue*)calloc((size_t)nst, sizeof(cpb_queue));
    pthread_t* th = (pthread_t*)calloc((size_t)nst, sizeof(pthread_t));
    for (int i = 0; i < nst; i++) q_init(&qs[i]);
    int k = 0;
    for (int c = 0; c < nchains; c++) {
        for (int j = 0; j < ST_N; j++, k++) {
            st[k].kind = j;
            st[k].in = j ? &qs[k - 1] : NULL;
            st[k].out = j + 1 < ST_N ? &qs[k] : NULL;
            st[k].iq = iq;
            st[k].n = n;
            st[k].p = &p[c];
        }
    }
    const int wf_kinds[3] = {ST_WF_FFT, ST_WF_SWAP, ST_WF_ADPCM};
    for (int j = 0; j < 3; j++, k++) {
        st[k].kind = wf_kinds[j];
        st[k].in = j ? &qs[k - 1] : NULL;
        st[k].out = j + 1 < 3 ? &qs[k] : NULL;
        st[k].iq = iq;
        st[k].n = n;
        st[k].N = N;
        st[k].hop = hop;
        st[k].avg = avg;
        st[k].add_db = add_db;
    }
    int started = 0;
    for (int i = 0; i < nst; i++)
        if (pthread_create(&th[i], NULL, cpb_stage_run, &st[i]) == 0) started++;
    int64_t total = 0;
    for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
    for (int i = 0; i < nst; i++) total += st[i].produced;
    for (int i = 0; i < nst; i++) q_free(&qs[i]);
    free(st);
    free(qs);
    free(th);
    if (nthreads_out) *nthreads_out = started;
    return started == nst ? total : -1;
}
