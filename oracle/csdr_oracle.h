/*
 * oracle/csdr_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * CPU restatement of the csdr DSP modules that sit on the OpenWebRX IQ hot path
 * (waterfall: owrx/fft.py -> csdr/chain/fft.py; demod: owrx/dsp.py ->
 * csdr/chain/{selector,analog,clientaudio}.py).  The arithmetic itself lives in the
 * third-party csdr library (luarvique fork, >= 0.18.36 per debian/control:22) which is
 * NOT in /root/reference; the algorithms here restate its published behaviour.
 * Parity with upstream csdr is "unpinned" except where a golden vector exists
 * (see DESIGN.md "Oracle"): firdes taps (htdocs/lib/AudioEngine.js:524-565), the
 * ADPCM bitstream (htdocs/lib/AudioEngine.js:410-509) and the chain parameter tables
 * recorded from the csdr/chain python modules (tests/golden/).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 */
#ifndef CSDR_ORACLE_H
#define CSDR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- filter design (float semantics of csdr's firdes_*; taps are parameters) ---- */
int  orc_firdes_filter_len(float transition_bw);
void orc_firdes_lowpass_f(float* out, int length, float cutoff_rate);
void orc_firdes_bandpass_c(float* out_cf, int length, float lowcut, float highcut);
void orc_hamming_window(float* out, int n);

/* ---- selector (DDC) ---- */
void    orc_shift(const float* in_cf, float* out_cf, int64_t n, float rate);
int64_t orc_fir_decimate(const float* in_cf, int64_t n, const float* taps, int ntaps,
                         int decimation, float* out_cf);
int64_t orc_fractional_decimator(const float* in_cf, int64_t n, double rate, float* out_cf);
void    orc_fir_complex(const float* in_cf, int64_t n, const float* taps_cf, int ntaps,
                        float* out_cf);
int64_t orc_squelch(const float* in_cf, int64_t n, int length, int decimation, int hang,
                    int flush, int report_interval, float level, float* out_cf,
                    float* power_out, int64_t* n_power);

/* ---- demodulators / audio (fp32, no contraction: bit-exact reference for the GPU) ---- */
void orc_fmdemod(const float* in_cf, int64_t n, float* out);
void orc_amdemod(const float* in_cf, int64_t n, float* out);
void orc_realpart(const float* in_cf, int64_t n, float* out);
void orc_limit(const float* in, int64_t n, float maxv, float* out);
void orc_dcblock(const float* in, int64_t n, float* out);
void orc_deemphasis(const float* in, int64_t n, float alpha, float* out);
float orc_nfm_deemphasis_alpha(int sample_rate);

typedef struct {
    float reference;
    float attack_rate;
    float decay_rate;
    float max_gain;
    float initial_gain;
    int   hang_time;
} orc_agc_params;
/* profile: 0 FAST, 1 SLOW, 2 MID, 3 LAGGY */
void orc_agc_profile(int profile, orc_agc_params* p);
void orc_agc(const float* in, int64_t n, const orc_agc_params* p, float* out);
void orc_convert_f_s16(const float* in, int64_t n, int16_t* out);
void orc_convert_s16_f(const int16_t* in, int64_t n, float* out);   /* n scalars */
void orc_gain(const float* in, int64_t n, float gain, float* out);

/* IMA-ADPCM.  sync=1: "SYNC" + s16 stepIndex + s16 predictor before data byte 0 and then
 * after every 1001 data bytes (the period htdocs/lib/AudioEngine.js:449-491 decodes). */
int64_t orc_adpcm_encode(const int16_t* in, int64_t n, int sync, uint8_t* out);
int64_t orc_adpcm_decode(const uint8_t* in, int64_t nbytes, int16_t* out);

/* ---- waterfall ---- */
/* Frames start at k*hop; rows sum avg frames (avg>=1) of |FFT(window*x)|^2 and map to
 * 10*log10(sum) + add_db - 10*log10(avg).  Returns number of rows written (N floats each),
 * NOT fft-swapped. */
int64_t orc_waterfall_rows(const float* in_cf, int64_t n, int N, int hop, int avg,
                           float add_db, float* rows_db);
void    orc_fftswap(const float* in, int N, float* out);
/* One FftAdpcm row: pad 10 copies of in[0], (short)(x*100), plain IMA-ADPCM, fresh state. */
int64_t orc_fft_adpcm_row(const float* row_db, int N, uint8_t* out);
/* Plain forward complex DFT (double, radix-2), N power of two. */
void    orc_fft(const double* in_cf, int N, double* out_cf);

/* ---- whole client chain (CPU baseline + end-to-end oracle) ---- */
typedef struct {
    float   shift_rate;
    int     decimation;
    int     ntaps;
    const float* taps;
    double  frac_rate;        /* 1.0 => no FractionalDecimator */
    int     bp_ntaps;         /* 0 => no Bandpass */
    const float* bp_taps;     /* complex */
    int     sq_length, sq_decimation, sq_hang, sq_flush, sq_report;
    float   sq_level;
    int     mode;             /* 0 NFM, 1 AM, 2 SSB(real part) */
    orc_agc_params agc;
    float   deemph_alpha;
    int     compression;      /* 0: s16 little endian, 1: ADPCM with sync */
} orc_chain_params;

/* Runs Shift->FirDecimate->[Frac]->[Bandpass]->Squelch->demod->...->Convert->[ADPCM].
 * Returns bytes written to out (<= out_cap), or -1 if out_cap is too small. */
int64_t orc_run_chain(const float* iq, int64_t n, const orc_chain_params* p, uint8_t* out,
                      int64_t out_cap, float* smeter, int64_t* n_smeter);

/* CPU baseline: run nchains chains over the same IQ with nthreads OpenMP threads. */
int64_t orc_run_chains_parallel(const float* iq, int64_t n, const orc_chain_params* p,
                                int nchains, int nthreads);
/* CPU baseline for the bench workload: the waterfall (one task) + nchains chains. */
int64_t orc_run_workload(const float* iq, int64_t n, int N, int hop, int avg, float add_db,
                         const orc_chain_params* p, int nchains, int nthreads);

void orc_fir_real(const float* in, int64_t n, const float* taps, int ntaps, float* out);
int64_t orc_fractional_decimator_f(const float* in, int64_t n, double rate, float* out);
float orc_wfm_deemphasis_alpha(int sample_rate, float tau);
int64_t orc_noise_filter(const float* in, int64_t n, float threshold_db, float* out);

#ifdef __cplusplus
}
#endif
#endif
