// owrx_types.h -- descriptors exchanged between the host engine (engine.hip) and the
// kernels.  Plain structs, identical layout on host and device.
#pragma once
#include <stdint.h>
#include "owrx_dev.h"

namespace owrx {

// ---- waterfall ---------------------------------------------------------------------------
// One workgroup computes sum_f |FFT(w * x_f)|^2 over `nframes` consecutive frames of one row.
struct WfGroup {
    int64_t start;    // absolute stream index of the first frame
    int32_t nframes;
    int32_t hop;
};
// One row touched by a finalize launch: sums its groups (in order) onto the carry.
struct WfRow {
    int32_t first_group;
    int32_t ngroups;
    int32_t use_carry;   // add the carried accumulator first
    int32_t complete;    // emit the row (else store the sum into the carry)
    int32_t out_index;   // row slot in the output staging buffer
    int32_t pad;         // wf_fft_l32 tail split: the descriptor of the row's first split frame
};

// ---- DDC (Shift + FirDecimate, fused, all chains of one (D, taps) group) ----------------
// One chain's filter-spectra build in a batched fc_make_w_jobs launch: its shift rate and the
// offset of its slot in the group's W.
struct FcWJob {
    uint64_t rate_fx;
    int64_t off;
};

struct DdcChain {
    uint64_t rate_fx;    // shift rate in 2^-64 turns per sample
    float2 wD;           // exp(j 2 pi D rate): rotator step between consecutive outputs
    int64_t n0;          // phase(n) = P0 + (n - n0 + 1) * rate_fx   (absolute n)
    uint64_t P0;
};

// ---- post-decimation chain state (device, persistent) -----------------------------------
// Owned by post_parallel (stream A).
struct ChainStateP {
    int64_t ddc_count;     // DDC outputs consumed so far (chain-local)
    int64_t fd_next;       // next FractionalDecimator output index
    int64_t fd_count;      // samples emitted by FractionalDecimator (or passthrough) so far
    int64_t sq_blocks;
    int32_t sq_pending;    // samples waiting for a full squelch block
    int32_t hang_ctr;
    int32_t flush_ctr;
    int32_t pad;
    float2 fm_last;
    // secondary FFT input (squelch output history): sf_buf[0, sf_fill) holds samples, the next
    // frame starts at sf_next (may exceed sf_fill when hop > N); post_parallel compacts and
    // appends, chain_sfft consumes frames
    int32_t sf_fill;
    int32_t sf_next;
    int32_t sf_row_frame;  // frames already summed into the open row (sf_acc)
    int32_t sf_pad;
    // WFM audio FractionalDecimator(FLOAT, 250000/hd_rate, prefilter=True) (analog.py:66-71)
    int64_t wf_count;      // FmDemod+Limit samples produced so far (IF rate)
    int64_t wf_next;       // next audio output index
};
// Owned by post_serial (stream B).
struct ChainStateS {
    int64_t adpcm_bytes;   // data bytes emitted (sync period bookkeeping)
    float deemph_y;
    float dc_xp, dc_yp;
    AgcState agc;
    AdpcmState adpcm;
    int32_t has_left;      // ADPCM: one encoded nibble waiting for its pair
    int32_t left_code;
    AfcState afc;          // SAm / RawSAm (chain_afc)
};
// NoiseFilter state (stream B; the host zeroes it with the filter's buffers on (re)start)
struct NrState {
    int32_t pend;          // input samples after nr_in[0, kNrHop) (the previous hop)
    int32_t frames;        // frames processed
};

// The per-block fields of a chain group's posts (post_parallel's argument): the slot's posts
// stay on the device across blocks and only this table changes.
// Caller blocks in one engine block (owrx_set_block_group: pairs, quads): sub-block s holds the
// DDC outputs [nk[s - 1], nk[s]) (nk[-1] = 0) from input up to the absolute sample end[s], in
// ceil((nk[s] - nk[s - 1]) / V) frames of its own with its own zero padding, so the fast DDC's
// frames and outputs are those of separate launches.  n = 1: one block (nk[0] = nk, end[0] =
// the block's end).
constexpr int kMaxSubBlocks = 4;
struct FcSubs {
    int n;
    int nk[kMaxSubBlocks];
    int64_t end[kMaxSubBlocks];
};

struct GroupStep {
    int64_t k_begin;
    int32_t nk;
    int32_t nseg;
};
constexpr int kMaxStepGroups = 32;
struct StepTable {
    GroupStep g[kMaxStepGroups];
};

// Static + per-step description of one chain, shared by post_parallel and post_serial.
struct ChainPost {
    // configuration
    int32_t demod;         // OWRX_DEMOD_*
    int32_t afc_update, afc_sample;  // OWRX_DEMOD_SAM: Afc(updatePeriod, samplePeriod)
    int32_t fixed_gain;    // Gain(agc.max_gain) instead of Agc (RawAm, RawSAm)
    int32_t output;        // OWRX_OUT_*
    int32_t frac_enabled;
    int32_t bp_ntaps;      // 0 => no bandpass
    int32_t bp_hist;       // bandpass history kept in fd_buf (>= bp_ntaps - 1, multiple of 256)
    int32_t bp_long;       // bp_ntaps > kBpHist + 1: the bandpass runs in bp_long (multi-WG)
    double frac_rate;
    const float2* bp_taps;
    int32_t sq_len, sq_dec, sq_hang, sq_flush, sq_report;
    float sq_level;
    float deemph_alpha, deemph_beta;
    // WFM: prefilter + 12-point Lagrange from the IF-rate FM demod output to the audio rate
    double wfm_rate;       // 250000 / hd_output_rate
    const float* pf_taps;  // prefilter lowpass
    int32_t pf_ntaps;
    float* wf_buf;         // [kWfHist + cap] FmDemod+Limit output (IF rate)
    float* pf_buf;         // [kWfHist + cap] prefiltered
    // NoiseFilter (ClientAudioChain, csdr/chain/clientaudio.py:12-13) between Agc and Convert
    int32_t nr_enabled;
    float nr_t;            // 10^(threshold_dB / 10)
    NrState* nr_state;
    float* nr_in;          // [kNrHop + cap + kNrN] AGC output not yet filtered
    float* nr_pow;         // [2 * (kNrN / 2 + 1)] smoothed power, noise floor per bin
    float* nr_ola;         // [kNrHop] overlap-add tail
    const float* nr_win;   // [kNrN] sqrt periodic Hann
    const float2* nr_tw;   // [kNrN] FFT twiddles
    AgcParams agc;
    // buffers
    ChainStateP* pstate;
    ChainStateS* sstate;
    float2* ddc_buf;       // [kFdHist + cap]
    float2* fd_buf;        // [kBpHist + cap]
    float2* sq_buf;        // [sq_len + cap]
    float* dem;            // this step's demodulator output slot [cap + sq_len + 16]
    int16_t* s16;          // Convert output feeding the ADPCM encoder [cap + sq_len + 16]
    // this step
    const float2* partial; // group partial sums [nseg][group_chains][nk]
    int32_t nseg;
    int32_t group_chains;
    int32_t chain_in_group;
    int32_t nk;            // group outputs this step (step_idx < 0; else StepTable)
    int32_t step_idx;      // the chain's group in this block's StepTable, or -1
    int64_t k_begin;       // absolute output index of partial column 0
    int64_t k_first;       // absolute output index of this chain's output 0
    // outputs
    uint8_t* out;          // staging slot
    int64_t out_cap;
    float* smeter;         // staging slot
    int32_t smeter_cap;
    int32_t debug;         // capture stage outputs
    float2* dbg_ddc;       // staging slots (only when debug)
    float2* dbg_fd;
    float2* dbg_bp;
    float2* dbg_sq;
    float* dbg_dem;
    float* dbg_agc;
    int64_t dbg_cap;
    // secondary FFT on the Selector output (owrx/dsp.py:220-225): FftChain(rate, sf_n, ...)
    int32_t sf_n;          // 0 => none
    int32_t sf_hop;        // Fft every_n_samples
    int32_t sf_avg;        // LogAveragePower avg_number (>= 1; LogPower == 1)
    int32_t sf_adpcm;      // FftAdpcm
    int32_t sf_reset;      // restart the secondary FFT stream this step
    float sf_corr;         // add_db - 10 log10(avg)
    float2* sf_buf;        // [sf_n + stage capacity]
    float* sf_acc;         // [sf_n] open-row accumulator
    const float* sf_window;
    const float2* sf_tw;
    uint8_t* sf_out;       // staging (rows of FftAdpcm bytes or f32 dB)
    int64_t sf_out_cap;
    // taps for secondary readers of ClientDemodulatorChain's buffers (owrx/dsp.py:185-206):
    // the squelched Selector output (selectorBuffer, cf32) and the demodulator chain's audio
    // before ClientAudioChain (audioBuffer, f32); null when nothing reads them
    float2* tap_sq;
    int64_t tap_sq_cap;
    float* tap_agc;
    int64_t tap_agc_cap;
};

// Per-chain counters written by the post kernels for the host (and n_sq for post_serial).
struct ChainCounts {
    int64_t out_bytes;
    int32_t smeter;
    int32_t sf_bytes;      // secondary FFT bytes staged this step
    int64_t n_ddc, n_fd, n_bp, n_sq;  // stage sample counts this step (n_sq: demod/audio)
    int64_t n_gate;        // squelch output samples (IF rate; == n_sq except WFM)
    int64_t n_front;       // samples through the demod front / AGC (n_sq before NoiseFilter)
};

}  // namespace owrx
