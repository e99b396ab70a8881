/*
 * owrx_amd.h -- C ABI of libowrx_amd.so, the MI355X-native IQ backend for OpenWebRX.
 *
 * Drop-in boundary.  In the reference the hot path ends at the pycsdr extension
 * (pycsdr.modules / pycsdr.types, C++ csdr underneath, not in /root/reference); its Python
 * callers are csdr/chain/{fft,selector,analog,clientaudio}.py, owrx/fft.py and owrx/dsp.py.
 * This library is what a pycsdr-compatible binding calls instead (the in-tree binding is the
 * ctypes package `pycsdr/` + `openwebrx_amd/`; INTEGRATION.md shows the stubs).  Plain
 * pointers and sizes only.
 *
 * Return codes: >= 0 ok (or a count), negative errno-style values below; the binding maps
 * OWRX_EINVAL to ValueError (the reference's format/parameter error convention,
 * csdr/chain/__init__.py:60-84) and the rest to OSError.  owrx_last_error() returns the
 * thread's last message.
 *
 * Threading: one engine per GPU; every call on an engine is serialised internally, setters may
 * be called from any thread and take effect at the next processed block (owrx/dsp.py:538-562
 * wires property callbacks from arbitrary threads).
 */
#ifndef OWRX_AMD_H
#define OWRX_AMD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OWRX_OK 0
#define OWRX_EIO (-5)       /* HIP runtime failure (engine marked failed) */
#define OWRX_EAGAIN (-11)   /* nothing to read yet */
#define OWRX_ENOMEM (-12)
#define OWRX_EINVAL (-22)
#define OWRX_ENOSPC (-28)   /* output ring overrun (oldest data dropped) */
#define OWRX_ENODEV (-19)   /* no gfx950 device */
#define OWRX_ETIMEDOUT (-110) /* a wait on the GPU exceeded the stall timeout (engine marked failed) */

#define OWRX_DEMOD_NFM 0
#define OWRX_DEMOD_AM 1
#define OWRX_DEMOD_SSB 2    /* RealPart: usb / lsb / cw (owrx/dsp.py:617-619) */
#define OWRX_DEMOD_WFM 3    /* WFm (csdr/chain/analog.py:55-116): FmDemod, Limit,
                               FractionalDecimator(FLOAT, IF/audio_rate, prefilter=True),
                               WfmDeemphasis(audio_rate, deemph_tau); no AGC.  The Selector
                               runs at the fixed 250 kHz IF (analog.py:81-82). */
#define OWRX_DEMOD_SAM 4    /* SAm / RawSAm (csdr/chain/analog.py:141-167): Afc(afc_update,
                               afc_sample) -> RealPart -> DcBlock -> Agc, or -> Gain(audio_gain)
                               with audio_gain > 0 (RawSAm); RawAm (analog.py:23-31) is
                               OWRX_DEMOD_AM with audio_gain > 0 (DcBlock -> Gain) */

#define OWRX_OUT_S16 0      /* Convert(FLOAT, SHORT) */
#define OWRX_OUT_ADPCM 1    /* Convert + AdpcmEncoder(sync=True) */
#define OWRX_OUT_F32 2      /* raw float audio (no Convert) */
#define OWRX_OUT_IQ 3       /* Shift + FirDecimate output only, cf32 at in/D: the service
                               Resampler (owrx/source/resampler.py:11-26) */
#define OWRX_OUT_SEL 4      /* the whole Selector's output, cf32 at the output rate (Shift,
                               FirDecimate, FractionalDecimator, Bandpass, Squelch if any): an
                               IQ-input decoder behind Selector(withSquelch=False), the
                               ServiceDemodulatorChain (owrx/service/chain.py:7-23); `demod`,
                               the AGC and the audio fields are unused */

#define OWRX_AGC_FAST 0
#define OWRX_AGC_SLOW 1
#define OWRX_AGC_MID 2
#define OWRX_AGC_LAGGY 3

typedef struct owrx_engine owrx_engine;

const char* owrx_version(void);               /* "0.18.x-amd" (owrx/feature.py:213-221 gate) */
const char* owrx_last_error(void);
int owrx_device_count(void);                   /* visible HIP devices, or OWRX_ENODEV */

/* ---- engine: one wideband IQ stream on one GPU ------------------------------------------
 * Replaces the wideband pycsdr Buffer(COMPLEX_FLOAT) fed by TcpSource
 * (owrx/source/__init__.py:307-330) and the per-module native threads. */
int owrx_engine_create(int device, double samp_rate, int64_t max_block, owrx_engine** out);
/* As owrx_engine_create, keeping `history` samples of the stream before each block readable
 * (<= 0: the minimum, 2^18: the longest FIR and the FFT overlap).  A longer history lets a
 * waterfall batch the frames of several blocks into one chip-filling launch
 * (owrx_waterfall_set_batch).  The push path keeps it in one device ring (the last `history`
 * samples are copied to the ring's start once per lap, not per block). */
int owrx_engine_create_ex(int device, double samp_rate, int64_t max_block, int64_t history,
                          owrx_engine** out);
int owrx_engine_destroy(owrx_engine* e);
/* samples that must precede a block handed to owrx_process_device (filter/FFT history) */
int64_t owrx_engine_history(owrx_engine* e);
int64_t owrx_engine_max_block(owrx_engine* e);

/* Host cf32 (interleaved little-endian float I,Q) -> device; processes whole blocks.
 * Equivalent of Writer.write() on the wideband Buffer. */
int owrx_push_iq(owrx_engine* e, const float* iq_cf32, int64_t nsamples);
/* Host cs16 (interleaved little-endian int16 I,Q) -> cf32 on the GPU, as the reference's
 * ingest conversion Chain([Convert(COMPLEX_SHORT, COMPLEX_FLOAT), Gain(COMPLEX_FLOAT, gain)])
 * (owrx/source/direct.py:51-71 getBuffer, fifi_sdr.py:27-28): x / 32767 * gain.  Half the
 * PCIe bytes of owrx_push_iq; the conversion kernel writes straight into the engine window. */
int owrx_push_iq_cs16(owrx_engine* e, const int16_t* iq_cs16, int64_t nsamples, float gain);
/* Device-resident cf32 block; iq_dev[-history, 0) must hold the previous samples of the stream
 * (e.g. a contiguous HBM recording, or an RCCL-broadcast window).  Zero-copy and asynchronous:
 * the block (with its history) must stay unmodified until the next owrx_process_device /
 * owrx_commit / owrx_push_iq / owrx_sync call on this engine has returned. */
int owrx_process_device(owrx_engine* e, const float* iq_dev, int64_t nsamples);
/* The engine's work from the next block on waits, on the GPU, for everything enqueued so far on
 * `stream` (a hipStream_t of the same device; NULL: the null stream), e.g. the collective that
 * writes the next owrx_process_device window (multi-GPU IQ broadcast).  The host
 * does not wait. */
int owrx_wait_stream(owrx_engine* e, void* stream);
/* Callers whose input blocks stay valid longer (a resident recording, a ring of windows): with
 * blocks = r the block handed to owrx_process_device (with its history) must stay unmodified
 * until r further owrx_process_device / owrx_commit calls (or owrx_sync) have returned, and the
 * engine waits only for block k - r + 1's stream-A work before returning from block k, so the
 * host runs up to r blocks ahead of stream A.  Default 1 (the contract above); 1 <= r <= 31, and
 * r >= 2 x the block group while grouping / pairing is on (OWRX_EINVAL otherwise). */
int owrx_set_input_retention(owrx_engine* e, int blocks);
/* Block pairing (enable = 1; input retention >= 4, before the first chain, waterfall and block):
 * owrx_process_device holds a block until the next call; when the next block follows it in
 * memory (block + nsamples == next) both run as one engine block, otherwise the held one runs
 * alone.  Every stage runs once per pair and the DDC's filter spectra are read once for both
 * blocks' frames; each block keeps its own DDC frames and zero padding, so every output is
 * byte-identical to unpaired processing.  A held block runs at the latest on the next call that
 * is not a read (owrx_sync, chain or waterfall changes, push / commit) or owrx_wait_stream's
 * successor, so it adds one block of latency: for callers that are blocks ahead of the stream
 * (a recording), not for a live source.  Staging is sized for 2 x max_block. */
int owrx_set_block_pairing(owrx_engine* e, int enable);
/* Block grouping, the general form of pairing (round 6): blocks = 1 (off), 2 (= pairing), 3 or 4
 * contiguous caller blocks run as one engine block, with input retention >= 2 x blocks; same
 * preconditions, contract and byte-identical outputs as owrx_set_block_pairing.  Each engine block
 * reads the DDC's filter spectra once for all its blocks' frames (quads: the per-bin GEMM at about
 * twice a pair's arithmetic intensity) and launches every stage once; it adds blocks - 1 blocks of
 * latency.  Staging is sized for blocks x max_block. */
int owrx_set_block_group(owrx_engine* e, int blocks);
/* Blocks of chain work in flight (streams A -> B -> C -> host rings), 1..16, default 8; only
 * before the first chain and block.  Each one holds pinned and device staging for every chain
 * (at 98 304 chains ~0.5 GB pinned per block), so deeper pipelines are for few-chain, high-rate
 * engines.  No reference counterpart: csdr runs each module in its own thread with its own
 * buffer (owrx/dsp.py:846-863 pumps); this is the engine's equivalent of that slack. */
int owrx_set_pipeline_depth(owrx_engine* e, int blocks);
/* Stall bound (default 20 000 ms): no call blocks longer than this waiting for the GPU.  When a
 * wait expires the engine is marked failed and the call, and every later one, returns
 * OWRX_ETIMEDOUT -- the engine-side counterpart of the reference's source failure
 * (owrx/source/__init__.py:432-448 fail() -> onFail, owrx/connection.py:292-295), which the
 * pycsdr shim turns into a FAILED driver with every output buffer ended.  owrx_engine_destroy
 * waits one more bound for the streams and then leaks the engine's buffers rather than free them
 * under a running kernel. */
int owrx_set_stall_timeout(owrx_engine* e, int64_t ms);
/* Test hook: enqueues a kernel that occupies stream 0 (A: FFT / DDC), 1 (B), 2 (C), 3 (R: the
 * output gathers) or 4 (the next waterfall row slot's stream) for `us` microseconds and then
 * exits (stall injection for the bounded-wait path; held copies for the reconfiguration tests). */
int owrx_debug_stall(owrx_engine* e, int stream, int64_t us);
/* Host self-test (no GPU needed): the fast-convolution DDC's tiled filter-spectrum layout maps
 * every (member slot < cap, branch < Dp) inside its bin's row of cap * Dp entries, one entry per
 * element.  OWRX_OK, or OWRX_EINVAL (the reason in owrx_last_error). */
int owrx_selftest_w_layout(int Dp, int cap);
/* Device window slot for the next block (write there, e.g. with ncclBroadcast), then commit. */
int owrx_ingest_buffer(owrx_engine* e, float** dev_ptr, int64_t* capacity);
int owrx_commit(owrx_engine* e, int64_t nsamples);
/* Waits for all enqueued device work and drains outputs into the host rings. */
int owrx_sync(owrx_engine* e);

/* ---- waterfall: FftChain (csdr/chain/fft.py:25-96) --------------------------------------
 * Fft(size=fft_size, every_n_samples) -> LogAveragePower(add_db, fft_size, avg_number) or
 * LogPower(add_db) when avg_number == 0 (fft.py:18-22) -> FftSwap -> FftAdpcm if compression.
 * fft_size: power of two, 256..65536.  The reference UI validates 256..16384
 * (owrx/controllers/settings/general.py:181); BASELINE config 4 asks for 65536 bins (sizes
 * above 16384 run a two-launch four-step FFT). */
int owrx_waterfall_create(owrx_engine* e, int fft_size, int every_n_samples, int avg_number,
                          float add_db, int adpcm, int* handle);
/* FftChain._setBlockSize / setFftAverages / setCompression (fft.py:51-55, 11-16, 87-96) */
int owrx_waterfall_set(owrx_engine* e, int handle, int every_n_samples, int avg_number,
                       int adpcm);
/* Launch granularity of the waterfall FFT (an engine-side choice; for a fixed batch setting the
 * rows, bit for bit, and their order do not depend on how the stream is cut into blocks -- the
 * setting picks the frames summed per workgroup, so rows under different settings may differ in
 * the last ulp of the dB value).  Complete frame groups are launched when at least
 * `min_frames` are ready, or when the oldest pending frame starts `max_lag` or more samples
 * before the end of the newest block, or before it would leave the engine history, and on
 * owrx_sync.  min_frames <= 1 (the default): every block's frames in that block.  max_lag <= 0:
 * as far as the history allows.  Rows then reach the reader up to max_lag samples later than
 * with per-block launches (the throughput / latency trade of Fft(every_n_samples) batching). */
int owrx_waterfall_set_batch(owrx_engine* e, int handle, int min_frames, int64_t max_lag);
/* Wall-clock bound on that batching (the row latency a client sees): pending frames are also
 * launched at the first block call at which waiting for one more block (the engine's running
 * estimate of the interval between block calls) would leave the oldest pending frame unlaunched
 * for more than `max_wall_ms` after the call that made it ready.  At the stream's real-time rate
 * this launches every block or two; fed faster than real time (a throughput run) the frame
 * count bound applies.  max_wall_ms <= 0: no wall-clock bound (the default). */
int owrx_waterfall_set_latency(owrx_engine* e, int handle, double max_wall_ms);
int owrx_waterfall_destroy(owrx_engine* e, int handle);
/* bytes of one output row: (fft_size+10)/2 with ADPCM, 4*fft_size without */
/* Frames one full round of this waterfall's FFT launch deals (stream A's resident workgroups x
 * frames per group; 0 where launches are not dealt in rounds): a caller that batches frames
 * (owrx_waterfall_set_batch) in whole rounds leaves no partial last round. */
int owrx_waterfall_round_frames(owrx_engine* e, int handle);
int64_t owrx_waterfall_row_bytes(owrx_engine* e, int handle);
/* copies whole rows (<= max_bytes) from the row ring; 0 when none; Reader.read() of the
 * spectrum buffer (owrx/fft.py:70-73) */
int64_t owrx_waterfall_read(owrx_engine* e, int handle, uint8_t* dst, int64_t max_bytes);

/* ---- client demod chain: ClientDemodulatorChain (owrx/dsp.py:39-72) ----------------------
 * [Selector(Shift, FirDecimate, [FractionalDecimator], [Bandpass], Squelch),
 *  NFm | Am | Ssb, ClientAudioChain(Convert, [AdpcmEncoder(sync=True)])]. */
typedef struct {
    float   shift_rate;      /* Shift.setRate(-offset/inRate)      selector.py:132-140 */
    int32_t decimation;      /* FirDecimate(decimation, transition, cutoff)  selector.py:29 */
    float   transition;
    float   cutoff;
    double  frac_rate;       /* FractionalDecimator rate; 1.0 => absent   selector.py:32-33 */
    int32_t bandpass;        /* 1 => Bandpass inserted (both cuts set)    selector.py:159-166 */
    float   bp_low;          /* normalised to the output rate */
    float   bp_high;
    float   bp_transition;   /* 320/outputRate                            selector.py:115-117 */
    int32_t sq_length;       /* Squelch(...)                              selector.py:119-130 */
    int32_t sq_decimation;
    int32_t sq_hang;
    int32_t sq_flush;
    int32_t sq_report;
    float   sq_level;        /* linear power, setSquelchLevel(10^(dB/10)) */
    int32_t demod;           /* OWRX_DEMOD_* */
    int32_t agc_profile;     /* OWRX_AGC_* */
    float   agc_initial_gain;/* < 0 => profile default; Am: 200 (analog.py:15) */
    float   agc_max_gain;    /* < 0 => profile default; NFm: 3 (analog.py:40) */
    int32_t audio_rate;      /* NfmDeemphasis(sampleRate) (analog.py:45) */
    int32_t output;          /* OWRX_OUT_* */
    float   deemph_tau;      /* WFM: WfmDeemphasis tau (wfm_deemphasis_tau, default 50e-6,
                                owrx/config/defaults.py:21); 0 => 50e-6 */
    double  if_rate;         /* WFM: the Selector output rate (250000); audio_rate is the HD
                                output rate (48000, owrx/dsp.py:494) */
    int32_t nr_enabled;      /* ClientAudioChain NoiseFilter(nr_threshold) before Convert
                                (csdr/chain/clientaudio.py:12-13; owrx/dsp.py:496-509) */
    float   nr_threshold;    /* dB, the UI's -20..20 slider (htdocs/index.html:278) */
    int32_t afc_update;      /* OWRX_DEMOD_SAM: Afc(updatePeriod, samplePeriod): SAm 10, 4;  */
    int32_t afc_sample;      /*   RawSAm 50, 8 (analog.py:143-144, :158-159) */
    float   audio_gain;      /* > 0 => Gain(FLOAT, audio_gain) after DcBlock instead of Agc
                                (RawAm, RawSAm: 100, analog.py:29, :165); 0 => Agc */
} owrx_chain_params;

/* Chains with the same FirDecimate design share one fast-convolution group; every output is
 * deterministic for a given membership, but the GEMM's K split across workgroups follows the
 * group's size (kernels_fcddc.hip fc_kslices), so a chain's DDC output can change at the float
 * rounding level (<= 1e-6 rel-RMS, tests/test_gpu_parity.py
 * test_ddc_group_size_changes_rounding_only) when other clients of its design join or leave. */
int owrx_chain_create(owrx_engine* e, const owrx_chain_params* p, int* handle);
int owrx_chain_destroy(owrx_engine* e, int handle);
int owrx_chain_set_shift_rate(owrx_engine* e, int handle, float rate);
int owrx_chain_set_bandpass(owrx_engine* e, int handle, int enabled, float low, float high);
int owrx_chain_set_squelch_level(owrx_engine* e, int handle, float level);
/* ClientAudioChain.setNrEnabled / setNrThreshold (csdr/chain/clientaudio.py:80-90): the
 * reference rebuilds the Converter, i.e. a fresh NoiseFilter; so does this (state reset at the
 * next block). */
int owrx_chain_set_noise_filter(owrx_engine* e, int handle, int enabled, float threshold_db);
/* audio bytes (s16 LE / ADPCM stream / f32) produced so far; Reader.read() of the audio
 * buffer (owrx/dsp.py:846-863) */
int64_t owrx_chain_read_audio(owrx_engine* e, int handle, uint8_t* dst, int64_t max_bytes);
/* Squelch power writer values (owrx/connection.py:483-489) */
int64_t owrx_chain_read_smeter(owrx_engine* e, int handle, float* dst, int64_t max_values);
/* Batched forms for a server pump that serves many clients from one thread (the reference runs
 * one pump thread per output, owrx/dsp.py:846-863): chain handles[i]'s available bytes / values
 * are appended to dst in order until max_bytes / max_values; lens[i] / counts[i] receive each
 * chain's share.  Returns the total.  Every handle may appear once: a repeated or unknown
 * handle returns OWRX_EINVAL and reads nothing.  dst == NULL with max_bytes / max_values == 0
 * is a size query: lens[i] / counts[i] receive what each chain holds, the sum is returned and
 * nothing is read (a pump sizes its buffer so one call drains every ring). */
int64_t owrx_chains_read_audio(owrx_engine* e, int n, const int* handles, uint8_t* dst,
                               int64_t max_bytes, int64_t* lens);
int64_t owrx_chains_read_smeter(owrx_engine* e, int n, const int* handles, float* dst,
                                int64_t max_values, int64_t* counts);
/* Secondary FFT of the chain's Selector output: ClientDemodulatorChain._createSecondaryFftChain
 * (owrx/dsp.py:220-225) = FftChain(selectorOutputRate, digimodes_fft_size, 0.3, 9, "adpcm")
 * reading selectorBuffer, i.e. Fft(size, every_n_samples) -> LogAveragePower(add_db, size,
 * avg_number) | LogPower when avg_number == 0 -> FftSwap -> FftAdpcm if adpcm
 * (csdr/chain/fft.py:25-96).  fft_size: 0 (remove) or a power of two in [1024, 8192];
 * setSecondaryFftSize / setSampleRate re-create it (owrx/dsp.py:357-363, :216-217), which
 * restarts the row stream.  Rows are owrx_chain_secondary_fft_row_bytes() each:
 * (fft_size+10)/2 ADPCM bytes or fft_size f32 dB. */
int owrx_chain_set_secondary_fft(owrx_engine* e, int handle, int fft_size, int every_n_samples,
                                 int avg_number, float add_db, int adpcm);
int64_t owrx_chain_secondary_fft_row_bytes(owrx_engine* e, int handle);
/* whole rows only (<= max_bytes); the secondary FFT Writer (frame type 0x03,
 * owrx/connection.py:500-501) */
int64_t owrx_chain_read_secondary_fft(owrx_engine* e, int handle, uint8_t* dst,
                                      int64_t max_bytes);
/* Taps for secondary readers of the chain's buffers (ClientDemodulatorChain, owrx/dsp.py:185-206):
 * selector != 0 publishes the Selector output (squelch-gated cf32 at the Selector rate, what
 * selectorBuffer carries to a SecondarySelector or a COMPLEX_FLOAT secondary demodulator);
 * audio != 0 the demodulator chain's f32 output before ClientAudioChain (what audioBuffer
 * carries to a FLOAT secondary demodulator).  The chain itself is unchanged. */
int owrx_chain_set_taps(owrx_engine* e, int handle, int selector, int audio);
/* which: 0 selector (cf32 items), 1 audio (f32 items); whole items only */
int64_t owrx_chain_read_tap(owrx_engine* e, int handle, int which, uint8_t* dst,
                            int64_t max_bytes);
/* absolute stream sample index of the chain's sample 0 (aligned to the decimation grid) */
int64_t owrx_chain_origin(owrx_engine* e, int handle);

/* ---- parity taps (tests): per-chain stage outputs captured while debug is enabled --------
 * stage 0: Selector DDC output (cf32), 1: after FractionalDecimator (cf32),
 * 2: after Bandpass (cf32), 3: after Squelch (cf32), 4: demod output before AGC (f32),
 * 5: AGC output (f32). */
int owrx_set_debug(owrx_engine* e, int enable);
int64_t owrx_chain_read_debug(owrx_engine* e, int handle, int stage, void* dst,
                              int64_t max_bytes);

typedef struct {
    int64_t samples_in;        /* IQ samples processed */
    int64_t blocks;            /* process calls */
    int64_t ddc_outputs;       /* sum over chains */
    int64_t waterfall_rows;
    int64_t audio_bytes;
    int64_t overruns;          /* host output ring drops */
    double  gpu_ms_ddc;        /* HIP-event time of the DDC kernels (when timing enabled) */
    double  gpu_ms_waterfall;
    double  gpu_ms_post;       /* stream A's post kernels (post_parallel, bp_long, chain_sfft) */
    int64_t ddc_launches;
    int64_t waterfall_launches;
    int64_t ddc_fast_launches; /* of ddc_launches: fast-convolution form (OWRX_DDC_FAST) */
    double  gpu_ms_ddc_mac;    /* HIP-event time of the fast form's GEMM (fc_mac), timed blocks */
    double  ddc_mac_flop;      /* its algorithmic flop (8 per complex MAC, frames with outputs) */
    double  ddc_mac_bytes;     /* its algorithmic bytes: filter spectra W + branch spectra U + Y */
    double  gpu_ms_serial;     /* post_parallel start -> encoder end (streams A, B, C) */
    double  host_ms_process;   /* host time inside block processing, of which waiting for: */
    double  host_ms_wait_input;/*   the previous block's stream-A work (input / descriptors) */
    double  host_ms_wait_slots;/*   block k - 4's chain outputs (the pipeline depth) */
    double  host_ms_wait_rows; /*   the oldest waterfall row slot */
    int64_t waterfall_frames;  /* FFT frames launched */
    int64_t waterfall_samples; /* stream samples those frames advanced over (frames x hop) */
    double  gpu_ms_waterfall_fft; /* HIP-event time of the waterfall FFT + finalize launches
                                     alone (timing enabled), for the HBM roofline */
    int64_t waterfall_timed_samples; /* stream samples of the frames those timed launches did */
    int64_t timed_blocks;      /* blocks whose kernel groups were timed (owrx_set_timing) */
    int64_t pipeline_drains;   /* full drains of the block pipeline (owrx_sync, waterfall
                                  reconfiguration, staging growth); chain joins / leaves and
                                  their setters do not drain */
    double  host_ms_build;     /* host time building a block's chain descriptors (of process) */
    double  host_ms_launch;    /* host time enqueueing its kernels, copies and events */
    double  host_ms_collect;   /* host time moving finished blocks into the output rings */
    /* waterfall row latency (wall clock): from the owrx_push_iq / owrx_process_device /
     * owrx_commit call that completed a row's last frame to the row being readable
     * (owrx_waterfall_read) */
    double  wf_row_latency_ms_max;
    double  wf_row_latency_ms_sum;
    int64_t wf_rows_latency_n;
    /* the fast-convolution GEMM form launched: fc_mac_lds (LDS-DMA ring) launches of all the
     * fast DDC launches, and the most K slices across workgroups one of them used */
    int64_t ddc_mac_lds_launches;
    int64_t ddc_mac_kslices_max;
    /* device (hipMalloc) and pinned (hipHostMalloc) allocations made by the engine's pools so
     * far: none should happen while blocks stream, since each stalls the GPU's running kernels */
    int64_t pool_allocs;
    double  gpu_ms_waterfall_fft_max;  /* the longest timed waterfall FFT + finalize launch */
    int64_t waterfall_timed_launches;  /* the launches gpu_ms_waterfall_fft and
                                          waterfall_timed_samples cover */
    /* finished blocks moved into the output rings (in host_ms_wait_slots and host_ms_collect):
     * waiting for a block's chain outputs to land in pinned memory, and copying them into the
     * chains' rings */
    double  host_ms_drain_wait;
    double  host_ms_drain_copy;
    int64_t ddc_frame_length;  /* the fast DDC's frame length M of the newest chain group */
} owrx_stats;
int owrx_get_stats(owrx_engine* e, owrx_stats* s);
/* n > 0 => record HIP events around each kernel group on the engine's streams in every n-th
 * block (the gpu_ms_* statistics average over those blocks); 0 => off */
int owrx_set_timing(owrx_engine* e, int every_n_blocks);
/* Form of the fused Shift + FirDecimate (csdr/chain/selector.py:11-35, :95, :132-140) every
 * chain group runs from the next block on.  Both compute y[k] = sum_t h[t] x[kD+t] e^{j phase}
 * exactly (fp32 rounding apart):
 *   OWRX_DDC_FAST   polyphase branches convolved through M-point DFTs, the per-chain filter
 *                   spectra applied as one f32-MFMA complex GEMM per bin (default)
 *   OWRX_DDC_DIRECT the direct polyphase FIR (4T + 6D flop per output and chain) */
#define OWRX_DDC_FAST 0
#define OWRX_DDC_DIRECT 1
int owrx_set_ddc_mode(owrx_engine* e, int mode);

/* ---- single-module runners (pycsdr module granularity, stateful, host buffers) -----------
 * Used by pycsdr.modules classes that run outside a fused chain and by the per-module parity
 * tests.  type: OWRX_MOD_*; params as documented per type; returns outputs produced. */
#define OWRX_MOD_FMDEMOD 1
#define OWRX_MOD_AMDEMOD 2
#define OWRX_MOD_REALPART 3
#define OWRX_MOD_LIMIT 4          /* p0 = max amplitude */
#define OWRX_MOD_DCBLOCK 5
#define OWRX_MOD_DEEMPH 6         /* p0 = alpha */
#define OWRX_MOD_AGC 7            /* p0 profile, p1 initial gain (<0 default), p2 max gain */
#define OWRX_MOD_CONVERT_F_S16 8
#define OWRX_MOD_ADPCM 9          /* p0 = sync (0/1); input s16 */
#define OWRX_MOD_FFTSWAP 10       /* p0 = fft size; input f32 rows */
#define OWRX_MOD_FFTADPCM 11      /* p0 = fft size; input f32 rows (already swapped) */
#define OWRX_MOD_CONVERT_CS16_CF32 12  /* Convert(COMPLEX_SHORT, COMPLEX_FLOAT); n = samples */
#define OWRX_MOD_GAIN 13          /* Gain(format, p0); p1 = 1 complex (n samples), 0 float */
#define OWRX_MOD_SHIFT 14         /* Shift(p0 = rate), cf32; phase continuous across calls */
#define OWRX_MOD_BANDPASS 15      /* Bandpass(p0 = low, p1 = high, p2 = transition), cf32 */
#define OWRX_MOD_AFC 17            /* Afc(p0 = updatePeriod, p1 = samplePeriod), cf32 -> cf32:
                                     carrier frequency tracking of SAm / RawSAm
                                     (csdr/chain/analog.py:141-167); csdr's algorithm is not in
                                     the reference: the build's documented choice */
#define OWRX_MOD_AUDIO_RESAMPLER 16 /* AudioResampler(p0 = input rate, p1 = output rate), f32:
                                       rational L/M polyphase lowpass (the build's choice) */
typedef struct owrx_module owrx_module;
int owrx_module_create(int device, int type, double p0, double p1, double p2,
                       owrx_module** out);
int owrx_module_destroy(owrx_module* m);
/* Shift.setRate(p0) (phase continuous) / Bandpass.setBandpass(p0, p1) with transition p2 */
int owrx_module_set(owrx_module* m, double p0, double p1, double p2);
/* in: n input items (cf32 for demods, f32, s16 for ADPCM); out: capacity in bytes */
int64_t owrx_module_process(owrx_module* m, const void* in, int64_t n, void* out,
                            int64_t out_cap_bytes);

/* ---- synthetic test source (benchmarks / tests; SURVEY.md 8d signal model) ---------------
 * Writes n cf32 samples of the stream starting at absolute sample `start` into device memory:
 * complex AWGN (sigma `noise`) + one carrier per entry of offsets_hz with modes[c] 0 NFM (1 kHz,
 * 2.5 kHz deviation), 1 AM (30 %, 1 kHz), 2 USB (+1 kHz tone), 3 CW (+800 Hz), 4 LSB (-1 kHz),
 * amplitude `amp`.  Synchronous.  Stands in for the SDR source (owrx/source/__init__.py:307-330). */
int owrx_synth_iq(int device, float* dst_dev, int64_t n, int64_t start, double samp_rate,
                  int ncarriers, const double* offsets_hz, const int* modes, uint64_t seed,
                  float noise, float amp);

#ifdef __cplusplus
}
#endif
#endif
