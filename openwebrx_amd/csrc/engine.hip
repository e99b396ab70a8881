// engine.hip -- host side of libowrx_amd.so: one engine per GPU and per wideband IQ stream.
//
// Replaces the reference's per-module native threads + ring buffers (pycsdr Buffer/Reader,
// csdr modules; callers owrx/fft.py:36-73 and owrx/dsp.py:39-72, 835-863) with a block
// scheduler over four HIP streams (one hardware queue each, GPU_MAX_HW_QUEUES = 4):
//   A (main):   wf_fft_power + wf_finalize per FftChain; DDC per (D, taps) group;
//               post_parallel for all client chains
//   B (serial): post_serial_front (deemphasis / DC block, AGC, Convert)
//   C (serial): chain_adpcm (AdpcmEncoder), back to back: the longest serial stage
//   R (rows):   wf_adpcm_rows + D2H of waterfall rows; D2H of audio, s-meter, debug taps
// B, C and R have a few dedicated CUs each (OWRX_SERIAL_CUS), so block k's serial work runs
// beside the next blocks' stream-A work; kSlots blocks are in flight and their outputs are
// drained, in order, into the host rings that the pycsdr binding reads.
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <chrono>
#include <cmath>
#include <deque>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include "../../include/owrx_amd.h"
#include "design.h"
#include "owrx_types.h"

// OWRX_SEGV_TRACE=1: a host SIGSEGV prints the faulting thread's native frames (library +
// offset, for addr2line) before the default action -- Python's faulthandler shows only the
// Python frames of a crash inside a C-ABI call
static void owrx_segv_trace(int sig) {
    void* fr[48];
    const int n = backtrace(fr, 48);
    for (int i = 0; i < n; ++i) {
        Dl_info di;
        char line[512];
        int len;
        if (dladdr(fr[i], &di) && di.dli_fname)
            len = snprintf(line, sizeof line, "  #%d %s +0x%lx (%s)\n", i, di.dli_fname,
                           (unsigned long)((char*)fr[i] - (char*)di.dli_fbase),
                           di.dli_sname ? di.dli_sname : "?");
        else
            len = snprintf(line, sizeof line, "  #%d %p\n", i, fr[i]);
        if (len > 0) (void)!write(2, line, (size_t)std::min(len, (int)sizeof line - 1));
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
static const bool g_segv_trace = [] {
    if (getenv("OWRX_SEGV_TRACE")) signal(SIGSEGV, owrx_segv_trace);
    return true;
}();

namespace owrx {

static thread_local std::string g_last_error;
void set_last_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

// kernel launchers (kernels_*.hip)
hipError_t launch_debug_sleep(int64_t us, hipStream_t st);  // synth.hip (stall injection)
hipError_t launch_wf_fft(int logn, const float2* blk, int64_t blk_start, const WfGroup* groups,
                         int ngroups, int fpg, const float* window, const float* ones,
                         const float2* tw, float* partial, float2* scratch, int* work, int cus,
                         hipStream_t st, int skip, int tail);
int wf_tail_split(int logn, int ngroups, int cus, int64_t frames, int fpg);
int wf_round_frames(int logn, int cus, int fpg);  // frames one full round of a launch deals
bool wf_uses_split(int logn);  // kernels_waterfall.hip: N = 32768 / 65536 via the DIF split
bool wf_uses_l32(int logn);  // kernels_waterfall.hip: N = 16384 on wf_fft_q16 / l32 (not r16)
int wf_default_fpg(int logn);
hipError_t launch_wf_finalize(const float* partial, const WfRow* rows, int nrows,
                              const float* carry_in, float* carry_out, int N, float add_corr,
                              int adpcm, int16_t* s16_out, float* f32_out, hipStream_t st,
                              const WfGroup* groups, int ngroups, int skip);
hipError_t launch_wf_adpcm(const int16_t* s16, int N, int nrows, uint8_t* out, int row_bytes,
                           int wgs, hipStream_t st);
hipError_t launch_ddc(int P, const float2* blk, int64_t blk_start, int64_t blk_end,
                      const float* taps_poly, const DdcChain* chains, int nchains, int D,
                      int64_t k_begin, int nk, int nseg, float2* partial, hipStream_t st);
int ddc_padded_p(int p);
int ddc_segments(int D, int nseg, int P, int nchains);
int ddc_blocks_per_cu(int P, int nchains);
int fc_frame_supported(int m);  // kernels_fcddc.hip
hipError_t launch_fc_make_w(int m, const float* h, int T, int D, int Dp, int P,
                            uint64_t rate_fx, float2* W, int64_t w_ks, hipStream_t st);
hipError_t launch_fc_move_w(int M, float2* W, int64_t w_ks, int Dp, int src, int dst, hipStream_t st);
hipError_t launch_fc_make_w_jobs(int m, const float* h, int T, int D, int Dp, int P,
                                 const FcWJob* jobs, int njobs, float2* W, int64_t w_ks,
                                 hipStream_t st);
int64_t fc_w_chain_offset(int c, int Dp);  // chain c's first entry in a bin's row of the tiled W
int fc_w_tile();                           // chains per W tile: capacities are multiples of it
int fc_w_layout_check(int Dp, int cap);    // host self-test of the tiled W layout
int fc_frames(const FcSubs& sb, int V);  // frames of a (grouped) engine block
hipError_t launch_fc_ddc(int M, const float2* blk, int64_t blk_start, const FcSubs& sb,
                         const DdcChain* chains, const float2* W, int64_t w_cs, int64_t w_ks,
                         int nchains, int D, int Dp, int V, int Fs, int64_t k_begin, int nk,
                         const float2* tw, float2* U, float2* Y, int64_t y_cap, float2* out,
                         int ncu, hipStream_t st, hipEvent_t mac0, hipEvent_t mac1, int* form);
int fc_kslices_max(int M, int nchains, int Dp, int ncu);  // Y slices a group may need
hipError_t launch_post_parallel(const ChainPost* posts, int nchains, ChainCounts* counts,
                                const StepTable& steps, hipStream_t st);
hipError_t launch_post_long(const ChainPost* posts, ChainCounts* counts, const int* idx,
                            int nlong, int64_t max_fd, int max_taps, hipStream_t st);
hipError_t launch_post_serial(const ChainPost* posts, ChainCounts* counts, const int* sel,
                              int nsel, int output, int debug, int nr, hipStream_t st);
hipError_t launch_chain_nr(const ChainPost* posts, int nposts, ChainCounts* counts,
                           hipStream_t st);
hipError_t launch_chain_sfft(int logn, const ChainPost* posts, int nposts, ChainCounts* counts,
                             hipStream_t st);
hipError_t launch_chain_afc(const ChainPost* posts, ChainCounts* counts, const int* sel, int nsel,
                            hipStream_t st);
hipError_t launch_chain_adpcm(const ChainPost* posts, ChainCounts* counts, const int* sel,
                              int nsel, hipStream_t st);

constexpr int kWfMaxFramesPerGroup = 16;  // frames one FFT workgroup sums (N <= kWfLdsMaxN)
constexpr int kWfLdsMaxN = 16384;      // largest FFT held in one CU's LDS
constexpr int kWfSplitMaxFpg = 4;      // frames per group of the DIF-split path (N > kWfLdsMaxN)
constexpr int kWfMaxN = 65536;
constexpr int kBlMaxTaps = 4095;       // longest bandpass of the bp_long path (kernels_post.hip)
constexpr int kSelPad = 64 * 4 * 6;    // serial lane lists: 64-lane padding per (output, NR, demod)
constexpr int64_t kDefaultHistory = 1 << 18;
constexpr int kDebugStages = 6;
#ifndef OWRX_SLOTS
#define OWRX_SLOTS 16
#endif
constexpr int kSlots = OWRX_SLOTS;  // the most blocks of chain work in flight (A -> B -> C)
constexpr int kDefaultSlots = 8;    // owrx_set_pipeline_depth: the engine's own (e->nslots)
constexpr int kInEv = 2 * kSlots;   // stream-A completion events kept (block index mod kInEv;
                                   // > kSlots: the slot-reuse wait reads block k - nslots's)
constexpr int kRowSlots = 4;  // waterfall row blocks in flight (each on its own stream, R CUs)

#define HIPCHK(expr)                                                                    \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) {                                                         \
            set_last_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),        \
                           __FILE__, __LINE__);                                         \
            return OWRX_EIO;                                                            \
        }                                                                               \
    } while (0)

#define RCCHK(expr)               \
    do {                          \
        int _rc = (expr);         \
        if (_rc) return _rc;      \
    } while (0)

template <typename T>
static hipError_t dalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, sizeof(T) * count);
    if (e == hipSuccess) e = hipMemset(*p, 0, sizeof(T) * count);
    // a failed allocation is reported here; clear the runtime's sticky last error, or the next
    // launch's hipGetLastError (any engine's, on this thread) would report it again
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
}
template <typename T>
static void dfree(T*& p) {
    if (p) hipFree((void*)p);
    p = nullptr;
}
template <typename T>
static hipError_t halloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    return hipHostMalloc((void**)p, sizeof(T) * count, 0);
}
template <typename T>
static void hfree(T*& p) {
    if (p) hipHostFree((void*)p);
    p = nullptr;
}

// Host worker pool for the per-chain loops that run every block (moving each chain's outputs
// into its ring, the batched reads): at tens of thousands of chains one host thread spent tens
// of milliseconds per block there (the real-time capacity was host-bound).  Chains are
// independent, so ranges of them go to the workers; below kParMin items the caller's thread
// does the loop alone.
class HostPool {
  public:
    explicit HostPool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { worker(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // fn(begin, end) over [0, n) in chunks of `chunk`, the caller's thread taking part
    void run(int64_t n, int64_t chunk, const std::function<void(int64_t, int64_t)>& fn) {
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &fn;
            n_ = n;
            chunk_ = std::max<int64_t>(1, chunk);
            next_.store(0);
            busy_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return busy_ == 0; });
        fn_ = nullptr;
    }

  private:
    void work() {
        for (;;) {
            const int64_t b = next_.fetch_add(chunk_);
            if (b >= n_) return;
            (*fn_)(b, std::min(n_, b + chunk_));
        }
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
            {
                std::lock_guard<std::mutex> lk(m_);
                if (--busy_ == 0) done_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int64_t, int64_t)>* fn_ = nullptr;
    std::atomic<int64_t> next_{0};
    int64_t n_ = 0, chunk_ = 1;
    int busy_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};
constexpr int64_t kParMin = 2048;  // per-chain loops shorter than this stay on one thread

struct ByteRing {  // host-side output queue
    std::vector<uint8_t> buf;
    size_t rd = 0;
    size_t cap = 64u << 20;
    int64_t dropped = 0;
    void push(const uint8_t* p, size_t n) {
        if (rd > 0 && rd * 2 >= buf.size()) {
            buf.erase(buf.begin(), buf.begin() + rd);
            rd = 0;
        }
        buf.insert(buf.end(), p, p + n);
        if (buf.size() - rd > cap) {  // overrun: drop oldest
            const size_t drop = buf.size() - rd - cap;
            rd += drop;
            dropped += (int64_t)drop;
        }
    }
    size_t avail() const { return buf.size() - rd; }
    // capacity for n bytes, its pages touched now: at 10^5 chains the rings otherwise grow
    // together (every chain's output is the same size) and one block's drain takes the page
    // faults of hundreds of MB of fresh heap (100-200 ms drains at 196 608 chains)
    void prime(size_t n) {
        if (buf.capacity() >= n) return;
        const size_t keep = buf.size();
        buf.resize(std::max(n, keep));
        buf.resize(keep);
    }
    void clear() {
        buf.clear();
        rd = 0;
    }
    size_t pop(uint8_t* dst, size_t n) {
        n = std::min(n, avail());
        memcpy(dst, buf.data() + rd, n);
        rd += n;
        return n;
    }
};

struct Waterfall {
    int N = 0, logn = 0, hop = 0, avg = 1, adpcm = 0;
    float add_db = -70.0f;
    int new_hop = 0, new_avg = 0, new_adpcm = 0;
    bool pending = false;
    int64_t next_start = 0;  // absolute index of the next frame
    int row_frame = 0;       // frames of the current row already scheduled
    int fpg = 1;             // frames per group (fixed per configuration: rows are bit-stable)
    int batch_min = 0;       // owrx_waterfall_set_batch: launch once this many frames are ready
    int64_t batch_lag = 0;   //   ... or the oldest pending frame is this far behind (0: history)
    double batch_wall_ms = 0;  // owrx_waterfall_set_latency: ... or it would wait longer than this
    double t_pending = -1;     // wall time (ms) of the block call that made the oldest pending frame ready
    // (stream end of a block, wall time of its call) for the blocks whose frames are not all
    // launched: a row's readiness time is the first block that covered its last frame
    std::deque<std::pair<int64_t, double>> blk_times;
    bool carry_valid = false;
    int carry_idx = 0;
    int64_t rows = 0;
    float* d_window = nullptr;
    float2* d_tw = nullptr;
    float* d_partial = nullptr;
    float2* d_y4 = nullptr;  // N > 16384: DIF-split sub-frames (fpg frames per group) or the
                             // four-step scratch (one cf32 frame per group)
    float* d_ones = nullptr; // DIF split: the sub-frames' window (the split applied the frame's)
    int* d_work = nullptr;   // wf_fft_l32's claim + exit counters (left zeroed by each launch)
    int partial_groups = 0;          // groups d_partial / d_groups hold
    WfGroup* h_groups[kSlots] = {};  // pinned copy sources, per slot of the launching block
    WfRow* h_rows[kSlots] = {};
    int h_cap[kSlots] = {};          // groups (and rows) each slot's pinned copy sources hold
    int row_slot_cap[kRowSlots] = {};  // rows each row slot's buffers hold
    float* d_carry[2] = {nullptr, nullptr};
    WfGroup* d_groups = nullptr;
    WfRow* d_rows = nullptr;
    int rows_cap = 0;
    // one set per row slot (kRowSlots blocks of rows in flight)
    int16_t* d_s16[kRowSlots] = {};
    float* d_f32[kRowSlots] = {};
    uint8_t* d_bytes[kRowSlots] = {};
    uint8_t* h_bytes[kRowSlots] = {};
    int pend_rows[kRowSlots] = {};
    int pend_adpcm[kRowSlots] = {};
    // the host buffer each row slot's copies went to: a reconfiguration (wf_reserve) may replace
    // h_bytes[ri] while the slot is in flight, and its drain must read the one the GPU wrote
    uint8_t* pend_h[kRowSlots] = {};
    std::vector<double> pend_t[kRowSlots];  // readiness time of each row in the slot
    ByteRing ring;
    std::vector<WfGroup> groups;
    std::vector<WfRow> rowdesc;
    int64_t row_bytes_for(int adp) const { return adp ? (N + 10) / 2 : 4 * (int64_t)N; }
    int64_t row_bytes() const { return row_bytes_for(adpcm); }
};

struct ChainGroup {
    int D = 0, T = 0, P = 0;
    uint32_t tbw_bits = 0, cutoff_bits = 0;
    float* d_taps = nullptr;
    std::vector<int> members;  // chain handles
    int64_t k_next = 0;
    DdcChain* d_chains = nullptr;
    int chains_cap = 0;
    float2* d_partial[kSlots] = {};  // DDC segment partials, per slot (A writes, B reads)
    size_t partial_elems = 0;
    int nseg = 1;
    DdcChain* h_chains[kSlots] = {};  // pinned copy sources, per slot
    bool chains_stale = true;  // d_chains needs an upload (membership changed, or a retune)
    int h_cap = 0;
    // fast-convolution form (kernels_fcddc.hip): frame length M; 0: direct form only
    int fc_M = 0;
    int fc_P = 0;                 // ceil(T / D), unpadded
    int fc_V = 0;                 // valid outputs per frame, M - P + 1
    int fc_Dp = 0;                // branches padded to a multiple of 96
    int fc_Fs = 0;                // frame stride of U / Y (>= frames of the largest block)
    float* d_h = nullptr;         // linear taps (T)
    float2* d_fc_tw = nullptr;    // M-point twiddles e^{-j 2 pi m / M}
    float2* d_fc_u = nullptr;     // U[M][Fs][Dp] (stream A only)
    float2* d_fc_y = nullptr;     // Y[chains][Fs][M] (stream A only)
    size_t fc_y_elems = 0;
    // filter spectra of every member, W[kappa][slot][Dp] (slot = index in `members`; a
    // destroyed member's slot is refilled by the last member's)
    float2* d_fc_w = nullptr;
    int fc_w_cap = 0;             // slots
    std::vector<FcWJob> w_pending;  // joins' spectra builds not yet launched (flush_uploads)
    int64_t fc_w_ks() const { return (int64_t)fc_w_cap * fc_Dp; }
};

// staging regions start 256-B aligned
static int64_t out_region(int64_t cap) { return (cap + 255) & ~(int64_t)255; }

struct Chain {
    owrx_chain_params prm;
    uint64_t read_mark = 0;  // batched reads: the call that listed it last (duplicate check)
    ChainGroup* group = nullptr;
    int64_t origin = 0;   // absolute sample index of chain sample 0
    int64_t k_first = 0;  // absolute output index of chain output 0
    // shift phase model: phase(n) = P0 + (n - n0 + 1) * rate
    uint64_t rate_fx = 0;
    uint64_t P0 = 0;
    int64_t n0 = 0;
    float rate = 0.0f;
    bool rate_pending = false;
    float new_rate = 0.0f;
    // device
    ChainStateP* d_pstate = nullptr;
    ChainStateS* d_sstate = nullptr;
    float2* d_ddc = nullptr;
    float2* d_fd = nullptr;
    float2* d_sq = nullptr;
    float* d_dem[kSlots] = {};
    int16_t* d_s16[kSlots] = {};  // ADPCM encoder input, per slot (B -> C)
    float2* d_bp_taps = nullptr;
    int bp_ntaps = 0;
    int bp_hist = kBpHist;      // fd_buf history; > kBpHist => long bandpass (bp_long kernel)
    int bp_design_taps = 0;     // taps of the chain's bandpass design (bp_transition)
    // WFM audio decimator (OWRX_DEMOD_WFM)
    float* d_wf = nullptr;
    float* d_pf = nullptr;
    float* d_pf_taps = nullptr;
    int pf_ntaps = 0;
    // NoiseFilter (nr_enabled); buffers allocated on first enable, zeroed on (re)start
    NrState* d_nr_state = nullptr;
    float* d_nr_in = nullptr;
    float* d_nr_pow = nullptr;
    float* d_nr_ola = nullptr;
    bool nr_reset = false;
    int64_t cap = 0;      // per-step sample capacity of stage buffers
    int64_t out_cap = 0;  // staging bytes per step
    int sm_cap = 0;
    ByteRing audio;
    ByteRing smeter;
    ByteRing dbg[kDebugStages];
    // secondary FFT (FftChain on the Selector output, owrx/dsp.py:220-225); sf_n == 0: none
    int sf_n = 0, sf_logn = 0, sf_hop = 0, sf_avg = 1, sf_adpcm = 0;
    float sf_add_db = -70.0f;
    bool sf_reset = false;
    float2* d_sf = nullptr;      // [sf_n + scap]
    float* d_sf_acc = nullptr;   // [sf_n]
    float* d_sf_window = nullptr;
    float2* d_sf_tw = nullptr;
    int64_t sf_out_cap = 0;      // staging bytes per step
    ByteRing sfft;
    // taps for secondary readers (owrx/dsp.py:185-206): selectorBuffer (cf32 after Squelch)
    // and audioBuffer (f32 demodulator-chain output); staging bytes per step, 0 = off
    int64_t tap_sq_cap = 0, tap_agc_cap = 0;
    ByteRing tap_sel, tap_audio;
    int64_t ring_dropped() const {
        return audio.dropped + smeter.dropped + sfft.dropped + tap_sel.dropped + tap_audio.dropped;
    }
    // bumped by owrx_chain_set_secondary_fft / owrx_chain_set_taps: blocks built before the
    // change (still in flight, they are not drained) deliver no rows / tap bytes afterwards
    uint32_t sf_gen = 0, tap_gen = 0;
    int64_t tap_bytes() const { return out_region(tap_sq_cap) + out_region(tap_agc_cap); }
    int64_t sf_row_bytes() const { return sf_adpcm ? (sf_n + 10) / 2 : 4 * (int64_t)sf_n; }
    // bytes of this chain's output region in a slot's staging (audio, secondary FFT, taps)
    int64_t staging_bytes() const { return out_region(out_cap) + out_region(sf_out_cap) + tap_bytes(); }
};

// A post's staging layout as built (drain_slot reads the block with the layout it was built
// with, whatever the chain's configuration is by then)
struct PostLayout {
    int64_t out_cap, sf_cap, tsq_cap, tagc_cap;
    uint32_t sf_gen, tap_gen;
};

// one descriptor upload of copy_jobs (process_block)
struct CopyJob {
    void* dst;
    const void* src;
    int64_t bytes;
};
constexpr int kMaxCopyJobs = 64;

struct Slot {  // one block's outputs in flight on streams B / C
    bool chains_pending = false;
    std::vector<int> post_ids;
    std::vector<int64_t> out_off;  // per post: byte offset of its output region
    std::vector<PostLayout> layout;
    bool debug = false;
    ChainPost* d_posts = nullptr;
    ChainPost* h_posts = nullptr;
    int* d_sel = nullptr;   // post indices grouped by output mode, then long-bandpass posts
    int* h_sel = nullptr;
    int long_off = 0;
    int afc_off = 0, nafc = 0;  // chain_afc's lane list (SAm chains) in d_sel
    ChainCounts* d_counts = nullptr;
    ChainCounts* h_counts = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* h_out = nullptr;
    float* d_sm = nullptr;
    float* h_sm = nullptr;
    uint8_t* d_dbg = nullptr;
    uint8_t* h_dbg = nullptr;
    hipEvent_t evA = nullptr;   // stream A finished this block's post_parallel
    hipEvent_t evF = nullptr;   // stream B finished this block's post_serial_front
    hipEvent_t evC = nullptr;   // stream C finished this block's encoder
    hipEvent_t evB = nullptr;   // stream R finished (audio copied to host)
    // timing brackets: A: [a0 waterfall + descriptors a1 DDC kernels a2 .. a3];
    // B/C: [b0 post_parallel, post_serial_front .. chain_adpcm b1]
    hipEvent_t a0 = nullptr, a1 = nullptr, a2 = nullptr, a3 = nullptr;
    hipEvent_t m0 = nullptr, m1 = nullptr;  // around the fast-convolution DDC's GEMM (fc_mac)
    bool timed_mac = false;
    hipEvent_t b0 = nullptr, b1 = nullptr;
    hipEvent_t w0 = nullptr, w1 = nullptr;  // around the waterfall FFT + finalize launches
    bool timed = false;
    bool timed_wf = false;
    bool timed_wff = false;
    // the slot's chain descriptors (h_posts, lane lists) as last built: rebuilt only when the
    // engine's chain epoch moved, the set of groups with outputs changed, or a one-shot reset
    // (NoiseFilter / secondary FFT) was carried; per block only nk / k_begin are patched
    uint64_t post_epoch = ~0ull;
    bool post_dirty = true;
    bool dev_stale = true;  // h_posts / h_sel rebuilt since the slot's device copy was made
    std::vector<const ChainGroup*> post_groups;
    std::vector<int> group_post0;  // first post of each group of post_groups
    int np = 0, nlong = 0, long_taps = 0, nfill = 0;
    int64_t long_fd = 0;
    uint32_t sf_sizes = 0;  // secondary FFT sizes (log2 bit set)
    bool any_nr = false;
    int nsel[3][2] = {}, off[3][2] = {};
    CopyJob* h_jobs = nullptr;  // pinned job table of copy_jobs
};

struct RowSlot {  // one block's waterfall rows being encoded / copied on stream R
    hipStream_t stream = nullptr;  // the row queue (W CUs), shared by the row slots
    hipEvent_t evWf = nullptr;  // stream A finished the block's finalize
    hipEvent_t evC = nullptr;   // rows copied to host
    bool pending = false;
    bool shared_stream = false;  // another row slot's stream (one row queue by default)
};


// Ingest conversion (owrx/source/direct.py:51-71): cs16 -> cf32 * gain straight into the engine
// window.  Two samples (8 B in, 16 B out) per thread, coalesced: HBM-bound at 12 B per sample.
__global__ void __launch_bounds__(256)
ingest_cs16(const int16_t* __restrict__ in, int64_t nsamples, float gain, float* __restrict__ out) {
    const int64_t pair = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t s0 = 2 * pair;
    if (s0 + 1 < nsamples) {
        const short4 v = *reinterpret_cast<const short4*>(in + 2 * s0);
        float4 o;
        o.x = gain_step(s16_to_f32(v.x), gain);
        o.y = gain_step(s16_to_f32(v.y), gain);
        o.z = gain_step(s16_to_f32(v.z), gain);
        o.w = gain_step(s16_to_f32(v.w), gain);
        *reinterpret_cast<float4*>(out + 2 * s0) = o;
    } else if (s0 < nsamples) {
        out[2 * s0] = gain_step(s16_to_f32(in[2 * s0]), gain);
        out[2 * s0 + 1] = gain_step(s16_to_f32(in[2 * s0 + 1]), gain);
    }
}

// Per-block host <-> device transfers run as kernels on the stream that owns them, reading or
// writing the pinned (GPU-mapped) host buffers directly.  hipMemcpyAsync of the same buffers
// shares the copy engines between streams: a 115 KB descriptor upload on stream A measured
// ~1.1 ms behind the other streams' output downloads (C3, 256 chains); as kernels they take a
// few microseconds and stay in their stream's order.
template <typename V>
__global__ void __launch_bounds__(256)
copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t n) {
    constexpr int W = sizeof(V);
    const int64_t nv = n / W;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv;
         i += (int64_t)gridDim.x * blockDim.x)
        reinterpret_cast<V*>(dst)[i] = reinterpret_cast<const V*>(src)[i];
    const int64_t t = nv * W + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && t < n) dst[t] = src[t];
}

// One block's descriptor uploads in one launch: job y copies its bytes (16 B per lane where
// both ends are 16-B aligned) from pinned host memory to the device.
__global__ void __launch_bounds__(256)
copy_jobs(const CopyJob* __restrict__ jobs) {
    const CopyJob j = jobs[blockIdx.y];
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if ((((uintptr_t)j.dst | (uintptr_t)j.src) & 15) == 0) {
        const int64_t n16 = j.bytes >> 4;
        for (int64_t i = t0; i < n16; i += stride)
            reinterpret_cast<uint4*>(j.dst)[i] = reinterpret_cast<const uint4*>(j.src)[i];
        for (int64_t i = (n16 << 4) + t0; i < j.bytes; i += stride)
            static_cast<uint8_t*>(j.dst)[i] = static_cast<const uint8_t*>(j.src)[i];
    } else {
        for (int64_t i = t0; i < j.bytes; i += stride)
            static_cast<uint8_t*>(j.dst)[i] = static_cast<const uint8_t*>(j.src)[i];
    }
}

// Zeroing of newly taken pool buffers, all of them in one launch: job y (read from the pinned
// upload ring) zeroes its bytes, 16 B per lane (pool sizes are multiples of 256 B).  One
// hipMemsetAsync per buffer was 21 972 fillBufferAligned dispatches in a C3 bench profile, a
// quarter of its GPU time, and 13-20 s of setup for 98 304-131 072 chains.
struct ZeroJob {
    void* dst;
    int64_t bytes;
};
__global__ void __launch_bounds__(256)
zero_jobs(const ZeroJob* __restrict__ jobs) {
    const ZeroJob j = jobs[blockIdx.y];
    const int64_t n16 = j.bytes >> 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (int64_t)gridDim.x * blockDim.x)
        reinterpret_cast<uint4*>(j.dst)[i] = make_uint4(0u, 0u, 0u, 0u);
}

static hipError_t kcopy(void* dst, const void* src, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const bool v16 = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
    const bool v4 = (((uintptr_t)dst | (uintptr_t)src) & 3) == 0;
    const int64_t nv = (int64_t)(n / (v16 ? 16 : v4 ? 4 : 1));
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(256, (nv + 255) / 256));
    if (v16)
        hipLaunchKernelGGL(copy_bytes<uint4>, dim3(blocks), dim3(256), 0, st, (uint8_t*)dst,
                           (const uint8_t*)src, (int64_t)n);
    else if (v4)
        hipLaunchKernelGGL(copy_bytes<uint32_t>, dim3(blocks), dim3(256), 0, st, (uint8_t*)dst,
                           (const uint8_t*)src, (int64_t)n);
    else
        hipLaunchKernelGGL(copy_bytes<uint8_t>, dim3(blocks), dim3(256), 0, st, (uint8_t*)dst,
                           (const uint8_t*)src, (int64_t)n);
    return hipGetLastError();
}

// One block's chain outputs to the pinned host staging, only what each chain produced: its
// counts record, its audio bytes, its secondary FFT bytes and its s-meter values (the staging
// regions are sized for the worst case: copying them whole moved ~10x the produced bytes).
__global__ void __launch_bounds__(256)
gather_outputs(const ChainPost* __restrict__ posts, const ChainCounts* __restrict__ counts,
               const uint8_t* __restrict__ d_out, uint8_t* __restrict__ h_out,
               const float* __restrict__ d_sm, float* __restrict__ h_sm, int sm_stride,
               ChainCounts* __restrict__ h_counts) {
    const int k = blockIdx.x;
    const ChainPost& p = posts[k];
    const ChainCounts c = counts[k];
    if (threadIdx.x == 0) h_counts[k] = c;
    auto move = [&](const uint8_t* src, int64_t n) {
        uint8_t* dst = h_out + (src - d_out);
        const int64_t nv = n >> 4;  // regions start 256-B aligned
        for (int64_t i = threadIdx.x; i < nv; i += blockDim.x)
            reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
        for (int64_t i = (nv << 4) + threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    };
    move(p.out, c.out_bytes < p.out_cap ? c.out_bytes : p.out_cap);
    if (p.sf_out && c.sf_bytes > 0) move(p.sf_out, c.sf_bytes < p.sf_out_cap ? c.sf_bytes : p.sf_out_cap);
    if (p.tap_sq) move((const uint8_t*)p.tap_sq, 8 * (c.n_gate < p.tap_sq_cap ? c.n_gate : p.tap_sq_cap));
    if (p.tap_agc)
        move((const uint8_t*)p.tap_agc, 4 * (c.n_front < p.tap_agc_cap ? c.n_front : p.tap_agc_cap));
    const int ns = c.smeter < sm_stride ? c.smeter : sm_stride;
    for (int i = threadIdx.x; i < ns; i += blockDim.x)
        h_sm[(int64_t)k * sm_stride + i] = d_sm[(int64_t)k * sm_stride + i];
}

}  // namespace owrx

using namespace owrx;

// One group's DDC work in a block (process_block)
struct GroupWork {
    ChainGroup* g;
    int64_t k_end;
    int nk;
    bool fast;
    FcSubs sub;  // the caller blocks' outputs and input ends (one block: n = 1)
};

struct owrx_engine {
    int device = 0;
    // A: waterfall FFT + DDC + post_parallel; B: post_serial_front; C: ADPCM; R: output
    // gathers + copies; the row slots' queue: waterfall row encoding + copies.  Each is a
    // CU-masked HSA queue of its own (none serialise on a shared queue); create_streams orders
    // them so A, B and C each have a CP pipe to themselves.
    hipStream_t sA = nullptr, sB = nullptr, sC = nullptr, sR = nullptr;
    // unmasked twins of B and C: past kWideSerialChains chains the serial kernels are
    // throughput-bound on their few CUs and spread over the chip instead (serial_wide)
    hipStream_t sBw = nullptr, sCw = nullptr;
    bool serial_wide = false;
    std::vector<int> sel_buckets[3][2][4];  // per-block scratch of the serial lane lists
    double samp_rate = 0;
    int64_t max_block = 0;
    int cus_a = 0;  // CUs of stream A (DDC launch shape)
    int rows_grid = 0;  // the row encoder's grid (2 x the row queue's CUs; 0: one per row)
    std::vector<float> wf_ms_log;  // timed waterfall launches (OWRX_WF_LOG=1: printed at destroy)
    // host time of the slot drains (OWRX_HOST_LOG=1: printed at destroy): the wait for the
    // block's stream-R event and the ring pushes, split by forced (process_block's slot reuse)
    // and opportunistic (the collect after each block)
    double hl_wait[2] = {}, hl_push[2] = {};
    // host time of owrx_chain_create by section (OWRX_HOST_LOG=1: printed at destroy):
    // setup, buffers + state uploads, bandpass taps, W reserve + build, group refresh, staging
    double cc_ms[6] = {};
    int64_t hl_n[2] = {};
    int64_t ring_dropped = 0;  // bytes the chains' host rings dropped (oldest first), all time
    bool hl_forced = false;
    int64_t history = kDefaultHistory;
    int64_t pos = 0;  // absolute samples processed
    int64_t block_index = 0;
    int64_t slot_tail = 0;  // oldest block whose outputs are not yet in the host rings
    bool failed = false;
    bool stalled = false;            // a bounded wait expired (owrx_set_stall_timeout)
    double t_block = 0;              // wall time (ms) of the current block call
    double t_last_block = -1;        // ... of the previous one
    double block_interval_ms = 0;    // running estimate of the interval between block calls
    int64_t stall_ms = 20000;        // the longest any host-side wait blocks before failing
    hipEvent_t evSync = nullptr;     // marker for bounded stream synchronisation
    hipEvent_t evExt = nullptr;      // owrx_wait_stream: the caller's stream position
    std::unique_ptr<HostPool> pool;  // host workers for per-chain loops (created on first use)
    bool debug = false;
    int timing = 0;                  // timing events every `timing` blocks (0: off)
    std::vector<GroupWork> work;     // per-block scratch: the groups with outputs
    std::vector<Chain*> nr_resets;   // NoiseFilter states to zero before the next serial work
    uint64_t chain_epoch = 0;        // bumped by every change of a chain's post descriptor
    uint64_t read_epoch = 0;         // bumped by every batched read (Chain::read_mark)
    int ddc_mode = OWRX_DDC_FAST;
    std::recursive_mutex mu;
    // push-path ring: blocks are appended at wp with `history` samples before them; when the
    // next block does not fit, the last `history` samples move to the start (once per lap)
    float2* d_ring = nullptr;
    int64_t ring_cap = 0, wp = 0;
    // the newest block's window (the waterfall flush at owrx_sync launches pending frames on it)
    const float2* last_blk = nullptr;
    int64_t last_start = 0, last_end = 0;
    float* h_in = nullptr;  // pinned staging for push_iq, two blocks (per block parity)
    int16_t* d_cs16 = nullptr;  // device staging of cs16 ingest (allocated on first use)
    // end of a block's stream-A work (its input and parity-indexed host descriptors reusable),
    // (evIn[k % kInEv] for block k); in_done: the newest block known to have finished it;
    // retention: blocks the caller keeps each input valid for (owrx_set_input_retention)
    hipEvent_t evIn[kInEv] = {};
    int64_t in_done = -1;
    int retention = 1;
    // block grouping (owrx_set_block_group; pairs: owrx_set_block_pairing): caller blocks held
    // until `group` contiguous ones arrived, then run as one engine block (pend_k held blocks from
    // pend_blk, pend_n[] samples each, pend_total in all; 0 = none)
    int group = 1;
    const float2* pend_blk = nullptr;
    int pend_k = 0;
    int64_t pend_n[kMaxSubBlocks] = {};
    int64_t pend_total = 0;
    // blocks of chain work in flight (owrx_set_pipeline_depth, <= kSlots): every slot holds
    // pinned and device staging for all chains, so the depth is the caller's memory trade
    int nslots = kDefaultSlots;
    std::map<int, std::unique_ptr<Waterfall>> wfs;
    // hashed: the per-block loops and the batched reads look every chain up (a tree of 65 536
    // chains costs ~16 cache misses per lookup)
    std::unordered_map<int, std::unique_ptr<Chain>> chains;
    std::vector<std::unique_ptr<ChainGroup>> groups;
    int next_handle = 1;
    // post staging (all chains), per block parity
    int post_cap = 0;
    int64_t out_total = 0, sm_stride = 0, dbg_stride = 0;  // out: sum of per-chain regions
    Slot slots[kSlots];
    RowSlot rslots[kRowSlots];
    int64_t row_head = 0;  // next row slot to fill
    int64_t row_tail = 0;  // oldest row slot not yet drained
    std::vector<ChainPost> posts;
    owrx_stats stats;
    float* d_nr_win = nullptr;    // NoiseFilter window and twiddles (shared by all chains)
    float2* d_nr_tw = nullptr;
    // Live reconfiguration without a drain (client join / leave, setBandpass, taps, secondary
    // FFT while other clients stream): chain buffers come from exact-size free lists, so joins
    // and leaves call neither hipMalloc nor hipFree (which synchronises the device) once warm;
    // a released buffer is parked until every block that may still read it has drained
    // (slot_tail >= the block index at its release); new buffers are zeroed and initial states
    // and taps uploaded on stream A, ordered before the first block that uses them.
    std::unordered_map<size_t, std::vector<void*>> pool_free;
    std::unordered_map<void*, size_t> pool_size;  // every pool buffer and its size class
    // small pool buffers are carved from slabs (palloc): a fresh engine creating 98 304 chains
    // made ~2 M hipMalloc calls, one per chain buffer; slabs and direct allocations are what
    // destroy frees (carved buffers live inside a slab)
    std::vector<void*> slabs;
    std::unordered_set<void*> pool_carved;
    char* slab_cur = nullptr;
    size_t slab_left = 0;
    struct Retired {
        int64_t block;
        void* p;
    };
    std::vector<Retired> pool_retired;
    // pinned host buffers (waterfall copy sources and row destinations): an exact-size pool,
    // released by block (stream-A copy sources) or by row slot (stream-R destinations)
    std::unordered_map<size_t, std::vector<void*>> hpool_free;
    std::unordered_map<void*, size_t> hpool_size;
    std::vector<Retired> hpool_retired;
    struct RowRetired {
        int64_t row;  // free once row_tail reaches this
        void* p;
        bool pinned;
    };
    std::vector<RowRetired> row_retired;
    uint8_t* h_up = nullptr;  // pinned staging of those uploads (a ring; wraps after stream A)
    size_t up_cap = 0, up_head = 0;
    std::vector<ZeroJob> zero_pending;  // pool buffers taken but not yet zeroed (flush_zero)
    // uploads not yet enqueued (upload()): their bytes, 16-B aligned, and (dst, offset, size)
    // records; flush_uploads() copies them into the pinned ring and launches one copy_jobs
    std::vector<uint8_t> up_data;
    std::vector<CopyJob> up_jobs;  // src = offset into up_data until the flush
    std::unordered_map<void*, size_t> up_index;  // dst -> its pending job (latest bytes win)
    // post staging needs of the current chains (kept as chains come and go)
    int64_t need_out = 256, need_sm = 4, need_dbg = 64;
};

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// fn(begin, end) over [0, n): on the engine's host workers when n is large, else inline
static void for_range(owrx_engine* e, int64_t n, const std::function<void(int64_t, int64_t)>& fn);

// Bounded waits.  The reference turns a source that stops producing into fail() -> every
// client's onFail (owrx/source/__init__.py:432-448, owrx/connection.py:292-295); here a GPU
// that stops completing work must do the same instead of blocking the OpenWebRX process in a
// HIP synchronisation call forever.  Every host-side wait polls its event against a deadline
// (e->stall_ms); an expired wait marks the engine failed (`stalled`) and returns
// OWRX_ETIMEDOUT, which the pycsdr shim turns into FAILED and ended outputs.
static int wait_ev(owrx_engine* e, hipEvent_t ev) {
    hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return OWRX_OK;
    const auto t0 = std::chrono::steady_clock::now();
    int polls = 0;
    while (q == hipErrorNotReady) {
        const double ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms > (double)e->stall_ms) {
            e->failed = true;
            e->stalled = true;
            set_last_error("GPU stalled: no progress for %lld ms (owrx_set_stall_timeout)",
                           (long long)e->stall_ms);
            return OWRX_ETIMEDOUT;
        }
        // spin briefly (a block's tail is typically tens of microseconds), then sleep
        if (++polls > 64) std::this_thread::sleep_for(std::chrono::microseconds(polls > 4096 ? 200 : 20));
        q = hipEventQuery(ev);
    }
    HIPCHK(q);
    return OWRX_OK;
}

static void for_range(owrx_engine* e, int64_t n, const std::function<void(int64_t, int64_t)>& fn) {
    if (n < kParMin) {
        fn(0, n);
        return;
    }
    if (!e->pool) {
        const unsigned hw = std::thread::hardware_concurrency();
        // OWRX_HOST_THREADS: workers besides the caller (default: up to 7, fewer on small hosts)
        int nt = (int)std::min(7u, hw > 1 ? hw - 1 : 1u);
        if (const char* v = getenv("OWRX_HOST_THREADS")) nt = std::max(0, atoi(v));
        e->pool = std::make_unique<HostPool>(nt);
    }
    e->pool->run(n, 1024, fn);
}

// everything enqueued on `st` so far, within the stall bound
static int sync_stream(owrx_engine* e, hipStream_t st) {
    HIPCHK(hipEventRecord(e->evSync, st));
    return wait_ev(e, e->evSync);
}

// the largest engine block: two caller blocks when pairing
static int64_t proc_block(const owrx_engine* e) { return (int64_t)e->group * e->max_block; }

static int64_t chain_stage_cap(const owrx_engine* e, int D, double frac) {
    int64_t nk = proc_block(e) / D + 4;
    if (frac > 0 && frac < 1.0) nk = (int64_t)std::ceil(nk / frac) + 4;
    return nk;
}

// pool allocation (see owrx_engine): zeroed on stream A.  Buffers up to kCarveMax come from
// kSlabBytes slabs (256-B aligned offsets), larger ones from hipMalloc.
constexpr size_t kCarveMax = 256u << 10;
constexpr size_t kSlabBytes = 64u << 20;
template <typename T>
static hipError_t palloc(owrx_engine* e, T** p, size_t count) {
    *p = nullptr;
    const size_t bytes = (sizeof(T) * std::max<size_t>(count, 1) + 255) & ~(size_t)255;
    void* q = nullptr;
    auto it = e->pool_free.find(bytes);
    if (it != e->pool_free.end() && !it->second.empty()) {
        q = it->second.back();
        it->second.pop_back();
    } else if (bytes <= kCarveMax) {
        if (e->slab_left < bytes) {
            void* sl = nullptr;
            const hipError_t r = hipMalloc(&sl, kSlabBytes);
            if (r != hipSuccess) {
                (void)hipGetLastError();
                return r;
            }
            e->slabs.push_back(sl);
            e->slab_cur = static_cast<char*>(sl);
            e->slab_left = kSlabBytes;
            e->stats.pool_allocs++;
        }
        q = e->slab_cur;
        e->slab_cur += bytes;
        e->slab_left -= bytes;
        e->pool_size[q] = bytes;
        e->pool_carved.insert(q);
    } else {
        const hipError_t r = hipMalloc(&q, bytes);
        if (r != hipSuccess) {
            (void)hipGetLastError();  // not sticky for the next launch (see dalloc)
            return r;
        }
        e->pool_size[q] = bytes;
        e->stats.pool_allocs++;
    }
    *p = static_cast<T*>(q);
    e->zero_pending.push_back({q, (int64_t)bytes});  // zeroed on stream A by flush_zero
    return hipSuccess;
}

static int flush_uploads(owrx_engine* e);

// release to the pool once the blocks enqueued so far have drained.  Pending uploads are
// enqueued first: one may target this buffer, and its next owner's zeroing and upload must run
// after it (copy_jobs does not order jobs to the same destination within a launch).
// A failed flush (a timed-out staging wait, no pinned memory) leaves its uploads and zeroing
// queued; one of them may target the buffer being released, which the pool then hands to another
// chain, so the later flush would write stale bytes over that chain's fresh state.  The queued
// work is dropped instead and the engine fails (every later call returns the error).
static void flush_before_release(owrx_engine* e) {
    if (e->up_jobs.empty()) return;
    if (flush_uploads(e) != OWRX_OK) {
        e->up_jobs.clear();
        e->up_data.clear();
        e->up_index.clear();
        e->zero_pending.clear();
        e->failed = true;
    }
}

template <typename T>
static void prel(owrx_engine* e, T*& p) {
    if (p) flush_before_release(e);
    if (p) e->pool_retired.push_back({e->block_index, (void*)p});
    p = nullptr;
}

template <typename T>
static hipError_t hpalloc(owrx_engine* e, T** p, size_t count) {
    *p = nullptr;
    const size_t bytes = (sizeof(T) * std::max<size_t>(count, 1) + 255) & ~(size_t)255;
    auto it = e->hpool_free.find(bytes);
    if (it != e->hpool_free.end() && !it->second.empty()) {
        *p = static_cast<T*>(it->second.back());
        it->second.pop_back();
        return hipSuccess;
    }
    void* q = nullptr;
    const hipError_t r = hipHostMalloc(&q, bytes, 0);
    if (r != hipSuccess) {
        (void)hipGetLastError();
        return r;
    }
    e->hpool_size[q] = bytes;
    e->stats.pool_allocs++;
    *p = static_cast<T*>(q);
    return hipSuccess;
}
// pinned / device buffers back to their pools: now (nothing can use them), after the blocks
// enqueued so far drained, or after the row slots enqueued so far drained
template <typename T>
static void hprel_now(owrx_engine* e, T*& p) {
    if (p) e->hpool_free[e->hpool_size[(void*)p]].push_back((void*)p);
    p = nullptr;
}
template <typename T>
static void prel_now(owrx_engine* e, T*& p) {
    if (p) flush_before_release(e);  // (see prel)
    if (p) e->pool_free[e->pool_size[(void*)p]].push_back((void*)p);
    p = nullptr;
}
template <typename T>
static void hprel(owrx_engine* e, T*& p) {
    if (p) e->hpool_retired.push_back({e->block_index, (void*)p});
    p = nullptr;
}
template <typename T>
static void rowrel(owrx_engine* e, T*& p, bool pinned) {
    if (p) e->row_retired.push_back({e->row_head, (void*)p, pinned});
    p = nullptr;
}

// Has stream A finished block j's work?  Non-blocking: evIn[j % kInEv] holds block j or a later
// block (stream order: a later block done implies j done).
static bool stream_a_done(owrx_engine* e, int64_t j) {
    if (j <= e->in_done || j < 0) return true;
    if (hipEventQuery(e->evIn[j % kInEv]) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    e->in_done = std::max(e->in_done, j);
    return true;
}

static void pool_collect(owrx_engine* e) {
    size_t k = 0;
    for (const auto& r : e->pool_retired) {
        if (r.block <= e->slot_tail)
            e->pool_free[e->pool_size[r.p]].push_back(r.p);
        else
            e->pool_retired[k++] = r;
    }
    e->pool_retired.resize(k);
    k = 0;
    // pinned copy sources (the waterfall's group / row descriptors) are read by stream-A kernel
    // copies of the blocks before r.block.  A drained slot does not prove that: a block with no
    // chain outputs and no timing drains without waiting for any event, so slot_tail can pass
    // blocks whose stream-A copies have not run yet, and a host memcpy into the reused buffer is
    // not stream-ordered.  So these wait for stream A itself (or an owrx_sync drain, which syncs
    // it and sets in_done).
    for (const auto& r : e->hpool_retired) {
        if (r.block <= e->slot_tail && stream_a_done(e, r.block - 1))
            e->hpool_free[e->hpool_size[r.p]].push_back(r.p);
        else
            e->hpool_retired[k++] = r;
    }
    e->hpool_retired.resize(k);
}

static void row_collect(owrx_engine* e) {
    size_t k = 0;
    for (const auto& r : e->row_retired) {
        if (r.row <= e->row_tail) {
            if (r.pinned) e->hpool_free[e->hpool_size[r.p]].push_back(r.p);
            else e->pool_free[e->pool_size[r.p]].push_back(r.p);
        } else {
            e->row_retired[k++] = r;
        }
    }
    e->row_retired.resize(k);
}

// n bytes from the host to device memory on stream A, through the pinned upload ring: the
// caller's buffer is free on return, and the copy runs before any later stream-A work
// n bytes of the pinned upload ring for a stream-A consumer enqueued right after
static int ring_take(owrx_engine* e, size_t n, uint8_t** h) {
    const size_t a = (n + 255) & ~(size_t)255;
    if (a > e->up_cap) {
        if (e->h_up) RCCHK(sync_stream(e, e->sA));
        hfree(e->h_up);
        e->up_cap = std::max<size_t>(4u << 20, a);
        HIPCHK(halloc(&e->h_up, e->up_cap));
        e->up_head = 0;
    }
    if (e->up_head + a > e->up_cap) {  // wrap: the ring's earlier copies must have run
        RCCHK(sync_stream(e, e->sA));
        e->up_head = 0;
    }
    *h = e->h_up + e->up_head;
    e->up_head += a;
    return OWRX_OK;
}

// Zero every pool buffer taken since the last flush, in one launch on stream A.  Called before
// any stream-A work that may touch them: uploads (initial states), the filter-spectra builds and
// moves, and each block.
static int flush_zero(owrx_engine* e) {
    while (!e->zero_pending.empty()) {
        const size_t nj = std::min<size_t>(e->zero_pending.size(), 65535);
        uint8_t* h = nullptr;
        RCCHK(ring_take(e, sizeof(ZeroJob) * nj, &h));
        memcpy(h, e->zero_pending.data(), sizeof(ZeroJob) * nj);
        int64_t most = 0;
        for (size_t i = 0; i < nj; ++i) most = std::max(most, e->zero_pending[i].bytes);
        const int gx = (int)std::max<int64_t>(1, std::min<int64_t>(64, (most / 16 + 255) / 256));
        hipLaunchKernelGGL(zero_jobs, dim3(gx, (unsigned)nj), dim3(256), 0, e->sA,
                           reinterpret_cast<const ZeroJob*>(h));
        HIPCHK(hipGetLastError());
        e->zero_pending.erase(e->zero_pending.begin(), e->zero_pending.begin() + nj);
    }
    return OWRX_OK;
}

// Device buffer zeroed on stream A with the other pending zeroing (one zero_jobs launch) instead
// of dalloc's synchronous hipMemset (a fillBufferAligned dispatch per buffer): for the slot and
// group buffers that capacity growth reallocates between blocks, after a drain.  The caller
// flushes the zeroing before anything can free the buffer again (flush_zero).
template <typename T>
static hipError_t dalloc_z(owrx_engine* e, T** p, size_t count) {
    *p = nullptr;
    const size_t bytes = (sizeof(T) * std::max<size_t>(count, 1) + 255) & ~(size_t)255;
    const hipError_t r = hipMalloc((void**)p, bytes);
    if (r != hipSuccess) {
        (void)hipGetLastError();  // not sticky for the next launch (see dalloc)
        *p = nullptr;
        return r;
    }
    e->zero_pending.push_back({(void*)*p, (int64_t)bytes});
    return hipSuccess;
}

// The filter-spectra builds of the chains that joined since the last flush, one launch per
// group (W is zeroed by fc_reserve before any build writes it).  Before anything that copies or
// moves W rows (fc_reserve's regrowth, a leave's swap-remove) and with every upload flush.
static int flush_wbuilds(owrx_engine* e) {
    for (auto& gp : e->groups) {
        ChainGroup* g = gp.get();
        size_t j0 = 0;
        while (j0 < g->w_pending.size()) {
            const size_t nj = std::min<size_t>(g->w_pending.size() - j0, 65535);
            uint8_t* h = nullptr;
            RCCHK(ring_take(e, sizeof(FcWJob) * nj, &h));
            memcpy(h, g->w_pending.data() + j0, sizeof(FcWJob) * nj);
            HIPCHK(launch_fc_make_w_jobs(g->fc_M, g->d_h, g->T, g->D, g->fc_Dp, g->fc_P,
                                         reinterpret_cast<const FcWJob*>(h), (int)nj, g->d_fc_w,
                                         g->fc_w_ks(), e->sA));
            j0 += nj;
        }
        g->w_pending.clear();
    }
    return OWRX_OK;
}

// Enqueue every pending upload on stream A: the pool buffers' zeroing first (a buffer's initial
// state is uploaded after it was zeroed), then one copy_jobs launch for all the uploads, their
// bytes and job table in one take of the pinned ring.  Called before any stream-A work that may
// read an uploaded buffer (each block, owrx_sync), and by upload() past kUpFlushBytes.
constexpr size_t kUpFlushBytes = 4u << 20;
static int flush_uploads(owrx_engine* e) {
    RCCHK(flush_zero(e));
    size_t j0 = 0;
    while (j0 < e->up_jobs.size()) {
        const size_t nj = std::min<size_t>(e->up_jobs.size() - j0, 65535);
        const size_t tab = (sizeof(CopyJob) * nj + 255) & ~(size_t)255;
        const size_t lo = (size_t)(intptr_t)e->up_jobs[j0].src;
        const CopyJob& last = e->up_jobs[j0 + nj - 1];
        const size_t hi = (size_t)(intptr_t)last.src + (size_t)last.bytes;
        uint8_t* h = nullptr;
        RCCHK(ring_take(e, tab + (hi - lo), &h));
        memcpy(h + tab, e->up_data.data() + lo, hi - lo);
        CopyJob* t = reinterpret_cast<CopyJob*>(h);
        int64_t most = 0;
        for (size_t i = 0; i < nj; ++i) {
            const CopyJob& u = e->up_jobs[j0 + i];
            t[i] = CopyJob{u.dst, h + tab + ((size_t)(intptr_t)u.src - lo), u.bytes};
            most = std::max(most, u.bytes);
        }
        hipLaunchKernelGGL(copy_jobs, dim3((unsigned)std::min<int64_t>(64, (most + 4095) / 4096), (unsigned)nj),
                           dim3(256), 0, e->sA, t);
        HIPCHK(hipGetLastError());
        j0 += nj;
    }
    e->up_jobs.clear();
    e->up_data.clear();
    e->up_index.clear();
    return flush_wbuilds(e);
}

// Host bytes -> device buffer on stream A, ordered before the next block (or flush_uploads).
// Chain joins upload their initial states this way: batched, ~no HIP calls per join.
static int upload(owrx_engine* e, void* dst, const void* src, size_t n) {
    if (n == 0) return OWRX_OK;
    // a second upload to a pending destination (setBandpass twice between blocks) replaces the
    // first one's bytes: one copy_jobs launch does not order two jobs on the same destination
    const auto hit = e->up_index.find(dst);
    if (hit != e->up_index.end()) {
        const CopyJob& j = e->up_jobs[hit->second];
        if ((size_t)j.bytes == n) {
            memcpy(e->up_data.data() + (size_t)(intptr_t)j.src, src, n);
            return OWRX_OK;
        }
        RCCHK(flush_uploads(e));
    }
    const size_t off = (e->up_data.size() + 15) & ~(size_t)15;
    e->up_data.resize(off + n);
    memcpy(e->up_data.data() + off, src, n);
    e->up_index[dst] = e->up_jobs.size();
    e->up_jobs.push_back(CopyJob{dst, (const void*)(intptr_t)off, (int64_t)n});
    if (e->up_data.size() >= kUpFlushBytes) RCCHK(flush_uploads(e));
    return OWRX_OK;
}

static void free_chain(owrx_engine* e, Chain* c) {
    prel(e, c->d_pstate);
    prel(e, c->d_sstate);
    prel(e, c->d_ddc);
    prel(e, c->d_fd);
    prel(e, c->d_sq);
    for (int i = 0; i < kSlots; ++i) prel(e, c->d_dem[i]);
    for (int i = 0; i < kSlots; ++i) prel(e, c->d_s16[i]);
    prel(e, c->d_bp_taps);
    prel(e, c->d_wf);
    prel(e, c->d_pf);
    prel(e, c->d_pf_taps);
    prel(e, c->d_nr_state);
    prel(e, c->d_nr_in);
    prel(e, c->d_nr_pow);
    prel(e, c->d_nr_ola);
    prel(e, c->d_sf);
    prel(e, c->d_sf_acc);
    prel(e, c->d_sf_window);
    prel(e, c->d_sf_tw);
}

// A waterfall's buffers back to the pools without waiting: device buffers read by stream A
// and the pinned copy sources once the blocks enqueued so far drained, the row-slot buffers
// (stream R encoders and copies) once the row slots enqueued so far drained.
static void free_wf(owrx_engine* e, Waterfall* w) {
    prel(e, w->d_window);
    prel(e, w->d_tw);
    prel(e, w->d_partial);
    prel(e, w->d_y4);
    prel(e, w->d_ones);
    prel(e, w->d_work);
    prel(e, w->d_carry[0]);
    prel(e, w->d_carry[1]);
    prel(e, w->d_groups);
    prel(e, w->d_rows);
    for (int b = 0; b < kSlots; ++b) {
        hprel(e, w->h_groups[b]);
        hprel(e, w->h_rows[b]);
    }
    for (int s = 0; s < kRowSlots; ++s) {
        rowrel(e, w->d_s16[s], false);
        rowrel(e, w->d_f32[s], false);
        rowrel(e, w->d_bytes[s], false);
        rowrel(e, w->h_bytes[s], true);
    }
}

static void free_slot_staging(Slot& s) {
    dfree(s.d_posts);
    dfree(s.d_sel);
    hfree(s.h_sel);
    dfree(s.d_counts);
    dfree(s.d_out);
    dfree(s.d_sm);
    dfree(s.d_dbg);
    hfree(s.h_posts);
    hfree(s.h_counts);
    hfree(s.h_out);
    hfree(s.h_sm);
    hfree(s.h_dbg);
}

// Drain one block's outputs (streams B / C) into the host rings.
static int drain_slot(owrx_engine* e, int si) {
    Slot& s = e->slots[si];
    if (s.chains_pending) {
        const int hk = e->hl_forced ? 1 : 0;
        const double th0 = now_ms();
        RCCHK(wait_ev(e, s.evB));
        const double th1 = now_ms();
        e->hl_wait[hk] += th1 - th0;
        e->hl_n[hk]++;
        s.chains_pending = false;
        if (s.timed) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, s.a1, s.a2) == hipSuccess) e->stats.gpu_ms_ddc += ms;
            // stream A's post kernels, and separately the span from post_parallel's start to the
            // end of the encoder (streams A -> B -> C)
            if (hipEventElapsedTime(&ms, s.a2, s.a3) == hipSuccess) e->stats.gpu_ms_post += ms;
            if (hipEventElapsedTime(&ms, s.b0, s.b1) == hipSuccess) e->stats.gpu_ms_serial += ms;
            if (s.timed_mac && hipEventElapsedTime(&ms, s.m0, s.m1) == hipSuccess)
                e->stats.gpu_ms_ddc_mac += ms;
            s.timed = false;
            s.timed_mac = false;
        }
        // each chain's outputs into its rings: chains are independent, so ranges of them on
        // the host workers; the counters are summed per range
        std::atomic<int64_t> ov{0}, ab{0}, dd{0}, dr{0};
        for_range(e, (int64_t)s.post_ids.size(), [&](int64_t k0, int64_t k1) {
        int64_t overruns = 0, audio_bytes = 0, ddc_outputs = 0, dropped = 0;
        for (int64_t k = k0; k < k1; ++k) {
            auto it = e->chains.find(s.post_ids[k]);
            if (it == e->chains.end()) continue;
            Chain* c = it->second.get();
            const int64_t dropped0 = c->ring_dropped();
            const ChainCounts& cc = s.h_counts[k];
            const PostLayout& L = s.layout[k];  // as this block was built
            const int64_t nb = std::min<int64_t>(cc.out_bytes, L.out_cap);
            if (cc.out_bytes > L.out_cap) overruns++;
            c->audio.push(s.h_out + s.out_off[k], (size_t)nb);
            if (cc.sf_bytes > 0 && L.sf_gen == c->sf_gen) {
                const int64_t sb = std::min<int64_t>(cc.sf_bytes, L.sf_cap);
                if (cc.sf_bytes > L.sf_cap) overruns++;
                c->sfft.push(s.h_out + s.out_off[k] + out_region(L.out_cap), (size_t)sb);
            }
            if (L.tsq_cap + L.tagc_cap > 0 && L.tap_gen == c->tap_gen) {
                const uint8_t* tb = s.h_out + s.out_off[k] + out_region(L.out_cap) +
                                    out_region(L.sf_cap);
                if (L.tsq_cap > 0) {
                    const int64_t b = std::min<int64_t>(8 * cc.n_gate, L.tsq_cap);
                    if (8 * cc.n_gate > L.tsq_cap) overruns++;
                    c->tap_sel.push(tb, (size_t)b);
                }
                if (L.tagc_cap > 0) {
                    const int64_t b = std::min<int64_t>(4 * cc.n_front, L.tagc_cap);
                    if (4 * cc.n_front > L.tagc_cap) overruns++;
                    c->tap_audio.push(tb + out_region(L.tsq_cap), (size_t)b);
                }
            }
            audio_bytes += nb;
            ddc_outputs += cc.n_ddc;
            c->smeter.push((const uint8_t*)(s.h_sm + (int64_t)k * e->sm_stride),
                           sizeof(float) * (size_t)std::min<int64_t>(cc.smeter, e->sm_stride));
            dropped += c->ring_dropped() - dropped0;
            if (s.debug && s.h_dbg) {
                const uint8_t* base = s.h_dbg + (int64_t)k * kDebugStages * e->dbg_stride;
                const int64_t cnt[kDebugStages] = {cc.n_ddc,  cc.n_fd,    cc.n_bp,
                                                   cc.n_gate, cc.n_front, cc.n_front};
                const int64_t isz[kDebugStages] = {8, 8, 8, 8, 4, 4};
                for (int st = 0; st < kDebugStages; ++st) {
                    const int64_t bytes = std::min(cnt[st] * isz[st], e->dbg_stride);
                    c->dbg[st].push(base + st * e->dbg_stride, (size_t)bytes);
                }
            }
        }
        ov += overruns;
        ab += audio_bytes;
        dd += ddc_outputs;
        dr += dropped;
        });
        e->stats.overruns += ov.load();
        e->ring_dropped += dr.load();
        e->stats.audio_bytes += ab.load();
        e->stats.ddc_outputs += dd.load();
        e->hl_push[hk] += now_ms() - th1;
        e->stats.host_ms_drain_wait += th1 - th0;
        e->stats.host_ms_drain_copy += now_ms() - th1;
    } else if (s.timed) {
        float ms = 0;
        RCCHK(wait_ev(e, s.a3));
        if (hipEventElapsedTime(&ms, s.a1, s.a2) == hipSuccess) e->stats.gpu_ms_ddc += ms;
        if (s.timed_mac && hipEventElapsedTime(&ms, s.m0, s.m1) == hipSuccess)
            e->stats.gpu_ms_ddc_mac += ms;
        s.timed = false;
        s.timed_mac = false;
    }
    if (s.timed_wf) {
        float ms = 0;
        RCCHK(wait_ev(e, s.a1));
        if (hipEventElapsedTime(&ms, s.a0, s.a1) == hipSuccess) e->stats.gpu_ms_waterfall += ms;
        s.timed_wf = false;
    }
    if (s.timed_wff) {
        float ms = 0;
        RCCHK(wait_ev(e, s.w1));
        if (hipEventElapsedTime(&ms, s.w0, s.w1) == hipSuccess) {
            e->stats.gpu_ms_waterfall_fft += ms;
            e->stats.gpu_ms_waterfall_fft_max = std::max<double>(e->stats.gpu_ms_waterfall_fft_max, ms);
            if (e->wf_ms_log.size() < 4096) e->wf_ms_log.push_back((float)ms);
        }
        s.timed_wff = false;
    }
    return OWRX_OK;
}

// Drain finished row slots in order; with `block` wait until `upto` slots remain in flight.
static int drain_rows(owrx_engine* e, bool block, int keep) {
    while (e->row_tail < e->row_head) {
        const int ri = (int)(e->row_tail % kRowSlots);
        RowSlot& r = e->rslots[ri];
        const bool must = block && (e->row_head - e->row_tail) > keep;
        if (!must) {
            hipError_t q = hipEventQuery(r.evC);
            if (q == hipErrorNotReady) break;
            HIPCHK(q);
        } else {
            RCCHK(wait_ev(e, r.evC));
        }
        for (auto& kv : e->wfs) {
            Waterfall* w = kv.second.get();
            const int nr = w->pend_rows[ri];
            if (nr <= 0) continue;
            const int64_t rb = w->row_bytes_for(w->pend_adpcm[ri]);
            w->ring.push(w->pend_h[ri], (size_t)(rb * nr));
            w->rows += nr;
            e->stats.waterfall_rows += nr;
            w->pend_rows[ri] = 0;
            const double tnow = now_ms();
            for (double tr : w->pend_t[ri]) {
                if (tr < 0) continue;
                const double lat = tnow - tr;
                e->stats.wf_row_latency_ms_max = std::max(e->stats.wf_row_latency_ms_max, lat);
                e->stats.wf_row_latency_ms_sum += lat;
                e->stats.wf_rows_latency_n++;
            }
            w->pend_t[ri].clear();
        }
        r.pending = false;
        e->row_tail++;
    }
    if (!e->row_retired.empty()) row_collect(e);
    return OWRX_OK;
}

// Drain finished chain slots in block order; with `block` wait until `keep` remain in flight.
static int drain_slots(owrx_engine* e, bool block, int keep) {
    while (e->slot_tail < e->block_index) {
        const int si = (int)(e->slot_tail % e->nslots);
        Slot& s = e->slots[si];
        const bool must = block && (e->block_index - e->slot_tail) > keep;
        if (!must) {
            hipEvent_t ev = s.chains_pending ? s.evB : (s.timed ? s.a3 : nullptr);
            if (ev) {
                hipError_t q = hipEventQuery(ev);
                if (q == hipErrorNotReady) break;
                HIPCHK(q);
            }
        }
        RCCHK(drain_slot(e, si));
        e->slot_tail++;
    }
    if (!e->pool_retired.empty() || !e->hpool_retired.empty()) pool_collect(e);
    return OWRX_OK;
}

static int drain_all(owrx_engine* e) {
    e->stats.pipeline_drains++;
    RCCHK(sync_stream(e, e->sA));
    e->in_done = e->block_index - 1;
    RCCHK(drain_rows(e, true, 0));
    return drain_slots(e, true, 0);
}

// Launch capacity of a waterfall (no drain: reconfiguration and joins run while blocks are in
// flight).  Buffers only grow, geometrically; a grown stream-A buffer replaces the old one for
// launches from now on and the old one returns to the pool once the blocks that used it
// drained; so are the pinned copy sources of slot bp (by block) and the buffers of row slot ri
// (by row slot), so a reservation may run while blocks are in flight.
static int wf_reserve(owrx_engine* e, Waterfall* w, int groups, int rows, int bp, int ri) {
    groups = std::max(groups, 1);
    rows = std::max(rows, 1);
    if (groups > w->partial_groups) {
        const int cap = std::max(groups, w->partial_groups + w->partial_groups / 2);
        prel(e, w->d_partial);
        prel(e, w->d_groups);
        prel(e, w->d_y4);
        HIPCHK(palloc(e, &w->d_partial, (size_t)cap * w->N));
        HIPCHK(palloc(e, &w->d_groups, (size_t)cap));
        if (w->N > kWfLdsMaxN)
            HIPCHK(palloc(e, &w->d_y4, (size_t)cap * w->N * (wf_uses_split(w->logn) ? kWfSplitMaxFpg : 1)));
        w->partial_groups = cap;
    }
    if (rows + 1 > w->rows_cap) {
        const int cap = std::max(rows + 1, w->rows_cap + w->rows_cap / 2);
        prel(e, w->d_rows);
        HIPCHK(palloc(e, &w->d_rows, (size_t)cap));
        w->rows_cap = cap;
    }
    if (bp >= 0 && std::max(groups, rows + 1) > w->h_cap[bp]) {
        const int cap = std::max(w->partial_groups, w->rows_cap);
        hprel(e, w->h_groups[bp]);
        hprel(e, w->h_rows[bp]);
        HIPCHK(hpalloc(e, &w->h_groups[bp], (size_t)cap));
        HIPCHK(hpalloc(e, &w->h_rows[bp], (size_t)cap));
        w->h_cap[bp] = cap;
    }
    if (ri >= 0 && rows > w->row_slot_cap[ri]) {
        const int cap = std::max(rows, w->row_slot_cap[ri] + w->row_slot_cap[ri] / 2);
        rowrel(e, w->d_s16[ri], false);
        rowrel(e, w->d_f32[ri], false);
        rowrel(e, w->d_bytes[ri], false);
        rowrel(e, w->h_bytes[ri], true);
        HIPCHK(palloc(e, &w->d_s16[ri], (size_t)cap * w->N));
        HIPCHK(palloc(e, &w->d_f32[ri], (size_t)cap * w->N));
        HIPCHK(palloc(e, &w->d_bytes[ri], (size_t)cap * 4 * w->N));
        HIPCHK(hpalloc(e, &w->h_bytes[ri], (size_t)cap * 4 * w->N));
        w->row_slot_cap[ri] = cap;
    }
    return OWRX_OK;
}

// the launch sizes a waterfall expects, for every block slot and row slot (its launches then
// allocate nothing: a hipMalloc / hipHostMalloc mid-stream maps pages into the GPU's address
// space, and the launches around one ran several times slower, measured 0.5-1 ms of stalled
// kernels per allocation).  Descriptors: the groups plus the tail split's single frames.
static int wf_initial_reserve(owrx_engine* e, Waterfall* w) {
    const int64_t span = w->batch_min > 1 ? e->history + proc_block(e) : proc_block(e);
    const int hop = std::max(1, w->pending ? std::min(w->hop, w->new_hop) : w->hop);
    const int avg = std::max(1, w->pending ? std::min(w->avg, w->new_avg) : w->avg);
    const int64_t frames = span / hop + 2;
    const int groups = (int)(frames / std::max(1, w->fpg) + frames / avg + 4);
    const int rows = (int)(frames / avg + 3);
    const int descs = groups + (int)frames;
    RCCHK(wf_reserve(e, w, descs, rows, -1, -1));
    for (int bp = 0; bp < kSlots; ++bp) RCCHK(wf_reserve(e, w, descs, rows, bp, -1));
    for (int ri = 0; ri < kRowSlots; ++ri) RCCHK(wf_reserve(e, w, descs, rows, -1, ri));
    return OWRX_OK;
}

static int ensure_post_capacity(owrx_engine* e) {
    const int n = (int)e->chains.size();
    // output staging: one region per chain, sized by that chain's own worst case (ADPCM audio
    // is ~2.6 KB per C2 block, a service resampler's cf32 IF up to 8 B per decimated sample);
    // the sums are kept by chain create / destroy / set_taps / set_secondary_fft (the staging
    // only grows: slots in flight were built within the current size)
    const int64_t need_out = e->need_out, need_sm = e->need_sm, need_dbg = e->need_dbg;
    if (n <= e->post_cap && need_out <= e->out_total && need_sm <= e->sm_stride &&
        (!e->debug || need_dbg <= e->dbg_stride))
        return OWRX_OK;
    RCCHK(drain_all(e));
    // posts capacity grows geometrically; the output region total is re-derived every time
    const int cap = n <= e->post_cap ? e->post_cap : std::max(n, e->post_cap ? e->post_cap * 2 : 16);
    e->out_total = need_out + need_out / 2;  // headroom: adding a chain rarely reallocates
    e->sm_stride = need_sm;
    e->dbg_stride = e->debug ? (need_dbg + 255) & ~(int64_t)255 : 0;
    for (int si = 0; si < e->nslots; ++si) {
        Slot& s = e->slots[si];
        free_slot_staging(s);
        HIPCHK(dalloc_z(e, &s.d_posts, cap));
        HIPCHK(halloc(&s.h_posts, cap));
        // serial lane lists (+ demodulator-run padding), then the long-bandpass post list and
        // chain_afc's list (a RawSAm chain at 48 kHz is on both: up to cap entries each)
        HIPCHK(dalloc_z(e, &s.d_sel, (size_t)3 * cap + kSelPad));
        HIPCHK(halloc(&s.h_sel, (size_t)3 * cap + kSelPad));
        HIPCHK(dalloc_z(e, &s.d_counts, cap));
        HIPCHK(dalloc_z(e, &s.d_out, (size_t)e->out_total));
        HIPCHK(dalloc_z(e, &s.d_sm, (size_t)cap * e->sm_stride));
        HIPCHK(halloc(&s.h_counts, (size_t)cap));
        HIPCHK(halloc(&s.h_out, (size_t)e->out_total));
        HIPCHK(halloc(&s.h_sm, (size_t)cap * e->sm_stride));
        if (!s.h_jobs) HIPCHK(halloc(&s.h_jobs, (size_t)kMaxCopyJobs));
        s.post_dirty = true;
        if (e->debug) {
            HIPCHK(dalloc_z(e, &s.d_dbg, (size_t)cap * kDebugStages * e->dbg_stride));
            HIPCHK(halloc(&s.h_dbg, (size_t)cap * kDebugStages * e->dbg_stride));
        }
    }
    e->post_cap = cap;
    RCCHK(flush_zero(e));  // the new buffers' zeroing, one launch (see dalloc_z)
    return OWRX_OK;
}

static int group_refresh_device(owrx_engine* e, ChainGroup* g) {
    // per-chain DDC descriptors + partial buffer sized for the current membership
    const int n = (int)g->members.size();
    if (n > g->chains_cap) {
        RCCHK(drain_all(e));
        dfree(g->d_chains);
        for (auto& h : g->h_chains) hfree(h);
        g->chains_cap = std::max(n, 2 * g->chains_cap);
        HIPCHK(dalloc_z(e, &g->d_chains, (size_t)g->chains_cap));
        for (auto& h : g->h_chains) HIPCHK(halloc(&h, (size_t)g->chains_cap));
        RCCHK(flush_zero(e));
    }
    const int64_t nk_max = proc_block(e) / g->D + 4;
    // Launch shape: each tile group's D phases are split into nseg segments, one 4-wave
    // workgroup each (kernels_ddc.hip); stream A's CUs hold ddc_blocks_per_cu of them.
    const int R = 32;
    int cpw = 1;
    while (cpw < n && cpw < 64) cpw <<= 1;
    const int tpw = 64 / cpw;
    const int64_t ntg = ((nk_max + R - 1) / R + tpw - 1) / tpw;
    const int64_t ncg = (n + cpw - 1) / cpw;
    const int64_t base = std::max<int64_t>(1, ntg * ncg);
    const int64_t slots = (int64_t)ddc_blocks_per_cu(g->P, n) * std::max(1, e->cus_a);
    // ~4 workgroups per resident slot: measured flat from 12 to 24 segments at C2 (a
    // rounds-quantisation model did not predict the timings; fewer segments starve the CUs,
    // more cost post_parallel extra partials)
    int nseg = (int)std::min<int64_t>(std::max<int64_t>(1, (2 * slots + base - 1) / base),
                                      std::max(1, g->D / 32));
    nseg = ddc_segments(g->D, nseg, g->P, n);
    if (const char* v = getenv("OWRX_DDC_NSEG")) nseg = ddc_segments(g->D, std::max(1, atoi(v)), g->P, n);
    if (getenv("OWRX_VERBOSE"))
        fprintf(stderr, "owrx: DDC group D=%d P=%d chains=%d: %lld tile groups x %d segments, "
                "%lld resident workgroups\n", g->D, g->P, n, (long long)base, nseg, (long long)slots);
    const size_t need = (size_t)nseg * std::max(1, n) * nk_max;
    // geometric growth (x1.5): adding chains one at a time must not reallocate every time
    // (buffers proportional to the membership: quadratic setup time at thousands of chains)
    if (need > g->partial_elems) {
        RCCHK(drain_all(e));
        const size_t alloc = need + need / 2;
        for (int i = 0; i < e->nslots; ++i) {  // the depth is fixed before the first chain
            dfree(g->d_partial[i]);
            HIPCHK(dalloc_z(e, &g->d_partial[i], alloc));
        }
        RCCHK(flush_zero(e));
        g->partial_elems = alloc;
    }
    g->nseg = nseg;
    if (g->fc_M) {  // fast-convolution product rows Y[chains][Fs][M]
        // times the K slices its smallest tile grid may be split into (fc_kslices)
        const size_t ny = (size_t)std::max(1, n) * g->fc_Fs * (size_t)g->fc_M *
                          (size_t)fc_kslices_max(g->fc_M, std::max(1, n), g->fc_Dp, e->cus_a);
        if (ny > g->fc_y_elems) {
            RCCHK(drain_all(e));
            dfree(g->d_fc_y);
            HIPCHK(dalloc_z(e, &g->d_fc_y, ny + ny / 2));
            RCCHK(flush_zero(e));
            g->fc_y_elems = ny + ny / 2;
        }
    }
    return OWRX_OK;
}

// Frame length M of the fast-convolution DDC for a group: the M (64, 128, 192, 256, 384) with
// the least modelled time per block and chain, max(f32 MFMA time of the padded frame tiles, HBM
// time of the W reads), ties to the longer frame (fewer frames: less U / Y traffic).  0 when
// the branch filters are too long for these frames (the group then runs the direct form).
//
// The frame length is chosen for the caller's block, so a grouped engine (owrx_set_block_group)
// keeps the ungrouped design and its outputs byte for byte.  C3 in fours would model faster at
// M = 192 (32 frames, no tile padding, against 52 frames of M = 128 padded to 64): fc_mac rose
// to 0.45-0.50 of the MFMA peak, but the job ran 2.5 % slower over eleven interleaved pairs of
// runs (stream C, the bound, slower with the GEMM's power drawn in a shorter time is the likely
// reading; profiles/r06_fc_m_ab.txt), so it is not the default (OWRX_FC_M=192 for the A/B).
static double fc_model_t(int M, int Dp, int P, int64_t nk_max) {
    const int V = M - P + 1;
    const int64_t F = (nk_max + V - 1) / V;
    const int64_t ft = F > 16 ? 32 : 16;
    const int64_t Fp = (F + ft - 1) / ft * ft;
    const double flop = 8.0 * M * Dp * Fp;
    const double wbytes = 8.0 * M * Dp * (Fp / ft);
    return std::max(flop / 150e12, wbytes / 5e12);
}
static int fc_choose_m(int D, int P, int64_t nk_max) {
    const int Dp = (D + 95) / 96 * 96;
    int best = 0;
    double best_t = 0;
    for (int M : {384, 256, 192, 128, 64}) {
        if (M - P + 1 < M / 2) continue;
        const double t = fc_model_t(M, Dp, P, nk_max);
        if (!best || t < best_t * 0.999) {
            best = M;
            best_t = t;
        }
    }
    return best;
}

// (Re)builds the W[kappa][r] of the chain in `slot` for its current shift rate on stream A,
// ordered before the next block's DDC (and after every earlier block's, which still read the
// old spectra).
static int fc_build_w(owrx_engine* e, Chain* c, int slot) {
    ChainGroup* g = c->group;
    if (!g->fc_M) return OWRX_OK;
    // (W is zeroed by fc_reserve before any build writes it; nothing else pending is read here)
    HIPCHK(launch_fc_make_w(g->fc_M, g->d_h, g->T, g->D, g->fc_Dp, g->fc_P, c->rate_fx,
                            g->d_fc_w + fc_w_chain_offset(slot, g->fc_Dp), g->fc_w_ks(), e->sA));
    return OWRX_OK;
}

// Room for `slots` members' spectra: grows W[kappa][slot tiles] (kernels_fcddc.hip: tiles of
// fc_w_tile() chains, so capacities are multiples of it and a bin's first cap Dp entries hold its
// first cap slots) by doubling, moving the existing rows with one strided copy.
static int fc_reserve(owrx_engine* e, ChainGroup* g, int slots) {
    if (!g->fc_M || slots <= g->fc_w_cap) return OWRX_OK;
    const int M = g->fc_M;
    const int tile = fc_w_tile();
    const int cap = (std::max(std::max(32, 2 * g->fc_w_cap), slots) + tile - 1) / tile * tile;
    float2* nw = nullptr;
    // on stream A behind the blocks that read the old spectra (those release it when drained)
    HIPCHK(palloc(e, &nw, (size_t)M * cap * g->fc_Dp));
    RCCHK(flush_zero(e));  // zeroed before the rows are copied in
    RCCHK(flush_wbuilds(e));  // the old rows complete before they move
    if (g->d_fc_w && g->fc_w_cap > 0) {
        const size_t row = sizeof(float2) * (size_t)g->fc_w_cap * g->fc_Dp;
        HIPCHK(hipMemcpy2DAsync(nw, sizeof(float2) * (size_t)cap * g->fc_Dp, g->d_fc_w, row, row,
                                (size_t)M, hipMemcpyDeviceToDevice, e->sA));
    }
    prel(e, g->d_fc_w);
    g->d_fc_w = nw;
    g->fc_w_cap = cap;
    return OWRX_OK;
}

// ------------------------------------------------------------------------------------------
// block processing
// ------------------------------------------------------------------------------------------

// Frames summed by one FFT workgroup (one partial |X|^2 row per group).  Fixed per waterfall
// configuration (engine geometry and hop -- not the launch batching) and groups start at fixed
// frame offsets of a row, so the summation order -- hence every row, bit for bit -- depends
// neither on how the stream is cut into blocks nor on how frames are batched into launches:
//  - N = 16384 on wf_fft_q16 (the default): 8 (wf_default_fpg; its group-end transpose and
//    partial row amortise over twice the frames, 0.291 vs 0.275 of HBM at 3840 C3 frames,
//    profiles/r05_wf_micro.txt); on wf_fft_l32 (OWRX_WF_KERNEL=l32) and after the DIF split
//    (N = 16384 Q): 4 (C3 geometry, 960 frames from HBM: F = 4 49 us vs F = 2 55 us,
//    profiles/r04*_wf_micro.txt);
//  - wf_fft_r16: enough that a block's frames occupy stream A's CUs about once;
//  - the four-step FFT (OWRX_WF_KERNEL=fourstep): one frame per group;
// always clamped so that a group still open at a block's end fits the next block's history.
static int wf_frames_per_group(const owrx_engine* e, const Waterfall* w) {
    const int64_t hop = std::max(1, w->hop);
    const int64_t frames = e->max_block / hop;  // not the batch: rows must not depend on it
    const int64_t cus = std::max(1, e->cus_a);
    // a group still open at the end of a block is read again from the next block's window, so
    // its span (fpg - 1) hop + N must fit the history (every kernel)
    const int64_t fit = std::max<int64_t>(1, (e->history - w->N) / hop + 1);
    int64_t fpg;
    if (w->N > kWfLdsMaxN) {
        if (!wf_uses_split(w->logn)) return 1;
        fpg = kWfSplitMaxFpg;
    } else if (wf_uses_l32(w->logn)) {
        static const int l32_fpg = [] {  // OWRX_WF_FPG: frames per group (A/B)
            const char* v = getenv("OWRX_WF_FPG");
            return v ? std::max(1, std::min(16, atoi(v))) : 0;
        }();
        fpg = l32_fpg ? l32_fpg : wf_default_fpg(w->logn);
    } else {
        fpg = std::min<int64_t>((frames + cus - 1) / cus, kWfMaxFramesPerGroup);
    }
    return (int)std::max<int64_t>(1, std::min(fpg, fit));
}

// Schedules and launches one FftChain's ready frames on stream A (when the batching rule says
// so, or `force`); completed rows are staged in row slot `ri` (their ADPCM / copy is enqueued
// by the caller on that slot's stream).
static int process_waterfall(owrx_engine* e, Waterfall* w, const float2* blk, int64_t blk_start,
                             int64_t blk_end, int ri, bool force, int* completed, bool timed,
                             Slot* S) {
    *completed = 0;
    w->groups.clear();
    w->rowdesc.clear();
    if (w->next_start + w->N > blk_end) return OWRX_OK;  // no frame complete
    if (w->t_pending < 0) w->t_pending = e->t_block;
    if (w->batch_min > 1 && !force) {
        // launch once enough frames are ready, or the oldest pending one is max_lag behind, or
        // it would leave the window of the next block (which starts at blk_end - history), or
        // waiting for the next block call would hold it past the wall-clock bound
        const int64_t ready = (blk_end - w->N - w->next_start) / std::max(1, w->hop) + 1;
        const int64_t lag = blk_end - w->next_start;
        const int64_t max_lag = w->batch_lag > 0 ? w->batch_lag : e->history;
        const bool leaving = w->next_start < blk_end + w->hop - e->history;
        const bool late = w->batch_wall_ms > 0 &&
                          e->t_block - w->t_pending + e->block_interval_ms >= w->batch_wall_ms;
        if (ready < w->batch_min && lag < max_lag && !leaving && !late) return OWRX_OK;
    }
    w->pend_t[ri].clear();
    {
        // capacity for every frame ready now (groups: at most one per fpg frames plus one short
        // group per row end; rows: one per avg frames plus a partial one)
        const int bp = (int)(e->block_index % e->nslots);
        const int64_t ready = (blk_end - w->N - w->next_start) / std::max(1, w->hop) + 1;
        const int64_t avg_min = std::max(1, std::min(w->avg, w->pending ? w->new_avg : w->avg));
        const int64_t rows = ready / avg_min + 2;
        RCCHK(wf_reserve(e, w, (int)(ready / std::max(1, w->fpg) + rows + 2), (int)rows, bp, ri));
    }
    int cur_row_first_group = 0;
    bool row_open = false;
    const int adpcm_now = w->adpcm;
    const int avg_now = w->avg;
    while (true) {
        const int gf = std::min(w->fpg, w->avg - w->row_frame);
        const int64_t last = w->next_start + (int64_t)(gf - 1) * w->hop;
        if (last + w->N > blk_end) break;
        if ((int)w->groups.size() >= w->partial_groups) break;
        if (!row_open) {
            cur_row_first_group = (int)w->groups.size();
            row_open = true;
        }
        w->groups.push_back(WfGroup{w->next_start, gf, w->hop});
        w->next_start += (int64_t)gf * w->hop;
        w->row_frame += gf;
        if (w->row_frame == w->avg) {
            // readiness: the first block call whose stream end covered the row's last frame
            double tr = -1;
            for (const auto& bt : w->blk_times)
                if (bt.first >= last + w->N) {
                    tr = bt.second;
                    break;
                }
            w->pend_t[ri].push_back(tr);
            WfRow r;
            r.first_group = cur_row_first_group;
            r.ngroups = (int)w->groups.size() - cur_row_first_group;
            r.use_carry = (w->rowdesc.empty() && w->carry_valid) ? 1 : 0;
            r.complete = 1;
            r.out_index = (int)w->rowdesc.size();
            r.pad = 0;
            w->rowdesc.push_back(r);
            w->row_frame = 0;
            w->carry_valid = false;
            row_open = false;
            if (w->pending) {  // parameter changes apply at row boundaries (next block)
                w->hop = w->new_hop;
                w->avg = w->new_avg;
                w->adpcm = w->new_adpcm;
                w->fpg = wf_frames_per_group(e, w);
                w->pending = false;
                break;
            }
            if ((int)w->rowdesc.size() + 1 >= w->rows_cap ||
                (int)w->rowdesc.size() >= w->row_slot_cap[ri])
                break;
        }
    }
    const int ncomplete = (int)w->rowdesc.size();
    // frames still ready after this launch keep the pending time; blocks wholly launched go
    while (!w->blk_times.empty() && w->blk_times.front().first < w->next_start + w->N)
        w->blk_times.pop_front();
    w->t_pending = w->next_start + w->N <= blk_end ? e->t_block : -1;
    if (row_open) {  // partially accumulated row: sum into the carry
        WfRow r;
        r.first_group = cur_row_first_group;
        r.ngroups = (int)w->groups.size() - cur_row_first_group;
        r.use_carry = (w->rowdesc.empty() && w->carry_valid) ? 1 : 0;
        r.complete = 0;
        r.out_index = 0;
        r.pad = 0;
        w->rowdesc.push_back(r);
    }
    if (w->groups.empty()) return OWRX_OK;
    int64_t nfr = 0;
    for (const WfGroup& g : w->groups) nfr += g.nframes;
    e->stats.waterfall_frames += nfr;
    e->stats.waterfall_samples += nfr * w->hop;
    // the launching block's slot (its previous user, block k - kSlots, has drained; at
    // owrx_sync every slot has)
    const int bp = (int)(e->block_index % e->nslots);
    // tail split (wf_fft_l32): the last `skip` groups are also listed frame by frame after the
    // groups, and the kernel deals those frames instead (the rows do not change)
    const int ngroups = (int)w->groups.size();
    const int skip = wf_tail_split(w->logn, ngroups, std::max(1, e->cus_a), nfr, w->fpg);
    int tail = 0;
    for (int gi = ngroups - skip; gi < ngroups; ++gi) {
        const WfGroup g = w->groups[gi];
        for (int j = 0; j < g.nframes; ++j) {
            w->groups.push_back(WfGroup{g.start + (int64_t)j * g.hop, 1, g.hop});
            ++tail;
        }
    }
    if (tail) {
        RCCHK(wf_reserve(e, w, (int)w->groups.size(), (int)w->rowdesc.size(), bp, ri));
        // each row reaching into the split groups: its first split frame's descriptor (pad)
        const int g_split = ngroups - skip;
        for (WfRow& r : w->rowdesc) {
            r.pad = ngroups;
            for (int gi = g_split; gi < std::max(g_split, r.first_group); ++gi)
                r.pad += w->groups[gi].nframes;
        }
    }
    memcpy(w->h_groups[bp], w->groups.data(), sizeof(WfGroup) * w->groups.size());
    memcpy(w->h_rows[bp], w->rowdesc.data(), sizeof(WfRow) * w->rowdesc.size());
    HIPCHK(kcopy(w->d_groups, w->h_groups[bp], sizeof(WfGroup) * w->groups.size(), e->sA));
    HIPCHK(kcopy(w->d_rows, w->h_rows[bp], sizeof(WfRow) * w->rowdesc.size(), e->sA));
    const bool tm = timed && S && !S->timed_wff;  // the first waterfall of a timed block
    if (tm) {
        HIPCHK(hipEventRecord(S->w0, e->sA));
        e->stats.waterfall_timed_samples += nfr * w->hop;
        e->stats.waterfall_timed_launches++;
    }
    HIPCHK(launch_wf_fft(w->logn, blk, blk_start, w->d_groups, ngroups, w->fpg,
                         w->d_window, w->d_ones, w->d_tw, w->d_partial, w->d_y4, w->d_work,
                         std::max(1, e->cus_a), e->sA, skip, tail));
    const float corr = (float)((double)w->add_db - 10.0 * std::log10((double)std::max(1, avg_now)));
    const int cin = w->carry_idx, cout = 1 - w->carry_idx;
    HIPCHK(launch_wf_finalize(w->d_partial, w->d_rows, (int)w->rowdesc.size(), w->d_carry[cin],
                              w->d_carry[cout], w->N, corr, adpcm_now, w->d_s16[ri],
                              w->d_f32[ri], e->sA, w->d_groups, ngroups, skip));
    if (tm) {
        HIPCHK(hipEventRecord(S->w1, e->sA));
        S->timed_wff = true;
    }
    if (row_open) {
        w->carry_idx = cout;
        w->carry_valid = true;
    }
    e->stats.waterfall_launches++;
    w->pend_rows[ri] = ncomplete;
    w->pend_adpcm[ri] = adpcm_now;
    w->pend_h[ri] = w->h_bytes[ri];
    *completed = ncomplete;
    return OWRX_OK;
}


// Every waterfall's ready frames (batching rule, or all of them with `force`) on stream A, then
// the completed rows' FftAdpcm + copy on a row slot's stream, or with `rows_on_a` on stream A
// behind their FFT, one workgroup per row (owrx_sync's flush: A has no block behind it, and the
// row queue's 4 CUs take ~3 ms for a 3 840-frame batch's 40 rows).
static int run_waterfalls(owrx_engine* e, const float2* blk, int64_t blk_start, int64_t blk_end,
                          bool force, bool timed, Slot* S, bool rows_on_a = false) {
    bool any_rows = false;
    if (!e->wfs.empty()) {
        const double t = now_ms();
        RCCHK(drain_rows(e, true, kRowSlots - 1));  // frees the slot about to be reused
        e->stats.host_ms_wait_rows += now_ms() - t;
        const int ri = (int)(e->row_head % kRowSlots);
        RowSlot& R = e->rslots[ri];
        for (auto& kv : e->wfs) {
            Waterfall* w = kv.second.get();
            int done = 0;
            RCCHK(process_waterfall(e, w, blk, blk_start, blk_end, ri, force, &done, timed, S));
            any_rows |= done > 0;
        }
        if (any_rows) {
            const hipStream_t rs = rows_on_a ? e->sA : R.stream;
            if (!rows_on_a) {
                HIPCHK(hipEventRecord(R.evWf, e->sA));
                HIPCHK(hipStreamWaitEvent(R.stream, R.evWf, 0));
            }
            for (auto& kv : e->wfs) {
                Waterfall* w = kv.second.get();
                const int nr = w->pend_rows[ri];
                if (nr <= 0) continue;
                const int64_t rb = w->row_bytes_for(w->pend_adpcm[ri]);
                if (w->pend_adpcm[ri]) {
                    HIPCHK(launch_wf_adpcm(w->d_s16[ri], w->N, nr, w->d_bytes[ri], (int)rb,
                                           rows_on_a ? 0 : e->rows_grid, rs));
                    HIPCHK(kcopy(w->h_bytes[ri], w->d_bytes[ri], rb * nr, rs));
                } else {
                    HIPCHK(kcopy(w->h_bytes[ri], w->d_f32[ri], rb * nr, rs));
                }
            }
            HIPCHK(hipEventRecord(R.evC, rs));
            R.pending = true;
            e->row_head++;
        }
    }
    return OWRX_OK;
}


// Chains per block above which the serial kernels (post_serial_front, chain_nr, chain_adpcm) run
// on unmasked streams: one lane per chain, so 1 024 chains are 16 waves = one per SIMD of
// stream B's / C's 4 CUs; beyond that those CUs time-slice while the rest of the chip waits.
// OWRX_WIDE_SERIAL_CHAINS overrides (A/B; a huge value keeps the masked streams).
static int wide_serial_chains() {
    static const int v = [] {
        const char* s = getenv("OWRX_WIDE_SERIAL_CHAINS");
        return s ? atoi(s) : 1024;
    }();
    return v;
}

// A slot's post descriptors (pinned S.h_posts), the lane lists of the serial kernels and the
// long-bandpass list (S.h_sel), for the groups of e->work in that order; the per-block fields
// (nk, k_begin, nseg) are patched by the caller.  One-shot flags (secondary FFT reset,
// NoiseFilter reset) are consumed here, so the next use of this slot rebuilds without them.
static int build_posts(owrx_engine* e, Slot& S, int si) {
    S.post_ids.clear();
    S.out_off.clear();
    S.layout.clear();
    S.post_groups.clear();
    S.group_post0.clear();
    S.sf_sizes = 0;
    S.any_nr = false;
    bool one_shot = false;
    int64_t out_off = 0;
    int np = 0;
    const bool use_steps = e->work.size() <= (size_t)kMaxStepGroups;
    for (size_t gi = 0; gi < e->work.size(); ++gi) {
        const GroupWork& gw = e->work[gi];
        const ChainGroup* g = gw.g;
        S.post_groups.push_back(g);
        S.group_post0.push_back(np);
        for (size_t i = 0; i < g->members.size(); ++i) {
            Chain* c = e->chains[g->members[i]].get();
            ChainPost& p = S.h_posts[np];
            memset(&p, 0, sizeof(p));
            const owrx_chain_params& q = c->prm;
            p.demod = q.demod;
            p.step_idx = use_steps ? (int)gi : -1;  // nk / k_begin / nseg: post_parallel's table
            p.afc_update = q.afc_update;
            p.afc_sample = q.afc_sample;
            p.output = q.output;
            p.frac_enabled = q.frac_rate != 1.0;
            p.frac_rate = q.frac_rate;
            p.bp_ntaps = q.bandpass ? c->bp_ntaps : 0;
            p.bp_taps = c->d_bp_taps;
            p.sq_len = q.sq_length;
            p.sq_dec = q.sq_decimation;
            p.sq_hang = q.sq_hang;
            p.sq_flush = q.sq_flush;
            p.sq_report = q.sq_report;
            p.sq_level = q.sq_level;
            p.deemph_alpha = nfm_deemphasis_alpha(q.audio_rate);
            p.bp_hist = c->bp_hist;
            p.bp_long = c->bp_hist > kBpHist ? 1 : 0;
            if (q.demod == OWRX_DEMOD_WFM) {
                // WfmDeemphasis(rate, tau): y += dt/(tau+dt) * (x - y) (csdr deemphasis_wfm_ff)
                const double dt = 1.0 / (double)q.audio_rate;
                const double tau = q.deemph_tau > 0 ? (double)q.deemph_tau : 50e-6;
                p.deemph_alpha = (float)(dt / (tau + dt));
                p.wfm_rate = q.if_rate / (double)q.audio_rate;
                p.pf_taps = c->d_pf_taps;
                p.pf_ntaps = c->pf_ntaps;
                p.wf_buf = c->d_wf;
                p.pf_buf = c->d_pf;
            }
            p.deemph_beta = 1.0f - p.deemph_alpha;
            if (q.nr_enabled && c->d_nr_state && q.output != OWRX_OUT_IQ) {
                if (c->nr_reset) {  // zeroed on the serial stream before this block's work
                    e->nr_resets.push_back(c);
                    c->nr_reset = false;
                    one_shot = true;
                }
                p.nr_enabled = 1;
                p.nr_t = (float)std::pow(10.0, (double)q.nr_threshold / 10.0);
                p.nr_state = c->d_nr_state;
                p.nr_in = c->d_nr_in;
                p.nr_pow = c->d_nr_pow;
                p.nr_ola = c->d_nr_ola;
                p.nr_win = e->d_nr_win;
                p.nr_tw = e->d_nr_tw;
                S.any_nr = true;
            }
            p.agc = agc_profile(q.agc_profile);
            if (q.agc_initial_gain >= 0) p.agc.initial_gain = q.agc_initial_gain;
            if (q.agc_max_gain >= 0) p.agc.max_gain = q.agc_max_gain;
            if (q.demod == OWRX_DEMOD_WFM) p.agc.max_gain = std::max(1.0f, p.agc.max_gain);
            if (q.audio_gain > 0) {  // Gain(audio_gain) replaces the Agc (post_serial_front)
                p.fixed_gain = 1;
                p.agc.max_gain = q.audio_gain;
            }
            p.pstate = c->d_pstate;
            p.sstate = c->d_sstate;
            p.ddc_buf = c->d_ddc;
            p.fd_buf = c->d_fd;
            p.sq_buf = c->d_sq;
            p.dem = c->d_dem[si];
            p.s16 = c->d_s16[si];
            p.partial = g->d_partial[si];
            p.nseg = gw.fast ? 1 : g->nseg;
            p.group_chains = (int)g->members.size();
            p.chain_in_group = (int)i;
            p.k_first = c->k_first;
            p.out = S.d_out + out_off;
            p.out_cap = c->out_cap;
            S.out_off.push_back(out_off);
            out_off += out_region(c->out_cap);
            if (c->sf_n > 0 && q.output != OWRX_OUT_IQ) {
                p.sf_n = c->sf_n;
                p.sf_hop = c->sf_hop;
                p.sf_avg = std::max(1, c->sf_avg);
                p.sf_adpcm = c->sf_adpcm;
                p.sf_reset = c->sf_reset ? 1 : 0;
                one_shot |= c->sf_reset;
                c->sf_reset = false;
                p.sf_corr = (float)((double)c->sf_add_db - 10.0 * std::log10((double)p.sf_avg));
                p.sf_buf = c->d_sf;
                p.sf_acc = c->d_sf_acc;
                p.sf_window = c->d_sf_window;
                p.sf_tw = c->d_sf_tw;
                p.sf_out = S.d_out + out_off;
                p.sf_out_cap = c->sf_out_cap;
                S.sf_sizes |= 1u << c->sf_logn;
            }
            out_off += out_region(c->sf_out_cap);
            if (c->tap_sq_cap > 0 && q.output != OWRX_OUT_IQ) {
                p.tap_sq = (float2*)(S.d_out + out_off);
                p.tap_sq_cap = c->tap_sq_cap / 8;
            }
            if (c->tap_agc_cap > 0 && q.output != OWRX_OUT_IQ) {
                p.tap_agc = (float*)(S.d_out + out_off + out_region(c->tap_sq_cap));
                p.tap_agc_cap = c->tap_agc_cap / 4;
            }
            out_off += c->tap_bytes();
            S.layout.push_back(PostLayout{c->out_cap, c->sf_out_cap, c->tap_sq_cap, c->tap_agc_cap,
                                          c->sf_gen, c->tap_gen});
            p.smeter = S.d_sm + (int64_t)np * e->sm_stride;
            p.smeter_cap = (int)e->sm_stride;
            p.debug = (e->debug && S.d_dbg) ? 1 : 0;
            if (p.debug) {
                uint8_t* base = S.d_dbg + (int64_t)np * kDebugStages * e->dbg_stride;
                p.dbg_ddc = (float2*)(base + 0 * e->dbg_stride);
                p.dbg_fd = (float2*)(base + 1 * e->dbg_stride);
                p.dbg_bp = (float2*)(base + 2 * e->dbg_stride);
                p.dbg_sq = (float2*)(base + 3 * e->dbg_stride);
                p.dbg_dem = (float*)(base + 4 * e->dbg_stride);
                p.dbg_agc = (float*)(base + 5 * e->dbg_stride);
                p.dbg_cap = e->dbg_stride / 8;
            }
            S.post_ids.push_back(g->members[i]);
            np++;
        }
    }
    S.np = np;
    // long-bandpass chains (indices after the serial lane lists in the sel buffer)
    S.nlong = 0;
    S.long_taps = 0;
    S.long_fd = 0;
    S.long_off = e->post_cap + kSelPad;
    for (int i = 0; i < np; ++i)
        if (S.h_posts[i].bp_long && S.h_posts[i].output != OWRX_OUT_IQ) {
            S.h_sel[S.long_off + S.nlong++] = i;
            S.long_taps = std::max(S.long_taps, S.h_posts[i].bp_ntaps);
            S.long_fd = std::max<int64_t>(S.long_fd, e->chains[S.post_ids[i]]->cap);
        }
    // one post_serial_front launch per output format present (S16 / ADPCM / F32); within a
    // format the chains are ordered by demodulator and every demodulator's run is padded to
    // whole 64-lane workgroups (-1 = idle lane), so each wave has a uniform demodulator; lists
    // per (output, NoiseFilter): a NoiseFilter chain's front stores for chain_nr instead of
    // converting; the two ADPCM lists are adjacent (one chain_adpcm launch)
    std::vector<int>(&bk)[3][2][4] = e->sel_buckets;
    for (auto& a : bk)
        for (auto& b : a)
            for (auto& v : b) v.clear();
    for (int i = 0; i < np; ++i) {
        const ChainPost& p = S.h_posts[i];
        // SAm's serial part after chain_afc is AM's (DcBlock -> Agc / Gain)
        const int dm = p.demod == OWRX_DEMOD_SAM ? OWRX_DEMOD_AM : p.demod;
        if (p.output >= 0 && p.output < 3 && dm >= 0 && dm < 4)
            bk[p.output][p.nr_enabled != 0][dm].push_back(i);
    }
    int nfill = 0;
    for (int o = 0; o < 3; ++o)
        for (int nr = 0; nr < 2; ++nr) {
            S.off[o][nr] = nfill;
            for (int dm = 0; dm < 4; ++dm) {
                const std::vector<int>& v = bk[o][nr][dm];
                for (int i : v) S.h_sel[nfill++] = i;
                for (size_t run = v.size(); run % 64; ++run) S.h_sel[nfill++] = -1;
            }
            S.nsel[o][nr] = nfill - S.off[o][nr];
        }
    S.nfill = nfill;
    // SAm chains: chain_afc's lane list after the long-bandpass list
    S.afc_off = S.long_off + S.nlong;
    S.nafc = 0;
    for (int i = 0; i < np; ++i)
        if (S.h_posts[i].demod == OWRX_DEMOD_SAM && S.h_posts[i].output != OWRX_OUT_IQ)
            S.h_sel[S.afc_off + S.nafc++] = i;
    S.post_epoch = e->chain_epoch;
    S.post_dirty = one_shot;
    S.dev_stale = true;
    return OWRX_OK;
}

// Wait until block j's stream-A work (which read its input and its staged descriptors) is done.
// engine blocks after which the caller's oldest retained input is read: `retention` caller
// blocks, each engine block of a paired engine holding up to two of them
static int in_keep(const owrx_engine* e) { return e->group > 1 ? (e->retention - 1) / e->group : e->retention; }

static int wait_input_block(owrx_engine* e, int64_t j) {
    if (j <= e->in_done || j < 0) return OWRX_OK;
    RCCHK(wait_ev(e, e->evIn[j % kInEv]));
    e->in_done = j;
    return OWRX_OK;
}

// `nsub` > 1: that many caller blocks of sub_n[] samples each (owrx_set_block_group); every stage
// runs once over all of them, the fast DDC with each block's own frame placement
static int process_block(owrx_engine* e, const float2* blk, int64_t n, int nsub = 1,
                         const int64_t* sub_n = nullptr) {
    const double t_enter = now_ms();
    RCCHK(flush_uploads(e));  // pool buffers and uploads of chains / waterfalls created since the last block
    // Block k's pinned descriptors are staged per slot (reused by block k + kSlots, after the
    // slot drained and block k's stream-A work is known done).  The caller's input: blocks
    // k - retention + 1 .. k may still be read on stream A when this call returns, block
    // k - retention is done (owrx_set_input_retention; 1 = the owrx_process_device contract:
    // the caller may reuse block k - 1's buffer).  The wait comes at the end, after block k is enqueued, so stream A
    // runs earlier blocks while the host builds block k; OWRX_IN_WAIT=start waits before the
    // build (the round-1/2 order, A/B).
    static const bool wait_first = [] {
        const char* v = getenv("OWRX_IN_WAIT");
        return v && strcmp(v, "start") == 0;
    }();
    if (wait_first) {
        const double t = now_ms();
        RCCHK(wait_input_block(e, e->block_index - in_keep(e)));
        e->stats.host_ms_wait_input += now_ms() - t;
    }
    const int bp = (int)(e->block_index % e->nslots);
    const int64_t blk_start = e->pos;
    const int64_t blk_end = e->pos + n;
    // wall-clock bookkeeping of the waterfall batching bound and row latency
    e->t_block = t_enter;
    if (e->t_last_block >= 0) {
        const double d = t_enter - e->t_last_block;
        e->block_interval_ms = e->block_interval_ms > 0 ? 0.75 * e->block_interval_ms + 0.25 * d : d;
    }
    e->t_last_block = t_enter;
    for (auto& kv : e->wfs) kv.second->blk_times.emplace_back(blk_end, t_enter);
    const int si = (int)(e->block_index % e->nslots);
    Slot& S = e->slots[si];
    // the slot's previous block (k - kSlots) must be drained before its buffers are reused
    // (and its stream-A work done: a block without chain outputs drains without a wait)
    {
        const double t = now_ms();
        e->hl_forced = true;
        const int rc = drain_slots(e, true, e->nslots - 1);
        e->hl_forced = false;
        RCCHK(rc);
        RCCHK(wait_input_block(e, e->block_index - e->nslots));
        e->stats.host_ms_wait_slots += now_ms() - t;
    }
    const bool timed = e->timing > 0 && e->block_index % e->timing == 0;
    if (timed) e->stats.timed_blocks++;
    if (timed) HIPCHK(hipEventRecord(S.a0, e->sA));

    // ---- waterfalls (stream A); row encoding + copy on the row slot's own stream
    // (every waterfall launch is timed when timing is on: batched launches are rare)
    RCCHK(run_waterfalls(e, blk, blk_start, blk_end, false, e->timing > 0, &S));
    e->last_blk = blk;
    e->last_start = blk_start;
    e->last_end = blk_end;
    // ---- chains: DDC per group (A); post_parallel + post_serial_front (B); ADPCM + copies (C)
    const double t_build = now_ms();
    std::vector<GroupWork>& work = e->work;
    work.clear();
    for (auto& gp : e->groups) {  // descriptors first, so the DDC bracket holds only kernels
        ChainGroup* g = gp.get();
        if (g->members.empty()) continue;
        if (blk_end < g->T) continue;
        const int64_t k_end = (blk_end - g->T) / g->D + 1;
        const int64_t nk64 = k_end - g->k_next;
        if (nk64 <= 0) continue;
        bool stale = g->chains_stale;
        for (size_t i = 0; i < g->members.size(); ++i) {
            Chain* c = e->chains[g->members[i]].get();
            if (c->rate_pending) {  // retune at output boundary k_next (phase continuous)
                const int64_t nb = std::max(g->k_next, c->k_first) * g->D;
                c->P0 = c->P0 + (uint64_t)(nb - c->n0) * c->rate_fx;
                c->n0 = nb;
                c->rate = c->new_rate;
                c->rate_fx = rate_to_fx(c->rate);
                c->rate_pending = false;
                RCCHK(fc_build_w(e, c, (int)i));
                stale = true;
            }
        }
        if (stale) {  // the group's DDC descriptors change only with its membership or a retune
            for (size_t i = 0; i < g->members.size(); ++i) {
                const Chain* c = e->chains[g->members[i]].get();
                DdcChain& d = g->h_chains[bp][i];
                d.rate_fx = c->rate_fx;
                d.wD = rate_rotator(c->rate, g->D);
                d.n0 = c->n0;
                d.P0 = c->P0;
            }
        }
        g->chains_stale = stale;  // consumed by this block's upload below
        // each caller block's outputs: those its own call would have produced
        FcSubs sb{};
        sb.n = std::max(1, std::min(nsub, kMaxSubBlocks));
        int64_t e_s = blk_start;
        for (int si = 0; si < sb.n; ++si) {
            e_s = si + 1 < sb.n ? e_s + sub_n[si] : blk_end;
            const int64_t ks = e_s < g->T ? g->k_next : (e_s - g->T) / g->D + 1;
            sb.nk[si] = (int)std::min(nk64, std::max<int64_t>(si ? sb.nk[si - 1] : 0, ks - g->k_next));
            sb.end[si] = e_s;
        }
        sb.nk[sb.n - 1] = (int)nk64;
        work.push_back(GroupWork{g, k_end, (int)nk64,
                                 g->fc_M != 0 && e->ddc_mode == OWRX_DDC_FAST, sb});
    }
    // the slot's post descriptors and lane lists: as built for its last block unless a chain
    // changed since (or the groups with outputs differ); then this block's nk / k_begin
    bool same_groups = S.post_groups.size() == work.size();
    for (size_t gi = 0; same_groups && gi < work.size(); ++gi) same_groups = S.post_groups[gi] == work[gi].g;
    if (S.post_dirty || S.post_epoch != e->chain_epoch || !same_groups) RCCHK(build_posts(e, S, si));
    // this block's group fields: post_parallel's StepTable argument (the slot's device posts are
    // reused as they are), or, past kMaxStepGroups groups, patched into every post
    StepTable steps;
    const bool use_steps = work.size() <= (size_t)kMaxStepGroups;
    for (size_t gi = 0; gi < work.size(); ++gi) {
        const GroupWork& gw = work[gi];
        const int nseg = gw.fast ? 1 : gw.g->nseg;
        if (use_steps) {
            steps.g[gi] = GroupStep{gw.g->k_next, gw.nk, nseg};
            continue;
        }
        ChainPost* p = S.h_posts + S.group_post0[gi];
        for (size_t i = 0; i < gw.g->members.size(); ++i) {
            p[i].nk = gw.nk;
            p[i].k_begin = gw.g->k_next;
            p[i].nseg = nseg;
        }
        S.dev_stale = true;
    }
    const int np = S.np;
    const double t_launch = now_ms();
    bool in_recorded = false;  // evIn of this block recorded (it doubles as the A -> B event)
    e->stats.host_ms_build += t_launch - t_build;
    // every descriptor of the block in one upload: the groups' DDC descriptors, the posts, the
    // serial lane lists and the long-bandpass list (stream B / C read them after stream A's
    // block event)
    {
        int nj = 0;
        int64_t maxb = 0;
        auto job = [&](void* dst, const void* src, int64_t bytes) {
            if (bytes <= 0) return;
            S.h_jobs[nj++] = CopyJob{dst, src, bytes};
            maxb = std::max(maxb, bytes);
        };
        for (const GroupWork& gw : work) {
            if (nj >= kMaxCopyJobs - 3) {  // many groups: flush this table
                hipLaunchKernelGGL(copy_jobs, dim3((unsigned)std::min<int64_t>(64, (maxb + 4095) / 4096), nj),
                                   dim3(256), 0, e->sA, S.h_jobs);
                HIPCHK(hipGetLastError());
                RCCHK(sync_stream(e, e->sA));  // the table is reused right away
                nj = 0;
                maxb = 0;
            }
            if (gw.g->chains_stale)
                job(gw.g->d_chains, gw.g->h_chains[bp], (int64_t)sizeof(DdcChain) * (int64_t)gw.g->members.size());
            gw.g->chains_stale = false;
        }
        if (S.dev_stale) {  // the slot's device posts and lane lists, when rebuilt
            job(S.d_posts, S.h_posts, (int64_t)sizeof(ChainPost) * np);
            job(S.d_sel, S.h_sel, (int64_t)sizeof(int) * S.nfill);
            job(S.d_sel + S.long_off, S.h_sel + S.long_off, (int64_t)sizeof(int) * (S.nlong + S.nafc));
            S.dev_stale = false;
        }
        if (nj > 0) {
            hipLaunchKernelGGL(copy_jobs, dim3((unsigned)std::min<int64_t>(64, (maxb + 4095) / 4096), nj),
                               dim3(256), 0, e->sA, S.h_jobs);
            HIPCHK(hipGetLastError());
        }
    }
    if (timed) {
        HIPCHK(hipEventRecord(S.a1, e->sA));
        S.timed_wf = !e->wfs.empty();
    }
    for (const GroupWork& gw : work) {
        ChainGroup* g = gw.g;
        const int64_t k_end = gw.k_end;
        const int nk = gw.nk;
        if (gw.fast) {
            // the first fast group's GEMM is timed (one group in the benchmark configurations)
            const bool tm = timed && !S.timed_mac;
            int form = 0;
            HIPCHK(launch_fc_ddc(g->fc_M, blk, blk_start, gw.sub,
                                 g->d_chains, g->d_fc_w,
                                 g->fc_Dp, g->fc_w_ks(), (int)g->members.size(), g->D, g->fc_Dp,
                                 g->fc_V, g->fc_Fs, g->k_next, nk, g->d_fc_tw, g->d_fc_u,
                                 g->d_fc_y, (int64_t)g->fc_y_elems, g->d_partial[si],
                                 std::max(1, e->cus_a), e->sA,
                                 tm ? S.m0 : nullptr,
                                 tm ? S.m1 : nullptr, &form));
            if (form > 0) e->stats.ddc_mac_lds_launches++;
            e->stats.ddc_mac_kslices_max = std::max<int64_t>(e->stats.ddc_mac_kslices_max, form);
            if (tm) {
                // algorithmic work of that GEMM: 8 flop per complex MAC over the frames that
                // carry outputs; bytes = W (every member's spectra) + U + Y, each moved once
                const double M = (double)g->fc_M;
                const double F = (double)fc_frames(gw.sub, g->fc_V);
                const double C = (double)g->members.size();
                e->stats.ddc_mac_flop += 8.0 * M * g->fc_Dp * C * F;
                e->stats.ddc_mac_bytes += 8.0 * M * g->fc_Dp * (C + F) + 8.0 * C * F * M;
                S.timed_mac = true;
            }
        } else
            HIPCHK(launch_ddc(g->P, blk, blk_start, blk_end, g->d_taps, g->d_chains,
                              (int)g->members.size(), g->D, g->k_next, nk, g->nseg,
                              g->d_partial[si], e->sA));
        e->stats.ddc_launches++;
        if (gw.fast) e->stats.ddc_fast_launches++;
        g->k_next = k_end;
    }
    if (timed) HIPCHK(hipEventRecord(S.a2, e->sA));
    if (np > 0) {
        // stream A: post_parallel (wide); stream B: post_serial_front (serial, own CUs)
        if (timed) HIPCHK(hipEventRecord(S.b0, e->sA));
        HIPCHK(launch_post_parallel(S.d_posts, np, S.d_counts, steps, e->sA));
        if (S.nlong > 0)  // long bandpass chains: bp_long + post_tail (after post_parallel)
            HIPCHK(launch_post_long(S.d_posts, S.d_counts, S.d_sel + S.long_off, S.nlong, S.long_fd,
                                    S.long_taps, e->sA));
        for (int lg = 0; lg < 32; ++lg)
            if (S.sf_sizes & (1u << lg)) HIPCHK(launch_chain_sfft(lg, S.d_posts, np, S.d_counts, e->sA));
        // stream A's last work of the block (the input's last reader too): one event serves both
        // stream B's wait and the input-retention check (evIn), one HIP call fewer per block
        HIPCHK(hipEventRecord(e->evIn[e->block_index % kInEv], e->sA));
        in_recorded = true;
        // serial streams for this block: the CU-masked pair, or past kWideSerialChains chains
        // (more waves than their CUs hold) the unmasked pair; on a switch the new pair first
        // waits for the old pair's last block, so every chain's state stays in block order
        const bool wide = np > wide_serial_chains();
        hipStream_t sB = wide ? e->sBw : e->sB, sC = wide ? e->sCw : e->sC;
        if (wide != e->serial_wide) {
            hipEvent_t fb, fc;
            HIPCHK(hipEventCreateWithFlags(&fb, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&fc, hipEventDisableTiming));
            HIPCHK(hipEventRecord(fb, e->serial_wide ? e->sBw : e->sB));
            HIPCHK(hipEventRecord(fc, e->serial_wide ? e->sCw : e->sC));
            HIPCHK(hipStreamWaitEvent(sB, fb, 0));
            HIPCHK(hipStreamWaitEvent(sC, fc, 0));
            HIPCHK(hipEventDestroy(fb));  // released once the waits are satisfied
            HIPCHK(hipEventDestroy(fc));
            e->serial_wide = wide;
        }
        HIPCHK(hipStreamWaitEvent(sB, e->evIn[e->block_index % kInEv], 0));
        // NoiseFilter resets the rebuild asked for (a fresh NoiseFilter: ClientAudioChain.
        // _updateConverter), on the serial stream in use, before this block's serial work
        for (Chain* c : e->nr_resets) {
            HIPCHK(hipMemsetAsync(c->d_nr_state, 0, sizeof(NrState), sB));
            HIPCHK(hipMemsetAsync(c->d_nr_in, 0, sizeof(float) * kNrHop, sB));
            HIPCHK(hipMemsetAsync(c->d_nr_pow, 0, sizeof(float) * 2 * (kNrN / 2 + 1), sB));
            HIPCHK(hipMemsetAsync(c->d_nr_ola, 0, sizeof(float) * kNrHop, sB));
        }
        e->nr_resets.clear();
        // SAm: Afc -> RealPart per chain (serial, lane per chain) ahead of the front
        if (S.nafc > 0) HIPCHK(launch_chain_afc(S.d_posts, S.d_counts, S.d_sel + S.afc_off, S.nafc, sB));
        const int dbg = (e->debug && S.d_dbg) ? 1 : 0;
        for (int o = 0; o < 3; ++o)
            for (int nr = 0; nr < 2; ++nr)
                HIPCHK(launch_post_serial(S.d_posts, S.d_counts, S.d_sel + S.off[o][nr],
                                          S.nsel[o][nr], o, dbg, nr, sB));
        if (S.any_nr) HIPCHK(launch_chain_nr(S.d_posts, np, S.d_counts, sB));
        HIPCHK(hipEventRecord(S.evF, sB));
        // stream C: ADPCM encoders (serial per chain, in block order) behind stream B's event.
        // (Round 4's in-kernel hand-off -- the encoder polling a flag stream B raised -- stalled
        // for its full 10 s bound and was removed in round 5: DESIGN.md §4, "A stall of our own".)
        HIPCHK(hipStreamWaitEvent(sC, S.evF, 0));
        const int nad = S.nsel[1][0] + S.nsel[1][1];
        HIPCHK(launch_chain_adpcm(S.d_posts, S.d_counts, S.d_sel + S.off[1][0], nad, sC));
        if (timed) HIPCHK(hipEventRecord(S.b1, sC));
        // the copies to host go on stream R (behind this block's encoder), so stream C runs
        // encoders back to back: its kernel is the pipeline's longest serial stage
        HIPCHK(hipEventRecord(S.evC, sC));
        HIPCHK(hipStreamWaitEvent(e->sR, S.evC, 0));
        hipLaunchKernelGGL(gather_outputs, dim3(np), dim3(256), 0, e->sR, S.d_posts, S.d_counts,
                           S.d_out, S.h_out, S.d_sm, S.h_sm, (int)e->sm_stride, S.h_counts);
        HIPCHK(hipGetLastError());
        S.debug = e->debug && S.d_dbg;
        if (S.debug)
            HIPCHK(hipMemcpyAsync(S.h_dbg, S.d_dbg, (size_t)np * kDebugStages * e->dbg_stride,
                                  hipMemcpyDeviceToHost, e->sR));
        HIPCHK(hipEventRecord(S.evB, e->sR));
        S.chains_pending = true;
    }
    if (timed) {
        HIPCHK(hipEventRecord(S.a3, e->sA));
        S.timed = true;
    }
    if (!in_recorded) HIPCHK(hipEventRecord(e->evIn[e->block_index % kInEv], e->sA));
    e->stats.host_ms_launch += now_ms() - t_launch;
    if (!wait_first) {  // the oldest input the caller may reuse now (see the top)
        const double t = now_ms();
        RCCHK(wait_input_block(e, e->block_index - in_keep(e)));
        e->stats.host_ms_wait_input += now_ms() - t;
    }
    e->pos = blk_end;
    e->stats.samples_in += n;
    e->stats.host_ms_process += now_ms() - t_enter;
    e->stats.blocks++;
    e->block_index++;
    // collect whatever earlier blocks have finished (B / C / R work overlaps later blocks)
    const double t_collect = now_ms();
    RCCHK(drain_slots(e, false, 0));
    RCCHK(drain_rows(e, false, 0));
    e->stats.host_ms_collect += now_ms() - t_collect;
    return OWRX_OK;
}

// the held caller blocks (owrx_set_block_group), contiguous, as one engine block
static int pair_flush(owrx_engine* e) {
    const float2* b = e->pend_blk;
    const int k = e->pend_k;
    const int64_t n = e->pend_total;
    int64_t sub[kMaxSubBlocks];
    for (int i = 0; i < k; ++i) sub[i] = e->pend_n[i];
    e->pend_k = 0;
    e->pend_total = 0;
    e->pend_blk = nullptr;
    return k > 0 ? process_block(e, b, n, k, sub) : OWRX_OK;
}

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------

#define ENGINE_GUARD_HELD(e)                                         \
    if (!(e)) {                                                      \
        set_last_error("null engine");                               \
        return OWRX_EINVAL;                                          \
    }                                                                \
    std::lock_guard<std::recursive_mutex> _lk((e)->mu);              \
    if ((e)->failed) {                                               \
        set_last_error((e)->stalled ? "engine failed earlier (GPU stalled)" \
                                    : "engine failed earlier (HIP error)"); \
        return (e)->stalled ? OWRX_ETIMEDOUT : OWRX_EIO;             \
    }                                                                \
    hipSetDevice((e)->device);

// every entry point except owrx_process_device, the reads and the stats: held caller blocks
// (owrx_set_block_group) run first, so the call sees the engine as after those blocks alone
#define ENGINE_GUARD(e)                                              \
    ENGINE_GUARD_HELD(e)                                             \
    if ((e)->pend_k > 0) {                                           \
        const int _prc = pair_flush(e);                              \
        if (_prc < 0) {                                              \
            if (_prc == OWRX_EIO || _prc == OWRX_ETIMEDOUT) (e)->failed = true; \
            return _prc;                                             \
        }                                                            \
    }

#define RC_FAIL(e, expr)                             \
    do {                                             \
        int _rc = (expr);                            \
        if (_rc < 0) {                               \
            if (_rc == OWRX_EIO || _rc == OWRX_ETIMEDOUT) (e)->failed = true; \
            return _rc;                              \
        }                                            \
    } while (0)

extern "C" {

const char* owrx_version(void) { return "0.18.99-amd"; }
const char* owrx_last_error(void) { return g_last_error.c_str(); }

int owrx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_last_error("no HIP device visible");
        return OWRX_ENODEV;
    }
    return n;
}

// Streams B, C and R run per-chain / per-row recurrences: a handful of waves whose speed is
// their own instruction issue, which halves when DDC waves share their SIMDs.  They get
// dedicated CUs (OWRX_SERIAL_CUS = "B,C,R,W" counts, default "4,4,4,4"; "0" = no masks) and
// stream A (FFT, DDC, post_parallel) the rest of the chip.  W: the waterfall row encoders'
// own CUs -- sharing R's, a batch of row encoders (one ~120 KiB-LDS workgroup per row, more
// rows than CUs) held the output gathers back by ~0.5 ms, and with them every slot's release.
static hipError_t create_streams(owrx_engine* e) {
    int ncu = 0;
    hipError_t err = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->device);
    if (err != hipSuccess) return err;
    for (hipStream_t* st : {&e->sBw, &e->sCw}) {
        err = hipStreamCreateWithFlags(st, hipStreamNonBlocking);
        if (err != hipSuccess) return err;
    }
    // B, C: the serial demodulator stages; R: the output gathers; W: the waterfall row encoders
    // B 8 and C 12 CUs: the serial one-lane-per-chain kernels are memory-latency bound, and
    // spread over more CUs they finish sooner (C3 6.0-6.3 -> 7.0 Gsps against 4 + 4; C4 and C5
    // +1.5-2 % with 8 + 8; A's 228 CUs cost the DDC GEMM nothing measurable:
    // profiles/r04_serial_cus_ab.txt)
    int nb = 8, nc = 12, nr = 4, nw = 4;
    if (const char* v = getenv("OWRX_SERIAL_CUS")) {
        const int k = sscanf(v, "%d,%d,%d,%d", &nb, &nc, &nr, &nw);
        if (k == 3) nw = 0;  // the row encoders share R's CUs (the round-2 layout)
        else if (k != 4) nb = nc = nr = 0;
    }
    e->cus_a = ncu;
    e->rows_grid = 2 * ncu;
    if (nb <= 0 || nc <= 0 || nr <= 0 || nw < 0 || nb + nc + nr + nw > ncu / 2) {
        for (hipStream_t* st : {&e->sA, &e->sB, &e->sC, &e->sR}) {
            err = hipStreamCreateWithFlags(st, hipStreamNonBlocking);
            if (err != hipSuccess) return err;
        }
        for (auto& r : e->rslots) {
            err = hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking);
            if (err != hipSuccess) return err;
        }
        return hipSuccess;
    }
    const int words = (ncu + 31) / 32;
    auto mask_range = [&](int lo, int hi) {  // CUs [lo, hi)
        std::vector<uint32_t> m((size_t)words, 0u);
        for (int c = lo; c < hi; ++c) m[(size_t)c / 32] |= 1u << (c % 32);
        return m;
    };
    const int a_end = ncu - nb - nc - nr - nw;
    e->cus_a = a_end;
    // the row encoder's grid: twice the row queue's CUs (measured: 2, 3, 4, 6, 8 workgroups on
    // its 4 CUs took 4.5, 3.1, 2.5, 1.8, 1.5 ms per batch against 1.4 with one per row, which
    // stalled stream R's gathers; profiles/r04_rows_grid_ab.txt).  OWRX_ROWS_GRID=rows: one
    // workgroup per row (the round-4 grid), =<n>: n (A/B)
    e->rows_grid = 2 * (nw > 0 ? nw : nr);
    if (const char* v = getenv("OWRX_ROWS_GRID")) e->rows_grid = strcmp(v, "rows") == 0 ? 0 : atoi(v);
    const std::vector<uint32_t> mA = mask_range(0, a_end);
    const std::vector<uint32_t> mB = mask_range(a_end, a_end + nb);
    const std::vector<uint32_t> mC = mask_range(a_end + nb, a_end + nb + nc);
    const std::vector<uint32_t> mR = mask_range(a_end + nb + nc, a_end + nb + nc + nr);
    std::vector<uint32_t> mW = nw > 0 ? mask_range(a_end + nb + nc + nr, ncu) : mR;
    // The row encoders may also use stream A's CUs, one workgroup per row, so a batch's rows (one
    // ~129 KiB-LDS workgroup each, near-serial per row) run side by side instead of eight at a
    // time on the row queue's own 4 CUs: a 35-row batch took ~2.4 ms there, and the last one
    // ended the 20-step C3 bench ~1.5 ms after the chain work (7 934-8 622 -> 9 373-9 555 Msps,
    // profiles/r05_rows_wide_ab.txt).  OWRX_ROWS_WIDE=0: the row queue's own CUs only (A/B).
    static const bool rows_wide = [] {
        const char* v = getenv("OWRX_ROWS_WIDE");
        return !(v && strcmp(v, "0") == 0);
    }();
    if (rows_wide) {
        const std::vector<uint32_t> mAw = mask_range(0, a_end);
        for (size_t i = 0; i < mW.size(); ++i) mW[i] |= mAw[i];
        if (!getenv("OWRX_ROWS_GRID")) e->rows_grid = 0;  // (an explicit grid still wins)
    }
    // Hardware queues and the command processor's pipes.  Every CU-masked stream is an HSA
    // queue of its own, and a process's queues are spread over the CP's four compute pipes in
    // creation order (measured: the 1st, 5th and 9th masked queue share one).  A queue holding a
    // cross-queue wait (hipStreamWaitEvent's barrier packet) slows the dispatch of a busy queue
    // on the same pipe: with the four row-slot queues created after A, B, C and R, every launch
    // whose rows went to the first of them (A's pipe) ran its waterfall FFT + finalize in
    // 0.15-0.20 ms instead of 0.072 and the following DDC launch up to 8x slower, and the
    // others (B's and C's pipes) slowed the serial stages (profiles/r04_pipe_layout_ab.txt).
    // So the row encoders get one queue, created first: it shares a pipe with R only (both
    // mostly waiting), and A, B and C each have a pipe to themselves.  All row slots encode on
    // it in order (~1 ms per 960-frame batch, one batch per ~2 ms at C3).  OWRX_ROW_STREAMS=4
    // restores the four row queues after R (A/B).
    static const int row_streams = [] {
        const char* v = getenv("OWRX_ROW_STREAMS");
        return v ? std::max(1, std::min(kRowSlots, atoi(v))) : 1;
    }();
    if (row_streams == 1) {
        err = hipExtStreamCreateWithCUMask(&e->rslots[0].stream, (uint32_t)words, mW.data());
        if (err != hipSuccess) return err;
    }
    const std::pair<hipStream_t*, const std::vector<uint32_t>*> sm[] = {
        {&e->sA, &mA}, {&e->sB, &mB}, {&e->sC, &mC}, {&e->sR, &mR}};
    // OWRX_MASK_A=0: stream A on every CU (the serial streams keep their own; A's waves may
    // then share their CUs) -- A/B of the CU mask's cost on A's full-chip kernels
    static const bool mask_a = [] {
        const char* v = getenv("OWRX_MASK_A");
        return !(v && strcmp(v, "0") == 0);
    }();
    for (auto& x : sm) {
        if (x.first == &e->sA && !mask_a) {
            err = hipStreamCreateWithFlags(x.first, hipStreamNonBlocking);
            e->cus_a = ncu;
        } else {
            err = hipExtStreamCreateWithCUMask(x.first, (uint32_t)words, x.second->data());
        }
        if (err != hipSuccess) return err;
    }
    for (int i = 0; i < kRowSlots; ++i) {
        auto& r = e->rslots[i];
        if (i >= row_streams) {
            r.stream = e->rslots[i % row_streams].stream;
            r.shared_stream = true;
        } else if (row_streams > 1) {
            err = hipExtStreamCreateWithCUMask(&r.stream, (uint32_t)words, mW.data());
            if (err != hipSuccess) return err;
        }
    }
    return hipSuccess;
}

int owrx_engine_create(int device, double samp_rate, int64_t max_block, owrx_engine** out) {
    return owrx_engine_create_ex(device, samp_rate, max_block, 0, out);
}

int owrx_engine_create_ex(int device, double samp_rate, int64_t max_block, int64_t history,
                          owrx_engine** out) {
    if (!out || samp_rate <= 0 || max_block <= 0) {
        set_last_error("owrx_engine_create: bad arguments");
        return OWRX_EINVAL;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        set_last_error("owrx_engine_create: device %d not available (%d visible)", device, n);
        return OWRX_ENODEV;
    }
    HIPCHK(hipSetDevice(device));
    (void)hipGetLastError();  // no stale error of an earlier engine on this thread
    owrx_engine* e = new owrx_engine();
    e->device = device;
    e->samp_rate = samp_rate;
    e->max_block = max_block;
    e->history = std::max<int64_t>(kDefaultHistory, (history + 255) & ~(int64_t)255);
    memset(&e->stats, 0, sizeof(e->stats));
    auto fail = [&](const char* what) {
        set_last_error("owrx_engine_create: %s", what);
        owrx_engine_destroy(e);
        return OWRX_EIO;
    };
    if (create_streams(e) != hipSuccess) return fail("stream");
    // Events that only order streams of this device (A -> B, B -> C, C -> R, A -> row queue) and
    // the input-retention poll (the host learns that stream A finished reading; it reads no data
    // through them) release at device scope; evB and the row slots' evC, after which the host
    // reads what the GPU wrote into pinned memory, keep the system-scope release.
    // OWRX_EVENT_FENCE=system: every event system-scope (A/B).
    static const unsigned dev_fence = [] {
        const char* v = getenv("OWRX_EVENT_FENCE");
        return (v && strcmp(v, "system") == 0) ? (unsigned)hipEventDisableTiming
                                               : (unsigned)(hipEventDisableTiming | hipEventDisableSystemFence);
    }();
    if (hipEventCreateWithFlags(&e->evSync, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->evExt, hipEventDisableTiming) != hipSuccess)
        return fail("event");
    for (auto& r : e->rslots) {
        if (hipEventCreateWithFlags(&r.evWf, dev_fence) != hipSuccess ||
            hipEventCreateWithFlags(&r.evC, hipEventDisableTiming) != hipSuccess)
            return fail("row stream");
    }
    for (auto& s : e->slots) {
        if (hipEventCreateWithFlags(&s.evA, dev_fence) != hipSuccess ||
            hipEventCreateWithFlags(&s.evF, dev_fence) != hipSuccess ||
            hipEventCreateWithFlags(&s.evB, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.evC, dev_fence) != hipSuccess ||
            // timing-only events: no system-scope fence, so the markers bracketing a kernel
            // do not add cache write-backs to the interval they measure
            hipEventCreateWithFlags(&s.a0, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.a1, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.a2, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.a3, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.b0, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.b1, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.m0, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.m1, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.w0, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&s.w1, hipEventDisableSystemFence) != hipSuccess)
            return fail("event");
    }
    // push-path ring: a lap holds >= 4 blocks past the history, so the per-lap move of the
    // history to the start never overlaps its source, and no block still read on stream A
    e->ring_cap = 2 * e->history + 4 * max_block;
    if (dalloc(&e->d_ring, (size_t)e->ring_cap) != hipSuccess) return fail("ring");
    if (hipMemset(e->d_ring, 0, sizeof(float2) * e->history) != hipSuccess) return fail("ring");
    e->wp = e->history;
    if (halloc(&e->h_in, 4 * (size_t)max_block) != hipSuccess) return fail("pinned input");
    for (hipEvent_t& ev : e->evIn)
        if (hipEventCreateWithFlags(&ev, dev_fence) != hipSuccess) return fail("event");
    *out = e;
    return OWRX_OK;
}

int owrx_engine_destroy(owrx_engine* e) {
    if (!e) return OWRX_EINVAL;
    hipSetDevice(e->device);
    if (getenv("OWRX_WF_LOG") && !e->wf_ms_log.empty()) {
        fprintf(stderr, "owrx waterfall launches (ms):");
        for (float v : e->wf_ms_log) fprintf(stderr, " %.3f", v);
        fprintf(stderr, "\n");
    }
    if (getenv("OWRX_HOST_LOG") && e->next_handle > 0)
        fprintf(stderr, "owrx chain create (ms over all creates): setup %.1f, buffers %.1f, bandpass %.1f, "
                "W %.1f, group %.1f, staging %.1f\n", e->cc_ms[0], e->cc_ms[1], e->cc_ms[2], e->cc_ms[3],
                e->cc_ms[4], e->cc_ms[5]);
    if (getenv("OWRX_HOST_LOG"))
        for (int k = 0; k < 2; ++k)
            fprintf(stderr, "owrx %s slot drains: %lld, wait %.3f ms, pushes %.3f ms (per drain %.4f / %.4f)\n",
                    k ? "forced" : "collect", (long long)e->hl_n[k], e->hl_wait[k], e->hl_push[k],
                    e->hl_n[k] ? e->hl_wait[k] / e->hl_n[k] : 0.0, e->hl_n[k] ? e->hl_push[k] / e->hl_n[k] : 0.0);
    // every stream drained, within the stall bound (a stalled engine gets one more bound to
    // finish; if its work still has not completed, its buffers are leaked rather than freed
    // under a running kernel, and the process keeps going)
    // The first stream still stuck after its bound ends the wait: the engine is leaked anyway,
    // and bounding every stream (or a shared row stream once per slot) in turn would block the
    // OpenWebRX process for many stall bounds.
    if (e->stalled) e->failed = false;
    std::vector<hipStream_t> streams = {e->sA, e->sB, e->sC, e->sR, e->sBw, e->sCw};
    for (auto& r : e->rslots)
        if (std::find(streams.begin(), streams.end(), r.stream) == streams.end()) streams.push_back(r.stream);
    for (hipStream_t st : streams)
        if (st && e->evSync && sync_stream(e, st) == OWRX_ETIMEDOUT) return OWRX_ETIMEDOUT;
    for (auto& kv : e->chains) free_chain(e, kv.second.get());
    for (auto& kv : e->wfs) free_wf(e, kv.second.get());
    for (auto& g : e->groups) {
        dfree(g->d_taps);
        dfree(g->d_h);
        dfree(g->d_fc_tw);
        dfree(g->d_fc_u);
        dfree(g->d_fc_y);
        prel(e, g->d_fc_w);
        dfree(g->d_chains);
        for (int i = 0; i < kSlots; ++i) dfree(g->d_partial[i]);
        for (auto& h : g->h_chains) hfree(h);
    }
    for (auto& kv : e->pool_size)  // the pool's buffers, in use or not (carved: in a slab)
        if (!e->pool_carved.count(kv.first)) hipFree(kv.first);
    for (void* sl : e->slabs) hipFree(sl);
    for (auto& kv : e->hpool_size) hipHostFree(kv.first);
    hfree(e->h_up);
    dfree(e->d_ring);
    dfree(e->d_cs16);
    hfree(e->h_in);
    for (hipEvent_t ev : e->evIn)
        if (ev) hipEventDestroy(ev);
    for (auto& s : e->slots) {
        free_slot_staging(s);
        hfree(s.h_jobs);
        for (hipEvent_t ev : {s.evA, s.evF, s.evB, s.evC, s.a0, s.a1, s.a2, s.a3, s.b0, s.b1, s.m0, s.m1,
                              s.w0, s.w1})
            if (ev) hipEventDestroy(ev);
    }
    for (auto& r : e->rslots) {
        if (r.evWf) hipEventDestroy(r.evWf);
        if (r.evC) hipEventDestroy(r.evC);
        if (r.stream && !r.shared_stream) hipStreamDestroy(r.stream);
    }
    for (hipStream_t st : {e->sA, e->sB, e->sC, e->sR, e->sBw, e->sCw})
        if (st) hipStreamDestroy(st);
    if (e->evSync) hipEventDestroy(e->evSync);
    if (e->evExt) hipEventDestroy(e->evExt);
    delete e;
    return OWRX_OK;
}

int64_t owrx_engine_history(owrx_engine* e) { return e ? e->history : OWRX_EINVAL; }

int owrx_set_pipeline_depth(owrx_engine* e, int blocks) {
    ENGINE_GUARD(e);
    // a chain created (and destroyed) before sized the per-slot staging for the old depth
    if (blocks < 1 || blocks > kSlots || e->block_index != 0 || !e->chains.empty() || e->post_cap > 0) {
        set_last_error("owrx_set_pipeline_depth: blocks must be in [1, %d], before the first "
                       "chain and block", kSlots);
        return OWRX_EINVAL;
    }
    e->nslots = blocks;
    return OWRX_OK;
}

int owrx_set_input_retention(owrx_engine* e, int blocks) {
    ENGINE_GUARD(e);
    if (blocks < 1 || blocks >= kInEv) {
        set_last_error("owrx_set_input_retention: blocks must be in [1, %d]", kInEv - 1);
        return OWRX_EINVAL;
    }
    // a grouping engine holds caller blocks until the group is complete: groups of g need
    // retention >= 2 g (owrx_set_block_group), so it may not be lowered below that afterwards
    if (e->group > 1 && blocks < 2 * e->group) {
        set_last_error("owrx_set_input_retention: block grouping of %d is on, blocks must be >= %d",
                       e->group, 2 * e->group);
        return OWRX_EINVAL;
    }
    e->retention = blocks;
    return OWRX_OK;
}
int64_t owrx_engine_max_block(owrx_engine* e) { return e ? e->max_block : OWRX_EINVAL; }

int owrx_selftest_w_layout(int Dp, int cap) {
    const int rc = fc_w_layout_check(Dp, cap);
    if (rc) set_last_error("owrx_selftest_w_layout(Dp=%d, cap=%d): %s", Dp, cap,
                           rc == -1 ? "not an engine geometry" : rc == -2 ? "entry outside the row"
                                                                          : "two entries on one element");
    return rc ? OWRX_EINVAL : OWRX_OK;
}

int owrx_set_stall_timeout(owrx_engine* e, int64_t ms) {
    ENGINE_GUARD(e);
    if (ms < 1) {
        set_last_error("owrx_set_stall_timeout: ms must be >= 1");
        return OWRX_EINVAL;
    }
    e->stall_ms = ms;
    return OWRX_OK;
}

int owrx_debug_stall(owrx_engine* e, int stream, int64_t us) {
    ENGINE_GUARD(e);
    hipStream_t st = stream == 0 ? e->sA : stream == 1 ? e->sB : stream == 2 ? e->sC
                   : stream == 3 ? e->sR : stream == 4 ? e->rslots[e->row_head % kRowSlots].stream
                   : nullptr;
    if (!st || us < 0 || us > 60000000) {
        set_last_error("owrx_debug_stall: stream 0..4, 0 <= us <= 60 s");
        return OWRX_EINVAL;
    }
    HIPCHK(launch_debug_sleep(us, st));
    return OWRX_OK;
}

// Stream A waits, on the GPU, for the work enqueued so far on the caller's stream (a collective
// that writes the next block's window: the broadcast of multi.IqBroadcast); no host wait.
int owrx_wait_stream(owrx_engine* e, void* stream) {
    ENGINE_GUARD_HELD(e);
    HIPCHK(hipEventRecord(e->evExt, (hipStream_t)stream));
    HIPCHK(hipStreamWaitEvent(e->sA, e->evExt, 0));
    return OWRX_OK;
}

int owrx_process_device(owrx_engine* e, const float* iq_dev, int64_t n) {
    ENGINE_GUARD_HELD(e);
    if (!iq_dev || n < 0 || n > e->max_block) {
        set_last_error("owrx_process_device: bad block (n=%lld, max %lld)", (long long)n,
                       (long long)e->max_block);
        return OWRX_EINVAL;
    }
    if (n == 0) return OWRX_OK;
    const float2* blk = (const float2*)iq_dev;
    if (e->group <= 1) {
        RC_FAIL(e, process_block(e, blk, n));
        return OWRX_OK;
    }
    // grouping: held blocks and this one, contiguous, run as one engine block once `group` of
    // them arrived; a block that does not follow the held ones runs them first, alone
    if (e->pend_k > 0 && blk != e->pend_blk + e->pend_total) RC_FAIL(e, pair_flush(e));
    if (e->pend_k == 0) e->pend_blk = blk;
    e->pend_n[e->pend_k++] = n;
    e->pend_total += n;
    if (e->pend_k >= e->group) {
        RC_FAIL(e, pair_flush(e));
        return OWRX_OK;
    }
    // input retention while held: the caller's block k - retention has been read.  The engine
    // blocks after the one holding it hold at least retention - pend_k - (group - 1) caller
    // blocks, at most `group` each, so engine block b - floor((retention - pend_k) / group)
    // covers it
    const double t = now_ms();
    RC_FAIL(e, wait_input_block(e, e->block_index - 1 - std::max(0, (e->retention - e->pend_k) / e->group)));
    e->stats.host_ms_wait_input += now_ms() - t;
    return OWRX_OK;
}

int owrx_set_block_group(owrx_engine* e, int blocks) {
    ENGINE_GUARD(e);
    // a grouping engine sizes its staging for `blocks` caller blocks: before the first chain and
    // block
    if (blocks < 1 || blocks > kMaxSubBlocks || e->block_index != 0 || !e->chains.empty() ||
        !e->wfs.empty() || e->post_cap > 0 || (blocks > 1 && e->retention < 2 * blocks)) {
        set_last_error("owrx_set_block_group: 1..%d, before the first chain, waterfall and "
                       "block, with input retention >= 2 x blocks", kMaxSubBlocks);
        return OWRX_EINVAL;
    }
    e->group = blocks;
    return OWRX_OK;
}

int owrx_set_block_pairing(owrx_engine* e, int enable) {
    if (e && (enable < 0 || enable > 1)) {
        set_last_error("owrx_set_block_pairing: 0 or 1");
        return OWRX_EINVAL;
    }
    return owrx_set_block_group(e, enable ? 2 : 1);
}

// Room for a block of n at the ring's write position: when it does not fit, the last `history`
// samples move to the ring's start on stream A (behind every kernel that read them).
static int ring_room(owrx_engine* e, int64_t n, bool* wrapped) {
    *wrapped = false;
    if (e->wp + n <= e->ring_cap) return OWRX_OK;
    HIPCHK(hipMemcpyAsync(e->d_ring, e->d_ring + (e->wp - e->history), sizeof(float2) * e->history,
                          hipMemcpyDeviceToDevice, e->sA));
    e->wp = e->history;
    *wrapped = true;
    return OWRX_OK;
}

int owrx_ingest_buffer(owrx_engine* e, float** dev_ptr, int64_t* capacity) {
    ENGINE_GUARD(e);
    if (!dev_ptr || !capacity) return OWRX_EINVAL;
    bool wrapped = false;
    RC_FAIL(e, ring_room(e, e->max_block, &wrapped));
    // the caller writes on a stream of its own: the move must be done first
    if (wrapped) RC_FAIL(e, sync_stream(e, e->sA));
    *dev_ptr = (float*)(e->d_ring + e->wp);
    *capacity = e->max_block;
    return OWRX_OK;
}

int owrx_commit(owrx_engine* e, int64_t n) {
    ENGINE_GUARD(e);
    if (n < 0 || n > e->max_block || e->wp + n > e->ring_cap) return OWRX_EINVAL;
    if (n == 0) return OWRX_OK;
    RC_FAIL(e, process_block(e, e->d_ring + e->wp, n));
    e->wp += n;
    return OWRX_OK;
}

int owrx_push_iq(owrx_engine* e, const float* iq, int64_t n) {
    ENGINE_GUARD(e);
    if (n < 0 || (n > 0 && !iq)) return OWRX_EINVAL;
    int64_t done = 0;
    while (done < n) {
        const int64_t m = std::min(n - done, e->max_block);
        // staging half (block parity) last used two blocks ago: its copy ran before that
        // block's stream-A work
        RC_FAIL(e, wait_input_block(e, e->block_index - 2));
        float* hb = e->h_in + 2 * (e->block_index & 1) * e->max_block;
        memcpy(hb, iq + 2 * done, sizeof(float2) * m);
        bool wrapped = false;
        RC_FAIL(e, ring_room(e, m, &wrapped));  // ordered with the copy below on stream A
        float2* dst = e->d_ring + e->wp;
        if (hipMemcpyAsync(dst, hb, sizeof(float2) * m, hipMemcpyHostToDevice, e->sA) !=
            hipSuccess) {
            e->failed = true;
            set_last_error("H2D copy failed");
            return OWRX_EIO;
        }
        int rc = owrx_commit(e, m);
        if (rc < 0) return rc;
        done += m;
    }
    return OWRX_OK;
}

int owrx_push_iq_cs16(owrx_engine* e, const int16_t* iq, int64_t n, float gain) {
    ENGINE_GUARD(e);
    if (n < 0 || (n > 0 && !iq)) return OWRX_EINVAL;
    if (n > 0 && !e->d_cs16) {
        if (dalloc(&e->d_cs16, 2 * (size_t)e->max_block) != hipSuccess) {
            set_last_error("cs16 staging allocation failed");
            return OWRX_ENOMEM;
        }
    }
    int64_t done = 0;
    while (done < n) {
        const int64_t m = std::min(n - done, e->max_block);
        // same staging discipline as owrx_push_iq (half the bytes per sample)
        RC_FAIL(e, wait_input_block(e, e->block_index - 2));
        int16_t* hb = reinterpret_cast<int16_t*>(e->h_in + 2 * (e->block_index & 1) * e->max_block);
        memcpy(hb, iq + 2 * done, 4 * (size_t)m);
        bool wrapped = false;
        RC_FAIL(e, ring_room(e, m, &wrapped));
        float* dst = reinterpret_cast<float*>(e->d_ring + e->wp);
        if (hipMemcpyAsync(e->d_cs16, hb, 4 * (size_t)m, hipMemcpyHostToDevice, e->sA) !=
            hipSuccess) {
            e->failed = true;
            set_last_error("H2D copy failed");
            return OWRX_EIO;
        }
        const int64_t pairs = (m + 1) / 2;
        hipLaunchKernelGGL(ingest_cs16, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, e->sA,
                           e->d_cs16, m, gain, dst);
        if (hipGetLastError() != hipSuccess) {
            e->failed = true;
            set_last_error("ingest_cs16 launch failed");
            return OWRX_EIO;
        }
        int rc = owrx_commit(e, m);
        if (rc < 0) return rc;
        done += m;
    }
    return OWRX_OK;
}

int owrx_sync(owrx_engine* e) {
    ENGINE_GUARD(e);
    // batched waterfalls: launch what is pending on the newest block's window (still valid:
    // owrx_process_device's contract, or the ring).  The flush stages its descriptors in the
    // next block's slot, so only that slot's previous block must have drained; the rest of the
    // pipeline (B's and C's last blocks) drains behind the flush instead of before it.
    RC_FAIL(e, flush_uploads(e));
    if (e->last_blk) {
        RC_FAIL(e, drain_slots(e, true, e->nslots - 1));
        RC_FAIL(e, run_waterfalls(e, e->last_blk, e->last_start, e->last_end, true, false, nullptr, true));
    }
    RC_FAIL(e, drain_all(e));
    return OWRX_OK;
}

// Chains per DDC group (see owrx_chain_create); OWRX_GROUP_CAP overrides (A/B).
static int group_cap() {
    static const int v = [] {
        const char* s = getenv("OWRX_GROUP_CAP");
        return s ? std::max(1, atoi(s)) : 16384;
    }();
    return v;
}

// ---- waterfall --------------------------------------------------------------------------

int owrx_waterfall_create(owrx_engine* e, int fft_size, int every_n_samples, int avg_number,
                          float add_db, int adpcm, int* handle) {
    ENGINE_GUARD(e);
    int logn = 0;
    while ((1 << logn) < fft_size) logn++;
    if (!handle || fft_size < 256 || fft_size > kWfMaxN || (1 << logn) != fft_size ||
        every_n_samples <= 0 || avg_number < 0) {
        set_last_error("owrx_waterfall_create: fft_size must be a power of two in [256, 65536], "
                       "every_n_samples > 0");
        return OWRX_EINVAL;
    }
    if ((int64_t)every_n_samples + fft_size > e->history) {
        set_last_error("owrx_waterfall_create: hop too large for engine history");
        return OWRX_EINVAL;
    }
    // no drain: the new FftChain's buffers come from the pools and its tables are uploaded on
    // stream A behind the blocks in flight (SpectrumThread restarts on an fft_size change,
    // owrx/fft.py:89-91, while every client keeps streaming)
    auto w = std::make_unique<Waterfall>();
    w->N = fft_size;
    w->logn = logn;
    w->hop = every_n_samples;
    w->avg = std::max(1, avg_number);
    w->adpcm = adpcm ? 1 : 0;
    w->add_db = add_db;
    w->next_start = e->pos;
    w->fpg = wf_frames_per_group(e, w.get());
    std::vector<float> win = hamming_window(fft_size);
    std::vector<float> tw = fft_twiddles(fft_size);
    int rc = OWRX_OK;
    auto setup = [&]() -> int {
        HIPCHK(palloc(e, &w->d_window, (size_t)fft_size));
        HIPCHK(palloc(e, &w->d_tw, (size_t)fft_size));
        HIPCHK(palloc(e, &w->d_work, 64));
        HIPCHK(palloc(e, &w->d_carry[0], (size_t)fft_size));
        HIPCHK(palloc(e, &w->d_carry[1], (size_t)fft_size));
        {
            // wf_fft_l32's claim and exit counters start at zero (the kernel's last workgroup
            // zeroes them again for the next launch)
            const int zero[2] = {0, 0};
            RCCHK(upload(e, w->d_work, zero, sizeof(zero)));
        }
        RCCHK(upload(e, w->d_window, win.data(), sizeof(float) * fft_size));
        RCCHK(upload(e, w->d_tw, tw.data(), sizeof(float) * 2 * fft_size));
        if (fft_size > kWfLdsMaxN) {
            const std::vector<float> ones(kWfLdsMaxN, 1.0f);
            HIPCHK(palloc(e, &w->d_ones, (size_t)kWfLdsMaxN));
            RCCHK(upload(e, w->d_ones, ones.data(), sizeof(float) * kWfLdsMaxN));
        }
        return wf_initial_reserve(e, w.get());
    };
    rc = setup();
    if (rc) {
        free_wf(e, w.get());
        return rc;
    }
    const int h = e->next_handle++;
    e->wfs[h] = std::move(w);
    *handle = h;
    return OWRX_OK;
}

int owrx_waterfall_set(owrx_engine* e, int handle, int every_n_samples, int avg_number,
                       int adpcm) {
    ENGINE_GUARD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end() || every_n_samples <= 0 || avg_number < 0) return OWRX_EINVAL;
    Waterfall* w = it->second.get();
    if ((int64_t)every_n_samples + w->N > e->history) return OWRX_EINVAL;
    // no drain: the new settings apply at the next row boundary (process_waterfall), blocks in
    // flight keep theirs, and launch buffers grow when a launch needs them (wf_reserve)
    w->new_hop = every_n_samples;
    w->new_avg = std::max(1, avg_number);
    w->new_adpcm = adpcm ? 1 : 0;
    if (w->row_frame == 0 && !w->carry_valid) {  // at a row boundary: apply now
        w->hop = w->new_hop;
        w->avg = w->new_avg;
        w->adpcm = w->new_adpcm;
        w->fpg = wf_frames_per_group(e, w);
        w->pending = false;
    } else {
        w->pending = true;
    }
    return wf_initial_reserve(e, w);
}

int owrx_waterfall_set_batch(owrx_engine* e, int handle, int min_frames, int64_t max_lag) {
    ENGINE_GUARD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end() || max_lag < 0) return OWRX_EINVAL;
    Waterfall* w = it->second.get();
    // the launch rule only: the groups (frames summed per workgroup) do not depend on it, so it
    // applies at once, mid-row and mid-stream, without a drain
    const int bmin = std::max(0, min_frames);
    // a deferred group must still fit the next block's window when its first frame leaves
    if (bmin > 1 && e->history < 2 * ((int64_t)w->fpg + 1) * w->hop + 2 * (int64_t)w->N) {
        set_last_error("owrx_waterfall_set_batch: engine history too short to batch (owrx_engine_create_ex)");
        return OWRX_EINVAL;
    }
    w->batch_min = bmin;
    w->batch_lag = max_lag;
    return wf_initial_reserve(e, w);
}

int owrx_waterfall_set_latency(owrx_engine* e, int handle, double max_wall_ms) {
    ENGINE_GUARD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end()) return OWRX_EINVAL;
    it->second->batch_wall_ms = max_wall_ms > 0 ? max_wall_ms : 0;
    return OWRX_OK;
}

int owrx_waterfall_destroy(owrx_engine* e, int handle) {
    ENGINE_GUARD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end()) return OWRX_EINVAL;
    // no drain: rows of it still in flight are dropped when their slot drains (drain_rows only
    // visits live waterfalls) and its buffers return to the pools once nothing can use them
    free_wf(e, it->second.get());
    e->wfs.erase(it);
    return OWRX_OK;
}

int owrx_waterfall_round_frames(owrx_engine* e, int handle) {
    ENGINE_GUARD_HELD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end()) return OWRX_EINVAL;
    return wf_round_frames(it->second->logn, std::max(1, e->cus_a), it->second->fpg);
}

int64_t owrx_waterfall_row_bytes(owrx_engine* e, int handle) {
    ENGINE_GUARD_HELD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end()) return OWRX_EINVAL;
    return it->second->row_bytes();
}

int64_t owrx_waterfall_read(owrx_engine* e, int handle, uint8_t* dst, int64_t max_bytes) {
    ENGINE_GUARD_HELD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end() || !dst || max_bytes < 0) return OWRX_EINVAL;
    Waterfall* w = it->second.get();
    const int64_t rb = w->row_bytes();
    const int64_t rows = std::min<int64_t>((int64_t)w->ring.avail() / rb, max_bytes / rb);
    return (int64_t)w->ring.pop(dst, (size_t)(rows * rb));
}

// ---- chains -----------------------------------------------------------------------------

static int64_t chain_nr_in_cap(const Chain* c) {
    return kNrHop + c->cap + c->prm.sq_length + 16 + kNrN;
}

// NoiseFilter buffers (first enable) and the engine's window / twiddle tables
static int chain_nr_alloc(owrx_engine* e, Chain* c) {
    if (!e->d_nr_win) {
        std::vector<float> w(kNrN);
        for (int i = 0; i < kNrN; ++i)
            w[i] = (float)std::sqrt(0.5 - 0.5 * std::cos(2.0 * M_PI * (double)i / kNrN));
        std::vector<float> tw = fft_twiddles(kNrN);
        HIPCHK(palloc(e, &e->d_nr_win, (size_t)kNrN));
        HIPCHK(palloc(e, &e->d_nr_tw, (size_t)kNrN));
        RCCHK(upload(e, e->d_nr_win, w.data(), sizeof(float) * kNrN));
        RCCHK(upload(e, e->d_nr_tw, tw.data(), sizeof(float) * 2 * kNrN));
    }
    if (!c->d_nr_state) {
        HIPCHK(palloc(e, &c->d_nr_state, 1));
        HIPCHK(palloc(e, &c->d_nr_in, (size_t)chain_nr_in_cap(c)));
        HIPCHK(palloc(e, &c->d_nr_pow, (size_t)2 * (kNrN / 2 + 1)));
        HIPCHK(palloc(e, &c->d_nr_ola, (size_t)kNrHop));
    }
    c->nr_reset = true;
    return OWRX_OK;
}

static int chain_validate(const owrx_chain_params* p) {
    if (p && p->output == OWRX_OUT_IQ)  // DDC only: the rest of the struct is unused
        return (p->decimation < 1 || p->transition <= 0 || p->cutoff <= 0 || p->frac_rate != 1.0)
                   ? OWRX_EINVAL : OWRX_OK;
    if (!p || p->decimation < 1 || p->transition <= 0 || p->cutoff <= 0 || p->frac_rate <= 0 ||
        p->sq_length <= 0 || p->sq_length > (1 << 20) || p->sq_decimation <= 0 || p->demod < 0 ||
        p->demod > OWRX_DEMOD_SAM || p->output < 0 || p->output > OWRX_OUT_SEL ||
        p->output == OWRX_OUT_IQ || p->audio_rate <= 0 ||
        p->agc_profile < 0 || p->agc_profile > 3)
        return OWRX_EINVAL;
    if (p->output == OWRX_OUT_SEL && (p->demod == OWRX_DEMOD_WFM || p->nr_enabled))
        return OWRX_EINVAL;
    if (p->demod == OWRX_DEMOD_WFM && (p->if_rate <= 0 || p->if_rate / p->audio_rate < 1.0))
        return OWRX_EINVAL;
    if (p->bandpass && (p->bp_transition <= 0 || p->bp_low >= p->bp_high)) return OWRX_EINVAL;
    if (p->demod == OWRX_DEMOD_SAM &&
        (p->afc_update <= 0 || p->afc_sample <= 0 || p->output == OWRX_OUT_SEL))
        return OWRX_EINVAL;
    if (p->audio_gain < 0 || (p->audio_gain > 0 && p->demod != OWRX_DEMOD_AM &&
                              p->demod != OWRX_DEMOD_SAM))
        return OWRX_EINVAL;
    return OWRX_OK;
}

static int chain_set_bandpass_taps(owrx_engine* e, Chain* c) {
    if (!c->prm.bandpass) return OWRX_OK;
    const int T = firdes_filter_len(c->prm.bp_transition);
    if (T > c->bp_hist + 1 || T > kBlMaxTaps) {
        set_last_error("bandpass transition too narrow (%d taps > %d)", T,
                       std::min(c->bp_hist + 1, kBlMaxTaps));
        return OWRX_EINVAL;
    }
    std::vector<float> taps = firdes_bandpass_c(T, c->prm.bp_low, c->prm.bp_high);
    // no drain: the bandpass FIR runs on stream A (post_parallel / bp_long), so blocks enqueued
    // before this copy filter with the old taps and every later block with the new ones
    if (!c->d_bp_taps) HIPCHK(palloc(e, &c->d_bp_taps, (size_t)c->bp_hist + 1));
    RCCHK(upload(e, c->d_bp_taps, taps.data(), sizeof(float) * 2 * T));
    c->bp_ntaps = T;
    return OWRX_OK;
}

int owrx_chain_create(owrx_engine* e, const owrx_chain_params* p, int* handle) {
    ENGINE_GUARD(e);
    double tcc = now_ms();
    auto lap = [&](int k) {
        const double t = now_ms();
        e->cc_ms[k] += t - tcc;
        tcc = t;
    };
    e->chain_epoch++;  // the slots rebuild their post descriptors
    if (!handle || chain_validate(p)) {
        set_last_error("owrx_chain_create: invalid chain parameters");
        return OWRX_EINVAL;
    }
    const int D = p->decimation;
    const int T = firdes_filter_len(p->transition);
    if (T + D > e->history) {
        set_last_error("owrx_chain_create: FIR (%d taps) longer than engine history", T);
        return OWRX_EINVAL;
    }
    const int P = ddc_padded_p((T + D - 1) / D);
    if (P < 0) {
        set_last_error("owrx_chain_create: polyphase depth %d unsupported", (T + D - 1) / D);
        return OWRX_EINVAL;
    }
    // no drain: the new chain starts at the next block (its origin is past every block in
    // flight); its buffers come from the pool and are initialised on stream A
    // group lookup by (D, transition, cutoff)
    uint32_t tb, cb;
    memcpy(&tb, &p->transition, 4);
    memcpy(&cb, &p->cutoff, 4);
    // A group holds at most group_cap() chains; past that the design opens another group.  The
    // filter spectra W of a group double as it grows and a regrown W returns to the engine's
    // exact-size pool, so one unbounded group kept every earlier capacity allocated (131 072
    // chains: ~115 GB of dead spectra) and needed old + new W at once; bounded groups grow
    // through the same sizes, reusing each other's pooled buffers (tools/dbg/mem_per_chain.py)
    ChainGroup* g = nullptr;
    for (auto& gp : e->groups)
        if (gp->D == D && gp->tbw_bits == tb && gp->cutoff_bits == cb &&
            (int)gp->members.size() < group_cap())
            g = gp.get();
    const int64_t aligned = ((e->pos + D - 1) / D) * D;
    if (!g) {
        auto ng = std::make_unique<ChainGroup>();
        ng->D = D;
        ng->T = T;
        ng->P = P;
        ng->tbw_bits = tb;
        ng->cutoff_bits = cb;
        // FirDecimate lowpass at cutoff/D (csdr LowPassFilter(cutoff / decimation, ...))
        const float fc = p->cutoff / (float)D;
        std::vector<float> h = firdes_lowpass(T, (double)fc);
        std::vector<float> poly((size_t)D * P, 0.0f);
        for (int r = 0; r < D; ++r)
            for (int q = 0; q < P; ++q) {
                const int64_t t = (int64_t)q * D + r;
                if (t < T) poly[(size_t)r * P + q] = h[t];
            }
        HIPCHK(dalloc(&ng->d_taps, poly.size()));
        HIPCHK(hipMemcpy(ng->d_taps, poly.data(), sizeof(float) * poly.size(),
                         hipMemcpyHostToDevice));
        // fast-convolution form: frame length, branch padding, U and twiddles
        ng->fc_P = (T + D - 1) / D;
        // the frame length from the caller's block (a paired engine keeps the unpaired design)
        const int64_t nk_max = e->max_block / D + 4;
        ng->fc_M = ng->fc_P <= 64 ? fc_choose_m(D, ng->fc_P, nk_max) : 0;
        if (const char* v = getenv("OWRX_FC_M")) {  // A/B: force the frame length
            const int m = atoi(v);
            if (ng->fc_M && fc_frame_supported(m) && m - ng->fc_P + 1 >= m / 2) ng->fc_M = m;
        }
        e->stats.ddc_frame_length = ng->fc_M;
        if (ng->fc_M) {
            const int M = ng->fc_M;
            ng->fc_V = M - ng->fc_P + 1;
            ng->fc_Dp = (D + 95) / 96 * 96;  // kFcDpAlign (kernels_fcddc.hip)
            // frames of the largest engine block; a pair cuts its frames at the caller blocks'
            // boundary, one frame more
            const int64_t nk_proc = proc_block(e) / D + 4;
            ng->fc_Fs = (int)((nk_proc + ng->fc_V - 1) / ng->fc_V + (e->group - 1) + 15) & ~15;
            HIPCHK(dalloc(&ng->d_h, (size_t)T));
            HIPCHK(hipMemcpy(ng->d_h, h.data(), sizeof(float) * T, hipMemcpyHostToDevice));
            std::vector<float> tw = fft_twiddles(M);
            HIPCHK(dalloc(&ng->d_fc_tw, (size_t)M));
            HIPCHK(hipMemcpy(ng->d_fc_tw, tw.data(), sizeof(float) * 2 * M, hipMemcpyHostToDevice));
            HIPCHK(dalloc(&ng->d_fc_u, (size_t)M * ng->fc_Fs * ng->fc_Dp));
            if (getenv("OWRX_VERBOSE"))
                fprintf(stderr, "owrx: DDC group D=%d T=%d: fast convolution M=%d V=%d Fs=%d\n",
                        D, T, M, ng->fc_V, ng->fc_Fs);
        }
        ng->k_next = aligned / D;
        e->groups.push_back(std::move(ng));
        g = e->groups.back().get();
    } else if (g->members.empty()) {
        g->k_next = std::max(g->k_next, aligned / D);
    }
    auto c = std::make_unique<Chain>();
    c->prm = *p;
    c->group = g;
    c->origin = std::max(aligned, g->k_next * (int64_t)D);
    c->k_first = c->origin / D;
    c->n0 = c->origin;
    c->P0 = 0;
    c->rate = p->shift_rate;
    c->rate_fx = rate_to_fx(p->shift_rate);
    c->cap = chain_stage_cap(e, D, p->frac_rate);
    const int64_t scap = c->cap + p->sq_length + 16;
    // output staging per block by output type: the encoder input holds up to scap + 160 + kNrN
    // samples (d_s16: a NoiseFilter emits up to a frame more than its input); ADPCM writes half a
    // byte per sample plus an 8-B sync frame per 1001 bytes (sizing every output at 4 B per
    // sample made 98 304 ADPCM chains allocate ~6x the pinned staging they use)
    const int64_t an = scap + 160 + kNrN;
    c->out_cap = p->output == OWRX_OUT_IQ    ? 8 * c->cap + 64
                 : p->output == OWRX_OUT_SEL ? 8 * scap + 64
                 : p->output == OWRX_OUT_ADPCM ? an / 2 + 1 + 8 * (an / 2 / kAdpcmSyncPeriod + 2) + 64
                 : p->output == OWRX_OUT_S16 ? 2 * an + 64
                                             : 4 * an + 64;
    c->sm_cap = p->output == OWRX_OUT_IQ ? 4 : (int)(scap / p->sq_length + 4);
    // the host rings: room for three blocks' outputs (the reader drains once per block; a drain
    // may land two or three blocks first)
    // (at most 1 MiB each: an IQ chain's block can be hundreds of KB)
    c->audio.prime(std::min<size_t>((size_t)(3 * c->out_cap), 1u << 20));
    c->smeter.prime(std::min<size_t>(3 * sizeof(float) * (size_t)c->sm_cap, 1u << 20));
    if (p->output != OWRX_OUT_IQ && scap / p->sq_length + 2 > 1024) {  // kMaxSqBlocks
        set_last_error("owrx_chain_create: squelch length %d too short for the block size",
                       p->sq_length);
        return OWRX_EINVAL;
    }
    // a bandpass design longer than the in-kernel FIR's history runs in bp_long (WFM)
    if (p->bp_transition > 0 && p->output != OWRX_OUT_IQ) {
        c->bp_design_taps = firdes_filter_len(p->bp_transition);
        if (c->bp_design_taps > kBlMaxTaps) {
            set_last_error("owrx_chain_create: bandpass of %d taps > %d", c->bp_design_taps,
                           kBlMaxTaps);
            return OWRX_EINVAL;
        }
        if (c->bp_design_taps - 1 > kBpHist) c->bp_hist = (c->bp_design_taps - 1 + 255) & ~255;
    }
    lap(0);
    ChainStateP ps;
    memset(&ps, 0, sizeof(ps));
    ChainStateS ss;
    memset(&ss, 0, sizeof(ss));
    AgcParams ap = agc_profile(p->agc_profile);
    if (p->agc_initial_gain >= 0) ap.initial_gain = p->agc_initial_gain;
    ss.agc.env = ap.reference / ap.initial_gain;
    HIPCHK(palloc(e, &c->d_pstate, 1));
    HIPCHK(palloc(e, &c->d_sstate, 1));
    RCCHK(upload(e, c->d_pstate, &ps, sizeof(ps)));
    RCCHK(upload(e, c->d_sstate, &ss, sizeof(ss)));
    HIPCHK(palloc(e, &c->d_ddc, (size_t)(kFdHist + c->cap)));
    HIPCHK(palloc(e, &c->d_fd, (size_t)(c->bp_hist + c->cap)));
    if (p->demod == OWRX_DEMOD_WFM && p->output != OWRX_OUT_IQ) {
        // FractionalDecimator(FLOAT, if_rate / audio_rate, prefilter=True): prefilter lowpass
        // at 0.5 / rate (output Nyquist), transition 0.03 (csdr's default; recalled, unpinned)
        const double r = p->if_rate / (double)p->audio_rate;
        c->pf_ntaps = firdes_filter_len(0.03f);
        std::vector<float> pf = firdes_lowpass(c->pf_ntaps, 0.5 / r);
        HIPCHK(palloc(e, &c->d_pf_taps, (size_t)c->pf_ntaps));
        RCCHK(upload(e, c->d_pf_taps, pf.data(), sizeof(float) * pf.size()));
        HIPCHK(palloc(e, &c->d_wf, (size_t)(kWfHist + scap)));
        HIPCHK(palloc(e, &c->d_pf, (size_t)(kWfHist + scap)));
    }
    HIPCHK(palloc(e, &c->d_sq, (size_t)scap));
    // slack: the serial kernels read whole 64-sample chunks / 8-sample prefetches unguarded
    // (SAm: the Selector output, cf32, until chain_afc leaves the RealPart in place)
    const size_t dem_n = (p->demod == OWRX_DEMOD_SAM ? 2 : 1) * ((size_t)scap + 160);
    for (int i = 0; i < e->nslots; ++i) HIPCHK(palloc(e, &c->d_dem[i], dem_n));
    // + kNrN: a NoiseFilter emits up to one frame more than its input per step
    for (int i = 0; i < e->nslots; ++i) HIPCHK(palloc(e, &c->d_s16[i], (size_t)scap + 160 + kNrN));
    lap(1);
    int rc = chain_set_bandpass_taps(e, c.get());
    if (!rc && p->nr_enabled && p->output != OWRX_OUT_IQ) rc = chain_nr_alloc(e, c.get());
    if (rc) {
        free_chain(e, c.get());
        return rc;
    }
    lap(2);
    if (g->fc_M) {
        int wrc = fc_reserve(e, g, (int)g->members.size() + 1);
        if (!wrc)  // built with the next flush, batched with the other joins (flush_wbuilds)
            g->w_pending.push_back(FcWJob{c->rate_fx, fc_w_chain_offset((int)g->members.size(), g->fc_Dp)});
        if (wrc) {
            free_chain(e, c.get());
            return wrc;
        }
    }
    lap(3);
    const int h = e->next_handle++;
    g->members.push_back(h);
    g->chains_stale = true;
    e->need_out += c->staging_bytes();
    e->need_sm = std::max<int64_t>(e->need_sm, c->sm_cap);
    // squelch / demod debug taps hold up to cap + sq_length samples per step
    e->need_dbg = std::max<int64_t>(e->need_dbg, (c->cap + c->prm.sq_length + 16) * 8 + 64);
    e->chains[h] = std::move(c);
    RC_FAIL(e, group_refresh_device(e, g));
    lap(4);
    RC_FAIL(e, ensure_post_capacity(e));
    lap(5);
    *handle = h;
    return OWRX_OK;
}

int owrx_chain_destroy(owrx_engine* e, int handle) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    // no drain: blocks in flight keep their descriptors (their outputs for this chain are
    // dropped at drain_slot), its buffers return to the pool once those blocks have drained,
    // and the spectra move below runs on stream A behind their DDC
    ChainGroup* g = it->second->group;
    // swap-remove: the last member takes the slot (and its filter spectra move with it)
    const int slot = (int)(std::find(g->members.begin(), g->members.end(), handle) - g->members.begin());
    const int last = (int)g->members.size() - 1;
    // pending spectra builds run first: before the last member's rows move, and before a later
    // join's build can target this slot (one fc_make_w_jobs launch does not order two jobs on
    // the same slot)
    if (!g->w_pending.empty()) RC_FAIL(e, flush_uploads(e));
    if (slot != last && g->fc_M) {
        HIPCHK(launch_fc_move_w(g->fc_M, g->d_fc_w, g->fc_w_ks(), g->fc_Dp, last, slot, e->sA));
    }
    g->members[slot] = g->members[last];
    g->members.pop_back();
    g->chains_stale = true;
    e->need_out -= it->second->staging_bytes();
    free_chain(e, it->second.get());
    e->chains.erase(it);
    if (!g->members.empty()) RC_FAIL(e, group_refresh_device(e, g));
    return OWRX_OK;
}

int owrx_chain_set_shift_rate(owrx_engine* e, int handle, float rate) {
    ENGINE_GUARD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    it->second->new_rate = rate;
    it->second->rate_pending = true;
    it->second->prm.shift_rate = rate;
    return OWRX_OK;
}

int owrx_chain_set_bandpass(owrx_engine* e, int handle, int enabled, float low, float high) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    Chain* c = it->second.get();
    if (enabled && low >= high) return OWRX_EINVAL;
    if (enabled && c->prm.bp_transition <= 0) return OWRX_EINVAL;
    c->prm.bandpass = enabled ? 1 : 0;
    c->prm.bp_low = low;
    c->prm.bp_high = high;
    RC_FAIL(e, chain_set_bandpass_taps(e, c));
    return OWRX_OK;
}

int owrx_chain_set_squelch_level(owrx_engine* e, int handle, float level) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    it->second->prm.sq_level = level;
    return OWRX_OK;
}

int owrx_chain_set_noise_filter(owrx_engine* e, int handle, int enabled, float threshold_db) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || it->second->prm.output == OWRX_OUT_IQ) return OWRX_EINVAL;
    Chain* c = it->second.get();
    if (enabled) RC_FAIL(e, chain_nr_alloc(e, c));
    c->prm.nr_enabled = enabled ? 1 : 0;
    c->prm.nr_threshold = threshold_db;
    return OWRX_OK;
}

int64_t owrx_chain_read_audio(owrx_engine* e, int handle, uint8_t* dst, int64_t max_bytes) {
    ENGINE_GUARD_HELD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || !dst || max_bytes < 0) return OWRX_EINVAL;
    return (int64_t)it->second->audio.pop(dst, (size_t)max_bytes);
}

int64_t owrx_chain_read_smeter(owrx_engine* e, int handle, float* dst, int64_t max_values) {
    ENGINE_GUARD_HELD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || !dst || max_values < 0) return OWRX_EINVAL;
    return (int64_t)it->second->smeter.pop((uint8_t*)dst, sizeof(float) * (size_t)max_values) /
           (int64_t)sizeof(float);
}

// A handle listed twice would have two host workers pop one ring at once: rejected (serial
// O(n) pass over the chains the lookups found)
static bool batched_duplicates(owrx_engine* e, const std::vector<Chain*>& cs) {
    const uint64_t ep = ++e->read_epoch;
    for (Chain* c : cs) {
        if (c->read_mark == ep) {
            set_last_error("owrx_chains_read_*: a chain handle is listed twice");
            return true;
        }
        c->read_mark = ep;
    }
    return false;
}

int64_t owrx_chains_read_audio(owrx_engine* e, int n, const int* handles, uint8_t* dst,
                               int64_t max_bytes, int64_t* lens) {
    ENGINE_GUARD_HELD(e);
    const bool query = !dst && max_bytes == 0;  // size query: nothing is read
    if (n < 0 || (n > 0 && (!handles || (!dst && !query) || !lens)) || max_bytes < 0) return OWRX_EINVAL;
    // sizes first (each chain's ring, on the host workers), offsets (in order, up to max_bytes),
    // then the copies (workers again)
    std::vector<Chain*> cs((size_t)n);
    std::atomic<bool> bad{false};
    for_range(e, n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            auto it = e->chains.find(handles[i]);
            if (it == e->chains.end()) { bad = true; continue; }
            cs[i] = it->second.get();
            lens[i] = (int64_t)cs[i]->audio.avail();
        }
    });
    if (bad || batched_duplicates(e, cs)) return OWRX_EINVAL;
    if (query) {
        int64_t total = 0;
        for (int i = 0; i < n; ++i) total += lens[i];
        return total;
    }
    std::vector<int64_t> offs((size_t)n);
    int64_t off = 0;
    for (int i = 0; i < n; ++i) {
        lens[i] = std::min(lens[i], max_bytes - off);
        offs[i] = off;
        off += lens[i];
    }
    for_range(e, n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) cs[i]->audio.pop(dst + offs[i], (size_t)lens[i]);
    });
    return off;
}

int64_t owrx_chains_read_smeter(owrx_engine* e, int n, const int* handles, float* dst,
                                int64_t max_values, int64_t* counts) {
    ENGINE_GUARD_HELD(e);
    const bool query = !dst && max_values == 0;  // size query: nothing is read
    if (n < 0 || (n > 0 && (!handles || (!dst && !query) || !counts)) || max_values < 0) return OWRX_EINVAL;
    std::vector<Chain*> cs((size_t)n);
    std::atomic<bool> bad{false};
    for_range(e, n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            auto it = e->chains.find(handles[i]);
            if (it == e->chains.end()) { bad = true; continue; }
            cs[i] = it->second.get();
            counts[i] = (int64_t)(cs[i]->smeter.avail() / sizeof(float));
        }
    });
    if (bad || batched_duplicates(e, cs)) return OWRX_EINVAL;
    if (query) {
        int64_t total = 0;
        for (int i = 0; i < n; ++i) total += counts[i];
        return total;
    }
    std::vector<int64_t> offs((size_t)n);
    int64_t off = 0;
    for (int i = 0; i < n; ++i) {
        counts[i] = std::min(counts[i], max_values - off);
        offs[i] = off;
        off += counts[i];
    }
    for_range(e, n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i)
            cs[i]->smeter.pop((uint8_t*)(dst + offs[i]), sizeof(float) * (size_t)counts[i]);
    });
    return off;
}

int owrx_chain_set_taps(owrx_engine* e, int handle, int selector, int audio) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    Chain* c = it->second.get();
    if (c->prm.output == OWRX_OUT_IQ && (selector || audio)) {
        set_last_error("owrx_chain_set_taps: the chain has no Selector output / audio");
        return OWRX_EINVAL;
    }
    // no drain: the slots in flight were built with the old layout (drain_slot uses theirs)
    const int64_t scap = c->cap + c->prm.sq_length + 16;  // samples per step, as the staging
    e->need_out -= c->staging_bytes();
    c->tap_sq_cap = selector ? 8 * scap : 0;
    c->tap_agc_cap = audio ? 4 * scap : 0;
    e->need_out += c->staging_bytes();
    c->tap_gen++;
    if (!selector) c->tap_sel.clear();
    if (!audio) c->tap_audio.clear();
    RC_FAIL(e, ensure_post_capacity(e));
    return OWRX_OK;
}

int64_t owrx_chain_read_tap(owrx_engine* e, int handle, int which, uint8_t* dst,
                            int64_t max_bytes) {
    ENGINE_GUARD_HELD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || !dst || max_bytes < 0 || which < 0 || which > 1)
        return OWRX_EINVAL;
    ByteRing& r = which == 0 ? it->second->tap_sel : it->second->tap_audio;
    const size_t item = which == 0 ? 8 : 4;
    const size_t n = std::min<size_t>((size_t)max_bytes, r.avail()) / item * item;
    return (int64_t)r.pop(dst, n);
}

int owrx_chain_set_secondary_fft(owrx_engine* e, int handle, int fft_size, int every_n_samples,
                                 int avg_number, float add_db, int adpcm) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    Chain* c = it->second.get();
    int logn = 0;
    while ((1 << logn) < fft_size) logn++;
    if (fft_size != 0 && (fft_size < 1024 || fft_size > 8192 || (1 << logn) != fft_size ||
                          every_n_samples <= 0 || avg_number < 0 ||
                          c->prm.output == OWRX_OUT_IQ)) {
        set_last_error("owrx_chain_set_secondary_fft: fft_size must be 0 or a power of two in "
                       "[1024, 8192], every_n_samples > 0, on an audio chain");
        return OWRX_EINVAL;
    }
    // no drain: the old buffers go back to the pool once the blocks in flight (built with
    // them) have drained; rows those blocks still produce are dropped (sf_gen)
    e->need_out -= c->staging_bytes();
    if (fft_size != c->sf_n) {
        prel(e, c->d_sf);
        prel(e, c->d_sf_acc);
        prel(e, c->d_sf_window);
        prel(e, c->d_sf_tw);
        c->sf_n = 0;
        c->sf_out_cap = 0;
        if (fft_size > 0) {
            const int64_t scap = c->cap + c->prm.sq_length + 16;
            HIPCHK(palloc(e, &c->d_sf, (size_t)(fft_size + scap + 64)));
            HIPCHK(palloc(e, &c->d_sf_acc, (size_t)fft_size));
            HIPCHK(palloc(e, &c->d_sf_window, (size_t)fft_size));
            HIPCHK(palloc(e, &c->d_sf_tw, (size_t)fft_size));
            std::vector<float> win = hamming_window(fft_size);
            std::vector<float> tw = fft_twiddles(fft_size);
            RCCHK(upload(e, c->d_sf_window, win.data(), sizeof(float) * fft_size));
            RCCHK(upload(e, c->d_sf_tw, tw.data(), sizeof(float) * 2 * fft_size));
        }
    }
    c->sf_gen++;
    c->sf_n = fft_size;
    c->sf_logn = logn;
    c->sf_hop = every_n_samples;
    c->sf_avg = avg_number;
    c->sf_add_db = add_db;
    c->sf_adpcm = adpcm ? 1 : 0;
    c->sf_reset = true;
    c->sfft.clear();
    if (fft_size > 0) {
        // rows per step: frames over (carried < N) + this step's samples, one row per avg frames
        const int64_t scap = c->cap + c->prm.sq_length + 16;
        const int64_t frames = (scap + fft_size) / every_n_samples + 2;
        const int64_t rows = frames / std::max(1, avg_number) + 2;
        c->sf_out_cap = rows * c->sf_row_bytes();
    }
    e->need_out += c->staging_bytes();
    RC_FAIL(e, ensure_post_capacity(e));
    return OWRX_OK;
}

int64_t owrx_chain_secondary_fft_row_bytes(owrx_engine* e, int handle) {
    ENGINE_GUARD_HELD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || it->second->sf_n == 0) return OWRX_EINVAL;
    return it->second->sf_row_bytes();
}

int64_t owrx_chain_read_secondary_fft(owrx_engine* e, int handle, uint8_t* dst,
                                      int64_t max_bytes) {
    ENGINE_GUARD_HELD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || !dst || max_bytes < 0) return OWRX_EINVAL;
    Chain* c = it->second.get();
    if (c->sf_n == 0) return 0;
    const int64_t rb = c->sf_row_bytes();
    return (int64_t)c->sfft.pop(dst, (size_t)((max_bytes / rb) * rb));
}

int64_t owrx_chain_origin(owrx_engine* e, int handle) {
    ENGINE_GUARD_HELD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    return it->second->origin;
}

int owrx_set_debug(owrx_engine* e, int enable) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    RC_FAIL(e, drain_all(e));
    e->debug = enable != 0;
    e->post_cap = 0;  // force reallocation with debug staging
    RC_FAIL(e, ensure_post_capacity(e));
    return OWRX_OK;
}

int64_t owrx_chain_read_debug(owrx_engine* e, int handle, int stage, void* dst,
                              int64_t max_bytes) {
    ENGINE_GUARD_HELD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || stage < 0 || stage >= kDebugStages || !dst || max_bytes < 0)
        return OWRX_EINVAL;
    return (int64_t)it->second->dbg[stage].pop((uint8_t*)dst, (size_t)max_bytes);
}

int owrx_get_stats(owrx_engine* e, owrx_stats* s) {
    ENGINE_GUARD_HELD(e);
    if (!s) return OWRX_EINVAL;
    *s = e->stats;
    // the chains' ring drops are summed as they happen (drain_slot): no pass over 10^5 chains
    // per call
    int64_t dropped = e->ring_dropped;
    for (auto& kv : e->wfs) dropped += kv.second->ring.dropped;
    s->overruns += dropped;
    return OWRX_OK;
}

int owrx_set_ddc_mode(owrx_engine* e, int mode) {
    ENGINE_GUARD(e);
    e->chain_epoch++;  // the slots rebuild their post descriptors
    if (mode != OWRX_DDC_FAST && mode != OWRX_DDC_DIRECT) return OWRX_EINVAL;
    e->ddc_mode = mode;
    return OWRX_OK;
}

int owrx_set_timing(owrx_engine* e, int enable) {
    ENGINE_GUARD(e);
    e->timing = std::max(0, enable);
    return OWRX_OK;
}

}  // extern "C"
