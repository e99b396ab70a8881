// engine.hip -- host side of libowrx_amd.so: one engine per GPU and per wideband IQ stream.
//
// Replaces the reference's per-module native threads + ring buffers (pycsdr Buffer/Reader,
// csdr modules; callers owrx/fft.py:36-73 and owrx/dsp.py:39-72, 835-863) with a block
// scheduler: each processed block runs
//   waterfall:  wf_fft_power -> wf_finalize -> wf_adpcm_rows      (per FftChain)
//   chains:     ddc_polyphase per (D, taps) group -> post_chains   (all client chains)
// on one HIP stream, then copies the finished waterfall rows, audio bytes and s-meter values
// to host rings that the pycsdr binding drains.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/owrx_amd.h"
#include "design.h"
#include "owrx_types.h"

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
hipError_t launch_wf_fft(int logn, const float2* blk, int64_t blk_start, const WfGroup* groups,
                         int ngroups, const float* window, const float2* tw, float* partial,
                         hipStream_t st);
hipError_t launch_wf_finalize(const float* partial, const WfRow* rows, int nrows,
                              const float* carry_in, float* carry_out, int N, float add_corr,
                              int adpcm, int16_t* s16_out, float* f32_out, hipStream_t st);
hipError_t launch_wf_adpcm(const int16_t* s16, int N, int nrows, uint8_t* out, int row_bytes,
                           hipStream_t st);
hipError_t launch_ddc(int P, const float2* blk, int64_t blk_start, int64_t blk_end,
                      const float* taps_poly, const DdcChain* chains, int nchains, int D,
                      int64_t k_begin, int nk, int nseg, float2* partial, hipStream_t st);
int ddc_padded_p(int p);
int ddc_segments(int D, int nseg);
hipError_t launch_post(const ChainPost* posts, int nchains, ChainCounts* counts,
                       hipStream_t st);

constexpr int kWfFramesPerGroup = 4;
constexpr int64_t kDefaultHistory = 1 << 18;
constexpr int kDebugStages = 6;

#define HIPCHK(expr)                                                                    \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) {                                                         \
            set_last_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),        \
                           __FILE__, __LINE__);                                         \
            return OWRX_EIO;                                                            \
        }                                                                               \
    } while (0)

template <typename T>
static hipError_t dalloc(T** p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, sizeof(T) * count);
    if (e == hipSuccess) e = hipMemset(*p, 0, sizeof(T) * count);
    return e;
}
template <typename T>
static void dfree(T*& p) {
    if (p) hipFree((void*)p);
    p = nullptr;
}

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
    bool carry_valid = false;
    int carry_idx = 0;
    int64_t rows = 0;
    float* d_window = nullptr;
    float2* d_tw = nullptr;
    float* d_partial = nullptr;
    int partial_groups = 0;
    float* d_carry[2] = {nullptr, nullptr};
    WfGroup* d_groups = nullptr;
    WfRow* d_rows = nullptr;
    int16_t* d_s16 = nullptr;
    float* d_f32 = nullptr;
    uint8_t* d_bytes = nullptr;
    uint8_t* h_bytes = nullptr;  // pinned
    int rows_cap = 0;
    ByteRing ring;
    std::vector<WfGroup> groups;
    std::vector<WfRow> rowdesc;
    int64_t row_bytes() const { return adpcm ? (N + 10) / 2 : 4 * (int64_t)N; }
};

struct ChainGroup {
    int D = 0, T = 0, P = 0;
    uint32_t tbw_bits = 0, cutoff_bits = 0;
    float* d_taps = nullptr;
    std::vector<int> members;  // chain handles
    int64_t k_next = 0;
    DdcChain* d_chains = nullptr;
    int chains_cap = 0;
    float2* d_partial = nullptr;
    size_t partial_elems = 0;
    int nseg = 1;
};

struct Chain {
    owrx_chain_params prm;
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
    ChainState* d_state = nullptr;
    float2* d_ddc = nullptr;
    float2* d_fd = nullptr;
    float2* d_sq = nullptr;
    float* d_dem = nullptr;
    float2* d_bp_taps = nullptr;
    int bp_ntaps = 0;
    int64_t cap = 0;      // per-step sample capacity of stage buffers
    int64_t out_cap = 0;  // staging bytes per step
    int sm_cap = 0;
    ByteRing audio;
    ByteRing smeter;
    ByteRing dbg[kDebugStages];
};

}  // namespace owrx

using namespace owrx;

struct owrx_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    double samp_rate = 0;
    int64_t max_block = 0;
    int64_t history = kDefaultHistory;
    int64_t pos = 0;  // absolute samples processed
    bool failed = false;
    bool debug = false;
    bool timing = false;
    std::recursive_mutex mu;
    // push-path window (ping-pong): [history | block]
    float2* d_win[2] = {nullptr, nullptr};
    int win_idx = 0;
    float* h_in = nullptr;  // pinned staging for push_iq
    std::map<int, std::unique_ptr<Waterfall>> wfs;
    std::map<int, std::unique_ptr<Chain>> chains;
    std::vector<std::unique_ptr<ChainGroup>> groups;
    int next_handle = 1;
    // post staging (all chains)
    int post_cap = 0;
    ChainPost* d_posts = nullptr;
    ChainCounts* d_counts = nullptr;
    ChainCounts* h_counts = nullptr;
    uint8_t* d_out = nullptr;
    uint8_t* h_out = nullptr;
    float* d_sm = nullptr;
    float* h_sm = nullptr;
    int64_t out_stride = 0, sm_stride = 0;
    uint8_t* d_dbg = nullptr;
    uint8_t* h_dbg = nullptr;
    int64_t dbg_stride = 0;  // bytes per chain per stage
    std::vector<ChainPost> posts;
    std::vector<int> post_ids;
    owrx_stats stats;
    hipEvent_t ev[6];
};

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------

static int64_t chain_stage_cap(const owrx_engine* e, int D, double frac) {
    int64_t nk = e->max_block / D + 4;
    if (frac > 0 && frac < 1.0) nk = (int64_t)std::ceil(nk / frac) + 4;
    return nk;
}

static void free_chain(Chain* c) {
    dfree(c->d_state);
    dfree(c->d_ddc);
    dfree(c->d_fd);
    dfree(c->d_sq);
    dfree(c->d_dem);
    dfree(c->d_bp_taps);
}

static void free_wf(Waterfall* w) {
    dfree(w->d_window);
    dfree(w->d_tw);
    dfree(w->d_partial);
    dfree(w->d_carry[0]);
    dfree(w->d_carry[1]);
    dfree(w->d_groups);
    dfree(w->d_rows);
    dfree(w->d_s16);
    dfree(w->d_f32);
    dfree(w->d_bytes);
    if (w->h_bytes) hipHostFree(w->h_bytes);
    w->h_bytes = nullptr;
}

static int wf_alloc_buffers(owrx_engine* e, Waterfall* w) {
    // capacities derived from the current hop/avg; re-run when they change
    const int64_t frames = e->max_block / std::max(1, w->hop) + 2 * kWfFramesPerGroup + 2;
    const int groups = (int)(frames / 1 + 2);  // a group may hold a single frame at row ends
    const int rows = (int)(frames / std::max(1, w->avg) + 3);
    if (groups > w->partial_groups) {
        dfree(w->d_partial);
        dfree(w->d_groups);
        HIPCHK(dalloc(&w->d_partial, (size_t)groups * w->N));
        HIPCHK(dalloc(&w->d_groups, (size_t)groups));
        w->partial_groups = groups;
    }
    if (rows > w->rows_cap) {
        dfree(w->d_rows);
        dfree(w->d_s16);
        dfree(w->d_f32);
        dfree(w->d_bytes);
        if (w->h_bytes) hipHostFree(w->h_bytes);
        w->h_bytes = nullptr;
        HIPCHK(dalloc(&w->d_rows, (size_t)rows + 1));
        HIPCHK(dalloc(&w->d_s16, (size_t)rows * w->N));
        HIPCHK(dalloc(&w->d_f32, (size_t)rows * w->N));
        HIPCHK(dalloc(&w->d_bytes, (size_t)rows * 4 * w->N));
        HIPCHK(hipHostMalloc((void**)&w->h_bytes, (size_t)rows * 4 * w->N, 0));
        w->rows_cap = rows;
    }
    return OWRX_OK;
}

static int ensure_post_capacity(owrx_engine* e) {
    const int n = (int)e->chains.size();
    int64_t need_out = 64, need_sm = 4, need_dbg = 64;
    for (auto& kv : e->chains) {
        need_out = std::max(need_out, kv.second->out_cap);
        need_sm = std::max<int64_t>(need_sm, kv.second->sm_cap);
        need_dbg = std::max<int64_t>(need_dbg, kv.second->cap * 8 + 64);
    }
    if (n <= e->post_cap && need_out <= e->out_stride && need_sm <= e->sm_stride &&
        (!e->debug || need_dbg <= e->dbg_stride))
        return OWRX_OK;
    const int cap = std::max(n, e->post_cap ? e->post_cap * 2 : 16);
    dfree(e->d_posts);
    dfree(e->d_counts);
    dfree(e->d_out);
    dfree(e->d_sm);
    dfree(e->d_dbg);
    if (e->h_counts) hipHostFree(e->h_counts);
    if (e->h_out) hipHostFree(e->h_out);
    if (e->h_sm) hipHostFree(e->h_sm);
    if (e->h_dbg) hipHostFree(e->h_dbg);
    e->h_counts = nullptr;
    e->h_out = nullptr;
    e->h_sm = nullptr;
    e->h_dbg = nullptr;
    e->out_stride = (need_out + 255) & ~(int64_t)255;
    e->sm_stride = need_sm;
    HIPCHK(dalloc(&e->d_posts, cap));
    HIPCHK(dalloc(&e->d_counts, cap));
    HIPCHK(dalloc(&e->d_out, (size_t)cap * e->out_stride));
    HIPCHK(dalloc(&e->d_sm, (size_t)cap * e->sm_stride));
    HIPCHK(hipHostMalloc((void**)&e->h_counts, sizeof(ChainCounts) * cap, 0));
    HIPCHK(hipHostMalloc((void**)&e->h_out, (size_t)cap * e->out_stride, 0));
    HIPCHK(hipHostMalloc((void**)&e->h_sm, sizeof(float) * cap * e->sm_stride, 0));
    if (e->debug) {
        e->dbg_stride = (need_dbg + 255) & ~(int64_t)255;
        HIPCHK(dalloc(&e->d_dbg, (size_t)cap * kDebugStages * e->dbg_stride));
        HIPCHK(hipHostMalloc((void**)&e->h_dbg, (size_t)cap * kDebugStages * e->dbg_stride, 0));
    } else {
        e->dbg_stride = 0;
    }
    e->post_cap = cap;
    return OWRX_OK;
}

static int group_refresh_device(owrx_engine* e, ChainGroup* g) {
    // per-chain DDC descriptors + partial buffer sized for the current membership
    const int n = (int)g->members.size();
    if (n > g->chains_cap) {
        dfree(g->d_chains);
        g->chains_cap = std::max(n, 2 * g->chains_cap);
        HIPCHK(dalloc(&g->d_chains, (size_t)g->chains_cap));
    }
    const int64_t nk_max = e->max_block / g->D + 4;
    // segments: enough waves to fill 256 CUs x 4 SIMDs x ~4 waves
    const int R = 32;
    int cpw = 1;
    while (cpw < n && cpw < 64) cpw <<= 1;
    const int tpw = 64 / cpw;
    const int64_t ntg = ((nk_max + R - 1) / R + tpw - 1) / tpw;
    const int64_t ncg = (n + cpw - 1) / cpw;
    const int64_t base = std::max<int64_t>(1, ntg * ncg);
    int nseg = (int)std::min<int64_t>(std::max<int64_t>(1, (4096 + base - 1) / base),
                                      std::max(1, g->D / 8));
    nseg = ddc_segments(g->D, nseg);
    const size_t need = (size_t)nseg * std::max(1, n) * nk_max;
    if (need > g->partial_elems) {
        dfree(g->d_partial);
        HIPCHK(dalloc(&g->d_partial, need));
        g->partial_elems = need;
    }
    g->nseg = nseg;
    return OWRX_OK;
}

// ------------------------------------------------------------------------------------------
// block processing
// ------------------------------------------------------------------------------------------

static int process_waterfall(owrx_engine* e, Waterfall* w, const float2* blk, int64_t blk_start,
                             int64_t blk_end) {
    w->groups.clear();
    w->rowdesc.clear();
    // schedule whole groups whose frames are inside the block (plus history)
    int cur_row_first_group = 0;
    bool row_open = false;
    while (true) {
        const int gf = std::min(kWfFramesPerGroup, w->avg - w->row_frame);
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
            if (w->pending) {  // parameter changes apply at row boundaries
                w->hop = w->new_hop;
                w->avg = w->new_avg;
                w->adpcm = w->new_adpcm;
                w->pending = false;
                int rc = wf_alloc_buffers(e, w);
                if (rc) return rc;
            }
            if ((int)w->rowdesc.size() + 1 >= w->rows_cap) break;
        }
    }
    int ncomplete = (int)w->rowdesc.size();
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
    HIPCHK(hipMemcpyAsync(w->d_groups, w->groups.data(), sizeof(WfGroup) * w->groups.size(),
                          hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(w->d_rows, w->rowdesc.data(), sizeof(WfRow) * w->rowdesc.size(),
                          hipMemcpyHostToDevice, e->stream));
    if (e->timing) hipEventRecord(e->ev[2], e->stream);
    HIPCHK(launch_wf_fft(w->logn, blk, blk_start, w->d_groups, (int)w->groups.size(),
                         w->d_window, w->d_tw, w->d_partial, e->stream));
    if (e->timing) hipEventRecord(e->ev[3], e->stream);
    const float corr = (float)((double)w->add_db - 10.0 * std::log10((double)std::max(1, w->avg)));
    const int cin = w->carry_idx, cout = 1 - w->carry_idx;
    HIPCHK(launch_wf_finalize(w->d_partial, w->d_rows, (int)w->rowdesc.size(), w->d_carry[cin],
                              w->d_carry[cout], w->N, corr, w->adpcm, w->d_s16, w->d_f32,
                              e->stream));
    if (row_open) {
        w->carry_idx = cout;
        w->carry_valid = true;
    }
    e->stats.waterfall_launches++;
    if (ncomplete > 0) {
        const int64_t rb = w->row_bytes();
        if (w->adpcm) {
            HIPCHK(launch_wf_adpcm(w->d_s16, w->N, ncomplete, w->d_bytes, (int)rb, e->stream));
            HIPCHK(hipMemcpyAsync(w->h_bytes, w->d_bytes, rb * ncomplete, hipMemcpyDeviceToHost,
                                  e->stream));
        } else {
            HIPCHK(hipMemcpyAsync(w->h_bytes, w->d_f32, rb * ncomplete, hipMemcpyDeviceToHost,
                                  e->stream));
        }
    }
    return OWRX_OK;
}

static int process_block(owrx_engine* e, const float2* blk, int64_t n) {
    const int64_t blk_start = e->pos;
    const int64_t blk_end = e->pos + n;
    if (e->timing) hipEventRecord(e->ev[0], e->stream);

    // ---- waterfalls
    std::vector<std::pair<Waterfall*, int>> wf_done;
    for (auto& kv : e->wfs) {
        Waterfall* w = kv.second.get();
        const size_t before = w->rowdesc.size();
        (void)before;
        int rc = process_waterfall(e, w, blk, blk_start, blk_end);
        if (rc) return rc;
        int complete = 0;
        for (auto& r : w->rowdesc) complete += r.complete;
        if (!w->groups.empty() && complete) wf_done.push_back({w, complete});
    }

    // ---- chains: apply pending setters, DDC per group, then one post launch
    e->posts.clear();
    e->post_ids.clear();
    if (e->timing) hipEventRecord(e->ev[4], e->stream);
    for (auto& gp : e->groups) {
        ChainGroup* g = gp.get();
        if (g->members.empty()) continue;
        if (blk_end < g->T) continue;
        const int64_t k_end = (blk_end - g->T) / g->D + 1;
        const int64_t nk64 = k_end - g->k_next;
        if (nk64 <= 0) continue;
        const int nk = (int)nk64;
        std::vector<DdcChain> dc(g->members.size());
        for (size_t i = 0; i < g->members.size(); ++i) {
            Chain* c = e->chains[g->members[i]].get();
            if (c->rate_pending) {  // retune at output boundary k_next (phase continuous)
                const int64_t nb = std::max(g->k_next, c->k_first) * g->D;
                const uint64_t ph_last = c->P0 + (uint64_t)(nb - c->n0) * c->rate_fx;
                c->P0 = ph_last;
                c->n0 = nb;
                c->rate = c->new_rate;
                c->rate_fx = rate_to_fx(c->rate);
                c->rate_pending = false;
            }
            dc[i].rate_fx = c->rate_fx;
            dc[i].wD = rate_rotator(c->rate, g->D);
            dc[i].n0 = c->n0;
            dc[i].P0 = c->P0;
        }
        HIPCHK(hipMemcpyAsync(g->d_chains, dc.data(), sizeof(DdcChain) * dc.size(),
                              hipMemcpyHostToDevice, e->stream));
        HIPCHK(launch_ddc(g->P, blk, blk_start, blk_end, g->d_taps, g->d_chains,
                          (int)g->members.size(), g->D, g->k_next, nk, g->nseg, g->d_partial,
                          e->stream));
        e->stats.ddc_launches++;
        for (size_t i = 0; i < g->members.size(); ++i) {
            Chain* c = e->chains[g->members[i]].get();
            ChainPost p;
            memset(&p, 0, sizeof(p));
            const owrx_chain_params& q = c->prm;
            p.demod = q.demod;
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
            p.deemph_beta = 1.0f - p.deemph_alpha;
            p.agc = agc_profile(q.agc_profile);
            if (q.agc_initial_gain >= 0) p.agc.initial_gain = q.agc_initial_gain;
            if (q.agc_max_gain >= 0) p.agc.max_gain = q.agc_max_gain;
            p.state = c->d_state;
            p.ddc_buf = c->d_ddc;
            p.fd_buf = c->d_fd;
            p.sq_buf = c->d_sq;
            p.dem_buf = c->d_dem;
            p.partial = g->d_partial;
            p.nseg = ddc_segments(g->D, g->nseg);
            p.group_chains = (int)g->members.size();
            p.chain_in_group = (int)i;
            p.nk = nk;
            p.k_begin = g->k_next;
            p.k_first = c->k_first;
            const int slot = (int)e->posts.size();
            p.out = e->d_out + (int64_t)slot * e->out_stride;
            p.out_cap = e->out_stride;
            p.smeter = e->d_sm + (int64_t)slot * e->sm_stride;
            p.smeter_cap = (int)e->sm_stride;
            p.debug = e->debug ? 1 : 0;
            if (e->debug) {
                uint8_t* base = e->d_dbg + (int64_t)slot * kDebugStages * e->dbg_stride;
                p.dbg_ddc = (float2*)(base + 0 * e->dbg_stride);
                p.dbg_fd = (float2*)(base + 1 * e->dbg_stride);
                p.dbg_bp = (float2*)(base + 2 * e->dbg_stride);
                p.dbg_sq = (float2*)(base + 3 * e->dbg_stride);
                p.dbg_dem = (float*)(base + 4 * e->dbg_stride);
                p.dbg_agc = (float*)(base + 5 * e->dbg_stride);
                p.dbg_cap = e->dbg_stride / 8;
            }
            e->posts.push_back(p);
            e->post_ids.push_back(g->members[i]);
        }
        g->k_next = k_end;
    }
    if (e->timing) hipEventRecord(e->ev[5], e->stream);
    const int np = (int)e->posts.size();
    if (np > 0) {
        HIPCHK(hipMemcpyAsync(e->d_posts, e->posts.data(), sizeof(ChainPost) * np,
                              hipMemcpyHostToDevice, e->stream));
        HIPCHK(launch_post(e->d_posts, np, e->d_counts, e->stream));
        HIPCHK(hipMemcpyAsync(e->h_counts, e->d_counts, sizeof(ChainCounts) * np,
                              hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipMemcpyAsync(e->h_out, e->d_out, (size_t)np * e->out_stride,
                              hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipMemcpyAsync(e->h_sm, e->d_sm, sizeof(float) * np * e->sm_stride,
                              hipMemcpyDeviceToHost, e->stream));
        if (e->debug)
            HIPCHK(hipMemcpyAsync(e->h_dbg, e->d_dbg, (size_t)np * kDebugStages * e->dbg_stride,
                                  hipMemcpyDeviceToHost, e->stream));
    }
    if (e->timing) hipEventRecord(e->ev[1], e->stream);
    HIPCHK(hipStreamSynchronize(e->stream));

    // ---- drain into host rings
    for (auto& wd : wf_done) {
        Waterfall* w = wd.first;
        const int64_t rb = w->row_bytes();
        w->ring.push(w->h_bytes, (size_t)(rb * wd.second));
        w->rows += wd.second;
        e->stats.waterfall_rows += wd.second;
    }
    for (int s = 0; s < np; ++s) {
        Chain* c = e->chains[e->post_ids[s]].get();
        const ChainCounts& cc = e->h_counts[s];
        const int64_t nb = std::min<int64_t>(cc.out_bytes, e->out_stride);
        if (cc.out_bytes > e->out_stride) e->stats.overruns++;
        c->audio.push(e->h_out + (int64_t)s * e->out_stride, (size_t)nb);
        e->stats.audio_bytes += nb;
        e->stats.ddc_outputs += cc.n_ddc;
        c->smeter.push((const uint8_t*)(e->h_sm + (int64_t)s * e->sm_stride),
                       sizeof(float) * (size_t)cc.smeter);
        if (e->debug) {
            const uint8_t* base = e->h_dbg + (int64_t)s * kDebugStages * e->dbg_stride;
            const int64_t cnt[kDebugStages] = {cc.n_ddc, cc.n_fd, cc.n_bp, cc.n_sq, cc.n_sq,
                                               cc.n_sq};
            const int64_t isz[kDebugStages] = {8, 8, 8, 8, 4, 4};
            for (int st = 0; st < kDebugStages; ++st) {
                const int64_t bytes = std::min(cnt[st] * isz[st], e->dbg_stride);
                c->dbg[st].push(base + st * e->dbg_stride, (size_t)bytes);
            }
        }
    }
    if (e->timing) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, e->ev[4], e->ev[5]) == hipSuccess) e->stats.gpu_ms_ddc += ms;
        if (!e->wfs.empty() && hipEventElapsedTime(&ms, e->ev[0], e->ev[4]) == hipSuccess)
            e->stats.gpu_ms_waterfall += ms;
        if (hipEventElapsedTime(&ms, e->ev[5], e->ev[1]) == hipSuccess) e->stats.gpu_ms_post += ms;
    }
    e->pos = blk_end;
    e->stats.samples_in += n;
    e->stats.blocks++;
    return OWRX_OK;
}

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------

#define ENGINE_GUARD(e)                                              \
    if (!(e)) {                                                      \
        set_last_error("null engine");                               \
        return OWRX_EINVAL;                                          \
    }                                                                \
    std::lock_guard<std::recursive_mutex> _lk((e)->mu);              \
    if ((e)->failed) {                                               \
        set_last_error("engine failed earlier (HIP error)");         \
        return OWRX_EIO;                                             \
    }                                                                \
    hipSetDevice((e)->device);

#define RC_FAIL(e, expr)          \
    do {                          \
        int _rc = (expr);         \
        if (_rc < 0) {            \
            if (_rc == OWRX_EIO) (e)->failed = true; \
            return _rc;           \
        }                         \
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

int owrx_engine_create(int device, double samp_rate, int64_t max_block, owrx_engine** out) {
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
    owrx_engine* e = new owrx_engine();
    e->device = device;
    e->samp_rate = samp_rate;
    e->max_block = max_block;
    memset(&e->stats, 0, sizeof(e->stats));
    int rc = OWRX_OK;
    auto fail = [&](const char* what) {
        set_last_error("owrx_engine_create: %s", what);
        owrx_engine_destroy(e);
        return OWRX_EIO;
    };
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
        return fail("stream");
    for (int i = 0; i < 6; ++i)
        if (hipEventCreate(&e->ev[i]) != hipSuccess) return fail("event");
    for (int i = 0; i < 2; ++i)
        if (dalloc(&e->d_win[i], (size_t)(e->history + max_block)) != hipSuccess)
            return fail("window");
    if (hipHostMalloc((void**)&e->h_in, sizeof(float2) * (size_t)max_block, 0) != hipSuccess)
        return fail("pinned input");
    (void)rc;
    *out = e;
    return OWRX_OK;
}

int owrx_engine_destroy(owrx_engine* e) {
    if (!e) return OWRX_EINVAL;
    hipSetDevice(e->device);
    if (e->stream) hipStreamSynchronize(e->stream);
    for (auto& kv : e->chains) free_chain(kv.second.get());
    for (auto& kv : e->wfs) free_wf(kv.second.get());
    for (auto& g : e->groups) {
        dfree(g->d_taps);
        dfree(g->d_chains);
        dfree(g->d_partial);
    }
    dfree(e->d_win[0]);
    dfree(e->d_win[1]);
    dfree(e->d_posts);
    dfree(e->d_counts);
    dfree(e->d_out);
    dfree(e->d_sm);
    dfree(e->d_dbg);
    if (e->h_in) hipHostFree(e->h_in);
    if (e->h_counts) hipHostFree(e->h_counts);
    if (e->h_out) hipHostFree(e->h_out);
    if (e->h_sm) hipHostFree(e->h_sm);
    if (e->h_dbg) hipHostFree(e->h_dbg);
    for (int i = 0; i < 6; ++i)
        if (e->ev[i]) hipEventDestroy(e->ev[i]);
    if (e->stream) hipStreamDestroy(e->stream);
    delete e;
    return OWRX_OK;
}

int64_t owrx_engine_history(owrx_engine* e) { return e ? e->history : OWRX_EINVAL; }
int64_t owrx_engine_max_block(owrx_engine* e) { return e ? e->max_block : OWRX_EINVAL; }

int owrx_process_device(owrx_engine* e, const float* iq_dev, int64_t n) {
    ENGINE_GUARD(e);
    if (!iq_dev || n < 0 || n > e->max_block) {
        set_last_error("owrx_process_device: bad block (n=%lld, max %lld)", (long long)n,
                       (long long)e->max_block);
        return OWRX_EINVAL;
    }
    if (n == 0) return OWRX_OK;
    RC_FAIL(e, process_block(e, (const float2*)iq_dev, n));
    return OWRX_OK;
}

int owrx_ingest_buffer(owrx_engine* e, float** dev_ptr, int64_t* capacity) {
    ENGINE_GUARD(e);
    if (!dev_ptr || !capacity) return OWRX_EINVAL;
    *dev_ptr = (float*)(e->d_win[e->win_idx] + e->history);
    *capacity = e->max_block;
    return OWRX_OK;
}

int owrx_commit(owrx_engine* e, int64_t n) {
    ENGINE_GUARD(e);
    if (n < 0 || n > e->max_block) return OWRX_EINVAL;
    if (n == 0) return OWRX_OK;
    float2* w = e->d_win[e->win_idx];
    RC_FAIL(e, process_block(e, w + e->history, n));
    // carry the last `history` samples into the other window
    float2* o = e->d_win[1 - e->win_idx];
    if (hipMemcpyAsync(o, w + n, sizeof(float2) * e->history, hipMemcpyDeviceToDevice,
                       e->stream) != hipSuccess) {
        e->failed = true;
        set_last_error("window carry copy failed");
        return OWRX_EIO;
    }
    e->win_idx = 1 - e->win_idx;
    return OWRX_OK;
}

int owrx_push_iq(owrx_engine* e, const float* iq, int64_t n) {
    ENGINE_GUARD(e);
    if (n < 0 || (n > 0 && !iq)) return OWRX_EINVAL;
    int64_t done = 0;
    while (done < n) {
        const int64_t m = std::min(n - done, e->max_block);
        memcpy(e->h_in, iq + 2 * done, sizeof(float2) * m);
        float2* dst = e->d_win[e->win_idx] + e->history;
        if (hipMemcpyAsync(dst, e->h_in, sizeof(float2) * m, hipMemcpyHostToDevice, e->stream) !=
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

int owrx_sync(owrx_engine* e) {
    ENGINE_GUARD(e);
    HIPCHK(hipStreamSynchronize(e->stream));
    return OWRX_OK;
}

// ---- waterfall --------------------------------------------------------------------------

int owrx_waterfall_create(owrx_engine* e, int fft_size, int every_n_samples, int avg_number,
                          float add_db, int adpcm, int* handle) {
    ENGINE_GUARD(e);
    int logn = 0;
    while ((1 << logn) < fft_size) logn++;
    if (!handle || fft_size < 256 || fft_size > 16384 || (1 << logn) != fft_size ||
        every_n_samples <= 0 || avg_number < 0) {
        set_last_error("owrx_waterfall_create: fft_size must be a power of two in [256, 16384], "
                       "every_n_samples > 0");
        return OWRX_EINVAL;
    }
    if ((int64_t)kWfFramesPerGroup * every_n_samples + fft_size > e->history) {
        set_last_error("owrx_waterfall_create: hop too large for engine history");
        return OWRX_EINVAL;
    }
    auto w = std::make_unique<Waterfall>();
    w->N = fft_size;
    w->logn = logn;
    w->hop = every_n_samples;
    w->avg = std::max(1, avg_number);
    w->adpcm = adpcm ? 1 : 0;
    w->add_db = add_db;
    w->next_start = e->pos;
    std::vector<float> win = hamming_window(fft_size);
    std::vector<float> tw = fft_twiddles(fft_size);
    HIPCHK(dalloc(&w->d_window, (size_t)fft_size));
    HIPCHK(dalloc(&w->d_tw, (size_t)fft_size));
    HIPCHK(dalloc(&w->d_carry[0], (size_t)fft_size));
    HIPCHK(dalloc(&w->d_carry[1], (size_t)fft_size));
    HIPCHK(hipMemcpy(w->d_window, win.data(), sizeof(float) * fft_size, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(w->d_tw, tw.data(), sizeof(float) * 2 * fft_size, hipMemcpyHostToDevice));
    int rc = wf_alloc_buffers(e, w.get());
    if (rc) {
        free_wf(w.get());
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
    if ((int64_t)kWfFramesPerGroup * every_n_samples + w->N > e->history) return OWRX_EINVAL;
    w->new_hop = every_n_samples;
    w->new_avg = std::max(1, avg_number);
    w->new_adpcm = adpcm ? 1 : 0;
    if (w->row_frame == 0 && !w->carry_valid) {  // at a row boundary: apply now
        w->hop = w->new_hop;
        w->avg = w->new_avg;
        w->adpcm = w->new_adpcm;
        w->pending = false;
        return wf_alloc_buffers(e, w);
    }
    w->pending = true;
    return OWRX_OK;
}

int owrx_waterfall_destroy(owrx_engine* e, int handle) {
    ENGINE_GUARD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end()) return OWRX_EINVAL;
    free_wf(it->second.get());
    e->wfs.erase(it);
    return OWRX_OK;
}

int64_t owrx_waterfall_row_bytes(owrx_engine* e, int handle) {
    ENGINE_GUARD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end()) return OWRX_EINVAL;
    return it->second->row_bytes();
}

int64_t owrx_waterfall_read(owrx_engine* e, int handle, uint8_t* dst, int64_t max_bytes) {
    ENGINE_GUARD(e);
    auto it = e->wfs.find(handle);
    if (it == e->wfs.end() || !dst || max_bytes < 0) return OWRX_EINVAL;
    Waterfall* w = it->second.get();
    const int64_t rb = w->row_bytes();
    const int64_t rows = std::min<int64_t>((int64_t)w->ring.avail() / rb, max_bytes / rb);
    return (int64_t)w->ring.pop(dst, (size_t)(rows * rb));
}

// ---- chains -----------------------------------------------------------------------------

static int chain_validate(const owrx_chain_params* p) {
    if (!p || p->decimation < 1 || p->transition <= 0 || p->cutoff <= 0 || p->frac_rate <= 0 ||
        p->sq_length <= 0 || p->sq_length > 3072 || p->sq_decimation <= 0 || p->demod < 0 ||
        p->demod > 2 || p->output < 0 || p->output > 2 || p->audio_rate <= 0 ||
        p->agc_profile < 0 || p->agc_profile > 3)
        return OWRX_EINVAL;
    if (p->bandpass && (p->bp_transition <= 0 || p->bp_low >= p->bp_high)) return OWRX_EINVAL;
    return OWRX_OK;
}

static int chain_set_bandpass_taps(owrx_engine* e, Chain* c) {
    if (!c->prm.bandpass) return OWRX_OK;
    const int T = firdes_filter_len(c->prm.bp_transition);
    if (T > kBpHist + 1) {
        set_last_error("bandpass transition too narrow (%d taps > %d)", T, kBpHist + 1);
        return OWRX_EINVAL;
    }
    std::vector<float> taps = firdes_bandpass_c(T, c->prm.bp_low, c->prm.bp_high);
    if (!c->d_bp_taps) HIPCHK(dalloc(&c->d_bp_taps, (size_t)kBpHist + 1));
    HIPCHK(hipMemcpyAsync(c->d_bp_taps, taps.data(), sizeof(float) * 2 * T,
                          hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    c->bp_ntaps = T;
    return OWRX_OK;
}

int owrx_chain_create(owrx_engine* e, const owrx_chain_params* p, int* handle) {
    ENGINE_GUARD(e);
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
    // group lookup by (D, transition, cutoff)
    uint32_t tb, cb;
    memcpy(&tb, &p->transition, 4);
    memcpy(&cb, &p->cutoff, 4);
    ChainGroup* g = nullptr;
    for (auto& gp : e->groups)
        if (gp->D == D && gp->tbw_bits == tb && gp->cutoff_bits == cb) g = gp.get();
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
    c->out_cap = 4 * scap + 8 * (scap / 2 / kAdpcmSyncPeriod + 2) + 64;
    c->sm_cap = (int)(scap / p->sq_length + 4);
    ChainState st;
    memset(&st, 0, sizeof(st));
    AgcParams ap = agc_profile(p->agc_profile);
    if (p->agc_initial_gain >= 0) ap.initial_gain = p->agc_initial_gain;
    st.agc.env = ap.reference / ap.initial_gain;
    HIPCHK(dalloc(&c->d_state, 1));
    HIPCHK(hipMemcpy(c->d_state, &st, sizeof(st), hipMemcpyHostToDevice));
    HIPCHK(dalloc(&c->d_ddc, (size_t)(kFdHist + c->cap)));
    HIPCHK(dalloc(&c->d_fd, (size_t)(kBpHist + c->cap)));
    HIPCHK(dalloc(&c->d_sq, (size_t)scap));
    HIPCHK(dalloc(&c->d_dem, (size_t)scap));
    int rc = chain_set_bandpass_taps(e, c.get());
    if (rc) {
        free_chain(c.get());
        return rc;
    }
    const int h = e->next_handle++;
    g->members.push_back(h);
    e->chains[h] = std::move(c);
    RC_FAIL(e, group_refresh_device(e, g));
    RC_FAIL(e, ensure_post_capacity(e));
    *handle = h;
    return OWRX_OK;
}

int owrx_chain_destroy(owrx_engine* e, int handle) {
    ENGINE_GUARD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    ChainGroup* g = it->second->group;
    g->members.erase(std::remove(g->members.begin(), g->members.end(), handle), g->members.end());
    free_chain(it->second.get());
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
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    Chain* c = it->second.get();
    if (enabled && low >= high) return OWRX_EINVAL;
    c->prm.bandpass = enabled ? 1 : 0;
    c->prm.bp_low = low;
    c->prm.bp_high = high;
    if (enabled && c->prm.bp_transition <= 0) return OWRX_EINVAL;
    return chain_set_bandpass_taps(e, c);
}

int owrx_chain_set_squelch_level(owrx_engine* e, int handle, float level) {
    ENGINE_GUARD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    it->second->prm.sq_level = level;
    return OWRX_OK;
}

int64_t owrx_chain_read_audio(owrx_engine* e, int handle, uint8_t* dst, int64_t max_bytes) {
    ENGINE_GUARD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || !dst || max_bytes < 0) return OWRX_EINVAL;
    return (int64_t)it->second->audio.pop(dst, (size_t)max_bytes);
}

int64_t owrx_chain_read_smeter(owrx_engine* e, int handle, float* dst, int64_t max_values) {
    ENGINE_GUARD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || !dst || max_values < 0) return OWRX_EINVAL;
    return (int64_t)it->second->smeter.pop((uint8_t*)dst, sizeof(float) * (size_t)max_values) /
           (int64_t)sizeof(float);
}

int64_t owrx_chain_origin(owrx_engine* e, int handle) {
    ENGINE_GUARD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end()) return OWRX_EINVAL;
    return it->second->origin;
}

int owrx_set_debug(owrx_engine* e, int enable) {
    ENGINE_GUARD(e);
    e->debug = enable != 0;
    e->post_cap = 0;  // force reallocation with debug staging
    return ensure_post_capacity(e);
}

int64_t owrx_chain_read_debug(owrx_engine* e, int handle, int stage, void* dst,
                              int64_t max_bytes) {
    ENGINE_GUARD(e);
    auto it = e->chains.find(handle);
    if (it == e->chains.end() || stage < 0 || stage >= kDebugStages || !dst || max_bytes < 0)
        return OWRX_EINVAL;
    return (int64_t)it->second->dbg[stage].pop((uint8_t*)dst, (size_t)max_bytes);
}

int owrx_get_stats(owrx_engine* e, owrx_stats* s) {
    ENGINE_GUARD(e);
    if (!s) return OWRX_EINVAL;
    *s = e->stats;
    int64_t dropped = 0;
    for (auto& kv : e->chains) dropped += kv.second->audio.dropped;
    for (auto& kv : e->wfs) dropped += kv.second->ring.dropped;
    s->overruns += dropped;
    return OWRX_OK;
}

int owrx_set_timing(owrx_engine* e, int enable) {
    ENGINE_GUARD(e);
    e->timing = enable != 0;
    return OWRX_OK;
}

}  // extern "C"
