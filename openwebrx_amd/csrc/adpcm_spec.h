// adpcm_spec.h -- speculative segment-parallel IMA-ADPCM window encoder (exact), shared by
// the waterfall row encoder (kernels_waterfall.hip).
#pragma once
#include "owrx_dev.h"

namespace owrx {

// Speculative segment-parallel IMA-ADPCM (exact).  IMA-ADPCM is a serial recurrence, but two
// encoders started from different states on the same input reach the same (index, predictor)
// state after a few samples and are identical from then on.  A window of up to kSpecWin
// samples (staged in LDS) is split into segments, one thread each:
//   pass 1: every segment encodes from a guessed state (segment 0 from the true state),
//           storing its codes and its state trajectory;
//   pass 2: a segment whose start differs from its predecessor's final state re-encodes from
//           that state until its state equals the stored trajectory (the stored codes are
//           exact from there on) or to its end (its trajectory / final state are replaced);
//           Jacobi rounds until no segment re-runs.
// The fixed point is the sequential trajectory, so codes are bit-identical to the serial
// encoder (oracle orc_adpcm_encode / orc_fft_adpcm_row).
constexpr int kSpecThreads = 256;

OWRX_DEV uint32_t pack_state(const AdpcmRem& s) {
    return ((uint32_t)s.index() << 16) | ((uint32_t)s.pred & 0xffffu);
}
OWRX_DEV AdpcmRem unpack_state(uint32_t v) {
    return adpcm_rem_state(AdpcmState{(int)(v >> 16), (int)(int16_t)(v & 0xffffu)});
}
// one sample with the remainder-form encoder (owrx_dev.h): its 4-bit code
OWRX_DEV uint8_t spec_encode(AdpcmRem& s, int x, const uint2* __restrict__ NSR) {
    return (uint8_t)((adpcm_encode_rem(s, x, NSR) & 15u) ^ 7u);
}

// Segment-transposed LDS layout: sample t of the window lives at (t % seg) * S + t / seg, so
// when every lane walks its own segment the 64 lanes of a wave touch 64 consecutive elements
// (a row-major layout put every lane's segment 2 * seg bytes apart: one LDS bank for the whole
// wave, a 64-way conflict on every access).  S = nseg rounded up to odd.
struct SpecGeom {
    int seg, nseg, S;
};
OWRX_DEV SpecGeom spec_geom(int n, int min_seg) {
    const int seg = max(min_seg, (((n + kSpecThreads - 1) / kSpecThreads) + 1) & ~1);
    const int nseg = (n + seg - 1) / seg;
    return SpecGeom{seg, nseg, nseg | 1};
}
OWRX_DEV int spec_at(const SpecGeom& g, int t) { return (t % g.seg) * g.S + t / g.seg; }

// capacity for a window of WIN samples in the transposed layout: seg * S <= n + 2 seg, and
// seg <= max(64, WIN / 256 + 2)
template <int WIN>
struct SpecLds {
    static constexpr int kCap = WIN + 2 * ((WIN / kSpecThreads + 2) > 64 ? (WIN / kSpecThreads + 2) : 64) + 2;
    uint2 NSR[kAdpcmRemEntries];  // adpcm_encode_rem successor records (round 5: ~25 % fewer
                                  // cycles per sample than the table step it replaced)
    int16_t x[kCap];
    uint8_t code[kCap];
    uint32_t traj[kCap];
    uint32_t seg_start[kSpecThreads], seg_final[kSpecThreads];
    int16_t T[96];
    int any;
};

// Encodes the window x[spec_at(g, t)], t < n, from `start` (block-uniform); g = spec_geom(n,
// min_seg) as the caller laid x out.  Returns with code / traj filled (same layout).
// Segments start from (index = `guess_index`, predictor = previous sample), or with
// guess_index < 0 from the step index matching the local slope.
template <int WIN>
OWRX_DEV void adpcm_spec_window(SpecLds<WIN>& L, int n, const SpecGeom& g, uint32_t start,
                                int guess_index) {
    const int tid = threadIdx.x;
    const int seg = g.seg, nseg = g.nseg, S = g.S;
    const int b0 = min(tid * seg, n), b1 = min(b0 + seg, n);
    const int len = b1 - b0;
    const int16_t* T = L.T;
    // pass 1
    if (tid < nseg) {
        AdpcmRem st;
        if (tid == 0) {
            st = unpack_state(start);
        } else {
            // the previous segment's last samples: x[b0 - 1], x[b0 - 2] at the tail of lane tid-1
            const int prev1 = (int)L.x[(seg - 1) * S + tid - 1];
            if (guess_index >= 0) {
                st = adpcm_rem_state(AdpcmState{guess_index, prev1});
            } else {
                // predictor = previous sample, step index from the local slope
                const int d = abs(prev1 - (int)L.x[(seg - 2) * S + tid - 1]);
                int lo = 0, hi = 88;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (T[mid] < d) lo = mid + 1; else hi = mid;
                }
                st = adpcm_rem_state(AdpcmState{lo, prev1});
            }
        }
        L.seg_start[tid] = pack_state(st);
        for (int j = 0, a = tid; j < len; ++j, a += S) {
            L.code[a] = spec_encode(st, L.x[a], L.NSR);
            L.traj[a] = pack_state(st);
        }
        L.seg_final[tid] = pack_state(st);
    }
    __syncthreads();
    // pass 2
    for (int round = 0; round < nseg; ++round) {
        if (tid == 0) L.any = 0;
        uint32_t want = 0, fin = 0;
        bool rerun = false;
        if (tid < nseg && tid > 0) {
            want = L.seg_final[tid - 1];
            rerun = want != L.seg_start[tid];
            fin = L.seg_final[tid];
        }
        __syncthreads();  // every start was read before any final changes
        if (rerun) {
            AdpcmRem r = unpack_state(want);
            bool merged = false;
            for (int j = 0, a = tid; j < len; ++j, a += S) {
                L.code[a] = spec_encode(r, L.x[a], L.NSR);
                const uint32_t ps = pack_state(r);
                if (ps == L.traj[a]) {
                    merged = true;
                    break;
                }
                L.traj[a] = ps;
            }
            if (!merged) fin = pack_state(r);
            L.seg_start[tid] = want;
            L.seg_final[tid] = fin;
            L.any = 1;
        }
        __syncthreads();
        if (!L.any) break;
        __syncthreads();
    }
}

}  // namespace owrx
