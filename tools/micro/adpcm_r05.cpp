// IMA-ADPCM serial encoder microbenchmark, round 5 (diagnostic; not part of the product):
// cycles per sample of one 64-lane wave (one lane per stream, 64 streams x 5000 samples) for the
// round 2-4 production encoder (byte-addressed masked successor table, tab2, defined below as the
// baseline) and its variants: 64-B threshold records, a ds_bpermute step, the successor row read
// beside the compares, reversed rows with accumulated compare bits (tab3), 8-B records with SDWA
// compares and a v_addc index in asm (tab4), the mask-free sub / alignbit / min form (tab6), and
// that form as shipped (adpcm_encode_rem, owrx_dev.h).  Every variant's codes are compared with
// tab2's.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 adpcm_r05.cpp -o adpcm_r05
#include "../../openwebrx_amd/csrc/owrx_dev.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace owrx;

// The round 2-4 production encoder (byte-addressed masked table), kept here as the baseline:
// NS2[index * 16 + sign * 8 + magnitude] = next step | (next index * 64) << 16 (the entry does
// not depend on the sign: each row is stored twice), so the next record's LDS byte address is
// the current record's high half + 32 * sign + 4 * magnitude -- one select after the last
// magnitude compare -- and the 4-bit code is that address's bits 2..5.  Each magnitude bit's
// remainder is selected from a subtraction done beside the compare.  Bit-identical to
// adpcm_encode.
constexpr int kAdpcmTab2Entries = 89 * 16;

template <int EXT>
OWRX_DEV void adpcm_tab2_fill(uint32_t (&NS2)[EXT], int tid, int nthreads) {
    static_assert(EXT >= kAdpcmTab2Entries, "byte-addressed successor table too small");
    for (int e = tid; e < kAdpcmTab2Entries; e += nthreads) {
        const int i = e >> 4, m = e & 7;
        int ni = i + kAdpcmIndex[m];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        NS2[e] = (uint32_t)kAdpcmStep[ni] | ((uint32_t)(ni * 64) << 16);
    }
}

struct AdpcmTab2 {
    uint32_t rec;  // step | (index * 64) << 16
    int pred;
    OWRX_DEV int index() const { return (int)(rec >> 22); }
};

OWRX_DEV AdpcmTab2 adpcm_tab2_state(AdpcmState s) {
    return AdpcmTab2{(uint32_t)kAdpcmStep[s.index] | ((uint32_t)(s.index * 64) << 16), s.pred};
}

OWRX_DEV int adpcm_encode_tab2(AdpcmTab2& s, int sample, const uint32_t* __restrict__ NS2) {
    // everything that needs only the predictor first, then a scheduling fence, so that it is
    // issued while this sample's record is still on its way from LDS (the record's first use
    // carries the wait)
    const int d = sample - s.pred;
    const int sgn = d >> 31;
    const int sg32 = sgn & 32;
    const int a0 = max(d, -d);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t rec = s.rec;
    const int step = (int)(rec & 0xffffu);
    const int h = step >> 1, q = step >> 2, s3 = step >> 3;
    const int rb = (int)(rec >> 16) + sg32;
    const bool m4 = a0 >= step;
    const int a1 = m4 ? a0 - step : a0;
    const bool m2 = a1 >= h;
    const int a2 = m2 ? a1 - h : a1;
    const bool m1 = a2 >= q;
    const int base = rb + (m4 ? 16 : 0) + (m2 ? 8 : 0);
    const int addr = m1 ? base + 4 : base;
    s.rec = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(NS2) + addr);
    // the predictor update after the lookup is issued (it fills the lookup's latency)
    __builtin_amdgcn_sched_barrier(0);
    const int dq = s3 + (m4 ? step : 0) + (m2 ? h : 0) + (m1 ? q : 0);
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    return (addr >> 2) & 15;  // magnitude bits and the sign (32 bytes = code bit 3)
}


constexpr int kThRec = 64;                 // bytes per record
constexpr int kThEntries = 89 * 8;         // (index, magnitude) -> the successor's record

struct ThState {
    uint32_t T4, T2, T6, T1, T3, T5, T7, S3, S3mQ, row;  // row: byte offset of TH[index][0]
    int pred;
};

__device__ void th_rec(uint32_t* r, int ni) {
    const uint32_t st = (uint32_t)kAdpcmStep[ni], h = st >> 1, q = st >> 2, s3 = st >> 3;
    r[0] = st; r[1] = h; r[2] = st + h; r[3] = q;
    r[4] = h + q; r[5] = st + q; r[6] = st + h + q; r[7] = s3;
    r[8] = s3 - q; r[9] = (uint32_t)(ni * 8 * kThRec);
}

__device__ void th_fill(uint32_t* TH, int tid, int nt) {
    for (int e = tid; e < kThEntries; e += nt) {
        const int i = e >> 3, m = e & 7;
        int ni = i + kAdpcmIndex[m];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        th_rec(TH + e * (kThRec / 4), ni);
    }
}

__device__ ThState th_state(int index, int pred) {
    uint32_t r[10];
    th_rec(r, index);
    return ThState{r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], r[8], r[9], pred};
}

__device__ __forceinline__ int th_encode(ThState& s, int x, const uint32_t* TH) {
    const int d = x - s.pred;
    const int sgn = d >> 31;
    const int a0 = max(d, -d);
    const bool m4 = a0 >= (int)s.T4;
    const int t2 = m4 ? (int)s.T6 : (int)s.T2;
    const uint32_t r4 = m4 ? s.row + 4 * kThRec : s.row;
    const int t1a = m4 ? (int)s.T5 : (int)s.T1;
    const int t1b = m4 ? (int)s.T7 : (int)s.T3;
    const bool m2 = a0 >= t2;
    const int t1 = m2 ? t1b : t1a;
    const uint32_t r42 = m2 ? r4 + 2 * kThRec : r4;
    const bool m1 = a0 >= t1;
    const uint32_t addr = m1 ? r42 + kThRec : r42;
    const char* base = reinterpret_cast<const char*>(TH) + addr;
    const uint4 q0 = *reinterpret_cast<const uint4*>(base);
    const uint4 q1 = *reinterpret_cast<const uint4*>(base + 16);
    const uint2 q2 = *reinterpret_cast<const uint2*>(base + 32);
    const int dq = t1 + (int)(m1 ? s.S3 : s.S3mQ);
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    const int code = (int)((addr - s.row) / kThRec) | (sgn & 8);
    s.T4 = q0.x; s.T2 = q0.y; s.T6 = q0.z; s.T1 = q0.w;
    s.T3 = q1.x; s.T5 = q1.y; s.T7 = q1.z; s.S3 = q1.w;
    s.S3mQ = q2.x; s.row = q2.y;
    return code;
}

// V == 2: the index in a register, the step fetched across lanes (ds_bpermute) from two VGPRs
// holding STEP[-1 .. 62] and STEP[63 .. 96] (ends clamped), so the index's clamp is off the path
struct BpState {
    int idx, step, pred;
};

__device__ __forceinline__ int bp_encode(BpState& s, int x, int tabA, int tabB) {
    const int d = x - s.pred;
    const int sgn = d >> 31;
    const int a0 = max(d, -d);
    const int step = s.step, h = step >> 1, q = step >> 2, s3 = step >> 3;
    const bool m4 = a0 >= step;
    const int a1 = m4 ? a0 - step : a0;
    const bool m2 = a1 >= h;
    const int a2 = m2 ? a1 - h : a1;
    const bool m1 = a2 >= q;
    const int nb = s.idx + (m4 ? (m2 ? 6 : 2) : -1);
    const int nr = nb + ((m4 && m1) ? 2 : 0);  // -1 .. 96
    const int slot = nr + 1;                    // 0 .. 97: tabA lanes 0..63, tabB lanes 0..33
    const int va = __builtin_amdgcn_ds_bpermute((slot & 63) << 2, tabA);
    const int vb = __builtin_amdgcn_ds_bpermute((slot & 63) << 2, tabB);
    s.step = slot >= 64 ? vb : va;
    s.idx = min(max(nr, 0), 88);
    const int dq = s3 + (m4 ? step : 0) + (m2 ? h : 0) + (m1 ? q : 0);
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    return (m4 ? 4 : 0) | (m2 ? 2 : 0) | (m1 ? 1 : 0) | (sgn & 8);
}

// V == 3: the production table (adpcm_tab2), but the row of 8 successor records for the
// current (index, sign) is read (two ds_read_b128) as soon as the current record arrives, beside
// the magnitude compares; the next record is then selected by m4, m2, m1 (three select levels)
__device__ __forceinline__ int row_encode(AdpcmTab2& s, int x, const uint32_t* NS2) {
    const int d = x - s.pred;
    const int sgn = d >> 31;
    const int a0 = max(d, -d);
    const uint32_t rec = s.rec;
    const int rb = (int)(rec >> 16) + (sgn & 32);
    const uint4 q0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(NS2) + rb);
    const uint4 q1 = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(NS2) + rb + 16);
    const int step = (int)(rec & 0xffffu);
    const int h = step >> 1, q = step >> 2, s3 = step >> 3;
    const bool m4 = a0 >= step;
    const int a1 = m4 ? a0 - step : a0;
    const bool m2 = a1 >= h;
    const int a2 = m2 ? a1 - h : a1;
    const bool m1 = a2 >= q;
    const int dq = s3 + (m4 ? step : 0) + (m2 ? h : 0) + (m1 ? q : 0);
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    const uint32_t e0 = m4 ? q1.x : q0.x, e1 = m4 ? q1.y : q0.y;
    const uint32_t e2 = m4 ? q1.z : q0.z, e3 = m4 ? q1.w : q0.w;
    const uint32_t f0 = m2 ? e2 : e0, f1 = m2 ? e3 : e1;
    s.rec = m1 ? f1 : f0;
    return (m4 ? 4 : 0) | (m2 ? 2 : 0) | (m1 ? 1 : 0) | (sgn & 8);
}

// V == 4: rows of 8 successor records in reverse magnitude order, indexed by (index * 2 + sign):
// NS3[(2 index + sign) * 8 + (7 - mag)] = next step | (2 next index) << 16.  The word index is
// built by doubling an accumulator and adding each inverted magnitude bit (a compare's result, a
// v_addc carry-in), so the code is the index's low nibble ^ 7 and no select builds an address.
constexpr int kAdpcmTab3Entries = 89 * 16;

__device__ void tab3_fill(uint32_t* NS3, int tid, int nt) {
    for (int e = tid; e < kAdpcmTab3Entries; e += nt) {
        const int index = e >> 4, mag = 7 - (e & 7);
        int ni = index + kAdpcmIndex[mag];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        NS3[e] = (uint32_t)kAdpcmStep[ni] | ((uint32_t)(ni * 2) << 16);
    }
}

struct Tab3 {
    uint32_t rec;  // step | (2 index) << 16
    int pred;
};

__device__ __forceinline__ uint32_t tab3_encode(Tab3& s, int x, const uint32_t* __restrict__ NS3) {
    const int d = x - s.pred;
    const int sgn = d >> 31;
    const uint32_t sb = (uint32_t)d >> 31;
    const int a0 = max(d, -d);
    const uint32_t rec = s.rec;
    const int step = (int)(rec & 0xffffu), h = step >> 1, q = step >> 2, s3 = step >> 3;
    uint32_t acc = (rec >> 16) + sb;
    const bool n4 = a0 < step;
    acc = 2 * acc + (uint32_t)n4;
    const int a1 = n4 ? a0 : a0 - step;
    const bool n2 = a1 < h;
    acc = 2 * acc + (uint32_t)n2;
    const int a2 = n2 ? a1 : a1 - h;
    const bool n1 = a2 < q;
    acc = 2 * acc + (uint32_t)n1;
    s.rec = NS3[acc];
    const int dq = s3 + (n4 ? 0 : step) + (n2 ? 0 : h) + (n1 ? 0 : q);
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    return acc;  // low nibble: code ^ 7
}

// V == 5: tab3's layout with 8-B records {step | (2 index) << 16, h | q << 16}, and the magnitude
// search in one asm block: SDWA compares / selects read the 16-bit fields in place (no unpacking),
// and each compare's VCC is the carry-in of a v_addc that doubles the word-index accumulator.
struct Tab4 {
    uint32_t w0, w1;  // step | (2 index) << 16, h | q << 16
    int pred;
};

__device__ void tab4_fill(uint2* NS4, int tid, int nt) {
    for (int e = tid; e < kAdpcmTab3Entries; e += nt) {
        const int index = e >> 4, mag = 7 - (e & 7);
        int ni = index + kAdpcmIndex[mag];
        ni = ni < 0 ? 0 : (ni > 88 ? 88 : ni);
        const uint32_t st = (uint32_t)kAdpcmStep[ni];
        NS4[e] = make_uint2(st | ((uint32_t)(ni * 2) << 16), (st >> 1) | ((st >> 2) << 16));
    }
}

__device__ __forceinline__ uint32_t tab4_encode(Tab4& s, int x, const uint2* __restrict__ NS4, int zero) {
    const int d = x - s.pred;
    const int sgn = d >> 31;
    const uint32_t sb = (uint32_t)d >> 31;
    int a = max(d, -d);
    uint32_t acc = sb + (s.w0 >> 16);
    int t4, t2, tq;
    uint64_t cy;
    asm volatile(
        "v_cmp_lt_u32_sdwa vcc, %[a], %[w0] src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_addc_co_u32_e64 %[acc], %[cy], %[acc], %[acc], vcc\n\t"
        "v_cndmask_b32_sdwa %[t4], %[w0], %[z], vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD\n\t"
        "v_sub_u32_e32 %[a], %[a], %[t4]\n\t"
        "v_cmp_lt_u32_sdwa vcc, %[a], %[w1] src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_addc_co_u32_e64 %[acc], %[cy], %[acc], %[acc], vcc\n\t"
        "v_cndmask_b32_sdwa %[t2], %[w1], %[z], vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD\n\t"
        "v_sub_u32_e32 %[a], %[a], %[t2]\n\t"
        "v_cmp_lt_u32_sdwa vcc, %[a], %[w1] src0_sel:DWORD src1_sel:WORD_1\n\t"
        "v_addc_co_u32_e64 %[acc], %[cy], %[acc], %[acc], vcc\n\t"
        "v_cndmask_b32_sdwa %[tq], %[w1], %[z], vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
        : [a] "+v"(a), [acc] "+v"(acc), [t4] "=&v"(t4), [t2] "=&v"(t2), [tq] "=&v"(tq), [cy] "=&s"(cy)
        : [w0] "v"(s.w0), [w1] "v"(s.w1), [z] "v"(zero)
        : "vcc");
    const int s3 = (int)((s.w1 & 0xffffu) >> 2);
    const uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(NS4) + (acc << 3));
    s.w0 = r.x;
    s.w1 = r.y;
    const int dq = s3 + t4 + t2 + tq;
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    return acc;  // low nibble: code ^ 7
}

// V == 6: tab4's records and rows, no lane masks at all: per magnitude bit u = a - t (t a 16-bit
// field of the record, read in place by SDWA), acc = alignbit(acc, u, 31) shifts u's sign (the
// inverted bit) into the word index, a = min_u32(a, u) keeps the remainder (u wraps above a when
// a < t); dq = s3 + a0 - a3.  Plain C++: the compiler schedules and pads it.
__device__ __forceinline__ uint32_t tab6_encode(Tab4& s, int x, const uint2* __restrict__ NS4) {
    const int d = x - s.pred;
    const int sgn = d >> 31;
    const uint32_t sb = (uint32_t)d >> 31;
    const uint32_t a0 = (uint32_t)max(d, -d);
    const uint32_t w0 = s.w0, w1 = s.w1;
    uint32_t acc = sb + (w0 >> 16);
    const uint32_t u4 = a0 - (w0 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u4, 31);
    const uint32_t a1 = min(a0, u4);
    const uint32_t u2 = a1 - (w1 & 0xffffu);
    acc = __builtin_amdgcn_alignbit(acc, u2, 31);
    const uint32_t a2 = min(a1, u2);
    const uint32_t u1 = a2 - (w1 >> 16);
    acc = __builtin_amdgcn_alignbit(acc, u1, 31);
    const uint32_t a3 = min(a2, u1);
    const uint2 r = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(NS4) + (acc << 3));
    const int dq = (int)(((w1 & 0xffffu) >> 2) + (a0 - a3));
    s.w0 = r.x;
    s.w1 = r.y;
    const int p = s.pred + ((dq ^ sgn) - sgn);
    s.pred = min(max(p, -32768), 32767);
    return acc;  // low nibble: code ^ 7
}

template <int V>
__global__ void __launch_bounds__(64) kern(const int16_t* __restrict__ x, int n, uint8_t* __restrict__ out,
                                           long long* cyc) {
    __shared__ __align__(16) uint2 NSR[V == 7 ? kAdpcmRemEntries : 1];
    if constexpr (V == 7) adpcm_rem_fill(NSR, threadIdx.x, 64);
    __shared__ __align__(16) uint32_t NS[(V == 5 || V == 6) ? 2 * kAdpcmTab3Entries : (V == 0 || V == 3 || V == 4) ? kAdpcmTab2Entries : kThEntries * (kThRec / 4)];
    if constexpr (V == 0 || V == 3) adpcm_tab2_fill(NS, threadIdx.x, 64);
    else if constexpr (V == 4) tab3_fill(NS, threadIdx.x, 64);
    else if constexpr (V == 5 || V == 6) tab4_fill(reinterpret_cast<uint2*>(NS), threadIdx.x, 64);
    else th_fill(NS, threadIdx.x, 64);
    __syncthreads();
    const int lane = threadIdx.x;
    const int16_t* src = x + (size_t)lane * (n + 16);
    uint8_t* o = out + (size_t)lane * n;
    auto ad2 = adpcm_tab2_state(AdpcmState{0, 0});
    ThState th = th_state(0, 0);
    BpState bp{0, kAdpcmStep[0], 0};
    Tab3 t3{(uint32_t)kAdpcmStep[0], 0};
    Tab4 t4s{(uint32_t)kAdpcmStep[0], (uint32_t)(kAdpcmStep[0] >> 1) | ((uint32_t)(kAdpcmStep[0] >> 2) << 16), 0};
    const int zero = __builtin_amdgcn_readfirstlane(n) * 0;
    AdpcmRem rem = adpcm_rem_state(AdpcmState{0, 0});
    const int la = lane - 1, lb = lane + 63;
    const int tabA = kAdpcmStep[la < 0 ? 0 : la];
    const int tabB = kAdpcmStep[lb > 88 ? 88 : lb];
    int cur[8], nxt[8];
    for (int q = 0; q < 8; ++q) cur[q] = src[q];
    const long long t0 = clock64();
    const long long r0 = wall_clock64();
    for (int j = 0; j < n; j += 8) {
        for (int q = 0; q < 8; ++q) nxt[q] = src[j + 8 + q];
        uint32_t w = 0;
        if constexpr (V == 7) {
#pragma unroll
            for (int u = 0; u < 8; ++u) w |= (adpcm_encode_rem(rem, cur[u], NSR) & 15u) << (4 * u);
            w ^= 0x77777777u;
        } else if constexpr (V == 6) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                w |= (tab6_encode(t4s, cur[u], reinterpret_cast<const uint2*>(NS)) & 15u) << (4 * u);
            w ^= 0x77777777u;
        } else if constexpr (V == 5) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                w |= (tab4_encode(t4s, cur[u], reinterpret_cast<const uint2*>(NS), zero) & 15u) << (4 * u);
            w ^= 0x77777777u;
        } else if constexpr (V == 4) {
#pragma unroll
            for (int u = 0; u < 8; ++u) w |= (tab3_encode(t3, cur[u], NS) & 15u) << (4 * u);
            w ^= 0x77777777u;
        } else
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            int c;
            if constexpr (V == 0) c = adpcm_encode_tab2(ad2, cur[u], NS);
            else if constexpr (V == 1) c = th_encode(th, cur[u], NS);
            else if constexpr (V == 3) c = row_encode(ad2, cur[u], NS);
            else c = bp_encode(bp, cur[u], tabA, tabB);
            w |= (uint32_t)c << (4 * u);
        }
        *reinterpret_cast<uint32_t*>(o + (j >> 1)) = w;
        for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
    }
    const long long t1 = clock64();
    const long long r1 = wall_clock64();
    if (lane == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = r1 - r0;
    }
}

int main() {
    const int S = 64, n = 5000;
    std::vector<int16_t> h((size_t)S * (n + 16));
    srand(3);
    for (int c = 0; c < S; ++c) {
        double y = 0, amp = 2000 + 15000.0 * (c % 7) / 6.0;
        for (int i = 0; i < n + 16; ++i) {
            y = 0.9 * y + (rand() / (double)RAND_MAX - 0.5);
            double v = amp * (0.6 * sin(0.05 * i * (1 + c % 11) + c) + 0.25 * y);
            if (c % 3 == 0) v = (rand() % 65536) - 32768;  // full-scale noise: large steps
            v = v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
            h[(size_t)c * (n + 16) + i] = (int16_t)v;
        }
    }
    int16_t* dx;
    uint8_t *d0, *d1;
    long long* dc;
    hipMalloc(&dx, h.size() * 2);
    hipMemcpy(dx, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&d0, (size_t)S * n);
    hipMalloc(&d1, (size_t)S * n);
    hipMalloc(&dc, 16);
    auto run = [&](const char* name, void (*k)(const int16_t*, int, uint8_t*, long long*), uint8_t* o) {
        long long cyc[2] = {0, 0};
        for (int rep = 0; rep < 5; ++rep) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, n, o, dc);
            hipDeviceSynchronize();
        }
        hipMemcpy(cyc, dc, 16, hipMemcpyDeviceToHost);
        int wrate = 0;
        hipDeviceGetAttribute(&wrate, hipDeviceAttributeWallClockRate, 0);  // kHz
        const double ns = cyc[1] * 1e6 / (double)wrate / n;
        printf("%-44s %7.1f cycles/sample, %6.1f ns/sample (%.2f GHz) (%s)\n", name, cyc[0] / (double)n, ns,
               cyc[0] / (double)n / ns, hipGetErrorString(hipGetLastError()));
    };
    run("tab2 (production chain_adpcm encoder)", kern<0>, d0);
    run("threshold records (64 B successor records)", kern<1>, d1);
    uint8_t* d2;
    hipMalloc(&d2, (size_t)S * n);
    run("index register + ds_bpermute step", kern<2>, d2);
    uint8_t* d3;
    hipMalloc(&d3, (size_t)S * n);
    run("tab2 + successor row read beside the compares", kern<3>, d3);
    std::vector<uint8_t> a((size_t)S * n / 2 * 2), b(a.size());
    hipMemcpy(a.data(), d0, a.size(), hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), d1, b.size(), hipMemcpyDeviceToHost);
    size_t diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("codes differing: %zu of %d bytes\n", diff, S * n / 2);
    hipMemcpy(b.data(), d2, b.size(), hipMemcpyDeviceToHost);
    diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("bpermute codes differing: %zu of %d bytes\n", diff, S * n / 2);
    hipMemcpy(b.data(), d3, b.size(), hipMemcpyDeviceToHost);
    diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("row-prefetch codes differing: %zu of %d bytes\n", diff, S * n / 2);
    uint8_t* d4;
    hipMalloc(&d4, (size_t)S * n);
    run("tab3: reversed rows, accumulated compare bits", kern<4>, d4);
    hipMemcpy(b.data(), d4, b.size(), hipMemcpyDeviceToHost);
    diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("tab3 codes differing: %zu of %d bytes\n", diff, S * n / 2);
    uint8_t* d5;
    hipMalloc(&d5, (size_t)S * n);
    run("tab4: 8-B records, SDWA compares + v_addc index", kern<5>, d5);
    hipMemcpy(b.data(), d5, b.size(), hipMemcpyDeviceToHost);
    diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("tab4 codes differing: %zu of %d bytes\n", diff, S * n / 2);
    uint8_t* d6;
    hipMalloc(&d6, (size_t)S * n);
    run("tab6: 8-B records, sub / alignbit / min (no masks)", kern<6>, d6);
    hipMemcpy(b.data(), d6, b.size(), hipMemcpyDeviceToHost);
    diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("tab6 codes differing: %zu of %d bytes\n", diff, S * n / 2);
    uint8_t* d7;
    hipMalloc(&d7, (size_t)S * n);
    run("adpcm_encode_rem (production, owrx_dev.h)", kern<7>, d7);
    hipMemcpy(b.data(), d7, b.size(), hipMemcpyDeviceToHost);
    diff = 0;
    for (int c = 0; c < S; ++c)
        for (int i = 0; i < n / 2; ++i) diff += a[(size_t)c * n + i] != b[(size_t)c * n + i];
    printf("adpcm_encode_rem codes differing: %zu of %d bytes\n", diff, S * n / 2);
    return 0;
}
