// wf_variants.hip -- waterfall FFT kernels that lost their same-box A/B against the production
// kernels (diagnostic only; included by tools/micro/wf_bench.hip after kernels_waterfall.hip,
// never built into libowrx_amd.so).  Measurements: DESIGN.md section 8 and profiles/r03*_wf_*.
//   wf_fft_lean  radix 16 with every twiddle from an LDS table (swizzled image): ~7 % slower than
//                wf_fft_r16 -- the table reads cost LDS time, which bounds the passes
//   wf_fft_h32   one frame per 512-thread workgroup through a half image, two workgroups per
//                CU: 19.6 us at C3 with one frame per group, but its 64 KiB partial row per
//                frame (or the in-kernel write-through group combine) costs what it gains
//   wf_fft_wl / wf_fft_ip / wf_fft_rx: round-2 variants (wave-local sub-transforms, in-place
//                DIF, power-chain radix 32), same time as wf_fft_r16 or slower
namespace owrx {
// ---- wf_fft_lean: the same product with every twiddle read from an LDS table ---------------
// Stockham radix-16 passes (+ one radix 2/4/8 pass), N/16 threads of 16 points, as wf_fft_r16,
// with the VALU work cut to the butterflies themselves:
//  - every twiddle of a radix-16 pass p >= 1 (Ns = 16^p) is one LDS read of a [15][Ns] table
//    W_(16 Ns)^(r k) (no power chains: 15 complex products per pass less); the last pass's
//    per-thread bases W_N^(q t) stay in registers for the whole group;
//  - the frame image is unpadded and XOR-swizzled (e ^ ((e >> 4) & 15)): conflict-free for the
//    stride-16 stores of pass 0 and every read, and the 8 KiB the padding took hold the tables
//    (N = 16384: 128 KiB image + 31.9 KiB of tables = 163 712 B, one workgroup per CU);
//  - plain FP32 (FMA-contracted) butterflies: a packed FP32 instruction issues in twice the
//    cycles of a scalar one on CDNA4's 32-lane SIMDs, so packing buys nothing here.
// Bins per thread (t + NT m) and the per-group |X|^2 partial rows are the production layout.
template <int LOGN>
struct WfLean {
    static constexpr int N = 1 << LOGN;
    static constexpr int NT = N / 16;
    static constexpr int P16 = LOGN / 4;              // radix-16 passes
    static constexpr int RL = 1 << (LOGN - 4 * P16);  // last radix (1: none)
    static constexpr int BL = 16 / RL;                 // last-pass butterflies per thread
    static constexpr int tsize(int p) { return 15 * (1 << (4 * p)); }
    static constexpr int toff(int p) {
        int o = N;
        for (int i = 1; i < p; ++i) o += tsize(i);
        return o;
    }
    static constexpr size_t kLds = sizeof(float2) * toff(P16);
    static_assert(kLds <= 163840, "one workgroup's LDS");
};

OWRX_DEV int wf_swz(int e) { return e ^ ((e >> 4) & 15); }

template <int LOGN>
__global__ void __launch_bounds__(WfLean<LOGN>::NT)
wf_fft_lean(const float2* __restrict__ blk, int64_t blk_start,
            const WfGroup* __restrict__ groups, const float* __restrict__ window,
            const float2* __restrict__ tw, float* __restrict__ partial) {
    using K = WfLean<LOGN>;
    constexpr int N = K::N, NT = K::NT, P16 = K::P16, RL = K::RL, BL = K::BL;
    // N >= 4096: NT is a multiple of 256, so swz(t + NT m) = swz(t) + NT m
    constexpr bool kLinSwz = (NT % 256) == 0;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int t0 = threadIdx.x;
    WF_RSTAMP(14);
    WF_STAMP(0);
    const WfGroup g = groups[blockIdx.x];
    const int64_t g0 = __builtin_amdgcn_readfirstlane((int)(g.start - blk_start));
    const int hop = __builtin_amdgcn_readfirstlane(g.hop);
    const int nfr = __builtin_amdgcn_readfirstlane(g.nframes);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(blk + g0), 0, (int)(sizeof(float2) * ((int64_t)(nfr - 1) * hop + N)),
        0x00020000);
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0,
                                                      (int)(sizeof(float) * N), 0x00020000);
    auto load_x = [&](int f, float2* v) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int vo = t0 * 8 + f * hop * 8;
            v[r] = make_float2(
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo, r * NT * 8, 0)),
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4, r * NT * 8, 0)));
        }
    };
    float2 nx[16];
    load_x(0, nx);
    // twiddle tables: pass p's [15][Ns] block holds W_(16 Ns)^(r k) = W_N^(r k N / (16 Ns))
#pragma unroll
    for (int p = 1; p < P16; ++p) {
        const int ns = 1 << (4 * p);
        const int sh = LOGN - 4 * (p + 1);
        for (int i = t0; i < K::tsize(p); i += NT) {
            const int r = i / ns + 1, k = i - (r - 1) * ns;
            sm[K::toff(p) + i] = tw[(r * k) << sh];
        }
    }
    float2 tb[RL > 1 ? RL - 1 : 1];  // last pass: W_N^(q t)
#pragma unroll
    for (int q = 1; q < RL; ++q) tb[q - 1] = tw[q * t0];
    float acc[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) acc[m] = 0.0f;
    auto rd = [&](int t, int m) -> float2 {
        return kLinSwz ? sm[wf_swz(t) + NT * m] : sm[wf_swz(t + NT * m)];
    };
#pragma unroll 1
    for (int f = 0; f < nfr; ++f) {
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        float2 a[16];
        const int sb = 1 + 6 * f;
        if (f < 2) WF_STAMP(sb);
        {
            float wv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                wv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, t0 * 4, r * NT * 4, 0));
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = make_float2(nx[r].x * wv[r], nx[r].y * wv[r]);
        }
        if (f + 1 < nfr) load_x(f + 1, nx);
        f2dft<16>(a);
        if (f < 2) WF_STAMP(sb + 1);
        __syncthreads();  // the previous frame's last reads (and, at f = 0, the tables)
        // pass 0 (Ns = 1): out[16 t + k]
#pragma unroll
        for (int k = 0; k < 16; ++k) sm[16 * t + (k ^ (t & 15))] = a[k];
        if (f < 2) WF_STAMP(sb + 2);
#pragma unroll
        for (int p = 1; p < P16; ++p) {
            const int ns = 1 << (4 * p);
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = rd(t, r);
            const int k = t & (ns - 1);
            const float2* T = sm + K::toff(p) + k;
#pragma unroll
            for (int r = 1; r < 16; ++r) a[r] = f2mul(a[r], T[(r - 1) * ns]);
            f2dft<16>(a);
            if (p == P16 - 1 && RL == 1) {
                // Ns = N / 16 = NT: outputs t + NT r are this thread's bins
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = fmaf(a[r].y, a[r].y, fmaf(a[r].x, a[r].x, acc[r]));
            } else {
                __syncthreads();  // every read of this pass before any store
                const int base = (t >> (4 * p)) * (16 * ns) + k;
#pragma unroll
                for (int r = 0; r < 16; ++r) sm[wf_swz(base + ns * r)] = a[r];
            }
            if (f < 2) WF_STAMP(sb + 2 + p);
        }
        if constexpr (RL > 1) {
            __syncthreads();
#pragma unroll
            for (int m = 0; m < 16; ++m) a[m] = rd(t, m);
            // butterfly j = t + NT b (b < BL), inputs a[b + BL q], twiddles W_N^(q t) W_16^(q b)
#pragma unroll
            for (int b = 0; b < BL; ++b) {
                float2 c[RL];
#pragma unroll
                for (int q = 0; q < RL; ++q) c[q] = a[b + BL * q];
#pragma unroll
                for (int q = 1; q < RL; ++q) {
                    float2 w = tb[q - 1];
                    if (b) w = f2mul(w, w16c((q * b) & 15));
                    c[q] = f2mul(c[q], w);
                }
                f2dft<RL>(c);
#pragma unroll
                for (int q = 0; q < RL; ++q)
                    acc[b + BL * q] = fmaf(c[q].y, c[q].y, fmaf(c[q].x, c[q].x, acc[b + BL * q]));
            }
        }
        if (f < 2) WF_STAMP(sb + 5);
    }
    float* out = partial + (int64_t)blockIdx.x * N;
#pragma unroll
    for (int m = 0; m < 16; ++m) out[t0 + NT * m] = acc[m];
    WF_STAMP(13);
    WF_RSTAMP(15);
}

// ---- wf_fft_h32: one frame per workgroup, two workgroups per CU ------------------------------
// The single-image kernels hold one frame per CU, so every pass is its LDS reads, then its VALU,
// then its LDS stores, one after the other (phase stamps: ~5 k cycles per pass = the three
// summed).  Here a 512-thread workgroup transforms ONE frame (16384 = 32 x 32 x 16, the l32
// factorisation) through a HALF image (8192 cf32 = 64 KiB): each exchange goes in two rounds
// (all threads store the half of their outputs that waves 0-3 read, barrier, waves 0-3 read,
// barrier, the other half for waves 4-7).  72 KiB of LDS and <= 128 VGPRs per workgroup put two
// workgroups (frames) on a CU, whose passes interleave: one's stores run under the other's
// butterflies.  No register prefetch and no accumulators across passes (the co-resident frame
// covers the load latency; one frame per workgroup).
// A group of G consecutive frames of a row (G = WfFrame::members) sums its |X|^2 in the kernel:
// every member writes its row to its slot, and the last member to finish (agent-scope ticket)
// adds the others' rows to its own in member order -- a fixed order whatever the arrival order,
// so the group's partial row is bit-reproducible -- and writes the group partial that
// wf_finalize reads.  Members of a group are placed on one XCD (host-side workgroup order).
struct WfFrame {
    int64_t start;    // stream index of the frame
    int32_t group;    // group (partial row) index
    int16_t member;   // index within the group
    int16_t members;  // frames in the group
};
struct WfH32 {
    static constexpr int LOGN = 14, N = 1 << LOGN, NT = 512, H = N / 2;
    static constexpr int TW2 = H;  // [31][32]: W_1024^(r k)
    static constexpr size_t kLds = sizeof(float2) * (H + 31 * 32);
};
OWRX_DEV int wf_swz16(int e) { return e ^ ((e >> 4) & 15); }

__global__ void __launch_bounds__(WfH32::NT, 4)
wf_fft_h32(const float2* __restrict__ blk, int64_t blk_start, const WfFrame* __restrict__ frames,
           const float* __restrict__ window, const float2* __restrict__ tw,
           float* __restrict__ member_rows, int* __restrict__ tickets, float* __restrict__ partial) {
    using K = WfH32;
    constexpr int N = K::N, NT = K::NT;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ int s_last;
    const int t = threadIdx.x;
    const WfFrame fr = frames[blockIdx.x];
    if (fr.members == 0) return;  // padding slot of the XCD-aware order
    const int64_t f0 = __builtin_amdgcn_readfirstlane((int)(fr.start - blk_start));
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(blk + f0), 0,
                                                      (int)(sizeof(float2) * N), 0x00020000);
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0,
                                                      (int)(sizeof(float) * N), 0x00020000);
    // L2-resident tables first (vmcnt retires in order), then the frame and its window taps
    float2 t2v[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int e = t + NT * i;
        t2v[i] = e < 31 * 32 ? tw[(((e >> 5) + 1) * (e & 31)) << 4] : make_float2(0.f, 0.f);
    }
    float2 tp[4];  // W_N^(2^i t)
#pragma unroll
    for (int i = 0; i < 4; ++i) tp[i] = tw[(t << i) & (N - 1)];
    float2 a[32];
    {
        float wv[32];
#pragma unroll
        for (int r = 0; r < 32; ++r) {
            a[r] = make_float2(
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, t * 8, r * NT * 8, 0)),
                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, t * 8 + 4, r * NT * 8, 0)));
            wv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, t * 4, r * NT * 4, 0));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if (t + NT * i < 31 * 32) sm[K::TW2 + t + NT * i] = t2v[i];
#pragma unroll
        for (int r = 0; r < 32; ++r) a[r] = make_float2(a[r].x * wv[r], a[r].y * wv[r]);
    }
    // P1 (Ns = 1): x[t + 512 r] -> DFT32 -> element 32 t + k
    f2dft32(a);
    // Both exchanges go through the image in halves: round h holds elements [8192 h, 8192 h +
    // 8192), which waves 4h..4h+3 write (all their outputs) and every thread reads (the 16 of
    // its 32 inputs there).  Stores are the conditional side, so no register array has two
    // definitions; at most 32 outputs + 16 inputs are live.  Swizzled as l32 (e ^ ((e >> 5) & 15)).
    const int h = t >> 8;
    const int sw = wf_swz32(t);  // swz(t + 512 r) = swz(t) + 512 r
    float2 b[32];
#pragma unroll
    for (int rnd = 0; rnd < 2; ++rnd) {
        if (rnd) __syncthreads();  // round 0's reads done
        if (h == rnd) {
#pragma unroll
            for (int k = 0; k < 32; ++k) sm[32 * (t & 255) + (k ^ (t & 15))] = a[l32_at(k)];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) b[16 * rnd + r] = sm[sw + NT * r];
    }
    // P2 (Ns = 32): butterfly j = t, k = t & 31, twiddles W_1024^(r k) from the table
    {
        const int k = t & 31;
        const float2* T = sm + K::TW2 + k;
#pragma unroll
        for (int r = 1; r < 32; ++r) {
            b[r] = f2mul(b[r], T[(r - 1) * 32]);
            if ((r & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // <= 8 twiddles in registers
        }
        f2dft32(b);
    }
    // exchange 2: element (t >> 5) 1024 + (t & 31) + 32 r' (half (t >> 8)); P3 reads t + 512 m
    {
        const int base = ((t & 255) >> 5) * 1024 + (t & 31);
#pragma unroll
        for (int rnd = 0; rnd < 2; ++rnd) {
            __syncthreads();  // the previous reads done
            if (h == rnd) {
#pragma unroll
                for (int r = 0; r < 32; ++r) sm[wf_swz32(base + 32 * r)] = b[l32_at(r)];
            }
            __syncthreads();
#pragma unroll
            for (int m = 0; m < 16; ++m) a[16 * rnd + m] = sm[sw + NT * m];
        }
    }
    // P3 (Ns = 1024): butterflies t + 512 bb, inputs a[bb + 2 r], twiddles W_N^(r t) W_32^(r bb),
    // W_N^(r t) the product of the exact powers W_N^(2^i t) of r's bits (registers are short at
    // four waves per SIMD); each |X|^2 goes straight to the partial row (a one-frame group) or
    // to this member's row, stored write-through (sc1) for the group's last member to read
    const int G = fr.members;
    float* const direct = partial + (int64_t)fr.group * N;
    const auto mr = __builtin_amdgcn_make_buffer_rsrc(member_rows + (int64_t)blockIdx.x * N, 0,
                                                      (int)(sizeof(float) * N), 0x00020000);
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
        float2 c[16];
        c[0] = a[bb];
#pragma unroll
        for (int r = 1; r < 16; ++r) {
            float2 w = make_float2(1.0f, 0.0f);
            bool first = true;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (r & (1 << i)) {
                    w = first ? tp[i] : f2mul(w, tp[i]);
                    first = false;
                }
            c[r] = f2mul(a[bb + 2 * r], bb ? f2mul32(w, r) : w);
        }
        f2dft<16>(c);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float p = fmaf(c[r].y, c[r].y, c[r].x * c[r].x);
            const int bin = t + NT * (bb + 2 * r);
            if (G == 1)
                direct[bin] = p;
            else
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, p), mr, bin * 4, 0, 16);
        }
    }
    if (G == 1) return;
    // hand-off without fences (cdna_hip_programming.md Guideline 16, R1): every storing wave
    // drains its write-through stores, the workgroup's barrier, one relaxed agent-scope ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
        const int old = __hip_atomic_fetch_add(tickets + fr.group, 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == G - 1;
        if (old == G - 1) __hip_atomic_store(tickets + fr.group, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the loads below the ticket
    // the members' workgroups: this one's index minus 8 per member before it (host order); every
    // load of their rows is write-through (sc1), each member's 32 values loaded together, then
    // added in member order
    float sacc[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) sacc[m] = 0.0f;
    for (int mb = 0; mb < G; ++mb) {
        const auto orr = __builtin_amdgcn_make_buffer_rsrc(
            member_rows + ((int64_t)blockIdx.x + 8 * (mb - fr.member)) * N, 0,
            (int)(sizeof(float) * N), 0x00020000);
        float v[32];
#pragma unroll
        for (int m = 0; m < 32; ++m)
            v[m] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(orr, (t + NT * m) * 4, 0, 16));
#pragma unroll
        for (int m = 0; m < 32; ++m) sacc[m] += v[m];
    }
#pragma unroll
    for (int m = 0; m < 32; ++m) direct[t + NT * m] = sacc[m];
}

// ---- wf_fft_wl: N = 16384 as 16 x 1024 with wave-local sub-transforms (production, C2/C3) --
// Same product as wf_fft_r16.  Only the first radix-16 pass is a workgroup step: thread t
// (1024 threads) takes x[t + 1024 r] from HBM (times the window), DFT16 over r, twiddles by
// W_N^(t k1) and stores Y[k1][t] into region k1 of LDS; one barrier.  Region k1 is then one
// independent 1024-point DFT (X[k1 + 16 k2] = sum_t Y[k1][t] W_1024^(t k2)), done by wave k1
// alone: t = l + 64 r (DFT16 over r, twiddle W_1024^(l j1)), l = s + 4 m (DFT16 over m, twiddle
// W_64^(s j2a)), DFT4 over s, with k2 = j1 + 16 j2a + 256 j2b.  Its two exchanges go through the
// wave's own region, ordered by the in-order LDS queue of one wave (no workgroup barrier), so
// sixteen waves interleave one's LDS traffic with another's butterflies instead of the whole
// workgroup alternating VALU and LDS phases between barriers.  One more barrier per frame
// before the next frame's first-pass stores reuse the regions.  All twiddles are powers of
// W_N^t, t < 1024 (an LDS table behind the regions).
struct WfWl {
    static constexpr int LOGN = 14, N = 1 << LOGN, NT = 1024;
    static constexpr int PT = 68;                  // exchange 1 row pitch: T[j1][l], 64 + 4
    static constexpr int PJ = 17;                  // exchange 2: U[s][j2a][j1] at s PU + j2a PJ + j1
    static constexpr int PU = 16 * PJ;
    static constexpr int REG = 16 * PT;            // region of one wave (>= 1024, >= 4 PU)
    static constexpr int TW0 = 16 * REG;
    static constexpr size_t kLds = sizeof(float2) * (TW0 + NT);
    static_assert(REG >= 1024 && REG >= 4 * PU, "region");
};

OWRX_DEV void wl_wave_fence() {  // order one wave's LDS accesses across lanes (in-order queue)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v_permlane32_swap: lanes 32..63 of p <-> lanes 0..31 of q; v_permlane16_swap: the odd rows
// of p <-> the even rows of q (rows of 16 lanes), both components.  (Scalar temporaries: this
// hipcc folds __builtin_bit_cast of a vector element into the wrong element.)
template <bool S32>
OWRX_DEV void wl_swap1(float& a, float& b) {
    const unsigned ua = __float_as_uint(a), ub = __float_as_uint(b);
    unsigned r0, r1;
    if constexpr (S32) {
        const auto r = __builtin_amdgcn_permlane32_swap(ua, ub, false, false);
        r0 = r[0];
        r1 = r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane16_swap(ua, ub, false, false);
        r0 = r[0];
        r1 = r[1];
    }
    a = __uint_as_float(r0);
    b = __uint_as_float(r1);
}
template <bool S32>
OWRX_DEV void wl_swap(c2& p, c2& q) {
    float px = p.x, py = p.y, qx = q.x, qy = q.y;
    wl_swap1<S32>(px, qx);
    wl_swap1<S32>(py, qy);
    p = c2{px, py};
    q = c2{qx, qy};
}

// XL: the last radix-4 stage across the wave's rows with lane swaps instead of an LDS exchange
template <bool XL>
__global__ void __launch_bounds__(WfWl::NT)
wf_fft_wl(const float2* __restrict__ blk, int64_t blk_start, const WfGroup* __restrict__ groups,
          const float* __restrict__ window, const float2* __restrict__ tw,
          float* __restrict__ partial) {
    using K = WfWl;
    constexpr int N = K::N, NT = K::NT;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int tid0 = threadIdx.x;
    const WfGroup g = groups[blockIdx.x];
    const int64_t g0 = __builtin_amdgcn_readfirstlane((int)(g.start - blk_start));
    const int hop = __builtin_amdgcn_readfirstlane(g.hop);
    const int nfr = __builtin_amdgcn_readfirstlane(g.nframes);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(blk + g0), 0, (int)(sizeof(float2) * ((int64_t)(nfr - 1) * hop + N)),
        0x00020000);
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0,
                                                      (int)(sizeof(float) * N), 0x00020000);
    auto load_x = [&](int f, c2* v) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int vo = tid0 * 8 + f * hop * 8;
            v[r] = c2{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo, r * NT * 8, 0)),
                      __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4, r * NT * 8, 0))};
        }
    };
    c2 nx[16];
    load_x(0, nx);
    sm[K::TW0 + tid0] = tw[tid0];  // W_N^t, t < 1024
    const int wave = tid0 >> 6, lane = tid0 & 63;
    float acc[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) acc[m] = 0.0f;
    __syncthreads();
#pragma unroll 1
    for (int f = 0; f < nfr; ++f) {
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        c2 a[16];
        {   // pass 0 (workgroup): windowed samples, DFT16 over r, twiddle W_N^(t k1), Y[k1][t]
            float wv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                wv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, tid0 * 4, r * NT * 4, 0));
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = nx[r] * wv[r];
        }
        __builtin_amdgcn_sched_barrier(0);
        dft_r<16>(a);
        if (tid) twiddle_r<16>(a, c2_of(sm[K::TW0 + tid]));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) sm[k1 * K::REG + tid] = f2_of(a[k1]);
        if (f + 1 < nfr) load_x(f + 1, nx);
        __syncthreads();
        // wave-local 1024-point DFT of region `wave`
        float2* R = sm + wave * K::REG;
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int r = 0; r < 16; ++r) a[r] = c2_of(R[ln + 64 * r]);
        __builtin_amdgcn_sched_barrier(0);
        dft_r<16>(a);
        if (ln) twiddle_r<16>(a, c2_of(sm[K::TW0 + 16 * ln]));  // W_1024^(l j1)
        __builtin_amdgcn_sched_barrier(0);
        wl_wave_fence();  // every lane's reads of Y before the region is rewritten
#pragma unroll
        for (int j1 = 0; j1 < 16; ++j1) R[j1 * K::PT + ln] = f2_of(a[j1]);
        wl_wave_fence();
        const int j1 = ln & 15, s = ln >> 4;
#pragma unroll
        for (int m = 0; m < 16; ++m) a[m] = c2_of(R[j1 * K::PT + s + 4 * m]);
        __builtin_amdgcn_sched_barrier(0);
        dft_r<16>(a);
        if (s) twiddle_r<16>(a, c2_of(sm[K::TW0 + 256 * s]));  // W_64^(s j2a)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!XL) {
            wl_wave_fence();
#pragma unroll
            for (int j2a = 0; j2a < 16; ++j2a) R[s * K::PU + j2a * K::PJ + j1] = f2_of(a[j2a]);
            wl_wave_fence();
            // lane (j1, gq = s): DFT4 over s of (j1, j2a = 4 gq + u), u < 4
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int j2a = 4 * s + u;
                c2 c[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) c[q] = c2_of(R[q * K::PU + j2a * K::PJ + j1]);
                dft4(c[0], c[1], c[2], c[3]);
#pragma unroll
                for (int j2b = 0; j2b < 4; ++j2b)
                    acc[4 * u + j2b] = fmaf(c[j2b].y, c[j2b].y, fmaf(c[j2b].x, c[j2b].x, acc[4 * u + j2b]));
            }
        } else {
            // DFT4 over s = the lane's row (16 lanes) without LDS: registers j2a = 2i, 2i + 1
            // meet in v_permlane32_swap (rows r, r + 2: s bit 1), then the b0 = 1 half of the
            // odd rows takes W4 = -i, then v_permlane16_swap (rows r, r + 1: s bit 0).  Lane
            // (j1, row) ends with register 2i + row / 2, outputs j2b = row % 2 (F0) and
            // row % 2 + 2 (F1).
            const bool odd = s & 1;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                c2 P = a[2 * i], Q = a[2 * i + 1];
                wl_swap<true>(P, Q);
                c2 X = P + Q, Y = P - Q;
                if (odd) Y = c2{Y.y, -Y.x};
                wl_swap<false>(X, Y);
                const c2 F0 = X + Y, F1 = X - Y;
                acc[2 * i] = fmaf(F0.y, F0.y, fmaf(F0.x, F0.x, acc[2 * i]));
                acc[2 * i + 1] = fmaf(F1.y, F1.y, fmaf(F1.x, F1.x, acc[2 * i + 1]));
            }
        }
        __syncthreads();  // regions reused by the next frame's first pass
    }
    // bin of acc[4 u + j2b]: k = wave + 16 j1 + 256 (4 gq + u) + 4096 j2b; the row goes out
    // through LDS in bin order (k + k/16 + k/1024 spreads one store's lanes over the banks) so
    // that the partial row is written with coalesced stores
    float* rowl = reinterpret_cast<float*>(sm);
    auto raddr = [](int k) { return k + (k >> 4) + (k >> 10); };
    {
        const int j1 = lane & 15, gq = lane >> 4;
        if constexpr (!XL) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int j2b = 0; j2b < 4; ++j2b)
                    rowl[raddr(wave + 16 * j1 + 256 * (4 * gq + u) + 4096 * j2b)] = acc[4 * u + j2b];
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    rowl[raddr(wave + 16 * j1 + 256 * (2 * i + (gq >> 1)) + 4096 * ((gq & 1) + 2 * h))] =
                        acc[2 * i + h];
        }
    }
    __syncthreads();
    float* out = partial + (int64_t)blockIdx.x * N;
#pragma unroll
    for (int r = 0; r < 16; ++r) out[tid0 + r * NT] = rowl[raddr(tid0 + r * NT)];
}

// ---- wf_fft_ip<LOGN>: in-place decimation-in-frequency (A/B: OWRX_WF_KERNEL=ip) ------------
// Same product as wf_fft_r16 (|X|^2 of the group's windowed frames summed per bin), with the
// passes done in place: stage s reads 16 samples of one length-L_s sub-transform (stride
// S_s = L_s / 16), takes the DFT16, twiddles output q by W_(L_s)^(n q) and writes it back to the
// addresses it read.  No thread overwrites another's inputs, so a stage needs one barrier (its
// reads after the previous stage's stores) instead of two, and each wave's stores follow its
// own DFT without waiting for every wave's reads.  The last stage (radix RL, or the last
// radix-16 stage when N is a power of 16) reads 16 consecutive samples per thread and leaves the
// bins in digit-reversed positions; the bin index is recomputed when the partial row goes out
// (through LDS, coalesced).  With the 1-in-16 padding every stage's reads and stores are free of
// LDS bank conflicts.  Twiddle bases W_(L_s)^n come from per-stage LDS tables.
template <int LOGN>
struct WfIp {
    static constexpr int N = 1 << LOGN;
    static constexpr int NT = N / 16;
    static constexpr int P16 = LOGN / 4;                      // radix-16 stages
    static constexpr int RL = 1 << (LOGN - 4 * P16);          // last radix (1: none)
    static constexpr int NS = RL > 1 ? P16 : P16 - 1;         // stages that twiddle and store
    static constexpr int stride(int s) { return N >> (4 * (s + 1)); }  // S_s
    static constexpr int tab(int s) {                         // table offset of stage s
        int o = 0;
        for (int i = 0; i < s; ++i) o += stride(i);
        return o;
    }
    static constexpr int TW0 = N + N / 16;
    static constexpr size_t kLds = sizeof(float2) * (TW0 + tab(NS));
    // The partial row goes through LDS by bin: thread t's bins differ from its neighbours' in
    // five bin bits (lane bit i moves position bit i + 4, i.e. digit bit kbit(i) of the bin).
    // The row is stored at k ^ swz(k), swz built from the bits above 4 only, so that those five
    // bits land on five different bank bits (stores conflict-free) while 32 consecutive bins
    // still cover all banks (the coalesced read-out conflict-free).
    static constexpr int kbit(int i) {
        const int e = i + 4, st = (LOGN - e - 1) / 4;  // stage whose stride S satisfies S <= 2^e < 16 S
        return 4 * st + e - (LOGN - 4 * st - 4);
    }
    static constexpr unsigned swz_vec(int b) {  // XOR vector of bin bit b >= 5 (0: none)
        unsigned used = 0;
        for (int i = 0; i < 5; ++i)
            if (kbit(i) < 5) used |= 1u << kbit(i);
        for (int i = 0, free_bit = 0; i < 5; ++i) {
            if (kbit(i) < 5) continue;
            while (used & (1u << free_bit)) ++free_bit;
            used |= 1u << free_bit;
            if (kbit(i) == b) return 1u << free_bit;
        }
        return 0;
    }
};

template <int LOGN>
OWRX_DEV int wf_ip_row_addr(int k) {
    unsigned x = 0;
#pragma unroll
    for (int b = 5; b < LOGN; ++b)
        if (WfIp<LOGN>::swz_vec(b)) x ^= ((k >> b) & 1) ? WfIp<LOGN>::swz_vec(b) : 0u;
    return k ^ (int)x;
}

template <int LOGN>
__global__ void __launch_bounds__(WfIp<LOGN>::NT)
wf_fft_ip(const float2* __restrict__ blk, int64_t blk_start, const WfGroup* __restrict__ groups,
          const float* __restrict__ window, const float2* __restrict__ tw, float* __restrict__ partial) {
    using K = WfIp<LOGN>;
    constexpr int N = K::N, NT = K::NT, P16 = K::P16, RL = K::RL, NS = K::NS;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int tid0 = threadIdx.x;
    const WfGroup g = groups[blockIdx.x];
    WF_STAMP(0);
    // frame samples and window taps through buffer descriptors (one VGPR of lane offset), the
    // first frame requested before the twiddle tables (vmcnt is in order)
    const int64_t g0 = __builtin_amdgcn_readfirstlane((int)(g.start - blk_start));
    const int hop = __builtin_amdgcn_readfirstlane(g.hop);
    const int nfr = __builtin_amdgcn_readfirstlane(g.nframes);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(blk + g0), 0, (int)(sizeof(float2) * ((int64_t)(nfr - 1) * hop + N)),
        0x00020000);
    const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(window), 0,
                                                      (int)(sizeof(float) * N), 0x00020000);
    auto load_x = [&](int f, c2* v) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // two dword loads paired into one dwordx2 (this hipcc's vector-returning
            // raw_buffer_load_b64 / _b128 builtins load one dword and splat it)
            const int vo = tid0 * 8 + f * hop * 8;
            v[r] = c2{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo, r * NT * 8, 0)),
                      __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, vo + 4, r * NT * 8, 0))};
        }
    };
    c2 nx[16];
    load_x(0, nx);
    // twiddle bases: stage 0's W_N^tid stays in a register (each thread uses only its own); the
    // later stages' tables (N/256 + N/4096 + ... entries) go to LDS, written in frame 0 before the
    // stage-1 barrier so no load latency is waited for before the first DFT
    const c2 tw0 = c2_of(tw[tid0]);
    constexpr int NTAB1 = K::tab(NS) - K::tab(1);  // entries of stages >= 1
    float2 tw1 = float2{0.0f, 0.0f};
    int tab_i = 0;
    if (NTAB1 > 0 && tid0 < NTAB1) {
        int s = 1, n = tid0;
        while (s < NS && n >= K::stride(s)) n -= K::stride(s++);
        tab_i = K::TW0 + K::tab(s) + n;
        tw1 = tw[n << (4 * s)];
    }
    float acc[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) acc[m] = 0.0f;
#pragma unroll 1
    for (int f = 0; f < nfr; ++f) {
        int tid = threadIdx.x;  // opaque: keeps the stage addresses inside the frame loop
        asm volatile("" : "+v"(tid));
        const int st0 = 1 + 6 * f;
        WF_STAMP(st0);
        c2 a[16];
        {
            float wv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r)
                wv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, tid0 * 4, r * NT * 4, 0));
#pragma unroll
            for (int r = 0; r < 16; ++r) a[r] = nx[r] * wv[r];
        }
        WF_STAMP(st0 + 1);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int S = K::stride(s);
            const int n = tid & (S - 1);
            const int base = (tid / S) * (16 * S) + n;  // sub-transform start + n
            if (s > 0) {
                __syncthreads();  // the previous stage's stores
#pragma unroll
                for (int m = 0; m < 16; ++m) a[m] = c2_of(sm[wf_pad(base + m * S)]);
            }
            __builtin_amdgcn_sched_barrier(0);
            dft_r<16>(a);
            if (n) twiddle_r<16>(a, s == 0 ? tw0 : c2_of(sm[K::TW0 + K::tab(s) + n]));  // W_(16 S)^(n q)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 16; ++q) sm[wf_pad(base + q * S)] = f2_of(a[q]);
            if (s == 0 && f == 0 && NTAB1 > 0 && tid0 < NTAB1) sm[tab_i] = tw1;
            if (s == 0 && f + 1 < nfr) load_x(f + 1, nx);
            WF_STAMP(st0 + 2 + s);
        }
        __syncthreads();
        // last stage: 16 consecutive samples per thread
        if constexpr (RL > 1) {
#pragma unroll
            for (int j = 0; j < 16 / RL; ++j) {
                c2 c[RL];
#pragma unroll
                for (int n = 0; n < RL; ++n) c[n] = c2_of(sm[wf_pad(16 * tid + RL * j + n)]);
                dft_r<RL>(c);
#pragma unroll
                for (int q = 0; q < RL; ++q)
                    acc[j * RL + q] = fmaf(c[q].y, c[q].y, fmaf(c[q].x, c[q].x, acc[j * RL + q]));
            }
        } else {
#pragma unroll
            for (int m = 0; m < 16; ++m) a[m] = c2_of(sm[wf_pad(16 * tid + m)]);
            dft_r<16>(a);
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = fmaf(a[q].y, a[q].y, fmaf(a[q].x, a[q].x, acc[q]));
        }
        WF_STAMP(st0 + 5);
        __syncthreads();  // LDS reused by the next frame (and by the row below)
    }
    // bins: position p = 16 tid + RL j holds, after stage s, digit q_s = (p / S_s) % 16 of the
    // bin (weight 16^s); the last stage's output q has weight 16^(number of earlier stages)
    float* rowl = reinterpret_cast<float*>(sm);
    constexpr int NE = RL > 1 ? P16 : P16 - 1;  // stages before the last
    constexpr int WL = 1 << (4 * NE);
#pragma unroll
    for (int j = 0; j < (RL > 1 ? 16 / RL : 1); ++j) {
        const int p = 16 * tid0 + (RL > 1 ? RL : 16) * j;
        int k0 = 0;
#pragma unroll
        for (int s = 0; s < NE; ++s) k0 += ((p / K::stride(s)) & 15) << (4 * s);
        constexpr int Q = RL > 1 ? RL : 16;
#pragma unroll
        for (int q = 0; q < Q; ++q) rowl[wf_ip_row_addr<LOGN>(k0 + q * WL)] = acc[j * Q + q];
    }
    __syncthreads();
    float* out = partial + (int64_t)blockIdx.x * N;
    for (int i = tid0; i < N; i += NT) out[i] = rowl[wf_ip_row_addr<LOGN>(i)];
    WF_STAMP(13);
}

// ---- wf_fft_rx<LOGN, R>: the same product with radix-R passes, N/R threads -----------------
// R = 32: 512 threads of 32 points at N = 16384, two LDS round trips per frame (radix 32, 32,
// then a last radix 16) instead of three; |X|^2 summed in fp32 per bin (one register per bin).
// The LDS image is padded one element in R.  Selected by OWRX_WF_KERNEL=r32 (A/B).
template <int LOGN, int R>
struct WfRx {
    static constexpr int LOGR = R == 16 ? 4 : 5;
    static constexpr int N = 1 << LOGN;
    static constexpr int NT = N / R;
    static constexpr int PR = LOGN / LOGR;                      // radix-R passes
    static constexpr int RL = 1 << (LOGN - LOGR * PR);          // last radix (1: none)
    static constexpr int BL = RL > 1 ? N / RL / NT : 1;         // butterflies / thread, last
    static constexpr int NACC = RL > 1 ? BL * RL : R;           // bins per thread
    static constexpr size_t kLds = sizeof(float2) * (N + N / R);
    OWRX_DEV static int pad(int i) { return i + (i >> LOGR); }
};

template <int LOGN, int R>
__global__ void __launch_bounds__((WfRx<LOGN, R>::NT))
wf_fft_rx(const float2* __restrict__ blk, int64_t blk_start,
          const WfGroup* __restrict__ groups, const float* __restrict__ window,
          const float2* __restrict__ tw, float* __restrict__ partial) {
    using K = WfRx<LOGN, R>;
    constexpr int N = K::N, NT = K::NT, PR = K::PR, RL = K::RL, BL = K::BL;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int tid0 = threadIdx.x;
    const WfGroup g = groups[blockIdx.x];
    float acc[K::NACC];  // sum |X|^2 per bin
#pragma unroll
    for (int m = 0; m < K::NACC; ++m) acc[m] = 0.0f;
    c2 nx[R];  // the next frame's samples, loaded while this frame's LDS passes run
#pragma unroll
    for (int r = 0; r < R; ++r) nx[r] = c2_of(blk[g.start - blk_start + tid0 + r * NT]);
#pragma unroll 1
    for (int f = 0; f < g.nframes; ++f) {
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));  // keeps each pass's address arithmetic in the loop
        c2 a[R];
#pragma unroll
        for (int r = 0; r < R; ++r) a[r] = nx[r] * window[tid + r * NT];
        int ns = 1;
#pragma unroll
        for (int pass = 0; pass < PR; ++pass) {
            if (pass > 0) {
                __syncthreads();  // the previous pass's stores
#pragma unroll
                for (int r = 0; r < R; ++r) a[r] = c2_of(sm[K::pad(tid + r * NT)]);
                const int k = tid & (ns - 1);
                if (k) twiddle_r<R>(a, c2_of(tw[k * (N / (ns * R))]));  // W_(R Ns)^k
            }
            __builtin_amdgcn_sched_barrier(0);
            dft_r<R>(a);
            __builtin_amdgcn_sched_barrier(0);
            const bool last = (pass == PR - 1) && RL == 1;
            if (last) {
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r] = fmaf(a[r].x, a[r].x, fmaf(a[r].y, a[r].y, acc[r]));
            } else {
                if (pass > 0) __syncthreads();  // every load of this pass before any store
                const int k = tid & (ns - 1);
                const int d = ((tid / ns) * ns * R) + k;
#pragma unroll
                for (int r = 0; r < R; ++r) sm[K::pad(d + r * ns)] = f2_of(a[r]);
                if (pass == 0 && f + 1 < g.nframes) {
                    const float2* xn = blk + (g.start + (int64_t)(f + 1) * g.hop - blk_start);
#pragma unroll
                    for (int r = 0; r < R; ++r) nx[r] = c2_of(xn[tid + r * NT]);
                }
            }
            ns *= R;
        }
        if constexpr (RL > 1) {
            // last pass: radix RL, Ns = N / RL, butterflies j = tid + b NT, outputs j + r N/RL
            __syncthreads();
#pragma unroll
            for (int b = 0; b < BL; ++b) {
                const int j = tid + b * NT;
                c2 c[RL];
#pragma unroll
                for (int r = 0; r < RL; ++r) c[r] = c2_of(sm[K::pad(j + r * (N / RL))]);
                if (j) twiddle_r<RL>(c, c2_of(tw[j]));  // W_N^(r j)
                dft_r<RL>(c);
#pragma unroll
                for (int r = 0; r < RL; ++r)
                    acc[b * RL + r] = fmaf(c[r].x, c[r].x, fmaf(c[r].y, c[r].y, acc[b * RL + r]));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __syncthreads();  // LDS reused by the next frame
    }
    float* out = partial + (int64_t)blockIdx.x * N;
    if constexpr (RL > 1) {
#pragma unroll
        for (int b = 0; b < BL; ++b)
#pragma unroll
            for (int r = 0; r < RL; ++r) out[tid0 + b * NT + r * (N / RL)] = acc[b * RL + r];
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) out[tid0 + r * NT] = acc[r];
    }
}

// ---- wf_fft_b2: N = 16384 at two workgroups per CU ------------------------------------------
// The one-workgroup-per-CU kernels above run a frame's loads, DFTs and LDS exchanges one after
// the other (the 128 KiB image fills the CU's LDS).  This one keeps the image to 66 KiB so two
// workgroups share a CU and each one's exchanges run under the other's DFTs, and inside a
// workgroup it splits every exchange into two rounds whose stores drain under the next stage's
// arithmetic.
//
// n = 1024 m1 + 64 m2 + 4 m3 + 2 n1 + n0, decimation in frequency:
//   S1: DFT16 over m1 -> k1, * W_16384^(k1 (n mod 1024))
//   S2: DFT16 over m2 -> k2, * W_1024^(k2 (n mod 64))
//   S3: DFT16 over m3 -> k3
//   S4: * W_64^(k3 (2 n1 + n0)), DFT4 over (n1, n0) -> k4;   bin k = k1 + 16 k2 + 256 k3 + 4096 k4.
// 512 threads hold 32 points each: two batches (n0 = 0, 1) of 16.  n0 stays a register index in
// every stage, so each exchange moves one batch at a time through a 64 KiB image (66 KiB for the
// padded X2 layout): W(b0) | R(b0) | W(b1) + the next stage on b0 | R(b1) + the next stage on b1.
// Thread layouts (t = 64 wave + lane) and images, chosen so every access is one ds_*_b64 with a
// compile-time offset and no bank conflict (16-lane store groups, 32-lane read groups):
//   S1 thread t = n1 + 2 m3 + 32 m2 (n mod 1024 = 2 t + n0: one 16-B load per m1 takes both batches)
//   X1 image [k1][m2][m3 n1] = t + 512 k1;   S2 thread (m3 n1) + 32 k1
//   X2 image (m3 n1) + 33 k1 + 528 k2;       S3 lane k1 + 16 (k2 & 1) + 32 n1, wave k2 >> 1
//   X3 image k1 + 16 (k2 & 1) + 32 n1 + 64 k3 + 1024 (k2 >> 1);
//   S4 lane k1 + 16 (k2 & 3) (the partial row's 64 contiguous bins), wave (k2 >> 2) + 4 (k3 >> 3),
//      so S4's twiddles are wave-uniform constants.
struct WfB2 {
    static constexpr int LOGN = 14, N = 1 << LOGN, NT = 512;
    static constexpr int kImage = 528 * 16;  // X2's padded image, the largest of the three
    static constexpr int kTw2 = 64 * 16;     // tw2[16 j + k] = W_1024^(j k)
    // S2's twiddles stay in LDS behind the image for the whole group, [k][n0][t & 31]: one
    // conflict-free ds_read_b64 each
    static constexpr size_t kLds = sizeof(float2) * (kImage + kTw2);
};

// workgroup barrier with only the LDS counter drained (global loads stay in flight across it);
// the memory clobber keeps every LDS access on its side
OWRX_DEV void wf_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// a[k] *= W_16384^(k nr), k = 1..15, from the powers w1 = W^nr, w2 = W^(2 nr), w4, w8
OWRX_DEV void b2_tw1(float2* a, float2 w1, float2 w2, float2 w4, float2 w8) {
    // each power is used as soon as it exists (a[k] and a[k + 8]), so few stay live
    a[8] = f2mul(a[8], w8);
    a[1] = f2mul(a[1], w1);
    a[9] = f2mul(a[9], f2mul(w1, w8));
    a[2] = f2mul(a[2], w2);
    a[10] = f2mul(a[10], f2mul(w2, w8));
    const float2 w3 = f2mul(w1, w2);
    a[3] = f2mul(a[3], w3);
    a[11] = f2mul(a[11], f2mul(w3, w8));
    a[4] = f2mul(a[4], w4);
    a[12] = f2mul(a[12], f2mul(w4, w8));
    const float2 w5 = f2mul(w1, w4);
    a[5] = f2mul(a[5], w5);
    a[13] = f2mul(a[13], f2mul(w5, w8));
    const float2 w6 = f2mul(w2, w4);
    a[6] = f2mul(a[6], w6);
    a[14] = f2mul(a[14], f2mul(w6, w8));
    const float2 w7 = f2mul(w3, w4);
    a[7] = f2mul(a[7], w7);
    a[15] = f2mul(a[15], f2mul(w7, w8));
}

#ifndef OWRX_B2_ABL
#define OWRX_B2_ABL 0
#endif
// PF = 0: two workgroups per CU (128 VGPRs), each frame's samples loaded when it starts.
// PF = 1: one workgroup per CU (256 VGPRs): the window stays in registers and the next frame's
//         samples load while this one transforms.
// ABL (tools/micro only): 1 = no frame loads, 2 = no barriers.
template <int PF, int ABL = OWRX_B2_ABL>
__global__ void __launch_bounds__(WfB2::NT) __attribute__((amdgpu_waves_per_eu(PF ? 2 : 4, PF ? 2 : 4)))
wf_fft_b2(const float2* __restrict__ blk, int64_t blk_start, const WfGroup* __restrict__ groups,
          const float* __restrict__ window, const float2* __restrict__ tw,
          const float2* __restrict__ tw2, float* __restrict__ partial) {
    using K = WfB2;
    constexpr int N = K::N;
    WF_RSTAMP(14);
    WF_STAMP(0);
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    {
        // S2's table into LDS: entry (2 k + n0) 32 + j of W_1024^((2 j + n0) k)
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int e = t + 512 * i, j = e & 31, kb = e >> 5;
            sm[K::kImage + e] = tw2[16 * (2 * j + (kb & 1)) + (kb >> 1)];
        }
    }
    // S1's exact powers W_N^(2 t 2^i), i < 4, for the whole group (batch 1 multiplies them by
    // the constants W_N^(2^i))
    float2 sb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sb[i] = tw[((int)threadIdx.x << (i + 1)) & (N - 1)];
    const WfGroup g = groups[blockIdx.x];
    const int64_t g0 = g.start - blk_start;
    const int hop = __builtin_amdgcn_readfirstlane(g.hop);
    const int nfr = __builtin_amdgcn_readfirstlane(g.nframes);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(blk + g0), 0, (int)(sizeof(float2) * ((int64_t)(nfr - 1) * hop + N)),
        0x00020000);
    const float2* __restrict__ win2 = reinterpret_cast<const float2*>(window);
    auto load_x = [&](int f, float4* v) {
        const int vo = ((int)threadIdx.x * 2 + f * hop) * 8;
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            if (ABL == 1)
                v[m] = make_float4(vo * 1e-9f + m, m - vo * 1e-9f, 0.5f * m, vo * 2e-9f);
            else
                v[m] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo, m * 1024 * 8, 0));
        }
    };
    float4 nx[PF ? 16 : 1];
    float2 wres[PF ? 16 : 1];
    if constexpr (PF) {
        load_x(0, nx);
#pragma unroll
        for (int m = 0; m < 16; ++m) wres[m] = win2[threadIdx.x + 512 * m];
    }
    float acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.0f;
    // S4's twiddles W_64^(k3 e), e = 1, 2, 3, k3 = kl + 8 (wave >> 2): wave-uniform, in SGPRs for
    // the whole group
    float2 t4[8][3];
    {
        const int k3h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
#pragma unroll
        for (int kl = 0; kl < 8; ++kl)
#pragma unroll
            for (int e = 1; e < 4; ++e) t4[kl][e - 1] = tw[(256 * e * (kl + 8 * k3h)) & (N - 1)];
    }
#pragma unroll 1
    for (int f = 0; f < nfr; ++f) {
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        // opaque per frame: otherwise the 30 twiddle products derived from them are hoisted out
        // of the loop and held in registers (spills)
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(sb[i].x), "+v"(sb[i].y));
        const int lane = t & 63, wv = t >> 6;
        // ---- S1: both batches' samples, 16 B per m1
        float2 a0[16], a1[16];
        if constexpr (PF) {
            float4 xs[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) xs[m] = nx[m];
            if (f + 1 < nfr) load_x(f + 1, nx);
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                a0[m] = make_float2(xs[m].x * wres[m].x, xs[m].y * wres[m].x);
                a1[m] = make_float2(xs[m].z * wres[m].y, xs[m].w * wres[m].y);
            }
        } else {
            float4 xs[16];
            load_x(f, xs);
            int wt = t;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float2 wp[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) wp[m] = win2[wt + 512 * (8 * h + m)];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const float4 x = xs[8 * h + m];
                    a0[8 * h + m] = make_float2(x.x * wp[m].x, x.y * wp[m].x);
                    a1[8 * h + m] = make_float2(x.z * wp[m].y, x.w * wp[m].y);
                }
                // the second half's taps load once the first half is applied (16 VGPRs, not 32)
                asm volatile("" : "+v"(wt) : "v"(a1[8 * h + 7].x));
            }
        }
        if (f == 1) WF_STAMP(1);
        f2dft<16>(a0);
        b2_tw1(a0, sb[0], sb[1], sb[2], sb[3]);
        if (ABL != 2) wf_bar();  // the previous frame's last reads
#pragma unroll
        for (int k = 0; k < 16; ++k) sm[t + 512 * k] = a0[k];
        f2dft<16>(a1);
        {
            // W_N^(2^i) = exp(-2 pi i 2^i / 16384), i < 4
            const float2 c1 = make_float2(0.99999992646571789f, -0.00038349518757139556f);
            const float2 c2 = make_float2(0.99999970586288223f, -0.00076699031874270449f);
            const float2 c4 = make_float2(0.99999882345170188f, -0.0015339801862847655f);
            const float2 c8 = make_float2(0.99999529380957619f, -0.0030679567629659761f);
            b2_tw1(a1, f2mul(sb[0], c1), f2mul(sb[1], c2), f2mul(sb[2], c4), f2mul(sb[3], c8));
        }
        if (ABL != 2) wf_bar();
        if (f == 1) WF_STAMP(2);
        // ---- S2 (thread (m3 n1) + 32 k1, j = n mod 64 = 2 (t & 31) + n0)
        const int r1 = (t & 31) + 512 * (t >> 5);
        const float2* T2 = sm + K::kImage + (t & 31);  // [k][n0][t & 31]
        float2 c0[16], c1[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) c0[m] = sm[r1 + 32 * m];
        if (ABL != 2) wf_bar();
#pragma unroll
        for (int k = 0; k < 16; ++k) sm[t + 512 * k] = a1[k];
        f2dft<16>(c0);
#pragma unroll
        for (int k = 1; k < 16; ++k) c0[k] = f2mul(c0[k], T2[64 * k]);
        if (ABL != 2) wf_bar();
#pragma unroll
        for (int m = 0; m < 16; ++m) c1[m] = sm[r1 + 32 * m];
        if (ABL != 2) wf_bar();
        const int w2 = (t & 31) + 33 * (t >> 5);
#pragma unroll
        for (int k = 0; k < 16; ++k) sm[w2 + 528 * k] = c0[k];
        f2dft<16>(c1);
#pragma unroll
        for (int k = 1; k < 16; ++k) c1[k] = f2mul(c1[k], T2[64 * k + 32]);
        if (ABL != 2) wf_bar();
        if (f == 1) WF_STAMP(3);
        // ---- S3 (lane k1 + 16 (k2 & 1) + 32 n1, wave k2 >> 1)
        const int r2 = (lane >> 5) + 33 * (lane & 15) + 528 * (((lane >> 4) & 1) + 2 * wv);
        float2 d0[16], d1[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) d0[m] = sm[r2 + 2 * m];
        if (ABL != 2) wf_bar();
#pragma unroll
        for (int k = 0; k < 16; ++k) sm[w2 + 528 * k] = c1[k];
        f2dft<16>(d0);
        if (ABL != 2) wf_bar();
#pragma unroll
        for (int m = 0; m < 16; ++m) d1[m] = sm[r2 + 2 * m];
        if (ABL != 2) wf_bar();
        const int w3 = lane + 1024 * wv;
#pragma unroll
        for (int k = 0; k < 16; ++k) sm[w3 + 64 * k] = d0[k];
        f2dft<16>(d1);
        if (ABL != 2) wf_bar();
        if (f == 1) WF_STAMP(4);
        // ---- S4 (lane k1 + 16 (k2 & 3), wave (k2 >> 2) + 4 (k3 >> 3)): with e = 2 n1 + n0 and
        // k4 = ka + 2 kb, X = sum_n0 W_2^(n0 kb) W_4^(n0 ka) y(ka, n0), y(ka, n0) = sum_n1 W_2^(n1 ka)
        // u(n1, n0), u = W_64^(k3 e) v: batch 0's half of the DFT4 runs before batch 1 arrives.
        // The twiddles are wave-uniform (k3 = kl + 8 (wave >> 2)): scalar loads of the table.
        const int r3 = (lane & 31) + 1024 * (lane >> 5) + 2048 * (wv & 3) + 512 * (wv >> 2);
        float2 y0[8][2];
#pragma unroll
        for (int kl = 0; kl < 8; ++kl) {
            const float2 u0 = sm[r3 + 64 * kl];
            const float2 u1 = f2mul(sm[r3 + 32 + 64 * kl], t4[kl][1]);
            y0[kl][0] = f2add(u0, u1);
            y0[kl][1] = f2sub(u0, u1);
        }
        if (ABL != 2) wf_bar();
#pragma unroll
        for (int k = 0; k < 16; ++k) sm[w3 + 64 * k] = d1[k];
        if (ABL != 2) wf_bar();
#pragma unroll
        for (int kl = 0; kl < 8; ++kl) {
            const float2 u0 = f2mul(sm[r3 + 64 * kl], t4[kl][0]);
            const float2 u1 = f2mul(sm[r3 + 32 + 64 * kl], t4[kl][2]);
            const float2 ya = f2add(u0, u1), yb = f2mi(f2sub(u0, u1));  // ka = 1: * W_4 = -i
            const float2 x0 = f2add(y0[kl][0], ya), x2 = f2sub(y0[kl][0], ya);
            const float2 x1 = f2add(y0[kl][1], yb), x3 = f2sub(y0[kl][1], yb);
            acc[kl][0] = fmaf(x0.y, x0.y, fmaf(x0.x, x0.x, acc[kl][0]));
            acc[kl][1] = fmaf(x1.y, x1.y, fmaf(x1.x, x1.x, acc[kl][1]));
            acc[kl][2] = fmaf(x2.y, x2.y, fmaf(x2.x, x2.x, acc[kl][2]));
            acc[kl][3] = fmaf(x3.y, x3.y, fmaf(x3.x, x3.x, acc[kl][3]));
        }
        if (f == 1) WF_STAMP(5);
    }
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    float* out = partial + (int64_t)blockIdx.x * N + lane + 64 * (wv & 3) + 2048 * (wv >> 2);
#pragma unroll
    for (int kl = 0; kl < 8; ++kl)
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) out[256 * kl + 4096 * k4] = acc[kl][k4];
    WF_STAMP(13);
    WF_RSTAMP(15);
#ifdef OWRX_WF_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 1024)
        g_wf_stamp[blockIdx.x][12] = ((unsigned long long)__builtin_amdgcn_s_getreg(63508) << 32) |
                                     (unsigned)__builtin_amdgcn_s_getreg(63492);
#endif
}

}  // namespace owrx
