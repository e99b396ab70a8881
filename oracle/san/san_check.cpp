// oracle/san/san_check.cpp -- TEST INFRASTRUCTURE ONLY (host sanitizer driver).
//
// Built by oracle/san/Makefile with AddressSanitizer + UndefinedBehaviorSanitizer on the
// HOST code only: the oracle restatement (oracle/csdr_oracle.c) and the engine's host-side
// parameter design (openwebrx_amd/csrc/design.cpp).  It drives every oracle entry point
// over ragged, empty and maximum-size inputs (the cases tests/test_oracle*.py cover) and
// cross-checks design.cpp's taps against the oracle's, so an out-of-bounds index, a
// signed overflow or a bad shift in either aborts the run (-fno-sanitize-recover=all).
// tests/test_sanitizers.py builds and runs it on the CPU.  SURVEY.md section 5.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <vector>
#include "csdr_oracle.h"
#include "design.h"

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static float frand() {
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (float)((double)(rng >> 11) / 9007199254740992.0 * 2.0 - 1.0);
}
static std::vector<float> noise(int64_t n, float amp) {
    std::vector<float> v((size_t)n);
    for (auto& x : v) x = amp * frand();
    return v;
}
static int fails = 0;
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); fails++; } } while (0)

static void check_design() {
    for (float tw : {0.001f, 0.01f, 0.05f, 0.15f, 0.4f}) {
        int a = owrx::firdes_filter_len(tw), b = orc_firdes_filter_len(tw);
        CHECK(a == b);
        std::vector<float> ref((size_t)b);
        orc_firdes_lowpass_f(ref.data(), b, 0.5f * tw + 0.01f);
        std::vector<float> d = owrx::firdes_lowpass(a, 0.5f * tw + 0.01f);
        CHECK((int)d.size() == a);
        double md = 0;
        for (int i = 0; i < a; i++) md = fmax(md, fabs((double)d[i] - ref[i]));
        CHECK(md < 1e-6);
        std::vector<float> bp = owrx::firdes_bandpass_c(a, -0.1f, 0.05f);
        std::vector<float> bref(2 * (size_t)a);
        orc_firdes_bandpass_c(bref.data(), a, -0.1f, 0.05f);
        CHECK((int)bp.size() == 2 * a);
        md = 0;
        for (int i = 0; i < 2 * a; i++) md = fmax(md, fabs((double)bp[i] - bref[i]));
        CHECK(md < 1e-5);
    }
    for (int n : {1, 2, 255, 256, 16384, 1 << 20}) {
        std::vector<float> w = owrx::hamming_window(n), r((size_t)n);
        orc_hamming_window(r.data(), n);
        CHECK((int)w.size() == n);
        double md = 0;
        for (int i = 0; i < n; i++) md = fmax(md, fabs((double)w[i] - r[i]));
        CHECK(md < 1e-6);
    }
    for (int n : {2, 256, 16384, 1 << 20}) CHECK((int)owrx::fft_twiddles(n).size() >= n / 2);
    for (int p = 0; p < 4; p++) {
        owrx::AgcParams a = owrx::agc_profile(p);
        orc_agc_params o;
        orc_agc_profile(p, &o);
        CHECK(a.reference == o.reference && a.attack == o.attack_rate && a.decay == o.decay_rate);
    }
    for (int sr : {8000, 12000, 44100, 48000}) CHECK(owrx::nfm_deemphasis_alpha(sr) == orc_nfm_deemphasis_alpha(sr));
    for (float r : {-0.5f, -0.4999f, -1e-7f, 0.f, 1e-7f, 0.25f, 0.4999f, 0.5f}) {
        (void)owrx::rate_to_fx(r);
        for (int64_t n : {(int64_t)0, (int64_t)1, (int64_t)1 << 20, (int64_t)1 << 40, INT64_MAX / 2}) {
            float2 z = owrx::rate_rotator(r, n);
            CHECK(fabsf(z.x * z.x + z.y * z.y - 1.f) < 1e-4f);
        }
    }
}

static void check_selector() {
    for (int64_t n : {0, 1, 7, 1000, 65537}) {
        std::vector<float> iq = noise(2 * n + 2, 0.5f), y(2 * (size_t)n + 2), z(2 * (size_t)n + 2);
        orc_shift(iq.data(), y.data(), n, 0.123f);
        int nt = orc_firdes_filter_len(0.05f);
        std::vector<float> taps((size_t)nt);
        orc_firdes_lowpass_f(taps.data(), nt, 0.1f);
        for (int dec : {1, 5, 25, 64}) {
            int64_t m = orc_fir_decimate(y.data(), n, taps.data(), nt, dec, z.data());
            CHECK(m >= 0 && m <= n / dec + 1);
        }
        for (double rate : {1.0, 1.3, 2.7182818}) {
            std::vector<float> fr(2 * (size_t)(n / rate + 4));
            int64_t m = orc_fractional_decimator(y.data(), n, rate, fr.data());
            CHECK(m >= 0 && (double)m <= n / rate + 2);
            std::vector<float> fr1((size_t)(n / rate + 4)), rin = noise(n + 1, 1.f);
            m = orc_fractional_decimator_f(rin.data(), n, rate, fr1.data());
            CHECK(m >= 0 && (double)m <= n / rate + 2);
        }
        std::vector<float> bp(2 * (size_t)nt);
        orc_firdes_bandpass_c(bp.data(), nt, -0.2f, 0.1f);
        orc_fir_complex(y.data(), n, bp.data(), nt, z.data());
        for (int len : {1, 128, 1024}) {
            std::vector<float> pw((size_t)(n / len + 1));  // one power per whole block
            int64_t np = 0;
            int64_t m = orc_squelch(y.data(), n, len, 5, 3, 1, 1, 0.01f, z.data(), pw.data(), &np);
            CHECK(m >= 0 && m <= n && np >= 0);
        }
    }
}

static void check_audio() {
    for (int64_t n : {0, 1, 2, 999, 48000}) {
        std::vector<float> iq = noise(2 * n + 2, 0.7f), a((size_t)n + 1), b((size_t)n + 1);
        orc_fmdemod(iq.data(), n, a.data());
        orc_amdemod(iq.data(), n, a.data());
        orc_realpart(iq.data(), n, a.data());
        orc_limit(a.data(), n, 0.5f, b.data());
        orc_dcblock(b.data(), n, a.data());
        orc_deemphasis(a.data(), n, orc_nfm_deemphasis_alpha(12000), b.data());
        for (int p = 0; p < 4; p++) {
            orc_agc_params ap;
            orc_agc_profile(p, &ap);
            orc_agc(b.data(), n, &ap, a.data());
        }
        orc_gain(a.data(), n, 3.f, b.data());
        std::vector<float> taps = noise(31, 0.1f);
        orc_fir_real(b.data(), n, taps.data(), 31, a.data());
        std::vector<float> nf((size_t)n + 1);
        (void)orc_noise_filter(a.data(), n, -20.f, nf.data());
        // full-scale and beyond: convert saturates, ADPCM clamps its predictor
        for (int64_t i = 0; i < n; i++) b[i] = 4.f * frand();
        std::vector<int16_t> s((size_t)n + 1), d(2 * (size_t)n + 16);
        orc_convert_f_s16(b.data(), n, s.data());
        orc_convert_s16_f(s.data(), n, a.data());
        for (int sync : {0, 1}) {
            std::vector<uint8_t> enc((size_t)n / 2 + 16 * ((size_t)n / 2002 + 2));
            int64_t nb = orc_adpcm_encode(s.data(), n, sync, enc.data());
            CHECK(nb >= 0 && (size_t)nb <= enc.size());
            std::vector<int16_t> dec(2 * (size_t)nb + 2);
            int64_t ns = orc_adpcm_decode(enc.data(), nb, dec.data());
            CHECK(ns >= 0 && ns <= 2 * nb);
        }
    }
    CHECK(orc_wfm_deemphasis_alpha(48000, 50e-6f) > 0.f);
}

static void check_waterfall() {
    for (int N : {16, 256, 1024, 16384}) {
        for (int64_t n : {(int64_t)0, (int64_t)N - 1, (int64_t)N, (int64_t)3 * N + 17}) {
            int hop = N / 2 + 3;
            std::vector<float> iq = noise(2 * n + 2, 0.3f);
            int64_t rows_cap = n >= N ? (n - N) / hop + 1 : 0;
            std::vector<float> rows((size_t)(rows_cap + 1) * N), sw((size_t)N);
            for (int avg : {1, 3}) {
                int64_t r = orc_waterfall_rows(iq.data(), n, N, hop, avg, -5.f, rows.data());
                CHECK(r >= 0 && r <= rows_cap);
                if (r > 0) {
                    orc_fftswap(rows.data(), N, sw.data());
                    std::vector<uint8_t> out((size_t)N / 2 + 16);
                    int64_t b = orc_fft_adpcm_row(sw.data(), N, out.data());
                    CHECK(b > 0 && (size_t)b <= out.size());
                }
            }
        }
        std::vector<double> x(2 * (size_t)N), X(2 * (size_t)N);
        for (auto& v : x) v = frand();
        orc_fft(x.data(), N, X.data());
    }
}

static void check_chain() {
    int64_t n = 1 << 16;
    std::vector<float> iq = noise(2 * n, 0.5f);
    int nt = orc_firdes_filter_len(0.02f);
    std::vector<float> taps((size_t)nt), bp(2 * (size_t)nt);
    orc_firdes_lowpass_f(taps.data(), nt, 0.02f);
    orc_firdes_bandpass_c(bp.data(), nt, -0.05f, 0.05f);
    for (int mode = 0; mode < 3; mode++)
        for (int comp = 0; comp < 2; comp++)
            for (int withbp = 0; withbp < 2; withbp++) {
                orc_chain_params p;
                memset(&p, 0, sizeof p);
                p.shift_rate = 0.0731f; p.decimation = 25; p.ntaps = nt; p.taps = taps.data();
                p.frac_rate = mode == 1 ? 1.25 : 1.0;
                p.bp_ntaps = withbp ? nt : 0; p.bp_taps = bp.data();
                p.sq_length = 1024; p.sq_decimation = 5; p.sq_hang = 3; p.sq_flush = 1;
                p.sq_report = 1; p.sq_level = 0.f; p.mode = mode;
                orc_agc_profile(mode == 2 ? 1 : 0, &p.agc);
                p.deemph_alpha = mode == 0 ? orc_nfm_deemphasis_alpha(12000) : 0.f;
                p.compression = comp;
                std::vector<uint8_t> out((size_t)n);
                std::vector<float> sm(1024);
                int64_t nsm = 0;
                int64_t b = orc_run_chain(iq.data(), n, &p, out.data(), (int64_t)out.size(), sm.data(), &nsm);
                CHECK(b > 0 && b <= (int64_t)out.size());
                CHECK(orc_run_chain(iq.data(), n, &p, out.data(), 1, sm.data(), &nsm) == -1);
            }
}

int main() {
    check_design();
    check_selector();
    check_audio();
    check_waterfall();
    check_chain();
    if (fails) { fprintf(stderr, "%d checks failed\n", fails); return 1; }
    printf("san_check ok\n");
    return 0;
}
