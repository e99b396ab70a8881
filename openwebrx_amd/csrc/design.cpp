// design.cpp -- see design.h.
#include "design.h"

#include <cmath>

namespace owrx {

int firdes_filter_len(float transition_bw) {
    // int(4.0/tbw) forced odd; tbw arrives as float (pycsdr float argument)
    int r = (int)(4.0 / (double)transition_bw);
    if (r % 2 == 0) r++;
    return r;
}

static double hamming(double r) { return 0.54 - 0.46 * std::cos(2.0 * M_PI * (0.5 + r / 2.0)); }

static std::vector<double> lowpass_d(int length, double cutoff) {
    std::vector<double> h(length);
    const int mid = length / 2;
    h[mid] = 2.0 * M_PI * cutoff * hamming(0.0);
    for (int i = 1; i <= mid; ++i) {
        const double v = (std::sin(2.0 * M_PI * cutoff * i) / i) * hamming((double)i / mid);
        h[mid - i] = v;
        h[mid + i] = v;
    }
    double sum = 0.0;
    for (double v : h) sum += v;
    for (double& v : h) v /= sum;
    return h;
}

std::vector<float> firdes_lowpass(int length, double cutoff) {
    std::vector<double> h = lowpass_d(length, cutoff);
    return std::vector<float>(h.begin(), h.end());
}

std::vector<float> firdes_bandpass_c(int length, float lo, float hi) {
    std::vector<double> h = lowpass_d(length, ((double)hi - (double)lo) / 2.0);
    const double fc = ((double)hi + (double)lo) / 2.0;
    std::vector<float> out(2 * (size_t)length);
    for (int i = 0; i < length; ++i) {
        const double ph = 2.0 * M_PI * std::fmod(fc * (double)i, 1.0);
        out[2 * i] = (float)(std::cos(ph) * h[i]);
        out[2 * i + 1] = (float)(std::sin(ph) * h[i]);
    }
    return out;
}

std::vector<float> hamming_window(int n) {
    std::vector<float> w(n);
    for (int i = 0; i < n; ++i) {
        const double r = n > 1 ? 2.0 * (double)i / (double)(n - 1) - 1.0 : 0.0;
        w[i] = (float)hamming(r);
    }
    return w;
}

std::vector<float> fft_twiddles(int n) {
    std::vector<float> t(2 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        const double a = -2.0 * M_PI * (double)i / (double)n;
        t[2 * i] = (float)std::cos(a);
        t[2 * i + 1] = (float)std::sin(a);
    }
    return t;
}

// Every profile has attack > decay > 0: post_serial_front's envelope step takes
// max(attack d, decay d) for (d > 0 ? attack : decay) d on that basis.
AgcParams agc_profile(int profile) {
    AgcParams p;
    p.reference = 0.8f;
    p.max_gain = 65535.0f;
    p.initial_gain = 1.0f;
    p.hang_time = 0;
    switch (profile) {
        case 0: p.attack = 0.1f; p.decay = 0.001f; break;    // FAST
        case 1: p.attack = 0.05f; p.decay = 0.0001f; break;  // SLOW
        case 2: p.attack = 0.1f; p.decay = 0.0005f; break;   // MID
        default: p.attack = 0.01f; p.decay = 0.0001f; break; // LAGGY
    }
    return p;
}

float nfm_deemphasis_alpha(int sample_rate) {
    const double dt = 1.0 / (double)sample_rate;
    const double tau = 1.0 / (2.0 * M_PI * 300.0);
    return (float)(dt / (tau + dt));
}

uint64_t rate_to_fx(float rate) {
    double r = (double)rate;
    r -= std::floor(r);
    const double s = r * 18446744073709551616.0;
    if (s >= 18446744073709551615.0) return 0;
    return (uint64_t)s;
}

float2 rate_rotator(float rate, int64_t nsamples) {
    const uint64_t ph = (uint64_t)nsamples * rate_to_fx(rate);
    const double a = 2.0 * M_PI * ((double)ph * (1.0 / 18446744073709551616.0));
    return make_float2((float)std::cos(a), (float)std::sin(a));
}

}  // namespace owrx
