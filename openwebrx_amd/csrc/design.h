// design.h -- host-side parameter design for the csdr modules on the hot path (filter taps,
// windows, twiddles, AGC profiles).  Taps are parameters shared by every chain of a group;
// they are computed once on the host in double and rounded to float, like the browser port
// of csdr's firdes (htdocs/lib/AudioEngine.js:540-565) that pins them.
#pragma once
#include <stdint.h>
#include <vector>
#include "owrx_dev.h"

namespace owrx {

int firdes_filter_len(float transition_bw);                       // csdr firdes_filter_len
std::vector<float> firdes_lowpass(int length, double cutoff);     // csdr firdes_lowpass_f
std::vector<float> firdes_bandpass_c(int length, float lo, float hi);  // interleaved re,im
std::vector<float> hamming_window(int n);                          // Fft window
std::vector<float> fft_twiddles(int n);                            // exp(-2 pi i t / n)
AgcParams agc_profile(int profile);
float nfm_deemphasis_alpha(int sample_rate);
uint64_t rate_to_fx(float rate);        // Shift rate -> 2^-64 turns per sample
float2 rate_rotator(float rate, int64_t nsamples);  // exp(j 2 pi nsamples rate)

}  // namespace owrx
