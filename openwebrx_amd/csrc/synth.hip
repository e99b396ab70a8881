// synth.hip -- synthetic wideband test source (benchmarks and tests; the reference's
// equivalent role is an SDR or csdr's test sources).  The signal model of SURVEY.md 8d and
// openwebrx_amd/synth.py: complex AWGN (sigma `noise` per component) plus one carrier per
// chain at offsets_hz[c]: NFM 1 kHz tone at 2.5 kHz deviation, AM 30 % at 1 kHz, USB / CW / LSB
// tones at +1000 / +800 / -1000 Hz, amplitude `amp`.  Carrier phases are exact 64-bit
// fixed-point turns; the noise is a counter-based hash (Box-Muller), so any range of the stream
// can be generated independently.  Not bit-identical to synth.py (numpy PCG64); same model.
#include <math.h>
#include <stdint.h>

#include "../../include/owrx_amd.h"
#include "owrx_dev.h"

namespace owrx {

OWRX_DEV uint64_t synth_mix(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}

__global__ void __launch_bounds__(256)
synth_iq(float2* __restrict__ out, int64_t n, int64_t start, double fs, int nc,
         const uint64_t* __restrict__ rate_fx, const int* __restrict__ modes, uint64_t seed,
         float noise, float amp) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t s = start + i;
    const uint64_t h = synth_mix(seed ^ synth_mix((uint64_t)s));
    const float u1 = ((float)(h >> 40) + 0.5f) * 5.9604645e-08f;           // (0, 1)
    const float u2 = (float)((h >> 16) & 0xffffff) * 5.9604645e-08f;        // [0, 1)
    const float r = noise * sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincospif(2.0f * u2, &sn, &cs);
    float re = r * cs, im = r * sn;
    // the 1 kHz modulating tone, shared by every carrier
    const double tm = (double)s * 1000.0 / fs;
    const float m = (float)sinpi(2.0 * (tm - floor(tm)));
    for (int c = 0; c < nc; ++c) {
        const uint64_t ph = (uint64_t)s * rate_fx[c];
        float t = (float)(int32_t)(uint32_t)(ph >> 32) * 2.3283064365386963e-10f;  // turns
        float a = amp;
        if (modes[c] == 0) t += 2.5f * m * 0.15915494f;   // NFM: +2.5 rad * sin
        else if (modes[c] == 1) a *= 1.0f + 0.3f * m;     // AM
        float ss, cc;
        sincospif(2.0f * t, &ss, &cc);
        re += a * cc;
        im += a * ss;
    }
    out[i] = make_float2(re, im);
}

// Stall injection for the bounded-wait test (owrx_debug_stall): one wave that sleeps for `us`
// microseconds of the 100 MHz real-time counter and exits -- a stream that stops completing
// work for a known time, ended by the kernel itself.
__global__ void __launch_bounds__(64) debug_sleep(int64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(127);
}

hipError_t launch_debug_sleep(int64_t us, hipStream_t st) {
    hipLaunchKernelGGL(debug_sleep, dim3(1), dim3(64), 0, st, us * 100);
    return hipGetLastError();
}

}  // namespace owrx

using namespace owrx;

extern "C" int owrx_synth_iq(int device, float* dst_dev, int64_t n, int64_t start,
                             double samp_rate, int ncarriers, const double* offsets_hz,
                             const int* modes, uint64_t seed, float noise, float amp) {
    if (n < 0 || ncarriers < 0 || !dst_dev || (ncarriers > 0 && (!offsets_hz || !modes)))
        return OWRX_EINVAL;
    if (hipSetDevice(device) != hipSuccess) return OWRX_ENODEV;
    // tone offsets folded into the carrier frequency: usb +1000, cw +800, lsb -1000 Hz
    uint64_t* h_rate = new uint64_t[ncarriers > 0 ? ncarriers : 1];
    int* h_mode = new int[ncarriers > 0 ? ncarriers : 1];
    for (int c = 0; c < ncarriers; ++c) {
        const double tone = modes[c] == 2 ? 1000.0 : modes[c] == 3 ? 800.0 : modes[c] == 4 ? -1000.0 : 0.0;
        const double turns = (offsets_hz[c] + tone) / samp_rate;
        h_rate[c] = (uint64_t)(int64_t)llround(ldexp(turns - floor(turns + 0.5), 63)) << 1;
        h_mode[c] = modes[c];
    }
    uint64_t* d_rate = nullptr;
    int* d_mode = nullptr;
    int rc = OWRX_OK;
    if (hipMalloc(&d_rate, sizeof(uint64_t) * (ncarriers + 1)) != hipSuccess ||
        hipMalloc(&d_mode, sizeof(int) * (ncarriers + 1)) != hipSuccess ||
        hipMemcpy(d_rate, h_rate, sizeof(uint64_t) * ncarriers, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_mode, h_mode, sizeof(int) * ncarriers, hipMemcpyHostToDevice) != hipSuccess) {
        rc = OWRX_EIO;
    } else {
        const int64_t chunk = 1 << 24;
        for (int64_t o = 0; o < n && rc == OWRX_OK; o += chunk) {
            const int64_t m = n - o < chunk ? n - o : chunk;
            hipLaunchKernelGGL(synth_iq, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, 0,
                               (float2*)dst_dev + o, m, start + o, samp_rate, ncarriers, d_rate,
                               d_mode, seed, noise, amp);
            if (hipGetLastError() != hipSuccess) rc = OWRX_EIO;
        }
        if (rc == OWRX_OK && hipDeviceSynchronize() != hipSuccess) rc = OWRX_EIO;
    }
    hipFree(d_rate);
    hipFree(d_mode);
    delete[] h_rate;
    delete[] h_mode;
    return rc;
}
