// modules.hip -- single csdr modules run on the GPU with persistent state, for pycsdr module
// objects that are not part of a fused chain and for per-module parity tests.  Each call copies
// the host input to HBM, runs the module's kernel (the same __device__ step functions the fused
// post kernel uses) and copies the output back.
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/owrx_amd.h"
#include "design.h"
#include "owrx_types.h"

namespace owrx {
void set_last_error(const char* fmt, ...);

struct ModState {
    float2 fm_last;
    float yp, xp, yp2;
    AgcState agc;
    AfcState afc;  // Afc (owrx_dev.h afc_step)
    AdpcmState adpcm;
    int64_t adpcm_bytes;
    int32_t has_left;
    int32_t left;
};

struct ModParams {
    int type;
    float f0;
    int i0, i1;
    AgcParams agc;
    float alpha, beta;
    int fft_size;
};

// serial modules: one lane walks the stream with the module state
__global__ void mod_serial(ModParams p, const void* __restrict__ in, int64_t n,
                           uint8_t* __restrict__ out, int64_t cap, ModState* __restrict__ st,
                           int64_t* __restrict__ produced) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    ModState s = *st;
    int64_t o = 0;
    const float2* ic = (const float2*)in;
    const float* iff = (const float*)in;
    const int16_t* is = (const int16_t*)in;
    float* of = (float*)out;
    int16_t* os = (int16_t*)out;
    switch (p.type) {
        case OWRX_MOD_FMDEMOD:
            for (int64_t k = 0; k < n; ++k) {
                of[k] = fm_step(ic[k], s.fm_last);
                s.fm_last = ic[k];
            }
            o = n;
            break;
        case OWRX_MOD_DCBLOCK:
            for (int64_t k = 0; k < n; ++k) of[k] = dcblock_step(iff[k], s.xp, s.yp2);
            o = n;
            break;
        case OWRX_MOD_DEEMPH:
            for (int64_t k = 0; k < n; ++k) of[k] = deemph_step(iff[k], p.alpha, p.beta, s.yp);
            o = n;
            break;
        case OWRX_MOD_AGC:
            for (int64_t k = 0; k < n; ++k) of[k] = agc_step(iff[k], p.agc, s.agc);
            o = n;
            break;
        case OWRX_MOD_AFC: {  // Afc(updatePeriod U, samplePeriod S): owrx_dev.h afc_step
            float2* oc = (float2*)out;
            for (int64_t k = 0; k < n; ++k) oc[k] = afc_step(s.afc, ic[k], p.i0, p.i1);
            o = n;
            break;
        }
        case OWRX_MOD_ADPCM:
            for (int64_t k = 0; k < n; ++k) {
                if (!s.has_left) {
                    s.left = is[k];
                    s.has_left = 1;
                    continue;
                }
                if (p.i0 && (s.adpcm_bytes % kAdpcmSyncPeriod) == 0) {
                    const int16_t ix = (int16_t)s.adpcm.index, pr = (int16_t)s.adpcm.pred;
                    const uint8_t hdr[8] = {'S', 'Y', 'N', 'C', (uint8_t)(ix & 0xff),
                                            (uint8_t)((ix >> 8) & 0xff), (uint8_t)(pr & 0xff),
                                            (uint8_t)((pr >> 8) & 0xff)};
                    for (int b = 0; b < 8; ++b)
                        if (o + b < cap) out[o + b] = hdr[b];
                    o += 8;
                }
                const int lo = adpcm_encode(s.adpcm, s.left);
                const int hi = adpcm_encode(s.adpcm, is[k]);
                if (o < cap) out[o] = (uint8_t)(lo | (hi << 4));
                o++;
                s.adpcm_bytes++;
                s.has_left = 0;
            }
            break;
        case OWRX_MOD_FFTADPCM: {
            const int N = p.fft_size;
            const int64_t rows = n / N;
            for (int64_t r = 0; r < rows; ++r) {
                AdpcmState a{0, 0};
                const float* row = iff + r * N;
                const int first = db_to_s16(row[0]);
                for (int t = 0; t < N + 10; t += 2) {
                    const int v0 = t < 10 ? first : db_to_s16(row[t - 10]);
                    const int v1 = t + 1 < 10 ? first : db_to_s16(row[t + 1 - 10]);
                    const int lo = adpcm_encode(a, v0);
                    const int hi = adpcm_encode(a, v1);
                    if (o < cap) out[o] = (uint8_t)(lo | (hi << 4));
                    o++;
                }
            }
            break;
        }
        default:
            break;
    }
    (void)os;
    *st = s;
    *produced = o;
}

// FmDemod, parallel: each output needs its sample and the previous one (the carried last sample
// of the previous call for k = 0)
__global__ void mod_fmdemod(const float2* __restrict__ in, int64_t n, float2 last,
                            float* __restrict__ out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x)
        out[k] = fm_step(in[k], k ? in[k - 1] : last);
}

// Shift(rate) standalone (csdr/chain/selector.py:95; the SecondarySelector at the Selector rate,
// selector.py:212-224): x[n] exp(j 2 pi phase(n)), phase(n) = P0 + (n - n0 + 1) rate in exact
// 64-bit fixed-point turns, continuous across calls and rate changes
__global__ void mod_shift(const float2* __restrict__ in, int64_t n, int64_t base, uint64_t P0,
                          int64_t n0, uint64_t rate_fx, float2* __restrict__ out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t ph = P0 + (uint64_t)(base + k - n0 + 1) * rate_fx;
        const float t = (float)(int32_t)(uint32_t)(ph >> 32) * 2.3283064365386963e-10f;
        float sn, cs;
        sincospif(2.0f * t, &sn, &cs);
        out[k] = cmul(in[k], make_float2(cs, sn));
    }
}

// Bandpass standalone (complex FIR of the Hamming bandpass design, selector.py:149-166):
// y[k] = sum_t g[t] x[k - t] over [history (ntaps - 1) | input]
__global__ void mod_cfir(const float2* __restrict__ x, int64_t n, const float2* __restrict__ g,
                         int ntaps, float2* __restrict__ out) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        const float2* xk = x + (ntaps - 1) + k;
        float ar = 0.0f, ai = 0.0f;
        for (int t = 0; t < ntaps; ++t) {
            const float2 a = g[t], v = xk[-t];
            ar = fmaf(a.x, v.x, ar);
            ar = fmaf(-a.y, v.y, ar);
            ai = fmaf(a.x, v.y, ai);
            ai = fmaf(a.y, v.x, ai);
        }
        out[k] = make_float2(ar, ai);
    }
}

// AudioResampler(in, out) (csdr/chain/clientaudio.py:15-16): rational L/M resampler,
// y[m] = L sum_j h[j] x_up[m M - j] with x_up = x upsampled by L (zeros between), polyphase:
// only the taps j = (m M mod L) + L q meet samples.  x = [history | block] on the device,
// sample index of x[0] = x0; output m of this call is absolute output m0 + m.
__global__ void mod_resample(const float* __restrict__ x, int64_t x0, int64_t m0, int64_t n_out,
                             const float* __restrict__ h, int ntaps, int L, int M,
                             float* __restrict__ out) {
    for (int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; m < n_out;
         m += (int64_t)gridDim.x * blockDim.x) {
        const int64_t up = (m0 + m) * (int64_t)M;   // position in the upsampled stream
        const int ph = (int)(up % L);
        const int64_t base = up / L;                 // input index of tap j = ph
        float acc = 0.0f;
        for (int j = ph, q = 0; j < ntaps; j += L, ++q) {
            const int64_t i = base - q - x0;
            if (i >= 0) acc = fmaf(h[j], x[i], acc);
        }
        out[m] = acc * (float)L;
    }
}

// stateless modules: grid-stride
__global__ void mod_parallel(ModParams p, const void* __restrict__ in, int64_t n,
                             uint8_t* __restrict__ out) {
    const float2* ic = (const float2*)in;
    const float* iff = (const float*)in;
    float* of = (float*)out;
    int16_t* os = (int16_t*)out;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x) {
        switch (p.type) {
            case OWRX_MOD_AMDEMOD: of[k] = am_step(ic[k]); break;
            case OWRX_MOD_REALPART: of[k] = ic[k].x; break;
            case OWRX_MOD_LIMIT: of[k] = limit_step(iff[k], p.f0); break;
            case OWRX_MOD_CONVERT_F_S16: os[k] = convert_s16(iff[k]); break;
            case OWRX_MOD_CONVERT_CS16_CF32: of[k] = s16_to_f32(((const int16_t*)in)[k]); break;
            case OWRX_MOD_GAIN: of[k] = gain_step(iff[k], p.f0); break;
            case OWRX_MOD_FFTSWAP: {
                const int N = p.fft_size;
                const int64_t r = k / N, i = k % N;
                of[k] = iff[r * N + ((i + N / 2) % N)];
                break;
            }
            default: break;
        }
    }
}

}  // namespace owrx

using namespace owrx;

struct owrx_module {
    int device;
    ModParams p;
    // FmDemod: the previous call's last sample; Shift: phase model and samples processed;
    // Bandpass: taps and the input history (ntaps - 1 samples)
    float2 fm_last = {0.0f, 0.0f};
    uint64_t P0 = 0, rate_fx = 0;
    int64_t n0 = 0, count = 0;
    float2* d_taps = nullptr;
    int ntaps = 0;
    std::vector<float2> hist;
    // AudioResampler: L / M, real taps, real history, outputs emitted so far
    int rs_L = 1, rs_M = 1;
    float* d_rtaps = nullptr;
    std::vector<float> rhist;
    int64_t rs_out = 0;
    ModState* d_state = nullptr;
    int64_t* d_produced = nullptr;
    void* d_in = nullptr;
    uint8_t* d_out = nullptr;
    int64_t in_cap = 0, out_cap = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
};

static int in_item_bytes(int type) {
    switch (type) {
        case OWRX_MOD_FMDEMOD:
        case OWRX_MOD_AMDEMOD:
        case OWRX_MOD_REALPART:
        case OWRX_MOD_AFC:
        case OWRX_MOD_SHIFT:
        case OWRX_MOD_BANDPASS: return 8;
        case OWRX_MOD_AUDIO_RESAMPLER: return 4;
        case OWRX_MOD_ADPCM: return 2;
        case OWRX_MOD_CONVERT_CS16_CF32: return 4;
        default: return 4;
    }
}

extern "C" int owrx_module_create(int device, int type, double p0, double p1, double p2,
                                  owrx_module** out) {
    if (!out || type < OWRX_MOD_FMDEMOD || type > OWRX_MOD_AFC) {
        set_last_error("owrx_module_create: bad type %d", type);
        return OWRX_EINVAL;
    }
    if (hipSetDevice(device) != hipSuccess) {
        set_last_error("owrx_module_create: hipSetDevice(%d) failed", device);
        return OWRX_ENODEV;
    }
    owrx_module* m = new owrx_module();
    m->device = device;
    memset(&m->p, 0, sizeof(m->p));
    m->p.type = type;
    ModState s;
    memset(&s, 0, sizeof(s));
    switch (type) {
        case OWRX_MOD_LIMIT: m->p.f0 = (float)p0; break;
        case OWRX_MOD_DEEMPH:
            m->p.alpha = (float)p0;
            m->p.beta = 1.0f - (float)p0;
            break;
        case OWRX_MOD_AGC:
            m->p.agc = agc_profile((int)p0);
            if (p1 >= 0) m->p.agc.initial_gain = (float)p1;
            if (p2 >= 0) m->p.agc.max_gain = (float)p2;
            s.agc.env = m->p.agc.reference / m->p.agc.initial_gain;
            break;
        case OWRX_MOD_ADPCM: m->p.i0 = (int)p0; break;
        case OWRX_MOD_AFC:
            if (p0 < 1 || p1 < 1 || p0 != (double)(int)p0 || p1 != (double)(int)p1) {
                delete m;
                set_last_error("Afc: integer updatePeriod, samplePeriod >= 1 required");
                return OWRX_EINVAL;
            }
            m->p.i0 = (int)p0;
            m->p.i1 = (int)p1;
            break;
        case OWRX_MOD_GAIN:
            m->p.f0 = (float)p0;
            m->p.i0 = p1 > 0 ? 1 : 0;  // complex: n samples = 2n floats
            break;
        case OWRX_MOD_SHIFT:
            m->rate_fx = rate_to_fx((float)p0);
            break;
        case OWRX_MOD_BANDPASS:
            if (!(p0 < p1) || p2 <= 0) {
                delete m;
                set_last_error("Bandpass: low < high and transition > 0 required");
                return OWRX_EINVAL;
            }
            break;
        case OWRX_MOD_AUDIO_RESAMPLER: {
            const int64_t a = (int64_t)p0, b = (int64_t)p1;
            if (a <= 0 || b <= 0 || (double)a != p0 || (double)b != p1) {
                delete m;
                set_last_error("AudioResampler: integer rates > 0 required");
                return OWRX_EINVAL;
            }
            int64_t g = a, r = b;
            while (r) {
                const int64_t t = g % r;
                g = r;
                r = t;
            }
            m->rs_L = (int)(b / g);
            m->rs_M = (int)(a / g);
            if (m->rs_L > 64 || m->rs_M > 4096) {
                delete m;
                set_last_error("AudioResampler: ratio %lld/%lld too fine", (long long)b, (long long)a);
                return OWRX_EINVAL;
            }
            // documented choice (csdr's filter is not in the reference): Hamming lowpass at
            // 0.5 / max(L, M) of the upsampled rate, transition a fifth of that, length by the
            // csdr firdes rule (int(4 / tbw), odd)
            const double c = 0.5 / (double)std::max(m->rs_L, m->rs_M);
            const int nt = firdes_filter_len((float)(0.2 * c));
            std::vector<float> h = firdes_lowpass(nt, c);
            m->ntaps = nt;
            if (hipSetDevice(device) != hipSuccess ||
                hipMalloc(&m->d_rtaps, sizeof(float) * nt) != hipSuccess ||
                hipMemcpy(m->d_rtaps, h.data(), sizeof(float) * nt, hipMemcpyHostToDevice) != hipSuccess) {
                owrx_module_destroy(m);
                set_last_error("AudioResampler: HIP allocation failed");
                return OWRX_EIO;
            }
            m->rhist.assign((size_t)(nt / m->rs_L + 2), 0.0f);
            break;
        }
        case OWRX_MOD_FFTSWAP:
        case OWRX_MOD_FFTADPCM:
            m->p.fft_size = (int)p0;
            if (m->p.fft_size <= 0 || (m->p.fft_size & 1)) {
                delete m;
                set_last_error("fft size must be even and positive");
                return OWRX_EINVAL;
            }
            break;
        default: break;
    }
    if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&m->d_state, sizeof(ModState)) != hipSuccess ||
        hipMalloc(&m->d_produced, sizeof(int64_t)) != hipSuccess ||
        hipMemcpy(m->d_state, &s, sizeof(s), hipMemcpyHostToDevice) != hipSuccess) {
        set_last_error("owrx_module_create: HIP allocation failed");
        owrx_module_destroy(m);
        return OWRX_EIO;
    }
    if (type == OWRX_MOD_BANDPASS) {
        const int rc = owrx_module_set(m, p0, p1, p2);
        if (rc) {
            owrx_module_destroy(m);
            return rc;
        }
    }
    *out = m;
    return OWRX_OK;
}

// Shift.setRate (phase continuous from the next sample) / Bandpass.setBandpass (history kept)
extern "C" int owrx_module_set(owrx_module* m, double p0, double p1, double p2) {
    if (!m) return OWRX_EINVAL;
    std::lock_guard<std::mutex> lk(m->mu);
    if (m->p.type == OWRX_MOD_SHIFT) {
        m->P0 = m->P0 + (uint64_t)(m->count - m->n0) * m->rate_fx;
        m->n0 = m->count;
        m->rate_fx = rate_to_fx((float)p0);
        return OWRX_OK;
    }
    if (m->p.type == OWRX_MOD_BANDPASS) {
        if (!(p0 < p1) || p2 <= 0) return OWRX_EINVAL;
        const int nt = firdes_filter_len((float)p2);
        std::vector<float> t = firdes_bandpass_c(nt, (float)p0, (float)p1);
        hipSetDevice(m->device);
        if (nt != m->ntaps) {
            if (m->d_taps) hipFree(m->d_taps);
            m->d_taps = nullptr;
            if (hipMalloc(&m->d_taps, sizeof(float2) * nt) != hipSuccess) return OWRX_ENOMEM;
            std::vector<float2> h((size_t)nt - 1, make_float2(0.0f, 0.0f));
            // keep the newest history samples when the length changes
            const size_t keep = std::min(h.size(), m->hist.size());
            for (size_t i = 0; i < keep; ++i) h[h.size() - 1 - i] = m->hist[m->hist.size() - 1 - i];
            m->hist.swap(h);
            m->ntaps = nt;
        }
        if (hipMemcpy(m->d_taps, t.data(), sizeof(float2) * nt, hipMemcpyHostToDevice) != hipSuccess)
            return OWRX_EIO;
        return OWRX_OK;
    }
    return OWRX_EINVAL;
}

extern "C" int owrx_module_destroy(owrx_module* m) {
    if (!m) return OWRX_EINVAL;
    hipSetDevice(m->device);
    if (m->d_state) hipFree(m->d_state);
    if (m->d_produced) hipFree(m->d_produced);
    if (m->d_in) hipFree(m->d_in);
    if (m->d_out) hipFree(m->d_out);
    if (m->d_taps) hipFree(m->d_taps);
    if (m->d_rtaps) hipFree(m->d_rtaps);
    if (m->stream) hipStreamDestroy(m->stream);
    delete m;
    return OWRX_OK;
}

extern "C" int64_t owrx_module_process(owrx_module* m, const void* in, int64_t n, void* out,
                                       int64_t out_cap_bytes) {
    if (!m || n < 0 || (n > 0 && (!in || !out))) return OWRX_EINVAL;
    std::lock_guard<std::mutex> lk(m->mu);
    if (n == 0) return 0;
    hipSetDevice(m->device);
    const int64_t in_bytes = n * in_item_bytes(m->p.type) * (m->p.type == OWRX_MOD_GAIN && m->p.i0 ? 2 : 1);
    if (in_bytes > m->in_cap) {
        if (m->d_in) hipFree(m->d_in);
        m->d_in = nullptr;
        if (hipMalloc(&m->d_in, in_bytes) != hipSuccess) return OWRX_ENOMEM;
        m->in_cap = in_bytes;
    }
    if (out_cap_bytes > m->out_cap) {
        if (m->d_out) hipFree(m->d_out);
        m->d_out = nullptr;
        if (hipMalloc(&m->d_out, out_cap_bytes) != hipSuccess) return OWRX_ENOMEM;
        m->out_cap = out_cap_bytes;
    }
    const int t = m->p.type;
    if (t == OWRX_MOD_AUDIO_RESAMPLER) {
        // outputs m with m M <= (last input index) L; x = [history | block]
        const int64_t H = (int64_t)m->rhist.size();
        const int64_t total = m->count + n;                  // inputs seen
        const int64_t last_out = ((total - 1) * m->rs_L) / m->rs_M;
        const int64_t n_out = std::max<int64_t>(0, last_out + 1 - m->rs_out);
        if (n_out * 4 > out_cap_bytes) return OWRX_ENOSPC;
        const int64_t need = sizeof(float) * (H + n);
        if (need > m->in_cap) {
            if (m->d_in) hipFree(m->d_in);
            m->d_in = nullptr;
            if (hipMalloc(&m->d_in, need) != hipSuccess) return OWRX_ENOMEM;
            m->in_cap = need;
        }
        if (n_out * 4 > m->out_cap) {
            if (m->d_out) hipFree(m->d_out);
            m->d_out = nullptr;
            if (hipMalloc(&m->d_out, n_out * 4) != hipSuccess) return OWRX_ENOMEM;
            m->out_cap = n_out * 4;
        }
        float* d = (float*)m->d_in;
        const float* src = (const float*)in;
        hipMemcpyAsync(d, m->rhist.data(), sizeof(float) * H, hipMemcpyHostToDevice, m->stream);
        hipMemcpyAsync(d + H, src, sizeof(float) * n, hipMemcpyHostToDevice, m->stream);
        if (n_out > 0) {
            const int blocks = (int)std::min<int64_t>(4096, (n_out + 255) / 256);
            hipLaunchKernelGGL(mod_resample, dim3(blocks), dim3(256), 0, m->stream, d,
                               m->count - H, m->rs_out, n_out, m->d_rtaps, m->ntaps, m->rs_L,
                               m->rs_M, (float*)m->d_out);
            hipMemcpyAsync(out, m->d_out, n_out * 4, hipMemcpyDeviceToHost, m->stream);
        }
        std::vector<float> nh((size_t)H);
        for (int64_t i = 0; i < H; ++i) {
            const int64_t j = n + i;
            nh[(size_t)i] = j < H ? m->rhist[(size_t)j] : src[j - H];
        }
        if (hipStreamSynchronize(m->stream) != hipSuccess) {
            set_last_error("owrx_module_process: HIP failure");
            return OWRX_EIO;
        }
        m->rhist.swap(nh);
        m->count = total;
        m->rs_out += n_out;
        return n_out * 4;
    }
    if (t == OWRX_MOD_FMDEMOD || t == OWRX_MOD_SHIFT || t == OWRX_MOD_BANDPASS) {
        // elementwise with carried state: many lanes, one launch per call
        const int64_t item_out = t == OWRX_MOD_FMDEMOD ? 4 : 8;
        if (n * item_out > out_cap_bytes) return OWRX_ENOSPC;
        const float2* src = (const float2*)in;
        const int blocks = (int)std::min<int64_t>(4096, (n + 255) / 256);
        if (t == OWRX_MOD_BANDPASS) {
            // device input = [history | block]
            const int64_t h = m->ntaps - 1;
            const int64_t need = sizeof(float2) * (h + n);
            if (need > m->in_cap) {
                if (m->d_in) hipFree(m->d_in);
                m->d_in = nullptr;
                if (hipMalloc(&m->d_in, need) != hipSuccess) return OWRX_ENOMEM;
                m->in_cap = need;
            }
            float2* d = (float2*)m->d_in;
            hipMemcpyAsync(d, m->hist.data(), sizeof(float2) * h, hipMemcpyHostToDevice, m->stream);
            hipMemcpyAsync(d + h, src, sizeof(float2) * n, hipMemcpyHostToDevice, m->stream);
            hipLaunchKernelGGL(mod_cfir, dim3(blocks), dim3(256), 0, m->stream, d, n, m->d_taps,
                               m->ntaps, (float2*)m->d_out);
            // new history: the last ntaps - 1 samples of [history | block]
            std::vector<float2> nh((size_t)h);
            for (int64_t i = 0; i < h; ++i) {
                const int64_t j = n + i;  // index into [history | block] of the kept sample
                nh[(size_t)i] = j < h ? m->hist[(size_t)j] : src[j - h];
            }
            m->hist.swap(nh);
        } else {
            hipMemcpyAsync(m->d_in, in, in_bytes, hipMemcpyHostToDevice, m->stream);
            if (t == OWRX_MOD_FMDEMOD) {
                hipLaunchKernelGGL(mod_fmdemod, dim3(blocks), dim3(256), 0, m->stream,
                                   (const float2*)m->d_in, n, m->fm_last, (float*)m->d_out);
                m->fm_last = src[n - 1];
            } else {
                hipLaunchKernelGGL(mod_shift, dim3(blocks), dim3(256), 0, m->stream,
                                   (const float2*)m->d_in, n, m->count, m->P0, m->n0, m->rate_fx,
                                   (float2*)m->d_out);
            }
        }
        m->count += n;
        hipMemcpyAsync(out, m->d_out, n * item_out, hipMemcpyDeviceToHost, m->stream);
        if (hipStreamSynchronize(m->stream) != hipSuccess) {
            set_last_error("owrx_module_process: HIP failure");
            return OWRX_EIO;
        }
        return n * item_out;
    }
    hipMemcpyAsync(m->d_in, in, in_bytes, hipMemcpyHostToDevice, m->stream);
    int64_t produced = 0;
    const bool parallel = t == OWRX_MOD_AMDEMOD || t == OWRX_MOD_REALPART || t == OWRX_MOD_LIMIT ||
                          t == OWRX_MOD_CONVERT_F_S16 || t == OWRX_MOD_FFTSWAP ||
                          t == OWRX_MOD_CONVERT_CS16_CF32 || t == OWRX_MOD_GAIN;
    if (parallel) {
        int64_t items = n;  // scalar items of the elementwise kernel
        if (t == OWRX_MOD_CONVERT_CS16_CF32 || (t == OWRX_MOD_GAIN && m->p.i0)) items = 2 * n;
        const int64_t item_out = (t == OWRX_MOD_CONVERT_F_S16) ? 2 : 4;
        if (t == OWRX_MOD_FFTSWAP) items = (n / m->p.fft_size) * m->p.fft_size;
        if (items * item_out > out_cap_bytes) return OWRX_EINVAL;
        const int blocks = (int)std::min<int64_t>(4096, (items + 255) / 256);
        if (items > 0)
            hipLaunchKernelGGL(mod_parallel, dim3(blocks), dim3(256), 0, m->stream, m->p, m->d_in,
                               items, m->d_out);
        produced = items * item_out;
    } else {
        // the elementwise serial modules write n outputs unconditionally
        const int64_t need = (t == OWRX_MOD_AFC) ? 8 * n
                             : (t == OWRX_MOD_DCBLOCK || t == OWRX_MOD_DEEMPH || t == OWRX_MOD_AGC) ? 4 * n
                                                                                                   : 0;
        if (need > out_cap_bytes) {
            set_last_error("owrx_module_process: output capacity %lld < %lld",
                           (long long)out_cap_bytes, (long long)need);
            return OWRX_ENOSPC;
        }
        hipLaunchKernelGGL(mod_serial, dim3(1), dim3(64), 0, m->stream, m->p, m->d_in, n,
                           m->d_out, out_cap_bytes, m->d_state, m->d_produced);
        hipMemcpyAsync(&produced, m->d_produced, sizeof(int64_t), hipMemcpyDeviceToHost, m->stream);
        if (hipStreamSynchronize(m->stream) != hipSuccess) return OWRX_EIO;
        if (t == OWRX_MOD_DCBLOCK || t == OWRX_MOD_DEEMPH || t == OWRX_MOD_AGC)
            produced *= 4;
        if (t == OWRX_MOD_AFC) produced *= 8;
        if (produced > out_cap_bytes) {
            set_last_error("owrx_module_process: output capacity %lld < %lld",
                           (long long)out_cap_bytes, (long long)produced);
            return OWRX_ENOSPC;
        }
    }
    if (produced > 0)
        hipMemcpyAsync(out, m->d_out, produced, hipMemcpyDeviceToHost, m->stream);
    if (hipStreamSynchronize(m->stream) != hipSuccess) {
        set_last_error("owrx_module_process: HIP failure");
        return OWRX_EIO;
    }
    return produced;
}
