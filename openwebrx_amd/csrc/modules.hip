// modules.hip -- single csdr modules run on the GPU with persistent state, for pycsdr module
// objects that are not part of a fused chain and for per-module parity tests.  Each call copies
// the host input to HBM, runs the module's kernel (the same __device__ step functions the fused
// post kernel uses) and copies the output back.
#include <string.h>

#include <mutex>

#include "../../include/owrx_amd.h"
#include "design.h"
#include "owrx_types.h"

namespace owrx {
void set_last_error(const char* fmt, ...);

struct ModState {
    float2 fm_last;
    float yp, xp, yp2;
    AgcState agc;
    AdpcmState adpcm;
    int64_t adpcm_bytes;
    int32_t has_left;
    int32_t left;
};

struct ModParams {
    int type;
    float f0;
    int i0;
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
        case OWRX_MOD_REALPART: return 8;
        case OWRX_MOD_ADPCM: return 2;
        case OWRX_MOD_CONVERT_CS16_CF32: return 4;
        default: return 4;
    }
}

extern "C" int owrx_module_create(int device, int type, double p0, double p1, double p2,
                                  owrx_module** out) {
    if (!out || type < OWRX_MOD_FMDEMOD || type > OWRX_MOD_GAIN) {
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
        case OWRX_MOD_GAIN:
            m->p.f0 = (float)p0;
            m->p.i0 = p1 > 0 ? 1 : 0;  // complex: n samples = 2n floats
            break;
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
    *out = m;
    return OWRX_OK;
}

extern "C" int owrx_module_destroy(owrx_module* m) {
    if (!m) return OWRX_EINVAL;
    hipSetDevice(m->device);
    if (m->d_state) hipFree(m->d_state);
    if (m->d_produced) hipFree(m->d_produced);
    if (m->d_in) hipFree(m->d_in);
    if (m->d_out) hipFree(m->d_out);
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
    hipMemcpyAsync(m->d_in, in, in_bytes, hipMemcpyHostToDevice, m->stream);
    int64_t produced = 0;
    const int t = m->p.type;
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
        hipLaunchKernelGGL(mod_serial, dim3(1), dim3(64), 0, m->stream, m->p, m->d_in, n,
                           m->d_out, out_cap_bytes, m->d_state, m->d_produced);
        hipMemcpyAsync(&produced, m->d_produced, sizeof(int64_t), hipMemcpyDeviceToHost, m->stream);
        if (hipStreamSynchronize(m->stream) != hipSuccess) return OWRX_EIO;
        if (t == OWRX_MOD_FMDEMOD || t == OWRX_MOD_DCBLOCK || t == OWRX_MOD_DEEMPH ||
            t == OWRX_MOD_AGC)
            produced *= 4;
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
