// pipeline.cpp -- the end-to-end host path (dspbench.h dsp_render_stft_host,
// wav.h dsp_render_stft_wav): a file in host memory streamed through HBM in
// time chunks, host -> HBM -> render (+ STFT) -> host.
//
// The reference loads a whole WAV into host memory (wav_reader.h:57-205),
// converts it (audio.h:66-121) and renders block by block
// (audio.cpp:13-175).  Here the file crosses PCIe once per chunk, three HIP
// streams deep:
//
//   up stream       chunk t's payload (or float rows) H2D into slot t % 2
//   compute stream  decode (WAV) + dsp_render_stft / dsp_render_offline of
//                   chunk t, with sample_offset = the chunk's start
//   down stream     chunk t's owned render rows and magnitude rows D2H
//
// so chunk t + 1's upload and chunk t - 1's download overlap chunk t's
// compute.  Chunks come from the time planner (dsp_shard_chunks, a one-rank
// shard): lcm(B, H)-aligned with an N - H halo, so chunked results equal the
// whole-file call bit for bit.  Plugins with state, and the FIR, run as one
// chunk.  Host buffers that are pinned (hipHostMalloc / hipHostRegister) are
// DMA'd directly; pageable ones go through pinned staging slots, copied by
// the calling thread while the GPU works on the other slot.  Downloads into
// HSA-allocated pinned memory run on an SDMA engine (sdma.hpp: the HIP
// runtime a PyTorch process uses would run them as blit kernels on the CUs,
// stalling the next chunk's kernel behind them); others go through
// hipMemcpyAsync on the down stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "dspbench/module.h"
#include "dspbench/shard.h"
#include "dspbench/wav.h"
#include "sdma.hpp"

namespace dspb {
void set_last_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);
}  // namespace dspb
using dspb::set_last_error;

#define PL_HIP(x)                                                  \
    do {                                                           \
        hipError_t e_ = (x);                                       \
        if (e_ != hipSuccess) return dspb::hip_fail(e_, #x);       \
    } while (0)

namespace {

bool is_pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

struct Source {  // what is streamed in: a WAV payload or planar float rows
    const unsigned char *payload = nullptr;  // WAV: concatenated data bytes
    dsp_wav_info info{};
    const float *const *rows = nullptr;      // float: in_channels rows of L
    uint32_t in_channels = 0;
    uint64_t L = 0;
    bool wav() const { return payload != nullptr; }
    uint64_t chunk_bytes(uint64_t frames) const {
        return wav() ? frames * info.block_align : frames * sizeof(float) * in_channels;
    }
};

struct Slot {
    void *d_up = nullptr;           // device: payload bytes or in_channels float rows
    float *d_in = nullptr;          // device: decoded planar input (WAV)
    float *d_out = nullptr;         // device: C render rows
    float *d_mag = nullptr;         // device: C magnitude rows
    unsigned char *h_up = nullptr;  // pinned staging (pageable source)
    float *h_out = nullptr;         // pinned staging (pageable outputs)
    float *h_mag = nullptr;
    hipEvent_t up_done = nullptr, comp_done = nullptr, down_done = nullptr;
    bool pending_down = false;      // a download into h_out / h_mag not yet copied out
    uint64_t t_start = 0, t_rlen = 0, t_frame0 = 0, t_frames = 0;
};

struct Resources {
    dspb::SdmaDownloader dl;        // SDMA downloads (when used): stopped first
    bool use_sdma = false;
    std::vector<Slot> slots;
    hipStream_t up = nullptr, down = nullptr;
    hipStream_t compute = nullptr;  // the caller's stream (not owned)
    bool compute_used = false;
    int prev_device = -1;           // restored on exit
    ~Resources() {
        // an early return leaves copies and kernels in flight on the slots'
        // buffers: drain them before the buffers go
        (void)dl.finish();
        if (up) (void)hipStreamSynchronize(up);
        if (compute_used) (void)hipStreamSynchronize(compute);
        if (down) (void)hipStreamSynchronize(down);
        (void)hipGetLastError();
        // downloads that never landed (SdmaDownloader::poisoned): the engine
        // may still read the device rows and write the pinned ones -- keep both
        const bool keep = dl.poisoned();
        for (Slot &s : slots) {
            if (s.d_up) (void)hipFree(s.d_up);
            if (s.d_in) (void)hipFree(s.d_in);
            if (s.d_out && !keep) (void)hipFree(s.d_out);
            if (s.d_mag && !keep) (void)hipFree(s.d_mag);
            if (s.h_up) (void)hipHostFree(s.h_up);
            if (s.h_out && !keep) (void)hipHostFree(s.h_out);
            if (s.h_mag && !keep) (void)hipHostFree(s.h_mag);
            for (hipEvent_t e : {s.up_done, s.comp_done, s.down_done})
                if (e) (void)hipEventDestroy(e);
        }
        if (up) (void)hipStreamDestroy(up);
        if (down) (void)hipStreamDestroy(down);
        if (prev_device >= 0) (void)hipSetDevice(prev_device);
    }
};

int invalid(const char *msg) {
    set_last_error("%s", msg);
    return DSP_ERR_INVALID;
}

int run(const Source &src, uint32_t C, uint32_t B, float sr, const dsp_plugin *plugin, bool stft, uint32_t N,
        uint32_t H, int32_t window, uint32_t K, float *const *out, float *const *mag, uint64_t ld, uint64_t chunk,
        const dsp_exec *ex) {
    if (ex && ex->result) *ex->result = 0;  // the chunks' DSP_RESULT_* bits are OR-ed in
    if (B == 0 || C == 0) return B == 0 ? invalid("block size B must be > 0") : DSP_OK;
    if (!out) return invalid("out is NULL");
    for (uint32_t c = 0; c < C; ++c)
        if (!out[c] || (stft && (!mag || !mag[c]))) return invalid("out / mag row is NULL");
    const uint64_t L = src.wav() ? src.info.frames : src.L;
    const uint32_t Cin = std::min<uint32_t>(src.wav() ? src.info.channels : src.in_channels, C);
    Resources R;  // declared first: restores the caller's device on every return
    int dev = -1;
    PL_HIP(hipGetDevice(&dev));
    if (ex && ex->device >= 0 && ex->device != dev) {
        PL_HIP(hipSetDevice(ex->device));
        R.prev_device = dev;
    }
    const hipStream_t cs = ex ? (hipStream_t)ex->stream : nullptr;
    R.compute = cs;
    const uint64_t goff = ex ? ex->sample_offset : 0;
    if (goff % B) return invalid("sample_offset must be a multiple of B");
    // render-only: chunks of whole blocks without a halo (N = H = B)
    const uint32_t pN = stft ? N : B, pH = stft ? H : B;
    // the FIR's and the BIQUAD's history and a GENERIC plugin's State carry across blocks:
    // one chunk (a GENERIC plugin without a State chunks like the map plugins)
    int stateless = 1;
    if (plugin && plugin->kind == DSP_PLUGIN_GENERIC) {
        if (!plugin->module) return invalid("GENERIC plugin needs a loaded dsp_module");
        if (int e = dsp_module_sizes((const dsp_module *)plugin->module, nullptr, nullptr, &stateless)) return e;
    }
    const bool one = plugin && (plugin->kind == DSP_PLUGIN_FIR || plugin->kind == DSP_PLUGIN_BIQUAD ||
                                (plugin->kind == DSP_PLUGIN_GENERIC && !stateless));
    dsp_shard whole{};
    int st = dsp_shard_plan(L, C, 1, 0, B, pN, pH, DSP_SHARD_TIME, 1, &whole);
    if (st) return st;
    const bool halo_fits = (uint64_t)(pN - pH + B - 1) / B * B < pN || pN == pH;
    const int64_t n = dsp_shard_chunks(&whole, L, B, pN, pH, 1, (one || !halo_fits) ? 0 : chunk, nullptr, 0);
    if (n < 0) return (int)n;
    std::vector<dsp_shard> ch((size_t)n);
    dsp_shard_chunks(&whole, L, B, pN, pH, 1, (one || !halo_fits) ? 0 : chunk, ch.data(), ch.size());
    const uint64_t Lpad = (L + B - 1) / B * B;
    if (n == 0) return DSP_OK;  // an empty file renders ceil(0 / B) = 0 blocks
    // slot sizes: the largest chunk
    uint64_t max_in = 0, max_pad = 0, max_fr = 0;
    for (const dsp_shard &c : ch) {
        const uint64_t nin = std::min<uint64_t>(L - c.start, c.owned + c.halo);
        max_in = std::max(max_in, nin);
        max_pad = std::max(max_pad, (nin + B - 1) / B * B);
        max_fr = std::max(max_fr, c.frames);
    }
    // row strides of the slots: whole 16-byte units, so every row is as
    // aligned as a fresh allocation (the fused kernels need 8-byte rows)
    max_in = (max_in + 3) & ~3ull;
    max_pad = (max_pad + 3) & ~3ull;
    bool in_pinned = true, out_pinned = true;
    if (src.wav()) in_pinned = is_pinned(src.payload);
    else
        for (uint32_t c = 0; c < Cin; ++c) in_pinned = in_pinned && is_pinned(src.rows[c]);
    for (uint32_t c = 0; c < C; ++c) out_pinned = out_pinned && is_pinned(out[c]) && (!stft || is_pinned(mag[c]));

    R.slots.resize(std::min<int64_t>(n, 2));
    PL_HIP(hipStreamCreateWithFlags(&R.up, hipStreamNonBlocking));
    PL_HIP(hipStreamCreateWithFlags(&R.down, hipStreamNonBlocking));
    const uint64_t up_bytes = src.chunk_bytes(max_in);
    for (Slot &s : R.slots) {
        if (Cin) PL_HIP(hipMalloc(&s.d_up, up_bytes + 16));
        if (Cin && src.wav()) PL_HIP(hipMalloc((void **)&s.d_in, sizeof(float) * src.info.channels * max_in + 16));
        PL_HIP(hipMalloc((void **)&s.d_out, sizeof(float) * C * max_pad));
        if (stft) PL_HIP(hipMalloc((void **)&s.d_mag, sizeof(float) * C * std::max<uint64_t>(max_fr, 1) * ld));
        if (Cin && !in_pinned) PL_HIP(hipHostMalloc((void **)&s.h_up, up_bytes + 16, hipHostMallocDefault));
        if (!out_pinned) {
            PL_HIP(hipHostMalloc((void **)&s.h_out, sizeof(float) * C * max_pad, hipHostMallocDefault));
            if (stft)
                PL_HIP(hipHostMalloc((void **)&s.h_mag, sizeof(float) * C * std::max<uint64_t>(max_fr, 1) * ld,
                                     hipHostMallocDefault));
        }
        PL_HIP(hipEventCreateWithFlags(&s.up_done, hipEventDisableTiming));
        PL_HIP(hipEventCreateWithFlags(&s.comp_done, hipEventDisableTiming));
        PL_HIP(hipEventCreateWithFlags(&s.down_done, hipEventDisableTiming));
    }
    // downloads on an SDMA engine when every destination allows it
    {
        int cur = -1;
        PL_HIP(hipGetDevice(&cur));
        bool ok = true;
        for (uint32_t c = 0; c < C && ok; ++c) {
            ok = dspb::SdmaDownloader::usable(cur, out_pinned ? (const void *)out[c] : R.slots[0].h_out);
            if (ok && stft) ok = dspb::SdmaDownloader::usable(cur, out_pinned ? (const void *)mag[c] : R.slots[0].h_mag);
        }
        if (ok && !out_pinned)
            for (const Slot &sl : R.slots)
                ok = ok && dspb::SdmaDownloader::usable(cur, sl.h_out) && (!stft || dspb::SdmaDownloader::usable(cur, sl.h_mag));
        R.use_sdma = ok;
        if (ok && (st = R.dl.start(cur, (int)R.slots.size()))) return st;
    }
    // a slot's downloads have landed
    auto landed = [&](Slot &s) -> int {
        if (R.use_sdma) return R.dl.wait_slot((int)(&s - R.slots.data()));
        PL_HIP(hipEventSynchronize(s.down_done));
        return DSP_OK;
    };
    // copy a finished download out of the pinned staging slot
    auto drain = [&](Slot &s) -> int {
        if (!s.pending_down) return DSP_OK;
        if (int e = landed(s)) return e;
        for (uint32_t c = 0; c < C; ++c) {
            std::memcpy(out[c] + s.t_start, s.h_out + (uint64_t)c * max_pad, s.t_rlen * sizeof(float));
            if (stft && s.t_frames)
                std::memcpy(mag[c] + s.t_frame0 * ld, s.h_mag + (uint64_t)c * max_fr * ld,
                            s.t_frames * ld * sizeof(float));
        }
        s.pending_down = false;
        return DSP_OK;
    };
    for (int64_t t = 0; t < n; ++t) {
        Slot &s = R.slots[(size_t)t % R.slots.size()];
        const dsp_shard &c = ch[(size_t)t];
        const uint64_t nin = std::min<uint64_t>(L - c.start, c.owned + c.halo);
        // the slot's previous chunk: its upload buffer and device rows are
        // free once its download finished
        if ((st = drain(s))) return st;
        if ((st = landed(s))) return st;
        // ---- upload
        if (Cin) {
            if (src.wav()) {
                const unsigned char *p = src.payload + c.start * src.info.block_align;
                const uint64_t bytes = nin * src.info.block_align;
                if (!in_pinned) {
                    std::memcpy(s.h_up, p, bytes);
                    p = s.h_up;
                }
                PL_HIP(hipMemcpyAsync(s.d_up, p, bytes, hipMemcpyHostToDevice, R.up));
            } else {
                for (uint32_t j = 0; j < Cin; ++j) {
                    const float *p = src.rows[j] + c.start;
                    float *d = (float *)s.d_up + (uint64_t)j * max_in;
                    if (!in_pinned) {
                        float *h = (float *)s.h_up + (uint64_t)j * max_in;
                        std::memcpy(h, p, nin * sizeof(float));
                        p = h;
                    }
                    PL_HIP(hipMemcpyAsync(d, p, nin * sizeof(float), hipMemcpyHostToDevice, R.up));
                }
            }
        }
        PL_HIP(hipEventRecord(s.up_done, R.up));
        // ---- compute (decode + render [+ STFT]) on the caller's stream
        R.compute_used = true;
        PL_HIP(hipStreamWaitEvent(cs, s.up_done, 0));
        dsp_exec e{};
        e.device = -1;
        e.flags = ex ? (ex->flags & DSP_EXEC_METHOD_FLAGS) : 0;
        e.stream = cs;
        e.sample_offset = goff + c.start;
        uint32_t chunk_res = 0;  // DSP_RESULT_* of this chunk, OR-ed into the caller's
        e.result = &chunk_res;
        std::vector<const float *> rin(Cin);
        std::vector<float *> rout(C), rmag(C);
        if (Cin && src.wav()) {
            dsp_wav_info ci = src.info;
            ci.frames = nin;
            ci.data_bytes = nin * src.info.block_align;
            // every file channel is decoded (the kernel writes all rows);
            // those past the device's C are not rendered (audio.cpp:66)
            std::vector<float *> dec(src.info.channels);
            for (uint32_t j = 0; j < src.info.channels; ++j) dec[j] = s.d_in + (uint64_t)j * max_in;
            if ((st = dsp_wav_decode(s.d_up, &ci, 0, nin, dec.data(), &e))) return st;
            for (uint32_t j = 0; j < Cin; ++j) rin[j] = s.d_in + (uint64_t)j * max_in;
        } else {
            for (uint32_t j = 0; j < Cin; ++j) rin[j] = (const float *)s.d_up + (uint64_t)j * max_in;
        }
        for (uint32_t j = 0; j < C; ++j) {
            rout[j] = s.d_out + (uint64_t)j * max_pad;
            if (stft) rmag[j] = s.d_mag + (uint64_t)j * std::max<uint64_t>(max_fr, 1) * ld;
        }
        if (stft)
            st = dsp_render_stft(rin.data(), Cin, nin, rout.data(), C, B, sr, plugin, N, H, window, K, rmag.data(), ld,
                                 &e);
        else
            st = dsp_render_offline(rin.data(), Cin, nin, rout.data(), C, B, sr, plugin, &e);
        if (st) return st;
        if (ex && ex->result) *ex->result |= chunk_res;
        PL_HIP(hipEventRecord(s.comp_done, cs));
        // ---- download the owned rows
        const uint64_t rlen = (c.start + c.owned >= L) ? Lpad - c.start : c.owned;
        s.t_start = c.start;
        s.t_rlen = rlen;
        s.t_frame0 = c.frame0;
        s.t_frames = stft ? c.frames : 0;
        std::vector<dspb::HostCopy> copies;
        for (uint32_t j = 0; j < C; ++j) {
            float *dst = out_pinned ? out[j] + c.start : s.h_out + (uint64_t)j * max_pad;
            copies.push_back({dst, rout[j], rlen * sizeof(float)});
            if (stft && c.frames) {
                float *md = out_pinned ? mag[j] + c.frame0 * ld : s.h_mag + (uint64_t)j * max_fr * ld;
                copies.push_back({md, rmag[j], c.frames * ld * sizeof(float)});
            }
        }
        if (R.use_sdma) {
            if ((st = R.dl.submit((int)(t % (int64_t)R.slots.size()), s.comp_done, std::move(copies)))) return st;
        } else {
            PL_HIP(hipStreamWaitEvent(R.down, s.comp_done, 0));
            for (const dspb::HostCopy &hc : copies)
                PL_HIP(hipMemcpyAsync(hc.dst, hc.src, hc.bytes, hipMemcpyDeviceToHost, R.down));
            PL_HIP(hipEventRecord(s.down_done, R.down));
        }
        s.pending_down = !out_pinned;
    }
    for (Slot &s : R.slots)
        if ((st = drain(s)) || (st = landed(s))) return st;
    if ((st = R.dl.finish())) return st;
    PL_HIP(hipStreamSynchronize(R.down));
    PL_HIP(hipStreamSynchronize(cs));
    return DSP_OK;
}

}  // namespace

extern "C" {

int dsp_render_stft_host(const float *const *in, uint32_t in_channels, uint64_t L, float *const *out, uint32_t C,
                         uint32_t B, float sr, const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window,
                         uint32_t K, float *const *mag, uint64_t ld, uint64_t chunk, const dsp_exec *ex) {
    if (in_channels && !in) return invalid("in is NULL");
    for (uint32_t c = 0; c < in_channels; ++c)
        if (!in[c]) return invalid("in row is NULL");
    Source s;
    s.rows = in;
    s.in_channels = in_channels;
    s.L = L;
    const bool stft = mag != nullptr;
    if (stft && (N == 0 || (N & (N - 1)) || N > 8192 || H == 0 || K == 0 || ld < K))
        return invalid("bad STFT arguments");
    return run(s, C, B, sr, plugin, stft, N, H, window, K, out, mag, ld, chunk, ex);
}

int dsp_render_stft_wav(const void *payload, const dsp_wav_info *info, uint32_t C, uint32_t B, float sr,
                        const dsp_plugin *plugin, uint32_t N, uint32_t H, int32_t window, uint32_t K,
                        float *const *out, float *const *mag, uint64_t ld, uint64_t chunk, const dsp_exec *ex) {
    if (!info || (info->frames && !payload)) return invalid("payload / info is NULL");
    if (info->channels == 0 || info->block_align == 0) return invalid("bad dsp_wav_info");
    Source s;
    s.payload = (const unsigned char *)payload;
    s.info = *info;
    const bool stft = mag != nullptr;
    if (stft && (N == 0 || (N & (N - 1)) || N > 8192 || H == 0 || K == 0 || ld < K))
        return invalid("bad STFT arguments");
    return run(s, C, B, sr, plugin, stft, N, H, window, K, out, mag, ld, chunk, ex);
}

}  // extern "C"
