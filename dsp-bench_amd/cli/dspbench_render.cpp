// dspbench_render -- the offline-render command line: a C++ host that drives
// the GPU path through the C ABI only (include/dspbench/*.h), the way the
// reference's host would ("called from: the build's
// offline-render CLI").
//
//   WAV file -> dsp_wav_parse -> payload to HBM -> dsp_wav_decode (planar)
//   -> dsp_render_offline / dsp_render_stft through a plugin -> dsp_wav_encode
//   -> output WAV (+ optional magnitude spectra as raw float32).
//
// It replaces the reference's load (wav_reader.h:57-205, audio.h:66-121),
// render loop (audio.cpp:13-175, pumped by wasapi_audio.cpp:223-251) and the
// analysis FFT (dsp.cpp:53-103) for a whole file, offline.
//
//   dspbench_render IN.wav OUT.wav [options]
//     --plugin NAME     gain_test (default) | IR_test | no_op | static_gain |
//                       PATH.cpp (any reference-style plugin source, compiled
//                       for gfx950 at run time: DSP_PLUGIN_GENERIC)
//     --gain G          gain_test / static_gain gain (0.2 / 0.1)
//     --ir G,STEP       IR_test parameters (0.9,0.002)
//     --block B         block size (512)
//     --bits 16|24|32|float   output sample format (default: the input's)
//     --stft FILE       also write the Hann 8192 / 4096 STFT magnitudes of the
//                       render: header "DSPMAG1\0", u32 C, u32 K, u64 F, then
//                       C x F x K float32
//     --device N        GPU ordinal (0; with --world: LOCAL_RANK if set, else the rank)
//     --device-channels C   render into C device channels, as the reference's
//                       device does (always 2, wasapi_audio.cpp:432-433): file
//                       channels past C are dropped, missing ones render from
//                       zeros (audio.cpp:65-81, 138-141).  Default: the file's.
//     --device-rate R   the sample rate handed to the plugin and written to the
//                       output header (the reference ignores the WAV's own rate,
//                       wav_reader.h:7-14).  Default: the file's.
//     --loop NBLOCKS    loop mode (audio.cpp:100-132): NBLOCKS blocks from a
//                       file that wraps around (no --stft)
//   multi-GPU (cfg 5, shard.h): one process per GPU, channels sharded one
//   run per rank, the render + STFT gathered to rank 0 over RCCL (needs --stft)
//     --world W --rank R    W processes, this one's rank (default: WORLD_SIZE /
//                       RANK from the environment when --comm-id is given)
//     --comm-id FILE    rendezvous file: rank 0 writes the RCCL id and the run
//                       id, the others wait for a file carrying their run id;
//                       rank 0 removes it once every rank has joined
//     --run-id STR      this launch's id (default: DSPB_RUN_ID, else
//                       TORCHELASTIC_RUN_ID, else none: then a file older than
//                       this process's start is taken as stale and ignored)
//     --chunk S         pipeline chunk in samples (default 16 Mi)
#include <hip/hip_runtime.h>

#include <sys/stat.h>
#include <unistd.h>

#include <ctime>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dspbench/dspbench.h"
#include "dspbench/module.h"
#include "dspbench/shard.h"
#include "dspbench/wav.h"

namespace {

int fail(const char *what, int st) {
    std::fprintf(stderr, "dspbench_render: %s: %s (%s)\n", what, dsp_status_string(st), dsp_last_error());
    return 1;
}

#define HIPCK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "dspbench_render: %s: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

bool read_file(const char *path, std::vector<unsigned char> &out) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const bool ok = n >= 0 && std::fread(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

void usage() {
    std::fprintf(stderr,
                 "usage: dspbench_render IN.wav OUT.wav [--plugin gain_test|IR_test|no_op|static_gain|PATH.cpp]\n"
                 "       [--gain G] [--ir G,STEP] [--block B] [--bits 16|24|32|float] [--stft MAG.f32]"
                 " [--device N]\n"
                 "       [--device-channels C] [--device-rate R] [--loop NBLOCKS]\n"
                 "       [--world W --rank R --comm-id FILE [--run-id STR] [--chunk SAMPLES]]\n");
}

// rank 0 writes the RCCL id and the run id to `path` (atomically: a temp
// file renamed); the other ranks wait up to two minutes for a file carrying
// their run id -- or, without one, a file written after they started -- so a
// file a previous launch left behind is never read
bool exchange_comm_id(const std::string &path, uint32_t rank, const std::string &run_id, time_t started,
                      unsigned char *id) {
    if (rank == 0) {
        if (dsp_comm_unique_id(id)) return false;
        const std::string tmp = path + ".tmp";
        FILE *f = std::fopen(tmp.c_str(), "wb");
        if (!f) return false;
        const bool ok = std::fwrite(id, 1, DSP_COMM_ID_BYTES, f) == DSP_COMM_ID_BYTES &&
                        std::fwrite(run_id.data(), 1, run_id.size(), f) == run_id.size();
        std::fclose(f);
        return ok && std::rename(tmp.c_str(), path.c_str()) == 0;
    }
    std::vector<unsigned char> buf(DSP_COMM_ID_BYTES + run_id.size() + 1);
    int tries = 1200;  // two minutes; DSPB_COMM_WAIT_S shortens it (tests)
    if (const char *w = std::getenv("DSPB_COMM_WAIT_S")) tries = std::max(1, std::atoi(w) * 10);
    for (int i = 0; i < tries; ++i, usleep(100000)) {
        struct stat sb;
        if (stat(path.c_str(), &sb) != 0) continue;
        if (run_id.empty() && sb.st_mtime < started) continue;  // stale: before this launch
        FILE *f = std::fopen(path.c_str(), "rb");
        if (!f) continue;
        const size_t n = std::fread(buf.data(), 1, buf.size(), f);
        std::fclose(f);
        if (n != DSP_COMM_ID_BYTES + run_id.size()) continue;  // another launch's run id (or a partial file)
        if (std::memcmp(buf.data() + DSP_COMM_ID_BYTES, run_id.data(), run_id.size()) != 0) continue;
        std::memcpy(id, buf.data(), DSP_COMM_ID_BYTES);
        return true;
    }
    return false;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        usage();
        return 2;
    }
    const char *in_path = argv[1], *out_path = argv[2];
    std::string plugin = "gain_test", stft_path, bits_opt;
    float gain = -1.f, ir_gain = 0.9f, ir_step = 0.002f;
    uint32_t B = 512;
    int device = -1;
    uint32_t dev_channels = 0, dev_rate = 0, world = 0, rank = 0;
    uint64_t loop_blocks = 0, chunk = 16ull << 20;
    bool have_rank = false;
    std::string comm_path, run_id;
    const time_t started = std::time(nullptr) - 2;  // (mtime has one-second resolution)
    if (const char *e = std::getenv("DSPB_RUN_ID")) run_id = e;
    else if (const char *e2 = std::getenv("TORCHELASTIC_RUN_ID")) run_id = e2;
    for (int i = 3; i < argc; i += 2) {  // every option takes one value
        const std::string a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : nullptr;
        if (!v) {
            usage();
            return 2;
        }
        if (a == "--plugin") plugin = v;
        else if (a == "--gain") gain = std::strtof(v, nullptr);
        else if (a == "--ir") {
            if (std::sscanf(v, "%f,%f", &ir_gain, &ir_step) != 2) {
                usage();
                return 2;
            }
        } else if (a == "--block") B = (uint32_t)std::strtoul(v, nullptr, 10);
        else if (a == "--bits") bits_opt = v;
        else if (a == "--stft") stft_path = v;
        else if (a == "--device") device = std::atoi(v);
        else if (a == "--device-channels") dev_channels = (uint32_t)std::strtoul(v, nullptr, 10);
        else if (a == "--device-rate") dev_rate = (uint32_t)std::strtoul(v, nullptr, 10);
        else if (a == "--loop") loop_blocks = std::strtoull(v, nullptr, 10);
        else if (a == "--world") world = (uint32_t)std::strtoul(v, nullptr, 10);
        else if (a == "--rank") rank = (uint32_t)std::strtoul(v, nullptr, 10), have_rank = true;
        else if (a == "--comm-id") comm_path = v;
        else if (a == "--run-id") run_id = v;
        else if (a == "--chunk") chunk = std::strtoull(v, nullptr, 10);
        else {
            usage();
            return 2;
        }
    }
    if (B == 0) {
        usage();
        return 2;
    }
    const bool multi = !comm_path.empty();
    if (multi) {  // torchrun-style environment when not given explicitly
        const char *ew = std::getenv("WORLD_SIZE"), *er = std::getenv("RANK");
        if (!world) world = ew ? (uint32_t)std::atoi(ew) : 1;
        if (!have_rank) rank = er ? (uint32_t)std::atoi(er) : 0;
        if (device < 0) {
            const char *lr = std::getenv("LOCAL_RANK");
            device = lr ? std::atoi(lr) : (int)rank;
        }
        if (world == 0 || rank >= world || stft_path.empty() || loop_blocks) {
            std::fprintf(stderr, "dspbench_render: --comm-id needs --stft, rank < world and no --loop\n");
            return 2;
        }
    }
    if (device < 0) device = 0;

    // ---- load + parse (wav_reader.h:57-205) --------------------------------
    std::vector<unsigned char> file;
    if (!read_file(in_path, file)) {
        std::fprintf(stderr, "dspbench_render: cannot read %s\n", in_path);
        return 1;
    }
    dsp_wav_info info{};
    int st = dsp_wav_parse(file.data(), file.size(), &info);
    if (st) return fail("dsp_wav_parse", st);
    const uint32_t Cf = info.channels;                // the file's channels
    const uint32_t C = dev_channels ? dev_channels : Cf;  // the device's (the render's)
    const uint32_t Cin = Cf < C ? Cf : C;             // channels_to_write (audio.cpp:66)
    const uint32_t rate = dev_rate ? dev_rate : info.sample_rate;
    const uint64_t L = info.frames;
    if (Cf == 0 || Cf > 16 || C == 0 || C > 16) {
        std::fprintf(stderr, "dspbench_render: %u file / %u device channels (1..16 supported)\n", Cf, C);
        return 1;
    }
    std::vector<unsigned char> payload(info.data_bytes);
    for (uint64_t c = 0, o = 0; c < info.n_data_chunks; ++c) {  // the data chunks, concatenated
        std::memcpy(payload.data() + o, file.data() + info.data_offset[c], info.data_size[c]);
        o += info.data_size[c];
    }
    file.clear();
    file.shrink_to_fit();

    HIPCK(hipSetDevice(device));
    hipStream_t s;
    HIPCK(hipStreamCreate(&s));
    dsp_exec ex{};
    ex.device = device;
    ex.stream = s;

    // ---- payload -> HBM, decode to planar float (audio.h:66-121) ----------
    const auto t0 = std::chrono::steady_clock::now();
    void *d_pay = nullptr;
    HIPCK(hipMalloc(&d_pay, payload.size() + 16));
    HIPCK(hipMemcpyAsync(d_pay, payload.data(), payload.size(), hipMemcpyHostToDevice, s));
    const uint64_t nblocks = loop_blocks ? loop_blocks : (L + B - 1) / B, Lr = nblocks * B;
    std::vector<float *> din(Cf), dout(C);
    for (uint32_t c = 0; c < Cf; ++c) HIPCK(hipMalloc(&din[c], (L ? L : 1) * sizeof(float)));
    for (uint32_t c = 0; c < C; ++c) HIPCK(hipMalloc(&dout[c], Lr * sizeof(float)));
    if ((st = dsp_wav_decode(d_pay, &info, 0, L, din.data(), &ex))) return fail("dsp_wav_decode", st);

    // ---- plugin ------------------------------------------------------------
    dsp_plugin p{};
    float pv[2] = {0.f, 0.f};
    dsp_module *mod = nullptr;
    std::vector<unsigned char> gparams;
    if (plugin == "gain_test") {
        pv[0] = gain >= 0.f ? gain : 0.2f;  // build/gain_test.cpp:23
        p.kind = DSP_PLUGIN_GAIN, p.params = pv, p.params_size = 4;
    } else if (plugin == "static_gain") {
        pv[0] = gain >= 0.f ? gain : 0.1f;  // test/static_gain_plugin.cpp:22
        p.kind = DSP_PLUGIN_STATIC_GAIN, p.state = pv, p.state_size = 4;
    } else if (plugin == "IR_test") {
        pv[0] = ir_gain, pv[1] = ir_step;  // build/IR_test.cpp:24
        p.kind = DSP_PLUGIN_IR_RAMP, p.params = pv, p.params_size = 8;
    } else if (plugin == "no_op") {
        p.kind = DSP_PLUGIN_NOOP;
    } else {  // a plugin source file: compile for gfx950, load, defaults, state
        std::vector<unsigned char> src;
        if (!read_file(plugin.c_str(), src)) {
            std::fprintf(stderr, "dspbench_render: cannot read plugin %s\n", plugin.c_str());
            return 1;
        }
        src.push_back(0);
        void *code = nullptr;
        uint64_t code_size = 0;
        std::vector<char> log(1 << 16);
        if ((st = dsp_module_compile((const char *)src.data(), plugin.c_str(), &code, &code_size, log.data(),
                                     log.size()))) {
            std::fprintf(stderr, "%s\n", log.data());
            return fail("dsp_module_compile", st);
        }
        st = dsp_module_load(code, code_size, device, &mod);
        dsp_module_free_code(code);
        if (st) return fail("dsp_module_load", st);
        uint32_t ps = 0, ss = 0;
        int stateless = 0;
        if ((st = dsp_module_sizes(mod, &ps, &ss, &stateless))) return fail("dsp_module_sizes", st);
        gparams.resize(ps ? ps : 1);
        if ((st = dsp_module_default_parameters(mod, gparams.data()))) return fail("dsp_module_default_parameters", st);
        if ((st = dsp_module_initialize_state(mod, gparams.data(), C, (float)rate, 16u << 20)))
            return fail("dsp_module_initialize_state", st);
        p.kind = DSP_PLUGIN_GENERIC, p.params = gparams.data(), p.params_size = ps, p.module = mod;
    }

    // ---- render (+ STFT) ---------------------------------------------------
    const float sr = (float)rate;
    const uint32_t N = 8192, H = 4096, K = N / 2 + 1;
    const uint64_t F = stft_path.empty() ? 0 : dsp_stft_frame_count(Lr, N, H);
    std::vector<float *> dmag(C, nullptr);
    hipEvent_t e0, e1;
    HIPCK(hipEventCreate(&e0));
    HIPCK(hipEventCreate(&e1));
    dsp_comm *comm = nullptr;
    if (multi) {
        unsigned char id[DSP_COMM_ID_BYTES];
        if (!exchange_comm_id(comm_path, rank, run_id, started, id)) {
            std::fprintf(stderr, "dspbench_render: rank %u: no communicator id at %s\n", rank, comm_path.c_str());
            return 1;
        }
        if ((st = dsp_comm_init(id, world, rank, device, &comm))) return fail("dsp_comm_init", st);
        // every rank has joined (the init is collective): the id is spent
        if (rank == 0) (void)std::remove(comm_path.c_str());
    }
    HIPCK(hipEventRecord(e0, s));
    if (multi) {
        // cfg 5: this rank renders + STFTs its run of channels, rank 0
        // gathers every channel (dout / dmag hold the whole file there)
        dsp_shard sh{};
        if ((st = dsp_shard_plan(L, C, world, rank, B, N, H, DSP_SHARD_CHANNELS, 1, &sh)))
            return fail("dsp_shard_plan", st);
        std::vector<float *> lout(sh.channels), lmag(sh.channels);
        std::vector<const float *> lin;
        for (uint32_t j = 0; j < sh.channels; ++j) {
            const uint32_t c = sh.chan0 + j;
            if (c < Cin) lin.push_back(din[c]);
            if (rank == 0) {
                lout[j] = dout[c];
            } else {
                HIPCK(hipMalloc(&lout[j], Lr * sizeof(float)));
            }
            HIPCK(hipMalloc(&lmag[j], (F ? F : 1) * K * sizeof(float)));
        }
        if (rank == 0)
            for (uint32_t c = 0; c < C; ++c) HIPCK(hipMalloc(&dmag[c], (F ? F : 1) * K * sizeof(float)));
        st = dsp_render_stft_sharded(lin.data(), (uint32_t)lin.size(), L, lout.data(), lmag.data(), K, C, B, sr, &p,
                                     N, H, DSP_WIN_HANN, K, &sh, chunk, comm, 0, rank == 0 ? dout.data() : nullptr,
                                     rank == 0 ? dmag.data() : nullptr, &ex);
        if (st) return fail("dsp_render_stft_sharded", st);
        HIPCK(hipStreamSynchronize(s));
        for (uint32_t j = 0; j < sh.channels; ++j) {
            if (rank != 0) (void)hipFree(lout[j]);
            (void)hipFree(lmag[j]);
        }
    } else if (loop_blocks) {
        uint64_t cursor = 0;
        if ((st = dsp_render_loop(din.data(), Cin, L, 0, dout.data(), C, B, nblocks, sr, &p, &cursor, &ex)))
            return fail("dsp_render_loop", st);
    } else if (!stft_path.empty() && F > 0) {
        for (uint32_t c = 0; c < C; ++c) HIPCK(hipMalloc(&dmag[c], F * K * sizeof(float)));
        st = dsp_render_stft(din.data(), Cin, L, dout.data(), C, B, sr, &p, N, H, DSP_WIN_HANN, K, dmag.data(), K,
                             &ex);
        if (st) return fail("dsp_render_stft", st);
    } else {
        if ((st = dsp_render_offline(din.data(), Cin, L, dout.data(), C, B, sr, &p, &ex)))
            return fail("dsp_render_offline", st);
    }
    HIPCK(hipEventRecord(e1, s));
    if (multi && rank != 0) {  // only the root writes
        HIPCK(hipStreamSynchronize(s));
        float ms = 0.f;
        HIPCK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("dspbench_render: rank %u of %u: channels rendered and gathered to rank 0 in %.3f ms\n", rank,
                    world, ms);
        dsp_comm_destroy(comm);
        return 0;
    }

    // ---- encode the render (audio.h:123-133 interleave) and write ----------
    uint16_t fmt = info.format, bits = info.bits_per_sample;
    if (bits_opt == "float") fmt = DSP_WAV_FORMAT_FLOAT, bits = 32;
    else if (!bits_opt.empty()) fmt = DSP_WAV_FORMAT_PCM, bits = (uint16_t)std::atoi(bits_opt.c_str());
    const uint64_t out_bytes = Lr * C * (bits / 8u);
    void *d_opay = nullptr;
    HIPCK(hipMalloc(&d_opay, out_bytes + 16));
    if ((st = dsp_wav_encode(dout.data(), C, Lr, fmt, bits, d_opay, &ex))) return fail("dsp_wav_encode", st);
    std::vector<unsigned char> out(64 + out_bytes);
    const int hdr = dsp_wav_write_header(out.data(), out.size(), fmt, (uint16_t)C, rate, bits, Lr);
    if (hdr < 0) return fail("dsp_wav_write_header", hdr);
    HIPCK(hipMemcpyAsync(out.data() + hdr, d_opay, out_bytes, hipMemcpyDeviceToHost, s));
    std::vector<float> mag;
    if (F > 0) {
        mag.resize((size_t)C * F * K);
        for (uint32_t c = 0; c < C; ++c)
            HIPCK(hipMemcpyAsync(mag.data() + (size_t)c * F * K, dmag[c], F * K * sizeof(float),
                                 hipMemcpyDeviceToHost, s));
    }
    HIPCK(hipStreamSynchronize(s));
    float render_ms = 0.f;
    HIPCK(hipEventElapsedTime(&render_ms, e0, e1));
    FILE *f = std::fopen(out_path, "wb");
    if (!f || std::fwrite(out.data(), 1, hdr + out_bytes, f) != hdr + out_bytes) {
        std::fprintf(stderr, "dspbench_render: cannot write %s\n", out_path);
        return 1;
    }
    std::fclose(f);
    if (F > 0) {
        f = std::fopen(stft_path.c_str(), "wb");
        const uint32_t hk[2] = {C, K};
        if (!f || std::fwrite("DSPMAG1", 1, 8, f) != 8 || std::fwrite(hk, 4, 2, f) != 2 ||
            std::fwrite(&F, 8, 1, f) != 1 || std::fwrite(mag.data(), 4, mag.size(), f) != mag.size()) {
            std::fprintf(stderr, "dspbench_render: cannot write %s\n", stft_path.c_str());
            return 1;
        }
        std::fclose(f);
    }
    std::printf("dspbench_render: %s: %u ch x %llu frames @ %u Hz -> %s (%s %u-bit, %llu blocks of %u)%s; "
                "render %.3f ms on the GPU, %.1f ms end to end\n",
                in_path, C, (unsigned long long)L, rate, out_path,
                fmt == DSP_WAV_FORMAT_FLOAT ? "float" : "PCM", bits, (unsigned long long)nblocks, B,
                F ? (" + STFT " + std::to_string(F) + " frames x " + std::to_string(K) + " bins").c_str() : "",
                render_ms, ms_since(t0));

    if (mod) dsp_module_destroy(mod);
    if (comm) dsp_comm_destroy(comm);
    for (uint32_t c = 0; c < Cf; ++c) (void)hipFree(din[c]);
    for (uint32_t c = 0; c < C; ++c) {
        (void)hipFree(dout[c]);
        if (dmag[c]) (void)hipFree(dmag[c]);
    }
    (void)hipFree(d_pay);
    (void)hipFree(d_opay);
    (void)hipStreamDestroy(s);
    return 0;
}
