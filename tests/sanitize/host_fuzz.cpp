// host_fuzz.cpp -- sanitizer fuzz of the library's host-side parsers, the
// code that reads untrusted bytes:
//   dsp_wav_parse   WAV file images (host/wav.cpp; the reference's
//                   wav_reader.h:57-205 reads the same headers)
//   desc::generate  plugin source text, the parameter annotations
//                   (csrc/descriptor.cpp; compiler.cpp:944-1164)
//   desc::read      a code object's ELF symbols and descriptor blob
// Seeded mutations of valid inputs; an ASan / UBSan report or a broken
// invariant fails the run.  Built and run by tests/test_host_sanitizers.py:
//   g++ -std=c++17 -g -O1 -fsanitize=address,undefined -fno-sanitize-recover=all
//       -Iinclude -Idsp-bench_amd/csrc tests/sanitize/host_fuzz.cpp
//       dsp-bench_amd/host/wav.cpp dsp-bench_amd/csrc/descriptor.cpp
//   ./host_fuzz <plugin_device.h> <code object> <plugin source>...
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "descriptor.hpp"
#include "dspbench/wav.h"

namespace {

uint64_t g_state = 0x9e3779b97f4a7c15ull;
uint64_t rnd() {  // xorshift64*
    g_state ^= g_state >> 12;
    g_state ^= g_state << 25;
    g_state ^= g_state >> 27;
    return g_state * 0x2545f4914f6cdd1dull;
}
size_t below(size_t n) { return n ? (size_t)(rnd() % n) : 0; }

#define CHECK(cond)                                                                 \
    do {                                                                            \
        if (!(cond)) {                                                              \
            std::fprintf(stderr, "invariant failed: %s (%s:%d)\n", #cond, __FILE__, \
                         __LINE__);                                                 \
            std::abort();                                                           \
        }                                                                           \
    } while (0)

std::string slurp(const char *path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream s;
    s << f.rdbuf();
    return s.str();
}

void put16(std::string &b, size_t at, uint16_t v) {
    if (at + 2 <= b.size()) std::memcpy(&b[at], &v, 2);
}
void put32(std::string &b, size_t at, uint32_t v) {
    if (at + 4 <= b.size()) std::memcpy(&b[at], &v, 4);
}

// byte-level mutations shared by the three targets
void mutate_bytes(std::string &b, int rounds) {
    static const uint32_t kInteresting[] = {0u, 1u, 2u, 7u, 8u, 16u, 0x7fu, 0x80u, 0xffu, 0x100u,
                                            0x7fffu, 0x8000u, 0xffffu, 0x10000u, 0x7fffffffu,
                                            0x80000000u, 0xfffffff8u, 0xffffffffu};
    for (int r = 0; r < rounds; ++r) {
        if (b.empty()) {
            b.push_back((char)rnd());
            continue;
        }
        switch (below(7)) {
        case 0: b[below(b.size())] = (char)rnd(); break;
        case 1: b[below(b.size())] ^= (char)(1u << below(8)); break;
        case 2: put32(b, below(b.size()) & ~(size_t)3, kInteresting[below(sizeof kInteresting / 4)]); break;
        case 3: put16(b, below(b.size()) & ~(size_t)1, (uint16_t)kInteresting[below(sizeof kInteresting / 4)]); break;
        case 4: b.resize(below(b.size() + 1)); break;  // truncate
        case 5: {                                      // duplicate a slice at the end
            const size_t a = below(b.size()), n = below(std::min<size_t>(b.size() - a, 256) + 1);
            b += b.substr(a, n);
            break;
        }
        default: {  // erase a slice
            const size_t a = below(b.size()), n = below(std::min<size_t>(b.size() - a, 64) + 1);
            b.erase(a, n);
        }
        }
    }
}

// ---- WAV ------------------------------------------------------------------
std::string wav_seed(int kind) {
    std::string f(64, '\0');
    uint16_t fmt = DSP_WAV_FORMAT_PCM, ch = 2, bits = 16;
    if (kind == 1) { fmt = DSP_WAV_FORMAT_FLOAT; ch = 1; bits = 32; }
    if (kind == 2) { bits = 24; ch = 3; }
    const uint64_t frames = 100 + below(300);
    const int h = dsp_wav_write_header(&f[0], f.size(), fmt, ch, 48000, bits, frames);
    CHECK(h > 0);
    f.resize((size_t)h);
    std::string payload(frames * ch * (bits / 8u), '\0');
    for (auto &c : payload) c = (char)rnd();
    f += payload;
    if (kind == 3) {  // a LIST chunk before the data and a second data chunk after it
        std::string list = std::string("LIST") + std::string(4, '\0') + "INFOabcd";
        put32(list, 4, 12);
        f.insert(36, list);
        std::string d2 = std::string("data") + std::string(4, '\0') + std::string(40, 'x');
        put32(d2, 4, 40);
        f += d2;
    }
    if (kind == 4) {  // WAVE_FORMAT_EXTENSIBLE, PCM sub-format
        std::string e(68, '\0');
        std::memcpy(&e[0], "RIFF", 4);
        std::memcpy(&e[8], "WAVEfmt ", 8);
        put32(e, 16, 40);
        put16(e, 20, 0xfffe);
        put16(e, 22, 2);
        put32(e, 24, 44100);
        put16(e, 32, 4);
        put16(e, 34, 16);
        put16(e, 36, 22);
        put16(e, 44, 1);  // sub-format code
        static const uint8_t tail[14] = {0x00, 0x00, 0x00, 0x00, 0x10, 0x00, 0x80,
                                         0x00, 0x00, 0xaa, 0x00, 0x38, 0x9b, 0x71};
        std::memcpy(&e[46], tail, 14);
        std::memcpy(&e[60], "data", 4);
        put32(e, 64, 400);
        e += std::string(400, 'y');
        put32(e, 4, (uint32_t)(e.size() - 8));
        f = e;
    }
    return f;
}

void check_wav(const dsp_wav_info &i, uint64_t n) {
    CHECK(i.n_data_chunks >= 1 && i.n_data_chunks <= DSP_WAV_MAX_DATA_CHUNKS);
    uint64_t sum = 0;
    for (uint32_t c = 0; c < i.n_data_chunks; ++c) {
        CHECK(i.data_offset[c] <= n && i.data_size[c] <= n - i.data_offset[c]);
        sum += i.data_size[c];
    }
    CHECK(sum == i.data_bytes);
    CHECK(i.channels > 0 && i.block_align > 0);
    CHECK(i.block_align == i.channels * (i.bits_per_sample / 8));
    CHECK(i.frames * i.block_align <= i.data_bytes);
    CHECK(i.format == DSP_WAV_FORMAT_PCM || i.format == DSP_WAV_FORMAT_FLOAT);
}

int fuzz_wav(int iters) {
    int ok = 0;
    for (int it = 0; it < iters; ++it) {
        std::string f = wav_seed((int)below(5));
        if (it) mutate_bytes(f, 1 + (int)below(8));
        // parse from an exact-size heap copy, so that ASan sees any read past the end
        std::vector<uint8_t> img(f.begin(), f.end());
        dsp_wav_info info;
        const int st = dsp_wav_parse(img.empty() ? nullptr : img.data(), img.size(), &info);
        if (st == DSP_OK) {
            check_wav(info, img.size());
            ++ok;
        } else {
            CHECK(st == DSP_ERR_INVALID || st == DSP_ERR_UNSUPPORTED);
        }
    }
    return ok;
}

// ---- descriptor generation from source text ----------------------------------
const char *kTokens[] = {"struct Parameters {", "struct State {", "}", "};", "FLOAT_PARAM(", "INT_PARAM(",
                         "ENUM_PARAM(", ")", "(", ",", ";", "/*", "*/", "//", "\n", "\"", "0.5f", "-1", "1e40",
                         "2.0f", "log", "enum E { A, B, C };", "enum class F : int { X = 3, Y = -2 };",
                         "#define P(a, b) FLOAT_PARAM(a, b)\n", "__attribute__((annotate(\"", "\")))",
                         "float x;", "int n;", "E e;", "typedef float real32;", "template <typename T>",
                         "\\", "{", "P(0.0f, 1.0f) q;", "ENUM_PARAM(E) sel;", "INT_PARAM(0, 4) k;"};

int fuzz_generate(const std::vector<std::string> &sources, const std::string &header, int iters) {
    int nonempty = 0;
    for (int it = 0; it < iters; ++it) {
        std::string s = sources[below(sources.size())];
        const int rounds = 1 + (int)below(6);
        for (int r = 0; r < rounds && it; ++r) {
            const size_t at = below(s.size() + 1);
            switch (below(4)) {
            case 0: s.insert(at, kTokens[below(sizeof kTokens / sizeof *kTokens)]); break;
            case 1: s.erase(at, below(32)); break;
            case 2: if (!s.empty()) s[below(s.size())] = (char)(rnd() & 0x7f); break;
            default: s.resize(at);
            }
        }
        std::string note;
        if (std::getenv("HOST_FUZZ_TRACE")) {
            std::fprintf(stderr, "generate %d (%zu bytes)\n", it, s.size());
            std::ofstream(std::getenv("HOST_FUZZ_TRACE"), std::ios::binary) << s;  // the input being run
        }
        const std::string gen = dspb::desc::generate(s.c_str(), header.c_str(), &note);
        nonempty += !gen.empty();
    }
    return nonempty;
}

// ---- descriptor read from a code object ----------------------------------------
int fuzz_read(const std::string &co, int iters) {
    int ok = 0;
    for (int it = 0; it < iters; ++it) {
        std::string b = co;
        if (it) {
            // mostly small changes (deep into the parser), some in the ELF header
            if (below(3) == 0) {
                put32(b, 0x20 + 4 * below(8), (uint32_t)rnd());  // e_shoff / e_flags / e_*size / counts
            }
            mutate_bytes(b, 1 + (int)below(4));
        }
        std::vector<uint8_t> img(b.begin(), b.end());
        if (std::getenv("HOST_FUZZ_TRACE")) std::fprintf(stderr, "read %d (%zu bytes)\n", it, b.size());
        dspb::desc::Descriptor d;
        std::string err;
        const int st = dspb::desc::read(img.empty() ? nullptr : img.data(), img.size(), &d, &err);
        if (st == 0) {
            ++ok;
            for (const auto &p : d.params) CHECK(p.offset <= d.params_size);
        }
    }
    return ok;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: host_fuzz <plugin_device.h> <code object> <plugin source>...\n");
        return 2;
    }
    const int iters = std::getenv("HOST_FUZZ_ITERS") ? std::atoi(std::getenv("HOST_FUZZ_ITERS")) : 20000;
    if (std::getenv("HOST_FUZZ_SEED")) g_state ^= std::strtoull(std::getenv("HOST_FUZZ_SEED"), nullptr, 0) * 0x9e37u;
    const std::string header = slurp(argv[1]);
    const std::string co = slurp(argv[2]);
    std::vector<std::string> sources;
    for (int i = 3; i < argc; ++i) sources.push_back(slurp(argv[i]));
    // inputs that once hung the scanner (kept as seeds): an ENUM_PARAM with no
    // type name searched for "" forever; __attribute__ with no group after it
    sources.push_back("struct Parameters{ENUM_PARAM(e);}");
    sources.push_back("struct Parameters { __attribute__ float g; };");
    // a seed with every annotation kind (the K3 shape of SURVEY 8c)
    sources.push_back("#include \"plugin_header.h\"\nenum Mode { A, B, C, D };\n"
                      "struct Parameters {\n  INT_PARAM(0, 4) n;\n  FLOAT_PARAM(0.0f, 1.0f) g;\n"
                      "  ENUM_PARAM(Mode) m;\n};\nstruct State { float s; };\n");
    CHECK(!header.empty() && !co.empty() && !sources.empty());

    const int wav_ok = fuzz_wav(iters);
    const int gen_ok = fuzz_generate(sources, header, iters / 4);
    const int read_ok = fuzz_read(co, iters / 4);
    std::printf("host fuzz ok: wav %d/%d parsed, generate %d/%d non-empty, read %d/%d parsed\n", wav_ok, iters,
                gen_ok, iters / 4, read_ok, iters / 4);
    CHECK(wav_ok > 0 && gen_ok > 0 && read_ok > 0);  // the unmutated seeds parse
    return 0;
}
