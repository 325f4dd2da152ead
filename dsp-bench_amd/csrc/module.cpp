// module.cpp -- generic GPU dispatch: plugin source -> hiprtc -> gfx950 code
// object -> kernels that call the plugin's own functions (module.h).
//
// The generated translation unit is, in order:
//   plugin_device.h          (as "plugin_header.h": device services)
//   #pragma clang force_cuda_host_device begin
//   #define annotate(...)     (the annotations are read from the text)
//   the plugin source         (unchanged; its #include of plugin_header.h
//                              hits the include guard)
//   #pragma clang force_cuda_host_device end
//   the descriptor            (dspb_desc_blob / dspb_desc_text, descriptor.cpp)
//   kDriver                   (dspb_sizes / _defaults / _init / _render /
//                              _callback kernels)
// compiled with -ffp-contract=off so the plugin's float / double arithmetic
// rounds as the CPU build of the same source does.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "descriptor.hpp"
#include "ir_proof.hpp"
#include "dspbench/module.h"
#include "kernels.hpp"

namespace {

#include "plugin_device_src.inc"  // const char kPluginDeviceSrc[] (generated from plugin_device.h)

constexpr uint64_t kStagedLdsBytes = 64 * 1024;  // stateful render's LDS double-buffer limit
#ifndef DSPB_LDS_ROUND
#define DSPB_LDS_ROUND (76 * 1024)
#define DSPB_LDS_WGS 2
#endif
// LDS per workgroup round of the stateless LDS-blocks path (kDriver
// dspb_lds_nb: the same formula, handed to hiprtc as DSPB_LDS_ROUND_BYTES),
// and the persistent grid's workgroups per CU
constexpr uint64_t kLdsRoundBytes = DSPB_LDS_ROUND;
constexpr uint64_t kLdsWgPerCu = DSPB_LDS_WGS;

// the LDS-blocks kernels of kDriver: (C, B) = 0 matches any value
struct LdsShape {
    const char *name;
    uint32_t C, B;
};
constexpr LdsShape kLdsShapes[7] = {{"dspb_render_lds", 0, 0},         {"dspb_render_lds_c2b512", 2, 512},
                                    {"dspb_render_lds_c2b256", 2, 256}, {"dspb_render_lds_c2b1024", 2, 1024},
                                    {"dspb_render_lds_c1b512", 1, 512}, {"dspb_render_lds_c1", 1, 0},
                                    {"dspb_render_lds_c2", 2, 0}};
// the stateful LDS path's kernels: dspb_render covers every other shape
constexpr LdsShape kStShapes[4] = {{"dspb_render_st_c2b512", 2, 512}, {"dspb_render_st_c2b256", 2, 256},
                                   {"dspb_render_st_c1", 1, 0}, {"dspb_render_st_c2", 2, 0}};
// speculative segments of a stateful render (kDriver dspb_segments): pass 1 /
// rerun kernels, most specific first, and the walk's
// (pass 1, its reruns; pipelined: blocks at a stride of C B + 2 and 4 | B)
struct SegShape {
    const char *name, *rerun;
    uint32_t C, B;
    bool pf;
};
constexpr SegShape kSegShapes[5] = {{"dspb_seg_c2b512", "dspb_seg_c2b512_rerun", 2, 512, true},
                                    {"dspb_seg_c2", "dspb_seg_c2_rerun", 2, 0, true},
                                    {"dspb_seg_c1", "dspb_seg_c1_rerun", 1, 0, true},
                                    {"dspb_seg_c4", "dspb_seg_c4_rerun", 4, 0, true},
                                    {"dspb_seg", nullptr, 0, 0, false}};
constexpr LdsShape kWalkShapes[2] = {{"dspb_seg_walk_c2b512", 2, 512}, {"dspb_seg_walk_any", 0, 0}};
// the chain kernels of a State that never forgets (kSegDriver dspb_seg_chain;
// B = 0: any B <= kChainMaxB, the private block sized for it)
constexpr LdsShape kChainShapes[4] = {{"dspb_seg_chain_c2b512", 2, 512}, {"dspb_seg_chain_c2", 2, 0},
                                      {"dspb_seg_chain_c1", 1, 0}, {"dspb_seg_chain_c4", 4, 0}};
// the chain of a split State's block-independent words, the same shapes
constexpr LdsShape kChainIndShapes[4] = {{"dspb_seg_chain_ind_c2b512", 2, 512}, {"dspb_seg_chain_ind_c2", 2, 0},
                                         {"dspb_seg_chain_ind_c1", 1, 0}, {"dspb_seg_chain_ind_c4", 4, 0}};
constexpr uint32_t kChainMaxB = 4096;
constexpr uint32_t kSegMaxState = 1024;   // bytes of State a lane copies (the walk keeps one in LDS)
constexpr uint32_t kSegWarm0 = 4;         // blocks of warm-up of a first render
constexpr uint32_t kSegWarmBumps = 2;     // at most this many blocks added for a few misses
constexpr uint32_t kSegWarmMax = 4096;    // the longest warm-up (blocks); past it, the chain is serial
constexpr uint32_t kSegLevels = 4;        // warm-up levels a render may try (x16 each)
constexpr uint32_t kSegMinBlocks = 4;     // blocks per segment at least

// Host mirror of the driver's argument block (same layout on both sides).
struct RenderArgsG {
    void *P;
    void *S;
    float *in[dspb::kMaxChannels];
    float *out[dspb::kMaxChannels];
    unsigned long long L;
    unsigned long long nblocks;
    unsigned long long block0;
    unsigned in_ch;
    unsigned C;
    unsigned B;
    float sr;
    unsigned lds;  // path: stateful 1 = LDS double buffer; stateless 1/2 private, 3 LDS blocks
    unsigned lds_nb;      // stateless LDS path: blocks per workgroup round
    unsigned lds_stride;  // stateless LDS path: floats per block in LDS (C B + 1)
    unsigned par;         // blocks render independently (dsp_module: par), in parallel
};
// Host mirror of kDriver's dspb_seg_args.
struct SegArgsG {
    RenderArgsG R;
    void *st_blk;
    void *st_end;
    unsigned *list;
    unsigned *count;
    unsigned *prev_count;
    unsigned char *flags;
    unsigned *stats;
    unsigned long long seg;
    unsigned K;
    unsigned warm;
    unsigned prev_warm;
    unsigned level;
    unsigned mode;
    unsigned pass;
    unsigned exact;
    unsigned long long perturb;
    void *st_ind;
    unsigned split;
};

// kDriver / kSegDriver: the driver kernels (csrc/plugin_driver.inl) and the
// speculative-segment kernels (csrc/plugin_driver_seg.inl), as strings
#include "plugin_driver_src.inc"

struct ArenaHost {  // mirror of dspb_arena
    char *base;
    unsigned long long capacity;
    unsigned long long used;
    float *fft_tmp;
    unsigned long long failed;
};

}  // namespace

struct dsp_descriptor {
    dspb::desc::Descriptor d;
};

struct dsp_module {
    dsp_descriptor *desc = nullptr;  // from the code object (NULL for code without one)
    int device = -1;
    hipModule_t mod = nullptr;
    hipModule_t chain_mod = nullptr;   // the State chain kernels from edited IR (dspb_chain_co), or NULL
    // the LDS-blocks kernels (NULL for code objects compiled before they
    // existed): [0] any (C, B), then the instantiations of kLdsShapes
    hipFunction_t f_render_lds[7] = {};
    hipFunction_t f_render_st[4] = {};  // kStShapes (NULL: dspb_render)
    // speculative segments (kSegShapes, the check, kWalkShapes; NULL in code
    // objects compiled before them: the serial chain)
    hipFunction_t f_seg[5] = {}, f_seg_rerun[5] = {}, f_seg_check = nullptr, f_seg_walk[2] = {};
    // kChainShapes and their private memory per lane: one whose compiled
    // form kept more than a State copy there kept (part of) the block, which
    // the State then depends on -- the serial chain renders instead
    hipFunction_t f_seg_chain[4] = {};
    int chain_priv[4] = {};
    hipFunction_t f_seg_chain_ind[4] = {};  // kChainIndShapes (facts.state_split), private memory as above
    int chain_ind_priv[4] = {};
    struct SegWork {
        void *blk = nullptr;           // [cap_blk] States: st_blk
        void *ind = nullptr;           // [cap_ind] States: a split State's independent words (st_ind, 4 K)
        uint64_t cap_ind = 0;
        void *end = nullptr;           // [cap] States: st_end
        uint64_t cap_blk = 0;
        unsigned *list = nullptr;      // [cap]
        unsigned char *flags = nullptr;  // [cap]
        unsigned *words = nullptr;     // [0] count, [4..8) stats
        uint32_t cap = 0;
        // the counters of the last two speculative renders: pinned copies
        // [2][4], each behind an event, read back without waiting by a later
        // call (what the module learns) or waiting by dsp_module_state_spec
        unsigned *h_stats = nullptr;
        hipEvent_t ev[2] = {};
        bool pending[2] = {};
        uint64_t seq[2] = {};
        dsp_state_spec_info info[2] = {};
        uint64_t calls = 0;
        dsp_state_spec_info last{};    // the newest render whose counters were read
        bool serial = false;           // the module's last State-writing render was the serial chain
        uint32_t warm = 0;             // learned warm-up for `params` (0: not yet)
        bool off = false;              // learned: the chain does not forget its State
        bool chain_bad = false;        // learned: the State chain's records failed their check
        bool one_level = false;        // learned: the first warm-up level suffices (two levels launched)
        uint32_t bumps = 0;            // warm-up blocks added after renders whose few misses took a rerun
        bool slot_one[2] = {};         // the render in the slot was launched with the first two levels alone
        uint64_t gen = 0;              // bumped when `params` change (learn only from renders with them)
        uint64_t slot_gen[2] = {};
        uint64_t perturb = 0;          // dsp_module_debug: the next State chain's wrong record (block + 1)
        std::vector<unsigned char> params;
        uint32_t C = 0, B = 0;         // ... and the shape it was learnt with (kernels differ by shape)
    } seg;
    hipFunction_t f_sizes = nullptr, f_defaults = nullptr, f_init = nullptr, f_render = nullptr,
                  f_callback = nullptr;
    uint32_t params_size = 0, state_size = 0;
    int stateless = 0;                 // State is empty
    // blocks render independently, so in parallel: the callback's IR was
    // analysed completely (no global memory written, no unknown call) and it
    // never writes its State (facts); otherwise the blocks run in order on
    // one lane, as the reference's audio thread runs them
    int par = 0;
    bool has_facts = false;            // the code object carries dspb_callback_facts
    dspb::irp::Facts facts;            // what the callback's IR shows (ir_proof.hpp)
    int cus = 256;                     // compute units of the device (persistent grids)
    void *h_params = nullptr;          // pinned staging of the Parameters upload
    hipEvent_t upload_ev = nullptr;    // the last upload from h_params
    hipEvent_t use_ev = nullptr;       // the last render launched with d_params / d_state
    void *d_params = nullptr;          // device Parameters
    void *d_state[2] = {nullptr, nullptr};  // [0] live State, [1] compute_IR scratch State
    ArenaHost *d_arena[2] = {nullptr, nullptr};
    char *arena_mem[2] = {nullptr, nullptr};
    bool initialized = false;
    // block classes found by module_specialize, per (Parameters, C, B, sr);
    // newest last, at most kSpecCache
    // a table class's block: the calls that hold it (module_specialize hands
    // it out, module_spec_done takes it back after the call's launches), an
    // event per stream after its last use, and whether a captured graph may
    // replay it (then it lives as long as the module)
    struct SpecUse {
        float *table = nullptr;
        std::map<hipStream_t, hipEvent_t> ev;
        int inflight = 0;
        bool captured = false;
    };
    struct Spec {
        std::vector<unsigned char> params;
        uint32_t C, B;
        float sr;
        dspb::ModuleSpec r;
        std::shared_ptr<SpecUse> use;  // table classes only
    };
    std::vector<Spec> spec;
    // tables of evicted entries: freed once no call holds them and their
    // streams have passed their last use (spec_reap), or by
    // dsp_module_destroy when a captured graph may replay them
    std::vector<std::shared_ptr<SpecUse>> retired;
    std::mutex mu;
};

namespace dspb {
void set_last_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);
int module_seg_collect(dsp_module *m, bool wait);
}  // namespace dspb
using dspb::set_last_error;

#define MOD_HIP(x)                                                   \
    do {                                                             \
        hipError_t e_ = (x);                                         \
        if (e_ != hipSuccess) return dspb::hip_fail(e_, #x);         \
    } while (0)

namespace {

int with_device(int device, int *prev) {
    MOD_HIP(hipGetDevice(prev));
    if (device >= 0 && device != *prev) MOD_HIP(hipSetDevice(device));
    return DSP_OK;
}

int launch1(hipFunction_t f, void **args, hipStream_t s = nullptr) {
    MOD_HIP(hipModuleLaunchKernel(f, 1, 1, 1, 1, 1, 1, 0, s, args, nullptr));
    return DSP_OK;
}

int make_arena(dsp_module *m, int slot, uint64_t bytes) {
    if (m->arena_mem[slot]) (void)hipFree(m->arena_mem[slot]);
    m->arena_mem[slot] = nullptr;
    if (!m->d_arena[slot]) MOD_HIP(hipMalloc(&m->d_arena[slot], sizeof(ArenaHost)));
    if (bytes) MOD_HIP(hipMalloc(&m->arena_mem[slot], bytes));
    if (bytes) MOD_HIP(hipMemset(m->arena_mem[slot], 0, bytes));
    ArenaHost h{m->arena_mem[slot], bytes, 0, nullptr, 0};
    MOD_HIP(hipMemcpy(m->d_arena[slot], &h, sizeof h, hipMemcpyHostToDevice));
    return DSP_OK;
}

// host-side writers of the device Parameters / State wait for the renders
// that use them
int wait_uses(dsp_module *m) {
    if (m->use_ev) MOD_HIP(hipEventSynchronize(m->use_ev));
    return DSP_OK;
}

int init_slot(dsp_module *m, int slot, const void *params, uint32_t C, float sr, uint64_t arena_bytes,
              hipStream_t s) {
    if (int st = wait_uses(m)) return st;
    if (!params && m->params_size > 0) {
        set_last_error("initialize_state: params blob is NULL");
        return DSP_ERR_INVALID;
    }
    int st = make_arena(m, slot, arena_bytes);
    if (st) return st;
    MOD_HIP(hipMemcpy(m->d_params, params, m->params_size, hipMemcpyHostToDevice));
    void *a_p = m->d_params, *a_s = m->d_state[slot], *a_a = m->d_arena[slot];
    unsigned a_c = C;
    float a_sr = sr;
    void *args[] = {&a_p, &a_s, &a_c, &a_sr, &a_a};
    if ((st = launch1(m->f_init, args, s))) return st;
    ArenaHost h{};
    MOD_HIP(hipMemcpyAsync(&h, m->d_arena[slot], sizeof h, hipMemcpyDeviceToHost, s));
    MOD_HIP(hipStreamSynchronize(s));
    if (h.failed) {  // an allocator returned NULL: Runtime_Low_Memory (errors.inc:22-23)
        set_last_error("initialize_state: arena of %llu bytes exhausted (%llu used, a request of %llu failed)",
                       (unsigned long long)h.capacity, (unsigned long long)h.used,
                       (unsigned long long)h.failed);
        return DSP_ERR_NOMEM;
    }
    return DSP_OK;
}

}  // namespace

namespace {

// The plugin source inside the device-service header and a
// force_cuda_host_device region: the head of both translation units (the
// module's and the analysis kernel's).
std::string plugin_prelude() {
    std::string tu;
    tu += "#include \"plugin_header.h\"\n";
    tu += "#pragma clang force_cuda_host_device begin\n";
    // the parameter annotations are read from the source text (descriptor.cpp);
    // compiled, each access to an annotated field would go through
    // llvm.ptr.annotation, an opaque pointer that keeps the field in memory
    // (a reload after every LDS store of the callback): drop the attribute
    tu += "#define annotate(...)\n#define __annotate__(...)\n";
    tu += "#include \"dspb_plugin_source.cpp\"\n";
    tu += "#undef annotate\n#undef __annotate__\n";
    tu += "#pragma clang force_cuda_host_device end\n";
    return tu;
}

// The callback's facts (ir_proof.hpp): the plugin compiled again, as a
// flattened analysis kernel, at -O2 without vectorisation or unrolling (the
// same IEEE semantics as the module's -O3 code; scalar IR is what the
// analysis reads), with the module compile's language options.
dspb::irp::Facts analyze_source(const char *source, bool shipped = false) {
    static const char *kProof =
        "extern \"C\" __global__ __attribute__((flatten)) void dspb_proof(Parameters *P, State *S, float **out, "
        "unsigned C, unsigned B, float sr) { audio_callback(*P, *S, out, C, B, sr); }\n";
    dspb::irp::Facts f;
    std::string ir, log;
    const int rc = dspb::irp::compile_to_ir(plugin_prelude() + kProof,
                                            {{"plugin_header.h", kPluginDeviceSrc}, {"dspb_plugin_source.cpp", source}},
                                            shipped ? std::vector<std::string>{"-O3", "-std=c++20", "-ffp-contract=off", "-w"}
                                                    : std::vector<std::string>{"-O2", "-std=c++20", "-ffp-contract=off", "-w",
                                                                               "-fno-vectorize", "-fno-slp-vectorize",
                                                                               "-fno-unroll-loops"},
                                            &ir, &log);
    if (rc != 0) {
        f.why = "the analysis compile failed: " + log.substr(0, 300);
        return f;
    }
    if (const char *dump = std::getenv("DSPB_PROOF_IR")) {  // diagnostics: the IR the analysis reads
        if (FILE *fp = std::fopen(dump, "w")) {
            std::fwrite(ir.data(), 1, ir.size(), fp);
            std::fclose(fp);
        }
    }
    return dspb::irp::analyze(ir, "dspb_proof");
}

}  // namespace

extern "C" {

int dsp_module_compile(const char *source, const char *name, void **code, uint64_t *code_size, char *log,
                       uint64_t log_cap) {
    if (log && log_cap) log[0] = 0;
    if (!source || !code || !code_size) {
        set_last_error("dsp_module_compile: NULL argument");
        return DSP_ERR_INVALID;
    }
    *code = nullptr;
    *code_size = 0;
    std::string tu = plugin_prelude();
    std::string note;
    tu += dspb::desc::generate(source, kPluginDeviceSrc, &note);
    // what the callback does with its block, from its own IR (ir_proof.cpp),
    // stored in the code object for dsp_module_load
    const dspb::irp::Facts facts = analyze_source(source);
    tu += "extern \"C\" __attribute__((used, visibility(\"default\"))) __device__ const unsigned char "
          "dspb_callback_facts[] = {" + dspb::desc::hex_literal(dspb::irp::encode(facts)) + "};\n";
    tu += kDriver;
    // the segment kernels only where they can run: a callback the analysis
    // bounded that writes its State (the loader treats them as optional)
    if (facts.analyzed && facts.writes_state) {
        // a split State: the words a block-dependent store may hit (kSegDriver
        // dspb_state_dep_words; the State chain of the others)
        if (facts.state_split && !facts.state_dep_words.empty()) {
            tu += "#define DSPB_STATE_DEP_WORDS ";
            for (size_t i = 0; i < facts.state_dep_words.size(); ++i)
                tu += (i ? "," : "") + std::to_string(facts.state_dep_words[i]);
            tu += "\n";
        }
        // diagnostics: pass 1's phase clocks (dsp_module_seg_timing)
        if (std::getenv("DSPB_SEG_TIMING")) tu += "#define DSPB_SEG_TIMING 1\n";
        tu += kSegDriver;
    }
    const std::string round = "-DDSPB_LDS_ROUND_BYTES=" + std::to_string(kLdsRoundBytes) + "u";
    // State chain kernels from the callback's IR with its block stores
    // deleted (ir_proof.cpp strip_chain_block_stores), so that they keep only
    // the State's arithmetic: every chain kernel when no State value depends
    // on the block (a tremolo's phase, not its output), the chain of a split
    // State's block-independent words (dspb_seg_chain_ind_*) when the State
    // splits.  Compiled through comgr from the same translation unit into a
    // code object of their own, carried inside the module's as the symbol
    // dspb_chain_co (dsp_module_load takes the chain kernels from it); every
    // other kernel is the hiprtc compile below.  Nothing is carried if any
    // step fails: the hiprtc chain kernels stand.
    if (facts.analyzed && facts.writes_state && (!facts.state_reads_block || facts.state_split)) {
        std::string ir, clog, co;
        int dropped = 0;
        const char *prefix = facts.state_reads_block ? "@dspb_seg_chain_ind_" : "@dspb_seg_chain_";
        if (dspb::irp::compile_to_ir(tu, {{"plugin_header.h", kPluginDeviceSrc}, {"dspb_plugin_source.cpp", source}},
                                     {"-O3", "-std=c++20", "-ffp-contract=off", "-w", "-fno-discard-value-names",
                                      round},
                                     &ir, &clog) == 0 &&
            (dropped = dspb::irp::strip_chain_block_stores(&ir, prefix)) > 0 &&
            dspb::irp::codegen_ir(ir, {"-O3", "-ffp-contract=off"}, &co, &clog) == 0) {
            tu += "extern \"C\" __attribute__((used, visibility(\"default\"))) __device__ const unsigned char "
                  "dspb_chain_co[] = {" + dspb::desc::hex_literal(co) + "};\n";
        } else if (dropped < 0) {
            note += "State chain: a store outside the block-store model, compiled from source\n";
        } else if (dropped == 0 && clog.empty()) {
            note += "State chain: no block store to drop\n";
        } else {
            note += "State chain compiled from source: " + clog.substr(0, 200) + "\n";
        }
    }
    std::vector<const char *> hdrs = {kPluginDeviceSrc, source}, hnames = {"plugin_header.h", "dspb_plugin_source.cpp"};
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, tu.c_str(), name ? name : "plugin.cpp", (int)hdrs.size(), hdrs.data(),
                            hnames.data()) != HIPRTC_SUCCESS) {
        set_last_error("hiprtcCreateProgram failed");
        return DSP_ERR_INVALID;
    }
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++20", "-ffp-contract=off", "-w", round.c_str()};
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof opts / sizeof *opts), opts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::vector<char> lg(ls + 1, 0);
    if (ls) hiprtcGetProgramLog(prog, lg.data());
    if (log && log_cap) {
        std::strncpy(log, lg.data(), log_cap - 1);
        log[log_cap - 1] = 0;
    }
    if (rc != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        set_last_error("plugin compile failed: %.400s", lg.data());
        return DSP_ERR_INVALID;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    void *buf = std::malloc(cs ? cs : 1);
    if (!buf) {
        hiprtcDestroyProgram(&prog);
        return DSP_ERR_NOMEM;
    }
    hiprtcGetCode(prog, (char *)buf);
    hiprtcDestroyProgram(&prog);
    // the parameter descriptor, validated as the reference's JIT does
    // (compiler.cpp:944-1164): an invalid annotation fails the compile
    dspb::desc::Descriptor d;
    std::string derr;
    if (dspb::desc::read(buf, cs, &d, &derr) != 0) note += "descriptor: " + derr + "\n";
    std::string bad;
    for (const auto &p : d.params)
        if (p.error != dspb::desc::kSuccess)
            bad += "parameter '" + p.name + "' (annotate \"" + p.annotation + "\"): " +
                   dspb::desc::error_name(p.error) + "\n";
    if (log && log_cap) {
        const std::string all = std::string(lg.data()) + note + bad;
        std::strncpy(log, all.c_str(), log_cap - 1);
        log[log_cap - 1] = 0;
    }
    if (!bad.empty()) {
        std::free(buf);
        set_last_error("plugin descriptor: %.400s", bad.c_str());
        return DSP_ERR_INVALID;
    }
    *code = buf;
    *code_size = cs;
    return DSP_OK;
}

void dsp_module_free_code(void *code) { std::free(code); }

int dsp_module_load(const void *code, uint64_t code_size, int device, dsp_module **out) {
    if (!code || !code_size || !out) {
        set_last_error("dsp_module_load: NULL argument");
        return DSP_ERR_INVALID;
    }
    *out = nullptr;
    int prev = -1;
    int st = with_device(device, &prev);
    if (st) return st;
    dsp_module *m = new dsp_module();
    (void)hipGetDevice(&m->device);
    if (hipDeviceGetAttribute(&m->cus, hipDeviceAttributeMultiprocessorCount, m->device) != hipSuccess || m->cus < 1)
        m->cus = 256;
    {
        dsp_descriptor *dd = new dsp_descriptor();
        if (dspb::desc::read(code, code_size, &dd->d, nullptr) == 0) m->desc = dd;
        else delete dd;
    }
    auto fail = [&](int s) {
        dsp_module_destroy(m);
        if (prev >= 0) (void)hipSetDevice(prev);
        return s;
    };
    hipError_t e = hipModuleLoadData(&m->mod, code);
    if (e != hipSuccess) return fail(dspb::hip_fail(e, "hipModuleLoadData"));
    struct { hipFunction_t *f; const char *n; } fs[] = {{&m->f_sizes, "dspb_sizes"}, {&m->f_defaults, "dspb_defaults"},
                                                        {&m->f_init, "dspb_init"}, {&m->f_render, "dspb_render"},
                                                        {&m->f_callback, "dspb_callback"}};
    for (auto &f : fs)
        if ((e = hipModuleGetFunction(f.f, m->mod, f.n)) != hipSuccess) return fail(dspb::hip_fail(e, f.n));
    for (int i = 0; i < 7; ++i) {
        if (hipModuleGetFunction(&m->f_render_lds[i], m->mod, kLdsShapes[i].name) != hipSuccess) {
            (void)hipGetLastError();
            m->f_render_lds[i] = nullptr;
        }
    }
    auto optional = [&](hipFunction_t *f, const char *name) {
        if (hipModuleGetFunction(f, m->mod, name) != hipSuccess) {
            (void)hipGetLastError();
            *f = nullptr;
        }
    };
    for (int i = 0; i < 4; ++i) optional(&m->f_render_st[i], kStShapes[i].name);
    for (int i = 0; i < 5; ++i) {
        optional(&m->f_seg[i], kSegShapes[i].name);
        if (kSegShapes[i].rerun) optional(&m->f_seg_rerun[i], kSegShapes[i].rerun);
    }
    for (int i = 0; i < 2; ++i) optional(&m->f_seg_walk[i], kWalkShapes[i].name);
    optional(&m->f_seg_check, "dspb_seg_check");
    for (int i = 0; i < 4; ++i) {
        optional(&m->f_seg_chain[i], kChainShapes[i].name);
        if (m->f_seg_chain[i] &&
            hipFuncGetAttribute(&m->chain_priv[i], HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, m->f_seg_chain[i]) !=
                hipSuccess) {
            (void)hipGetLastError();
            m->f_seg_chain[i] = nullptr;
        }
        optional(&m->f_seg_chain_ind[i], kChainIndShapes[i].name);
        if (m->f_seg_chain_ind[i] &&
            hipFuncGetAttribute(&m->chain_ind_priv[i], HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, m->f_seg_chain_ind[i]) !=
                hipSuccess) {
            (void)hipGetLastError();
            m->f_seg_chain_ind[i] = nullptr;
        }
    }
    {
        // the State chain kernels compiled from the callback's edited IR
        // (dsp_module_compile: the symbol dspb_chain_co), a code object of
        // their own; the module's facts say which of them it holds
        std::string cco, ft;
        dspb::irp::Facts cf;
        if (dspb::desc::code_symbol(code, code_size, "dspb_chain_co", &cco) && !cco.empty() &&
            dspb::desc::code_symbol(code, code_size, "dspb_callback_facts", &ft)) {
            while (!ft.empty() && ft.back() == '\0') ft.pop_back();
            if (dspb::irp::decode(ft, &cf) && hipModuleLoadData(&m->chain_mod, cco.data()) == hipSuccess) {
                auto from_chain = [&](hipFunction_t *f, int *priv, const char *name) {
                    hipFunction_t g = nullptr;
                    if (hipModuleGetFunction(&g, m->chain_mod, name) != hipSuccess ||
                        hipFuncGetAttribute(priv, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, g) != hipSuccess) {
                        (void)hipGetLastError();
                        *f = nullptr;  // (the edited chain is all or nothing)
                        return;
                    }
                    *f = g;
                };
                for (int i = 0; i < 4; ++i) {
                    if (!cf.state_reads_block) from_chain(&m->f_seg_chain[i], &m->chain_priv[i], kChainShapes[i].name);
                    from_chain(&m->f_seg_chain_ind[i], &m->chain_ind_priv[i], kChainIndShapes[i].name);
                }
            } else {
                (void)hipGetLastError();
                m->chain_mod = nullptr;
            }
        }
    }
    unsigned *d_o = nullptr;
    if ((e = hipMalloc(&d_o, 4 * sizeof(unsigned))) != hipSuccess) return fail(dspb::hip_fail(e, "hipMalloc"));
    void *args[] = {&d_o};
    st = launch1(m->f_sizes, args);
    unsigned h[4] = {0, 0, 0, 0};
    if (!st && (e = hipMemcpy(h, d_o, sizeof h, hipMemcpyDeviceToHost)) != hipSuccess) st = dspb::hip_fail(e, "sizes");
    (void)hipFree(d_o);
    if (st) return fail(st);
    m->params_size = h[0];
    m->state_size = h[1];
    m->stateless = (int)h[2];
    {
        std::string ft;
        if (dspb::desc::code_symbol(code, code_size, "dspb_callback_facts", &ft)) {
            while (!ft.empty() && ft.back() == '\0') ft.pop_back();
            m->has_facts = dspb::irp::decode(ft, &m->facts);
        }
        m->par = (m->has_facts && m->facts.analyzed && !m->facts.writes_state) ? 1 : 0;
    }
    if ((e = hipMalloc(&m->d_params, m->params_size ? m->params_size : 1)) != hipSuccess ||
        (e = hipMalloc(&m->d_state[0], m->state_size ? m->state_size : 1)) != hipSuccess ||
        (e = hipMalloc(&m->d_state[1], m->state_size ? m->state_size : 1)) != hipSuccess)
        return fail(dspb::hip_fail(e, "hipMalloc"));
    (void)hipMemset(m->d_state[0], 0, m->state_size ? m->state_size : 1);
    (void)hipMemset(m->d_state[1], 0, m->state_size ? m->state_size : 1);
    if (prev >= 0 && prev != m->device) (void)hipSetDevice(prev);
    *out = m;
    return DSP_OK;
}

void dsp_module_destroy(dsp_module *m) {
    if (!m) return;
    int prev = -1;
    if (with_device(m->device, &prev) == DSP_OK) {
        for (int i = 0; i < 2; ++i) {
            if (m->d_state[i]) (void)hipFree(m->d_state[i]);
            if (m->d_arena[i]) (void)hipFree(m->d_arena[i]);
            if (m->arena_mem[i]) (void)hipFree(m->arena_mem[i]);
        }
        if (m->d_params) (void)hipFree(m->d_params);
        (void)hipDeviceSynchronize();  // no launch may still read a table
        for (auto &e : m->spec)
            if (e.use) m->retired.push_back(e.use);
        for (auto &u : m->retired) {
            (void)hipFree(u->table);
            for (auto &kv : u->ev) (void)hipEventDestroy(kv.second);
        }
        for (hipEvent_t e : {m->upload_ev, m->use_ev, m->seg.ev[0], m->seg.ev[1]})
            if (e) {
                (void)hipEventSynchronize(e);
                (void)hipEventDestroy(e);
            }
        if (m->h_params) (void)hipHostFree(m->h_params);
        if (m->seg.h_stats) (void)hipHostFree(m->seg.h_stats);
        for (void *p : {m->seg.blk, m->seg.ind, m->seg.end, (void *)m->seg.list, (void *)m->seg.flags,
                        (void *)m->seg.words})
            if (p) (void)hipFree(p);
        if (m->mod) (void)hipModuleUnload(m->mod);
        if (m->chain_mod) (void)hipModuleUnload(m->chain_mod);
        if (prev >= 0 && prev != m->device) (void)hipSetDevice(prev);
    }
    delete m->desc;
    delete m;
}

int dsp_module_block_class(dsp_module *m, const void *params, uint32_t params_size, uint32_t C, uint32_t B,
                           float sr, int32_t *block_class, float *gain, const dsp_exec *ex) {
    if (!m || !block_class) {
        set_last_error("dsp_module_block_class: NULL argument");
        return DSP_ERR_INVALID;
    }
    int prev = -1;
    if (int st = with_device(ex && ex->device >= 0 ? ex->device : m->device, &prev)) return st;
    dspb::ModuleSpec r;
    const int st = dspb::module_specialize(m, params, params_size, C, B, sr, ex ? (hipStream_t)ex->stream : nullptr, &r);
    if (!st && r.use) (void)dspb::module_spec_done(m, r.use, ex ? (hipStream_t)ex->stream : nullptr);  // no launch
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && prev >= 0 && prev != cur) (void)hipSetDevice(prev);
    if (st) return st;
    *block_class = r.kind == dspb::kSpecTable ? DSP_BLOCK_TABLE
                   : r.kind == dspb::kSpecGain ? DSP_BLOCK_GAIN
                   : r.kind == dspb::kSpecGainTable ? DSP_BLOCK_GAIN_TABLE
                                                   : DSP_BLOCK_CALLBACK;
    if (gain) *gain = r.gain;
    return DSP_OK;
}

int dsp_module_retired_tables(dsp_module *m, uint64_t *n) {
    if (!m || !n) return DSP_ERR_INVALID;
    *n = dspb::module_spec_retired(m);
    return DSP_OK;
}

int dsp_module_state_spec(dsp_module *m, dsp_state_spec_info *out) {
    if (!m || !out) {
        set_last_error("dsp_module_state_spec: NULL argument");
        return DSP_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    if (int st = dspb::module_seg_collect(m, true)) return st;
    *out = m->seg.serial ? dsp_state_spec_info{} : m->seg.last;
    out->disabled = (m->seg.off || m->seg.chain_bad) ? 1 : 0;
    return DSP_OK;
}

int dsp_ir_strip_chain_stores(const char *ir, char *out, uint64_t out_cap, int32_t *dropped) {
    if (!ir || !dropped) {
        set_last_error("dsp_ir_strip_chain_stores: NULL argument");
        return DSP_ERR_INVALID;
    }
    std::string t(ir);
    *dropped = dspb::irp::strip_chain_block_stores(&t);
    if (out && out_cap) {
        if (t.size() + 1 > out_cap) {
            set_last_error("dsp_ir_strip_chain_stores: %llu bytes needed", (unsigned long long)t.size() + 1);
            return DSP_ERR_INVALID;
        }
        std::memcpy(out, t.c_str(), t.size() + 1);
    }
    return DSP_OK;
}

int dsp_module_debug(dsp_module *m, int what, uint64_t value) {
    if (!m || what != DSP_MODULE_DEBUG_PERTURB_CHAIN || value == ~0ull) {
        set_last_error("dsp_module_debug: unknown hook");
        return DSP_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    m->seg.perturb = value + 1;
    return DSP_OK;
}

int dsp_module_seg_timing(dsp_module *m, uint32_t out[8]) {
    if (!m || !out) return DSP_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    std::memset(out, 0, 8 * sizeof(uint32_t));
    if (!m->seg.words) return DSP_OK;
    MOD_HIP(hipDeviceSynchronize());
    MOD_HIP(hipMemcpy(out, m->seg.words + 24, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return DSP_OK;
}

int dsp_module_sizes(const dsp_module *m, uint32_t *params_size, uint32_t *state_size, int *stateless) {
    if (!m) return DSP_ERR_INVALID;
    if (params_size) *params_size = m->params_size;
    if (state_size) *state_size = m->state_size;
    if (stateless) *stateless = m->par;
    return DSP_OK;
}

int dsp_module_default_parameters(dsp_module *m, void *params) {
    if (!m || (!params && m->params_size)) return DSP_ERR_INVALID;
    std::lock_guard<std::mutex> lk(m->mu);
    if (int st = wait_uses(m)) return st;
    int prev = -1;
    int st = with_device(m->device, &prev);
    if (st) return st;
    void *a_p = m->d_params;
    void *args[] = {&a_p};
    if ((st = launch1(m->f_defaults, args))) return st;
    MOD_HIP(hipMemcpy(params, m->d_params, m->params_size, hipMemcpyDeviceToHost));
    if (prev >= 0 && prev != m->device) (void)hipSetDevice(prev);
    return DSP_OK;
}

int dsp_module_initialize_state(dsp_module *m, const void *params, uint32_t C, float sr, uint64_t arena_bytes) {
    if (!m) return DSP_ERR_INVALID;
    if (C == 0 || C > (uint32_t)dspb::kMaxChannels) {
        set_last_error("channels must be 1..%d", dspb::kMaxChannels);
        return DSP_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    int prev = -1;
    int st = with_device(m->device, &prev);
    if (st) return st;
    st = init_slot(m, 0, params, C, sr, arena_bytes, nullptr);
    m->initialized = (st == DSP_OK);
    // block classes were found with the previous State: forget them (their
    // tables are freed once no call holds them, dspb::spec_reap)
    for (auto &e : m->spec)
        if (e.use) m->retired.push_back(e.use);
    m->spec.clear();
    dspb::spec_reap(m);
    if (prev >= 0 && prev != m->device) (void)hipSetDevice(prev);
    return st;
}

// ---- parameter descriptor (module.h) ----------------------------------------
int dsp_descriptor_from_code(const void *code, uint64_t code_size, dsp_descriptor **out) {
    if (!code || !code_size || !out) {
        set_last_error("dsp_descriptor_from_code: NULL argument");
        return DSP_ERR_INVALID;
    }
    *out = nullptr;
    dsp_descriptor *d = new dsp_descriptor();
    std::string err;
    if (dspb::desc::read(code, code_size, &d->d, &err) != 0) {
        delete d;
        set_last_error("%s", err.c_str());
        return DSP_ERR_INVALID;
    }
    *out = d;
    return DSP_OK;
}

void dsp_descriptor_destroy(dsp_descriptor *d) { delete d; }

const dsp_descriptor *dsp_module_descriptor(const dsp_module *m) { return m ? m->desc : nullptr; }

int dsp_descriptor_info(const dsp_descriptor *d, dsp_plugin_descriptor *out) {
    if (!d || !out) return DSP_ERR_INVALID;
    out->params_size = d->d.params_size;
    out->params_align = d->d.params_align;
    out->state_size = d->d.state_size;
    out->state_align = d->d.state_align;
    out->num_parameters = (uint32_t)d->d.params.size();
    out->error = d->d.error;
    return DSP_OK;
}

int dsp_descriptor_param(const dsp_descriptor *d, uint32_t i, dsp_param_desc *out) {
    if (!d || !out || i >= d->d.params.size()) return DSP_ERR_INVALID;
    const dspb::desc::Param &p = d->d.params[i];
    std::memset(out, 0, sizeof *out);
    std::strncpy(out->name, p.name.c_str(), DSP_PARAM_NAME_MAX - 1);
    out->offset = p.offset;
    out->type = p.type;
    out->error = p.error;
    out->int_min = p.int_min;
    out->int_max = p.int_max;
    out->float_min = p.float_min;
    out->float_max = p.float_max;
    out->float_log = p.float_log ? 1 : 0;
    out->num_entries = (uint32_t)p.entries.size();
    return DSP_OK;
}

int dsp_descriptor_enum_entry(const dsp_descriptor *d, uint32_t i, uint32_t e, int64_t *value, char *name,
                              uint32_t name_cap) {
    if (!d || i >= d->d.params.size() || e >= d->d.params[i].entries.size()) return DSP_ERR_INVALID;
    const dspb::desc::Entry &en = d->d.params[i].entries[e];
    if (value) *value = en.value;
    if (name && name_cap) {
        std::strncpy(name, en.name.c_str(), name_cap - 1);
        name[name_cap - 1] = 0;
    }
    return DSP_OK;
}

int dsp_params_from_values(const dsp_descriptor *d, const dsp_param_value *values, void *holder) {
    if (!d || (!d->d.params.empty() && (!values || !holder))) return DSP_ERR_INVALID;
    char *h = (char *)holder;
    for (size_t i = 0; i < d->d.params.size(); ++i) {
        const dspb::desc::Param &p = d->d.params[i];
        if (p.offset + 4ull > d->d.params_size) return DSP_ERR_INVALID;
        switch (p.type) {  // plugin.cpp:155-168: every kind is a 4-byte store
        case dspb::desc::kInt: std::memcpy(h + p.offset, &values[i].int_value, 4); break;
        case dspb::desc::kFloat: std::memcpy(h + p.offset, &values[i].float_value, 4); break;
        default: std::memcpy(h + p.offset, &values[i].enum_value, 4); break;
        }
    }
    return DSP_OK;
}

int dsp_params_to_values(const dsp_descriptor *d, const void *holder, dsp_param_value *values) {
    if (!d || (!d->d.params.empty() && (!values || !holder))) return DSP_ERR_INVALID;
    const char *h = (const char *)holder;
    for (size_t i = 0; i < d->d.params.size(); ++i) {
        const dspb::desc::Param &p = d->d.params[i];
        if (p.offset + 4ull > d->d.params_size) return DSP_ERR_INVALID;
        std::memcpy(&values[i], h + p.offset, 4);  // plugin.cpp:129-142
    }
    return DSP_OK;
}

int dsp_descriptor_equal(const dsp_descriptor *a, const dsp_descriptor *b) {
    if (!a || !b) return 0;
    const dspb::desc::Descriptor &x = a->d, &y = b->d;
    if (x.params_size != y.params_size || x.params_align != y.params_align || x.state_size != y.state_size ||
        x.state_align != y.state_align || x.params.size() != y.params.size())
        return 0;
    for (size_t i = 0; i < x.params.size(); ++i) {
        const dspb::desc::Param &p = x.params[i], &q = y.params[i];
        // (the reference compares a's name with itself, plugin.cpp:74; the
        // names are compared here)
        if (p.offset != q.offset || p.type != q.type || p.name != q.name) return 0;
        if (p.type == dspb::desc::kInt && (p.int_min != q.int_min || p.int_max != q.int_max)) return 0;
        if (p.type == dspb::desc::kFloat && (p.float_min != q.float_min || p.float_max != q.float_max)) return 0;
        if (p.type == dspb::desc::kEnum) {
            if (p.entries.size() != q.entries.size()) return 0;
            for (size_t e = 0; e < p.entries.size(); ++e)
                if (p.entries[e].value != q.entries[e].value || p.entries[e].name != q.entries[e].name) return 0;
        }
    }
    return 1;
}

// plugin.h:173-233, in fp32 as the reference computes them (real32
// arguments: the float overloads of log / exp)
int dsp_param_normalize(const dsp_param_desc *p, const int64_t *enum_values, dsp_param_value v, float *out) {
    if (!p || !out) return DSP_ERR_INVALID;
    switch (p->type) {
    case DSP_PARAM_INT:  // normalize_parameter_int_value
        *out = (float)((float)v.int_value - (float)p->int_min) / (float)(p->int_max - p->int_min);
        return DSP_OK;
    case DSP_PARAM_FLOAT: {  // normalize_parameter_float_value
        float x = v.float_value;
        x = x < p->float_min ? p->float_min : (x > p->float_max ? p->float_max : x);
        if (x == p->float_min) *out = 0.0f;
        else if (p->float_log) *out = std::log(x / p->float_min) / std::log(p->float_max / p->float_min);
        else *out = (x - p->float_min) / (p->float_max - p->float_min);
        return DSP_OK;
    }
    case DSP_PARAM_ENUM: {  // enum_value_to_index + normalize_parameter_enum_index
        if (!enum_values || p->num_entries == 0) return DSP_ERR_INVALID;
        uint32_t idx = 0;
        for (; idx < p->num_entries && enum_values[idx] != (int64_t)v.enum_value; ++idx) {
        }
        if (idx == p->num_entries) return DSP_ERR_INVALID;
        *out = p->num_entries == 1 ? 0.0f : (float)idx / (float)(p->num_entries - 1);
        return DSP_OK;
    }
    default: return DSP_ERR_INVALID;
    }
}

int dsp_param_denormalize(const dsp_param_desc *p, const int64_t *enum_values, float x, dsp_param_value *out) {
    if (!p || !out) return DSP_ERR_INVALID;
    switch (p->type) {
    case DSP_PARAM_INT:  // denormalize_int_value
        out->int_value = (int32_t)(x * (float)(p->int_max - p->int_min) + (float)p->int_min);
        return DSP_OK;
    case DSP_PARAM_FLOAT:  // denormalize_float_value
        out->float_value = p->float_log ? p->float_min * std::exp(x * std::log(p->float_max / p->float_min))
                                        : x * (p->float_max - p->float_min) + p->float_min;
        return DSP_OK;
    case DSP_PARAM_ENUM: {  // denormalize_enum_index + enum_index_to_value
        if (!enum_values || p->num_entries == 0) return DSP_ERR_INVALID;
        const uint32_t idx = (uint32_t)(x * (float)(p->num_entries - 1));
        if (idx >= p->num_entries) return DSP_ERR_INVALID;
        out->enum_value = (int32_t)enum_values[idx];
        return DSP_OK;
    }
    default: return DSP_ERR_INVALID;
    }
}

static void facts_out(const dspb::irp::Facts &f, bool present, dsp_callback_facts *o) {
    std::memset(o, 0, sizeof *o);
    o->present = present ? 1 : 0;
    o->analyzed = f.analyzed;
    o->reads_block = f.reads_block;
    o->writes_state = f.writes_state;
    o->input_control = f.input_control;
    o->gain_form = f.gain_form;
    std::strncpy(o->gain, f.gain_expr.c_str(), sizeof o->gain - 1);
    o->gain_source = f.gain_src;
    o->gain_offset = f.gain_off;
    std::memcpy(&o->gain_constant, &f.gain_bits, 4);
    std::strncpy(o->why, f.why.c_str(), sizeof o->why - 1);
    o->gain_table_form = f.gain_table_form;
    std::strncpy(o->table_why, f.table_why.c_str(), sizeof o->table_why - 1);
    o->state_reads_block = f.state_reads_block;
    o->state_split = f.state_split;
    std::string dw;
    for (int64_t w : f.state_dep_words)
        dw += (dw.empty() ? "" : ",") + (w >= 0 ? std::to_string(w) : std::to_string(-w - 2) + "-");
    std::strncpy(o->state_dep_words, dw.c_str(), sizeof o->state_dep_words - 1);
}

int dsp_module_facts(const dsp_module *m, dsp_callback_facts *out) {
    if (!m || !out) return DSP_ERR_INVALID;
    facts_out(m->facts, m->has_facts, out);
    return DSP_OK;
}

int dsp_code_facts(const void *code, uint64_t code_size, dsp_callback_facts *out) {
    if (!code || !out) return DSP_ERR_INVALID;
    dspb::irp::Facts f;
    std::string ft;
    bool present = false;
    if (dspb::desc::code_symbol(code, code_size, "dspb_callback_facts", &ft)) {
        while (!ft.empty() && ft.back() == '\0') ft.pop_back();
        present = dspb::irp::decode(ft, &f);
    }
    facts_out(f, present, out);
    return DSP_OK;
}

int dsp_plugin_analyze(const char *source, dsp_callback_facts *out) {
    if (!source || !out) {
        set_last_error("dsp_plugin_analyze: NULL argument");
        return DSP_ERR_INVALID;
    }
    facts_out(analyze_source(source), true, out);
    return DSP_OK;
}

int dsp_plugin_analyze_shipped(const char *source, dsp_callback_facts *out) {
    if (!source || !out) {
        set_last_error("dsp_plugin_analyze_shipped: NULL argument");
        return DSP_ERR_INVALID;
    }
    facts_out(analyze_source(source, true), true, out);
    return DSP_OK;
}

int dsp_module_read_state(const dsp_module *m, void *state) {
    if (!m || (!state && m->state_size)) return DSP_ERR_INVALID;
    if (int st = wait_uses(const_cast<dsp_module *>(m))) return st;
    MOD_HIP(hipMemcpy(state, m->d_state[0], m->state_size, hipMemcpyDeviceToHost));
    return DSP_OK;
}

}  // extern "C"

namespace dspb {

// DSPB_STATELESS_PATH=0 / 3 forces the in-place wave path / the LDS-blocks
// path for a stateless plugin (tools/generic_probe.py A/B); -1: by size
static int stateless_path_forced() {
    static const int v = [] {
        const char *e = std::getenv("DSPB_STATELESS_PATH");
        return e && (e[0] == '0' || e[0] == '3') ? e[0] - '0' : -1;
    }();
    return v;
}
// the LDS-blocks path: LDS per workgroup round (two workgroups per CU)


// the caller's Parameters blob -> the module's device Parameters, stream
// ordered: through a pinned staging copy (reused once the previous upload
// from it has completed), behind every earlier render's use of the device
// Parameters on any stream (use_ev), so the call returns without a sync
static int upload_params(dsp_module *m, const void *params, uint32_t n, hipStream_t s) {
    if (!m->upload_ev) {
        MOD_HIP(hipEventCreateWithFlags(&m->upload_ev, hipEventDisableTiming));
        MOD_HIP(hipEventCreateWithFlags(&m->use_ev, hipEventDisableTiming));
        MOD_HIP(hipEventRecord(m->upload_ev, s));
        MOD_HIP(hipEventRecord(m->use_ev, s));
    }
    MOD_HIP(hipStreamWaitEvent(s, m->use_ev, 0));
    if (!n) return DSP_OK;
    if (!m->h_params) MOD_HIP(hipHostMalloc(&m->h_params, n, hipHostMallocDefault));
    MOD_HIP(hipEventSynchronize(m->upload_ev));
    std::memcpy(m->h_params, params, n);
    MOD_HIP(hipMemcpyAsync(m->d_params, m->h_params, n, hipMemcpyHostToDevice, s));
    MOD_HIP(hipEventRecord(m->upload_ev, s));
    return DSP_OK;
}

// A GENERIC render cannot be captured into a graph: its Parameters upload
// waits on the host for the pinned staging buffer and copies from it, so a
// replay would upload whatever a later call left there.  Refused instead.
static int refuse_capture(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
        set_last_error("GENERIC plugin: calls cannot be captured into a graph (the Parameters upload is "
                       "host-staged); call it eagerly");
        return DSP_ERR_INVALID;
    }
    return DSP_OK;
}

// the module's code object, Parameters and State live on m->device: a call
// made on another device (e.g. a mis-wired shard rank) is refused
static int check_device(const dsp_module *m) {
    int dev = -1;
    MOD_HIP(hipGetDevice(&dev));
    if (dev != m->device) {
        set_last_error("GENERIC plugin: module loaded on device %d, called on device %d", m->device, dev);
        return DSP_ERR_INVALID;
    }
    return DSP_OK;
}

// The last speculative render's counters (pinned copy, behind an event):
// into m->seg.last, and what they teach about the current Parameters.  The
// render tried warm-up levels (x16 each, on the GPU) until no more than 1/8
// of the segments it guessed started from a State that was not the true one;
// the level that stood is where the next render with these Parameters
// starts.  When even the last level it could try failed (kSegWarmMax, or a
// warm-up half the file), the chain does not forget: these Parameters render
// serially from now on.  wait = false reads the counters only if they have
// landed (a render never waits for them).
int module_seg_collect(dsp_module *m, bool wait) {
    auto &W = m->seg;
    const int older = W.seq[0] < W.seq[1] ? 0 : 1;  // the older slot first
    for (int pass = 0; pass < 2; ++pass) {
        const int i = pass == 0 ? older : 1 - older;
        if (!W.pending[i]) continue;
        if (wait) MOD_HIP(hipEventSynchronize(W.ev[i]));
        else if (hipEventQuery(W.ev[i]) != hipSuccess) {
            (void)hipGetLastError();
            continue;
        }
        W.pending[i] = false;
        dsp_state_spec_info &r = W.info[i];
        const unsigned *h = W.h_stats + 16 * i;  // [0, 4) levels, [4] [5] reruns, [7] walk, [8, 12) levels run,
                                                 // [12] the State chain ran
        const uint32_t first_warm = r.warmup_blocks;
        const bool spec = r.levels > 0;  // a speculative render (else the learnt State chain alone)
        uint32_t last = 0, warm = first_warm;
        for (uint32_t L = 1; L < r.levels && h[8 + L]; ++L) {
            last = L;
            warm = std::min<uint32_t>(warm * 16, kSegWarmMax);
        }
        if (spec) {
            r.levels = last + 1;
            r.warmup_blocks = warm;
            r.differed[0] = h[last];
            r.differed[1] = h[4];
            r.differed[2] = h[5];
        }
        r.serial_reruns = h[7];
        r.chain = (h[12] || !spec) ? 1 : 0;
        r.chain_mismatch = h[13];
        r.chain_records_differed = h[14];
        // (split: set at launch, kept)
        if (W.seq[i] == W.calls) W.last = r;
        if (W.slot_gen[i] != W.gen) continue;  // rendered with other Parameters: nothing to learn
        // the chain's records failed their check (the walk rendered the call
        // right): these Parameters render serially from now on
        if (r.chain && (r.chain_mismatch || r.chain_records_differed)) W.off = W.chain_bad = true;
        // learn only from renders that started with the warm-up now in force
        if (!spec || first_warm != W.warm || W.off) continue;
        const uint64_t early = std::min<uint64_t>(r.segments - 1, warm / r.blocks_per_segment);
        const uint64_t guessed = r.segments - 1 - early;
        const bool failed = guessed && r.differed[0] * 8ull > guessed;
        if (W.slot_one[i]) {  // launched with the first two levels alone
            if (failed || r.levels > 1) {
                W.one_level = false;  // every level again from the next call
            } else if (r.differed[0] && W.bumps < kSegWarmBumps) {
                // a few segments missed and took a rerun (its rounds cost more
                // than one more warm-up round for all): one block longer
                W.warm += 1;
                ++W.bumps;
            }
            continue;
        }
        if (failed) {
            W.off = true;  // the longest warm-up it could try failed
        } else {
            W.warm = warm;
            W.one_level = r.levels == 1;  // the first level sufficed
        }
    }
    return DSP_OK;
}

// rows [in[c], in[c] + L) and [out[c'], out[c'] + Lr) share an element
static bool module_rows_overlap(const float *const *in, uint32_t in_ch, uint64_t L, const float *const *out,
                                uint32_t C, uint64_t Lr) {
    for (uint32_t a = 0; a < in_ch; ++a)
        for (uint32_t b = 0; b < C; ++b)
            if (in[a] < out[b] + Lr && out[b] < in[a] + L) return true;
    return false;
}

// A State-writing callback over the whole file as speculative segments
// (kDriver dspb_segments); returns 1 (nothing launched) when the shape does
// not fit them -- the caller renders the serial chain.  `chain` (a State
// learned not to forget): the chain kernel records every block's State, and
// the exact rerun renders the segments from them (dspb_seg_chain).
static int module_render_seg(dsp_module *m, RenderArgsG &A, hipStream_t s, bool chain) {
    const uint32_t C = A.C, B = A.B;
    if (2ull * C * B * sizeof(float) > kStagedLdsBytes) return 1;  // the walk's double buffer
    // the chain kernel of this shape, if its compiled form dropped the block
    hipFunction_t fc = nullptr;
    for (int i = 0; i < 4 && !fc; ++i)
        if (m->f_seg_chain[i] && kChainShapes[i].C == C &&
            (kChainShapes[i].B ? kChainShapes[i].B == B : B <= kChainMaxB) &&
            (uint64_t)m->chain_priv[i] <= (uint64_t)m->state_size + 64)
            fc = m->f_seg_chain[i];
    if (chain && !fc) return 1;
    hipFunction_t f = nullptr, fw = nullptr;
    int fi = -1;
    for (int i = 0; i < 5 && !f; ++i) {
        const SegShape &sh = kSegShapes[i];
        if (!m->f_seg[i] || (sh.C && sh.C != C) || (sh.B && sh.B != B) || (sh.pf && B % 4)) continue;
        if (sh.rerun && !m->f_seg_rerun[i]) continue;
        f = m->f_seg[fi = i];
    }
    if (!f) return 1;
    // the pipelined kernels (dspb_segments_pf) stride blocks by C B + 2
    const uint64_t stride = (uint64_t)C * B + (kSegShapes[fi].pf ? 2 : 1);
    // lanes per workgroup (kDriver dspb_seg_nb: the same formula)
    const uint64_t nb = std::min<uint64_t>(64, kLdsRoundBytes / (stride * sizeof(float)));
    if (nb < 4) return 1;
    for (int i = 0; i < 2 && !fw; ++i)
        if (m->f_seg_walk[i] && (!kWalkShapes[i].C || kWalkShapes[i].C == C) &&
            (!kWalkShapes[i].B || kWalkShapes[i].B == B))
            fw = m->f_seg_walk[i];
    if (!fw || !m->f_seg_check) return 1;
    hipFunction_t fr = kSegShapes[fi].rerun ? m->f_seg_rerun[fi] : f;  // the reruns' kernel
    auto &W = m->seg;
    // segments: as many as the chip runs lanes at once (two workgroups per
    // CU, nb lanes each), kSegMinBlocks blocks at least
    const uint64_t lanes = kLdsWgPerCu * (uint64_t)m->cus * nb;
    const uint64_t seg = std::max<uint64_t>((A.nblocks + lanes - 1) / lanes, kSegMinBlocks);
    const uint64_t K = (A.nblocks + seg - 1) / seg;
    // (block indices in 32 bits; one recorded State per block, at most 8 GB of them)
    if (K < 2 || A.nblocks >= (1ull << 32) || A.nblocks * m->state_size > (8ull << 30)) return 1;
    // a split State: the chain of its independent words, when the compiled
    // kernel of the shape dropped the block (no private block: the words
    // need no sample), and the records for it
    hipFunction_t fsplit = nullptr;
    if (!chain && m->facts.state_split)
        for (int i = 0; i < 4 && !fsplit; ++i)
            if (m->f_seg_chain_ind[i] && kChainIndShapes[i].C == C &&
                (kChainIndShapes[i].B ? kChainIndShapes[i].B == B : B <= kChainMaxB) &&
                (uint64_t)m->chain_ind_priv[i] <= (uint64_t)m->state_size + 64)
                fsplit = m->f_seg_chain_ind[i];
    if (fsplit && 4 * K > W.cap_ind) {
        if (int st = wait_uses(m)) return st;
        if (W.ind) (void)hipFree(W.ind);
        W.ind = nullptr;
        W.cap_ind = 0;
        const uint64_t cap = std::max<uint64_t>(4 * K, 4096);
        if (hipMalloc(&W.ind, cap * m->state_size) != hipSuccess) {
            (void)hipGetLastError();
            W.ind = nullptr;
            fsplit = nullptr;  // no room: plain speculation
        } else {
            W.cap_ind = cap;
        }
    }
    if (K > W.cap || A.nblocks > W.cap_blk) {
        if (int st = wait_uses(m)) return st;
        for (void *p : {W.blk, W.end, (void *)W.list, (void *)W.flags}) if (p) (void)hipFree(p);
        W.blk = W.end = nullptr, W.list = nullptr, W.flags = nullptr, W.cap = 0, W.cap_blk = 0;
        const uint32_t cap = (uint32_t)std::max<uint64_t>(K, 1024);
        const uint64_t cap_blk = std::max<uint64_t>(A.nblocks, 4096);
        if (hipMalloc(&W.blk, cap_blk * m->state_size) != hipSuccess ||
            hipMalloc(&W.end, (uint64_t)cap * m->state_size) != hipSuccess ||
            hipMalloc(&W.list, cap * sizeof(unsigned)) != hipSuccess || hipMalloc(&W.flags, cap) != hipSuccess) {
            (void)hipGetLastError();  // no room for the records: the serial chain renders this call
            for (void *p : {W.blk, W.end, (void *)W.list, (void *)W.flags}) if (p) (void)hipFree(p);
            W.blk = W.end = nullptr, W.list = nullptr, W.flags = nullptr;
            return 1;
        }
        W.cap = cap;
        W.cap_blk = cap_blk;
    }
    if (!W.words) {
        MOD_HIP(hipMalloc(&W.words, 32 * sizeof(unsigned)));
        MOD_HIP(hipHostMalloc(&W.h_stats, 32 * sizeof(unsigned), hipHostMallocDefault));
        for (hipEvent_t &e : W.ev) MOD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // the slot this call fills: the one of the render two calls back, whose
    // counters have landed by now in a stream of back-to-back calls
    const int slot = W.seq[0] <= W.seq[1] ? 0 : 1;
    if (W.pending[slot]) {
        MOD_HIP(hipEventSynchronize(W.ev[slot]));
        if (int st = module_seg_collect(m, false)) return st;
    }
    W.slot_one[slot] = false;  // (set below when the levels are cut to the first)
    SegArgsG G{};
    G.R = A;
    G.R.lds_nb = (unsigned)nb;
    G.R.lds_stride = (unsigned)stride;
    G.st_blk = W.blk;
    G.st_end = W.end;
    G.list = W.list;
    G.flags = W.flags;
    G.stats = W.words + 8;  // words: [0] pass 1's listing, [2] / [3] the reruns' listings
    G.seg = seg;
    G.K = (unsigned)K;
    void *args[] = {&G};
    const unsigned lds = (unsigned)(nb * stride * sizeof(float));
    const unsigned gseg = (unsigned)((K + nb - 1) / nb), gchk = (unsigned)((K + 3) / 4);  // 4 segments per 256 threads
    G.perturb = chain || fc || fsplit ? W.perturb : 0;  // (test hook: consumed by the render that may run a chain)
    if (G.perturb) W.perturb = 0;
    MOD_HIP(hipMemsetAsync(W.words, 0, 32 * sizeof(unsigned), s));
    // the State chain's records checked: every boundary against the State the
    // segment before ended with (stats[13]), then the walk renders serially
    // from the true State whatever differs and writes the live State
    auto checked = [&](unsigned exact) -> int {
        G.exact = exact;
        G.mode = 0;
        G.pass = 13;
        G.level = 0xffffffffu;
        MOD_HIP(hipModuleLaunchKernel(m->f_seg_check, gchk, 1, 1, 256, 1, 1, 0, s, args, nullptr));
        MOD_HIP(hipModuleLaunchKernel(fw, 1, 1, 1, 256, 1, 1, (unsigned)(2ull * C * B * sizeof(float)), s, args,
                                      nullptr));
        return DSP_OK;
    };
    uint32_t levels = 0;
    if (chain) {
        G.mode = 1;
        MOD_HIP(hipModuleLaunchKernel(fc, 1, 1, 1, 64, 1, 1, 0, s, args, nullptr));
        G.exact = 1;
        MOD_HIP(hipModuleLaunchKernel(fr, gseg, 1, 1, 256, 1, 1, lds, s, args, nullptr));
        if (int st = checked(1)) return st;
    } else {
        // a split State: its independent words' chain first, pass 1 then
        // starts every warm-up from them (the other words from the live State)
        // the warm-up of each level pass 1 may run: the learnt one, then 16x
        // longer ones while too many segments started wrong (each level
        // decides on the GPU whether it runs: dspb_seg_level_runs)
        uint32_t lw[kSegLevels] = {}, nlev = 0;
        for (uint32_t L = 0, warm = W.warm; L < kSegLevels; ++L) {
            if (L > 0) {
                const uint32_t next = std::min<uint32_t>(warm * 16, kSegWarmMax);
                if (next <= warm || 2ull * next >= A.nblocks) break;  // no longer, or as long as the file
                // with a State chain to fall back on, a level whose rounds (its
                // warm-up and a segment of full callbacks) exceed 1/16 of the
                // file costs more than the chain (the State arithmetic alone over
                // every block) is likely to: not tried
                if (fc && 16ull * (next + seg) > A.nblocks) break;
                warm = next;
            }
            lw[nlev++] = warm;
        }
        // learnt: the first level meets the State (the later ones would only
        // return at once, a launch each of pass 1, its check and the split
        // chain): the first two levels alone -- the second one is there for
        // a render whose input keeps the first from meeting the State (it
        // unlearns this; without it such a render fell to the reruns and the
        // walk's serial chain, 465 segments of a 20 s peak follower)
        if (W.one_level) nlev = std::min<uint32_t>(nlev, 2);
        W.slot_one[slot] = W.one_level;
        if (fsplit) {
            G.st_ind = W.ind;
            G.split = 1;
        }
        uint32_t warm = W.warm, prev = 0;
        G.count = W.words;
        for (uint32_t L = 0; L < nlev; ++L) {
            prev = L ? lw[L - 1] : 0;
            warm = lw[L];
            G.level = L;
            G.warm = warm;
            G.prev_warm = prev;
            // a split State: the chain of its independent words first, recording
            // them where this level's warm-ups start (it runs only where the
            // level does); pass 1 starts from them and the live State's others
            if (fsplit) MOD_HIP(hipModuleLaunchKernel(fsplit, 1, 1, 1, 64, 1, 1, 0, s, args, nullptr));
            G.mode = 0;
            MOD_HIP(hipModuleLaunchKernel(f, gseg, 1, 1, 256, 1, 1, lds, s, args, nullptr));
            G.pass = L;
            G.mode = 1;  // the check lists the differing segments for the rerun
            MOD_HIP(hipModuleLaunchKernel(m->f_seg_check, gchk, 1, 1, 256, 1, 1, 0, s, args, nullptr));
            ++levels;
        }
        // the last level failed (decided on the GPU): the State chain and the
        // exact rerun take over, the reruns and the walk below return at once
        if (fc) {
            G.level = levels;
            G.prev_warm = warm;
            G.mode = 2;
            MOD_HIP(hipModuleLaunchKernel(fc, 1, 1, 1, 64, 1, 1, 0, s, args, nullptr));
        }
        // two reruns of the listed segments, each checked; the last check only flags
        G.level = 0xffffffffu;
        unsigned *listing = W.words;
        for (unsigned p = 0; p < 2; ++p) {
            G.count = listing;
            G.mode = 1;
            MOD_HIP(hipModuleLaunchKernel(fr, gseg, 1, 1, 256, 1, 1, lds, s, args, nullptr));
            G.prev_count = listing;
            listing = W.words + 2 + p;
            G.count = listing;
            G.pass = 4 + p;
            G.mode = p == 0 ? 1 : 0;
            MOD_HIP(hipModuleLaunchKernel(m->f_seg_check, gchk, 1, 1, 256, 1, 1, 0, s, args, nullptr));
        }
        MOD_HIP(hipModuleLaunchKernel(fw, 1, 1, 1, 256, 1, 1, (unsigned)(2ull * C * B * sizeof(float)), s, args,
                                      nullptr));
        if (fc) {  // (each returns at once unless the chain ran)
            G.mode = 1;
            G.exact = 2;
            MOD_HIP(hipModuleLaunchKernel(fr, gseg, 1, 1, 256, 1, 1, lds, s, args, nullptr));
            if (int st = checked(2)) return st;
        }
    }
    MOD_HIP(hipMemcpyAsync(W.h_stats + 16 * slot, W.words + 8, 16 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
    MOD_HIP(hipEventRecord(W.ev[slot], s));
    W.pending[slot] = true;
    W.seq[slot] = ++W.calls;
    W.slot_gen[slot] = W.gen;
    dsp_state_spec_info &r = W.info[slot];
    r = dsp_state_spec_info{};
    r.used = 1;
    r.segments = (uint32_t)K;
    r.blocks_per_segment = (uint32_t)seg;
    r.warmup_blocks = chain ? 0 : W.warm;  // the first level's; module_seg_collect names the one that stood
    r.levels = levels;                     // 0: the learnt State chain alone
    r.chain = chain ? 1 : 0;
    r.split = fsplit ? 1 : 0;
    MOD_HIP(hipEventRecord(m->use_ev, s));
    return DSP_OK;
}

// dsp_render_offline / dsp_render_stft with DSP_PLUGIN_GENERIC (device buffers)
int module_render(dsp_module *m, const void *params, uint32_t params_size, const float *const *in,
                  uint32_t in_ch, uint64_t L, float *const *out, uint32_t C, uint32_t B, float sr,
                  uint64_t goff, hipStream_t s, uint32_t flags) {
    if (!m || !m->initialized) {
        set_last_error("GENERIC plugin: module not loaded / initialize_state not run");
        return DSP_ERR_INVALID;
    }
    if (int st = check_device(m)) return st;
    if (int st = refuse_capture(s)) return st;
    if (params_size != m->params_size || (!params && params_size)) {
        set_last_error("GENERIC plugin: params blob is %u bytes, the plugin's Parameters %u", params_size,
                       m->params_size);
        return DSP_ERR_INVALID;
    }
    if (C > (uint32_t)kMaxChannels || in_ch > (uint32_t)kMaxChannels) {
        set_last_error("GENERIC plugin: at most %d channels", kMaxChannels);
        return DSP_ERR_INVALID;
    }
    if (goff % B) {
        set_last_error("sample_offset must be a multiple of B");
        return DSP_ERR_INVALID;
    }
    const bool par = m->par != 0;
    if (!par && goff) {
        set_last_error("GENERIC plugin with State: whole files only (sample_offset 0)");
        return DSP_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    if (int st = upload_params(m, params, params_size, s)) return st;
    RenderArgsG A{};
    A.P = m->d_params;
    A.S = m->d_state[0];
    for (uint32_t c = 0; c < in_ch; ++c) A.in[c] = const_cast<float *>(in[c]);
    for (uint32_t c = 0; c < C; ++c) A.out[c] = out[c];
    A.L = L;
    A.nblocks = (L + B - 1) / B;
    A.block0 = goff / B;
    A.in_ch = in_ch;
    A.C = C;
    A.B = B;
    A.sr = sr;
    A.par = (unsigned)m->par;
    if (A.nblocks == 0) return DSP_OK;
    void *args[] = {&A};
    unsigned grid = 1, block = 1, lds_bytes = 0;
    if (par) {
        // default: the LDS-blocks path (dspb_render_lds) when a round of at
        // least 4 blocks fits the per-workgroup LDS budget, else the
        // in-place wave path; DSPB_STATELESS_PATH=0/3 forces one
        uint64_t stride = (uint64_t)C * B + 1;
        // the most specific instantiation for (C, B): exact shapes first (the
        // software-pipelined rounds of dspb_stateless_lds_pf, on a persistent
        // grid of two workgroups per CU)
        hipFunction_t f = nullptr;
        bool persistent = false;
        for (int i = 6; i >= 0 && !f; --i)
            if (m->f_render_lds[i] && kLdsShapes[i].C == C && kLdsShapes[i].B == B) {
                f = m->f_render_lds[i];
                persistent = B % 4 == 0;
            }
        for (int i = 6; i >= 0 && !f; --i)
            if (m->f_render_lds[i] && (!kLdsShapes[i].C || kLdsShapes[i].C == C) && !kLdsShapes[i].B)
                f = m->f_render_lds[i];
        // rounds of nb blocks at a block stride of C B + 1 floats, C B + 2 for
        // the pipelined kernels (kDriver dspb_lds_nb: the same formula)
        if (persistent) stride = (uint64_t)C * B + 2;
        const uint64_t nb = std::min<uint64_t>(64, kLdsRoundBytes / (stride * sizeof(float)) / 4 * 4);
        int path = stateless_path_forced();
        if (path < 0) path = nb >= 4 ? 3 : 0;
        if (path == 3 && (nb < 4 || !f)) path = 0;
        if (path == 3) {
            A.lds = 3;
            A.lds_nb = (unsigned)nb;
            A.lds_stride = (unsigned)stride;
            uint64_t g = (A.nblocks + nb - 1) / nb;
            if (persistent) g = std::min<uint64_t>(g, kLdsWgPerCu * m->cus);
            MOD_HIP(hipModuleLaunchKernel(f, (unsigned)(g < (1u << 20) ? g : (1u << 20)), 1, 1, 256, 1, 1,
                                          (unsigned)(nb * stride * sizeof(float)), s, args, nullptr));
            MOD_HIP(hipEventRecord(m->use_ev, s));
            return DSP_OK;
        }
        block = 64;  // one wave per 64 blocks
        const uint64_t g = (A.nblocks + 63) / 64;
        grid = (unsigned)(g < 65535 ? g : 65535);
    }
    // a State the callback writes, and no other memory (the analysis), a
    // State a lane can copy, rows apart: speculative segments, the serial
    // chain's bits (module_render_seg)
    if (!par && !(flags & DSP_EXEC_SERIAL_STATE) && m->has_facts && m->facts.analyzed && m->facts.writes_state &&
        m->state_size > 0 && m->state_size <= kSegMaxState &&
        !module_rows_overlap(in, in_ch, L, out, C, A.nblocks * B)) {
        auto &W = m->seg;
        if (int st = module_seg_collect(m, false)) return st;
        const unsigned char *pb = (const unsigned char *)params;
        if (!W.warm || W.C != C || W.B != B || W.params.size() != params_size ||
            (params_size && std::memcmp(W.params.data(), pb, params_size))) {
            // new Parameters, or a new shape (whether a State chain or a split
            // State's chain exists depends on it): learn again
            W.params.assign(pb, pb + params_size);
            W.C = C, W.B = B;
            W.warm = kSegWarm0;
            W.off = W.chain_bad = W.one_level = false;
            W.bumps = 0;
            ++W.gen;
        }
        // (learned never to forget: the State chain, then the segments exactly)
        // (the chain's records failed their check once: the serial chain)
        const int st = W.chain_bad ? 1 : module_render_seg(m, A, s, W.off);
        W.serial = st > 0;
        if (st <= 0) return st;
    }
    if (!par) m->seg.serial = true;
    hipFunction_t f = m->f_render;
    if (!par && 2ull * C * B * sizeof(float) <= kStagedLdsBytes) {
        // stateful: 4 waves, the block double-buffer in LDS (the callback's
        // loads and stores hit LDS, the copies run on 192 lanes beside it)
        A.lds = 1;
        block = 256;
        lds_bytes = (unsigned)(2ull * C * B * sizeof(float));
        for (int i = 0; i < 4; ++i)
            if (m->f_render_st[i] && kStShapes[i].C == C && (!kStShapes[i].B || kStShapes[i].B == B)) {
                f = m->f_render_st[i];
                break;
            }
    }
    MOD_HIP(hipModuleLaunchKernel(f, grid, 1, 1, block, 1, 1, lds_bytes, s, args, nullptr));
    MOD_HIP(hipEventRecord(m->use_ev, s));
    return DSP_OK;
}

// The callback once on device buffers, with the live State (DSP_EXEC_VERIFY_CLASS:
// blocks of a call rendered by a block class, re-run through the callback).
// Only for a module whose blocks are independent (par): its callback never
// writes the State, so this run leaves it as it was.
int module_callback_once(dsp_module *m, const void *params, uint32_t params_size, float *const *bufs, uint32_t C,
                         uint32_t B, float sr, hipStream_t s) {
    if (!m || !m->par || !m->initialized) {
        set_last_error("module_callback_once: a loaded module with independent blocks is needed");
        return DSP_ERR_INVALID;
    }
    if (C == 0 || C > (uint32_t)kMaxChannels || params_size != m->params_size) return DSP_ERR_INVALID;
    if (int st = check_device(m)) return st;
    std::lock_guard<std::mutex> lk(m->mu);
    if (int st = upload_params(m, params, params_size, s)) return st;
    RenderArgsG A{};
    A.P = m->d_params;
    A.S = m->d_state[0];
    for (uint32_t c = 0; c < C; ++c) A.out[c] = bufs[c];
    A.C = C;
    A.B = B;
    A.sr = sr;
    void *args[] = {&A};
    MOD_HIP(hipModuleLaunchKernel(m->f_callback, 1, 1, 1, 1, 1, 1, 0, s, args, nullptr));
    MOD_HIP(hipEventRecord(m->use_ev, s));
    return DSP_OK;
}

// dsp_ir_analysis with DSP_PLUGIN_GENERIC: fresh scratch State (compute_IR,
// plugin.cpp:33-49), then the callback once on the impulse buffers.
int module_ir(dsp_module *m, const void *params, uint32_t params_size, float *const *bufs, uint32_t C,
              uint32_t n, float sr, hipStream_t s) {
    if (!m) return DSP_ERR_INVALID;
    if (C == 0 || C > (uint32_t)kMaxChannels) {  // the driver's channel table holds 16 pointers
        set_last_error("GENERIC plugin: 1..%d channels", kMaxChannels);
        return DSP_ERR_INVALID;
    }
    if (int st = check_device(m)) return st;
    if (int st = refuse_capture(s)) return st;
    if (params_size != m->params_size || (!params && params_size)) {
        set_last_error("GENERIC plugin: params blob is %u bytes, the plugin's Parameters %u", params_size,
                       m->params_size);
        return DSP_ERR_INVALID;
    }
    std::lock_guard<std::mutex> lk(m->mu);
    int st = init_slot(m, 1, params, C, sr, 16ull << 20, s);
    if (st) return st;
    RenderArgsG A{};
    A.P = m->d_params;
    A.S = m->d_state[1];
    for (uint32_t c = 0; c < C; ++c) A.out[c] = bufs[c];
    A.C = C;
    A.B = n;
    A.sr = sr;
    void *args[] = {&A};
    MOD_HIP(hipModuleLaunchKernel(m->f_callback, 1, 1, 1, 1, 1, 1, 0, s, args, nullptr));
    if (!m->use_ev) MOD_HIP(hipEventCreateWithFlags(&m->use_ev, hipEventDisableTiming));
    MOD_HIP(hipEventRecord(m->use_ev, s));
    return DSP_OK;
}


// ---------------------------------------------------------------------------
// Block classes (kernels.hpp ModuleSpec).  A plugin whose blocks are
// independent (an empty State, or one its callback never writes) computes
// each block as f(Parameters, State, block, C, B, sr): it cannot see where
// the block lies in the file.  A class is taken only when the callback's own
// IR proves it (dsp_module_facts, ir_proof.cpp) and the callback, run on
// probe blocks, pins what the IR leaves open:
//   TABLE  the callback reads no sample of its block (IR), so its output is
//          one block B for every input; two probes that differ in every
//          element (zeros, noise) render the same values, so every element
//          is written: the render is that block (computed by the callback)
//          tiled, read by the fused kernels as a block table
//          (MapKind::Ramp).  All channels must render the same row.
//   GAIN   every block store is fl(x g) at the address x was loaded from,
//          with one call-invariant g, under input-independent control flow
//          (IR); a probe of ones renders g in every element, so every element
//          is stored exactly once (or the map is fl(x g) anyway): the gain
//          map with that g (MapKind::Gain).  A callback with no block store
//          at all is the identity (g = 1).
// The other probes (uniform in [-1000, 1000], signed steps with a -0) are a
// second check of the same class.  Without facts (a code object compiled
// before them) or without a proof, the callback runs on every block.
constexpr int kProbes = 5;  // zeros, noise [-1, 1], noise [-1000, 1000], steps, ones
constexpr uint32_t kSpecMaxB = 1u << 16;
constexpr size_t kSpecCache = 4;

static uint32_t xorshift(uint32_t &x) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return x;
}

static bool same_bits(float a, float b) { return std::memcmp(&a, &b, 4) == 0; }

// Is the callback's block t[0, B) an f64 ramp rounded to f32 -- t[i] =
// (float)fma(-i, s, g0), the closed form common.hpp ramp_value evaluates --
// for some (g0, s)?  IR_test.cpp (build/IR_test.cpp:47-58: `gain -= step` in
// double from float Parameters) gives one whenever its recurrence is exact.
// Candidates: g0 = t[0]; s = the float nearest the end-to-end slope and its
// neighbours (a float Parameter widened to double), then the slope itself.
// Only a candidate that reproduces all B values bit for bit is taken, so the
// closed form renders exactly the callback's block.
static bool affine_ramp(const float *t, uint32_t B, double *g0, double *s) {
    const double a = t[0];
    auto fits = [&](double sc) {
        for (uint32_t i = 0; i < B; ++i)
            if (!same_bits((float)std::fma(-(double)i, sc, a), t[i])) return false;
        return true;
    };
    if (!std::isfinite(a)) return false;
    // (a subnormal value keeps the table: the device's f64 -> f32 conversion
    // is not checked against the host's there)
    for (uint32_t i = 0; i < B; ++i)
        if (t[i] != 0.f && std::fabs(t[i]) < FLT_MIN) return false;
    if (B == 1) {
        *g0 = a;
        *s = 0.0;
        return true;
    }
    const double slope = (a - (double)t[B - 1]) / (double)(B - 1);
    if (!std::isfinite(slope)) return false;
    std::vector<double> cand;
    const float sf = (float)slope;
    cand.push_back(sf);
    float up = sf, dn = sf;
    for (int k = 0; k < 8; ++k) {
        up = std::nextafter(up, INFINITY);
        dn = std::nextafter(dn, -INFINITY);
        cand.push_back(up);
        cand.push_back(dn);
    }
    cand.push_back(slope);
    for (double sc : cand)
        if (fits(sc)) {
            *g0 = a;
            *s = sc;
            return true;
        }
    return false;
}

static bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// frees the retired tables no call holds and no stream still reads (m->mu held)
void spec_reap(dsp_module *m) {
    for (size_t i = 0; i < m->retired.size();) {
        auto &u = m->retired[i];
        bool done = !u->captured && u->inflight == 0;
        for (auto &kv : u->ev) done = done && hipEventQuery(kv.second) == hipSuccess;
        if (!done) {
            ++i;
            continue;
        }
        (void)hipFree(u->table);
        for (auto &kv : u->ev) (void)hipEventDestroy(kv.second);
        m->retired.erase(m->retired.begin() + (long)i);
    }
}

// a call that rendered with a table class's block releases it: an event on
// its stream after its launches (none under capture: the table then stays
// until dsp_module_destroy)
int module_spec_done(dsp_module *m, void *use, hipStream_t s) {
    if (!m || !use) return DSP_OK;
    std::lock_guard<std::mutex> lk(m->mu);
    auto *u = static_cast<dsp_module::SpecUse *>(use);
    --u->inflight;
    if (capturing(s)) {
        u->captured = true;
    } else {
        hipEvent_t &e = u->ev[s];
        if (!e) MOD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        MOD_HIP(hipEventRecord(e, s));
    }
    spec_reap(m);
    return DSP_OK;
}

size_t module_spec_retired(dsp_module *m) {
    std::lock_guard<std::mutex> lk(m->mu);
    spec_reap(m);
    return m->retired.size();
}

int module_specialize(dsp_module *m, const void *params, uint32_t params_size, uint32_t C, uint32_t B, float sr,
                      hipStream_t s, ModuleSpec *out) {
    *out = ModuleSpec{};
    if (!m || !m->initialized || !m->par || C == 0 || C > (uint32_t)kMaxChannels || B == 0 || B > kSpecMaxB)
        return DSP_OK;
    const dspb::irp::Facts &F = m->facts;
    const bool may_table = m->has_facts && F.analyzed && !F.writes_state && !F.reads_block;
    const bool may_gain = m->has_facts && F.analyzed && !F.writes_state && F.gain_form && !F.input_control;
    const bool may_gtab = m->has_facts && F.analyzed && !F.writes_state && F.gain_table_form && !F.input_control;
    if (!may_table && !may_gain && !may_gtab) return DSP_OK;  // the callback on every block
    if (params_size != m->params_size || (!params && params_size)) return DSP_OK;  // module_render reports it
    if (int st = check_device(m)) return st;
    std::lock_guard<std::mutex> lk(m->mu);
    spec_reap(m);
    for (const auto &e : m->spec)
        if (e.C == C && e.B == B && same_bits(e.sr, sr) && e.params.size() == params_size &&
            (!params_size || std::memcmp(e.params.data(), params, params_size) == 0)) {
            *out = e.r;
            if (e.use) {
                ++e.use->inflight;
                out->use = e.use.get();
            }
            return DSP_OK;
        }
    if (int st = refuse_capture(s)) return st;  // probing allocates and synchronises
    if (int st = upload_params(m, params, params_size, s)) return st;
    const uint64_t n = (uint64_t)C * B;
    std::vector<float> h((size_t)(kProbes * n), 0.f);
    uint32_t seed = 0x9e3779b9u;
    for (uint64_t i = 0; i < n; ++i) {
        // (xorshift32 never yields 0, so no noise element is 0: probes 0 and
        // 1 differ in every element)
        h[n + i] = (float)((int32_t)xorshift(seed)) * (1.0f / 2147483648.0f);
        h[2 * n + i] = (float)((int32_t)xorshift(seed)) * (1000.0f / 2147483648.0f);
        h[3 * n + i] = (float)((int)(i % 13) - 6) * 0.125f;
        h[4 * n + i] = 1.0f;
    }
    for (uint32_t c = 0; c < C; ++c) h[n + (uint64_t)c * B] = 1.0f;
    h[3 * n + (B > 1 ? 1 : 0)] = -0.0f;
    float *d = nullptr;
    MOD_HIP(hipMalloc(&d, sizeof(float) * h.size()));
    struct Free {
        float **p;
        ~Free() { if (*p) (void)hipFree(*p); }
    } fr{&d};
    MOD_HIP(hipMemcpyAsync(d, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice, s));
    for (int p = 0; p < kProbes; ++p) {
        RenderArgsG A{};
        A.P = m->d_params;
        A.S = m->d_state[0];
        for (uint32_t c = 0; c < C; ++c) A.out[c] = d + (uint64_t)(p * C + c) * B;
        A.C = C;
        A.B = B;
        A.sr = sr;
        void *args[] = {&A};
        MOD_HIP(hipModuleLaunchKernel(m->f_callback, 1, 1, 1, 1, 1, 1, 0, s, args, nullptr));
    }
    MOD_HIP(hipEventRecord(m->use_ev, s));
    std::vector<float> r(h.size());
    MOD_HIP(hipMemcpyAsync(r.data(), d, sizeof(float) * r.size(), hipMemcpyDeviceToHost, s));
    // g's value from where the IR says the callback reads it -- not from the
    // callback's output -- so that the probe of ones checks how often each
    // element is scaled: fl(g^k) == g for k != 1 only for g = 0, 1, -1,
    // where x g ... g = x g for every x
    float ge = 0.f;
    bool have_ge = false;
    if (may_gain) {
        if (F.gain_src == 'K') {
            std::memcpy(&ge, &F.gain_bits, 4);
            have_ge = true;
        } else if (F.gain_src == 'R') {
            ge = sr;
            have_ge = true;
        } else if (F.gain_src == 'P' && (uint64_t)F.gain_off + 4 <= params_size) {
            std::memcpy(&ge, (const char *)params + F.gain_off, 4);
            have_ge = true;
        } else if (F.gain_src == 'S' && (uint64_t)F.gain_off + 4 <= m->state_size) {
            MOD_HIP(hipMemcpyAsync(&ge, (const char *)m->d_state[0] + F.gain_off, 4, hipMemcpyDeviceToHost, s));
            have_ge = true;
        }
    }
    MOD_HIP(hipStreamSynchronize(s));
    ModuleSpec res{};
    bool table = may_table;
    for (uint64_t i = 0; i < kProbes * n && table; ++i) table = same_bits(r[i], r[i % B]);
    const float g = ge;
    bool gain = !table && may_gain && have_ge && std::isfinite(g);
    for (uint64_t i = 4 * n; i < 5 * n && gain; ++i) gain = same_bits(r[i], g);  // ones -> g, every element
    for (uint64_t i = 0; i < kProbes * n && gain; ++i) gain = same_bits(r[i], h[i] * g);
    // a gain table (IR: every store x G at x's address, G free of samples,
    // each element stored at most once): G[c][s] is what the probe of ones
    // renders (fl(1 G) = G; 1 where nothing is stored), and every probe must
    // render fl(x G) element by element
    bool gtab = !table && !gain && may_gtab;
    for (uint64_t i = 0; i < kProbes * n && gtab; ++i) gtab = same_bits(r[i], h[i] * r[4 * n + i % n]);
    if (table) {
        float *t = nullptr;
        MOD_HIP(hipMalloc(&t, sizeof(float) * B));
        MOD_HIP(hipMemcpyAsync(t, d, sizeof(float) * B, hipMemcpyDeviceToDevice, s));
        res.kind = kSpecTable;
        res.table = t;
        res.affine = affine_ramp(r.data(), B, &res.rg0, &res.rs);
    } else if (gain) {
        res.kind = kSpecGain;
        res.gain = g;
    } else if (gtab) {
        float *t = nullptr;
        MOD_HIP(hipMalloc(&t, sizeof(float) * n));
        MOD_HIP(hipMemcpyAsync(t, d + 4 * n, sizeof(float) * n, hipMemcpyDeviceToDevice, s));
        res.kind = kSpecGainTable;
        res.table = t;
    }
    // an evicted entry's table is retired, not freed: a call (this thread's
    // or another's) or a captured graph may still read it (spec_reap)
    if (m->spec.size() >= kSpecCache) {
        if (m->spec.front().use) m->retired.push_back(m->spec.front().use);
        m->spec.erase(m->spec.begin());
    }
    std::shared_ptr<dsp_module::SpecUse> use;
    if (res.table) {
        use = std::make_shared<dsp_module::SpecUse>();
        use->table = const_cast<float *>(res.table);
        use->inflight = 1;
    }
    m->spec.push_back({std::vector<unsigned char>((const unsigned char *)params,
                                                  (const unsigned char *)params + params_size),
                       C, B, sr, res, use});
    *out = res;
    out->use = use.get();
    return DSP_OK;
}

}  // namespace dspb
