// ir_proof.hpp -- what a plugin's audio_callback does with its block, read
// from the callback's own LLVM IR (ir_proof.cpp).
//
// The reference calls the compiled callback on every block
// (audio.cpp:160-165 -> compiler.cpp:1181-1187).  The product may render a
// block class instead (module.h DSP_BLOCK_TABLE / DSP_BLOCK_GAIN) or run the
// blocks of a plugin with a State in parallel; it does so only on facts this
// analysis establishes about the callback's code, never on probe outputs
// alone.
#pragma once
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace dspb {
namespace irp {

struct Facts {
    bool analyzed = false;      // every instruction of the callback was inside the analysis
    bool reads_block = false;   // a load (or memcpy source) through a block sample pointer
    bool writes_state = false;  // a store (or memset / memcpy destination) through State
    bool input_control = false; // a branch / switch condition depends on a block sample
    bool gain_form = false;     // every block store is fl(x g) at the address x was loaded
                                // from, with one g for the whole call (no sample, no
                                // loop-carried value, no address in it); no block store
                                // at all is the identity (g = 1)
    std::string gain_expr;      // g, canonical (diagnostics)
    // gain_form: where g comes from -- 'P' / 'S' a float at byte gain_off of
    // Parameters / State, 'K' the constant with bits gain_bits, 'R' the
    // sample-rate argument -- so that its value is known without the callback
    char gain_src = 0;
    uint32_t gain_off = 0, gain_bits = 0;
    // every block store is fl(x G) at the address x was loaded from, G free
    // of any sample (it may vary with the channel, the position, Parameters,
    // a State the callback only reads), and each element is stored at most
    // once: the store addresses are (a constant channel or a loop's induction
    // variable, a loop's induction variable), each store inside exactly the
    // loops its address uses, different store instructions on different
    // constant channels (the CFG's natural loops, ir_proof.cpp)
    bool gain_table_form = false;
    std::string table_why;      // why not gain_table_form
    // a value stored to State, or a branch condition, depends on a block
    // sample (true unless the analysis completed and showed otherwise): when
    // false the State's trajectory is the same whatever the block holds
    bool state_reads_block = true;
    // state_reads_block, but with no branch on a sample and every store of a
    // block-dependent value at an offset of known range (a constant, a
    // channel loop's counter bounded by its exit test) or known lower bound:
    // the State's 4-byte words split into the block-dependent ones
    // (state_dep_words: word indices, and -(T + 2) for every word from T on)
    // and the others, which at least one store writes -- whose trajectory is
    // the same whatever the block holds (a block counter beside an envelope)
    bool state_split = false;
    std::vector<int64_t> state_dep_words;
    std::string why;            // the first construct that ended the analysis, or why a
                                // property does not hold
};

// Analyse kernel `fn` of module text `ir`, a kernel of the form
//   fn(Parameters *P, State *S, float **out, unsigned C, unsigned B, float sr)
//   { audio_callback(*P, *S, out, C, B, sr); }   (flattened: the callback inlined)
Facts analyze(const std::string &ir, const char *fn);

// Compile a HIP translation unit to optimised LLVM IR text for gfx950 through
// comgr (the same front end hiprtc drives), with the hiprtc runtime header
// pre-included as hiprtc does.  0 on success, else -1 with *log set.
int compile_to_ir(const std::string &tu, const std::vector<std::pair<std::string, std::string>> &includes,
                  const std::vector<std::string> &options, std::string *ir, std::string *log);

// The State chain of a callback whose State never depends on its block
// (facts: writes_state, !state_reads_block): in every `dspb_seg_chain_*`
// function of the module's IR text, delete the stores through pointers
// derived from the private block `dspb_chain_blk` other than the copy of the
// input into it (non-temporal stores) -- the callback's outputs, which by
// that fact reach no State and no branch -- so that code generation drops the
// arithmetic that only fed them.  `prefix`: the functions edited (the chain
// of a split State's block-independent words: "@dspb_seg_chain_ind_").
// Returns the stores deleted, -1 for a store outside the pass's model.
int strip_chain_block_stores(std::string *ir, const char *prefix = "@dspb_seg_chain_");

// LLVM IR text -> a gfx950 code object (comgr: codegen at `options`, link).
int codegen_ir(const std::string &ir, const std::vector<std::string> &options, std::string *code, std::string *log);

// Facts <-> the compact text stored in a code object (dspb_callback_facts).
std::string encode(const Facts &f);
bool decode(const std::string &s, Facts *f);

}  // namespace irp
}  // namespace dspb
