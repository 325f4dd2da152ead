// ir_proof.cpp -- facts about a plugin's audio_callback from its LLVM IR
// (ir_proof.hpp).
//
// dsp_module_compile compiles the plugin a second time, through comgr, into
// a flattened analysis kernel
//
//   dspb_proof(Parameters *P, State *S, float **out, unsigned C, unsigned B, float sr)
//   { audio_callback(*P, *S, out, C, B, sr); }
//
// at -O2 without vectorisation or unrolling (the same source and IEEE
// semantics as the code that runs: only the schedule differs), and reads the
// optimised IR of that kernel.  Every SSA value gets
//
//   an origin (pointers): BUF (a block sample pointer: an element of `out`),
//     TBL (`out` itself), PRM (Parameters), STA (State), LOC (private
//     memory), GC / GM (constant / mutable global), EXT (a pointer read from
//     memory other than `out`), UNK (made from an integer);
//   dependence bits: IN (depends on a block sample), VAR (may differ between
//     the callback's iterations: a phi, a private or block load, State that
//     is written), ADDR (depends on an address as a number),
//
// iterated to a fixpoint over the phis.  Anything outside the model -- a call
// that may touch memory, an atomic, a store to Parameters / `out` / a global,
// a pointer stored to memory, a block address compared or turned into an
// integer -- ends the analysis with `analyzed` false, and the product then
// runs the callback on every block.
//
// What the facts prove (module.cpp uses them, plus probes of the callback):
//   !reads_block: the callback reads no sample of its block (nor an address
//       of one), so its output is a function of (Parameters, State, C, B, sr)
//       only -- every block renders the same values (DSP_BLOCK_TABLE; which
//       elements are written is pinned by two probes that differ everywhere);
//   gain_form && !input_control: the sequence of block stores is the same on
//       every call and each stores fl(x g) for the x loaded from that same
//       address and one call-invariant g (DSP_BLOCK_GAIN; a probe of ones
//       pins g and that every element is stored once);
//   !writes_state: blocks are independent given the State, so a plugin with
//       a State it only reads renders its blocks in parallel.
#include "ir_proof.hpp"

#include <dlfcn.h>

#include <amd_comgr/amd_comgr.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <sstream>

namespace dspb {
namespace irp {

namespace {

enum : uint32_t { O_BUF = 1, O_TBL = 2, O_PRM = 4, O_STA = 8, O_LOC = 16, O_GC = 32, O_GM = 64, O_EXT = 128, O_UNK = 256 };
enum : uint32_t { D_IN = 1, D_VAR = 2, D_ADDR = 4 };

// soff / shi: for a pointer into State alone (org == O_STA), the range of its
// byte offset from the State's base, [soff, shi] (shi = kShiInf: no upper
// bound -- an index the analysis knows only to be non-negative): kSoffUnset
// before the fixpoint has seen a definition, kSoffUnknown when no range is
// known (a negative or unparsed offset)
constexpr int64_t kSoffUnset = -2, kSoffUnknown = -1, kShiInf = INT64_MAX;
struct Val {
    uint32_t org = 0, data = 0;
    int64_t soff = kSoffUnset, shi = kSoffUnset;
};
// the hull of two offset ranges
void join_off(Val &a, const Val &b) {
    if (b.soff == kSoffUnset) return;
    if (a.soff == kSoffUnset) {
        a.soff = b.soff, a.shi = b.shi;
    } else if (a.soff == kSoffUnknown || b.soff == kSoffUnknown) {
        a.soff = a.shi = kSoffUnknown;
    } else {
        a.soff = std::min(a.soff, b.soff);
        a.shi = std::max(a.shi, b.shi);
    }
}

// bytes of an IR scalar or vector type (0: not one this analysis sizes)
int64_t type_bytes(const std::string &t) {
    static const std::map<std::string, int64_t> kScalar = {
        {"i8", 1}, {"i16", 2}, {"i32", 4}, {"i64", 8}, {"half", 2}, {"bfloat", 2}, {"float", 4}, {"double", 8},
        {"ptr", 8}, {"ptr addrspace(1)", 8}, {"ptr addrspace(5)", 4}, {"i1", 1}};
    auto it = kScalar.find(t);
    if (it != kScalar.end()) return it->second;
    if (t.size() > 4 && ((t[0] == '<' && t.back() == '>') || (t[0] == '[' && t.back() == ']'))) {  // <N x T>, [N x T]
        const size_t x = t.find(" x ");
        if (x == std::string::npos) return 0;
        const int64_t n = std::strtoll(t.c_str() + 1, nullptr, 10);
        const int64_t e = type_bytes(t.substr(x + 3, t.size() - x - 4));
        return (n > 0 && e > 0 && n < (1ll << 32)) ? n * e : 0;
    }
    return 0;
}
// the element type of an array type [N x T] ("" if not one)
std::string array_elem(const std::string &t) {
    if (t.size() < 6 || t[0] != '[' || t.back() != ']') return "";
    const size_t x = t.find(" x ");
    return x == std::string::npos ? "" : t.substr(x + 3, t.size() - x - 4);
}

struct Inst {
    std::string res, op, text;      // result (or ""), opcode, operand text after the opcode
    std::vector<std::string> parts; // `text` split at top-level commas
    int blk = 0;                    // its basic block (Analysis::blk_name)
    bool nuw = false;               // a `nuw` flag (a getelementptr's offsets are non-negative)
    std::string pred;               // icmp / fcmp: the predicate
};

bool ident_char(char c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '.' || c == '_' ||
           c == '$' || c == '-';
}

std::string trim(const std::string &s) {
    size_t a = 0, b = s.size();
    while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
    while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) --b;
    return s.substr(a, b - a);
}

// the line without its `;` comment (outside string literals)
std::string strip_comment(const std::string &s) {
    bool q = false;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == '"') q = !q;
        else if (s[i] == ';' && !q) return s.substr(0, i);
    }
    return s;
}

std::vector<std::string> split_top(const std::string &s) {
    std::vector<std::string> out;
    int depth = 0;
    bool q = false;
    size_t start = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        const char c = s[i];
        if (c == '"') q = !q;
        if (q) continue;
        if (c == '(' || c == '[' || c == '{' || c == '<') ++depth;
        else if (c == ')' || c == ']' || c == '}' || c == '>') --depth;
        else if (c == ',' && depth == 0) {
            out.push_back(trim(s.substr(start, i - start)));
            start = i + 1;
        }
    }
    const std::string last = trim(s.substr(start));
    if (!last.empty()) out.push_back(last);
    return out;
}

struct Module {
    std::set<std::string> types;                       // %named types (numbered ones too: %0 = type ...)
    std::set<std::string> locals;                      // the analysed function's arguments and results
    std::map<std::string, bool> global_const;          // @global -> constant
    std::map<std::string, std::string> fn_attrs;       // @function -> its attribute groups' text
    std::map<std::string, std::string> attr_groups;    // #N -> text
    std::map<std::string, std::vector<std::string>> fn_groups;  // @function -> #N ids
};

// value tokens (%x / @x) of an operand text, in order; named types and
// `label %x` operands excluded
std::vector<std::string> values_in(const std::string &s, const Module &M) {
    std::vector<std::string> v;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] != '%' && s[i] != '@') continue;
        size_t j = i + 1;
        if (j < s.size() && s[j] == '"') {
            const size_t e = s.find('"', j + 1);
            if (e == std::string::npos) break;
            j = e + 1;
        } else {
            while (j < s.size() && ident_char(s[j])) ++j;
        }
        const std::string tok = s.substr(i, j - i);
        const bool is_label = i >= 6 && s.compare(i - 6, 6, "label ") == 0;
        // a numbered type (%0 = type ...) and a numbered value (%0, an
        // unnamed argument) share their spelling: a token the function
        // defines is taken as the value (at worst an extra dependence)
        const bool is_type = s[i] == '%' && M.types.count(tok) && !M.locals.count(tok);
        if (tok.size() > 1 && !is_label && !is_type) v.push_back(tok);
        i = j - 1;
    }
    return v;
}

std::string first_value(const std::string &s, const Module &M) {
    const auto v = values_in(s, M);
    return v.empty() ? std::string() : v.front();
}

// the attribute-group ids (#N) after the argument list of a define / declare / call
std::vector<std::string> groups_after_args(const std::string &s, size_t open) {
    std::vector<std::string> g;
    int depth = 0;
    size_t i = open;
    for (; i < s.size(); ++i) {
        if (s[i] == '(') ++depth;
        else if (s[i] == ')' && --depth == 0) break;
    }
    for (; i < s.size(); ++i) {
        if (s[i] == '#') {
            size_t j = i + 1;
            while (j < s.size() && s[j] >= '0' && s[j] <= '9') ++j;
            g.push_back(s.substr(i, j - i));
            i = j;
        }
    }
    return g;
}

bool starts_with(const std::string &s, const char *p) { return s.compare(0, std::strlen(p), p) == 0; }

struct Analysis {
    const Module &M;
    std::map<std::string, Val> val;
    std::map<std::string, const Inst *> def;
    std::vector<Inst> body;
    std::vector<std::string> args;  // the kernel's six parameters
    uint32_t loc_data = 0, sta_data = 0;
    // State stores by byte: the data bits stored at each known offset, those
    // of stores with a lower bound alone (every byte from there on), and those
    // of stores whose offset or extent is not known (any byte)
    std::map<int64_t, uint32_t> sta_byte, sta_tail;
    uint32_t sta_any = 0;
    Facts f;
    std::string fail;
    std::vector<std::string> blk_name;  // "%label" per basic block; block 0 is the entry

    explicit Analysis(const Module &m) : M(m) {}

    void stop(const std::string &why) {
        if (fail.empty()) fail = why;
    }

    Val get(const std::string &tok) const {
        Val v;
        if (tok.empty()) return v;
        if (tok[0] == '@') {
            auto g = M.global_const.find(tok);
            if (g != M.global_const.end()) v.org = g->second ? O_GC : O_GM;
            return v;
        }
        auto it = val.find(tok);
        return it == val.end() ? v : it->second;
    }

    bool callee_pure(const std::string &callee, const std::string &site_attrs) const {
        std::string attrs = site_attrs;
        auto g = M.fn_attrs.find(callee);
        if (g != M.fn_attrs.end()) attrs += " " + g->second;
        if (attrs.find("memory(none)") != std::string::npos) return true;
        // device-library routines that only read constant tables
        if (starts_with(callee, "@__ocml_") || starts_with(callee, "@__ockl_")) {
            const size_t m = attrs.find("memory(");
            if (m != std::string::npos) {
                const size_t e = attrs.find(')', m);
                const std::string mem = attrs.substr(m, e == std::string::npos ? std::string::npos : e - m);
                if (mem.find("write") == std::string::npos) return true;
            }
        }
        return false;
    }

    // the bytes [lo, end) a pointer with offset range P touches with an access
    // of n bytes (end = kShiInf: every byte from lo on); false: unknown
    static bool extent(const Val &P, int64_t n, int64_t *lo, int64_t *end) {
        if (P.org != O_STA || P.soff < 0 || n <= 0) return false;
        *lo = P.soff;
        *end = (P.shi == kShiInf || P.shi - P.soff > (1 << 16)) ? kShiInf : P.shi + n;
        return true;
    }
    // a store of data bits d through State pointer P of n bytes (0: extent unknown)
    void state_store(const Val &P, uint32_t d, int64_t n) {
        f.writes_state = true;
        sta_data |= d;
        int64_t lo, end;
        if (!extent(P, n, &lo, &end))
            sta_any |= d;
        else if (end == kShiInf)
            sta_tail[lo] |= d;
        else
            for (int64_t b = lo; b < end; ++b) sta_byte[b] |= d;
    }
    // the data bits a load of n bytes through State pointer P can see
    uint32_t state_load(const Val &P, int64_t n) const {
        uint32_t d = sta_any;
        int64_t lo = 0, end = kShiInf;
        if (!extent(P, n, &lo, &end)) lo = 0, end = kShiInf;
        for (auto it = sta_byte.lower_bound(lo); it != sta_byte.end() && it->first < end; ++it) d |= it->second;
        for (const auto &t : sta_tail)
            if (t.first < end) d |= t.second;
        return d;
    }

    // one transfer step for instruction I; returns true when a value grew
    bool step(const Inst &I, bool final_pass) {
        Val r;
        const std::string &op = I.op;
        auto merge_all = [&](const std::string &s) {
            for (const auto &t : values_in(s, M)) {
                const Val v = get(t);
                r.org |= v.org;
                r.data |= v.data;
            }
        };
        auto store_to = [&](const Val &P, const Val &Vv, bool val_is_ptr, const std::string &what, int64_t n) {
            if (P.org == 0) {  // (store_to runs in the final pass: every origin has propagated)
                stop(what + " through a pointer of unknown origin");
                return;
            }
            if (P.org & (O_TBL | O_PRM | O_GC | O_GM | O_EXT | O_UNK)) {
                stop(what + " to " + (P.org & O_TBL ? "the block pointer table" : P.org & O_PRM ? "Parameters" :
                                      (P.org & (O_GC | O_GM)) ? "global memory" : "memory behind a loaded pointer"));
                return;
            }
            if (val_is_ptr && (Vv.org & (O_BUF | O_TBL | O_STA | O_PRM | O_LOC | O_EXT))) {
                stop("a pointer is stored to memory");
                return;
            }
            if (P.org & O_STA) state_store(P, Vv.data | P.data, n);
            if (P.org & O_LOC) loc_data |= Vv.data | P.data;
            if ((P.org & O_BUF) && (P.data & D_IN)) f.input_control = true;  // an input-dependent address
        };
        auto load_from = [&](const Val &P, bool ptr_result, int64_t n) {
            Val v;
            if (final_pass && P.org == 0) stop("a load through a pointer of unknown origin");
            if (P.org & O_GM) stop("a load of mutable global memory");
            if (P.org & O_UNK) stop("a load through a pointer made from an integer");
            v.data = P.data & (D_IN | D_VAR | D_ADDR);
            if (P.org & O_BUF) {
                v.data |= D_IN | D_VAR;
                f.reads_block = true;
            }
            if (P.org & O_LOC) v.data |= loc_data | D_VAR;
            if (P.org & O_STA) v.data |= f.writes_state ? (state_load(P, n) | D_VAR) : 0u;
            if (P.org & O_TBL) {
                if (ptr_result) v.org |= O_BUF;
                else stop("the block pointer table is read as data");
            }
            if (ptr_result && (P.org & (O_PRM | O_STA | O_LOC | O_GC | O_EXT))) v.org |= O_EXT;
            if (ptr_result && (P.org & O_BUF)) v.org |= O_UNK;
            return v;
        };
        if (op == "alloca") {
            r.org = O_LOC;
        } else if (op == "load") {
            if (I.parts.size() < 2) return stop("unparsed load: " + I.text), false;
            if (starts_with(I.text, "atomic")) return stop("an atomic load"), false;
            const std::string &ty = I.parts[0];
            const bool ptr_result = starts_with(ty, "ptr") || ty.find("x ptr") != std::string::npos ||
                                    starts_with(ty, "volatile ptr");
            r = load_from(get(first_value(I.parts[1], M)), ptr_result, type_bytes(ty));
        } else if (op == "store") {
            if (I.parts.size() < 2) return stop("unparsed store: " + I.text), false;
            if (starts_with(I.text, "atomic")) return stop("an atomic store"), false;
            const std::string vt = first_value(I.parts[0], M);
            const Val P = get(first_value(I.parts[1], M));
            const Val Vv = get(vt);
            const bool val_is_ptr = starts_with(I.parts[0], "ptr") || starts_with(I.parts[0], "volatile ptr") ||
                                    I.parts[0].find("x ptr>") != std::string::npos;
            // the stored value's type: the operand text before its value token
            std::string vty = I.parts[0];
            if (starts_with(vty, "volatile ")) vty = vty.substr(9);
            const size_t vs = vty.rfind(' ');
            const int64_t n = type_bytes(vs == std::string::npos ? vty : trim(vty.substr(0, vs)));
            if (final_pass) store_to(P, Vv, val_is_ptr, "a store", n);
            else {
                if (P.org & O_STA) state_store(P, Vv.data | P.data, n);
                if (P.org & O_LOC) loc_data |= Vv.data | P.data;
            }
            return false;
        } else if (op == "getelementptr") {
            if (I.parts.size() < 2) return stop("unparsed getelementptr: " + I.text), false;
            const Val b = get(first_value(I.parts[1], M));
            r.org = b.org;
            r.data = b.data;
            for (size_t k = 2; k < I.parts.size(); ++k)
                for (const auto &t : values_in(I.parts[k], M)) r.data |= get(t).data;
            // a State pointer plus one index of a sized element type: a
            // constant, an index of known range (a loop's counter bounded by
            // its exit test), or (nuw) any non-negative one
            // (an older LLVM -- the comgr a process gets once PyTorch's ROCm
            // libraries are loaded -- keeps array GEPs: [N x T], 0, i; each
            // index steps through the array types)
            r.soff = r.shi = kSoffUnknown;
            if (b.org == O_STA && b.soff >= 0 && I.parts.size() >= 3) {
                std::string ty = trim(I.parts[0]);
                int64_t lo = b.soff, hi = b.shi;
                bool ok = true;
                for (size_t k = 2; k < I.parts.size() && ok; ++k) {
                    if (k > 2) ty = array_elem(ty);  // the next index steps inside an array
                    const int64_t es = ty.empty() ? 0 : type_bytes(ty);
                    int64_t ilo = 0, ihi = kShiInf;
                    const bool known = es > 0 && index_range(I.parts[k], &ilo, &ihi);
                    if (!known && !(es > 0 && I.nuw)) { ok = false; break; }
                    if (!known || (ilo < 0 && I.nuw)) ilo = 0;  // nuw: the offsets are non-negative
                    if (ilo > (1ll << 32) || ilo < -(1ll << 32)) { ok = false; break; }
                    lo += ilo * es;
                    hi = (hi == kShiInf || ihi == kShiInf || ihi > (1ll << 32)) ? kShiInf : hi + ihi * es;
                }
                if (ok && lo >= 0) r.soff = lo, r.shi = hi;
            } else if (b.soff == kSoffUnset) {
                r.soff = r.shi = kSoffUnset;
            }
        } else if (op == "bitcast" || op == "addrspacecast" || op == "freeze") {
            merge_all(I.text);
            const Val p = get(first_value(I.text, M));
            r.soff = p.soff, r.shi = p.shi;
        } else if (op == "ptrtoint") {
            const Val p = get(first_value(I.text, M));
            if (p.org & (O_BUF | O_TBL | O_LOC | O_STA | O_PRM | O_EXT)) stop("an address is turned into an integer");
            r.data = p.data | D_ADDR;
        } else if (op == "inttoptr") {
            r.org = O_UNK;
            r.data = get(first_value(I.text, M)).data;
        } else if (op == "icmp") {
            merge_all(I.text);
            if (r.org & (O_BUF | O_TBL)) stop("block addresses are compared");
            r.org = 0;
        } else if (op == "phi") {
            // [ value, %block ], ...
            for (const auto &p : split_top(I.text.substr(I.text.find('[') == std::string::npos ? 0
                                                                                                : I.text.find('[')))) {
                std::string in = p;
                const size_t a = in.find('['), b = in.rfind(']');
                if (a != std::string::npos && b != std::string::npos && b > a) in = in.substr(a + 1, b - a - 1);
                const auto two = split_top(in);
                if (two.empty()) continue;
                const Val v = get(first_value(two[0], M));
                r.org |= v.org;
                r.data |= v.data;
                join_off(r, v);
            }
            r.data |= D_VAR;
        } else if (op == "call") {
            // the callee: the first value token directly followed by its
            // argument list (`@f(` direct, `%fp(` indirect)
            std::string callee;
            size_t e = std::string::npos;
            for (size_t i = 0; i < I.text.size(); ++i) {
                if (I.text[i] != '@' && I.text[i] != '%') continue;
                size_t j = i + 1;
                while (j < I.text.size() && ident_char(I.text[j])) ++j;
                if (j < I.text.size() && I.text[j] == '(') {
                    callee = I.text.substr(i, j - i);
                    e = j;
                    break;
                }
                i = j - 1;
            }
            if (callee.empty()) return stop("an unparsed call: " + I.text), false;
            if (callee[0] == '%') return stop("an indirect call"), false;
            const size_t open = I.text.find('(', e);
            std::string argtext;
            if (open != std::string::npos) {
                int depth = 0;
                size_t k = open;
                for (; k < I.text.size(); ++k) {
                    if (I.text[k] == '(') ++depth;
                    else if (I.text[k] == ')' && --depth == 0) break;
                }
                argtext = I.text.substr(open + 1, k > open ? k - open - 1 : 0);
            }
            const auto a = split_top(argtext);
            std::string site;
            for (const auto &g : groups_after_args(I.text, open == std::string::npos ? I.text.size() : open)) {
                auto it = M.attr_groups.find(g);
                if (it != M.attr_groups.end()) site += " " + it->second;
            }
            if (starts_with(callee, "@llvm.memcpy") || starts_with(callee, "@llvm.memmove")) {
                if (a.size() < 3) return stop("unparsed memcpy"), false;
                const Val src = get(first_value(a[1], M));
                Val v = load_from(src, false, 0);
                v.data |= get(first_value(a[2], M)).data;
                const Val dst = get(first_value(a[0], M));
                if (final_pass) store_to(dst, v, false, "a memcpy", 0);
                else {
                    if (dst.org & O_STA) state_store(dst, v.data | dst.data, 0);
                    if (dst.org & O_LOC) loc_data |= v.data | dst.data;
                }
                if (final_pass && (dst.org & O_BUF)) gain_breakers.insert("a memcpy into the block"),
                    table_breakers.insert("a memcpy into the block");
                return false;
            }
            if (starts_with(callee, "@llvm.memset")) {
                if (a.size() < 3) return stop("unparsed memset"), false;
                Val v = get(first_value(a[1], M));
                v.data |= get(first_value(a[2], M)).data;
                const Val dst = get(first_value(a[0], M));
                if (final_pass) store_to(dst, v, false, "a memset", 0);
                else {
                    if (dst.org & O_STA) state_store(dst, v.data | dst.data, 0);
                    if (dst.org & O_LOC) loc_data |= v.data | dst.data;
                }
                if (final_pass && (dst.org & O_BUF)) gain_breakers.insert("a memset of the block"),
                    table_breakers.insert("a memset of the block");
                return false;
            }
            static const char *kIgnore[] = {"@llvm.lifetime.", "@llvm.assume", "@llvm.experimental.noalias.scope.decl",
                                            "@llvm.dbg.", "@llvm.donothing", "@llvm.trap", "@llvm.debugtrap",
                                            "@llvm.sideeffect", "@llvm.pseudoprobe"};
            for (const char *p : kIgnore)
                if (starts_with(callee, p)) return false;
            static const char *kLane[] = {"workitem", "workgroup", "dispatch", "implicitarg", "readfirstlane",
                                          "readlane", "ballot", "mbcnt", ".ds.", "getreg", "memtime", "memrealtime",
                                          "s.sleep", "wave", "lds", "cluster", "queue", "permlane", "update.dpp",
                                          "mov.dpp", "icmp", "fcmp", "wqm", "wwm", "barrier", "s.wait"};
            if (starts_with(callee, "@llvm.amdgcn."))
                for (const char *p : kLane)
                    if (callee.find(p) != std::string::npos) return stop("a lane-dependent builtin: " + callee), false;
            if (!callee_pure(callee, site)) return stop("a call that may touch memory: " + callee), false;
            for (const auto &x : a)
                for (const auto &t : values_in(x, M)) {
                    const Val v = get(t);
                    r.data |= v.data;
                    // a pointer it returns may be any argument moved (llvm.ptrmask
                    // of __builtin_align_down): it keeps their origins
                    r.org |= v.org;
                    if (v.org & (O_BUF | O_TBL)) stop("a block pointer is passed to " + callee);
                }
        } else if (op == "atomicrmw" || op == "cmpxchg" || op == "fence" || op == "va_arg" || op == "invoke" ||
                   op == "callbr" || op == "indirectbr" || op == "landingpad" || op == "resume") {
            stop("a `" + op + "` instruction");
        } else if (op == "br" || op == "switch") {
            if (final_pass) {
                const std::string c = first_value(I.text, M);
                if (get(c).data & D_IN) f.input_control = true;
            }
            return false;
        } else if (op == "ret" || op == "unreachable") {
            return false;
        } else {  // arithmetic, casts, compares, selects, aggregates, vectors
            merge_all(I.text);
            for (const auto &t : values_in(I.text, M)) {
                const Val v = get(t);
                if (v.org & O_STA) join_off(r, v);
            }
        }
        if (I.res.empty()) return false;
        Val &cur = val[I.res];
        const Val before = cur;
        cur.org |= r.org;
        cur.data |= r.data;
        // the range this definition has had over every pass, widened: a bound
        // that moves once more (a pointer stepped through a loop) is dropped,
        // so that the fixpoint ends
        if (r.soff != kSoffUnset) {
            if (cur.soff == kSoffUnset) {
                cur.soff = r.soff, cur.shi = r.shi;
            } else if (cur.soff == kSoffUnknown || r.soff == kSoffUnknown || r.soff < cur.soff) {
                cur.soff = cur.shi = kSoffUnknown;
            } else if (r.shi > cur.shi) {
                cur.shi = kShiInf;
            }
        }
        return cur.org != before.org || cur.data != before.data || cur.soff != before.soff || cur.shi != before.shi;
    }

    std::set<std::string> gain_breakers, table_breakers;
    std::map<std::string, std::string> canon_memo;

    // ---- the gain-table form: at most one store per block element --------
    // The control flow graph from the terminators' `label %x` operands, its
    // dominators and natural loops; a loop's canonical induction variable
    // (phi [0, outside], [iv + 1, inside] in its header) takes distinct
    // values in one run of the loop.  A store whose address is (channel,
    // sample) = (a constant or a loop's IV, a loop's IV), inside exactly the
    // loops whose IVs its address uses, hits each element at most once; two
    // store instructions must name different constant channels.
    struct Loop {
        int header;
        std::vector<bool> body;
    };
    std::vector<std::vector<int>> succ_;
    std::vector<std::vector<bool>> dom_;  // dom_[b][a]: block a dominates block b
    std::vector<Loop> loops_;
    bool loops_ok_ = false;

    static std::vector<std::string> labels_in(const std::string &t) {
        std::vector<std::string> out;
        for (size_t i = t.find("label %"); i != std::string::npos; i = t.find("label %", i + 1)) {
            size_t j = i + 7;
            while (j < t.size() && ident_char(t[j])) ++j;
            out.push_back(t.substr(i + 6, j - i - 6));
        }
        return out;
    }

    bool build_loops(std::string *why) {
        loops_.clear();
        loops_ok_ = false;
        iv_max_memo_.clear();
        const int n = (int)blk_name.size();
        std::map<std::string, int> id;
        for (int b = 0; b < n; ++b)
            if (!blk_name[b].empty()) id[blk_name[b]] = b;
        succ_.assign(n, {});
        std::vector<std::vector<int>> pred(n);
        for (const Inst &I : body) {
            if (I.op != "br" && I.op != "switch" && I.op != "indirectbr" && I.op != "callbr") continue;
            for (const auto &l : labels_in(I.text)) {
                auto it = id.find(l);
                if (it == id.end()) return *why = "a branch to an unknown block " + l, false;
                succ_[I.blk].push_back(it->second);
                pred[it->second].push_back(I.blk);
            }
        }
        // dominators, iteratively (a few hundred blocks at most)
        std::vector<std::vector<bool>> dom(n, std::vector<bool>(n, true));
        dom[0].assign(n, false);
        dom[0][0] = true;
        for (bool changed = true; changed;) {
            changed = false;
            for (int b = 1; b < n; ++b) {
                std::vector<bool> d(n, pred[b].empty() ? false : true);
                for (int p : pred[b])
                    for (int k = 0; k < n; ++k) d[k] = d[k] && dom[p][k];
                d[b] = true;
                if (d != dom[b]) dom[b] = d, changed = true;
            }
        }
        // every cycle must be a natural loop: without the back edges (t -> h,
        // h dominating t) the graph is acyclic, else the control flow is
        // irreducible and a block could run more than once per iteration of
        // the loops found below
        {
            std::vector<int> color(n, 0);  // 0 new, 1 on the stack, 2 done
            std::vector<std::pair<int, size_t>> st;
            for (int r = 0; r < n; ++r) {
                if (color[r]) continue;
                st.push_back({r, 0});
                color[r] = 1;
                while (!st.empty()) {
                    auto &[b, k] = st.back();
                    if (k == succ_[b].size()) {
                        color[b] = 2;
                        st.pop_back();
                        continue;
                    }
                    const int t = succ_[b][k++];
                    if (dom[b][t]) continue;  // a back edge
                    if (color[t] == 1) return *why = "irreducible control flow", false;
                    if (!color[t]) color[t] = 1, st.push_back({t, 0});
                }
            }
        }
        // natural loops of the back edges t -> h (h dominates t), one per header
        std::map<int, int> by_header;
        for (int t = 0; t < n; ++t)
            for (int h : succ_[t]) {
                if (!dom[t][h]) continue;
                auto it = by_header.find(h);
                if (it == by_header.end()) {
                    by_header[h] = (int)loops_.size();
                    loops_.push_back(Loop{h, std::vector<bool>(n, false)});
                    it = by_header.find(h);
                }
                std::vector<bool> &in = loops_[it->second].body;
                in[h] = true;
                std::vector<int> work;
                if (!in[t]) in[t] = true, work.push_back(t);
                while (!work.empty()) {
                    const int b = work.back();
                    work.pop_back();
                    for (int p : pred[b])
                        if (!in[p]) in[p] = true, work.push_back(p);
                }
            }
        dom_ = std::move(dom);
        loops_ok_ = true;
        return true;
    }

    // an integer literal operand ("i64 8", or the bare value)
    static bool int_literal(const std::string &operand, int64_t *c) {
        std::string lit = trim(operand);
        const size_t sp = lit.rfind(' ');
        if (sp != std::string::npos) {
            if (lit[0] != 'i') return false;
            lit = trim(lit.substr(sp + 1));
        }
        if (lit.empty()) return false;
        char *e = nullptr;
        const long long v = std::strtoll(lit.c_str(), &e, 10);
        if (!e || *e != 0) return false;
        *c = v;
        return true;
    }
    // an upper bound of a loop-invariant integer: a literal, or
    // llvm.umin / llvm.smin with a literal argument (through zext)
    bool int_max(const std::string &operand, int64_t *hi) const {
        if (int_literal(operand, hi)) return true;
        std::string tok = first_value(operand, M);
        for (int hop = 0; hop < 3 && !tok.empty(); ++hop) {
            auto d = def.find(tok);
            if (d == def.end()) return false;
            const Inst &I = *d->second;
            if (I.op == "zext") {
                tok = first_value(I.text, M);
                continue;
            }
            if (I.op != "call" || (I.text.find("@llvm.umin.") == std::string::npos &&
                                   I.text.find("@llvm.smin.") == std::string::npos))
                return false;
            const size_t open = I.text.find('(');
            const size_t close = I.text.rfind(')');
            if (open == std::string::npos || close == std::string::npos || close <= open) return false;
            bool have = false;
            for (const auto &a : split_top(I.text.substr(open + 1, close - open - 1))) {
                int64_t c;
                if (int_literal(a, &c)) *hi = have ? std::min(*hi, c) : c, have = true;
            }
            return have;
        }
        return false;
    }
    // the largest value loop li's canonical IV `iv` takes in the loop, from an
    // exit test every iteration runs (its block dominates each latch) that
    // compares the IV or its increment with a loop-invariant bound
    mutable std::map<std::string, std::pair<bool, int64_t>> iv_max_memo_;  // (the CFG is fixed: per IV once)
    bool iv_max(const std::string &iv, int li, int64_t *hi) const {
        auto memo = iv_max_memo_.find(iv);
        if (memo != iv_max_memo_.end()) {
            if (memo->second.first) *hi = memo->second.second;
            return memo->second.first;
        }
        int64_t m = 0;
        const bool ok = iv_max_scan(iv, li, &m);
        iv_max_memo_[iv] = {ok, m};
        if (ok) *hi = m;
        return ok;
    }
    bool iv_max_scan(const std::string &iv, int li, int64_t *hi) const {
        const Loop &L = loops_[li];
        const int n = (int)blk_name.size();
        std::string next;  // the IV's increment (the phi's value from inside)
        for (const Inst &I : body)
            if (I.op == "add" && I.parts.size() == 2 && first_value(I.parts[0], M) == iv && trim(I.parts[1]) == "1" &&
                L.body[I.blk])
                next = I.res;
        std::map<std::string, int> id;
        for (int b = 0; b < n; ++b) id[blk_name[b]] = b;
        bool found = false;
        for (const Inst &B : body) {
            if (B.op != "br" || !L.body[B.blk]) continue;
            const auto lab = labels_in(B.text);
            if (lab.size() != 2 || !id.count(lab[0]) || !id.count(lab[1])) continue;
            const bool out0 = !L.body[id[lab[0]]], out1 = !L.body[id[lab[1]]];
            if (out0 == out1) continue;
            bool every = true;  // the test's block dominates every latch
            for (int t = 0; t < n; ++t)
                if (L.body[t])
                    for (int h : succ_[t])
                        if (h == L.header && !dom_[t][B.blk]) every = false;
            if (!every) continue;
            auto c = def.find(first_value(B.text, M));
            if (c == def.end() || c->second->op != "icmp" || c->second->parts.size() != 2) continue;
            const Inst &C = *c->second;
            std::string x = first_value(C.parts[0], M), y = C.parts[1], p = C.pred;
            // the counter on the left: swap a bound-first test
            if (x != iv && (x.empty() || x != next)) {
                x = first_value(C.parts[1], M), y = C.parts[0];
                static const std::map<std::string, std::string> kSwap = {
                    {"eq", "eq"}, {"ne", "ne"}, {"ult", "ugt"}, {"ugt", "ult"}, {"ule", "uge"}, {"uge", "ule"},
                    {"slt", "sgt"}, {"sgt", "slt"}, {"sle", "sge"}, {"sge", "sle"}};
                auto s = kSwap.find(p);
                if (s == kSwap.end()) continue;
                p = s->second;
            }
            if (x != iv && (x.empty() || x != next)) continue;
            // bounds must not change inside the loop
            const std::string yt = first_value(y, M);
            if (!yt.empty()) {
                auto yd = def.find(yt);
                if (yd != def.end() && L.body[yd->second->blk]) continue;
            }
            int64_t bmax;
            if (!int_max(y, &bmax)) continue;
            // the loop leaves when the counter reaches the bound: exit on
            // eq / uge / sge, stay on ne / ult / slt
            const bool exit_on_true = out0;
            const bool reach = exit_on_true ? (p == "eq" || p == "uge" || p == "sge")
                                            : (p == "ne" || p == "ult" || p == "slt");
            if (!reach) continue;
            // the IV before the test is at most bound - 1 when the increment
            // is compared, bound when the IV itself is (its last value runs the
            // code before the test)
            const int64_t m = x == next ? bmax - 1 : bmax;
            *hi = found ? std::min(*hi, m) : m;
            found = true;
        }
        return found;
    }
    // the range of an integer index operand: a literal, or a loop's canonical
    // IV (through zext / sext) with the bound its exit test sets
    bool index_range(const std::string &operand, int64_t *lo, int64_t *hi) const {
        int64_t c;
        if (int_literal(operand, &c)) return *lo = *hi = c, true;
        if (!loops_ok_) return false;
        std::string tok = first_value(operand, M);
        for (int hop = 0; hop < 2 && !tok.empty(); ++hop) {
            auto d = def.find(tok);
            if (d == def.end()) return false;
            if (d->second->op != "zext" && d->second->op != "sext") break;
            tok = first_value(d->second->text, M);
        }
        const int li = iv_loop(tok);
        int64_t m;
        if (li < 0 || !iv_max(tok, li, &m) || m < 0) return false;
        *lo = 0, *hi = m;
        return true;
    }

    // the loop whose canonical IV `tok` is (through zext / sext), or -1
    int iv_loop(std::string tok) const {
        for (int hop = 0; hop < 2; ++hop) {
            auto d = def.find(tok);
            if (d == def.end()) return -1;
            const Inst &I = *d->second;
            if (I.op == "zext" || I.op == "sext") {
                tok = first_value(I.text, M);
                continue;
            }
            if (I.op != "phi") return -1;
            // an i8 / i16 counter can wrap inside one run of its loop (distinct
            // values only up to 2^N iterations): i32 and i64 only
            if (!starts_with(I.text, "i32 ") && !starts_with(I.text, "i64 ")) return -1;
            int li = -1;
            for (size_t k = 0; k < loops_.size(); ++k)
                if (loops_[k].header == I.blk) li = (int)k;
            if (li < 0) return -1;
            // [ value, %block ], ...: 0 from outside the loop, tok + 1 from inside
            bool zero_in = false, step_in = false;
            const size_t lb = I.text.find('[');
            if (lb == std::string::npos) return -1;
            for (const auto &pp : split_top(I.text.substr(lb))) {
                const size_t a = pp.find('['), b = pp.rfind(']');
                if (a == std::string::npos || b == std::string::npos || b <= a) return -1;
                const auto two = split_top(pp.substr(a + 1, b - a - 1));
                if (two.size() != 2) return -1;
                int from = -1;
                for (size_t q = 0; q < blk_name.size(); ++q)
                    if (blk_name[q] == two[1]) from = (int)q;
                if (from < 0) return -1;
                if (!loops_[li].body[from]) {
                    if (two[0] != "0" || zero_in) return -1;
                    zero_in = true;
                } else {
                    auto n = def.find(two[0]);
                    if (n == def.end() || n->second->op != "add" || n->second->parts.size() != 2) return -1;
                    const std::string x0 = first_value(n->second->parts[0], M);
                    const std::string one = trim(n->second->parts[1]);
                    if (x0 != tok || one != "1") return -1;
                    step_in = true;
                }
            }
            return zero_in && step_in ? li : -1;
        }
        return -1;
    }

    void check_gain_table() {
        std::string why;
        auto refuse = [&](const std::string &w) {
            if (why.empty()) why = w;
        };
        if (!table_breakers.empty()) refuse(*table_breakers.begin());
        if (why.empty() && !build_loops(&why)) {}
        struct StoreAt {
            int chan_const = -1, chan_loop = -1, samp_loop = -1;
        };
        std::vector<StoreAt> seen;
        for (const Inst &I : body) {
            if (!why.empty()) break;
            if (I.op != "store" || I.parts.size() < 2) continue;
            const std::string ptr = first_value(I.parts[1], M);
            if (!(get(ptr).org & O_BUF)) continue;
            if (!starts_with(I.parts[0], "float ")) { refuse("a block store that is not one float"); break; }
            // the value: x * G with x loaded from this address, G free of samples
            const std::string v = first_value(I.parts[0], M);
            auto d = def.find(v);
            if (v.empty() || d == def.end() || d->second->op != "fmul" || d->second->parts.size() != 2) {
                refuse("a block store that is not a product");
                break;
            }
            std::string g_tok;
            bool have_x = false;
            for (int k = 0; k < 2; ++k) {
                const std::string t = first_value(d->second->parts[k], M);
                auto ld = def.find(t);
                if (!have_x && !t.empty() && ld != def.end() && ld->second->op == "load" &&
                    ld->second->parts.size() >= 2 && first_value(ld->second->parts[1], M) == ptr) {
                    have_x = true;
                    g_tok = first_value(d->second->parts[1 - k], M);
                }
            }
            if (!have_x) { refuse("a block store of a product that is not x * G at its own address"); break; }
            if (!g_tok.empty() && (get(g_tok).data & (D_IN | D_ADDR))) { refuse("a gain that depends on a sample"); break; }
            // the address: getelementptr float, (load of the channel's pointer), sample index
            auto gp = def.find(ptr);
            if (gp == def.end() || gp->second->op != "getelementptr" || gp->second->parts.size() != 3 ||
                trim(gp->second->parts[0]) != "float") {
                refuse("a block address that is not row[index]");
                break;
            }
            StoreAt sa;
            sa.samp_loop = iv_loop(first_value(gp->second->parts[2], M));
            if (sa.samp_loop < 0) { refuse("a sample index that is not a loop's induction variable"); break; }
            const std::string row = first_value(gp->second->parts[1], M);
            auto rl = def.find(row);
            if (rl == def.end() || rl->second->op != "load" || rl->second->parts.size() < 2) {
                refuse("a row pointer not read from the pointer table");
                break;
            }
            const std::string tp = first_value(rl->second->parts[1], M);
            if (args.size() == 6 && tp == args[2]) {
                sa.chan_const = 0;
            } else {
                auto tg = def.find(tp);
                if (tg == def.end() || tg->second->op != "getelementptr" || tg->second->parts.size() != 3 ||
                    first_value(tg->second->parts[1], M) != args[2]) {
                    refuse("a row pointer not read from the pointer table");
                    break;
                }
                const std::string et = trim(tg->second->parts[0]);
                std::string ix = trim(tg->second->parts[2]);
                const size_t sp = ix.find(' ');
                const std::string ixv = sp == std::string::npos ? ix : trim(ix.substr(sp + 1));
                char *end = nullptr;
                const long long k = std::strtoll(ixv.c_str(), &end, 10);
                if (end && *end == 0 && !ixv.empty() && ixv[0] != '%') {
                    const long long esz = et == "ptr" ? 8 : et == "i8" ? 1 : 0;
                    if (!esz || k < 0 || (k * (esz) % 8) != 0) { refuse("an unparsed channel index"); break; }
                    sa.chan_const = (int)(k * esz / 8);
                } else if (et == "ptr") {
                    sa.chan_loop = iv_loop(first_value(ix, M));
                    if (sa.chan_loop < 0) { refuse("a channel index that is not a loop's induction variable"); break; }
                } else {
                    refuse("an unparsed channel index");
                    break;
                }
            }
            if (sa.chan_loop == sa.samp_loop) { refuse("channel and sample from one loop"); break; }
            // inside exactly the loops its address uses
            for (size_t li = 0; li < loops_.size(); ++li) {
                const bool in = loops_[li].body[I.blk];
                const bool used = (int)li == sa.samp_loop || (int)li == sa.chan_loop;
                if (in != used) {
                    refuse(in ? "a block store inside a loop its address does not use"
                              : "a block store outside its index's loop");
                    break;
                }
            }
            for (const StoreAt &o : seen)
                if (o.chan_loop >= 0 || sa.chan_loop >= 0 || o.chan_const == sa.chan_const)
                    refuse("two block stores that may hit one element");
            seen.push_back(sa);
        }
        f.gain_table_form = why.empty() && !f.input_control;
        if (!f.gain_table_form) f.table_why = why.empty() ? "the stored samples depend on a sample" : why;
    }

    // canonical text of a call-invariant value (an operand part or a token)
    std::string canon_tok(const std::string &tok, int depth) {
        if (depth > 48) return "?";
        if (tok[0] == '@') return tok;
        for (size_t i = 0; i < args.size(); ++i)
            if (args[i] == tok) return "arg" + std::to_string(i);
        auto m = canon_memo.find(tok);
        if (m != canon_memo.end()) return m->second;
        auto d = def.find(tok);
        if (d == def.end()) return "?";
        const Inst &I = *d->second;
        if (I.op == "phi") return "?";
        std::string c = I.op + "(";
        for (const auto &p : I.parts)
            if (p.empty() || p[0] != '!') c += canon_part(p, depth + 1) + ",";  // (metadata dropped)
        c += ")";
        canon_memo[tok] = c;
        return c;
    }
    std::string canon_part(const std::string &part, int depth) {
        std::string out;
        const auto toks = values_in(part, M);
        size_t pos = 0;
        for (const auto &t : toks) {
            const size_t at = part.find(t, pos);
            if (at == std::string::npos) break;
            out += part.substr(pos, at - pos) + "{" + canon_tok(t, depth) + "}";
            pos = at + t.size();
        }
        return out + part.substr(pos);
    }

    void check_gain() {
        std::string g_all;
        int stores = 0;
        for (const Inst &I : body) {
            if (I.op != "store" || I.parts.size() < 2) continue;
            const std::string ptr = first_value(I.parts[1], M);
            if (!(get(ptr).org & O_BUF)) continue;
            ++stores;
            auto fail_gain = [&](const std::string &w) { gain_breakers.insert(w); };
            if (!starts_with(I.parts[0], "float ")) { fail_gain("a block store that is not one float"); continue; }
            if (get(ptr).data & (D_IN | D_ADDR)) { fail_gain("an input-dependent block address"); continue; }
            const std::string v = first_value(I.parts[0], M);
            auto d = def.find(v);
            if (v.empty() || d == def.end() || d->second->op != "fmul") {
                fail_gain("a block store that is not a product");
                continue;
            }
            const Inst &mul = *d->second;
            const auto ops = values_in(mul.text, M);
            std::string load_tok, g_part;
            const auto mparts = split_top(mul.text);
            if (mparts.size() != 2) { fail_gain("an unparsed product"); continue; }
            for (int k = 0; k < 2; ++k) {
                const std::string t = first_value(mparts[k], M);
                auto ld = def.find(t);
                if (load_tok.empty() && !t.empty() && ld != def.end() && ld->second->op == "load" &&
                    ld->second->parts.size() >= 2 && first_value(ld->second->parts[1], M) == ptr) {
                    load_tok = t;
                    g_part = mparts[1 - k];
                }
            }
            if (load_tok.empty()) { fail_gain("a block store of a product that is not x * g at its own address"); continue; }
            const std::string gt = first_value(g_part, M);
            if (!gt.empty() && (get(gt).data & (D_IN | D_VAR | D_ADDR))) {
                fail_gain("a gain that varies within the call");
                continue;
            }
            // the type word of the first operand part ("float %x") is dropped
            std::string gp = g_part;
            if (starts_with(gp, "float ")) gp = gp.substr(6);
            const std::string c = canon_part(gp, 0);
            if (c.find('?') != std::string::npos) { fail_gain("a gain outside the canonical forms"); continue; }
            if (g_all.empty()) {
                g_all = c;
                if (!gain_source(gp, gt)) fail_gain("a gain not read directly from Parameters / State / a constant");
            } else if (g_all != c) {
                fail_gain("two different gains");
            }
        }
        // (no block store at all: the identity, g = 1)
        f.gain_form = gain_breakers.empty();
        if (f.gain_form && !stores) {
            f.gain_src = 'K';
            f.gain_bits = 0x3f800000u;
        }
        if (f.gain_form) f.gain_expr = stores ? g_all : "1 (no block store)";
        else if (f.why.empty()) f.why = "not a gain: " + *gain_breakers.begin();
    }

    // Where g comes from, so that the host knows its value without running
    // the callback: a float constant, the sample rate argument, or a float
    // load at a constant byte offset of Parameters / State.
    bool gain_source(const std::string &gp, const std::string &gt) {
        if (gt.empty()) {  // a constant: LLVM writes floats as decimal or as the f64 bits in hex
            double v = 0.0;
            if (starts_with(gp, "0x") && gp.size() == 18) {
                const unsigned long long b = std::strtoull(gp.c_str() + 2, nullptr, 16);
                std::memcpy(&v, &b, 8);
            } else {
                char *e = nullptr;
                v = std::strtod(gp.c_str(), &e);
                if (!e || e == gp.c_str()) return false;
            }
            const float fv = (float)v;
            if ((double)fv != v) return false;
            f.gain_src = 'K';
            std::memcpy(&f.gain_bits, &fv, 4);
            return true;
        }
        if (args.size() == 6 && gt == args[5]) {
            f.gain_src = 'R';
            return true;
        }
        auto d = def.find(gt);
        if (d == def.end() || d->second->op != "load" || d->second->parts.size() < 2 ||
            d->second->parts[0] != "float")
            return false;
        const std::string p = first_value(d->second->parts[1], M);
        uint64_t off = 0;
        std::string base = p;
        auto g = def.find(p);
        if (g != def.end() && g->second->op == "getelementptr") {
            const Inst &G = *g->second;
            if (G.parts.size() != 3) return false;
            const std::string &et = G.parts[0];
            const uint64_t esz = et == "i8" ? 1 : (et == "float" || et == "i32") ? 4 : (et == "double" || et == "i64") ? 8 : 0;
            if (!esz || !values_in(G.parts[2], M).empty()) return false;
            const size_t sp = G.parts[2].find(' ');
            if (sp == std::string::npos) return false;
            char *e = nullptr;
            const long long k = std::strtoll(G.parts[2].c_str() + sp + 1, &e, 10);
            if (k < 0 || k > (1 << 20)) return false;
            off = (uint64_t)k * esz;
            base = first_value(G.parts[1], M);
        }
        if (args.size() != 6 || (base != args[0] && base != args[1])) return false;
        f.gain_src = base == args[0] ? 'P' : 'S';
        f.gain_off = (uint32_t)off;
        return true;
    }
};

Module scan_module(const std::string &ir) {
    Module M;
    std::istringstream in(ir);
    std::string line;
    while (std::getline(in, line)) {
        if (starts_with(line, "%")) {
            const size_t e = line.find(" = type ");
            if (e != std::string::npos) M.types.insert(line.substr(0, e));
        } else if (starts_with(line, "@")) {
            const size_t e = line.find(" = ");
            if (e == std::string::npos) continue;
            const std::string name = line.substr(0, e);
            std::istringstream w(line.substr(e + 3));
            std::string tok;
            bool is_const = false, found = false;
            while (w >> tok) {
                if (tok == "constant") { is_const = true; found = true; break; }
                if (tok == "global") { found = true; break; }
            }
            if (found) M.global_const[name] = is_const;
        } else if (starts_with(line, "attributes #")) {
            const size_t e = line.find(" = ");
            if (e != std::string::npos) M.attr_groups[line.substr(11, e - 11)] = line.substr(e + 3);
        } else if (starts_with(line, "define ") || starts_with(line, "declare ")) {
            const size_t at = line.find('@');
            if (at == std::string::npos) continue;
            size_t e = at + 1;
            while (e < line.size() && ident_char(line[e])) ++e;
            M.fn_groups[line.substr(at, e - at)] = groups_after_args(line, line.find('(', e));
        }
    }
    for (auto &fg : M.fn_groups) {
        std::string t;
        for (const auto &g : fg.second) {
            auto it = M.attr_groups.find(g);
            if (it != M.attr_groups.end()) t += " " + it->second;
        }
        M.fn_attrs[fg.first] = t;
    }
    return M;
}

}  // namespace

Facts analyze(const std::string &ir, const char *fn) {
    Module M = scan_module(ir);
    Analysis A(M);
    std::istringstream in(ir);
    std::string line;
    const std::string want = std::string("@") + fn + "(";
    bool inside = false;
    std::string pending;  // a switch spanning lines
    A.blk_name.push_back("");  // the entry block (no label)
    while (std::getline(in, line)) {
        if (!inside) {
            if (starts_with(line, "define ") && line.find(want) != std::string::npos) {
                inside = true;
                const size_t open = line.find(want) + want.size() - 1;
                int depth = 0;
                size_t k = open;
                for (; k < line.size(); ++k) {
                    if (line[k] == '(') ++depth;
                    else if (line[k] == ')' && --depth == 0) break;
                }
                for (const auto &p : split_top(line.substr(open + 1, k - open - 1))) {
                    // the parameter's name: its last %token (the type before it
                    // may itself be a %type)
                    const size_t at = p.rfind('%');
                    std::string name;
                    if (at != std::string::npos) {
                        size_t e = at + 1;
                        while (e < p.size() && ident_char(p[e])) ++e;
                        name = p.substr(at, e - at);
                    }
                    A.args.push_back(name.size() > 1 ? name : std::string());
                }
            }
            continue;
        }
        std::string s = trim(strip_comment(line));
        if (s == "}") break;
        if (s.empty()) continue;
        if (!pending.empty()) {
            pending += " " + s;
            if (s.find(']') == std::string::npos) continue;
            s = pending;
            pending.clear();
        } else if (starts_with(s, "switch ") && s.find(']') == std::string::npos) {
            pending = s;
            continue;
        }
        if (s.back() == ':' && s.find(' ') == std::string::npos) {  // a block label
            A.blk_name.push_back("%" + s.substr(0, s.size() - 1));
            continue;
        }
        Inst I;
        std::string rest = s;
        if (s[0] == '%') {
            const size_t e = s.find(" = ");
            if (e == std::string::npos) continue;
            I.res = s.substr(0, e);
            rest = s.substr(e + 3);
        }
        std::istringstream w(rest);
        std::string word;
        w >> word;
        while (word == "tail" || word == "musttail" || word == "notail") w >> word;
        I.op = word;
        std::string tail;
        std::getline(w, tail);
        tail = trim(tail);
        // fast-math and wrap flags before the operands
        static const std::set<std::string> kFlags = {"nnan", "ninf", "nsz", "arcp", "contract", "afn", "reassoc",
                                                     "fast", "nuw", "nsw", "nusw", "exact", "disjoint", "nneg", "samesign",
                                                     "volatile", "inbounds", "inrange"};
        for (;;) {
            const size_t sp = tail.find(' ');
            if (sp == std::string::npos || !kFlags.count(tail.substr(0, sp))) break;
            if (tail.compare(0, sp, "nuw") == 0) I.nuw = true;
            tail = trim(tail.substr(sp + 1));
        }
        if (I.op == "icmp" || I.op == "fcmp") {  // the predicate
            const size_t sp = tail.find(' ');
            if (sp != std::string::npos) I.pred = tail.substr(0, sp), tail = trim(tail.substr(sp + 1));
        }
        I.text = tail;
        I.parts = split_top(tail);
        I.blk = (int)A.blk_name.size() - 1;
        A.body.push_back(I);
    }
    if (!inside) {
        A.f.why = std::string("no function ") + fn + " in the IR";
        return A.f;
    }
    if (A.args.size() != 6) {
        A.f.why = "the analysis kernel does not have six parameters";
        return A.f;
    }
    for (const auto &a : A.args)
        if (a.empty()) {
            A.f.why = "unparsed parameters of the analysis kernel";
            return A.f;
        }
    // the function's own names: a numbered value shadows a numbered type
    for (const auto &a : A.args) M.locals.insert(a);
    for (const Inst &I : A.body)
        if (!I.res.empty()) M.locals.insert(I.res);
    for (const Inst &I : A.body)
        if (!I.res.empty()) A.def[I.res] = &I;
    A.val[A.args[0]].org = O_PRM;
    A.val[A.args[1]].org = O_STA;
    A.val[A.args[1]].soff = 0;
    A.val[A.args[2]].org = O_TBL;
    A.val[A.args[1]].shi = 0;
    // the loops first: the ranges of their counters bound State offsets
    {
        std::string why;
        (void)A.build_loops(&why);  // (irreducible: no ranges; check_gain_table says why)
    }
    bool settled = false;
    for (int it = 0; it < 64 && !settled; ++it) {
        bool grew = false;
        const uint32_t ld = A.loc_data, sd = A.sta_data, sa = A.sta_any;
        const auto sb = A.sta_byte, stl = A.sta_tail;
        const bool ws = A.f.writes_state;
        for (const Inst &I : A.body) grew |= A.step(I, false);
        settled = !grew && ld == A.loc_data && sd == A.sta_data && ws == A.f.writes_state && sa == A.sta_any &&
                  sb == A.sta_byte && stl == A.sta_tail;
    }
    // facts from values still growing would not be conservative
    if (!settled) A.stop("no fixpoint after 64 passes");
    for (const Inst &I : A.body) A.step(I, true);
    if (!A.fail.empty()) {
        A.f.why = A.fail;
        A.f.analyzed = false;
        A.f.gain_form = false;
        return A.f;
    }
    A.f.analyzed = true;
    A.f.state_reads_block = A.f.writes_state && ((A.sta_data & D_IN) || A.f.input_control);
    // the State's words by dependence on the block: a word is block-dependent
    // when a store that may hit it carries a block sample (a store of unknown
    // offset, or with a lower bound alone, may hit any word / every word from
    // its bound on); with a branch on a sample, every word is
    if (A.f.state_reads_block && !A.f.input_control && !(A.sta_any & D_IN)) {
        std::set<int64_t> dep, written;
        int64_t dep_from = kShiInf, written_from = kShiInf;  // the tails' first words
        for (const auto &e : A.sta_tail) {
            written_from = std::min(written_from, e.first / 4);
            if (e.second & D_IN) dep_from = std::min(dep_from, e.first / 4);
        }
        for (const auto &e : A.sta_byte) {
            if (e.first / 4 >= dep_from) continue;
            written.insert(e.first / 4);
            if (e.second & D_IN) dep.insert(e.first / 4);
        }
        bool indep_written = written_from < dep_from;
        for (int64_t w : written) indep_written = indep_written || !dep.count(w);
        const bool any_dep = !dep.empty() || dep_from != kShiInf;
        const int64_t last = dep_from != kShiInf ? dep_from : dep.empty() ? 0 : *dep.rbegin();
        if (indep_written && any_dep && last < 256) {
            A.f.state_dep_words.assign(dep.begin(), dep.end());
            // every word from dep_from on: one entry -(dep_from + 2)
            if (dep_from != kShiInf) A.f.state_dep_words.push_back(-(dep_from + 2));
            A.f.state_split = true;
        }
    }
    A.check_gain();
    A.check_gain_table();
    if (A.f.input_control && A.f.gain_form) {
        A.f.gain_form = false;
        A.f.why = "not a gain: which samples are stored depends on a sample (a branch or an address)";
    }
    return A.f;
}

// ---------------------------------------------------------------------------
// comgr: plugin TU -> optimised IR text
// ---------------------------------------------------------------------------
namespace {

struct Comgr {
    amd_comgr_data_set_t in{}, out{};
    amd_comgr_action_info_t ai{};
    bool have_in = false, have_out = false, have_ai = false;
    ~Comgr() {
        if (have_ai) amd_comgr_destroy_action_info(ai);
        if (have_out) amd_comgr_destroy_data_set(out);
        if (have_in) amd_comgr_destroy_data_set(in);
    }
};

bool add_data(amd_comgr_data_set_t set, amd_comgr_data_kind_t k, const std::string &txt, const char *name) {
    amd_comgr_data_t d;
    if (amd_comgr_create_data(k, &d)) return false;
    const bool ok = !amd_comgr_set_data(d, txt.size(), txt.data()) && !amd_comgr_set_data_name(d, name) &&
                    !amd_comgr_data_set_add(set, d);
    amd_comgr_release_data(d);
    return ok;
}

bool get_data(amd_comgr_data_set_t set, amd_comgr_data_kind_t k, std::string *out) {
    size_t n = 0;
    if (amd_comgr_action_data_count(set, k, &n) || n == 0) return false;
    amd_comgr_data_t d;
    if (amd_comgr_action_data_get_data(set, k, 0, &d)) return false;
    size_t sz = 0;
    bool ok = !amd_comgr_get_data(d, &sz, nullptr);
    if (ok) {
        out->assign(sz, '\0');
        ok = !amd_comgr_get_data(d, &sz, &(*out)[0]);
    }
    amd_comgr_release_data(d);
    return ok;
}

// hiprtc's runtime header (libhiprtc-builtins), which hiprtc pre-includes
bool hiprtc_runtime_header(std::string *out) {
    static std::string text;
    static bool ok = false;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("libhiprtc-builtins.so.7", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libhiprtc-builtins.so", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            const char *hdr = (const char *)dlsym(h, "__hipRTC_header");
            const unsigned *sz = (const unsigned *)dlsym(h, "__hipRTC_header_size");
            if (hdr && sz) {
                text.assign(hdr, *sz);
                ok = true;
            }
        }
    });
    *out = text;
    return ok;
}

}  // namespace

int compile_to_ir(const std::string &tu, const std::vector<std::pair<std::string, std::string>> &includes,
                  const std::vector<std::string> &options, std::string *ir, std::string *log) {
    std::string rt;
    if (!hiprtc_runtime_header(&rt)) {
        *log = "libhiprtc-builtins (the hiprtc runtime header) not found";
        return -1;
    }
    Comgr c;
    if (amd_comgr_create_data_set(&c.in)) return *log = "comgr: data set", -1;
    c.have_in = true;
    if (amd_comgr_create_data_set(&c.out)) return *log = "comgr: data set", -1;
    c.have_out = true;
    if (!add_data(c.in, AMD_COMGR_DATA_KIND_SOURCE, tu, "dspb_proof.hip") ||
        !add_data(c.in, AMD_COMGR_DATA_KIND_INCLUDE, rt, "hiprtc_runtime.h"))
        return *log = "comgr: input", -1;
    for (const auto &inc : includes)
        if (!add_data(c.in, AMD_COMGR_DATA_KIND_INCLUDE, inc.second, inc.first.c_str()))
            return *log = "comgr: include " + inc.first, -1;
    if (amd_comgr_create_action_info(&c.ai)) return *log = "comgr: action info", -1;
    c.have_ai = true;
    std::vector<const char *> opts = {"-S", "-emit-llvm", "-nogpuinc", "-D__HIPCC_RTC__", "-include", "hiprtc_runtime.h"};
    for (const auto &o : options) opts.push_back(o.c_str());
    if (amd_comgr_action_info_set_language(c.ai, AMD_COMGR_LANGUAGE_HIP) ||
        amd_comgr_action_info_set_isa_name(c.ai, "amdgcn-amd-amdhsa--gfx950") ||
        amd_comgr_action_info_set_option_list(c.ai, opts.data(), opts.size()) ||
        amd_comgr_action_info_set_logging(c.ai, true))
        return *log = "comgr: options", -1;
    const amd_comgr_status_t st =
        amd_comgr_do_action(AMD_COMGR_ACTION_COMPILE_SOURCE_WITH_DEVICE_LIBS_TO_BC, c.ai, c.in, c.out);
    std::string lg;
    get_data(c.out, AMD_COMGR_DATA_KIND_LOG, &lg);
    *log = lg;
    if (st != AMD_COMGR_STATUS_SUCCESS || !get_data(c.out, AMD_COMGR_DATA_KIND_BC, ir)) {
        if (log->empty()) *log = "comgr: compile failed";
        return -1;
    }
    if (ir->compare(0, 1, ";") != 0 && ir->find("define ") == std::string::npos) {
        *log = "comgr returned no IR text";
        return -1;
    }
    return 0;
}

// ---------------------------------------------------------------------------
int strip_chain_block_stores(std::string *ir, const char *prefix) {
    std::istringstream in(*ir);
    std::vector<std::string> lines;
    for (std::string l; std::getline(in, l);) lines.push_back(l);
    auto name_at = [](const std::string &l, size_t p) {  // %name starting at p
        size_t e = p + 1;
        while (e < l.size() && (std::isalnum((unsigned char)l[e]) || l[e] == '_' || l[e] == '.' || l[e] == '-')) ++e;
        return l.substr(p, e - p);
    };
    int dropped = 0;
    std::vector<char> keep(lines.size(), 1);
    for (size_t i = 0; i < lines.size(); ++i) {
        if (lines[i].compare(0, 6, "define") != 0 || lines[i].find(prefix) == std::string::npos) continue;
        size_t end = i;
        while (end < lines.size() && lines[end] != "}") ++end;
        std::set<std::string> blk;
        for (size_t k = i; k < end; ++k) {
            const std::string &l = lines[k];
            const size_t p = l.find("%dspb_chain_blk");
            if (p != std::string::npos && l.find(" = alloca ") != std::string::npos && l.find('%') == p)
                blk.insert(name_at(l, p));
        }
        for (bool grew = true; grew && !blk.empty();) {  // pointers derived from the block
            grew = false;
            for (size_t k = i; k < end; ++k) {
                const std::string &l = lines[k];
                const size_t eq = l.find(" = ");
                if (eq == std::string::npos) continue;
                const size_t p0 = l.find('%');
                if (p0 == std::string::npos || p0 > eq) continue;
                const std::string res = name_at(l, p0);
                if (blk.count(res)) continue;
                const std::string rhs = l.substr(eq + 3);
                if (rhs.compare(0, 13, "getelementptr") && rhs.compare(0, 3, "phi") && rhs.compare(0, 6, "select") &&
                    rhs.compare(0, 13, "addrspacecast") && rhs.compare(0, 7, "bitcast"))
                    continue;
                for (size_t q = rhs.find('%'); q != std::string::npos; q = rhs.find('%', q + 1))
                    if (blk.count(name_at(rhs, q))) {
                        blk.insert(res);
                        grew = true;
                        break;
                    }
            }
        }
        for (size_t k = i; k < end && !blk.empty(); ++k) {
            const std::string &l = lines[k];
            const size_t st = l.find_first_not_of(' ');
            if (st == std::string::npos || l.compare(st, 6, "store ") != 0) continue;
            // store [atomic] [volatile] <ty> <value>, ptr addrspace(5) <address>[, ...]: the
            // address is the operand after the first comma outside brackets
            size_t v = st + 6;
            for (const char *kw : {"atomic ", "volatile "})
                if (l.compare(v, std::strlen(kw), kw) == 0) v += std::strlen(kw);
            size_t comma = std::string::npos;
            int depth = 0;
            for (size_t q = v; q < l.size() && comma == std::string::npos; ++q) {
                const char ch = l[q];
                if (ch == '(' || ch == '<' || ch == '[' || ch == '{') ++depth;
                else if (ch == ')' || ch == '>' || ch == ']' || ch == '}') --depth;
                else if (ch == ',' && depth == 0) comma = q;
            }
            if (comma == std::string::npos) return -1;  // not a store this parser understands
            const std::string value = l.substr(v, comma - v);
            // a pointer derived from the block stored anywhere: outside the
            // model (the analysis refuses it too); keep the hiprtc code
            for (size_t q = value.find('%'); q != std::string::npos; q = value.find('%', q + 1))
                if (blk.count(name_at(value, q)) && value.compare(0, 4, "ptr ") == 0) return -1;
            size_t a = l.find_first_not_of(' ', comma + 1);
            static const char kAddr[] = "ptr addrspace(5) %";
            if (a == std::string::npos || l.compare(a, sizeof kAddr - 1, kAddr) != 0) continue;
            if (!blk.count(name_at(l, a + sizeof kAddr - 2))) continue;
            if (l.find("!nontemporal", comma) != std::string::npos) continue;  // the input's copy into the block
            if (value.compare(0, 4, "ptr ") == 0) return -1;
            keep[k] = 0;
            ++dropped;
        }
        i = end;
    }
    if (dropped) {
        std::string o;
        o.reserve(ir->size());
        for (size_t i = 0; i < lines.size(); ++i)
            if (keep[i]) o += lines[i], o += '\n';
        *ir = o;
    }
    return dropped;
}

int codegen_ir(const std::string &ir, const std::vector<std::string> &options, std::string *code, std::string *log) {
    Comgr c;
    amd_comgr_data_set_t exe{};
    if (amd_comgr_create_data_set(&c.in)) return *log = "comgr: data set", -1;
    c.have_in = true;
    if (amd_comgr_create_data_set(&c.out)) return *log = "comgr: data set", -1;
    c.have_out = true;
    if (amd_comgr_create_data_set(&exe)) return *log = "comgr: data set", -1;
    struct Drop {
        amd_comgr_data_set_t s;
        ~Drop() { amd_comgr_destroy_data_set(s); }
    } drop{exe};
    if (!add_data(c.in, AMD_COMGR_DATA_KIND_BC, ir, "dspb_chain.ll")) return *log = "comgr: input", -1;
    if (amd_comgr_create_action_info(&c.ai)) return *log = "comgr: action info", -1;
    c.have_ai = true;
    std::vector<const char *> opts;
    for (const auto &o : options) opts.push_back(o.c_str());
    if (amd_comgr_action_info_set_isa_name(c.ai, "amdgcn-amd-amdhsa--gfx950") ||
        amd_comgr_action_info_set_option_list(c.ai, opts.data(), opts.size()) ||
        amd_comgr_action_info_set_logging(c.ai, true))
        return *log = "comgr: options", -1;
    if (amd_comgr_do_action(AMD_COMGR_ACTION_CODEGEN_BC_TO_RELOCATABLE, c.ai, c.in, c.out) ||
        amd_comgr_do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, c.ai, c.out, exe)) {
        get_data(c.out, AMD_COMGR_DATA_KIND_LOG, log);
        if (log->empty()) *log = "comgr: codegen failed";
        return -1;
    }
    if (!get_data(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, code) || code->empty()) return *log = "comgr: no code", -1;
    return 0;
}

// ---------------------------------------------------------------------------
std::string encode(const Facts &f) {
    auto clean = [](std::string s) {
        for (char &c : s)
            if (c == '\n' || c == '\0') c = ' ';
        return s;
    };
    std::string s = "dspb_facts 1\n";
    s += "analyzed=" + std::to_string(f.analyzed) + "\n";
    s += "reads_block=" + std::to_string(f.reads_block) + "\n";
    s += "writes_state=" + std::to_string(f.writes_state) + "\n";
    s += "input_control=" + std::to_string(f.input_control) + "\n";
    s += "gain_form=" + std::to_string(f.gain_form) + "\n";
    s += "gain=" + clean(f.gain_expr.substr(0, 512)) + "\n";
    s += "gain_src=" + std::string(f.gain_src ? 1 : 0, f.gain_src) + "\n";
    s += "gain_off=" + std::to_string(f.gain_off) + "\n";
    s += "gain_bits=" + std::to_string(f.gain_bits) + "\n";
    s += "gain_table_form=" + std::to_string(f.gain_table_form) + "\n";
    s += "table_why=" + clean(f.table_why.substr(0, 256)) + "\n";
    s += "state_reads_block=" + std::to_string(f.state_reads_block) + "\n";
    s += "state_split=" + std::to_string(f.state_split) + "\n";
    s += "state_dep_words=";
    for (size_t i = 0; i < f.state_dep_words.size(); ++i) s += (i ? "," : "") + std::to_string(f.state_dep_words[i]);
    s += "\n";
    s += "why=" + clean(f.why.substr(0, 512)) + "\n";
    return s;
}

bool decode(const std::string &s, Facts *f) {
    *f = Facts{};
    std::istringstream in(s);
    std::string line;
    if (!std::getline(in, line) || line != "dspb_facts 1") return false;
    bool have_analyzed = false;
    while (std::getline(in, line)) {
        const size_t e = line.find('=');
        if (e == std::string::npos) continue;
        const std::string k = line.substr(0, e), v = line.substr(e + 1);
        if (k == "analyzed") f->analyzed = v == "1", have_analyzed = true;
        else if (k == "reads_block") f->reads_block = v == "1";
        else if (k == "writes_state") f->writes_state = v == "1";
        else if (k == "input_control") f->input_control = v == "1";
        else if (k == "gain_form") f->gain_form = v == "1";
        else if (k == "gain") f->gain_expr = v;
        else if (k == "gain_src") f->gain_src = v.empty() ? 0 : v[0];
        else if (k == "gain_off") f->gain_off = (uint32_t)std::strtoul(v.c_str(), nullptr, 10);
        else if (k == "gain_bits") f->gain_bits = (uint32_t)std::strtoul(v.c_str(), nullptr, 10);
        else if (k == "gain_table_form") f->gain_table_form = v == "1";
        else if (k == "table_why") f->table_why = v;
        else if (k == "state_reads_block") f->state_reads_block = v == "1";
        else if (k == "state_split") f->state_split = v == "1";
        else if (k == "state_dep_words") {
            f->state_dep_words.clear();
            for (size_t a = 0; a < v.size();) {
                size_t b = v.find(',', a);
                if (b == std::string::npos) b = v.size();
                if (b > a) f->state_dep_words.push_back(std::strtoll(v.substr(a, b - a).c_str(), nullptr, 10));
                a = b + 1;
            }
        }
        else if (k == "why") f->why = v;
    }
    return have_analyzed;
}

}  // namespace irp
}  // namespace dspb
