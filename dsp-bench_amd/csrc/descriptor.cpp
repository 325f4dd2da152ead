// descriptor.cpp -- the plugin parameter descriptor of a module (module.h,
// SURVEY 8 a8): what the reference's JIT reads from the plugin's AST
// (compiler.cpp:944-1164, parse_plugin_descriptor) rebuilt for a plugin
// compiled by hiprtc, plus the host-side marshalling of parameter values
// (plugin.cpp:121-171) and their normalisation (plugin.h:173-233).
//
// The reference walks the clang AST of `struct Parameters` and, for every
// field that carries an `annotate` attribute, records its name, its byte
// offset and the min / max / log / enumerators of the annotation.  hiprtc
// gives no AST, so the descriptor is built in two halves:
//
//   * text: a small scanner finds `struct Parameters { ... }` in the plugin
//     source, expands the annotation macros (plugin_header.h's INT_PARAM /
//     FLOAT_PARAM / FLOAT_PARAM_LOG / ENUM_PARAM, or the plugin's own
//     #defines of them, with # stringisation), and collects each annotated
//     field's name, annotation string and type spelling, and the enumerator
//     names of an Enum field's type;
//   * compiler: generated code appended to the translation unit lets the
//     device compiler itself evaluate everything layout-dependent --
//     sizeof / alignof of Parameters and State, __builtin_offsetof of every
//     field, whether the field is int, float or an enum, and the value of
//     every enumerator -- into a constant array, dspb_desc_blob.
//
// Both halves are stored in the code object (dspb_desc_blob, dspb_desc_text)
// and read back from its ELF symbol table on the host, so the descriptor of
// a code object needs no GPU.  The annotation is then validated with the
// reference's rules and error flags (errors.inc:1-19).
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "descriptor.hpp"

namespace dspb {
namespace desc {

namespace {

constexpr unsigned long long kMagic = 0x3145445342505344ull;  // "DSPBSDE1"
constexpr char kRecSep = '\x1e', kFieldSep = '\x1f';

bool ident_start(char c) { return std::isalpha((unsigned char)c) || c == '_'; }
bool ident_char(char c) { return std::isalnum((unsigned char)c) || c == '_'; }

// strip /* */ and // comments, keep string / char literals intact
std::string strip_comments(const std::string &s) {
    std::string o;
    o.reserve(s.size());
    for (size_t i = 0; i < s.size();) {
        if (s[i] == '"' || s[i] == '\'') {
            const char q = s[i];
            o += s[i++];
            while (i < s.size() && s[i] != q) {
                if (s[i] == '\\' && i + 1 < s.size()) o += s[i++];
                o += s[i++];
            }
            if (i < s.size()) o += s[i++];
        } else if (s.compare(i, 2, "//") == 0) {
            while (i < s.size() && s[i] != '\n') ++i;
        } else if (s.compare(i, 2, "/*") == 0) {
            const size_t e = s.find("*/", i + 2);
            i = e == std::string::npos ? s.size() : e + 2;
            o += ' ';
        } else {
            o += s[i++];
        }
    }
    return o;
}

struct Macro {
    bool function = false;
    std::vector<std::string> params;
    std::string body;
};

std::string trim(const std::string &s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

// whitespace runs -> one space, as # stringisation does
std::string collapse_ws(const std::string &s) {
    std::string o;
    bool ws = false;
    for (char c : trim(s)) {
        if (std::isspace((unsigned char)c)) {
            ws = true;
        } else {
            if (ws) o += ' ';
            ws = false;
            o += c;
        }
    }
    return o;
}

std::string stringize(const std::string &arg) {
    std::string o = "\"";
    for (char c : collapse_ws(arg)) {
        if (c == '"' || c == '\\') o += '\\';
        o += c;
    }
    return o + "\"";
}

// #define lines (with \-continuations), in order: later ones override
void collect_macros(const std::string &src, std::map<std::string, Macro> &out) {
    std::string s;
    for (size_t i = 0; i < src.size(); ++i) {  // join continuation lines
        if (src[i] == '\\' && i + 1 < src.size() && src[i + 1] == '\n') { ++i; continue; }
        s += src[i];
    }
    size_t pos = 0;
    while (pos < s.size()) {
        size_t e = s.find('\n', pos);
        if (e == std::string::npos) e = s.size();
        std::string line = trim(s.substr(pos, e - pos));
        pos = e + 1;
        if (line.empty() || line[0] != '#') continue;
        line = trim(line.substr(1));
        if (line.compare(0, 6, "define") != 0 || line.size() < 7 || !std::isspace((unsigned char)line[6]))
            continue;
        line = trim(line.substr(6));
        size_t n = 0;
        while (n < line.size() && ident_char(line[n])) ++n;
        if (n == 0) continue;
        Macro m;
        const std::string name = line.substr(0, n);
        if (n < line.size() && line[n] == '(') {  // function-like: no space before '('
            m.function = true;
            const size_t close = line.find(')', n);
            if (close == std::string::npos) continue;
            std::string plist = line.substr(n + 1, close - n - 1);
            size_t p0 = 0;
            while (p0 <= plist.size()) {
                size_t c = plist.find(',', p0);
                if (c == std::string::npos) c = plist.size();
                const std::string p = trim(plist.substr(p0, c - p0));
                if (!p.empty()) m.params.push_back(p);
                p0 = c + 1;
            }
            m.body = trim(line.substr(close + 1));
        } else {
            m.body = trim(line.substr(n));
        }
        out[name] = m;
    }
}

// split "a, (b, c), d" at top-level commas
std::vector<std::string> split_args(const std::string &s) {
    std::vector<std::string> out;
    int depth = 0;
    std::string cur;
    for (size_t i = 0; i < s.size(); ++i) {
        const char c = s[i];
        if (c == '"' || c == '\'') {
            const char q = c;
            cur += s[i++];
            while (i < s.size() && s[i] != q) {
                if (s[i] == '\\' && i + 1 < s.size()) cur += s[i++];
                cur += s[i++];
            }
            if (i < s.size()) cur += s[i];
            continue;
        }
        if (c == '(' || c == '[' || c == '{') ++depth;
        if (c == ')' || c == ']' || c == '}') --depth;
        if (c == ',' && depth == 0) {
            out.push_back(cur);
            cur.clear();
        } else {
            cur += c;
        }
    }
    out.push_back(cur);
    return out;
}

// one expansion pass over `s`; returns true when something was expanded
bool expand_once(std::string &s, const std::map<std::string, Macro> &macros) {
    std::string o;
    bool any = false;
    for (size_t i = 0; i < s.size();) {
        if (s[i] == '"') {  // copy string literals verbatim
            o += s[i++];
            while (i < s.size() && s[i] != '"') {
                if (s[i] == '\\' && i + 1 < s.size()) o += s[i++];
                o += s[i++];
            }
            if (i < s.size()) o += s[i++];
            continue;
        }
        if (!ident_start(s[i]) || (i > 0 && ident_char(s[i - 1]))) {
            o += s[i++];
            continue;
        }
        size_t j = i;
        while (j < s.size() && ident_char(s[j])) ++j;
        const std::string id = s.substr(i, j - i);
        auto it = macros.find(id);
        if (it == macros.end()) {
            o += id;
            i = j;
            continue;
        }
        const Macro &m = it->second;
        if (!m.function) {
            o += m.body;
            i = j;
            any = true;
            continue;
        }
        size_t k = j;
        while (k < s.size() && std::isspace((unsigned char)s[k])) ++k;
        if (k >= s.size() || s[k] != '(') {
            o += id;
            i = j;
            continue;
        }
        int depth = 0;
        size_t e = k;
        for (; e < s.size(); ++e) {
            if (s[e] == '(') ++depth;
            else if (s[e] == ')' && --depth == 0) break;
        }
        if (e >= s.size()) {
            o += id;
            i = j;
            continue;
        }
        std::vector<std::string> args = split_args(s.substr(k + 1, e - k - 1));
        // substitute parameters (and #parameter) in the body
        std::string b;
        const std::string &body = m.body;
        for (size_t p = 0; p < body.size();) {
            if (body[p] == '"') {
                b += body[p++];
                while (p < body.size() && body[p] != '"') {
                    if (body[p] == '\\' && p + 1 < body.size()) b += body[p++];
                    b += body[p++];
                }
                if (p < body.size()) b += body[p++];
                continue;
            }
            bool hash = false;
            size_t q = p;
            if (body[q] == '#' && !(q + 1 < body.size() && body[q + 1] == '#')) {
                hash = true;
                ++q;
                while (q < body.size() && std::isspace((unsigned char)body[q])) ++q;
            }
            if (q < body.size() && ident_start(body[q]) && (q == 0 || !ident_char(body[q - 1]) || hash)) {
                size_t r = q;
                while (r < body.size() && ident_char(body[r])) ++r;
                const std::string pid = body.substr(q, r - q);
                size_t idx = 0;
                for (; idx < m.params.size() && m.params[idx] != pid; ++idx) {
                }
                if (idx < m.params.size() && idx < args.size()) {
                    b += hash ? stringize(args[idx]) : trim(args[idx]);
                    p = r;
                    continue;
                }
                if (!hash) {
                    b += pid;
                    p = r;
                    continue;
                }
            }
            b += body[p++];
        }
        o += b;
        i = e + 1;
        any = true;
    }
    s = o;
    return any;
}

std::string expand(std::string s, const std::map<std::string, Macro> &macros) {
    for (int pass = 0; pass < 8 && expand_once(s, macros); ++pass) {
    }
    return s;
}

// body text between the braces of `struct|class NAME {` (or of
// `typedef struct ... { } NAME;`), "" when absent
std::string find_record_body(const std::string &s, const std::string &name) {
    if (name.empty()) return "";  // find("") matches everywhere: the loop would not advance
    for (size_t pos = 0; (pos = s.find(name, pos)) != std::string::npos; pos += name.size()) {
        if ((pos > 0 && ident_char(s[pos - 1])) || (pos + name.size() < s.size() && ident_char(s[pos + name.size()])))
            continue;
        // `struct NAME {`
        size_t b = pos;
        while (b > 0 && std::isspace((unsigned char)s[b - 1])) --b;
        const bool tagged = (b >= 6 && s.compare(b - 6, 6, "struct") == 0) ||
                            (b >= 5 && s.compare(b - 5, 5, "class") == 0);
        size_t a = pos + name.size();
        while (a < s.size() && s[a] != '{' && s[a] != ';' && s[a] != '(' && s[a] != ')') ++a;
        if (tagged && a < s.size() && s[a] == '{') {
            int depth = 0;
            for (size_t e = a; e < s.size(); ++e) {
                if (s[e] == '{') ++depth;
                else if (s[e] == '}' && --depth == 0) return s.substr(a + 1, e - a - 1);
            }
        }
        // `typedef struct { ... } NAME;`
        if (b > 0 && s[b - 1] == '}') {
            int depth = 0;
            for (size_t e = b; e-- > 0;) {
                if (s[e] == '}') ++depth;
                else if (s[e] == '{' && --depth == 0) {
                    size_t t = e;
                    while (t > 0 && std::isspace((unsigned char)s[t - 1])) --t;
                    // accept `typedef struct [tag] {`
                    const size_t st = s.rfind("typedef", t);
                    if (st != std::string::npos && t - st < 64) return s.substr(e + 1, b - 1 - e - 1);
                    break;
                }
            }
        }
    }
    return "";
}

// enumerator names of `enum [class|struct] NAME [: T] { ... }` or
// `typedef enum [tag] { ... } NAME;`
bool find_enumerators(const std::string &s, const std::string &name, std::vector<std::string> *out) {
    auto names_of = [&](size_t open) {
        int depth = 0;
        size_t e = open;
        for (; e < s.size(); ++e) {
            if (s[e] == '{') ++depth;
            else if (s[e] == '}' && --depth == 0) break;
        }
        out->clear();
        for (const std::string &item : split_args(s.substr(open + 1, e - open - 1))) {
            const std::string t = trim(item);
            size_t n = 0;
            while (n < t.size() && ident_char(t[n])) ++n;
            if (n) out->push_back(t.substr(0, n));
        }
        return true;
    };
    if (name.empty()) return false;  // an ENUM_PARAM without a type name (tests/sanitize/host_fuzz.cpp)
    for (size_t pos = 0; (pos = s.find(name, pos)) != std::string::npos; pos += name.size()) {
        if ((pos > 0 && ident_char(s[pos - 1])) || (pos + name.size() < s.size() && ident_char(s[pos + name.size()])))
            continue;
        size_t b = pos;
        while (b > 0 && std::isspace((unsigned char)s[b - 1])) --b;
        size_t w = b;
        while (w > 0 && ident_char(s[w - 1])) --w;
        std::string kw = s.substr(w, b - w);
        if (kw == "class" || kw == "struct") {  // enum class NAME
            size_t b2 = w;
            while (b2 > 0 && std::isspace((unsigned char)s[b2 - 1])) --b2;
            size_t w2 = b2;
            while (w2 > 0 && ident_char(s[w2 - 1])) --w2;
            kw = s.substr(w2, b2 - w2);
        }
        if (kw == "enum") {
            size_t a = pos + name.size();
            while (a < s.size() && s[a] != '{' && s[a] != ';') ++a;
            if (a < s.size() && s[a] == '{') return names_of(a);
        }
        if (b > 0 && s[b - 1] == '}') {  // typedef enum { ... } NAME;
            int depth = 0;
            for (size_t e = b; e-- > 0;) {
                if (s[e] == '}') ++depth;
                else if (s[e] == '{' && --depth == 0) {
                    const size_t en = s.rfind("enum", e);
                    if (en != std::string::npos && e - en < 64) return names_of(e);
                    break;
                }
            }
        }
    }
    return false;
}

// string literals inside annotate( ... ), concatenated
bool annotation_of(const std::string &decl, std::string *ann) {
    const size_t a = decl.find("annotate");
    if (a == std::string::npos) return false;
    size_t p = decl.find('(', a);
    if (p == std::string::npos) return false;
    int depth = 0;
    std::string out;
    for (size_t i = p; i < decl.size(); ++i) {
        const char c = decl[i];
        if (c == '(') ++depth;
        else if (c == ')') {
            if (--depth == 0) break;
        } else if (c == '"') {
            for (++i; i < decl.size() && decl[i] != '"'; ++i) {
                if (decl[i] == '\\' && i + 1 < decl.size()) ++i;
                out += decl[i];
            }
        }
    }
    *ann = out;
    return true;
}

// remove every __attribute__((...)) group
std::string strip_attributes(const std::string &decl) {
    std::string o;
    for (size_t i = 0; i < decl.size();) {
        if (decl.compare(i, 13, "__attribute__") == 0) {
            const size_t p = decl.find('(', i);
            if (p == std::string::npos) {  // no group follows: i would wrap to 0 (tests/sanitize/host_fuzz.cpp)
                o += ' ';
                break;
            }
            int depth = 0;
            size_t e = p;
            for (; e < decl.size(); ++e) {
                if (decl[e] == '(') ++depth;
                else if (decl[e] == ')' && --depth == 0) break;
            }
            i = e + 1;
            o += ' ';
        } else {
            o += decl[i++];
        }
    }
    return o;
}

// "const float gain = 1.0f" -> type "const float", names {"gain"}
void split_declaration(const std::string &decl, std::string *type, std::vector<std::string> *names) {
    std::vector<std::string> parts = split_args(decl);
    names->clear();
    type->clear();
    for (size_t k = 0; k < parts.size(); ++k) {
        std::string d = parts[k];
        const size_t eq = d.find_first_of("={");
        if (eq != std::string::npos) d = d.substr(0, eq);
        const size_t br = d.find('[');
        if (br != std::string::npos) d = d.substr(0, br);
        d = trim(d);
        size_t e = d.size();
        while (e > 0 && !ident_char(d[e - 1])) --e;
        size_t s = e;
        while (s > 0 && ident_char(d[s - 1])) --s;
        if (s == e) continue;
        names->push_back(d.substr(s, e - s));
        if (k == 0) *type = collapse_ws(d.substr(0, s));
    }
    // a type spelled with pointer / reference declarators stays as written
    while (!type->empty() && (type->back() == '*' || type->back() == '&' || type->back() == ' '))
        type->pop_back();
}

std::string hex_bytes(const std::string &s) {
    std::string o;
    char buf[8];
    for (unsigned char c : s) {
        std::snprintf(buf, sizeof buf, "%u,", (unsigned)c);
        o += buf;
    }
    return o + "0";
}

// the enumerator list's type name as written in the field's type, minus
// cv-qualifiers / elaborated keywords
std::string enum_name_of(const std::string &type) {
    std::string t = " " + type + " ";
    for (const char *kw : {" const ", " volatile ", " enum ", " class ", " struct "}) {
        size_t p;
        while ((p = t.find(kw)) != std::string::npos) t.replace(p, std::strlen(kw), " ");
    }
    t = trim(t);
    const size_t c = t.rfind("::");
    return c == std::string::npos ? t : t.substr(c + 2);
}

}  // namespace

// ---------------------------------------------------------------------------
// compile side: scan the source, generate the blob / text definitions
// ---------------------------------------------------------------------------
std::string generate(const char *source, const char *device_header, std::string *note) {
    const std::string src = strip_comments(source ? source : "");
    std::map<std::string, Macro> macros;
    collect_macros(strip_comments(device_header ? device_header : ""), macros);
    collect_macros(src, macros);

    struct Field {
        std::string name, annotation, type, enum_type;
        std::vector<std::string> enumerators;
    };
    std::vector<Field> fields;
    std::string body = find_record_body(src, "Parameters");
    bool parsed = !body.empty() || src.find("Parameters") == std::string::npos;
    if (body.empty() && note) *note += "descriptor: no `struct Parameters { ... }` found in the source text\n";
    // drop preprocessor lines inside the body, then split at top-level ';'
    {
        std::string b;
        size_t pos = 0;
        while (pos < body.size()) {
            size_t e = body.find('\n', pos);
            if (e == std::string::npos) e = body.size();
            const std::string line = body.substr(pos, e - pos);
            if (trim(line).empty() || trim(line)[0] != '#') b += line + "\n";
            pos = e + 1;
        }
        body = b;
    }
    int depth = 0;
    std::string cur;
    std::vector<std::string> decls;
    for (char c : body) {
        if (c == '{' || c == '(') ++depth;
        if (c == '}' || c == ')') --depth;
        if (c == ';' && depth == 0) {
            decls.push_back(cur);
            cur.clear();
        } else {
            cur += c;
        }
    }
    for (const std::string &raw : decls) {
        const std::string d = expand(raw, macros);
        std::string ann;
        if (!annotation_of(d, &ann)) continue;  // not a parameter (compiler.cpp:963-966)
        const std::string plain = strip_attributes(d);
        if (plain.find('(') != std::string::npos) continue;  // a member function, not a field
        std::string type;
        std::vector<std::string> names;
        split_declaration(plain, &type, &names);
        for (const std::string &n : names) {
            Field f;
            f.name = n;
            f.annotation = ann;
            f.type = type;
            if (ann.compare(0, 4, "Enum") == 0) {
                f.enum_type = enum_name_of(type);
                if (!find_enumerators(src, f.enum_type, &f.enumerators) && note)
                    *note += "descriptor: enumerators of `" + f.enum_type + "` not found\n";
            }
            fields.push_back(f);
        }
    }

    // the compiler evaluates the layout: offsets, type classes, enumerators
    std::string g;
    g += "\ntemplate <class T> struct dspb_desc_typecode {\n"
         "  static constexpr unsigned long long v = __is_same(T, int) ? 1ull : __is_same(T, float) ? 2ull :\n"
         "                                         __is_enum(T) ? 3ull : 0ull;\n};\n";
    // a name the scanner got wrong must not break the build: the helpers
    // answer ~0 (no such field) instead of failing to compile
    for (const Field &f : fields) {
        g += "template <class P> constexpr unsigned long long dspb_desc_off_" + f.name + "() {\n"
             "  if constexpr (requires { &P::" + f.name + "; }) return __builtin_offsetof(P, " + f.name + ");\n"
             "  else return ~0ull;\n}\n";
        g += "template <class P> constexpr unsigned long long dspb_desc_tc_" + f.name + "() {\n"
             "  if constexpr (requires { &P::" + f.name + "; }) return dspb_desc_typecode<decltype(((P *)0)->" + f.name +
             ")>::v;\n  else return 0ull;\n}\n";
    }
    g += "extern \"C\" __attribute__((used, visibility(\"default\"))) __device__ const unsigned long long dspb_desc_blob[] = {\n";
    g += "  " + std::to_string(kMagic) + "ull, 1ull, sizeof(Parameters), alignof(Parameters), sizeof(State), "
         "alignof(State), (unsigned long long)__is_empty(State), " + std::to_string(fields.size()) + "ull, " +
         (parsed ? "1ull" : "0ull") + ",\n";
    for (const Field &f : fields) {
        g += "  dspb_desc_off_" + f.name + "<Parameters>(), dspb_desc_tc_" + f.name + "<Parameters>(), " +
             std::to_string(f.enumerators.size()) + "ull,\n";
        for (const std::string &e : f.enumerators)
            g += "  (unsigned long long)(long long)(" + f.enum_type + "::" + e + "),\n";
    }
    g += "  0ull};\n";
    std::string text;
    for (const Field &f : fields) {
        text += f.name + kFieldSep + f.annotation;
        for (const std::string &e : f.enumerators) text += kFieldSep + e;
        text += kRecSep;
    }
    g += "extern \"C\" __attribute__((used, visibility(\"default\"))) __device__ const unsigned char dspb_desc_text[] = {" +
         hex_bytes(text) + "};\n";
    return g;
}

// ---------------------------------------------------------------------------
// host side: the two symbols out of the code object's ELF
// ---------------------------------------------------------------------------
namespace {

struct Elf64Ehdr {
    unsigned char ident[16];
    uint16_t type, machine;
    uint32_t version;
    uint64_t entry, phoff, shoff;
    uint32_t flags;
    uint16_t ehsize, phentsize, phnum, shentsize, shnum, shstrndx;
};
struct Elf64Shdr {
    uint32_t name, type;
    uint64_t flags, addr, offset, size;
    uint32_t link, info;
    uint64_t addralign, entsize;
};
struct Elf64Sym {
    uint32_t name;
    unsigned char info, other;
    uint16_t shndx;
    uint64_t value, size;
};

// bytes of symbol `want` (a defined object) in an ELF64 image, or false
bool elf_symbol(const unsigned char *img, size_t size, const char *want, std::string *out) {
    if (size < sizeof(Elf64Ehdr) || std::memcmp(img, "\x7f" "ELF", 4) != 0 || img[4] != 2) return false;
    Elf64Ehdr eh;
    std::memcpy(&eh, img, sizeof eh);
    // every range check below is written so that no sum can wrap
    // (a corrupted header must not pass them: tests/sanitize/host_fuzz.cpp)
    auto in_image = [size](uint64_t off, uint64_t len) { return off <= size && len <= size - off; };
    if (eh.shentsize != sizeof(Elf64Shdr) || eh.shnum == 0 ||
        !in_image(eh.shoff, (uint64_t)eh.shnum * sizeof(Elf64Shdr)))
        return false;
    std::vector<Elf64Shdr> sh(eh.shnum);
    std::memcpy(sh.data(), img + eh.shoff, sh.size() * sizeof(Elf64Shdr));
    for (const Elf64Shdr &s : sh) {
        if (s.type != 2 && s.type != 11) continue;  // SHT_SYMTAB / SHT_DYNSYM
        if (s.link >= sh.size() || !in_image(s.offset, s.size) || s.entsize != sizeof(Elf64Sym)) continue;
        const Elf64Shdr &strs = sh[s.link];
        if (!in_image(strs.offset, strs.size)) continue;
        for (uint64_t k = 0; k < s.size / sizeof(Elf64Sym); ++k) {
            Elf64Sym sym;
            std::memcpy(&sym, img + s.offset + k * sizeof(Elf64Sym), sizeof sym);
            if (sym.name >= strs.size || sym.shndx == 0 || sym.shndx >= sh.size()) continue;
            // the name and its terminator must both lie inside the string table
            const char *nm = (const char *)img + strs.offset + sym.name;
            const size_t wl = std::strlen(want);
            if (strs.size - sym.name < wl + 1 || std::memcmp(nm, want, wl) != 0 || nm[wl] != 0) continue;
            const Elf64Shdr &sec = sh[sym.shndx];
            if (sec.type == 8) return false;  // NOBITS: no initialiser in the file
            if (sym.value < sec.addr || sym.value - sec.addr > sec.size || sym.size > sec.size - (sym.value - sec.addr))
                return false;
            if (!in_image(sec.offset, sec.size)) return false;
            const uint64_t off = sec.offset + (sym.value - sec.addr);  // within [sec.offset, sec.offset + sec.size]
            out->assign((const char *)img + off, sym.size);
            return true;
        }
    }
    return false;
}

// std::getline(iss, token, ' ') over the annotation (compiler.cpp:992-997)
std::vector<std::string> tokens_of(const std::string &a) {
    std::vector<std::string> t;
    if (a.empty()) return t;
    size_t p = 0;
    while (true) {
        const size_t e = a.find(' ', p);
        t.push_back(a.substr(p, e == std::string::npos ? std::string::npos : e - p));
        if (e == std::string::npos || e + 1 == a.size()) break;
        p = e + 1;
    }
    return t;
}

}  // namespace

int read(const void *code, size_t size, Descriptor *d, std::string *err) {
    *d = Descriptor{};
    std::string blob, text;
    const unsigned char *img = (const unsigned char *)code;
    if (!elf_symbol(img, size, "dspb_desc_blob", &blob) || !elf_symbol(img, size, "dspb_desc_text", &text)) {
        if (err) *err = "code object has no descriptor (dspb_desc_blob): compiled by an older dsp_module_compile";
        return -1;
    }
    std::vector<unsigned long long> v(blob.size() / 8);
    if (!v.empty()) std::memcpy(v.data(), blob.data(), v.size() * 8);
    if (v.size() < 9 || v[0] != kMagic || v[1] != 1) {
        if (err) *err = "descriptor blob: bad magic / version";
        return -1;
    }
    d->params_size = v[2];
    d->params_align = v[3];
    d->state_size = v[4];
    d->state_align = v[5];
    d->state_empty = v[6] != 0;
    const uint64_t n = v[7];
    d->source_parsed = v[8] != 0;
    auto pow2 = [](uint64_t a) { return a && a <= 4096 && !(a & (a - 1)); };
    if (d->params_size > (1u << 24) || d->state_size > (1ull << 32) || !pow2(d->params_align) ||
        !pow2(d->state_align) || n > 4096) {
        if (err) *err = "descriptor blob: implausible layout";
        return -1;
    }
    // text records: name \x1f annotation [\x1f enumerator ...] \x1e
    std::vector<std::vector<std::string>> recs;
    {
        std::vector<std::string> rec;
        std::string cur;
        for (char c : text) {
            if (c == 0) break;
            if (c == kFieldSep) {
                rec.push_back(cur);
                cur.clear();
            } else if (c == kRecSep) {
                rec.push_back(cur);
                cur.clear();
                recs.push_back(rec);
                rec.clear();
            } else {
                cur += c;
            }
        }
    }
    if (recs.size() != n) {
        if (err) *err = "descriptor blob / text disagree";
        return -1;
    }
    size_t at = 9;
    d->error = kSuccess;
    for (uint64_t i = 0; i < n; ++i) {
        if (at + 3 > v.size()) {
            if (err) *err = "descriptor blob truncated";
            return -1;
        }
        Param p;
        p.name = recs[i][0];
        p.annotation = recs[i].size() > 1 ? recs[i][1] : "";
        if (v[at] > d->params_size || d->params_size - v[at] < 4) {  // int, float and enum fields: 4 bytes
            if (err) *err = "descriptor blob: a field lies outside Parameters";
            return -1;
        }
        p.offset = (uint32_t)v[at];
        const unsigned long long tc = v[at + 1];
        const uint64_t ne = v[at + 2];
        at += 3;
        for (uint64_t e = 0; e < ne && at < v.size(); ++e, ++at) {
            Entry en;
            en.value = (int64_t)v[at];
            en.name = 2 + e < recs[i].size() ? recs[i][2 + e] : "";
            p.entries.push_back(en);
        }
        // validation: compiler.cpp:1009-1146
        const std::vector<std::string> tok = tokens_of(p.annotation);
        p.error = kSuccess;
        if (tok.empty()) {
            p.error = kEmptyAnnotation;
        } else if (tok[0] == "Int") {
            p.type = kInt;
            if (tc != 1) p.error = kTypeMismatch;
            else if (tok.size() != 3) p.error = kMissingMinMax;
            else {
                char *e1 = nullptr, *e2 = nullptr;
                const long mn = std::strtol(tok[1].c_str(), &e1, 0);
                const long mx = std::strtol(tok[2].c_str(), &e2, 0);
                // the reference tests end_ptr against nullptr, which strtol never
                // returns; a token with no number at all is flagged here
                if (e1 == tok[1].c_str()) p.error = kInvalidMin;
                else if (e2 == tok[2].c_str()) p.error = kInvalidMax;
                else if (mn >= mx) p.error = kMinGreaterThanMax;
                p.int_min = (int32_t)mn;
                p.int_max = (int32_t)mx;
            }
        } else if (tok[0] == "Float") {
            p.type = kFloat;
            if (tc != 2) p.error = kTypeMismatch;
            else if (tok.size() != 3 && tok.size() != 4) p.error = kMissingMinMax;
            else {
                char *e1 = nullptr, *e2 = nullptr;
                const float mn = std::strtof(tok[1].c_str(), &e1);
                const float mx = std::strtof(tok[2].c_str(), &e2);
                if (e1 == tok[1].c_str()) p.error = kInvalidMin;
                else if (e2 == tok[2].c_str()) p.error = kInvalidMax;
                else if (mn >= mx) p.error = kMinGreaterThanMax;
                p.float_min = mn;
                p.float_max = mx;
                if (tok.size() == 4) {
                    if (tok[3] == "log") p.float_log = true;
                    else if (p.error == kSuccess) p.error = kInvalidAnnotation;
                }
            }
        } else if (tok[0] == "Enum") {
            p.type = kEnum;
            if (tc != 3) p.error = kTypeMismatch;
            else if (p.entries.empty()) p.error = kInvalidAnnotation;  // enumerators not found in the source
        } else {
            p.error = kInvalidAnnotation;
        }
        if (p.error != kSuccess) d->error = kErrorRecurse;
        d->params.push_back(p);
    }
    return 0;
}

const char *error_name(int e) {
    switch (e) {  // errors.inc:1-19
    case kSuccess: return "Compiler_Success";
    case kErrorRecurse: return "Compiler_Error_Recurse";
    case kEmptyAnnotation: return "Compiler_Empty_Annotation";
    case kInvalidAnnotation: return "Compiler_Invalid_Annotation";
    case kMissingMinMax: return "Compiler_Missing_Min_Max";
    case kMinGreaterThanMax: return "Compiler_Min_Greater_Than_Max";
    case kInvalidMin: return "Compiler_Invalid_Min_Value";
    case kInvalidMax: return "Compiler_Invalid_Max_Value";
    case kTypeMismatch: return "Compiler_Annotation_Type_Mismatch";
    default: return "unknown";
    }
}

std::string hex_literal(const std::string &s) { return hex_bytes(s); }

bool code_symbol(const void *code, size_t size, const char *name, std::string *out) {
    return elf_symbol((const unsigned char *)code, size, name, out);
}

}  // namespace desc
}  // namespace dspb
