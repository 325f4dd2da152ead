// descriptor.hpp -- a module's plugin parameter descriptor (descriptor.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace dspb {
namespace desc {

// Plugin_Parameter_Type (plugin.h:15-19)
enum { kInt = 0, kFloat = 1, kEnum = 2 };

// the compiler error flags a descriptor can carry (errors.inc:1-19), as
// dsp_desc_error values (module.h)
enum {
    kSuccess = 0,
    kErrorRecurse = 1,
    kEmptyAnnotation = 2,
    kInvalidAnnotation = 3,
    kMissingMinMax = 4,
    kMinGreaterThanMax = 5,
    kInvalidMin = 6,
    kInvalidMax = 7,
    kTypeMismatch = 8
};

struct Entry {  // Parameter_Enum_Entry (plugin.h:36-39)
    int64_t value = 0;
    std::string name;
};

struct Param {  // Plugin_Descriptor_Parameter (plugin.h:47-55)
    std::string name, annotation;
    uint32_t offset = 0;
    int type = kFloat;
    int error = kSuccess;
    int32_t int_min = 0, int_max = 0;
    float float_min = 0.f, float_max = 0.f;
    bool float_log = false;
    std::vector<Entry> entries;
};

struct Descriptor {  // Plugin_Descriptor (plugin.h:57-74)
    uint64_t params_size = 0, params_align = 0, state_size = 0, state_align = 0;
    bool state_empty = false;
    bool source_parsed = false;
    int error = kSuccess;
    std::vector<Param> params;
};

// The definitions to append to a plugin's translation unit (after the
// plugin): dspb_desc_blob / dspb_desc_text.  `note` collects scanner remarks.
std::string generate(const char *source, const char *device_header, std::string *note);

// The descriptor stored in a code object (host only, no GPU); 0 or -1.
int read(const void *code, size_t size, Descriptor *d, std::string *err);

const char *error_name(int e);

// "0x.., 0x.., ..." initialiser text of a byte string (generated device arrays)
std::string hex_literal(const std::string &s);

// the bytes of a defined object symbol of a code object's ELF (host only)
bool code_symbol(const void *code, size_t size, const char *name, std::string *out);

}  // namespace desc
}  // namespace dspb
