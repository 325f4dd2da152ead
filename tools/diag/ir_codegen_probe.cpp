// ir_codegen_probe -- does comgr turn LLVM IR *text* into a gfx950 code
// object (CODEGEN_BC_TO_RELOCATABLE, then LINK_RELOCATABLE_TO_EXECUTABLE)?
// The question behind DESIGN 9's State chain for callbacks that read their
// block: a chain compiled from the callback's IR with its block stores
// removed needs exactly this path.  CPU only.
//   build: g++ -O1 -std=c++17 -I/opt/rocm/include ir_codegen_probe.cpp -L/opt/rocm/lib -lamd_comgr -o probe
//   usage: probe in.ll out.co
#include <amd_comgr/amd_comgr.h>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

static bool add(amd_comgr_data_set_t set, amd_comgr_data_kind_t k, const std::string &t, const char *name) {
    amd_comgr_data_t d;
    if (amd_comgr_create_data(k, &d)) return false;
    bool ok = !amd_comgr_set_data(d, t.size(), t.data()) && !amd_comgr_set_data_name(d, name) &&
              !amd_comgr_data_set_add(set, d);
    amd_comgr_release_data(d);
    return ok;
}
static std::string get(amd_comgr_data_set_t set, amd_comgr_data_kind_t k) {
    size_t n = 0;
    if (amd_comgr_action_data_count(set, k, &n) || !n) return "";
    amd_comgr_data_t d;
    amd_comgr_action_data_get_data(set, k, 0, &d);
    size_t sz = 0;
    amd_comgr_get_data(d, &sz, nullptr);
    std::string s(sz, '\0');
    amd_comgr_get_data(d, &sz, &s[0]);
    amd_comgr_release_data(d);
    return s;
}
int main(int argc, char **argv) {
    if (argc < 3) return 2;
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    amd_comgr_data_set_t in, rel, exe;
    amd_comgr_create_data_set(&in);
    amd_comgr_create_data_set(&rel);
    amd_comgr_create_data_set(&exe);
    if (!add(in, AMD_COMGR_DATA_KIND_BC, ss.str(), "probe.ll")) return 3;
    amd_comgr_action_info_t ai;
    amd_comgr_create_action_info(&ai);
    amd_comgr_action_info_set_isa_name(ai, "amdgcn-amd-amdhsa--gfx950");
    amd_comgr_action_info_set_logging(ai, true);
    const char *opts[] = {"-O3"};
    amd_comgr_action_info_set_option_list(ai, opts, 1);
    amd_comgr_status_t st = amd_comgr_do_action(AMD_COMGR_ACTION_CODEGEN_BC_TO_RELOCATABLE, ai, in, rel);
    std::printf("codegen: %d\n%s\n", (int)st, get(rel, AMD_COMGR_DATA_KIND_LOG).substr(0, 800).c_str());
    if (st) return 4;
    st = amd_comgr_do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, ai, rel, exe);
    std::printf("link: %d\n%s\n", (int)st, get(exe, AMD_COMGR_DATA_KIND_LOG).substr(0, 800).c_str());
    if (st) return 5;
    const std::string co = get(exe, AMD_COMGR_DATA_KIND_EXECUTABLE);
    std::ofstream(argv[2], std::ios::binary).write(co.data(), (std::streamsize)co.size());
    std::printf("code object: %zu bytes\n", co.size());
    return co.empty() ? 6 : 0;
}
