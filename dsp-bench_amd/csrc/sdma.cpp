// sdma.cpp -- device -> pinned host downloads on an SDMA engine (sdma.hpp).
//
// The HSA runtime is the one the process has already loaded with its HIP
// runtime (dlopen by soname with RTLD_NOLOAD only: a PyTorch process carries
// its own copy, and a second runtime in one process would be fatal -- when
// none is loaded, the downloads take hipMemcpyAsync instead); the types come
// from /opt/rocm/include/hsa.
#include "sdma.hpp"

#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>

#include "dspbench/dspbench.h"

namespace dspb {
void set_last_error(const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);

namespace {

constexpr int kCopyTimeoutS = 120;  // one chunk's downloads: ~10 ms at the engine's 57 GB/s

struct Hsa {
    bool ok = false;
    decltype(&hsa_iterate_agents) iterate_agents;
    decltype(&hsa_agent_get_info) agent_get_info;
    decltype(&hsa_signal_create) signal_create;
    decltype(&hsa_signal_destroy) signal_destroy;
    decltype(&hsa_signal_wait_scacquire) signal_wait_scacquire;
    decltype(&hsa_signal_store_screlease) signal_store_screlease;
    decltype(&hsa_amd_memory_async_copy_on_engine) copy_on_engine;
    decltype(&hsa_amd_memory_copy_engine_status) engine_status;
    decltype(&hsa_amd_pointer_info) pointer_info;
    decltype(&hsa_amd_memory_get_preferred_copy_engine) preferred;  // may be NULL (older runtimes)
};

Hsa &hsa() {
    static Hsa h;
    static std::once_flag once;
    std::call_once(once, [] {
        void *l = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!l) return;  // never a runtime of our own: not usable
        bool all = true;
        auto sym = [&](const char *n) {
            void *p = dlsym(l, n);
            all = all && p;
            return p;
        };
        h.iterate_agents = (decltype(h.iterate_agents))sym("hsa_iterate_agents");
        h.agent_get_info = (decltype(h.agent_get_info))sym("hsa_agent_get_info");
        h.signal_create = (decltype(h.signal_create))sym("hsa_signal_create");
        h.signal_destroy = (decltype(h.signal_destroy))sym("hsa_signal_destroy");
        h.signal_wait_scacquire = (decltype(h.signal_wait_scacquire))sym("hsa_signal_wait_scacquire");
        h.signal_store_screlease = (decltype(h.signal_store_screlease))sym("hsa_signal_store_screlease");
        h.copy_on_engine = (decltype(h.copy_on_engine))sym("hsa_amd_memory_async_copy_on_engine");
        h.engine_status = (decltype(h.engine_status))sym("hsa_amd_memory_copy_engine_status");
        h.pointer_info = (decltype(h.pointer_info))sym("hsa_amd_pointer_info");
        h.ok = all;
        h.preferred = (decltype(h.preferred))dlsym(l, "hsa_amd_memory_get_preferred_copy_engine");
    });
    return h;
}

// a HIP device's HSA agent (matched by PCI domain / bus / device), a CPU
// agent, and the SDMA engines free for GPU -> CPU copies
struct Agents {
    bool ok = false;
    hsa_agent_t gpu{}, cpu{};
    uint32_t engines = 0;    // free for GPU -> CPU copies
    uint32_t preferred = 0;  // the runtime's preferred ones (0: unknown)
};

struct Find {
    uint32_t domain, bdf;
    hsa_agent_t gpu{}, cpu{};
    bool have_gpu = false, have_cpu = false;
};

hsa_status_t find_agent(hsa_agent_t a, void *u) {
    Find &f = *(Find *)u;
    Hsa &h = hsa();
    hsa_device_type_t t;
    if (h.agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !f.have_cpu) {
        f.cpu = a;
        f.have_cpu = true;
    } else if (t == HSA_DEVICE_TYPE_GPU && !f.have_gpu) {
        uint32_t bdf = 0, dom = 0;
        if (h.agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
            h.agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
            (bdf & ~7u) == f.bdf && dom == f.domain) {
            f.gpu = a;
            f.have_gpu = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

Agents agents_of(int dev) {
    static std::mutex mu;
    static std::map<int, Agents> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    Agents a;
    Hsa &h = hsa();
    int bus = -1, device = -1, domain = -1;
    if (h.ok && hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) == hipSuccess &&
        hipDeviceGetAttribute(&device, hipDeviceAttributePciDeviceId, dev) == hipSuccess &&
        hipDeviceGetAttribute(&domain, hipDeviceAttributePciDomainId, dev) == hipSuccess) {
        Find f{(uint32_t)domain, ((uint32_t)bus << 8) | ((uint32_t)device << 3)};
        if (h.iterate_agents(find_agent, &f) == HSA_STATUS_SUCCESS && f.have_gpu && f.have_cpu) {
            a.gpu = f.gpu;
            a.cpu = f.cpu;
            a.ok = h.engine_status(a.cpu, a.gpu, &a.engines) == HSA_STATUS_SUCCESS && a.engines != 0;
            if (h.preferred && h.preferred(a.cpu, a.gpu, &a.preferred) != HSA_STATUS_SUCCESS) a.preferred = 0;
        }
    }
    (void)hipGetLastError();
    cache[dev] = a;
    return a;
}

}  // namespace

bool SdmaDownloader::usable(int dev, const void *host) {
    if (std::getenv("DSPB_NO_SDMA")) return false;  // A/B: the HIP runtime's own copy
    Hsa &h = hsa();
    if (!h.ok || !agents_of(dev).ok) return false;
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof info);
    info.size = sizeof info;
    if (h.pointer_info(host, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
    // an HSA allocation (hipHostMalloc, torch's pinned memory) is addressed
    // by the engine at its host address; locked (registered) memory is not
    return info.type == HSA_EXT_POINTER_TYPE_HSA && info.hostBaseAddress == info.agentBaseAddress;
}

SdmaDownloader::~SdmaDownloader() { (void)finish(); }

int SdmaDownloader::start(int dev, int nslots) {
    dev_ = dev;
    submitted_.assign((size_t)nslots, 0);
    landed_.assign((size_t)nslots, 0);
    stop_ = false;
    err_ = 0;
    th_ = std::thread([this] { run(); });
    started_ = true;
    return DSP_OK;
}

int SdmaDownloader::submit(int slot, hipEvent_t after, std::vector<HostCopy> copies) {
    {
        std::lock_guard<std::mutex> g(mu_);
        if (err_) return err_;
        q_.push_back(Job{slot, after, std::move(copies)});
        ++submitted_[(size_t)slot];
    }
    cv_.notify_all();
    return DSP_OK;
}

int SdmaDownloader::wait_slot(int slot) {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] { return err_ || landed_[(size_t)slot] == submitted_[(size_t)slot]; });
    if (err_) set_last_error("%s", msg_.c_str());
    return err_;
}

int SdmaDownloader::finish() {
    if (!started_) return err_;
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    th_.join();
    started_ = false;
    if (err_) set_last_error("%s", msg_.c_str());
    return err_;
}

void SdmaDownloader::run() {
    (void)hipSetDevice(dev_);
    Hsa &h = hsa();
    const Agents ag = agents_of(dev_);
    hsa_signal_t sig{};
    int st = h.signal_create(1, 0, nullptr, &sig) == HSA_STATUS_SUCCESS ? DSP_OK : DSP_ERR_HIP;
    if (st) set_last_error("SDMA download: hsa_signal_create failed");
    // the engine: the highest of the runtime's preferred ones for this
    // direction.  Measured on MI355X (preferred 0x6 for D2H, 0x1 for H2D):
    // 0x4 or 0x8 alone download 1 h of render + spectra in 54.5-55.5 ms
    // beside the uploads, 0x2 (alone or with 0x4) in 60-67 ms, 0x10 in
    // 222 ms (profiles/r03_e2e_sdma_engines.txt).  DSPB_SDMA_ENGINES (a hex
    // mask) overrides, for A/B runs.
    // A runtime that reports no preference (the ROCm 7.0 runtime PyTorch
    // bundles: preferred 0x0) gets what ROCm 7.2 prefers for D2H on MI355X
    // (0x6) -> 0x4; its lowest free engine, 0x1, downloads 1 h in 65 ms.
    uint32_t mask = (ag.preferred ? ag.preferred : 0x6u) & ag.engines;
    if (mask) mask = 1u << (31 - __builtin_clz(mask));
    if (!mask) mask = ag.engines & (0u - ag.engines);  // the lowest free one
    if (const char *e = std::getenv("DSPB_SDMA_ENGINES")) mask = (uint32_t)std::strtoul(e, nullptr, 16) & ag.engines;
    if (!mask) mask = ag.engines & (0u - ag.engines);
    std::vector<hsa_amd_sdma_engine_id_t> eng;
    for (uint32_t b = 0; b < 32; ++b)
        if (mask & (1u << b)) eng.push_back((hsa_amd_sdma_engine_id_t)(1u << b));
    if (std::getenv("DSPB_SDMA_VERBOSE"))
        std::fprintf(stderr, "dspbench: SDMA downloads on engine mask 0x%x (free 0x%x, preferred 0x%x)\n", mask,
                     ag.engines, ag.preferred);
    size_t next = 0;
    while (true) {
        Job job;
        {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] { return stop_ || !q_.empty(); });
            if (q_.empty()) break;  // stop_ and drained
            job = std::move(q_.front());
            q_.pop_front();
        }
        if (!st) {
            const hipError_t e = hipEventSynchronize(job.after);
            if (e != hipSuccess) st = hip_fail(e, "SDMA download: the chunk's compute");
        }
        uint64_t n = 0;
        for (const HostCopy &c : job.copies) n += c.bytes ? 1 : 0;
        if (!st && n) {
            // every copy decrements the signal once: it reaches 0 when all
            // have landed (after a failed issue: when the issued ones have)
            h.signal_store_screlease(sig, (hsa_signal_value_t)n);
            uint64_t issued = 0;
            for (const HostCopy &c : job.copies) {
                if (!c.bytes) continue;
                const hsa_status_t hs = h.copy_on_engine(c.dst, ag.cpu, c.src, ag.gpu, c.bytes, 0, nullptr, sig,
                                                         eng[next++ % eng.size()], true);
                if (hs != HSA_STATUS_SUCCESS) {
                    set_last_error("SDMA download: hsa_amd_memory_async_copy_on_engine failed (0x%x)", (unsigned)hs);
                    st = DSP_ERR_HIP;
                    break;
                }
                ++issued;
            }
            // bounded: a copy that never lands fails the render instead of
            // hanging this worker (and the join in finish())
            const hsa_signal_value_t want = (hsa_signal_value_t)(n - issued + 1);
            const auto t0 = std::chrono::steady_clock::now();
            while (h.signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, want, 1000000ull, HSA_WAIT_STATE_BLOCKED) >=
                   want) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(kCopyTimeoutS)) {
                    set_last_error("SDMA download: copies did not land within %d s (their buffers are kept: "
                                   "the engine may still write them)", kCopyTimeoutS);
                    if (!st) st = DSP_ERR_HIP;
                    std::lock_guard<std::mutex> g(mu_);
                    poisoned_ = true;
                    break;
                }
            }
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            if (st && !err_) {
                err_ = st;
                msg_ = dsp_last_error();  // (the worker thread's own error text)
            }
            ++landed_[(size_t)job.slot];
        }
        cv_.notify_all();
    }
    // a copy still in flight may decrement the signal: keep it then (leaked)
    bool keep = false;
    {
        std::lock_guard<std::mutex> g(mu_);
        keep = poisoned_;
    }
    if (sig.handle && !keep) h.signal_destroy(sig);
}

}  // namespace dspb
