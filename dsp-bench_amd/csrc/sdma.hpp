// sdma.hpp -- device -> pinned host downloads on an SDMA copy engine.
//
// Inside a PyTorch process the HIP runtime in use is the one torch bundles,
// and it moves a device -> pinned-host hipMemcpyAsync with a blit kernel
// (__amd_rocclr_copyBuffer) on the compute units: the waves sit on PCIe
// writes for the whole copy and the pipeline's next chunk kernel waits for CU
// slots behind them (tools/copy_engine_probe.py: a 0.03 ms chunk kernel took
// 2.4 ms beside a copy), and H2D + D2H together reach no more than either
// alone.  The same copies on an SDMA engine leave the CUs alone and run
// beside the SDMA uploads (tools/d2h_probe.hip: 57 GB/s alone, 97 GB/s with
// an upload).  So the host pipeline issues its downloads itself, through the
// HSA runtime the process already has loaded (hsa_amd_memory_async_copy_on_
// engine), from a worker thread that waits for each chunk's compute event.
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dspb {

struct HostCopy {
    void *dst;        // pinned host memory (hipHostMalloc'd)
    const void *src;  // device memory
    uint64_t bytes;
};

class SdmaDownloader {
public:
    // whether `host` (pinned host memory from hipHostMalloc) can be written
    // by an SDMA engine of device `dev` through the HSA runtime in this process
    static bool usable(int dev, const void *host);
    ~SdmaDownloader();
    int start(int dev, int nslots);
    // the copies of `slot`, issued once `after` (recorded on the compute
    // stream) has completed
    int submit(int slot, hipEvent_t after, std::vector<HostCopy> copies);
    // block until every download of `slot` submitted so far has landed
    int wait_slot(int slot);
    // drain and stop the worker; the first error of any copy
    int finish();
    // a copy did not land within the bounded wait: the engine may still
    // write the destinations and read the sources, so their owners must keep
    // them (the worker keeps its signal for the same reason)
    bool poisoned() {
        std::lock_guard<std::mutex> g(mu_);
        return poisoned_;
    }

private:
    struct Job {
        int slot;
        hipEvent_t after;
        std::vector<HostCopy> copies;
    };
    void run();
    int dev_ = -1;
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job> q_;
    std::vector<uint64_t> submitted_, landed_;
    bool stop_ = false, started_ = false, poisoned_ = false;
    int err_ = 0;
    std::string msg_;  // the worker's error text, re-raised on the caller's thread
};

}  // namespace dspb
