// gpu_devices.hpp -- GPU set the extension shards row groups over.
// FLS_GPU_DEVICES="0,1,2,3" selects HIP ordinals; default: every visible GPU.
#pragma once
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/flsgpu.h"

namespace duckdb {
namespace ext_fastlane {

// A deployment knob's value in effect (the environment's, else the default
// from the engine's one table, fls_config_value in flsgpu.h).
inline int64_t KnobValue(const char *name) {
    int64_t v = 0;
    if (fls_config_value(name, &v) != 0) std::abort();  // not a knob: a programming error
    return v;
}

inline std::vector<int> GpuDevices() {
    std::vector<int> d;
    if (const char *e = std::getenv("FLS_GPU_DEVICES")) {
        std::string s(e);
        size_t p = 0;
        while (p < s.size()) {
            size_t q = s.find(',', p);
            if (q == std::string::npos) q = s.size();
            if (q > p) d.push_back(std::atoi(s.substr(p, q - p).c_str()));
            p = q + 1;
        }
    }
    if (d.empty()) {
        int n = fls_device_count();
        for (int i = 0; i < (n > 0 ? n : 1); ++i) d.push_back(i);
    }
    return d;
}

// The engine connections, one per device set for the whole process.
struct SharedConnections {
    std::mutex mu;
    std::map<std::vector<int>, fls_connection *> conns;
    static SharedConnections &Get() {
        static auto *s = new SharedConnections();  // process lifetime (tables may outlive static destruction order)
        return *s;
    }
};

// The engine connection over GpuDevices(): every file the extension opens
// shares it, so its per-GPU scan pipelines (streams, device slots, pinned
// host batches) and staging threads carry over from one query to the next.
// The pinned memory idle pipelines keep is capped per GPU by the engine
// (FLS_IDLE_PINNED_MB) and handed back by TrimSharedConnections (SQL:
// fastlane_release_memory()).
inline fls_connection *SharedConnection() {
    auto &s = SharedConnections::Get();
    const std::vector<int> devs = GpuDevices();
    std::lock_guard<std::mutex> lk(s.mu);
    auto it = s.conns.find(devs);
    if (it != s.conns.end()) return it->second;
    fls_connection *c = nullptr;
    if (fls_connect(devs.data(), (int)devs.size(), &c) != 0) return nullptr;
    s.conns[devs] = c;
    return c;
}

// Free the idle scan pipelines of every shared connection down to keep_bytes
// of pinned memory per GPU; returns the pinned bytes still idle.
inline uint64_t TrimSharedConnections(uint64_t keep_bytes) {
    auto &s = SharedConnections::Get();
    std::lock_guard<std::mutex> lk(s.mu);
    uint64_t left = 0;
    for (auto &kv : s.conns) {
        uint64_t idle = 0;
        if (fls_connection_trim(kv.second, keep_bytes, &idle) == 0) left += idle;
    }
    return left;
}

// fastlane_release_memory(): the idle pinned host memory (above) and every
// HBM-resident file image no running scan uses (fls_release_device_memory);
// returns the bytes of both still held.
inline uint64_t ReleaseMemory() {
    uint64_t left = TrimSharedConnections(0), freed = 0, resident = 0;
    fls_release_device_memory(-1, &freed);
    if (fls_resident_info(-1, &resident, nullptr) == 0) left += resident;
    return left;
}

}  // namespace ext_fastlane
}  // namespace duckdb
