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

// The engine connection over GpuDevices(), one per device set for the whole
// process: every file the extension opens shares it, so its per-GPU scan
// pipelines (streams, device slots, pinned host batches) and staging threads
// carry over from one query to the next.  Never closed (process lifetime).
inline fls_connection *SharedConnection() {
    static std::mutex mu;
    static auto *conns = new std::map<std::vector<int>, fls_connection *>();
    const std::vector<int> devs = GpuDevices();
    std::lock_guard<std::mutex> lk(mu);
    auto it = conns->find(devs);
    if (it != conns->end()) return it->second;
    fls_connection *c = nullptr;
    if (fls_connect(devs.data(), (int)devs.size(), &c) != 0) return nullptr;
    (*conns)[devs] = c;
    return c;
}

}  // namespace ext_fastlane
}  // namespace duckdb
