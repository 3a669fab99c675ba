// gpu_devices.hpp -- GPU set the extension shards row groups over.
// FLS_GPU_DEVICES="0,1,2,3" selects HIP ordinals; default: every visible GPU.
#pragma once
#include <cstdlib>
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

}  // namespace ext_fastlane
}  // namespace duckdb
