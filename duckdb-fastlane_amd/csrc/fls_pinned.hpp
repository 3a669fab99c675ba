// fls_pinned.hpp -- page-locked host memory for the scan pipeline's host
// batches and the writer's GPU staging.
//
// hipHostMalloc pins at 4.3-5.0 GB/s on the GPU box (scripts/pin_bench.cpp,
// profiles/r5/pin_bench_r5g.txt), and a cold query's first batches wait for
// it (about 100 ms of a 0.2-0.3 s first query, FLS_SCAN_PROFILE).  Memory that
// is allocated 2 MB-aligned, marked for transparent huge pages, touched once
// and then registered (hipHostRegister) pins at 22 GB/s on one thread: the
// kernel hands out 2 MB pages and the registration walks 512x fewer of them.
// Registered memory is device-accessible at the same address on ROCm (checked:
// otherwise the allocation falls back to hipHostMalloc).  FLS_PIN_MODE=hostmalloc
// keeps hipHostMalloc for every allocation (A/B).
#pragma once
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>

namespace fls {

struct PinnedRegistry {
    std::mutex mu;
    std::unordered_map<void *, size_t> registered;  // pointer -> registered length
    static PinnedRegistry &get() {
        static auto *r = new PinnedRegistry();  // process lifetime
        return *r;
    }
    static bool use_register() {
        static const bool on = [] {
            const char *e = getenv("FLS_PIN_MODE");
            return !(e && strcmp(e, "hostmalloc") == 0);
        }();
        return on;
    }
};

inline hipError_t pinned_alloc(void **out, size_t bytes) {
    *out = nullptr;
    bytes = bytes ? bytes : 1;
    if (PinnedRegistry::use_register()) {
        constexpr size_t kHuge = 2u << 20;
        const size_t align = bytes >= kHuge ? kHuge : 4096;
        const size_t len = (bytes + align - 1) / align * align;
        void *m = nullptr;
        if (posix_memalign(&m, align, len) == 0) {
            if (align == kHuge) madvise(m, len, MADV_HUGEPAGE);
            memset(m, 0, len);  // fault every page in before the registration walks them
            if (hipHostRegister(m, len, hipHostRegisterMapped) == hipSuccess) {
                void *dp = nullptr;
                if (hipHostGetDevicePointer(&dp, m, 0) == hipSuccess && dp == m) {
                    PinnedRegistry &r = PinnedRegistry::get();
                    std::lock_guard<std::mutex> lk(r.mu);
                    r.registered[m] = len;
                    *out = m;
                    return hipSuccess;
                }
                hipHostUnregister(m);
            }
            (void)hipGetLastError();
            free(m);
        }
    }
    return hipHostMalloc(out, bytes, hipHostMallocDefault);
}

// Like hipHostFree, which waits for the device before it releases the pages,
// every GPU is synchronised before registered memory is unregistered: a copy
// still in flight into memory being freed must land in mapped pages (a
// registered block unmapped under a running copy faults the GPU).
inline void pinned_free(void *p) {
    if (!p) return;
    bool reg = false;
    {
        PinnedRegistry &r = PinnedRegistry::get();
        std::lock_guard<std::mutex> lk(r.mu);
        auto it = r.registered.find(p);
        if (it != r.registered.end()) {
            r.registered.erase(it);
            reg = true;
        }
    }
    if (!reg) {
        hipHostFree(p);
        return;
    }
    int n = 0, cur = 0;
    if (hipGetDeviceCount(&n) == hipSuccess && hipGetDevice(&cur) == hipSuccess) {
        for (int d = 0; d < n; ++d)
            if (hipSetDevice(d) == hipSuccess) hipDeviceSynchronize();
        hipSetDevice(cur);
    }
    (void)hipGetLastError();
    hipHostUnregister(p);
    free(p);
}

}  // namespace fls
