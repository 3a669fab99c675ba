// fls_pinned.hpp -- page-locked host memory for the scan pipeline's host
// batches and the writer's GPU staging: one place for the allocation policy.
//
// hipHostMalloc pins at 4.3-5.0 GB/s on the GPU box (scripts/pin_bench.cpp,
// profiles/r5/pin_bench_r5g.txt), and a cold query's first batches wait for
// it.  2 MB-aligned memory marked for transparent huge pages, touched, then
// hipHostRegister'ed pins at 22 GB/s on one thread (76 GB/s on four), but
// with every pinned buffer of the engine allocated, registered, unregistered
// and freed that way the GPU test suite faulted twice ("illegal memory
// access" in a later pageable D2H copy, profiles/r5/pytest_gpu_r5h_fault.log,
// _r5j_fault.log; the same suite passed with hipHostMalloc,
// pytest_gpu_hostmalloc_r5i.log) -- most likely a freed registration's
// address range handed out again by the allocator while the runtime still
// mapped it (round 6: scripts/pin_probe.cpp checks the runtime's view of such
// ranges).
//
// Round 6: the arena (FLS_PIN_ARENA_MB > 0) keeps the fast registration and
// removes that hazard by construction: memory is registered in large chunks
// that are NEVER unregistered or unmapped (process lifetime), and buffers are
// carved out of them and returned to a free list, so no registered range is
// ever handed back to the allocator.  Beyond the cap, or if a registration
// fails, buffers come from hipHostMalloc as before.
#pragma once
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>

#include "fls_config.hpp"

namespace fls {

class PinnedArena {
  public:
    static PinnedArena &get() {
        static auto *a = new PinnedArena();  // process lifetime: chunks are never released
        return *a;
    }
    // a buffer of at least `bytes` from the arena, or nullptr (off / cap reached)
    void *alloc(size_t bytes) {
        const size_t need = (bytes + kGrain - 1) / kGrain * kGrain;
        std::lock_guard<std::mutex> lk(mu_);
        if (cap_ == 0) return nullptr;
        for (int pass = 0; pass < 2; ++pass) {
            for (auto it = free_.begin(); it != free_.end(); ++it) {  // first fit, address order
                if (it->second < need) continue;
                char *p = it->first;
                const size_t rest = it->second - need;
                free_.erase(it);
                if (rest) free_[p + need] = rest;
                used_[p] = need;
                in_use_ += need;
                return p;
            }
            if (pass == 0 && !grow(need)) return nullptr;
        }
        return nullptr;
    }
    // true if p came from the arena (and is now free again)
    bool release(void *vp) {
        char *p = (char *)vp;
        std::lock_guard<std::mutex> lk(mu_);
        auto u = used_.find(p);
        if (u == used_.end()) return false;
        size_t len = u->second;
        used_.erase(u);
        in_use_ -= len;
        // coalesce with the free neighbours (within one chunk: chunks are
        // separate mappings, so an adjacent chunk's range never merges)
        auto next = free_.find(p + len);
        if (next != free_.end() && same_chunk(p, next->first)) {
            len += next->second;
            free_.erase(next);
        }
        auto prev = free_.lower_bound(p);
        if (prev != free_.begin()) {
            --prev;
            if (prev->first + prev->second == p && same_chunk(prev->first, p)) {
                prev->second += len;
                return true;
            }
        }
        free_[p] = len;
        return true;
    }
    bool owns(void *vp) {
        std::lock_guard<std::mutex> lk(mu_);
        return used_.count((char *)vp) != 0;
    }
    size_t registered_bytes() {
        std::lock_guard<std::mutex> lk(mu_);
        return total_;
    }

  private:
    static constexpr size_t kGrain = 4096, kHuge = 2u << 20;
    std::mutex mu_;
    std::map<char *, size_t> free_, used_;
    std::map<char *, size_t> chunks_;  // base -> length
    size_t total_ = 0, in_use_ = 0, next_chunk_ = 64u << 20;
    size_t cap_ = (size_t)std::max<int64_t>(0, knob_value("FLS_PIN_ARENA_MB")) << 20;

    bool same_chunk(const char *a, const char *b) const {
        auto it = chunks_.upper_bound((char *)a);
        if (it == chunks_.begin()) return false;
        --it;
        return b >= it->first && b < it->first + it->second;
    }
    // register a new chunk of at least need bytes (64 MB, doubling to 1 GB)
    bool grow(size_t need) {
        size_t len = std::max(need, next_chunk_);
        len = (len + kHuge - 1) / kHuge * kHuge;
        if (total_ + len > cap_) {
            if (total_ + need > cap_) return false;
            len = (need + kHuge - 1) / kHuge * kHuge;
            if (total_ + len > cap_) return false;
        }
        // 2 MB-aligned anonymous mapping (huge pages: the registration walks
        // 512x fewer pages), populated before it is registered
        const size_t map_len = len + kHuge;
        char *raw = (char *)mmap(nullptr, map_len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (raw == MAP_FAILED) return false;
        char *base = (char *)(((uintptr_t)raw + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
        if (base > raw) munmap(raw, (size_t)(base - raw));
        const size_t tail = (size_t)(raw + map_len - (base + len));
        if (tail) munmap(base + len, tail);
        madvise(base, len, MADV_HUGEPAGE);
        memset(base, 0, len);
        void *dp = nullptr;
        if (hipHostRegister(base, len, hipHostRegisterMapped) != hipSuccess) {
            (void)hipGetLastError();
            munmap(base, len);  // never registered: safe to unmap
            cap_ = 0;           // registration unavailable: hipHostMalloc from now on
            return false;
        }
        if (hipHostGetDevicePointer(&dp, base, 0) != hipSuccess || dp != base) {
            // mapped at another device address: not usable as a plain pinned
            // buffer by the copy paths; keep it registered (never unregister)
            // but unused, and stop using the arena
            (void)hipGetLastError();
            cap_ = 0;
            return false;
        }
        chunks_[base] = len;
        free_[base] = len;
        total_ += len;
        next_chunk_ = std::min<size_t>(next_chunk_ * 2, 1u << 30);
        return true;
    }
};

inline hipError_t pinned_alloc(void **out, size_t bytes) {
    *out = nullptr;
    if (void *p = PinnedArena::get().alloc(bytes ? bytes : 1)) {
        *out = p;
        return hipSuccess;
    }
    return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
}

// Like hipHostFree, which waits for the device before it releases the pages,
// every GPU is synchronised before an arena buffer goes back to the free list:
// a copy still in flight into it must land before another owner gets it.
inline void pinned_free(void *p) {
    if (!p) return;
    if (!PinnedArena::get().owns(p)) {
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
    PinnedArena::get().release(p);
}

}  // namespace fls
