// fls_pinned.hpp -- page-locked host memory for the scan pipeline's host
// batches and the writer's GPU staging: one place for the allocation policy.
//
// hipHostMalloc pins at 4.3-5.0 GB/s on the GPU box (scripts/pin_bench.cpp,
// profiles/r5/pin_bench_r5g.txt), and a cold query's first batches wait for
// it.  2 MB-aligned memory marked for transparent huge pages, touched, then
// hipHostRegister'ed pins at 22 GB/s on one thread (76 GB/s on four), but
// with every pinned buffer of the engine allocated that way the GPU test
// suite faulted twice ("illegal memory access" in a later pageable D2H copy,
// profiles/r5/pytest_gpu_r5h_fault.log, _r5j_fault.log; the same suite passed with
// hipHostMalloc, pytest_gpu_hostmalloc_r5i.log), although the registration's device pointer was
// checked and the GPUs were synchronised before every unregister -- most
// likely a freed registration's address range reused by the allocator while
// the runtime still mapped it.  So hipHostMalloc it is; the finding is in
// DESIGN.md section 14.
#pragma once
#include <hip/hip_runtime.h>

namespace fls {

inline hipError_t pinned_alloc(void **out, size_t bytes) {
    *out = nullptr;
    return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
}

inline void pinned_free(void *p) {
    if (p) hipHostFree(p);
}

}  // namespace fls
