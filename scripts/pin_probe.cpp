// pin_probe.cpp -- VERDICT r5 item 3: does the HIP runtime still track a host
// range after hipHostUnregister + free, when the allocator hands the same
// addresses out again?  (Round 5's registered pinned memory faulted the GPU
// suite twice in a later PAGEABLE D2H copy, profiles/r5/pytest_gpu_r5h_fault.log,
// _r5j_fault.log; the hypothesis was a freed registration's range reused while
// the runtime still mapped it.)
//
// No device access touches freed memory here: every check is
// hipPointerGetAttributes on the host address, so a stale registration shows
// up as an attribute, not as a fault.  Per iteration, on T threads at once
// (the scan pipelines allocate from several threads):
//   1. mmap a block of 2-16 MB (posix_memalign hands out such blocks as
//      mappings), madvise(MADV_HUGEPAGE), touch, hipHostRegister(Mapped),
//      hipHostGetDevicePointer, one H2D copy out of it (registered use);
//   2. hipHostUnregister -> its return code; hipPointerGetAttributes(block):
//      what the runtime reports right after unregistering;
//   3. munmap; map the same addresses again (MAP_FIXED_NOREPLACE: what a
//      later large malloc, e.g. numpy's, may get); hipPointerGetAttributes on
//      it: what a pageable copy into it would see.
// Counters per thread and in total; any "tracked after unregister/free" is
// the stale registration the hypothesis names.
//   hipcc -O2 -std=c++17 scripts/pin_probe.cpp -o scripts/pin_probe -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static std::atomic<long> n_iter{0}, n_unreg_fail{0}, n_tracked_after_unreg{0}, n_same_va{0}, n_tracked_reuse{0},
    n_reg_fail{0};

static bool tracked(void *p, int *type) {
    hipPointerAttribute_t a;
    memset(&a, 0, sizeof(a));
    const hipError_t e = hipPointerGetAttributes(&a, p);
    (void)hipGetLastError();
    *type = (int)a.type;
    // an untracked pageable pointer: an error, or type unregistered
    return e == hipSuccess && a.type != hipMemoryTypeUnregistered;
}

static void worker(int tid, int iters, size_t base_len, void *dev) {
    for (int i = 0; i < iters; ++i) {
        const size_t len = base_len << (i % 4);  // 2, 4, 8, 16 MB (as batches vary)
        const size_t kHuge = 2u << 20;
        // an anonymous mapping (what posix_memalign hands out for blocks this
        // large), so the block's addresses can be mapped again after munmap
        void *m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) continue;
        (void)kHuge;
        madvise(m, len, MADV_HUGEPAGE);
        memset(m, tid + 1, len);
        if (hipHostRegister(m, len, hipHostRegisterMapped) != hipSuccess) {
            (void)hipGetLastError();
            ++n_reg_fail;
            munmap(m, len);
            continue;
        }
        void *dp = nullptr;
        hipHostGetDevicePointer(&dp, m, 0);
        hipMemcpy(dev, m, 1 << 20, hipMemcpyHostToDevice);  // used for a copy while registered
        int ty = 0;
        const hipError_t ue = hipHostUnregister(m);
        if (ue != hipSuccess) {
            (void)hipGetLastError();
            ++n_unreg_fail;
        }
        if (tracked(m, &ty)) {
            ++n_tracked_after_unreg;
            if (n_tracked_after_unreg < 5)
                fprintf(stderr, "thread %d iter %d: %p still tracked after hipHostUnregister (rc %d, type %d)\n", tid,
                        i, m, (int)ue, ty);
        }
        munmap(m, len);
        // the same addresses mapped again (as malloc / numpy would get them)
        void *n = mmap(m, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED_NOREPLACE, -1, 0);
        if (n == MAP_FAILED) n = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (n == MAP_FAILED) continue;
        if (n == m) ++n_same_va;
        memset(n, 0, 4096);
        if (tracked(n, &ty)) {
            ++n_tracked_reuse;
            if (n_tracked_reuse < 5)
                fprintf(stderr, "thread %d iter %d: reused block %p (old %p) tracked, type %d\n", tid, i, n, m, ty);
        }
        munmap(n, len);
        ++n_iter;
    }
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 8;
    const int iters = argc > 2 ? atoi(argv[2]) : 200;
    void *dev = nullptr;
    if (hipMalloc(&dev, 1 << 20) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    for (int t : {1, threads}) {
        n_iter = n_unreg_fail = n_tracked_after_unreg = n_same_va = n_tracked_reuse = n_reg_fail = 0;
        std::vector<std::thread> th;
        for (int k = 0; k < t; ++k) th.emplace_back(worker, k, iters, (size_t)2 << 20, dev);
        for (auto &x : th) x.join();
        printf("threads %d: iterations %ld, register failures %ld, unregister failures %ld, tracked right after "
               "unregister %ld, freed block reused at the same address %ld, reused block tracked %ld\n",
               t, n_iter.load(), n_reg_fail.load(), n_unreg_fail.load(), n_tracked_after_unreg.load(),
               n_same_va.load(), n_tracked_reuse.load());
        fflush(stdout);
    }
    hipFree(dev);
    return 0;
}
