// pin_bench.cpp -- what page-locking host memory costs on the GPU box (the
// scan pipeline's pinned host batches are the cold query's largest one-time
// cost, profiles/r5/): hipHostMalloc against malloc + hipHostRegister, with
// and without transparent huge pages, in 1 and 4 threads.  Host-side probe,
// no kernels.
//   hipcc -O2 scripts/pin_bench.cpp -o scripts/pin_bench && scripts/pin_bench [MB]
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const size_t mb = argc > 1 ? (size_t)atol(argv[1]) : 512;
    const size_t chunk = 16ull << 20, n = (mb << 20) / chunk;
    if (hipSetDevice(0) != hipSuccess) return 1;
    hipFree(nullptr);
    for (int mode = 0; mode < 4; ++mode) {
        for (int threads : {1, 4}) {
            std::vector<void *> p(n, nullptr);
            const double t0 = now();
            auto work = [&](int t) {
                for (size_t i = t; i < n; i += threads) {
                    if (mode == 0) {
                        if (hipHostMalloc(&p[i], chunk, hipHostMallocDefault) != hipSuccess) p[i] = nullptr;
                    } else {
                        void *m = nullptr;
                        if (posix_memalign(&m, 2u << 20, chunk)) continue;
                        if (mode >= 2) madvise(m, chunk, MADV_HUGEPAGE);
                        if (mode == 3) memset(m, 0, chunk);  // fault the pages in first
                        if (hipHostRegister(m, chunk, hipHostRegisterDefault) != hipSuccess) {
                            free(m);
                            continue;
                        }
                        p[i] = m;
                    }
                }
            };
            std::vector<std::thread> th;
            for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
            work(0);
            for (auto &x : th) x.join();
            const double t1 = now();
            size_t ok = 0;
            for (void *q : p) ok += q != nullptr;
            const char *names[] = {"hipHostMalloc", "malloc+register", "malloc+THP+register", "malloc+THP+touch+register"};
            printf("%-28s %d thread(s): %zu x 16 MB in %7.1f ms = %6.2f GB/s\n", names[mode], threads, ok,
                   (t1 - t0) * 1e3, ok * chunk / (t1 - t0) / 1e9);
            for (void *q : p) {
                if (!q) continue;
                if (mode == 0) hipHostFree(q);
                else {
                    hipHostUnregister(q);
                    free(q);
                }
            }
        }
    }
    return 0;
}
