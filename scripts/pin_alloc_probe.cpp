// pin_alloc_probe.cpp -- how fast a process gets pinned host memory, by thread
// count (round 6: the file's first read_fastlanes query runs ~220 M rows/s
// against ~830 warm, and its pinned host batches come from hipHostMalloc at
// 4-5 GB/s on one thread).  Per config: T threads together allocate TOTAL
// bytes in CHUNK-sized hipHostMalloc calls (then the same with hipHostFree
// timed), GB/s of the aggregate.  A fresh process per run: argv threads chunk_mb
// total_mb.
//   hipcc -O2 scripts/pin_alloc_probe.cpp -o scripts/pin_alloc_probe -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 1;
    const size_t chunk = (size_t)(argc > 2 ? atoi(argv[2]) : 8) << 20;
    const size_t total = (size_t)(argc > 3 ? atoi(argv[3]) : 2048) << 20;
    if (hipFree(nullptr) != hipSuccess) return 1;  // runtime up before timing
    const size_t n = total / chunk;
    std::vector<void *> p(n, nullptr);
    auto run = [&](auto f) {
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (size_t i = t; i < n; i += T) f(i);
            });
        for (auto &x : th) x.join();
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    };
    int bad = 0;
    const double ta = run([&](size_t i) { bad |= hipHostMalloc(&p[i], chunk, hipHostMallocDefault) != hipSuccess; });
    const double tf = run([&](size_t i) { bad |= hipHostFree(p[i]) != hipSuccess; });
    const double ta2 = run([&](size_t i) { bad |= hipHostMalloc(&p[i], chunk, hipHostMallocDefault) != hipSuccess; });
    printf("threads %d chunk %zu MB total %zu MB: alloc %.2f GB/s (again after free %.2f), free %.2f GB/s%s\n", T,
           chunk >> 20, total >> 20, total / ta / 1e9, total / ta2 / 1e9, total / tf / 1e9, bad ? " ERRORS" : "");
    for (auto q : p) (void)hipHostFree(q);
    return bad;
}
