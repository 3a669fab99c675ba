// d2h_probe.hip -- PCIe copy rates of one process, by copy engine (round 6:
// a plain 1 GiB hipMemcpy D2H into hipHostMalloc memory ran 57.1 GB/s in some
// fresh processes and 30.2 in others on one box, link at 32 GT/s x16 and clocks
// unchanged throughout, profiles/r6/e2e_numa_r6am.txt).  Per process:
//   memcpy      hipMemcpy D2H / H2D (SDMA unless HSA_ENABLE_SDMA=0)
//   async2      two hipMemcpyAsync D2H halves on two streams
//   kernel      a copy kernel: device loads, stores to the pinned host buffer
//               (D2H) or host loads, device stores (H2D); 16 B per lane
// argv: MiB (default 1024)
//   hipcc -O3 --offload-arch=gfx950 scripts/d2h_probe.hip -o scripts/d2h_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ __launch_bounds__(256) void k_copy(v4u *__restrict__ dst, const v4u *__restrict__ src, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

int main(int argc, char **argv) {
    const size_t nb = (size_t)(argc > 1 ? atoi(argv[1]) : 1024) << 20;
    void *h, *d;
    CK(hipHostMalloc(&h, nb, 0));
    CK(hipMalloc(&d, nb));
    CK(hipMemset(d, 1, nb));
    memset(h, 2, nb);
    hipStream_t s[2];
    for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    auto best = [&](auto f) {
        f();
        CK(hipDeviceSynchronize());
        double b = 0;
        for (int r = 0; r < 3; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            f();
            CK(hipDeviceSynchronize());
            double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            b = b > nb / sec / 1e9 ? b : nb / sec / 1e9;
        }
        return b;
    };
    const double md = best([&] { CK(hipMemcpy(h, d, nb, hipMemcpyDeviceToHost)); });
    const double mh = best([&] { CK(hipMemcpy(d, h, nb, hipMemcpyHostToDevice)); });
    const double a2 = best([&] {
        for (int i = 0; i < 2; ++i)
            CK(hipMemcpyAsync((char *)h + i * nb / 2, (char *)d + i * nb / 2, nb / 2, hipMemcpyDeviceToHost, s[i]));
    });
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double kd[3], kh[3];
    const int grids[3] = {cus, cus * 4, cus * 16};
    for (int g = 0; g < 3; ++g) {
        kd[g] = best([&] { k_copy<<<grids[g], 256>>>((v4u *)h, (const v4u *)d, nb / 16); });
        kh[g] = best([&] { k_copy<<<grids[g], 256>>>((v4u *)d, (const v4u *)h, nb / 16); });
    }
    printf("memcpy d2h %.1f h2d %.1f | async2 d2h %.1f | kernel d2h %.1f/%.1f/%.1f h2d %.1f/%.1f/%.1f GB/s "
           "(grids %d/%d/%d)\n",
           md, mh, a2, kd[0], kd[1], kd[2], kh[0], kh[1], kh[2], grids[0], grids[1], grids[2]);
    CK(hipHostFree(h));
    CK(hipFree(d));
    return 0;
}
