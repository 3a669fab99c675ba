// membw10.hip -- the ceiling for the main decode's traffic MIX on a rated
// placement: the decode reads ~1 byte of packed input per 8 bytes it writes
// (SF100 main columns: 10.65 GB packed + 0.36 GB metadata read, 76.8 GB
// written).  How fast does a pure stream of that mix run, without any decode
// work?  (Round 6: the fused SF100 step moves 5.79 TB/s, the main decode alone
// 5.68 TB/s, a pure write of the same outputs 6.9 TB/s.)
//
// Per trial: the decode's output shape (16 column buffers, lineitem_full
// SF12.5) and an input buffer of 1/8 of it.  Kernels (persistent 1-wave
// blocks, 16 per CU, wave w takes row-group chunks w, w + NW, ... in
// largest-first order, 1 KiB per store instruction):
//   write      stores only (the placement probe's stream)
//   mix1       per 8 KiB of output one 1 KiB load, consumed one vector later
//   mix2       the same, loads issued two vectors ahead
//   fill       a linear fill (4 KiB per 256-thread workgroup) of the buffers
// argv: trials
//   hipcc -O3 --offload-arch=gfx950 scripts/membw10.hip -o scripts/membw10
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

struct Chunk {
    v4u *out;
    const v4u *in;   // 1/8 of the chunk's output bytes
    uint32_t kib;    // output KiB (a multiple of 8)
    uint32_t pad;
};

template <int MODE>  // 0 write, 1 one vector ahead, 2 two vectors ahead
__global__ __launch_bounds__(64) void k_mix(const Chunk *__restrict__ ch, uint32_t n) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        const Chunk k = ch[c];
        const uint32_t nv = k.kib / 8;
        v4u acc = {lane, c, 7u, 9u};
        v4u a = acc, b = acc;
        if (MODE >= 1) a = k.in[lane];
        if (MODE == 2 && nv > 1) b = k.in[64 + lane];
        for (uint32_t v = 0; v < nv; ++v) {
            v4u cur = acc;
            if (MODE == 1) {
                cur = a;
                if (v + 1 < nv) a = k.in[(size_t)(v + 1) * 64 + lane];
            } else if (MODE == 2) {
                cur = a;
                a = b;
                if (v + 2 < nv) b = k.in[(size_t)(v + 2) * 64 + lane];
            }
            v4u *o = k.out + (size_t)v * 512;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) o[j * 64 + lane] = cur + j;
        }
    }
}

__global__ __launch_bounds__(256) void k_fill(v4u *__restrict__ out) {
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = v4u{(uint32_t)blockIdx.x, 1u, 2u, 3u};
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 6;
    const uint64_t rows = 75004738, rg = 65536;
    const int ob[16] = {8, 8, 8, 4, 8, 8, 8, 8, 16, 16, 4, 4, 4, 16, 16, 16};
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t nrg = (uint32_t)(rows / rg);
    uint64_t wr = 0;
    for (int c = 0; c < 16; ++c) wr += (uint64_t)nrg * rg * ob[c];
    Chunk *dch;
    CK(hipMalloc(&dch, sizeof(Chunk) * 16 * nrg));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float sum = 0;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            sum += ms;
        }
        return sum / 6;
    };
    for (int t = 0; t < trials; ++t) {
        std::vector<v4u *> bufs(16);
        for (int c = 0; c < 16; ++c) CK(hipMalloc(&bufs[c], rows * ob[c] + 4096));
        v4u *in;
        CK(hipMalloc(&in, wr / 8 + 4096));
        CK(hipMemset(in, 1, wr / 8));
        std::vector<Chunk> lpt;
        uint64_t ioff = 0;
        for (int c = 0; c < 16; ++c)
            for (uint32_t g = 0; g < nrg; ++g) {
                const uint32_t kib = (uint32_t)(rg * ob[c] / 1024);
                lpt.push_back({bufs[c] + (size_t)g * rg * ob[c] / 16, in + ioff / 16, kib, 0});
                ioff += (uint64_t)kib * 128;
            }
        std::stable_sort(lpt.begin(), lpt.end(), [](const Chunk &a, const Chunk &b) { return a.kib > b.kib; });
        CK(hipMemcpy(dch, lpt.data(), lpt.size() * sizeof(Chunk), hipMemcpyHostToDevice));
        const uint32_t n = (uint32_t)lpt.size();
        const float mw = timeit([&] { k_mix<0><<<cus * 16, 64>>>(dch, n); });
        const float m1 = timeit([&] { k_mix<1><<<cus * 16, 64>>>(dch, n); });
        const float m2 = timeit([&] { k_mix<2><<<cus * 16, 64>>>(dch, n); });
        const float mf = timeit([&] {
            for (int c = 0; c < 16; ++c) k_fill<<<(unsigned)(nrg * rg * ob[c] / 4096), 256>>>(bufs[c]);
        });
        const double rd = (double)wr / 8;
        printf("trial %d: write %.0f GB/s (q %.3f) | mix1 %.0f GB/s total (%.0f written) | mix2 %.0f total (%.0f "
               "written) | fill %.0f GB/s\n",
               t, wr / mw / 1e6, mf / mw, (wr + rd) / m1 / 1e6, wr / m1 / 1e6, (wr + rd) / m2 / 1e6, wr / m2 / 1e6,
               wr / mf / 1e6);
        fflush(stdout);
        for (int c = 0; c < 16; ++c) CK(hipFree(bufs[c]));
        CK(hipFree(in));
    }
    return 0;
}
