// membw9.hip -- what makes a write sweep fast on every allocation?
// (membw8: a non-persistent fill, one 4 KiB block per 256-thread workgroup,
// wrote the decode's 16 output buffers at 6.82-6.93 TB/s on all 8
// allocations, while persistent waves that each own whole row-group chunks
// ran 5.3-6.75 TB/s depending on the allocation.)
//
// Same buffers (lineitem_full SF12.5 output shape), re-allocated per trial;
// every variant writes each buffer completely, one launch per buffer (like
// a torch fill) unless noted:
//   torch     non-persistent, 256 threads x 16 B = 4 KiB per workgroup
//   np1k      non-persistent, 64 threads = 1 KiB per workgroup
//   np16k     non-persistent, 256 threads x 4 stores = 16 KiB per workgroup
//   pw<G>     persistent 1-wave blocks (16 per CU), wave w writes G KiB granules
//             w, w + NW, ... (G = 1, 4, 8, 16)
//   pg4       persistent 4-wave blocks (4 per CU), block b writes 4 KiB
//             granules b, b + NB, ... (one 1 KiB store per wave)
//   chunks    persistent 1-wave blocks, ONE launch, wave w owns row-group
//             chunks w, w + NW, ... in largest-first order (the decode)
// argv: trials
//   hipcc -O3 --offload-arch=gfx950 scripts/membw9.hip -o scripts/membw9
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

template <int TPB, int PER>
__global__ __launch_bounds__(TPB) void k_np(v4u *__restrict__ out) {
    const size_t base = (size_t)blockIdx.x * TPB * PER + threadIdx.x;
#pragma unroll
    for (int k = 0; k < PER; ++k) out[base + k * TPB] = v4u{(uint32_t)base, 1u, 2u, (uint32_t)k};
}

// persistent 1-wave blocks, granules of G KiB (G stores of 1 KiB per wave)
template <int G>
__global__ __launch_bounds__(64) void k_pw(v4u *__restrict__ out, size_t ngran) {
    const uint32_t lane = threadIdx.x;
    for (size_t g = blockIdx.x; g < ngran; g += gridDim.x) {
        v4u *o = out + g * G * 64;
#pragma unroll
        for (int j = 0; j < G; ++j) o[j * 64 + lane] = v4u{lane, (uint32_t)g, 7u, (uint32_t)j};
    }
}

// persistent 4-wave blocks, 4 KiB per block per iteration
__global__ __launch_bounds__(256) void k_pg4(v4u *__restrict__ out, size_t ngran) {
    for (size_t g = blockIdx.x; g < ngran; g += gridDim.x) out[g * 256 + threadIdx.x] = v4u{threadIdx.x, (uint32_t)g, 7u, 9u};
}

struct Chunk {
    v4u *out;
    uint32_t kib;
};
__global__ __launch_bounds__(64) void k_chunks(const Chunk *__restrict__ ch, uint32_t n) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        const Chunk k = ch[c];
        for (uint32_t b = 0; b < k.kib; ++b) k.out[b * 64 + lane] = v4u{lane, c, 7u, b};
    }
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 6;
    const uint64_t rows = 75004738, rg = 65536;
    const int ob[16] = {8, 8, 8, 4, 8, 8, 8, 8, 16, 16, 4, 4, 4, 16, 16, 16};
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t nrg = (uint32_t)(rows / rg);
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
    uint64_t wr = 0;
    for (int c = 0; c < 16; ++c) wr += nrg * rg * ob[c];
    for (int t = 0; t < trials; ++t) {
        std::vector<v4u *> bufs(16);
        std::vector<size_t> kib(16);
        for (int c = 0; c < 16; ++c) {
            CK(hipMalloc(&bufs[c], rows * ob[c] + 4096));
            kib[c] = nrg * rg * ob[c] / 1024;
        }
        std::vector<Chunk> lpt;
        for (int c = 0; c < 16; ++c)
            for (uint32_t g = 0; g < nrg; ++g) lpt.push_back({bufs[c] + (size_t)g * rg * ob[c] / 16, (uint32_t)(rg * ob[c] / 1024)});
        std::stable_sort(lpt.begin(), lpt.end(), [](const Chunk &a, const Chunk &b) { return a.kib > b.kib; });
        CK(hipMemcpy(dch, lpt.data(), lpt.size() * sizeof(Chunk), hipMemcpyHostToDevice));
        auto gbs = [&](float ms) { return wr / ms / 1e6; };
        const int nw = cus * 16;
        printf("trial %d:", t);
        printf(" torch %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_np<256, 1><<<kib[c] / 4, 256>>>(bufs[c]); })));
        printf(" np1k %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_np<64, 1><<<kib[c], 64>>>(bufs[c]); })));
        printf(" np16k %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_np<256, 4><<<kib[c] / 16, 256>>>(bufs[c]); })));
        printf(" pw1 %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_pw<1><<<nw, 64>>>(bufs[c], kib[c]); })));
        printf(" pw4 %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_pw<4><<<nw, 64>>>(bufs[c], kib[c] / 4); })));
        printf(" pw8 %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_pw<8><<<nw, 64>>>(bufs[c], kib[c] / 8); })));
        printf(" pw16 %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_pw<16><<<nw, 64>>>(bufs[c], kib[c] / 16); })));
        printf(" pg4 %.0f", gbs(timeit([&] { for (int c = 0; c < 16; ++c) k_pg4<<<cus * 4, 256>>>(bufs[c], kib[c] / 4); })));
        printf(" chunks %.0f GB/s\n", gbs(timeit([&] { k_chunks<<<nw, 64>>>(dch, (uint32_t)lpt.size()); })));
        fflush(stdout);
        for (int c = 0; c < 16; ++c) CK(hipFree(bufs[c]));
    }
    return 0;
}
