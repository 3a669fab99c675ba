// membw8.hip -- which write ORDER is fast on every allocation?
// (Round 6: a pure write of the decode's output shape ran 5.66-6.89 TB/s from
// one allocation to the next at identical virtual addresses, membw7; the
// decode itself 2.63-3.13 ms on lineitem_full SF12.5.)
//
// Each trial allocates the decode's output shape (16 column buffers, lineitem_
// full SF12.5: 75,004,738 rows x {8,8,8,4,8,8,8,8,16,16,4,4,4,16,16,16} B) and
// writes every (column, row group) chunk -- 1 KiB per wave store, 1-wave
// persistent blocks, 16 per CU -- in several orders on the SAME buffers:
//   colmajor   chunks in column-major order, wave w takes chunks w, w+NW, ...,
//              each front to back (membw7)
//   lpt        chunks largest output first (the decode's queue order)
//   lpt-rot    lpt, but a wave starts its chunk at vector r = hash(chunk) % nvec
//              and wraps (concurrent waves at different offsets)
//   lpt-rev    lpt, odd chunks written back to front
//   shuffled   chunks in a random order
//   vecint     the flattened (chunk, vector) list in lpt order, wave w taking
//              vectors w, w+NW, ... (consecutive waves write consecutive vectors)
//   torch      one 4 KiB block per 256-thread workgroup over each buffer in turn
// argv: trials
//   hipcc -O3 --offload-arch=gfx950 scripts/membw8.hip -o scripts/membw8
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
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
    uint32_t nvec;  // 8 KiB... vectors of vbytes each
    uint32_t vkb;   // KiB per vector (4, 8, 16)
    uint32_t flags; // 1: rotate, 2: reverse
    uint32_t rot;
};

__global__ __launch_bounds__(64) void k_chunks(const Chunk *__restrict__ ch, uint32_t n) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        const Chunk k = ch[c];
        v4u x = {lane, c, 7u, 9u};
        for (uint32_t i = 0; i < k.nvec; ++i) {
            uint32_t v = i;
            if (k.flags & 1) {
                v = i + k.rot;
                if (v >= k.nvec) v -= k.nvec;
            }
            if (k.flags & 2) v = k.nvec - 1 - i;
            v4u *o = k.out + (size_t)v * k.vkb * 64;
            for (uint32_t b = 0; b < k.vkb; ++b) o[b * 64 + lane] = x + b;
        }
    }
}

// flattened vectors: item i -> (chunk, vector) via prefix of nvec
__global__ __launch_bounds__(64) void k_vecint(const Chunk *__restrict__ ch, const uint32_t *__restrict__ first,
                                               uint32_t n, uint32_t total) {
    const uint32_t lane = threadIdx.x;
    uint32_t c = 0;
    for (uint32_t it = blockIdx.x; it < total; it += gridDim.x) {
        while (c + 1 < n && first[c + 1] <= it) ++c;  // items ascend per wave
        const Chunk k = ch[c];
        const uint32_t v = it - first[c];
        v4u x = {lane, it, 7u, 9u};
        v4u *o = k.out + (size_t)v * k.vkb * 64;
        for (uint32_t b = 0; b < k.vkb; ++b) o[b * 64 + lane] = x + b;
    }
}

__global__ __launch_bounds__(256) void k_torch(v4u *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    out[i] = v4u{(uint32_t)i, 1u, 2u, 3u};
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 6;
    const uint64_t rows = 75004738, rg = 65536;
    const int ob[16] = {8, 8, 8, 4, 8, 8, 8, 8, 16, 16, 4, 4, 4, 16, 16, 16};
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 16;
    const uint32_t nrg = (uint32_t)(rows / rg);  // full row groups only
    Chunk *dch;
    uint32_t *dfirst;
    CK(hipMalloc(&dch, sizeof(Chunk) * 16 * nrg));
    CK(hipMalloc(&dfirst, sizeof(uint32_t) * 16 * nrg));
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
    std::mt19937 rng(42);
    for (int t = 0; t < trials; ++t) {
        std::vector<char *> bufs(16);
        for (int c = 0; c < 16; ++c) CK(hipMalloc(&bufs[c], rows * ob[c] + 4096));
        std::vector<Chunk> col;
        uint64_t wr = 0;
        for (int c = 0; c < 16; ++c)
            for (uint32_t g = 0; g < nrg; ++g) {
                col.push_back({(v4u *)(bufs[c] + g * rg * ob[c]), 64, (uint32_t)ob[c], 0, 0});
                wr += rg * ob[c];
            }
        std::vector<Chunk> lpt = col;
        std::stable_sort(lpt.begin(), lpt.end(), [](const Chunk &a, const Chunk &b) { return a.vkb > b.vkb; });
        auto run = [&](const std::vector<Chunk> &h) {
            CK(hipMemcpy(dch, h.data(), h.size() * sizeof(Chunk), hipMemcpyHostToDevice));
            return timeit([&] { k_chunks<<<grid, 64>>>(dch, (uint32_t)h.size()); });
        };
        printf("trial %d (first buffer %p):", t, (void *)bufs[0]);
        const float m_col = run(col);
        const float m_lpt = run(lpt);
        std::vector<Chunk> rot = lpt;
        for (size_t i = 0; i < rot.size(); ++i) {
            rot[i].flags = 1;
            rot[i].rot = (uint32_t)((i * 2654435761u) >> 26) & 63;
        }
        const float m_rot = run(rot);
        std::vector<Chunk> rev = lpt;
        for (size_t i = 1; i < rev.size(); i += 2) rev[i].flags = 2;
        const float m_rev = run(rev);
        std::vector<Chunk> shuf = col;
        std::shuffle(shuf.begin(), shuf.end(), rng);
        const float m_shuf = run(shuf);
        std::vector<uint32_t> first(lpt.size());
        uint32_t tot = 0;
        for (size_t i = 0; i < lpt.size(); ++i) {
            first[i] = tot;
            tot += lpt[i].nvec;
        }
        CK(hipMemcpy(dch, lpt.data(), lpt.size() * sizeof(Chunk), hipMemcpyHostToDevice));
        CK(hipMemcpy(dfirst, first.data(), first.size() * 4, hipMemcpyHostToDevice));
        const float m_vi = timeit([&] { k_vecint<<<grid, 64>>>(dch, dfirst, (uint32_t)lpt.size(), tot); });
        const float m_torch = timeit([&] {
            for (int c = 0; c < 16; ++c) k_torch<<<(unsigned)(nrg * rg * ob[c] / 4096), 256>>>((v4u *)bufs[c]);
        });
        auto gbs = [&](float ms) { return wr / ms / 1e6; };
        printf(" colmajor %.0f | lpt %.0f | lpt-rot %.0f | lpt-rev %.0f | shuffled %.0f | vecint %.0f | torch %.0f GB/s\n",
               gbs(m_col), gbs(m_lpt), gbs(m_rot), gbs(m_rev), gbs(m_shuf), gbs(m_vi), gbs(m_torch));
        fflush(stdout);
        for (int c = 0; c < 16; ++c) CK(hipFree(bufs[c]));
    }
    return 0;
}
