// membw7.hip -- does a pure write stream's speed change from one allocation
// to the next?  (Round 6: the same decode at the same virtual addresses ran
// 2.78 or 3.12 ms on lineitem_full SF12.5 depending on the trial,
// profiles/r6/placement_*.txt.)
//
// Each trial allocates the decode's output shape -- 16 column buffers of
// 75,004,738 rows x {8,8,8,4,8,8,8,8,16,16,4,4,4,16,16,16} bytes (lineitem_full
// SF12.5: int64 keys/decimals, int32 dates/codes, 16-B string_t) -- writes
// every row group's output chunk (65,536 rows) with persistent 1-wave blocks
// (wave w takes chunks w, w + NW, ...; column-major order like the decode's
// queue), 1 KiB per store instruction, and then the same bytes as ONE buffer;
// times both, frees everything.  argv: trials, allocation flags (4 = contiguous).
//   hipcc -O3 --offload-arch=gfx950 scripts/membw7.hip -o scripts/membw7
#include <hip/hip_runtime.h>

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
    uint64_t bytes;
};

__global__ __launch_bounds__(64) void k_chunks(const Chunk *__restrict__ ch, uint32_t n) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t c = blockIdx.x; c < n; c += gridDim.x) {
        v4u *o = ch[c].out;
        const uint64_t nb = ch[c].bytes >> 10;
        v4u x = {lane, c, 7u, 9u};
        for (uint64_t b = 0; b < nb; ++b) o[b * 64 + lane] = x + (uint32_t)b;
    }
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 8;
    // allocation flags: 0 = hipMalloc, else hipExtMallocWithFlags (4 = hipDeviceMallocContiguous)
    const unsigned flags = argc > 2 ? (unsigned)atoi(argv[2]) : 0;
    auto dmalloc = [&](char **p, size_t n) {
        if (!flags) return hipMalloc(p, n);
        return hipExtMallocWithFlags((void **)p, n, flags);
    };
    printf("allocation flags %u\n", flags);
    const uint64_t rows = 75004738, rg = 65536;
    const int ob[16] = {8, 8, 8, 4, 8, 8, 8, 8, 16, 16, 4, 4, 4, 16, 16, 16};
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 16;
    uint64_t total = 0;
    for (int c = 0; c < 16; ++c) total += rows * ob[c];
    Chunk *dch;
    const uint32_t nrg = (uint32_t)((rows + rg - 1) / rg);
    CK(hipMalloc(&dch, sizeof(Chunk) * 16 * nrg));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const std::vector<Chunk> &h) {
        CK(hipMemcpy(dch, h.data(), h.size() * sizeof(Chunk), hipMemcpyHostToDevice));
        k_chunks<<<grid, 64>>>(dch, (uint32_t)h.size());
        CK(hipDeviceSynchronize());
        float best = 1e9, sum = 0;
        for (int r = 0; r < 10; ++r) {
            CK(hipEventRecord(e0));
            k_chunks<<<grid, 64>>>(dch, (uint32_t)h.size());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        return sum / 10;
    };
    for (int t = 0; t < trials; ++t) {
        // 16 column buffers
        std::vector<char *> bufs(16);
        for (int c = 0; c < 16; ++c) CK(dmalloc(&bufs[c], rows * ob[c] + 4096));
        std::vector<Chunk> h;
        for (int c = 0; c < 16; ++c)
            for (uint64_t g = 0; g < nrg; ++g) {
                const uint64_t r0 = g * rg, n = (r0 + rg <= rows ? rg : rows - r0);
                h.push_back({(v4u *)(bufs[c] + r0 * ob[c]), (n * ob[c]) & ~1023ull});
            }
        uint64_t wr = 0;
        for (auto &x : h) wr += x.bytes;
        const float ms16 = timed(h);
        for (int c = 0; c < 16; ++c) CK(hipFree(bufs[c]));
        // one buffer of the same total
        char *one;
        CK(dmalloc(&one, total + 4096 * 16));
        std::vector<Chunk> h1;
        uint64_t off = 0;
        for (int c = 0; c < 16; ++c) {
            for (uint64_t g = 0; g < nrg; ++g) {
                const uint64_t r0 = g * rg, n = (r0 + rg <= rows ? rg : rows - r0);
                h1.push_back({(v4u *)(one + off + r0 * ob[c]), (n * ob[c]) & ~1023ull});
            }
            off += (rows * ob[c] + 4095) & ~4095ull;
        }
        const float ms1 = timed(h1);
        printf("trial %d: 16 buffers %.4f ms = %.1f GB/s (first %p) | one buffer %.4f ms = %.1f GB/s (%p)\n", t, ms16,
               wr / ms16 / 1e6, (void *)bufs[0], ms1, wr / ms1 / 1e6, (void *)one);
        fflush(stdout);
        CK(hipFree(one));
    }
    return 0;
}
