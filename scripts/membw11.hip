// membw11.hip -- is C3's DELTA64 store ORDER what keeps it below the write
// ceiling?  (c3: 1e9 INT64 keys, 8 GB written at 4.9-5.2 TB/s, 81.5 % of wave
// cycles waiting to issue stores, PMC traffic = algorithmic.)  delta64_vec
// (csrc/fls_decode_dev.hpp) writes a vector's 8 KiB in 8 store instructions,
// instruction j putting lane group g's 128 B at segment 8 bitrev3(g) + j:
// eight 128-B pieces 1 KiB apart per instruction.  The FFOR path writes 1 KiB
// contiguous per instruction.  Same buffers, same chunk order (c3's shape:
// 15,259 chunks of 64 vectors, 512 KiB each, whole chunks per wave, 4-wave
// blocks, persistent), store forms:
//   contig    instruction j: bytes [1024 j, 1024 j + 1024) of the vector
//   delta     instruction j: 128 (8 bitrev3(g) + j) + 16 q  (g = lane>>3, q = lane&7)
// each with the default policy and with sc1 nt (DELTA64's, policy bits 18).
// Per trial a new allocation (placement), the four modes interleaved on it.
// argv: trials blocks_per_cu
//   hipcc -O3 --offload-arch=gfx950 scripts/membw11.hip -o scripts/membw11
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t bitrev3(uint32_t g) { return ((g & 1) << 2) | (g & 2) | ((g >> 2) & 1); }
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

template <int CPOL>
__device__ __forceinline__ void st(uint8_t *vec, uint32_t off, v4u v) {
    if constexpr (CPOL != 0) {
        const uint64_t b = (uint64_t)vec;
        void *ub = (void *)((uint64_t)uni((uint32_t)(b >> 32)) << 32 | (uint64_t)uni((uint32_t)b));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, CPOL);
    } else {
        *reinterpret_cast<v4u *>(vec + off) = v;
    }
}

template <bool DELTA, int CPOL>
__global__ __launch_bounds__(256) void k_write(uint8_t *__restrict__ out, uint32_t nchunks) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t g = lane >> 3, q = lane & 7, s = bitrev3(g);
    const uint32_t stride = gridDim.x * 4;
    for (uint32_t c = blockIdx.x * 4 + w; c < nchunks; c += stride) {
        for (uint32_t v = 0; v < 64; ++v) {
            uint8_t *vec = out + ((size_t)c * 64 + v) * 8192;
            v4u x = {lane, v, c, 7u};
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t off = DELTA ? 128 * (8 * s + j) + 16 * q : 1024 * j + 16 * lane;
                st<CPOL>(vec, off, x + j);
            }
        }
    }
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 4;
    const int bpc = argc > 2 ? atoi(argv[2]) : 4;
    const uint32_t nchunks = 15259;
    const size_t bytes = (size_t)nchunks * 64 * 8192;
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        return bytes / best / 1e6;  // GB/s
    };
    const dim3 grid(cus * bpc), blk(256);
    printf("c3-shaped write, %zu bytes, %u chunks, grid %d x 256 (%d blocks per CU)\n", bytes, nchunks, cus * bpc, bpc);
    for (int t = 0; t < trials; ++t) {
        uint8_t *out;
        CK(hipMalloc(&out, bytes));
        const double c0 = timeit([&] { k_write<false, 0><<<grid, blk>>>(out, nchunks); });
        const double d0 = timeit([&] { k_write<true, 0><<<grid, blk>>>(out, nchunks); });
        const double c18 = timeit([&] { k_write<false, 18><<<grid, blk>>>(out, nchunks); });
        const double d18 = timeit([&] { k_write<true, 18><<<grid, blk>>>(out, nchunks); });
        printf("trial %d: contig %.0f / delta %.0f GB/s (default) | contig %.0f / delta %.0f GB/s (sc1 nt)\n", t, c0, d0,
               c18, d18);
        fflush(stdout);
        CK(hipFree(out));
    }
    return 0;
}
