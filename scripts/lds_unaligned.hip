// lds_unaligned.hip -- does gfx950 honour byte-unaligned ds_write_b64 (the
// FSST ring writer's exact-window stores), and what does it cost against
// aligned ds_write_b64 and ds_or_b64?  Standalone probe, not product code.
//   hipcc -O3 --offload-arch=gfx950 scripts/lds_unaligned.hip -o scripts/lds_unaligned
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__device__ __forceinline__ void ds_w64(uint32_t addr, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// correctness: lane l writes bytes (l*7+1)+[0,8) = l*16+k ... lanes in
// descending order of issue? no: one instruction, disjoint ranges 7 apart would
// overlap, so lanes write at stride 9 (disjoint) with arbitrary misalignment.
__global__ void probe(uint8_t *out, uint32_t stride, uint32_t off) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 4096; i += 64) lds[i] = 0xEE;
    __syncthreads();
    uint64_t v = 0;
    for (int k = 0; k < 8; ++k) v |= (uint64_t)((lane * 8 + k) & 0xFF) << (8 * k);
    const uint32_t base = (uint32_t)(uintptr_t)(&lds[0]);
    ds_w64(base + off + stride * lane, v);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    for (uint32_t i = lane; i < 4096; i += 64) out[i] = lds[i];
}

// throughput: each wave does N rounds of 8 stores; mode 0 aligned b64,
// 1 unaligned b64 (lane stride 17 B), 2 ds_or_b64 aligned at stride 16 B
template <int MODE>
__global__ void tput(uint32_t *sink, int rounds) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t *L = lds + w * 2048;
    const uint32_t base = (uint32_t)(uintptr_t)L;
    uint64_t v = lane * 0x0101010101010101ull;
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (MODE == 0) ds_w64(base + 16 * lane + 8 * (k & 1), v + k);
            if (MODE == 1) ds_w64(base + 17 * lane + 3 * k, v + k);
            if (MODE == 2)
                __hip_atomic_fetch_or((__attribute__((address_space(3))) uint64_t *)(L + 16 * lane + 8 * (k & 1)), v + k,
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        v += 0x9E3779B97F4A7C15ull;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) sink[blockIdx.x] = L[5];
}

int main() {
    uint8_t *d;
    CK(hipMalloc(&d, 4096));
    std::vector<uint8_t> h(4096);
    int bad = 0;
    for (uint32_t off : {0u, 1u, 2u, 3u, 5u, 7u}) {
        for (uint32_t stride : {8u, 9u, 11u, 13u}) {
            probe<<<1, 64>>>(d, stride, off);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), d, 4096, hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < 4096; ++i) {
                uint8_t exp = 0xEE;
                if (i >= off) {
                    const uint32_t l = (i - off) / stride, k = (i - off) % stride;
                    if (l < 64 && k < 8) exp = (uint8_t)((l * 8 + k) & 0xFF);
                }
                if (h[i] != exp) {
                    if (bad < 10) printf("off %u stride %u byte %u: got %02x want %02x\n", off, stride, i, h[i], exp);
                    ++bad;
                }
            }
        }
    }
    printf("unaligned ds_write_b64 correctness: %s (%d bad bytes)\n", bad ? "FAIL" : "ok", bad);
    uint32_t *sink;
    CK(hipMalloc(&sink, 1 << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int blocks = 256 * 4, rounds = 4096, threads = 256;  // 4 waves/block, 16 waves/CU
    const char *names[3] = {"aligned ds_write_b64", "unaligned ds_write_b64", "aligned ds_or_b64"};
    for (int rep = 0; rep < 2; ++rep)
        for (int m = 0; m < 3; ++m) {
            CK(hipEventRecord(a));
            if (m == 0) tput<0><<<blocks, threads, 4 * 2048>>>(sink, rounds);
            if (m == 1) tput<1><<<blocks, threads, 4 * 2048>>>(sink, rounds);
            if (m == 2) tput<2><<<blocks, threads, 4 * 2048>>>(sink, rounds);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double ops = (double)blocks * 4 * rounds * 8;  // wave-instructions
            if (rep) printf("%-24s %8.3f ms  %.2f wave-instr per CU-cycle (2.4 GHz)\n", names[m], ms,
                            ops / 256 / (ms * 1e-3 * 2.4e9));
        }
    return bad ? 1 : 0;
}
