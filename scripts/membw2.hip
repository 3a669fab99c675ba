// membw2.hip -- which WRITE pattern reaches the fill rate on this GPU?
// torch.fill_ of 8 GiB runs ~6.3 TB/s on the box while membw.hip's persistent
// grid-stride store loop tops at ~5.4.  The decode kernel writes per-wave
// private streams (a wave owns a column chunk: up to 1 MiB contiguous output),
// so this compares, at 8 GiB of 16-B-per-lane stores:
//   memset      hipMemsetD32 (the runtime's fill kernel)
//   oneshot U   one block per 256*U*16 B, block exits after U stores per lane
//   stride  B   persistent grid-stride, B blocks per CU
//   private R   persistent waves, each owning R-byte contiguous regions,
//               8 x 1 KiB store instructions per iteration (the decode shape)
//   privil  R   as private, but region r is split over 8 waves interleaved
//               at 8 KiB (concurrent waves write adjacent 8 KiB blocks)
//   hipcc -O3 --offload-arch=gfx950 scripts/membw2.hip -o /tmp/membw2 && /tmp/membw2
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

template <int U, int NT>
__global__ __launch_bounds__(256) void k_oneshot(v4u *__restrict__ out) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    const v4u v = {threadIdx.x, blockIdx.x, 7u, 9u};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (NT) __builtin_nontemporal_store(v, out + base + (size_t)u * 256);
        else out[base + (size_t)u * 256] = v;
    }
}

__global__ __launch_bounds__(256) void k_stride(v4u *__restrict__ out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    const v4u v = {threadIdx.x, blockIdx.x, 7u, 9u};
    for (size_t i = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; i < n16; i += stride) {
#pragma unroll
        for (int u = 0; u < 4; ++u) out[i + (size_t)u * 256] = v;
    }
}

// wave-private regions of R bytes: wave w takes regions w, w+nw, ...
__global__ __launch_bounds__(256) void k_private(v4u *__restrict__ out, size_t nreg, size_t r16) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (size_t)gridDim.x * 4;
    for (size_t r = wave; r < nreg; r += nw) {
        v4u *o = out + r * r16;
        for (size_t b = 0; b < r16; b += 512) {
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const v4u v = {lane, j, (uint32_t)b, 1u};
                o[b + 64 * j + lane] = v;
            }
        }
    }
}

// region-owning groups of 8 waves: wave k of a group writes 8 KiB blocks k, k+8, ...
__global__ __launch_bounds__(256) void k_privil(v4u *__restrict__ out, size_t nreg, size_t r16) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (size_t)gridDim.x * 4;
    const size_t grp = wave / 8, ng = nw / 8, k = wave % 8;
    for (size_t r = grp; r < nreg; r += ng) {
        v4u *o = out + r * r16;
        for (size_t b = k * 512; b < r16; b += 8 * 512) {
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const v4u v = {lane, j, (uint32_t)b, 1u};
                o[b + 64 * j + lane] = v;
            }
        }
    }
}

template <class F>
double time_ms(F f, int reps = 10) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t bytes = 8ull << 30;
    const size_t n16 = bytes / 16;
    v4u *out;
    CK(hipMalloc(&out, bytes));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double ms;
    for (int rep = 0; rep < 2; ++rep) {
        ms = time_ms([&] { CK(hipMemsetD32((hipDeviceptr_t)out, 0x01020304, bytes / 4)); });
        printf("memset D32             : %7.1f GB/s\n", bytes / ms / 1e6);
        ms = time_ms([&] { k_oneshot<1, 0><<<n16 / 256, 256>>>(out); });
        printf("oneshot U1             : %7.1f GB/s\n", bytes / ms / 1e6);
        ms = time_ms([&] { k_oneshot<4, 0><<<n16 / 1024, 256>>>(out); });
        printf("oneshot U4             : %7.1f GB/s\n", bytes / ms / 1e6);
        ms = time_ms([&] { k_oneshot<8, 0><<<n16 / 2048, 256>>>(out); });
        printf("oneshot U8             : %7.1f GB/s\n", bytes / ms / 1e6);
        ms = time_ms([&] { k_oneshot<4, 1><<<n16 / 1024, 256>>>(out); });
        printf("oneshot U4 nt          : %7.1f GB/s\n", bytes / ms / 1e6);
        for (int bpc : {2, 4, 8, 16}) {
            ms = time_ms([&] { k_stride<<<cus * bpc, 256>>>(out, n16); });
            printf("stride  %2d blk/CU      : %7.1f GB/s\n", bpc, bytes / ms / 1e6);
        }
        for (size_t R : {65536ul, 262144ul, 1048576ul}) {
            for (int bpc : {2, 4, 8}) {
                ms = time_ms([&] { k_private<<<cus * bpc, 256>>>(out, bytes / R, R / 16); });
                printf("private %7zu B %d blk/CU: %7.1f GB/s\n", R, bpc, bytes / ms / 1e6);
                ms = time_ms([&] { k_privil<<<cus * bpc, 256>>>(out, bytes / R, R / 16); });
                printf("privil  %7zu B %d blk/CU: %7.1f GB/s\n", R, bpc, bytes / ms / 1e6);
            }
        }
    }
    return 0;
}
