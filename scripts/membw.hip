// membw.hip -- HBM ceilings for the decode kernel's traffic mix on this GPU:
// pure 16-B stores (plain / nontemporal), pure loads, copy, and the decode's
// ~1:7 read:write mix, at several occupancies.  Informs roofline.frac's
// practical ceiling.  Build + run:
//   hipcc -O3 --offload-arch=gfx950 scripts/membw.hip -o /tmp/membw && /tmp/membw
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

template <int NT, int U>
__global__ __launch_bounds__(256) void k_write(v4u *__restrict__ out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    const v4u v = {threadIdx.x, blockIdx.x, 7u, 9u};
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + (size_t)u * 256;
            if (j < n16) {
                if (NT) __builtin_nontemporal_store(v, out + j);
                else out[j] = v;
            }
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const v4u *__restrict__ in, size_t n16, v4u *sink) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    v4u acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + (size_t)u * 256;
            if (j < n16) acc ^= in[j];
        }
    }
    if (acc.x == 0x12345678u) sink[0] = acc;
}

// reads 1 x 16 B per R x 16 B written (the decode writes ~7x what it reads)
template <int R>
__global__ __launch_bounds__(256) void k_mix(const v4u *__restrict__ in, v4u *__restrict__ out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i * R < n16; i += stride) {
        const v4u x = in[i];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t j = (i / 64) * 64 * R + (size_t)r * 64 + (i % 64);
            if (j < n16) out[j] = x + (uint32_t)r;
        }
    }
}

__global__ __launch_bounds__(256) void k_copy(const v4u *__restrict__ in, v4u *__restrict__ out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

// one wave writes 8 KB blocks with 8 store instructions, either each
// instruction 1 KB contiguous (SEG=0) or 8 x 128-B segments 1 KB apart (SEG=1,
// the DELTA64 register layout)
template <int SEG>
__global__ __launch_bounds__(256) void k_block(v4u *__restrict__ out, size_t nblk) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (size_t)gridDim.x * 4;
    const uint32_t g = lane >> 3, q = lane & 7;
    for (size_t b = wave; b < nblk; b += nw) {
        v4u *o = out + b * 512;  // 8 KB = 512 x 16 B
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const v4u v = {lane, j, (uint32_t)b, 1u};
            if (SEG) o[8 * (8 * g + j) + q] = v;
            else o[64 * j + lane] = v;
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
    const size_t bytes = 8ull << 30;  // 8 GiB output, like one SF100 slice of columns
    const size_t n16 = bytes / 16;
    v4u *out, *in, *sink;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&sink, 16));
    CK(hipMemset(in, 1, bytes));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int per_cu : {4, 16}) {
        const int grid = cus * per_cu;
        double ms;
        ms = time_ms([&] { k_write<0, 4><<<grid, 256>>>(out, n16); });
        printf("write plain  grid %5d: %7.1f GB/s\n", grid, bytes / ms / 1e6);
        ms = time_ms([&] { k_write<1, 4><<<grid, 256>>>(out, n16); });
        printf("write nt     grid %5d: %7.1f GB/s\n", grid, bytes / ms / 1e6);
        ms = time_ms([&] { k_write<0, 1><<<grid, 256>>>(out, n16); });
        printf("write U1     grid %5d: %7.1f GB/s\n", grid, bytes / ms / 1e6);
        ms = time_ms([&] { k_read<4><<<grid, 256>>>(in, n16, sink); });
        printf("read         grid %5d: %7.1f GB/s\n", grid, bytes / ms / 1e6);
        ms = time_ms([&] { k_copy<<<grid, 256>>>(in, out, n16 / 2); });
        printf("copy (r+w)   grid %5d: %7.1f GB/s\n", grid, bytes / ms / 1e6);
        ms = time_ms([&] { k_mix<7><<<grid, 256>>>(in, out, n16); });
        printf("mix 1:7      grid %5d: %7.1f GB/s (read+write)\n", grid, (bytes + bytes / 7) / ms / 1e6);
        ms = time_ms([&] { k_mix<3><<<grid, 256>>>(in, out, n16); });
        printf("mix 1:3      grid %5d: %7.1f GB/s (read+write)\n", grid, (bytes + bytes / 3) / ms / 1e6);
        ms = time_ms([&] { k_block<0><<<grid, 256>>>(out, bytes / 8192); });
        printf("8K blk 1KB   grid %5d: %7.1f GB/s\n", grid, bytes / ms / 1e6);
        ms = time_ms([&] { k_block<1><<<grid, 256>>>(out, bytes / 8192); });
        printf("8K blk 8x128 grid %5d: %7.1f GB/s\n", grid, bytes / ms / 1e6);
    }
    return 0;
}
