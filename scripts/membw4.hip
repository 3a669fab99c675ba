// membw4.hip -- is there XCD <-> HBM address locality for writes (and reads)?
// membw3: one-shot grids whose block b writes 4 KiB piece b (blocks dealt
// round-robin over XCDs, so XCD x writes pieces = x mod 8) reach ~6.8 TB/s;
// other piece sizes 6.0-6.5.  Here persistent waves read their XCD id and
// write only pieces p of G bytes with (p mod 8) == (xcd + shift) mod 8.  If
// memory is interleaved over stacks at G with a fixed XCD affinity, one
// shift is much faster than the others.
//   hipcc -O3 --offload-arch=gfx950 scripts/membw4.hip -o scripts/membw4
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

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7;
}

// G16 = piece size in 16-B units (multiple of 64: whole 1 KiB wave stores)
template <int G16>
__global__ __launch_bounds__(256) void k_xw(v4u *__restrict__ out, size_t npieces, uint32_t shift) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t x = (xcc_id() + shift) & 7;
    const size_t wix = (size_t)(blockIdx.x / 8) * 4 + (threadIdx.x >> 6);
    const size_t nwx = (size_t)(gridDim.x / 8) * 4;
    for (size_t k = wix; 8 * k + x < npieces; k += nwx) {
        v4u *o = out + (8 * k + x) * G16;
#pragma unroll
        for (int j = 0; j < G16 / 64; ++j) {
            const v4u v = {lane, (uint32_t)j, (uint32_t)k, 1u};
            o[64 * j + lane] = v;
        }
    }
}

template <int G16>
__global__ __launch_bounds__(256) void k_xr(const v4u *__restrict__ in, size_t npieces, uint32_t shift, v4u *sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t x = (xcc_id() + shift) & 7;
    const size_t wix = (size_t)(blockIdx.x / 8) * 4 + (threadIdx.x >> 6);
    const size_t nwx = (size_t)(gridDim.x / 8) * 4;
    v4u acc = {0, 0, 0, 0};
    for (size_t k = wix; 8 * k + x < npieces; k += nwx) {
        const v4u *p = in + (8 * k + x) * G16;
#pragma unroll
        for (int j = 0; j < G16 / 64; ++j) acc ^= p[64 * j + lane];
    }
    if (acc.x == 0x12345678u) sink[0] = acc;
}

__global__ void k_ids(uint32_t *ids) {
    if (threadIdx.x == 0) ids[blockIdx.x] = xcc_id();
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

template <int G16>
void sweep(v4u *out, v4u *sink, size_t bytes, int grid) {
    const size_t np = bytes / (G16 * 16);
    printf("piece %6d B  write:", G16 * 16);
    for (uint32_t s = 0; s < 8; ++s) {
        const double ms = time_ms([&] { k_xw<G16><<<grid, 256>>>(out, np, s); });
        printf(" %6.0f", bytes / ms / 1e6);
    }
    printf("\n               read: ");
    for (uint32_t s = 0; s < 8; ++s) {
        const double ms = time_ms([&] { k_xr<G16><<<grid, 256>>>(out, np, s, sink); });
        printf(" %6.0f", bytes / ms / 1e6);
    }
    printf("\n");
}

int main() {
    const size_t bytes = 8ull << 30;
    v4u *out, *sink;
    uint32_t *ids;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&ids, 4 * 64));
    CK(hipMemset(out, 1, bytes));
    k_ids<<<16, 64>>>(ids);
    uint32_t h[16];
    CK(hipMemcpy(h, ids, sizeof h, hipMemcpyDeviceToHost));
    printf("xcc of blocks 0..15:");
    for (int i = 0; i < 16; ++i) printf(" %u", h[i]);
    printf("\nbase %p\n", (void *)out);
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 4;
    printf("GB/s by shift 0..7 (pieces written by XCD x: p mod 8 == x + shift)\n");
    for (int rep = 0; rep < 2; ++rep) {
        sweep<64>(out, sink, bytes, grid);
        sweep<128>(out, sink, bytes, grid);
        sweep<256>(out, sink, bytes, grid);
        sweep<512>(out, sink, bytes, grid);
        sweep<1024>(out, sink, bytes, grid);
    }
    return 0;
}
