// membw3.hip -- follow-up to membw2: write patterns a decode kernel could use.
// membw2 found one-shot grids (a block writes 4 KiB and exits) at ~6.85 TB/s,
// persistent grid-stride loops at ~5.4 and wave-private contiguous regions at
// 5.7-6.1.  Here, at 8 GiB of output:
//   os  B U      one-shot, B threads per block, U 16-B stores per lane, the
//                block's stores contiguous (lane-fastest, then wave, then u)
//   vec B K      one-shot "decode shape": a wave loads K*16 B per lane of input
//                (K x 1 KiB), then writes an 8 KiB vector (8 x 1 KiB stores)
//   pull G       persistent, G blocks/CU; waves pull 8 KiB units from an
//                atomic counter (sliding window like a one-shot grid)
//   rot R        persistent wave-private R-byte regions, each wave starting at
//                a different 8 KiB block of its region and wrapping
//   hipcc -O3 --offload-arch=gfx950 scripts/membw3.hip -o scripts/membw3
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

template <int B, int U>
__global__ __launch_bounds__(B) void k_os(v4u *__restrict__ out) {
    const size_t base = (size_t)blockIdx.x * B * U + threadIdx.x;
    const v4u v = {threadIdx.x, blockIdx.x, 7u, 9u};
#pragma unroll
    for (int u = 0; u < U; ++u) out[base + (size_t)u * B] = v;
}

// one 8 KiB vector per wave; K x 1 KiB of input per wave
template <int B, int K>
__global__ __launch_bounds__(B) void k_vec(const v4u *__restrict__ in, v4u *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t vec = (size_t)blockIdx.x * (B / 64) + (threadIdx.x >> 6);
    v4u acc = {lane, 1u, 2u, 3u};
#pragma unroll
    for (int k = 0; k < K; ++k) acc ^= in[vec * 64 * K + 64 * k + lane];
    v4u *o = out + vec * 512;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[64 * j + lane] = acc + (uint32_t)j;
}

__global__ __launch_bounds__(256) void k_pull(v4u *__restrict__ out, size_t nunits, unsigned *ctr) {
    const uint32_t lane = threadIdx.x & 63;
    for (;;) {
        unsigned u = 0;
        if (lane == 0) u = atomicAdd(ctr, 1u);
        u = __shfl(u, 0);
        if (u >= nunits) break;
        v4u *o = out + (size_t)u * 512;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const v4u v = {lane, (uint32_t)j, u, 1u};
            o[64 * j + lane] = v;
        }
    }
}

__global__ __launch_bounds__(256) void k_rot(v4u *__restrict__ out, size_t nreg, size_t nblk) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (size_t)gridDim.x * 4;
    for (size_t r = wave; r < nreg; r += nw) {
        v4u *o = out + r * nblk * 512;
        for (size_t i = 0; i < nblk; ++i) {
            const size_t b = (i + wave) % nblk;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const v4u v = {lane, j, (uint32_t)b, 1u};
                o[b * 512 + 64 * j + lane] = v;
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
    v4u *out, *in;
    unsigned *ctr;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&in, bytes / 2));
    CK(hipMalloc(&ctr, 4));
    CK(hipMemset(in, 3, bytes / 2));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double ms;
    const size_t nvec = bytes / 8192;
#define GBS(name) printf("%-26s: %7.1f GB/s\n", name, bytes / ms / 1e6)
    for (int rep = 0; rep < 2; ++rep) {
        ms = time_ms([&] { k_os<256, 1><<<n16 / 256, 256>>>(out); });      GBS("os 256 U1");
        ms = time_ms([&] { k_os<256, 2><<<n16 / 512, 256>>>(out); });      GBS("os 256 U2");
        ms = time_ms([&] { k_os<64, 1><<<n16 / 64, 64>>>(out); });         GBS("os 64 U1");
        ms = time_ms([&] { k_os<64, 4><<<n16 / 256, 64>>>(out); });        GBS("os 64 U4");
        ms = time_ms([&] { k_os<64, 8><<<n16 / 512, 64>>>(out); });        GBS("os 64 U8");
        ms = time_ms([&] { k_os<512, 1><<<n16 / 512, 512>>>(out); });      GBS("os 512 U1");
        ms = time_ms([&] { k_os<1024, 1><<<n16 / 1024, 1024>>>(out); });   GBS("os 1024 U1");
        ms = time_ms([&] { k_vec<64, 1><<<nvec, 64>>>(in, out); });        GBS("vec 64 K1");
        ms = time_ms([&] { k_vec<64, 2><<<nvec, 64>>>(in, out); });        GBS("vec 64 K2");
        ms = time_ms([&] { k_vec<256, 1><<<nvec / 4, 256>>>(in, out); });  GBS("vec 256 K1");
        ms = time_ms([&] { k_vec<256, 2><<<nvec / 4, 256>>>(in, out); });  GBS("vec 256 K2");
        for (int g : {2, 4, 8}) {
            char nm[64];
            ms = time_ms([&] {
                CK(hipMemsetAsync(ctr, 0, 4));
                k_pull<<<cus * g, 256>>>(out, nvec, ctr);
            });
            snprintf(nm, sizeof nm, "pull %d blk/CU", g); GBS(nm);
        }
        for (size_t R : {65536ul, 262144ul, 1048576ul}) {
            char nm[64];
            ms = time_ms([&] { k_rot<<<cus * 4, 256>>>(out, bytes / R, R / 8192); });
            snprintf(nm, sizeof nm, "rot %zu 4 blk/CU", R); GBS(nm);
        }
    }
    return 0;
}
