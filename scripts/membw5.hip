// membw5.hip -- does the DELTA64 store shape cost write bandwidth?
// Persistent waves (16 per CU, like the decode kernel) each own chunks of 64
// "vectors" of 8 KiB (512 KiB contiguous), grid-stride over chunks, and per
// vector read K x 1 KiB of input then issue 8 store instructions:
//   contig   store j writes bytes [1024 j, 1024 j + 1024) of the vector
//            (lane = 16 B column; the FFOR shape)
//   lines    store j writes 128 B at line 8 g + j for lane group g = lane / 8
//            (eight 128 B lines 1 KiB apart; the DELTA64 shape)
//   hipcc -O3 --offload-arch=gfx950 scripts/membw5.hip -o scripts/membw5
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

template <int MODE, int K>
__global__ __launch_bounds__(256) void k_vec(const v4u *__restrict__ in, v4u *__restrict__ out, size_t nchunks) {
    const uint32_t lane = threadIdx.x & 63, g = lane >> 3, q = lane & 7;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (size_t)gridDim.x * 4;
    for (size_t c = wave; c < nchunks; c += nw) {
        for (uint32_t v = 0; v < 64; ++v) {
            const size_t vec = c * 64 + v;
            v4u acc = {lane, v, 7u, 9u};
            if (K > 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) acc ^= in[(vec * K + k) * 64 + lane];
            }
            v4u *o = out + vec * 512;
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                const v4u x = acc + j;
                if (MODE == 0) o[64 * j + lane] = x;
                else o[8 * (8 * g + j) + q] = x;
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
    const size_t bytes = 8ull << 30;            // output
    const size_t nvec = bytes / 8192, nchunks = nvec / 64;
    v4u *out, *in;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&in, nvec * 1024));
    CK(hipMemset(in, 3, nvec * 1024));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 4;
    for (int rep = 0; rep < 2; ++rep) {
        double ms;
        ms = time_ms([&] { k_vec<0, 0><<<grid, 256>>>(in, out, nchunks); });
        printf("contig K0 : %7.1f GB/s written\n", bytes / ms / 1e6);
        ms = time_ms([&] { k_vec<1, 0><<<grid, 256>>>(in, out, nchunks); });
        printf("lines  K0 : %7.1f GB/s written\n", bytes / ms / 1e6);
        ms = time_ms([&] { k_vec<0, 1><<<grid, 256>>>(in, out, nchunks); });
        printf("contig K1 : %7.1f GB/s written (+1/8 read)\n", bytes / ms / 1e6);
        ms = time_ms([&] { k_vec<1, 1><<<grid, 256>>>(in, out, nchunks); });
        printf("lines  K1 : %7.1f GB/s written (+1/8 read)\n", bytes / ms / 1e6);
    }
    return 0;
}
