// membw6.hip -- the HBM write ceiling by address pattern and store form
// (round 6: VERDICT r5 item 1 asks for the write ceiling re-measured with the
// guide's store forms; the round-1 microbenchmark membw5 measured only the
// decode's own "each wave owns a 512 KiB chunk" pattern).
//
// Every kernel writes OUT bytes with 16-B-per-lane stores, one 1 KiB block per
// wave store instruction.  Waves are 1-wave workgroups (as the fused decode
// launches them), persistent, CUs x WPC of them.  Patterns:
//   linear    wave w writes blocks w, w + NW, w + 2 NW ... (all waves inside
//             one NW KiB window at a time: a torch fill's footprint)
//   chunk C   wave w owns chunks of C KiB (w, w + NW, ...) and writes each
//             front to back (the decode: C = 256/512/1024 KiB row-group
//             outputs of int32/int64/string_t columns; C = 8 is "vector
//             interleaved": consecutive waves write consecutive 8 KiB vectors)
//   group C,G G consecutive waves share a C-KiB chunk, wave r of the group
//             writing its 8 KiB vectors r, r + G, ... (G streams per chunk)
//   torch     non-persistent 256-thread blocks of 4 KiB each (torch.fill_'s
//             shape), for reference
// Store forms: plain, nt, sc1, sc0 sc1 (vector stores only).
// K = 1 adds one 1 KiB load per 8 KiB written (the decode's ~1/8 read share),
// loaded one vector ahead.
//   hipcc -O3 --offload-arch=gfx950 scripts/membw6.hip -o scripts/membw6
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

template <int FORM>
__device__ __forceinline__ void st16(v4u *p, v4u x) {
    if constexpr (FORM == 0) {
        *p = x;
    } else if constexpr (FORM == 1) {
        __builtin_nontemporal_store(x, p);
    } else if constexpr (FORM == 2) {
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
    } else {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
    }
}

// write one 8 KiB vector (8 blocks) starting at block b; optional 1 KiB read
template <int FORM, int K>
__device__ __forceinline__ void put_vec(v4u *out, const v4u *in, size_t b, uint32_t lane, v4u &acc) {
    v4u nxt = acc;
    if (K) nxt ^= in[(b >> 3) * 64 + lane];  // this vector's input
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) st16<FORM>(out + (b + j) * 64 + lane, acc + j);
    acc = nxt;
}

// PAT 0 linear, 1 chunk (C blocks), 2 group (C blocks, G waves)
template <int PAT, int FORM, int K>
__global__ __launch_bounds__(64) void k_write(const v4u *__restrict__ in, v4u *__restrict__ out, size_t nblocks,
                                              uint32_t C, uint32_t G) {
    const uint32_t lane = threadIdx.x;
    const size_t w = blockIdx.x, nw = gridDim.x;
    v4u acc = {lane, (uint32_t)w, 7u, 9u};
    if constexpr (PAT == 0) {
        for (size_t b = w; b < nblocks; b += nw) {
            if (K && (b & 7) == 0) acc ^= in[(b >> 3) * 64 + lane];
            st16<FORM>(out + b * 64 + lane, acc);
        }
    } else if constexpr (PAT == 1) {
        const size_t nch = nblocks / C;
        for (size_t c = w; c < nch; c += nw)
            for (uint32_t v = 0; v < C; v += 8) put_vec<FORM, K>(out, in, c * C + v, lane, acc);
    } else {
        const size_t nch = nblocks / C, grp = w / G, ngrp = nw / G;
        const uint32_t r = (uint32_t)(w % G);
        for (size_t c = grp; c < nch; c += ngrp)
            for (uint32_t v = 8 * r; v < C; v += 8 * G) put_vec<FORM, K>(out, in, c * C + v, lane, acc);
    }
}

__global__ __launch_bounds__(256) void k_torch(v4u *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    out[i] = v4u{(uint32_t)i, 1u, 2u, 3u};
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
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

static const char *kForm[] = {"plain", "nt", "sc1", "sc0sc1"};

template <int PAT, int FORM, int K>
void run(const char *name, const v4u *in, v4u *out, size_t bytes, int cus, int wpc, uint32_t C, uint32_t G) {
    const size_t nb = bytes / 1024;
    const size_t written = PAT == 0 ? nb * 1024 : nb / C * C * 1024;
    const double ms = time_ms([&] { k_write<PAT, FORM, K><<<cus * wpc, 64>>>(in, out, nb, C, G); });
    printf("%-7s C=%5u KiB G=%2u form=%-6s K=%d wpc=%2d : %7.1f GB/s written%s\n", name, C, G, kForm[FORM], K, wpc,
           written / ms / 1e6, K ? " (+1/8 read)" : "");
    fflush(stdout);
}

template <int FORM>
void forms(const v4u *in, v4u *out, size_t bytes, int cus) {
    run<0, FORM, 0>("linear", in, out, bytes, cus, 16, 1, 1);
    run<1, FORM, 0>("chunk", in, out, bytes, cus, 16, 512, 1);
    run<1, FORM, 0>("chunk", in, out, bytes, cus, 16, 8, 1);
}

int main(int argc, char **argv) {
    const size_t bytes = 8ull << 30;  // output
    size_t off = argc > 1 ? strtoull(argv[1], nullptr, 0) : 0;  // byte offset of the output
    v4u *out0, *in;
    CK(hipMalloc(&out0, bytes + (4u << 20)));
    CK(hipMalloc(&in, bytes / 8));
    CK(hipMemset(in, 3, bytes / 8));
    v4u *out = (v4u *)((char *)out0 + off);
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("out %p (+%zu), in %p, %d CUs\n", (void *)out, off, (void *)in, cus);
    for (int rep = 0; rep < 2; ++rep) {
        printf("-- rep %d\n", rep);
        {
            const double ms = time_ms([&] { k_torch<<<bytes / 4096, 256>>>(out); });
            printf("torch   (4 KiB blocks, non-persistent)            : %7.1f GB/s written\n", bytes / ms / 1e6);
        }
        // store forms on three patterns
        forms<0>(in, out, bytes, cus);
        forms<1>(in, out, bytes, cus);
        forms<2>(in, out, bytes, cus);
        forms<3>(in, out, bytes, cus);
        // chunk size sweep (plain), the decode's sizes and finer
        for (uint32_t C : {8u, 16u, 32u, 64u, 128u, 256u, 1024u}) run<1, 0, 0>("chunk", in, out, bytes, cus, 16, C, 1);
        // waves per CU
        for (int wpc : {4, 8, 12, 24, 32}) {
            run<0, 0, 0>("linear", in, out, bytes, cus, wpc, 1, 1);
            run<1, 0, 0>("chunk", in, out, bytes, cus, wpc, 512, 1);
        }
        // G waves sharing a chunk
        for (uint32_t G : {2u, 4u, 8u, 16u, 64u}) run<2, 0, 0>("group", in, out, bytes, cus, 16, 512, G);
        // with the decode's 1/8 read share
        run<0, 0, 1>("linear", in, out, bytes, cus, 16, 1, 1);
        run<1, 0, 1>("chunk", in, out, bytes, cus, 16, 512, 1);
        run<1, 0, 1>("chunk", in, out, bytes, cus, 16, 8, 1);
        run<2, 0, 1>("group", in, out, bytes, cus, 16, 512, 8);
        run<1, 1, 1>("chunk", in, out, bytes, cus, 16, 512, 1);
        run<1, 2, 1>("chunk", in, out, bytes, cus, 16, 512, 1);
    }
    return 0;
}
