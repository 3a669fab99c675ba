// fls_unpack.hpp -- gfx950 device primitives shared by the decode kernels:
// unified-transposed index map, 16-byte-chunk interleaved unpack at any
// width (v_alignbit for T=32/64, SWAR funnel shifts for T=8/16), wrapping
// frame-of-reference add, tail-guarded 16-byte stores.
//
// Pointer parameters are templates so callers can pass address-space
// qualified pointers (FLS_GLOBAL / FLS_LDS): pointers read out of descriptors
// are otherwise generic, hipcc then emits flat_* instructions, which complete
// out of order and force s_waitcnt vmcnt(0) & lgkmcnt(0) around every access.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#define FLS_GLOBAL __attribute__((address_space(1)))
#define FLS_LDS __attribute__((address_space(3)))

namespace fls {
namespace dev {

// 16-byte register vector usable through address-space qualified pointers
// (HIP's uint4 is a class whose operator= cannot bind a qualified object)
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v4u mk4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    v4u r;
    r.x = a; r.y = b; r.z = c; r.w = d;
    return r;
}

template <class T>
__device__ __forceinline__ FLS_GLOBAL T *gptr(T *p) {
    return (FLS_GLOBAL T *)p;
}
template <class T>
__device__ __forceinline__ const FLS_GLOBAL T *gptr(const T *p) {
    return (const FLS_GLOBAL T *)p;
}

__device__ __forceinline__ void wave_sync() {
    // One wave talks to itself through LDS: the DS instructions of a wave are
    // executed in issue order, so only the COMPILER must not move LDS accesses
    // across this point.  A memory-clobbering empty asm does exactly that;
    // memory-model fences (even wavefront scope) would also make hipcc emit
    // s_waitcnt vmcnt(0), draining the global prefetch this kernel pipelines.
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint32_t tau(uint32_t p) {
    // FL_ORDER = {0,4,2,6,1,5,3,7} is the 3-bit bit reversal
    const uint32_t b = (p >> 4) & 7;
    const uint32_t rb = ((b & 1) << 2) | (b & 2) | ((b >> 2) & 1);
    return (rb << 7) | (((p >> 7) & 7) << 4) | (p & 15);
}

// SWAR funnel shift of packed 16-bit (or 8-bit) words inside a dword
template <int T>
__device__ __forceinline__ uint32_t swar_funnel(uint32_t lo, uint32_t hi, uint32_t s, uint32_t m1, uint32_t m2,
                                                uint32_t mw) {
    return (((lo >> s) & m1) | ((hi << (T - s)) & m2)) & mw;
}

// ---- unpack one 16-byte chunk of T-bit values ------------------------------
// P: staged packed words (128-byte word-rows, 8 x 16-byte columns), plus one
// zero pad row.  Chunk ci = (row R = ci/8, column qc = ci%8) holds 128/T lanes.
template <int T, class PP>
__device__ __forceinline__ v4u unpack_chunk(PP P, uint32_t W, uint32_t ci) {
    const uint32_t R = ci >> 3, qc = ci & 7;
    const uint32_t bit = R * W;
    constexpr uint32_t sh = T == 64 ? 6 : T == 32 ? 5 : T == 16 ? 4 : 3;
    const uint32_t k = bit >> sh, s = bit & (T - 1);
    const v4u lo = P[k * 8 + qc], hi = P[(k + 1) * 8 + qc];
    v4u r;
    if constexpr (T == 32) {
        const uint32_t m = W >= 32 ? 0xFFFFFFFFu : ((1u << W) - 1u);
        r.x = __builtin_amdgcn_alignbit(hi.x, lo.x, s) & m;
        r.y = __builtin_amdgcn_alignbit(hi.y, lo.y, s) & m;
        r.z = __builtin_amdgcn_alignbit(hi.z, lo.z, s) & m;
        r.w = __builtin_amdgcn_alignbit(hi.w, lo.w, s) & m;
    } else if constexpr (T == 64) {
        const uint32_t s5 = s & 31;
        const bool big = s >= 32;
        const uint32_t mlo = W >= 32 ? 0xFFFFFFFFu : ((1u << W) - 1u);
        const uint32_t mhi = W >= 64 ? 0xFFFFFFFFu : (W > 32 ? ((1u << (W - 32)) - 1u) : 0u);
        // lane 0 = (lo.y:lo.x), next word row (hi.y:hi.x); lane 1 = (.w:.z)
        r.x = __builtin_amdgcn_alignbit(big ? hi.x : lo.y, big ? lo.y : lo.x, s5) & mlo;
        r.y = __builtin_amdgcn_alignbit(big ? hi.y : hi.x, big ? hi.x : lo.y, s5) & mhi;
        r.z = __builtin_amdgcn_alignbit(big ? hi.z : lo.w, big ? lo.w : lo.z, s5) & mlo;
        r.w = __builtin_amdgcn_alignbit(big ? hi.w : hi.z, big ? hi.z : lo.w, s5) & mhi;
    } else {
        constexpr uint32_t rep = T == 16 ? 0x00010001u : 0x01010101u;
        constexpr uint32_t full = T == 16 ? 0xFFFFu : 0xFFu;
        const uint32_t m1 = rep * (full >> s);
        const uint32_t m2 = rep * ((full << (T - s)) & full);
        const uint32_t mw = W >= (uint32_t)T ? 0xFFFFFFFFu : rep * ((1u << W) - 1u);
        r.x = swar_funnel<T>(lo.x, hi.x, s, m1, m2, mw);
        r.y = swar_funnel<T>(lo.y, hi.y, s, m1, m2, mw);
        r.z = swar_funnel<T>(lo.z, hi.z, s, m1, m2, mw);
        r.w = swar_funnel<T>(lo.w, hi.w, s, m1, m2, mw);
    }
    return r;
}

// ---- frame-of-reference add on a 16-byte chunk (wrapping T-bit) ----------
__device__ __forceinline__ uint32_t swar_add(uint32_t a, uint32_t b, uint32_t hi) {
    return ((a & ~hi) + (b & ~hi)) ^ ((a ^ b) & hi);
}
template <int T>
__device__ __forceinline__ v4u add_base(v4u a, uint64_t base) {
    if constexpr (T == 64) {
        const uint64_t v0 = (((uint64_t)a.y << 32) | a.x) + base;
        const uint64_t v1 = (((uint64_t)a.w << 32) | a.z) + base;
        return mk4((uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32));
    } else if constexpr (T == 32) {
        const uint32_t b = (uint32_t)base;
        return mk4(a.x + b, a.y + b, a.z + b, a.w + b);
    } else if constexpr (T == 16) {
        const uint32_t b = 0x00010001u * (uint32_t)(base & 0xFFFF), hi = 0x80008000u;
        return mk4(swar_add(a.x, b, hi), swar_add(a.y, b, hi), swar_add(a.z, b, hi), swar_add(a.w, b, hi));
    } else {
        const uint32_t b = 0x01010101u * (uint32_t)(base & 0xFF), hi = 0x80808080u;
        return mk4(swar_add(a.x, b, hi), swar_add(a.y, b, hi), swar_add(a.z, b, hi), swar_add(a.w, b, hi));
    }
}

// ---- stores with tail guard ----------------------------------------------
// store 16 bytes at out + off, or only the EB-byte elements below `limit`.
// Global (address space 1) byte pointers.
#define FLS_DEFINE_STORE16(AS)                                                                   \
    template <int EB>                                                                            \
    __device__ __forceinline__ void store16(AS uint8_t *__restrict__ out, uint32_t off, uint32_t limit, \
                                            v4u v) {                                             \
        if (off + 16 <= limit) {                                                                 \
            *reinterpret_cast<AS v4u *>(out + off) = v;                                          \
            return;                                                                              \
        }                                                                                        \
        if (off >= limit) return;                                                                \
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};                                              \
        _Pragma("unroll") for (int e = 0; e < 16 / EB; ++e) {                                    \
            const uint32_t o = off + e * EB;                                                     \
            if (o < limit) {                                                                     \
                if (EB == 8) {                                                                   \
                    *reinterpret_cast<AS uint64_t *>(out + o) = ((uint64_t)w[2 * e + 1] << 32) | w[2 * e]; \
                } else if (EB == 4) {                                                            \
                    *reinterpret_cast<AS uint32_t *>(out + o) = w[e];                            \
                } else if (EB == 2) {                                                            \
                    *reinterpret_cast<AS uint16_t *>(out + o) = (uint16_t)(w[e / 2] >> (16 * (e & 1))); \
                } else {                                                                         \
                    out[o] = (uint8_t)(w[e / 4] >> (8 * (e & 3)));                               \
                }                                                                                \
            }                                                                                    \
        }                                                                                        \
    }
FLS_DEFINE_STORE16(FLS_GLOBAL)
#undef FLS_DEFINE_STORE16

}  // namespace dev
}  // namespace fls
