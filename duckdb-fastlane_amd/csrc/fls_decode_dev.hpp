// fls_decode_dev.hpp -- the main decode kernel's device code (every path,
// run_chunk, decode_chunk, decode_range), shared by decode_kernel
// (fls_decode.hip) and the fused decode + FSST kernel (fls_fsst.hip), each
// translation unit with its own copy (namespace fls::dec, internal linkage).
// See fls_decode.hip for the design.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "fls_alp.hpp"
#include "fls_decode.hpp"
#include "fls_format.hpp"
#include "fls_unpack.hpp"

namespace fls {
namespace dec {
namespace {
using namespace dev;

constexpr int kWaves = 4;  // waves per 256-thread block

// address-space qualified views (global = 1, LDS = 3): see fls_unpack.hpp
using gv4 = const FLS_GLOBAL v4u;
using gu8 = const FLS_GLOBAL uint8_t;
using ov4 = FLS_GLOBAL v4u;
using ou8 = FLS_GLOBAL uint8_t;
using lv4 = FLS_LDS v4u;
using lu8 = FLS_LDS uint8_t;

template <int T>
struct UInt;
template <> struct UInt<8> { using type = uint8_t; };
template <> struct UInt<16> { using type = uint16_t; };
template <> struct UInt<32> { using type = uint32_t; };
template <> struct UInt<64> { using type = uint64_t; };

__device__ __forceinline__ uint32_t rl(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }

__constant__ double kF10D[kAlpMaxExpD + 1] = {FLS_ALP_F10_D};
__constant__ double kIF10D[kAlpMaxExpD + 1] = {FLS_ALP_IF10_D};
__constant__ float kF10F[kAlpMaxExpF + 1] = {FLS_ALP_F10_F};
__constant__ float kIF10F[kAlpMaxExpF + 1] = {FLS_ALP_IF10_F};
// keep unrolled iterations in program order: bounds register pressure to one
// iteration (the occupancy, not the ILP of one wave, hides latency here)
// full 16-byte output store at byte off of the vector's (wave-uniform) output
// out.  CPOL != 0: a buffer store with that cache policy (2 = nt, 16 = sc1,
// 17 = sc0 sc1).  Chosen per path by build A/B over re-drawn placements
// (scripts/ab_builds.py, profiles/r6/ab_builds_*): nt stores made DELTA64
// (c3, 1e9 INT64 keys) 5.0-7.2 % faster and sc1 4.4 %, while nt cost the
// FFOR / DICT paths 1.8-2.9 % (c4, lineitem SF10) and nothing at SF100; so
// only the DELTA64 path leaves the default, with sc1 | nt (c3 1.671 ms
// against 1.720 with nt alone, sc0 sc1 nt 1.684, sc0 nt 1.705,
// profiles/r6/ab_builds_c3_cpol_r6s.txt).  FLS_STORE_CPOL (experiment
// builds, make cpol) overrides every path's policy.
#ifdef FLS_STORE_CPOL
constexpr int kCpolAll = FLS_STORE_CPOL;
#else
constexpr int kCpolAll = -1;
#endif
constexpr int kCpolDelta64 = 18;  // sc1 | nt
template <int CPOL = 0>
__device__ __forceinline__ void st16(ou8 *out, uint32_t off, v4u v) {
    constexpr int cp = kCpolAll >= 0 ? kCpolAll : CPOL;
    if constexpr (cp != 0) {
        const uint64_t b = (uint64_t)out;
        void *ub = (void *)((uint64_t)uni((uint32_t)(b >> 32)) << 32 | (uint64_t)uni((uint32_t)b));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, cp);
    } else {
        *reinterpret_cast<ov4 *>(out + off) = v;
    }
}
// packed-bit load (FLS_NT_LOAD: non-temporal, read-once stream)
__device__ __forceinline__ v4u ld16(const FLS_GLOBAL v4u *p) {
#ifdef FLS_NT_LOAD
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// Scheduling fence between unrolled 16-byte-chunk steps: one step's registers
// live at a time (occupancy, not one wave's ILP, hides latency here).
// Measured: fencing every second step instead (LDS reads of two steps in
// flight) was neutral to 2 % slower (profiles/r1/abenv_prefetch_width_*.txt,
// arm p8).
__device__ __forceinline__ void seq() { __builtin_amdgcn_sched_barrier(0); }
__device__ __forceinline__ uint32_t bitrev3(uint32_t g) { return ((g & 1) << 2) | (g & 2) | ((g >> 2) & 1); }

// per-lane copy of the chunk's VecMeta[lane]
struct ChunkMetas {
    uint32_t poff, blo, bhi, aoff, nvbw, acnt;
};
__device__ __forceinline__ ChunkMetas load_metas(const DevChunk &c, uint32_t lane) {
    ChunkMetas m{0, 0, 0, 0, 0, 0};
    if (lane < c.nvec) {
        gv4 *p = reinterpret_cast<gv4 *>(gptr(c.chunk) + c.meta_off) + 2 * lane;
        const v4u a = p[0], b = p[1];
        m.poff = a.x;
        m.blo = a.z;
        m.bhi = a.w;
        m.aoff = b.x;
        m.nvbw = b.z;
        m.acnt = b.w;
    }
    return m;
}

struct VecInfo {
    uint32_t poff16;   // packed offset (uint4 units) inside the packed area
    uint32_t W, nvals, aoff, acount;
    uint64_t base;
};
__device__ __forceinline__ VecInfo vec_info(const ChunkMetas &m, uint32_t v) {
    VecInfo x;
    x.poff16 = rl(m.poff, v) >> 4;
    x.base = ((uint64_t)rl(m.bhi, v) << 32) | rl(m.blo, v);
    x.aoff = rl(m.aoff, v);
    const uint32_t nb = rl(m.nvbw, v);
    x.nvals = nb & 0xFFFF;
    x.W = (nb >> 16) & 0xFF;
    x.acount = rl(m.acnt, v);
    return x;
}

// ---- packed-bit prefetch (registers) and staging (LDS) --------------------
// L = T/8 = max 16-byte loads per lane (W <= T -> 8W <= 8T per vector).  Load
// instruction i is issued only when some lane needs it (a wave-uniform
// branch on W); inside it, lanes past the end re-read a safe dummy line.  The
// waits stay exact: what follows the prefetch (the stores) is fixed per path.
// ALL: every one of the L loads is issued (past the end: the dummy line), so
// the number of memory operations between a load and its use is fixed and
// the compiler's vmcnt waits can leave a second vector's loads in flight
template <int L, bool ALL = false>
__device__ __forceinline__ void prefetch(gv4 *__restrict__ src, uint32_t n16, gv4 *__restrict__ dummy,
                                         uint32_t lane, v4u (&r)[L]) {
#pragma unroll
    for (int i = 0; i < L; ++i) {
        if (ALL || 64 * i < n16) {
            const uint32_t idx = lane + 64 * i;
            r[i] = ld16(idx < n16 ? src + idx : dummy);
        }
    }
}
template <int L>
__device__ __forceinline__ void stage(lv4 *__restrict__ P, const v4u (&r)[L], uint32_t n16, uint32_t lane) {
#pragma unroll
    for (int i = 0; i < L; ++i) {
        if (64 * i < n16) {
            const uint32_t idx = lane + 64 * i;
            if (idx < n16) P[idx] = r[i];
        }
    }
    if (lane < 8) P[n16 + lane] = mk4(0, 0, 0, 0);
}

// ---- per-path vector processing ---------------------------------------------
// Each path: aux prefetch (registers, issued with the packed prefetch) and
// vec<FULL>(...) writing one vector; FULL=false guards the partial tail.

struct NoAux {
    __device__ __forceinline__ void load(gu8 *, uint32_t) {}
};

template <int T, bool FULL>
__device__ __forceinline__ void ffor_vec(const lv4 *__restrict__ P, uint32_t W, uint64_t base, ou8 *__restrict__ out,
                                         uint32_t nvals, uint32_t lane) {
    const uint32_t limit = nvals * (T / 8);
#pragma unroll
    for (uint32_t j = 0; j < T / 8; ++j) {
        const uint32_t ci = lane + 64 * j;
        const v4u v = add_base<T>(unpack_chunk<T>(P, W, ci), base);
        if (FULL) st16(out, 16 * ci, v);
        else store16<T / 8>(out, 16 * ci, limit, v);
        seq();
    }
}

// DELTA T=64 bases: lane q = lane&7 needs chains 2q, 2q+1 -> one 16 B load
struct Aux64 {
    v4u b;
    __device__ __forceinline__ void load(gu8 *bases, uint32_t lane) {
        b = *reinterpret_cast<gv4 *>(bases + 16 * (lane & 7));
    }
};

template <bool FULL>
__device__ __forceinline__ void delta64_vec(const lv4 *__restrict__ P, uint32_t W, uint64_t base, const Aux64 &aux,
                                            ou8 *__restrict__ out, uint32_t nvals, uint32_t lane) {
    // chunk ci = lane + 64 j holds positions p = 16 R + 2q + e with R = g + 8 j
    // (g = lane>>3, q = lane&7): tuple 16 (8 FL[g] + j) + 2q + e, i.e. steps
    // 8 FL[g] + j of chains 2q, 2q+1 -- a contiguous 8-step segment s = FL[g].
    const uint32_t g = lane >> 3, q = lane & 7, s = bitrev3(g);
    uint64_t a0[8], a1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const v4u x = add_base<64>(unpack_chunk<64>(P, W, lane + 64 * j), base);
        a0[j] = ((uint64_t)x.y << 32) | x.x;
        a1[j] = ((uint64_t)x.w << 32) | x.z;
        seq();
    }
#pragma unroll
    for (int j = 1; j < 8; ++j) {
        a0[j] += a0[j - 1];
        a1[j] += a1[j - 1];
    }
    // inclusive scan of segment totals in segment order; segment t lives in
    // lane group FL[t] (FL is an involution)
    uint64_t x0 = a0[7], x1 = a1[7];
#pragma unroll
    for (uint32_t d = 1; d < 8; d <<= 1) {
        const uint32_t src = 8 * bitrev3((s - d) & 7) + q;
        const uint64_t y0 = __shfl((unsigned long long)x0, (int)src, 64);
        const uint64_t y1 = __shfl((unsigned long long)x1, (int)src, 64);
        if (s >= d) {
            x0 += y0;
            x1 += y1;
        }
    }
    const uint64_t p0 = x0 - a0[7] + (((uint64_t)aux.b.y << 32) | aux.b.x);
    const uint64_t p1 = x1 - a1[7] + (((uint64_t)aux.b.w << 32) | aux.b.z);
    const uint32_t limit = nvals * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint64_t v0 = p0 + a0[j], v1 = p1 + a1[j];
        const v4u v = mk4((uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32));
        const uint32_t off = 128 * (8 * s + j) + 16 * q;
        if (FULL) st16<kCpolDelta64>(out, off, v);
        else store16<8>(out, off, limit, v);
    }
}

// DELTA T<64 / RLE index bases: lane's chain(s) base(s), loaded as registers
template <int T>
struct AuxSmall {
    uint32_t b0, b1;
    __device__ __forceinline__ void load(gu8 *bases, uint32_t lane) {
        if (T == 32) {
            b0 = reinterpret_cast<const FLS_GLOBAL uint32_t *>(bases)[lane & 31];
        } else if (T == 16) {
            b0 = reinterpret_cast<const FLS_GLOBAL uint16_t *>(bases)[lane];
        } else {
            b0 = bases[lane];
            b1 = bases[lane + 64];
        }
    }
};

// unpack + base into LDS at transposed (DELTA/RLE) or natural (DICT) position
template <int T, bool TRANSPOSED>
__device__ __forceinline__ void unpack_to_lds(const lv4 *__restrict__ P, uint32_t W, uint64_t base,
                                              lu8 *__restrict__ V, uint32_t lane) {
#pragma unroll
    for (uint32_t j = 0; j < T / 8; ++j) {
        const uint32_t ci = lane + 64 * j;
        const v4u v = add_base<T>(unpack_chunk<T>(P, W, ci), base);
        const uint32_t p0 = ci * (128 / T);
        const uint32_t i0 = TRANSPOSED ? tau(p0) : p0;
        *reinterpret_cast<lv4 *>(V + i0 * (T / 8)) = v;
        seq();
    }
}

// in-place chain scan in LDS (T = 8/16/32); bases from registers
template <int T>
__device__ __forceinline__ void chain_scan_lds(lu8 *__restrict__ V, const AuxSmall<T> &aux, uint32_t lane) {
    using UT = typename UInt<T>::type;
    FLS_LDS UT *v = reinterpret_cast<FLS_LDS UT *>(V);
    if (T == 8) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = lane + 64 * h;
            const uint32_t i0 = (c >> 4) * 128 + (c & 15);
            UT acc = (UT)(h ? aux.b1 : aux.b0);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                acc = (UT)(acc + v[i0 + 16 * k]);
                v[i0 + 16 * k] = acc;
            }
        }
        return;
    }
    constexpr uint32_t nchains = 1024 / T;  // 32 or 64
    const uint32_t c = lane % nchains, seg = lane / nchains;
    const uint32_t i0 = (c >> 4) * 16 * T + (c & 15) + 256 * seg;
    UT run[16];
    UT acc = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        acc = (UT)(acc + v[i0 + 16 * j]);
        run[j] = acc;
    }
    uint32_t pre = 0;
    if (nchains == 32) {  // two 16-step segments per chain
        const uint32_t y = __shfl_up((uint32_t)acc, 32, 64);
        pre = seg ? y : 0u;
    }
    const UT p = (UT)(pre + aux.b0);
#pragma unroll
    for (int j = 0; j < 16; ++j) v[i0 + 16 * j] = (UT)(p + run[j]);
}

// 16 B/lane copy of a decoded vector (tuple order, EB bytes each) LDS -> HBM
template <int EB, bool FULL>
__device__ __forceinline__ void copy_out(const lu8 *__restrict__ V, ou8 *__restrict__ out, uint32_t nvals,
                                         uint32_t lane) {
    const uint32_t limit = nvals * EB;
#pragma unroll
    for (uint32_t j = 0; j < EB; ++j) {
        const uint32_t ci = lane + 64 * j;
        const v4u x = *reinterpret_cast<const lv4 *>(V + 16 * ci);
        if (FULL) st16(out, 16 * ci, x);
        else store16<EB>(out, 16 * ci, limit, x);
        seq();
    }
}

// gather OB-byte table entries by index and store 16 B/lane
template <int OB, bool FULL, typename TabF, typename IdxF>
__device__ __forceinline__ void gather_out(TabF tab, ou8 *__restrict__ out, uint32_t nvals, uint32_t lane, IdxF idx) {
    const uint32_t limit = nvals * OB;
    constexpr int per = 16 / OB;
#pragma unroll
    for (uint32_t j = 0; j < OB; ++j) {
        const uint32_t oc = lane + 64 * j;
        uint32_t w[4] = {0, 0, 0, 0};
        if (OB == 16) {
            const v4u e = tab.v16(idx(oc));
            w[0] = e.x; w[1] = e.y; w[2] = e.z; w[3] = e.w;
        } else {
#pragma unroll
            for (int e = 0; e < per; ++e) {
                const uint32_t t = idx(oc * per + e);
                if (OB == 8) {
                    const uint64_t x = tab.u64(t);
                    w[2 * e] = (uint32_t)x;
                    w[2 * e + 1] = (uint32_t)(x >> 32);
                } else if (OB == 4) {
                    w[e] = tab.u32(t);
                } else if (OB == 2) {
                    w[e / 2] |= tab.u16(t) << (16 * (e & 1));
                } else {
                    w[e / 4] |= tab.u8(t) << (8 * (e & 3));
                }
            }
        }
        const v4u v = mk4(w[0], w[1], w[2], w[3]);
        if (FULL) st16(out, 16 * oc, v);
        else store16<OB == 16 ? 8 : OB>(out, 16 * oc, limit, v);
        seq();
    }
}

// table readers over an address space AS (LDS-staged or global dictionary)
#define FLS_DEFINE_TAB(NAME, AS)                                                                          \
    struct NAME {                                                                                         \
        const AS uint8_t *p;                                                                              \
        __device__ __forceinline__ v4u v16(uint32_t i) const { return reinterpret_cast<const AS v4u *>(p)[i]; } \
        __device__ __forceinline__ uint64_t u64(uint32_t i) const {                                      \
            return reinterpret_cast<const AS uint64_t *>(p)[i];                                           \
        }                                                                                                 \
        __device__ __forceinline__ uint32_t u32(uint32_t i) const {                                      \
            return reinterpret_cast<const AS uint32_t *>(p)[i];                                           \
        }                                                                                                 \
        __device__ __forceinline__ uint32_t u16(uint32_t i) const {                                      \
            return reinterpret_cast<const AS uint16_t *>(p)[i];                                           \
        }                                                                                                 \
        __device__ __forceinline__ uint32_t u8(uint32_t i) const { return p[i]; }                         \
    };
FLS_DEFINE_TAB(TabL, FLS_LDS)
FLS_DEFINE_TAB(TabG, FLS_GLOBAL)
#undef FLS_DEFINE_TAB

// ---- the pipelined chunk loop ------------------------------------------------
struct Lds {
    lv4 *P;          // packed staging (p_bytes)
    lu8 *V;          // decoded scratch; DICT: codes [0,4K) + staged dictionary
    uint32_t v_bytes;
};

// Path concept: T (packing width), Aux (registers prefetched with the packed
// bits), aux_ptr(chunk, vec), template<bool FULL> vec(...).
template <int T_>
struct PathFfor {
    __device__ __forceinline__ PathFfor(const DevChunk &, const Lds &, uint32_t, uint32_t *) {}
    static constexpr int T = T_;
    using Aux = NoAux;
    __device__ __forceinline__ gu8 *aux_ptr(const DevChunk &, const VecInfo &) const { return nullptr; }
    template <bool FULL>
    __device__ __forceinline__ void vec(const Lds &s, const VecInfo &x, const Aux &, ou8 *out, uint32_t lane) const {
        ffor_vec<T, FULL>(s.P, x.W, x.base, out, x.nvals, lane);
    }
};

struct PathDelta64 {
    __device__ __forceinline__ PathDelta64(const DevChunk &, const Lds &, uint32_t, uint32_t *) {}
    static constexpr int T = 64;
    using Aux = Aux64;
    __device__ __forceinline__ gu8 *aux_ptr(const DevChunk &c, const VecInfo &x) const {
        return gptr(c.chunk) + c.aux_off + x.aoff;
    }
    template <bool FULL>
    __device__ __forceinline__ void vec(const Lds &s, const VecInfo &x, const Aux &a, ou8 *out, uint32_t lane) const {
        delta64_vec<FULL>(s.P, x.W, x.base, a, out, x.nvals, lane);
    }
};

template <int T_>
struct PathDeltaSmall {
    __device__ __forceinline__ PathDeltaSmall(const DevChunk &, const Lds &, uint32_t, uint32_t *) {}
    static constexpr int T = T_;
    using Aux = AuxSmall<T_>;
    __device__ __forceinline__ gu8 *aux_ptr(const DevChunk &c, const VecInfo &x) const {
        return gptr(c.chunk) + c.aux_off + x.aoff;
    }
    template <bool FULL>
    __device__ __forceinline__ void vec(const Lds &s, const VecInfo &x, const Aux &a, ou8 *out, uint32_t lane) const {
        unpack_to_lds<T, true>(s.P, x.W, x.base, s.V, lane);
        wave_sync();
        chain_scan_lds<T>(s.V, a, lane);
        wave_sync();
        copy_out<T / 8, FULL>(s.V, out, x.nvals, lane);
    }
};

template <int OB, bool STAGED>
struct PathDict {
    static constexpr int T = 32;
    using Aux = NoAux;
    using Tab = typename std::conditional<STAGED, TabL, TabG>::type;
    Tab tab;              // LDS-staged or global dictionary (OB-byte entries)
    uint32_t count;
    uint32_t *err;
    __device__ __forceinline__ PathDict(const DevChunk &c, const Lds &s, uint32_t lane, uint32_t *e)
        : count(c.dict_count), err(e) {
        if constexpr (STAGED) {
            // copy the small dictionary into LDS (V + 4 KiB): the gather stays on-chip
            const uint32_t bytes = c.dict_count * OB;
            lv4 *dst = reinterpret_cast<lv4 *>(s.V + 4096);
            gu8 *src = gptr(c.dict);
            if (((uintptr_t)c.dict & 15) == 0) {
                for (uint32_t i = lane; i < (bytes + 15) / 16; i += 64) dst[i] = reinterpret_cast<gv4 *>(src)[i];
            } else {
                for (uint32_t i = lane; i < bytes; i += 64) s.V[4096 + i] = src[i];
            }
            wave_sync();
            tab.p = s.V + 4096;
        } else {
            tab.p = gptr(c.dict);
        }
    }
    __device__ __forceinline__ gu8 *aux_ptr(const DevChunk &, const VecInfo &) const { return nullptr; }
    template <bool FULL>
    __device__ __forceinline__ void vec(const Lds &s, const VecInfo &x, const Aux &, ou8 *out, uint32_t lane) const {
        unpack_to_lds<32, false>(s.P, x.W, x.base, s.V, lane);
        wave_sync();
        const FLS_LDS uint32_t *codes = reinterpret_cast<const FLS_LDS uint32_t *>(s.V);
        const uint32_t n = count;
        bool bad = false;
        gather_out<OB, FULL>(tab, out, x.nvals, lane, [&](uint32_t i) {
            uint32_t k = codes[i];
            if (k >= n) { bad = true; k = n - 1; }
            return k;
        });
        if (bad) atomicOr(err, KERR_DICT_CODE);
    }
};

template <int OB>
struct PathRle {
    static constexpr int T = 16;
    using Aux = AuxSmall<16>;
    gu8 *aux_base;
    uint32_t *err;
    __device__ __forceinline__ PathRle(const DevChunk &c, const Lds &, uint32_t, uint32_t *e)
        : aux_base(gptr(c.chunk) + c.aux_off), err(e) {}
    __device__ __forceinline__ gu8 *aux_ptr(const DevChunk &ch, const VecInfo &x) const {
        return gptr(ch.chunk) + ch.aux_off + x.aoff;
    }
    template <bool FULL>
    __device__ __forceinline__ void vec(const Lds &s, const VecInfo &x, const Aux &a, ou8 *out, uint32_t lane) const {
        unpack_to_lds<16, true>(s.P, x.W, x.base, s.V, lane);
        wave_sync();
        chain_scan_lds<16>(s.V, a, lane);
        wave_sync();
        const FLS_LDS uint16_t *idx = reinterpret_cast<const FLS_LDS uint16_t *>(s.V);
        const TabG runs{aux_base + x.aoff + 128};
        const uint32_t n = x.acount;
        bool bad = false;
        gather_out<OB, FULL>(runs, out, x.nvals, lane, [&](uint32_t i) {
            uint32_t r = idx[i];
            if (r >= n) { bad = true; r = n - 1; }
            return r;
        });
        if (bad) atomicOr(err, KERR_RUN_INDEX);
    }
};

// ALP: (F)d * 10^f * 10^-e, evaluated left to right in F (as the encoder checks)
template <int T>
struct AlpScale;
template <>
struct AlpScale<64> {
    double fm, im;
    __device__ __forceinline__ AlpScale(uint32_t e, uint32_t f) : fm(kF10D[f]), im(kIF10D[e]) {}
    __device__ __forceinline__ v4u apply(v4u x) const {
        const double a = (double)(int64_t)(((uint64_t)x.y << 32) | x.x) * fm * im;
        const double b = (double)(int64_t)(((uint64_t)x.w << 32) | x.z) * fm * im;
        const uint64_t ua = __double_as_longlong(a), ub = __double_as_longlong(b);
        return mk4((uint32_t)ua, (uint32_t)(ua >> 32), (uint32_t)ub, (uint32_t)(ub >> 32));
    }
};
template <>
struct AlpScale<32> {
    float fm, im;
    __device__ __forceinline__ AlpScale(uint32_t e, uint32_t f) : fm(kF10F[f]), im(kIF10F[e]) {}
    __device__ __forceinline__ uint32_t one(uint32_t d) const {
        return __float_as_uint((float)(int32_t)d * fm * im);
    }
    __device__ __forceinline__ v4u apply(v4u x) const { return mk4(one(x.x), one(x.y), one(x.z), one(x.w)); }
};

template <int T_>
struct PathAlp {
    static constexpr int T = T_;
    static constexpr uint32_t kMaxE = T_ == 64 ? kAlpMaxExpD : kAlpMaxExpF;
    using Aux = NoAux;
    gu8 *aux_base;
    uint32_t *err;
    __device__ __forceinline__ PathAlp(const DevChunk &c, const Lds &, uint32_t, uint32_t *e)
        : aux_base(gptr(c.chunk) + c.aux_off), err(e) {}
    __device__ __forceinline__ gu8 *aux_ptr(const DevChunk &, const VecInfo &) const { return nullptr; }
    template <bool FULL>
    __device__ __forceinline__ void vec(const Lds &s, const VecInfo &x, const Aux &, ou8 *out, uint32_t lane) const {
        const uint32_t exc = x.acount & 0xFFFF;
        const uint32_t e = min((x.acount >> 16) & 0xFF, kMaxE), f = min(x.acount >> 24, e);
        const AlpScale<T> sc(e, f);
        // registers straight to HBM, like FFOR
        const uint32_t limit = x.nvals * (T / 8);
#pragma unroll
        for (uint32_t j = 0; j < T / 8; ++j) {
            const uint32_t ci = lane + 64 * j;
            const v4u v = sc.apply(add_base<T>(unpack_chunk<T>(s.P, x.W, ci), x.base));
            if (FULL) st16(out, 16 * ci, v);
            else store16<T / 8>(out, 16 * ci, limit, v);
            seq();
        }
        if (exc == 0) return;
        // exceptions overwrite their positions (ascending, so lanes write
        // consecutive slots).  Same-wave stores to one address already land in
        // issue order; vmcnt(0) makes that explicit at the cost of one wait in
        // the (rare) vectors that have exceptions.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0), expcnt/lgkmcnt untouched
        gu8 *ea = aux_base + x.aoff;
        const FLS_GLOBAL uint16_t *pos = reinterpret_cast<const FLS_GLOBAL uint16_t *>(ea);
        gu8 *val = ea + ((2 * exc + 15) & ~15u);
        bool bad = false;
        for (uint32_t k = lane; k < exc; k += 64) {
            const uint32_t p = pos[k];
            if (p >= x.nvals) { bad = true; continue; }
            if (T == 64) {
                reinterpret_cast<FLS_GLOBAL uint64_t *>(out)[p] = reinterpret_cast<const FLS_GLOBAL uint64_t *>(val)[k];
            } else {
                reinterpret_cast<FLS_GLOBAL uint32_t *>(out)[p] = reinterpret_cast<const FLS_GLOBAL uint32_t *>(val)[k];
            }
        }
        if (bad) atomicOr(err, KERR_BAD_DESC);
    }
};

// One out-of-line function per path: each gets its own register allocation
// (inlined into one switch, hipcc allocated the union of all paths: 292 VGPRs,
// one wave per SIMD).  Arguments arrive in VGPRs, which a callee must assume
// divergent, so everything uniform is re-established with readfirstlane.
// L = 16-byte prefetch loads per lane the chunk's widest vector needs
// (8 W / 64 rounded up): the register prefetch holds only that many.
template <class Path, int L>
__device__ __attribute__((noinline)) void run_chunk(const DevChunk *chunk_generic, uint32_t lds_p, uint32_t lds_v,
                                                    uint32_t v_bytes, uint32_t *err_generic, uint32_t vrange) {
    const uint64_t cp = (uint64_t)chunk_generic;
    const FLS_GLOBAL DevChunk *cptr =
        (const FLS_GLOBAL DevChunk *)((uint64_t)uni((uint32_t)(cp >> 32)) << 32 | uni((uint32_t)cp));
    DevChunk c;
    {
        const FLS_GLOBAL v4u *q = reinterpret_cast<const FLS_GLOBAL v4u *>(cptr);
        v4u *d = reinterpret_cast<v4u *>(&c);
        d[0] = q[0];
        d[1] = q[1];
        d[2] = q[2];
        d[3] = q[3];
    }
    Lds s;
    s.P = (lv4 *)(size_t)uni(lds_p);
    s.V = (lu8 *)(size_t)uni(lds_v);
    s.v_bytes = uni(v_bytes);
    const uint64_t ep = (uint64_t)err_generic;
    uint32_t *err = (uint32_t *)((uint64_t)uni((uint32_t)(ep >> 32)) << 32 | uni((uint32_t)ep));
    const uint32_t lane = __lane_id();
    const Path path(c, s, lane, err);
    using Aux = typename Path::Aux;
    const uint32_t nvec = c.nvec;
    const uint32_t ob = c.ob;
    const ChunkMetas m = load_metas(c, lane);
    gv4 *packed = reinterpret_cast<gv4 *>(gptr(c.chunk) + c.packed_off);
    gv4 *dummy = reinterpret_cast<gv4 *>(gptr(c.chunk));
    ou8 *out = gptr(c.out);
    // this call decodes vectors [vb, ve) of the chunk (vrange = vb | ve << 8;
    // a balanced split may cut a chunk between waves)
    const uint32_t vb = uni(vrange) & 0xFF, ve = min(uni(vrange) >> 8, nvec);
    const uint32_t last_nvals = rl(m.nvbw, nvec - 1) & 0xFFFF;
    const uint32_t nfull = (ve == nvec && last_nvals != kVectorSize) ? ve - 1 : ve;

#ifdef FLS_PREFETCH2
    // (experiment build) two vectors ahead: the packed bits of v + 1 and v + 2
    // in flight while v decodes (two register sets, the loop unrolled by two
    // so each set keeps its registers; every prefetch issues all L loads, so
    // the compiler's vmcnt waits leave the second set in flight).  Not a
    // gain: with the load order of the two builds in one process swapped,
    // each build measured the same when loaded first (3.109 / 3.109 ms,
    // lineitem_full SF12.5) -- the 2.85 ms first seen was the second-loaded
    // build's advantage (profiles/r5/ab_prefetch_order_r6b.txt).
    if (vb < ve) {
        v4u ra[L], rb[L];
        VecInfo xa = vec_info(m, vb);
        Aux aa, ab;
        aa.load(path.aux_ptr(c, xa), lane);
        prefetch<L, true>(packed + xa.poff16, 8 * xa.W, dummy, lane, ra);
        VecInfo xb = vec_info(m, min(vb + 1, ve - 1));
        ab.load(path.aux_ptr(c, xb), lane);
        prefetch<L, true>(packed + xb.poff16, 8 * xb.W, dummy, lane, rb);
        uint32_t v = vb;
        for (;;) {
            if (v >= nfull) break;
            wave_sync();
            stage<L>(s.P, ra, 8 * xa.W, lane);
            {
                const VecInfo xn = vec_info(m, min(v + 2, ve - 1));
                Aux an;
                an.load(path.aux_ptr(c, xn), lane);
                prefetch<L, true>(packed + xn.poff16, 8 * xn.W, dummy, lane, ra);
                wave_sync();
                path.template vec<true>(s, xa, aa, out + (size_t)v * kVectorSize * ob, lane);
                xa = xn;
                aa = an;
            }
            ++v;
            if (v >= nfull) break;
            wave_sync();
            stage<L>(s.P, rb, 8 * xb.W, lane);
            {
                const VecInfo xn = vec_info(m, min(v + 2, ve - 1));
                Aux an;
                an.load(path.aux_ptr(c, xn), lane);
                prefetch<L, true>(packed + xn.poff16, 8 * xn.W, dummy, lane, rb);
                wave_sync();
                path.template vec<true>(s, xb, ab, out + (size_t)v * kVectorSize * ob, lane);
                xb = xn;
                ab = an;
            }
            ++v;
        }
        if (nfull < ve) {  // partial tail vector: in ra after an even number of full ones
            wave_sync();
            const bool in_a = ((v - vb) & 1) == 0;
            if (in_a) stage<L>(s.P, ra, 8 * xa.W, lane);
            else stage<L>(s.P, rb, 8 * xb.W, lane);
            wave_sync();
            if (in_a) path.template vec<false>(s, xa, aa, out + (size_t)v * kVectorSize * ob, lane);
            else path.template vec<false>(s, xb, ab, out + (size_t)v * kVectorSize * ob, lane);
        }
    }
    return;
#endif
    v4u r[L];
    Aux aux, aux_next;
    // aux (DELTA / RLE bases) is loaded before the packed bits of the same
    // vector: waiting for the packed bits (stage) then covers it, so no wait
    // on the aux load ever depends on the W-dependent number of packed loads
    VecInfo cur = vec_info(m, vb);
    aux.load(path.aux_ptr(c, cur), lane);
    prefetch<L>(packed + cur.poff16, 8 * cur.W, dummy, lane, r);
    uint32_t v = vb;
    if (vb < nfull) {
        // peeled first iteration: the loop header then only sees the steady state
        stage<L>(s.P, r, 8 * cur.W, lane);
        VecInfo nxt = vec_info(m, vb + 1 < ve ? vb + 1 : vb);
        aux_next.load(path.aux_ptr(c, nxt), lane);
        prefetch<L>(packed + nxt.poff16, 8 * nxt.W, dummy, lane, r);
        wave_sync();
        path.template vec<true>(s, cur, aux, out + (size_t)vb * kVectorSize * ob, lane);
        cur = nxt;
        aux = aux_next;
        for (v = vb + 1; v < nfull; ++v) {
            wave_sync();
            stage<L>(s.P, r, 8 * cur.W, lane);
            nxt = vec_info(m, v + 1 < ve ? v + 1 : v);
            aux_next.load(path.aux_ptr(c, nxt), lane);
            prefetch<L>(packed + nxt.poff16, 8 * nxt.W, dummy, lane, r);
            wave_sync();
            path.template vec<true>(s, cur, aux, out + (size_t)v * kVectorSize * ob, lane);
            cur = nxt;
            aux = aux_next;
        }
    }
    if (nfull < ve) {  // partial tail vector (only the last row group of a table)
        wave_sync();
        stage<L>(s.P, r, 8 * cur.W, lane);
        wave_sync();
        path.template vec<false>(s, cur, aux, out + (size_t)v * kVectorSize * ob, lane);
    }
}

// The register prefetch holds L = 8 W / 64 (rounded up to a power of two)
// 16-byte loads per lane for the chunk's widest vector W, not T / 8: fewer
// live VGPRs, no spills of in-flight prefetch data (measured: halving L for
// W <= T/2 took c3's DELTA64 keys from 2.01 to 1.88 ms,
// profiles/r1/abenv_prefetch_width_c3.txt).
template <class Path, int L>
__device__ __forceinline__ void call_l(const DevChunk *c, uint32_t lp, uint32_t lv, uint32_t vb, uint32_t *err,
                                       uint32_t max_w, uint32_t vr) {
    if constexpr (L > 1) {
        if (max_w <= 4 * L) {  // W <= 8 (L / 2): half as many loads suffice
            call_l<Path, L / 2>(c, lp, lv, vb, err, max_w, vr);
            return;
        }
    }
    run_chunk<Path, L>(c, lp, lv, vb, err, vr);
}
template <class Path>
__device__ __forceinline__ void call(const DevChunk *c, uint32_t lp, uint32_t lv, uint32_t vb, uint32_t *err,
                                     uint32_t max_w, uint32_t vr) {
    call_l<Path, Path::T / 8>(c, lp, lv, vb, err, max_w, vr);
}

template <int OB>
__device__ __forceinline__ void call_dict(const DevChunk *c, uint32_t lp, uint32_t lv, uint32_t vb, uint32_t *err,
                                          uint32_t dict_count, uint32_t max_w, uint32_t vr) {
    if (dict_count * OB + 4096 <= vb) call<PathDict<OB, true>>(c, lp, lv, vb, err, max_w, vr);
    else call<PathDict<OB, false>>(c, lp, lv, vb, err, max_w, vr);
}

// Next chunk of this wave: from the launch's work queue (one atomic per chunk,
// lane 0, broadcast) when there is one -- chunks are then taken in the host's
// largest-first order, so the launch ends on small chunks -- else grid-stride.
// The first chunk of every wave is static (no burst of same-address atomics
// at launch); the queue hands out the chunks after the grid's first round.
// stride == 0: every chunk from the queue (several grids share it).
__device__ __forceinline__ uint32_t next_chunk(uint32_t *queue, uint32_t prev, uint32_t first, uint32_t stride) {
    if (prev == UINT32_MAX && stride) return first;
    if (!queue) return prev + stride;
    uint32_t ci = 0;
    if (__lane_id() == 0) ci = atomicAdd(queue, 1u);
    return stride + uni(ci);
}

#ifdef FLS_WAVE_TRACE
// Timing build (make trace, libflsgpu_trace.so; scripts/wave_trace.py): one
// record per decode_chunk call -- start / end (s_memrealtime, 100 MHz), the
// wave, its hardware slot and XCD, the vector range and the chunk's shape.
struct TraceRec {
    uint64_t t0, t1;
    uint32_t wave, vr, hw_id, xcc_id, shape, max_w;
};
constexpr uint32_t kTraceCap = 1u << 20;
__device__ TraceRec g_trace[kTraceCap];
__device__ uint32_t g_trace_n;
#endif

__device__ __forceinline__ void decode_chunk_body(const DevChunk *cg, uint32_t lp, uint32_t lv, uint32_t v_bytes,
                                                  uint32_t *err, uint32_t vr);
// Decode vectors [vr & 0xFF, vr >> 8) of one chunk: the chunk's (encoding, T,
// output width) picks the path instantiation.
__device__ __forceinline__ void decode_chunk(const DevChunk *cg, uint32_t lp, uint32_t lv, uint32_t v_bytes,
                                             uint32_t *err, uint32_t vr) {
#ifdef FLS_WAVE_TRACE
    const uint64_t t0 = wall_clock64();
    decode_chunk_body(cg, lp, lv, v_bytes, err, vr);
    const uint64_t t1 = wall_clock64();
    if (__lane_id() == 0) {
        const uint32_t i = atomicAdd(&g_trace_n, 1u);
        if (i < kTraceCap) {
            const FLS_GLOBAL DevChunk *c = gptr(cg);
            TraceRec &r = g_trace[i];
            r.t0 = t0;
            r.t1 = t1;
            r.wave = blockIdx.x * kWaves + (threadIdx.x >> 6);
            r.vr = vr;
            r.hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            r.xcc_id = __builtin_amdgcn_s_getreg((31 << 11) | 20);
            r.shape = (uint32_t)c->enc | (uint32_t)c->T << 8 | (uint32_t)c->ob << 16 | c->nvec << 24;
            r.max_w = c->max_w;
        }
    }
#else
    decode_chunk_body(cg, lp, lv, v_bytes, err, vr);
#endif
}
__device__ __forceinline__ void decode_chunk_body(const DevChunk *cg, uint32_t lp, uint32_t lv, uint32_t v_bytes,
                                                  uint32_t *err, uint32_t vr) {
    const FLS_GLOBAL DevChunk *c = gptr(cg);
    const uint32_t dc = c->dict_count, mw = c->max_w;
    const uint32_t enc = c->enc, T = c->T, ob = c->ob;
    switch (enc) {
    case ENC_FFOR:
        switch (T) {
        case 64: call<PathFfor<64>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        case 32: call<PathFfor<32>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        case 16: call<PathFfor<16>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        default: call<PathFfor<8>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        }
        break;
    case ENC_DELTA:
        switch (T) {
        case 64: call<PathDelta64>(cg, lp, lv, v_bytes, err, mw, vr); break;
        case 32: call<PathDeltaSmall<32>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        case 16: call<PathDeltaSmall<16>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        default: call<PathDeltaSmall<8>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        }
        break;
    case ENC_DICT:
        switch (ob) {
        case 16: call_dict<16>(cg, lp, lv, v_bytes, err, dc, mw, vr); break;
        case 8: call_dict<8>(cg, lp, lv, v_bytes, err, dc, mw, vr); break;
        case 4: call_dict<4>(cg, lp, lv, v_bytes, err, dc, mw, vr); break;
        case 2: call_dict<2>(cg, lp, lv, v_bytes, err, dc, mw, vr); break;
        default: call_dict<1>(cg, lp, lv, v_bytes, err, dc, mw, vr); break;
        }
        break;
    case ENC_ALP:
        if (T == 64) call<PathAlp<64>>(cg, lp, lv, v_bytes, err, mw, vr);
        else call<PathAlp<32>>(cg, lp, lv, v_bytes, err, mw, vr);
        break;
    case ENC_RLE:
        switch (ob) {
        case 8: call<PathRle<8>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        case 4: call<PathRle<4>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        case 2: call<PathRle<2>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        default: call<PathRle<1>>(cg, lp, lv, v_bytes, err, mw, vr); break;
        }
        break;
    default:
        if ((threadIdx.x & 63) == 0) atomicOr(err, KERR_BAD_DESC);
        break;
    }
}

// vectors from position s0 to s1 (position = chunk << 7 | vector)
__device__ __forceinline__ void decode_range(const DevChunk *chunks, uint32_t nchunks, uint32_t s0, uint32_t s1,
                                             uint32_t lp, uint32_t lv, uint32_t v_bytes, uint32_t *err) {
    const uint32_t ce = min(s1 >> 7, nchunks), vend = s1 & 127;
    uint32_t vb = s0 & 127;
    for (uint32_t ci = s0 >> 7; ci < ce || (ci == ce && ci < nchunks && vb < vend); ++ci, vb = 0) {
        const uint32_t nvec = gptr(chunks)[ci].nvec;
        const uint32_t ve = min(ci == ce ? vend : nvec, nvec);
        if (vb < ve) decode_chunk(chunks + ci, lp, lv, v_bytes, err, vb | ve << 8);
    }
}

}  // namespace
}  // namespace dec
}  // namespace fls
