// fls_fsst_lab.hip -- the FSST decode EXPERIMENT library (round 1-3 variants).
//
// Built only into libflsgpu_lab.so (`make lab`, -DFLS_EXPERIMENTS), never into
// the product libflsgpu.so: it holds every kernel variant the product kernels
// in fls_fsst.hip were A/B-measured against, selected with FLS_FSST_VARIANT,
// including cost ablations (kFsstAblate*) whose output is WRONG by design
// (timing only).  Load it with FLS_LIB=libflsgpu_lab.so for same-buffer A/B
// runs (scripts/ab_env.py).
#ifndef FLS_EXPERIMENTS
#error "fls_fsst_lab.hip is the experiment library: build it with make lab (-DFLS_EXPERIMENTS)"
#endif
//
// (original header)
// fls_fsst.hip -- MI355X (gfx950) FSST string decode into DuckDB string_t.
//
// Replaces the FSST step inside RowgroupReader::materialize()
// (reference src/fastlanes_facade.cpp:48, the FLSStrColumn consumer at
// :163-170) for VARCHAR chunks written with ENC_FSST (fls_format.hpp).
//
// One wave per 64-thread block; a CU holds as many waves as its LDS fits
// (10.6 KB each at 8 B per lane per round).  Waves take contiguous ranges of
// the launch's vectors (so a wave reloads the chunk's symbol table only when
// its range crosses into the next chunk).  Per vector:
//   1. the FFOR-packed string lengths are unpacked into LDS and scanned into
//      exclusive offsets (doff[0..1024]) inside the vector's decompressed bytes;
//   2. the compressed code stream is decoded CODE-PARALLEL in rounds of
//      64 x BPL bytes (BPL = 8 per lane, one coalesced load each, the next
//      round's load in flight while this one decodes): a lane looks up its
//      codes' symbol lengths (all LDS reads issued together), a DPP wave scan
//      turns them into output positions and the lane ORs its symbols into the
//      zeroed LDS ring as aligned dwords.  The escape code (255: next byte is
//      a literal) makes a code's meaning depend on its predecessor; a lane then
//      evaluates its bytes for both entry states and a wave scan composes those
//      2-state maps (only in rounds that contain an escape byte or start right
//      after one; escape-free rounds take a branch-free path);
//   3. every string whose first min(len, 12) bytes are decoded gets its 16 B
//      string_t (inline bytes, or 4-byte prefix + pointer into the heap's host
//      copy), stored 64 records = 1 KiB at a time;
//   4. complete 16 B blocks of the ring are streamed to the chunk's heap in
//      HBM (16 B stores); the unfinished tail (< 32 B) moves to the ring start.
// Strings never straddle a vector, and every vector's heap starts 16-byte
// aligned, so only this wave writes its heap lines.
// Corrupt input (lengths that disagree with the stream, truncated escapes,
// oversized symbols) is clamped and reported through KERR_FSST.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>

#include "fls_decode.hpp"
#include "fls_format.hpp"
#include "fls_unpack.hpp"

namespace fls {
namespace {
using namespace dev;

using gv4 = const FLS_GLOBAL v4u;
using gu8 = const FLS_GLOBAL uint8_t;
using ov4 = FLS_GLOBAL v4u;
using lv4 = FLS_LDS v4u;
using lu8 = FLS_LDS uint8_t;
using lu32 = FLS_LDS uint32_t;

// One wave per 64-thread block (LDS is allocated per wave, so a CU holds as
// many waves as its LDS fits).  BPL = compressed bytes per lane per round
// (a round decodes 64 * BPL codes); the LDS ring must hold one round's output
// (<= 8 B per code) plus a carried tail.  Per-wave LDS layout (bytes, all
// 16-aligned): the vector's string lengths -- SMALL chunks (every string
// <= 255 bytes, DevChunk.vbits = 1) keep them as u8[1024], others as exclusive
// u32 offsets doff[1025] -- then u64 symbol[256], u8 length[256] and the ring.
// The packed string lengths of step 1 are staged in the ring, which is free
// until the rounds start.
template <int BPL, bool SMALL, int SEG = 0, bool D8 = false>
struct Lds {
    static constexpr uint32_t kOffD = 0;
    // string lengths / offsets: SMALL u8 lengths (1 KB), SMALL segmented
    // u16 offsets mod 65536 (1025 entries) or u8 lengths (D8), others u32
    // offsets (1025 entries)
    static constexpr uint32_t kOffSym = SMALL ? ((SEG && !D8) ? 2064 : 1024) : 4112;
    static constexpr uint32_t kOffLen = kOffSym + 2048;
    // D8: no length table (the segmented kernel reads lengths packed in the
    // staged symbols)
    static constexpr uint32_t kOffRing = kOffLen + (D8 ? 0 : 256);
    static constexpr uint32_t kPackedMax = SMALL ? 128 * 8 + 128 : 128 * 32 + 128;  // W <= 8 | 32, + zero row
    static constexpr uint32_t kRound = 64 * BPL;
    // 2 KiB holds a round's output at up to ~4 bytes per code; a round that
    // decodes to more is written in parts (lanes [l0, l1) at a time)
    // SEG: a round is 64 segments of 16 codes (about 2.8 KB of l_comment);
    // kSegCap bytes of decoded output per part, plus the slack a lane may
    // write past its segment's claimed end (16 codes x 8 B + a qword) when a
    // corrupt table understates it
    static constexpr uint32_t kSegCap = SEG > 0 ? (uint32_t)SEG : 4096u;  // SEG = the cap (bytes)
    static constexpr uint32_t kSegSlack = 2 * 16 * 8 + 16;   // up to 2 segments per lane
    static constexpr uint32_t kRingPlain = kPackedMax > 2048 + 64 ? kPackedMax : 2048 + 64;
    static constexpr uint32_t kRingSeg = kPackedMax > kSegCap + kSegSlack ? kPackedMax : kSegCap + kSegSlack;
    static constexpr uint32_t kRing = SEG ? kRingSeg : kRingPlain;
    static constexpr uint32_t kWave = kOffRing + kRing;
    static_assert(kOffSym % 16 == 0 && kOffRing % 16 == 0 && kWave % 16 == 0, "LDS layout alignment");
};

__device__ __forceinline__ uint32_t rl(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint32_t byte_of(const v4u &r, uint32_t k) {
    const uint32_t w = k < 4 ? r.x : k < 8 ? r.y : k < 12 ? r.z : r.w;
    return (w >> (8 * (k & 3))) & 0xFF;
}
// Inclusive wave-64 prefix sum on DPP (row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast 15/31 across rows): six VALU steps, no LDS round trip.
__device__ __forceinline__ uint32_t scan_incl(uint32_t x, uint32_t /*lane*/) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

struct Wave {
    lv4 *P;
    lu32 *D;
    const FLS_LDS uint64_t *sym;
    const lu8 *len;
    lu8 *ring;
};

// Escape state entering a lane's first code (the parity rule).  Code 255 is
// the escape (the next byte is a literal).  After any byte other than 0xFF
// the decoder is in the normal state (that byte was a symbol code, or the
// literal of an escape), so the state entering byte p is the parity of the
// run of 0xFF bytes that ends at p - 1.  A lane holding some non-0xFF byte
// therefore leaves its segment in state (length of its trailing 0xFF run) & 1
// whatever its entry state; a lane of BPL (even) 0xFF bytes leaves it in its
// entry state.  So a lane's entry state is the exit state of the nearest
// earlier lane holding a non-0xFF byte (one ballot + one ds_bpermute), or the
// state the previous round ended in.  No 2-state maps, no per-round wave
// composition, no special path for rounds that contain escapes.
__device__ __forceinline__ uint32_t entry_state(bool has_plain, uint32_t exit_if_plain, uint32_t carry,
                                                uint32_t lane) {
    const uint64_t m = __ballot(has_plain) & ((1ull << lane) - 1ull);  // lane 0: 0
    const uint32_t src = m ? 63u - (uint32_t)__builtin_clzll(m) : 0u;
    const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)exit_if_plain);
    return m ? v : carry;
}

// Appends symbols to the zeroed ring at byte wp through a 64-bit accumulator
// that is OR-ed (ds_or_b64) into its aligned qword after every symbol: OR is
// idempotent, so no select on whether the qword is complete; a lane's edge
// qwords are shared with its neighbours' output and OR-ing merges them.
// Symbols must be masked to their length (the staged table is).  Measured
// against OR-ing every symbol into both qwords it spans (no accumulator,
// fewer VALU, twice the ds_or_b64): 1-2 % faster on l_comment.
// QMask: qword index mask of a circular ring (kFsstCirc), ~0 for a flat one.
template <uint32_t QMask = ~0u>
struct QwordWriter {
    FLS_LDS uint64_t *o64;
    uint64_t acc;
    uint32_t q, bits;
    __device__ __forceinline__ QwordWriter(lu8 *ring, uint32_t wp)
        : o64(reinterpret_cast<FLS_LDS uint64_t *>(ring)), acc(0), q((wp >> 3) & QMask), bits(8 * (wp & 7)) {}
    __device__ __forceinline__ void put(uint64_t v, uint32_t n) {  // n <= 8 bytes
        // v << bits spans qwords q (lo) and q + 1 (hi); (v >> 1) >> (63 - bits)
        // is v >> (64 - bits) without the bits == 0 case
        const uint64_t lo = v << bits, hi = (v >> 1) >> (63 - bits);
        acc |= lo;
        __hip_atomic_fetch_or(o64 + q, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t nb = bits + 8 * n;
        const bool e = nb >= 64;
        q = (q + (e ? 1u : 0u)) & QMask;
        acc = e ? hi : acc;
        bits = nb & 63;
    }
    __device__ __forceinline__ void finish() {
        __hip_atomic_fetch_or(o64 + q, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
};

// One round's codes of this lane (nb valid bytes of raw) from the escape
// state the previous round ended in (carry): the symbols v[k] and their byte
// counts n[k] (a literal is one byte, the escape code none -- its staged table
// entry is {0, 0} -- and a symbol its length; nothing past the stream end,
// FULL = no lane of the round reaches it).  Returns the lane's byte count;
// st_out = the state after its last valid byte (held across an empty tail).
// Byte count of a staged symbol from its bits (LFS, kFsstLenFromSym): the
// table is masked to the symbols' lengths, so a symbol whose last byte is not
// zero has length ceil(bit length / 8), and the escape entry (0) length 0.
__device__ __forceinline__ uint32_t len_from_sym(uint64_t x) { return (71u - (uint32_t)__clzll((long long)x)) >> 3; }

// The table entries of a lane's BPL codes (kFsstEarlyGather: read before the
// previous round's retire(), so their LDS latency runs under its work).
template <int BPL>
struct Gathered {
    uint64_t sy[BPL];
    uint32_t sl[BPL];
};
template <int BPL>
__device__ __forceinline__ void gather_codes(const Wave &w, const v4u &raw, Gathered<BPL> &g) {
#pragma unroll
    for (uint32_t k = 0; k < BPL; ++k) {
        const uint32_t c = byte_of(raw, k);
        g.sy[k] = w.sym[c];
        g.sl[k] = w.len[c];
    }
}

template <int BPL, bool FULL, bool LFS = false>
__device__ __forceinline__ uint32_t lane_codes(const Wave &w, const v4u &raw, uint32_t nb, uint32_t carry,
                                               uint32_t lane, uint64_t (&v)[BPL], uint32_t (&n)[BPL],
                                               uint32_t &st_out, const Gathered<BPL> *pre = nullptr) {
    uint32_t code[BPL], sl[BPL];
    uint64_t sy[BPL];
    int32_t last = -1;  // last non-0xFF byte of the lane's segment
#pragma unroll
    for (uint32_t k = 0; k < BPL; ++k) {  // all table reads issued together
        code[k] = byte_of(raw, k);
        sy[k] = pre ? pre->sy[k] : w.sym[code[k]];
        sl[k] = pre ? pre->sl[k] : LFS ? len_from_sym(sy[k]) : (uint32_t)w.len[code[k]];
        if ((FULL || k < nb) && code[k] != kFsstEscape) last = (int32_t)k;
    }
    const uint32_t end = FULL ? (uint32_t)BPL : nb;
    uint32_t st = entry_state(last >= 0, ((int32_t)end - 1 - last) & 1, carry, lane);
    uint32_t out = 0;
#pragma unroll
    for (uint32_t k = 0; k < BPL; ++k) {
        const bool lit = st != 0, in = FULL || k < nb;
        const uint64_t vk = lit ? (uint64_t)code[k] : sy[k];
        const uint32_t nk = lit ? 1u : sl[k];
        v[k] = in ? vk : 0ull;
        n[k] = in ? nk : 0u;
        st = in ? (uint32_t)(!lit && code[k] == kFsstEscape) : st;
        out += n[k];
    }
    st_out = st;
    return out;
}

// A round in which no lane holds an escape byte (and that does not start
// inside an escape): every code is a symbol, so no entry state and no
// literal selects.
template <int BPL>
__device__ __forceinline__ uint32_t lane_codes_plain(const Wave &w, const v4u &raw, uint64_t (&v)[BPL],
                                                     uint32_t (&n)[BPL]) {
    uint32_t out = 0;
#pragma unroll
    for (uint32_t k = 0; k < BPL; ++k) {
        const uint32_t c = byte_of(raw, k);
        v[k] = w.sym[c];
        n[k] = w.len[c];
        out += n[k];
    }
    return out;
}
// does any of the lane's BPL bytes equal the escape code 0xFF?  (x has an
// 0xFF byte iff ~x has a zero byte)
template <int BPL>
__device__ __forceinline__ bool has_escape(const v4u &raw) {
    auto ff = [](uint32_t x) -> uint32_t { return (~x - 0x01010101u) & x & 0x80808080u; };
    return (BPL == 8 ? (ff(raw.x) | ff(raw.y)) : (ff(raw.x) | ff(raw.y) | ff(raw.z) | ff(raw.w))) != 0;
}

// One lane's segment (segmented kernel): its nb (<= 16) code bytes in raw,
// decoded from escape state st into the ring at byte wp; returns the bytes
// written, st = the state after its last code.  FULL: all 16 bytes are codes;
// ESC: the vector holds escape codes (without them every code is a symbol,
// and a stray escape decodes to nothing -- its staged entry is {0, 0} -- which
// the byte-count check catches).  Table reads go out 8 codes at a time.
// Every symbol OR-ed into both qwords it spans (kFsstTwoQ: one more ds_or_b64
// per code, half the VALU of the accumulator's carry logic)
struct TwoQWriter {
    FLS_LDS uint64_t *o64;
    uint32_t p;
    __device__ __forceinline__ TwoQWriter(lu8 *ring, uint32_t wp) : o64(reinterpret_cast<FLS_LDS uint64_t *>(ring)), p(wp) {}
    __device__ __forceinline__ void put(uint64_t v, uint32_t n) {
        // shift counts are taken mod 64 by the hardware: 8p mod 64 is the bit
        // offset inside qword p / 8, ~(8p) mod 64 = 63 - it
        const uint32_t b8 = p << 3;
        const uint64_t lo = v << (b8 & 63), hi = (v >> 1) >> (~b8 & 63);
        __hip_atomic_fetch_or(o64 + (p >> 3), lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_or(o64 + (p >> 3) + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        p += n;
    }
    __device__ __forceinline__ void finish() {}
};

// The accumulator writer, storing only when a qword is complete (kFsstSegSparse):
// ~1 lane in 4 takes part in a code step's ds_or_b64 instead of all 64, which
// is where the LDS bank conflicts of the per-code OR came from
struct SparseWriter {
    FLS_LDS uint64_t *o64;
    uint64_t acc;
    uint32_t q, bits;
    __device__ __forceinline__ SparseWriter(lu8 *ring, uint32_t wp)
        : o64(reinterpret_cast<FLS_LDS uint64_t *>(ring)), acc(0), q(wp >> 3), bits(8 * (wp & 7)) {}
    __device__ __forceinline__ void put(uint64_t v, uint32_t n) {
        const uint64_t lo = v << bits, hi = (v >> 1) >> (63 - bits);
        acc |= lo;
        const uint32_t nb = bits + 8 * n;
        if (nb >= 64) {
            __hip_atomic_fetch_or(o64 + q, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            ++q;
            acc = hi;
        }
        bits = nb & 63;
    }
    __device__ __forceinline__ void finish() {
        if (bits) __hip_atomic_fetch_or(o64 + q, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
};

// PL: the staged table holds each symbol's length in its top byte (symbols of
// at most 7 bytes, kFsstSegPackedLen): one table read per code instead of two
// FB: codes per batch of table reads on the fast path (FULL, no escapes): 8,
// or all 16 issued together (kFsstSegWide)
// cost ablation (kFsstAblateWrite, wrong output): the symbols are read and
// summed but never written
struct NullWriter {
    uint64_t acc = 0;
    lu8 *ring;
    uint32_t wp;
    __device__ __forceinline__ NullWriter(lu8 *r, uint32_t p) : ring(r), wp(p) {}
    __device__ __forceinline__ void put(uint64_t v, uint32_t n) { acc += v + n; }
    __device__ __forceinline__ void finish() {
        if (acc == 0x123456789ull) ring[wp] = 1;  // keeps the reads alive
    }
};
// The sparse writer with lengths in bits (kFsstSegLean: the staged table's
// top byte holds 8 x the symbol length, so no multiply per code), the ring
// position kept as the byte address of the open qword plus a bit offset, and
// the carry out of a completed qword as one shift (the bit offset is >= 8
// whenever a qword completes: symbols are <= 7 bytes).  The staged symbol's
// top byte is masked off by the caller.
struct LeanWriter {
    lu8 *ring;
    uint64_t acc;
    uint32_t a, b, start;   // open qword's ring byte, bit offset in it, start position (bits)
    __device__ __forceinline__ LeanWriter(lu8 *r, uint32_t wp)
        : ring(r), acc(0), a(wp & ~7u), b(8 * (wp & 7)), start(8 * wp) {}
    __device__ __forceinline__ void put(uint64_t v, uint32_t bl) {  // bl = 8 x length, <= 56
        acc |= v << b;
        const uint32_t nb = b + bl;
        if (nb >= 64) {
            __hip_atomic_fetch_or(reinterpret_cast<FLS_LDS uint64_t *>(ring + a), acc, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
            a += 8;
            acc = v >> (64 - b);
        }
        b = nb & 63;
    }
    // an entry as staged (8 x length in the top byte): the length is added
    // straight from the top byte (one v_add_u32_sdwa), then the high dword
    // masked in place -- the empty asm orders the two, otherwise the compiler
    // masks into a new register first and copies the low dword beside it
    __device__ __forceinline__ void put_tagged(uint32_t lo, uint32_t hi) {
        uint32_t nb = b + (hi >> 24);
        asm("" : "+v"(hi), "+v"(nb));
        hi &= 0x00FFFFFFu;
        const uint64_t v = (uint64_t)hi << 32 | lo;
        acc |= v << b;
        if (nb >= 64) {
            __hip_atomic_fetch_or(reinterpret_cast<FLS_LDS uint64_t *>(ring + a), acc, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
            a += 8;
            acc = v >> (64 - b);
        }
        b = nb & 63;
    }
    __device__ __forceinline__ void finish() {
        if (b) __hip_atomic_fetch_or(reinterpret_cast<FLS_LDS uint64_t *>(ring + a), acc, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    __device__ __forceinline__ uint32_t bytes() const { return (8 * a + b - start) >> 3; }
};
template <int WR>   // 0 accumulator, 1 two-qword, 2 sparse, 3 none (ablation), 4 lean
using SegWriter = typename std::conditional<
    WR == 1, TwoQWriter,
    typename std::conditional<
        WR == 2, SparseWriter,
        typename std::conditional<WR == 3, NullWriter,
                                  typename std::conditional<WR == 4, LeanWriter, QwordWriter<>>::type>::type>::type>::type;

template <bool FULL, bool ESC, int WR = 0, bool PL = false, uint32_t FB = 8>
__device__ __forceinline__ uint32_t seg_lane(const Wave &w, const v4u &raw_in, uint32_t nb, uint32_t &st,
                                             SegWriter<WR> &qw) {
    // an opaque copy: the callers' variants would otherwise share (hoist) the
    // byte extraction and table addresses of all 16 codes ahead of their
    // branch, all of them live at once
    v4u raw = raw_in;
    asm volatile("" : "+v"(raw.x), "+v"(raw.y), "+v"(raw.z), "+v"(raw.w));
    // codes per batch of table reads: the general path keeps each code byte
    // (a literal's value) beside its table entry, so it reads 4 at a time to
    // stay in the fast path's register budget
    constexpr uint32_t B = (FULL && !ESC) ? FB : 4;
    // lean writer: lengths in bits (the staged top byte is 8 x the length)
    constexpr bool LEAN = WR == 4;
    static_assert(!LEAN || PL, "the lean writer reads packed lengths");
    constexpr uint32_t kLitLen = LEAN ? 8u : 1u;
    uint32_t got = 0;
#pragma unroll
    for (uint32_t h = 0; h < 16 / B; ++h) {
        uint32_t c[B], sl[B];
        uint64_t sy[B];
#pragma unroll
        for (uint32_t k = 0; k < B; ++k) {
            c[k] = byte_of(raw, B * h + k);
            sy[k] = w.sym[c[k]];
            if constexpr (LEAN && FULL && !ESC) {
                sl[k] = 0;   // put_tagged() reads the length from the entry
            } else if constexpr (PL) {
                sl[k] = (uint32_t)(sy[k] >> 56);
                sy[k] &= 0x00FFFFFFFFFFFFFFull;
            } else {
                sl[k] = w.len[c[k]];
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < B; ++k) {
            // selects as bit masks (v_bfi), not compares: per-code lane masks
            // would each take an SGPR pair, and 16 live ones spill
            uint32_t vlo = (uint32_t)sy[k], vhi = (uint32_t)(sy[k] >> 32), n = sl[k];
            if constexpr (ESC) {
                const uint32_t lit = 0u - st;                        // all ones after an escape
                vlo = (vlo & ~lit) | (c[k] & lit);
                vhi &= ~lit;
                n = (n & ~lit) | (kLitLen & lit);
                uint32_t ns = ((c[k] + 1u) >> 8) & ~st;             // an escape code, not a literal
                if constexpr (!FULL) {
                    const uint32_t in = 0u - (((B * h + k) - nb) >> 31);  // all ones iff Bh + k < nb
                    ns = (ns & in) | (st & ~in);
                }
                st = ns;
            }
            if constexpr (!FULL) {
                const uint32_t in = 0u - (((B * h + k) - nb) >> 31);
                vlo &= in;
                vhi &= in;
                n &= in;
            }
            if constexpr (LEAN && FULL && !ESC) {
                qw.put_tagged(vlo, vhi);
                continue;
            }
            qw.put((uint64_t)vhi << 32 | vlo, n);
            if constexpr (!LEAN) got += n;
        }
        // the next batch's table reads stay behind this batch's writes:
        // hoisted, their values would be live across them (spills)
        wave_sync();
    }
    if constexpr (LEAN) return qw.bytes();
    return got;
}

// string_t of a string of n bytes at ring byte x, host pointer p (DMask:
// dword index mask of a circular ring, ~0 for a flat one)
template <uint32_t DMask = ~0u>
__device__ __forceinline__ v4u make_record_at(const lu8 *ring, uint32_t x, uint32_t n, uint64_t p) {
    const lu32 *r32 = reinterpret_cast<const lu32 *>(ring);
    const uint32_t i0 = x >> 2, sh = x & 3;
    const uint32_t w0 = r32[i0 & DMask], w1 = r32[(i0 + 1) & DMask], w2 = r32[(i0 + 2) & DMask],
                   w3 = r32[(i0 + 3) & DMask];
    const uint32_t b0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
    if (n > 12) return mk4(n, b0, (uint32_t)p, (uint32_t)(p >> 32));
    const uint32_t b1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    const uint32_t b2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
    auto keep = [n](uint32_t word, uint32_t first) -> uint32_t {  // zero bytes at index >= n
        if (n >= first + 4) return word;
        if (n <= first) return 0u;
        return word & ((1u << (8 * (n - first))) - 1u);
    };
    return mk4(n, keep(b0, 0), keep(b1, 4), keep(b2, 8));
}

// string_t of string i (doff d0, length n) from the ring: a flat ring holds
// byte ring_base at ring byte 0, a circular one (CircBytes) byte g at g mod CircBytes
template <uint32_t CircBytes>
__device__ __forceinline__ v4u make_record(const Wave &w, uint32_t d0, uint32_t n, uint32_t ring_base,
                                           uint64_t ptr_base) {
    if constexpr (CircBytes != 0) return make_record_at<CircBytes / 4 - 1>(w.ring, d0, n, ptr_base + d0);
    else return make_record_at(w.ring, d0 - ring_base, n, ptr_base + d0);
}

template <int BPL, bool SMALL, int V, int SEG = 0>
__device__ void fsst_vector(const Wave &w, gu8 *packed_vec, uint32_t W, uint32_t base, uint32_t nvals,
                            uint32_t dbytes, gu8 *vh, FLS_GLOBAL uint8_t *heap, uint32_t heap_bytes,
                            uint64_t heap_host, FLS_GLOBAL uint8_t *out, uint32_t lane, uint32_t *err,
                            bool table_lfs = false) {
    static_assert(!SEG || (BPL == 16 && (V & kFsstZeroFlush)),
                  "the segmented kernel: 16 codes per lane, zero-at-flush ring");
    constexpr bool D8 = SMALL && SEG && (V & kFsstSegD8) != 0;
    static_assert(!D8 || ((V & kFsstSegBatch) && (V & kFsstSegPackedLen)), "u8 lengths: batched records, packed lengths");
    using Layout = Lds<BPL, SMALL, SEG, D8>;
    bool bad = false;
    // kFsstCirc: a circular ring of kCirc bytes (a power of two) indexed by
    // decoded byte position mod kCirc, so retire() moves no tail, it only
    // advances ring_base (needs the zero-at-flush invariant)
    constexpr uint32_t kCirc = (!SEG && (V & kFsstCirc)) ? (Layout::kRing >= 4096 ? 4096u : 2048u) : 0u;
    static_assert(!(V & kFsstCirc) || ((V & kFsstZeroFlush) && !(V & kFsstTwoQ)), "kFsstCirc needs zero-at-flush");
    static_assert(kCirc <= Layout::kRing, "circular ring fits the ring area");
    // ---- 1. string lengths: u8 lengths (SMALL) or exclusive u32 offsets -----
    W = SMALL ? min(W, 8u) : W;
    const uint32_t n16 = 8 * W;
    gv4 *pk = reinterpret_cast<gv4 *>(packed_vec);
    for (uint32_t i = lane; i < n16; i += 64) w.P[i] = pk[i];
    if (lane < 8) w.P[n16 + lane] = mk4(0, 0, 0, 0);
    wave_sync();
    uint32_t total = 0;
    if constexpr (SMALL && SEG && !D8) {
        // u8 lengths staged in the ring past the packed words, then each lane
        // turns 16 consecutive ones into u16 exclusive offsets (mod 65536:
        // finalize_seg rebuilds the high bits, strings being <= 255 bytes)
        lu32 *L8 = reinterpret_cast<lu32 *>(w.ring + 2048);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t ci = lane + 64 * j;
            const v4u v = add_base<32>(unpack_chunk<32>(w.P, W, ci), base);
            const uint32_t b0 = 4 * ci < nvals ? v.x & 255 : 0, b1 = 4 * ci + 1 < nvals ? v.y & 255 : 0;
            const uint32_t b2 = 4 * ci + 2 < nvals ? v.z & 255 : 0, b3 = 4 * ci + 3 < nvals ? v.w & 255 : 0;
            L8[ci] = b0 | b1 << 8 | b2 << 16 | b3 << 24;
        }
        wave_sync();
        const v4u q = reinterpret_cast<const lv4 *>(L8)[lane];
        const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
        uint32_t a[16], run = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            a[k] = run;
            run += (wd[k >> 2] >> (8 * (k & 3))) & 255;
        }
        const uint32_t incl = scan_incl(run, lane);
        const uint32_t excl = incl - run;
        lu32 *D32 = reinterpret_cast<lu32 *>(w.D);
#pragma unroll
        for (int k = 0; k < 16; k += 2) D32[8 * lane + k / 2] = ((excl + a[k]) & 0xFFFF) | (excl + a[k + 1]) << 16;
        if (lane == 63) reinterpret_cast<FLS_LDS uint16_t *>(w.D)[1024] = (uint16_t)incl;
        total = rl(incl, 63);
        wave_sync();
    } else if constexpr (SMALL) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t ci = lane + 64 * j;
            const v4u v = add_base<32>(unpack_chunk<32>(w.P, W, ci), base);
            const uint32_t b0 = 4 * ci < nvals ? v.x & 255 : 0, b1 = 4 * ci + 1 < nvals ? v.y & 255 : 0;
            const uint32_t b2 = 4 * ci + 2 < nvals ? v.z & 255 : 0, b3 = 4 * ci + 3 < nvals ? v.w & 255 : 0;
            reinterpret_cast<lu32 *>(w.D)[ci] = b0 | b1 << 8 | b2 << 16 | b3 << 24;
            run += b0 + b1 + b2 + b3;
        }
        total = rl(scan_incl(run, lane), 63);
        wave_sync();
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t ci = lane + 64 * j;
            v4u v = add_base<32>(unpack_chunk<32>(w.P, W, ci), base);
            if (4 * ci + 0 >= nvals) v.x = 0;
            if (4 * ci + 1 >= nvals) v.y = 0;
            if (4 * ci + 2 >= nvals) v.z = 0;
            if (4 * ci + 3 >= nvals) v.w = 0;
            reinterpret_cast<lv4 *>(w.D)[ci] = v;
        }
        wave_sync();
        uint32_t a[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u v = reinterpret_cast<const lv4 *>(w.D)[4 * lane + q];
            a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
        }
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t t = a[k];
            a[k] = run;  // exclusive
            run += t;
        }
        const uint32_t incl = scan_incl(run, lane);
        const uint32_t excl = incl - run;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            reinterpret_cast<lv4 *>(w.D)[4 * lane + q] =
                mk4(excl + a[4 * q], excl + a[4 * q + 1], excl + a[4 * q + 2], excl + a[4 * q + 3]);
        if (lane == 63) w.D[1024] = incl;
        total = rl(incl, 63);
        wave_sync();
    }
    if (total != dbytes) bad = true;
    if constexpr ((V & kFsstZeroFlush) != 0) {
        // the ring (which staged the packed lengths) starts all zero; from
        // here on every byte past the decoded ones stays zero: flush() zeroes
        // the blocks it streams out and retire() the bytes its tail vacates,
        // so the rounds OR into zeros without zeroing first
        for (uint32_t q = lane; q < Layout::kRing / 16; q += 64)
            reinterpret_cast<lv4 *>(w.ring)[q] = mk4(0, 0, 0, 0);
        wave_sync();
    }
    const FLS_GLOBAL FsstVecHeader *hp = reinterpret_cast<const FLS_GLOBAL FsstVecHeader *>(vh);
    const uint32_t heap_off = uni(hp->heap_off), comp_len = uni(hp->comp_len), clen_w = uni(min(hp->clen_w, 32u));
    const uint32_t hlim = min((dbytes + 15) & ~15u, heap_bytes > heap_off ? heap_bytes - heap_off : 0u);
    FLS_GLOBAL uint8_t *vheap = heap + heap_off;
    const uint64_t ptr_base = heap_host + heap_off;
    gv4 *comp = reinterpret_cast<gv4 *>(vh + sizeof(FsstVecHeader) + 128 * clen_w);

    // next_str = first string without its string_t yet, str_base = its offset
    uint32_t out_pos = 0, ring_base = 0, carry_lit = 0, next_str = 0, str_base = 0;
    // strings whose leading bytes are all decoded get their string_t
    auto finalize = [&]() {
        while (next_str < nvals) {
            const uint32_t i = next_str + lane;
            uint32_t d0 = 0, n = 0, incl = 0;
            if constexpr (SMALL) {
                n = i < nvals ? (uint32_t)reinterpret_cast<const lu8 *>(w.D)[i] : 0u;
                incl = scan_incl(n, lane);
                d0 = str_base + incl - n;
            } else if (i < nvals) {
                d0 = w.D[i];
                n = w.D[i + 1] - d0;
            }
            const bool ok = i < nvals && d0 + min(n, 12u) <= out_pos;
            const uint64_t m = __ballot(ok);
            const uint32_t n_ok = ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (lane < n_ok)
                *reinterpret_cast<ov4 *>(out + 16ull * i) = make_record<kCirc>(w, d0, n, ring_base, ptr_base);
            if constexpr (SMALL) {
                if (n_ok > 0) str_base += rl(incl, n_ok - 1);
            }
            next_str += n_ok;
            if (n_ok < 64) break;
        }
        if constexpr (!SMALL) str_base = next_str < nvals ? uni(w.D[next_str]) : out_pos;
    };
    // Segmented kernel: records in whole batches of 64 strings (no partial
    // batch per round; the ring keeps an unfinished batch's bytes), offsets
    // read straight from D (no length scan), the record assembled without
    // branches.  force: also a partial batch (vector end, ring full).
    auto finalize_seg = [&](bool force) {
        if constexpr ((V & kFsstAblateRecords) != 0) {  // cost ablation (wrong output): no records
            next_str = nvals;
            return;
        }
        if constexpr ((V & kFsstSegBatch) == 0) {
            // two batches of 64 strings per pass (strings i and i + 64 of
            // every lane): both offset reads, then both sets of ring reads are
            // in flight together, two LDS round trips per 128 records
            while (next_str < nvals) {
                uint32_t d0[2], n[2], rel1[2];
                bool ok[2];
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
                    const uint32_t i = next_str + 64 * h + lane;
                    uint32_t r0, r1;  // string start / end relative to str_base
                    if constexpr (SMALL) {   // u16 offsets mod 65536: 128 strings span < 32 KB
                        const FLS_LDS uint16_t *D16 = reinterpret_cast<const FLS_LDS uint16_t *>(w.D);
                        const uint32_t b16 = D16[next_str];
                        r0 = (D16[min(i, nvals)] - b16) & 0xFFFF;
                        r1 = (D16[min(i + 1, nvals)] - b16) & 0xFFFF;
                    } else {
                        r0 = w.D[min(i, nvals)] - str_base;
                        r1 = w.D[min(i + 1, nvals)] - str_base;
                    }
                    d0[h] = str_base + r0;
                    n[h] = r1 - r0;
                    rel1[h] = r1;
                    ok[h] = i < nvals && d0[h] + min(n[h], 12u) <= out_pos;
                }
                const uint64_t ma = __ballot(ok[0]), mb = __ballot(ok[1]);
                const uint32_t na = ~ma == 0 ? 64u : (uint32_t)__builtin_ctzll(~ma);
                const uint32_t nb = na < 64 ? 0u : ~mb == 0 ? 64u : (uint32_t)__builtin_ctzll(~mb);
                const lu32 *r32 = reinterpret_cast<const lu32 *>(w.ring);
                uint32_t wd[2][4];
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {  // (lanes past the complete ones read harmless ring words)
                    const uint32_t i0 = min(d0[h] - ring_base, Layout::kRing - 16) >> 2;
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) wd[h][k] = r32[i0 + k];
                }
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
                    if (lane < (h ? nb : na)) {
                        const uint32_t sh = (d0[h] - ring_base) & 3, nn = n[h];
                        const uint32_t b0 = __builtin_amdgcn_alignbyte(wd[h][1], wd[h][0], sh);
                        const uint32_t b1 = __builtin_amdgcn_alignbyte(wd[h][2], wd[h][1], sh);
                        const uint32_t b2 = __builtin_amdgcn_alignbyte(wd[h][3], wd[h][2], sh);
                        auto keep = [nn](uint32_t word, uint32_t first) -> uint32_t {  // bytes [first, nn) of 4
                            const uint32_t c = nn > first ? min(nn - first, 4u) : 0u;
                            return c >= 4 ? word : word & ((1u << (8 * c)) - 1u);
                        };
                        const uint64_t p = ptr_base + d0[h];
                        const bool inl = nn <= 12;
                        *reinterpret_cast<ov4 *>(out + 16ull * (next_str + 64 * h + lane)) =
                            mk4(nn, inl ? keep(b0, 0) : b0, inl ? keep(b1, 4) : (uint32_t)p,
                                inl ? keep(b2, 8) : (uint32_t)(p >> 32));
                    }
                }
                const uint32_t tot = na + nb;
                if (nb > 0) str_base += rl(rel1[1], nb - 1);
                else if (na > 0) str_base += rl(rel1[0], na - 1);
                next_str += tot;
                if (tot < 128) break;
            }
            return;
        }
        while (next_str < nvals) {
            const uint32_t i = next_str + lane;
            const bool valid = i < nvals;
            uint32_t rel0, rel1;  // string start / end relative to str_base
            if constexpr (D8) {  // u8 lengths: offsets by a wave scan
                const uint32_t n8 = valid ? (uint32_t)reinterpret_cast<const lu8 *>(w.D)[i] : 0u;
                rel1 = scan_incl(n8, lane);
                rel0 = rel1 - n8;
            } else if constexpr (SMALL) {
                const FLS_LDS uint16_t *D16 = reinterpret_cast<const FLS_LDS uint16_t *>(w.D);
                const uint32_t a = D16[min(i, nvals)], b = D16[min(i + 1, nvals)];
                const uint32_t b16 = rl(a, 0);
                rel0 = (a - b16) & 0xFFFF;
                rel1 = (b - b16) & 0xFFFF;
            } else {
                rel0 = w.D[min(i, nvals)] - str_base;
                rel1 = w.D[min(i + 1, nvals)] - str_base;
            }
            const uint32_t d0 = str_base + rel0, n = rel1 - rel0;
            const bool ok = valid && d0 + min(n, 12u) <= out_pos;
            const uint64_t m = __ballot(ok), vm = __ballot(valid);
            // kFsstSegBatch: wait for the whole batch, unless its bytes fill
            // half the ring (long strings: a batch of 64 may not fit the ring
            // at all); measured slower (the kept tail moves every round)
            if ((V & kFsstSegBatch) && !force && m != vm && out_pos - str_base <= Layout::kSegCap / 2) break;
            const uint32_t n_ok = ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (lane < n_ok) {
                const lu32 *r32 = reinterpret_cast<const lu32 *>(w.ring);
                const uint32_t x = d0 - ring_base, i0 = x >> 2, sh = x & 3;
                const uint32_t w0 = r32[i0], w1 = r32[i0 + 1], w2 = r32[i0 + 2], w3 = r32[i0 + 3];
                const uint64_t p = ptr_base + d0;
                const bool inl = n <= 12;
                if constexpr ((V & kFsstSegLean) != 0) {
                    // one v_perm_b32 per word aligns and masks: selector byte
                    // j is sh + j (a byte of the ring dword pair) while
                    // 4k + j < n, else 12 (a zero byte); the bytes at or past
                    // the length come from a 64-bit shift of ones by
                    // 8 x clamp(n - 4k, 0, 4) (amounts 0..32, no wrap)
                    const uint32_t base = 0x03020100u + sh * 0x01010101u, t = 8 * n;
                    auto word = [&](uint32_t hi, uint32_t lo, int k) -> uint32_t {
                        const uint32_t sk = (uint32_t)min(max((int)t - 32 * k, 0), 32);
                        const uint32_t past = (uint32_t)(0xFFFFFFFFull << sk);
                        const uint32_t sel = (past & 0x0C0C0C0Cu) | (~past & base);
                        return __builtin_amdgcn_perm(hi, lo, sel);
                    };
                    *reinterpret_cast<ov4 *>(out + 16ull * i) =
                        mk4(n, word(w1, w0, 0), inl ? word(w2, w1, 1) : (uint32_t)p, inl ? word(w3, w2, 2) : (uint32_t)(p >> 32));
                } else {
                    const uint32_t b0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
                    const uint32_t b1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
                    const uint32_t b2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
                    auto keep = [n](uint32_t word, uint32_t first) -> uint32_t {  // bytes [first, n) of 4
                        const uint32_t c = n > first ? min(n - first, 4u) : 0u;
                        return c >= 4 ? word : word & ((1u << (8 * c)) - 1u);
                    };
                    *reinterpret_cast<ov4 *>(out + 16ull * i) =
                        mk4(n, inl ? keep(b0, 0) : b0, inl ? keep(b1, 4) : (uint32_t)p, inl ? keep(b2, 8) : (uint32_t)(p >> 32));
                }
            }
            if (n_ok > 0) str_base += rl(rel1, n_ok - 1);
            next_str += n_ok;
            if (n_ok < 64) break;
        }
    };
    // stream complete 16 B blocks below `upto` (16-aligned) to the heap
    auto flush = [&](uint32_t upto) {
        // (a ring never holds more than kRing bytes: the clamp bounds the
        // loop whatever a corrupt stream did to the positions)
        const uint32_t nblk = (V & kFsstAblateFlush) ? 0u : min((upto - ring_base) >> 4, Layout::kRing / 16);
        for (uint32_t q = lane; q < nblk; q += 64) {
            const uint32_t g = ring_base + 16 * q;
            const uint32_t slot = kCirc ? (g >> 4) & (kCirc / 16 - 1) : q;
            const v4u b = reinterpret_cast<const lv4 *>(w.ring)[slot];
            if constexpr ((V & kFsstZeroFlush) != 0) reinterpret_cast<lv4 *>(w.ring)[slot] = mk4(0, 0, 0, 0);
            if (g + 16 <= hlim) *reinterpret_cast<ov4 *>(vheap + g) = b;
            else bad = true;
        }
    };

    // ---- 2-4. code-parallel rounds -----------------------------------------
    constexpr uint32_t kRound = Layout::kRound;
    // a lane's compressed bytes of the round starting at r0 (zeros past the end)
    auto load_raw = [&](uint32_t r0) -> v4u {
        const uint32_t idx0 = r0 + BPL * lane;
        v4u x = mk4(0, 0, 0, 0);
        if (idx0 < comp_len) {
            if constexpr (BPL == 16) {
                x = comp[(r0 >> 4) + lane];
            } else {  // 8 B per lane: one dwordx2 load (the stream is 16 B aligned)
                const v2u h = reinterpret_cast<const FLS_GLOBAL v2u *>(comp)[(r0 >> 3) + lane];
                x = mk4(h.x, h.y, 0, 0);
            }
        }
        return x;
    };
    // string_t records of the strings decoded so far, complete 16 B blocks of
    // the ring to the heap, the unfinished tail (< 32 B) to the ring start
    // segmented kernel's flush: up to 4 blocks per lane per pass, all ring
    // reads in flight before the zeroing and the heap stores
    // (kFsstSegLazy: blocks [flushed, upto), which lie from ring slot
    // (flushed - ring_base) / 16 on)
    uint32_t flushed = 0;
    auto flush_seg = [&](uint32_t upto) {
        constexpr bool kLazy = (V & kFsstSegLazy) != 0;
        const uint32_t from = kLazy ? flushed : ring_base;
        const uint32_t q_off = (from - ring_base) >> 4;
        const uint32_t nblk = (V & kFsstAblateFlush) ? 0u : min((upto - from) >> 4, Layout::kRing / 16 - min(q_off, Layout::kRing / 16));
        lv4 *r16 = reinterpret_cast<lv4 *>(w.ring) + (kLazy ? q_off : 0u);
        if constexpr (kLazy) flushed = max(flushed, upto);
        for (uint32_t q0 = 0; q0 < nblk; q0 += 256) {
            v4u b[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t q = q0 + 64 * j + lane;
                b[j] = q < nblk ? r16[q] : mk4(0, 0, 0, 0);
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t q = q0 + 64 * j + lane;
                if (q < nblk) {
                    r16[q] = mk4(0, 0, 0, 0);
                    const uint32_t g = from + 16 * q;
                    if (g + 16 <= hlim) *reinterpret_cast<ov4 *>(vheap + g) = b[j];
                    else bad = true;
                }
            }
        }
    };
    // segmented kernel: the kept tail (an unfinished batch of strings, up to
    // a few KB) moves to the ring start 1 KB at a time, the bytes it vacates
    // back to zero
    auto retire_seg = [&](bool force, bool compact = true) {
        finalize_seg(force);
        const uint32_t keep_from = next_str < nvals ? min(str_base, out_pos) : out_pos;
        const uint32_t new_base = keep_from & ~15u;
        flush_seg(new_base);
        wave_sync();
        if (!compact) return;   // kFsstSegLazy: the tail stays where it is
        const uint32_t src = min(new_base - ring_base, Layout::kRing);
        const uint32_t len = min((out_pos - new_base + 15) & ~15u, Layout::kRing - 16);
        lv4 *r16 = reinterpret_cast<lv4 *>(w.ring);
        if (src > 0) {
            for (uint32_t o = 0; o < len; o += 1024) {
                const uint32_t k = (o >> 4) + lane;
                v4u t = mk4(0, 0, 0, 0);
                if (16 * k < len) t = r16[(src >> 4) + k];
                wave_sync();
                if (16 * k < len) r16[k] = t;
                wave_sync();
            }
            // vacated: [max(src, len), src + len)
            for (uint32_t b = max(src, len) + 16 * lane; b < src + len; b += 1024) r16[b >> 4] = mk4(0, 0, 0, 0);
        }
        ring_base = new_base;
        wave_sync();
    };
    auto retire = [&]() {
        finalize();
        const uint32_t keep_from = next_str < nvals ? min(str_base, out_pos) : out_pos;
        const uint32_t new_base = keep_from & ~15u;
        flush(new_base);
        wave_sync();
        if constexpr (kCirc != 0) {  // the tail stays where it is
            ring_base = new_base;
            return;
        }
        const uint32_t src = (new_base - ring_base) >> 2;
        uint32_t t = 0;
        if (lane < 8) t = reinterpret_cast<const lu32 *>(w.ring)[src + lane];
        wave_sync();
        if (lane < 8) reinterpret_cast<lu32 *>(w.ring)[lane] = t;
        if constexpr ((V & kFsstZeroFlush) != 0) {  // the vacated tail bytes back to zero
            if (lane < 8 && src + lane >= 8) reinterpret_cast<lu32 *>(w.ring)[src + lane] = 0;
        }
        ring_base = new_base;
        wave_sync();
    };
    if constexpr (SEG) {
        // ---- segmented rounds: lane l decodes segment 64r + l (16 codes) at
        // the ring offset the segment table gives, from the escape state it
        // gives: no gathered lengths to scan first, no entry-state hand-off
        const uint32_t soff = sizeof(FsstVecHeader) + 128 * clen_w + ((comp_len + 15) & ~15u);
        const FLS_GLOBAL FsstSegHeader *shp = reinterpret_cast<const FLS_GLOBAL FsstSegHeader *>(vh + soff);
        const uint32_t nseg = (comp_len + kFsstSegCodes - 1) / kFsstSegCodes;
        const bool vec_esc = (uni(shp->flags) & FSST_SEG_HAS_ESCAPE) != 0;
        if (uni(shp->nseg) != nseg) bad = true;
        gu8 *segv = vh + soff + sizeof(FsstSegHeader);
        // NS consecutive segments per lane (kFsstSegDouble: 2, a round of
        // 2048 codes, so the per-round work is spread over twice the codes)
        constexpr uint32_t NS = (V & kFsstSegDouble) ? 2 : 1;
        constexpr uint32_t kRoundSeg = 64 * 16 * NS;
        const uint32_t n16 = (comp_len + 15) >> 4;
        auto load_seg = [&](uint32_t r0, uint32_t j) -> uint32_t {
            const uint32_t k = (r0 >> 4) + NS * lane + j;
            return k < nseg ? (uint32_t)segv[k] : 0u;
        };
        auto load_codes = [&](uint32_t r0, uint32_t j) -> v4u {
            const uint32_t k = (r0 >> 4) + NS * lane + j;
            return k < n16 ? comp[k] : mk4(0, 0, 0, 0);
        };
        v4u raw_next[NS];
        uint32_t sv_next[NS];
#pragma unroll
        for (uint32_t j = 0; j < NS; ++j) {
            raw_next[j] = load_codes(0, j);
            sv_next[j] = load_seg(0, j);
        }
        constexpr int WR = (V & kFsstAblateWrite) ? 3 : (V & kFsstTwoQ) ? 1 : (V & kFsstSegLean) ? 4 : (V & kFsstSegSparse) ? 2 : 0;
        static_assert(WR != 4 || !(V & kFsstSegDouble), "the lean writer counts one segment");
        constexpr bool PL = (V & kFsstSegPackedLen) != 0;
        constexpr uint32_t FB = (V & kFsstSegWide) ? 16 : 8;
        for (uint32_t r0 = 0; r0 < comp_len; r0 += kRoundSeg) {
            const uint32_t idx0 = r0 + 16 * NS * lane;
            v4u raw[NS];
            uint32_t dlj[NS], entj[NS], dl = 0;
#pragma unroll
            for (uint32_t j = 0; j < NS; ++j) {
                raw[j] = raw_next[j];
                entj[j] = sv_next[j] > 128 ? 1u : 0u;
                dlj[j] = entj[j] ? sv_next[j] - 129 : sv_next[j];
                dl += dlj[j];
            }
            if (r0 + kRoundSeg < comp_len) {
#pragma unroll
                for (uint32_t j = 0; j < NS; ++j) {
                    raw_next[j] = load_codes(r0 + kRoundSeg, j);
                    sv_next[j] = load_seg(r0 + kRoundSeg, j);
                }
            }
            const bool full = r0 + kRoundSeg <= comp_len;
            // the previous round's stores, after this round's loads
            // (kFsstSegLazy: the tail moves only once the ring is half full)
            if (r0 > 0) retire_seg(false, !(V & kFsstSegLazy) || out_pos - ring_base > Layout::kSegCap / 2);
            const uint32_t entry = entj[0];
            const uint32_t incl = scan_incl(dl, lane);
            uint32_t st = entry, l0 = 0, done = 0, guard = 0;
            for (;;) {  // the lanes whose output fits the ring, then the rest
                if (++guard > 130) {  // at most 64 parts + 64 retires: a corrupt table
                    bad = true;
                    break;
                }
                const uint32_t p0 = out_pos - ring_base;
                const bool fits = lane < l0 || p0 + (incl - done) <= Layout::kSegCap;
                const uint64_t fm = __ballot(fits);
                const uint32_t l1 = ~fm == 0 ? 64u : (uint32_t)__builtin_ctzll(~fm);
                if (l1 == l0) {  // nothing fits beside the kept tail: retire it first
                    retire_seg(true);
                    continue;    // then the tail is < 32 B and lane l0 (<= 256 B) fits
                }
                const uint32_t part = rl(incl, l1 - 1) - done;
                wave_sync();
                if (lane >= l0 && lane < l1) {
                    SegWriter<WR> qw(w.ring, p0 + (incl - dl - done));
#pragma unroll
                    for (uint32_t j = 0; j < NS; ++j) {
                        if (j > 0 && st != entj[j]) bad = true;   // the state between a lane's segments
                        st = entj[j];
                        const uint32_t e0 = idx0 + 16 * j;
                        const uint32_t nb = e0 < comp_len ? min(comp_len - e0, 16u) : 0u;
                        const uint32_t got = !full   ? seg_lane<false, true, WR, PL>(w, raw[j], nb, st, qw)
                                             : vec_esc ? seg_lane<true, true, WR, PL>(w, raw[j], nb, st, qw)
                                                       : seg_lane<true, false, WR, PL, FB>(w, raw[j], nb, st, qw);
                        if (got != dlj[j]) bad = true;
                    }
                    qw.finish();
                }
                wave_sync();
                out_pos += part;
                done += part;
                if (l1 == 64) break;
                retire_seg(true);
                l0 = l1;
            }
            // a lane's exit state is the entry state of the segment after it
            const uint32_t nxt = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane + 1) & 63) << 2), (int)entry);
            if (lane < 63 && idx0 + 16 * NS < comp_len && st != nxt) bad = true;
            if (lane == 0 && entry != carry_lit) bad = true;
            carry_lit = rl(st, min(63u, (comp_len - 1 - r0) / (16 * NS)));
        }
    } else {
    v4u raw_next = load_raw(0);
    for (uint32_t r0 = 0; r0 < comp_len; r0 += kRound) {
        const uint32_t idx0 = r0 + BPL * lane;
        const uint32_t nb = idx0 < comp_len ? min(comp_len - idx0, (uint32_t)BPL) : 0u;
        const v4u raw = raw_next;  // the next round's bytes load while this one decodes
        if (r0 + kRound < comp_len) raw_next = load_raw(r0 + kRound);
        const bool full = r0 + kRound <= comp_len;
        Gathered<BPL> pre;
        if constexpr ((V & kFsstEarlyGather) != 0) {
            if (full) gather_codes<BPL>(w, raw, pre);
        }
        // the previous round's stores go out now, after this round's load was
        // issued and a whole decode before the next wait (vmcnt counts loads
        // and stores in issue order, and the variable store count makes that
        // wait a vmcnt(0): issued at the end of their own round, the stores'
        // latency was exposed every round)
        if (r0 > 0) retire();
        uint32_t n[BPL], lane_end = 0;
        uint64_t v[BPL];
        bool plain = false;
        if constexpr ((V & kFsstPlain) != 0) plain = full && carry_lit == 0 && __ballot(has_escape<BPL>(raw)) == 0;
        const uint32_t lane_out = plain  ? lane_codes_plain<BPL>(w, raw, v, n)
                                  : full ? ((V & kFsstLenFromSym) && table_lfs
                                                ? lane_codes<BPL, true, (V & kFsstLenFromSym) != 0>(w, raw, nb, carry_lit,
                                                                                                    lane, v, n, lane_end)
                                                : lane_codes<BPL, true>(w, raw, nb, carry_lit, lane, v, n, lane_end,
                                                                        (V & kFsstEarlyGather) ? &pre : nullptr))
                                         : lane_codes<BPL, false>(w, raw, nb, carry_lit, lane, v, n, lane_end);
        const uint32_t incl = scan_incl(lane_out, lane);
        // write the round into the ring: normally all 64 lanes at once; when
        // their output would overrun the ring, the lanes that fit first, then
        // retire() to empty the ring and continue (a lane writes <= 8 BPL bytes)
        // slack: qword ORs, retire()'s 32 B tail read (circular: the bytes
        // from ring_base to the round's end must not wrap onto ring_base)
        constexpr uint32_t kCap = kCirc ? kCirc - 16 : Layout::kRingPlain - 48;
        uint32_t l0 = 0, done = 0;
        for (;;) {
            const uint32_t p0 = out_pos - ring_base;
            const bool fits = lane < l0 || p0 + (incl - done) <= kCap;
            const uint64_t fm = __ballot(fits);
            const uint32_t l1 = ~fm == 0 ? 64u : (uint32_t)__builtin_ctzll(~fm);
            const uint32_t part = rl(incl, l1 - 1) - done;
            // zero the ring dwords these lanes OR into, keeping the already
            // decoded bytes below out_pos in the first one
            if constexpr ((V & kFsstZeroFlush) == 0) {
                FLS_LDS uint32_t *r32 = reinterpret_cast<FLS_LDS uint32_t *>(w.ring);
                const uint32_t z0 = (p0 + 3) >> 2, z1 = ((p0 + part + 7) & ~7u) >> 2;
                for (uint32_t q = z0 + lane; q < z1; q += 64) r32[q] = 0;
                if (lane == 0 && (p0 & 3)) r32[p0 >> 2] &= (1u << (8 * (p0 & 3))) - 1u;
            }
            wave_sync();
            if (lane >= l0 && lane < l1) {
                const uint32_t wp = (kCirc ? out_pos : p0) + (incl - lane_out - done);
                if constexpr ((V & kFsstTwoQ) != 0) {
                    // every symbol OR-ed into both qwords it spans: the shift
                    // counts are taken mod 64 by the hardware (8 * p mod 64 is
                    // the bit offset inside qword p / 8; ~(8p) mod 64 = 63 - it)
                    FLS_LDS uint64_t *o64 = reinterpret_cast<FLS_LDS uint64_t *>(w.ring);
                    uint32_t p = wp;
#pragma unroll
                    for (uint32_t k = 0; k < BPL; ++k) {
                        const uint32_t b8 = p << 3;
                        const uint64_t lo = v[k] << (b8 & 63), hi = (v[k] >> 1) >> (~b8 & 63);
                        __hip_atomic_fetch_or(o64 + (p >> 3), lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        __hip_atomic_fetch_or(o64 + (p >> 3) + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        p += n[k];
                    }
                } else {
                    QwordWriter<kCirc ? kCirc / 8 - 1 : ~0u> qw(w.ring, wp);
#pragma unroll
                    for (uint32_t k = 0; k < BPL; ++k) qw.put(v[k], n[k]);
                    qw.finish();
                }
            }
            wave_sync();
            out_pos += part;
            done += part;
            if (l1 == 64) break;
            retire();
            l0 = l1;
        }
        // state after the round's last valid byte (lane 63 unless the stream ends here)
        carry_lit = rl(lane_end, min(63u, (comp_len - 1 - r0) / BPL));
    }
    }  // SEG
    if (carry_lit) bad = true;  // stream ends inside an escape
    if constexpr (SEG) retire_seg(true);
    else retire();
    if (next_str < nvals) {     // lengths claim more bytes than the stream holds
        bad = true;
        for (uint32_t i = next_str + lane; i < nvals; i += 64)
            *reinterpret_cast<ov4 *>(out + 16ull * i) = mk4(0, 0, 0, 0);
    }
    // zero the padding of the last block, then flush everything
    const uint32_t end = (out_pos + 15) & ~15u;
    if (lane < 16 && out_pos + lane < end) w.ring[kCirc ? (out_pos + lane) & (kCirc - 1) : out_pos - ring_base + lane] = 0;
    wave_sync();
    flush(end);
    if (bad) atomicOr(err, KERR_FSST);
}

__device__ __forceinline__ DevChunk load_chunk(const DevChunk *chunks, uint32_t ci) {
    const FLS_GLOBAL v4u *q = reinterpret_cast<const FLS_GLOBAL v4u *>(gptr(chunks + ci));
    // wave-uniform: the descriptor lives in SGPRs, not in 16 VGPRs
    DevChunk c;
    uint32_t *d = reinterpret_cast<uint32_t *>(&c);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const v4u x = q[k];
        d[4 * k] = uni(x.x);
        d[4 * k + 1] = uni(x.y);
        d[4 * k + 2] = uni(x.z);
        d[4 * k + 3] = uni(x.w);
    }
    return c;
}

// The wave's vectors (items numbered chunk by chunk through DevChunk.vec_base):
// without a queue the contiguous range [item0, item1); with one, pieces of
// `piece` consecutive items taken from the shared counter until it runs out
// (a wave's pieces come in increasing order, so its chunk cursor only moves
// forward).  The wave loads a chunk's symbol table once per stay in it.
template <int BPL, bool SMALL, bool QUEUE, int V, int SEG = 0>
__device__ __forceinline__ void fsst_range(const DevChunk *chunks_generic, uint32_t nchunks, uint32_t nitems,
                                           uint32_t item0, uint32_t item1, uint32_t *queue, uint32_t piece, lu8 *L,
                                           uint32_t *err_generic) {
    const uint64_t cp = (uint64_t)chunks_generic;
    const DevChunk *chunks = (const DevChunk *)((uint64_t)uni((uint32_t)(cp >> 32)) << 32 | uni((uint32_t)cp));
    const uint64_t ep = (uint64_t)err_generic;
    uint32_t *err = (uint32_t *)((uint64_t)uni((uint32_t)(ep >> 32)) << 32 | uni((uint32_t)ep));
    nchunks = uni(nchunks);
    const uint32_t lane = __lane_id();
    // next piece of the queue into [item0, item1); false when none is left
    // (every wave reaches that exit)
    auto take = [&]() -> bool {
        uint32_t p = 0;
        if (lane == 0) p = atomicAdd(queue, 1u);
        p = rl(p, 0);
        if (p >= (nitems + piece - 1) / piece) return false;
        item0 = p * piece;
        item1 = min(item0 + piece, nitems);
        return true;
    };
    if constexpr (QUEUE) {
        if (!take()) return;
    }
    item0 = uni(item0);
    item1 = uni(item1);
    constexpr bool D8 = SMALL && SEG && (V & kFsstSegD8) != 0;
    using Layout = Lds<BPL, SMALL, SEG, D8>;
    Wave w;
    w.P = reinterpret_cast<lv4 *>(L + Layout::kOffRing);
    w.D = reinterpret_cast<lu32 *>(L + Layout::kOffD);
    w.sym = reinterpret_cast<const FLS_LDS uint64_t *>(L + Layout::kOffSym);
    w.len = L + Layout::kOffLen;
    w.ring = L + Layout::kOffRing;
    // chunk holding item0: last ci with vec_base <= item0
    uint32_t lo = 0, hi = nchunks;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (uni(gptr(chunks + mid)->vec_base) <= item0) lo = mid;
        else hi = mid;
    }
    uint32_t ci = lo;
    DevChunk c = load_chunk(chunks, ci);
    bool have_table = false;
    bool table_lfs = false;  // kFsstLenFromSym: every symbol's last byte is non-zero
    for (uint32_t item = item0;;) {
        if (item >= item1) {
            if constexpr (!QUEUE) break;
            if (!take()) break;
            item = item0;
        }
        const uint32_t v = item - uni(c.vec_base);
        if (v >= uni(c.nvec)) {  // next chunk
            if (++ci >= nchunks) break;
            c = load_chunk(chunks, ci);
            have_table = false;
            continue;
        }
        gu8 *chunk = gptr(c.chunk);
        gu8 *aux = chunk + c.aux_off;
        if (!have_table) {
            // symbol table, sanitised: each symbol masked to its length (so
            // OR-ing whole symbols is exact), the escape code's entry {0, 0}
            wave_sync();
            const FLS_GLOBAL uint64_t *gs = reinterpret_cast<const FLS_GLOBAL uint64_t *>(aux);
            FLS_LDS uint64_t *ls = reinterpret_cast<FLS_LDS uint64_t *>(L + Layout::kOffSym);
            bool zero_last = false, long8 = false;
            for (uint32_t k = lane; k < 256; k += 64) {
                const uint32_t n = k == kFsstEscape ? 0u : min((uint32_t)aux[8 * 256 + k], 8u);
                const uint64_t sy = n >= 8 ? gs[k] : gs[k] & ((1ull << (8 * n)) - 1);
                // kFsstSegPackedLen: the length rides in the top byte (the
                // host sends only tables of symbols <= 7 bytes)
                // (kFsstSegLean: 8 x the length, the bit count)
                ls[k] = (SEG && (V & kFsstSegPackedLen)) ? sy | (uint64_t)((V & kFsstSegLean) ? 8 * n : n) << 56 : sy;
                if constexpr (!D8) L[Layout::kOffLen + k] = (uint8_t)n;
                zero_last |= n > 0 && ((sy >> (8 * (n - 1))) & 0xFF) == 0;
                long8 |= n >= 8;
            }
            table_lfs = __ballot(zero_last) == 0;
            if (SEG && (V & kFsstSegPackedLen) && __ballot(long8) != 0 && lane == 0) atomicOr(err, KERR_BAD_DESC);
            wave_sync();
            have_table = true;
        }
        const FLS_GLOBAL VecMeta *meta = reinterpret_cast<const FLS_GLOBAL VecMeta *>(chunk + c.meta_off) + v;
        const uint32_t poff = uni((uint32_t)meta->packed_off);
        const uint32_t base = uni((uint32_t)meta->for_base);
        const uint32_t aoff = uni((uint32_t)meta->aux_off);
        const uint32_t nvals = uni(meta->nvals);
        const uint32_t W = uni(min((uint32_t)meta->bw, 32u));
        const uint32_t dbytes = uni(meta->aux_count);
        fsst_vector<BPL, SMALL, V, SEG>(w, chunk + c.packed_off + poff, W, base, nvals, dbytes, aux + aoff,
                    (FLS_GLOBAL uint8_t *)(size_t)c.dict, c.heap_bytes, c.heap_host,
                    gptr(c.out) + 16ull * kVectorSize * v, lane, err, table_lfs);
        wave_sync();
        ++item;
    }
}

// Work distribution.  Standalone launches: contiguous vector ranges per wave
// (a wave mostly stays inside one chunk and stages its symbol table once).
// Overlapped launches (queue != nullptr, FsstLaunch::overlap): pieces of
// `piece` consecutive vectors from a counter shared by the narrow grid that
// runs beside the main decode kernel and the full grid that follows it, one
// atomic per piece, so no vector is decoded twice and late waves find work.
// (A piece queue for standalone launches measured 2-4 % slower on l_comment
// at SF10: more symbol-table reloads.)  The piece loop is the range loop's
// own (a loop around the range decoder needed 98-124 VGPRs instead of 82).
#ifndef FLS_FSST_WAVES
#define FLS_FSST_WAVES 4  // minimum waves per SIMD the register budget must allow
#endif
#ifndef FLS_FSST_SEG_WAVES
#define FLS_FSST_SEG_WAVES 5  // the segmented kernel: 96 VGPRs, no spill (its LDS admits about 5 waves per SIMD)
#endif
template <int BPL, bool SMALL, bool QUEUE, int V, int SEG = 0>
__global__ __launch_bounds__(64, SEG ? (((V & kFsstSegDouble) || (V & kFsstSegW4)) ? 4 : FLS_FSST_SEG_WAVES) : (V & kFsstW6) ? 6 : FLS_FSST_WAVES) void fsst_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                     uint32_t nitems, uint32_t *__restrict__ err,
                                                     uint32_t *__restrict__ queue, uint32_t piece) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw_generic[];
    // an LDS-typed pointer to the dynamic LDS (a known constant address, so
    // table and ring offsets fold into the DS instructions' offset fields)
    // kFsstAbsLds: the same addresses as plain integers (the kernel has no
    // static LDS, so its dynamic LDS starts at address 0; checked), which lets
    // the compiler fold table and ring offsets without adding a symbol base
    if constexpr ((V & kFsstAbsLds) != 0) {
        if ((uint32_t)(size_t)lds_raw_generic != 0u) {
            if (threadIdx.x == 0) atomicOr(err, KERR_LDS_BASE);
            return;
        }
    }
    lu8 *lds_raw = (V & kFsstAbsLds) ? (lu8 *)(size_t)0 : (lu8 *)lds_raw_generic;
    uint32_t i0 = 0, i1 = 0;
    if (!QUEUE) {
        const uint32_t nwaves = gridDim.x, wave = blockIdx.x;
        const uint32_t per = (nitems + nwaves - 1) / nwaves;
        i0 = min(wave * per, nitems);
        i1 = min(i0 + per, nitems);
        if (i0 >= i1) return;
    }
    fsst_range<BPL, SMALL, QUEUE, V, SEG>(chunks, nchunks, nitems, i0, i1, queue, piece, lds_raw, err);
}

template <int BPL, bool SMALL, bool QUEUE, int V, int SEG = 0>
hipError_t launch_fsst_q(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                         hipStream_t stream, const FsstLaunch &how) {
    const uint32_t shmem = Lds<BPL, SMALL, SEG, SMALL && SEG && (V & kFsstSegD8) != 0>::kWave;
    if constexpr ((V & kFsstAbsLds) != 0) {
        // the variant addresses its dynamic LDS from 0, which holds only for a
        // kernel without static LDS: refuse to launch one that has some
        static const bool lds_at_zero = [] {
            hipFuncAttributes a{};
            return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(fsst_kernel<BPL, SMALL, QUEUE, V, SEG>)) ==
                       hipSuccess &&
                   a.sharedSizeBytes == 0;
        }();
        if (!lds_at_zero) {
            fprintf(stderr, "fsst_kernel<%d,%d,%d,%d,%d>: static LDS present or attributes unavailable; the "
                            "kFsstAbsLds variant cannot run\n", BPL, (int)SMALL, (int)QUEUE, V, SEG);
            return hipErrorInvalidDeviceFunction;
        }
    }
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fsst_kernel<BPL, SMALL, QUEUE, V, SEG>, 64, shmem) !=
            hipSuccess)
            per_cu = 1;
    }
    if (how.grid_cus > 0) cus = std::min(cus, how.grid_cus);   // a CU-masked stream
    const int full = cus * std::max(1, per_cu);
    int wpc = how.waves_per_cu;
    if (const char *e = getenv("FLS_FSST_WPC"); e && wpc == 0) wpc = std::max(0, atoi(e));  // A/B knob (standalone launches)
    const int grid = std::min<int>(wpc > 0 ? cus * std::min(wpc, per_cu) : full, (int)nvecs);
    // overlapped: pieces of ~1/4 of a wave's share of a full grid, <= 16 vectors
    uint32_t piece = std::max<uint32_t>(1, std::min<uint32_t>(16, nvecs / (4u * (uint32_t)full)));
    if (const char *e = getenv("FLS_FSST_PIECE")) piece = (uint32_t)std::max(1, std::min(64, atoi(e)));  // A/B knob
    if (how.queue && how.reset_queue) {
        const hipError_t e = hipMemsetAsync(how.queue, 0, sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
    }
    if (getenv("FLS_DEBUG"))
        fprintf(stderr, "DEBUG: fsst_kernel<%d,%s%s>: variant %d, %d blocks of 1 wave (%d per CU, %u B LDS), %u vectors%s\n",
                BPL, SMALL ? "small" : "any", SEG ? ",seg" : "", V, grid, per_cu, shmem, nvecs,
                how.queue ? " (piece queue)" : "");
    hipLaunchKernelGGL((fsst_kernel<BPL, SMALL, QUEUE, V, SEG>), dim3(grid), dim3(64), shmem, stream, d_chunks, nchunks, nvecs,
                       d_err, how.queue, piece);
    return hipGetLastError();
}
template <int BPL, bool SMALL, int V>
hipError_t launch_fsst_v(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                         hipStream_t stream, const FsstLaunch &how) {
    return how.queue ? launch_fsst_q<BPL, SMALL, true, V>(d_chunks, nchunks, nvecs, d_err, stream, how)
                     : launch_fsst_q<BPL, SMALL, false, V>(d_chunks, nchunks, nvecs, d_err, stream, how);
}
// code-parallel variants (FsstLaunch::variant, FLS_FSST_VARIANT): BPL = 8
// instantiates the ones A/B-measured (profiles/r2/abenv_fsst_var*.txt),
// BPL = 16 only the default
template <int BPL, bool SMALL>
hipError_t launch_fsst_t(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                         hipStream_t stream, const FsstLaunch &how) {
    if constexpr (BPL == 8) {
        switch (how.variant & 255) {
        case 0: return launch_fsst_v<BPL, SMALL, 0>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstPlain: return launch_fsst_v<BPL, SMALL, kFsstPlain>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstTwoQ: return launch_fsst_v<BPL, SMALL, kFsstTwoQ>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstW6 | kFsstTwoQ:
            return launch_fsst_v<BPL, SMALL, kFsstW6 | kFsstTwoQ>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstW6: return launch_fsst_v<BPL, SMALL, kFsstW6>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstZeroFlush:
            return launch_fsst_v<BPL, SMALL, kFsstZeroFlush>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstW6 | kFsstZeroFlush:
            return launch_fsst_v<BPL, SMALL, kFsstW6 | kFsstZeroFlush>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstZeroFlush | kFsstAbsLds | kFsstEarlyGather:
            return launch_fsst_v<BPL, SMALL, kFsstZeroFlush | kFsstAbsLds | kFsstEarlyGather>(d_chunks, nchunks, nvecs,
                                                                                            d_err, stream, how);
        case kFsstDefault | kFsstEarlyGather:
            return launch_fsst_v<BPL, SMALL, kFsstDefault | kFsstEarlyGather>(d_chunks, nchunks, nvecs, d_err, stream,
                                                                            how);
        case kFsstW6 | kFsstZeroFlush | kFsstLenFromSym:
            return launch_fsst_v<BPL, SMALL, kFsstW6 | kFsstZeroFlush | kFsstLenFromSym>(d_chunks, nchunks, nvecs,
                                                                                       d_err, stream, how);
        case kFsstW6 | kFsstZeroFlush | kFsstCirc:
            return launch_fsst_v<BPL, SMALL, kFsstW6 | kFsstZeroFlush | kFsstCirc>(d_chunks, nchunks, nvecs, d_err,
                                                                                 stream, how);
        default:
            return launch_fsst_v<BPL, SMALL, kFsstDefault>(d_chunks, nchunks, nvecs, d_err, stream, how);
        }
    }
    return launch_fsst_v<BPL, SMALL, kFsstDefault>(d_chunks, nchunks, nvecs, d_err, stream, how);
}

// ============================================================================
// String-parallel path (chunks whose strings are all <= 255 bytes, both
// decompressed and compressed: the host marks them, DevChunk.vbits = 1).
// Every string is compressed on its own and the vector stores the strings'
// compressed lengths, so lane j decodes string s + j of a round by itself: no
// escape-state composition, no per-code wave scans.  Per vector:
//   1. both length streams (FFOR, W <= 8) are unpacked into u8 arrays;
//   2. rounds of up to 64 strings (as many as fit the LDS rings: inclusive
//      wave scans of the lengths + ballot): the round's compressed bytes are
//      staged into the IN ring with 16 B coalesced loads, the OUT ring's
//      dwords for the round are zeroed, then every lane walks its string 4
//      codes at a time (one unaligned dword of codes, the 4 symbol / length
//      lookups issued together) and ORs the symbols into OUT as aligned
//      dwords (a string's edge dwords are shared with its neighbours);
//   3. the round's string_t records (64 x 16 B) and the complete 16 B blocks
//      of OUT go to HBM; the unfinished tail (< 16 B) moves to the ring start.
// Corrupt lengths (a string that expands to more or fewer bytes than its
// length, a truncated escape, streams that do not add up) are clamped to the
// string's own bytes and reported through KERR_FSST.
constexpr uint32_t kSpIncap = 1536;   // IN ring: compressed bytes of a round (+16 B slack)
constexpr uint32_t kSpOutcap = 2560;  // OUT ring: decoded bytes of a round incl. the carried tail
constexpr uint32_t kSpSym = 0, kSpLen = 2048, kSpDL = 2304, kSpCL = kSpDL + 1024, kSpIn = kSpCL + 1024;
constexpr uint32_t kSpOut = kSpIn + kSpIncap + 16;
constexpr uint32_t kSpWave = kSpOut + kSpOutcap + 16;
static_assert(kSpIncap >= 128 * 8 + 128 && kSpIncap >= 255 + 16 && kSpOutcap >= 255 + 16, "SP ring sizes");
static_assert(kSpIn % 16 == 0 && kSpOut % 16 == 0 && kSpWave % 16 == 0, "SP LDS layout alignment");

struct SpWave {
    const FLS_LDS uint64_t *sym;
    const lu8 *len;
    lu8 *DL, *CL, *IN, *OUT;
};

// u8 lengths of the vector (base + FFOR(T=32, W <= 8), zero past nvals); the
// packed bits are staged in the IN ring
__device__ __forceinline__ void unpack_u8(const SpWave &w, gu8 *packed, uint32_t W, uint32_t base, uint32_t nvals,
                                          lu8 *dst, uint32_t lane) {
    lv4 *P = reinterpret_cast<lv4 *>(w.IN);
    const uint32_t n16 = 8 * W;
    gv4 *pk = reinterpret_cast<gv4 *>(packed);
    for (uint32_t i = lane; i < n16; i += 64) P[i] = pk[i];
    if (lane < 8) P[n16 + lane] = mk4(0, 0, 0, 0);
    wave_sync();
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t ci = lane + 64 * j;
        const v4u v = add_base<32>(unpack_chunk<32>(P, W, ci), base);
        const uint32_t b0 = 4 * ci < nvals ? v.x & 255 : 0, b1 = 4 * ci + 1 < nvals ? v.y & 255 : 0;
        const uint32_t b2 = 4 * ci + 2 < nvals ? v.z & 255 : 0, b3 = 4 * ci + 3 < nvals ? v.w & 255 : 0;
        reinterpret_cast<lu32 *>(dst)[ci] = b0 | b1 << 8 | b2 << 16 | b3 << 24;
    }
    wave_sync();
}

// Wave-64 maximum (DPP, like scan_incl), valid in every lane after readlane
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false));  // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false));  // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return rl(x, 63);
}

// The round's strings, one per lane: codes IN[cb, cb + cl) -> OUT[wp, wp + dl).
// Branch-free: the wave walks the round's longest compressed string (maxcl,
// uniform) 4 codes per step and every lane predicates its codes with
// selects, not branches (divergent control flow cost more scalar exec-mask
// instructions than the decode itself).  A lane assembles its bytes in a
// 64-bit accumulator and ORs them into the zeroed OUT ring as aligned qwords
// (a string's edge qwords are shared with its neighbours); the accumulator is
// OR-ed into its qword every step, full or not.  The symbol table is
// sanitised (symbols masked to their length, the escape code = {0, 0}).
// Returns false on corrupt input (wrong byte count, truncated escape).
__device__ __forceinline__ bool sp_decode(const SpWave &w, uint32_t cb, uint32_t cl, uint32_t wp, uint32_t dl,
                                          uint32_t maxcl) {
    const lu32 *in32 = reinterpret_cast<const lu32 *>(w.IN);
    FLS_LDS uint64_t *o64 = reinterpret_cast<FLS_LDS uint64_t *>(w.OUT);
    constexpr uint32_t kLastQ = (kSpOutcap + 16) / 8 - 1;
    const uint32_t ce = cb + cl;
    uint32_t q = wp >> 3, bits = 8 * (wp & 7), pos = 0;
    uint64_t acc = 0;
    bool lit = false;
    for (uint32_t it = 0; it < maxcl; it += 4) {
        const uint32_t c = cb + it;
        const uint32_t x = __builtin_amdgcn_alignbyte(in32[(c >> 2) + 1], in32[c >> 2], c & 3);
        const uint32_t nk = c < ce ? min(ce - c, 4u) : 0u;
        // codes past the string's end read as the escape code, whose table
        // entry is {0, 0} (and which then starts no literal)
        uint32_t b[4], sl[4];
        uint64_t sy[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            b[k] = k < nk ? (x >> (8 * k)) & 255 : kFsstEscape;
            sy[k] = w.sym[b[k]];
            sl[k] = w.len[b[k]];
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const bool l = lit;
            lit = k < nk && !l && b[k] == kFsstEscape;
            const uint64_t v = l ? (uint64_t)b[k] : sy[k];
            const uint32_t n = l ? 1u : sl[k];
            pos += n;
            // v << bits spans qwords q (lo) and q + 1 (hi); (v >> 1) >> (63 - bits)
            // is v >> (64 - bits) without the bits == 0 case
            const uint64_t lo = v << bits, hi = (v >> 1) >> (63 - bits);
            acc |= lo;
            // OR the accumulator every step (OR is idempotent): no select on
            // whether qword q is complete
            __hip_atomic_fetch_or(o64 + min(q, kLastQ), acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            const uint32_t nb = bits + 8 * n;
            const bool e = nb >= 64;
            q += e ? 1u : 0u;
            acc = e ? hi : acc;
            bits = nb & 63;
        }
    }
    __hip_atomic_fetch_or(o64 + min(q, kLastQ), acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    return !lit && pos == dl;
}

__device__ void fsst_vector_sp(const SpWave &w, gu8 *packed_vec, uint32_t W, uint32_t base, uint32_t nvals,
                               uint32_t dbytes, gu8 *vh, FLS_GLOBAL uint8_t *heap, uint32_t heap_bytes,
                               uint64_t heap_host, FLS_GLOBAL uint8_t *out, uint32_t lane, uint32_t *err) {
    const FLS_GLOBAL FsstVecHeader *hp = reinterpret_cast<const FLS_GLOBAL FsstVecHeader *>(vh);
    const uint32_t heap_off = uni(hp->heap_off), comp_len = uni(hp->comp_len);
    const uint32_t cbase = uni(hp->clen_base), cw = uni(min(hp->clen_w, 8u));
    bool bad = false;
    const uint32_t hlim = min((dbytes + 15) & ~15u, heap_bytes > heap_off ? heap_bytes - heap_off : 0u);
    FLS_GLOBAL uint8_t *vheap = heap + heap_off;
    const uint64_t ptr_base = heap_host + heap_off;
    gv4 *cs = reinterpret_cast<gv4 *>(vh + sizeof(FsstVecHeader) + 128 * cw);
    const uint32_t lim16 = (comp_len + 15) >> 4;
    lu32 *o32 = reinterpret_cast<lu32 *>(w.OUT);
    lv4 *in16 = reinterpret_cast<lv4 *>(w.IN);
    const lv4 *out16 = reinterpret_cast<const lv4 *>(w.OUT);
    // stream complete 16 B blocks [ring_base, upto) of OUT to the heap
    auto flush = [&](uint32_t ring_base, uint32_t upto) {
        const uint32_t nblk = (upto - ring_base) >> 4;
        for (uint32_t q = lane; q < nblk; q += 64) {
            const uint32_t g = ring_base + 16 * q;
            if (g + 16 <= hlim) *reinterpret_cast<ov4 *>(vheap + g) = out16[q];
            else bad = true;
        }
    };
    // ---- 2-3. rounds of up to 64 strings, one per lane ----------------------
    // The IN window of a round (kSpIncap bytes from the 16 B block holding its
    // first code) is loaded into registers one round ahead, so the round only
    // waits for loads issued before the previous round's decode.
    constexpr uint32_t kInBlocks = kSpIncap / 16;
    static_assert(kInBlocks > 64 && kInBlocks <= 128, "two 16 B prefetch loads per lane");
    v4u pf0 = mk4(0, 0, 0, 0), pf1 = mk4(0, 0, 0, 0);
    auto prefetch_in = [&](uint32_t from) {
        const uint32_t g = from >> 4;
        pf0 = g + lane < lim16 ? cs[g + lane] : mk4(0, 0, 0, 0);
        pf1 = lane + 64 < kInBlocks && g + lane + 64 < lim16 ? cs[g + lane + 64] : mk4(0, 0, 0, 0);
    };
    prefetch_in(0);
    // ---- 1. both length streams -> u8 arrays (the first window in flight) ---
    unpack_u8(w, packed_vec, min(W, 8u), base, nvals, w.DL, lane);
    unpack_u8(w, vh + sizeof(FsstVecHeader), cw, cbase, nvals, w.CL, lane);
    uint32_t s = 0, dpos = 0, cpos = 0, ring_base = 0;
    while (s < nvals) {
        const uint32_t i = s + lane;
        const uint32_t dl = i < nvals ? (uint32_t)w.DL[i] : 0u, cl = i < nvals ? (uint32_t)w.CL[i] : 0u;
        const uint32_t dinc = scan_incl(dl, lane), cinc = scan_incl(cl, lane);
        const uint32_t tail = dpos - ring_base, cskew = cpos & 15;
        const bool fits = i < nvals && tail + dinc <= kSpOutcap && cskew + cinc <= kSpIncap;
        const uint64_t m = __ballot(fits);
        const uint32_t nr = ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m);  // >= 1: one string always fits
        const uint32_t rd = rl(dinc, nr - 1), rc = rl(cinc, nr - 1);
        // stage the round's compressed bytes (prefetched window), then start
        // loading the next round's window
        in16[lane] = pf0;
        if (lane + 64 < kInBlocks) in16[lane + 64] = pf1;
        prefetch_in(cpos + rc);
        // zero the OUT dwords the round ORs into, keeping the carried tail bytes
        {
            const uint32_t z0 = (tail + 3) >> 2, z1 = (tail + rd + 3) >> 2;
            for (uint32_t q = z0 + lane; q < z1; q += 64) o32[q] = 0;
            if (lane == 0 && (tail & 3)) o32[tail >> 2] &= (1u << (8 * (tail & 3))) - 1u;
        }
        wave_sync();
        const uint32_t wp = tail + dinc - dl;
        {
            const bool act = lane < nr;
            const uint32_t acl = act ? cl : 0u;
            const uint32_t maxcl = wave_max(acl);
            if (!sp_decode(w, act ? cskew + cinc - cl : 0u, acl, act ? wp : 0u, act ? dl : 0u, maxcl)) bad = true;
        }
        wave_sync();
        // string_t records of the round's strings (64 x 16 B = one 1 KiB store)
        if (lane < nr)
            *reinterpret_cast<ov4 *>(out + 16ull * i) = make_record_at(w.OUT, wp, dl, ptr_base + (dpos + dinc - dl));
        const uint32_t new_base = (dpos + rd) & ~15u;
        flush(ring_base, new_base);
        wave_sync();
        // move the unfinished tail (< 16 B) to the ring start
        const uint32_t src = (new_base - ring_base) >> 2;
        uint32_t t = 0;
        if (lane < 4) t = o32[src + lane];
        wave_sync();
        if (lane < 4) o32[lane] = t;
        wave_sync();
        dpos += rd;
        cpos += rc;
        s += nr;
        ring_base = new_base;
    }
    if (dpos != dbytes || cpos != comp_len) bad = true;
    // zero the padding of the last block, then flush it
    const uint32_t end = (dpos + 15) & ~15u;
    if (lane < 16 && dpos + lane < end) w.OUT[dpos - ring_base + lane] = 0;
    wave_sync();
    flush(ring_base, end);
    if (bad) atomicOr(err, KERR_FSST);
}

// Vectors [item0, item1) of the launch's string-parallel chunks (numbered
// through DevChunk.vec_base); a chunk's symbol table is staged once, each
// symbol masked to its length (so OR-ing whole symbols is exact) and the
// escape code's entry emptied.
__device__ __forceinline__ void fsst_sp_range(const DevChunk *chunks, uint32_t nchunks, uint32_t item0, uint32_t item1,
                                              lu8 *L, uint32_t *err) {
    const uint32_t lane = __lane_id();
    SpWave w;
    w.sym = reinterpret_cast<const FLS_LDS uint64_t *>(L + kSpSym);
    w.len = L + kSpLen;
    w.DL = L + kSpDL;
    w.CL = L + kSpCL;
    w.IN = L + kSpIn;
    w.OUT = L + kSpOut;
    uint32_t lo = 0, hi = nchunks;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (uni(gptr(chunks + mid)->vec_base) <= item0) lo = mid;
        else hi = mid;
    }
    uint32_t ci = lo;
    DevChunk c = load_chunk(chunks, ci);
    bool have_table = false;
    for (uint32_t item = item0; item < item1;) {
        const uint32_t v = item - uni(c.vec_base);
        if (v >= uni(c.nvec)) {
            if (++ci >= nchunks) break;
            c = load_chunk(chunks, ci);
            have_table = false;
            continue;
        }
        gu8 *chunk = gptr(c.chunk);
        gu8 *aux = chunk + c.aux_off;
        if (!have_table) {
            wave_sync();
            const FLS_GLOBAL uint64_t *gs = reinterpret_cast<const FLS_GLOBAL uint64_t *>(aux);
            FLS_LDS uint64_t *ls = reinterpret_cast<FLS_LDS uint64_t *>(L + kSpSym);
            for (uint32_t k = lane; k < 256; k += 64) {
                const uint32_t n = k == kFsstEscape ? 0u : min((uint32_t)aux[8 * 256 + k], 8u);
                const uint64_t sy = gs[k];
                ls[k] = n >= 8 ? sy : sy & ((1ull << (8 * n)) - 1);
                L[kSpLen + k] = (uint8_t)n;
            }
            wave_sync();
            have_table = true;
        }
        const FLS_GLOBAL VecMeta *meta = reinterpret_cast<const FLS_GLOBAL VecMeta *>(chunk + c.meta_off) + v;
        const uint32_t poff = uni((uint32_t)meta->packed_off);
        const uint32_t base = uni((uint32_t)meta->for_base);
        const uint32_t aoff = uni((uint32_t)meta->aux_off);
        const uint32_t nvals = uni(meta->nvals);
        const uint32_t W = uni((uint32_t)meta->bw);
        const uint32_t dbytes = uni(meta->aux_count);
        fsst_vector_sp(w, chunk + c.packed_off + poff, W, base, nvals, dbytes, aux + aoff,
                       (FLS_GLOBAL uint8_t *)(size_t)c.dict, c.heap_bytes, c.heap_host,
                       gptr(c.out) + 16ull * kVectorSize * v, lane, err);
        wave_sync();
        ++item;
    }
}

__global__ __launch_bounds__(64) void fsst_sp_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                      uint32_t nitems, uint32_t *__restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    const uint32_t nwaves = gridDim.x, wave = blockIdx.x;
    const uint32_t per = (nitems + nwaves - 1) / nwaves;
    const uint32_t i0 = min(wave * per, nitems), i1 = min(i0 + per, nitems);
    if (i0 < i1) fsst_sp_range(chunks, uni(nchunks), uni(i0), uni(i1), (lu8 *)(size_t)(uint32_t)(size_t)lds_raw, err);
}

}  // namespace

hipError_t launch_fsst_sp(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                          hipStream_t stream) {
    if (nchunks == 0 || nvecs == 0) return hipSuccess;
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fsst_sp_kernel, 64, kSpWave) != hipSuccess)
            per_cu = 1;
    }
    const int grid = std::min<int>(cus * std::max(1, per_cu), (int)nvecs);
    if (getenv("FLS_DEBUG"))
        fprintf(stderr, "DEBUG: fsst_sp_kernel: %d blocks of 1 wave (%d per CU, %u B LDS), %u vectors\n", grid, per_cu,
                kSpWave, nvecs);
    hipLaunchKernelGGL(fsst_sp_kernel, dim3(grid), dim3(64), kSpWave, stream, d_chunks, nchunks, nvecs, d_err);
    return hipGetLastError();
}

// the segmented kernel's instantiations: variant V, ring cap CAP
template <int V, int CAP>
hipError_t launch_seg(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err, hipStream_t stream,
                      const FsstLaunch &how) {
    return how.queue ? (how.small ? launch_fsst_q<16, true, true, V, CAP>(d_chunks, nchunks, nvecs, d_err, stream, how)
                                  : launch_fsst_q<16, false, true, V, CAP>(d_chunks, nchunks, nvecs, d_err, stream, how))
                     : (how.small ? launch_fsst_q<16, true, false, V, CAP>(d_chunks, nchunks, nvecs, d_err, stream, how)
                                  : launch_fsst_q<16, false, false, V, CAP>(d_chunks, nchunks, nvecs, d_err, stream, how));
}

// every variant of the switches below (an unlisted one falls back to the default)
bool fsst_variant_built(int, bool, int) { return true; }

hipError_t launch_fsst(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                       hipStream_t stream, const FsstLaunch &how) {
    if (nchunks == 0 || nvecs == 0) return hipSuccess;
    if (how.seg) {  // segmented kernel; variants and ring caps for A/B (FLS_FSST_VARIANT, FLS_FSST_SEG_CAP)
        constexpr int SPLW = kFsstDefault | kFsstSegSparse | kFsstSegPackedLen | kFsstSegWide;
        constexpr int SPLWD = SPLW | kFsstSegDouble;
        constexpr int SPLWB = SPLW | kFsstSegBatch;
        // default: sparse stores, packed lengths, 16 reads in flight, records
        // in whole batches, ring cap 5120 (same-buffer A/B on l_comment SF10,
        // profiles/r3/abenv_fsst_r3j.txt, abenv_fsst_r3l.txt: 2 % ahead of the
        // same without batches, 2-3 % ahead of the code-parallel kernel), and
        // the lean writer and records (abenv_fsst_lean_r3za.txt: 0.847 against
        // 0.920 ms without)
        switch (how.variant) {
        case SPLWD:
            return launch_seg<SPLWD, 6144>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLWB:
            return launch_seg<SPLWB, 5120>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case kFsstDefault:
        case SPLWB | kFsstSegLean:
            return launch_seg<SPLWB | kFsstSegLean, 5120>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLWB | kFsstSegLean | kFsstSegW4:
            return launch_seg<SPLWB | kFsstSegLean | kFsstSegW4, 5120>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLWB | kFsstSegLean | kFsstSegLazy:
            return launch_seg<SPLWB | kFsstSegLean | kFsstSegLazy, 5120>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLWB | kFsstSegLean | kFsstSegD8 | kFsstSegLazy:
            return launch_seg<SPLWB | kFsstSegLean | kFsstSegD8 | kFsstSegLazy, 4832>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLWB | kFsstSegLean | kFsstSegD8:
            return launch_seg<SPLWB | kFsstSegLean | kFsstSegD8, 4832>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLW | kFsstAblateRecords:
            return launch_seg<SPLW | kFsstAblateRecords, 4096>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLW | kFsstAblateFlush:
            return launch_seg<SPLW | kFsstAblateFlush, 4096>(d_chunks, nchunks, nvecs, d_err, stream, how);
        case SPLW | kFsstAblateWrite:
            return launch_seg<SPLW | kFsstAblateWrite, 4096>(d_chunks, nchunks, nvecs, d_err, stream, how);
        default:
            return how.seg_cap == 5120 ? launch_seg<SPLW, 5120>(d_chunks, nchunks, nvecs, d_err, stream, how)
                                       : launch_seg<SPLW, 4096>(d_chunks, nchunks, nvecs, d_err, stream, how);
        }
    }
    if (how.bytes_per_lane == 16)
        return how.small ? launch_fsst_t<16, true>(d_chunks, nchunks, nvecs, d_err, stream, how)
                         : launch_fsst_t<16, false>(d_chunks, nchunks, nvecs, d_err, stream, how);
    return how.small ? launch_fsst_t<8, true>(d_chunks, nchunks, nvecs, d_err, stream, how)
                     : launch_fsst_t<8, false>(d_chunks, nchunks, nvecs, d_err, stream, how);
}

}  // namespace fls
