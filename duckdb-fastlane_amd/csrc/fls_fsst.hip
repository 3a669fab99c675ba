// fls_fsst.hip -- MI355X (gfx950) FSST string decode into DuckDB string_t.
//
// Replaces the FSST step inside RowgroupReader::materialize()
// (reference src/fastlanes_facade.cpp:48, the FLSStrColumn consumer at
// :163-170) for VARCHAR / BLOB chunks written with ENC_FSST (fls_format.hpp).
//
// The product build holds one kernel per chunk layout, each in its measured
// best configuration:
//   1. segmented kernel (every chunk the writer produces since round 3: a
//      segment table per vector gives each 16-code segment its decoded length
//      and entry escape state, so lane l decodes segment l of a round on its
//      own, no hand-off between lanes);
//   2. code-parallel kernel (chunks without segment tables: each round's
//      output positions come from a wave scan of the lanes' decoded lengths
//      and the escape state from the parity rule);
//   3. string-parallel kernel (policy bit 7, FLS_DECODE_POLICY=128: chunks
//      whose strings are all <= 255 bytes, one string per lane).
// The variants, ablations and ring sizes they were chosen against (DESIGN.md
// §5 item 9, §12) live in fls_fsst_lab.hip, built only into the
// experiment library (`make lab`, -DFLS_EXPERIMENTS, FLS_LIB=libflsgpu_lab.so).
//
// Common to all three: one wave per 64-thread block (LDS is per wave, so a CU
// holds as many waves as its LDS fits); the chunk's symbol table is staged in
// LDS sanitised (each symbol masked to its length so whole symbols can be
// OR-ed, the escape code's entry empty); decoded bytes go through a per-wave
// LDS ring that is kept zero past the decoded bytes (the flush zeroes what it
// streams out), complete 16 B blocks stream to the chunk's heap in HBM, and
// every string gets its 16 B string_t (inline bytes, or a 4-byte prefix plus
// a pointer into the heap's host copy).  Strings never straddle a vector and
// every vector's heap starts 16-byte aligned, so only one wave writes a heap
// line.  Corrupt input (lengths that disagree with the stream, truncated
// escapes, segment tables that disagree with the codes) is clamped and
// reported through KERR_FSST.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "fls_decode.hpp"
#include "fls_decode_dev.hpp"
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
using lu16 = FLS_LDS uint16_t;
using lu32 = FLS_LDS uint32_t;
using lu64 = FLS_LDS uint64_t;

__device__ __forceinline__ uint32_t rl(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint32_t byte_of(const v4u &r, uint32_t k) {
    const uint32_t w = k < 4 ? r.x : k < 8 ? r.y : k < 12 ? r.z : r.w;
    return (w >> (8 * (k & 3))) & 0xFF;
}
// Inclusive wave-64 prefix sum on DPP (row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast 15/31 across rows): six VALU steps, no LDS round trip.
__device__ __forceinline__ uint32_t scan_incl(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}
// lanes [0, k) of a ballot mask all set: k = count of trailing ones
__device__ __forceinline__ uint32_t leading_ok(uint64_t m) { return ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m); }

// The chunk descriptor, wave-uniform: read into SGPRs (readfirstlane of its
// 16 dwords), not 16 VGPRs.
__device__ __forceinline__ DevChunk load_chunk(const DevChunk *chunks, uint32_t ci) {
    const FLS_GLOBAL v4u *q = reinterpret_cast<const FLS_GLOBAL v4u *>(gptr(chunks + ci));
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
// A wave-uniform 64-bit pointer (readfirstlane of both halves).
template <class T>
__device__ __forceinline__ T *uni_ptr(T *p) {
    const uint64_t v = (uint64_t)p;
    return (T *)((uint64_t)uni((uint32_t)(v >> 32)) << 32 | uni((uint32_t)v));
}
// Index of the chunk holding launch item `item` (last ci with vec_base <= item).
// Chunks of full row groups hold 64 vectors, so item / 64 is checked first
// (one descriptor read); a binary search otherwise.
__device__ __forceinline__ uint32_t chunk_of(const DevChunk *chunks, uint32_t nchunks, uint32_t item) {
    const uint32_t g = min(item / 64, nchunks - 1);
    const uint32_t gb = uni(gptr(chunks + g)->vec_base), gn = uni(gptr(chunks + g)->nvec);
    if (gb <= item && item - gb < gn) return g;
    uint32_t lo = 0, hi = nchunks;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (uni(gptr(chunks + mid)->vec_base) <= item) lo = mid;
        else hi = mid;
    }
    return lo;
}
// The per-vector fields every kernel reads from its VecMeta (wave-uniform).
struct VecArgs {
    gu8 *packed;          // FFOR stream of the decompressed string lengths
    gu8 *vh;              // FsstVecHeader
    uint32_t W, base, nvals, dbytes;
    FLS_GLOBAL uint8_t *out;   // the vector's string_t records
};
__device__ __forceinline__ VecArgs vec_args(const DevChunk &c, uint32_t v) {
    gu8 *chunk = gptr(c.chunk);
    const FLS_GLOBAL VecMeta *meta = reinterpret_cast<const FLS_GLOBAL VecMeta *>(chunk + c.meta_off) + v;
    VecArgs a;
    a.packed = chunk + c.packed_off + uni((uint32_t)meta->packed_off);
    a.vh = chunk + c.aux_off + uni((uint32_t)meta->aux_off);
    a.base = uni((uint32_t)meta->for_base);
    a.nvals = uni(meta->nvals);
    a.W = uni(min((uint32_t)meta->bw, 32u));
    a.dbytes = uni(meta->aux_count);
    a.out = gptr(c.out) + 16ull * kVectorSize * v;
    return a;
}
// The FsstVecHeader fields and the vector's heap window.
struct VecHeap {
    uint32_t heap_off, comp_len, clen_w, hlim;
    FLS_GLOBAL uint8_t *heap;   // the vector's heap bytes
    uint64_t ptr_base;          // host address string_t pointers use for its byte 0
};
__device__ __forceinline__ VecHeap vec_heap(const DevChunk &c, const VecArgs &a) {
    const FLS_GLOBAL FsstVecHeader *hp = reinterpret_cast<const FLS_GLOBAL FsstVecHeader *>(a.vh);
    VecHeap h;
    h.heap_off = uni(hp->heap_off);
    h.comp_len = uni(hp->comp_len);
    h.clen_w = uni(min(hp->clen_w, 32u));
    // blocks past the vector's padded bytes or the chunk's heap are refused
    h.hlim = min((a.dbytes + 15) & ~15u, c.heap_bytes > h.heap_off ? c.heap_bytes - h.heap_off : 0u);
    h.heap = (FLS_GLOBAL uint8_t *)(size_t)c.dict + h.heap_off;
    h.ptr_base = c.heap_host + h.heap_off;
    return h;
}

// Stage the chunk's symbol table into LDS, sanitised: symbol k masked to its
// length, the escape code's entry {0, 0}.  TAG: the length (in bits, 8 x
// bytes) rides in the top byte of the entry (the segmented kernel: tables of
// symbols <= 7 bytes only; a longer one is reported as a bad descriptor).
// Else the byte lengths go to len[256].
template <bool TAG, bool SPLIT = false>
__device__ __forceinline__ void stage_table(gu8 *aux, lu64 *sym, lu8 *len, uint32_t lane, uint32_t *err) {
    wave_sync();
    const FLS_GLOBAL uint64_t *gs = reinterpret_cast<const FLS_GLOBAL uint64_t *>(aux);
    bool long8 = false;
    for (uint32_t k = lane; k < 256; k += 64) {
        const uint32_t n = k == kFsstEscape ? 0u : min((uint32_t)aux[8 * 256 + k], 8u);
        const uint64_t sy = n >= 8 ? gs[k] : gs[k] & ((1ull << (8 * n)) - 1);
        if constexpr (TAG && SPLIT) {  // (experiment) low dwords at [0, 256), high at [256, 512)
            const uint64_t t = sy | (uint64_t)(8 * n) << 56;
            reinterpret_cast<lu32 *>(sym)[k] = (uint32_t)t;
            reinterpret_cast<lu32 *>(sym)[256 + k] = (uint32_t)(t >> 32);
            long8 |= n >= 8;
        } else if constexpr (TAG) {
            sym[k] = sy | (uint64_t)(8 * n) << 56;
            long8 |= n >= 8;
        } else {
            sym[k] = sy;
            len[k] = (uint8_t)n;
        }
    }
    if (TAG && __ballot(long8) != 0 && lane == 0) atomicOr(err, KERR_BAD_DESC);
    wave_sync();
}

// Unpack a vector's FFOR string lengths (T = 32, W bits, base) for values
// 4 ci .. 4 ci + 3 of the 256 16-byte chunks, zero past nvals.
__device__ __forceinline__ v4u length_chunk(lv4 *P, uint32_t W, uint32_t base, uint32_t nvals, uint32_t ci) {
    v4u v = add_base<32>(unpack_chunk<32>(P, W, ci), base);
    if (4 * ci + 0 >= nvals) v.x = 0;
    if (4 * ci + 1 >= nvals) v.y = 0;
    if (4 * ci + 2 >= nvals) v.z = 0;
    if (4 * ci + 3 >= nvals) v.w = 0;
    return v;
}
// Stage a vector's packed lengths (8 W 16-byte rows plus a zero row) at P.
__device__ __forceinline__ void stage_packed(lv4 *P, gu8 *packed, uint32_t W, uint32_t lane) {
    const uint32_t n16 = 8 * W;
    gv4 *pk = reinterpret_cast<gv4 *>(packed);
    for (uint32_t i = lane; i < n16; i += 64) P[i] = pk[i];
    if (lane < 8) P[n16 + lane] = mk4(0, 0, 0, 0);
    wave_sync();
}

// string_t fields of a string of n bytes whose first bytes are the ring
// dwords w0..w3 shifted by sh bytes: inline (n <= 12: bytes past n zeroed) or
// prefix + host pointer p.  One v_perm_b32 per word aligns and masks:
// selector byte j is sh + j (a byte of the dword pair) while 4k + j < n, else
// 12 (a zero byte); the bytes at or past the length come from a 64-bit shift
// of ones by 8 x clamp(n - 4k, 0, 4) (amounts 0..32, no wrap).
template <bool SEL = false>
__device__ __forceinline__ v4u make_record(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t sh,
                                           uint32_t n, uint64_t p) {
    const uint32_t base = 0x03020100u + sh * 0x01010101u, t = 8 * n;
    auto word = [&](uint32_t hi, uint32_t lo, int k) -> uint32_t {
        const uint32_t sk = (uint32_t)min(max((int)t - 32 * k, 0), 32);
        const uint32_t past = (uint32_t)(0xFFFFFFFFull << sk);
        const uint32_t sel = (past & 0x0C0C0C0Cu) | (~past & base);
        return __builtin_amdgcn_perm(hi, lo, sel);
    };
    const bool inl = n <= 12;
    if constexpr (SEL) {  // both forms computed, picked by bit select: no branch (kSegXRecSel: the branch)
        const uint32_t m = 0u - (uint32_t)inl;
        uint32_t a = word(w2, w1, 1), b = word(w3, w2, 2);
        asm volatile("" : "+v"(a), "+v"(b));
        return mk4(n, word(w1, w0, 0), (a & m) | ((uint32_t)p & ~m), (b & m) | ((uint32_t)(p >> 32) & ~m));
    }
    return mk4(n, word(w1, w0, 0), inl ? word(w2, w1, 1) : (uint32_t)p, inl ? word(w3, w2, 2) : (uint32_t)(p >> 32));
}

// Stream complete 16 B blocks [from, upto) of the ring (ring byte 0 = decoded
// byte ring_base) to the vector's heap, zeroing each block as it leaves (the
// ring stays zero past the decoded bytes).  Up to 4 blocks per lane per pass,
// all ring reads in flight before the zeroing and the heap stores.  A block
// past the vector's heap window is refused (bad).
template <bool UNIFORM = false, bool CLAMP = false>
__device__ __forceinline__ void flush_ring(lu8 *ring, uint32_t ring_bytes, uint32_t ring_base, uint32_t upto,
                                           const VecHeap &h, uint32_t lane, bool &bad) {
    // (a ring never holds more than ring_bytes: the clamp bounds the loop
    // whatever a corrupt stream did to the positions)
    const uint32_t nblk = min((upto - ring_base) >> 4, ring_bytes / 16);
    lv4 *r16 = reinterpret_cast<lv4 *>(ring);
    if constexpr (CLAMP) {
        // (experiment kSegXClamp) no exec-masked stores: the window is checked
        // once for the wave, a pass's rows of 64 blocks past the end are
        // skipped by a wave-uniform test, and in the last row the lanes past
        // nblk take block nblk - 1 -- they read, zero and store the same bytes
        // as its own lane, which is harmless
        if (ring_base + 16 * nblk <= h.hlim) {
            for (uint32_t q0 = 0; q0 < nblk; q0 += 256) {
                const uint32_t nj = min(4u, (nblk - q0 + 63) >> 6);
                v4u b[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (j < nj) b[j] = r16[min(q0 + 64 * j + lane, nblk - 1)];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if (j < nj) {
                        const uint32_t q = min(q0 + 64 * j + lane, nblk - 1);
                        r16[q] = mk4(0, 0, 0, 0);
                        *reinterpret_cast<ov4 *>(h.heap + ring_base + 16 * q) = b[j];
                    }
            }
            return;
        }
    }
    if constexpr (UNIFORM) {
        // every block inside the heap window, checked once for the wave: no
        // per-block bound test (kSegXFlush: the per-block test below)
        if (ring_base + 16 * nblk <= h.hlim) {
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
                        *reinterpret_cast<ov4 *>(h.heap + ring_base + 16 * q) = b[j];
                    }
                }
            }
            return;
        }
    }
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
                const uint32_t g = ring_base + 16 * q;
                if (g + 16 <= h.hlim) *reinterpret_cast<ov4 *>(h.heap + g) = b[j];
                else bad = true;
            }
        }
    }
}

// ============================================================================
// 1. Segmented kernel.
//
// Per vector:
//   a. the FFOR string lengths become exclusive offsets in LDS (u16 mod 65536
//      for chunks whose strings are all <= 255 bytes, "SMALL", else u32);
//   b. rounds of 64 segments of 16 code bytes (one 16 B load per lane, the
//      next round's in flight while this one decodes): lane l decodes segment
//      64 r + l at the output offset the segment table gives (a wave scan of
//      the segments' decoded lengths) from the entry escape state it gives,
//      ORing completed qwords into the zeroed ring; a round whose output
//      exceeds the ring cap is written in parts (lanes [l0, l1) at a time);
//   c. after the next round's loads are issued (the stores' vmcnt must not
//      sit in front of the next wait): the string_t records of every batch of
//      64 strings whose first bytes are decoded, the complete 16 B blocks of
//      the ring to the heap, and the unfinished tail to the ring start.
// What shaped it (same-buffer A/B on l_comment SF10, profiles/r3/): the
// segment table instead of the ballot/bpermute escape hand-off
// (abenv_fsst_seg_r3*.txt), sparse qword stores (abenv_fsst_sparse_r3d.txt),
// lengths packed in the symbols' top byte (abenv_fsst_pl_r3e.txt), 16 table
// reads in flight on the escape-free path, records in whole batches of 64
// (abenv_fsst_batch_r3i.txt), a 5120-byte ring cap (abenv_fsst_r3j/l.txt) and
// the lean writer and records (abenv_fsst_lean_r3za.txt): 0.90-0.93 ms for the
// code-parallel kernel -> 0.80-0.85 ms.
// ============================================================================
constexpr uint32_t kSegRingCap = 5120;             // decoded bytes per part of a round
constexpr uint32_t kSegSlack = 2 * 16 * 8 + 16;    // a lane may write past its claimed end on a corrupt table

// Per-wave LDS layout (bytes, 16-aligned): string offsets (SMALL: u16 x 1025;
// else u32 x 1025), the tagged symbol table u64[256], 256 B kept free (the
// occupancy the kernel was measured at: 16 waves per CU), the ring.  The
// packed lengths are staged in the ring before the rounds start.
// Experiment bits of the segmented kernel (0 in the product build; the
// experiment library, make exp, instantiates the others for same-buffer A/B:
// FLS_FSST_VARIANT = kFsstDefault | x << kSegXShift).
enum : int {
    kSegXShift = 20,
    kSegXInline = 1,   // records read a string's bytes 4..11 only for inline (<= 12-byte) strings
    kSegXNoPad = 2,    // no 256 B pad in the per-wave LDS (17 waves per CU instead of 16 for SMALL)
    kSegXSplit = 4,    // symbol table as two u32 arrays (low / high dwords): two b32 gathers per code
    kSegXDouble = 8,   // two consecutive segments (32 code bytes) per lane per round: half the rounds
    // round 5: the next two are the default (a ring flush bound-checked once
    // per wave; string_t records with both forms computed and bit-selected,
    // no branch), -1.2 % on l_comment SF10 on two boxes
    // (profiles/r5/abenv_fsst_segx_r5a.txt, abenv_r5n_lineitem_full_10.txt);
    // the bits now select round 4's forms
    kSegXFlush = 16,   // ring flush bound-checked per block
    kSegXRecSel = 32,  // string_t records: a branch between the inline and the pointer form
    kSegXClamp = 64,   // ring flush without exec-masked stores (clamped block index, uniform row skips)
    kSegXNoBranch = 128,  // escape-free codes: every code ORs (an incomplete qword into a dummy slot), no exec mask
    kSegXTwo = 256,       // escape-free segments as two independent 8-code chains (the second's start from the first's lengths)
};
template <bool SMALL, int X = 0>
struct SegLds {
    static constexpr uint32_t kOffD = 0;
    static constexpr uint32_t kOffSym = SMALL ? 2064 : 4112;
    static constexpr uint32_t kOffRing = kOffSym + 2048 + ((X & kSegXNoPad) ? 0 : 256);
    static constexpr uint32_t kPackedMax = SMALL ? 128 * 8 + 128 : 128 * 32 + 128;  // W <= 8 | 32, + zero row
    static constexpr uint32_t kSlack = (X & kSegXDouble) ? 2 * 32 * 8 + 16 : kSegSlack;  // 32 codes per lane
    static constexpr uint32_t kRing = kPackedMax > kSegRingCap + kSlack ? kPackedMax : kSegRingCap + kSlack;
    static constexpr uint32_t kWave = kOffRing + kRing;
    static_assert(kOffSym % 16 == 0 && kOffRing % 16 == 0 && kWave % 16 == 0, "LDS layout alignment");
};

// A lane's decoded bytes, appended to the zeroed ring through a 64-bit
// accumulator that is OR-ed (ds_or_b64) into its qword only once the qword is
// complete (about one lane in four per code step, which is what kept the LDS
// bank conflicts of a per-code OR down); lengths in bits (the staged table's
// top byte is 8 x the symbol length); the position is the open qword's ring
// byte plus a bit offset, and the carry out of a completed qword is one shift
// (the offset is >= 8 whenever a qword completes: symbols are <= 7 bytes).
// The first and last qwords of a lane are shared with its neighbours; OR
// merges them.
struct LeanWriter {
    lu8 *ring;
    uint64_t acc;
    uint32_t a, b, start;   // open qword's ring byte, bit offset in it, start position (bits)
    __device__ __forceinline__ LeanWriter(lu8 *r, uint32_t wp)
        : ring(r), acc(0), a(wp & ~7u), b(8 * (wp & 7)), start(8 * wp) {}
    __device__ __forceinline__ void complete(uint64_t carry) {
        __hip_atomic_fetch_or(reinterpret_cast<lu64 *>(ring + a), acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        a += 8;
        acc = carry;
    }
    // a symbol v of bl bits (<= 56)
    __device__ __forceinline__ void put(uint64_t v, uint32_t bl) {
        acc |= v << b;
        const uint32_t nb = b + bl;
        if (nb >= 64) complete(v >> (64 - b));
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
        if (nb >= 64) complete(v >> (64 - b));
        b = nb & 63;
    }
    // (experiment kSegXNoBranch) the same without the exec-masked branch:
    // every code ORs, an incomplete qword into the lane's dummy slot (two
    // lanes share one) -- two SALU instructions per code fewer
    __device__ __forceinline__ void put_tagged_nb(uint32_t lo, uint32_t hi, lu64 *dummy) {
        uint32_t nb = b + (hi >> 24);
        asm("" : "+v"(hi), "+v"(nb));
        hi &= 0x00FFFFFFu;
        const uint64_t v = (uint64_t)hi << 32 | lo;
        acc |= v << b;
        const bool c = nb >= 64;
        lu64 *dst = c ? reinterpret_cast<lu64 *>(ring + a) : dummy;
        __hip_atomic_fetch_or(dst, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        a += c ? 8u : 0u;
        acc = c ? v >> ((64u - b) & 63u) : acc;
        b = nb & 63;
    }
    __device__ __forceinline__ void finish() {
        if (b) __hip_atomic_fetch_or(reinterpret_cast<lu64 *>(ring + a), acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    __device__ __forceinline__ uint32_t bytes() const { return (8 * a + b - start) >> 3; }
};

// One lane's segment: its nb (<= 16) code bytes in raw, decoded from escape
// state st into the ring through qw; returns the bytes written, st = the state
// after its last code.  FULL: all 16 bytes are codes.  ESC: the vector holds
// escape codes (without them every code is a symbol, and a stray escape
// decodes to nothing -- its staged entry is {0, 0} -- which the byte-count
// check catches).  The fast path (FULL, no escapes) issues all 16 table reads
// together; the general one keeps each code byte (a literal's value) beside
// its entry and reads 4 at a time to stay in the fast path's registers.
template <bool FULL, bool ESC, bool SPLIT = false, bool NOBRANCH = false, bool TWO = false>
__device__ __forceinline__ uint32_t seg_lane(const lu64 *sym, const v4u &raw_in, uint32_t nb, uint32_t &st,
                                             LeanWriter &qw, lu64 *dummy = nullptr) {
    // an opaque copy: the callers' variants would otherwise share (hoist) the
    // byte extraction and table addresses of all 16 codes ahead of their
    // branch, all of them live at once
    v4u raw = raw_in;
    asm volatile("" : "+v"(raw.x), "+v"(raw.y), "+v"(raw.z), "+v"(raw.w));
    constexpr bool kFast = FULL && !ESC;
    constexpr uint32_t B = kFast ? 16 : 4;
#pragma unroll
    for (uint32_t h = 0; h < 16 / B; ++h) {
        uint32_t c[B], sl[B];
        uint64_t sy[B];
#pragma unroll
        for (uint32_t k = 0; k < B; ++k) {
            c[k] = byte_of(raw, B * h + k);
            if constexpr (SPLIT) {
                const lu32 *s32 = reinterpret_cast<const lu32 *>(sym);
                sy[k] = (uint64_t)s32[256 + c[k]] << 32 | s32[c[k]];
            } else {
                sy[k] = sym[c[k]];
            }
            if constexpr (!kFast) {
                sl[k] = (uint32_t)(sy[k] >> 56);
                sy[k] &= 0x00FFFFFFFFFFFFFFull;
            }
        }
        if constexpr (kFast && TWO) {
            // (kSegXTwo) codes 0-7 and 8-15 as two independent chains: the
            // second starts where the first 8 symbols end (their lengths, in
            // bits, ride in the entries' top bytes); the chains share at most
            // the qword at the seam, and OR merges it
            uint32_t h8 = 0;
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) h8 += (uint32_t)(sy[k] >> 56);
            LeanWriter q2(qw.ring, (8 * qw.a + qw.b + h8) >> 3);
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                qw.put_tagged((uint32_t)sy[k], (uint32_t)(sy[k] >> 32));
                q2.put_tagged((uint32_t)sy[k + 8], (uint32_t)(sy[k + 8] >> 32));
            }
            qw.finish();
            qw.acc = q2.acc;  // the lane goes on as the second chain (start kept: bytes() counts both)
            qw.a = q2.a;
            qw.b = q2.b;
            return qw.bytes();
        }
#pragma unroll
        for (uint32_t k = 0; k < B; ++k) {
            if constexpr (kFast) {
                if constexpr (NOBRANCH) qw.put_tagged_nb((uint32_t)sy[k], (uint32_t)(sy[k] >> 32), dummy);
                else qw.put_tagged((uint32_t)sy[k], (uint32_t)(sy[k] >> 32));
                continue;
            }
            // selects as bit masks (v_bfi), not compares: per-code lane masks
            // would each take an SGPR pair, and 16 live ones spill
            uint32_t vlo = (uint32_t)sy[k], vhi = (uint32_t)(sy[k] >> 32), n = sl[k];
            if constexpr (ESC) {
                const uint32_t lit = 0u - st;                        // all ones after an escape
                vlo = (vlo & ~lit) | (c[k] & lit);
                vhi &= ~lit;
                n = (n & ~lit) | (8u & lit);
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
            qw.put((uint64_t)vhi << 32 | vlo, n);
        }
        // the next batch's table reads stay behind this batch's writes:
        // hoisted, their values would be live across them (spills)
        wave_sync();
    }
    return qw.bytes();
}

template <bool SMALL, int X = 0>
__device__ void seg_vector(lu8 *L, const lu64 *sym, const DevChunk &c, const VecArgs &a, uint32_t lane,
                           uint32_t *err) {
    using Layout = SegLds<SMALL, X>;
    lu8 *ring = L + Layout::kOffRing;
    lu32 *D = reinterpret_cast<lu32 *>(L + Layout::kOffD);
    const uint32_t nvals = a.nvals;
    bool bad = false;

    // ---- a. string offsets ---------------------------------------------------
    const uint32_t W = SMALL ? min(a.W, 8u) : a.W;
    stage_packed(reinterpret_cast<lv4 *>(ring), a.packed, W, lane);
    uint32_t total = 0;
    if constexpr (SMALL) {
        // u8 lengths staged in the ring past the packed words, then each lane
        // turns 16 consecutive ones into u16 exclusive offsets (mod 65536:
        // the records rebuild the high bits, strings being <= 255 bytes)
        lu32 *L8 = reinterpret_cast<lu32 *>(ring + 2048);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t ci = lane + 64 * j;
            const v4u v = length_chunk(reinterpret_cast<lv4 *>(ring), W, a.base, nvals, ci);
            L8[ci] = (v.x & 255) | (v.y & 255) << 8 | (v.z & 255) << 16 | (v.w & 255) << 24;
        }
        wave_sync();
        const v4u q = reinterpret_cast<const lv4 *>(L8)[lane];
        const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
        uint32_t o[16], run = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            o[k] = run;
            run += (wd[k >> 2] >> (8 * (k & 3))) & 255;
        }
        const uint32_t incl = scan_incl(run);
        const uint32_t excl = incl - run;
#pragma unroll
        for (int k = 0; k < 16; k += 2) D[8 * lane + k / 2] = ((excl + o[k]) & 0xFFFF) | (excl + o[k + 1]) << 16;
        if (lane == 63) reinterpret_cast<lu16 *>(D)[1024] = (uint16_t)incl;
        total = rl(incl, 63);
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t ci = lane + 64 * j;
            reinterpret_cast<lv4 *>(D)[ci] = length_chunk(reinterpret_cast<lv4 *>(ring), W, a.base, nvals, ci);
        }
        wave_sync();
        uint32_t o[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u v = reinterpret_cast<const lv4 *>(D)[4 * lane + q];
            o[4 * q] = v.x; o[4 * q + 1] = v.y; o[4 * q + 2] = v.z; o[4 * q + 3] = v.w;
        }
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t t = o[k];
            o[k] = run;  // exclusive
            run += t;
        }
        const uint32_t incl = scan_incl(run);
        const uint32_t excl = incl - run;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            reinterpret_cast<lv4 *>(D)[4 * lane + q] = mk4(excl + o[4 * q], excl + o[4 * q + 1], excl + o[4 * q + 2], excl + o[4 * q + 3]);
        if (lane == 63) D[1024] = incl;
        total = rl(incl, 63);
    }
    wave_sync();
    if (total != a.dbytes) bad = true;
    // the ring (which staged the packed lengths) starts all zero; from here on
    // every byte past the decoded ones stays zero: the flush zeroes the blocks
    // it streams out and the tail move the bytes it vacates
    for (uint32_t q = lane; q < Layout::kRing / 16; q += 64) reinterpret_cast<lv4 *>(ring)[q] = mk4(0, 0, 0, 0);
    wave_sync();

    const VecHeap h = vec_heap(c, a);
    gv4 *comp = reinterpret_cast<gv4 *>(a.vh + sizeof(FsstVecHeader) + 128 * h.clen_w);
    const uint32_t comp_len = h.comp_len;

    // out_pos = decoded bytes so far; ring byte 0 is decoded byte ring_base;
    // next_str = first string without its string_t, str_base = its offset
    uint32_t out_pos = 0, ring_base = 0, carry_lit = 0, next_str = 0, str_base = 0;
    // ---- c. records: whole batches of 64 strings whose first min(n, 12)
    // bytes are decoded (a partial batch waits, unless `force` -- vector end,
    // ring full -- or its bytes fill half the ring: a batch of long strings
    // may not fit it at all); offsets straight from D, no length scan
    auto records = [&](bool force) {
        while (next_str < nvals) {
            const uint32_t i = next_str + lane;
            const bool valid = i < nvals;
            uint32_t rel0, rel1;  // string start / end relative to str_base
            if constexpr (SMALL) {
                const lu16 *D16 = reinterpret_cast<const lu16 *>(D);
                const uint32_t x = D16[min(i, nvals)], y = D16[min(i + 1, nvals)];
                const uint32_t b16 = rl(x, 0);
                rel0 = (x - b16) & 0xFFFF;
                rel1 = (y - b16) & 0xFFFF;
            } else {
                rel0 = D[min(i, nvals)] - str_base;
                rel1 = D[min(i + 1, nvals)] - str_base;
            }
            const uint32_t d0 = str_base + rel0, n = rel1 - rel0;
            const bool ok = valid && d0 + min(n, 12u) <= out_pos;
            const uint64_t m = __ballot(ok), vm = __ballot(valid);
            if (!force && m != vm && out_pos - str_base <= kSegRingCap / 2) break;
            const uint32_t n_ok = leading_ok(m);
            if (lane < n_ok) {
                const lu32 *r32 = reinterpret_cast<const lu32 *>(ring);
                const uint32_t x = d0 - ring_base, i0 = x >> 2;
                uint32_t w2 = 0, w3 = 0;
                if constexpr ((X & kSegXInline) != 0) {
                    if (n <= 12) {  // a pointer record needs only the 4-byte prefix
                        w2 = r32[i0 + 2];
                        w3 = r32[i0 + 3];
                    }
                } else {
                    w2 = r32[i0 + 2];
                    w3 = r32[i0 + 3];
                }
                *reinterpret_cast<ov4 *>(a.out + 16ull * i) =
                    make_record<(X & kSegXRecSel) == 0>(r32[i0], r32[i0 + 1], w2, w3, x & 3, n, h.ptr_base + d0);
            }
            if (n_ok > 0) str_base += rl(rel1, n_ok - 1);
            next_str += n_ok;
            if (n_ok < 64) break;
        }
    };
    // records, then the complete blocks below the first byte still needed (the
    // oldest string without a record, or the decode position) to the heap,
    // then the kept tail (an unfinished batch, up to a few KB) to the ring
    // start 1 KB at a time, the bytes it vacates back to zero
    auto retire = [&](bool force) {
        records(force);
        const uint32_t keep_from = next_str < nvals ? min(str_base, out_pos) : out_pos;
        const uint32_t new_base = keep_from & ~15u;
        flush_ring<(X & kSegXFlush) == 0, (X & kSegXClamp) != 0>(ring, Layout::kRing, ring_base, new_base, h, lane, bad);
        wave_sync();
        const uint32_t src = min(new_base - ring_base, Layout::kRing);
        const uint32_t len = min((out_pos - new_base + 15) & ~15u, Layout::kRing - 16);
        lv4 *r16 = reinterpret_cast<lv4 *>(ring);
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

    // ---- b. rounds of 64 segments ---------------------------------------------
    const uint32_t soff = sizeof(FsstVecHeader) + 128 * h.clen_w + ((comp_len + 15) & ~15u);
    const FLS_GLOBAL FsstSegHeader *shp = reinterpret_cast<const FLS_GLOBAL FsstSegHeader *>(a.vh + soff);
    const uint32_t nseg = (comp_len + kFsstSegCodes - 1) / kFsstSegCodes;
    const bool vec_esc = (uni(shp->flags) & FSST_SEG_HAS_ESCAPE) != 0;
    if (uni(shp->nseg) != nseg) bad = true;
    gu8 *segv = a.vh + soff + sizeof(FsstSegHeader);
    // (experiment kSegXDouble: lane l decodes segments 2l and 2l + 1 of a round)
    constexpr uint32_t SEGS = (X & kSegXDouble) ? 2 : 1;
    constexpr uint32_t kRoundCodes = 64 * 16 * SEGS;
    const uint32_t n16 = (comp_len + 15) >> 4;
    auto load_seg = [&](uint32_t r0, uint32_t j) -> uint32_t {
        const uint32_t k = (r0 >> 4) + SEGS * lane + j;
        return k < nseg ? (uint32_t)segv[k] : 0u;
    };
    auto load_codes = [&](uint32_t r0, uint32_t j) -> v4u {
        const uint32_t k = (r0 >> 4) + SEGS * lane + j;
        return k < n16 ? comp[k] : mk4(0, 0, 0, 0);
    };
    v4u raw_next = load_codes(0, 0), raw_next1 = mk4(0, 0, 0, 0);
    uint32_t sv_next = load_seg(0, 0), sv_next1 = 0;
    if constexpr (SEGS == 2) {
        raw_next1 = load_codes(0, 1);
        sv_next1 = load_seg(0, 1);
    }
    for (uint32_t r0 = 0; r0 < comp_len; r0 += kRoundCodes) {
        const uint32_t idx0 = r0 + 16 * SEGS * lane;
        const v4u raw = raw_next, raw1 = raw_next1;
        // segment value: dlen (entry state 0) or 129 + dlen (state 1)
        const uint32_t entry = sv_next > 128 ? 1u : 0u;
        const uint32_t dl0 = entry ? sv_next - 129 : sv_next;
        const uint32_t entry1 = sv_next1 > 128 ? 1u : 0u;
        const uint32_t dl = dl0 + (SEGS == 2 ? (entry1 ? sv_next1 - 129 : sv_next1) : 0u);
        if (r0 + kRoundCodes < comp_len) {
            raw_next = load_codes(r0 + kRoundCodes, 0);
            sv_next = load_seg(r0 + kRoundCodes, 0);
            if constexpr (SEGS == 2) {
                raw_next1 = load_codes(r0 + kRoundCodes, 1);
                sv_next1 = load_seg(r0 + kRoundCodes, 1);
            }
        }
        const bool full = r0 + kRoundCodes <= comp_len;
        // the previous round's stores, after this round's loads
        if (r0 > 0) retire(false);
        const uint32_t incl = scan_incl(dl);
        uint32_t st = entry, l0 = 0, done = 0, guard = 0;
        for (;;) {  // the lanes whose output fits the ring, then the rest
            if (++guard > 130) {  // at most 64 parts + 64 retires: a corrupt table
                bad = true;
                break;
            }
            const uint32_t p0 = out_pos - ring_base;
            const bool fits = lane < l0 || p0 + (incl - done) <= kSegRingCap;
            const uint32_t l1 = leading_ok(__ballot(fits));
            if (l1 == l0) {  // nothing fits beside the kept tail: retire it first
                retire(true);
                continue;    // then the tail is < 32 B and lane l0 (<= 256 B) fits
            }
            const uint32_t part = rl(incl, l1 - 1) - done;
            wave_sync();
            if (lane >= l0 && lane < l1) {
                LeanWriter qw(ring, p0 + (incl - dl - done));
                const uint32_t nb = idx0 < comp_len ? min(comp_len - idx0, 16u) : 0u;
                constexpr bool kSplit = (X & kSegXSplit) != 0;
                // (kSegXNoBranch) the lane's dummy slot: the 256 B pad before the ring
                constexpr bool kNoBr = (X & kSegXNoBranch) != 0 && (X & kSegXNoPad) == 0;
                constexpr bool kTwo = (X & kSegXTwo) != 0 && !kNoBr && !kSplit;
                lu64 *dummy = reinterpret_cast<lu64 *>(ring - 256) + (lane & 31);
                uint32_t got = !full   ? seg_lane<false, true, kSplit>(sym, raw, nb, st, qw)
                               : vec_esc ? seg_lane<true, true, kSplit>(sym, raw, nb, st, qw)
                                         : seg_lane<true, false, kSplit, kNoBr, kTwo>(sym, raw, nb, st, qw, dummy);
                if constexpr (SEGS == 2) {
                    const uint32_t nb1 = idx0 + 16 < comp_len ? min(comp_len - idx0 - 16, 16u) : 0u;
                    if (got != dl0 || (nb1 > 0 && st != entry1)) bad = true;
                    got = !full   ? seg_lane<false, true, kSplit>(sym, raw1, nb1, st, qw)
                          : vec_esc ? seg_lane<true, true, kSplit>(sym, raw1, nb1, st, qw)
                                    : seg_lane<true, false, kSplit>(sym, raw1, nb1, st, qw);
                }
                if (got != dl) bad = true;
                qw.finish();
            }
            wave_sync();
            out_pos += part;
            done += part;
            if (l1 == 64) break;
            retire(true);
            l0 = l1;
        }
        // a lane's exit state is the entry state of the segment after it
        const uint32_t nxt = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane + 1) & 63) << 2), (int)entry);
        if (lane < 63 && idx0 + 16 * SEGS < comp_len && st != nxt) bad = true;
        if (lane == 0 && entry != carry_lit) bad = true;
        carry_lit = rl(st, min(63u, (comp_len - 1 - r0) / (16 * SEGS)));
    }
    if (carry_lit) bad = true;  // stream ends inside an escape
    retire(true);
    if (next_str < nvals) {     // lengths claim more bytes than the stream holds
        bad = true;
        for (uint32_t i = next_str + lane; i < nvals; i += 64) *reinterpret_cast<ov4 *>(a.out + 16ull * i) = mk4(0, 0, 0, 0);
    }
    // zero the padding of the last block, then flush everything
    const uint32_t end = (out_pos + 15) & ~15u;
    if (lane < 16 && out_pos + lane < end) ring[out_pos - ring_base + lane] = 0;
    wave_sync();
    flush_ring(ring, Layout::kRing, ring_base, end, h, lane, bad);
    if (bad) atomicOr(err, KERR_FSST);
}

// ============================================================================
// 2. Code-parallel kernel (chunks without segment tables).
//
// A round is 512 consecutive compressed bytes of the vector's stream, 8 per
// lane (one 8 B load each, the next round's in flight): a lane looks up its
// codes' symbols (all table reads issued together), a wave scan turns the
// lanes' decoded lengths into output positions, and each lane ORs its symbols
// into the zeroed ring through a 64-bit accumulator OR-ed into its qword after
// every symbol (OR is idempotent: no select on whether the qword is complete;
// lanes sharing an edge qword merge).  The escape code (255: the next byte is
// a literal) makes a code's meaning depend on its predecessors; after any
// byte other than 0xFF the decoder is in the normal state, so a lane holding
// some non-0xFF byte leaves its bytes in a fixed state, and a lane's entry
// state is the exit state of the nearest earlier such lane (one ballot + one
// ds_bpermute per round).  Records are written for every string whose first
// bytes are decoded, after the next round's load.
// Chunks whose strings are all <= 255 bytes ("SMALL") keep u8 lengths, offsets
// from a wave scan as the records are made.
// ============================================================================
template <bool SMALL>
struct CpLds {
    static constexpr uint32_t kOffD = 0;
    static constexpr uint32_t kOffSym = SMALL ? 1024 : 4112;  // u8 lengths | u32 offsets x 1025
    static constexpr uint32_t kOffLen = kOffSym + 2048;
    static constexpr uint32_t kOffRing = kOffLen + 256;
    static constexpr uint32_t kPackedMax = SMALL ? 128 * 8 + 128 : 128 * 32 + 128;
    // 2 KiB holds a round's output at up to ~4 bytes per code; a round that
    // decodes to more is written in parts (lanes [l0, l1) at a time)
    static constexpr uint32_t kRing = kPackedMax > 2048 + 64 ? kPackedMax : 2048 + 64;
    static constexpr uint32_t kCap = kRing - 48;  // slack: qword ORs, the 32 B tail read
    static constexpr uint32_t kWave = kOffRing + kRing;
    static_assert(kOffSym % 16 == 0 && kOffRing % 16 == 0 && kWave % 16 == 0, "LDS layout alignment");
};
constexpr uint32_t kCpBytes = 8;   // compressed bytes per lane per round

// Appends symbols at ring byte wp through a 64-bit accumulator OR-ed into its
// aligned qword after every symbol (measured against OR-ing every symbol into
// both qwords it spans, fewer VALU and twice the ds_or_b64: 1-2 % faster).
struct QwordWriter {
    lu64 *o64;
    uint64_t acc;
    uint32_t q, bits;
    __device__ __forceinline__ QwordWriter(lu8 *ring, uint32_t wp)
        : o64(reinterpret_cast<lu64 *>(ring)), acc(0), q(wp >> 3), bits(8 * (wp & 7)) {}
    __device__ __forceinline__ void put(uint64_t v, uint32_t n) {  // n <= 8 bytes
        // v << bits spans qwords q (lo) and q + 1 (hi); (v >> 1) >> (63 - bits)
        // is v >> (64 - bits) without the bits == 0 case
        const uint64_t lo = v << bits, hi = (v >> 1) >> (63 - bits);
        acc |= lo;
        __hip_atomic_fetch_or(o64 + q, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t nb = bits + 8 * n;
        const bool e = nb >= 64;
        q += e ? 1u : 0u;
        acc = e ? hi : acc;
        bits = nb & 63;
    }
    __device__ __forceinline__ void finish() {
        __hip_atomic_fetch_or(o64 + q, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
};

// Escape state entering a lane's first code (the parity rule): the exit state
// of the nearest earlier lane holding a non-0xFF byte, or `carry` (the state
// the previous round ended in) when there is none.
__device__ __forceinline__ uint32_t entry_state(bool has_plain, uint32_t exit_if_plain, uint32_t carry, uint32_t lane) {
    const uint64_t m = __ballot(has_plain) & ((1ull << lane) - 1ull);  // lane 0: 0
    const uint32_t src = m ? 63u - (uint32_t)__builtin_clzll(m) : 0u;
    const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)exit_if_plain);
    return m ? v : carry;
}

// One round's codes of this lane (nb valid bytes of raw) from the escape state
// the previous round ended in (carry): the symbols v[k] and their byte counts
// n[k] (a literal is one byte, the escape code none -- its staged entry is
// {0, 0} -- and a symbol its length; nothing past the stream end; FULL = no
// lane of the round reaches it).  Returns the lane's byte count; st_out = the
// state after its last valid byte.
template <bool FULL>
__device__ __forceinline__ uint32_t cp_lane_codes(const lu64 *sym, const lu8 *len, const v4u &raw, uint32_t nb,
                                                  uint32_t carry, uint32_t lane, uint64_t (&v)[kCpBytes],
                                                  uint32_t (&n)[kCpBytes], uint32_t &st_out) {
    uint32_t code[kCpBytes], sl[kCpBytes];
    uint64_t sy[kCpBytes];
    int32_t last = -1;  // last non-0xFF byte of the lane's bytes
#pragma unroll
    for (uint32_t k = 0; k < kCpBytes; ++k) {  // all table reads issued together
        code[k] = byte_of(raw, k);
        sy[k] = sym[code[k]];
        sl[k] = len[code[k]];
        if ((FULL || k < nb) && code[k] != kFsstEscape) last = (int32_t)k;
    }
    const uint32_t end = FULL ? kCpBytes : nb;
    uint32_t st = entry_state(last >= 0, ((int32_t)end - 1 - last) & 1, carry, lane);
    uint32_t out = 0;
#pragma unroll
    for (uint32_t k = 0; k < kCpBytes; ++k) {
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

template <bool SMALL>
__device__ void cp_vector(lu8 *L, const DevChunk &c, const VecArgs &a, uint32_t lane, uint32_t *err) {
    using Layout = CpLds<SMALL>;
    lu8 *ring = L + Layout::kOffRing;
    lu32 *D = reinterpret_cast<lu32 *>(L + Layout::kOffD);
    const lu64 *sym = reinterpret_cast<const lu64 *>(L + Layout::kOffSym);
    const lu8 *len = L + Layout::kOffLen;
    const uint32_t nvals = a.nvals;
    bool bad = false;
    // ---- string lengths: u8 (SMALL) or exclusive u32 offsets ---------------
    const uint32_t W = SMALL ? min(a.W, 8u) : a.W;
    stage_packed(reinterpret_cast<lv4 *>(ring), a.packed, W, lane);
    uint32_t total = 0;
    if constexpr (SMALL) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t ci = lane + 64 * j;
            const v4u v = length_chunk(reinterpret_cast<lv4 *>(ring), W, a.base, nvals, ci);
            const uint32_t b0 = v.x & 255, b1 = v.y & 255, b2 = v.z & 255, b3 = v.w & 255;
            D[ci] = b0 | b1 << 8 | b2 << 16 | b3 << 24;
            run += b0 + b1 + b2 + b3;
        }
        total = rl(scan_incl(run), 63);
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t ci = lane + 64 * j;
            reinterpret_cast<lv4 *>(D)[ci] = length_chunk(reinterpret_cast<lv4 *>(ring), W, a.base, nvals, ci);
        }
        wave_sync();
        uint32_t o[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u v = reinterpret_cast<const lv4 *>(D)[4 * lane + q];
            o[4 * q] = v.x; o[4 * q + 1] = v.y; o[4 * q + 2] = v.z; o[4 * q + 3] = v.w;
        }
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t t = o[k];
            o[k] = run;
            run += t;
        }
        const uint32_t incl = scan_incl(run);
        const uint32_t excl = incl - run;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            reinterpret_cast<lv4 *>(D)[4 * lane + q] = mk4(excl + o[4 * q], excl + o[4 * q + 1], excl + o[4 * q + 2], excl + o[4 * q + 3]);
        if (lane == 63) D[1024] = incl;
        total = rl(incl, 63);
    }
    wave_sync();
    if (total != a.dbytes) bad = true;
    for (uint32_t q = lane; q < Layout::kRing / 16; q += 64) reinterpret_cast<lv4 *>(ring)[q] = mk4(0, 0, 0, 0);
    wave_sync();

    const VecHeap h = vec_heap(c, a);
    const uint32_t comp_len = h.comp_len;
    gv4 *comp = reinterpret_cast<gv4 *>(a.vh + sizeof(FsstVecHeader) + 128 * h.clen_w);
    uint32_t out_pos = 0, ring_base = 0, carry_lit = 0, next_str = 0, str_base = 0;
    // string_t records of every string whose first min(n, 12) bytes are decoded
    auto records = [&]() {
        while (next_str < nvals) {
            const uint32_t i = next_str + lane;
            uint32_t d0 = 0, n = 0, incl = 0;
            if constexpr (SMALL) {
                n = i < nvals ? (uint32_t)reinterpret_cast<const lu8 *>(D)[i] : 0u;
                incl = scan_incl(n);
                d0 = str_base + incl - n;
            } else if (i < nvals) {
                d0 = D[i];
                n = D[i + 1] - d0;
            }
            const bool ok = i < nvals && d0 + min(n, 12u) <= out_pos;
            const uint32_t n_ok = leading_ok(__ballot(ok));
            if (lane < n_ok) {
                const lu32 *r32 = reinterpret_cast<const lu32 *>(ring);
                const uint32_t x = d0 - ring_base, i0 = x >> 2;
                *reinterpret_cast<ov4 *>(a.out + 16ull * i) =
                    make_record(r32[i0], r32[i0 + 1], r32[i0 + 2], r32[i0 + 3], x & 3, n, h.ptr_base + d0);
            }
            if constexpr (SMALL) {
                if (n_ok > 0) str_base += rl(incl, n_ok - 1);
            }
            next_str += n_ok;
            if (n_ok < 64) break;
        }
        if constexpr (!SMALL) str_base = next_str < nvals ? uni(D[next_str]) : out_pos;
    };
    // records, complete 16 B blocks to the heap, the unfinished tail (< 32 B)
    // to the ring start (the bytes it vacates back to zero)
    auto retire = [&]() {
        records();
        const uint32_t keep_from = next_str < nvals ? min(str_base, out_pos) : out_pos;
        const uint32_t new_base = keep_from & ~15u;
        flush_ring(ring, Layout::kRing, ring_base, new_base, h, lane, bad);
        wave_sync();
        const uint32_t src = (new_base - ring_base) >> 2;
        uint32_t t = 0;
        if (lane < 8) t = reinterpret_cast<const lu32 *>(ring)[src + lane];
        wave_sync();
        if (lane < 8) reinterpret_cast<lu32 *>(ring)[lane] = t;
        if (lane < 8 && src + lane >= 8) reinterpret_cast<lu32 *>(ring)[src + lane] = 0;
        ring_base = new_base;
        wave_sync();
    };
    constexpr uint32_t kRound = 64 * kCpBytes;
    // a lane's compressed bytes of the round starting at r0 (zeros past the end)
    auto load_raw = [&](uint32_t r0) -> v4u {
        v4u x = mk4(0, 0, 0, 0);
        if (r0 + kCpBytes * lane < comp_len) {  // one dwordx2 load (the stream is 16 B aligned)
            const v2u q = reinterpret_cast<const FLS_GLOBAL v2u *>(comp)[(r0 >> 3) + lane];
            x = mk4(q.x, q.y, 0, 0);
        }
        return x;
    };
    v4u raw_next = load_raw(0);
    for (uint32_t r0 = 0; r0 < comp_len; r0 += kRound) {
        const uint32_t idx0 = r0 + kCpBytes * lane;
        const uint32_t nb = idx0 < comp_len ? min(comp_len - idx0, kCpBytes) : 0u;
        const v4u raw = raw_next;  // the next round's bytes load while this one decodes
        if (r0 + kRound < comp_len) raw_next = load_raw(r0 + kRound);
        const bool full = r0 + kRound <= comp_len;
        // the previous round's stores go out now, after this round's load was
        // issued and a whole decode before the next wait (vmcnt counts loads
        // and stores in issue order)
        if (r0 > 0) retire();
        uint32_t n[kCpBytes], lane_end = 0;
        uint64_t v[kCpBytes];
        const uint32_t lane_out = full ? cp_lane_codes<true>(sym, len, raw, nb, carry_lit, lane, v, n, lane_end)
                                       : cp_lane_codes<false>(sym, len, raw, nb, carry_lit, lane, v, n, lane_end);
        const uint32_t incl = scan_incl(lane_out);
        // the lanes whose output fits the ring, then retire() and the rest
        // (a lane writes <= 8 x 8 bytes)
        uint32_t l0 = 0, done = 0;
        for (;;) {
            const uint32_t p0 = out_pos - ring_base;
            const bool fits = lane < l0 || p0 + (incl - done) <= Layout::kCap;
            const uint32_t l1 = leading_ok(__ballot(fits));
            const uint32_t part = rl(incl, l1 - 1) - done;
            wave_sync();
            if (lane >= l0 && lane < l1) {
                QwordWriter qw(ring, p0 + (incl - lane_out - done));
#pragma unroll
                for (uint32_t k = 0; k < kCpBytes; ++k) qw.put(v[k], n[k]);
                qw.finish();
            }
            wave_sync();
            out_pos += part;
            done += part;
            if (l1 == 64) break;
            retire();
            l0 = l1;
        }
        // state after the round's last valid byte (lane 63 unless the stream ends here)
        carry_lit = rl(lane_end, min(63u, (comp_len - 1 - r0) / kCpBytes));
    }
    if (carry_lit) bad = true;  // stream ends inside an escape
    retire();
    if (next_str < nvals) {     // lengths claim more bytes than the stream holds
        bad = true;
        for (uint32_t i = next_str + lane; i < nvals; i += 64) *reinterpret_cast<ov4 *>(a.out + 16ull * i) = mk4(0, 0, 0, 0);
    }
    const uint32_t end = (out_pos + 15) & ~15u;
    if (lane < 16 && out_pos + lane < end) ring[out_pos - ring_base + lane] = 0;
    wave_sync();
    flush_ring(ring, Layout::kRing, ring_base, end, h, lane, bad);
    if (bad) atomicOr(err, KERR_FSST);
}

// ============================================================================
// Work distribution of the segmented and code-parallel kernels.  Standalone
// launches: contiguous vector ranges per wave (a wave mostly stays inside one
// chunk and stages its symbol table once).  Overlapped launches (queue !=
// nullptr, FsstLaunch::queue): pieces of `piece` consecutive vectors from a
// counter shared by the narrow grid that runs beside the main decode kernel
// and the full grid that follows it, one atomic per piece, so no vector is
// decoded twice and late waves find work (a piece queue for standalone
// launches measured 2-4 % slower on l_comment: more table reloads).  The piece
// loop is the range loop's own (a loop around the range decoder needed 98-124
// VGPRs instead of 82).  Every wave reaches the exit: the range ends, the
// chunks run out, or the queue is empty.
// LDS is addressed with plain integers from 0 (the kernels have no static LDS,
// so their dynamic LDS starts at address 0, checked at entry and at launch):
// table and ring offsets fold into the DS instructions' offset fields instead
// of adding the dynamic-LDS symbol to every address (1.2 % on l_comment,
// profiles/r2/abenv_fsst_abslds.txt).
// ============================================================================
enum class Kind { Seg, Cp };
constexpr uint32_t kHalving = 0x80000000u;  // fsst_range's piece: halving piece sizes

// Items [item0, item1) first, then (QUEUE) pieces of `piece` items from
// `queue`: piece p = [qbase + p * piece, ...) up to nitems.  A queue launch
// may pass an empty first range (then the first piece comes from the queue).
template <Kind K, bool SMALL, bool QUEUE, int X = 0>
__device__ __forceinline__ void fsst_range(const DevChunk *chunks, uint32_t nchunks, uint32_t nitems, uint32_t item0,
                                           uint32_t item1, uint32_t *queue, uint32_t piece, lu8 *L, uint32_t *err,
                                           uint32_t qbase = 0) {
    chunks = uni_ptr(chunks);
    err = uni_ptr(err);
    nchunks = uni(nchunks);
    qbase = uni(qbase);
    const uint32_t lane = __lane_id();
    // next piece of the queue into [item0, item1); false when none is left
    // piece & kHalving: pieces of (piece & 0xFFFF) vectors over the first
    // half of the queue's items, half that over the next quarter, ... down to
    // single vectors (few table stagings early, a fine-grained end)
    auto take = [&]() -> bool {
        uint32_t p = 0;
        if (lane == 0) p = atomicAdd(queue, 1u);
        p = rl(p, 0);
        if (qbase >= nitems) return false;
        if (!(piece & kHalving)) {
            if (p >= (nitems - qbase + piece - 1) / piece) return false;
            item0 = qbase + p * piece;
            item1 = min(item0 + piece, nitems);
            return true;
        }
        uint32_t base = qbase, rem = nitems - qbase, ps = max(1u, piece & 0xFFFFu);
        for (;;) {
            const uint32_t span = ps > 1 ? max(1u, rem / 2) : rem;
            const uint32_t cnt = (span + ps - 1) / ps;
            if (p < cnt) {
                item0 = base + p * ps;
                item1 = min(item0 + ps, base + span);
                return true;
            }
            p -= cnt;
            base += span;
            rem -= span;
            if (ps == 1 || rem == 0) return false;
            ps >>= 1;
        }
    };
    if constexpr (QUEUE) {
        if (uni(item0) >= uni(item1) && !take()) return;
    }
    item0 = uni(item0);
    item1 = uni(item1);
    constexpr uint32_t kOffSym = K == Kind::Seg ? SegLds<SMALL, X>::kOffSym : CpLds<SMALL>::kOffSym;
    lu64 *sym = reinterpret_cast<lu64 *>(L + kOffSym);
    uint32_t ci = chunk_of(chunks, nchunks, item0);
    DevChunk c = load_chunk(chunks, ci);
    bool have_table = false;
    for (uint32_t item = item0;;) {
        if (item >= item1) {
            if constexpr (!QUEUE) break;
            if (!take()) break;
            item = item0;
            // the next piece is usually far ahead (the other waves took the
            // ones between): find its chunk instead of walking there
            if (item - uni(c.vec_base) >= uni(c.nvec)) {
                ci = chunk_of(chunks, nchunks, item);
                c = load_chunk(chunks, ci);
                have_table = false;
            }
        }
        const uint32_t v = item - uni(c.vec_base);
        if (v >= uni(c.nvec)) {  // next chunk
            if (++ci >= nchunks) break;
            c = load_chunk(chunks, ci);
            have_table = false;
            continue;
        }
        if (!have_table) {
            gu8 *aux = gptr(c.chunk) + c.aux_off;
            if constexpr (K == Kind::Seg) stage_table<true, (X & kSegXSplit) != 0>(aux, sym, nullptr, lane, err);
            else stage_table<false>(aux, sym, L + CpLds<SMALL>::kOffLen, lane, err);
            have_table = true;
        }
        const VecArgs a = vec_args(c, v);
#ifdef FLS_WAVE_TRACE
        const uint64_t tr0 = wall_clock64();
#endif
        if constexpr (K == Kind::Seg) seg_vector<SMALL, X>(L, sym, c, a, lane, err);
        else cp_vector<SMALL>(L, c, a, lane, err);
        wave_sync();
#ifdef FLS_WAVE_TRACE
        // (timing build) one record per FSST vector: shape enc 0xFE, ob 0,
        // max_w = its bytes / 128 (records + heap + compressed, estimated)
        const uint64_t tr1 = wall_clock64();
        if (lane == 0) {
            const uint32_t i = atomicAdd(&dec::g_trace_n, 1u);
            if (i < dec::kTraceCap) {
                dec::TraceRec &r = dec::g_trace[i];
                r.t0 = tr0;
                r.t1 = tr1;
                r.wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
                r.vr = item;
                r.hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);
                r.xcc_id = __builtin_amdgcn_s_getreg((31 << 11) | 20);
                r.shape = 0xFEu | 1u << 24;
                r.max_w = (16u * 1024u + a.dbytes + a.dbytes / 2) / 128u;
            }
        }
#endif
        ++item;
    }
}

// register budgets: the segmented kernel 5 waves per SIMD (96 VGPRs, no
// spill; its LDS admits 16 waves per CU), the code-parallel one 6 (80 VGPRs)
template <Kind K, bool SMALL, bool QUEUE, int X = 0>
__global__ __launch_bounds__(64, K == Kind::Seg ? ((X & kSegXDouble) ? 4 : 5) : 6) void fsst_kernel(const DevChunk *__restrict__ chunks,
                                                                         uint32_t nchunks, uint32_t nitems,
                                                                         uint32_t *__restrict__ err,
                                                                         uint32_t *__restrict__ queue, uint32_t piece) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    if ((uint32_t)(size_t)lds_raw != 0u) {  // LDS addressed from 0 (see above)
        if (threadIdx.x == 0) atomicOr(err, KERR_LDS_BASE);
        return;
    }
    uint32_t i0 = 0, i1 = 0;
    if (!QUEUE) {
        const uint32_t nwaves = gridDim.x, wave = blockIdx.x;
        const uint32_t per = (nitems + nwaves - 1) / nwaves;
        i0 = min(wave * per, nitems);
        i1 = min(i0 + per, nitems);
        if (i0 >= i1) return;
    }
    fsst_range<K, SMALL, QUEUE, X>(chunks, nchunks, nitems, i0, i1, queue, piece, (lu8 *)(size_t)0, err);
}

template <Kind K, bool SMALL, bool QUEUE, int X = 0>
hipError_t launch_kind(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err, hipStream_t stream,
                       const FsstLaunch &how) {
    const uint32_t shmem = K == Kind::Seg ? SegLds<SMALL, X>::kWave : CpLds<SMALL>::kWave;
    auto kern = fsst_kernel<K, SMALL, QUEUE, X>;
    // the kernel addresses its dynamic LDS from 0, which holds only without
    // static LDS: refuse to launch one that has some
    static const bool lds_at_zero = [kern] {
        hipFuncAttributes a{};
        return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(kern)) == hipSuccess && a.sharedSizeBytes == 0;
    }();
    if (!lds_at_zero) {
        fprintf(stderr, "fsst_kernel: static LDS present or attributes unavailable; cannot address LDS from 0\n");
        return hipErrorInvalidDeviceFunction;
    }
    int cus = device_cus(), per_cu = occupancy(reinterpret_cast<const void *>(kern), 64, shmem);
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
        fprintf(stderr, "DEBUG: fsst_kernel<%d,%s%s>: %d blocks of 1 wave (%d per CU, %u B LDS), %u vectors%s\n",
                K == Kind::Seg ? 16 : 8, SMALL ? "small" : "any", K == Kind::Seg ? ",seg" : "", grid, per_cu, shmem,
                nvecs, how.queue ? " (piece queue)" : "");
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), shmem, stream, d_chunks, nchunks, nvecs, d_err, how.queue, piece);
    return hipGetLastError();
}
template <Kind K, int X = 0>
hipError_t launch_kind2(const DevChunk *d, uint32_t nchunks, uint32_t nvecs, uint32_t *err, hipStream_t stream,
                        const FsstLaunch &how) {
    if (how.queue) return how.small ? launch_kind<K, true, true, X>(d, nchunks, nvecs, err, stream, how)
                                    : launch_kind<K, false, true, X>(d, nchunks, nvecs, err, stream, how);
    return how.small ? launch_kind<K, true, false, X>(d, nchunks, nvecs, err, stream, how)
                     : launch_kind<K, false, false, X>(d, nchunks, nvecs, err, stream, how);
}

// ============================================================================
// 4. Fused kernel: the main decode (fls_decode_dev.hpp) and the segmented FSST
// decode in ONE launch of 1-wave blocks.  The main decode is HBM-bound and
// the FSST decode VALU / LDS-bound, so they share each CU better than either
// runs alone; run one after the other, each kernel's tail idles the CUs and
// the second kernel waits for the first one's drain.  Every wave pulls from
// two queues: whole main chunks (the host's largest-output-first order) and
// FSST pieces of `piece` vectors; fsst_per16 of every 16 waves start on the
// FSST queue, the rest on the main one, and a wave whose queue runs dry
// moves to the other, so both end together whatever the mix.  LDS per wave:
// the larger of the two kernels' (dynamic LDS from address 0, as the FSST
// code addresses it), registers: the main decode's budget (4 waves / SIMD).
// ============================================================================
// The FSST part out of line: its own register allocation, as the main
// decode's paths have theirs (run_chunk); arguments arrive in VGPRs and are
// made uniform again inside (fsst_range).
template <bool SMALL, int X>
__device__ __attribute__((noinline)) void fused_fsst_part(const DevChunk *fchunks, uint32_t nfsst, uint32_t nfvecs,
                                                          uint32_t item0, uint32_t item1, uint32_t *queue,
                                                          uint32_t piece, uint32_t qbase, uint32_t *err) {
    fsst_range<Kind::Seg, SMALL, true, X>(fchunks, nfsst, nfvecs, uni(item0), uni(item1), uni_ptr(queue), uni(piece),
                                          (lu8 *)(size_t)0, err, uni(qbase));
}

template <bool SMALL, int X = 0, bool RATING = false>
__global__ __launch_bounds__(64, 4) void fused_kernel(const DevChunk *__restrict__ mchunks, uint32_t nmain,
                                                      const DevChunk *__restrict__ fchunks, uint32_t nfsst,
                                                      uint32_t nfvecs, uint32_t *__restrict__ err,
                                                      uint32_t *__restrict__ queues, uint32_t p_bytes,
                                                      uint32_t v_bytes, uint32_t piece, uint32_t fsst_per16,
                                                      uint32_t fsst_static, uint32_t nf_waves, uint32_t nwhole,
                                                      uint32_t tsplit) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    if ((uint32_t)(size_t)lds_raw != 0u) {  // LDS addressed from 0 (fsst_kernel)
        if (threadIdx.x == 0) atomicOr(err, KERR_LDS_BASE);
        return;
    }
    // every wave's first item is static (no burst of same-address atomics at
    // launch): main-first wave m takes main chunk m (the queue starts past
    // them), FSST-first wave f the f-th equal share of the first fsst_static
    // FSST vectors (the queue's pieces start after those)
    const uint32_t b = blockIdx.x, k = fsst_per16, grp = b >> 4, r = b & 15;
    const bool fsst_first = r < k;
    // main items: chunks [0, nwhole) whole, then each later chunk as tsplit
    // pieces (FusedLaunch::tail_chunks / tail_split)
    const uint32_t nitems = nwhole + (nmain - nwhole) * tsplit;
    auto main_part = [&](bool first) {
        uint32_t it = first ? grp * (16 - k) + (r - k) : 0u;
        for (;; first = false) {
            if (!first) {
                if (__lane_id() == 0) it = atomicAdd(queues, 1u);
                it = uni(it);
            }
            if (it >= nitems) {
                if (first) continue;  // (fewer main items than waves: the queue is empty too)
                break;
            }
            uint32_t ci = it, p = 0;
            if (it >= nwhole) {
                ci = nwhole + (it - nwhole) / tsplit;
                p = (it - nwhole) % tsplit;
            }
            const uint32_t nvec = gptr(mchunks)[ci].nvec;
            const uint32_t vb = it >= nwhole ? nvec * p / tsplit : 0u, ve = it >= nwhole ? nvec * (p + 1) / tsplit : nvec;
            if (vb < ve) dec::decode_chunk(mchunks + ci, 0u, p_bytes, v_bytes, err, vb | ve << 8);
        }
    };
    auto fsst_part = [&](bool first) {
        uint32_t i0 = 0, i1 = 0;
        if (first) {
            const uint32_t f = grp * k + r;
            i0 = (uint32_t)((uint64_t)fsst_static * f / nf_waves);
            i1 = (uint32_t)((uint64_t)fsst_static * (f + 1) / nf_waves);
        }
        if (nfsst) fused_fsst_part<SMALL, X>(fchunks, nfsst, nfvecs, i0, i1, queues + 1, piece, fsst_static, err);
        wave_sync();
    };
    const bool stat = nf_waves != 0;  // 0: every item from the queues (FusedLaunch::static_first)
    if (fsst_first) {
        fsst_part(stat);
        main_part(false);
    } else {
        main_part(stat);
        fsst_part(false);
    }
}

template <bool SMALL, int X = 0>
hipError_t launch_fused_t(const DevChunk *d_main, uint32_t nmain, const DevChunk *d_fsst, uint32_t nfsst,
                          uint32_t nfvecs, uint32_t *d_err, const DecodeGeom &geom, hipStream_t stream,
                          uint32_t *d_queues, const FusedLaunch &how) {
    // (the rating instantiation: the same code under another name, rating_launch())
    auto kern = rating_launch() ? fused_kernel<SMALL, X, true> : fused_kernel<SMALL, X, false>;
    const uint32_t shmem = std::max<uint32_t>(geom.p_bytes + geom.v_bytes, SegLds<SMALL>::kWave);
    static const bool lds_at_zero = [] {
        auto zero = [](auto k) {
            hipFuncAttributes a{};
            return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(k)) == hipSuccess && a.sharedSizeBytes == 0;
        };
        return zero(fused_kernel<SMALL, X, false>) && zero(fused_kernel<SMALL, X, true>);
    }();
    if (!lds_at_zero) return hipErrorInvalidDeviceFunction;
    const int cus = device_cus();
    int per_cu = occupancy(reinterpret_cast<const void *>(kern), 64, shmem);
    if (how.waves_per_cu > 0) per_cu = std::min(per_cu, how.waves_per_cu);
    const int grid = cus * std::max(1, per_cu);
    // waves starting on each queue (blockIdx & 15 < k: FSST first), and the
    // static first items: main chunk m of main-first wave m, the first
    // fsst_static_pct % of the FSST vectors split over the FSST-first waves
    const uint32_t k = std::min(16u, how.fsst_per16);
    uint32_t nf = 0;
    for (int bb = 0; bb < grid; ++bb) nf += (uint32_t)(bb & 15) < k;
    const uint32_t nm = (uint32_t)grid - nf;
    const bool stat = how.static_first;
    const uint32_t tsplit = std::max(1u, std::min(64u, how.tail_split));
    const uint32_t nwhole = tsplit > 1 ? nmain - std::min(nmain, how.tail_chunks) : nmain;
    const uint32_t nitems = nwhole + (nmain - nwhole) * tsplit;
    const uint32_t fstat = stat && nf ? (uint32_t)((uint64_t)nfvecs * std::min(100u, how.fsst_static_pct) / 100) : 0u;
    hipError_t e = hipMemsetD32Async((hipDeviceptr_t)d_queues, stat ? std::min(nm, nitems) : 0u, 1, stream);
    if (e == hipSuccess) e = hipMemsetD32Async((hipDeviceptr_t)(d_queues + 1), 0, 1, stream);
    if (e != hipSuccess) return e;
    if (getenv("FLS_DEBUG"))
        fprintf(stderr, "DEBUG: fused_kernel<%s>: %d blocks of 1 wave (%d per CU, %u B LDS), %u main chunks, %u FSST "
                        "vectors in pieces of %u, %u of 16 waves FSST first\n",
                SMALL ? "small" : "any", grid, per_cu, shmem, nmain, nfvecs, how.piece, how.fsst_per16);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), shmem, stream, d_main, nmain, d_fsst, nfsst, nfvecs, d_err,
                       d_queues, geom.p_bytes, geom.v_bytes, std::max(1u, std::min(64u, how.piece)) | (how.halving ? kHalving : 0u),
                       k, fstat, stat ? std::max(1u, nf) : 0u, nwhole, tsplit);
    return hipGetLastError();
}

// ============================================================================
// 3. String-parallel kernel (chunks whose strings are all <= 255 bytes, both
// decompressed and compressed: the host marks them, DevChunk.vbits = 1;
// FLS_DECODE_POLICY bit 7).  Every string is compressed on its own and the
// vector stores the strings' compressed lengths, so lane j decodes string
// s + j of a round by itself: no escape-state composition, no per-code wave
// scans.  Per vector:
//   1. both length streams (FFOR, W <= 8) are unpacked into u8 arrays;
//   2. rounds of up to 64 strings (as many as fit the LDS rings: inclusive
//      wave scans of the lengths + ballot): the round's compressed bytes are
//      staged into the IN ring with 16 B coalesced loads, the OUT ring's
//      dwords for the round are zeroed, then every lane walks its string 4
//      codes at a time (one unaligned dword of codes, the 4 symbol / length
//      lookups issued together) and ORs the symbols into OUT as aligned
//      qwords (a string's edge qwords are shared with its neighbours);
//   3. the round's string_t records (64 x 16 B) and the complete 16 B blocks
//      of OUT go to HBM; the unfinished tail (< 16 B) moves to the ring start.
// It measured slower than the code-parallel kernel on l_comment (lanes idle on
// short strings: profiles/r1/fsst_sp_sq_counters.txt) and stays as a policy.
// ============================================================================
constexpr uint32_t kSpIncap = 1536;   // IN ring: compressed bytes of a round (+16 B slack)
constexpr uint32_t kSpOutcap = 2560;  // OUT ring: decoded bytes of a round incl. the carried tail
constexpr uint32_t kSpSym = 0, kSpLen = 2048, kSpDL = 2304, kSpCL = kSpDL + 1024, kSpIn = kSpCL + 1024;
constexpr uint32_t kSpOut = kSpIn + kSpIncap + 16;
constexpr uint32_t kSpWave = kSpOut + kSpOutcap + 16;
static_assert(kSpIncap >= 128 * 8 + 128 && kSpIncap >= 255 + 16 && kSpOutcap >= 255 + 16, "SP ring sizes");
static_assert(kSpIn % 16 == 0 && kSpOut % 16 == 0 && kSpWave % 16 == 0, "SP LDS layout alignment");

struct SpWave {
    const lu64 *sym;
    const lu8 *len;
    lu8 *DL, *CL, *IN, *OUT;
};

// u8 lengths of the vector (base + FFOR(T=32, W <= 8), zero past nvals); the
// packed bits are staged in the IN ring
__device__ __forceinline__ void unpack_u8(const SpWave &w, gu8 *packed, uint32_t W, uint32_t base, uint32_t nvals,
                                          lu8 *dst, uint32_t lane) {
    lv4 *P = reinterpret_cast<lv4 *>(w.IN);
    stage_packed(P, packed, W, lane);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t ci = lane + 64 * j;
        const v4u v = length_chunk(P, W, base, nvals, ci);
        reinterpret_cast<lu32 *>(dst)[ci] = (v.x & 255) | (v.y & 255) << 8 | (v.z & 255) << 16 | (v.w & 255) << 24;
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
// uniform) 4 codes per step and every lane predicates its codes with selects
// (divergent control flow cost more scalar exec-mask instructions than the
// decode itself); the accumulator is OR-ed into its qword every step.
// Returns false on corrupt input (wrong byte count, truncated escape).
__device__ __forceinline__ bool sp_decode(const SpWave &w, uint32_t cb, uint32_t cl, uint32_t wp, uint32_t dl,
                                          uint32_t maxcl) {
    const lu32 *in32 = reinterpret_cast<const lu32 *>(w.IN);
    lu64 *o64 = reinterpret_cast<lu64 *>(w.OUT);
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
            const uint64_t lo = v << bits, hi = (v >> 1) >> (63 - bits);
            acc |= lo;
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

__device__ void sp_vector(const SpWave &w, const DevChunk &c, const VecArgs &a, uint32_t lane, uint32_t *err) {
    const FLS_GLOBAL FsstVecHeader *hp = reinterpret_cast<const FLS_GLOBAL FsstVecHeader *>(a.vh);
    const uint32_t cbase = uni(hp->clen_base), cw = uni(min(hp->clen_w, 8u));
    const VecHeap h = vec_heap(c, a);
    const uint32_t comp_len = h.comp_len, nvals = a.nvals;
    bool bad = false;
    gv4 *cs = reinterpret_cast<gv4 *>(a.vh + sizeof(FsstVecHeader) + 128 * cw);
    const uint32_t lim16 = (comp_len + 15) >> 4;
    lu32 *o32 = reinterpret_cast<lu32 *>(w.OUT);
    lv4 *in16 = reinterpret_cast<lv4 *>(w.IN);
    const lv4 *out16 = reinterpret_cast<const lv4 *>(w.OUT);
    // stream complete 16 B blocks [ring_base, upto) of OUT to the heap
    auto flush = [&](uint32_t ring_base, uint32_t upto) {
        const uint32_t nblk = (upto - ring_base) >> 4;
        for (uint32_t q = lane; q < nblk; q += 64) {
            const uint32_t g = ring_base + 16 * q;
            if (g + 16 <= h.hlim) *reinterpret_cast<ov4 *>(h.heap + g) = out16[q];
            else bad = true;
        }
    };
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
    unpack_u8(w, a.packed, min(a.W, 8u), a.base, nvals, w.DL, lane);
    unpack_u8(w, a.vh + sizeof(FsstVecHeader), cw, cbase, nvals, w.CL, lane);
    uint32_t s = 0, dpos = 0, cpos = 0, ring_base = 0;
    while (s < nvals) {
        const uint32_t i = s + lane;
        const uint32_t dl = i < nvals ? (uint32_t)w.DL[i] : 0u, cl = i < nvals ? (uint32_t)w.CL[i] : 0u;
        const uint32_t dinc = scan_incl(dl), cinc = scan_incl(cl);
        const uint32_t tail = dpos - ring_base, cskew = cpos & 15;
        const bool fits = i < nvals && tail + dinc <= kSpOutcap && cskew + cinc <= kSpIncap;
        const uint32_t nr = leading_ok(__ballot(fits));  // >= 1: one string always fits
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
        if (lane < nr) {
            const lu32 *r32 = reinterpret_cast<const lu32 *>(w.OUT);
            const uint32_t i0 = wp >> 2;
            *reinterpret_cast<ov4 *>(a.out + 16ull * i) =
                make_record(r32[i0], r32[i0 + 1], r32[i0 + 2], r32[i0 + 3], wp & 3, dl, h.ptr_base + (dpos + dinc - dl));
        }
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
    if (dpos != a.dbytes || cpos != comp_len) bad = true;
    // zero the padding of the last block, then flush it
    const uint32_t end = (dpos + 15) & ~15u;
    if (lane < 16 && dpos + lane < end) w.OUT[dpos - ring_base + lane] = 0;
    wave_sync();
    flush(ring_base, end);
    if (bad) atomicOr(err, KERR_FSST);
}

__global__ __launch_bounds__(64) void fsst_sp_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                      uint32_t nitems, uint32_t *__restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    const uint32_t nwaves = gridDim.x, wave = blockIdx.x;
    const uint32_t per = (nitems + nwaves - 1) / nwaves;
    const uint32_t item0 = uni(min(wave * per, nitems)), item1 = uni(min(item0 + per, nitems));
    if (item0 >= item1) return;
    nchunks = uni(nchunks);
    const uint32_t lane = __lane_id();
    lu8 *L = (lu8 *)(size_t)(uint32_t)(size_t)lds_raw;
    SpWave w;
    w.sym = reinterpret_cast<const lu64 *>(L + kSpSym);
    w.len = L + kSpLen;
    w.DL = L + kSpDL;
    w.CL = L + kSpCL;
    w.IN = L + kSpIn;
    w.OUT = L + kSpOut;
    uint32_t ci = chunk_of(chunks, nchunks, item0);
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
        if (!have_table) {
            stage_table<false>(gptr(c.chunk) + c.aux_off, reinterpret_cast<lu64 *>(L + kSpSym), L + kSpLen, lane, err);
            have_table = true;
        }
        sp_vector(w, c, vec_args(c, v), lane, err);
        wave_sync();
        ++item;
    }
}

}  // namespace

hipError_t launch_fsst_sp(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                          hipStream_t stream) {
    if (nchunks == 0 || nvecs == 0) return hipSuccess;
    const int cus = device_cus(), per_cu = occupancy(reinterpret_cast<const void *>(fsst_sp_kernel), 64, kSpWave);
    const int grid = std::min<int>(cus * std::max(1, per_cu), (int)nvecs);
    if (getenv("FLS_DEBUG"))
        fprintf(stderr, "DEBUG: fsst_sp_kernel: %d blocks of 1 wave (%d per CU, %u B LDS), %u vectors\n", grid, per_cu,
                kSpWave, nvecs);
    hipLaunchKernelGGL(fsst_sp_kernel, dim3(grid), dim3(64), kSpWave, stream, d_chunks, nchunks, nvecs, d_err);
    return hipGetLastError();
}

bool fsst_variant_built(int variant, bool seg, int bytes_per_lane) {
    if (seg || bytes_per_lane == 8) {
        if (variant == kFsstDefault) return true;  // the product build has each kernel's default only
#ifdef FLS_EXPERIMENTS
        const int x = variant >> kSegXShift;
        if ((variant & ((1 << kSegXShift) - 1)) == kFsstDefault &&
            ((x >= 1 && x <= 9) || x == 16 || x == 32 || x == 48 || x == 64 || x == 128 || x == 256))
            return true;
#endif
    }
    return false;
}

bool fused_x_built(int x) {
    if (x == 0) return true;
#ifdef FLS_EXPERIMENTS
    return x == (kSegXFlush | kSegXRecSel) || x == kSegXTwo || x == kSegXNoBranch;
#else
    return false;
#endif
}

hipError_t launch_fused(const DevChunk *d_main, uint32_t nmain, const DevChunk *d_fsst, uint32_t nfsst,
                        uint32_t nfvecs, bool small, uint32_t *d_err, const DecodeGeom &geom, hipStream_t stream,
                        uint32_t *d_queues, const FusedLaunch &how) {
    if (nmain == 0 && nfsst == 0) return hipSuccess;
#ifdef FLS_EXPERIMENTS
    // (experiment library) the FSST part's segmented-kernel bits, FusedLaunch::x
    if (how.x == (kSegXFlush | kSegXRecSel))
        return small ? launch_fused_t<true, kSegXFlush | kSegXRecSel>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom,
                                                                       stream, d_queues, how)
                     : launch_fused_t<false, kSegXFlush | kSegXRecSel>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom,
                                                                        stream, d_queues, how);
    if (how.x == kSegXTwo)
        return small ? launch_fused_t<true, kSegXTwo>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom, stream,
                                                      d_queues, how)
                     : launch_fused_t<false, kSegXTwo>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom, stream,
                                                       d_queues, how);
    if (how.x == kSegXNoBranch)
        return small ? launch_fused_t<true, kSegXNoBranch>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom, stream,
                                                           d_queues, how)
                     : launch_fused_t<false, kSegXNoBranch>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom, stream,
                                                            d_queues, how);
#endif
    if (how.x != 0) return hipErrorInvalidValue;
    return small ? launch_fused_t<true>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom, stream, d_queues, how)
                 : launch_fused_t<false>(d_main, nmain, d_fsst, nfsst, nfvecs, d_err, geom, stream, d_queues, how);
}

hipError_t launch_fsst(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                       hipStream_t stream, const FsstLaunch &how) {
    if (nchunks == 0 || nvecs == 0) return hipSuccess;
    if (!fsst_variant_built(how.variant, how.seg, how.bytes_per_lane)) return hipErrorInvalidValue;
    if (!how.seg) return launch_kind2<Kind::Cp>(d_chunks, nchunks, nvecs, d_err, stream, how);
#ifdef FLS_EXPERIMENTS
    switch (how.variant >> kSegXShift) {
    case 1: return launch_kind2<Kind::Seg, 1>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 2: return launch_kind2<Kind::Seg, 2>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 3: return launch_kind2<Kind::Seg, 3>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 4: return launch_kind2<Kind::Seg, 4>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 5: return launch_kind2<Kind::Seg, 5>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 6: return launch_kind2<Kind::Seg, 6>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 7: return launch_kind2<Kind::Seg, 7>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 8: return launch_kind2<Kind::Seg, 8>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 9: return launch_kind2<Kind::Seg, 9>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 16: return launch_kind2<Kind::Seg, 16>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 32: return launch_kind2<Kind::Seg, 32>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 48: return launch_kind2<Kind::Seg, 48>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 64: return launch_kind2<Kind::Seg, 64>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 128: return launch_kind2<Kind::Seg, 128>(d_chunks, nchunks, nvecs, d_err, stream, how);
    case 256: return launch_kind2<Kind::Seg, 256>(d_chunks, nchunks, nvecs, d_err, stream, how);
    default: break;
    }
#endif
    return launch_kind2<Kind::Seg>(d_chunks, nchunks, nvecs, d_err, stream, how);
}

#ifdef FLS_WAVE_TRACE
// (timing build) this file's trace records: the fused kernel's main chunks
// and every FSST vector (fls_decode.hip holds decode_kernel's)
extern "C" int fls_trace_fsst_reset(void) {
    const uint32_t z = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(dec::g_trace_n), &z, sizeof(z)) == hipSuccess ? 0 : -1;
}
extern "C" int64_t fls_trace_fsst_read(void *dst, uint32_t cap) {
    uint32_t n = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(&n, HIP_SYMBOL(dec::g_trace_n), sizeof(n)) != hipSuccess)
        return -1;
    const uint32_t k = std::min(std::min(n, cap), dec::kTraceCap);
    if (k && hipMemcpyFromSymbol(dst, HIP_SYMBOL(dec::g_trace), k * sizeof(dec::TraceRec)) != hipSuccess) return -1;
    return n;
}
#endif

}  // namespace fls
