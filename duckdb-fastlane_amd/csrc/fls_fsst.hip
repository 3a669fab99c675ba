// fls_fsst.hip -- MI355X (gfx950) FSST string decode into DuckDB string_t.
//
// Replaces the FSST step inside RowgroupReader::materialize()
// (reference src/fastlanes_facade.cpp:48, the FLSStrColumn consumer at
// :163-170) for VARCHAR chunks written with ENC_FSST (fls_format.hpp).
//
// Waves take contiguous ranges of the launch's vectors (so a wave reloads the
// chunk's symbol table only when its range crosses into the next chunk).
// Per vector:
//   1. the FFOR-packed string lengths are unpacked into LDS and scanned into
//      exclusive offsets (doff[0..1024]) inside the vector's decompressed bytes;
//   2. the compressed code stream is decoded CODE-PARALLEL in rounds of 1024
//      bytes (16 per lane, one coalesced 16 B load each): a lane sums its
//      codes' symbol lengths, a wave scan turns them into output positions and
//      the lane writes its symbols into an LDS ring.  The escape code (255:
//      next byte is a literal) makes a code's meaning depend on its
//      predecessor; a lane therefore evaluates its bytes for both entry
//      states and a wave scan composes those 2-state maps (only in rounds that
//      contain an escape byte or start right after one);
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

constexpr int kWaves = 4;
// per-wave LDS layout (bytes, all 16-aligned)
constexpr uint32_t kOffP = 0;                      // packed lengths: 128*32 + 128
constexpr uint32_t kOffD = kOffP + 128 * 32 + 128;  // doff[1025] (u32)
constexpr uint32_t kOffSym = kOffD + 4112;         // u64 symbol[256]
constexpr uint32_t kOffLen = kOffSym + 2048;       // u8 length[256]
constexpr uint32_t kOffRing = kOffLen + 256;       // decoded bytes
constexpr uint32_t kRing = 8192 + 64;              // one round (<= 1024 codes x 8 B) + carry
constexpr uint32_t kWaveLds = kOffRing + kRing;
static_assert(kOffSym % 16 == 0 && kOffRing % 16 == 0 && kWaveLds % 16 == 0, "LDS layout alignment");

__device__ __forceinline__ uint32_t rl(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint32_t byte_of(const v4u &r, uint32_t k) {
    const uint32_t w = k < 4 ? r.x : k < 8 ? r.y : k < 12 ? r.z : r.w;
    return (w >> (8 * (k & 3))) & 0xFF;
}
__device__ __forceinline__ uint32_t scan_incl(uint32_t x, uint32_t lane) {
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

struct Wave {
    lv4 *P;
    lu32 *D;
    const FLS_LDS uint64_t *sym;
    const lu8 *len;
    lu8 *ring;
};

// 2-state escape automaton over a lane's bytes from entry state s:
// returns the exit state, adds the produced bytes to out
__device__ __forceinline__ uint32_t simulate(const Wave &w, const v4u &raw, uint32_t nb, uint32_t s, uint32_t &out) {
    for (uint32_t k = 0; k < 16; ++k) {
        if (k >= nb) break;
        const uint32_t b = byte_of(raw, k);
        if (s) {
            out += 1;
            s = 0;
        } else if (b == kFsstEscape) {
            s = 1;
        } else {
            out += min((uint32_t)w.len[b], 8u);
        }
    }
    return s;
}

// string_t of string i (doff d0, length n) from the ring (ring_base = global
// position of ring byte 0)
__device__ __forceinline__ v4u make_record(const Wave &w, uint32_t d0, uint32_t n, uint32_t ring_base,
                                           uint64_t ptr_base) {
    const uint32_t x = d0 - ring_base;
    const lu32 *r32 = reinterpret_cast<const lu32 *>(w.ring) + (x >> 2);
    const uint32_t sh = x & 3;
    const uint32_t w0 = r32[0], w1 = r32[1], w2 = r32[2], w3 = r32[3];
    const uint32_t b0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
    if (n > 12) {
        const uint64_t p = ptr_base + d0;
        return mk4(n, b0, (uint32_t)p, (uint32_t)(p >> 32));
    }
    const uint32_t b1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
    const uint32_t b2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
    auto keep = [n](uint32_t word, uint32_t first) -> uint32_t {  // zero bytes at index >= n
        if (n >= first + 4) return word;
        if (n <= first) return 0u;
        return word & ((1u << (8 * (n - first))) - 1u);
    };
    return mk4(n, keep(b0, 0), keep(b1, 4), keep(b2, 8));
}

__device__ void fsst_vector(const Wave &w, gu8 *packed_vec, uint32_t W, uint32_t base, uint32_t nvals,
                            uint32_t dbytes, gu8 *vh, FLS_GLOBAL uint8_t *heap, uint32_t heap_bytes,
                            uint64_t heap_host, FLS_GLOBAL uint8_t *out, uint32_t lane, uint32_t *err) {
    bool bad = false;
    // ---- 1. lengths -> offsets --------------------------------------------
    const uint32_t n16 = 8 * W;
    gv4 *pk = reinterpret_cast<gv4 *>(packed_vec);
    for (uint32_t i = lane; i < n16; i += 64) w.P[i] = pk[i];
    if (lane < 8) w.P[n16 + lane] = mk4(0, 0, 0, 0);
    wave_sync();
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
    {
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
    }
    wave_sync();
    const uint32_t total = uni(w.D[1024]);
    if (total != dbytes) bad = true;
    const FLS_GLOBAL FsstVecHeader *hp = reinterpret_cast<const FLS_GLOBAL FsstVecHeader *>(vh);
    const uint32_t heap_off = uni(hp->heap_off), comp_len = uni(hp->comp_len);
    const uint32_t hlim = min((dbytes + 15) & ~15u, heap_bytes > heap_off ? heap_bytes - heap_off : 0u);
    FLS_GLOBAL uint8_t *vheap = heap + heap_off;
    const uint64_t ptr_base = heap_host + heap_off;
    gv4 *comp = reinterpret_cast<gv4 *>(vh + sizeof(FsstVecHeader));

    uint32_t out_pos = 0, ring_base = 0, carry_lit = 0, next_str = 0;
    // strings whose leading bytes are all decoded get their string_t
    auto finalize = [&]() {
        while (next_str < nvals) {
            const uint32_t i = next_str + lane;
            bool ok = false;
            uint32_t d0 = 0, n = 0;
            if (i < nvals) {
                d0 = w.D[i];
                n = w.D[i + 1] - d0;
                ok = d0 + min(n, 12u) <= out_pos;
            }
            const uint64_t m = __ballot(ok);
            const uint32_t n_ok = ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m);
            if (lane < n_ok)
                *reinterpret_cast<ov4 *>(out + 16ull * i) = make_record(w, d0, n, ring_base, ptr_base);
            next_str += n_ok;
            if (n_ok < 64) break;
        }
    };
    // stream complete 16 B blocks below `upto` (16-aligned) to the heap
    auto flush = [&](uint32_t upto) {
        const uint32_t nblk = (upto - ring_base) >> 4;
        for (uint32_t q = lane; q < nblk; q += 64) {
            const uint32_t g = ring_base + 16 * q;
            if (g + 16 <= hlim) *reinterpret_cast<ov4 *>(vheap + g) = reinterpret_cast<const lv4 *>(w.ring)[q];
            else bad = true;
        }
    };

    // ---- 2-4. code-parallel rounds -----------------------------------------
    for (uint32_t r0 = 0; r0 < comp_len; r0 += 1024) {
        const uint32_t idx0 = r0 + 16 * lane;
        const uint32_t nb = idx0 < comp_len ? min(comp_len - idx0, 16u) : 0u;
        const v4u raw = nb ? comp[(r0 >> 4) + lane] : mk4(0, 0, 0, 0);
        bool has_esc = false;
        for (uint32_t k = 0; k < nb; ++k) has_esc |= byte_of(raw, k) == kFsstEscape;
        uint32_t start = 0, lane_out = 0, lane_end = 0;
        if (__ballot(has_esc) == 0 && carry_lit == 0) {  // no escape anywhere: every code is a symbol
            for (uint32_t k = 0; k < nb; ++k) lane_out += min((uint32_t)w.len[byte_of(raw, k)], 8u);
        } else {
            uint32_t o0 = 0, o1 = 0;
            const uint32_t e0 = simulate(w, raw, nb, 0, o0), e1 = simulate(w, raw, nb, 1, o1);
            // inclusive scan of the lanes' state maps f (bit s = f(s)); apply earlier first
            uint32_t f = e0 | (e1 << 1);
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t g = __shfl_up(f, d, 64);
                if (lane >= d) f = (((f >> (g & 1)) & 1)) | (((f >> ((g >> 1) & 1)) & 1) << 1);
            }
            uint32_t pre = __shfl_up(f, 1, 64);
            if (lane == 0) pre = 2;  // identity map
            start = (pre >> carry_lit) & 1;
            lane_out = start ? o1 : o0;
            lane_end = start ? e1 : e0;
        }
        const uint32_t incl = scan_incl(lane_out, lane);
        const uint32_t round_total = rl(incl, 63);
        // write this lane's symbols into the ring
        uint32_t wp = out_pos - ring_base + (incl - lane_out);
        uint32_t st = start;
        for (uint32_t k = 0; k < nb; ++k) {
            const uint32_t b = byte_of(raw, k);
            if (st) {
                w.ring[wp++] = (uint8_t)b;
                st = 0;
            } else if (b == kFsstEscape) {
                st = 1;
            } else {
                const uint32_t L = min((uint32_t)w.len[b], 8u);
                const uint64_t sy = w.sym[b];
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q)
                    if (q < L) w.ring[wp + q] = (uint8_t)(sy >> (8 * q));
                wp += L;
            }
        }
        carry_lit = rl(lane_end, 63);
        wave_sync();
        out_pos += round_total;
        finalize();
        const uint32_t keep_from = next_str < nvals ? min(uni(w.D[next_str]), out_pos) : out_pos;
        const uint32_t new_base = keep_from & ~15u;
        flush(new_base);
        wave_sync();
        // move the unfinished tail (< 32 B) to the ring start
        const uint32_t src = (new_base - ring_base) >> 2;
        uint32_t t = 0;
        if (lane < 8) t = reinterpret_cast<const lu32 *>(w.ring)[src + lane];
        wave_sync();
        if (lane < 8) reinterpret_cast<lu32 *>(w.ring)[lane] = t;
        ring_base = new_base;
        wave_sync();
    }
    if (carry_lit) bad = true;  // stream ends inside an escape
    finalize();
    if (next_str < nvals) {     // lengths claim more bytes than the stream holds
        bad = true;
        for (uint32_t i = next_str + lane; i < nvals; i += 64)
            *reinterpret_cast<ov4 *>(out + 16ull * i) = mk4(0, 0, 0, 0);
    }
    // zero the padding of the last block, then flush everything
    const uint32_t end = (out_pos + 15) & ~15u;
    if (lane < 16 && out_pos + lane < end) w.ring[out_pos - ring_base + lane] = 0;
    wave_sync();
    flush(end);
    if (bad) atomicOr(err, KERR_FSST);
}

__device__ __forceinline__ DevChunk load_chunk(const DevChunk *chunks, uint32_t ci) {
    const FLS_GLOBAL v4u *q = reinterpret_cast<const FLS_GLOBAL v4u *>(gptr(chunks + ci));
    DevChunk c;
    v4u *d = reinterpret_cast<v4u *>(&c);
    d[0] = q[0];
    d[1] = q[1];
    d[2] = q[2];
    d[3] = q[3];
    return c;
}

// Vectors [item0, item1) of the launch (items numbered chunk by chunk through
// DevChunk.vec_base): the wave loads a chunk's symbol table once and decodes
// its vectors in order.
__device__ __attribute__((noinline)) void fsst_range(const DevChunk *chunks_generic, uint32_t nchunks, uint32_t item0,
                                                     uint32_t item1, uint8_t *lds_generic, uint32_t *err_generic) {
    const uint64_t cp = (uint64_t)chunks_generic;
    const DevChunk *chunks = (const DevChunk *)((uint64_t)uni((uint32_t)(cp >> 32)) << 32 | uni((uint32_t)cp));
    const uint64_t ep = (uint64_t)err_generic;
    uint32_t *err = (uint32_t *)((uint64_t)uni((uint32_t)(ep >> 32)) << 32 | uni((uint32_t)ep));
    lu8 *L = (lu8 *)(size_t)uni((uint32_t)(size_t)lds_generic);
    nchunks = uni(nchunks);
    item0 = uni(item0);
    item1 = uni(item1);
    const uint32_t lane = __lane_id();
    Wave w;
    w.P = reinterpret_cast<lv4 *>(L + kOffP);
    w.D = reinterpret_cast<lu32 *>(L + kOffD);
    w.sym = reinterpret_cast<const FLS_LDS uint64_t *>(L + kOffSym);
    w.len = L + kOffLen;
    w.ring = L + kOffRing;
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
    for (uint32_t item = item0; item < item1;) {
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
            // symbol table (u64[256] then u8[256]: 144 x 16 B, contiguous in both places)
            wave_sync();
            for (uint32_t i = lane; i < kFsstTableBytes / 16; i += 64)
                reinterpret_cast<lv4 *>(L + kOffSym)[i] = reinterpret_cast<gv4 *>(aux)[i];
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
        fsst_vector(w, chunk + c.packed_off + poff, W, base, nvals, dbytes, aux + aoff,
                    (FLS_GLOBAL uint8_t *)(size_t)c.dict, c.heap_bytes, c.heap_host,
                    gptr(c.out) + 16ull * kVectorSize * v, lane, err);
        wave_sync();
        ++item;
    }
}

__global__ __launch_bounds__(256, 2) void fsst_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                      uint32_t nitems, uint32_t *__restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    const uint32_t w = uni(threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * kWaves, wave = blockIdx.x * kWaves + w;
    // contiguous vector ranges per wave: a wave mostly stays inside one chunk
    const uint32_t per = (nitems + nwaves - 1) / nwaves;
    const uint32_t i0 = min(wave * per, nitems), i1 = min(i0 + per, nitems);
    if (i0 < i1) fsst_range(chunks, nchunks, i0, i1, lds_raw + w * kWaveLds, err);
}

}  // namespace

hipError_t launch_fsst(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                       hipStream_t stream) {
    if (nchunks == 0 || nvecs == 0) return hipSuccess;
    const uint32_t shmem = kWaves * kWaveLds;
    int dev = 0, cus = 256, per_cu = 1;
    if (hipGetDevice(&dev) == hipSuccess) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fsst_kernel, 64 * kWaves, shmem) != hipSuccess)
            per_cu = 1;
    }
    const int grid = std::min<int>(cus * std::max(1, per_cu), (int)((nvecs + kWaves - 1) / kWaves));
    hipLaunchKernelGGL(fsst_kernel, dim3(grid), dim3(64 * kWaves), shmem, stream, d_chunks, nchunks, nvecs, d_err);
    return hipGetLastError();
}

}  // namespace fls
