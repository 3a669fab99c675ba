// fls_encode.hip -- MI355X (gfx950) FastLanes chunk encoder: FFOR and
// unified-transposed DELTA for integer columns, byte-identical to the CPU
// writer's chunks (fls_writer.cpp enc_ffor / enc_delta / assemble_chunk).
//
// The write side of the scan path (COPY ... TO (FORMAT
// FLS); the reference's writer is a stub, src/writer/write_fastlane_stream.cpp
// :65-314).  The arithmetic is the decode kernel's run backwards:
//   * one 256-thread block (4 waves) per column chunk (<= 64 vectors);
//   * the waves take the vectors in rounds of four, one vector per wave, one
//     pass each: the 1024 values (tail padded with the last value, as the CPU
//     writer does) are staged in LDS; DELTA turns them into per-chain deltas
//     in transposed position order (chain c = tuples blk*16T + l + 16k,
//     FL_ORDER = {0,4,2,6,1,5,3,7}) and writes the chain bases to scratch;
//     the 16 position-ordered values of each lane are read once into
//     registers, and the wave reduces their signed minimum (FOR base) and
//     maximum together (W = bit width of max - min, which equals the width of
//     OR(value - base) that the CPU writer computes); value - base goes back
//     to LDS in position order;
//   * one block barrier per round makes the round's widths visible; a vector's
//     packed rows start where those of the vectors before it end, so every
//     lane then assembles 16-byte rows of the interleaved packing (word k of
//     FastLanes lane L = bits [kT, kT + T) of lane L's stream of T values of
//     W bits -- the inverse of fls_unpack.hpp) straight at their place;
//   * wave 0 scans the vectors' 128 W packed bytes into offsets and writes the
//     chunk header and the VecMeta records; the waves then move the DELTA
//     bases after the packed area and write the zero padding.
//   History (profiles/r1/encode_*): v1 read the input twice (analyse, then
//   pack): 3.16 ms for 1e9 INT64 keys.  v2 packed into a scratch area at the
//   vector's widest position and moved the rows once every width was known:
//   2.09-2.23 ms.  Reading the values into registers once (one min/max
//   reduction instead of a min pass and an OR pass over LDS) took INT64 DELTA
//   2.11 -> 1.96 ms and INT32 FFOR 1.87 -> 1.78 ms; packing straight to the
//   final place, INT64 FFOR 2.29 -> 1.78 ms; the T <= 32 register prefetch,
//   INT32 FFOR 1.71 -> 1.39 ms.
// Integer work, HBM-bound: per value it reads T/8 bytes and writes W/8 bytes.
// No MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/flsgpu.h"
#include "../../include/flswriter.h"
#include "fls_common.hpp"
#include "fls_decode.hpp"
#include "fls_encode.hpp"
#include "fls_alp.hpp"
#include "fls_format.hpp"
#include "fls_unpack.hpp"

namespace fls {
namespace {
using namespace dev;

constexpr int kEncWaves = 4;

__device__ __forceinline__ uint64_t tmask_d(uint32_t T) { return T >= 64 ? ~0ull : ((1ull << T) - 1ull); }
__device__ __forceinline__ int64_t sext_d(uint64_t v, uint32_t T) {
    if (T >= 64) return (int64_t)v;
    const uint64_t sign = 1ull << (T - 1);
    v &= tmask_d(T);
    return (int64_t)((v ^ sign) - sign);
}
// transposed position p -> tuple index (FL_ORDER is the 3-bit bit reversal)
__device__ __forceinline__ uint32_t tau_d(uint32_t p) {
    const uint32_t b = (p >> 4) & 7;
    const uint32_t rb = ((b & 1) << 2) | (b & 2) | ((b >> 2) & 1);
    return (rb << 7) | (((p >> 7) & 7) << 4) | (p & 15);
}
__device__ __forceinline__ uint32_t rl(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }
// The wave's index in the block, wave-uniform: as an SGPR its LDS and input
// offsets are scalar too.  Held in a VGPR (FLS_ENC_VECTOR_WAVE_INDEX, the
// round-2 code) the narrow kernel needed 93 VGPRs, and its 6-wave build spilled
// the wave's LDS base (w * 4096) to one 8-byte scratch slot whose store sat
// inside the prefetch branch of a full next vector: waves that skipped the
// branch reloaded a stale slot.  Scalar: 80 VGPRs, no
// spill at 5 or 6 waves per SIMD.
__device__ __forceinline__ uint32_t wave_index() {
#ifdef FLS_ENC_VECTOR_WAVE_INDEX
    return threadIdx.x >> 6;
#else
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#endif
}
// min and max together: two independent shuffle chains, one latency
__device__ __forceinline__ void wave_minmax_i64(int64_t &mn, int64_t &mx) {
    for (int d = 32; d >= 1; d >>= 1) {
        const int64_t a = (int64_t)__shfl_xor((unsigned long long)mn, d, 64);
        const int64_t b = (int64_t)__shfl_xor((unsigned long long)mx, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
}

// LDS / register storage of a T-bit value: u32 for T <= 32 (half the LDS
// and VGPRs of u64), u64 for T = 64
template <int T>
using Sto = typename std::conditional<T == 64, uint64_t, uint32_t>::type;

// 1024 values of vector v of the chunk into V (zero-extended T-bit), the
// tail past vn padded with the last value
template <int T, typename S>
__device__ __forceinline__ void stage_values(const uint8_t *in, uint32_t v, uint32_t vn, FLS_LDS S *V,
                                             uint32_t lane) {
    using U = typename std::conditional<T == 8, uint8_t,
              typename std::conditional<T == 16, uint16_t,
              typename std::conditional<T == 32, uint32_t, uint64_t>::type>::type>::type;
    const FLS_GLOBAL U *src = (const FLS_GLOBAL U *)in + (size_t)v * kVectorSize;
    if (vn == kVectorSize) {
        // 16-byte loads: 16 / (T/8) values each
        constexpr uint32_t per = 16 / (T / 8);
        const FLS_GLOBAL v4u *s16 = reinterpret_cast<const FLS_GLOBAL v4u *>(src);
        for (uint32_t q = lane; q < kVectorSize / per; q += 64) {
            const v4u x = s16[q];
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (uint32_t i = 0; i < per; ++i) {
                uint64_t val;
                if (T == 64) val = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
                else val = (w[(i * T) / 32] >> ((i * T) % 32)) & (uint32_t)tmask_d(T);
                V[q * per + i] = (S)val;
            }
        }
    } else {
        for (uint32_t j = lane; j < kVectorSize; j += 64) V[j] = (S)src[j < vn ? j : vn - 1];
    }
}

// Register prefetch of a full vector (T <= 32: T/8 16-byte loads per lane,
// at most 16 VGPRs) and its staging, the full-vector case of stage_values
template <int T>
__device__ __forceinline__ void load_vec(const uint8_t *in, uint32_t v, uint32_t lane, v4u (&r)[T / 8]) {
    const FLS_GLOBAL v4u *s16 = (const FLS_GLOBAL v4u *)(in + (size_t)v * kVectorSize * (T / 8));
#pragma unroll
    for (uint32_t i = 0; i < T / 8; ++i) r[i] = s16[lane + 64 * i];
}
template <int T, typename S>
__device__ __forceinline__ void stage_regs(const v4u (&r)[T / 8], FLS_LDS S *V, uint32_t lane) {
    constexpr uint32_t per = 16 / (T / 8);
#pragma unroll
    for (uint32_t i = 0; i < T / 8; ++i) {
        const uint32_t q = lane + 64 * i;
        const uint32_t w[4] = {r[i].x, r[i].y, r[i].z, r[i].w};
#pragma unroll
        for (uint32_t j = 0; j < per; ++j)
            V[q * per + j] = (S)(T == 64 ? ((uint64_t)w[2 * j] | ((uint64_t)w[2 * j + 1] << 32))
                                         : (w[(j * T) / 32] >> ((j * T) % 32)) & (uint32_t)tmask_d(T));
    }
}

// position-ordered value p of the vector staged in V: FFOR the value itself,
// DELTA the delta of tuple tau(p) on its chain (0 at a chain start)
template <int T, bool DELTA, typename S>
__device__ __forceinline__ S pos_value(const FLS_LDS S *V, uint32_t p) {
    if (!DELTA) return V[p];
    const uint32_t i = tau_d(p);
    return ((i >> 4) % T == 0) ? (S)0 : (S)((V[i] - V[i - 16]) & (S)tmask_d(T));
}

struct VecStat {
    int64_t base;
    uint32_t W;
};

// FOR base and bit width of the vector's 16 position-ordered values per lane,
// held in registers (read from LDS once): base = signed minimum; W = bit
// width of max - min, which is the width of OR(x - min) that the CPU writer
// computes (the highest set bit of an OR is that of its largest operand).
template <int T>
__device__ __forceinline__ VecStat analyze_regs(const uint64_t (&x)[16]) {
    int64_t mn = INT64_MAX, mx = INT64_MIN;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const int64_t y = sext_d(x[k], T);
        mn = y < mn ? y : mn;
        mx = y > mx ? y : mx;
    }
    wave_minmax_i64(mn, mx);
    const uint64_t range = ((uint64_t)mx - (uint64_t)mn) & tmask_d(T);
    VecStat s;
    s.base = mn;
    s.W = range ? 64u - (uint32_t)__builtin_clzll(range) : 0u;
    return s;
}
// T <= 32: the same in 32-bit registers and shuffles
template <int T>
__device__ __forceinline__ VecStat analyze_regs(const uint32_t (&x)[16]) {
    int32_t mn = INT32_MAX, mx = INT32_MIN;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        const uint32_t sign = 1u << (T - 1);
        const int32_t y = T == 32 ? (int32_t)x[k] : (int32_t)(((x[k] & (uint32_t)tmask_d(T)) ^ sign) - sign);
        mn = y < mn ? y : mn;
        mx = y > mx ? y : mx;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const int32_t a = __shfl_xor(mn, d, 64);
        const int32_t b = __shfl_xor(mx, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
    }
    const uint32_t range = ((uint32_t)mx - (uint32_t)mn) & (uint32_t)tmask_d(T);
    VecStat s;
    s.base = mn;
    s.W = range ? 32u - (uint32_t)__builtin_clz(range) : 0u;
    return s;
}

// Interleaved packing of the position-ordered u = value - base staged in U:
// 16-byte row chunk ci = (word row k = ci / 8, byte column 16 (ci % 8)) holds
// word k of FastLanes lanes L = (ci % 8) * 128/T + j, j < 128/T; word k of lane
// L = OR over rows r of u[r * 1024/T + L] << (r W - k T) (bits [kT, kT + T) of
// the lane's stream).
template <int T, typename S>
__device__ void pack_vector(const FLS_LDS S *U, uint32_t W, FLS_GLOBAL uint8_t *dst, uint32_t lane) {
    constexpr uint32_t nl = kVectorSize / T, wpc = 128 / T;  // lanes, words per 16 B
    const uint64_t tm = tmask_d(T);
    for (uint32_t ci = lane; ci < 8 * W; ci += 64) {
        const uint32_t k = ci >> 3, L0 = (ci & 7) * wpc;
        const uint32_t r0 = (k * T) / W, r1 = min((uint32_t)T - 1, ((k + 1) * T - 1) / W);
        uint32_t out[4] = {0, 0, 0, 0};
#pragma unroll
        for (uint32_t j = 0; j < wpc; ++j) {
            uint64_t word = 0;
            for (uint32_t r = r0; r <= r1; ++r) {
                const uint64_t u = U[r * nl + L0 + j];
                const int32_t sh = (int32_t)(r * W) - (int32_t)(k * T);
                word |= sh >= 0 ? (sh < 64 ? u << sh : 0ull) : u >> (uint32_t)(-sh);
            }
            word &= tm;
            // place word j (T bits) into the 16-byte chunk
            if (T == 64) {
                out[2 * j] = (uint32_t)word;
                out[2 * j + 1] = (uint32_t)(word >> 32);
            } else {
                out[(j * T) / 32] |= (uint32_t)word << ((j * T) % 32);
            }
        }
        *reinterpret_cast<FLS_GLOBAL v4u *>(dst + 16ull * ci) = mk4(out[0], out[1], out[2], out[3]);
    }
}

template <int T, bool DELTA>
__device__ void encode_chunk(const EncChunk &c, FLS_LDS Sto<T> *Vall, FLS_LDS uint32_t *Wv,
                             FLS_LDS int64_t *Bv, FLS_LDS uint64_t *Ov) {
    using S = Sto<T>;
    const uint32_t lane = threadIdx.x & 63, w = wave_index();
    FLS_LDS S *V = Vall + w * kVectorSize;
    const uint32_t n = c.nrows, nvec = (n + kVectorSize - 1) / kVectorSize;
    const uint8_t *in = (const uint8_t *)c.in;
    FLS_GLOBAL uint8_t *out = (FLS_GLOBAL uint8_t *)c.out;
    FLS_GLOBAL uint8_t *scratch = (FLS_GLOBAL uint8_t *)c.scratch;
    // ---- one pass per vector: base, width, DELTA bases, packing.  The waves
    // take the vectors in rounds of kEncWaves; a vector's packed rows start
    // where the packed rows of the vectors before it end, so once a round's
    // widths are in LDS (one block barrier) every wave packs straight to its
    // vector's place in the chunk.  The DELTA bases go to scratch: their place
    // follows the packed area.
    const uint64_t meta_off = sizeof(ChunkHeader);
    const uint64_t packed_off = (meta_off + sizeof(VecMeta) * nvec + 15) & ~15ull;
    FLS_GLOBAL uint8_t *sbases = scratch;
    uint32_t done = 0;  // packed bytes of the earlier rounds' vectors
    // T <= 32: the wave's next full vector (v + kEncWaves) is loaded into
    // registers while this one is analysed and packed (INT32 FFOR 1.70 ->
    // see DESIGN.md section 10; T = 64 would hold 32 more VGPRs and measured slower)
#ifndef FLS_ENC_PF_MAX_T
#define FLS_ENC_PF_MAX_T 32
#endif
    constexpr bool kPf = T <= FLS_ENC_PF_MAX_T;
    constexpr int TP = kPf ? T : 8;  // prefetch instantiation (unused when !kPf)
    constexpr uint32_t kPfN = TP / 8;
    v4u pf[kPfN];
    auto full = [&](uint32_t x) { return (x + 1) * kVectorSize <= n; };
    if (kPf && w < nvec && full(w)) load_vec<TP>(in, w, lane, pf);
    for (uint32_t r = 0; r < nvec; r += kEncWaves) {
        const uint32_t v = r + w;
        const bool act = v < nvec;  // wave-uniform
        VecStat s{0, 0};
        if (act) {
            const uint32_t vn = min(kVectorSize, n - v * kVectorSize);
            if (kPf && vn == kVectorSize) stage_regs<TP>(pf, V, lane);
            else stage_values<T>(in, v, vn, V, lane);
            if (kPf && v + kEncWaves < nvec && full(v + kEncWaves))
                load_vec<TP>(in, v + kEncWaves, lane, pf);
            wave_sync();
            S x[16];
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) x[k] = pos_value<T, DELTA>(V, lane + 64 * k);
            s = analyze_regs<T>(x);
            if (lane == 0) {
                Wv[v] = s.W;
                Bv[v] = s.base;
            }
            if (DELTA) {
                // chain c's base = its first tuple blk*16T + l (put_word layout, T/8 bytes)
                if (lane < kVectorSize / T) {
                    const uint64_t b = V[(lane / 16) * 16 * T + (lane % 16)];
                    FLS_GLOBAL uint8_t *bp = sbases + 128ull * v + lane * (T / 8);
                    if (T == 64) *(FLS_GLOBAL uint64_t *)bp = b;
                    else if (T == 32) *(FLS_GLOBAL uint32_t *)bp = (uint32_t)b;
                    else if (T == 16) *(FLS_GLOBAL uint16_t *)bp = (uint16_t)b;
                    else *bp = (uint8_t)b;
                }
                if (T == 8 && lane < 64) {  // 128 chains of T = 8: lanes 0..63 take chains 64..127 too
                    const uint32_t c2 = lane + 64;
                    sbases[128ull * v + c2] = (uint8_t)V[(c2 / 16) * 16 * T + (c2 % 16)];
                }
            }
            S u[16];
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) u[k] = (S)((x[k] - (S)s.base) & (S)tmask_d(T));
            wave_sync();
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) V[lane + 64 * k] = u[k];
            wave_sync();
        }
        __syncthreads();  // this round's widths are in Wv
        if (act) {
            uint32_t off = done;
            for (uint32_t i = r; i < v; ++i) off += 128u * Wv[i];
            pack_vector<T>(V, s.W, out + packed_off + off, lane);
        }
        for (uint32_t i = r; i < min(r + (uint32_t)kEncWaves, nvec); ++i) done += 128u * Wv[i];
        wave_sync();
    }
    __syncthreads();
    // ---- chunk layout (assemble_chunk) --------------------------------------
    if (w == 0) {
        const uint32_t pw = lane < nvec ? 128u * Wv[lane] : 0u;
        uint32_t incl = pw;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        const uint64_t packed_total = rl(incl, 63);
        const uint64_t aux_off = (packed_off + packed_total + 15) & ~15ull;
        const uint64_t aux_len = DELTA ? 128ull * nvec : 0ull;
        const uint64_t total = (aux_off + aux_len + kChunkAlign - 1) & ~(uint64_t)(kChunkAlign - 1);
        if (lane < nvec) {
            VecMeta m;
            m.packed_off = incl - pw;
            m.for_base = Bv[lane];
            m.aux_off = DELTA ? 128ull * lane : 0ull;
            m.nvals = (uint16_t)min(kVectorSize, n - lane * kVectorSize);
            m.bw = (uint8_t)Wv[lane];
            m.pad = 0;
            m.aux_count = 0;
            const uint32_t *mw = reinterpret_cast<const uint32_t *>(&m);
            FLS_GLOBAL uint32_t *dm = reinterpret_cast<FLS_GLOBAL uint32_t *>(out + meta_off + sizeof(VecMeta) * lane);
#pragma unroll
            for (int i = 0; i < 8; ++i) dm[i] = mw[i];
            Ov[lane] = incl - pw;
        }
        if (lane == 0) {
            ChunkHeader h;
            h.magic = kChunkMagic;
            h.enc = DELTA ? ENC_DELTA : ENC_FFOR;
            h.T = (uint8_t)T;
            h.vbits = (uint8_t)T;
            h.is_str = 0;
            h.nvec = nvec;
            h.nvals = n;
            h.meta_off = meta_off;
            h.packed_off = packed_off;
            h.aux_off = aux_off;
            h.aux_len = aux_len;
            h.dict_count = 0;
            h.reserved0 = 0;
            h.reserved1 = 0;
            const uint32_t *hw = reinterpret_cast<const uint32_t *>(&h);
            FLS_GLOBAL uint32_t *dh = reinterpret_cast<FLS_GLOBAL uint32_t *>(out);
#pragma unroll
            for (int i = 0; i < 16; ++i) dh[i] = hw[i];
            Ov[64] = packed_total;
            Ov[65] = aux_off;
            Ov[66] = total;
            *(FLS_GLOBAL uint64_t *)c.len_out = total | (uint64_t)(DELTA ? ENC_DELTA : ENC_FFOR) << kEncShift;
        }
    }
    __syncthreads();
    const uint64_t packed_total = Ov[64], aux_off = Ov[65], total = Ov[66];
    // ---- DELTA bases after the packed area; padding.  Each wave moves the
    // bases of its own vectors, which its own lanes wrote to scratch in the
    // round loop: a wave's global store and later load of the same address
    // are ordered, while a hand-off of global memory between the waves would
    // rely on the barrier alone (it waits for LDS traffic, lgkmcnt, not for
    // stores still in flight, vmcnt).  The block-strided copy this replaces
    // was the one cross-wave global hand-off in the kernel.
    if (DELTA) {
        const FLS_GLOBAL v4u *src = reinterpret_cast<const FLS_GLOBAL v4u *>(sbases);
        FLS_GLOBAL v4u *dst = reinterpret_cast<FLS_GLOBAL v4u *>(out + aux_off);
        for (uint32_t v = w; v < nvec; v += kEncWaves)
            if (lane < 8) dst[8 * v + lane] = src[8 * v + lane];
    }
    {
        const uint64_t gaps[3][2] = {{meta_off + sizeof(VecMeta) * nvec, packed_off},
                                     {packed_off + packed_total, aux_off},
                                     {aux_off + (DELTA ? 128ull * nvec : 0ull), total}};
        for (int g = 0; g < 3; ++g)
            for (uint64_t b = gaps[g][0] + threadIdx.x; b < gaps[g][1]; b += blockDim.x) out[b] = 0;
    }
}

// FastLanes-RLE chunk (fls_writer.cpp enc_rle, byte for byte): per vector the
// run index of every value (the tail padded with the last value, so it adds
// no run), DELTA(T = 16)-coded in the unified transposed order and
// FFOR-packed at T = 16, plus an aux block of 128 B of chain bases (u16) and
// the run values (T/8 bytes each), 16-aligned per vector.  Two passes over
// the vectors: the first finds every vector's runs and width (so the packed
// and aux offsets are known), the second writes each vector at its place.
// Per vector, lane L takes values [16L, 16L + 16): run starts, a wave scan of
// their counts, then the run index per value.  No MFMA; HBM-bound like the
// other encoders (reads T/8 bytes per value twice).
template <int T>
__device__ uint32_t run_index(FLS_LDS Sto<T> *V, uint32_t lane, uint32_t (&idx)[16], uint32_t &flags) {
    using S = Sto<T>;
    S x[16];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) x[j] = V[16 * lane + j];
    const S prev = lane > 0 ? V[16 * lane - 1] : x[0];
    flags = 0;
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        const bool start = j == 0 ? (lane == 0 || x[0] != prev) : x[j] != x[j - 1];
        flags |= start ? 1u << j : 0u;
        cnt += start ? 1u : 0u;
        idx[j] = cnt;  // inclusive within the lane
    }
    uint32_t incl = cnt;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    const uint32_t base = incl - cnt;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) idx[j] = base + idx[j] - 1;
    return __shfl(incl, 63, 64);  // the vector's runs
}

template <int T>
__device__ void encode_rle_chunk(const EncChunk &c, FLS_LDS Sto<T> *Vall, FLS_LDS uint32_t *Wv, FLS_LDS int64_t *Bv,
                                 FLS_LDS uint64_t *Ov) {
    using S = Sto<T>;
    const uint32_t lane = threadIdx.x & 63, w = wave_index();
    FLS_LDS S *V = Vall + w * kVectorSize;
    const uint32_t n = c.nrows, nvec = (n + kVectorSize - 1) / kVectorSize;
    const uint8_t *in = (const uint8_t *)c.in;
    FLS_GLOBAL uint8_t *out = (FLS_GLOBAL uint8_t *)c.out;
    // the transposed deltas of the run indices (T = 16 chains) in registers,
    // their FOR base and width
    auto idx_deltas = [&](uint32_t (&idx)[16], S (&x)[16]) -> VecStat {
        wave_sync();
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) V[16 * lane + j] = (S)idx[j];
        wave_sync();
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) x[k] = pos_value<16, true>(V, lane + 64 * k);
        return analyze_regs<16>(x);
    };
    // ---- pass 1: runs and width of every vector
    for (uint32_t v = w; v < nvec; v += kEncWaves) {
        stage_values<T>(in, v, min(kVectorSize, n - v * kVectorSize), V, lane);
        wave_sync();
        uint32_t idx[16], flags;
        const uint32_t runs = run_index<T>(V, lane, idx, flags);
        S x[16];
        const VecStat st = idx_deltas(idx, x);
        if (lane == 0) {
            Wv[v] = st.W;
            Bv[v] = st.base;
            Ov[v] = runs;
        }
        wave_sync();
    }
    __syncthreads();
    // ---- layout (assemble_chunk): every wave computes the offsets it needs
    const uint64_t meta_off = sizeof(ChunkHeader);
    const uint64_t packed_off = (meta_off + sizeof(VecMeta) * nvec + 15) & ~15ull;
    const uint32_t pw = lane < nvec ? 128u * Wv[lane] : 0u;
    const uint32_t va = lane < nvec ? 128u + (uint32_t)Ov[lane] * (T / 8) : 0u;  // aux bytes of vector lane
    uint32_t pincl = pw, aincl = (va + 15) & ~15u;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(pincl, d, 64), z = __shfl_up(aincl, d, 64);
        if (lane >= d) { pincl += y; aincl += z; }
    }
    const uint32_t poff = pincl - pw, aoff = aincl - ((va + 15) & ~15u);  // exclusive
    const uint64_t packed_total = __shfl(pincl, 63, 64);
    const uint64_t aux_off = (packed_off + packed_total + 15) & ~15ull;
    const uint64_t aux_len = __shfl(aoff, nvec - 1, 64) + __shfl(va, nvec - 1, 64);
    const uint64_t total = (aux_off + aux_len + kChunkAlign - 1) & ~(uint64_t)(kChunkAlign - 1);
    if (w == 0) {
        if (lane < nvec) {
            VecMeta m;
            m.packed_off = poff;
            m.for_base = Bv[lane];
            m.aux_off = aoff;
            m.nvals = (uint16_t)min(kVectorSize, n - lane * kVectorSize);
            m.bw = (uint8_t)Wv[lane];
            m.pad = 0;
            m.aux_count = (uint32_t)Ov[lane];
            const uint32_t *mw = reinterpret_cast<const uint32_t *>(&m);
            FLS_GLOBAL uint32_t *dm = reinterpret_cast<FLS_GLOBAL uint32_t *>(out + meta_off + sizeof(VecMeta) * lane);
#pragma unroll
            for (int i = 0; i < 8; ++i) dm[i] = mw[i];
        }
        if (lane == 0) {
            ChunkHeader h;
            h.magic = kChunkMagic;
            h.enc = ENC_RLE;
            h.T = 16;
            h.vbits = (uint8_t)T;
            h.is_str = 0;
            h.nvec = nvec;
            h.nvals = n;
            h.meta_off = meta_off;
            h.packed_off = packed_off;
            h.aux_off = aux_off;
            h.aux_len = aux_len;
            h.dict_count = 0;
            h.reserved0 = 0;
            h.reserved1 = 0;
            const uint32_t *hw = reinterpret_cast<const uint32_t *>(&h);
            FLS_GLOBAL uint32_t *dh = reinterpret_cast<FLS_GLOBAL uint32_t *>(out);
#pragma unroll
            for (int i = 0; i < 16; ++i) dh[i] = hw[i];
            *(FLS_GLOBAL uint64_t *)c.len_out = total | (uint64_t)ENC_RLE << kEncShift;
        }
    }
    // ---- pass 2: run values, chain bases and packed run-index deltas of
    // every vector at their places
    for (uint32_t v = w; v < nvec; v += kEncWaves) {
        const uint32_t vn = min(kVectorSize, n - v * kVectorSize);
        const uint32_t p_off = __shfl(poff, v, 64), a_off = __shfl(aoff, v, 64);
        FLS_GLOBAL uint8_t *aux = out + aux_off + a_off;
        stage_values<T>(in, v, vn, V, lane);
        wave_sync();
        uint32_t idx[16], flags;
        run_index<T>(V, lane, idx, flags);
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j)
            if (flags >> j & 1u) {  // run idx[j] starts here: its value
                const S val = V[16 * lane + j];
                FLS_GLOBAL uint8_t *rp = aux + 128 + (size_t)idx[j] * (T / 8);
                if (T == 64) *(FLS_GLOBAL uint64_t *)rp = (uint64_t)val;
                else if (T == 32) *(FLS_GLOBAL uint32_t *)rp = (uint32_t)val;
                else if (T == 16) *(FLS_GLOBAL uint16_t *)rp = (uint16_t)val;
                else *rp = (uint8_t)val;
            }
        S x[16];
        const VecStat st = idx_deltas(idx, x);
        // chain c's base = run index of its first tuple (blk*256 + l), u16
        *(FLS_GLOBAL uint16_t *)(aux + 2 * lane) = (uint16_t)V[(lane / 16) * 256 + (lane % 16)];
        S u[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) u[k] = (S)((x[k] - (S)st.base) & (S)0xFFFFu);
        wave_sync();
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) V[lane + 64 * k] = u[k];
        wave_sync();
        pack_vector<16>(V, st.W, out + packed_off + p_off, lane);
        // zero padding after this vector's aux block (up to the next one's start)
        const uint32_t a_end = a_off + 128u + __shfl(va, v, 64) - 128u;
        const uint32_t a_next = (a_end + 15) & ~15u;
        if (v + 1 < nvec && lane < a_next - a_end) aux[a_end - a_off + lane] = 0;
        wave_sync();
    }
    // header / meta / packed / aux gaps
    {
        const uint64_t gaps[3][2] = {{meta_off + sizeof(VecMeta) * nvec, packed_off},
                                     {packed_off + packed_total, aux_off},
                                     {aux_off + aux_len, total}};
        for (int g = 0; g < 3; ++g)
            for (uint64_t b = gaps[g][0] + threadIdx.x; b < gaps[g][1]; b += blockDim.x) out[b] = 0;
    }
}

// ENC_AUTO on the GPU: the encoding fls_writer.cpp encode_int_chunk(ENC_AUTO)
// picks, from the same estimates computed the same way -- per vector the
// FFOR width of the values and of their transposed deltas (the tail padded
// with the last value, as load_vec does), and the chunk's runs (adjacent
// values that differ, over its nrows values):
//   FFOR  sum(128 W + 32)          DELTA sum(128 W + 32 + 128)
//   RLE   runs (T/8) + nvec (32 + 128 + 640), none when 4 runs > nrows
//   DICT  the host's estimate (c.est_dict: a distinct count needs a hash set)
// smallest wins, ties to the earlier of FFOR, DELTA, RLE, DICT.  One extra
// read of the chunk's values.  Returns the encoding (block-uniform).
template <int T>
__device__ uint8_t choose_encoding(const EncChunk &c, FLS_LDS Sto<T> *Vall, FLS_LDS uint64_t *acc) {
    using S = Sto<T>;
    const uint32_t lane = threadIdx.x & 63, w = wave_index();
    FLS_LDS S *V = Vall + w * kVectorSize;
    const uint32_t n = c.nrows, nvec = (n + kVectorSize - 1) / kVectorSize;
    const uint8_t *in = (const uint8_t *)c.in;
    if (threadIdx.x < 3) acc[threadIdx.x] = 0;
    __syncthreads();
    uint64_t ffor = 0, delta = 0, diffs = 0;  // this wave's sums
    for (uint32_t v = w; v < nvec; v += kEncWaves) {
        const uint32_t vn = min(kVectorSize, n - v * kVectorSize);
        stage_values<T>(in, v, vn, V, lane);
        wave_sync();
        S x[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) x[k] = V[lane + 64 * k];
        const VecStat f = analyze_regs<T>(x);
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) x[k] = pos_value<T, true>(V, lane + 64 * k);
        const VecStat d = analyze_regs<T>(x);
        ffor += 128u * f.W + 32u;
        delta += 128u * d.W + 32u + 128u;
        // values that differ from their predecessor (row 0 of the vector
        // against the previous vector's last value)
        uint32_t nd = 0;
        for (uint32_t j = lane; j < vn; j += 64)
            if (j > 0) nd += V[j] != V[j - 1] ? 1u : 0u;
        if (lane == 0 && v > 0) {
            using U = typename std::conditional<T == 8, uint8_t,
                      typename std::conditional<T == 16, uint16_t,
                      typename std::conditional<T == 32, uint32_t, uint64_t>::type>::type>::type;
            const U last = ((const FLS_GLOBAL U *)in)[(size_t)v * kVectorSize - 1];
            nd += (S)last != V[0];
        }
        for (int o = 32; o >= 1; o >>= 1) nd += __shfl_xor(nd, o, 64);
        diffs += nd;
        wave_sync();
    }
    if (lane == 0) {
        __hip_atomic_fetch_add(acc + 0, ffor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(acc + 1, delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(acc + 2, diffs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    const uint64_t e_ffor = acc[0], e_delta = acc[1], runs = acc[2] + 1;
    const uint64_t e_rle = runs * 4 > n ? UINT64_MAX : runs * (T / 8) + (uint64_t)nvec * (32 + 128 + 640);
    uint64_t best = e_ffor;
    uint8_t enc = ENC_FFOR;
    if (e_delta < best) { best = e_delta; enc = ENC_DELTA; }
    if (e_rle < best) { best = e_rle; enc = ENC_RLE; }
    if (c.est_dict < best) { best = c.est_dict; enc = ENC_DICT; }
    __syncthreads();  // acc and V are reused by the encode
    return enc;
}

// One kernel per storage width: S = uint64_t for T = 64 chunks, uint32_t for
// T <= 32 (half the LDS and VGPRs: more waves per SIMD for the narrow types).
// The narrow kernel runs at 5 waves per SIMD (93 VGPRs, no spills): INT32
// FFOR 1.38 ms with u64 storage -> 1.08 ms (u32, 4 waves) -> 1.03 ms.  Forcing
// 6 waves (80 VGPRs, 6 spilled to scratch) gave byte mismatches in mixed
// launches, intermittently, so it is not used.
#ifndef FLS_ENC_NARROW_WAVES
#define FLS_ENC_NARROW_WAVES 5
#endif
template <typename S>
__global__ __launch_bounds__(256, sizeof(S) == 8 ? 4 : FLS_ENC_NARROW_WAVES) void encode_kernel(const EncChunk *__restrict__ chunks, uint32_t nchunks) {
    __shared__ S Vall[kEncWaves * kVectorSize];
    __shared__ uint32_t Wv[64];
    __shared__ int64_t Bv[64];
    __shared__ uint64_t Ov[67];
    const EncChunk c = chunks[blockIdx.x];
    FLS_LDS S *V = (FLS_LDS S *)Vall;
    FLS_LDS uint32_t *W = (FLS_LDS uint32_t *)Wv;
    FLS_LDS int64_t *B = (FLS_LDS int64_t *)Bv;
    FLS_LDS uint64_t *O = (FLS_LDS uint64_t *)Ov;
    uint8_t enc = c.enc;
    if (enc == ENC_ALP) return;  // alp_encode_kernel
    if (enc == ENC_AUTO) {
        if constexpr (sizeof(S) == 8) {
            enc = choose_encoding<64>(c, V, O);
        } else {
            switch (c.T) {
            case 8: enc = choose_encoding<8>(c, V, O); break;
            case 16: enc = choose_encoding<16>(c, V, O); break;
            default: enc = choose_encoding<32>(c, V, O); break;
            }
        }
        if (enc != ENC_FFOR && enc != ENC_DELTA) {
            // RLE: encode_rle_kernel, launched next, writes the chunk; DICT:
            // dict_encode_kernel (or the host, without a table)
            if (threadIdx.x == 0) *(FLS_GLOBAL uint64_t *)c.len_out = (uint64_t)enc << kEncShift;
            return;
        }
    }
    if (enc == ENC_RLE) return;  // explicit RLE chunks: encode_rle_kernel
    if (enc == ENC_DICT) {       // explicit DICT chunks: dict_encode_kernel (or the host)
        if (threadIdx.x == 0) *(FLS_GLOBAL uint64_t *)c.len_out = (uint64_t)ENC_DICT << kEncShift;
        return;
    }
    const bool delta = enc == ENC_DELTA;
    if constexpr (sizeof(S) == 8) {
        delta ? encode_chunk<64, true>(c, V, W, B, O) : encode_chunk<64, false>(c, V, W, B, O);
    } else {
        switch (c.T) {
        case 8: delta ? encode_chunk<8, true>(c, V, W, B, O) : encode_chunk<8, false>(c, V, W, B, O); break;
        case 16: delta ? encode_chunk<16, true>(c, V, W, B, O) : encode_chunk<16, false>(c, V, W, B, O); break;
        default: delta ? encode_chunk<32, true>(c, V, W, B, O) : encode_chunk<32, false>(c, V, W, B, O); break;
        }
    }
}

// RLE chunks in a kernel of their own (inlined into encode_kernel its
// registers made the FFOR / DELTA paths spill): explicit ENC_RLE chunks, and
// ENC_AUTO chunks for which encode_kernel, launched before it on the same
// stream, chose RLE (length 0, ENC_RLE in the top byte).  Every other chunk's
// block returns at once.
// (Its run-index, delta and packing registers get a budget of 2 waves per
// SIMD: at the FFOR kernel's 4-5 it spilled, and a spilling encoder build is
// the one that once wrote wrong rows)
template <typename S>
__global__ __launch_bounds__(256, 2) void encode_rle_kernel(const EncChunk *__restrict__ chunks, uint32_t nchunks) {
    __shared__ S Vall[kEncWaves * kVectorSize];
    __shared__ uint32_t Wv[64];
    __shared__ int64_t Bv[64];
    __shared__ uint64_t Ov[67];
    const EncChunk c = chunks[blockIdx.x];
    if (c.enc != ENC_RLE) {
        if (c.enc != ENC_AUTO) return;
        const uint64_t chosen = __builtin_amdgcn_readfirstlane(
            (uint32_t)(*(const FLS_GLOBAL uint64_t *)c.len_out >> kEncShift));
        if (chosen != ENC_RLE || (*(const FLS_GLOBAL uint64_t *)c.len_out & ((1ull << kEncShift) - 1)) != 0) return;
    }
    FLS_LDS S *V = (FLS_LDS S *)Vall;
    FLS_LDS uint32_t *W = (FLS_LDS uint32_t *)Wv;
    FLS_LDS int64_t *B = (FLS_LDS int64_t *)Bv;
    FLS_LDS uint64_t *O = (FLS_LDS uint64_t *)Ov;
    if constexpr (sizeof(S) == 8) {
        encode_rle_chunk<64>(c, V, W, B, O);
    } else {
        switch (c.T) {
        case 8: encode_rle_chunk<8>(c, V, W, B, O); break;
        case 16: encode_rle_chunk<16>(c, V, W, B, O); break;
        default: encode_rle_chunk<32>(c, V, W, B, O); break;
        }
    }
}



// ============================================================================
// ALP chunks of FLOAT / DOUBLE columns (fls_writer.cpp enc_alp, byte for
// byte).  One 256-thread block per chunk:
//   1. the chunk's (e, f) candidates: min(8, nvec) sampled vectors (32
//      values each) score every e <= kMaxE, f <= e by the CPU's cost
//      (bit width of the encoded range x samples + exceptions x (16 + T)),
//      each votes for its first cheapest; the up to five most-voted (ties to
//      the lower e (kMaxE + 1) + f, as the CPU's stable sort) are kept;
//   2. per vector (a wave each): the cheapest candidate on its own sample,
//      every value encoded (d = rint(n 10^e 10^-f), kept when d 10^f 10^-e
//      gives n's bits back), exceptions replaced by the first encoded value,
//      FOR base and width; then the layout (packed rows, 16-aligned aux
//      blocks of u16 positions + original values), and a second pass that
//      writes each vector at its place.
// The arithmetic is the CPU's, operation for operation, in the value's own
// precision (no contraction: products only), so the same values encode and
// the file is the CPU writer's.  Compute-light, HBM-bound (T/8 bytes read
// twice per value, the chunk written once).
// ============================================================================
__constant__ double kAlpF10D[kAlpMaxExpD + 1] = {FLS_ALP_F10_D};
__constant__ double kAlpIF10D[kAlpMaxExpD + 1] = {FLS_ALP_IF10_D};
__constant__ float kAlpF10F[kAlpMaxExpF + 1] = {FLS_ALP_F10_F};
__constant__ float kAlpIF10F[kAlpMaxExpF + 1] = {FLS_ALP_IF10_F};

template <class F>
struct AlpDev;
template <>
struct AlpDev<double> {
    using I = int64_t;
    using U = uint64_t;
    static constexpr int T = 64, kMaxE = kAlpMaxExpD;
    __device__ static double f10(int e) { return kAlpF10D[e]; }
    __device__ static double if10(int e) { return kAlpIF10D[e]; }
    __device__ static bool in_range(double x) { return __builtin_fabs(x) < 9.2233720368547748e18; }
    __device__ static I round(double x) { return (I)__builtin_rint(x); }
    __device__ static U bits(double x) { return (U)__double_as_longlong(x); }
    __device__ static double from_bits(U u) { return __longlong_as_double((long long)u); }
};
template <>
struct AlpDev<float> {
    using I = int32_t;
    using U = uint32_t;
    static constexpr int T = 32, kMaxE = kAlpMaxExpF;
    __device__ static float f10(int e) { return kAlpF10F[e]; }
    __device__ static float if10(int e) { return kAlpIF10F[e]; }
    __device__ static bool in_range(float x) { return __builtin_fabsf(x) < 2.1474835e9f; }
    __device__ static I round(float x) { return (I)__builtin_rintf(x); }
    __device__ static U bits(float x) { return (U)__float_as_uint(x); }
    __device__ static float from_bits(U u) { return __uint_as_float(u); }
};
// fls_writer.cpp alp_encode_one: n * 10^e * 10^-f rounded, verified bit-exact
template <class F>
__device__ __forceinline__ bool alp_enc1(F n, int e, int f, typename AlpDev<F>::I &d) {
    using A = AlpDev<F>;
    const F tmp = n * A::f10(e) * A::if10(f);
    if (!A::in_range(tmp)) return false;  // also NaN / inf
    d = A::round(tmp);
    const F back = (F)d * A::f10(f) * A::if10(e);
    return A::bits(back) == A::bits(n);
}
__device__ __forceinline__ uint32_t bitlen_u64(uint64_t x) { return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u; }
// (e, f) of combination index k in the CPU's loop order (e outer, f <= e inner)
__device__ __forceinline__ void alp_combo(uint32_t k, int &e, int &f) {
    int x = 0;
    while ((uint32_t)((x + 1) * (x + 2) / 2) <= k) ++x;
    e = x;
    f = (int)k - x * (x + 1) / 2;
}
// alp_cost over the wave's lanes < sn (one sample each): every lane gets the cost
template <class F>
__device__ __forceinline__ uint64_t alp_cost_wave(F x, bool have, uint32_t sn, int e, int f) {
    using A = AlpDev<F>;
    typename A::I d = 0;
    const bool ok = have && alp_enc1<F>(x, e, f, d);
    int64_t mn = ok ? (int64_t)d : INT64_MAX, mx = ok ? (int64_t)d : INT64_MIN;
    wave_minmax_i64(mn, mx);
    const uint32_t exc = (uint32_t)__popcll(__ballot(have && !ok));
    const uint64_t range = mn <= mx ? (uint64_t)((typename A::U)(typename A::I)mx - (typename A::U)(typename A::I)mn) : 0u;
    return (uint64_t)bitlen_u64(range) * sn + (uint64_t)exc * (16u + A::T);
}
constexpr uint32_t kAlpSampleVecs = 8, kAlpSamples = 32, kAlpCombos = 5;
constexpr uint32_t kAlpNcD = (kAlpMaxExpD + 1) * (kAlpMaxExpD + 2) / 2;  // 190 (e, f) pairs

template <class F>
__device__ void alp_chunk(const EncChunk &c, uint64_t *lds_v, uint64_t *lds_cost, uint32_t *lds_votes,
                          uint32_t *Wv, int64_t *Bv, uint64_t *Ov, int *combo) {
    using A = AlpDev<F>;
    using I = typename A::I;
    using U = typename A::U;
    constexpr int T = A::T, M = A::kMaxE;
    constexpr uint32_t NC = (M + 1) * (M + 2) / 2;
    using S = Sto<T>;
    const uint32_t lane = threadIdx.x & 63, w = wave_index();
    const uint32_t n = c.nrows, nvec = (n + kVectorSize - 1) / kVectorSize;
    const FLS_GLOBAL U *in = (const FLS_GLOBAL U *)c.in;
    FLS_GLOBAL uint8_t *out = (FLS_GLOBAL uint8_t *)c.out;
    // ---- 1. candidates: sampled vectors score every (e, f)
    const uint32_t nsv = min(kAlpSampleVecs, nvec);
    for (uint32_t t = threadIdx.x; t < nsv * NC; t += blockDim.x) {
        const uint32_t k = t / NC, ci = t % NC;
        const uint32_t v = (uint32_t)((uint64_t)k * nvec / nsv), b = v * kVectorSize;
        const uint32_t vn = min(kVectorSize, n - b), sn = min(kAlpSamples, vn);
        int e, f;
        alp_combo(ci, e, f);
        int64_t mn = INT64_MAX, mx = INT64_MIN;
        uint32_t exc = 0;
        for (uint32_t i = 0; i < sn; ++i) {
            const F x = A::from_bits(in[b + (uint64_t)i * vn / sn]);
            I d;
            if (!alp_enc1<F>(x, e, f, d)) { ++exc; continue; }
            mn = (int64_t)d < mn ? (int64_t)d : mn;
            mx = (int64_t)d > mx ? (int64_t)d : mx;
        }
        const uint64_t range = mn <= mx ? (uint64_t)((U)(I)mx - (U)(I)mn) : 0u;
        lds_cost[k * kAlpNcD + ci] = (uint64_t)bitlen_u64(range) * sn + (uint64_t)exc * (16u + T);
    }
    for (uint32_t i = threadIdx.x; i < (M + 1) * (M + 1); i += blockDim.x) lds_votes[i] = 0;
    __syncthreads();
    if (threadIdx.x < nsv) {  // each sampled vector votes for its first cheapest
        uint64_t best = UINT64_MAX;
        uint32_t bi = 0;
        for (uint32_t ci = 0; ci < NC; ++ci) {
            const uint64_t x = lds_cost[threadIdx.x * kAlpNcD + ci];
            if (x < best) { best = x; bi = ci; }
        }
        int e, f;
        alp_combo(bi, e, f);
        atomicAdd(&lds_votes[e * (M + 1) + f], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the most voted, ties to the lower index (stable sort)
        int nc = 0;
        for (; nc < (int)kAlpCombos; ++nc) {
            uint32_t bv = 0, bi = 0;
            for (uint32_t i = 0; i < (M + 1) * (M + 1); ++i)
                if (lds_votes[i] > bv) { bv = lds_votes[i]; bi = i; }
            if (bv == 0) break;
            combo[1 + nc] = (int)bi;
            lds_votes[bi] = 0;
        }
        if (nc == 0) { combo[1] = 0; nc = 1; }
        combo[0] = nc;
    }
    __syncthreads();
    const int ncombo = combo[0];
    FLS_LDS S *V = (FLS_LDS S *)lds_v + w * kVectorSize;
    // one vector: its (e, f), every value's d in V (exceptions replaced by the
    // first encoded value, the tail by the last), the exception bits per row k
    auto encode_vec = [&](uint32_t v, int &e, int &f, uint64_t (&excm)[16]) {
        const uint32_t b = v * kVectorSize, vn = min(kVectorSize, n - b);
        e = combo[1] / (M + 1);
        f = combo[1] % (M + 1);
        if (ncombo > 1) {  // level 2: the cheapest candidate on this vector's sample
            const uint32_t sn = min(kAlpSamples, vn);
            const bool have = lane < sn;
            const F x = have ? A::from_bits(in[b + (uint64_t)lane * vn / sn]) : (F)0;
            uint64_t best = UINT64_MAX;
            for (int k = 0; k < ncombo; ++k) {
                const int ek = combo[1 + k] / (M + 1), fk = combo[1 + k] % (M + 1);
                const uint64_t cst = alp_cost_wave<F>(x, have, sn, ek, fk);
                if (cst < best) { best = cst; e = ek; f = fk; }
            }
        }
        uint32_t first = kVectorSize;  // first encoded index of this lane
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t i = lane + 64 * k;
            I d = 0;
            const bool ok = i < vn && alp_enc1<F>(A::from_bits(in[b + i]), e, f, d);
            excm[k] = __ballot(i < vn && !ok);
            if (ok && i < first) first = i;
            V[i] = (S)(U)d;
        }
        for (int o = 32; o >= 1; o >>= 1) first = min(first, (uint32_t)__shfl_xor((int)first, o, 64));
        wave_sync();
        const S fill = first < kVectorSize ? V[first] : (S)0;
        wave_sync();
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k)
            if ((excm[k] >> lane) & 1ull) V[lane + 64 * k] = fill;
        wave_sync();
        const S last = V[vn - 1];
        for (uint32_t i = vn + lane; i < kVectorSize; i += 64) V[i] = last;
        wave_sync();
    };
    // ---- 2a. per vector: (e, f), exceptions, FOR base and width
    for (uint32_t v = w; v < nvec; v += kEncWaves) {
        int e, f;
        uint64_t excm[16];
        encode_vec(v, e, f, excm);
        S x[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) x[k] = V[lane + 64 * k];
        const VecStat st = analyze_regs<T>(x);
        uint32_t npos = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) npos += (uint32_t)__popcll(excm[k]);
        if (lane == 0) {
            Wv[v] = st.W;
            Bv[v] = st.base;
            Ov[v] = (uint64_t)npos | ((uint64_t)e << 16) | ((uint64_t)f << 24);
        }
        wave_sync();
    }
    __syncthreads();
    // ---- layout (assemble_chunk): packed rows back to back; the aux blocks of
    // vectors with exceptions, each 16-aligned; aux_len ends at the last block
    const uint64_t meta_off = sizeof(ChunkHeader);
    const uint64_t packed_off = (meta_off + sizeof(VecMeta) * nvec + 15) & ~15ull;
    const uint32_t pw = lane < nvec ? 128u * Wv[lane] : 0u;
    const uint32_t npos_l = lane < nvec ? (uint32_t)(Ov[lane] & 0xFFFF) : 0u;
    // this vector's aux block (fls_format.hpp alp_aux_bytes)
    const uint32_t sz = npos_l ? ((2u * npos_l + 15u) & ~15u) + npos_l * (uint32_t)(T / 8) : 0u;
    const uint32_t va = (sz + 15) & ~15u;
    uint32_t pincl = pw, aincl = va;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(pincl, d, 64), z = __shfl_up(aincl, d, 64);
        if (lane >= d) { pincl += y; aincl += z; }
    }
    const uint32_t poff = pincl - pw, aoff = aincl - va;
    const uint64_t packed_total = __shfl(pincl, 63, 64);
    const uint64_t aux_off = (packed_off + packed_total + 15) & ~15ull;
    uint32_t aend = npos_l ? aoff + sz : 0u;
    for (int o = 32; o >= 1; o >>= 1) aend = max(aend, (uint32_t)__shfl_xor((int)aend, o, 64));
    const uint64_t aux_len = aend;
    const uint64_t total = (aux_off + aux_len + kChunkAlign - 1) & ~(uint64_t)(kChunkAlign - 1);
    if (w == 0) {
        if (lane < nvec) {
            VecMeta m;
            m.packed_off = poff;
            m.for_base = Bv[lane];
            m.aux_off = npos_l ? aoff : 0u;
            m.nvals = (uint16_t)min(kVectorSize, n - lane * kVectorSize);
            m.bw = (uint8_t)Wv[lane];
            m.pad = 0;
            m.aux_count = (uint32_t)Ov[lane];
            const uint32_t *mw = reinterpret_cast<const uint32_t *>(&m);
            FLS_GLOBAL uint32_t *dm = reinterpret_cast<FLS_GLOBAL uint32_t *>(out + meta_off + sizeof(VecMeta) * lane);
#pragma unroll
            for (int i = 0; i < 8; ++i) dm[i] = mw[i];
        }
        if (lane == 0) {
            ChunkHeader h;
            h.magic = kChunkMagic;
            h.enc = ENC_ALP;
            h.T = (uint8_t)T;
            h.vbits = (uint8_t)T;
            h.is_str = 0;
            h.nvec = nvec;
            h.nvals = n;
            h.meta_off = meta_off;
            h.packed_off = packed_off;
            h.aux_off = aux_off;
            h.aux_len = aux_len;
            h.dict_count = 0;
            h.reserved0 = 0;
            h.reserved1 = 0;
            const uint32_t *hw = reinterpret_cast<const uint32_t *>(&h);
            FLS_GLOBAL uint32_t *dh = reinterpret_cast<FLS_GLOBAL uint32_t *>(out);
#pragma unroll
            for (int i = 0; i < 16; ++i) dh[i] = hw[i];
            *(FLS_GLOBAL uint64_t *)c.len_out = total | (uint64_t)ENC_ALP << kEncShift;
        }
    }
    // ---- 2b. every vector at its place: exceptions (positions, original
    // values), the packed d - base, the zero gaps of its aux block
    for (uint32_t v = w; v < nvec; v += kEncWaves) {
        int e, f;
        uint64_t excm[16];
        encode_vec(v, e, f, excm);
        const uint32_t b = v * kVectorSize;
        const uint32_t p_off = __shfl(poff, v, 64), a_off = __shfl(aoff, v, 64);
        const uint32_t npos = __shfl(npos_l, v, 64), vsz = __shfl(sz, v, 64);
        if (npos) {
            FLS_GLOBAL uint8_t *aux = out + aux_off + a_off;
            const uint32_t voff = (2u * npos + 15) & ~15u;
            uint32_t before = 0;
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) {
                const uint64_t m = excm[k];
                if ((m >> lane) & 1ull) {
                    const uint32_t r = before + (uint32_t)__popcll(m & ((1ull << lane) - 1));
                    const uint32_t i = lane + 64 * k;
                    *(FLS_GLOBAL uint16_t *)(aux + 2 * r) = (uint16_t)i;
                    *(FLS_GLOBAL U *)(aux + voff + (size_t)r * sizeof(F)) = in[b + i];
                }
                before += (uint32_t)__popcll(m);
            }
            for (uint32_t j = 2 * npos + lane; j < voff; j += 64) aux[j] = 0;   // positions' padding
            // up to the next vector's aux block (16-aligned)
            const uint32_t a_next = (a_off + vsz + 15) & ~15u;
            if (lane < a_next - (a_off + vsz) && a_off + vsz < aux_len) aux[vsz + lane] = 0;
        }
        const VecStat st{Bv[v], Wv[v]};
        S u[16];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) u[k] = (S)((uint64_t)V[lane + 64 * k] - (uint64_t)st.base) & (S)tmask_d(T);
        wave_sync();
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) V[lane + 64 * k] = u[k];
        wave_sync();
        pack_vector<T>(V, st.W, out + packed_off + p_off, lane);
        wave_sync();
    }
    // header / meta / packed / aux gaps
    {
        const uint64_t gaps[3][2] = {{meta_off + sizeof(VecMeta) * nvec, packed_off},
                                     {packed_off + packed_total, aux_off},
                                     {aux_off + aux_len, total}};
        for (int g = 0; g < 3; ++g)
            for (uint64_t q = gaps[g][0] + threadIdx.x; q < gaps[g][1]; q += blockDim.x) out[q] = 0;
    }
}

__global__ __launch_bounds__(256) void alp_encode_kernel(const EncChunk *__restrict__ chunks) {
    __shared__ uint64_t Vall[kEncWaves * kVectorSize];
    __shared__ uint64_t cost[kAlpSampleVecs * kAlpNcD];
    __shared__ uint32_t votes[(kAlpMaxExpD + 1) * (kAlpMaxExpD + 1)];
    __shared__ uint32_t Wv[64];
    __shared__ int64_t Bv[64];
    __shared__ uint64_t Ov[64];
    __shared__ int combo[1 + kAlpCombos];
    const EncChunk c = chunks[blockIdx.x];
    if (c.enc != ENC_ALP) return;
    if (c.T == 64) alp_chunk<double>(c, Vall, cost, votes, Wv, Bv, Ov, combo);
    else alp_chunk<float>(c, Vall, cost, votes, Wv, Bv, Ov, combo);
}

// ============================================================================
// DICT chunks of integer columns (fls_writer.cpp enc_dict_int, byte for byte):
// the chunk's distinct values sorted by their signed T-bit value form the
// dictionary (T/8 bytes each, the chunk's aux area), and each value's code --
// its position in the dictionary -- is FFOR-packed at T = 32 per vector, the
// tail padded with the last code.  Two kernels around encode_kernel:
//   dict_analyze_kernel: the distinct values of every ENC_DICT chunk and of
//     every ENC_AUTO chunk whose DICT estimate the GPU makes (kEstDictGpu):
//     first the CPU writer's 1,024-value sample rule (a chunk of more than
//     4,096 values whose sample holds more than 512 distinct values gets no
//     estimate), then every value into an open-addressing table in HBM
//     (atomicCAS on the key), and the estimate d T/8 + nvec (32 + 128
//     bitlen(d - 1)) -- est_dict's, so ENC_AUTO picks what the CPU picks;
//   dict_encode_kernel: for chunks that came out of encode_kernel as DICT,
//     the table's keys into LDS, a bitonic sort by signed value, each key's
//     position written back into the table as its code, then per vector the
//     values' codes looked up, FFOR-analysed and packed as encode_chunk does.
// Integer work bound by the table probes (L2-resident: 1.5 MB per 65,536-row
// chunk) and the input reads; no MFMA.
// ============================================================================
constexpr uint64_t kDictEmpty = ~0ull;   // an empty slot (the value ~0 itself is kept in the header)
struct DictHeader {                      // the table's first 64 bytes
    uint32_t count;                      // distinct values in keys[] (kDictEmpty excluded)
    uint32_t has_empty;                  // the value ~0ull (T = 64 only) occurs
    uint32_t empty_code;                 // its code (dict_encode_kernel)
    uint32_t pad[13];
};
static_assert(sizeof(DictHeader) == 64, "DICT table header is 64 B");

__device__ __forceinline__ uint64_t dict_hash(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
// value i of a chunk (zero-extended T-bit)
__device__ __forceinline__ uint64_t load_value(const uint8_t *in, uint32_t T, uint64_t i) {
    switch (T) {
    case 8: return ((const FLS_GLOBAL uint8_t *)in)[i];
    case 16: return ((const FLS_GLOBAL uint16_t *)in)[i];
    case 32: return ((const FLS_GLOBAL uint32_t *)in)[i];
    default: return ((const FLS_GLOBAL uint64_t *)in)[i];
    }
}
// Bitonic sort of the n (a power of two) keys of K ascending, by the block.
__device__ __forceinline__ void block_bitonic(FLS_LDS uint64_t *K, uint32_t n) {
    for (uint32_t k = 2; k <= n; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = K[i], b = K[l];
                    const bool up = (i & k) == 0;
                    if (up ? a > b : a < b) {
                        K[i] = b;
                        K[l] = a;
                    }
                }
            }
            __syncthreads();
        }
}
__device__ __forceinline__ uint32_t block_sum(uint32_t x, FLS_LDS uint32_t *red) {
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t t = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; ++w) t += red[w];
    __syncthreads();
    return t;
}

__global__ __launch_bounds__(256) void dict_analyze_kernel(EncChunk *__restrict__ chunks) {
    __shared__ uint64_t smp[1024];
    __shared__ uint32_t red[4];
    __shared__ uint32_t cnt, has_empty;
    EncChunk &cref = chunks[blockIdx.x];
    const EncChunk c = cref;
    const bool auto_est = c.enc == ENC_AUTO && c.est_dict == kEstDictGpu;
    if (!c.dict_tab || !(c.enc == ENC_DICT || auto_est)) return;
    const uint32_t n = c.nrows, T = c.T, nvec = (n + kVectorSize - 1) / kVectorSize;
    const uint8_t *in = (const uint8_t *)c.in;
    FLS_LDS uint64_t *S = (FLS_LDS uint64_t *)smp;
    if (auto_est && n > 4096) {
        // the CPU's sample: values i n / 1024, i < 1024, more than 512 distinct = no DICT
        for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) S[i] = load_value(in, T, (uint64_t)i * n / 1024);
        __syncthreads();
        block_bitonic(S, 1024);
        uint32_t dd = 0;
        for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) dd += (i == 0 || S[i] != S[i - 1]) ? 1u : 0u;
        dd = block_sum(dd, (FLS_LDS uint32_t *)red);
        if (dd > 512) {
            if (threadIdx.x == 0) cref.est_dict = UINT64_MAX;
            return;
        }
    }
    DictHeader *hdr = (DictHeader *)c.dict_tab;
    uint64_t *keys = (uint64_t *)(c.dict_tab + sizeof(DictHeader));
    const uint32_t cap = enc_dict_cap(n), mask = cap - 1;
    for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) keys[i] = kDictEmpty;
    if (threadIdx.x == 0) {
        cnt = 0;
        has_empty = 0;
    }
    __syncthreads();  // (also orders the block's key stores before its CAS probes)
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t x = load_value(in, T, i);
        if (x == kDictEmpty) {
            has_empty = 1;
            continue;
        }
        uint32_t h = (uint32_t)dict_hash(x) & mask;
        for (uint32_t probe = 0; probe < cap; ++probe) {
            // a plain read first: a value already in the table (every repeat
            // of a low-cardinality column) costs no atomic
            uint64_t old = __hip_atomic_load(keys + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == kDictEmpty) {
                old = atomicCAS((unsigned long long *)(keys + h), (unsigned long long)kDictEmpty, (unsigned long long)x);
                if (old == kDictEmpty) {
                    atomicAdd(&cnt, 1u);
                    break;
                }
            }
            if (old == x) break;
            h = (h + 1) & mask;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        hdr->count = cnt;
        hdr->has_empty = has_empty;
        if (auto_est) {
            const uint64_t d = (uint64_t)cnt + has_empty;
            const uint64_t dm1 = d - 1 ? d - 1 : 0;
            const uint32_t bl = dm1 ? 64u - (uint32_t)__builtin_clzll(dm1) : 0u;
            cref.est_dict = d > 65536 ? UINT64_MAX : d * (T / 8) + (uint64_t)nvec * (32 + 128ull * bl);
        }
    }
}

// code of value x: its slot's code (the table holds every value of the chunk)
__device__ __forceinline__ uint32_t dict_code(const uint64_t *keys, const uint32_t *codes, uint32_t mask,
                                              uint32_t empty_code, uint64_t x) {
    if (x == kDictEmpty) return empty_code;
    uint32_t h = (uint32_t)dict_hash(x) & mask;
    for (uint32_t probe = 0; probe <= mask && keys[h] != x; ++probe) h = (h + 1) & mask;
    return codes[h];
}

__global__ __launch_bounds__(256) void dict_encode_kernel(const EncChunk *__restrict__ chunks) {
    __shared__ uint64_t U[kDictGpuMax];              // the sorted distinct values (order keys)
    __shared__ uint32_t Vall[kEncWaves * kVectorSize];
    __shared__ uint32_t Wv[64];
    __shared__ int64_t Bv[64];
    __shared__ uint64_t Ov[67];
    __shared__ uint32_t fill;
    const EncChunk c = chunks[blockIdx.x];
    if (!c.dict_tab || !(c.enc == ENC_DICT || c.enc == ENC_AUTO)) return;
    const uint64_t lw = *(const FLS_GLOBAL uint64_t *)c.len_out;
    if ((uint32_t)(lw >> kEncShift) != ENC_DICT || (lw & ((1ull << kEncShift) - 1)) != 0) return;
    const DictHeader *hdr = (const DictHeader *)c.dict_tab;
    uint64_t *keys = (uint64_t *)(c.dict_tab + sizeof(DictHeader));
    const uint32_t n = c.nrows, T = c.T, nvec = (n + kVectorSize - 1) / kVectorSize;
    const uint32_t cap = enc_dict_cap(n), mask = cap - 1;
    uint32_t *codes = (uint32_t *)(keys + cap);
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(hdr->count);
    const uint32_t has_empty = __builtin_amdgcn_readfirstlane(hdr->has_empty);
    const uint32_t d = cnt + has_empty;
    if (d > kDictGpuMax || d == 0) return;  // the host encodes it (length stays 0)
    FLS_LDS uint64_t *K = (FLS_LDS uint64_t *)U;
    // ---- the distinct values, ordered by their signed T-bit value: the sort
    // key is sext(x) with the sign bit flipped (unsigned order = signed order)
    const uint64_t flip = 1ull << 63;
    if (threadIdx.x == 0) fill = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
        const uint64_t x = keys[i];
        if (x != kDictEmpty) K[atomicAdd(&fill, 1u)] = (uint64_t)sext_d(x, T) ^ flip;
    }
    __syncthreads();
    uint32_t P = 1;
    while (P < d) P <<= 1;
    if (threadIdx.x == 0 && has_empty) K[cnt] = (uint64_t)sext_d(kDictEmpty, T) ^ flip;
    for (uint32_t i = d + threadIdx.x; i < P; i += blockDim.x) K[i] = ~0ull;  // padding sorts last
    __syncthreads();
    block_bitonic(K, P);
    // ---- each value's code = its position; the dictionary (put_word layout)
    const uint64_t tm = tmask_d(T);
    const uint64_t packed_off = (sizeof(ChunkHeader) + sizeof(VecMeta) * (uint64_t)nvec + 15) & ~15ull;
    FLS_GLOBAL uint8_t *out = (FLS_GLOBAL uint8_t *)c.out;
    __shared__ uint32_t empty_code_s;
    for (uint32_t i = threadIdx.x; i < d; i += blockDim.x) {
        const uint64_t x = (K[i] ^ flip) & tm;
        if (x == kDictEmpty) {
            empty_code_s = i;
        } else {
            uint32_t h = (uint32_t)dict_hash(x) & mask;
            for (uint32_t probe = 0; probe < cap && keys[h] != x; ++probe) h = (h + 1) & mask;
            codes[h] = i;
        }
    }
    __syncthreads();  // codes[] written by the block before it reads them
    const uint32_t empty_code = has_empty ? empty_code_s : 0u;
    // ---- codes -> FFOR (T = 32) per vector, as encode_chunk<32, false>
    const uint32_t lane = threadIdx.x & 63, w = wave_index();
    FLS_LDS uint32_t *V = (FLS_LDS uint32_t *)Vall + w * kVectorSize;
    FLS_LDS uint32_t *W = (FLS_LDS uint32_t *)Wv;
    FLS_LDS int64_t *B = (FLS_LDS int64_t *)Bv;
    FLS_LDS uint64_t *O = (FLS_LDS uint64_t *)Ov;
    const uint8_t *in = (const uint8_t *)c.in;
    uint32_t done = 0;
    for (uint32_t r = 0; r < nvec; r += kEncWaves) {
        const uint32_t v = r + w;
        const bool act = v < nvec;
        VecStat st{0, 0};
        if (act) {
            const uint32_t vn = min(kVectorSize, n - v * kVectorSize);
            for (uint32_t j = lane; j < kVectorSize; j += 64)
                V[j] = dict_code(keys, codes, mask, empty_code, load_value(in, T, (uint64_t)v * kVectorSize + min(j, vn - 1)));
            wave_sync();
            uint32_t x[16];
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) x[k] = V[lane + 64 * k];
            st = analyze_regs<32>(x);
            if (lane == 0) {
                W[v] = st.W;
                B[v] = st.base;
            }
            wave_sync();
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k) V[lane + 64 * k] = x[k] - (uint32_t)st.base;
            wave_sync();
        }
        __syncthreads();
        if (act) {
            uint32_t off = done;
            for (uint32_t i = r; i < v; ++i) off += 128u * W[i];
            pack_vector<32>(V, st.W, out + packed_off + off, lane);
        }
        for (uint32_t i = r; i < min(r + (uint32_t)kEncWaves, nvec); ++i) done += 128u * W[i];
        wave_sync();
    }
    __syncthreads();
    // ---- chunk layout (assemble_chunk): the dictionary is the aux area, padded to 16 B
    const uint64_t meta_off = sizeof(ChunkHeader);
    const uint64_t dict_bytes = (uint64_t)d * (T / 8);
    const uint64_t aux_len = (dict_bytes + 15) & ~15ull;
    if (w == 0) {
        const uint32_t pw = lane < nvec ? 128u * W[lane] : 0u;
        uint32_t incl = pw;
        for (uint32_t dd = 1; dd < 64; dd <<= 1) {
            const uint32_t y = __shfl_up(incl, dd, 64);
            if (lane >= dd) incl += y;
        }
        const uint64_t packed_total = rl(incl, 63);
        const uint64_t aux_off = (packed_off + packed_total + 15) & ~15ull;
        const uint64_t total = (aux_off + aux_len + kChunkAlign - 1) & ~(uint64_t)(kChunkAlign - 1);
        if (lane < nvec) {
            VecMeta m;
            m.packed_off = incl - pw;
            m.for_base = B[lane];
            m.aux_off = 0;
            m.nvals = (uint16_t)min(kVectorSize, n - lane * kVectorSize);
            m.bw = (uint8_t)W[lane];
            m.pad = 0;
            m.aux_count = 0;
            const uint32_t *mw = reinterpret_cast<const uint32_t *>(&m);
            FLS_GLOBAL uint32_t *dm = reinterpret_cast<FLS_GLOBAL uint32_t *>(out + meta_off + sizeof(VecMeta) * lane);
#pragma unroll
            for (int i = 0; i < 8; ++i) dm[i] = mw[i];
        }
        if (lane == 0) {
            ChunkHeader h;
            h.magic = kChunkMagic;
            h.enc = ENC_DICT;
            h.T = 32;
            h.vbits = (uint8_t)T;
            h.is_str = 0;
            h.nvec = nvec;
            h.nvals = n;
            h.meta_off = meta_off;
            h.packed_off = packed_off;
            h.aux_off = aux_off;
            h.aux_len = aux_len;
            h.dict_count = d;
            h.reserved0 = 0;
            h.reserved1 = 0;
            const uint32_t *hw = reinterpret_cast<const uint32_t *>(&h);
            FLS_GLOBAL uint32_t *dh = reinterpret_cast<FLS_GLOBAL uint32_t *>(out);
#pragma unroll
            for (int i = 0; i < 16; ++i) dh[i] = hw[i];
            O[64] = packed_total;
            O[65] = aux_off;
            O[66] = total;
        }
    }
    __syncthreads();
    const uint64_t packed_total = O[64], aux_off = O[65], total = O[66];
    // the dictionary, byte by byte in the put_word layout (little-endian T/8 bytes)
    for (uint32_t i = threadIdx.x; i < d; i += blockDim.x) {
        const uint64_t x = (K[i] ^ flip) & tm;
        FLS_GLOBAL uint8_t *dp = out + aux_off + (uint64_t)i * (T / 8);
        for (uint32_t b = 0; b < T / 8; ++b) dp[b] = (uint8_t)(x >> (8 * b));
    }
    {
        const uint64_t gaps[3][2] = {{meta_off + sizeof(VecMeta) * nvec, packed_off},
                                     {packed_off + packed_total, aux_off},
                                     {aux_off + dict_bytes, total}};
        for (int g = 0; g < 3; ++g)
            for (uint64_t b = gaps[g][0] + threadIdx.x; b < gaps[g][1]; b += blockDim.x) out[b] = 0;
    }
    if (threadIdx.x == 0) *(FLS_GLOBAL uint64_t *)c.len_out = total | (uint64_t)ENC_DICT << kEncShift;
}


// ---- VARCHAR / BLOB dictionaries (build_str_dict's order: first appearance) ----
// Four steps on the context's stream, no host round trip between them:
//   insert (a thread per row, the whole grid): the row's bytes hashed a word
//     at a time, then linear probing of an open-addressing table in HBM whose
//     slot holds the row that claimed it (atomicCAS on an empty slot; a slot
//     already held is compared word by word, no atomic), the smallest row
//     holding its string (atomicMin: the first appearance) and, once sorted,
//     its code; a global count of distinct strings, and past `limit` an
//     overflow flag that ends the other rows early;
//   sort (one block): the distinct strings as (first row, slot) in LDS, a
//     bitonic sort by first row numbers the codes;
//   codes (the grid): each row's code through its slot.
// The bytes are 8-aligned with 16 readable bytes past the last string, so a
// string is read as aligned qwords whatever its offset.
__device__ __forceinline__ uint64_t str_word(const uint8_t *bytes, uint32_t p, uint32_t left) {
    const uint64_t *q = reinterpret_cast<const uint64_t *>(bytes + (p & ~7u));
    const uint32_t sh = 8 * (p & 7);
    uint64_t w = q[0] >> sh;
    if (sh) w |= q[1] << (64 - sh);
    return left >= 8 ? w : w & ((1ull << (8 * left)) - 1);
}
__device__ __forceinline__ uint64_t str_hash_d(const uint8_t *bytes, uint32_t p, uint32_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    for (uint32_t k = 0; k < n; k += 8) h = dict_hash(h ^ str_word(bytes, p + k, n - k));
    return h;
}
__device__ __forceinline__ bool str_eq_d(const uint8_t *bytes, const uint32_t *offs, uint32_t a, uint32_t b) {
    const uint32_t a0 = offs[a], la = offs[a + 1] - a0, b0 = offs[b], lb = offs[b + 1] - b0;
    if (la != lb) return false;
    for (uint32_t k = 0; k < la; k += 8)
        if (str_word(bytes, a0 + k, la - k) != str_word(bytes, b0 + k, la - k)) return false;
    return true;
}
constexpr uint32_t kStrEmpty = 0xFFFFFFFFu;

__global__ __launch_bounds__(256) void str_dict_insert_kernel(const uint8_t *__restrict__ bytes,
                                                              const uint32_t *__restrict__ offs, uint32_t n,
                                                              uint32_t limit, uint32_t *__restrict__ slots,
                                                              uint32_t *__restrict__ row_slot, StrDictInfo *info) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (__hip_atomic_load(&info->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const uint32_t cap = enc_dict_cap(n), mask = cap - 1;
    uint32_t *srow = slots, *sfirst = slots + cap;
    const uint32_t p = offs[i], len = offs[i + 1] - p;
    uint32_t s = (uint32_t)str_hash_d(bytes, p, len) & mask;
    for (uint32_t probe = 0; probe < cap; ++probe) {
        uint32_t r = __hip_atomic_load(srow + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (r == kStrEmpty) {
            r = atomicCAS(srow + s, kStrEmpty, i);
            if (r == kStrEmpty) {
                if (atomicAdd(&info->count, 1u) >= limit) atomicOr(&info->overflow, 1u);
                break;
            }
        }
        if (str_eq_d(bytes, offs, r, i)) break;
        s = (s + 1) & mask;
    }
    // first appearance: only a row below the slot's current first row takes
    // the atomic (a low-cardinality column would otherwise send every row's
    // atomicMin to the same few addresses)
    if (__hip_atomic_load(sfirst + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > i) atomicMin(sfirst + s, i);
    row_slot[i] = s;
}

__global__ __launch_bounds__(1024) void str_dict_sort_kernel(const uint32_t *__restrict__ offs, uint32_t n,
                                                             uint32_t *__restrict__ slots, uint32_t *__restrict__ entries,
                                                             StrDictInfo *__restrict__ info) {
    __shared__ uint64_t K[kDictGpuMax];
    __shared__ uint32_t fill;
    __shared__ unsigned long long ebytes;
    const uint32_t cap = enc_dict_cap(n);
    const uint32_t *srow = slots, *sfirst = slots + cap;
    uint32_t *scode = slots + 2 * cap;
    const uint32_t d = info->count;
    if (info->overflow || d > kDictGpuMax) {
        if (threadIdx.x == 0) info->big = !info->overflow;
        return;
    }
    if (threadIdx.x == 0) {
        fill = 0;
        ebytes = 0;
    }
    __syncthreads();
    // the distinct strings as (first row << 32 | slot), sorted by first row
    for (uint32_t s = threadIdx.x; s < cap; s += blockDim.x) {
        const uint32_t r = srow[s];
        if (r == kStrEmpty) continue;
        K[atomicAdd(&fill, 1u)] = (uint64_t)sfirst[s] << 32 | s;
        atomicAdd(&ebytes, (unsigned long long)(offs[r + 1] - offs[r]));
    }
    uint32_t P = 1;
    while (P < d) P <<= 1;
    __syncthreads();
    for (uint32_t i = d + threadIdx.x; i < P; i += blockDim.x) K[i] = ~0ull;
    __syncthreads();
    block_bitonic((FLS_LDS uint64_t *)K, P);
    for (uint32_t k = threadIdx.x; k < d; k += blockDim.x) {
        scode[(uint32_t)K[k]] = k;
        entries[k] = (uint32_t)(K[k] >> 32);
    }
    if (threadIdx.x == 0) {
        info->big = 0;
        info->entry_bytes = ebytes;
    }
}

__global__ __launch_bounds__(256) void str_dict_codes_kernel(uint32_t n, const uint32_t *__restrict__ slots,
                                                             const uint32_t *__restrict__ row_slot,
                                                             uint32_t *__restrict__ codes, const StrDictInfo *info) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || info->overflow || info->big) return;
    codes[i] = slots[2 * enc_dict_cap(n) + row_slot[i]];
}

// One lane per string.  The table is staged in LDS; a lane reads its string
// 8 bytes at a time from two aligned qwords (the L1 serves the overlap of
// consecutive steps) and writes its codes byte by byte into its own region.
__global__ __launch_bounds__(256) void fsst_compress_kernel(const uint8_t *__restrict__ bytes,
                                                            const uint32_t *__restrict__ offs, uint32_t n,
                                                            const FsstCTable *__restrict__ tab,
                                                            uint8_t *__restrict__ codes, uint32_t *__restrict__ clen) {
    __shared__ FsstCTable t;
    {
        const v4u *src = reinterpret_cast<const v4u *>(tab);
        v4u *dst = reinterpret_cast<v4u *>(&t);
        for (uint32_t k = threadIdx.x; k < sizeof(FsstCTable) / 16; k += blockDim.x) dst[k] = src[k];
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t p = offs[i];
    const uint32_t e = offs[i + 1];
    uint8_t *out = codes + 2ull * p;
    uint32_t o = 0;
    while (p < e) {
        const uint32_t r = e - p;
        const uint64_t *q = reinterpret_cast<const uint64_t *>(bytes + (p & ~7u));
        const uint32_t sh = 8 * (p & 7);
        const uint64_t lo = q[0], hi = q[1];
        uint64_t w = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
        if (r < 8) w &= (1ull << (8 * r)) - 1;
        int c = -1;
        if (r >= 2) {
            const uint32_t b = fsst_cbucket((uint32_t)(w & 0xFFFF));
            for (uint32_t j = t.start[b], j1 = t.start[b + 1]; j < j1; ++j) {
                const uint32_t cc = t.codes[j], L = t.len[cc];
                const uint64_t m = L >= 8 ? ~0ull : (1ull << (8 * L)) - 1;
                if (L <= r && ((w ^ t.sym[cc]) & m) == 0) {
                    c = (int)cc;
                    break;
                }
            }
        }
        if (c < 0) c = t.one[w & 0xFF];
        if (c >= 0) {
            out[o++] = (uint8_t)c;
            p += max(1u, (uint32_t)t.len[c]);
        } else {
            out[o++] = (uint8_t)kFsstEscape;
            out[o++] = (uint8_t)(w & 0xFF);
            ++p;
        }
    }
    clen[i] = o;
}

}  // namespace

hipError_t launch_fsst_compress(const uint8_t *d_bytes, const uint32_t *d_offs, uint32_t n, const FsstCTable *d_tab,
                                uint8_t *d_codes, uint32_t *d_clen, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(fsst_compress_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_bytes, d_offs, n, d_tab,
                       d_codes, d_clen);
    return hipGetLastError();
}

hipError_t launch_str_dict(const uint8_t *d_bytes, const uint32_t *d_offs, uint32_t n, uint32_t limit,
                           uint32_t *d_slots, uint32_t *d_row_slot, uint32_t *d_codes, uint32_t *d_entries,
                           StrDictInfo *d_info, hipStream_t stream) {
    if (n == 0) return hipErrorInvalidValue;
    const uint32_t cap = enc_dict_cap(n), grid = (n + 255) / 256;
    hipError_t e = hipMemsetAsync(d_slots, 0xFF, 8ull * cap, stream);   // row and first row: empty
    if (e == hipSuccess) e = hipMemsetAsync(d_info, 0, sizeof(StrDictInfo), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(str_dict_insert_kernel, dim3(grid), dim3(256), 0, stream, d_bytes, d_offs, n, limit, d_slots,
                       d_row_slot, d_info);
    hipLaunchKernelGGL(str_dict_sort_kernel, dim3(1), dim3(1024), 0, stream, d_offs, n, d_slots, d_entries, d_info);
    hipLaunchKernelGGL(str_dict_codes_kernel, dim3(grid), dim3(256), 0, stream, n, d_slots, d_row_slot, d_codes,
                       d_info);
    return hipGetLastError();
}

uint64_t enc_slot_bytes(uint32_t T, uint32_t nrows, uint8_t enc) {
    const uint64_t nvec = (nrows + kVectorSize - 1) / kVectorSize;
    const uint64_t packed_off = (sizeof(ChunkHeader) + sizeof(VecMeta) * nvec + 15) & ~15ull;
    const uint64_t delta = packed_off + 128ull * T * nvec + (enc == ENC_FFOR ? 0ull : 128ull * nvec);
    // RLE: T = 16 packing, aux = 128 B of bases + up to 1,024 run values per vector
    const uint64_t rle = packed_off + 128ull * 16 * nvec + nvec * ((128ull + 1024ull * (T / 8) + 15) & ~15ull);
    // DICT: codes of at most 16 bits (65,536 distinct values) FFOR-packed at T = 32, the dictionary
    const uint64_t dict = packed_off + 128ull * 17 * nvec + (((uint64_t)nrows * (T / 8) + 15) & ~15ull);
    // ALP: W <= T, and at most every value an exception (16-aligned aux blocks)
    const uint64_t alp = packed_off + 128ull * T * nvec + nvec * ((alp_aux_bytes(kVectorSize, T) + 15) & ~15ull);
    if (enc == ENC_ALP) return (alp + kChunkAlign - 1) & ~(uint64_t)(kChunkAlign - 1);
    const uint64_t need = enc == ENC_RLE    ? rle
                          : enc == ENC_AUTO ? std::max({delta, rle, dict})  // AUTO may pick any
                          : enc == ENC_DICT ? dict
                                            : delta;
    return (need + kChunkAlign - 1) & ~(uint64_t)(kChunkAlign - 1);
}

hipError_t launch_encode(EncChunk *d_chunks, uint32_t n_wide, uint32_t n_narrow, hipStream_t stream, bool rle,
                         bool dict, bool alp) {
    if (alp && n_wide + n_narrow)
        hipLaunchKernelGGL(alp_encode_kernel, dim3(n_wide + n_narrow), dim3(256), 0, stream, d_chunks);
    if (dict && n_wide + n_narrow)
        hipLaunchKernelGGL(dict_analyze_kernel, dim3(n_wide + n_narrow), dim3(256), 0, stream, d_chunks);
    if (n_wide) hipLaunchKernelGGL(encode_kernel<uint64_t>, dim3(n_wide), dim3(64 * kEncWaves), 0, stream, d_chunks, n_wide);
    if (n_narrow)
        hipLaunchKernelGGL(encode_kernel<uint32_t>, dim3(n_narrow), dim3(64 * kEncWaves), 0, stream, d_chunks + n_wide,
                           n_narrow);
    if (rle && n_wide)
        hipLaunchKernelGGL(encode_rle_kernel<uint64_t>, dim3(n_wide), dim3(64 * kEncWaves), 0, stream, d_chunks, n_wide);
    if (rle && n_narrow)
        hipLaunchKernelGGL(encode_rle_kernel<uint32_t>, dim3(n_narrow), dim3(64 * kEncWaves), 0, stream,
                           d_chunks + n_wide, n_narrow);
    if (dict && n_wide + n_narrow)
        hipLaunchKernelGGL(dict_encode_kernel, dim3(n_wide + n_narrow), dim3(256), 0, stream, d_chunks);
    return hipGetLastError();
}


}  // namespace fls

using namespace fls;

#define ENC_HIP(expr)                                                                           \
    do {                                                                                        \
        const hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) return fail(FLS_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

extern "C" {

uint64_t fls_encode_slot_bytes(uint8_t type, uint8_t encoding, uint32_t rowgroup_rows) {
    const int T = type_value_bits(type);
    if (T == 0 || type_is_float(type)) return 0;
    return enc_slot_bytes((uint32_t)T, rowgroup_rows, encoding);
}

int fls_encode_device(int device, uint8_t type, uint8_t encoding, const void *d_values, uint64_t nrows,
                      uint32_t rowgroup_rows, void *d_out, uint64_t *chunk_lens, float *kernel_ms) {
    const int T = type_value_bits(type);
    if (T == 0 || type_is_float(type) || type_is_string(type))
        return fail(FLS_ERR_ARG, "fls_encode_device: integer types only (type %u)", type);
    if (encoding != ENC_FFOR && encoding != ENC_DELTA)
        return fail(FLS_ERR_ARG, "fls_encode_device: FFOR or DELTA only (encoding %u)", encoding);
    if (!d_values || !d_out || !chunk_lens || nrows == 0) return fail(FLS_ERR_ARG, "fls_encode_device: bad argument");
    if (rowgroup_rows == 0 || rowgroup_rows > kRowGroupSize || rowgroup_rows % kVectorSize)
        return fail(FLS_ERR_ARG, "fls_encode_device: row group size %u", rowgroup_rows);
    if (((uintptr_t)d_values & 15) || ((uintptr_t)d_out & 15))
        return fail(FLS_ERR_ARG, "fls_encode_device: buffers must be 16-byte aligned");
    const uint64_t nrg = (nrows + rowgroup_rows - 1) / rowgroup_rows;
    const uint64_t slot = enc_slot_bytes((uint32_t)T, rowgroup_rows, encoding);
    ENC_HIP(hipSetDevice(device));
    // scratch: one area per chunk, kept per device across calls (grown as needed)
    static std::mutex mu;
    static std::vector<std::pair<uint8_t *, uint64_t>> cache;
    std::lock_guard<std::mutex> lock(mu);
    if ((size_t)device >= cache.size()) cache.resize(device + 1, {nullptr, 0});
    const uint64_t need = nrg * enc_scratch_bytes();
    if (cache[device].second < need) {
        hipFree(cache[device].first);
        cache[device] = {nullptr, 0};
        ENC_HIP(hipMalloc((void **)&cache[device].first, need));
        cache[device].second = need;
    }
    uint8_t *scratch = cache[device].first;
    std::vector<EncChunk> desc(nrg);
    EncChunk *d_desc = nullptr;
    uint64_t *d_lens = nullptr;
    ENC_HIP(hipMalloc((void **)&d_desc, nrg * sizeof(EncChunk)));
    const hipError_t ea = hipMalloc((void **)&d_lens, nrg * sizeof(uint64_t));
    if (ea != hipSuccess) {
        hipFree(d_desc);
        return fail(FLS_ERR_DEVICE, "hipMalloc: %s", hipGetErrorString(ea));
    }
    for (uint64_t i = 0; i < nrg; ++i) {
        EncChunk &c = desc[i];
        c.in = (uint64_t)(uintptr_t)d_values + i * rowgroup_rows * (uint64_t)(T / 8);
        c.out = (uint64_t)(uintptr_t)d_out + i * slot;
        c.len_out = (uint64_t)(uintptr_t)(d_lens + i);
        c.scratch = (uint64_t)(uintptr_t)(scratch + i * enc_scratch_bytes());
        c.nrows = (uint32_t)std::min<uint64_t>(rowgroup_rows, nrows - i * rowgroup_rows);
        c.T = (uint8_t)T;
        c.enc = encoding;
        c.pad[0] = c.pad[1] = 0;
        c.est_dict = UINT64_MAX;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipMemcpy(d_desc, desc.data(), nrg * sizeof(EncChunk), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipEventRecord(e0, nullptr);
    if (e == hipSuccess)
        e = launch_encode(d_desc, T == 64 ? (uint32_t)nrg : 0u, T == 64 ? 0u : (uint32_t)nrg, nullptr, false);
    if (e == hipSuccess) e = hipEventRecord(e1, nullptr);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess) e = hipMemcpy(chunk_lens, d_lens, nrg * sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess)  // the kernel puts the encoding in the top byte
        for (uint64_t i = 0; i < nrg; ++i) chunk_lens[i] &= (1ull << kEncShift) - 1;
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    hipFree(d_desc);
    hipFree(d_lens);
    if (e != hipSuccess) return fail(FLS_ERR_DEVICE, "fls_encode_device: %s", hipGetErrorString(e));
    if (kernel_ms) *kernel_ms = ms;
    return 0;
}

}  // extern "C"
