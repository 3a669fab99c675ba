// fls_decode.hip -- MI355X (gfx950) FastLanes vector decode.
//
// Replaces the decode inside RowgroupReader::materialize()
// (reference src/fastlanes_facade.cpp:48) for the north-star codecs:
// interleaved bit-unpack at every width, FFOR, unified-transposed DELTA,
// DICT gather (integers and DuckDB string_t) and FastLanes-RLE.
//
// Work decomposition: one 64-lane wave decodes one 1024-value vector.
//   1. stage: the vector's 128*W packed bytes are streamed HBM -> LDS with
//      16 B/lane loads (1 KiB per wave-instruction), plus one zero word-row;
//   2. unpack: lane handles 16-byte "chunks" ci (row R = ci/8, 16-byte column
//      qc = ci%8 of the 128-byte word-row).  For any T the chunk's values are
//      a funnel shift of word-rows k = R*W/T and k+1 (two ds_read_b128),
//      computed with v_alignbit (T=32/64) or SWAR shifts (T=8/16), then masked;
//      bit width W is a runtime, wave-uniform value (no 124-way template
//      explosion, no runtime-indexed register arrays);
//   3. FFOR stores chunk ci straight to output bytes [16ci, 16ci+16): the 64
//      lanes of one store instruction write 1 KiB contiguously;
//      DELTA / RLE scatter the chunk into LDS at its transposed position, scan
//      the 1024/T lane chains (16 serial steps per lane + a wave shuffle across
//      chain segments), add the lane bases and copy out with 16 B/lane stores;
//      DICT / RLE gather through the dictionary / run values and store
//      16 B/lane.
// The path is HBM-bound integer work: no MFMA.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fls_decode.hpp"
#include "fls_format.hpp"

namespace fls {
namespace {

constexpr int kWaves = 4;                         // waves per 256-thread block
constexpr int kPackedU4 = (128 * 64 + 128) / 16;  // max packed bytes (T=64,W=64) + pad row
constexpr int kValBytes = 1024 * 8;               // max decoded vector (T=64)

__device__ __forceinline__ void wave_sync() {
    // one wave talks to itself through LDS: DS ops of a wave execute in order;
    // the fences stop the compiler from moving LDS accesses across.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint32_t tau(uint32_t p) {
    // FL_ORDER = {0,4,2,6,1,5,3,7} is the 3-bit bit reversal
    const uint32_t b = (p >> 4) & 7;
    const uint32_t rb = ((b & 1) << 2) | (b & 2) | ((b >> 2) & 1);
    return (rb << 7) | (((p >> 7) & 7) << 4) | (p & 15);
}

// ---- unpack one 16-byte chunk of T-bit values ------------------------------
template <int T>
__device__ __forceinline__ uint4 unpack_chunk(const uint4 *__restrict__ P, uint32_t W, uint32_t ci);

template <>
__device__ __forceinline__ uint4 unpack_chunk<32>(const uint4 *__restrict__ P, uint32_t W, uint32_t ci) {
    const uint32_t R = ci >> 3, qc = ci & 7;
    const uint32_t bit = R * W, k = bit >> 5, s = bit & 31;
    const uint4 lo = P[k * 8 + qc], hi = P[(k + 1) * 8 + qc];
    const uint32_t m = W >= 32 ? 0xFFFFFFFFu : ((1u << W) - 1u);
    uint4 r;
    r.x = __builtin_amdgcn_alignbit(hi.x, lo.x, s) & m;
    r.y = __builtin_amdgcn_alignbit(hi.y, lo.y, s) & m;
    r.z = __builtin_amdgcn_alignbit(hi.z, lo.z, s) & m;
    r.w = __builtin_amdgcn_alignbit(hi.w, lo.w, s) & m;
    return r;
}

template <>
__device__ __forceinline__ uint4 unpack_chunk<64>(const uint4 *__restrict__ P, uint32_t W, uint32_t ci) {
    const uint32_t R = ci >> 3, qc = ci & 7;
    const uint32_t bit = R * W, k = bit >> 6, s = bit & 63, s5 = s & 31;
    const uint4 lo = P[k * 8 + qc], hi = P[(k + 1) * 8 + qc];
    const bool big = s >= 32;
    const uint32_t mlo = W >= 32 ? 0xFFFFFFFFu : ((1u << W) - 1u);
    const uint32_t mhi = W >= 64 ? 0xFFFFFFFFu : (W > 32 ? ((1u << (W - 32)) - 1u) : 0u);
    uint4 r;
    // lane 0 = (lo.y:lo.x), next word row (hi.y:hi.x); lane 1 = (.w:.z)
    r.x = __builtin_amdgcn_alignbit(big ? hi.x : lo.y, big ? lo.y : lo.x, s5) & mlo;
    r.y = __builtin_amdgcn_alignbit(big ? hi.y : hi.x, big ? hi.x : lo.y, s5) & mhi;
    r.z = __builtin_amdgcn_alignbit(big ? hi.z : lo.w, big ? lo.w : lo.z, s5) & mlo;
    r.w = __builtin_amdgcn_alignbit(big ? hi.w : hi.z, big ? hi.z : lo.w, s5) & mhi;
    return r;
}

// SWAR funnel shift of packed 16-bit (or 8-bit) words inside a dword
template <int T>
__device__ __forceinline__ uint32_t swar_funnel(uint32_t lo, uint32_t hi, uint32_t s, uint32_t m1, uint32_t m2,
                                                uint32_t mw) {
    return (((lo >> s) & m1) | ((hi << (T - s)) & m2)) & mw;
}

template <>
__device__ __forceinline__ uint4 unpack_chunk<16>(const uint4 *__restrict__ P, uint32_t W, uint32_t ci) {
    const uint32_t R = ci >> 3, qc = ci & 7;
    const uint32_t bit = R * W, k = bit >> 4, s = bit & 15;
    const uint4 lo = P[k * 8 + qc], hi = P[(k + 1) * 8 + qc];
    const uint32_t rep = 0x00010001u;
    const uint32_t m1 = rep * (0xFFFFu >> s);
    const uint32_t m2 = rep * ((0xFFFFu << (16 - s)) & 0xFFFFu);
    const uint32_t mw = W >= 16 ? 0xFFFFFFFFu : rep * ((1u << W) - 1u);
    uint4 r;
    r.x = swar_funnel<16>(lo.x, hi.x, s, m1, m2, mw);
    r.y = swar_funnel<16>(lo.y, hi.y, s, m1, m2, mw);
    r.z = swar_funnel<16>(lo.z, hi.z, s, m1, m2, mw);
    r.w = swar_funnel<16>(lo.w, hi.w, s, m1, m2, mw);
    return r;
}

template <>
__device__ __forceinline__ uint4 unpack_chunk<8>(const uint4 *__restrict__ P, uint32_t W, uint32_t ci) {
    const uint32_t R = ci >> 3, qc = ci & 7;
    const uint32_t bit = R * W, k = bit >> 3, s = bit & 7;
    const uint4 lo = P[k * 8 + qc], hi = P[(k + 1) * 8 + qc];
    const uint32_t rep = 0x01010101u;
    const uint32_t m1 = rep * (0xFFu >> s);
    const uint32_t m2 = rep * ((0xFFu << (8 - s)) & 0xFFu);
    const uint32_t mw = W >= 8 ? 0xFFFFFFFFu : rep * ((1u << W) - 1u);
    uint4 r;
    r.x = swar_funnel<8>(lo.x, hi.x, s, m1, m2, mw);
    r.y = swar_funnel<8>(lo.y, hi.y, s, m1, m2, mw);
    r.z = swar_funnel<8>(lo.z, hi.z, s, m1, m2, mw);
    r.w = swar_funnel<8>(lo.w, hi.w, s, m1, m2, mw);
    return r;
}

// ---- frame-of-reference add on a 16-byte chunk (wrapping T-bit) ----------
template <int T>
__device__ __forceinline__ uint4 add_base(uint4 a, uint64_t base);

template <>
__device__ __forceinline__ uint4 add_base<64>(uint4 a, uint64_t base) {
    const uint64_t v0 = (((uint64_t)a.y << 32) | a.x) + base;
    const uint64_t v1 = (((uint64_t)a.w << 32) | a.z) + base;
    return make_uint4((uint32_t)v0, (uint32_t)(v0 >> 32), (uint32_t)v1, (uint32_t)(v1 >> 32));
}
template <>
__device__ __forceinline__ uint4 add_base<32>(uint4 a, uint64_t base) {
    const uint32_t b = (uint32_t)base;
    return make_uint4(a.x + b, a.y + b, a.z + b, a.w + b);
}
__device__ __forceinline__ uint32_t swar_add(uint32_t a, uint32_t b, uint32_t hi) {
    return ((a & ~hi) + (b & ~hi)) ^ ((a ^ b) & hi);
}
template <>
__device__ __forceinline__ uint4 add_base<16>(uint4 a, uint64_t base) {
    const uint32_t b = 0x00010001u * (uint32_t)(base & 0xFFFF), hi = 0x80008000u;
    return make_uint4(swar_add(a.x, b, hi), swar_add(a.y, b, hi), swar_add(a.z, b, hi), swar_add(a.w, b, hi));
}
template <>
__device__ __forceinline__ uint4 add_base<8>(uint4 a, uint64_t base) {
    const uint32_t b = 0x01010101u * (uint32_t)(base & 0xFF), hi = 0x80808080u;
    return make_uint4(swar_add(a.x, b, hi), swar_add(a.y, b, hi), swar_add(a.z, b, hi), swar_add(a.w, b, hi));
}

// ---- stores with tail guard ----------------------------------------------
// store 16 bytes at out + off, or only the bytes below `limit`
template <int EB>  // element bytes for the partial path
__device__ __forceinline__ void store16(uint8_t *__restrict__ out, uint32_t off, uint32_t limit, uint4 v) {
    if (off + 16 <= limit) {
        *reinterpret_cast<uint4 *>(out + off) = v;
        return;
    }
    if (off >= limit) return;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 16 / EB; ++e) {
        const uint32_t o = off + e * EB;
        if (o < limit) {
            if (EB == 8) {
                *reinterpret_cast<uint64_t *>(out + o) = ((uint64_t)w[2 * e + 1] << 32) | w[2 * e];
            } else if (EB == 4) {
                *reinterpret_cast<uint32_t *>(out + o) = w[e];
            } else if (EB == 2) {
                *reinterpret_cast<uint16_t *>(out + o) = (uint16_t)(w[e / 2] >> (16 * (e & 1)));
            } else {
                out[o] = (uint8_t)(w[e / 4] >> (8 * (e & 3)));
            }
        }
    }
}

// ---- LDS chain scan (DELTA / RLE index) -------------------------------------
// vals: 1024 T-bit deltas in tuple order (LDS).  bases: 1024/T chain bases
// (global).  In place: vals[i] = base[chain] + sum of the chain's deltas <= i.
template <int T>
__device__ __forceinline__ void chain_scan(uint8_t *__restrict__ V, const uint8_t *__restrict__ bases, uint32_t lane) {
    using UT = typename std::conditional<T == 64, uint64_t,
               typename std::conditional<T == 32, uint32_t,
               typename std::conditional<T == 16, uint16_t, uint8_t>::type>::type>::type;
    UT *v = reinterpret_cast<UT *>(V);
    const UT *b = reinterpret_cast<const UT *>(bases);
    if (T == 8) {
        // 128 chains of 8 steps: two chains per lane
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t c = lane + 64 * h;
            const uint32_t i0 = (c >> 4) * 128 + (c & 15);
            UT acc = b[c];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                acc = (UT)(acc + v[i0 + 16 * k]);
                v[i0 + 16 * k] = acc;
            }
        }
        return;
    }
    constexpr uint32_t nchains = 1024 / T;  // 16, 32, 64
    const uint32_t c = lane % nchains, seg = lane / nchains;
    const uint32_t i0 = (c >> 4) * 16 * T + (c & 15) + 256 * seg;
    UT run[16];
    UT acc = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        acc = (UT)(acc + v[i0 + 16 * j]);
        run[j] = acc;
    }
    // exclusive prefix of segment totals across the lanes of one chain
    uint64_t tot = (uint64_t)acc, x = tot;
    if (nchains <= 32) {  // T >= 32: >= 2 segments
        uint64_t y = __shfl_up((unsigned long long)x, nchains, 64);
        if (seg >= 1) x += y;
        if (nchains == 16) {
            y = __shfl_up((unsigned long long)x, 32, 64);
            if (seg >= 2) x += y;
        }
    }
    const UT pre = (UT)((x - tot) + (uint64_t)b[c]);
#pragma unroll
    for (int j = 0; j < 16; ++j) v[i0 + 16 * j] = (UT)(pre + run[j]);
}

// copy the decoded vector (tuple order, EB bytes each) from LDS to HBM
template <int EB>
__device__ __forceinline__ void copy_out(const uint8_t *__restrict__ V, uint8_t *__restrict__ out, uint32_t nvals,
                                         uint32_t lane) {
    const uint32_t limit = nvals * EB;
#pragma unroll
    for (uint32_t ci = lane; ci < 64 * EB; ci += 64) {
        const uint4 x = *reinterpret_cast<const uint4 *>(V + 16 * ci);
        store16<EB>(out, 16 * ci, limit, x);
    }
}

// gather values through a table and store 16 B/lane.  idx(i) yields the
// table index of tuple i, tab holds OB-byte entries.
template <int OB, typename IdxF>
__device__ __forceinline__ void gather_out(const uint8_t *__restrict__ tab, uint8_t *__restrict__ out, uint32_t nvals,
                                           uint32_t lane, IdxF idx) {
    const uint32_t limit = nvals * OB;
    constexpr int per = 16 / OB;
#pragma unroll
    for (uint32_t oc = lane; oc < 64 * OB; oc += 64) {
        uint32_t w[4] = {0, 0, 0, 0};
        if (OB == 16) {
            const uint4 e = reinterpret_cast<const uint4 *>(tab)[idx(oc)];
            w[0] = e.x; w[1] = e.y; w[2] = e.z; w[3] = e.w;
        } else {
#pragma unroll
            for (int e = 0; e < per; ++e) {
                const uint32_t t = idx(oc * per + e);
                if (OB == 8) {
                    const uint64_t x = reinterpret_cast<const uint64_t *>(tab)[t];
                    w[2 * e] = (uint32_t)x;
                    w[2 * e + 1] = (uint32_t)(x >> 32);
                } else if (OB == 4) {
                    w[e] = reinterpret_cast<const uint32_t *>(tab)[t];
                } else if (OB == 2) {
                    w[e / 2] |= (uint32_t)reinterpret_cast<const uint16_t *>(tab)[t] << (16 * (e & 1));
                } else {
                    w[e / 4] |= (uint32_t)tab[t] << (8 * (e & 3));
                }
            }
        }
        store16<OB == 16 ? 8 : OB>(out, 16 * oc, limit, make_uint4(w[0], w[1], w[2], w[3]));
    }
}

struct VecCtx {
    const uint4 *P;       // staged packed bits (LDS)
    uint8_t *V;           // decoded vector scratch (LDS)
    uint32_t W, nvals, lane;
    uint64_t base;
};

// FFOR: unpack + base, straight to HBM
template <int T>
__device__ __forceinline__ void do_ffor(const VecCtx &x, uint8_t *__restrict__ out) {
    const uint32_t limit = x.nvals * (T / 8);
#pragma unroll
    for (uint32_t ci = x.lane; ci < 8 * T; ci += 64) {
        const uint4 v = add_base<T>(unpack_chunk<T>(x.P, x.W, ci), x.base);
        store16<T / 8>(out, 16 * ci, limit, v);
    }
}

// unpack + base into LDS at transposed (DELTA) or natural position
template <int T, bool TRANSPOSED>
__device__ __forceinline__ void unpack_to_lds(const VecCtx &x) {
#pragma unroll
    for (uint32_t ci = x.lane; ci < 8 * T; ci += 64) {
        const uint4 v = add_base<T>(unpack_chunk<T>(x.P, x.W, ci), x.base);
        const uint32_t p0 = ci * (128 / T);                     // first position of the chunk
        const uint32_t i0 = TRANSPOSED ? tau(p0) : p0;          // its tuple index
        *reinterpret_cast<uint4 *>(x.V + i0 * (T / 8)) = v;
    }
}

template <int T>
__device__ __forceinline__ void do_delta(const VecCtx &x, const uint8_t *__restrict__ bases, uint8_t *__restrict__ out) {
    unpack_to_lds<T, true>(x);
    wave_sync();
    chain_scan<T>(x.V, bases, x.lane);
    wave_sync();
    copy_out<T / 8>(x.V, out, x.nvals, x.lane);
}

template <int OB>
__device__ __forceinline__ void dict_gather(const VecCtx &x, const uint8_t *__restrict__ dict, uint32_t dict_count,
                                            uint8_t *__restrict__ out, uint32_t *err) {
    const uint32_t *codes = reinterpret_cast<const uint32_t *>(x.V);
    bool bad = false;
    gather_out<OB>(dict, out, x.nvals, x.lane, [&](uint32_t i) {
        uint32_t c = codes[i];
        if (c >= dict_count) { bad = true; c = dict_count - 1; }
        return c;
    });
    if (bad) atomicOr(err, KERR_DICT_CODE);
}

template <int OB>
__device__ __forceinline__ void rle_gather(const VecCtx &x, const uint8_t *__restrict__ runs, uint32_t nruns,
                                           uint8_t *__restrict__ out, uint32_t *err) {
    const uint16_t *idx = reinterpret_cast<const uint16_t *>(x.V);
    bool bad = false;
    gather_out<OB>(runs, out, x.nvals, x.lane, [&](uint32_t i) {
        uint32_t r = idx[i];
        if (r >= nruns) { bad = true; r = nruns - 1; }
        return r;
    });
    if (bad) atomicOr(err, KERR_RUN_INDEX);
}

__global__ __launch_bounds__(256) void decode_kernel(const DevChunk *__restrict__ chunks, uint32_t ntasks,
                                                     uint32_t *__restrict__ err) {
    __shared__ uint4 lds_p[kWaves][kPackedU4];
    __shared__ __attribute__((aligned(16))) uint8_t lds_v[kWaves][kValBytes];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = uni(threadIdx.x >> 6);
    uint4 *P = lds_p[w];
    uint8_t *V = lds_v[w];
    const uint32_t stride = gridDim.x * kWaves;
    for (uint32_t task = blockIdx.x * kWaves + w; task < ntasks; task += stride) {
        const DevChunk &c = chunks[task >> 6];
        const uint32_t v = task & 63;
        if (v >= c.nvec) continue;
        const VecMeta *vm = reinterpret_cast<const VecMeta *>(c.chunk + c.meta_off) + v;
        const uint32_t W = vm->bw, nvals = vm->nvals;
        const uint64_t base = (uint64_t)vm->for_base;
        const uint8_t *aux = c.chunk + c.aux_off + vm->aux_off;
        const uint4 *src = reinterpret_cast<const uint4 *>(c.chunk + c.packed_off + vm->packed_off);
        uint8_t *out = c.out + (size_t)v * kVectorSize * c.ob;
        // 1. stage packed bits (W word-rows of 128 B) + a zero pad row
        wave_sync();
        const uint32_t n16 = 8 * W;
        for (uint32_t i = lane; i < n16; i += 64) P[i] = src[i];
        if (lane < 8) P[n16 + lane] = make_uint4(0, 0, 0, 0);
        wave_sync();
        VecCtx x{P, V, W, nvals, lane, base};
        switch (c.enc) {
        case ENC_FFOR:
            switch (c.T) {
            case 64: do_ffor<64>(x, out); break;
            case 32: do_ffor<32>(x, out); break;
            case 16: do_ffor<16>(x, out); break;
            default: do_ffor<8>(x, out); break;
            }
            break;
        case ENC_DELTA:
            switch (c.T) {
            case 64: do_delta<64>(x, aux, out); break;
            case 32: do_delta<32>(x, aux, out); break;
            case 16: do_delta<16>(x, aux, out); break;
            default: do_delta<8>(x, aux, out); break;
            }
            break;
        case ENC_DICT:
            unpack_to_lds<32, false>(x);
            wave_sync();
            switch (c.ob) {
            case 16: dict_gather<16>(x, c.dict, c.dict_count, out, err); break;
            case 8: dict_gather<8>(x, c.dict, c.dict_count, out, err); break;
            case 4: dict_gather<4>(x, c.dict, c.dict_count, out, err); break;
            case 2: dict_gather<2>(x, c.dict, c.dict_count, out, err); break;
            default: dict_gather<1>(x, c.dict, c.dict_count, out, err); break;
            }
            break;
        case ENC_RLE: {
            unpack_to_lds<16, true>(x);
            wave_sync();
            chain_scan<16>(V, aux, lane);
            wave_sync();
            const uint8_t *runs = aux + 128;
            const uint32_t nruns = vm->aux_count;
            switch (c.ob) {
            case 8: rle_gather<8>(x, runs, nruns, out, err); break;
            case 4: rle_gather<4>(x, runs, nruns, out, err); break;
            case 2: rle_gather<2>(x, runs, nruns, out, err); break;
            default: rle_gather<1>(x, runs, nruns, out, err); break;
            }
        } break;
        default:
            if (lane == 0) atomicOr(err, KERR_BAD_DESC);
            break;
        }
    }
}

}  // namespace

hipError_t launch_decode(const DevChunk *d_chunks, uint32_t nchunks, uint32_t *d_err, int grid, hipStream_t stream) {
    const uint64_t ntasks = (uint64_t)nchunks * 64;
    if (ntasks == 0) return hipSuccess;
    if (ntasks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint64_t need = (ntasks + kWaves - 1) / kWaves;
    const int g = (int)std::min<uint64_t>(need, (uint64_t)grid);
    hipLaunchKernelGGL(decode_kernel, dim3(g), dim3(64 * kWaves), 0, stream, d_chunks, (uint32_t)ntasks, d_err);
    return hipGetLastError();
}

int decode_grid_size() {
    int dev = 0, cus = 256, per_cu = 2;
    if (hipGetDevice(&dev) == hipSuccess) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_kernel, 64 * kWaves, 0) != hipSuccess)
            per_cu = 2;
    }
    if (per_cu < 1) per_cu = 1;
    return cus * per_cu;
}

}  // namespace fls
