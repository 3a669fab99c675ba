// fls_decode.hip -- MI355X (gfx950) FastLanes vector decode, pipelined (v2).
//
// Replaces the decode inside RowgroupReader::materialize()
// (reference src/fastlanes_facade.cpp:48) for the north-star codecs:
// interleaved bit-unpack at every width, FFOR, unified-transposed DELTA,
// DICT gather (integers and DuckDB string_t) and FastLanes-RLE.
//
// Work decomposition
//   * a 64-lane wave owns whole column chunks (one column of one row group,
//     <= 64 vectors), walking them grid-stride so every wave sees every column;
//   * per chunk the 64 VecMeta records are loaded once, one per lane, and
//     read with v_readlane when needed (no dependent metadata load per vector);
//   * the chunk's (encoding, T, output width) selects a templated inner loop, so
//     each loop body has a fixed instruction sequence and hipcc can count
//     vmcnt exactly;
//   * software pipeline, depth 1: while vector v is unpacked and stored, the
//     packed bits (and DELTA lane bases) of vector v+1 are already in flight
//     into registers.  gfx950's vmcnt counts stores and loads in issue order, so
//     the prefetch is issued BEFORE v's stores: the wait for v+1's data never
//     waits for v's stores;
//   * unpack: a lane handles 16-byte chunks ci (row R = ci/8, 16-byte column
//     qc = ci%8 of the 128-byte word-row) = funnel shift of word-rows R*W/T and
//     +1 (two ds_read_b128 from the staged LDS copy); W is runtime/uniform;
//   * FFOR stores chunk ci straight to output bytes [16ci, 16ci+16): one store
//     instruction writes 1 KiB contiguously;
//   * DELTA T=64 (BIGINT keys) is scanned entirely in registers: after the
//     unpack a lane already holds 8 consecutive steps of 2 chains (segment
//     FL_ORDER[lane/8]); in-lane prefix + a 3-step ds_bpermute scan across the
//     8 segments + lane bases -> 8 x 16 B stores (128 B lines);
//   * DELTA T<64 and RLE indices scatter into LDS at their transposed position
//     and scan the 1024/T chains there; DICT codes go through LDS and gather
//     from the dictionary (staged in LDS when small) with 16 B/lane stores;
//   * ALP (FLOAT/DOUBLE): the FFOR stream's integers are converted and scaled
//     in registers ((F)d * 10^f * 10^-e) and stored like FFOR; exception
//     values are then stored over their positions by the same wave.
// FSST strings have their own kernel (fls_fsst.hip).
// The path is HBM-bound integer work: no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "fls_alp.hpp"
#include "fls_decode.hpp"
#include "fls_format.hpp"
#include "fls_unpack.hpp"

#include "fls_decode_dev.hpp"

namespace fls {
using namespace dec;
namespace {

#ifndef FLS_WAVES_PER_SIMD
#define FLS_WAVES_PER_SIMD 4
#endif
// Work distribution, one of:
//   split != NULL: balanced split (balanced_split) -- wave gw first decodes
//     its static range [split[gw], split[gw + 1]), then pulls tail pieces p
//     = [split[nw + 1 + p], split[nw + 2 + p]) from the queue; a chunk may be
//     shared by several waves;
//   queue != NULL: whole chunks, the first static, then from the work queue;
//   neither: whole chunks, grid-stride.
// RATING: the same kernel under another name, for the upload's placement
// rating launches (rating_launch(), flsgpu.hip decode_rating), so a profile
// tells them from the decode's own launches
template <bool RATING>
__global__ __launch_bounds__(256, FLS_WAVES_PER_SIMD) void decode_kernel(const DevChunk *__restrict__ chunks, uint32_t nchunks,
                                                        uint32_t *__restrict__ err, uint32_t p_bytes,
                                                        uint32_t v_bytes, uint32_t *__restrict__ queue,
                                                        const uint32_t *__restrict__ split, uint32_t npieces,
                                                        uint32_t flags) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    // flags bit 0: the queue is shared by several grids; bits 1-2: wave issue
    // priority (s_setprio) for a grid that runs beside the FSST kernel
    const uint32_t shared_queue = flags & 1u, prio = (flags >> 1) & 3u;
    if (prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (prio == 3) __builtin_amdgcn_s_setprio(3);
    const uint32_t w = uni(threadIdx.x >> 6);
    const uint32_t lp = (uint32_t)(size_t)((lu8 *)lds_raw + w * (p_bytes + v_bytes));
    const uint32_t lv = lp + p_bytes;
    const uint32_t stride = shared_queue ? 0u : gridDim.x * kWaves, first = blockIdx.x * kWaves + w;
    if (split && shared_queue) {
        // several grids drain one guided plan: queue value q < nst is static
        // item q, the rest tail pieces (nst = the plan's waves, flags >> 8)
        const FLS_GLOBAL uint32_t *sp = gptr(split);
        const uint32_t nst = flags >> 8;
        for (;;) {
            uint32_t q = 0;
            if (__lane_id() == 0) q = atomicAdd(queue, 1u);
            q = uni(q);
            if (q >= nst + npieces) break;
            const uint32_t i = q < nst ? q : q + 1;  // pieces start one entry past the static boundaries
            decode_range(chunks, nchunks, uni(sp[i]), uni(sp[i + 1]), lp, lv, v_bytes, err);
        }
        return;
    }
    if (split) {
        const FLS_GLOBAL uint32_t *sp = gptr(split);
        decode_range(chunks, nchunks, uni(sp[first]), uni(sp[first + 1]), lp, lv, v_bytes, err);
        if (!queue) return;
        const FLS_GLOBAL uint32_t *pp = sp + stride + 1;
        for (;;) {
            uint32_t p = 0;
            if (__lane_id() == 0) p = atomicAdd(queue, 1u);
            p = uni(p);
            if (p >= npieces) break;
            decode_range(chunks, nchunks, uni(pp[p]), uni(pp[p + 1]), lp, lv, v_bytes, err);
        }
        return;
    }
    for (uint32_t ci = next_chunk(queue, UINT32_MAX, first, stride); ci < nchunks;
         ci = next_chunk(queue, ci, first, stride)) {
        const uint32_t nvec = gptr(chunks)[ci].nvec;
        if (nvec == 0) continue;
        decode_chunk(chunks + ci, lp, lv, v_bytes, err, nvec << 8);
    }
}

}  // namespace

#ifdef FLS_WAVE_TRACE
extern "C" int fls_trace_reset(void) {
    const uint32_t z = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace_n), &z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// copies up to cap records (40 B each) to dst; returns how many were recorded
extern "C" int64_t fls_trace_read(void *dst, uint32_t cap) {
    uint32_t n = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_trace_n), sizeof(n)) != hipSuccess)
        return -1;
    const uint32_t k = std::min(std::min(n, cap), kTraceCap);
    if (k && hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_trace), (size_t)k * sizeof(TraceRec)) != hipSuccess) return -1;
    return n;
}
#endif

namespace {
std::mutex g_occ_mu;
std::map<int, int> g_cus;
std::map<std::tuple<int, const void *, int, size_t>, int> g_occ;
}  // namespace

int device_cus() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    {
        std::lock_guard<std::mutex> lk(g_occ_mu);
        if (auto it = g_cus.find(dev); it != g_cus.end()) return it->second;
    }
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
    std::lock_guard<std::mutex> lk(g_occ_mu);
    g_cus[dev] = cus;
    return cus;
}

int occupancy(const void *kernel, int block, size_t shmem) {
    int dev = 0, per_cu = 1;
    if (hipGetDevice(&dev) != hipSuccess) return 1;
    const auto key = std::make_tuple(dev, kernel, block, shmem);
    {
        std::lock_guard<std::mutex> lk(g_occ_mu);
        if (auto it = g_occ.find(key); it != g_occ.end()) return it->second;
    }
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, shmem) != hipSuccess) return 1;
    std::lock_guard<std::mutex> lk(g_occ_mu);
    g_occ[key] = per_cu;
    return per_cu;
}

int decode_grid_size(uint32_t shmem_per_block) {
    const int cus = device_cus();
    int per_cu = occupancy(reinterpret_cast<const void *>(decode_kernel<false>), 64 * kWaves, shmem_per_block);
    // A/B knob: blocks per CU below what the occupancy query reports
    if (const char *e = getenv("FLS_BLOCKS_PER_CU")) per_cu = std::min(per_cu, std::max(1, atoi(e)));
    return cus * std::max(1, per_cu);
}

uint32_t decode_waves(const DecodeGeom &geom) {
    const uint32_t shmem = kWaves * (geom.p_bytes + geom.v_bytes);
    return (uint32_t)(geom.grid > 0 ? geom.grid : decode_grid_size(shmem)) * kWaves;
}

// Cost of one vector of chunk d in the balanced split: the bytes it moves
// (output + packed estimate at the chunk's widest W) plus a fixed per-vector
// term for the work that does not scale with bytes (metadata, LDS staging).
static inline uint64_t vec_cost(const DevChunk &d) { return 1024ull * d.ob + 128ull * d.max_w + 512; }

SplitPlan balanced_split(const DevChunk *h, uint32_t n, uint32_t nw, uint32_t static_pct, uint32_t pieces_per_wave,
                         std::vector<uint32_t> &pos) {
    uint64_t total = 0, nvecs = 0;
    for (uint32_t i = 0; i < n; ++i) {
        total += h[i].nvec * vec_cost(h[i]);
        nvecs += h[i].nvec;
    }
    SplitPlan plan;
    // no more waves than vectors (rounded to whole blocks)
    plan.waves = (uint32_t)std::min<uint64_t>(nw, (nvecs + kWaves - 1) / kWaves * kWaves);
    if (plan.waves == 0) plan.waves = kWaves;
    static_pct = std::min(static_pct, 100u);
    plan.pieces = static_pct < 100 ? plan.waves * std::max(1u, pieces_per_wave) : 0;
    const uint64_t stat = (uint64_t)((unsigned __int128)total * static_pct / 100);
    pos.clear();
    pos.reserve(plan.positions());
    // one monotone walk over the targets: static boundaries, then tail pieces
    uint64_t acc = 0;
    uint32_t i = 0;
    auto at = [&](uint64_t tgt) {
        while (i < n && acc + h[i].nvec * vec_cost(h[i]) <= tgt) {
            acc += h[i].nvec * vec_cost(h[i]);
            ++i;
        }
        pos.push_back(i < n ? (i << 7 | (uint32_t)((tgt - acc) / vec_cost(h[i]))) : n << 7);
    };
    // static boundaries 0..waves (the last one = where the tail starts)
    for (uint32_t w = 0; w <= plan.waves; ++w) at((uint64_t)((unsigned __int128)stat * w / plan.waves));
    // tail piece boundaries 0..pieces (pieces == 0: one unused entry)
    at(stat);
    for (uint32_t p = 1; p < plan.pieces; ++p) at(stat + (uint64_t)((unsigned __int128)(total - stat) * p / plan.pieces));
    if (plan.pieces) pos.push_back(n << 7);
    return plan;
}

SplitPlan guided_split(const DevChunk *h, uint32_t n, uint32_t nw, uint32_t factor, uint32_t min_vecs,
                       std::vector<uint32_t> &pos) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += h[i].nvec * vec_cost(h[i]);
    factor = std::max(1u, factor);
    min_vecs = std::max(1u, min_vecs);
    nw = std::max<uint32_t>(nw, kWaves);
    // item starts (positions chunk << 7 | vector), one walk in list order
    std::vector<uint32_t> b;
    b.reserve(n + n / 4);
    uint64_t acc = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t nv = h[i].nvec;
        if (nv == 0) continue;
        const uint64_t vc = vec_cost(h[i]), cc = nv * vc;
        const uint64_t target = std::max<uint64_t>((total - acc) / ((uint64_t)factor * nw), (uint64_t)min_vecs * vc);
        uint32_t parts = 1;
        if (cc > target)
            parts = (uint32_t)std::min<uint64_t>((cc + target - 1) / target, (nv + min_vecs - 1) / min_vecs);
        for (uint32_t p = 0; p < parts; ++p) b.push_back(i << 7 | (uint32_t)((uint64_t)nv * p / parts));
        acc += cc;
    }
    const uint32_t items = (uint32_t)b.size();
    b.push_back(n << 7);
    SplitPlan plan;
    plan.guided = true;
    plan.waves = std::min<uint32_t>(nw, std::max<uint32_t>(kWaves, (items + kWaves - 1) / kWaves * kWaves));
    plan.pieces = items > plan.waves ? items - plan.waves : 0;
    pos.clear();
    pos.reserve(plan.positions());
    // static: wave w takes item w (an empty range past the last item)
    for (uint32_t w = 0; w <= plan.waves; ++w) pos.push_back(b[std::min(w, items)]);
    // tail pieces: items waves .. items - 1 (pieces == 0: one unused entry)
    for (uint32_t p = 0; p <= plan.pieces; ++p) pos.push_back(b[std::min(plan.waves + p, items)]);
    return plan;
}

hipError_t launch_decode(const DevChunk *d_chunks, uint32_t nchunks, uint32_t *d_err, const DecodeGeom &geom,
                         hipStream_t stream, uint32_t *d_queue, const uint32_t *d_split, SplitPlan plan,
                         bool shared_queue, int prio) {
    if (nchunks == 0) return hipSuccess;
    const uint32_t shmem = kWaves * (geom.p_bytes + geom.v_bytes);
    int grid;
    if (d_split && shared_queue) {
        grid = std::min<int>(geom.grid > 0 ? geom.grid : decode_grid_size(shmem), (int)(plan.waves / kWaves));
    } else if (d_split) {
        grid = (int)(plan.waves / kWaves);
        if (!plan.pieces) d_queue = nullptr;
    } else {
        grid = std::min<int>(geom.grid > 0 ? geom.grid : decode_grid_size(shmem), (nchunks + kWaves - 1) / kWaves);
    }
    if (d_queue && !shared_queue) {
        const hipError_t e = hipMemsetAsync(d_queue, 0, sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(rating_launch() ? decode_kernel<true> : decode_kernel<false>, dim3(grid), dim3(64 * kWaves), shmem,
                       stream, d_chunks, nchunks, d_err,
                       geom.p_bytes, geom.v_bytes, d_queue, d_split, plan.pieces,
                       (uint32_t)(shared_queue && d_queue) | (uint32_t)(prio & 3) << 1 |
                           (d_split && shared_queue ? plan.waves << 8 : 0u));
    return hipGetLastError();
}

bool &rating_launch() {
    static thread_local bool f = false;
    return f;
}

// ---- HBM placement probe ---------------------------------------
namespace {
// the decode's write stream without the decode: wave w writes regions w, w+NW,
// ... front to back, 1 KiB per store instruction
__global__ __launch_bounds__(64) void probe_regions_kernel(const ProbeRegion *__restrict__ r, uint32_t n) {
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t p = (uint64_t)r[i].out, nb = r[i].bytes >> 10;
        // uni() returns the readfirstlane value as uint32_t: the builtin's int
        // would sign-extend a low word >= 2^31 across the high word
        FLS_GLOBAL v4u *o = (FLS_GLOBAL v4u *)((uint64_t)uni((uint32_t)(p >> 32)) << 32 | (uint64_t)uni((uint32_t)p));
        const v4u z = {0u, 0u, 0u, 0u};
        for (uint64_t b = 0; b < nb; ++b) o[b * 64 + lane] = z;
    }
}
// a linear fill: one 4 KiB block per 256-thread workgroup, dispatch order =
// address order (placement-insensitive in every measurement)
__global__ __launch_bounds__(256) void probe_fill_kernel(v4u *__restrict__ out) {
    ((FLS_GLOBAL v4u *)out)[(size_t)blockIdx.x * 256 + threadIdx.x] = v4u{0u, 0u, 0u, 0u};
}
}  // namespace

hipError_t probe_placement(const ProbeRegion *d_regions, uint32_t nregions, uint8_t *const *bufs,
                           const uint64_t *buf_bytes, uint32_t nbuf, int reps, hipStream_t stream, float *chunk_ms,
                           float *fill_ms) {
    int dev = 0, cus = 256;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    hipEvent_t a, b;
    if ((e = hipEventCreate(&a)) != hipSuccess) return e;
    if ((e = hipEventCreate(&b)) != hipSuccess) {
        hipEventDestroy(a);
        return e;
    }
    float best_c = 1e30f, best_f = 1e30f;
    for (int r = 0; r <= reps && e == hipSuccess; ++r) {  // r == 0 warms up
        float ms = 0;
        hipEventRecord(a, stream);
        hipLaunchKernelGGL(probe_regions_kernel, dim3(cus * 16), dim3(64), 0, stream, d_regions, nregions);
        hipEventRecord(b, stream);
        if ((e = hipEventSynchronize(b)) != hipSuccess) break;
        hipEventElapsedTime(&ms, a, b);
        if (r) best_c = std::min(best_c, ms);
        hipEventRecord(a, stream);
        for (uint32_t i = 0; i < nbuf; ++i)
            if (buf_bytes[i] >= 4096)
                hipLaunchKernelGGL(probe_fill_kernel, dim3((uint32_t)(buf_bytes[i] >> 12)), dim3(256), 0, stream,
                                   (v4u *)bufs[i]);
        hipEventRecord(b, stream);
        if ((e = hipEventSynchronize(b)) != hipSuccess) break;
        hipEventElapsedTime(&ms, a, b);
        if (r) best_f = std::min(best_f, ms);
    }
    if (e == hipSuccess) e = hipGetLastError();
    hipEventDestroy(a);
    hipEventDestroy(b);
    *chunk_ms = best_c;
    *fill_ms = best_f;
    return e;
}

}  // namespace fls
