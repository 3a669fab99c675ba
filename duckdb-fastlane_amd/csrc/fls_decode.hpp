// fls_decode.hpp -- device-side descriptors shared by the decode kernel and the
// host engine.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace fls {

// One column chunk (one column of one row group) resident in HBM.  Built by
// the host from the chunk header so the kernel never chases a dependent
// header load before it can start streaming.
struct DevChunk {              // 64 B
    const uint8_t *chunk;      // HBM address of the chunk (ChunkHeader)
    const uint8_t *dict;       // DICT: int dictionary, or string_t table (VARCHAR);
                               // FSST: HBM address of the chunk's string heap (written)
    uint8_t *out;              // HBM address of output row 0 of this chunk
    uint32_t nvec;             // vectors (<= 64)
    uint32_t dict_count;
    uint32_t meta_off;         // VecMeta array, relative to chunk
    uint32_t packed_off;       // packed area, relative to chunk
    uint32_t aux_off;          // aux area, relative to chunk
    uint8_t enc, T, vbits, ob; // encoding, packing width, value bits, output bytes/value
    uint64_t heap_host;        // FSST: address string_t pointers use for heap byte 0
                               // (the pinned host copy the heap lands in)
    uint32_t heap_bytes;       // FSST: heap bytes of the chunk (ChunkHeader.reserved1)
    union {
        uint32_t vec_base;     // FSST: vectors of the FSST chunks before this one in the launch
        uint32_t max_w;        // other encodings: widest vector of the chunk (bits) -- sizes the
                               // register prefetch, so narrow chunks hold fewer VGPRs in flight
    };
};
static_assert(sizeof(DevChunk) == 64, "DevChunk is 64 B");

// error flags raised by the kernel (corrupt codes / run indices are clamped)
enum : uint32_t { KERR_DICT_CODE = 1, KERR_RUN_INDEX = 2, KERR_BAD_DESC = 4, KERR_FSST = 8 };
// (16: KERR_FILTER_STR, fls_filter.hpp) an FSST kernel built with
// kFsstAbsLds found its dynamic LDS not at address 0: a build problem, not
// corrupt data (the launcher checks the kernel's static LDS first)
enum : uint32_t { KERR_LDS_BASE = 32 };

// Per-launch LDS geometry: per-wave packed staging (>= 128*maxW + 128 bytes)
// and decoded-vector scratch (path dependent), both multiples of 16; grid = 0
// picks the resident grid for that LDS size.
struct DecodeGeom {
    uint32_t p_bytes = 256, v_bytes = 0;
    int grid = 0;
};

// Balanced split of a launch's vectors (positions = chunk << 7 | vector):
// waves + 1 static boundaries (wave w decodes [pos[w], pos[w + 1])), then
// pieces + 1 boundaries of the tail pieces the waves pull from the work queue
// when their static range is done.  waves == 0: no split.
struct SplitPlan {
    uint32_t waves = 0, pieces = 0;
    bool guided = false;  // guided_split (whole chunks, then ever smaller pieces), else balanced_split
    size_t positions() const { return waves ? (size_t)waves + pieces + 2 : 0; }
};

// Launch the fused decode over every vector of nchunks chunks (no FSST).
// d_split (plan.positions() positions from balanced_split, may be NULL): each
// wave decodes its own balanced range of vectors, then tail pieces from
// d_queue; else d_queue (one zeroed word, may be NULL): waves take whole
// chunks from this work queue in list order; else a static grid-stride split
// of whole chunks.  shared_queue: the caller zeroed d_queue and several grids
// drain it (every chunk from the queue, none static).
hipError_t launch_decode(const DevChunk *d_chunks, uint32_t nchunks, uint32_t *d_err, const DecodeGeom &geom,
                         hipStream_t stream, uint32_t *d_queue = nullptr, const uint32_t *d_split = nullptr,
                         SplitPlan plan = SplitPlan(), bool shared_queue = false, int prio = 0);
// Waves of a resident decode launch with this LDS geometry.
uint32_t decode_waves(const DecodeGeom &geom);
// Split the vectors of h[0, n) over at most nw waves: static_pct % of the
// estimated bytes as equal static ranges, the rest as pieces_per_wave * waves
// equal tail pieces (dynamic: the waves that finish first take them).
SplitPlan balanced_split(const DevChunk *h, uint32_t n, uint32_t nw, uint32_t static_pct, uint32_t pieces_per_wave,
                         std::vector<uint32_t> &pos);
// Guided split of h[0, n) in list order (largest output first) over at most
// nw waves: work items are whole chunks while a chunk costs at most the
// remaining work / (factor * nw), then pieces of that size, never below
// min_vecs vectors, so the launch ends on pieces a few vectors long instead
// of whole chunks.  Item w < waves is wave w's first (static) item, the rest
// are tail pieces from the queue.
SplitPlan guided_split(const DevChunk *h, uint32_t n, uint32_t nw, uint32_t factor, uint32_t min_vecs,
                       std::vector<uint32_t> &pos);
// Code-parallel FSST kernel variants (bits): kFsstPlain = escape-free rounds
// skip the escape-state logic; kFsstTwoQ = each symbol OR-ed into both
// qwords it spans instead of through a 64-bit accumulator; kFsstZeroFlush =
// the ring is kept zero past the decoded bytes by the flush (no zeroing pass
// per round); kFsstW6 = registers budgeted for 6 waves per SIMD instead of 4;
// kFsstCirc = circular ring indexed by decoded position (no tail move per
// round; with zero-at-flush); kFsstLenFromSym = a symbol's length taken from
// its bits instead of a second table read, in chunks whose symbols all end in
// a non-zero byte (the others keep the table read); kFsstAbsLds = LDS
// addresses as integers from 0 (no symbol base added per access);
// kFsstEarlyGather = a round's table reads issued before the previous round's
// retire() (slower: spills at 6 waves, 5 waves without).
// Default kFsstW6 | kFsstZeroFlush | kFsstAbsLds (80 VGPRs, no spill in the
// standalone kernel): l_comment SF10 1.074 -> 1.012 (descriptor in SGPRs) ->
// 0.969 (6-wave budget) -> 0.922 ms (zero at flush) -> 1.2 % less (absolute
// LDS addresses, profiles/r2/abenv_fsst_abslds.txt); Plain, TwoQ, Circ and
// LenFromSym measured slower (profiles/r2/abenv_fsst_*.txt).
enum : int {
    kFsstPlain = 1, kFsstTwoQ = 2, kFsstZeroFlush = 4, kFsstW6 = 8, kFsstCirc = 16, kFsstLenFromSym = 32, kFsstAbsLds = 64, kFsstEarlyGather = 128,
    kFsstDefault = kFsstW6 | kFsstZeroFlush | kFsstAbsLds,
    // segmented kernel (FsstLaunch::seg): bit 0 = store a qword only once
    // complete (kFsstSegSparse), bit 1 = two-qword writer (kFsstTwoQ)
    kFsstSegSparse = kFsstPlain,
    // bit 5 = symbol length packed into the staged symbol's top byte
    // (tables of symbols <= 7 bytes only; kFsstSegPackedLen)
    kFsstSegPackedLen = kFsstLenFromSym,
    // bit 4 = all 16 table reads of a lane's segment issued together on the
    // fast path (kFsstSegWide)
    kFsstSegWide = kFsstCirc,
    // bit 7 = two consecutive segments (32 codes) per lane per round
    // (kFsstSegDouble)
    kFsstSegDouble = kFsstEarlyGather,
    // bit 8 = string_t records in whole batches of 64 strings (kFsstSegBatch)
    kFsstSegBatch = 256,
    // cost ablations of the segmented kernel (wrong output, timing only):
    // no string_t records / no heap flush / no ring writes
    kFsstAblateRecords = 512, kFsstAblateFlush = 1024, kFsstAblateWrite = 2048,
    // bit 12 = lean writer and records (kFsstSegLean): lengths staged in bits,
    // fewer VALU per code and per string_t record
    kFsstSegLean = 4096,
    // bit 13 = 8 KB of LDS per wave (kFsstSegD8: string lengths kept as u8,
    // offsets scanned per batch of records; no separate length table; ring
    // cap 4832), so 20 waves fit a CU instead of 16
    kFsstSegD8 = 8192,
    // bit 14 = lazy ring compaction (kFsstSegLazy): a round's retire streams
    // the finished blocks to the heap where they lie and moves the kept tail
    // to the ring start only when the ring is past half full
    kFsstSegLazy = 16384,
    // bit 15 = registers budgeted for 4 waves per SIMD (128 VGPRs) instead of
    // 5: the LDS admits only 16 waves per CU anyway (kFsstSegW4)
    kFsstSegW4 = 32768
};
// How one FSST launch runs (launch_fsst).
struct FsstLaunch {
    int bytes_per_lane = 8;       // compressed bytes a lane decodes per round (8 or 16)
    bool small = false;           // every string of these chunks is <= 255 bytes (DevChunk.vbits = 1)
    uint32_t *queue = nullptr;    // piece counter (overlapped launches); nullptr: contiguous ranges
    bool reset_queue = true;      // zero it first (false: drain a queue another launch started)
    int waves_per_cu = 0;         // grid: 0 = as many as fit, else at most this many per CU
    int grid_cus = 0;             // grid: the CUs it may run on (a CU-masked stream); 0 = all
    int variant = kFsstDefault;   // code-parallel kernel variant (kFsst* bits; FLS_FSST_VARIANT)
    bool seg = false;             // the chunks carry segment tables (DevChunk.vbits bit 1): segmented kernel
    int seg_cap = 4096;           // its ring: decoded bytes per part of a round (4096 or 5120; FLS_FSST_SEG_CAP)
};
// Launch the FSST string decode over nchunks FSST chunks holding nvecs vectors
// (DevChunk.vec_base numbers them) (fls_fsst.hip).
hipError_t launch_fsst(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                       hipStream_t stream, const FsstLaunch &how);
// The fused launch (fls_fsst.hip fused_kernel): the main decode of nmain
// chunks and the segmented FSST decode of nfsst chunks (nfvecs vectors, all
// of one kind: small = every string <= 255 bytes) in one kernel of 1-wave
// blocks that pull from two queues (d_queues[0] main chunks, [1] FSST
// pieces; zeroed by the launch).
struct FusedLaunch {
    uint32_t fsst_per16 = 6;   // of every 16 waves, how many start on the FSST queue
    uint32_t piece = 2;        // FSST vectors per queue item (halving: the largest piece)
    bool halving = false;      // pieces of `piece` vectors over half the queue's items, half that over a quarter, ...
    uint32_t fsst_static_pct = 0;   // % of the FSST vectors split statically over the FSST-first waves
    bool static_first = true;       // every wave's first item static (false: all from the queues)
    int waves_per_cu = 0;      // 0: as many as fit
    int x = 0;                 // the FSST part's experiment bits (FLS_FUSED_X; the experiment library only)
    // main-queue tail: the last tail_chunks main chunks (the smallest: the
    // host orders largest output first) are queued as tail_split pieces of
    // about nvec / tail_split vectors each, so the launch ends on short items
    uint32_t tail_chunks = 0, tail_split = 1;
};
hipError_t launch_fused(const DevChunk *d_main, uint32_t nmain, const DevChunk *d_fsst, uint32_t nfsst,
                        uint32_t nfvecs, bool small, uint32_t *d_err, const DecodeGeom &geom, hipStream_t stream,
                        uint32_t *d_queues, const FusedLaunch &how);
// Whether this build holds the FSST kernel for (variant, segmented, bytes per
// lane): the product build only each kernel's default (kFsstDefault, 8 bytes
// per lane for the code-parallel one); the experiment library (`make lab`,
// fls_fsst_lab.hip) every variant.  launch_fsst refuses the others.
bool fsst_variant_built(int variant, bool seg, int bytes_per_lane);
// Whether this build holds the fused kernel's FSST-part bits x
// (FusedLaunch::x, FLS_FUSED_X): 0 always, the others in the experiment
// library only.
bool fused_x_built(int x);
// Launch the string-parallel FSST decode over nchunks FSST chunks whose
// strings are all <= 255 bytes (DevChunk.vbits = 1), nvecs vectors numbered
// through DevChunk.vec_base (fls_fsst.hip).
hipError_t launch_fsst_sp(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                          hipStream_t stream);
// Resident-grid size of the v2 kernel for the given dynamic LDS per block.
int decode_grid_size(uint32_t shmem_per_block);
// The current device's CU count and a kernel's resident blocks per CU
// (hipOccupancyMaxActiveBlocksPerMultiprocessor), cached per device / (device,
// kernel, block size, dynamic LDS bytes): the scan's refill sizes several
// grids per batch, and these queries cost more host time than the launches.
// A failed query returns the fallback (256 CUs, 1 block) uncached.
int device_cus();
int occupancy(const void *kernel, int block, size_t shmem);

// Placement rating (flsgpu.hip decode_rating): decode launches made by this
// thread while it is set use the kernels' RATING instantiations -- the same
// code under another name (decode_kernel<true>, fused_kernel<.., .., true>),
// so profiles and step spans tell the upload's rating launches from the
// decode's own.
bool &rating_launch();

// HBM placement probe (round 6).  How fast the decode's write
// stream runs depends on where the driver placed the output buffers: the same
// pure write of the decode's output shape ran 5.66-6.89 TB/s from one
// allocation to the next at identical virtual addresses, while a linear fill
// (one 4 KiB block per 256-thread workgroup) ran 6.82-6.94 TB/s on every one
// (profiles/r6/membw7_*.txt, membw8_*.txt, membw9_*.txt).  The probe times
// both on a candidate set of output buffers; their ratio rates the placement.
struct ProbeRegion {  // 16 B: one output chunk, written front to back by one wave
    uint8_t *out;
    uint64_t bytes;   // a multiple of 1 KiB
};
// Time (ms, HIP events, best of `reps`) of the chunk-order write over the
// regions (persistent 1-wave blocks, wave w takes regions w, w + NW, ...) and
// of a linear fill of each of the `nbuf` buffers.
hipError_t probe_placement(const ProbeRegion *d_regions, uint32_t nregions, uint8_t *const *bufs,
                           const uint64_t *buf_bytes, uint32_t nbuf, int reps, hipStream_t stream, float *chunk_ms,
                           float *fill_ms);
// LDS bytes per wave the v2 kernel needs for one chunk (given its max width)
inline void chunk_lds_need(uint8_t enc, uint8_t T, uint8_t ob, uint32_t dict_count, uint32_t max_w,
                           uint32_t &p_bytes, uint32_t &v_bytes) {
    p_bytes = 128 * max_w + 128;
    v_bytes = 0;
    if (enc == 2 /*DELTA*/ && T < 64) v_bytes = 128 * T;
    if (enc == 4 /*RLE*/) v_bytes = 2048;
    if (enc == 3 /*DICT*/) {
        const uint32_t d = dict_count * ob;
        v_bytes = 4096 + (d <= 4096 ? ((d + 15) & ~15u) : 0);
    }
}

}  // namespace fls
