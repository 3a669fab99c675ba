// fls_decode.hpp -- device-side descriptors shared by the decode kernel and the
// host engine.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

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

// Per-launch LDS geometry: per-wave packed staging (>= 128*maxW + 128 bytes)
// and decoded-vector scratch (path dependent), both multiples of 16; grid = 0
// picks the resident grid for that LDS size.
struct DecodeGeom {
    uint32_t p_bytes = 256, v_bytes = 0;
    int grid = 0;
};

// Launch the fused decode over every vector of nchunks chunks (no FSST).
// d_queue (one zeroed word, may be NULL): waves take chunks from this work
// queue in list order instead of a static grid-stride split.
hipError_t launch_decode(const DevChunk *d_chunks, uint32_t nchunks, uint32_t *d_err, const DecodeGeom &geom,
                         hipStream_t stream, uint32_t *d_queue = nullptr);
// Launch the FSST string decode over nchunks FSST chunks holding nvecs vectors
// (DevChunk.vec_base numbers them) (fls_fsst.hip).
// bytes_per_lane: compressed bytes a lane decodes per round (8 or 16).
hipError_t launch_fsst(const DevChunk *d_chunks, uint32_t nchunks, uint32_t nvecs, uint32_t *d_err,
                       hipStream_t stream, int bytes_per_lane = 8);
// Resident-grid size of the v2 kernel for the given dynamic LDS per block.
int decode_grid_size(uint32_t shmem_per_block);
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
