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
    const uint8_t *dict;       // DICT: int dictionary, or string_t table (VARCHAR)
    uint8_t *out;              // HBM address of output row 0 of this chunk
    uint32_t nvec;             // vectors (<= 64)
    uint32_t dict_count;
    uint32_t meta_off;         // VecMeta array, relative to chunk
    uint32_t packed_off;       // packed area, relative to chunk
    uint32_t aux_off;          // aux area, relative to chunk
    uint8_t enc, T, vbits, ob; // encoding, packing width, value bits, output bytes/value
    uint32_t pad[4];
};
static_assert(sizeof(DevChunk) == 64, "DevChunk is 64 B");

// error flags raised by the kernel (corrupt codes / run indices are clamped)
enum : uint32_t { KERR_DICT_CODE = 1, KERR_RUN_INDEX = 2, KERR_BAD_DESC = 4 };

// Launch the fused decode over ntasks = nchunks * 64 vector tasks.
hipError_t launch_decode(const DevChunk *d_chunks, uint32_t nchunks, uint32_t *d_err, int grid,
                         hipStream_t stream);
// Resident-grid size for the decode kernel on the current device.
int decode_grid_size();

}  // namespace fls
