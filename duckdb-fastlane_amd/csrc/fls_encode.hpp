// fls_encode.hpp -- GPU chunk encoder (fls_encode.hip): launch descriptors.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fls {

// One column chunk to encode (one block of encode_kernel).
struct EncChunk {
    uint64_t in;       // device address of the chunk's first value (T/8 bytes each)
    uint64_t out;      // device address of the chunk's output slot (enc_slot_bytes)
    uint64_t len_out;  // device address of a uint64: the chunk's byte length (written)
    uint64_t scratch;  // device address of enc_scratch_bytes() bytes (the DELTA chain bases)
    uint32_t nrows;    // rows of the chunk (1..65536)
    uint8_t T, enc;    // packing width 8/16/32/64; ENC_FFOR, ENC_DELTA, ENC_RLE, ENC_DICT or ENC_AUTO
    uint8_t pad[2];
    uint64_t est_dict; // ENC_AUTO: the DICT size estimate (UINT64_MAX: DICT not worth it;
                       // kEstDictGpu: dict_analyze_kernel computes it, as the CPU writer's est_dict)
    uint64_t dict_tab; // ENC_DICT / ENC_AUTO: device address of enc_dict_tab_bytes(nrows) bytes (the
                       // chunk's distinct-value hash table), 0 = the host encodes DICT chunks
    uint64_t reserved;
};
// *len_out = chunk bytes | encoding << kEncShift.  Chunks the GPU does not
// write (ENC_AUTO picking RLE is written by encode_rle_kernel; a DICT chunk
// without a table or with more distinct values than dict_encode_kernel sorts
// in LDS) come back with length 0, the encoding in the top byte, and the host
// encodes them from the staged values (fls_writer.cpp GpuEncoder::complete).
constexpr int kEncShift = 56;
constexpr uint64_t kEstDictGpu = UINT64_MAX - 1;
static_assert(sizeof(EncChunk) == 64, "EncChunk is 64 B");

// The DICT hash table of a chunk of nrows values: a 64-byte header (distinct
// count, ...), keys u64[cap], codes u32[cap], cap = the power of two >= 2 nrows.
__host__ __device__ inline uint32_t enc_dict_cap(uint32_t nrows) {
    uint32_t cap = 64;
    while (cap < 2u * nrows) cap <<= 1;
    return cap;
}
inline uint64_t enc_dict_tab_bytes(uint32_t nrows) { return 64ull + 12ull * enc_dict_cap(nrows); }
// Distinct values dict_encode_kernel sorts in LDS (more: the host encodes the chunk).
constexpr uint32_t kDictGpuMax = 16384;

// Scratch bytes per chunk: 64 x 128 B of DELTA chain bases (their place in
// the chunk follows the packed area, known only once every width is).
inline uint64_t enc_scratch_bytes() { return 64ull * 128ull; }

// Bytes an output slot needs for a chunk of nrows values (the chunk at W = T).
uint64_t enc_slot_bytes(uint32_t T, uint32_t nrows, uint8_t enc);
// Encode nchunks chunks (d_chunks in device memory), one block each.
// Launch over chunks [0, n_wide) of T = 64 and then [n_wide, n_wide + n_narrow)
// of T <= 32 (one kernel each: u64 or u32 registers and LDS).
// rle: some chunk is ENC_RLE or ENC_AUTO (encode_rle_kernel follows).
// dict: some chunk is ENC_DICT or ENC_AUTO with a dict_tab (dict_analyze_kernel
// runs first, dict_encode_kernel after).  d_chunks is written (est_dict).
// alp: some chunk is ENC_ALP (FLOAT T = 32 / DOUBLE T = 64: alp_encode_kernel).
hipError_t launch_encode(EncChunk *d_chunks, uint32_t n_wide, uint32_t n_narrow, hipStream_t stream, bool rle,
                         bool dict = false, bool alp = false);

// GPU FSST compression (writer side of ENC_FSST chunks; fls_writer.cpp
// enc_fsst).  The host builds the chunk's symbol table from its sample
// (fsst_build) and lays it out as an FsstCTable; the GPU applies it, one lane
// per string, with the host compressor's greedy longest match
// (FsstTable::match2), so the code bytes are the host's.  Codes of length >= 2
// sit in buckets of their first two bytes (fsst_cbucket), each bucket's codes
// in the order the host tries them (length descending, then code), so the
// first full match in a bucket is the host's match.
constexpr uint32_t kFsstCBuckets = 1024;
struct FsstCTable {
    uint64_t sym[256];                   // symbols, zero past their length
    uint8_t len[256];                    // their lengths (1..8)
    int16_t one[256];                    // the one-byte symbol of each byte value, -1: escape it
    uint16_t start[kFsstCBuckets + 1];   // bucket b's codes: codes[start[b] .. start[b + 1])
    uint8_t codes[256];
    uint8_t pad[14];
};
static_assert(sizeof(FsstCTable) % 16 == 0, "FsstCTable is copied in 16 B words");
__host__ __device__ inline uint32_t fsst_cbucket(uint32_t two_bytes) { return (two_bytes * 0x9E3779B1u) >> 22; }
// Compress strings [offs[i], offs[i + 1]) of d_bytes (offsets from 0, d_bytes
// 8-aligned and readable 16 bytes past offs[n]): string i's codes go to
// d_codes + 2 * offs[i] (room for every byte escaped), their count to d_clen[i].
hipError_t launch_fsst_compress(const uint8_t *d_bytes, const uint32_t *d_offs, uint32_t n, const FsstCTable *d_tab,
                                uint8_t *d_codes, uint32_t *d_clen, hipStream_t stream);

// GPU dictionary of a VARCHAR / BLOB chunk (fls_writer.cpp build_str_dict:
// the distinct strings in order of first appearance, each row's code): one
// block per chunk.  limit: more distinct strings than this (ENC_AUTO: n / 8)
// stops the build (info->overflow); more than kDictGpuMax leaves it to the
// host (info->big).  Tables in device memory: slots u32[3 cap] (cap =
// enc_dict_cap(n)), row_slot u32[n]; outputs codes u32[n], entries u32[n]
// (the first row of each distinct string, in code order).
struct StrDictInfo {
    uint32_t count;       // distinct strings
    uint32_t overflow;    // more than limit
    uint32_t big;         // more than kDictGpuMax (the host builds it)
    uint32_t pad;
    uint64_t entry_bytes; // sum of the distinct strings' lengths
};
hipError_t launch_str_dict(const uint8_t *d_bytes, const uint32_t *d_offs, uint32_t n, uint32_t limit,
                           uint32_t *d_slots, uint32_t *d_row_slot, uint32_t *d_codes, uint32_t *d_entries,
                           StrDictInfo *d_info, hipStream_t stream);

}  // namespace fls
