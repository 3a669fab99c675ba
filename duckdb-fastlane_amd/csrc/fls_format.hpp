// fls_format.hpp -- on-disk / in-HBM layout of a FastLanes row-group file.
//
// The reference reads `.fls` files through cwida/FastLanes
// (src/fastlanes_facade.cpp:33-56: connect -> read_fls -> get_rowgroup_reader
// -> materialize).  That library's byte format is not available here (empty
// submodule, .gitmodules:9-12), so this container is our own restatement of the
// FastLanes layout (paper: 1024-value vectors, interleaved bit-packing, FFOR,
// unified-transposed DELTA, DICT, FastLanes-RLE) designed so that the file body
// can be uploaded to HBM verbatim and decoded in place: every column chunk is
// 256-byte aligned, every packed vector 16-byte aligned, per-vector metadata is
// a flat 32-byte record array.  DESIGN.md "Container format" is the spec.
#pragma once
#include <algorithm>
#include <cstdint>

namespace fls {

constexpr uint32_t kVectorSize = 1024;      // values per FastLanes vector
constexpr uint32_t kRowGroupSize = 65536;   // rows per row group (64 vectors);
                                            // src/writer/write_fastlane_stream.cpp:21-24
constexpr uint32_t kVectorsPerRowGroup = kRowGroupSize / kVectorSize;
constexpr uint32_t kChunkAlign = 256;
constexpr uint32_t kChunkMagic = 0x43534C46u;  // "FLSC"
constexpr char kFileMagic[8] = {'F', 'L', 'S', 'A', 'M', 'D', '0', '1'};
constexpr char kTailMagic[4] = {'F', 'L', 'S', 'F'};

// Encodings (FastLanes expression kinds used on the north-star path)
enum Encoding : uint8_t {
    ENC_AUTO = 0,
    ENC_FFOR = 1,   // fused frame-of-reference + interleaved bit-packing
    ENC_DELTA = 2,  // unified-transposed delta, deltas FFOR-packed, per-lane bases
    ENC_DICT = 3,   // dictionary codes FFOR-packed (T=32), per-row-group dictionary
    ENC_RLE = 4,    // FastLanes-RLE: run values + DELTA(T=16) run-index vector
    ENC_ALP = 5,    // ALP (FLOAT/DOUBLE): decimal-exponent ints FFOR-packed + exceptions
    ENC_FSST = 7,   // FSST (VARCHAR): 255-symbol table, byte codes, FFOR-packed lengths
};

// Logical column types (cf. reference src/type_mapping.cpp:64-109)
enum TypeId : uint8_t {
    TY_INT8 = 1, TY_INT16 = 2, TY_INT32 = 3, TY_INT64 = 4,
    TY_UINT8 = 5, TY_UINT16 = 6, TY_UINT32 = 7, TY_UINT64 = 8,
    TY_BOOLEAN = 9,   // u8 0 / 1 (DuckDB bool), FFOR-packed like UINT8 (W <= 1)
    TY_DATE = 10,     // int32 days since 1970-01-01 (DuckDB date_t)
    TY_DECIMAL = 11,  // int64 scaled integer (DuckDB DECIMAL(w<=18, s))
    TY_FLOAT = 12,    // IEEE binary32 (FastLanes flt_col_t)
    TY_DOUBLE = 13,   // IEEE binary64 (FastLanes dbl_col_t)
    TY_VARCHAR = 20,  // DICT or FSST strings, decoded to DuckDB string_t (16 B)
    TY_BLOB = 21,     // byte strings: VARCHAR's layout and encodings (DuckDB BLOB)
};

inline int type_value_bits(uint8_t t) {
    switch (t) {
    case TY_INT8: case TY_UINT8: case TY_BOOLEAN: return 8;
    case TY_INT16: case TY_UINT16: return 16;
    case TY_INT32: case TY_UINT32: case TY_DATE: case TY_FLOAT: return 32;
    case TY_INT64: case TY_UINT64: case TY_DECIMAL: case TY_DOUBLE: return 64;
    default: return 0;
    }
}
inline bool type_is_float(uint8_t t) { return t == TY_FLOAT || t == TY_DOUBLE; }
inline bool type_is_string(uint8_t t) { return t == TY_VARCHAR || t == TY_BLOB; }
// bytes per decoded value in the output column (string_t = 16 B)
inline int type_out_bytes(uint8_t t) { return type_is_string(t) ? 16 : type_value_bits(t) / 8; }
inline bool type_valid(uint8_t t) { return type_out_bytes(t) > 0; }

struct ChunkHeader {          // 64 B, at the start of every column chunk
    uint32_t magic;           // kChunkMagic
    uint8_t enc;              // Encoding
    uint8_t T;                // packing width of the bit-packed stream (8/16/32/64)
    uint8_t vbits;            // value width in bits (0 for VARCHAR)
    uint8_t is_str;           // 1 for VARCHAR dictionary
    uint32_t nvec;            // vectors in this chunk (<= 64)
    uint32_t nvals;           // rows in this chunk
    uint64_t meta_off;        // VecMeta[nvec], relative to chunk start
    uint64_t packed_off;      // packed area, relative to chunk start
    uint64_t aux_off;         // aux area (bases / dictionary / run values)
    uint64_t aux_len;
    uint32_t dict_count;      // DICT: dictionary entries
    uint32_t reserved0;
    uint64_t reserved1;
};
struct VecMeta {              // 32 B per 1024-value vector
    uint64_t packed_off;      // relative to packed area; multiple of 16; 128*bw bytes
    int64_t for_base;         // frame of reference (sign-extended T-bit)
    uint64_t aux_off;         // relative to aux area (DELTA bases, RLE bases+runs)
    uint16_t nvals;           // 1..1024
    uint8_t bw;               // bit width 0..T
    uint8_t pad;
    uint32_t aux_count;       // RLE: number of runs
};
// ALP chunk (FLOAT T=vbits=32 / DOUBLE T=vbits=64): per vector the FFOR
// stream holds the encoded integers d, value = (float_t)d * kAlpF10[f] *
// kAlpIF10[e] (fls_alp.hpp); VecMeta.aux_count = exceptions | e << 16 | f << 24;
// VecMeta.aux_off -> u16 positions[exceptions] (padded to 16 B), then the
// exception values (T/8 bytes each) that replace the decoded value there.
inline uint32_t alp_exceptions(uint32_t aux_count) { return aux_count & 0xFFFF; }
inline uint32_t alp_e(uint32_t aux_count) { return (aux_count >> 16) & 0xFF; }
inline uint32_t alp_f(uint32_t aux_count) { return aux_count >> 24; }
inline uint64_t alp_aux_bytes(uint32_t exc, uint32_t vbits) { return ((2ull * exc + 15) & ~15ull) + exc * (vbits / 8ull); }

// FSST chunk (VARCHAR, T=32, vbits=0, is_str=1):
//   aux[0, 2304): symbol table, u64 symbol[256] (little-endian bytes) then
//                 u8 length[256] (1..8; code 255 is the escape, unused);
//   ChunkHeader.dict_count = symbols in use, reserved1 = heap bytes of the
//   chunk (sum of the vectors' 16-byte-padded decompressed sizes);
//   per vector: FFOR stream (T=32) of the decompressed string lengths;
//   VecMeta.aux_count = decompressed bytes of the vector;
//   VecMeta.aux_off -> FsstVecHeader, then the FFOR stream (T=32, clen_w bits,
//   base clen_base: 128 * clen_w bytes) of the strings' COMPRESSED lengths,
//   then the vector's compressed byte stream (every string compressed on its
//   own, codes concatenated; code 255 = next byte is a literal, never the
//   last code of a string).  The compressed lengths let a decoder start every
//   string independently (fls_fsst.hip's string-parallel path).
//   ChunkHeader.reserved0 = kFsstSegCodes when every vector carries a segment
//   table after its stream (below), else 0.
constexpr uint32_t kFsstTableBytes = 256 * 8 + 256;
constexpr uint32_t kFsstEscape = 255;
struct FsstVecHeader {        // 16 B
    uint32_t heap_off;        // start of this vector's strings in the chunk heap (16-aligned)
    uint32_t comp_len;        // compressed bytes (after the compressed-length stream)
    uint32_t clen_base;       // FOR base of the compressed string lengths
    uint32_t clen_w;          // their bit width (<= 32)
};
// compressed stream of a vector, relative to its FsstVecHeader
inline uint64_t fsst_stream_off(const FsstVecHeader &h) { return sizeof(FsstVecHeader) + 128ull * h.clen_w; }
static_assert(sizeof(FsstVecHeader) == 16, "FSST vector header is 16 B");

// FSST segment table (round 3; present when ChunkHeader.reserved0 ==
// kFsstSegCodes, readers that ignore it see the same stream).  The compressed
// stream of a vector is cut into segments of kFsstSegCodes code bytes (the
// last one shorter); per vector, 16-byte aligned after the stream:
//   FsstSegHeader, then u8 seg[nseg], nseg = ceil(comp_len / kFsstSegCodes):
//   the decoded bytes of segment k's codes and the escape state entering it,
//   as dlen (state 0, dlen <= 128) or 129 + dlen (state 1: the segment starts
//   with the literal byte of an escape, so dlen <= 1 + 15 * 8 = 121).
// With it a GPU lane decodes its own segment at its own output offset with no
// hand-off from the lanes before it (fls_fsst.hip, the segmented kernel).
constexpr uint32_t kFsstSegCodes = 16;
enum : uint32_t { FSST_SEG_HAS_ESCAPE = 1 };  // FsstSegHeader.flags: the stream holds an escape code
struct FsstSegHeader {        // 16 B
    uint32_t flags;
    uint32_t nseg;
    uint32_t reserved0, reserved1;
};
static_assert(sizeof(FsstSegHeader) == 16, "FSST segment header is 16 B");
inline uint64_t fsst_seg_off(const FsstVecHeader &h) { return fsst_stream_off(h) + ((h.comp_len + 15ull) & ~15ull); }
inline uint32_t fsst_nseg(uint32_t comp_len) { return (comp_len + kFsstSegCodes - 1) / kFsstSegCodes; }
inline uint64_t fsst_seg_bytes(uint32_t comp_len) { return sizeof(FsstSegHeader) + ((fsst_nseg(comp_len) + 15ull) & ~15ull); }
inline uint8_t fsst_seg_value(uint32_t dlen, uint32_t entry_state) { return (uint8_t)(entry_state ? 129 + dlen : dlen); }

// Validity (NULLs, round 3).  A chunk with at least one NULL row sets
// kChunkValidity in ChunkHeader.reserved0 and ends with nvec x 128 B of
// bitmaps, 16-aligned at chunk_len - 128 * nvec: bit i of u64 word j of vector
// v is 1 when row 1024 v + 64 j + i is valid (DuckDB's ValidityMask layout,
// so a row group's bitmaps are its validity mask); bits past nvals are 0.
// VecMeta.pad bit 0 (kVecHasNull) marks the vectors holding a NULL.  The
// encoded values at NULL rows are placeholders the writer chose so they cost
// nothing to encode (the chunk's previous valid value, 0 before the first;
// the empty string): every reader masks them with the bitmap.  A chunk without
// NULLs is byte-identical to a round-2 chunk.
constexpr uint32_t kChunkValidity = 1u << 31;
constexpr uint8_t kVecHasNull = 1;
constexpr uint32_t kValidityVecBytes = kVectorSize / 8;  // 128
inline bool chunk_has_validity(const ChunkHeader &h) { return (h.reserved0 & kChunkValidity) != 0; }
// ChunkHeader.reserved0 without the validity flag (FSST: kFsstSegCodes or 0)
inline uint32_t chunk_seg_codes(const ChunkHeader &h) { return h.reserved0 & ~kChunkValidity; }
inline uint64_t validity_off(uint64_t chunk_len, uint32_t nvec) { return chunk_len - (uint64_t)kValidityVecBytes * nvec; }

static_assert(sizeof(ChunkHeader) == 64, "chunk header is 64 B");
static_assert(sizeof(VecMeta) == 32, "vector meta is 32 B");
static_assert(alignof(VecMeta) == 8 && alignof(ChunkHeader) == 8, "natural alignment, no padding");

// Footer (little-endian):
//   u32 version=1, u32 ncols, u64 nrows, u32 nrowgroups, u32 rowgroup_size,
//   u64 row_offset,
//   per column: u8 type, u8 width, u8 scale, u8 pad, u16 name_len, name[name_len]
//   per row group: u32 nrows, per column {u64 chunk_off, u64 chunk_len}
//   optional zone-map section (readers that stop after the row-group table,
//   e.g. oracle/flsref.c, ignore it):
//   u32 kZoneMagic, u32 entry bytes (24), then per row group per column a
//   ZoneMap.  Zone maps feed row-group pruning of pushed-down filters
//   (read_fastlanes filter_pushdown; reference src/scanner/scan_fastlanes.cpp:154
//   leaves it off).
// File tail (16 B): u64 footer_off, u32 footer_len, "FLSF".
constexpr uint32_t kFooterVersion = 1;
constexpr uint32_t kFooterFixed = 32;
constexpr uint32_t kZoneMagic = 0x50414D5Au;  // "ZMAP"

// min / max of one column chunk in the column's comparison domain:
// signed integers (INT*, DATE, DECIMAL) as int64, unsigned as uint64,
// FLOAT/DOUBLE as the IEEE bits of a double over the non-NaN values (NaN
// sorts above every number, as in DuckDB).  VARCHAR has none: DICT chunks are
// pruned on their dictionary instead.  Over the valid rows only: ZM_HAS_NULL
// when the chunk has a NULL, ZM_ALL_NULL (and no ZM_VALID) when every row is
// NULL; string columns carry these two flags alone.
enum : uint32_t { ZM_VALID = 1, ZM_HAS_NAN = 2, ZM_ALL_NAN = 4, ZM_HAS_NULL = 8, ZM_ALL_NULL = 16 };
struct ZoneMap {              // 24 B
    uint64_t min, max;
    uint32_t flags;
    uint32_t pad;
};
static_assert(sizeof(ZoneMap) == 24, "zone map entry is 24 B");

inline bool type_is_signed(uint8_t t) {
    return t == TY_INT8 || t == TY_INT16 || t == TY_INT32 || t == TY_INT64 || t == TY_DATE || t == TY_DECIMAL;
}

// Zone map of n values given as raw T-bit patterns (T = type_value_bits).
inline ZoneMap zone_of(uint8_t type, const uint64_t *raw, uint32_t n) {
    ZoneMap z{0, 0, 0, 0};
    const int T = type_value_bits(type);
    if (T == 0 || n == 0) return z;
    z.flags = ZM_VALID;
    if (type_is_float(type)) {
        bool any = false;
        double mn = 0, mx = 0;
        for (uint32_t i = 0; i < n; ++i) {
            double d;
            if (T == 32) {
                float f;
                const uint32_t b = (uint32_t)raw[i];
                __builtin_memcpy(&f, &b, 4);
                d = f;
            } else {
                __builtin_memcpy(&d, &raw[i], 8);
            }
            if (d != d) { z.flags |= ZM_HAS_NAN; continue; }
            if (d == 0) d = 0.0;  // -0 == 0: one canonical zero
            if (!any || d < mn) mn = d;
            if (!any || d > mx) mx = d;
            any = true;
        }
        if (!any) z.flags |= ZM_ALL_NAN;
        __builtin_memcpy(&z.min, &mn, 8);
        __builtin_memcpy(&z.max, &mx, 8);
        return z;
    }
    const uint64_t m = T >= 64 ? ~0ull : ((1ull << T) - 1);
    if (type_is_signed(type)) {
        int64_t mn = INT64_MAX, mx = INT64_MIN;
        for (uint32_t i = 0; i < n; ++i) {
            uint64_t v = raw[i] & m;
            if (T < 64) { const uint64_t s = 1ull << (T - 1); v = (v ^ s) - s; }
            mn = std::min(mn, (int64_t)v);
            mx = std::max(mx, (int64_t)v);
        }
        z.min = (uint64_t)mn;
        z.max = (uint64_t)mx;
    } else {
        uint64_t mn = UINT64_MAX, mx = 0;
        for (uint32_t i = 0; i < n; ++i) {
            mn = std::min(mn, raw[i] & m);
            mx = std::max(mx, raw[i] & m);
        }
        z.min = mn;
        z.max = mx;
    }
    return z;
}

// Zone map of n integer values stored in the column's own width (1/2/4/8 B):
// the same result as zone_of over their raw patterns, one vectorisable pass
// without widening (the writer's GPU-encoded columns never widen their data).
template <class I>
inline ZoneMap zone_of_ints(const I *v, uint32_t n) {
    ZoneMap z{0, 0, ZM_VALID, 0};
    I mn = v[0], mx = v[0];
    for (uint32_t i = 1; i < n; ++i) {
        mn = v[i] < mn ? v[i] : mn;
        mx = v[i] > mx ? v[i] : mx;
    }
    if (I(-1) < I(0)) {  // signed: sign-extended int64 patterns
        z.min = (uint64_t)(int64_t)mn;
        z.max = (uint64_t)(int64_t)mx;
    } else {
        z.min = (uint64_t)mn;
        z.max = (uint64_t)mx;
    }
    return z;
}
inline ZoneMap zone_of_typed(uint8_t type, const void *data, uint32_t n) {
    if (n == 0 || type_value_bits(type) == 0) return ZoneMap{0, 0, 0, 0};
    if (type_is_float(type)) {  // zone_of's rule (NaN flags, one canonical zero) over the typed values
        ZoneMap z{0, 0, ZM_VALID, 0};
        bool any = false;
        double mn = 0, mx = 0;
        for (uint32_t i = 0; i < n; ++i) {
            double d = type_value_bits(type) == 32 ? (double)((const float *)data)[i] : ((const double *)data)[i];
            if (d != d) { z.flags |= ZM_HAS_NAN; continue; }
            if (d == 0) d = 0.0;
            if (!any || d < mn) mn = d;
            if (!any || d > mx) mx = d;
            any = true;
        }
        if (!any) z.flags |= ZM_ALL_NAN;
        __builtin_memcpy(&z.min, &mn, 8);
        __builtin_memcpy(&z.max, &mx, 8);
        return z;
    }
    const bool sg = type_is_signed(type);
    switch (type_value_bits(type)) {
    case 8: return sg ? zone_of_ints((const int8_t *)data, n) : zone_of_ints((const uint8_t *)data, n);
    case 16: return sg ? zone_of_ints((const int16_t *)data, n) : zone_of_ints((const uint16_t *)data, n);
    case 32: return sg ? zone_of_ints((const int32_t *)data, n) : zone_of_ints((const uint32_t *)data, n);
    default: return sg ? zone_of_ints((const int64_t *)data, n) : zone_of_ints((const uint64_t *)data, n);
    }
}

}  // namespace fls
