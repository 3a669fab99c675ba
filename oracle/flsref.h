/*
 * flsref.h -- CPU restatement of the FastLanes decode path (ORACLE).
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * or the timed CPU baseline.  The product (duckdb-fastlane_amd/) never links it.
 *
 * PARITY UNPINNED.  The reference (lmangani/duckdb-fastlane @ 2025-08-24)
 * delegates every decode step to the cwida/FastLanes library
 * (.gitmodules:9-12, branch `dev`, commit unknown, vcpkg port 0.1.0 at
 * vcpkg_ports/fastlanes/vcpkg.json:3).  That submodule is empty in
 * /root/reference and no .fls fixture exists (test/sql/fastlane.test:15-66
 * needs third_party/fastlanes/data/fls/data.fls, absent), so neither the
 * library nor its byte format can be executed or compared here.  This file
 * restates the published FastLanes algorithm (Afroozeh & Boncz, "The
 * FastLanes Compression Layout", VLDB 2023) over this repo's container
 * format (DESIGN.md "Container format"), and is pinned by hand-computed
 * known-answer tests, an independent numpy restatement (oracle/flsref_np.py)
 * and the seeded generators' ground truth (integer codecs are lossless).
 *
 * Upstream facts this restatement assumes (what an upstream .fls fixture or
 * the cwida/FastLanes sources would have to confirm; each is checked against
 * the restatement mechanically by the named test):
 *   F1 interleaved packing: vector = 1024 values, 1024/T lanes; value at
 *      (row r, lane l) starts in word floor(rW/T)*(1024/T)+l at bit (rW) mod T
 *      and straddles into the next word of the same lane; W = 0 stores no
 *      bytes, W = T is the identity layout.  Matches SURVEY.md section 5
 *      bit for bit (tests/test_oracle.py::test_survey_layout_statements,
 *      test_kat_pack_t32_w7, test_kat_pack_t64_w64_identity).
 *   F2 FFOR: value = base + unpacked, wrapping at T bits, base = the
 *      vector's minimum (sign-extended T-bit); W = bit width of max - min.
 *   F3 DELTA, unified transposed order FL_ORDER = {0,4,2,6,1,5,3,7}:
 *      position p = 128a + 16b + l holds tuple 128*FL_ORDER[b] + 16a + l
 *      (flsref_tau).  Each lane holds one delta chain, tuples blk*16T + l + 16k,
 *      k = 0..T-1, with one base (its first tuple) per lane, 1024/T bases =
 *      128 bytes per vector.  For T = 64 the lane's tuple SET equals SURVEY's
 *      index(r,l) = FL_ORDER[r/8]*16 + (r%8)*128 + l; the ROW ORDER differs by
 *      the fixed permutation r -> 8*FL_ORDER[r/8] + FL_ORDER[r%8]
 *      (test_survey_layout_statements).  Which row order upstream stores is
 *      the open fact; an adapter for the other one is that permutation.
 *   F4 DICT: codes FFOR-packed at T = 32, value = dict[code]; VARCHAR
 *      dictionaries decode to DuckDB string_t (16 B, <= 12 bytes inline).
 *   F5 RLE (FastLanes-RLE): per vector a u16 run index per value, DELTA(T=16)
 *      coded as in F3, plus the run values; value = runs[index].
 *   F6 ALP: value = (float)digits * 10^f * 10^-e with per-vector (e, f) and
 *      exceptions patched by position; FSST: 255-symbol table of <= 8-byte
 *      symbols, code 255 escapes one literal byte.
 *   The container around the vectors (FLSAMD01 header, chunk headers, VecMeta,
 *   footer) is this repo's own; upstream's .fls framing is unknown here.
 *
 * Call sites of the replaced decode in the reference:
 *   src/fastlanes_facade.cpp:33  fastlanes::connect()
 *   src/fastlanes_facade.cpp:34  Connection::read_fls(path)
 *   src/fastlanes_facade.cpp:41  TableReader::get_rowgroup_reader(0)
 *   src/fastlanes_facade.cpp:48  RowgroupReader::materialize()   <- decode
 *   src/fastlanes_facade.cpp:112-183  per-type column access
 */
#ifndef FLSREF_H
#define FLSREF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* --- layout primitives (paper section 3/4) --------------------------------- */

/* Original tuple index stored at position p (0..1023) of the unified
 * transposed layout.  FL_ORDER = {0,4,2,6,1,5,3,7}. */
uint32_t flsref_tau(uint32_t p);

/* Interleaved bit-unpack of one 1024-value vector: T in {8,16,32,64},
 * 0 <= W <= T.  packed holds 128*W bytes (W words of T bits per lane,
 * word k of lane L at word index k*(1024/T)+L).  out[p] = unsigned value at
 * position p = row*(1024/T)+lane. */
void flsref_unpack(int T, int W, const void *packed, uint64_t *out);

/* Inverse of flsref_unpack (used only by tests to build KATs). */
void flsref_pack(int T, int W, const uint64_t *in, void *packed);

/* --- container decode ---------------------------------------------------- */

typedef struct {
    const uint8_t *img;
    size_t len;
    uint32_t ncols;
    uint64_t nrows;
    uint32_t nrowgroups;
    uint32_t rowgroup_size;
    uint64_t row_offset;
    const uint8_t *footer;
    uint32_t footer_len;
} flsref_file;

/* Parse the footer of an in-memory image.  Returns 0 on success. */
int flsref_open(const void *img, size_t len, flsref_file *f);

/* Column schema: logical type id, decimal width/scale, name (not NUL
 * terminated; *name_len bytes). Returns 0 on success. */
int flsref_column(const flsref_file *f, uint32_t col, int *type, int *width,
                  int *scale, const char **name, int *name_len);

/* Rows in row group rg (or -1 on error). */
int64_t flsref_rowgroup_rows(const flsref_file *f, uint32_t rg);

/* Decode column `col` of row group `rg`.
 * Integer columns: out receives nrows values of the column's value width
 *   (1/2/4/8 bytes, little-endian two's complement); FLOAT/DOUBLE (ALP) their
 *   IEEE bits.  FSST columns are decoded with flsref_decode_strings.
 * VARCHAR columns: out receives nrows pairs {uint64 byte offset into the
 *   image, uint64 length} naming each value's bytes inside the image.
 * Returns number of rows decoded, or -1 on a malformed chunk. */
int64_t flsref_decode(const flsref_file *f, uint32_t col, uint32_t rg, void *out);

/* Strings of VARCHAR column col, row group rg (DICT or FSST): offs receives
 * nrows+1 offsets into heap (cap bytes), heap the concatenated bytes.
 * Returns the byte count, or -1 on error / insufficient cap. */
int64_t flsref_decode_strings(const flsref_file *f, uint32_t col, uint32_t rg, uint32_t *offs,
                              uint8_t *heap, uint64_t cap);

/* Decode every row group of `col` into out (rows concatenated).  Threads:
 * nthreads > 1 decodes row groups in parallel (CPU baseline).  Returns rows. */
int64_t flsref_decode_column(const flsref_file *f, uint32_t col, void *out, int nthreads);

/* Validity of column col, row group rg (NULLs; csrc/fls_format.hpp): when the
 * chunk carries bitmaps (ChunkHeader.reserved0 bit 31), words receives
 * 16 * nvec u64 words (bit i of word j: row 64 j + i valid) and 1 is
 * returned; 0 when every row is valid (words untouched); -1 when the bitmaps
 * are out of bounds, set bits past the chunk's rows, or disagree with the
 * vectors' has-NULL marks (VecMeta.pad bit 0). */
int flsref_validity(const flsref_file *f, uint32_t col, uint32_t rg, uint64_t *words);

/* Bytes per output value of column col (1/2/4/8, or 16 for VARCHAR pairs). */
int flsref_out_width(const flsref_file *f, uint32_t col);

#ifdef __cplusplus
}
#endif
#endif
