/*
 * flswriter.h -- C-ABI of the CPU FastLanes writer and the seeded workload
 * generators (libflsgpu.so).
 *
 * Reference interfaces this replaces / serves:
 *   - ext_fastlane::FastLanesFacade::createFile / writeChunk / finalizeFile
 *     (src/include/fastlanes_facade.hpp:39-43; declared, never implemented in
 *     the reference) and the COPY ... TO 'x.fls' (FORMAT FLS) writer stub
 *     (src/writer/write_fastlane_stream.cpp:65-314, row_group_size default
 *     65,536 at :21-24).  Exposed as the copy function in SURVEY.md 8(f) row 1.
 *   - the data file third_party/fastlanes/data/fls/data.fls that
 *     test/sql/fastlane.test:15-66 scans (absent; regenerated synthetically).
 *
 * All functions return 0 on success and a negative fls_status on error;
 * fls_last_error() (flsgpu.h) describes the last error of the calling thread.
 */
#ifndef FLSWRITER_H
#define FLSWRITER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fls_writer fls_writer;

/* Column types (cf. reference src/type_mapping.cpp:64-109). */
enum fls_type {
    FLS_INT8 = 1, FLS_INT16 = 2, FLS_INT32 = 3, FLS_INT64 = 4,
    FLS_UINT8 = 5, FLS_UINT16 = 6, FLS_UINT32 = 7, FLS_UINT64 = 8,
    FLS_BOOLEAN = 9,  /* u8 0/1, DuckDB bool (reference type_mapping.cpp:13-14) */
    FLS_DATE = 10, FLS_DECIMAL = 11, FLS_FLOAT = 12, FLS_DOUBLE = 13, FLS_VARCHAR = 20,
    FLS_BLOB = 21     /* byte strings, VARCHAR's layout (reference type_mapping.cpp:40-42, BYTE_ARRAY) */
};
/* Encodings; FLS_ENC_AUTO picks per chunk: the smallest of FFOR/DELTA/DICT/RLE
 * for integers, ALP for FLOAT/DOUBLE, DICT or FSST for VARCHAR. */
enum fls_encoding {
    FLS_ENC_AUTO = 0, FLS_ENC_FFOR = 1, FLS_ENC_DELTA = 2, FLS_ENC_DICT = 3, FLS_ENC_RLE = 4,
    FLS_ENC_ALP = 5,  /* FLOAT/DOUBLE */
    FLS_ENC_FSST = 7  /* VARCHAR */
};

/* New writer; row_offset = global index of the first row (shards). */
fls_writer *fls_writer_new(uint64_t row_offset);
void fls_writer_free(fls_writer *w);
int fls_writer_add_column(fls_writer *w, const char *name, uint8_t type, uint8_t width,
                          uint8_t scale, uint8_t encoding);
/* Rows per row group (multiple of 1024 in [1024, 65536]; default 65536, the
 * reference's ROW_GROUP_SIZE default, src/writer/write_fastlane_stream.cpp:21-24).
 * Must be called before the first row group. */
int fls_writer_set_rowgroup_size(fls_writer *w, uint32_t rows);
/* Threads encoding the columns of a row group in parallel (0 = default:
 * min(16, hardware threads)).  Output bytes do not depend on it. */
int fls_writer_set_threads(fls_writer *w, int nthreads);
/* Encode the FFOR and DELTA integer columns of every later row group on GPU
 * `device` (fls_encode.hip: one block per column chunk); -1 = CPU (default).
 * The chunks are byte-identical to the CPU writer's.  Other columns (AUTO,
 * DICT, RLE, ALP, VARCHAR) stay on the CPU threads. */
int fls_writer_set_device(fls_writer *w, int device);

/* GPU chunk encoder over a device-resident integer column (the write side of
 * the scan path).  nrows values of `type` (1/2/4/8 B,
 * 16-byte aligned) at d_values become ceil(nrows / rowgroup_rows) FFOR or
 * DELTA chunks, chunk i at d_out + i * fls_encode_slot_bytes(type, encoding,
 * rowgroup_rows), byte-identical to the CPU writer's; chunk_lens (host, one per
 * chunk) receive their lengths, kernel_ms (may be NULL) the kernel time. */
uint64_t fls_encode_slot_bytes(uint8_t type, uint8_t encoding, uint32_t rowgroup_rows);
int fls_encode_device(int device, uint8_t type, uint8_t encoding, const void *d_values, uint64_t nrows,
                      uint32_t rowgroup_rows, void *d_out, uint64_t *chunk_lens, float *kernel_ms);
/* Append one row group of nrows (1..row group size) rows; only the last row
 * group of a file may be short.  Integer / FLOAT / DOUBLE column c:
 * data[c] -> nrows values of the column's width (1/2/4/8 B).  VARCHAR column c:
 * data[c] -> concatenated bytes, str_offsets[c] -> nrows+1 uint32 offsets
 * (str_offsets may be NULL when there is no VARCHAR column). */
int fls_writer_add_rowgroup(fls_writer *w, uint32_t nrows, const void *const *data,
                            const uint32_t *const *str_offsets);
/* Append nrg row groups in one call (rows nrows[k]; data / str_offsets hold
 * nrg * ncols pointers, row group k's column c at [k * ncols + c], as in
 * fls_writer_add_rowgroup).  The file is the same as from nrg calls of
 * fls_writer_add_rowgroup; the (row group, column) chunks are encoded in
 * parallel across the row groups, so a row group's slowest column does not
 * idle the other threads (the COPY sink hands over 8 row groups at a time). */
int fls_writer_add_rowgroups(fls_writer *w, uint32_t nrg, const uint32_t *nrows, const void *const *data,
                             const uint32_t *const *str_offsets);
/* The same with NULLs: validity[k * ncols + c] is row group k's validity mask
 * of column c in DuckDB's layout (u64 words, bit i of word j set when row
 * 64 j + i is valid) or NULL when every row is valid; validity itself may be
 * NULL.  Values (and string bytes) at NULL rows are ignored.  A chunk with a
 * NULL stores its bitmaps (csrc/fls_format.hpp, "Validity"); replaces the
 * reference writer's NULL tracking (src/writer/write_fastlane.cpp:207-208). */
int fls_writer_add_rowgroups_v(fls_writer *w, uint32_t nrg, const uint32_t *nrows, const void *const *data,
                               const uint32_t *const *str_offsets, const uint64_t *const *validity);
/* Stream the file to `path` while it is written: row groups whose chunks are
 * all encoded go to a temporary file beside `path` (their bytes freed once
 * written), and fls_writer_finish_file(w, path) -- the same path -- adds the
 * footer and renames the file over `path`.  Before the first row group.
 * fls_writer_free without a finish removes the temporary file; nothing is
 * left at `path`.  Not in the reference, whose writer is a stub
 * (src/writer/write_fastlane_stream.cpp:65-107). */
int fls_writer_set_output(fls_writer *w, const char *path);
/* Pipelined adds (on != 0): an add call returns once its row groups' chunk
 * tasks are queued behind the previous call's, not when they are encoded, so
 * the caller prepares the next batch while the threads encode this one.  The
 * file is the same.  The buffers of call k (the pointer arrays included) must
 * stay valid until call k+1, a finish, fls_writer_set_pipelined(w, 0) or
 * fls_writer_free returns.
 * on == 0 waits for the pending call's row groups.  No reference counterpart
 * (the reference's COPY writer is a stub, src/writer/write_fastlane_stream.cpp:
 * 65-107); the COPY sink of extension/src/scanner/ext_fastlanes_facade.cpp
 * uses it. */
int fls_writer_set_pipelined(fls_writer *w, int on);
/* Assemble the file: to `path` (written beside it, then renamed over it), or
 * into a malloc'ed buffer freed with fls_image_free. */
int fls_writer_finish_file(fls_writer *w, const char *path);
int fls_writer_finish_image(fls_writer *w, uint8_t **img, uint64_t *len);
void fls_image_free(uint8_t *img);

/* ---- seeded synthetic workloads (fls_gen.hpp) -------------------------
 * workload: "c1", "lineitem", "c3", "c4"; "lineitem_full" (16 columns,
 * l_comment FSST), "lineitem_dbl" (the DECIMAL columns as DOUBLE, ALP).
 * scale: lineitem scale factor
 * (ignored otherwise).  nrows: 0 = workload default (c1 1e6, c3/c4 1e9,
 * lineitem dbgen row count for the scale).  Row groups [rg_begin, rg_end) of
 * the full table are encoded into one image (a shard) using nthreads. */
int64_t fls_gen_nrows(const char *workload, double scale, uint64_t nrows);
int fls_gen_ncols(const char *workload);
int fls_gen_image(const char *workload, double scale, uint64_t nrows, uint32_t rg_begin,
                  uint32_t rg_end, int nthreads, uint8_t **img, uint64_t *len);
/* Ground truth of column col for rows [row_begin, row_begin+n): integer columns
 * in their value width, VARCHAR columns as uint32 dictionary codes. */
int fls_gen_values(const char *workload, double scale, uint64_t nrows, int col,
                   uint64_t row_begin, uint64_t n, void *out);
/* Strings of VARCHAR column col (dictionary or l_comment text) for rows
 * [row_begin, row_begin+n): offs receives n+1 offsets into bytes (cap bytes).
 * Returns the byte count. */
int64_t fls_gen_strings(const char *workload, double scale, uint64_t nrows, int col, uint64_t row_begin, uint64_t n,
                        uint32_t *offs, char *bytes, uint64_t cap);
/* Dictionary string `code` of VARCHAR column col (NULL if none). */
const char *fls_gen_dict_string(const char *workload, int col, uint32_t code);

#ifdef __cplusplus
}
#endif
#endif
