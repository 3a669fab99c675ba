/*
 * flsgpu.h -- C-ABI of the MI355X FastLanes decode engine (libflsgpu.so).
 *
 * This is the seam the reference's FastLanesFacade::Impl
 * (src/fastlanes_facade.cpp:12-20) crosses into its decode library.  Each
 * entry point names the cwida/FastLanes call it replaces:
 *
 *   fls_connect            fastlanes::connect()                src/fastlanes_facade.cpp:33
 *   fls_read_fls           Connection::read_fls(path)          src/fastlanes_facade.cpp:34
 *   fls_table_nrows/...    Rowgroup::RowCount()/ColCount()     src/fastlanes_facade.cpp:52-56,85
 *   fls_table_column       Rowgroup::internal_rowgroup[c] type src/fastlanes_facade.cpp:112-183
 *                          (typed schema: ext_fastlane::FastLanesFacade::
 *                          getColumnTypes/getColumnNames,
 *                          src/include/fastlanes_facade.hpp:34-35)
 *   fls_materialize        TableReader::get_rowgroup_reader(rg)
 *                          + RowgroupReader::materialize()     src/fastlanes_facade.cpp:41,48
 *   fls_scan_begin/next    the row-group loop the reference never wrote
 *                          (it decodes row group 0 only, :41)
 *   fls_scan_acquire/release  the same loop for a parallel DuckDB scan
 *                          (MaxThreads > 1, batch index = row group; the
 *                          reference pins MaxThreads to 1,
 *                          src/scanner/scan_fastlanes.cpp:43-45)
 *   fls_table_close/fls_disconnect  FastLanesFacade::closeFile  src/fastlanes_facade.cpp:202-210
 *
 * Conventions: plain pointers and sizes, no exceptions across the ABI; every
 * function returns 0 (or a count) on success and a negative fls_status on
 * error, with fls_last_error() holding a message for the calling thread.
 * Decoded columns are DuckDB physical layouts: int8..int64 little-endian,
 * DATE int32 days, DECIMAL int64 scaled, VARCHAR duckdb::string_t (16 B:
 * u32 length + 12 inline bytes, or u32 length + 4-byte prefix + char* into a
 * pinned host dictionary heap owned by the table).
 * A table handle is used by one host thread at a time (DuckDB's scan thread,
 * src/scanner/scan_fastlanes.cpp:43-45), except fls_scan_acquire/release,
 * which any number of threads may call concurrently between fls_scan_begin
 * and the next begin/close; internally there is one HIP stream set per GPU.
 */
#ifndef FLSGPU_H
#define FLSGPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum fls_status {
    FLS_OK = 0,
    FLS_ERR_IO = -1,        /* cannot open / read the file */
    FLS_ERR_FORMAT = -2,    /* not an .fls file or corrupt footer / chunk */
    FLS_ERR_ARG = -3,       /* bad argument (index out of range, NULL) */
    FLS_ERR_DEVICE = -4,    /* HIP runtime error or no usable GPU */
    FLS_ERR_STATE = -5,     /* call out of order (e.g. decode before upload) */
    FLS_ERR_NOMEM = -6,
    FLS_ERR_CONFIG = -7     /* an FLS_* tuning variable names a kernel this build does not hold */
} fls_status;

typedef struct fls_connection fls_connection;
typedef struct fls_table fls_table;

typedef struct fls_column_info {
    const char *name;   /* NUL-terminated, owned by the table */
    uint8_t type;       /* enum fls_type (flswriter.h) */
    uint8_t width;      /* DECIMAL width */
    uint8_t scale;      /* DECIMAL scale */
    uint8_t out_bytes;  /* bytes per decoded value (string_t = 16) */
} fls_column_info;

typedef struct fls_rowgroup {
    uint32_t rowgroup;            /* row-group index within the table */
    uint32_t nrows;               /* rows delivered (after a pushed-down filter) */
    uint64_t first_row;           /* global row index of the row group's first row */
    uint32_t ncols;
    const void *const *columns;   /* ncols pointers into pinned host memory;
                                     NULL for columns not selected */
    uint32_t nrows_scanned;       /* rows of the row group */
    const uint32_t *sel;          /* filtered scan: the delivered rows' indices
                                     within the row group (ascending); NULL
                                     when every row is delivered */
    const uint64_t *const *validity; /* ncols pointers: the delivered rows'
                                     validity mask in DuckDB's layout (bit i
                                     of word i / 64 set when delivered row i
                                     is not NULL), or NULL when every
                                     delivered row is valid (and for columns
                                     not selected).  Values at NULL rows are
                                     placeholders.  Valid as long as columns. */
    const void *const *dict;      /* ncols pointers (fls_scan_dict_codes): for a
                                     column delivered as dictionary codes in
                                     this row group, its dictionary as 16-byte
                                     string_t records (host); columns[c] then
                                     holds one code per delivered row,
                                     dict_width[c] bytes each (1 or 2, little
                                     endian).  NULL for other columns. */
    const uint32_t *dict_size;    /* ncols: entries of dict[c] */
    const uint8_t *dict_width;    /* ncols: bytes per delivered value */
    const uint8_t *narrow;        /* ncols (fls_scan_narrow): 1 when columns[c]
                                     holds value - narrow_base[c] as an
                                     unsigned dict_width[c]-byte integer (the
                                     value, mod 2^64, is their sum) */
    const uint64_t *narrow_base;  /* ncols: this row group's base */
} fls_rowgroup;

/* Pushed-down filter term: `column <op> constant` (DuckDB TableFilterSet:
 * ConstantFilter / IsNullFilter / IsNotNullFilter; ConjunctionOr and InFilter
 * become several terms of one clause, ConjunctionAnd several clauses).
 * Terms with equal `clause` are OR-ed, clauses are AND-ed. */
typedef enum fls_cmp {
    FLS_CMP_EQ = 0, FLS_CMP_NE = 1, FLS_CMP_LT = 2, FLS_CMP_LE = 3, FLS_CMP_GT = 4, FLS_CMP_GE = 5,
    FLS_CMP_IS_NULL = 6, FLS_CMP_IS_NOT_NULL = 7,
    FLS_CMP_FALSE = 8             /* holds for no row (a comparison with a NULL constant) */
} fls_cmp;
typedef struct fls_predicate {
    uint32_t col;                 /* table column */
    uint32_t clause;
    uint8_t op;                   /* fls_cmp */
    uint8_t pad[7];
    uint64_t value;               /* constant in the column's physical type:
                                     signed ints / DATE days / DECIMAL scaled as
                                     int64, unsigned as uint64, FLOAT as IEEE
                                     binary32 bits (low 32), DOUBLE binary64 bits */
    const char *str;              /* VARCHAR constant (copied) */
    uint64_t str_len;
} fls_predicate;

typedef struct fls_decode_stats {
    double kernel_ms;             /* duration of the last decode launch (HIP events) */
    uint64_t values;              /* values decoded by that launch */
    uint64_t packed_bytes;        /* algorithmic bytes read: bit-packed streams */
    uint64_t meta_bytes;          /* per-vector metadata, bases, dictionaries, run values */
    uint64_t out_bytes;           /* algorithmic bytes written: decoded columns */
    uint32_t launches;            /* decode launches since upload */
    uint32_t timed_launches;      /* launches since the previous fls_device_sync */
    double kernel_ms_total;       /* sum of their kernel durations (HIP events on the
                                     decode stream, one start/stop pair per launch) */
} fls_decode_stats;

const char *fls_last_error(void);
const char *fls_version(void);
/* Deployment knobs: the environment variables the library and the extension
 * read (FLS_IDLE_PINNED_MB, FLS_SCAN_RESIDENT_MB, FLS_COPY_BATCH, ...; the
 * list with each meaning is in INTEGRATION.md), defaults kept in one table
 * (csrc/fls_config.hpp).  fls_config_default: the compiled default;
 * fls_config_value: the value in effect (the environment's, else the
 * default); FLS_ERR_ARG for a name that is not a knob.  fls_config_count /
 * fls_config_name enumerate the knobs (NULL past the end).  Not in the
 * reference, which reads no environment. */
int fls_config_default(const char *name, int64_t *value);
int fls_config_value(const char *name, int64_t *value);
int fls_config_count(void);
const char *fls_config_name(int i);
/* Number of HIP devices visible (0 when there is no GPU). */
int fls_device_count(void);
/* Raw device buffers and copies on GPU `device`, for callers that hold no HIP
 * runtime of their own (bindings, tests, the encoder bench): kind 0 = host to
 * device, 1 = device to host, 2 = device to device. */
int fls_device_alloc(int device, uint64_t bytes, void **ptr);
int fls_device_free(int device, void *ptr);
int fls_device_memcpy(int device, void *dst, const void *src, uint64_t bytes, int kind);

/* fastlanes::connect(): devices = HIP ordinals to shard row groups over
 * (NULL/0 = device 0). */
int fls_connect(const int *devices, int ndevices, fls_connection **out);
void fls_disconnect(fls_connection *conn);
/* Free the connection's idle scan pipelines (streams, device slots, pinned
 * host batches kept for the next scan) down to keep_bytes of pinned memory
 * per GPU (0: all of them); idle_bytes (may be NULL) receives what stays.
 * Idle pinned memory is also capped per GPU when a scan ends
 * (FLS_IDLE_PINNED_MB, default 1024).  Not in the reference: a long-lived
 * host (DuckDB) uses it to hand page-locked memory back. */
int fls_connection_trim(fls_connection *conn, uint64_t keep_bytes, uint64_t *idle_bytes);
/* HBM-resident compressed images (the scan pipeline keeps a scanned file's
 * bytes in HBM so warm queries skip the H2D): one byte budget per GPU over
 * every cached file (FLS_SCAN_RESIDENT_MB, default 65,536), least recently
 * used images evicted first, never one a running scan uses.  Not in the
 * reference, whose closeFile (src/fastlanes_facade.cpp:202-210) releases
 * everything it holds.
 * fls_release_device_memory: free every image no running scan uses on
 * device (-1: every GPU); freed_bytes (may be NULL) receives the bytes freed.
 * fls_resident_info: the images' bytes and count on device (-1: every GPU). */
int fls_release_device_memory(int device, uint64_t *freed_bytes);
int fls_resident_info(int device, uint64_t *bytes, uint32_t *images);

/* Connection::read_fls(): parse footer + schema (no GPU work). */
int fls_read_fls(fls_connection *conn, const char *path, fls_table **out);
/* Same over an in-memory image (copy=0: caller keeps img alive). */
int fls_read_fls_image(fls_connection *conn, const void *img, uint64_t len, int copy, fls_table **out);
void fls_table_close(fls_table *t);

uint32_t fls_table_ncols(const fls_table *t);
uint64_t fls_table_nrows(const fls_table *t);
uint64_t fls_table_row_offset(const fls_table *t);
uint32_t fls_table_nrowgroups(const fls_table *t);
int64_t fls_table_rowgroup_rows(const fls_table *t, uint32_t rg);
int fls_table_column(const fls_table *t, uint32_t col, fls_column_info *out);

/* Decode the selected columns (col_mask[c] != 0; NULL = all) of one row group
 * on the GPU that owns it and deliver them into pinned host buffers owned by
 * the table, valid until the next materialize/scan call. */
int fls_materialize(fls_table *t, uint32_t rg, const uint8_t *col_mask, fls_rowgroup *out);

/* Streaming scan over row groups [rg_begin, rg_end) in order: row groups are
 * sharded contiguously over the connection's GPUs, uploaded once, decoded in
 * batches and copied to pinned host memory ahead of the consumer. */
int fls_scan_begin(fls_table *t, const uint8_t *col_mask, uint32_t rg_begin, uint32_t rg_end);
/* 1 = a row group was delivered into *out, 0 = end of scan, <0 = error.
 * The previous row group's buffers are released by the call. */
int fls_scan_next(fls_table *t, fls_rowgroup *out);
/* Filter for the following fls_scan_begin calls on this table (n = 0
 * clears).  The scan then skips row groups whose zone maps / dictionaries
 * rule every row out, evaluates the filter per row on the GPU and delivers
 * only qualifying rows (fls_rowgroup.nrows / sel), in row order.  The
 * filter's columns are decoded whether or not col_mask delivers them. */
int fls_scan_filter(fls_table *t, const fls_predicate *preds, uint32_t n);
/* Row groups the current scan skipped by zone maps / dictionaries. */
int fls_scan_pruned(const fls_table *t);
/* Zone map of column col in row group rg: 1 and *min / *max (int64, uint64
 * or double bits by column type, see fls_predicate.value; FLOAT widened to
 * double) and *flags (1 valid, 2 / 4 has / all NaN, 8 / 16 has / all NULL;
 * min / max over the non-NULL rows) when present, 0 when the file has none
 * for it. */
int fls_table_zonemap(const fls_table *t, uint32_t rg, uint32_t col, uint64_t *min, uint64_t *max, uint32_t *flags);
/* Dictionary-coded delivery for the next fls_scan_begin (enable != 0): a
 * delivered VARCHAR / BLOB column no filter term reads, whose chunks in a
 * batch are all DICT, crosses PCIe as 1- or 2-byte codes instead of 16-byte
 * string_t records (fls_rowgroup.dict / dict_width); what a DuckDB
 * dictionary vector needs.  Off by default. */
int fls_scan_dict_codes(fls_table *t, int enable);
/* Narrowed delivery for the next fls_scan_begin (enable != 0): a delivered
 * integer / DATE / DECIMAL column whose zone maps put every value of a
 * batch's row groups within 2^8, 2^16 or 2^32 of its row group's minimum
 * crosses PCIe as the 1-, 2- or 4-byte difference (fls_rowgroup.narrow /
 * narrow_base); the consumer adds the base back while filling its vectors.
 * Off by default. */
int fls_scan_narrow(fls_table *t, int enable);
/* With fls_scan_narrow (FLS_SCAN_STRLEN, default 1; 0 ships string_t
 * records instead: the lengths measured 7.81e8 against 6.78e8 rows/s on the
 * link-bound 16-thread read_fastlanes, profiles/r4/e2e_arms_strlen_r4t.txt),
 * an unfiltered scan also delivers FSST string columns
 * as their lengths (1, 2 or 4 bytes per row) plus the string heap, and the
 * string_t records are rebuilt on the host; fls_rowgroup shows them as
 * ordinary string_t columns.  fls_scan_acquire builds them unless
 * fls_scan_defer_records(t, 1) was set before fls_scan_begin: then the
 * consumer calls fls_scan_build_records(t, &rg) for each acquired row group
 * before reading its string columns (so a consumer that serialises its
 * acquires builds them in parallel, outside its lock). */
int fls_scan_defer_records(fls_table *t, int enable);
int fls_scan_build_records(fls_table *t, const fls_rowgroup *rg);
/* Validity of column col in row group rg: 1 and *words = its bitmaps in the
 * host image (16 u64 words per 1024-row vector, DuckDB's layout: bit i of
 * word j set when row 64 j + i is valid) when the chunk holds a NULL, 0 (and
 * *words = NULL) when every row is valid.  Valid while the table is open;
 * for consumers of the device-resident columns (fls_device_column). */
int fls_table_validity(const fls_table *t, uint32_t rg, uint32_t col, const uint64_t **words);
/* May a row of row group rg satisfy the filter?  (1 yes / 0 no; host only) */
int fls_rowgroup_may_match(const fls_table *t, uint32_t rg, const fls_predicate *preds, uint32_t n);

/* Thread-safe form for parallel consumers: claims the next row group in order
 * (1 = delivered, 0 = end, <0 = error); its buffers stay valid until
 * fls_scan_release(t, out->rowgroup), so a consumer may keep several row
 * groups (DuckDB vectors referencing the pinned columns, zero-copy).  A GPU's
 * batch slot is refilled as soon as every row group of its batch has been
 * handed out; the pinned host side of a batch goes back to a per-GPU pool when
 * its last row group is released (pool cap FLS_SCAN_HOST_BATCHES, default 64;
 * at the cap a refill waits for a release).  A failed refill is sticky: every
 * later acquire returns its error.  Do not mix with fls_scan_next on one scan. */
int fls_scan_acquire(fls_table *t, fls_rowgroup *out);
int fls_scan_release(fls_table *t, uint32_t rowgroup);

/* ---- device-resident mode (HBM roofline measurement, bench.py) ---------
 * Upload row groups [rg_begin, rg_end) of the table to HBM, split into
 * contiguous parts over the connection's GPUs (as a scan shards them; a GPU
 * gets no part when there are fewer row groups than GPUs), and allocate HBM
 * output columns for them. */
int fls_device_upload(fls_table *t, uint32_t rg_begin, uint32_t rg_end);
/* Enqueue ONE decode launch per GPU over every resident vector of the
 * selected columns (col_mask NULL = all) into HBM.  Asynchronous: the parts
 * decode concurrently. */
int fls_device_decode(fls_table *t, const uint8_t *col_mask);
/* Wait for the table's GPU work; fills *stats if non-NULL: values and bytes
 * summed over the parts, kernel_ms = the last launch, kernel_ms_total over the
 * launches since the previous sync, a launch timed as its slowest part. */
int fls_device_sync(fls_table *t, fls_decode_stats *stats);

typedef struct {
    int device;               /* HIP ordinal */
    uint32_t rg_begin, rg_end;
    uint64_t first_row;       /* first resident row, relative to the table's first row */
    uint64_t nrows;
} fls_device_part_info;
/* Number of resident parts (GPUs holding row groups) and each one's extent. */
int fls_device_parts(const fls_table *t);
int fls_device_part(const fls_table *t, uint32_t part, fls_device_part_info *out);
/* HBM address and byte size of a resident output column of one part. */
int fls_device_part_column(fls_table *t, uint32_t part, uint32_t col, void **dev_ptr, uint64_t *nbytes);
/* String heap of a part's resident FSST VARCHAR column (see fls_device_heap). */
int fls_device_part_heap(fls_table *t, uint32_t part, uint32_t col, void **dev_ptr, const void **host_ptr,
                         uint64_t *nbytes);
/* HBM address and byte size of a resident output column (single-part tables;
 * FLS_ERR_STATE when the table is split over several GPUs). */
int fls_device_column(fls_table *t, uint32_t col, void **dev_ptr, uint64_t *nbytes);
/* String heap of a resident FSST (free-text) VARCHAR column: its HBM address,
 * the host address the column's string_t pointers are based on (the heap's
 * host copy, filled by fls_device_copy_out) and its size.  Returns 1, or 0
 * (pointers NULL) for a column without one. */
int fls_device_heap(fls_table *t, uint32_t col, void **dev_ptr, const void **host_ptr, uint64_t *nbytes);
/* Copy rows [row, row+n) (relative to the first resident row, counted over
 * the parts in order) of a decoded column into host memory. */
int fls_device_copy_out(fls_table *t, uint32_t col, uint64_t row, uint64_t n, void *host_dst);
/* Rows resident on the GPUs (all parts). */
uint64_t fls_device_rows(const fls_table *t);

#ifdef __cplusplus
}
#endif
#endif
