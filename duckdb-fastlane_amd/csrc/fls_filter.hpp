// fls_filter.hpp -- pushed-down scan filters (read_fastlanes filter_pushdown).
//
// The reference registers its scanner with filter_pushdown = false
// (src/scanner/scan_fastlanes.cpp:154), so DuckDB filters every decoded row on
// the CPU after the scan.  Here a filter is a conjunction of clauses, each a
// disjunction of terms `column <op> constant` -- the shape of DuckDB's
// TableFilterSet (ConstantFilter, ConjunctionAnd/Or, InFilter, IS [NOT] NULL).
// It is applied twice:
//   * on the host, per row group, against the footer zone maps and the DICT
//     dictionaries: row groups no row of which can qualify are never uploaded;
//   * on the GPU, per row, over the decoded batch in HBM (fls_filter.hip):
//     a selection mask, then only the qualifying rows of the delivered
//     columns are compacted and written to pinned host memory.
// The comparison semantics are DuckDB's, shared by both sides: signed /
// unsigned integers, IEEE floats with NaN equal to NaN and above every
// number and -0 == 0, strings compared bytewise (memcmp order, a proper
// prefix sorts first).  NULL rows (the chunks' validity bitmaps) satisfy
// IS NULL and no comparison, as in DuckDB; IS NOT NULL holds for the rest.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fls {

enum FilterKind : uint8_t {
    FK_INT = 0,    // signed integer (INT*, DATE days, DECIMAL scaled int64)
    FK_UINT = 1,   // unsigned integer
    FK_FLOAT = 2,  // FLOAT / DOUBLE, compared as double
    FK_STR = 3,    // VARCHAR (string_t records)
};
enum FilterOp : uint8_t {
    OP_EQ = 0, OP_NE = 1, OP_LT = 2, OP_LE = 3, OP_GT = 4, OP_GE = 5, OP_IS_NULL = 6, OP_IS_NOT_NULL = 7,
    OP_FALSE = 8  // no row (col <op> NULL)
};

__host__ __device__ inline bool op_holds(uint8_t op, int c) {
    switch (op) {
    case OP_EQ: return c == 0;
    case OP_NE: return c != 0;
    case OP_LT: return c < 0;
    case OP_LE: return c <= 0;
    case OP_GT: return c > 0;
    case OP_GE: return c >= 0;
    case OP_IS_NULL: return false;
    case OP_FALSE: return false;
    default: return true;  // IS NOT NULL
    }
}

__host__ __device__ inline int cmp_int(int64_t a, int64_t b) { return a < b ? -1 : (a > b ? 1 : 0); }
__host__ __device__ inline int cmp_uint(uint64_t a, uint64_t b) { return a < b ? -1 : (a > b ? 1 : 0); }
// DuckDB float ordering: NaN == NaN, NaN > every number; -0 == 0
__host__ __device__ inline int cmp_float(double a, double b) {
    const bool na = a != a, nb = b != b;
    if (na || nb) return na == nb ? 0 : (na ? 1 : -1);
    return a < b ? -1 : (a > b ? 1 : 0);
}
__host__ __device__ inline double as_double(uint64_t bits) {
    double d;
    __builtin_memcpy(&d, &bits, 8);
    return d;
}
// bytewise string comparison (DuckDB string_t ordering)
__host__ __device__ inline int cmp_bytes(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb) {
    const uint32_t n = la < lb ? la : lb;
    for (uint32_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

// One term of the filter as the kernel sees it, rebuilt per scan batch.
struct DevTerm {              // 64 B
    const uint8_t *col;       // decoded column of the batch in HBM (row 0 of the batch)
    const uint8_t *str;       // FK_STR: constant bytes in HBM
    uint64_t value;           // constant: int64 / uint64 / double bits
    uint64_t host_lo, host_hi;  // FK_STR: host range the long strings' pointers fall in
    int64_t dev_delta;        // ... and device address = host address + dev_delta
    uint32_t str_len;
    uint8_t kind, op, ob;     // FilterKind, FilterOp, bytes per decoded value
    uint8_t end_clause;       // 1 on the last term of a clause
    const uint64_t *valid;    // the column's validity words for the batch rows (HBM), or
                              // NULL when no row of the batch is NULL
};
static_assert(sizeof(DevTerm) == 64, "DevTerm is 64 B");

// One delivered column of a filtered batch: qualifying rows of src (HBM) are
// compacted into dst (pinned host memory, written by the kernel over PCIe).
struct DevOut {               // 32 B
    const uint8_t *src;
    uint8_t *dst;
    uint32_t ob;
    uint32_t pad[3];
};
static_assert(sizeof(DevOut) == 32, "DevOut is 32 B");

enum : uint32_t { KERR_FILTER_STR = 16 };
// a narrowed column's decoded value outside [base, base + 2^(8 nw)): the zone
// maps the narrowing trusted do not bound the data (corrupt or foreign file)
enum : uint32_t { KERR_NARROW = 64 };

// Selection mask (one bit per row: 16 x u64 words per 1024-row vector) and
// per-vector counts for the nrows decoded rows of a batch.
hipError_t launch_filter(const DevTerm *d_terms, uint32_t nterms, uint32_t nrows, uint64_t *d_mask,
                         uint32_t *d_counts, uint32_t *d_err, hipStream_t stream);
// Compact the selected rows of nouts columns (and their row indices within
// their row group of rg_rows rows, into sel) in row order.
hipError_t launch_compact(const DevOut *d_outs, uint32_t nouts, const uint64_t *d_mask, const uint32_t *d_counts,
                          uint32_t nrows, uint32_t rg_rows, uint32_t *sel, hipStream_t stream);

// Narrowed delivery (fls_scan_narrow): an integer column of a batch whose
// values, per row group, lie in [base, base + 2^(8 nw)) crosses PCIe as the
// nw-byte differences value - base (the host adds the base back).  Reads ob
// bytes and writes nw per row: HBM-side work that saves (ob - nw) bytes of
// PCIe per row.
struct DevNarrow {            // 32 B
    const uint8_t *src;       // decoded column of the batch (HBM, ob bytes per row)
    uint8_t *dst;             // narrowed copy (HBM, nw bytes per row)
    const uint64_t *base;     // per row group of the batch (row / rg_rows): the value subtracted
    uint8_t ob, nw, sign;     // widths; sign: values sign-extend from ob bytes
    uint8_t pad[5];
};
static_assert(sizeof(DevNarrow) == 32, "DevNarrow is 32 B");
hipError_t launch_narrow(const DevNarrow *d_cols, uint32_t ncols, uint32_t nrows, uint32_t rg_rows,
                         uint32_t *d_err, hipStream_t stream);

// Delivery of a batch's decoded columns and string heaps into pinned host
// memory by a copy kernel (FLS_SCAN_COPY_KERNEL, default 1) instead of the DMA engines: a
// hipMemcpy D2H ran 57.1 GB/s in some processes and 30.2 in others on one box (link at 32 GT/s x16 throughout), a copy kernel 54.7 in
// every process (profiles/r6/d2h_probe_r6an.txt).  Both pointers of a copy
// are 16-byte aligned (the caller sends the others through hipMemcpyAsync);
// up to kHostCopyMax copies per launch, passed by value.
struct HostCopy {
    const uint8_t *src;  // HBM or pinned host memory
    uint8_t *dst;        // the other
    uint64_t bytes;
};
constexpr uint32_t kHostCopyMax = 40;
constexpr uint32_t kHostCopyPiece = 64u << 10;  // bytes per block iteration
struct HostCopyList {
    HostCopy c[kHostCopyMax];
    uint32_t first[kHostCopyMax + 1];  // first piece of each copy; first[n] = total pieces
    uint32_t n;
};
hipError_t launch_host_copy(const HostCopy *copies, uint32_t n, hipStream_t stream);

}  // namespace fls
