/*
 * flscheck.h -- full-size GPU verification of decoded columns against the
 * seeded generators (libflscheck.so).  Test / bench support: it answers
 * "is every decoded value of a 1e9-row / SF100 scan bit-exact?" without a host
 * copy, by regenerating the ground truth (duckdb-fastlane_amd/csrc/fls_gen.hpp)
 * on the GPU next to the decoded columns.  Not part of the decode product.
 */
#ifndef FLSCHECK_H
#define FLSCHECK_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Compare decoded rows [0, n) -- global rows [row_begin, row_begin+n) of the
 * workload (c1, lineitem, lineitem_full, lineitem_dbl, c3, c4) -- of ncols
 * columns resident on the current HIP device.
 * d_cols[c]: device column (NULL = skip); out_bytes[c]: 1/2/4/8 or 16 for
 * string_t; dicts[c]: for dictionary VARCHAR columns a NUL-separated,
 * double-NUL-ended list of the dictionary strings (codes 0..7);
 * heap_delta[c]: for the free-text column (lineitem_full's l_comment, FSST) the
 * device address of its string heap minus the host address its string_t
 * pointers carry (NULL when there is none).  mismatches[c] receives the
 * number of mismatching rows.  Returns 0, or -1 with fls_check_last_error(). */
int fls_check_workload(const char *workload, double scale, uint64_t nrows_total, uint64_t row_begin,
                       uint64_t n, const void *const *d_cols, const uint8_t *out_bytes, int ncols,
                       const void *const *dicts, const int64_t *heap_delta, uint64_t *mismatches);
/* The same on HIP device `device` (one part of a table resident on several GPUs). */
int fls_check_workload_on(int device, const char *workload, double scale, uint64_t nrows_total, uint64_t row_begin,
                          uint64_t n, const void *const *d_cols, const uint8_t *out_bytes, int ncols,
                          const void *const *dicts, const int64_t *heap_delta, uint64_t *mismatches);
const char *fls_check_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
