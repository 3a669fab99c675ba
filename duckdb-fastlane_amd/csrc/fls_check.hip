// fls_check.hip -- full-size bit-exact verification on the GPU (libflscheck.so).
//
// Test / bench support, not the decode product: at BASELINE.json's full sizes
// (1e9 rows, SF100) copying decoded columns back to the host for a CPU
// comparison would dominate the run, so this kernel regenerates the seeded
// ground truth (fls_gen.hpp -- the same pure functions of (seed, row) the
// writer encoded) next to the decoded columns in HBM and counts mismatching
// rows per column.  Integer codecs are lossless: any mismatch is a decode bug.
// VARCHAR string_t records are compared in full when inlined (<= 12 bytes) and
// on length + 4-byte prefix when they point into the host dictionary heap.
// Free text (l_comment, FSST, workload lineitem_full) is compared in full:
// length, inline bytes or prefix, and every byte of a long string read from
// the column's device heap (string_t pointer + heap_delta) against the text
// pool uploaded next to it.  lineitem_dbl's ALP columns are compared as the
// IEEE bits of cents / 100.0.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/flscheck.h"
#include "fls_gen.hpp"
#include "fls_text.hpp"

namespace {

constexpr int kMaxCols = 16;
constexpr int kMaxDict = 8;
constexpr int kRowsPerThread = 256;

struct CheckArgs {
    const uint8_t *col[kMaxCols];   // decoded columns (device), nullptr = skip
    uint32_t ob[kMaxCols];          // output bytes per value
    uint32_t str_cmp[kMaxCols];     // VARCHAR: per code bytes to compare (16 or 8), packed 4 bits x 8
    uint4 dict[kMaxCols][kMaxDict]; // expected string_t per code (pointer bytes zero)
    int64_t heap_delta[kMaxCols];   // free-text column: device heap address - string_t pointer base
    uint32_t text_col;              // free-text column (l_comment) or kMaxCols
    uint32_t dbl_mask;              // columns decoded as DOUBLE = cents / 100.0 (lineitem_dbl)
    const uint8_t *pool;            // text pool (device), pool_size bytes
    uint64_t pool_size;
    int ncols;
    int workload;                   // 0 c1, 1 lineitem (+ _full, _dbl), 2 c3, 3 c4
    fls::gen::LineitemParams li;
    uint64_t row_begin;             // global row of decoded row 0
    uint64_t n;
};

__device__ __forceinline__ bool eq_col(const CheckArgs &a, int c, uint64_t i, int64_t v) {
    const uint8_t *p = a.col[c];
    switch (a.ob[c]) {
    case 1: return *(const int8_t *)(p + i) == (int8_t)v;
    case 2: return *(const int16_t *)(p + 2 * i) == (int16_t)v;
    case 4: return *(const int32_t *)(p + 4 * i) == (int32_t)v;
    case 8: return *(const int64_t *)(p + 8 * i) == v;
    default: {
        const uint4 got = *(const uint4 *)(p + 16 * i);
        const uint32_t code = (uint32_t)v;
        if (code >= kMaxDict) return false;
        const uint4 e = a.dict[c][code];
        const uint32_t nb = (a.str_cmp[c] >> (4 * code)) & 0xF;  // 4 -> 16 bytes, 2 -> 8 bytes
        if (got.x != e.x || got.y != e.y) return false;
        return nb == 2 || (got.z == e.z && got.w == e.w);
    }
    }
}

// l_comment of global row `row` against its decoded string_t record
__device__ __forceinline__ bool eq_text(const CheckArgs &a, int c, uint64_t i, uint64_t row) {
    uint64_t off;
    uint32_t len;
    fls::gen::comment_span(a.li.seed, row, a.pool_size, off, len);
    const uint4 got = *(const uint4 *)(a.col[c] + 16 * i);
    if (got.x != len) return false;
    const uint8_t *want = a.pool + off;
    if (len <= 12) {
        const uint8_t *b = (const uint8_t *)&got + 4;
        for (uint32_t k = 0; k < 12; ++k)
            if (b[k] != (k < len ? want[k] : 0)) return false;
        return true;
    }
    const uint8_t *pre = (const uint8_t *)&got + 4;
    for (uint32_t k = 0; k < 4; ++k)
        if (pre[k] != want[k]) return false;
    const uint8_t *str = (const uint8_t *)(((uint64_t)got.w << 32 | got.z) + (uint64_t)a.heap_delta[c]);
    for (uint32_t k = 0; k < len; ++k)
        if (str[k] != want[k]) return false;
    return true;
}

__device__ __forceinline__ int64_t dbl_bits(int64_t cents) {
    const double d = (double)cents / 100.0;
    return __double_as_longlong(d);
}

__global__ void check_kernel(CheckArgs a, unsigned long long *mism) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * kRowsPerThread;
    if (i0 >= a.n) return;
    const uint64_t i1 = i0 + kRowsPerThread < a.n ? i0 + kRowsPerThread : a.n;
    uint32_t bad[kMaxCols];
    for (int c = 0; c < kMaxCols; ++c) bad[c] = 0;
    const uint64_t seed = a.li.seed;
    if (a.workload == 1) {
        fls::gen::OrderWalker ow;
        ow.start(seed, a.row_begin + i0);
        fls::gen::LineitemRow r;
        for (uint64_t i = i0; i < i1; ++i, ow.next()) {
            fls::gen::lineitem_row_at(a.li, a.row_begin + i, ow.cur(), r);
            for (int c = 0; c < a.ncols; ++c) {
                if (!a.col[c]) continue;
                if ((uint32_t)c == a.text_col) {
                    if (!eq_text(a, c, i, a.row_begin + i)) bad[c]++;
                    continue;
                }
                const int64_t v = fls::gen::lineitem_col(r, c);
                if (!eq_col(a, c, i, (a.dbl_mask >> c) & 1 ? dbl_bits(v) : v)) bad[c]++;
            }
        }
    } else if (a.workload == 2) {
        fls::gen::OrderWalker ow;
        ow.start(seed, a.row_begin + i0);
        for (uint64_t i = i0; i < i1; ++i, ow.next())
            if (!eq_col(a, 0, i, fls::gen::orderkey(ow.cur().order))) bad[0]++;
    } else {
        for (uint64_t i = i0; i < i1; ++i) {
            const int64_t v = a.workload == 0 ? fls::gen::c1_value(seed, a.row_begin + i)
                                              : fls::gen::c4_code(seed, a.row_begin + i);
            if (!eq_col(a, 0, i, v)) bad[0]++;
        }
    }
    for (int c = 0; c < a.ncols; ++c)
        if (bad[c]) atomicAdd(&mism[c], (unsigned long long)bad[c]);
}

thread_local std::string g_err;

int err(const std::string &s) {
    g_err = s;
    return -1;
}

}  // namespace

extern "C" {

const char *fls_check_last_error(void) { return g_err.c_str(); }

int fls_check_workload(const char *workload, double scale, uint64_t nrows_total, uint64_t row_begin, uint64_t n,
                       const void *const *d_cols, const uint8_t *out_bytes, int ncols, const void *const *dicts,
                       const int64_t *heap_delta, uint64_t *mismatches) {
    if (!workload || !d_cols || !out_bytes || !mismatches || ncols < 1 || ncols > kMaxCols)
        return err("fls_check_workload: bad arguments");
    CheckArgs a;
    memset(&a, 0, sizeof(a));
    std::string w = workload;
    const bool li = w == "lineitem" || w == "lineitem_full" || w == "lineitem_dbl";
    a.workload = w == "c1" ? 0 : li ? 1 : w == "c3" ? 2 : w == "c4" ? 3 : -1;
    if (a.workload < 0) return err("unknown workload " + w);
    a.text_col = kMaxCols;
    if (w == "lineitem_dbl") a.dbl_mask = 0xF0u;  // quantity, extendedprice, discount, tax
    uint8_t *d_pool = nullptr;
    if (w == "lineitem_full" && ncols > 15 && d_cols[15]) {
        if (!heap_delta) return err("lineitem_full: l_comment needs its heap_delta");
        const std::string &pool = fls::gen::text_pool();
        if (hipMalloc(&d_pool, pool.size()) != hipSuccess) return err("hipMalloc failed");
        if (hipMemcpy(d_pool, pool.data(), pool.size(), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d_pool);
            return err("hipMemcpy failed");
        }
        a.text_col = 15;
        a.pool = d_pool;
        a.pool_size = pool.size();
        a.heap_delta[15] = heap_delta[15];
    }
    a.ncols = ncols;
    a.li.seed = fls::gen::kSeed;
    a.li.nrows = nrows_total;
    a.li.n_part = std::max<int64_t>(1, (int64_t)(200000.0 * scale + 0.5));
    a.li.n_supp = std::max<int64_t>(4, (int64_t)(10000.0 * scale + 0.5));
    a.row_begin = row_begin;
    a.n = n;
    for (int c = 0; c < ncols; ++c) {
        a.col[c] = (const uint8_t *)d_cols[c];
        a.ob[c] = out_bytes[c];
        if (out_bytes[c] == 16 && (uint32_t)c != a.text_col) {
            // dicts[c]: NUL-separated list of the column's dictionary strings (<= 8)
            const char *s = dicts ? (const char *)dicts[c] : nullptr;
            if (!s) return err("VARCHAR column needs its dictionary");
            for (int k = 0; k < kMaxDict && *s; ++k) {
                const size_t len = strlen(s);
                uint8_t rec[16] = {0};
                const uint32_t l32 = (uint32_t)len;
                memcpy(rec, &l32, 4);
                memcpy(rec + 4, s, len <= 12 ? len : 4);
                memcpy(&a.dict[c][k], rec, 16);
                a.str_cmp[c] |= (len <= 12 ? 4u : 2u) << (4 * k);
                s += len + 1;
            }
        }
    }
    unsigned long long *d_m = nullptr;
    if (hipMalloc(&d_m, sizeof(unsigned long long) * kMaxCols) != hipSuccess) {
        if (d_pool) (void)hipFree(d_pool);
        return err("hipMalloc failed");
    }
    if (hipMemset(d_m, 0, sizeof(unsigned long long) * kMaxCols) != hipSuccess) return err("hipMemset failed");
    const uint64_t threads = (n + kRowsPerThread - 1) / kRowsPerThread;
    const uint32_t blocks = (uint32_t)((threads + 255) / 256);
    if (blocks) hipLaunchKernelGGL(check_kernel, dim3(blocks), dim3(256), 0, 0, a, d_m);
    hipError_t e = hipDeviceSynchronize();
    if (d_pool) (void)hipFree(d_pool);
    if (e != hipSuccess) {
        (void)hipFree(d_m);
        return err(std::string("check kernel failed: ") + hipGetErrorString(e));
    }
    unsigned long long h[kMaxCols];
    (void)hipMemcpy(h, d_m, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d_m);
    for (int c = 0; c < ncols; ++c) mismatches[c] = h[c];
    return 0;
}

int fls_check_workload_on(int device, const char *workload, double scale, uint64_t nrows_total, uint64_t row_begin,
                          uint64_t n, const void *const *d_cols, const uint8_t *out_bytes, int ncols,
                          const void *const *dicts, const int64_t *heap_delta, uint64_t *mismatches) {
    if (hipSetDevice(device) != hipSuccess) return err("hipSetDevice failed");
    return fls_check_workload(workload, scale, nrows_total, row_begin, n, d_cols, out_bytes, ncols, dicts, heap_delta,
                              mismatches);
}

}  // extern "C"
