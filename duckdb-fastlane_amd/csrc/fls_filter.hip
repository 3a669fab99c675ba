// fls_filter.hip -- gfx950 kernels of the pushed-down scan filter
// (fls_filter.hpp): row selection over a decoded batch in HBM, then
// compaction of the qualifying rows straight into pinned host memory.
//
// Both kernels are byte-moving, HBM-bound integer work (no MFMA):
//   filter:  reads ob bytes per row per term column, writes 1 bit per row;
//   compact: reads the mask + ob bytes per selected row per delivered column
//            (whole 128-B lines of HBM wherever rows qualify), writes the
//            selected values over PCIe.
// A 256-thread block owns one 1024-row vector; wave w handles its 64-row
// words 4w..4w+3 (lane = row within the word), so every term load is one
// coalesced wave access and a word's selection is one ballot.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "fls_decode.hpp"
#include "fls_filter.hpp"

namespace fls {
namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t readlane64(uint64_t x, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

__device__ __forceinline__ int64_t load_int(const uint8_t *p, uint32_t ob) {
    switch (ob) {
    case 1: return *(const int8_t *)p;
    case 2: return *(const int16_t *)p;
    case 4: return *(const int32_t *)p;
    default: return *(const int64_t *)p;
    }
}
__device__ __forceinline__ uint64_t load_uint(const uint8_t *p, uint32_t ob) {
    switch (ob) {
    case 1: return *p;
    case 2: return *(const uint16_t *)p;
    case 4: return *(const uint32_t *)p;
    default: return *(const uint64_t *)p;
    }
}

// string_t record at p against the term's constant
__device__ __forceinline__ int cmp_string(const DevTerm &t, const uint8_t *p, bool &bad) {
    const v4u rec = *(const v4u *)p;
    const uint32_t len = rec.x;
    // the 4 bytes after the length are the string's first bytes in both the
    // inlined and the pointer form: most comparisons end there
    const uint32_t k = min(4u, min(len, t.str_len));
    for (uint32_t i = 0; i < k; ++i) {
        const uint8_t a = p[4 + i], b = t.str[i];
        if (a != b) return a < b ? -1 : 1;
    }
    if (len <= 4 || t.str_len <= 4) return len < t.str_len ? -1 : (len > t.str_len ? 1 : 0);
    if ((t.op == OP_EQ || t.op == OP_NE) && len != t.str_len) return 1;
    const uint8_t *s;
    if (len <= 12) {
        s = p + 4;
    } else {
        const uint64_t hp = ((uint64_t)rec.w << 32) | rec.z;
        if (hp < t.host_lo || hp > t.host_hi || len > t.host_hi - hp) {
            bad = true;
            return 1;
        }
        s = (const uint8_t *)(hp + t.dev_delta);
    }
    return cmp_bytes(s + 4, len - 4, t.str + 4, t.str_len - 4);
}

__device__ __forceinline__ bool eval_term(const DevTerm &t, uint64_t row, bool &bad) {
    // one word per 64 rows: a wave's lanes read the same word (a broadcast)
    const bool valid = !t.valid || ((t.valid[row >> 6] >> (row & 63)) & 1);
    if (t.op == OP_FALSE) return false;
    if (t.op >= OP_IS_NULL) return (t.op == OP_IS_NOT_NULL) == valid;
    if (!valid) return false;  // a NULL row satisfies no comparison
    const uint8_t *p = t.col + row * t.ob;
    int c;
    switch (t.kind) {
    case FK_INT: c = cmp_int(load_int(p, t.ob), (int64_t)t.value); break;
    case FK_UINT: c = cmp_uint(load_uint(p, t.ob), t.value); break;
    case FK_FLOAT: c = cmp_float(t.ob == 4 ? (double)*(const float *)p : *(const double *)p, as_double(t.value)); break;
    default: c = cmp_string(t, p, bad); break;
    }
    return op_holds(t.op, c);
}

__global__ __launch_bounds__(256) void filter_kernel(const DevTerm *__restrict__ terms, uint32_t nterms,
                                                     uint32_t nrows, uint64_t *__restrict__ mask,
                                                     uint32_t *__restrict__ counts, uint32_t *__restrict__ err) {
    __shared__ uint32_t wave_cnt[4];
    const uint32_t v = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t cnt = 0;
    bool bad = false;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t word = 4 * w + k;
        const uint64_t row = (uint64_t)v * 1024 + 64 * word + lane;
        const bool ok = row < nrows;
        bool res = ok, acc = false;
        for (uint32_t i = 0; i < nterms; ++i) {
            const DevTerm &t = terms[i];
            acc = acc || (ok && eval_term(t, row, bad));
            if (t.end_clause) {
                res = res && acc;
                acc = false;
            }
        }
        const uint64_t b = __ballot(res);
        if (lane == 0) mask[(size_t)v * 16 + word] = b;
        cnt += (uint32_t)__popcll(b);
    }
    if (lane == 0) wave_cnt[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) counts[v] = wave_cnt[0] + wave_cnt[1] + wave_cnt[2] + wave_cnt[3];
    if (__ballot(bad) && lane == 0) atomicOr(err, KERR_FILTER_STR);
}

__device__ __forceinline__ void copy_value(const uint8_t *src, uint8_t *dst, uint32_t ob) {
    switch (ob) {
    case 1: *dst = *src; break;
    case 2: *(uint16_t *)dst = *(const uint16_t *)src; break;
    case 4: *(uint32_t *)dst = *(const uint32_t *)src; break;
    case 8: *(uint64_t *)dst = *(const uint64_t *)src; break;
    default: *(v4u *)dst = *(const v4u *)src; break;
    }
}

__global__ __launch_bounds__(256) void compact_kernel(const DevOut *__restrict__ outs, uint32_t nouts,
                                                      const uint64_t *__restrict__ mask,
                                                      const uint32_t *__restrict__ counts, uint32_t rg_rows,
                                                      uint32_t *__restrict__ sel) {
    const uint32_t v = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // selected rows of the batch's earlier vectors (<= 512 counts per batch)
    uint32_t base = 0;
    for (uint32_t k = lane; k < v; k += 64) base += counts[k];
    base = wave_sum(base);
    const uint64_t mw = lane < 16 ? mask[(size_t)v * 16 + lane] : 0;
    uint32_t pre = 0;
    for (uint32_t i = 0; i < 4 * w; ++i) pre += (uint32_t)__popcll(readlane64(mw, i));
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t word = 4 * w + k;
        const uint64_t b = readlane64(mw, word);
        if (b == 0) continue;
        if ((b >> lane) & 1) {
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0));
            const uint64_t row = (uint64_t)v * 1024 + 64 * word + lane;
            const uint64_t dest = base + pre + rank;
            for (uint32_t o = 0; o < nouts; ++o) {
                const DevOut &d = outs[o];
                copy_value(d.src + row * d.ob, d.dst + dest * d.ob, d.ob);
            }
            if (sel) sel[dest] = (uint32_t)(row % rg_rows);
        }
        pre += (uint32_t)__popcll(b);
    }
}

// one 1024-row tile of one narrowed column per block, 4 rows per thread
__global__ __launch_bounds__(256) void narrow_kernel(const DevNarrow *__restrict__ cols, uint32_t nrows,
                                                     uint32_t rg_rows, uint32_t *__restrict__ err) {
    const DevNarrow c = cols[blockIdx.y];
    bool bad = false;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t row = (uint64_t)blockIdx.x * 1024 + k * 256 + threadIdx.x;
        if (row >= nrows) break;
        const uint8_t *p = c.src + row * c.ob;
        // (a string_t record, ob 16, narrows its 4-byte length word)
        const uint32_t vb = c.ob == 16 ? 4u : c.ob;
        const uint64_t v = c.sign ? (uint64_t)load_int(p, vb) : load_uint(p, vb);
        const uint64_t d = v - c.base[row / rg_rows];
        // the difference must fit nw bytes: the zone maps bound a sound file's
        // values (NULL placeholders included), so a value outside them is
        // reported, never truncated into a wrong integer
        bad |= (d >> (8 * c.nw)) != 0;
        uint8_t *q = c.dst + row * c.nw;
        switch (c.nw) {
        case 1: *q = (uint8_t)d; break;
        case 2: *(uint16_t *)q = (uint16_t)d; break;
        default: *(uint32_t *)q = (uint32_t)d; break;
        }
    }
    if (__ballot(bad) != 0 && __lane_id() == 0) atomicOr(err, KERR_NARROW);
}

// 64 KiB pieces of the copies over a grid-stride block loop: 256 lanes x 16 B
// per iteration (a 4 KiB contiguous write burst per block), the copy's last
// (bytes mod 16) bytes one per lane
__global__ __launch_bounds__(256) void host_copy_kernel(const HostCopyList l) {
    const uint32_t total = l.first[l.n];
    uint32_t i = 0;
    for (uint32_t p = blockIdx.x; p < total; p += gridDim.x) {
        while (p >= l.first[i + 1]) ++i;  // pieces ascend with p
        const HostCopy c = l.c[i];
        const uint64_t base = (uint64_t)(p - l.first[i]) * kHostCopyPiece;
        const uint32_t len = (uint32_t)min<uint64_t>(kHostCopyPiece, c.bytes - base);
        const v4u *__restrict__ s = (const v4u *)(c.src + base);
        v4u *__restrict__ d = (v4u *)(c.dst + base);
        const uint32_t nv = len / 16;
#pragma unroll 4
        for (uint32_t v = threadIdx.x; v < nv; v += 256) d[v] = s[v];
        for (uint32_t b = nv * 16 + threadIdx.x; b < len; b += 256) c.dst[base + b] = c.src[base + b];
    }
}

}  // namespace

hipError_t launch_host_copy(const HostCopy *copies, uint32_t n, hipStream_t stream) {
    const int cus = device_cus();
    uint32_t k = 0;
    while (k < n) {
        HostCopyList l;
        memset(&l, 0, sizeof(l));
        uint64_t pieces = 0;
        for (; k < n && l.n < kHostCopyMax; ++k) {
            if (!copies[k].bytes) continue;
            if (((uintptr_t)copies[k].src | (uintptr_t)copies[k].dst) & 15) return hipErrorInvalidValue;
            l.first[l.n] = (uint32_t)pieces;
            l.c[l.n++] = copies[k];
            pieces += (copies[k].bytes + kHostCopyPiece - 1) / kHostCopyPiece;
            if (pieces >= (1ull << 31)) return hipErrorInvalidValue;
        }
        if (!l.n) continue;
        l.first[l.n] = (uint32_t)pieces;
        // 2 blocks per CU keep the link busy (256-4096 blocks measured equal)
        const uint32_t grid = (uint32_t)std::min<uint64_t>(pieces, 2ull * cus);
        hipLaunchKernelGGL(host_copy_kernel, dim3(grid), dim3(256), 0, stream, l);
        if (const hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
}

hipError_t launch_narrow(const DevNarrow *d_cols, uint32_t ncols, uint32_t nrows, uint32_t rg_rows,
                         uint32_t *d_err, hipStream_t stream) {
    if (ncols == 0 || nrows == 0 || rg_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(narrow_kernel, dim3((nrows + 1023) / 1024, ncols), dim3(256), 0, stream, d_cols, nrows,
                       rg_rows, d_err);
    return hipGetLastError();
}

hipError_t launch_filter(const DevTerm *d_terms, uint32_t nterms, uint32_t nrows, uint64_t *d_mask,
                         uint32_t *d_counts, uint32_t *d_err, hipStream_t stream) {
    const uint32_t nvec = (nrows + 1023) / 1024;
    if (nvec == 0) return hipSuccess;
    hipLaunchKernelGGL(filter_kernel, dim3(nvec), dim3(256), 0, stream, d_terms, nterms, nrows, d_mask, d_counts,
                       d_err);
    return hipGetLastError();
}

hipError_t launch_compact(const DevOut *d_outs, uint32_t nouts, const uint64_t *d_mask, const uint32_t *d_counts,
                          uint32_t nrows, uint32_t rg_rows, uint32_t *sel, hipStream_t stream) {
    const uint32_t nvec = (nrows + 1023) / 1024;
    if (nvec == 0 || rg_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(compact_kernel, dim3(nvec), dim3(256), 0, stream, d_outs, nouts, d_mask, d_counts, rg_rows,
                       sel);
    return hipGetLastError();
}

}  // namespace fls
