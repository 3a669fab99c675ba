// flsfast.cpp -- FastLanes-shaped CPU decoder: the CPU BASELINE of bench.py.
//
// TEST / BENCH INFRASTRUCTURE ONLY (like flsref.c): bench.py's cpu_baseline
// leg times it, tests/test_flsfast.py checks it against the oracle
// (oracle/flsref.c).  The product (duckdb-fastlane_amd/) never links it.
//
// What it stands in for: the reference's CPU decode, cwida/FastLanes'
// RowgroupReader::materialize() (reference src/fastlanes_facade.cpp:48),
// built by vcpkg as a static library with the project's default flags and no
// -march=native (vcpkg_ports/fastlanes/portfile.cmake:19-45,50-61).  That
// library is absent here (empty submodule), so this restates
// the SHAPE of its generated kernels, which is what makes FastLanes fast on a
// CPU: one function per (T, W) in which the loop runs over the 1024/T lanes
// (independent, contiguous words -> the compiler vectorises it) and the T rows
// are fully unrolled with compile-time shifts and masks, the FOR base / delta
// / dictionary step fused into the same pass (Afroozeh & Boncz, "The FastLanes
// Compression Layout", VLDB 2023, sections 3-5).  Unlike flsref.c (the
// per-value checker) it has no division, modulo, type switch or straddle
// branch per value.
//
// DELTA: position p = r*(1024/T) + c of the interleaved layout holds tuple
// tau(p) (flsref_tau).  For every T, lane c holds one delta chain and row r is
// step k(r) of it, with k(r) = tau(r*L)/16 independent of the lane, and lane
// group g (lanes 16g..16g+15) holds chain block blk(g) = tau(16g)/(16T); so the
// fused loop walks k = 0..T-1 (row r(k)), adds each lane's unpacked delta to
// its running sum and stores it at tuple blk(g)*16T + (c mod 16) + 16k, the
// same value flsref.c's delta_vector computes.
//
// Output: DuckDB physical layouts, as the GPU path writes them: integers in
// the column's width, DATE int32, DECIMAL int64, FLOAT/DOUBLE, VARCHAR 16-byte
// string_t (inline <= 12 bytes, else 4-byte prefix + pointer into the file
// image (DICT) or the column's decoded FSST heap).  Row groups are spread over
// threads (dynamic), each thread decoding every column of its row group.
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <utility>
#include <vector>

namespace {

constexpr uint32_t kVec = 1024;
constexpr uint32_t FL_ORDER[8] = {0, 4, 2, 6, 1, 5, 3, 7};
enum { ENC_FFOR = 1, ENC_DELTA = 2, ENC_DICT = 3, ENC_RLE = 4, ENC_ALP = 5, ENC_FSST = 7 };
enum { TY_BOOLEAN = 9, TY_FLOAT = 12, TY_DOUBLE = 13, TY_VARCHAR = 20, TY_BLOB = 21 };

constexpr uint32_t tau(uint32_t p) { return 128u * FL_ORDER[(p >> 4) & 7] + 16u * ((p >> 7) & 7) + (p & 15); }

template <class T>
inline T ld(const uint8_t *p) {
    T v;
    memcpy(&v, p, sizeof(T));
    return v;
}

#define FLS_INLINE inline __attribute__((always_inline))

template <uint32_t R, uint32_t N, class F>
FLS_INLINE void static_for(F &&f) {
    if constexpr (R < N) {
        f(std::integral_constant<uint32_t, R>{});
        static_for<R + 1, N>(f);
    }
}

// value of row R of lane i (words in[k*L + i]), compile-time W
template <class T, uint32_t W, uint32_t R>
FLS_INLINE T row_value(const T *__restrict in, uint32_t i) {
    constexpr uint32_t B = sizeof(T) * 8, L = kVec / B;
    if constexpr (W == 0) {
        return 0;
    } else {
        constexpr uint32_t bit = R * W, k = bit / B, s = bit % B;
        constexpr T M = W >= B ? (T)~T(0) : (T)((T(1) << W) - 1);
        if constexpr (s + W <= B) {
            return (T)((T)(in[k * L + i] >> s) & M);
        } else {
            return (T)(((T)(in[k * L + i] >> s) | (T)(in[(k + 1) * L + i] << (B - s))) & M);
        }
    }
}

// FFOR: out[r*L + i] = base + unpack  (lanes vectorised, rows unrolled)
template <class T, uint32_t W>
void unffor(const T *__restrict in, T *__restrict out, T base) {
    constexpr uint32_t B = sizeof(T) * 8, L = kVec / B;
    for (uint32_t i = 0; i < L; ++i)
        static_for<0, B>([&](auto r) { out[r * L + i] = (T)(row_value<T, W, r>(in, i) + base); });
}

// DELTA over the unified transposed layout (see the header comment)
template <class T>
constexpr uint32_t row_of_step(uint32_t k) {  // r with k(r) == k
    constexpr uint32_t B = sizeof(T) * 8, L = kVec / B;
    for (uint32_t r = 0; r < B; ++r)
        if (tau(r * L) / 16 == k) return r;
    return 0;
}
template <class T, uint32_t W>
void undelta(const T *__restrict in, T *__restrict out, T for_base, const T *__restrict bases) {
    constexpr uint32_t B = sizeof(T) * 8, L = kVec / B;
    T acc[L];
    for (uint32_t g = 0; g < L / 16; ++g) {
        const uint32_t blk = tau(16 * g) / (16 * B);
        for (uint32_t l = 0; l < 16; ++l) acc[16 * g + l] = bases[blk * 16 + l];
    }
    static_for<0, B>([&](auto k) {
        constexpr uint32_t r = row_of_step<T>(k);
        for (uint32_t i = 0; i < L; ++i) {
            acc[i] = (T)(acc[i] + (T)(row_value<T, W, r>(in, i) + for_base));
            const uint32_t blk = tau(16 * (i / 16)) / (16 * B);
            out[blk * 16 * B + (i % 16) + 16 * k] = acc[i];
        }
    });
}

template <class T>
using UnfforFn = void (*)(const T *, T *, T);
template <class T>
using UndeltaFn = void (*)(const T *, T *, T, const T *);
template <class T, size_t... W>
constexpr auto unffor_table(std::index_sequence<W...>) {
    return std::vector<UnfforFn<T>>{&unffor<T, (uint32_t)W>...};
}
template <class T, size_t... W>
constexpr auto undelta_table(std::index_sequence<W...>) {
    return std::vector<UndeltaFn<T>>{&undelta<T, (uint32_t)W>...};
}
template <class T>
const std::vector<UnfforFn<T>> &unffor_fns() {
    static const auto t = unffor_table<T>(std::make_index_sequence<sizeof(T) * 8 + 1>{});
    return t;
}
template <class T>
const std::vector<UndeltaFn<T>> &undelta_fns() {
    static const auto t = undelta_table<T>(std::make_index_sequence<sizeof(T) * 8 + 1>{});
    return t;
}

// ---- container (FLSAMD01) --------------------------
struct Col {
    uint8_t type;
    uint32_t ob;  // output bytes per value
};
struct File {
    const uint8_t *img = nullptr;
    uint64_t len = 0, nrows = 0;
    uint32_t ncols = 0, nrg = 0;
    std::vector<Col> cols;
    std::vector<uint32_t> rg_rows;
    std::vector<uint64_t> rg_first;   // first row of each row group
    std::vector<uint64_t> chunk_off;  // [rg * ncols + c]
};

uint32_t out_bytes(uint8_t t) {
    switch (t) {
    case 1: case 5: case TY_BOOLEAN: return 1;
    case 2: case 6: return 2;
    case 3: case 7: case 10: case TY_FLOAT: return 4;
    case 4: case 8: case 11: case TY_DOUBLE: return 8;
    case TY_VARCHAR: case TY_BLOB: return 16;
    default: return 0;
    }
}

bool open_file(const uint8_t *img, uint64_t len, File &f) {
    if (len < 32 || memcmp(img, "FLSAMD01", 8) != 0 || memcmp(img + len - 4, "FLSF", 4) != 0) return false;
    const uint64_t foff = ld<uint64_t>(img + len - 16);
    const uint8_t *p = img + foff;
    f.img = img;
    f.len = len;
    f.ncols = ld<uint32_t>(p + 4);
    f.nrows = ld<uint64_t>(p + 8);
    f.nrg = ld<uint32_t>(p + 16);
    p += 32;
    for (uint32_t c = 0; c < f.ncols; ++c) {
        f.cols.push_back({p[0], out_bytes(p[0])});
        p += 6 + ld<uint16_t>(p + 4);
    }
    uint64_t row = 0;
    for (uint32_t r = 0; r < f.nrg; ++r) {
        f.rg_rows.push_back(ld<uint32_t>(p));
        f.rg_first.push_back(row);
        row += f.rg_rows.back();
        for (uint32_t c = 0; c < f.ncols; ++c) f.chunk_off.push_back(ld<uint64_t>(p + 4 + 16 * c));
        p += 4 + 16ull * f.ncols;
    }
    return true;
}

// 16-byte duckdb::string_t
FLS_INLINE void make_string_t(uint8_t *dst, const uint8_t *s, uint32_t n) {
    uint8_t rec[16] = {0};
    memcpy(rec, &n, 4);
    if (n <= 12) {
        memcpy(rec + 4, s, n);
    } else {
        memcpy(rec + 4, s, 4);
        const uint64_t ptr = (uint64_t)(uintptr_t)s;
        memcpy(rec + 8, &ptr, 8);
    }
    memcpy(dst, rec, 16);
}

struct Scratch {
    alignas(64) uint64_t u64[kVec];
    alignas(64) uint32_t u32[kVec];
    alignas(64) uint16_t u16[kVec];
    std::vector<uint8_t> strtab;  // DICT string_t table of the chunk
};

template <class T>
FLS_INLINE void ffor_vec(const uint8_t *packed, uint32_t W, uint64_t base, uint32_t n, uint8_t *out, Scratch &s) {
    if (n == kVec) {
        unffor_fns<T>()[W]((const T *)packed, (T *)out, (T)base);
    } else {
        T *tmp = (T *)s.u64;
        unffor_fns<T>()[W]((const T *)packed, tmp, (T)base);
        memcpy(out, tmp, (size_t)n * sizeof(T));
    }
}
template <class T>
FLS_INLINE void delta_vec(const uint8_t *packed, uint32_t W, uint64_t base, const uint8_t *bases, uint32_t n,
                          uint8_t *out, Scratch &s) {
    if (n == kVec) {
        undelta_fns<T>()[W]((const T *)packed, (T *)out, (T)base, (const T *)bases);
    } else {
        T *tmp = (T *)s.u64;
        undelta_fns<T>()[W]((const T *)packed, tmp, (T)base, (const T *)bases);
        memcpy(out, tmp, (size_t)n * sizeof(T));
    }
}

template <class V>
FLS_INLINE void gather(const uint32_t *codes, const V *dict, uint32_t nd, uint32_t n, V *out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = dict[codes[i] < nd ? codes[i] : 0];
}
template <class V>
FLS_INLINE void gather16(const uint16_t *idx, const V *runs, uint32_t nr, uint32_t n, V *out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = runs[idx[i] < nr ? idx[i] : 0];
}

const double kF10D[19] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18};
const double kIF10D[19] = {1e-0, 1e-1, 1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7, 1e-8, 1e-9, 1e-10,
                           1e-11, 1e-12, 1e-13, 1e-14, 1e-15, 1e-16, 1e-17, 1e-18};
const float kF10F[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
const float kIF10F[11] = {1e-0f, 1e-1f, 1e-2f, 1e-3f, 1e-4f, 1e-5f, 1e-6f, 1e-7f, 1e-8f, 1e-9f, 1e-10f};

// FSST: the classic decoder loop (8-byte symbol store, advance by its
// length); the heap has >= 8 bytes of slack after every chunk
FLS_INLINE uint8_t *fsst_expand(const uint8_t *table, const uint8_t *c, const uint8_t *end, uint8_t *o) {
    const uint8_t *lens = table + 8 * 256;
    while (c < end) {
        const uint32_t code = *c++;
        if (code != 255) {
            memcpy(o, table + 8 * code, 8);
            o += lens[code];
        } else {
            *o++ = *c++;
        }
    }
    return o;
}

// one chunk (column c of row group rg) into out (+ heap for FSST)
bool decode_chunk(const File &f, uint32_t rg, uint32_t c, uint8_t *out, uint8_t *heap, Scratch &s) {
    const uint8_t *ch = f.img + f.chunk_off[(size_t)rg * f.ncols + c];
    const uint32_t enc = ch[4], T = ch[5], vbits = ch[6], is_str = ch[7];
    const uint32_t nvec = ld<uint32_t>(ch + 8);
    const uint8_t *meta = ch + ld<uint64_t>(ch + 16);
    const uint8_t *packed = ch + ld<uint64_t>(ch + 24);
    const uint8_t *aux = ch + ld<uint64_t>(ch + 32);
    const uint32_t dict_count = ld<uint32_t>(ch + 48);
    const uint32_t ob = f.cols[c].ob;
    if (enc == ENC_DICT && is_str) {  // per-chunk string_t table, gathered below
        s.strtab.resize(16ull * dict_count);
        const uint8_t *bytes = aux + 4ull * (dict_count + 1);
        for (uint32_t k = 0; k < dict_count; ++k) {
            const uint32_t b0 = ld<uint32_t>(aux + 4ull * k), b1 = ld<uint32_t>(aux + 4ull * (k + 1));
            make_string_t(s.strtab.data() + 16ull * k, bytes + b0, b1 - b0);
        }
    }
    for (uint32_t v = 0; v < nvec; ++v) {
        const uint8_t *m = meta + 32ull * v;
        const uint8_t *pk = packed + ld<uint64_t>(m);
        const uint64_t base = ld<uint64_t>(m + 8);
        const uint8_t *va = aux + ld<uint64_t>(m + 16);
        const uint32_t n = ld<uint16_t>(m + 24), W = m[26], acount = ld<uint32_t>(m + 28);
        uint8_t *o = out + (size_t)v * kVec * ob;
        switch (enc) {
        case ENC_FFOR:
            switch (T) {
            case 8: ffor_vec<uint8_t>(pk, W, base, n, o, s); break;
            case 16: ffor_vec<uint16_t>(pk, W, base, n, o, s); break;
            case 32: ffor_vec<uint32_t>(pk, W, base, n, o, s); break;
            default: ffor_vec<uint64_t>(pk, W, base, n, o, s); break;
            }
            break;
        case ENC_DELTA:
            switch (T) {
            case 8: delta_vec<uint8_t>(pk, W, base, va, n, o, s); break;
            case 16: delta_vec<uint16_t>(pk, W, base, va, n, o, s); break;
            case 32: delta_vec<uint32_t>(pk, W, base, va, n, o, s); break;
            default: delta_vec<uint64_t>(pk, W, base, va, n, o, s); break;
            }
            break;
        case ENC_DICT: {
            unffor_fns<uint32_t>()[W]((const uint32_t *)pk, s.u32, (uint32_t)base);
            if (is_str) {
                gather(s.u32, (const __uint128_t *)s.strtab.data(), dict_count, n, (__uint128_t *)o);
            } else {
                switch (vbits) {
                case 8: gather(s.u32, (const uint8_t *)aux, dict_count, n, (uint8_t *)o); break;
                case 16: gather(s.u32, (const uint16_t *)aux, dict_count, n, (uint16_t *)o); break;
                case 32: gather(s.u32, (const uint32_t *)aux, dict_count, n, (uint32_t *)o); break;
                default: gather(s.u32, (const uint64_t *)aux, dict_count, n, (uint64_t *)o); break;
                }
            }
        } break;
        case ENC_RLE: {
            undelta_fns<uint16_t>()[W]((const uint16_t *)pk, s.u16, (uint16_t)base, (const uint16_t *)va);
            const uint8_t *runs = va + 128;
            switch (vbits) {
            case 8: gather16(s.u16, runs, acount, n, o); break;
            case 16: gather16(s.u16, (const uint16_t *)runs, acount, n, (uint16_t *)o); break;
            case 32: gather16(s.u16, (const uint32_t *)runs, acount, n, (uint32_t *)o); break;
            default: gather16(s.u16, (const uint64_t *)runs, acount, n, (uint64_t *)o); break;
            }
        } break;
        case ENC_ALP: {
            const uint32_t exc = acount & 0xFFFF, e = (acount >> 16) & 0xFF, fct = acount >> 24;
            if (T == 64) {
                unffor_fns<uint64_t>()[W]((const uint64_t *)pk, s.u64, base);
                double *od = (double *)o;
                const double a = kF10D[fct], b = kIF10D[e];
                for (uint32_t i = 0; i < n; ++i) od[i] = (double)(int64_t)s.u64[i] * a * b;
            } else {
                unffor_fns<uint32_t>()[W]((const uint32_t *)pk, s.u32, (uint32_t)base);
                float *of = (float *)o;
                const float a = kF10F[fct], b = kIF10F[e];
                for (uint32_t i = 0; i < n; ++i) of[i] = (float)(int32_t)s.u32[i] * a * b;
            }
            const uint8_t *val = va + ((2ull * exc + 15) & ~15ull);
            for (uint32_t k = 0; k < exc; ++k) {
                const uint32_t p = ld<uint16_t>(va + 2ull * k);
                if (p < n) memcpy(o + (size_t)(T / 8) * p, val + (size_t)(T / 8) * k, T / 8);
            }
        } break;
        case ENC_FSST: {
            // string lengths, then the vector's code stream in one pass (every
            // string is compressed on its own, so no escape spans two strings)
            unffor_fns<uint32_t>()[W]((const uint32_t *)pk, s.u32, (uint32_t)base);
            const uint32_t heap_off = ld<uint32_t>(va), clen = ld<uint32_t>(va + 4), cw = ld<uint32_t>(va + 12);
            const uint8_t *cs = va + 16 + 128ull * cw;
            uint8_t *h = heap + heap_off;
            fsst_expand(aux, cs, cs + clen, h);
            uint8_t *rec = o;
            for (uint32_t i = 0; i < n; ++i) {
                make_string_t(rec + 16ull * i, h, s.u32[i]);
                h += s.u32[i];
            }
        } break;
        default: return false;
        }
    }
    return true;
}

}  // namespace

extern "C" {

// Per column: out (rows x out-bytes, DuckDB layout) and, for FSST VARCHAR
// columns, heap (flsfast_heap_bytes).  Decodes row groups [rg0, rg1) (rows
// placed from the first of them) with nthreads threads; returns the values
// decoded (rows x columns) or -1.
int64_t flsfast_decode(const void *img, uint64_t len, uint32_t rg0, uint32_t rg1, int nthreads, void *const *outs,
                       void *const *heaps) {
    File f;
    if (!open_file((const uint8_t *)img, len, f) || rg1 > f.nrg || rg0 > rg1) return -1;
    // heap offset of each (rg, col) FSST chunk, chunks 16 bytes apart (slack
    // for the decoder's 8-byte symbol stores)
    std::vector<uint64_t> hoff((size_t)(rg1 - rg0) * f.ncols, 0);
    for (uint32_t c = 0; c < f.ncols; ++c) {
        uint64_t acc = 0;
        for (uint32_t r = rg0; r < rg1; ++r) {
            const uint8_t *ch = f.img + f.chunk_off[(size_t)r * f.ncols + c];
            hoff[(size_t)(r - rg0) * f.ncols + c] = acc;
            if (ch[4] == ENC_FSST) acc += ((ld<uint64_t>(ch + 56) + 15) & ~15ull) + 16;
        }
    }
    std::atomic<uint32_t> next{rg0};
    std::atomic<bool> ok{true};
    const uint64_t row0 = f.rg_first[rg0];
    auto work = [&]() {
        Scratch s;
        for (uint32_t r; (r = next.fetch_add(1)) < rg1;)
            for (uint32_t c = 0; c < f.ncols; ++c) {
                uint8_t *o = (uint8_t *)outs[c] + (f.rg_first[r] - row0) * f.cols[c].ob;
                uint8_t *h = heaps && heaps[c] ? (uint8_t *)heaps[c] + hoff[(size_t)(r - rg0) * f.ncols + c] : nullptr;
                if (!decode_chunk(f, r, c, o, h, s)) ok = false;
            }
    };
    if (nthreads < 1) nthreads = 1;
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    if (!ok) return -1;
    const uint64_t rows = f.rg_first[rg1 - 1] + f.rg_rows[rg1 - 1] - row0;
    return rg1 > rg0 ? (int64_t)(rows * f.ncols) : 0;
}

// Bytes of column col's FSST heap for row groups [rg0, rg1) (0 if none).
uint64_t flsfast_heap_bytes(const void *img, uint64_t len, uint32_t rg0, uint32_t rg1, uint32_t col) {
    File f;
    if (!open_file((const uint8_t *)img, len, f) || rg1 > f.nrg || col >= f.ncols) return 0;
    uint64_t acc = 0;
    for (uint32_t r = rg0; r < rg1; ++r) {
        const uint8_t *ch = f.img + f.chunk_off[(size_t)r * f.ncols + col];
        if (ch[4] == ENC_FSST) acc += ((ld<uint64_t>(ch + 56) + 15) & ~15ull) + 16;
    }
    return acc;
}

}  // extern "C"
