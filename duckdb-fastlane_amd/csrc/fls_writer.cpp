// fls_writer.cpp -- CPU FastLanes encoder + file assembler + seeded workloads.
//
// Encodes row groups of 65,536 rows (src/writer/write_fastlane_stream.cpp:21-24)
// into 1024-value vectors with the FastLanes codecs the decode path supports:
// FFOR, unified-transposed DELTA, DICT (int and string) and FastLanes-RLE.
// This is the write path the reference only stubs
// (src/writer/write_fastlane.cpp:227, src/include/fastlanes_facade.hpp:39-43)
// and the producer of every benchmark / test input (fls_gen.hpp).
#include <algorithm>
#include <cstddef>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/flsgpu.h"
#include "../../include/flswriter.h"
#include "fls_alp.hpp"
#include "fls_common.hpp"
#include "fls_config.hpp"
#include "fls_encode.hpp"
#include "fls_format.hpp"
#include "fls_gen.hpp"
#include "fls_pinned.hpp"
#include "fls_text.hpp"

namespace fls {

std::string &last_error() {
    static thread_local std::string e;
    return e;
}

namespace {

constexpr uint8_t kFLOrder[8] = {0, 4, 2, 6, 1, 5, 3, 7};

inline uint64_t tmask(int T) { return T >= 64 ? ~0ull : ((1ull << T) - 1ull); }
inline int bitlen(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }
inline int64_t sext(uint64_t v, int T) {
    if (T >= 64) return (int64_t)v;
    const uint64_t sign = 1ull << (T - 1);
    v &= tmask(T);
    return (int64_t)((v ^ sign) - sign);
}
// transposed position p -> original tuple index
inline uint32_t tau(uint32_t p) { return 128u * kFLOrder[(p >> 4) & 7] + 16u * (p >> 7) + (p & 15); }

struct TauTable {
    uint16_t t[1024];
    TauTable() { for (uint32_t p = 0; p < 1024; ++p) t[p] = (uint16_t)tau(p); }
};
const TauTable &tau_table() { static TauTable tt; return tt; }

void put_word(uint8_t *dst, int T, uint64_t idx, uint64_t v) {
    switch (T) {
    case 8: dst[idx] = (uint8_t)v; break;
    case 16: { uint16_t x = (uint16_t)v; memcpy(dst + 2 * idx, &x, 2); } break;
    case 32: { uint32_t x = (uint32_t)v; memcpy(dst + 4 * idx, &x, 4); } break;
    default: memcpy(dst + 8 * idx, &v, 8); break;
    }
}

// Interleaved bit-packing of 1024 values in position order (lane-major
// accumulation; lane L's k-th word goes to word index k*(1024/T)+L).
void pack(int T, int W, const uint64_t *vals, uint8_t *dst) {
    if (W == 0) return;
    const int lanes = 1024 / T;
    const uint64_t wm = tmask(W), tm = tmask(T);
    for (int lane = 0; lane < lanes; ++lane) {
        unsigned __int128 acc = 0;
        int nbits = 0, k = 0;
        for (int row = 0; row < T; ++row) {
            acc |= (unsigned __int128)(vals[row * lanes + lane] & wm) << nbits;
            nbits += W;
            while (nbits >= T) {
                put_word(dst, T, (uint64_t)k * lanes + lane, (uint64_t)acc & tm);
                acc >>= T;
                nbits -= T;
                ++k;
            }
        }
    }
}

// FFOR over 1024 unsigned T-bit values (already in position order).
// Returns bw, sets base; u receives value - base (mod 2^T).
int ffor_prepare(int T, const uint64_t *v, int64_t &base, uint64_t *u) {
    int64_t mn = sext(v[0], T);
    for (int i = 1; i < 1024; ++i) mn = std::min(mn, sext(v[i], T));
    const uint64_t tm = tmask(T);
    uint64_t mx = 0;
    for (int i = 0; i < 1024; ++i) {
        u[i] = (v[i] - (uint64_t)mn) & tm;
        mx |= u[i];
    }
    base = mn;
    return bitlen(mx);
}

struct VecOut {
    VecMeta meta;
    std::vector<uint8_t> packed;
    std::vector<uint8_t> aux;  // per-vector aux (DELTA bases, RLE bases + runs)
};

void align_to(std::vector<uint8_t> &b, size_t a) {
    while (b.size() % a) b.push_back(0);
}

// Assemble one chunk from encoded vectors + chunk-level aux (dictionary).
std::vector<uint8_t> assemble_chunk(uint8_t enc, uint8_t T, uint8_t vbits, bool is_str,
                                    uint32_t nvals, std::vector<VecOut> &vecs,
                                    const std::vector<uint8_t> &chunk_aux, uint32_t dict_count,
                                    uint64_t reserved1 = 0, uint32_t reserved0 = 0) {
    ChunkHeader h{};
    h.magic = kChunkMagic;
    h.enc = enc;
    h.T = T;
    h.vbits = vbits;
    h.is_str = is_str ? 1 : 0;
    h.nvec = (uint32_t)vecs.size();
    h.nvals = nvals;
    h.meta_off = sizeof(ChunkHeader);
    size_t packed_total = 0;
    for (auto &v : vecs) packed_total += v.packed.size();
    size_t off = h.meta_off + sizeof(VecMeta) * vecs.size();
    off = (off + 15) & ~size_t(15);
    h.packed_off = off;
    off += packed_total;
    off = (off + 15) & ~size_t(15);
    h.aux_off = off;
    // aux: chunk-level dictionary first, then per-vector aux (8-B aligned)
    std::vector<uint8_t> aux = chunk_aux;
    align_to(aux, 16);
    uint64_t poff = 0;
    for (auto &v : vecs) {
        v.meta.packed_off = poff;
        poff += v.packed.size();
        if (!v.aux.empty()) {
            align_to(aux, 16);
            v.meta.aux_off = aux.size();
            aux.insert(aux.end(), v.aux.begin(), v.aux.end());
        }
    }
    h.aux_len = aux.size();
    h.dict_count = dict_count;
    h.reserved0 = reserved0;
    h.reserved1 = reserved1;
    size_t total = h.aux_off + aux.size();
    total = (total + kChunkAlign - 1) & ~size_t(kChunkAlign - 1);
    std::vector<uint8_t> out(total, 0);
    memcpy(out.data(), &h, sizeof(h));
    for (size_t i = 0; i < vecs.size(); ++i) memcpy(out.data() + h.meta_off + 32 * i, &vecs[i].meta, 32);
    size_t p = h.packed_off;
    for (auto &v : vecs) {
        if (!v.packed.empty()) memcpy(out.data() + p, v.packed.data(), v.packed.size());
        p += v.packed.size();
    }
    if (!aux.empty()) memcpy(out.data() + h.aux_off, aux.data(), aux.size());
    return out;
}

// load 1024 values of vector v (padding the tail with the last value)
void load_vec(const uint64_t *vals, uint32_t n, uint32_t v, uint64_t *out, uint32_t &vn) {
    const uint32_t b = v * 1024;
    vn = std::min<uint32_t>(1024, n - b);
    for (uint32_t i = 0; i < vn; ++i) out[i] = vals[b + i];
    for (uint32_t i = vn; i < 1024; ++i) out[i] = vals[b + vn - 1];
}

// ---- integer chunk encoders (vals: n values as unsigned T-bit in uint64) --

std::vector<uint8_t> enc_ffor(int T, const uint64_t *vals, uint32_t n) {
    const uint32_t nvec = (n + 1023) / 1024;
    std::vector<VecOut> vecs(nvec);
    uint64_t v[1024], u[1024];
    for (uint32_t k = 0; k < nvec; ++k) {
        uint32_t vn;
        load_vec(vals, n, k, v, vn);
        int64_t base;
        int W = ffor_prepare(T, v, base, u);
        VecOut &o = vecs[k];
        o.meta = VecMeta{};
        o.meta.for_base = base;
        o.meta.bw = (uint8_t)W;
        o.meta.nvals = (uint16_t)vn;
        o.packed.assign((size_t)128 * W, 0);
        pack(T, W, u, o.packed.data());
    }
    return assemble_chunk(ENC_FFOR, (uint8_t)T, (uint8_t)T, false, n, vecs, {}, 0);
}

// deltas of one vector in the unified transposed layout; bases (128 B) out
void delta_vector(int T, const uint64_t *v, uint64_t *pos_vals, uint8_t *bases) {
    const uint64_t tm = tmask(T);
    uint64_t d[1024];
    const int nchains = 1024 / T;
    for (int c = 0; c < nchains; ++c) {
        const int blk = c / 16, l = c % 16;
        const uint32_t i0 = (uint32_t)(blk * 16 * T + l);
        put_word(bases, T, (uint64_t)c, v[i0]);
        d[i0] = 0;
        for (int k = 1; k < T; ++k) {
            const uint32_t i = i0 + 16u * k;
            d[i] = (v[i] - v[i - 16]) & tm;
        }
    }
    const TauTable &tt = tau_table();
    for (uint32_t p = 0; p < 1024; ++p) pos_vals[p] = d[tt.t[p]];
}

std::vector<uint8_t> enc_delta(int T, const uint64_t *vals, uint32_t n) {
    const uint32_t nvec = (n + 1023) / 1024;
    std::vector<VecOut> vecs(nvec);
    uint64_t v[1024], pv[1024], u[1024];
    for (uint32_t k = 0; k < nvec; ++k) {
        uint32_t vn;
        load_vec(vals, n, k, v, vn);
        VecOut &o = vecs[k];
        o.aux.assign(128, 0);
        delta_vector(T, v, pv, o.aux.data());
        int64_t base;
        int W = ffor_prepare(T, pv, base, u);
        o.meta = VecMeta{};
        o.meta.for_base = base;
        o.meta.bw = (uint8_t)W;
        o.meta.nvals = (uint16_t)vn;
        o.packed.assign((size_t)128 * W, 0);
        pack(T, W, u, o.packed.data());
    }
    return assemble_chunk(ENC_DELTA, (uint8_t)T, (uint8_t)T, false, n, vecs, {}, 0);
}

// DICT codes (u32, T=32 packing) + chunk dictionary bytes
std::vector<uint8_t> enc_dict_codes(const uint32_t *codes, uint32_t n, uint8_t vbits, bool is_str,
                                    const std::vector<uint8_t> &dict, uint32_t dict_count) {
    const uint32_t nvec = (n + 1023) / 1024;
    std::vector<VecOut> vecs(nvec);
    uint64_t v[1024], u[1024];
    for (uint32_t k = 0; k < nvec; ++k) {
        const uint32_t b = k * 1024, vn = std::min<uint32_t>(1024, n - b);
        for (uint32_t i = 0; i < 1024; ++i) v[i] = codes[b + std::min(i, vn - 1)];
        int64_t base;
        int W = ffor_prepare(32, v, base, u);
        VecOut &o = vecs[k];
        o.meta = VecMeta{};
        o.meta.for_base = base;
        o.meta.bw = (uint8_t)W;
        o.meta.nvals = (uint16_t)vn;
        o.packed.assign((size_t)128 * W, 0);
        pack(32, W, u, o.packed.data());
    }
    return assemble_chunk(ENC_DICT, 32, vbits, is_str, n, vecs, dict, dict_count);
}

// Open-addressing set / map of 64-bit values (row-group sized: n <= 65,536),
// the distinct-value pass of ENC_AUTO's dictionary estimate and of DICT.
struct U64Table {
    std::vector<uint64_t> key;
    std::vector<uint32_t> val;  // UINT32_MAX = empty slot
    uint64_t mask;
    size_t count = 0;
    explicit U64Table(uint32_t n) {
        size_t cap = 16;
        while (cap < 2ull * n) cap <<= 1;
        key.resize(cap);
        val.assign(cap, UINT32_MAX);
        mask = cap - 1;
    }
    static uint64_t h(uint64_t x) {
        x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33;
        return x;
    }
    size_t slot(uint64_t x) const {
        size_t i = h(x) & mask;
        while (val[i] != UINT32_MAX && key[i] != x) i = (i + 1) & mask;
        return i;
    }
    void insert(uint64_t x) {
        const size_t i = slot(x);
        if (val[i] == UINT32_MAX) { key[i] = x; val[i] = 0; ++count; }
    }
};

std::vector<uint8_t> enc_dict_int(int T, const uint64_t *vals, uint32_t n) {
    U64Table tab(n);
    for (uint32_t i = 0; i < n; ++i) tab.insert(vals[i]);
    std::vector<uint64_t> uniq;
    uniq.reserve(tab.count);
    for (size_t i = 0; i <= tab.mask; ++i)
        if (tab.val[i] != UINT32_MAX) uniq.push_back(tab.key[i]);
    std::sort(uniq.begin(), uniq.end(), [T](uint64_t a, uint64_t b) { return sext(a, T) < sext(b, T); });
    for (uint32_t i = 0; i < uniq.size(); ++i) tab.val[tab.slot(uniq[i])] = i;
    std::vector<uint32_t> codes(n);
    for (uint32_t i = 0; i < n; ++i) codes[i] = tab.val[tab.slot(vals[i])];
    std::vector<uint8_t> dict((size_t)uniq.size() * (T / 8));
    for (size_t i = 0; i < uniq.size(); ++i) put_word(dict.data(), T, i, uniq[i]);
    return enc_dict_codes(codes.data(), n, (uint8_t)T, false, dict, (uint32_t)uniq.size());
}

std::vector<uint8_t> str_dict_bytes(const std::vector<std::string_view> &entries) {
    std::vector<uint8_t> d(4 * (entries.size() + 1));
    uint32_t off = 0;
    for (size_t i = 0; i < entries.size(); ++i) {
        memcpy(d.data() + 4 * i, &off, 4);
        off += (uint32_t)entries[i].size();
    }
    memcpy(d.data() + 4 * entries.size(), &off, 4);
    for (auto &e : entries) d.insert(d.end(), e.begin(), e.end());
    return d;
}

// Dictionary of a chunk's strings in first-appearance order plus the codes,
// one pass over the rows with an open-addressing table of (hash, entry)
// (a std::unordered_map<string_view> here cost 2 hash-map passes per row and
// bounded the ENC_AUTO writer at ~18 M rows/s on 16 threads).  Stops, and
// returns false, once more than `limit` distinct strings are seen.
struct StrDict {
    std::vector<std::string_view> entries;
    std::vector<uint32_t> codes;
    uint64_t entry_bytes = 0;  // sum of the entries' lengths
};
static inline uint64_t str_hash(const char *p, uint32_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
    }
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = (h ^ w) * 0xc4ceb9fe1a85ec53ull;
    return h ^ (h >> 29);
}
bool build_str_dict(const uint32_t *offs, const char *bytes, uint32_t n, uint32_t limit, StrDict &d) {
    size_t cap = 16;
    while (cap < 2ull * (std::min(limit, n) + 1)) cap <<= 1;
    // (hash high 32 bits << 32) | (entry + 1); 0 = empty.  Kept per thread:
    // fresh 100+ KiB vectors per chunk are mmap'd and page-faulted, and the
    // faults serialise the column threads
    thread_local std::vector<uint64_t> slot;
    slot.assign(cap, 0);
    const size_t mask = cap - 1;
    d.entries.clear();
    d.codes.resize(n);
    d.entry_bytes = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const char *p = bytes + offs[i];
        const uint32_t len = offs[i + 1] - offs[i];
        const uint64_t h = str_hash(p, len);
        const uint64_t tag = h >> 32 << 32;
        size_t k = (size_t)h & mask;
        for (;;) {
            const uint64_t e = slot[k];
            if (e == 0) {
                if (d.entries.size() >= limit) return false;
                d.entries.emplace_back(p, len);
                d.entry_bytes += len;
                slot[k] = tag | d.entries.size();
                d.codes[i] = (uint32_t)d.entries.size() - 1;
                break;
            }
            if ((e & ~0xFFFFFFFFull) == tag) {
                const std::string_view &sv = d.entries[(uint32_t)e - 1];
                if (sv.size() == len && memcmp(sv.data(), p, len) == 0) {
                    d.codes[i] = (uint32_t)e - 1;
                    break;
                }
            }
            k = (k + 1) & mask;
        }
    }
    return true;
}

std::vector<uint8_t> enc_dict_str(const StrDict &d, uint32_t n) {
    return enc_dict_codes(d.codes.data(), n, 0, true, str_dict_bytes(d.entries), (uint32_t)d.entries.size());
}
std::vector<uint8_t> enc_dict_str(const uint32_t *offs, const char *bytes, uint32_t n) {
    StrDict d;
    build_str_dict(offs, bytes, n, n, d);
    return enc_dict_str(d, n);
}

// ---- FSST (VARCHAR) ----------------------------------------------------------
// Boncz, Neumann, Leis, "FSST: Fast Random Access String Compression", VLDB
// 2020: a table of up to 255 symbols of 1..8 bytes; a string becomes byte codes
// (greedy longest match), code 255 escapes one literal byte.  The table is
// built from a sample in five rounds: compress the sample with the current
// table, count symbol and adjacent-pair occurrences, keep the 255 candidates
// (symbols, pair concatenations cut to 8 bytes, single bytes) of highest gain
// = count x length.  One table per chunk (row group), so chunks stay
// self-contained; the GPU decodes a vector's code stream code-parallel.

struct FsstTable {
    uint64_t sym[256] = {};
    uint8_t len[256] = {};
    int n = 0;
    std::vector<uint8_t> by_first[256];  // codes starting with a byte, longest first

    // the final table's codes of length >= 2 by their first two bytes (CSR,
    // each list longest first as in by_first) and its one-byte symbol per
    // byte: the compressor then tries the few symbols that share a position's
    // first two bytes instead of every symbol sharing its first byte (text
    // puts 50+ symbols behind ' ')
    std::vector<uint32_t> start2;       // 65536 + 1 offsets into codes2
    std::vector<uint8_t> codes2;
    int16_t one[256];

    void index() {
        for (auto &v : by_first) v.clear();
        for (int c = 0; c < n; ++c) by_first[sym[c] & 0xFF].push_back((uint8_t)c);
        for (auto &v : by_first)
            std::stable_sort(v.begin(), v.end(), [this](uint8_t a, uint8_t b) { return len[a] > len[b]; });
    }
    void index2() {
        start2.assign(65537, 0);
        for (int b = 0; b < 256; ++b) one[b] = -1;
        for (int b = 0; b < 256; ++b)
            for (uint8_t c : by_first[b]) {
                if (len[c] >= 2) start2[(sym[c] & 0xFFFF) + 1]++;
                else if (one[b] < 0) one[b] = c;  // the first one-byte symbol by_first would reach
            }
        for (uint32_t k = 0; k < 65536; ++k) start2[k + 1] += start2[k];
        codes2.assign(start2[65536], 0);
        std::vector<uint32_t> fill(start2.begin(), start2.end() - 1);
        for (int b = 0; b < 256; ++b)  // by_first order: longest first, then code order
            for (uint8_t c : by_first[b])
                if (len[c] >= 2) codes2[fill[sym[c] & 0xFFFF]++] = c;
    }
    // the same longest match as match(), through the two-byte index
    int match2(const uint8_t *p, size_t r) const {
        if (r >= 2) {
            uint64_t w = 0;
            if (r >= 8) memcpy(&w, p, 8);
            else memcpy(&w, p, r);
            const uint32_t k = (uint32_t)(w & 0xFFFF);
            for (uint32_t j = start2[k]; j < start2[k + 1]; ++j) {
                const uint8_t c = codes2[j];
                const uint32_t L = len[c];
                const uint64_t m = L >= 8 ? ~0ull : (1ull << (8 * L)) - 1;
                if (L <= r && ((w ^ sym[c]) & m) == 0) return c;
            }
        }
        return one[p[0]];
    }
    // the longest symbol matching at p (r bytes left), or -1: one 8-byte load
    // of the input and a masked compare per candidate (a symbol's bytes past
    // its length are zero) instead of a memcmp call each
    int match(const uint8_t *p, size_t r) const {
        uint64_t w = 0;
        if (r >= 8) memcpy(&w, p, 8);  // (a fixed-size copy is one load; a variable one is a call)
        else memcpy(&w, p, r);
        for (uint8_t c : by_first[p[0]]) {
            const uint32_t L = len[c];
            const uint64_t m = L >= 8 ? ~0ull : (1ull << (8 * L)) - 1;
            if (L <= r && ((w ^ sym[c]) & m) == 0) return c;
        }
        return -1;
    }
    void compress(const uint8_t *p, size_t n_, std::vector<uint8_t> &out) const {
        for (size_t i = 0; i < n_;) {
            const int c = match2(p + i, n_ - i);
            if (c >= 0) {
                out.push_back((uint8_t)c);
                i += len[c];
            } else {
                out.push_back((uint8_t)kFsstEscape);
                out.push_back(p[i]);
                ++i;
            }
        }
    }
};

FsstTable fsst_build(const uint32_t *offs, const char *bytes, uint32_t n) {
    // FLS_FSST_MAX_SYMBOLS (tests): a smaller table forces escapes
    const char *ms = getenv("FLS_FSST_MAX_SYMBOLS");
    const int max_symbols = ms ? std::max(0, std::min(255, atoi(ms))) : 255;
    // sample: whole strings at evenly spaced rows, about 16 KiB
    const char *se = getenv("FLS_FSST_SAMPLE");
    const uint64_t sample_bytes = se ? std::max(1024, atoi(se)) : 16384;
    const char *re = getenv("FLS_FSST_ROUNDS");
    const int rounds = re ? std::max(1, atoi(re)) : 5;
    const char *ml = getenv("FLS_FSST_MAX_LEN");
    // symbols of at most 7 bytes (FSST allows 8): the GPU's segmented kernel
    // keeps a symbol's length in its top byte, one table read per code; on
    // l_comment the 8th byte bought 0.6 % of compression
    const uint32_t max_len = ml ? (uint32_t)std::max(1, std::min(8, atoi(ml))) : 7;
    std::vector<std::pair<uint32_t, uint32_t>> smp;  // (offset, length)
    const uint64_t total = offs[n] - offs[0];
    const uint32_t step = (uint32_t)std::max<uint64_t>(1, total / sample_bytes);  // rows between samples
    uint64_t taken = 0;
    for (uint32_t i = 0; i < n && taken < sample_bytes; i += step) {
        smp.emplace_back(offs[i], offs[i + 1] - offs[i]);
        taken += offs[i + 1] - offs[i];
    }
    FsstTable st;
    struct Key {
        uint64_t sym;
        uint32_t len;
        bool operator==(const Key &o) const { return sym == o.sym && len == o.len; }
        bool operator<(const Key &o) const { return sym != o.sym ? sym < o.sym : len < o.len; }
    };
    for (int round = 0; round < rounds; ++round) {
        st.index();
        st.index2();
        // ids: 0..n-1 symbols, 256 + b escaped byte b
        std::vector<uint64_t> c1(512, 0);
        // adjacent-pair counts: a flat 512 x 512 table (the pairs that occur
        // listed once each) instead of a hash map
        thread_local std::vector<uint32_t> c2(512 * 512, 0);
        std::vector<uint32_t> pairs;
        auto sym_of = [&](int id, uint64_t &s, uint32_t &l) {
            if (id < 256) { s = st.sym[id]; l = st.len[id]; }
            else { s = (uint64_t)(id - 256); l = 1; }
        };
        for (auto &sp : smp) {
            const uint8_t *p = (const uint8_t *)bytes + sp.first;
            int prev = -1;
            for (uint32_t i = 0; i < sp.second;) {
                const int c = st.match2(p + i, sp.second - i);
                const int id = c >= 0 ? c : 256 + p[i];
                i += c >= 0 ? st.len[c] : 1;
                c1[id]++;
                if (prev >= 0) {
                    const uint32_t k = ((uint32_t)prev << 9) | (uint32_t)id;
                    if (c2[k]++ == 0) pairs.push_back(k);
                }
                prev = id;
            }
        }
        // candidate symbol -> gain (the largest of its occurrences), kept as a
        // list merged by sorting rather than a hash map
        std::vector<std::pair<Key, uint64_t>> gain;
        gain.reserve(512 + pairs.size());
        auto add = [&](uint64_t sym, uint32_t l, uint64_t g) { gain.push_back({Key{sym, l}, g}); };
        for (int id = 0; id < 512; ++id) {
            if (!c1[id]) continue;
            uint64_t sy;
            uint32_t l;
            sym_of(id, sy, l);
            add(sy, l, c1[id] * l);
        }
        for (uint32_t k : pairs) {
            const uint64_t cnt = c2[k];
            c2[k] = 0;  // (the table is all zero again for the next round)
            uint64_t s1, s2;
            uint32_t l1, l2;
            sym_of((int)(k >> 9), s1, l1);
            sym_of((int)(k & 511), s2, l2);
            if (l1 >= max_len) continue;
            const uint32_t l = std::min<uint32_t>(max_len, l1 + l2);
            uint64_t sy = s1 | (s2 << (8 * l1));
            if (l < 8) sy &= (1ull << (8 * l)) - 1;
            add(sy, l, cnt * l);
        }
        std::sort(gain.begin(), gain.end(), [](const auto &a, const auto &b) {
            return a.first < b.first || (a.first == b.first && a.second > b.second);
        });
        std::vector<std::pair<Key, uint64_t>> cand;  // one entry per key, its largest gain
        cand.reserve(gain.size());
        for (auto &g : gain)
            if (cand.empty() || !(cand.back().first == g.first)) cand.push_back(g);
        std::sort(cand.begin(), cand.end(), [](const auto &a, const auto &b) {
            return a.second != b.second ? a.second > b.second : a.first < b.first;
        });
        st = FsstTable();
        for (auto &c : cand) {
            if (st.n == max_symbols) break;
            st.sym[st.n] = c.first.sym;
            st.len[st.n] = (uint8_t)c.first.len;
            st.n++;
        }
    }
    // Every byte value that occurs in the chunk gets a one-byte symbol when
    // the table has room for all of them (it always does for text: l_comment
    // uses 35 byte values), displacing the lowest-gain multi-byte symbols.  A
    // byte the sample missed would otherwise be escaped wherever it occurs:
    // two code bytes instead of one, and the GPU decoder's slower escape path
    // for every vector holding one.  Tables capped below 255 symbols
    // (FLS_FSST_MAX_SYMBOLS, tests forcing escapes) are left as built.
    if (max_symbols == 255) {
        bool seen[256] = {};
        const uint8_t *b = (const uint8_t *)bytes;
        for (uint64_t i = offs[0]; i < offs[n]; ++i) seen[b[i]] = true;
        bool single[256] = {};
        int nsingle = 0;
        for (int c = 0; c < st.n; ++c)
            if (st.len[c] == 1) single[st.sym[c] & 0xFF] = true;
        std::vector<uint8_t> missing;
        for (int v = 0; v < 256; ++v) {
            nsingle += seen[v] ? 1 : 0;
            if (seen[v] && !single[v]) missing.push_back((uint8_t)v);
        }
        if (!missing.empty() && nsingle <= max_symbols) {
            // candidates are in decreasing gain order: replace from the end,
            // skipping one-byte symbols (they stay)
            int c = st.n;
            for (uint8_t v : missing) {
                if (st.n < max_symbols) {
                    st.sym[st.n] = v;
                    st.len[st.n] = 1;
                    st.n++;
                    continue;
                }
                do { --c; } while (c > 0 && st.len[c] == 1);
                if (c < 0 || st.len[c] == 1) break;  // no multi-byte symbol left to replace
                st.sym[c] = v;
                st.len[c] = 1;
            }
        }
    }
    st.index();
    st.index2();
    return st;
}

// The segment table of a vector's code stream (fls_format.hpp): per
// kFsstSegCodes code bytes the bytes they decode to and the escape state
// entering them, so a GPU lane can decode its segment with no hand-off.
void fsst_segments(const FsstTable &st, const std::vector<uint8_t> &comp, uint8_t *out) {
    FsstSegHeader sh{};
    sh.nseg = fsst_nseg((uint32_t)comp.size());
    uint8_t *seg = out + sizeof(sh);
    uint32_t state = 0;  // 1: the next byte is an escape's literal
    for (uint32_t k = 0; k < sh.nseg; ++k) {
        const uint32_t entry = state;
        uint32_t d = 0;
        const size_t e = std::min<size_t>(comp.size(), (size_t)(k + 1) * kFsstSegCodes);
        for (size_t j = (size_t)k * kFsstSegCodes; j < e; ++j) {
            const uint8_t c = comp[j];
            if (state) { d += 1; state = 0; }
            else if (c == kFsstEscape) { state = 1; sh.flags |= FSST_SEG_HAS_ESCAPE; }
            else d += st.len[c];
        }
        seg[k] = fsst_seg_value(d, entry);
    }
    memcpy(out, &sh, sizeof(sh));
}

// GPU FSST compression (fls_writer_set_device): the chunk's table is built
// here, the strings are compressed on the GPU (launch_fsst_compress, the same
// greedy longest match as FsstTable::compress, so the same code bytes) and
// the vectors are assembled here as for the host compressor.  One context per
// concurrently encoding worker (its own stream and buffers), from a free list.
// The same context builds VARCHAR / BLOB dictionaries on the GPU (run_dict,
// launch_str_dict: build_str_dict's first-appearance order and codes).
struct FsstGpuCtx {
    hipStream_t stream = nullptr;
    uint8_t *h_in = nullptr, *d_in = nullptr, *h_codes = nullptr, *d_codes = nullptr;
    uint32_t *h_offs = nullptr, *d_offs = nullptr, *h_clen = nullptr, *d_clen = nullptr;
    FsstCTable *h_tab = nullptr, *d_tab = nullptr;
    size_t in_cap = 0, n_cap = 0;
    // string dictionaries: slots u32[3 cap], row slots, codes and entries u32[n]
    uint32_t *d_slots = nullptr, *d_rows = nullptr, *d_dcodes = nullptr, *d_entries = nullptr;
    uint32_t *h_dcodes = nullptr, *h_entries = nullptr;
    StrDictInfo *d_info = nullptr, *h_info = nullptr;
    size_t dict_n_cap = 0;

    void release_dict() {
        hipFree(d_slots);
        hipFree(d_rows);
        hipFree(d_dcodes);
        hipFree(d_entries);
        hipFree(d_info);
        pinned_free(h_dcodes);
        pinned_free(h_entries);
        pinned_free(h_info);
        d_slots = d_rows = d_dcodes = d_entries = h_dcodes = h_entries = nullptr;
        d_info = h_info = nullptr;
        dict_n_cap = 0;
    }
    void release() {
        if (stream) hipStreamSynchronize(stream);
        release_dict();
        pinned_free(h_in);
        pinned_free(h_codes);
        pinned_free(h_offs);
        pinned_free(h_clen);
        pinned_free(h_tab);
        hipFree(d_in);
        hipFree(d_codes);
        hipFree(d_offs);
        hipFree(d_clen);
        hipFree(d_tab);
        if (stream) hipStreamDestroy(stream);
        *this = FsstGpuCtx();
    }
#define FHIP(expr)                                                                                  \
    do {                                                                                            \
        const hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(FLS_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)
    // Strings [offs[0], offs[n]) of bytes into d_in (8-aligned, 16 zero bytes
    // after) and their offsets from 0 into d_offs, on this context's stream.
    int upload(int dev, const uint32_t *offs, const char *bytes, uint32_t n) {
        FHIP(hipSetDevice(dev));
        if (!stream) FHIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        const size_t nb = offs[n] - offs[0];
        if (nb + 16 > in_cap) {
            pinned_free(h_in);
            pinned_free(h_codes);
            hipFree(d_in);
            hipFree(d_codes);
            h_in = h_codes = d_in = d_codes = nullptr;
            in_cap = 0;
            const size_t cap = std::max<size_t>(nb + 16, 1 << 20) * 5 / 4;
            FHIP(pinned_alloc((void **)&h_in, cap));
            FHIP(pinned_alloc((void **)&h_codes, 2 * cap));
            FHIP(hipMalloc((void **)&d_in, cap));
            FHIP(hipMalloc((void **)&d_codes, 2 * cap));
            in_cap = cap;
        }
        if (n + 1 > n_cap) {
            pinned_free(h_offs);
            pinned_free(h_clen);
            hipFree(d_offs);
            hipFree(d_clen);
            h_offs = h_clen = d_offs = d_clen = nullptr;
            n_cap = 0;
            FHIP(pinned_alloc((void **)&h_offs, 4ull * (n + 1)));
            FHIP(pinned_alloc((void **)&h_clen, 4ull * (n + 1)));
            FHIP(hipMalloc((void **)&d_offs, 4ull * (n + 1)));
            FHIP(hipMalloc((void **)&d_clen, 4ull * (n + 1)));
            n_cap = n + 1;
        }
        if (!h_tab) {
            FHIP(pinned_alloc((void **)&h_tab, sizeof(FsstCTable)));
            FHIP(hipMalloc((void **)&d_tab, sizeof(FsstCTable)));
        }
        memcpy(h_in, bytes + offs[0], nb);
        memset(h_in + nb, 0, 16);
        for (uint32_t i = 0; i <= n; ++i) h_offs[i] = offs[i] - offs[0];
        FHIP(hipMemcpyAsync(d_in, h_in, nb + 16, hipMemcpyHostToDevice, stream));
        FHIP(hipMemcpyAsync(d_offs, h_offs, 4ull * (n + 1), hipMemcpyHostToDevice, stream));
        return 0;
    }

    // The dictionary of the n strings (build_str_dict on the GPU): d.entries
    // in first-appearance order and d.codes; few = false once more than
    // `limit` distinct strings occur.  A chunk with more than kDictGpuMax
    // distinct strings is built on the host (same result).
    int run_dict(int dev, const uint32_t *offs, const char *bytes, uint32_t n, uint32_t limit, StrDict &d, bool &few) {
        if (const char *f = getenv("FLS_TEST_FAIL_FSST_GPU"); f && atoi(f) != 0)
            return fail(FLS_ERR_DEVICE, "injected GPU string dictionary failure");
        if (int rc = upload(dev, offs, bytes, n)) return rc;
        if (n > dict_n_cap) {
            release_dict();
            FHIP(hipMalloc((void **)&d_slots, 12ull * enc_dict_cap(n)));
            FHIP(hipMalloc((void **)&d_rows, 4ull * n));
            FHIP(hipMalloc((void **)&d_dcodes, 4ull * n));
            FHIP(hipMalloc((void **)&d_entries, 4ull * n));
            FHIP(hipMalloc((void **)&d_info, sizeof(StrDictInfo)));
            FHIP(pinned_alloc((void **)&h_dcodes, 4ull * n));
            FHIP(pinned_alloc((void **)&h_entries, 4ull * n));
            FHIP(pinned_alloc((void **)&h_info, sizeof(StrDictInfo)));
            dict_n_cap = n;
        }
        // one round trip: the codes and entries come back with the outcome
        // (unused when the build overflowed or is left to the host)
        FHIP(launch_str_dict(d_in, d_offs, n, limit, d_slots, d_rows, d_dcodes, d_entries, d_info, stream));
        FHIP(hipMemcpyAsync(h_info, d_info, sizeof(StrDictInfo), hipMemcpyDeviceToHost, stream));
        FHIP(hipMemcpyAsync(h_dcodes, d_dcodes, 4ull * n, hipMemcpyDeviceToHost, stream));
        FHIP(hipMemcpyAsync(h_entries, d_entries, 4ull * std::min<uint32_t>(n, kDictGpuMax), hipMemcpyDeviceToHost,
                            stream));
        FHIP(hipStreamSynchronize(stream));
        const StrDictInfo info = *h_info;
        if (info.overflow) {
            few = false;
            return 0;
        }
        if (info.big) {  // more distinct strings than the GPU sorts: the host's build
            few = build_str_dict(offs, bytes, n, limit, d);
            return 0;
        }
        if (info.count > std::min<uint32_t>(n, kDictGpuMax))
            return fail(FLS_ERR_DEVICE, "GPU string dictionary: %u entries for %u rows", info.count, n);
        d.entries.resize(info.count);
        for (uint32_t k = 0; k < info.count; ++k) {
            const uint32_t r = h_entries[k];
            if (r >= n) return fail(FLS_ERR_DEVICE, "GPU string dictionary: entry %u names row %u of %u", k, r, n);
            d.entries[k] = std::string_view(bytes + offs[r], offs[r + 1] - offs[r]);
        }
        d.codes.assign(h_dcodes, h_dcodes + n);
        d.entry_bytes = info.entry_bytes;
        few = true;
        return 0;
    }

    // compress strings [offs[0], offs[n]) of bytes with table st: string i's
    // codes at h_codes + 2 * (offs[i] - offs[0]), their count h_clen[i]
    // (uploaded: these strings are already in d_in / d_offs, from run_dict)
    int run(int dev, const FsstTable &st, const uint32_t *offs, const char *bytes, uint32_t n, bool uploaded = false) {
        // test hook: a failed device compression (the writer's error path)
        if (const char *f = getenv("FLS_TEST_FAIL_FSST_GPU"); f && atoi(f) != 0)
            return fail(FLS_ERR_DEVICE, "injected GPU FSST compression failure");
        if (!uploaded)
            if (int rc = upload(dev, offs, bytes, n)) return rc;
        const size_t nb = offs[n] - offs[0];
        // the table: codes of length >= 2 bucketed by their first two bytes in
        // the order the host's two-byte index lists them (by_first order)
        FsstCTable &t = *h_tab;
        memset(&t, 0, sizeof(t));
        memcpy(t.sym, st.sym, sizeof(t.sym));
        memcpy(t.len, st.len, sizeof(t.len));
        memcpy(t.one, st.one, sizeof(t.one));
        uint32_t cnt[kFsstCBuckets + 1] = {};
        for (int b = 0; b < 256; ++b)
            for (uint8_t c : st.by_first[b])
                if (st.len[c] >= 2) cnt[fsst_cbucket((uint32_t)(st.sym[c] & 0xFFFF)) + 1]++;
        for (uint32_t k = 0; k < kFsstCBuckets; ++k) cnt[k + 1] += cnt[k];
        for (uint32_t k = 0; k <= kFsstCBuckets; ++k) t.start[k] = (uint16_t)cnt[k];
        for (int b = 0; b < 256; ++b)
            for (uint8_t c : st.by_first[b])
                if (st.len[c] >= 2) t.codes[cnt[fsst_cbucket((uint32_t)(st.sym[c] & 0xFFFF))]++] = c;
        FHIP(hipMemcpyAsync(d_tab, h_tab, sizeof(FsstCTable), hipMemcpyHostToDevice, stream));
        FHIP(launch_fsst_compress(d_in, d_offs, n, d_tab, d_codes, d_clen, stream));
        FHIP(hipMemcpyAsync(h_clen, d_clen, 4ull * n, hipMemcpyDeviceToHost, stream));
        FHIP(hipMemcpyAsync(h_codes, d_codes, 2 * nb, hipMemcpyDeviceToHost, stream));
        FHIP(hipStreamSynchronize(stream));
        for (uint32_t i = 0; i < n; ++i)
            if (h_clen[i] > 2ull * (h_offs[i + 1] - h_offs[i]))
                return fail(FLS_ERR_DEVICE, "GPU FSST compression: string %u: %u codes for %u bytes", i, h_clen[i],
                            h_offs[i + 1] - h_offs[i]);
        return 0;
    }
#undef FHIP
};
struct FsstGpu {
    int dev = -1;
    std::mutex mu;
    std::vector<FsstGpuCtx *> idle, all;
    std::atomic<int> err{0};   // first failure's code (the message is in the failing thread's fls_last_error)
    std::string err_msg;
    FsstGpuCtx *take() {
        std::lock_guard<std::mutex> lk(mu);
        if (idle.empty()) {
            all.push_back(new FsstGpuCtx());
            return all.back();
        }
        FsstGpuCtx *g = idle.back();
        idle.pop_back();
        return g;
    }
    void give(FsstGpuCtx *g) {
        std::lock_guard<std::mutex> lk(mu);
        idle.push_back(g);
    }
    void failed(int rc) {
        std::lock_guard<std::mutex> lk(mu);
        if (err.load() == 0) {
            err_msg = fls_last_error();
            err.store(rc);
        }
    }
    void release() {
        if (dev >= 0) hipSetDevice(dev);
        for (FsstGpuCtx *g : all) {
            g->release();
            delete g;
        }
        all.clear();
        idle.clear();
        err.store(0);
    }
    ~FsstGpu() { release(); }
};

// FLS_WRITER_PROFILE=1: time in the string chunk steps, summed over worker
// threads (printed with the writer's phases)
struct StrProfile {
    std::atomic<uint64_t> dict_ns{0}, table_ns{0}, compress_ns{0}, chunks{0};
    static uint64_t now_ns() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
};
StrProfile g_str_prof;
bool g_str_prof_on = getenv("FLS_WRITER_PROFILE") != nullptr;  // (re-read by fls_writer_new)

// gpu: compress on that GPU (fls_writer_set_device); a failure is recorded in
// gpu->err (the caller reports it) and leaves an empty chunk.  held: a context
// taken from gpu that already holds these strings (ENC_AUTO's dictionary
// attempt uploaded them); it is given back here.
std::vector<uint8_t> enc_fsst(const uint32_t *offs, const char *bytes, uint32_t n, FsstGpu *gpu = nullptr,
                              FsstGpuCtx *held = nullptr) {
    const uint64_t t0 = g_str_prof_on ? StrProfile::now_ns() : 0;
    const FsstTable st = fsst_build(offs, bytes, n);
    const uint64_t t1 = g_str_prof_on ? StrProfile::now_ns() : 0;
    if (g_str_prof_on) g_str_prof.table_ns += t1 - t0;
    FsstGpuCtx *g = nullptr;
    if (gpu) {
        g = held ? held : gpu->take();
        if (const int rc = g->run(gpu->dev, st, offs, bytes, n, held != nullptr)) {
            gpu->give(g);
            gpu->failed(rc);
            return {};
        }
        if (g_str_prof_on) g_str_prof.compress_ns += StrProfile::now_ns() - t1;
    }
    std::vector<uint8_t> table(kFsstTableBytes, 0);
    memcpy(table.data(), st.sym, 8 * 256);
    memcpy(table.data() + 8 * 256, st.len, 256);
    const uint32_t nvec = (n + 1023) / 1024;
    std::vector<VecOut> vecs(nvec);
    uint64_t lens[1024], clens[1024], u[1024];
    uint64_t heap = 0;
    std::vector<uint8_t> comp;
    for (uint32_t k = 0; k < nvec; ++k) {
        const uint32_t b = k * 1024, vn = std::min<uint32_t>(1024, n - b);
        comp.clear();
        for (uint32_t i = 0; i < 1024; ++i) {
            const size_t c0 = comp.size();
            if (i < vn && g) {
                const uint8_t *cs = g->h_codes + 2ull * (offs[b + i] - offs[0]);
                comp.insert(comp.end(), cs, cs + g->h_clen[b + i]);
            } else if (i < vn) {
                st.compress((const uint8_t *)bytes + offs[b + i], offs[b + i + 1] - offs[b + i], comp);
            }
            clens[i] = comp.size() - c0;
        }
        for (uint32_t i = 0; i < 1024; ++i) lens[i] = i < vn ? offs[b + i + 1] - offs[b + i] : 0;
        const uint64_t dbytes = offs[b + vn] - offs[b];
        int64_t base;
        const int W = ffor_prepare(32, lens, base, u);
        VecOut &o = vecs[k];
        o.meta = VecMeta{};
        o.meta.for_base = base;
        o.meta.bw = (uint8_t)W;
        o.meta.nvals = (uint16_t)vn;
        o.meta.aux_count = (uint32_t)dbytes;
        o.packed.assign((size_t)128 * W, 0);
        pack(32, W, u, o.packed.data());
        FsstVecHeader vh{};
        vh.heap_off = (uint32_t)heap;
        vh.comp_len = (uint32_t)comp.size();
        int64_t cbase;
        const int Wc = ffor_prepare(32, clens, cbase, u);
        vh.clen_base = (uint32_t)cbase;
        vh.clen_w = (uint32_t)Wc;
        o.aux.assign(fsst_seg_off(vh) + fsst_seg_bytes(vh.comp_len), 0);
        memcpy(o.aux.data(), &vh, sizeof(vh));
        pack(32, Wc, u, o.aux.data() + sizeof(vh));
        if (!comp.empty()) memcpy(o.aux.data() + fsst_stream_off(vh), comp.data(), comp.size());
        fsst_segments(st, comp, o.aux.data() + fsst_seg_off(vh));
        heap += (dbytes + 15) & ~15ull;
    }
    if (g) gpu->give(g);
    return assemble_chunk(ENC_FSST, 32, 0, true, n, vecs, table, (uint32_t)st.n, heap, kFsstSegCodes);
}

// VARCHAR: DICT when the distinct values are few (at most n / 8, and their
// bytes + 4 each under half the chunk's bytes), else FSST.  ENC_AUTO builds
// the dictionary once: it is the estimate and, when DICT wins, the encoding.
// With a device (gpu) and FLS_WRITER_STRDICT_GPU=1 the dictionary is built
// on the GPU (FsstGpuCtx::run_dict): same entries, same codes, same bytes.
std::vector<uint8_t> encode_str_chunk(uint8_t enc, const uint32_t *offs, const char *bytes, uint32_t n,
                                      FsstGpu *gpu = nullptr) {
    if (enc == ENC_FSST) return enc_fsst(offs, bytes, n, gpu);
    StrDict d;
    const uint32_t limit = enc == ENC_AUTO ? n / 8 : n;
    bool few;
    // VARCHAR dictionaries on the GPU are opt-in (FLS_WRITER_STRDICT_GPU=1):
    // a chunk's build is one synchronous round trip (~0.45 ms of copies and
    // kernels, queued behind the other workers' on the device), slower in
    // COPY than the host threads' build
    const uint64_t t0 = g_str_prof_on ? StrProfile::now_ns() : 0;
    if (g_str_prof_on) ++g_str_prof.chunks;
    if (gpu && n > 0 && knob_value("FLS_WRITER_DICT_GPU") != 0 && knob_value("FLS_WRITER_STRDICT_GPU") != 0) {
        FsstGpuCtx *g = gpu->take();
        const int rc = g->run_dict(gpu->dev, offs, bytes, n, limit, d, few);
        if (g_str_prof_on) g_str_prof.dict_ns += StrProfile::now_ns() - t0;
        if (rc) {
            gpu->give(g);
            gpu->failed(rc);
            return {};
        }
        if (enc == ENC_AUTO &&
            !(few && d.entry_bytes + 4ull * d.entries.size() < (uint64_t)(offs[n] - offs[0]) / 2))
            return enc_fsst(offs, bytes, n, gpu, g);   // the strings are on the GPU already
        gpu->give(g);
    } else {
        few = build_str_dict(offs, bytes, n, limit, d);
        if (g_str_prof_on) g_str_prof.dict_ns += StrProfile::now_ns() - t0;
    }
    if (enc == ENC_AUTO &&
        !(few && d.entry_bytes + 4ull * d.entries.size() < (uint64_t)(offs[n] - offs[0]) / 2))
        return enc_fsst(offs, bytes, n, gpu);
    return enc_dict_str(d, n);
}

// FastLanes-RLE: per vector run values + run-index vector (u16) DELTA-coded
std::vector<uint8_t> enc_rle(int T, const uint64_t *vals, uint32_t n) {
    const uint32_t nvec = (n + 1023) / 1024;
    std::vector<VecOut> vecs(nvec);
    uint64_t v[1024], idx[1024], pv[1024], u[1024];
    for (uint32_t k = 0; k < nvec; ++k) {
        uint32_t vn;
        load_vec(vals, n, k, v, vn);
        std::vector<uint64_t> runs;
        for (int i = 0; i < 1024; ++i) {
            if (i == 0 || v[i] != v[i - 1]) runs.push_back(v[i]);
            idx[i] = runs.size() - 1;
        }
        VecOut &o = vecs[k];
        o.aux.assign(128 + runs.size() * (T / 8), 0);
        delta_vector(16, idx, pv, o.aux.data());
        for (size_t r = 0; r < runs.size(); ++r) put_word(o.aux.data() + 128, T, r, runs[r]);
        int64_t base;
        int W = ffor_prepare(16, pv, base, u);
        o.meta = VecMeta{};
        o.meta.for_base = base;
        o.meta.bw = (uint8_t)W;
        o.meta.nvals = (uint16_t)vn;
        o.meta.aux_count = (uint32_t)runs.size();
        o.packed.assign((size_t)128 * W, 0);
        pack(16, W, u, o.packed.data());
    }
    return assemble_chunk(ENC_RLE, 16, (uint8_t)T, false, n, vecs, {}, 0);
}

// ---- ALP (FLOAT / DOUBLE) ----------------------------------------------------
// Afroozeh et al., SIGMOD 2024: per vector an exponent e and factor f (f <= e)
// such that most values n satisfy n == (F)d * 10^f * 10^-e for the integer
// d = round(n * 10^e * 10^-f); the d are FFOR-packed, the rest are exceptions
// (position + original value).  (e, f) selection is ALP's two-level sampling:
// the chunk's sampled vectors vote for their best combination, each vector
// then picks the cheapest of the top five on its own sample.

template <class F>
struct AlpT;
template <>
struct AlpT<double> {
    using I = int64_t;
    using U = uint64_t;
    static constexpr int T = 64, kMaxE = kAlpMaxExpD;
    static constexpr double F10[] = {FLS_ALP_F10_D};
    static constexpr double IF10[] = {FLS_ALP_IF10_D};
    static constexpr double kLimit = 9.2233720368547748e18;  // below 2^63
};
template <>
struct AlpT<float> {
    using I = int32_t;
    using U = uint32_t;
    static constexpr int T = 32, kMaxE = kAlpMaxExpF;
    static constexpr float F10[] = {FLS_ALP_F10_F};
    static constexpr float IF10[] = {FLS_ALP_IF10_F};
    static constexpr float kLimit = 2.1474835e9f;  // below 2^31
};

template <class F>
inline bool alp_encode_one(F n, int e, int f, typename AlpT<F>::I &d) {
    using A = AlpT<F>;
    const F tmp = n * A::F10[e] * A::IF10[f];
    if (!(std::fabs(tmp) < A::kLimit)) return false;  // also rejects NaN / inf
    d = (typename A::I)std::nearbyint(tmp);
    const F back = (F)d * A::F10[f] * A::IF10[e];
    return memcmp(&back, &n, sizeof(F)) == 0;  // bit-exact (keeps -0.0 as an exception)
}

// estimated bits of one sample under (e, f)
template <class F>
uint64_t alp_cost(const F *x, int n, int e, int f) {
    using A = AlpT<F>;
    typename A::I mn = 0, mx = 0, d;
    bool any = false;
    int exc = 0;
    for (int i = 0; i < n; ++i) {
        if (!alp_encode_one<F>(x[i], e, f, d)) { ++exc; continue; }
        if (!any) { mn = mx = d; any = true; }
        mn = std::min(mn, d);
        mx = std::max(mx, d);
    }
    const uint64_t range = any ? (uint64_t)((typename A::U)mx - (typename A::U)mn) : 0;
    return (uint64_t)bitlen(range) * n + (uint64_t)exc * (16 + A::T);
}

template <class F>
void alp_sample(const F *v, uint32_t vn, F *s, int &n) {
    n = (int)std::min<uint32_t>(32, vn);
    for (int i = 0; i < n; ++i) s[i] = v[(uint64_t)i * vn / n];
}

template <class F>
std::vector<uint8_t> enc_alp(const uint64_t *bits, uint32_t n) {
    using A = AlpT<F>;
    constexpr int T = A::T;
    const uint32_t nvec = (n + 1023) / 1024;
    std::vector<F> vals(n);
    for (uint32_t i = 0; i < n; ++i) {
        typename A::U u = (typename A::U)bits[i];
        memcpy(&vals[i], &u, sizeof(F));
    }
    // level 1: sampled vectors vote for their best (e, f)
    std::vector<std::pair<int, int>> combos;
    {
        std::vector<int> votes((A::kMaxE + 1) * (A::kMaxE + 1), 0);
        const uint32_t nsv = std::min<uint32_t>(8, nvec);
        F smp[32];
        int sn;
        for (uint32_t k = 0; k < nsv; ++k) {
            const uint32_t v = (uint32_t)((uint64_t)k * nvec / nsv);
            const uint32_t b = v * 1024, vn = std::min<uint32_t>(1024, n - b);
            alp_sample<F>(vals.data() + b, vn, smp, sn);
            uint64_t best = UINT64_MAX;
            int be = 0, bf = 0;
            for (int e = 0; e <= A::kMaxE; ++e)
                for (int f = 0; f <= e; ++f) {
                    const uint64_t c = alp_cost<F>(smp, sn, e, f);
                    if (c < best) { best = c; be = e; bf = f; }
                }
            votes[be * (A::kMaxE + 1) + bf]++;
        }
        std::vector<int> order(votes.size());
        for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return votes[a] > votes[b]; });
        for (int i = 0; i < 5 && votes[order[i]] > 0; ++i)
            combos.emplace_back(order[i] / (A::kMaxE + 1), order[i] % (A::kMaxE + 1));
        if (combos.empty()) combos.emplace_back(0, 0);
    }
    std::vector<VecOut> vecs(nvec);
    uint64_t u64v[1024], u[1024];
    for (uint32_t k = 0; k < nvec; ++k) {
        const uint32_t b = k * 1024, vn = std::min<uint32_t>(1024, n - b);
        const F *v = vals.data() + b;
        // level 2: cheapest of the chunk's combinations on this vector's sample
        int e = combos[0].first, f = combos[0].second;
        if (combos.size() > 1) {
            F smp[32];
            int sn;
            alp_sample<F>(v, vn, smp, sn);
            uint64_t best = UINT64_MAX;
            for (auto &c : combos) {
                const uint64_t cost = alp_cost<F>(smp, sn, c.first, c.second);
                if (cost < best) { best = cost; e = c.first; f = c.second; }
            }
        }
        typename A::I d[1024];
        std::vector<uint16_t> pos;
        bool have_fill = false;
        typename A::I fill = 0;
        for (uint32_t i = 0; i < vn; ++i) {
            if (alp_encode_one<F>(v[i], e, f, d[i])) {
                if (!have_fill) { fill = d[i]; have_fill = true; }
            } else {
                pos.push_back((uint16_t)i);
            }
        }
        for (uint16_t p : pos) d[p] = fill;           // keep the FFOR range tight
        for (uint32_t i = 0; i < 1024; ++i) {
            const typename A::I x = i < vn ? d[i] : d[vn - 1];
            u64v[i] = (uint64_t)(typename A::U)x;
        }
        int64_t base;
        const int W = ffor_prepare(T, u64v, base, u);
        VecOut &o = vecs[k];
        o.meta = VecMeta{};
        o.meta.for_base = base;
        o.meta.bw = (uint8_t)W;
        o.meta.nvals = (uint16_t)vn;
        o.meta.aux_count = (uint32_t)pos.size() | ((uint32_t)e << 16) | ((uint32_t)f << 24);
        o.packed.assign((size_t)128 * W, 0);
        pack(T, W, u, o.packed.data());
        if (!pos.empty()) {
            o.aux.assign(alp_aux_bytes((uint32_t)pos.size(), T), 0);
            memcpy(o.aux.data(), pos.data(), 2 * pos.size());
            uint8_t *ev = o.aux.data() + ((2 * pos.size() + 15) & ~size_t(15));
            for (size_t j = 0; j < pos.size(); ++j) memcpy(ev + j * sizeof(F), &v[pos[j]], sizeof(F));
        }
    }
    return assemble_chunk(ENC_ALP, (uint8_t)T, (uint8_t)T, false, n, vecs, {}, 0);
}

// estimated encoded bytes for ENC_AUTO
size_t est_ffor(int T, const uint64_t *vals, uint32_t n) {
    size_t b = 0;
    uint64_t v[1024], u[1024];
    for (uint32_t k = 0; k < (n + 1023) / 1024; ++k) {
        uint32_t vn;
        load_vec(vals, n, k, v, vn);
        int64_t base;
        b += 128 * (size_t)ffor_prepare(T, v, base, u) + 32;
    }
    return b;
}
size_t est_delta(int T, const uint64_t *vals, uint32_t n) {
    size_t b = 0;
    uint64_t v[1024], pv[1024], u[1024];
    uint8_t bases[128];
    for (uint32_t k = 0; k < (n + 1023) / 1024; ++k) {
        uint32_t vn;
        load_vec(vals, n, k, v, vn);
        delta_vector(T, v, pv, bases);
        int64_t base;
        b += 128 * (size_t)ffor_prepare(T, pv, base, u) + 32 + 128;
    }
    return b;
}
size_t est_rle(int T, const uint64_t *vals, uint32_t n) {
    size_t runs = 1;
    for (uint32_t i = 1; i < n; ++i) runs += vals[i] != vals[i - 1];
    if (runs * 4 > n) return SIZE_MAX;  // not worth it
    // idx deltas over stride 16 are <= 16 -> at most 5 bits
    return runs * (T / 8) + ((n + 1023) / 1024) * (32 + 128 + 128 * 5);
}
size_t est_dict(int T, const uint64_t *vals, uint32_t n) {
    // a 1,024-value sample first: high-cardinality columns (keys, prices)
    // skip the full distinct count, which dominated ENC_AUTO's cost
    if (n > 4096) {
        uint64_t smp[1024];
        for (uint32_t i = 0; i < 1024; ++i) smp[i] = vals[(uint64_t)i * n / 1024];
        std::sort(smp, smp + 1024);
        if (std::unique(smp, smp + 1024) - smp > 512) return SIZE_MAX;
    }
    U64Table tab(n);
    for (uint32_t i = 0; i < n; ++i) tab.insert(vals[i]);
    const size_t d = tab.count;
    if (d > 65536) return SIZE_MAX;
    return d * (T / 8) + ((n + 1023) / 1024) * (32 + 128 * (size_t)bitlen(d - 1 ? d - 1 : 0));
}

// est_dict over a column chunk held in its own width (T/8 bytes per value):
// the 1,024-value sample reads the typed values directly, so the common
// high-cardinality case converts nothing (the GPU ENC_AUTO path)
uint64_t load_typed(const uint8_t *p, int T, uint64_t i) {
    uint64_t x = 0;
    memcpy(&x, p + i * (T / 8), T / 8);
    return x;
}
size_t est_dict_typed(int T, const void *data, uint32_t n) {
    const uint8_t *p = (const uint8_t *)data;
    if (n > 4096) {
        uint64_t smp[1024];
        for (uint32_t i = 0; i < 1024; ++i) smp[i] = load_typed(p, T, (uint64_t)i * n / 1024);
        std::sort(smp, smp + 1024);
        if (std::unique(smp, smp + 1024) - smp > 512) return SIZE_MAX;
    }
    std::vector<uint64_t> v(n);
    for (uint32_t i = 0; i < n; ++i) v[i] = load_typed(p, T, i);
    return est_dict(T, v.data(), n);
}

struct ColSpec {
    std::string name;
    uint8_t type, width, scale, enc;
};

}  // namespace

// Encode one integer chunk with a chosen (or automatic) encoding.
std::vector<uint8_t> encode_int_chunk(uint8_t type, uint8_t enc, const uint64_t *vals, uint32_t n) {
    if (type == TY_DOUBLE) return enc_alp<double>(vals, n);
    if (type == TY_FLOAT) return enc_alp<float>(vals, n);
    const int T = type_value_bits(type);
    if (enc == ENC_AUTO) {
        size_t best = est_ffor(T, vals, n);
        enc = ENC_FFOR;
        size_t d = est_delta(T, vals, n);
        if (d < best) { best = d; enc = ENC_DELTA; }
        size_t r = est_rle(T, vals, n);
        if (r < best) { best = r; enc = ENC_RLE; }
        size_t x = est_dict(T, vals, n);
        if (x < best) { best = x; enc = ENC_DICT; }
    }
    switch (enc) {
    case ENC_DELTA: return enc_delta(T, vals, n);
    case ENC_DICT: return enc_dict_int(T, vals, n);
    case ENC_RLE: return enc_rle(T, vals, n);
    default: return enc_ffor(T, vals, n);
    }
}

// ---- file assembly -------------------------------------------------------

struct FileBuilder {
    std::vector<ColSpec> cols;
    uint64_t row_offset = 0;
    uint32_t rowgroup_size = kRowGroupSize;  // rows per row group (all but the last)
    struct RG {
        uint32_t nrows;
        std::vector<std::vector<uint8_t>> chunks;
        std::vector<ZoneMap> zones;  // per column (VARCHAR: none)
        // per column: the chunk's validity bitmaps (nvec x 128 B) when it has
        // a NULL, else empty; appended to the chunk by finish()
        std::vector<std::vector<uint64_t>> valid;
        // per column: the chunk's final length once it was handed to the
        // output stream (its bytes are gone then)
        std::vector<uint64_t> flen;
        uint64_t chunk_len(size_t c) const {
            if (!flen.empty()) return flen[c];
            const uint64_t n = chunks[c].size();
            return c < valid.size() && !valid[c].empty() ? ((n + 15) & ~15ull) + 8ull * valid[c].size() : n;
        }
    };
    std::vector<RG> rgs;

    // ---- streamed output (fls_writer_set_output) ------------------------------
    // Row groups whose chunks are all encoded are handed, in order, to
    // threads that pwrite() them at their final offsets in a temporary file in
    // the destination's directory, so the file is written while later row
    // groups encode instead of all at the end; finish writes the footer and
    // renames the file over the destination (a failed or abandoned write
    // leaves no partial file there).  Chunk bytes are freed once written.
    // FLS_WRITER_STREAM_THREADS (default 1) threads: 4 did not speed up the
    // end of an unordered COPY, whose last ~1 GB of row groups complete at
    // once (34.16 vs 34.39 M rows/s, profiles/r5/copy_stream_threads_r5v.txt).
    struct Stream {
        struct Job {
            uint64_t at = 0, len = 0;
            std::vector<uint8_t> bytes;
            std::vector<uint64_t> valid;
        };
        int fd = -1;
        std::string path, tmp;
        uint64_t off = 256;              // next chunk's offset
        size_t next_rg = 0;              // first row group not handed over yet
        std::vector<uint64_t> offs;      // per chunk handed over (footer)
        std::vector<std::thread> th;
        std::mutex mu;
        std::condition_variable cv, room;
        std::deque<Job> q;
        uint64_t queued = 0;             // bytes waiting in q
        bool stop = false;
        std::atomic<int> err{0};         // errno of a failed write (read by writer threads without mu)
        static constexpr uint64_t kMaxQueued = 512ull << 20;
    };
    std::unique_ptr<Stream> out;

    static int pwrite_all(int fd, const void *p, uint64_t n, uint64_t at) {
        const uint8_t *b = (const uint8_t *)p;
        while (n > 0) {
            const ssize_t k = ::pwrite(fd, b, std::min<uint64_t>(n, 1ull << 30), (off_t)at);
            if (k < 0 && errno == EINTR) continue;
            if (k <= 0) return errno ? errno : EIO;
            b += k;
            at += (uint64_t)k;
            n -= (uint64_t)k;
        }
        return 0;
    }
    static std::string tmp_name(const std::string &path) {
        return path + ".tmp." + std::to_string((long)getpid()) + "." +
               std::to_string((unsigned long long)(uintptr_t)&path % 100000);
    }
    int open_stream(const char *path) {
        if (out) return fail(FLS_ERR_STATE, "fls_writer_set_output: output already set");
        if (!rgs.empty()) return fail(FLS_ERR_STATE, "fls_writer_set_output: after first row group");
        auto st = std::make_unique<Stream>();
        st->path = path;
        st->tmp = tmp_name(st->path);
        st->fd = ::open(st->tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (st->fd < 0) return fail(FLS_ERR_IO, "cannot create %s: %s", st->tmp.c_str(), strerror(errno));
        uint8_t head[256] = {};
        memcpy(head, kFileMagic, 8);
        const uint64_t version = 1;
        memcpy(head + 8, &version, 8);
        if (const int e = pwrite_all(st->fd, head, sizeof(head), 0)) {
            ::close(st->fd);
            ::unlink(st->tmp.c_str());
            return fail(FLS_ERR_IO, "write to %s: %s", st->tmp.c_str(), strerror(e));
        }
        Stream *sp = st.get();
        const int nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(16, knob_value("FLS_WRITER_STREAM_THREADS")));
        for (int t = 0; t < nthreads; ++t) st->th.emplace_back([sp] {
            static const uint8_t zeros[16] = {};
            std::vector<uint8_t> tmp;
            for (;;) {
                Stream::Job j;
                {
                    std::unique_lock<std::mutex> lk(sp->mu);
                    sp->cv.wait(lk, [&] { return sp->stop || !sp->q.empty(); });
                    if (sp->q.empty()) return;
                    j = std::move(sp->q.front());
                    sp->q.pop_front();
                }
                int e = 0;
                if (!sp->err) {
                    const uint64_t padded = (j.len + 15) & ~15ull;
                    if (!j.valid.empty()) {
                        tmp.assign(padded, 0);
                        memcpy(tmp.data(), j.bytes.data(), j.bytes.size());
                        append_validity(tmp.data(), j.bytes.size(), j.len, j.valid);
                        e = pwrite_all(sp->fd, tmp.data(), padded, j.at);
                    } else {
                        e = pwrite_all(sp->fd, j.bytes.data(), j.bytes.size(), j.at);
                        if (!e && padded > j.bytes.size()) e = pwrite_all(sp->fd, zeros, padded - j.bytes.size(), j.at + j.bytes.size());
                    }
                }
                std::lock_guard<std::mutex> lk(sp->mu);
                if (e && !sp->err) sp->err = e;
                sp->queued -= j.bytes.size();
                sp->room.notify_all();
            }
        });
        out = std::move(st);
        return 0;
    }
    // hand the complete row groups from next_rg on to the stream (all: every
    // row group must be complete -- after the GPU encoder's last batch)
    int flush_stream(bool all) {
        if (!out) return 0;
        Stream &st = *out;
        for (; st.next_rg < rgs.size(); ++st.next_rg) {
            RG &r = rgs[st.next_rg];
            bool done = true;
            for (auto &ch : r.chunks) done = done && !ch.empty();
            if (!done) {
                if (all) return fail(FLS_ERR_STATE, "row group %zu incomplete at finish", st.next_rg);
                break;
            }
            std::vector<uint64_t> lens(r.chunks.size());
            for (size_t c = 0; c < r.chunks.size(); ++c) lens[c] = r.chunk_len(c);
            for (size_t c = 0; c < r.chunks.size(); ++c) {
                Stream::Job j;
                j.at = st.off;
                j.len = lens[c];
                j.bytes = std::move(r.chunks[c]);
                if (c < r.valid.size()) j.valid = std::move(r.valid[c]);
                st.offs.push_back(st.off);
                st.off += (lens[c] + 15) & ~15ull;
                std::unique_lock<std::mutex> lk(st.mu);
                st.room.wait(lk, [&] { return st.queued < Stream::kMaxQueued || st.err; });
                st.queued += j.bytes.size();
                st.q.push_back(std::move(j));
                st.cv.notify_one();
            }
            r.flen = std::move(lens);
            r.chunks.assign(r.chunks.size(), {});
        }
        return 0;
    }
    // stop the thread after the queue drains; the first write error (0: none)
    int drain_stream() {
        if (!out || out->th.empty()) return out ? out->err.load() : 0;
        {
            std::lock_guard<std::mutex> lk(out->mu);
            out->stop = true;
        }
        out->cv.notify_all();
        for (auto &t : out->th) t.join();
        out->th.clear();
        return out->err.load();
    }
    void abandon_stream() {
        if (!out) return;
        drain_stream();
        if (out->fd >= 0) ::close(out->fd);
        ::unlink(out->tmp.c_str());
        out.reset();
    }
    ~FileBuilder() { abandon_stream(); }
    FileBuilder() = default;
    FileBuilder(const FileBuilder &) = delete;
    FileBuilder &operator=(const FileBuilder &) = delete;
    // the streamed file: remaining row groups, footer, tail, rename over path
    int finish_stream(const char *path) {
        Stream &st = *out;
        if (st.path != path) {
            abandon_stream();
            return fail(FLS_ERR_ARG, "fls_writer_finish_file: the output was set to another path");
        }
        if (const int rc = flush_stream(true)) {
            abandon_stream();
            return rc;
        }
        const int e = drain_stream();
        if (e) {
            const std::string t = st.tmp;
            abandon_stream();
            return fail(FLS_ERR_IO, "write to %s: %s", t.c_str(), strerror(e));
        }
        std::vector<uint8_t> ft = footer(st.offs);
        uint8_t tail[16];
        const uint32_t flen = (uint32_t)ft.size();
        memcpy(tail, &st.off, 8);
        memcpy(tail + 8, &flen, 4);
        memcpy(tail + 12, kTailMagic, 4);
        ft.insert(ft.end(), tail, tail + 16);
        int rc = pwrite_all(st.fd, ft.data(), ft.size(), st.off);
        if (!rc && ftruncate(st.fd, (off_t)(st.off + ft.size())) != 0) rc = errno;
        if (::close(st.fd) != 0 && !rc) rc = errno;
        st.fd = -1;
        if (!rc && ::rename(st.tmp.c_str(), st.path.c_str()) != 0) rc = errno;
        if (rc) {
            const std::string t = st.tmp;
            abandon_stream();
            return fail(FLS_ERR_IO, "write to %s: %s", t.c_str(), strerror(rc));
        }
        out.reset();
        return 0;
    }

    std::vector<uint8_t> footer(const std::vector<uint64_t> &chunk_offs) const {
        std::vector<uint8_t> f;
        auto put = [&f](const void *p, size_t n) { f.insert(f.end(), (const uint8_t *)p, (const uint8_t *)p + n); };
        uint32_t ver = kFooterVersion, ncols = (uint32_t)cols.size(), nrg = (uint32_t)rgs.size(), rgsz = rowgroup_size;
        uint64_t nrows = 0;
        for (auto &r : rgs) nrows += r.nrows;
        put(&ver, 4); put(&ncols, 4); put(&nrows, 8); put(&nrg, 4); put(&rgsz, 4); put(&row_offset, 8);
        for (auto &c : cols) {
            uint8_t d[4] = {c.type, c.width, c.scale, 0};
            put(d, 4);
            uint16_t nl = (uint16_t)c.name.size();
            put(&nl, 2);
            put(c.name.data(), nl);
        }
        size_t k = 0;
        for (auto &r : rgs) {
            put(&r.nrows, 4);
            for (size_t c = 0; c < cols.size(); ++c, ++k) {
                uint64_t off = chunk_offs[k], len = r.chunk_len(c);
                put(&off, 8);
                put(&len, 8);
            }
        }
        // zone-map section (fls_format.hpp)
        uint32_t zm[2] = {kZoneMagic, (uint32_t)sizeof(ZoneMap)};
        put(zm, 8);
        const ZoneMap none{0, 0, 0, 0};
        for (auto &r : rgs)
            for (size_t c = 0; c < cols.size(); ++c) put(c < r.zones.size() ? &r.zones[c] : &none, sizeof(ZoneMap));
        return f;
    }

    // A chunk's validity (fls_format.hpp): the bitmaps at its end, the flag in
    // its header and the has-NULL mark of each vector holding a NULL.
    static void append_validity(uint8_t *chunk, uint64_t enc_len, uint64_t len, const std::vector<uint64_t> &w) {
        memcpy(chunk + len - 8 * w.size(), w.data(), 8 * w.size());
        ChunkHeader h;
        memcpy(&h, chunk, sizeof(h));
        h.reserved0 |= kChunkValidity;
        memcpy(chunk, &h, sizeof(h));
        for (uint32_t v = 0; v < h.nvec; ++v) {
            const uint32_t n = std::min<uint32_t>(kVectorSize, h.nvals - v * kVectorSize);
            bool null = false;
            for (uint32_t j = 0; j < 16; ++j) {
                const uint32_t r0 = 64 * j;
                const uint64_t live = r0 >= n ? 0 : (n - r0 >= 64 ? ~0ull : ((1ull << (n - r0)) - 1));
                null |= (w[16 * v + j] & live) != live;
            }
            if (null) chunk[h.meta_off + 32ull * v + offsetof(VecMeta, pad)] |= kVecHasNull;
        }
        (void)enc_len;
    }

    // Assemble into one malloc'ed image; chunk buffers are released as copied.
    int finish(uint8_t **img, uint64_t *len, int nthreads) {
        std::vector<uint64_t> offs;
        uint64_t off = 256;  // 8 B magic + 8 B version, padded to the chunk alignment
        for (auto &r : rgs)
            for (size_t c = 0; c < r.chunks.size(); ++c) {
                offs.push_back(off);
                off += (r.chunk_len(c) + 15) & ~15ull;  // chunks start 16-aligned
            }
        std::vector<uint8_t> ft = footer(offs);
        const uint64_t foot_off = off;
        const uint64_t total = off + ft.size() + 16;
        uint8_t *buf = (uint8_t *)malloc(total);
        if (!buf) return fail(FLS_ERR_NOMEM, "out of host memory assembling %llu bytes", (unsigned long long)total);
        memset(buf, 0, 256);
        memcpy(buf, kFileMagic, 8);
        uint64_t version = 1;
        memcpy(buf + 8, &version, 8);
        // parallel copy by row group
        std::atomic<size_t> next{0};
        std::vector<size_t> rg_first(rgs.size() + 1, 0);
        for (size_t i = 0; i < rgs.size(); ++i) rg_first[i + 1] = rg_first[i] + rgs[i].chunks.size();
        auto work = [&]() {
            for (size_t r; (r = next.fetch_add(1)) < rgs.size();) {
                for (size_t c = 0; c < rgs[r].chunks.size(); ++c) {
                    auto &ch = rgs[r].chunks[c];
                    uint8_t *dst = buf + offs[rg_first[r] + c];
                    const uint64_t len = rgs[r].chunk_len(c);
                    memcpy(dst, ch.data(), ch.size());
                    memset(dst + ch.size(), 0, ((len + 15) & ~15ull) - ch.size());
                    if (c < rgs[r].valid.size() && !rgs[r].valid[c].empty())
                        append_validity(dst, ch.size(), len, rgs[r].valid[c]);
                    std::vector<uint8_t>().swap(ch);
                }
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
        work();
        for (auto &t : th) t.join();
        memcpy(buf + foot_off, ft.data(), ft.size());
        uint32_t flen = (uint32_t)ft.size();
        memcpy(buf + foot_off + ft.size(), &foot_off, 8);
        memcpy(buf + foot_off + ft.size() + 8, &flen, 4);
        memcpy(buf + foot_off + ft.size() + 12, kTailMagic, 4);
        *img = buf;
        *len = total;
        return 0;
    }

    // The same bytes written straight to a file: every chunk pwrite()n at its
    // offset by the row group's thread (no image of the whole file in memory,
    // no single-threaded write of it).  Padding is written, not left as holes.
    int write_file(const char *path, int nthreads) {
        std::vector<uint64_t> offs;
        uint64_t off = 256;
        for (auto &r : rgs)
            for (size_t c = 0; c < r.chunks.size(); ++c) {
                offs.push_back(off);
                off += (r.chunk_len(c) + 15) & ~15ull;
            }
        std::vector<uint8_t> ft = footer(offs);
        const uint64_t foot_off = off;
        // written beside path and renamed over it once complete: a failed write
        // leaves no partial file at path, and tables still mapping the old file
        // keep its inode
        const std::string tmp = tmp_name(path);
        const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0) return fail(FLS_ERR_IO, "cannot create %s: %s", tmp.c_str(), strerror(errno));
        std::atomic<int> bad{0};
        auto put = [&](const void *p, uint64_t n, uint64_t at) {
            const uint8_t *b = (const uint8_t *)p;
            while (n > 0) {
                const ssize_t k = ::pwrite(fd, b, std::min<uint64_t>(n, 1ull << 30), (off_t)at);
                if (k < 0 && errno == EINTR) continue;
                if (k <= 0) {
                    bad.store(errno ? errno : EIO);
                    return;
                }
                b += k;
                at += (uint64_t)k;
                n -= (uint64_t)k;
            }
        };
        uint8_t head[256] = {};
        memcpy(head, kFileMagic, 8);
        const uint64_t version = 1;
        memcpy(head + 8, &version, 8);
        put(head, sizeof(head), 0);
        std::atomic<size_t> next{0};
        std::vector<size_t> rg_first(rgs.size() + 1, 0);
        for (size_t i = 0; i < rgs.size(); ++i) rg_first[i + 1] = rg_first[i] + rgs[i].chunks.size();
        static const uint8_t zeros[16] = {};
        auto work = [&]() {
            std::vector<uint8_t> tmp;
            for (size_t r; !bad.load() && (r = next.fetch_add(1)) < rgs.size();) {
                for (size_t c = 0; c < rgs[r].chunks.size(); ++c) {
                    auto &ch = rgs[r].chunks[c];
                    const uint64_t at = offs[rg_first[r] + c], len = rgs[r].chunk_len(c), padded = (len + 15) & ~15ull;
                    if (c < rgs[r].valid.size() && !rgs[r].valid[c].empty()) {
                        tmp.assign(padded, 0);
                        memcpy(tmp.data(), ch.data(), ch.size());
                        append_validity(tmp.data(), ch.size(), len, rgs[r].valid[c]);
                        put(tmp.data(), padded, at);
                    } else {
                        put(ch.data(), ch.size(), at);
                        if (padded > ch.size()) put(zeros, padded - ch.size(), at + ch.size());
                    }
                    std::vector<uint8_t>().swap(ch);
                }
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
        work();
        for (auto &t : th) t.join();
        uint8_t tail[16];
        const uint32_t flen = (uint32_t)ft.size();
        memcpy(tail, &foot_off, 8);
        memcpy(tail + 8, &flen, 4);
        memcpy(tail + 12, kTailMagic, 4);
        ft.insert(ft.end(), tail, tail + 16);
        put(ft.data(), ft.size(), foot_off);
        int e = bad.load();
        if (::close(fd) != 0 && !e) e = errno ? errno : EIO;
        if (!e && ::rename(tmp.c_str(), path) != 0) e = errno ? errno : EIO;
        if (e) {
            ::unlink(tmp.c_str());
            return fail(FLS_ERR_IO, "write to %s: %s", path, strerror(e));
        }
        return 0;
    }
};

// ---- seeded workloads ----------------------------------------------------

namespace {

const char *const kReturnFlag[] = {"A", "N", "R"};
const char *const kLineStatus[] = {"F", "O"};
const char *const kShipInstruct[] = {"DELIVER IN PERSON", "COLLECT COD", "NONE", "TAKE BACK RETURN"};
const char *const kShipMode[] = {"REG AIR", "AIR", "RAIL", "SHIP", "TRUCK", "MAIL", "FOB"};

struct Workload {
    std::string name;
    std::vector<ColSpec> cols;
    uint64_t nrows;
    gen::LineitemParams li;
    bool lineitem = false;   // lineitem, lineitem_full, lineitem_dbl
    bool dbl = false;        // quantity / extendedprice / discount / tax as DOUBLE (ALP)
    int comment_col = -1;    // l_comment (FSST) column
};

uint64_t lineitem_rows(double sf) {
    // dbgen row counts at the standard scale factors
    if (sf == 0.01) return 60175;
    if (sf == 0.1) return 600572;
    if (sf == 1) return 6001215;
    if (sf == 10) return 59986052;
    if (sf == 100) return 600037902;
    if (sf == 1000) return 5999989709ull;
    return (uint64_t)(6000000.0 * sf + 0.5);
}

bool make_workload(const char *wl, double sf, uint64_t nrows, Workload &w) {
    if (!wl) return false;
    w.name = wl;
    w.cols.clear();
    if (w.name == "c1") {
        w.cols = {{"value", TY_INT32, 0, 0, ENC_FFOR}};
        w.nrows = nrows ? nrows : 1000000;
    } else if (w.name == "c3") {
        w.cols = {{"key", TY_INT64, 0, 0, ENC_DELTA}};
        w.nrows = nrows ? nrows : 1000000000ull;
    } else if (w.name == "c4") {
        w.cols = {{"mode", TY_VARCHAR, 0, 0, ENC_DICT}};
        w.nrows = nrows ? nrows : 1000000000ull;
    } else if (w.name == "lineitem" || w.name == "lineitem_full" || w.name == "lineitem_dbl") {
        if (!(sf > 0)) return false;
        w.lineitem = true;
        w.cols = {
            {"l_orderkey", TY_INT64, 0, 0, ENC_DELTA},   {"l_partkey", TY_INT32, 0, 0, ENC_FFOR},
            {"l_suppkey", TY_INT32, 0, 0, ENC_FFOR},     {"l_linenumber", TY_INT32, 0, 0, ENC_FFOR},
            {"l_quantity", TY_DECIMAL, 15, 2, ENC_FFOR}, {"l_extendedprice", TY_DECIMAL, 15, 2, ENC_FFOR},
            {"l_discount", TY_DECIMAL, 15, 2, ENC_FFOR}, {"l_tax", TY_DECIMAL, 15, 2, ENC_FFOR},
            {"l_returnflag", TY_VARCHAR, 0, 0, ENC_DICT}, {"l_linestatus", TY_VARCHAR, 0, 0, ENC_DICT},
            {"l_shipdate", TY_DATE, 0, 0, ENC_FFOR},     {"l_commitdate", TY_DATE, 0, 0, ENC_FFOR},
            {"l_receiptdate", TY_DATE, 0, 0, ENC_FFOR},  {"l_shipinstruct", TY_VARCHAR, 0, 0, ENC_DICT},
            {"l_shipmode", TY_VARCHAR, 0, 0, ENC_DICT},
        };
        if (w.name == "lineitem_dbl") {
            // the four DECIMAL(15,2) columns as DOUBLE (cents / 100.0), ALP-encoded
            w.dbl = true;
            for (int c = 4; c < 8; ++c) w.cols[c] = {w.cols[c].name, TY_DOUBLE, 0, 0, ENC_ALP};
        }
        if (w.name == "lineitem_full") {  // all 16 TPC-H columns: l_comment FSST
            w.comment_col = 15;
            w.cols.push_back({"l_comment", TY_VARCHAR, 0, 0, ENC_FSST});
        }
        w.nrows = nrows ? nrows : lineitem_rows(sf);
        w.li.n_part = std::max<int64_t>(1, (int64_t)(200000.0 * sf + 0.5));
        w.li.n_supp = std::max<int64_t>(4, (int64_t)(10000.0 * sf + 0.5));
    } else {
        return false;
    }
    w.li.seed = gen::kSeed;
    w.li.nrows = w.nrows;
    return true;
}

// dictionary (string table) of a generated VARCHAR column
bool gen_dict(const Workload &w, int col, std::vector<std::string_view> &d) {
    auto fill = [&d](const char *const *t, size_t n) { d.assign(t, t + n); };
    if (w.name == "c4" && col == 0) { fill(kShipMode, 7); return true; }
    if (w.lineitem) {
        switch (col) {
        case 8: fill(kReturnFlag, 3); return true;
        case 9: fill(kLineStatus, 2); return true;
        case 13: fill(kShipInstruct, 4); return true;
        case 14: fill(kShipMode, 7); return true;
        }
    }
    return false;
}

// Fill raw values (sign-extended ints / codes) of all columns for rows
// [row0, row0+n).  out[c] holds n uint64.
void gen_rows(const Workload &w, uint64_t row0, uint32_t n, std::vector<std::vector<uint64_t>> &out) {
    out.resize(w.cols.size());
    for (auto &o : out) o.resize(n);
    if (w.name == "c1") {
        for (uint32_t i = 0; i < n; ++i) out[0][i] = (uint64_t)gen::c1_value(w.li.seed, row0 + i);
    } else if (w.name == "c4") {
        for (uint32_t i = 0; i < n; ++i) out[0][i] = (uint64_t)gen::c4_code(w.li.seed, row0 + i);
    } else if (w.name == "c3") {
        gen::OrderWalker ow;
        ow.start(w.li.seed, row0);
        for (uint32_t i = 0; i < n; ++i, ow.next()) out[0][i] = (uint64_t)gen::orderkey(ow.cur().order);
    } else {
        gen::OrderWalker ow;
        ow.start(w.li.seed, row0);
        gen::LineitemRow r;
        for (uint32_t i = 0; i < n; ++i, ow.next()) {
            gen::lineitem_row_at(w.li, row0 + i, ow.cur(), r);
            for (int c = 0; c < gen::kLineitemCols; ++c) out[c][i] = (uint64_t)gen::lineitem_col(r, c);
            if (w.dbl)
                for (int c = 4; c < 8; ++c) {
                    const double x = (double)(int64_t)out[c][i] / 100.0;
                    memcpy(&out[c][i], &x, 8);
                }
            if (w.comment_col >= 0) out[w.comment_col][i] = row0 + i;  // strings come from gen::comment
        }
    }
}

// l_comment strings of rows [row0, row0+n) as offsets + bytes
void gen_comments(const Workload &w, uint64_t row0, uint32_t n, std::vector<uint32_t> &offs, std::string &bytes) {
    offs.assign(n + 1, 0);
    bytes.clear();
    for (uint32_t i = 0; i < n; ++i) {
        const std::string_view c = gen::comment(w.li.seed, row0 + i);
        bytes.append(c.data(), c.size());
        offs[i + 1] = (uint32_t)bytes.size();
    }
}

std::vector<uint8_t> encode_gen_chunk(const Workload &w, int c, const std::vector<uint64_t> &vals,
                                      ZoneMap *zone = nullptr) {
    const ColSpec &cs = w.cols[c];
    const uint32_t n = (uint32_t)vals.size();
    if (c == w.comment_col) {
        std::vector<uint32_t> offs;
        std::string bytes;
        gen_comments(w, vals[0], n, offs, bytes);
        return enc_fsst(offs.data(), bytes.data(), n);
    }
    if (type_is_string(cs.type)) {
        std::vector<std::string_view> d;
        gen_dict(w, c, d);
        std::vector<uint32_t> codes(vals.begin(), vals.end());
        return enc_dict_codes(codes.data(), n, 0, true, str_dict_bytes(d), (uint32_t)d.size());
    }
    const int T = type_value_bits(cs.type);
    std::vector<uint64_t> tv(vals);
    for (auto &x : tv) x &= tmask(T);
    if (zone) *zone = zone_of(cs.type, tv.data(), n);
    return encode_int_chunk(cs.type, cs.enc, tv.data(), n);
}

}  // namespace
}  // namespace fls

using namespace fls;

// ---- C-ABI ----------------------------------------------------------------

namespace {
int default_writer_threads() {
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::min(16u, std::max(1u, hw));
}
}  // namespace

// FLS_WRITER_PROFILE=1: wall time of the writer's phases, summed over the
// writer's calls and printed to stderr when the image is finished
struct WriterProfile {
    bool on = getenv("FLS_WRITER_PROFILE") != nullptr;
    double cpu = 0, submit = 0, gpu_wait = 0, copy_out = 0, finish = 0;
    uint64_t flushes = 0;
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void print() const {
        if (on)
            fprintf(stderr,
                    "fls_writer profile: CPU columns, GPU staging and zone maps %.3f s, submit %.3f s, gpu wait %.3f s, "
                    "copy out %.3f s (%llu flushes), finish %.3f s\n",
                    cpu, submit, gpu_wait, copy_out, (unsigned long long)flushes, finish);
        if (on)
            fprintf(stderr,
                    "fls_writer profile: string chunks %llu: dictionaries %.3f s, FSST tables %.3f s, "
                    "FSST compression (GPU round trips) %.3f s (summed over worker threads)\n",
                    (unsigned long long)g_str_prof.chunks.load(), g_str_prof.dict_ns.load() * 1e-9,
                    g_str_prof.table_ns.load() * 1e-9, g_str_prof.compress_ns.load() * 1e-9);
    }
};
static WriterProfile g_prof;

// GPU chunk encoding of the FFOR / DELTA integer columns (fls_writer_set_device).
// Row groups are batched, kBatch per launch, in two buffer sets used in turn.
// add() reserves a row group's room in the current set (the caller stages the
// values into pinned memory in the same worker pass as the zone maps) and
// records one job per chunk.  A full set is submitted -- one H2D copy, the
// encode launches (a block per chunk), the lengths and the slots back in two
// D2H copies, all async on the encoder's stream -- and staging continues in
// the other set.  A set's chunks move into their row groups when the set is
// needed again or at finish(); by then its GPU work has run under the staging
// of the next batch.  (Per-row-group launches of ~11 blocks left the GPU
// idle: 46 M rows/s against 65 M on 16 CPU threads for lineitem SF10; one
// synchronous flush per batch with a separate staging pass: 54 M rows/s.)
struct GpuEncoder {
    static constexpr uint32_t kBatch = 32;  // row groups per launch
    struct Job {
        size_t rg, col;
        uint64_t in_off, out_off;
        uint32_t nrows;
        uint8_t T, enc;         // enc may be ENC_AUTO: the kernel chooses (fls_encode.hip choose_encoding)
        uint64_t est_dict = UINT64_MAX;  // ENC_AUTO: the DICT estimate (set by the staging pass, or kEstDictGpu)
        uint64_t dict_off = UINT64_MAX;  // ENC_DICT / ENC_AUTO: its DICT table in d_dict (UINT64_MAX: none)
    };
    struct Set {
        uint8_t *h_stage = nullptr, *d_in = nullptr, *d_out = nullptr, *d_scratch = nullptr, *h_out = nullptr;
        uint8_t *d_dict = nullptr;    // DICT hash tables of the set's ENC_DICT / ENC_AUTO jobs
        size_t dict_cap = 0;
        uint64_t dict_used = 0;
        uint64_t *h_lens = nullptr, *d_lens = nullptr;
        EncChunk *h_desc = nullptr, *d_desc = nullptr;
        size_t in_cap = 0, out_cap = 0, job_cap = 0;
        std::vector<Job> jobs;
        uint64_t in_used = 0, out_used = 0;
        uint32_t batched = 0;  // row groups in the set
        bool in_flight = false;
        hipEvent_t done = nullptr;
    };
    int dev = -1;
    hipStream_t stream = nullptr;
    Set sets[2];
    int cur = 0;

    static void free_set(Set &b) {
        pinned_free(b.h_stage);
        pinned_free(b.h_lens);
        pinned_free(b.h_out);
        pinned_free(b.h_desc);
        hipFree(b.d_in);
        hipFree(b.d_out);
        hipFree(b.d_lens);
        hipFree(b.d_desc);
        hipFree(b.d_scratch);
        hipFree(b.d_dict);
        if (b.done) hipEventDestroy(b.done);
        b = Set();
    }
    void release() {
        if (dev < 0) return;
        hipSetDevice(dev);
        if (stream) hipStreamSynchronize(stream);
        free_set(sets[0]);
        free_set(sets[1]);
        if (stream) hipStreamDestroy(stream);
        stream = nullptr;
        cur = 0;
    }
    ~GpuEncoder() { release(); }
    bool full() const { return sets[cur].batched >= kBatch; }

#define WHIP(expr)                                                                                  \
    do {                                                                                            \
        const hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(FLS_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

    // Room for a full batch of row groups needing in_rg / out_rg / nj /
    // dict_rg each (the set is empty and idle here).
    int ensure(Set &b, uint64_t in_rg, uint64_t out_rg, size_t nj, uint64_t dict_rg) {
        if (!b.done) WHIP(hipEventCreateWithFlags(&b.done, hipEventDisableTiming));
        if (kBatch * dict_rg > b.dict_cap) {
            hipFree(b.d_dict);
            b.d_dict = nullptr;
            b.dict_cap = 0;
            WHIP(hipMalloc((void **)&b.d_dict, kBatch * dict_rg));
            b.dict_cap = kBatch * dict_rg;
        }
        if (kBatch * in_rg > b.in_cap) {
            pinned_free(b.h_stage);
            hipFree(b.d_in);
            b.h_stage = b.d_in = nullptr;
            b.in_cap = 0;
            WHIP(pinned_alloc((void **)&b.h_stage, kBatch * in_rg));
            WHIP(hipMalloc((void **)&b.d_in, kBatch * in_rg));
            b.in_cap = kBatch * in_rg;
        }
        if (kBatch * out_rg > b.out_cap) {
            hipFree(b.d_out);
            pinned_free(b.h_out);
            b.d_out = b.h_out = nullptr;
            b.out_cap = 0;
            WHIP(hipMalloc((void **)&b.d_out, kBatch * out_rg));
            WHIP(pinned_alloc((void **)&b.h_out, kBatch * out_rg));
            b.out_cap = kBatch * out_rg;
        }
        if (kBatch * nj > b.job_cap) {
            hipFree(b.d_desc);
            hipFree(b.d_lens);
            pinned_free(b.h_lens);
            pinned_free(b.h_desc);
            hipFree(b.d_scratch);
            b.d_desc = b.h_desc = nullptr;
            b.d_lens = b.h_lens = nullptr;
            b.d_scratch = nullptr;
            b.job_cap = 0;
            const size_t n = kBatch * nj;
            WHIP(hipMalloc((void **)&b.d_desc, n * sizeof(EncChunk)));
            WHIP(pinned_alloc((void **)&b.h_desc, n * sizeof(EncChunk)));
            WHIP(hipMalloc((void **)&b.d_lens, n * sizeof(uint64_t)));
            WHIP(pinned_alloc((void **)&b.h_lens, n * sizeof(uint64_t)));
            WHIP(hipMalloc((void **)&b.d_scratch, n * enc_scratch_bytes()));
            b.job_cap = n;
        }
        // add() hands out pointers into jobs (est_dict) that must stay valid
        // while later row groups join the set (fls_writer_add_rowgroups)
        b.jobs.reserve(b.job_cap);
        return 0;
    }

    // Pinned staging / slot bytes columns cols of an nrows row group need.
    // DICT chunks on the GPU (FLS_WRITER_DICT_GPU=0: DICT estimates and DICT
    // chunks on the host, the round-3 path)
    static bool dict_gpu() {
        return knob_value("FLS_WRITER_DICT_GPU") != 0;
    }
    static bool dict_job(uint8_t enc) { return (enc == ENC_DICT || enc == ENC_AUTO) && dict_gpu(); }
    // ALP chunks of FLOAT / DOUBLE columns on the GPU only with
    // FLS_WRITER_ALP_GPU=1: the host threads won every same-box A/B (COPY
    // lineitem_dbl SF10: 55.2 vs 51.1 M rows/s unordered, 44.2 vs 38.4 ordered,
    // profiles/r5/copy_r5o_lineitem_dbl_10.txt; r4: ordered -10 %), and the
    // byte-identical GPU kernel stays as the opt-in
    static bool alp_gpu() {
        return knob_value("FLS_WRITER_ALP_GPU") != 0;
    }
    // the encoding a job asks the kernels for: FLOAT / DOUBLE columns are ALP
    // (ENC_AUTO included, as encode_int_chunk does)
    static uint8_t job_enc(const ColSpec &cs) { return type_is_float(cs.type) ? (uint8_t)ENC_ALP : cs.enc; }
    static void need(const std::vector<ColSpec> &specs, const std::vector<size_t> &cols, uint32_t nrows,
                     uint64_t &in_rg, uint64_t &out_rg, uint64_t &dict_rg) {
        in_rg = out_rg = dict_rg = 0;
        for (size_t c : cols) {
            const int T = type_value_bits(specs[c].type);
            const uint8_t enc = job_enc(specs[c]);
            in_rg += ((uint64_t)nrows * (T / 8) + 15) & ~15ull;
            out_rg += enc_slot_bytes((uint32_t)T, nrows, enc);
            if (dict_job(enc)) dict_rg += (enc_dict_tab_bytes(nrows) + 255) & ~255ull;
        }
    }
    // Whether add() would take this row group into the current set without
    // first submitting it (submitting needs every row group of the set staged).
    bool has_room(const std::vector<ColSpec> &specs, const std::vector<size_t> &cols, uint32_t nrows) const {
        uint64_t in_rg, out_rg, dict_rg;
        need(specs, cols, nrows, in_rg, out_rg, dict_rg);
        const Set &b = sets[cur];
        return !b.in_flight && b.in_used + in_rg <= b.in_cap && b.out_used + out_rg <= b.out_cap &&
               b.jobs.size() + cols.size() <= b.job_cap && b.dict_used + dict_rg <= b.dict_cap;
    }

    // Reserve the current set's room for columns cols of row group rg (nrows
    // rows); stage[c] = where column c's values go in pinned memory (the
    // caller copies them there, together with the column's zone map pass).
    int add(const std::vector<ColSpec> &specs, const std::vector<size_t> &cols, size_t rg, uint32_t nrows,
            int nthreads, std::vector<FileBuilder::RG> &rgs, std::vector<uint8_t *> &stage,
            std::vector<uint64_t *> &est_dict) {
        WHIP(hipSetDevice(dev));
        if (!stream) WHIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        // capacity for a full batch of row groups like this one (the first
        // row group is the largest: only the last one may be short)
        uint64_t in_rg, out_rg, dict_rg;
        need(specs, cols, nrows, in_rg, out_rg, dict_rg);
        if (sets[cur].in_flight) {
            const int rc = complete(sets[cur], rgs, nthreads);
            if (rc) return rc;
        }
        Set *b = &sets[cur];
        if (b->in_used + in_rg > b->in_cap || b->out_used + out_rg > b->out_cap ||
            b->jobs.size() + cols.size() > b->job_cap || b->dict_used + dict_rg > b->dict_cap) {
            if (!b->jobs.empty()) {
                int rc = submit();
                if (rc) return rc;
                b = &sets[cur];
                if (b->in_flight && (rc = complete(*b, rgs, nthreads))) return rc;
            }
            const int rc = ensure(*b, in_rg, out_rg, cols.size(), dict_rg);
            if (rc) return rc;
        }
        const size_t j0 = b->jobs.size();
        for (size_t c : cols) {
            const int T = type_value_bits(specs[c].type);
            const uint8_t enc = job_enc(specs[c]);
            Job jb{rg, c, b->in_used, b->out_used, nrows, (uint8_t)T, enc};
            if (dict_job(enc)) {
                jb.dict_off = b->dict_used;
                b->dict_used += (enc_dict_tab_bytes(nrows) + 255) & ~255ull;
            }
            b->jobs.push_back(jb);
            stage[c] = b->h_stage + b->in_used;
            b->in_used += ((uint64_t)nrows * (T / 8) + 15) & ~15ull;
            b->out_used += enc_slot_bytes((uint32_t)T, nrows, enc);
        }
        for (size_t k = 0; k < cols.size(); ++k) est_dict[cols[k]] = &b->jobs[j0 + k].est_dict;
        ++b->batched;  // the caller submits a full set once this row group is in rgs
        return 0;
    }

    // Send the current set to the GPU (async) and switch to the other set.
    int submit() {
        Set &b = sets[cur];
        if (b.jobs.empty()) return 0;
        const double t0 = g_prof.on ? WriterProfile::now() : 0;
        WHIP(hipSetDevice(dev));
        for (size_t i = 0; i < b.jobs.size(); ++i) {
            const Job &jb = b.jobs[i];
            EncChunk &c = b.h_desc[i];
            c.in = (uint64_t)(uintptr_t)(b.d_in + jb.in_off);
            c.out = (uint64_t)(uintptr_t)(b.d_out + jb.out_off);
            c.len_out = (uint64_t)(uintptr_t)(b.d_lens + i);
            c.scratch = (uint64_t)(uintptr_t)(b.d_scratch + i * enc_scratch_bytes());
            c.nrows = jb.nrows;
            c.T = jb.T;
            c.enc = jb.enc;
            c.pad[0] = c.pad[1] = 0;
            c.est_dict = jb.est_dict;
            c.dict_tab = jb.dict_off == UINT64_MAX ? 0 : (uint64_t)(uintptr_t)(b.d_dict + jb.dict_off);
            c.reserved = 0;
        }
        // T = 64 chunks first (launch_encode); each carries its own addresses
        EncChunk *first = b.h_desc, *last = b.h_desc + b.jobs.size();
        const uint32_t n_wide =
            (uint32_t)(std::stable_partition(first, last, [](const EncChunk &c) { return c.T == 64; }) - first);
        WHIP(hipMemcpyAsync(b.d_in, b.h_stage, b.in_used, hipMemcpyHostToDevice, stream));
        WHIP(hipMemcpyAsync(b.d_desc, b.h_desc, b.jobs.size() * sizeof(EncChunk), hipMemcpyHostToDevice, stream));
        bool rle = false, dict = false, alp = false;
        for (const Job &jb : b.jobs) {
            rle |= jb.enc == ENC_RLE || jb.enc == ENC_AUTO;
            dict |= jb.dict_off != UINT64_MAX;
            alp |= jb.enc == ENC_ALP;
        }
        WHIP(launch_encode(b.d_desc, n_wide, (uint32_t)b.jobs.size() - n_wide, stream, rle, dict, alp));
        WHIP(hipMemcpyAsync(b.h_lens, b.d_lens, b.jobs.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        // the slots come back in one pinned copy (slots are sized for W = T,
        // so this moves more than the chunks hold, but one large copy beats
        // a small copy per chunk); complete() moves each chunk's bytes out
        WHIP(hipMemcpyAsync(b.h_out, b.d_out, b.out_used, hipMemcpyDeviceToHost, stream));
        WHIP(hipEventRecord(b.done, stream));
        b.in_flight = true;
        cur ^= 1;
        if (g_prof.on) g_prof.submit += WriterProfile::now() - t0;
        return 0;
    }

    // Wait for a submitted set and move its chunks into their row groups (on
    // up to nthreads threads); the set is then empty.
    int complete(Set &b, std::vector<FileBuilder::RG> &rgs, int nthreads) {
        const double t0 = g_prof.on ? WriterProfile::now() : 0;
        WHIP(hipEventSynchronize(b.done));
        const double t1 = g_prof.on ? WriterProfile::now() : 0;
        std::atomic<size_t> next{0};
        std::atomic<size_t> empty{SIZE_MAX};  // a job whose chunk came back empty (a kernel that did not write it)
        auto move_out = [&]() {
            for (size_t i; (i = next.fetch_add(1)) < b.jobs.size();) {
                const Job &jb = b.jobs[i];
                std::vector<uint8_t> &dst = rgs[jb.rg].chunks[jb.col];
                const uint64_t len = b.h_lens[i] & ((1ull << kEncShift) - 1);
                const uint8_t enc = (uint8_t)(b.h_lens[i] >> kEncShift);
                if (len == 0 && (enc == ENC_RLE || enc == ENC_DICT)) {
                    // ENC_AUTO chose an encoding the GPU does not write: encode
                    // it here from the staged values (still in this set)
                    std::vector<uint64_t> v(jb.nrows);
                    for (uint32_t r = 0; r < jb.nrows; ++r) v[r] = load_typed(b.h_stage + jb.in_off, jb.T, r);
                    dst = enc == ENC_RLE ? enc_rle(jb.T, v.data(), jb.nrows) : enc_dict_int(jb.T, v.data(), jb.nrows);
                    continue;
                }
                if (len == 0) {
                    empty.store(i);
                    continue;
                }
                dst.assign(b.h_out + jb.out_off, b.h_out + jb.out_off + len);
            }
        };
        std::vector<std::thread> th;
        const size_t nth = std::min<size_t>(b.jobs.size(), (size_t)std::max(1, nthreads));
        for (size_t t = 1; t < nth; ++t) th.emplace_back(move_out);
        move_out();
        for (auto &t : th) t.join();
        // test hook: a set whose first chunk came back empty (the error path)
        if (const char *f = getenv("FLS_TEST_FAIL_GPU_ENCODE"); f && atoi(f) != 0 && !b.jobs.empty()) empty.store(0);
        if (const size_t e = empty.load(); e != SIZE_MAX) {
            const Job &jb = b.jobs[e];
            const int rc = fail(FLS_ERR_DEVICE, "GPU encoder: no chunk for row group %zu column %zu (encoding %u)", jb.rg,
                                jb.col, (unsigned)jb.enc);
            b.jobs.clear();
            b.in_used = b.out_used = 0;
            b.dict_used = 0;
            b.batched = 0;
            b.in_flight = false;
            return rc;
        }
        b.jobs.clear();
        b.in_used = b.out_used = 0;
        b.dict_used = 0;
        b.batched = 0;
        b.in_flight = false;
        if (g_prof.on) {
            g_prof.gpu_wait += t1 - t0;
            g_prof.copy_out += WriterProfile::now() - t1;
            ++g_prof.flushes;
        }
        return 0;
    }

    // Every staged row group encoded and in place (before the file is assembled).
    int finish(std::vector<FileBuilder::RG> &rgs, int nthreads) {
        int rc = submit();
        for (int k = 0; k < 2 && !rc; ++k)
            if (sets[k].in_flight) rc = complete(sets[k], rgs, nthreads);
        return rc;
    }
#undef WHIP
};

// The writer's persistent threads (created per row group before: 15 thread
// starts per 65,536-row group): a FIFO of jobs, each n independent tasks; workers take
// the front job's next task.  run() submits and waits; submit() / wait()
// split it, so a pipelined writer (fls_writer_set_pipelined) lets the next
// call's tasks start while the previous call's last ones finish.  The caller
// of wait() runs its own job's remaining tasks before it sleeps.
class WorkerPool {
public:
    struct Job {
        std::function<void(size_t)> fn;
        size_t n = 0;
        std::atomic<size_t> next{0}, done{0};
    };
    ~WorkerPool() { stop(); }
    // nthreads in total, the calling thread included
    void resize(int nthreads) {
        const size_t want = (size_t)std::max(0, nthreads - 1);
        if (want == th_.size()) return;
        stop();
        quit_ = false;
        for (size_t i = 0; i < want; ++i) th_.emplace_back([this] { loop(); });
    }
    std::shared_ptr<Job> submit(size_t n, std::function<void(size_t)> fn) {
        auto j = std::make_shared<Job>();
        j->fn = std::move(fn);
        j->n = n;
        if (n > 1 && !th_.empty()) {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(j);
            cv_.notify_all();
        }
        return j;
    }
    void wait(const std::shared_ptr<Job> &j) {
        if (!j) return;
        for (size_t i; (i = j->next.fetch_add(1)) < j->n;) finish_task(*j, i);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return j->done.load() == j->n; });
    }
    void run(size_t n, const std::function<void(size_t)> &fn) { wait(submit(n, fn)); }

private:
    void finish_task(Job &j, size_t i) {
        j.fn(i);
        if (j.done.fetch_add(1) + 1 == j.n) {
            std::lock_guard<std::mutex> lk(mu_);
            done_.notify_all();
        }
    }
    void loop() {
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_ || !q_.empty(); });
                if (quit_) return;
                j = q_.front();
                if (j->next.load() >= j->n) {  // every task taken: the job leaves the queue
                    q_.pop_front();
                    continue;
                }
            }
            const size_t i = j->next.fetch_add(1);
            if (i < j->n) finish_task(*j, i);
        }
    }
    void stop() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
        th_.clear();
        q_.clear();
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::deque<std::shared_ptr<Job>> q_;  // jobs with tasks not taken yet
    bool quit_ = false;
};

namespace {
struct RgArgs {
    uint32_t nrows;
    const void *const *data;
    const uint32_t *const *offs;
    const uint64_t *const *valid = nullptr;  // per column: validity words, or NULL (all valid)
};
// A row group being encoded: its chunks, zone maps and bitmaps, the caller's
// columns, and (GPU columns) where its values are staged.
struct PendingRg {
    FileBuilder::RG rg;
    RgArgs in;
    std::vector<uint8_t *> stage;     // GPU columns: where their values go in pinned memory
    std::vector<uint64_t *> est_dict; // GPU ENC_AUTO columns: the host's DICT estimate
};
// A pipelined writer's segment still encoding on the pool after its call
// returned (fls_writer_set_pipelined): appended by the next call or finish.
struct PendingSeg {
    std::vector<PendingRg> seg;
    std::shared_ptr<WorkerPool::Job> job;
    double t0 = 0;
};
}  // namespace

struct fls_writer {
    FileBuilder fb;
    int threads = default_writer_threads();  // (row group, column) tasks run on this many threads
    GpuEncoder gpu;                          // fls_writer_set_device
    FsstGpu fsst_gpu;                        // fls_writer_set_device: FSST chunks compressed on the GPU
    WorkerPool pool;
    // a failure that left work queued for row groups that were dropped (the
    // GPU encoder's batch holds jobs indexed by them): every later add or
    // finish fails with this instead of completing those jobs
    int broken = 0;
    std::string broken_msg;
    bool pipelined = false;                  // fls_writer_set_pipelined
    std::unique_ptr<PendingSeg> pend;        // pipelined: the last call's segment, still encoding
    ~fls_writer() {
        if (pend) pool.wait(pend->job);      // its tasks read the caller's buffers and our row groups
    }
};

namespace {
// a segment's tasks done: its row groups appended in order (none when a GPU
// FSST compression failed; the caller reports that, seg_failed / finish_writer)
void append_segment(fls_writer *w, std::unique_ptr<PendingSeg> ps) {
    if (!ps) return;
    w->pool.wait(ps->job);
    if (w->fsst_gpu.err.load()) return;
    for (PendingRg &p : ps->seg) w->fb.rgs.push_back(std::move(p.rg));
    if (g_prof.on) g_prof.cpu += WriterProfile::now() - ps->t0;
}
// the last call's segment of a pipelined writer, and its FSST failure if any
int drain_pending(fls_writer *w) {
    append_segment(w, std::move(w->pend));
    if (const int rc = w->fsst_gpu.err.exchange(0)) {
        w->broken = rc;
        w->broken_msg = w->fsst_gpu.err_msg;
        return fail(rc, "%s", w->fsst_gpu.err_msg.c_str());
    }
    return 0;
}
}  // namespace

extern "C" {

fls_writer *fls_writer_new(uint64_t row_offset) {
    auto *w = new fls_writer();
    w->fb.row_offset = row_offset;
    g_prof.on = g_str_prof_on = getenv("FLS_WRITER_PROFILE") != nullptr;  // (profiles the writers made from here on)
    return w;
}

void fls_writer_free(fls_writer *w) { delete w; }

int fls_writer_add_column(fls_writer *w, const char *name, uint8_t type, uint8_t width, uint8_t scale,
                          uint8_t encoding) {
    if (!w || !name) return fail(FLS_ERR_ARG, "fls_writer_add_column: NULL argument");
    if (!type_valid(type)) return fail(FLS_ERR_ARG, "fls_writer_add_column: unsupported type %u", type);
    if (encoding > ENC_FSST || encoding == 6) return fail(FLS_ERR_ARG, "fls_writer_add_column: bad encoding %u", encoding);
    if (type_is_string(type) && encoding != ENC_AUTO && encoding != ENC_DICT && encoding != ENC_FSST)
        return fail(FLS_ERR_ARG, "fls_writer_add_column: VARCHAR/BLOB support DICT and FSST");
    if (type_is_float(type) && encoding != ENC_AUTO && encoding != ENC_ALP)
        return fail(FLS_ERR_ARG, "fls_writer_add_column: FLOAT/DOUBLE support ALP");
    if (!type_is_float(type) && encoding == ENC_ALP)
        return fail(FLS_ERR_ARG, "fls_writer_add_column: ALP needs FLOAT/DOUBLE");
    if (!type_is_string(type) && encoding == ENC_FSST)
        return fail(FLS_ERR_ARG, "fls_writer_add_column: FSST needs VARCHAR/BLOB");
    if (!w->fb.rgs.empty()) return fail(FLS_ERR_STATE, "fls_writer_add_column: after first row group");
    if (strlen(name) > 65535) return fail(FLS_ERR_ARG, "column name too long");
    w->fb.cols.push_back(ColSpec{name, type, width, scale, encoding});
    return 0;
}

}  // extern "C"

namespace {

// The chunk bitmaps of n rows from the caller's validity words (bits past n
// cleared); false when every row is valid.  nnull: NULL rows.
bool chunk_validity(const uint64_t *in, uint32_t n, std::vector<uint64_t> &w, uint32_t &nnull) {
    nnull = 0;
    if (!in) return false;
    const uint32_t nw = (n + 63) / 64;
    for (uint32_t j = 0; j < nw; ++j) {
        const uint32_t r0 = 64 * j;
        const uint64_t live = n - r0 >= 64 ? ~0ull : ((1ull << (n - r0)) - 1);
        nnull += (uint32_t)__builtin_popcountll(~in[j] & live);
    }
    if (!nnull) return false;
    w.assign(16ull * ((n + kVectorSize - 1) / kVectorSize), 0);
    for (uint32_t j = 0; j < nw; ++j) {
        const uint32_t r0 = 64 * j;
        w[j] = in[j] & (n - r0 >= 64 ? ~0ull : ((1ull << (n - r0)) - 1));
    }
    return true;
}
inline bool row_valid(const std::vector<uint64_t> &w, uint32_t i) { return (w[i / 64] >> (i % 64)) & 1; }

// Placeholders at NULL rows (fls_format.hpp): the previous valid value, the
// first valid one for leading NULLs, 0 when every row is NULL; w bytes each.
void fill_nulls(uint8_t *vals, uint32_t w, uint32_t n, const std::vector<uint64_t> &valid) {
    uint32_t first = 0;
    while (first < n && !row_valid(valid, first)) ++first;
    if (first == n) {
        memset(vals, 0, (size_t)n * w);
        return;
    }
    for (uint32_t i = 0; i < first; ++i) memcpy(vals + (size_t)i * w, vals + (size_t)first * w, w);
    for (uint32_t i = first + 1; i < n; ++i)
        if (!row_valid(valid, i)) memcpy(vals + (size_t)i * w, vals + (size_t)(i - 1) * w, w);
}

// Append row groups a[0..nrg): every (row group, column) chunk is an
// independent task on the writer's threads, VARCHAR chunks (the slowest) first,
// so a row group's slowest column no longer idles the other threads.  With a
// GPU (fls_writer_set_device) the integer columns are staged into the GPU
// encoder's current batch by the same tasks; the row groups go in in segments
// that end where the batch is full or out of room, since a batch is only
// submitted once every row group in it is staged.
int add_rowgroups_impl(fls_writer *w, uint32_t nrg, const RgArgs *a) {
    // a pipelined writer's previous call is done when this one returns with
    // an error (its caller may then free that call's buffers)
    struct SettleOnError {
        fls_writer *w;
        bool ok = false;
        ~SettleOnError() {
            if (!ok && w->pend) append_segment(w, std::move(w->pend));
        }
    } settle{w};
    if (w->fb.cols.empty()) return fail(FLS_ERR_STATE, "no columns");
    if (w->broken) return fail(FLS_ERR_STATE, "writer failed earlier: %s", w->broken_msg.c_str());
    const size_t ncols = w->fb.cols.size();
    const uint32_t rgsz = w->fb.rowgroup_size;
    // row groups so far, a pipelined writer's pending segment included
    const size_t nprev = w->fb.rgs.size() + (w->pend ? w->pend->seg.size() : 0);
    const uint32_t last_rows = w->pend ? w->pend->seg.back().rg.nrows : nprev ? w->fb.rgs.back().nrows : rgsz;
    // validate every row group before any is added
    for (uint32_t k = 0; k < nrg; ++k) {
        const uint32_t nrows = a[k].nrows;
        if (nrows == 0 || nrows > rgsz) return fail(FLS_ERR_ARG, "row group needs 1..%u rows, got %u", rgsz, nrows);
        const bool prev_short = (k == 0 ? last_rows : a[k - 1].nrows) != rgsz;
        if (prev_short) return fail(FLS_ERR_STATE, "only the last row group may be short");
        if (!a[k].data) return fail(FLS_ERR_ARG, "fls_writer_add_rowgroup: NULL argument");
        // test hook: fail the call that would add row group k (error paths of callers)
        if (const char *f = getenv("FLS_TEST_FAIL_WRITER_RG"))
            if (nprev + k == (size_t)atoi(f)) return fail(FLS_ERR_STATE, "injected writer failure at row group %s", f);
        for (size_t c = 0; c < ncols; ++c) {
            const ColSpec &cs = w->fb.cols[c];
            if (!a[k].data[c]) return fail(FLS_ERR_ARG, "column %zu: NULL data", c);
            if (type_is_string(cs.type)) {
                if (!a[k].offs || !a[k].offs[c]) return fail(FLS_ERR_ARG, "column %zu: VARCHAR needs offsets", c);
                const uint32_t *o = a[k].offs[c];
                for (uint32_t i = 0; i < nrows; ++i)
                    if (o[i + 1] < o[i]) return fail(FLS_ERR_ARG, "column %zu: offsets not monotone", c);
            }
            if (cs.type == TY_BOOLEAN) {  // DuckDB's bool bytes: 0 or 1
                const uint8_t *b = (const uint8_t *)a[k].data[c];
                uint8_t any = 0;
                for (uint32_t i = 0; i < nrows; ++i) any |= b[i];
                if (any > 1) return fail(FLS_ERR_ARG, "column %zu: BOOLEAN bytes must be 0 or 1", c);
            }
        }
    }
    // GPU-encoded columns (fls_writer_set_device): integer FFOR / DELTA / RLE /
    // DICT / AUTO, FLOAT / DOUBLE (ALP)
    std::vector<size_t> gcols;
    if (w->gpu.dev >= 0)
        for (size_t c = 0; c < ncols; ++c) {
            const ColSpec &cs = w->fb.cols[c];
            if (type_is_float(cs.type)) {
                if (GpuEncoder::alp_gpu()) gcols.push_back(c);
            } else if (!type_is_string(cs.type) &&
                       (cs.enc == ENC_FFOR || cs.enc == ENC_DELTA || cs.enc == ENC_RLE || cs.enc == ENC_AUTO ||
                        (cs.enc == ENC_DICT && GpuEncoder::dict_gpu()))) {
                gcols.push_back(c);
            }
        }
    std::vector<uint8_t> on_gpu(ncols, 0);
    for (size_t c : gcols) on_gpu[c] = 1;
    w->pool.resize(w->threads);
    // FSST chunks compressed on the GPU (FLS_WRITER_FSST_GPU=0: on the host)
    FsstGpu *fsst_gpu = w->fsst_gpu.dev >= 0 && knob_value("FLS_WRITER_FSST_GPU") != 0 ? &w->fsst_gpu : nullptr;

    using Pending = PendingRg;
    std::vector<Pending> seg;
    // (by value: a pipelined call's tasks outlive this call)
    auto encode_col = [w, on_gpu, fsst_gpu](Pending &p, size_t c) {
        const ColSpec &cs = w->fb.cols[c];
        const uint32_t nrows = p.in.nrows;
        const void *data = p.in.data[c];
        // NULLs: the chunk's bitmaps, placeholders at the NULL rows, zone-map flags
        uint32_t nnull = 0;
        const bool nulls = chunk_validity(p.in.valid ? p.in.valid[c] : nullptr, nrows, p.rg.valid[c], nnull);
        const std::vector<uint64_t> &vw = p.rg.valid[c];
        auto null_flags = [&](ZoneMap &z) {
            if (!nulls) return;
            z.flags |= ZM_HAS_NULL;
            if (nnull == nrows) z = ZoneMap{0, 0, ZM_HAS_NULL | ZM_ALL_NULL, 0};
        };
        if (type_is_string(cs.type)) {
            if (!nulls) {
                p.rg.chunks[c] = encode_str_chunk(cs.enc, p.in.offs[c], (const char *)data, nrows, fsst_gpu);
                return;
            }
            // NULL rows as empty strings
            const uint32_t *o = p.in.offs[c];
            std::vector<uint32_t> no(nrows + 1, 0);
            std::string bytes;
            for (uint32_t i = 0; i < nrows; ++i) {
                if (row_valid(vw, i)) bytes.append((const char *)data + o[i], o[i + 1] - o[i]);
                no[i + 1] = (uint32_t)bytes.size();
            }
            p.rg.chunks[c] = encode_str_chunk(cs.enc, no.data(), bytes.data(), nrows, fsst_gpu);
            null_flags(p.rg.zones[c]);
            return;
        }
        const uint32_t vbytes = type_value_bits(cs.type) / 8;
        if (on_gpu[c]) {  // encoded by the GPU batch: staging copy and zone map here
            memcpy(p.stage[c], data, (size_t)nrows * vbytes);
            if (nulls) fill_nulls(p.stage[c], vbytes, nrows, vw);
            p.rg.zones[c] = zone_of_typed(cs.type, p.stage[c], nrows);
            null_flags(p.rg.zones[c]);
            if (cs.enc == ENC_AUTO && !type_is_float(cs.type)) {
                if (GpuEncoder::dict_gpu()) {  // dict_analyze_kernel makes the DICT estimate
                    *p.est_dict[c] = kEstDictGpu;
                } else {                       // the host's (FLS_WRITER_DICT_GPU=0)
                    const size_t d = est_dict_typed(type_value_bits(cs.type), p.stage[c], nrows);
                    *p.est_dict[c] = d == SIZE_MAX ? UINT64_MAX : (uint64_t)d;
                }
            }
            return;
        }
        const int T = type_value_bits(cs.type);
        std::vector<uint64_t> v(nrows);
        const uint8_t *src = (const uint8_t *)data;
        for (uint32_t i = 0; i < nrows; ++i) {
            uint64_t x = 0;
            memcpy(&x, src + (size_t)i * (T / 8), T / 8);
            v[i] = x;
        }
        if (nulls) fill_nulls((uint8_t *)v.data(), 8, nrows, vw);
        p.rg.chunks[c] = encode_int_chunk(cs.type, cs.enc, v.data(), nrows);
        p.rg.zones[c] = zone_of(cs.type, v.data(), nrows);
        null_flags(p.rg.zones[c]);
    };
    // encode the segment's chunks (submitted to the pool), then append its
    // row groups in order; a pipelined writer leaves the call's last segment
    // encoding (w->pend) and appends it at the start of the next call
    auto start_seg = [&]() -> std::unique_ptr<PendingSeg> {
        if (seg.empty()) return nullptr;
        auto ps = std::make_unique<PendingSeg>();
        ps->t0 = g_prof.on ? WriterProfile::now() : 0;
        ps->seg = std::move(seg);
        seg.clear();
        std::vector<std::pair<uint32_t, uint32_t>> tasks;  // (row group in segment, column)
        tasks.reserve(ps->seg.size() * ncols);
        for (int pass = 0; pass < 2; ++pass)
            for (uint32_t k = 0; k < ps->seg.size(); ++k)
                for (uint32_t c = 0; c < ncols; ++c)
                    if ((type_is_string(w->fb.cols[c].type)) == (pass == 0)) tasks.emplace_back(k, c);
        PendingSeg *pp = ps.get();
        ps->job = w->pool.submit(tasks.size(), [pp, tasks, encode_col](size_t t) {
            encode_col(pp->seg[tasks[t].first], tasks[t].second);
        });
        return ps;
    };
    auto finish_pend = [&]() { append_segment(w, std::move(w->pend)); };
    auto run_seg = [&]() {
        finish_pend();
        append_segment(w, start_seg());
    };
    // a GPU FSST compression that failed in the last segment
    // The segment's row groups were dropped, but the GPU encoder's current
    // batch (and a set in flight) may hold jobs indexed by them: the writer is
    // marked failed, so no later call completes those jobs into row groups
    // that do not exist (or into the wrong ones).
    auto seg_failed = [&]() -> int {
        if (!fsst_gpu || !fsst_gpu->err.load()) return 0;
        const int rc = fsst_gpu->err.exchange(0);
        w->broken = rc;
        w->broken_msg = fsst_gpu->err_msg;
        return fail(rc, "%s", fsst_gpu->err_msg.c_str());
    };
    // a GPU encoder failure (a set that did not come back whole) leaves row
    // groups without some of their chunks: the writer is failed from here on
    auto gpu_failed = [&](int rc) -> int {
        w->broken = rc;
        w->broken_msg = fls_last_error();
        return rc;
    };
    seg.reserve(nrg);
    for (uint32_t k = 0; k < nrg; ++k) {
        Pending p;
        p.in = a[k];
        p.rg.nrows = a[k].nrows;
        p.rg.chunks.resize(ncols);
        p.rg.zones.assign(ncols, ZoneMap{0, 0, 0, 0});
        p.rg.valid.assign(ncols, {});
        p.stage.assign(ncols, nullptr);
        p.est_dict.assign(ncols, nullptr);
        if (!gcols.empty()) {
            // room in the batch now; the values are staged by the tasks (the
            // caller's buffers are only valid during this call)
            if (!w->gpu.has_room(w->fb.cols, gcols, a[k].nrows)) run_seg();
            if (const int rc = seg_failed()) return rc;
            // (its position in the file: a pending segment's row groups are
            // appended before any set holding them is submitted -- run_seg
            // before every submit, drain_pending before gpu.finish -- so a
            // completing set only touches row groups already in rgs)
            const size_t at = w->fb.rgs.size() + (w->pend ? w->pend->seg.size() : 0) + seg.size();
            const int rc = w->gpu.add(w->fb.cols, gcols, at, a[k].nrows, w->threads, w->fb.rgs, p.stage, p.est_dict);
            if (rc) {
                run_seg();
                return gpu_failed(rc);
            }
        }
        seg.push_back(std::move(p));
        // a full batch is encoded once its last row group is in place
        if (w->gpu.dev >= 0 && w->gpu.full()) {
            run_seg();
            if (const int rc = seg_failed()) return rc;
            const int rc = w->gpu.submit();
            if (rc) return gpu_failed(rc);
        }
    }
    if (w->pipelined) {
        // the previous call's segment first (row groups stay in call order),
        // this one's tasks already queued behind it
        auto mine = start_seg();
        finish_pend();
        w->pend = std::move(mine);
    } else {
        run_seg();
    }
    if (const int rc = seg_failed()) return rc;
    const int rc = w->fb.flush_stream(false);  // streamed output: the complete row groups go to the file
    settle.ok = rc == 0;
    return rc;
}
}  // namespace

extern "C" {

int fls_writer_add_rowgroup(fls_writer *w, uint32_t nrows, const void *const *data,
                            const uint32_t *const *str_offsets) {
    if (!w || !data) return fail(FLS_ERR_ARG, "fls_writer_add_rowgroup: NULL argument");
    const RgArgs a{nrows, data, str_offsets};
    return add_rowgroups_impl(w, 1, &a);
}

int fls_writer_add_rowgroups(fls_writer *w, uint32_t nrg, const uint32_t *nrows, const void *const *data,
                             const uint32_t *const *str_offsets) {
    return fls_writer_add_rowgroups_v(w, nrg, nrows, data, str_offsets, nullptr);
}

int fls_writer_add_rowgroups_v(fls_writer *w, uint32_t nrg, const uint32_t *nrows, const void *const *data,
                               const uint32_t *const *str_offsets, const uint64_t *const *validity) {
    if (!w || !nrows || !data) return fail(FLS_ERR_ARG, "fls_writer_add_rowgroups: NULL argument");
    const size_t ncols = w->fb.cols.size();
    std::vector<RgArgs> a(nrg);
    for (uint32_t k = 0; k < nrg; ++k)
        a[k] = RgArgs{nrows[k], data + k * ncols, str_offsets ? str_offsets + k * ncols : nullptr,
                      validity ? validity + k * ncols : nullptr};
    return add_rowgroups_impl(w, nrg, a.data());
}

int fls_writer_set_threads(fls_writer *w, int nthreads) {
    if (!w) return fail(FLS_ERR_ARG, "fls_writer_set_threads: NULL writer");
    w->threads = nthreads > 0 ? nthreads : default_writer_threads();
    return 0;
}

int fls_writer_set_device(fls_writer *w, int device) {
    if (!w) return fail(FLS_ERR_ARG, "fls_writer_set_device: NULL writer");
    if (const int rc = drain_pending(w)) return rc;  // (its FSST chunks may be on the old device)
    w->gpu.release();
    w->gpu.dev = -1;
    w->fsst_gpu.release();
    w->fsst_gpu.dev = -1;
    if (device < 0) return 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device >= n)
        return fail(FLS_ERR_DEVICE, "fls_writer_set_device: no GPU %d (%d visible)", device, n);
    w->gpu.dev = device;
    w->fsst_gpu.dev = device;
    return 0;
}

int fls_writer_set_rowgroup_size(fls_writer *w, uint32_t rows) {
    if (!w) return fail(FLS_ERR_ARG, "fls_writer_set_rowgroup_size: NULL writer");
    if (rows == 0 || rows > kRowGroupSize || rows % kVectorSize)
        return fail(FLS_ERR_ARG, "row group size must be a multiple of %u in [%u, %u], got %u", kVectorSize, kVectorSize,
                    kRowGroupSize, rows);
    if (!w->fb.rgs.empty() || w->pend) return fail(FLS_ERR_STATE, "fls_writer_set_rowgroup_size: after first row group");
    w->fb.rowgroup_size = rows;
    return 0;
}

namespace {
// the image (img) or the file (path): the GPU encoder's last batch completed,
// then the row groups assembled
int finish_writer(fls_writer *w, uint8_t **img, uint64_t *len, const char *path) {
    if (w->fb.cols.empty()) return fail(FLS_ERR_STATE, "no columns");
    if (w->broken) return fail(FLS_ERR_STATE, "writer failed earlier: %s", w->broken_msg.c_str());
    if (const int rc = drain_pending(w)) return rc;
    if (w->gpu.dev >= 0) {
        const int rc = w->gpu.finish(w->fb.rgs, w->threads);
        if (rc) {  // row groups without some of their chunks: no file from this writer
            w->broken = rc;
            w->broken_msg = fls_last_error();
            return rc;
        }
    }
    const double tf = g_prof.on ? WriterProfile::now() : 0;
    if (w->fb.out && !path) return fail(FLS_ERR_STATE, "fls_writer_finish_image: the writer streams to a file");
    const bool streaming = w->fb.out != nullptr;
    const int rc = streaming ? w->fb.finish_stream(path)
                   : path    ? w->fb.write_file(path, w->threads)
                             : w->fb.finish(img, len, w->threads);
    if (rc && streaming) {
        // row groups handed to the stream gave their chunk bytes away (flen
        // set, chunks empty): a later finish would write blank chunks under a
        // valid footer, so this writer makes no file any more
        bool handed = false;
        for (const auto &r : w->fb.rgs) handed = handed || !r.flen.empty();
        if (handed) {
            w->broken = rc;
            w->broken_msg = fls_last_error();
        }
    }
    if (g_prof.on) {
        g_prof.finish += WriterProfile::now() - tf;
        g_prof.print();
        g_prof = WriterProfile();
        g_str_prof.dict_ns = g_str_prof.table_ns = g_str_prof.compress_ns = g_str_prof.chunks = 0;
    }
    return rc;
}
}  // namespace

int fls_writer_finish_image(fls_writer *w, uint8_t **img, uint64_t *len) {
    if (!w || !img || !len) return fail(FLS_ERR_ARG, "fls_writer_finish_image: NULL argument");
    return finish_writer(w, img, len, nullptr);
}

int fls_writer_set_pipelined(fls_writer *w, int on) {
    if (!w) return fail(FLS_ERR_ARG, "fls_writer_set_pipelined: NULL writer");
    if (!on)
        if (const int rc = drain_pending(w)) return rc;
    w->pipelined = on != 0;
    return 0;
}

int fls_writer_set_output(fls_writer *w, const char *path) {
    if (!w || !path) return fail(FLS_ERR_ARG, "fls_writer_set_output: NULL argument");
    return w->fb.open_stream(path);
}

int fls_writer_finish_file(fls_writer *w, const char *path) {
    if (!w || !path) return fail(FLS_ERR_ARG, "fls_writer_finish_file: NULL argument");
    return finish_writer(w, nullptr, nullptr, path);
}

void fls_image_free(uint8_t *img) { free(img); }

int64_t fls_gen_nrows(const char *workload, double scale, uint64_t nrows) {
    Workload w;
    if (!make_workload(workload, scale, nrows, w)) return fail(FLS_ERR_ARG, "unknown workload '%s'", workload ? workload : "(null)");
    return (int64_t)w.nrows;
}

int fls_gen_ncols(const char *workload) {
    Workload w;
    if (!make_workload(workload, 1.0, 0, w)) return fail(FLS_ERR_ARG, "unknown workload '%s'", workload ? workload : "(null)");
    return (int)w.cols.size();
}

int fls_gen_image(const char *workload, double scale, uint64_t nrows, uint32_t rg_begin, uint32_t rg_end,
                  int nthreads, uint8_t **img, uint64_t *len) {
    Workload w;
    if (!make_workload(workload, scale, nrows, w)) return fail(FLS_ERR_ARG, "unknown workload '%s'", workload ? workload : "(null)");
    const uint64_t nrg_total = (w.nrows + kRowGroupSize - 1) / kRowGroupSize;
    if (rg_end > nrg_total) rg_end = (uint32_t)nrg_total;
    if (rg_begin > rg_end || !img || !len) return fail(FLS_ERR_ARG, "bad row-group range [%u,%u)", rg_begin, rg_end);
    if (nthreads < 1) nthreads = 1;
    FileBuilder fb;
    fb.cols = w.cols;
    fb.row_offset = (uint64_t)rg_begin * kRowGroupSize;
    fb.rgs.resize(rg_end - rg_begin);
    std::atomic<uint32_t> next{rg_begin};
    auto work = [&]() {
        std::vector<std::vector<uint64_t>> vals;
        for (uint32_t rg; (rg = next.fetch_add(1)) < rg_end;) {
            const uint64_t r0 = (uint64_t)rg * kRowGroupSize;
            const uint32_t n = (uint32_t)std::min<uint64_t>(kRowGroupSize, w.nrows - r0);
            gen_rows(w, r0, n, vals);
            auto &out = fb.rgs[rg - rg_begin];
            out.nrows = n;
            out.chunks.resize(w.cols.size());
            out.zones.assign(w.cols.size(), ZoneMap{0, 0, 0, 0});
            for (size_t c = 0; c < w.cols.size(); ++c)
                out.chunks[c] = encode_gen_chunk(w, (int)c, vals[c], &out.zones[c]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    return fb.finish(img, len, nthreads);
}

int fls_gen_values(const char *workload, double scale, uint64_t nrows, int col, uint64_t row_begin, uint64_t n,
                   void *out) {
    Workload w;
    if (!make_workload(workload, scale, nrows, w)) return fail(FLS_ERR_ARG, "unknown workload '%s'", workload ? workload : "(null)");
    if (col < 0 || col >= (int)w.cols.size() || !out) return fail(FLS_ERR_ARG, "bad column %d", col);
    if (col == w.comment_col) return fail(FLS_ERR_ARG, "column %d holds strings: use fls_gen_strings", col);
    if (row_begin + n > w.nrows) return fail(FLS_ERR_ARG, "rows out of range");
    const int vb = type_is_string(w.cols[col].type) ? 4 : type_value_bits(w.cols[col].type) / 8;
    std::vector<std::vector<uint64_t>> vals;
    uint8_t *o = (uint8_t *)out;
    for (uint64_t r = 0; r < n;) {
        const uint32_t k = (uint32_t)std::min<uint64_t>(65536, n - r);
        gen_rows(w, row_begin + r, k, vals);
        for (uint32_t i = 0; i < k; ++i) memcpy(o + (r + i) * vb, &vals[col][i], vb);
        r += k;
    }
    return 0;
}

int64_t fls_gen_strings(const char *workload, double scale, uint64_t nrows, int col, uint64_t row_begin, uint64_t n,
                        uint32_t *offs, char *bytes, uint64_t cap) {
    Workload w;
    if (!make_workload(workload, scale, nrows, w)) return fail(FLS_ERR_ARG, "unknown workload '%s'", workload ? workload : "(null)");
    if (col < 0 || col >= (int)w.cols.size() || !type_is_string(w.cols[col].type) || !offs)
        return fail(FLS_ERR_ARG, "column %d is not a VARCHAR column", col);
    if (row_begin + n > w.nrows) return fail(FLS_ERR_ARG, "rows out of range");
    uint64_t o = 0;
    offs[0] = 0;
    std::vector<std::vector<uint64_t>> vals;
    std::vector<std::string_view> dict;
    const bool is_dict = col != w.comment_col && gen_dict(w, col, dict);
    for (uint64_t r = 0; r < n;) {
        const uint32_t k = (uint32_t)std::min<uint64_t>(65536, n - r);
        if (is_dict) gen_rows(w, row_begin + r, k, vals);
        for (uint32_t i = 0; i < k; ++i) {
            const std::string_view sv = is_dict ? dict[vals[col][i]] : gen::comment(w.li.seed, row_begin + r + i);
            if (o + sv.size() > cap || o + sv.size() > UINT32_MAX) return fail(FLS_ERR_ARG, "string buffer too small");
            if (bytes) memcpy(bytes + o, sv.data(), sv.size());
            o += sv.size();
            offs[r + i + 1] = (uint32_t)o;
        }
        r += k;
    }
    return (int64_t)o;
}

const char *fls_gen_dict_string(const char *workload, int col, uint32_t code) {
    Workload w;
    if (!make_workload(workload, 1.0, 0, w)) return nullptr;
    static thread_local std::vector<std::string_view> d;
    if (!gen_dict(w, col, d) || code >= d.size()) return nullptr;
    return d[code].data();  // entries are NUL-terminated literals
}

}  // extern "C"
