/*
 * flsref.c -- CPU restatement of the FastLanes decode path (ORACLE).
 *
 * TEST INFRASTRUCTURE ONLY -- see flsref.h for who may call this and why
 * parity with upstream cwida/FastLanes bytes is UNPINNED.
 *
 * The algorithm follows the FastLanes paper (VLDB 2023) as used by the
 * reference's decode call RowgroupReader::materialize()
 * (src/fastlanes_facade.cpp:48) and its per-type consumers
 * (src/fastlanes_facade.cpp:125-172):
 *   - 1024-value vectors, T-bit "virtual lanes" (1024/T lanes of T rows);
 *   - interleaved bit-packing: lane L's W-bit values are concatenated into W
 *     T-bit words; word k of lane L is stored at word index k*(1024/T)+L;
 *   - FFOR: value = base + unpacked (wrapping T-bit);
 *   - DELTA over the unified transposed layout (FL_ORDER 0,4,2,6,1,5,3,7):
 *     each lane holds one chain of T tuples at stride 16 inside a block of
 *     16*T tuples; value = lane base + running sum of deltas;
 *   - DICT: value = dict[base + unpacked code];
 *   - RLE (FastLanes-RLE): run index vector decoded as DELTA(T=16), then
 *     value = run_values[index];
 *   - ALP (Afroozeh, Kuffo, Boncz, SIGMOD 2024) for FLOAT/DOUBLE: the FFOR
 *     stream holds integers d, value = (F)d * 10^f * 10^-e, then exceptions
 *     (position, original value) are patched in;
 *   - FSST (Boncz, Neumann, Leis, VLDB 2020) for VARCHAR: a string is a run
 *     of byte codes, code c < 255 expands to symbol[c] (1..8 bytes), code 255
 *     is followed by one literal byte; every string is compressed on its
 *     own and a vector stores its strings' compressed lengths (FFOR), so the
 *     checker expands and bounds-checks string by string.
 * It is written as plain scalar loops on purpose: it is the checker, not the
 * thing measured (besides the cpu_baseline leg of bench.py).
 */
#include "flsref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t FL_ORDER[8] = {0, 4, 2, 6, 1, 5, 3, 7};

enum { ENC_FFOR = 1, ENC_DELTA = 2, ENC_DICT = 3, ENC_RLE = 4, ENC_ALP = 5, ENC_FSST = 7 };
enum {
    TY_INT8 = 1, TY_INT16 = 2, TY_INT32 = 3, TY_INT64 = 4,
    TY_UINT8 = 5, TY_UINT16 = 6, TY_UINT32 = 7, TY_UINT64 = 8, TY_BOOLEAN = 9,
    TY_DATE = 10, TY_DECIMAL = 11, TY_FLOAT = 12, TY_DOUBLE = 13, TY_VARCHAR = 20, TY_BLOB = 21
};

/* ALP: 10^i and the nearest binary64/binary32 to 10^-i */
static const double ALP_F10_D[19] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10,
                                     1e11, 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18};
static const double ALP_IF10_D[19] = {1e-0, 1e-1, 1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7, 1e-8, 1e-9, 1e-10,
                                      1e-11, 1e-12, 1e-13, 1e-14, 1e-15, 1e-16, 1e-17, 1e-18};
static const float ALP_F10_F[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
static const float ALP_IF10_F[11] = {1e-0f, 1e-1f, 1e-2f, 1e-3f, 1e-4f, 1e-5f, 1e-6f, 1e-7f, 1e-8f, 1e-9f, 1e-10f};

/* little-endian readers; the image is not necessarily aligned for us */
static uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

static uint64_t mask_bits(int w) { return w >= 64 ? ~0ULL : ((1ULL << w) - 1ULL); }

uint32_t flsref_tau(uint32_t p)
{
    uint32_t a = (p >> 7) & 7, b = (p >> 4) & 7, l = p & 15;
    return 128u * FL_ORDER[b] + 16u * a + l;
}

/* read T-bit word number `idx` (0-based, in units of T bits) */
static uint64_t rd_word(int T, const uint8_t *packed, uint64_t idx)
{
    const uint8_t *p = packed + idx * (uint64_t)(T / 8);
    switch (T) {
    case 8: return p[0];
    case 16: return rd16(p);
    case 32: return rd32(p);
    default: return rd64(p);
    }
}

static void wr_word(int T, uint8_t *packed, uint64_t idx, uint64_t v)
{
    uint8_t *p = packed + idx * (uint64_t)(T / 8);
    switch (T) {
    case 8: p[0] = (uint8_t)v; break;
    case 16: { uint16_t x = (uint16_t)v; memcpy(p, &x, 2); } break;
    case 32: { uint32_t x = (uint32_t)v; memcpy(p, &x, 4); } break;
    default: memcpy(p, &v, 8); break;
    }
}

void flsref_unpack(int T, int W, const void *packed_v, uint64_t *out)
{
    const uint8_t *packed = (const uint8_t *)packed_v;
    const int lanes = 1024 / T;
    const uint64_t m = mask_bits(W);
    for (int lane = 0; lane < lanes; ++lane) {
        for (int row = 0; row < T; ++row) {
            uint64_t v = 0;
            if (W > 0) {
                /* bit offset of this row inside the lane's concatenated stream */
                uint64_t bit = (uint64_t)row * (uint64_t)W;
                uint64_t k = bit / (uint64_t)T;
                int s = (int)(bit % (uint64_t)T);
                uint64_t lo = rd_word(T, packed, k * lanes + lane);
                v = lo >> s;
                if (s + W > T) {
                    uint64_t hi = rd_word(T, packed, (k + 1) * lanes + lane);
                    v |= hi << (T - s);
                }
                v &= m;
            }
            out[row * lanes + lane] = v;
        }
    }
}

void flsref_pack(int T, int W, const uint64_t *in, void *packed_v)
{
    uint8_t *packed = (uint8_t *)packed_v;
    const int lanes = 1024 / T;
    const uint64_t m = mask_bits(W);
    const uint64_t tmask = mask_bits(T);
    memset(packed, 0, (size_t)128 * W);
    for (int lane = 0; lane < lanes; ++lane) {
        for (int row = 0; row < T; ++row) {
            if (W == 0) continue;
            uint64_t v = in[row * lanes + lane] & m;
            uint64_t bit = (uint64_t)row * (uint64_t)W;
            uint64_t k = bit / (uint64_t)T;
            int s = (int)(bit % (uint64_t)T);
            uint64_t lo = rd_word(T, packed, k * lanes + lane);
            lo |= (v << s) & tmask;
            wr_word(T, packed, k * lanes + lane, lo);
            if (s + W > T) {
                uint64_t hi = rd_word(T, packed, (k + 1) * lanes + lane);
                hi |= (v >> (T - s)) & tmask;
                wr_word(T, packed, (k + 1) * lanes + lane, hi);
            }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* container                                                                 */

int flsref_open(const void *img_v, size_t len, flsref_file *f)
{
    const uint8_t *img = (const uint8_t *)img_v;
    memset(f, 0, sizeof(*f));
    if (len < 32 || memcmp(img, "FLSAMD01", 8) != 0) return -1;
    if (memcmp(img + len - 4, "FLSF", 4) != 0) return -2;
    uint64_t foff = rd64(img + len - 16);
    uint32_t flen = rd32(img + len - 8);
    if (foff + flen + 16 > len) return -3;
    const uint8_t *p = img + foff;
    if (rd32(p) != 1) return -4;
    f->img = img;
    f->len = len;
    f->ncols = rd32(p + 4);
    f->nrows = rd64(p + 8);
    f->nrowgroups = rd32(p + 16);
    f->rowgroup_size = rd32(p + 20);
    f->row_offset = rd64(p + 24);
    f->footer = p;
    f->footer_len = flen;
    return 0;
}

/* walk the footer: column descriptors start at byte 32 */
static const uint8_t *col_desc(const flsref_file *f, uint32_t col)
{
    const uint8_t *p = f->footer + 32;
    for (uint32_t c = 0; c < col; ++c) p += 6 + rd16(p + 4);
    return p;
}

static const uint8_t *rg_desc(const flsref_file *f, uint32_t rg)
{
    const uint8_t *p = col_desc(f, f->ncols);
    return p + (size_t)rg * (4 + 16 * (size_t)f->ncols);
}

int flsref_column(const flsref_file *f, uint32_t col, int *type, int *width,
                  int *scale, const char **name, int *name_len)
{
    if (col >= f->ncols) return -1;
    const uint8_t *p = col_desc(f, col);
    *type = p[0];
    *width = p[1];
    *scale = p[2];
    *name_len = rd16(p + 4);
    *name = (const char *)(p + 6);
    return 0;
}

int64_t flsref_rowgroup_rows(const flsref_file *f, uint32_t rg)
{
    if (rg >= f->nrowgroups) return -1;
    return rd32(rg_desc(f, rg));
}

static int value_bytes(int type)
{
    switch (type) {
    case TY_INT8: case TY_UINT8: case TY_BOOLEAN: return 1;
    case TY_INT16: case TY_UINT16: return 2;
    case TY_INT32: case TY_UINT32: case TY_DATE: case TY_FLOAT: return 4;
    case TY_INT64: case TY_UINT64: case TY_DECIMAL: case TY_DOUBLE: return 8;
    case TY_VARCHAR: case TY_BLOB: return 16;
    default: return 0;
    }
}

int flsref_out_width(const flsref_file *f, uint32_t col)
{
    int type, w, s, nl;
    const char *n;
    if (flsref_column(f, col, &type, &w, &s, &n, &nl)) return 0;
    return value_bytes(type);
}

static void store_val(uint8_t *out, int vb, uint64_t idx, uint64_t v)
{
    switch (vb) {
    case 1: out[idx] = (uint8_t)v; break;
    case 2: { uint16_t x = (uint16_t)v; memcpy(out + 2 * idx, &x, 2); } break;
    case 4: { uint32_t x = (uint32_t)v; memcpy(out + 4 * idx, &x, 4); } break;
    default: memcpy(out + 8 * idx, &v, 8); break;
    }
}

/* DELTA reconstruction of one vector: u[p] are unpacked values at transposed
 * positions, for_base the frame of reference of the deltas, bases[c] the
 * chain (lane) bases.  Writes 1024 tuple values (mod 2^T) to vals. */
static void delta_vector(int T, const uint64_t *u, uint64_t for_base,
                         const uint8_t *bases, uint64_t *vals)
{
    const uint64_t tm = mask_bits(T);
    uint64_t d[1024];
    for (uint32_t p = 0; p < 1024; ++p) d[flsref_tau(p)] = (for_base + u[p]) & tm;
    const int nchains = 1024 / T;
    for (int c = 0; c < nchains; ++c) {
        int blk = c / 16, l = c % 16;
        uint64_t acc = rd_word(T, bases, (uint64_t)c);
        for (int k = 0; k < T; ++k) {
            uint32_t i = (uint32_t)(blk * 16 * T + l + 16 * k);
            acc = (acc + d[i]) & tm;
            vals[i] = acc;
        }
    }
}

int flsref_validity(const flsref_file *f, uint32_t col, uint32_t rg, uint64_t *words)
{
    if (col >= f->ncols || rg >= f->nrowgroups) return -1;
    const uint8_t *rgp = rg_desc(f, rg);
    const uint64_t coff = rd64(rgp + 4 + 16 * (size_t)col);
    const uint64_t clen = rd64(rgp + 4 + 16 * (size_t)col + 8);
    if (coff + clen > f->len || clen < 64) return -1;
    const uint8_t *ch = f->img + coff;
    if (!(rd32(ch + 52) & 0x80000000u)) return 0;
    const uint32_t nvec = rd32(ch + 8), nvals = rd32(ch + 12);
    if (clen < 64 + 128ull * nvec) return -1;
    const uint8_t *bits = ch + clen - 128ull * nvec;
    const uint8_t *meta = ch + rd64(ch + 16);
    for (uint32_t v = 0; v < nvec; ++v) {
        const uint32_t n = nvals - 1024 * v < 1024 ? nvals - 1024 * v : 1024;
        int has_null = 0;
        for (uint32_t j = 0; j < 16; ++j) {
            const uint64_t w = rd64(bits + 128ull * v + 8 * j);
            const uint32_t r0 = 64 * j;
            const uint64_t live = r0 >= n ? 0 : (n - r0 >= 64 ? ~0ull : ((1ull << (n - r0)) - 1));
            if (w & ~live) return -1;            /* bits past the rows */
            if ((w & live) != live) has_null = 1;
            words[16 * (size_t)v + j] = w;
        }
        if (has_null != (meta[32 * (size_t)v + 27] & 1)) return -1;  /* VecMeta.pad */
    }
    return 1;
}

int64_t flsref_decode(const flsref_file *f, uint32_t col, uint32_t rg, void *out_v)
{
    uint8_t *out = (uint8_t *)out_v;
    if (col >= f->ncols || rg >= f->nrowgroups) return -1;
    int type, w, s, nl;
    const char *nm;
    flsref_column(f, col, &type, &w, &s, &nm, &nl);
    const int vb = value_bytes(type);
    const uint8_t *rgp = rg_desc(f, rg);
    const uint32_t rg_rows = rd32(rgp);
    const uint64_t coff = rd64(rgp + 4 + 16 * (size_t)col);
    const uint64_t clen = rd64(rgp + 4 + 16 * (size_t)col + 8);
    if (coff + clen > f->len || clen < 64) return -1;
    const uint8_t *ch = f->img + coff;
    if (rd32(ch) != 0x43534C46u) return -1; /* 'FLSC' */
    const int enc = ch[4], T = ch[5], vbits = ch[6], is_str = ch[7];
    const uint32_t nvec = rd32(ch + 8), nvals = rd32(ch + 12);
    const uint8_t *meta = ch + rd64(ch + 16);
    const uint8_t *packed = ch + rd64(ch + 24);
    const uint8_t *aux = ch + rd64(ch + 32);
    const uint32_t dict_count = rd32(ch + 48);
    if (nvals != rg_rows) return -1;
    if (T != 8 && T != 16 && T != 32 && T != 64) return -1;
    const uint64_t tm = mask_bits(T);
    const uint64_t vm = mask_bits(vbits ? vbits : 64);

    uint64_t u[1024], vals[1024];
    uint64_t row = 0;
    for (uint32_t v = 0; v < nvec; ++v) {
        const uint8_t *vm_p = meta + 32 * (size_t)v;
        const uint64_t poff = rd64(vm_p);
        const uint64_t for_base = rd64(vm_p + 8);
        const uint64_t aoff = rd64(vm_p + 16);
        const uint32_t vn = rd16(vm_p + 24);
        const int W = vm_p[26];
        const uint32_t acount = rd32(vm_p + 28);
        if (W > T || vn > 1024) return -1;
        flsref_unpack(T, W, packed + poff, u);
        switch (enc) {
        case ENC_FFOR:
            for (uint32_t i = 0; i < vn; ++i) store_val(out, vb, row + i, (for_base + u[i]) & tm);
            break;
        case ENC_DELTA:
            delta_vector(T, u, for_base, aux + aoff, vals);
            for (uint32_t i = 0; i < vn; ++i) store_val(out, vb, row + i, vals[i]);
            break;
        case ENC_DICT:
            for (uint32_t i = 0; i < vn; ++i) {
                uint64_t code = (for_base + u[i]) & tm;
                if (code >= dict_count) return -1;
                if (is_str) {
                    const uint8_t *offs = aux;
                    uint32_t b0 = rd32(offs + 4 * code), b1 = rd32(offs + 4 * (code + 1));
                    uint64_t bytes_at = (uint64_t)(aux - f->img) + 4ull * (dict_count + 1) + b0;
                    uint64_t pair[2] = {bytes_at, (uint64_t)(b1 - b0)};
                    memcpy(out + 16 * (row + i), pair, 16);
                } else {
                    store_val(out, vb, row + i, rd_word(vbits, aux, code) & vm);
                }
            }
            break;
        case ENC_RLE: {
            /* index vector: DELTA with T=16 over 64 u16 lane bases */
            if (T != 16) return -1;
            delta_vector(16, u, for_base, aux + aoff, vals);
            const uint8_t *runs = aux + aoff + 128;
            for (uint32_t i = 0; i < vn; ++i) {
                uint64_t idx = vals[i];
                if (idx >= acount) return -1;
                store_val(out, vb, row + i, rd_word(vbits, runs, idx) & vm);
            }
        } break;
        case ENC_ALP: {
            const uint32_t exc = acount & 0xFFFF, e = (acount >> 16) & 0xFF, fct = acount >> 24;
            if (T == 64 ? (e > 18 || fct > e) : (T != 32 || e > 10 || fct > e)) return -1;
            if (exc > vn) return -1;
            for (uint32_t i = 0; i < vn; ++i) {
                const uint64_t d = (for_base + u[i]) & tm;
                if (T == 64) {
                    double x = (double)(int64_t)d * ALP_F10_D[fct] * ALP_IF10_D[e];
                    memcpy(out + 8 * (row + i), &x, 8);
                } else {
                    float x = (float)(int32_t)(uint32_t)d * ALP_F10_F[fct] * ALP_IF10_F[e];
                    memcpy(out + 4 * (row + i), &x, 4);
                }
            }
            const uint8_t *pos = aux + aoff;
            const uint8_t *val = pos + ((2 * (size_t)exc + 15) & ~(size_t)15);
            for (uint32_t k = 0; k < exc; ++k) {
                const uint32_t p = rd16(pos + 2 * k);
                if (p >= vn) return -1;
                memcpy(out + (size_t)(T / 8) * (row + p), val + (size_t)(T / 8) * k, T / 8);
            }
        } break;
        default:
            return -1;  /* FSST strings: flsref_decode_strings */
        }
        row += vn;
    }
    return (int64_t)row;
}

/* FSST: expand the compressed stream [c, c+clen) into dst (cap bytes).
 * Returns bytes written, or -1 on a truncated escape / overflow. */
static int64_t fsst_expand(const uint8_t *table, const uint8_t *c, uint32_t clen, uint8_t *dst, uint64_t cap)
{
    uint64_t o = 0;
    for (uint32_t i = 0; i < clen; ++i) {
        const uint32_t code = c[i];
        if (code == 255) {
            if (++i >= clen || o + 1 > cap) return -1;
            dst[o++] = c[i];
        } else {
            const uint32_t L = table[8 * 256 + code];
            if (o + L > cap) return -1;
            memcpy(dst + o, table + 8 * code, L); /* symbol bytes, little-endian order */
            o += L;
        }
    }
    return (int64_t)o;
}

/* The segment table after a vector's code stream (round-3 container, chunk
 * header reserved0 == 16; the GPU's segmented FSST kernel reads it, this
 * decoder does not need it): for every 16 code bytes, the bytes they decode to
 * and whether they start with an escape's literal, as dlen or 129 + dlen.
 * Recomputed here from the stream by the sequential decoder's own state
 * machine and compared; 0 = consistent.  Serves fastlanes_facade.cpp:48
 * (materialize), whose FSST step the kernel restates lane-parallel. */
static int fsst_check_segments(const uint8_t *table, const uint8_t *cs, uint32_t clen, const uint8_t *seg_area)
{
    const uint32_t nseg = (clen + 15) / 16;
    if (rd32(seg_area + 4) != nseg) return -1;
    uint32_t has_esc = 0, st = 0;
    for (uint32_t k = 0; k < nseg; ++k) {
        const uint32_t entry = st;
        uint32_t d = 0;
        for (uint32_t j = 16 * k; j < clen && j < 16 * k + 16; ++j) {
            if (st) { d += 1; st = 0; }
            else if (cs[j] == 255) { st = 1; has_esc = 1; }
            else d += table[8 * 256 + cs[j]];
        }
        const uint32_t want = entry ? 129 + d : d;
        if (want > 255 || seg_area[16 + k] != want) return -1;
    }
    if ((rd32(seg_area) & 1) != has_esc) return -1;
    return 0;
}

int64_t flsref_decode_strings(const flsref_file *f, uint32_t col, uint32_t rg, uint32_t *offs,
                              uint8_t *heap, uint64_t cap)
{
    if (col >= f->ncols || rg >= f->nrowgroups) return -1;
    int type, w, s, nl;
    const char *nm;
    flsref_column(f, col, &type, &w, &s, &nm, &nl);
    if (type != TY_VARCHAR && type != TY_BLOB) return -1;
    const uint8_t *rgp = rg_desc(f, rg);
    const uint32_t rg_rows = rd32(rgp);
    const uint64_t coff = rd64(rgp + 4 + 16 * (size_t)col);
    const uint8_t *ch = f->img + coff;
    const int enc = ch[4];
    if (enc == ENC_DICT) {
        uint64_t *pairs = (uint64_t *)malloc(16 * (size_t)rg_rows);
        if (!pairs) return -1;
        if (flsref_decode(f, col, rg, pairs) != rg_rows) { free(pairs); return -1; }
        uint64_t o = 0;
        offs[0] = 0;
        for (uint32_t i = 0; i < rg_rows; ++i) {
            const uint64_t at = pairs[2 * i], len = pairs[2 * i + 1];
            if (o + len > cap) { free(pairs); return -1; }
            memcpy(heap + o, f->img + at, len);
            o += len;
            offs[i + 1] = (uint32_t)o;
        }
        free(pairs);
        return (int64_t)o;
    }
    if (enc != ENC_FSST || ch[5] != 32) return -1;
    const uint32_t nvec = rd32(ch + 8);
    const uint8_t *meta = ch + rd64(ch + 16);
    const uint8_t *packed = ch + rd64(ch + 24);
    const uint8_t *aux = ch + rd64(ch + 32);
    uint64_t u[1024];
    uint64_t o = 0, row = 0;
    offs[0] = 0;
    for (uint32_t v = 0; v < nvec; ++v) {
        const uint8_t *vm_p = meta + 32 * (size_t)v;
        const uint64_t poff = rd64(vm_p), for_base = rd64(vm_p + 8), aoff = rd64(vm_p + 16);
        const uint32_t vn = rd16(vm_p + 24), W = vm_p[26], dbytes = rd32(vm_p + 28);
        if (W > 32 || vn > 1024) return -1;
        flsref_unpack(32, (int)W, packed + poff, u);
        /* FsstVecHeader: heap_off, comp_len, clen_base, clen_w; then the FFOR
         * stream of the compressed string lengths; then the code stream */
        const uint8_t *vh = aux + aoff;
        const uint32_t clen = rd32(vh + 4), cbase = rd32(vh + 8), cw = rd32(vh + 12);
        if (cw > 32 || o + dbytes > cap) return -1;
        uint64_t cu[1024];
        flsref_unpack(32, (int)cw, vh + 16, cu);
        const uint8_t *cs = vh + 16 + 128 * (size_t)cw;
        if ((rd32(ch + 52) & 0x7FFFFFFFu) == 16 && fsst_check_segments(aux, cs, clen, cs + ((clen + 15u) & ~15u)) != 0) return -1;
        /* every string is compressed on its own: expand string by string */
        uint64_t sum = 0, cpos = 0;
        for (uint32_t i = 0; i < vn; ++i) {
            const uint32_t dl = (uint32_t)((for_base + u[i]) & 0xFFFFFFFFull);
            const uint32_t cl = (uint32_t)((cbase + cu[i]) & 0xFFFFFFFFull);
            if (cpos + cl > clen || sum + dl > dbytes) return -1;
            if (fsst_expand(aux, cs + cpos, cl, heap + o + sum, dl) != (int64_t)dl) return -1;
            cpos += cl;
            sum += dl;
            offs[row + i + 1] = (uint32_t)(o + sum);
        }
        if (sum != dbytes || cpos != clen) return -1;
        o += dbytes;
        row += vn;
    }
    return row == rg_rows ? (int64_t)o : -1;
}

/* ---- parallel column decode (CPU baseline) ------------------------------ */

typedef struct {
    const flsref_file *f;
    uint32_t col;
    uint8_t *out;
    int vb;
    uint32_t rg_begin, rg_end;
    const uint64_t *rg_row;
    int64_t rc;
} job_t;

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    j->rc = 0;
    for (uint32_t rg = j->rg_begin; rg < j->rg_end; ++rg) {
        int64_t n = flsref_decode(j->f, j->col, rg, j->out + j->rg_row[rg] * (uint64_t)j->vb);
        if (n < 0) { j->rc = -1; return NULL; }
        j->rc += n;
    }
    return NULL;
}

int64_t flsref_decode_column(const flsref_file *f, uint32_t col, void *out, int nthreads)
{
    if (col >= f->ncols) return -1;
    const int vb = flsref_out_width(f, col);
    uint64_t *rg_row = (uint64_t *)malloc(sizeof(uint64_t) * (f->nrowgroups + 1));
    rg_row[0] = 0;
    for (uint32_t rg = 0; rg < f->nrowgroups; ++rg) rg_row[rg + 1] = rg_row[rg] + (uint64_t)flsref_rowgroup_rows(f, rg);
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > f->nrowgroups) nthreads = f->nrowgroups ? (int)f->nrowgroups : 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].f = f;
        jobs[t].col = col;
        jobs[t].out = (uint8_t *)out;
        jobs[t].vb = vb;
        jobs[t].rg_begin = (uint32_t)((uint64_t)f->nrowgroups * t / nthreads);
        jobs[t].rg_end = (uint32_t)((uint64_t)f->nrowgroups * (t + 1) / nthreads);
        jobs[t].rg_row = rg_row;
        if (nthreads > 1) pthread_create(&th[t], NULL, worker, &jobs[t]);
        else worker(&jobs[t]);
    }
    int64_t total = 0;
    for (int t = 0; t < nthreads; ++t) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        if (jobs[t].rc < 0) total = -1;
        else if (total >= 0) total += jobs[t].rc;
    }
    free(jobs);
    free(th);
    free(rg_row);
    return total;
}
