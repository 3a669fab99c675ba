// fls_reader.hpp -- footer / schema parser (Connection::read_fls counterpart,
// reference src/fastlanes_facade.cpp:34).  Host only; validates every offset
// so a corrupt file is reported as FLS_ERR_FORMAT instead of faulting a GPU.
#pragma once
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "fls_alp.hpp"
#include "fls_format.hpp"

namespace fls {

struct ColumnMeta {
    std::string name;
    uint8_t type, width, scale;
};

struct ChunkRef {
    uint64_t off, len;
    ChunkHeader hdr;
};

struct RowGroupMeta {
    uint32_t nrows;
    uint64_t first_row;            // relative to the file's first row
    std::vector<ChunkRef> chunks;  // one per column
    std::vector<ZoneMap> zones;    // one per column, empty without a zone-map section
};

struct FileMeta {
    uint64_t nrows = 0, row_offset = 0;
    uint32_t rowgroup_size = kRowGroupSize;
    std::vector<ColumnMeta> cols;
    std::vector<RowGroupMeta> rgs;
};

// Is [off, off + n) inside [0, lim)?  Each term is compared on its own, so a
// u64 field near 2^64 taken from the file cannot wrap the sum past the check.
inline bool fits(uint64_t off, uint64_t n, uint64_t lim) { return off <= lim && n <= lim - off; }

// Chunk c of row group r against its header, the column type and every
// vector's extents (the GPU reads nothing these checks have not bounded).
// Returns nullptr or the reason.
inline const char *validate_chunk(const uint8_t *img, const FileMeta &m, uint32_t r, uint32_t c) {
    const RowGroupMeta &rg = m.rgs[r];
    const ChunkRef &ch = rg.chunks[c];
    const ChunkHeader &h = ch.hdr;
    if (h.magic != kChunkMagic) return "bad chunk magic";
    if (h.nvals != rg.nrows || h.nvec != (rg.nrows + kVectorSize - 1) / kVectorSize) return "chunk row count mismatch";
    if (h.T != 8 && h.T != 16 && h.T != 32 && h.T != 64) return "bad packing width";
    if ((h.enc < ENC_FFOR || h.enc > ENC_ALP) && h.enc != ENC_FSST) return "bad encoding";
    const uint8_t ty = m.cols[c].type;
    const bool is_str = type_is_string(ty);
    if ((bool)h.is_str != is_str) return "chunk/column type mismatch";
    if (is_str ? (h.enc != ENC_DICT && h.enc != ENC_FSST) : h.vbits != type_value_bits(ty))
        return "chunk/column type mismatch";
    if (type_is_float(ty) != (h.enc == ENC_ALP)) return "chunk/column type mismatch";
    if ((h.enc == ENC_ALP) && h.T != h.vbits) return "bad packing width";
    if (h.enc == ENC_FSST && h.T != 32) return "bad string length width";
    if ((h.enc == ENC_FFOR || h.enc == ENC_DELTA) && h.T != h.vbits) return "bad packing width";
    if (h.enc == ENC_DICT && h.T != 32) return "bad dictionary code width";
    if (h.enc == ENC_RLE && h.T != 16) return "bad run-index width";
    if (!fits(h.meta_off, 32ull * h.nvec, ch.len) || h.packed_off > h.aux_off || !fits(h.aux_off, h.aux_len, ch.len) ||
        h.packed_off % 16 || h.meta_off % 16 || h.aux_off % 16)
        return "chunk layout out of bounds";
    // per-vector validation: packed extents, widths, aux extents
    for (uint32_t v = 0; v < h.nvec; ++v) {
        VecMeta vm;
        memcpy(&vm, img + ch.off + h.meta_off + 32ull * v, 32);
        if (vm.bw > h.T || vm.nvals == 0 || vm.nvals > kVectorSize) return "bad vector meta";
        if (v + 1 < h.nvec && vm.nvals != kVectorSize) return "short vector before the last";
        if (vm.packed_off % 16 || !fits(vm.packed_off, 128ull * vm.bw, h.aux_off - h.packed_off))
            return "packed vector out of bounds";
        if (h.enc == ENC_DELTA && (vm.aux_off % 16 || !fits(vm.aux_off, 128, h.aux_len))) return "delta bases out of bounds";
        if (h.enc == ENC_RLE) {
            if (vm.aux_off % 16 || vm.aux_count == 0 || vm.aux_count > kVectorSize ||
                !fits(vm.aux_off, 128 + (uint64_t)vm.aux_count * (h.vbits / 8), h.aux_len))
                return "run values out of bounds";
        }
        if (h.enc == ENC_ALP) {
            const uint32_t exc = alp_exceptions(vm.aux_count), e = alp_e(vm.aux_count), f = alp_f(vm.aux_count);
            const uint32_t maxe = h.T == 64 ? kAlpMaxExpD : kAlpMaxExpF;
            if (e > maxe || f > e || exc > vm.nvals) return "bad ALP exponent or exception count";
            if (exc && (vm.aux_off % 16 || !fits(vm.aux_off, alp_aux_bytes(exc, h.vbits), h.aux_len)))
                return "ALP exceptions out of bounds";
        }
        if (h.enc == ENC_FSST) {
            FsstVecHeader fh;
            if (vm.aux_off % 16 || vm.aux_off < kFsstTableBytes || !fits(vm.aux_off, sizeof(fh), h.aux_len))
                return "FSST vector out of bounds";
            memcpy(&fh, img + ch.off + h.aux_off + vm.aux_off, sizeof(fh));
            if (fh.clen_w > 32 || !fits(vm.aux_off, fsst_stream_off(fh) + fh.comp_len, h.aux_len) ||
                fh.heap_off % 16 || fh.heap_off + (uint64_t)vm.aux_count > h.reserved1)
                return "FSST vector out of bounds";
            if (chunk_seg_codes(h) == kFsstSegCodes) {  // segment table after the stream
                if (!fits(vm.aux_off, fsst_seg_off(fh) + fsst_seg_bytes(fh.comp_len), h.aux_len))
                    return "FSST segment table out of bounds";
                FsstSegHeader sh;
                memcpy(&sh, img + ch.off + h.aux_off + vm.aux_off + fsst_seg_off(fh), sizeof(sh));
                if (sh.nseg != fsst_nseg(fh.comp_len)) return "bad FSST segment table";
            }
        }
    }
    if (h.enc == ENC_FSST) {
        if (h.aux_len < kFsstTableBytes || h.dict_count > 255) return "bad FSST symbol table";
        if (chunk_seg_codes(h) != 0 && chunk_seg_codes(h) != kFsstSegCodes) return "bad FSST segment size";
        for (uint32_t k = 0; k < h.dict_count; ++k) {
            const uint8_t l = img[ch.off + h.aux_off + 8 * 256 + k];
            if (l < 1 || l > 8) return "bad FSST symbol length";
        }
        if (h.reserved1 > (1ull << 32)) return "FSST heap too large";
    }
    if (h.enc != ENC_FSST && chunk_seg_codes(h) != 0) return "bad chunk flags";
    if (chunk_has_validity(h)) {  // bitmaps at the chunk's end, after everything else
        if (ch.len < (uint64_t)kValidityVecBytes * h.nvec + sizeof(ChunkHeader)) return "validity out of bounds";
        const uint64_t vo = validity_off(ch.len, h.nvec);
        if (vo % 16 || vo < h.aux_off + h.aux_len || vo < h.meta_off + 32ull * h.nvec) return "validity out of bounds";
    }
    if (h.enc == ENC_DICT) {
        if (h.dict_count == 0) return "empty dictionary";
        if (is_str) {
            uint64_t need = 4ull * (h.dict_count + 1);
            if (need > h.aux_len) return "dictionary out of bounds";
            uint32_t last;
            memcpy(&last, img + ch.off + h.aux_off + 4ull * h.dict_count, 4);
            if (need + last > h.aux_len) return "dictionary out of bounds";
            // entry i is bytes [off[i], off[i+1]): offsets start at 0 and never decrease
            uint32_t prev = 0;
            for (uint32_t k = 0; k <= h.dict_count; ++k) {
                uint32_t o;
                memcpy(&o, img + ch.off + h.aux_off + 4ull * k, 4);
                if ((k == 0 && o != 0) || o < prev) return "dictionary offsets not monotone";
                prev = o;
            }
        } else if ((uint64_t)h.dict_count * (h.vbits / 8) > h.aux_len) {
            return "dictionary out of bounds";
        }
    }
    return nullptr;
}

// Parse and validate; returns empty string on success, else the reason.
// Chunk validation runs on up to 8 threads for large files (it touches
// every chunk's vector metadata: ~26 ms single-threaded for 15k chunks); the
// reported reason is the first failing row group's, as a serial pass would.
inline std::string parse_file(const uint8_t *img, uint64_t len, FileMeta &m) {
    auto rd = [&](uint64_t off, void *dst, size_t n) -> bool {
        if (off > len || n > len - off) return false;
        memcpy(dst, img + off, n);
        return true;
    };
    if (len < 16 + 16 || memcmp(img, kFileMagic, 8) != 0) return "bad file magic";
    if (memcmp(img + len - 4, kTailMagic, 4) != 0) return "bad tail magic";
    uint64_t foff;
    uint32_t flen;
    rd(len - 16, &foff, 8);
    rd(len - 8, &flen, 4);
    if (foff > len - 16 || flen > len - 16 - foff || flen < kFooterFixed) return "bad footer offset";
    uint64_t p = foff;
    const uint64_t fend = foff + flen;
    uint32_t ver, ncols, nrg, rgsz;
    rd(p, &ver, 4);
    rd(p + 4, &ncols, 4);
    rd(p + 8, &m.nrows, 8);
    rd(p + 16, &nrg, 4);
    rd(p + 20, &rgsz, 4);
    rd(p + 24, &m.row_offset, 8);
    if (ver != kFooterVersion) return "unsupported footer version";
    if (rgsz == 0 || rgsz > kRowGroupSize || rgsz % kVectorSize) return "unsupported row-group size";
    if (ncols == 0 || ncols > 4096) return "bad column count";
    m.rowgroup_size = rgsz;
    p += kFooterFixed;
    m.cols.resize(ncols);
    for (auto &c : m.cols) {
        uint8_t d[4];
        uint16_t nl;
        if (p + 6 > fend || !rd(p, d, 4) || !rd(p + 4, &nl, 2) || p + 6 + nl > fend) return "truncated column descriptor";
        c.type = d[0];
        c.width = d[1];
        c.scale = d[2];
        if (!type_valid(c.type)) return "unsupported column type";
        c.name.assign((const char *)img + p + 6, nl);
        p += 6 + nl;
    }
    if ((uint64_t)nrg * (4 + 16ull * ncols) > fend - p) return "truncated row-group descriptor";
    m.rgs.resize(nrg);
    uint64_t rows = 0;
    for (uint32_t r = 0; r < nrg; ++r) {
        auto &rg = m.rgs[r];
        if (p + 4 + 16ull * ncols > fend) return "truncated row-group descriptor";
        rd(p, &rg.nrows, 4);
        if (rg.nrows == 0 || rg.nrows > rgsz) return "bad row-group row count";
        if (r + 1 < nrg && rg.nrows != rgsz) return "short row group before the last";
        rg.first_row = rows;
        rows += rg.nrows;
        rg.chunks.resize(ncols);
        for (uint32_t c = 0; c < ncols; ++c) {
            auto &ch = rg.chunks[c];
            rd(p + 4 + 16ull * c, &ch.off, 8);
            rd(p + 12 + 16ull * c, &ch.len, 8);
            if (ch.off > foff || ch.len > foff - ch.off || ch.len < sizeof(ChunkHeader) || ch.off % 16)
                return "chunk out of bounds";
            memcpy(&ch.hdr, img + ch.off, sizeof(ChunkHeader));
        }
        p += 4 + 16ull * ncols;
    }
    if (rows != m.nrows) return "row count mismatch";
    {   // chunk validation, row groups split over threads for large files
        const uint32_t T = nrg >= 64 ? std::min<uint32_t>(8, std::max(1u, std::thread::hardware_concurrency())) : 1;
        std::vector<const char *> why(T, nullptr);
        auto work = [&](uint32_t t) {
            for (uint32_t r = nrg * t / T; r < nrg * (t + 1) / T && !why[t]; ++r)
                for (uint32_t c = 0; c < ncols && !why[t]; ++c)
                    why[t] = validate_chunk(img, m, r, c);
        };
        std::vector<std::thread> th;
        for (uint32_t t = 1; t < T; ++t) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
        for (uint32_t t = 0; t < T; ++t)  // ranges are in row-group order
            if (why[t]) return why[t];
    }
    // optional zone-map section
    uint32_t zh[2];
    if (p + 8 <= fend && rd(p, zh, 8) && zh[0] == kZoneMagic) {
        if (zh[1] != sizeof(ZoneMap) || p + 8 + (uint64_t)nrg * ncols * sizeof(ZoneMap) > fend)
            return "truncated zone-map section";
        for (uint32_t r = 0; r < nrg; ++r) {
            auto &z = m.rgs[r].zones;
            z.resize(ncols);
            rd(p + 8 + (uint64_t)r * ncols * sizeof(ZoneMap), z.data(), ncols * sizeof(ZoneMap));
            for (uint32_t c = 0; c < ncols; ++c)
                if (type_is_string(m.cols[c].type)) z[c].flags &= ZM_HAS_NULL | ZM_ALL_NULL;
        }
    }
    return "";
}

// String i of a validated VARCHAR DICT chunk (aux area: u32 offsets[n + 1],
// then the bytes).  The offsets were checked monotone and inside the chunk.
inline void dict_string(const uint8_t *aux, uint32_t n, uint32_t i, const uint8_t *&p, uint32_t &len) {
    uint32_t b0, b1;
    memcpy(&b0, aux + 4ull * i, 4);
    memcpy(&b1, aux + 4ull * (i + 1), 4);
    p = aux + 4ull * (n + 1) + b0;
    len = b1 - b0;
}

}  // namespace fls
