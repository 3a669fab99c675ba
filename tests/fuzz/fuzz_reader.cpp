// fuzz_reader.cpp -- mutation fuzzing of the .fls footer / chunk validation
// (csrc/fls_reader.hpp) under AddressSanitizer + UBSan, host only.
//
// parse_file is the gate between an untrusted file and the GPU: every offset
// the host or the decode kernels follow must have been checked by it.  The
// harness mutates a valid image (bytes, bits, 32-bit fields, truncation; biased
// towards the footer and the chunk headers / vector metadata), parses it, and
// for every image the parser accepts walks all bytes the host side reads after
// parsing (vector metadata, DICT dictionaries via dict_string, FSST symbol
// tables and vector headers, ALP exception areas, RLE run values, zone maps).
// Any out-of-bounds read aborts the process (-fno-sanitize-recover).
//
//   fuzz_reader <image.fls> <iterations> <seed>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "fls_reader.hpp"

using namespace fls;

static uint64_t g_sink = 0;

static void touch(const uint8_t *p, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) g_sink += p[i];
}

// everything the host reads from an accepted image (make_devchunk,
// build_strtabs, term_may_match, rg_byte_range)
static void walk(const std::vector<uint8_t> &img, const FileMeta &m) {
    const uint8_t *b = img.data();
    for (auto &rg : m.rgs) {
        for (size_t c = 0; c < rg.chunks.size(); ++c) {
            const ChunkRef &ch = rg.chunks[c];
            const ChunkHeader &h = ch.hdr;
            const uint8_t *chunk = b + ch.off;
            for (uint32_t v = 0; v < h.nvec; ++v) {
                VecMeta vm;
                memcpy(&vm, chunk + h.meta_off + 32ull * v, 32);
                touch(chunk + h.packed_off + vm.packed_off, 128ull * vm.bw);
                const uint8_t *aux = chunk + h.aux_off;
                if (h.enc == ENC_DELTA) touch(aux + vm.aux_off, 128);
                if (h.enc == ENC_RLE) touch(aux + vm.aux_off, 128 + (uint64_t)vm.aux_count * (h.vbits / 8));
                if (h.enc == ENC_ALP && alp_exceptions(vm.aux_count))
                    touch(aux + vm.aux_off, alp_aux_bytes(alp_exceptions(vm.aux_count), h.vbits));
                if (h.enc == ENC_FSST) {
                    FsstVecHeader fh;
                    memcpy(&fh, aux + vm.aux_off, sizeof(fh));
                    touch(aux + vm.aux_off + sizeof(fh), fsst_stream_off(fh) - sizeof(fh) + fh.comp_len);
                }
            }
            if (h.enc == ENC_DICT) {
                const uint8_t *aux = chunk + h.aux_off;
                if (h.is_str) {
                    for (uint32_t i = 0; i < h.dict_count; ++i) {
                        const uint8_t *p;
                        uint32_t len;
                        dict_string(aux, h.dict_count, i, p, len);
                        touch(p, len);
                    }
                } else {
                    touch(aux, (uint64_t)h.dict_count * (h.vbits / 8));
                }
            }
            if (h.enc == ENC_FSST) touch(chunk + h.aux_off, kFsstTableBytes);
            if (!rg.zones.empty()) g_sink += rg.zones[c].min ^ rg.zones[c].max;
        }
    }
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s image iterations seed\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> orig;
    int ch;
    while ((ch = fgetc(f)) != EOF) orig.push_back((uint8_t)ch);
    fclose(f);
    const long iters = atol(argv[2]);
    std::mt19937_64 rng(strtoull(argv[3], nullptr, 10));
    FileMeta base;
    if (!parse_file(orig.data(), orig.size(), base).empty()) {
        fprintf(stderr, "seed image does not parse\n");
        return 2;
    }
    walk(orig, base);
    // interesting offsets: chunk headers, vector metadata, aux starts, footer
    std::vector<uint64_t> hot;
    for (auto &rg : base.rgs)
        for (auto &c : rg.chunks) {
            hot.push_back(c.off);
            hot.push_back(c.off + c.hdr.meta_off);
            hot.push_back(c.off + c.hdr.aux_off);
        }
    // targeted u64 wrap-around cases: offsets chosen so that
    // `a + b > lim` checks would wrap and accept an image whose streams start
    // before the chunk; every one must be rejected
    long wrap_cases = 0;
    for (auto &rg : base.rgs)
        for (auto &c : rg.chunks) {
            const ChunkHeader &h = c.hdr;
            auto reject = [&](uint64_t at, uint64_t val, const char *what) {
                std::vector<uint8_t> img = orig;
                memcpy(img.data() + at, &val, 8);
                FileMeta m;
                ++wrap_cases;
                if (parse_file(img.data(), img.size(), m).empty()) {
                    fprintf(stderr, "wrap case accepted: %s = 0x%llx at %llu\n", what, (unsigned long long)val,
                            (unsigned long long)at);
                    exit(3);
                }
            };
            const uint64_t hm = c.off + offsetof(ChunkHeader, meta_off);
            reject(hm, ~0ull - 31, "meta_off");
            reject(c.off + offsetof(ChunkHeader, aux_off), ~0ull - 15, "aux_off");
            reject(c.off + offsetof(ChunkHeader, aux_len), ~0ull - 15, "aux_len");
            for (uint32_t v = 0; v < h.nvec; ++v) {
                const uint64_t vo = c.off + h.meta_off + 32ull * v;
                VecMeta vm;
                memcpy(&vm, orig.data() + vo, 32);
                reject(vo + offsetof(VecMeta, packed_off), (uint64_t)0 - (h.packed_off + 128ull * vm.bw), "vm.packed_off");
                reject(vo + offsetof(VecMeta, packed_off), ~0ull - 15, "vm.packed_off");
                if (h.enc == ENC_DELTA || h.enc == ENC_RLE || h.enc == ENC_FSST ||
                    (h.enc == ENC_ALP && alp_exceptions(vm.aux_count)))
                    reject(vo + offsetof(VecMeta, aux_off), (uint64_t)0 - 128, "vm.aux_off");
            }
        }
    uint64_t foot;
    memcpy(&foot, orig.data() + orig.size() - 16, 8);
    long accepted = 0;
    for (long it = 0; it < iters; ++it) {
        std::vector<uint8_t> img = orig;
        const int nm = 1 + (int)(rng() % 6);
        for (int k = 0; k < nm; ++k) {
            uint64_t at;
            const unsigned where = rng() % 8;
            if (where < 3) at = foot + rng() % (img.size() - foot);                // footer / tail
            else if (where < 6) at = hot[rng() % hot.size()] + rng() % 96;          // headers, metas, aux
            else at = rng() % img.size();                                           // anywhere
            if (at >= img.size()) at = img.size() - 1;
            switch (rng() % 5) {
            case 0: img[at] = (uint8_t)rng(); break;
            case 1: img[at] ^= (uint8_t)(1u << (rng() % 8)); break;
            case 2: img[at] = 0xFF; break;
            case 3: {  // a 32-bit field: 0, huge, or a small perturbation
                const uint64_t a = at & ~3ull;
                if (a + 4 <= img.size()) {
                    uint32_t x;
                    memcpy(&x, img.data() + a, 4);
                    const unsigned kind = rng() % 3;
                    x = kind == 0 ? 0u : kind == 1 ? 0xFFFFFFF0u + (uint32_t)(rng() % 16) : x + (uint32_t)(rng() % 64) - 32;
                    memcpy(img.data() + a, &x, 4);
                }
                break;
            }
            default:  // truncate (keeping the tail magic rarely valid)
                if (rng() % 4 == 0 && img.size() > 64) img.resize(img.size() - 1 - rng() % 64);
                break;
            }
        }
        FileMeta m;
        if (parse_file(img.data(), img.size(), m).empty()) {
            ++accepted;
            walk(img, m);
        }
    }
    printf("iterations %ld accepted %ld wrap_cases %ld sink %llu\n", iters, accepted, wrap_cases,
           (unsigned long long)(g_sink & 0xFF));
    return 0;
}
