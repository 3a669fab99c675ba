// fls_config.hpp -- the deployment knobs (environment variables) of the
// library and the extension, with their defaults in ONE table.  The code reads
// a knob only through knob_value(), the C-ABI reports the table
// (fls_config_default / fls_config_value, include/flsgpu.h), and
// tests/test_config.py checks every default that include/*.h and
// INTEGRATION.md state against it (the header had said 512
// for FLS_IDLE_PINNED_MB after the code moved to 1024).
//
// The other FLS_* variables in csrc/ are A/B-measurement and test hooks, not
// deployment settings, and stay where they are read.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>

namespace fls {

struct Knob {
    const char *name;
    int64_t def;
};

inline constexpr Knob kKnobs[] = {
    // scan pipeline (flsgpu.hip)
    {"FLS_IDLE_PINNED_MB", 1024},     // pinned host memory idle pipelines keep per GPU
    {"FLS_SCAN_RESIDENT_MB", 65536},  // HBM budget per GPU for resident file images (0: off)
    {"FLS_SCAN_HOST_BATCHES", 64},    // host-batch pool cap per GPU
    {"FLS_SCAN_SLOTS", 2},            // device slots (batches in flight) per GPU, 1-4
    {"FLS_SCAN_BATCH", 8},            // row groups per scan batch
    {"FLS_SCAN_STRLEN", 1},           // narrowed scans ship FSST columns as lengths + heap
    {"FLS_SCAN_COPY_KERNEL", 1},      // batches reach pinned host memory by a copy kernel (0: DMA engines)
    {"FLS_SCAN_EARLY_REFILL", 1},     // a slot refills once its batch's D2H is seen complete (0: once handed out)
    {"FLS_OPEN_CACHE", 16},           // opened files kept mapped with their metadata (0: off)
    {"FLS_COPY_THREADS", 4},          // staging copy threads per connection
    {"FLS_PIN_ARENA_MB", 0},          // registered pinned arena cap (fls_pinned.hpp; 0: hipHostMalloc only)
    {"FLS_PLACEMENT_DECODE", 6},      // output-buffer sets rated by decode launches per resident part (0/1: write probe)
    {"FLS_PLACEMENT_HEAPS", 1},       // candidate sets include new FSST heaps
    {"FLS_PLACEMENT_IMAGE", 1},       // candidate sets include a new copy of the compressed image
    {"FLS_PLACEMENT_TRIES", 8},       // write-probe mode: output-buffer sets tried per resident part
    {"FLS_PLACEMENT_GOOD", 990},      // placement rating (per mille) that ends the search
    // writer (fls_writer.cpp)
    {"FLS_WRITER_STREAM_THREADS", 1}, // write threads of a streamed file
    {"FLS_WRITER_ALP_GPU", 0},        // FLOAT / DOUBLE ALP chunks on the writer's GPU
    {"FLS_WRITER_FSST_GPU", 1},       // FSST compression on the writer's GPU
    {"FLS_WRITER_DICT_GPU", 1},       // integer DICT chunks and estimates on the writer's GPU
    {"FLS_WRITER_STRDICT_GPU", 0},    // VARCHAR / BLOB dictionaries on the writer's GPU too
    // extension (extension/src/scanner)
    {"FLS_READ_DICT", 1},             // read_fastlanes delivers DICT strings as dictionary vectors
    {"FLS_COPY_GPU", 1},              // COPY encodes on a GPU when one is visible
    {"FLS_COPY_PIPELINE", 1},         // the COPY sink pipelines its writer calls
    {"FLS_COPY_STREAM", 1},           // the COPY sink streams the file while it is written
    {"FLS_COPY_BATCH", 8},            // row groups the COPY sink hands the writer per call
    {"FLS_COPY_STAGED_MB", 1024},     // bytes all COPY sink stages may buffer together
    {"FLS_COPY_SINK_THREADS", 4},     // column helper threads of a lone COPY sink (0: none)
};

inline const Knob *find_knob(const char *name) {
    if (!name) return nullptr;
    for (const Knob &k : kKnobs)
        if (!strcmp(k.name, name)) return &k;
    return nullptr;
}

// The value in effect: the environment's (decimal integer) or the default.
// An unknown name is a programming error: abort rather than guess.
inline int64_t knob_value(const char *name) {
    const Knob *k = find_knob(name);
    if (!k) abort();
    const char *e = getenv(name);
    return e && *e ? strtoll(e, nullptr, 10) : k->def;
}

}  // namespace fls
