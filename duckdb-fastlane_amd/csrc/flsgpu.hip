// flsgpu.hip -- host engine behind include/flsgpu.h.
//
// Replaces FastLanes' connect/read_fls/get_rowgroup_reader/materialize
// (reference src/fastlanes_facade.cpp:33-56) with:
//   * footer parse on the host (fls_reader.hpp) -- no GPU needed for schema;
//   * device-resident mode: a shard of row groups is uploaded verbatim to HBM
//     and decoded by ONE fused kernel launch per pass (bench / roofline);
//   * streaming scan: row groups sharded contiguously over the connection's
//     GPUs (no collectives: row groups are independent); per
//     GPU a two-slot pipeline H2D(compressed batch) -> decode -> D2H(pinned)
//     runs ahead of the consumer (DuckDB's scan thread).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <memory>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/flsgpu.h"
#include "fls_common.hpp"
#include "fls_config.hpp"
#include "fls_decode.hpp"
#include "fls_filter.hpp"
#include "fls_format.hpp"
#include "fls_pinned.hpp"
#include "fls_reader.hpp"
#include "fls_resident.hpp"

using namespace fls;

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(FLS_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                 \
    } while (0)

namespace {

// DuckDB v1.3.2 string_t (16 B): len <= 12 inlined, else 4-byte prefix + pointer
struct StrT {
    uint32_t len;
    char data[12];
};
static_assert(sizeof(StrT) == 16, "string_t is 16 B");

StrT make_string_t(const char *p, uint32_t n) {
    StrT s;
    memset(&s, 0, sizeof(s));
    s.len = n;
    if (n <= 12) {
        memcpy(s.data, p, n);
    } else {
        memcpy(s.data, p, 4);
        memcpy(s.data + 4, &p, sizeof(p));
    }
    return s;
}

// Scan set-up profile (FLS_SCAN_PROFILE=1): process-wide time and bytes per
// phase, printed to stderr when a table that scanned closes -- where a cold
// query's first milliseconds go (pinned and device allocations, string_t
// tables, the resident image, staging copies, the consumers' waits), and
// per batch on the GPU (HIP events on the slot's stream: the decode kernels,
// then the D2H of its columns; batches of different slots overlap, so these
// are summed stream time, not wall time).
enum ProfPhase {
    PROF_PIN_ALLOC, PROF_DEV_ALLOC, PROF_SETUP, PROF_STRTABS, PROF_IMAGE, PROF_STAGE_COPY, PROF_FILL, PROF_FILL_DESC,
    PROF_FILL_LIST, PROF_REFILL_LAT, PROF_WAIT, PROF_GPU_DECODE, PROF_D2H, PROF_N
};
struct ScanProf {
    std::atomic<uint64_t> ns[PROF_N] = {}, bytes[PROF_N] = {}, calls[PROF_N] = {};
    static bool on() {
        static const bool e = getenv("FLS_SCAN_PROFILE") && atoi(getenv("FLS_SCAN_PROFILE")) != 0;
        return e;
    }
    void print() {
        static const char *names[PROF_N] = {"pinned host alloc", "device alloc", "scan_setup", "string_t tables",
                                            "resident image", "staging copy", "fill_batch (all)",
                                            "fill: descriptors", "fill: chunk list", "batch seen -> refill",
                                            "consumer wait",
                                            "GPU decode (events)", "D2H (events)"};
        fprintf(stderr, "FLS_SCAN_PROFILE (process, since the last report):\n");
        for (int i = 0; i < PROF_N; ++i)
            fprintf(stderr, "  %-20s %9.3f ms  %8llu calls  %10.1f MB\n", names[i], ns[i].exchange(0) / 1e6,
                    (unsigned long long)calls[i].exchange(0), bytes[i].exchange(0) / 1e6);
    }
};
ScanProf &scan_prof() {
    static auto *p = new ScanProf();
    return *p;
}
struct ProfTimer {
    int ph;
    uint64_t b;
    std::chrono::steady_clock::time_point t0;
    explicit ProfTimer(int phase, uint64_t bytes = 0) : ph(ScanProf::on() ? phase : -1), b(bytes) {
        if (ph >= 0) t0 = std::chrono::steady_clock::now();
    }
    void stop() {  // record now (once)
        if (ph < 0) return;
        ScanProf &p = scan_prof();
        p.ns[ph] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        p.bytes[ph] += b;
        p.calls[ph] += 1;
        ph = -1;
    }
    void cancel() { ph = -1; }
    ~ProfTimer() { stop(); }
};

// Frees every HBM-resident image no running scan uses on GPU dev (defined
// with the image registry); a device allocation that runs out of memory calls
// it once and retries, so the image cache never fails a scan's own buffers.
uint64_t release_idle_images(int dev);

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    int dev = -1;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p), n(o.n), dev(o.dev) { o.p = nullptr; o.n = 0; }
    void release() {
        if (p) {
            int cur;
            hipGetDevice(&cur);
            hipSetDevice(dev);
            hipFree(p);
            hipSetDevice(cur);
        }
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(int d, size_t count) {
        if (count <= n && p && d == dev) return hipSuccess;
        release();
        dev = d;
        n = count;
        ProfTimer pt(PROF_DEV_ALLOC, count * sizeof(T));
        hipError_t e = hipMalloc((void **)&p, std::max<size_t>(1, count * sizeof(T)));
        if (e == hipErrorOutOfMemory && release_idle_images(d) > 0) {
            (void)hipGetLastError();
            e = hipMalloc((void **)&p, std::max<size_t>(1, count * sizeof(T)));
        }
        if (e != hipSuccess) {
            p = nullptr;
            n = 0;
        }
        return e;
    }
    ~DevBuf() { release(); }
};

template <typename T>
struct PinBuf {
    T *p = nullptr;
    size_t n = 0;
    PinBuf() = default;
    PinBuf(const PinBuf &) = delete;
    PinBuf &operator=(const PinBuf &) = delete;
    PinBuf(PinBuf &&o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    void release() {
        if (p) pinned_free(p);
        p = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t count) {
        if (count <= n && p) return hipSuccess;
        release();
        n = count;
        ProfTimer pt(PROF_PIN_ALLOC, count * sizeof(T));
        const hipError_t e = pinned_alloc((void **)&p, std::max<size_t>(1, count * sizeof(T)));
        if (e != hipSuccess) {
            p = nullptr;
            n = 0;
        }
        return e;
    }
    ~PinBuf() { release(); }
};

// Host threads that split a large memcpy: a scan stages each batch's
// compressed bytes from the mapped file into pinned memory for its H2D
// (instead of pinning the whole file up front, which cost ~0.12 s per GB
// before the first row group could move).  The copy must keep pace with
// compressed/decoded x the D2H rate (lineitem: ~9 GB/s at 50 GB/s D2H), more
// than one thread's page-cache copy rate.  Threads start on first use;
// FLS_COPY_THREADS (default 4) sets how many besides the caller.
class CopyPool {
  public:
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    void copy(void *dst, const void *src, size_t n) {
        constexpr size_t kMinPart = 2u << 20;
        start();
        const size_t parts = std::min<size_t>(th_.size() + 1, std::max<size_t>(1, n / kMinPart));
        if (parts <= 1) {
            memcpy(dst, src, n);
            return;
        }
        Call call;
        call.left = (int)parts - 1;
        const size_t per = (n / parts + 63) & ~size_t(63);
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (size_t p = 1; p < parts; ++p) {
                const size_t o = std::min(n, p * per), e = std::min(n, o + per);
                jobs_.push_back({(uint8_t *)dst + o, (const uint8_t *)src + o, p + 1 == parts ? n - o : e - o, &call});
            }
        }
        cv_.notify_all();
        memcpy(dst, src, std::min(n, per));
        std::unique_lock<std::mutex> lk(call.m);
        call.cv.wait(lk, [&] { return call.left == 0; });
    }

  private:
    struct Call {
        std::mutex m;
        std::condition_variable cv;
        int left = 0;
    };
    struct Job {
        uint8_t *d;
        const uint8_t *s;
        size_t n;
        Call *call;
    };
    void start() {
        std::lock_guard<std::mutex> lk(mu_);
        if (started_) return;
        started_ = true;
        const int n = (int)std::max<int64_t>(0, std::min<int64_t>(64, knob_value("FLS_COPY_THREADS")));
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { run(); });
    }
    void run() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !jobs_.empty(); });
                if (jobs_.empty()) return;
                j = jobs_.back();
                jobs_.pop_back();
            }
            memcpy(j.d, j.s, j.n);
            std::lock_guard<std::mutex> lk(j.call->m);
            if (--j.call->left == 0) j.call->cv.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<Job> jobs_;
    std::vector<std::thread> th_;
    bool started_ = false, stop_ = false;
};

}  // namespace

struct DevImage;  // a file's compressed image resident in HBM (defined with MappedFile)
namespace {

// Device images are allocated this much past their last chunk: kernels read
// whole 16 B blocks of a stream whose last block may end inside it.
constexpr uint64_t kImagePad = 256;

// FSST chunks of a launch, one kernel group after another (order_for_launch):
// 0 = segment tables and every string <= 255 bytes, 1 = segment tables,
// 2 = strings <= 255 bytes, 3 = the rest (DevChunk.vbits: bit 0 = small
// strings, bit 1 = segment tables); each group numbers its vectors through
// DevChunk.vec_base.
constexpr int kFsstGroups = 4;
inline int fsst_group(uint8_t vbits) { return vbits == 3 ? 0 : vbits == 2 ? 1 : vbits == 1 ? 2 : 3; }
struct FsstCounts {
    uint32_t n[kFsstGroups] = {}, vecs[kFsstGroups] = {};
    uint32_t first(int g) const {
        uint32_t f = 0;
        for (int k = 0; k < g; ++k) f += n[k];
        return f;
    }
    uint64_t total_vecs() const {
        uint64_t t = 0;
        for (int k = 0; k < kFsstGroups; ++k) t += vecs[k];
        return t;
    }
};

// Per-chunk algorithmic byte accounting (roofline numerator).
struct ByteCount {
    uint64_t values = 0, packed = 0, meta = 0, out = 0;
    DecodeGeom geom;   // max LDS need over the counted chunks
};

// Byte range of the file covering row groups [rg0, rg1).
void rg_byte_range(const FileMeta &m, uint32_t rg0, uint32_t rg1, uint64_t &lo, uint64_t &hi) {
    lo = UINT64_MAX;
    hi = 0;
    for (uint32_t r = rg0; r < rg1; ++r)
        for (auto &c : m.rgs[r].chunks) {
            lo = std::min(lo, c.off);
            hi = std::max(hi, c.off + c.len);
        }
    lo &= ~uint64_t(255);
}

// Pinned host side of one decoded batch: what consumers read.  It belongs to
// the batch's row groups, not to the device slot that produced it: once every
// row group of the batch has been handed out (fls_scan_acquire) the slot is
// refilled with a fresh HostBatch from the pool, and this one goes back to the
// pool when the last of its row groups is released.  So a consumer that keeps
// a row group (DuckDB vectors that reference the pinned columns) never holds
// up the GPU pipeline, and no consumer waits for another one's release.
struct HostBatch {
    uint32_t rg0 = 0, nrg = 0;
    uint32_t handed = 0, released = 0;    // row groups handed out / handed back
    std::vector<PinBuf<uint8_t>> h_out;   // per delivered column (pinned)
    std::vector<PinBuf<uint8_t>> h_heap;  // per FSST column: pinned copy string_t points into
    std::vector<const void *> col_ptrs;   // per (rg - rg0) * ncols + col: pinned host column start
    PinBuf<uint32_t> h_counts;            // filtered: selected rows per vector
    PinBuf<uint32_t> h_sel;               // filtered: selected row indices within their row group
    uint32_t nvec = 0;                    // vectors of the batch
    bool sel_ready = false;               // sel_off computed from h_counts
    std::vector<uint32_t> sel_off;        // per row group of the batch (+1): first selected row
    // per (rg - rg0) * ncols + col: the delivered rows' validity words (NULL:
    // all valid) -- the file image's bitmaps, or, filtered, gathered into vbits
    std::vector<const uint64_t *> valid_ptrs;
    std::vector<std::vector<uint64_t>> vbits;
    // dictionary-coded delivery (fls_scan_dict_codes): per column the bytes
    // delivered per row (string_t 16, or a code width 1 / 2), per (rg - rg0) *
    // ncols + col the host string_t dictionary and its size (NULL: not coded)
    std::vector<uint8_t> ob;
    std::vector<const void *> dict_ptrs;
    std::vector<uint32_t> dict_sizes;
    // narrowed delivery (fls_scan_narrow): per column 1 when it crosses PCIe
    // as value - base in ob bytes, per (rg - rg0) * ncols + col that base
    std::vector<uint8_t> narrowed;
    std::vector<uint64_t> nbase;
    // FSST columns delivered as string lengths (fls_scan_narrow, unfiltered
    // scans): per column the length width (0: string_t records cross PCIe);
    // per (rg - rg0) * ncols + col the row group's heap offset in h_heap; the
    // string_t records rebuilt on the consumer's thread (scan_acquire) into
    // h_rec; narrow_out = narrowed with these columns cleared (the consumer
    // sees string_t)
    std::vector<uint8_t> strlen_w, narrow_out, ob_out;
    std::vector<uint64_t> heap_off;
    std::vector<std::unique_ptr<uint8_t[]>> h_rec;
    std::vector<uint64_t> h_rec_cap;      // rows h_rec[c] holds
    // completion of the batch's device work, per batch rather than per slot:
    // the slot takes its next batch as soon as this one's D2H is complete (its
    // first acquire), while consumers still take this one's row groups
    hipEvent_t done = nullptr;            // recorded after the D2H (fill_batch)
    hipEvent_t pt[3] = {};                // FLS_SCAN_PROFILE: decode start, D2H start, end (timing events)
    uint64_t prof_d2h = 0;                // ... and the batch's D2H bytes
    std::atomic<bool> prof_pending{false};  // the batch's times not yet counted (its first acquire does)
    std::atomic<bool> upload_resident{false};  // the batch uploads into the resident image (marked present once done)
    PinBuf<uint32_t> h_err;               // the device error flags, copied after the batch's kernels
    HostBatch() = default;
    HostBatch(const HostBatch &) = delete;
    HostBatch &operator=(const HostBatch &) = delete;
    ~HostBatch() {
        if (done) hipEventDestroy(done);
        for (hipEvent_t e : pt)
            if (e) hipEventDestroy(e);
    }
};

struct Slot {                       // one batch of row groups in flight
    uint32_t rg0 = 0, nrg = 0;      // absolute row groups (consecutive, all surviving pruning)
    bool busy = false;              // a batch is enqueued and its D2H not yet seen complete by an acquire
    bool filling = false;           // claimed, its work being enqueued (fill_batch, outside s.mu)
    bool starved = false;           // refill deferred: the host-batch pool is at its cap
    HostBatch *hb = nullptr;        // host side of the batch in flight
    std::vector<DevBuf<uint8_t>> d_out;   // per decoded column
    std::vector<DevBuf<uint8_t>> d_heap;  // per FSST column: decoded string bytes
    std::vector<uint64_t> heap_bytes;     // per column: heap bytes of this batch
    PinBuf<DevChunk> h_chunks;
    DevBuf<DevChunk> d_chunks;
    DevBuf<uint8_t> d_in;           // streamed compressed bytes of the batch (no resident image)
    const uint8_t *in_dev = nullptr;  // device address of the batch's first compressed byte
    PinBuf<uint8_t> h_stage;        // pinned bounce buffer when the image cannot be pinned
    DevBuf<uint32_t> queue;         // decode work-queue counter
    uint64_t in_base = 0;
    hipStream_t stream = nullptr;   // one stream per slot: slot b's H2D+decode overlap slot a's D2H
    // filtered batches (fls_scan_filter)
    DevBuf<uint64_t> d_mask;        // selection bits, 16 words per 1024-row vector
    DevBuf<uint32_t> d_counts;      // selected rows per vector
    PinBuf<uint8_t> h_fdesc;        // DevTerm[] + DevOut[] + constant strings
    DevBuf<uint8_t> d_fdesc;
    std::vector<DevBuf<uint64_t>> d_valid;  // per filtered column with a NULL: batch validity words
    std::vector<DevBuf<uint8_t>> d_narrow;  // per narrowed column: its narrowed copy
    PinBuf<uint8_t> h_ndesc;                // DevNarrow[] + per-row-group bases
    DevBuf<uint8_t> d_ndesc;
};

// One GPU's scan pipeline: streams, the two device slots and the pinned
// host-batch pool.  A scan borrows one per GPU from its connection
// (ConnRes::take) and the table gives it back when it closes, so the next
// table -- a new DuckDB query -- starts without stream creation, hipMalloc or
// hipHostMalloc.
constexpr size_t kIdent16 = 256;  // ScanDev::ident: where the u16 identity table starts

struct ScanDev {
    int dev = -1;
    hipStream_t stream = nullptr;
    uint32_t rg0 = 0, rg1 = 0;      // span of row groups this GPU owns within the scan
    uint32_t p0 = 0, p1 = 0;        // ... as positions in ScanCtx::rgs
    uint32_t next_p = 0;            // next position to enqueue
    // device slots: batches in flight at once (ScanCtx::nslots of them used)
    static constexpr int kMaxSlots = 4;
    Slot slots[kMaxSlots];
    std::shared_ptr<DevImage> dimg;  // the scanned file's resident image on this GPU (none: per-slot uploads)
    std::vector<std::unique_ptr<HostBatch>> batches;  // host-batch pool of this GPU
    std::vector<HostBatch *> free_batches;
    DevBuf<StrT> strtab;
    std::vector<uint64_t> strtab_off;
    std::vector<StrT> h_strtab;     // host copy of strtab (the dictionaries coded columns reference)
    // identity "dictionaries" a coded column gathers its codes from: u8 0..255
    // at byte 0, u16 0..65535 at byte kIdent16
    DevBuf<uint8_t> ident;
    DevBuf<uint32_t> err;
    int grid = 0;
    ScanDev() = default;
    ScanDev(const ScanDev &) = delete;
    ScanDev &operator=(const ScanDev &) = delete;
    void sync() {
        if (dev < 0) return;
        hipSetDevice(dev);
        if (stream) hipStreamSynchronize(stream);
        for (auto &sl : slots)
            if (sl.stream) hipStreamSynchronize(sl.stream);
    }
    ~ScanDev() {
        sync();
        for (auto &sl : slots)
            if (sl.stream) hipStreamDestroy(sl.stream);
        if (stream) hipStreamDestroy(stream);
    }
};

// One term of a pushed-down filter (fls_scan_filter), host side.
struct HostTerm {
    uint32_t col = 0, clause = 0;
    uint8_t op = 0, kind = 0;
    uint64_t value = 0;             // comparison domain: int64 / uint64 / double bits
    std::string str;
};

struct ScanCtx {
    bool active = false;
    std::vector<uint8_t> mask;      // delivered columns
    std::vector<uint8_t> dmask;     // decoded columns (delivered + filter columns)
    std::vector<HostTerm> terms;    // filter of this scan, sorted by clause (empty: none)
    bool dict_codes = false;        // deliver DICT string chunks as codes + dictionary
    bool narrow = false;            // deliver integer columns narrowed to their row groups' ranges
    bool defer_records = false;     // FSST-as-lengths records built by fls_scan_build_records, not scan_acquire
    std::vector<uint32_t> rgs;      // row groups to scan, in order (pruned ones left out)
    uint32_t cur = 0;               // next position in rgs to hand out
    uint32_t pruned = 0;
    uint32_t batch = 8;
    std::vector<std::unique_ptr<ScanDev>> devs;  // borrowed from the connection (ConnRes)
    int64_t held = -1;              // row group fls_scan_next handed out last (released on the next call)
    std::vector<std::pair<uint32_t, HostBatch *>> out;  // row groups handed out and not yet released
    // batches whose D2H an acquire saw complete and whose slot took its next
    // batch: (device index, batch) until their last row group is handed out
    std::vector<std::pair<int, HostBatch *>> ready;
    bool early_refill = true;       // FLS_SCAN_EARLY_REFILL
    bool spin_wait = false;         // FLS_SCAN_SPIN_WAIT (A/B): acquires poll the batch event
    uint32_t max_batches = 64;      // host-batch pool cap per GPU (FLS_SCAN_HOST_BATCHES)
    int nslots = 2;                 // device slots per GPU (FLS_SCAN_SLOTS, 1..ScanDev::kMaxSlots)
    // sticky error of a failed batch refill (scan_release): consumers waiting
    // for a row group of that batch, and every later acquire, return it
    // instead of waiting for a batch that will never be enqueued
    int err_rc = 0;
    std::string err_msg;
    // fls_scan_acquire/release may be called from several consumer threads:
    // claiming a row group, releasing one and refilling a slot happen under mu;
    // waiting for a batch's decode does not.
    std::mutex mu;
    std::condition_variable cv;
};

// Pinned bytes a host batch holds (its columns, FSST heaps, selection).
size_t pinned_bytes(const HostBatch &b) {
    size_t t = b.h_counts.n * sizeof(uint32_t) + b.h_sel.n * sizeof(uint32_t);
    for (auto &x : b.h_out) t += x.n;
    for (auto &x : b.h_heap) t += x.n;
    return t;
}
size_t pinned_bytes(const ScanDev &d) {
    size_t t = 0;
    for (auto &b : d.batches) t += pinned_bytes(*b);
    for (auto &sl : d.slots) t += sl.h_chunks.n * sizeof(DevChunk) + sl.h_stage.n + sl.h_fdesc.n;
    return t;
}

// What a connection keeps between scans: idle per-GPU pipelines (at most
// kIdlePerDev per GPU) and the staging copy threads.  The idle pipelines'
// pinned host batches are capped by BYTES per GPU (FLS_IDLE_PINNED_MB, default
// 1024; 0 keeps none): a batch is up to 8 row groups of every delivered column,
// about 150 MB at lineitem_full widths, so a count cap alone let a long-lived
// process (DuckDB) keep more page-locked memory than it uses.  512 MB was
// below a 16-thread scan's working set: every other warm query re-pinned
// ~100 MB at hipHostMalloc's 4-5 GB/s (profiles/r5/e2e_env_r5p_prof.txt: the
// 492 M rows/s query of a 660 M median); at 1024 no warm query allocates
// (e2e_env_r5o_cap1024.txt).  fls_connection_trim frees the idle pipelines on
// demand.  Tables share ConnRes by reference, so
// it lives until the connection and every table opened on it are closed.
struct ConnRes {
    static constexpr size_t kIdlePerDev = 2;
    std::mutex mu;
    std::vector<std::unique_ptr<ScanDev>> idle;
    CopyPool copy;
    static size_t idle_cap_bytes() {
        return (size_t)std::max<int64_t>(0, knob_value("FLS_IDLE_PINNED_MB")) << 20;
    }
    // free idle pipelines until the pinned bytes they hold on GPU dev (every
    // GPU: dev < 0) are at most keep (caller holds mu)
    void trim_locked(int dev, size_t keep) {
        std::map<int, size_t> held;
        for (size_t i = idle.size(); i-- > 0;) {
            ScanDev &d = *idle[i];
            if (dev >= 0 && d.dev != dev) continue;
            // drop batches of this pipeline while over the cap, then the pipeline
            while (!d.batches.empty() && held[d.dev] + pinned_bytes(d) > keep) {
                d.batches.pop_back();
                d.free_batches.clear();
                for (auto &b : d.batches) d.free_batches.push_back(b.get());
            }
            if (held[d.dev] + pinned_bytes(d) > keep) {
                idle.erase(idle.begin() + (long)i);
                continue;
            }
            held[d.dev] += pinned_bytes(d);
        }
    }
    std::unique_ptr<ScanDev> take(int dev) {
        {
            std::lock_guard<std::mutex> lk(mu);
            for (size_t i = 0; i < idle.size(); ++i)
                if (idle[i]->dev == dev) {
                    auto d = std::move(idle[i]);
                    idle.erase(idle.begin() + (long)i);
                    return d;
                }
        }
        auto d = std::make_unique<ScanDev>();
        d->dev = dev;
        return d;
    }
    // back from a closing table; a pipeline with a host batch still out (a
    // row group never released) is freed rather than reused
    void give(std::unique_ptr<ScanDev> d) {
        if (!d) return;
        d->sync();
        if (d->free_batches.size() != d->batches.size()) return;
        for (auto &sl : d->slots) {
            sl.busy = sl.starved = false;
            sl.hb = nullptr;
        }
        d->free_batches.clear();
        for (auto &b : d->batches) d->free_batches.push_back(b.get());
        std::lock_guard<std::mutex> lk(mu);
        size_t same = 0;
        for (auto &x : idle) same += x->dev == d->dev;
        if (same >= kIdlePerDev) return;
        const int dev = d->dev;
        idle.push_back(std::move(d));
        trim_locked(dev, idle_cap_bytes());
    }
    // pinned bytes the idle pipelines hold (all GPUs)
    size_t idle_pinned() {
        std::lock_guard<std::mutex> lk(mu);
        size_t t = 0;
        for (auto &d : idle) t += pinned_bytes(*d);
        return t;
    }
};

}  // namespace

struct fls_connection {
    std::vector<int> devices;
    std::shared_ptr<ConnRes> res = std::make_shared<ConnRes>();
};

// Second stream a table decode overlaps its FSST kernels on (launch_all).
struct SideStream {
    hipStream_t stream = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // CU-partitioned overlap (FLS_OVERLAP_CU_SPLIT = m): two streams whose
    // kernels may only use disjoint CU sets -- set A (CU index mod 32 < m) for
    // the main decode, set B for FSST -- made on first use for that m
    int cu_m = 0;
    hipStream_t cu_a = nullptr, cu_b = nullptr;
    hipEvent_t join_a = nullptr, join_b = nullptr;
    void release_cu() {
        for (hipStream_t *st : {&cu_a, &cu_b})
            if (*st) {
                hipStreamSynchronize(*st);
                hipStreamDestroy(*st);
                *st = nullptr;
            }
        for (hipEvent_t *e : {&join_a, &join_b})
            if (*e) {
                hipEventDestroy(*e);
                *e = nullptr;
            }
        cu_m = 0;
    }
};

namespace {

// One GPU's part of a device-resident table (fls_device_*): a contiguous
// range of row groups uploaded verbatim to its HBM with their string_t
// tables, the decoded columns, the launch descriptor list and the streams and
// events of its decode launches.  A table is split over the connection's GPUs
// like a scan (no data crosses GPUs: row groups are independent).
struct Resident {
    int dev = -1;
    uint32_t rg0 = 0, rg1 = 0;
    uint64_t base = 0;                 // file offset of img[0]
    uint64_t first_row = 0, rows = 0;  // resident rows, relative to the file's first row
    DevBuf<uint8_t> img;               // compressed bytes of [rg0, rg1)
    DevBuf<StrT> strtab;               // string_t tables of VARCHAR chunks
    std::vector<uint64_t> strtab_off;  // per (rg - rg0) * ncols + col: index into strtab
    DevBuf<uint32_t> err;
    DevBuf<uint32_t> queue;                // decode work-queue counters
    std::vector<DevBuf<uint8_t>> d_heap;   // per FSST column: decoded string bytes
    std::vector<PinBuf<uint8_t>> h_heap;   // per FSST column: host copy string_t points into
    std::vector<uint64_t> heap_off;        // per (rg - rg0) * ncols + col: chunk heap offset
    std::vector<DevBuf<uint8_t>> d_out;    // per column, rows of [rg0, rg1)
    double placement_q = 0;                // write-probe rating of d_out's placement (choose_placement; 0: not rated)
    float placement_ms = 0;                // decode-time rating of d_out's placement (0: not rated)
    DevBuf<DevChunk> d_chunks;
    std::vector<DevChunk> h_chunks;
    std::vector<uint8_t> mask;         // column mask h_chunks was built for
    uint32_t nmain = 0;                // h_chunks[0, nmain) main kernel, the rest FSST
    int64_t policy = -1;               // decode_policy() h_chunks was ordered for
    int64_t lpolicy = 0;                // ... and the launch policy it resolved to (launch_policy)
    FsstCounts fsst;                   // FSST chunks of h_chunks
    SplitPlan split;                   // balanced split after h_chunks on the device (waves 0: none)
    ByteCount bytes;                   // algorithmic bytes of one launch
    hipStream_t stream = nullptr;
    SideStream side;                   // FSST kernels overlapping the main decode kernel
    std::vector<hipEvent_t> ev_pool;   // per-launch (start, stop) pairs since last sync
    uint32_t ev_used = 0;
    Resident() = default;
    Resident(const Resident &) = delete;
    Resident &operator=(const Resident &) = delete;
    ~Resident() {
        if (dev < 0) return;
        hipSetDevice(dev);
        if (stream) hipStreamSynchronize(stream);
        if (side.stream) hipStreamSynchronize(side.stream);
        if (stream) hipStreamDestroy(stream);
        if (side.stream) hipStreamDestroy(side.stream);
        if (side.fork) hipEventDestroy(side.fork);
        if (side.join) hipEventDestroy(side.join);
        side.release_cu();
        for (auto e : ev_pool) hipEventDestroy(e);
    }
};

}  // namespace

// A mapped, validated file shared by the tables that read it: fls_read_fls
// keeps the last few in a process-wide cache keyed by (device, inode, size,
// mtime), so reopening an unchanged file (DuckDB opens files at every query)
// skips the chunk-header validation (10-30 ms at SF10).
// A file's compressed image kept in one GPU's HBM by the scan pipeline: the
// first scan's batches are uploaded into it instead of a per-slot buffer, and
// later scans of the same (cached, unchanged) file decode its row groups from
// it with no staging copy and no H2D -- a warm query moves only decoded bytes
// over PCIe, in one direction.  Lives with the open-file cache entry.
// One GPU's image holds the file bytes of that GPU's shard of the whole
// table (its row groups when the table is split over the connection's GPUs),
// not the whole file.  Images live in a process-wide registry with one byte
// budget per GPU (ResidentSet, resident_image).
struct DevImage {
    uint8_t *p = nullptr;                              // file bytes [lo, hi) + kImagePad
    int dev = -1;
    uint64_t lo = 0, hi = 0;
    std::unique_ptr<std::atomic<uint8_t>[]> present;   // per row group of the file: its chunks are in p
    uint32_t nrg = 0;
    ~DevImage() {
        if (p) {
            int cur = 0;
            hipGetDevice(&cur);
            hipSetDevice(dev);
            hipFree(p);
            hipSetDevice(cur);
        }
    }
};
void drop_file_images(const void *owner);
struct MappedFile {
    void *map = nullptr;
    size_t len = 0;
    FileMeta meta;
    ~MappedFile() {
        drop_file_images(this);
        if (map) munmap(map, len);
    }
};

// Every GPU's resident images, under one lock (process lifetime: tables may
// outlive static destruction order).
struct ImageRegistry {
    std::mutex mu;
    ResidentSet<DevImage> set;
};
ImageRegistry &image_registry() {
    static auto *r = new ImageRegistry();
    return *r;
}
// FLS_SCAN_RESIDENT_MB: the image budget per GPU over every cached file (0 = off)
uint64_t resident_budget() {
    return (uint64_t)std::max<int64_t>(0, knob_value("FLS_SCAN_RESIDENT_MB")) << 20;
}
namespace {
uint64_t release_idle_images(int dev) {
    ImageRegistry &R = image_registry();
    ResidentSet<DevImage>::Evicted ev;
    std::lock_guard<std::mutex> lk(R.mu);
    const uint64_t b = R.set.release_idle(dev, ev);
    ev.clear();
    return b;
}
}  // namespace
void drop_file_images(const void *owner) {
    ImageRegistry &R = image_registry();
    ResidentSet<DevImage>::Evicted ev;
    std::lock_guard<std::mutex> lk(R.mu);
    R.set.drop_owner(owner, ev);
    ev.clear();
}

struct fls_table {
    std::vector<int> devices;          // the connection's GPUs (row groups shard over them)
    std::shared_ptr<MappedFile> mapped;  // fls_read_fls: the file and its validated metadata (shared)
    std::shared_ptr<ConnRes> res;      // the connection's scan resources (outlive a disconnect)
    std::vector<uint8_t> owned;
    const uint8_t *img = nullptr;
    uint64_t len = 0;
    FileMeta meta;
    std::vector<std::string> names;
    bool registered = false;        // img pinned with hipHostRegister (FLS_SCAN_PIN=1)
    bool pin_tried = false;
    void *map = nullptr;            // fls_read_fls: the file, mapped read-only
    size_t map_len = 0;

    // device-resident mode: one part per GPU (fls_device_upload)
    std::vector<std::unique_ptr<Resident>> resident;
    uint32_t launches = 0;

    ScanCtx scan, mat;
    std::vector<HostTerm> filter;   // fls_scan_filter: applies to the next fls_scan_begin
    bool dict_codes = false;        // fls_scan_dict_codes: applies to the next fls_scan_begin
    bool narrow = false;            // fls_scan_narrow: applies to the next fls_scan_begin
    bool defer_records = false;     // fls_scan_defer_records: applies to the next fls_scan_begin
    bool profiled = false;          // scanned with FLS_SCAN_PROFILE=1 (prints the totals at close)
    ~fls_table();
};

namespace {

int out_bytes_of(const fls_table *t, uint32_t c) { return type_out_bytes(t->meta.cols[c].type); }

// The validity bitmaps of chunk (rg, c) in the host image, or nullptr when the
// chunk has no NULL (fls_format.hpp "Validity")
const uint64_t *chunk_validity_host(const fls_table *t, uint32_t rg, uint32_t c) {
    const ChunkRef &ch = t->meta.rgs[rg].chunks[c];
    if (!chunk_has_validity(ch.hdr)) return nullptr;
    return (const uint64_t *)(t->img + ch.off + validity_off(ch.len, ch.hdr.nvec));
}

// Build host string_t tables for the VARCHAR chunks of [rg0, rg1) and upload.
int build_strtabs(const fls_table *t, int dev, uint32_t rg0, uint32_t rg1, DevBuf<StrT> &tab,
                  std::vector<uint64_t> &offs, std::vector<StrT> &host) {
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    offs.assign((size_t)(rg1 - rg0) * ncols, UINT64_MAX);
    host.clear();
    for (uint32_t r = rg0; r < rg1; ++r)
        for (uint32_t c = 0; c < ncols; ++c) {
            if (!type_is_string(t->meta.cols[c].type)) continue;
            const ChunkRef &ch = t->meta.rgs[r].chunks[c];
            if (ch.hdr.enc != ENC_DICT) continue;  // FSST strings are decoded on the GPU
            const uint8_t *aux = t->img + ch.off + ch.hdr.aux_off;
            const uint32_t n = ch.hdr.dict_count;
            offs[(size_t)(r - rg0) * ncols + c] = host.size();
            for (uint32_t i = 0; i < n; ++i) {
                const uint8_t *p;
                uint32_t len;
                dict_string(aux, n, i, p, len);
                host.push_back(make_string_t((const char *)p, len));
            }
        }
    HIP_TRY(hipSetDevice(dev));
    HIP_TRY(tab.alloc(dev, host.size()));
    if (!host.empty()) HIP_TRY(hipMemcpy(tab.p, host.data(), host.size() * sizeof(StrT), hipMemcpyHostToDevice));
    return 0;
}

// Describe chunk (rg, col) located at d_chunk_base (device) for the kernel.
// code_w (1 or 2): a DICT string chunk delivered as its codes, gathered from
// the identity table d_ident instead of the string_t dictionary
DevChunk make_devchunk(const fls_table *t, uint32_t rg, uint32_t col, const uint8_t *d_chunk, const uint8_t *d_dict,
                       uint8_t *d_out, ByteCount *bc, uint8_t *d_heap = nullptr, const uint8_t *h_heap = nullptr,
                       uint32_t code_w = 0, const uint8_t *d_ident = nullptr) {
    const ChunkRef &ch = t->meta.rgs[rg].chunks[col];
    const ChunkHeader &h = ch.hdr;
    DevChunk d;
    memset(&d, 0, sizeof(d));
    d.chunk = d_chunk;
    d.out = d_out;
    d.nvec = h.nvec;
    d.dict_count = h.dict_count;
    d.meta_off = (uint32_t)h.meta_off;
    d.packed_off = (uint32_t)h.packed_off;
    d.aux_off = (uint32_t)h.aux_off;
    d.enc = h.enc;
    d.T = h.T;
    d.vbits = h.vbits;
    d.ob = (uint8_t)out_bytes_of(t, col);
    if (h.enc == ENC_DICT) d.dict = h.is_str ? d_dict : d_chunk + h.aux_off;
    if (code_w && h.enc == ENC_DICT && h.is_str) {
        d.ob = (uint8_t)code_w;
        d.dict = code_w == 1 ? d_ident : d_ident + kIdent16;
    }
    bc->values += h.nvals;
    if (h.enc == ENC_FSST) {
        d.dict = d_heap;
        d.heap_host = (uint64_t)(uintptr_t)h_heap;
        d.heap_bytes = (uint32_t)h.reserved1;
        bc->out += (uint64_t)h.nvals * 16 + h.reserved1;
        bc->meta += 32ull * h.nvec + kFsstTableBytes;
        const uint8_t *meta = t->img + ch.off + h.meta_off;
        bool sp = true;
        for (uint32_t v = 0; v < h.nvec; ++v) {
            VecMeta vm;
            memcpy(&vm, meta + 32ull * v, 32);
            FsstVecHeader fh;
            memcpy(&fh, t->img + ch.off + h.aux_off + vm.aux_off, sizeof(fh));
            bc->packed += 128ull * vm.bw + 128ull * fh.clen_w + fh.comp_len;
            bc->meta += sizeof(fh);
            if (chunk_seg_codes(h) == kFsstSegCodes) bc->meta += sizeof(FsstSegHeader) + fsst_nseg(fh.comp_len);
            // string-parallel kernel iff every string of the chunk is <= 255
            // bytes, decompressed and compressed (bounds from the two FFOR streams)
            const uint64_t dmax = (uint64_t)vm.for_base + (vm.bw >= 32 ? 0xFFFFFFFFull : (1ull << vm.bw) - 1);
            const uint64_t cmax = (uint64_t)fh.clen_base + (fh.clen_w >= 32 ? 0xFFFFFFFFull : (1ull << fh.clen_w) - 1);
            if (vm.for_base < 0 || dmax > 255 || cmax > 255) sp = false;
        }
        // bit 1: segment tables (the segmented kernel; FLS_FSST_SEG=0 keeps
        // the code-parallel one, an A/B knob)
        // and symbols of at most 7 bytes (the segmented kernel stages each
        // symbol with its length in the top byte)
        const char *sg = getenv("FLS_FSST_SEG");
        bool short_syms = true;
        const uint8_t *lens = t->img + ch.off + h.aux_off + 8 * 256;
        for (uint32_t k = 0; k < h.dict_count && k < 255; ++k) short_syms &= lens[k] <= 7;
        const bool seg = chunk_seg_codes(h) == kFsstSegCodes && short_syms && !(sg && atoi(sg) == 0);
        d.vbits = (sp ? 1 : 0) | (seg ? 2 : 0);
        return d;  // separate kernels, fixed LDS layouts
    }
    bc->out += (uint64_t)h.nvals * d.ob;
    bc->meta += 32ull * h.nvec;
    const uint8_t *meta = t->img + ch.off + h.meta_off;
    uint32_t max_w = 0;
    for (uint32_t v = 0; v < h.nvec; ++v) {
        VecMeta vm;
        memcpy(&vm, meta + 32ull * v, 32);
        bc->packed += 128ull * vm.bw;
        max_w = std::max<uint32_t>(max_w, vm.bw);
        if (h.enc == ENC_DELTA) bc->meta += 128;
        if (h.enc == ENC_RLE) bc->meta += 128 + (uint64_t)vm.aux_count * (h.vbits / 8);
        if (h.enc == ENC_ALP && alp_exceptions(vm.aux_count))
            bc->meta += alp_aux_bytes(alp_exceptions(vm.aux_count), h.vbits);
    }
    if (h.enc == ENC_DICT) bc->meta += (uint64_t)h.dict_count * (h.is_str ? d.ob : h.vbits / 8);
    d.max_w = max_w;
    uint32_t pb, vb;
    chunk_lds_need(h.enc, h.T, d.ob, h.dict_count, max_w, pb, vb);
    bc->geom.p_bytes = std::max(bc->geom.p_bytes, pb);
    bc->geom.v_bytes = std::max(bc->geom.v_bytes, vb);
    return d;
}

bool col_selected(const std::vector<uint8_t> &mask, uint32_t c) { return mask.empty() || mask[c]; }

bool is_fsst(const fls_table *t, uint32_t rg, uint32_t c) { return t->meta.rgs[rg].chunks[c].hdr.enc == ENC_FSST; }

// Decode work distribution (A/B knob FLS_DECODE_POLICY, read per call so both
// arms run on the same buffers): 0 = work queue, largest chunks first
// (default); bit 0 = static grid-stride split; bit 1 = keep column order.
// bit 2 = full-width register prefetch for every chunk (descriptor max_w = T).
// bit 3 = FSST chunks with segment tables on the code-parallel kernel
// (FLS_FSST_SEG=0) instead of the segmented one.
// bit 4 = FSST rounds of 16 compressed bytes per lane instead of 8.
// bit 5 = balanced static split of vectors over the resident waves, chunks in
// file (row-group-major) order (balanced_split).  bit 6 = work queue even for
// small launches (launch_policy).  bit 7 = FSST chunks whose strings are all
// <= 255 bytes on the string-parallel kernel (default: every FSST chunk on the
// code-parallel kernel; same-buffer A/B profiles/r1/abenv_fsst_cp.txt).
enum : int {
    POLICY_STATIC = 1, POLICY_NO_LPT = 2, POLICY_FULL_PREFETCH = 4, POLICY_FSST_NOSEG = 8, POLICY_FSST16 = 16,
    POLICY_BALANCED = 32, POLICY_QUEUE = 64, POLICY_FSST_SP = 128
};
// Balanced-split knobs, folded into the policy word (so a change rebuilds the
// cached launch list): FLS_STATIC_PCT = % of the bytes split statically
// (bits 8-15, default 100), FLS_TAIL_PIECES = tail pieces per wave for the
// rest (bits 16-23, default 2), FLS_BLOCKS_PER_CU (bits 24-30, 0 = unset).
// Guided tail defaults (FLS_GUIDED_MIN_VECS / FLS_GUIDED_FACTOR, guided_split)
constexpr int kGuidedMinVecs = 0, kGuidedFactor = 2;
int64_t decode_policy() {
    const char *e = getenv("FLS_DECODE_POLICY");
    const char *sp = getenv("FLS_STATIC_PCT");
    const char *tp = getenv("FLS_TAIL_PIECES");
    const int pct = sp ? std::min(100, std::max(0, atoi(sp))) : 100;
    const int pieces = tp ? std::min(255, std::max(1, atoi(tp))) : 2;
    // FLS_BLOCKS_PER_CU (decode_grid_size) only enters the grid when the
    // launch list is rebuilt: fold it in so a change rebuilds it
    const char *bp = getenv("FLS_BLOCKS_PER_CU");
    const int bpc = bp ? std::min(127, std::max(0, atoi(bp))) : 0;
    // FLS_FSST_SEG=0 (make_devchunk: FSST chunks with segment tables go to the
    // code-parallel kernel) changes the descriptors: fold it in too
    const char *sg = getenv("FLS_FSST_SEG");
    const int noseg = sg && atoi(sg) == 0 ? POLICY_FSST_NOSEG : 0;
    // guided tail (guided_split): FLS_GUIDED_MIN_VECS = smallest piece in
    // vectors (bits 32-39, 0 = whole chunks only), FLS_GUIDED_FACTOR = pieces
    // per wave of the remaining work (bits 40-47)
    const char *gm = getenv("FLS_GUIDED_MIN_VECS");
    const char *gf = getenv("FLS_GUIDED_FACTOR");
    const int64_t gmin = gm ? std::min(64, std::max(0, atoi(gm))) : kGuidedMinVecs;
    const int64_t gfac = gf ? std::min(255, std::max(1, atoi(gf))) : kGuidedFactor;
    return (int64_t)(((e ? (atoi(e) & 0xFF) : 0) | noseg) | pct << 8 | pieces << 16 | bpc << 24) | gmin << 32 |
           gfac << 40;
}

// Policy for one launch: the default (no distribution bits) switches to the
// balanced split when the launch has fewer main-kernel chunks than resident
// waves (the scan pipeline's 8-row-group batches: ~120 chunks for ~4,096
// waves), where whole-chunk work items would leave most waves idle.  Large
// launches keep the work queue: same-buffer A/B on SF100 lineitem, c3 and c4
// found the split no faster than the queue (profiles/r1/abenv_bal_*.txt).
int64_t launch_policy(int64_t policy, const std::vector<DevChunk> &v, DecodeGeom &geom) {
    if (policy & (POLICY_STATIC | POLICY_BALANCED | POLICY_QUEUE)) return policy;
    size_t nmain = 0;
    for (const DevChunk &d : v) nmain += d.enc != ENC_FSST;
    if (geom.grid <= 0) geom.grid = decode_grid_size(4 * (geom.p_bytes + geom.v_bytes));
    return nmain < decode_waves(geom) ? (policy | POLICY_BALANCED) : policy;
}

// FSST chunks go last (their own kernels: string-parallel ones first, then
// code-parallel ones, each group numbering its vectors through vec_base);
// returns how many lead (main kernel) and the FSST counts
uint32_t order_for_launch(std::vector<DevChunk> &v, FsstCounts *fc, int64_t policy) {
    auto mid = std::stable_partition(v.begin(), v.end(), [](const DevChunk &d) { return d.enc != ENC_FSST; });
    std::stable_sort(mid, v.end(), [](const DevChunk &a, const DevChunk &b) {
        return fsst_group(a.vbits) < fsst_group(b.vbits);
    });
    if (policy & POLICY_FULL_PREFETCH)
        for (auto it = v.begin(); it != mid; ++it) it->max_w = it->T;
    if (policy & POLICY_BALANCED) {
        // file order = row-group-major: every wave's range mixes all columns
        // (paths that run slower per byte are spread over the waves)
        std::stable_sort(v.begin(), mid, [](const DevChunk &a, const DevChunk &b) { return a.chunk < b.chunk; });
    } else if (!(policy & (POLICY_STATIC | POLICY_NO_LPT))) {
        // largest output first: the work queue then ends the launch on small chunks
        std::stable_sort(v.begin(), mid, [](const DevChunk &a, const DevChunk &b) {
            return (uint64_t)a.nvec * a.ob > (uint64_t)b.nvec * b.ob;
        });
    }
    *fc = FsstCounts();
    for (auto it = mid; it != v.end(); ++it) {
        const int g = fsst_group(it->vbits);
        it->vec_base = fc->vecs[g];
        fc->vecs[g] += it->nvec;
        fc->n[g]++;
    }
    return (uint32_t)(mid - v.begin());
}

// Append the balanced split of the main chunks to the descriptor list (as
// extra DevChunk slots, so it uploads with it); plan.waves == 0 when the
// policy does not split.
SplitPlan append_split(std::vector<DevChunk> &list, uint32_t nmain, const DecodeGeom &geom, int64_t policy) {
    if (nmain == 0) return SplitPlan();
    std::vector<uint32_t> pos;
    SplitPlan plan;
    if (policy & POLICY_BALANCED)
        plan = balanced_split(list.data(), nmain, decode_waves(geom), (policy >> 8) & 0xFF, (policy >> 16) & 0xFF, pos);
    else if (!(policy & (POLICY_STATIC | POLICY_NO_LPT)) && ((policy >> 32) & 0xFF))
        plan = guided_split(list.data(), nmain, decode_waves(geom), (uint32_t)((policy >> 40) & 0xFF),
                            (uint32_t)((policy >> 32) & 0xFF), pos);
    else
        return SplitPlan();
    const size_t k = list.size();
    list.resize(k + (pos.size() * 4 + sizeof(DevChunk) - 1) / sizeof(DevChunk));
    memcpy(list.data() + k, pos.data(), pos.size() * 4);
    return plan;
}

// Overlap split (launch_all): blocks per CU of the narrow main decode grid
// and FSST waves per CU of the narrow FSST grid; knobs FLS_OVERLAP_DECODE_BPC /
// FLS_OVERLAP_FSST_WPC (0 FSST waves = no overlap).
// Overlap vs one-after-the-other at the per-GPU shares of 1/2/4/8-GPU runs
// (same-buffer A/B on lineitem_full, profiles/r2/abenv_overlap_scales.txt,
// abenv_sf12p5.txt, abenv_minvecs.txt, abenv_overlap_grid.txt,
// abenv_overlap_prio.txt): overlapped is faster at SF25 (5.90 vs 6.26 ms),
// SF50 (12.0 vs 12.9) and SF100 (23.1 vs 26.0, 23.9 vs 26.4); at SF12.5 (286
// FSST vectors per CU, the per-GPU share of an 8-GPU run) serial was faster on
// three boxes of four (3.41 vs 3.46, 3.11 vs 3.18, 3.36 vs 3.45 ms; 3.16 vs
// 3.09 on the fourth).  So launches with fewer than 400 FSST vectors per CU
// ran serially (FLS_OVERLAP_MIN_VECS_PER_CU).  With round 3's faster FSST
// kernel serial also wins at SF25 (572 vectors per CU: 6.41 vs 6.51 ms) and
// at SF12.5 against every split tried (3.22 vs 3.34-3.45 ms;
// profiles/r3/abenv_sf25_split_r3zl.txt, abenv_sf12_split_r3zl.txt), so the
// threshold is 800; SF50 (1,144 vectors per CU) and SF100 (2,288) stay
// overlapped: 11.17 vs 11.82 and 22.14 vs 23.80 ms (abenv_sf50_split_r3zm.txt,
// abenv_sf100_split_r3zm.txt).  The main kernel's wave issue
// priority while overlapped (FLS_OVERLAP_DECODE_PRIO, s_setprio 1-3) measured
// within 0.1 % of the default.
struct OverlapSplit {
    // 12 FSST waves per CU beside 1 decode block: 1.6-2 % faster than 16 at
    // SF100 and SF12.5 (profiles/r2/abenv_v12.txt)
    int decode_bpc = 1, fsst_wpc = 12;
    uint32_t min_vecs_per_cu = 800;
    int decode_prio = 0;  // FLS_OVERLAP_DECODE_PRIO: s_setprio of the main kernel's waves while overlapped
    // FLS_OVERLAP_CU_SPLIT = m in 1..31: the main decode starts on the CUs whose
    // index mod 32 is < m, FSST on the others, each kind alone on its CUs
    // (0 = the co-resident split above)
    int cu_split = 0;
    // FLS_OVERLAP_GUIDED=1: the overlapped decode grids drain the guided plan's
    // items (whole chunks, then pieces) instead of whole chunks
    bool guided = false;
};
OverlapSplit overlap_split() {
    OverlapSplit o;
    if (const char *e = getenv("FLS_OVERLAP_CU_SPLIT")) o.cu_split = std::min(31, std::max(0, atoi(e)));
    if (const char *e = getenv("FLS_OVERLAP_DECODE_BPC")) o.decode_bpc = std::max(1, atoi(e));
    if (const char *e = getenv("FLS_OVERLAP_FSST_WPC")) o.fsst_wpc = std::max(0, atoi(e));
    if (const char *e = getenv("FLS_OVERLAP_MIN_VECS_PER_CU")) o.min_vecs_per_cu = (uint32_t)std::max(0, atoi(e));
    if (const char *e = getenv("FLS_OVERLAP_DECODE_PRIO")) o.decode_prio = std::min(3, std::max(0, atoi(e)));
    if (const char *e = getenv("FLS_OVERLAP_GUIDED")) o.guided = atoi(e) != 0;
    return o;
}

// d_queue[0] = main decode work queue, [1 + g] = FSST piece counter of kernel
// group g (FsstCounts).
//
// Without a side stream (scan batches) the FSST kernels follow the main one
// on its stream.  With one (a table decode), the FSST kernels (VALU-bound)
// overlap the main decode kernel (HBM-bound):
//   main stream: narrow decode grid (decode_bpc blocks per CU), then a full
//                FSST grid;
//   side stream: narrow FSST grid (fsst_wpc waves per CU), then a full decode
//                grid.
// Every grid of a kind drains one shared queue (decode chunks / FSST pieces),
// so no work is done twice, and whichever kind runs out first, its stream
// follows with a full grid of the other kind onto the freed wave slots.  The
// split holds whichever kernel the hardware dispatches first.
// Measured on lineitem_full SF100 (same-buffer A/B, profiles/r1/abenv_overlap.txt):
// 26.7 ms serial -> 24.3 ms at 1 decode block + 12..20 FSST waves per CU
// (2 blocks + 8..12 waves: 24.7 ms).  The kernel trace shows the overlap phase
// moving ~4.9 TB/s together, below the 5.6 TB/s of the main kernel alone: the
// two compete for the CUs' LDS and issue slots as well as for HBM.
// The FSST kernels a launch with this policy and FLS_FSST_VARIANT would run
// must be in this build: the product library holds each kernel's default only
// (fls_fsst.hip), the experiment library every variant (make lab).  A stale
// tuning variable fails the decode with FLS_ERR_CONFIG instead of running a
// kernel it did not ask for.
int fsst_config_check(int64_t policy) {
    int variant = kFsstDefault;
    const char *fv = getenv("FLS_FSST_VARIANT");
    if (fv) {
        char *end = nullptr;
        const long v = strtol(fv, &end, 10);
        if (end == fv || *end != 0 || v < 0 || v > 0x7FFFFFFF)
            return fail(FLS_ERR_CONFIG, "FLS_FSST_VARIANT=%s is not a variant number", fv);
        variant = (int)v;
    }
    if (const char *fx = getenv("FLS_FUSED_X")) {  // the fused kernel's FSST-part bits (experiments)
        char *end = nullptr;
        const long x = strtol(fx, &end, 10);
        if (end == fx || *end != 0 || x < 0 || x > 0x7FFFFFFF || !fused_x_built((int)x))
            return fail(FLS_ERR_CONFIG,
                        "FLS_FUSED_X=%s is not in this build: the product library holds the default fused kernel "
                        "only; experiments need FLS_LIB=libflsgpu_lab.so (make lab) -- unset FLS_FUSED_X",
                        fx);
    }
    const int bpl = (policy & POLICY_FSST16) ? 16 : 8;
    if (!fsst_variant_built(variant, true, bpl) || !fsst_variant_built(variant, false, bpl))
        return fail(FLS_ERR_CONFIG,
                    "FSST kernel variant %d (%d bytes per lane) is not in this build: the product library holds the "
                    "default kernels only; experiments need FLS_LIB=libflsgpu_lab.so (make lab)%s",
                    variant, bpl, fv ? " -- unset FLS_FSST_VARIANT" : "");
    return 0;
}

constexpr uint32_t kQueueWords = 1 + kFsstGroups;

// Fused launch knobs (launch_all -> launch_fused): the default for a table
// decode whose FSST chunks are of one segmented kind; FLS_FUSED=0 turns it
// off (serial or overlapped kernels), FLS_FUSED=1 forces it even without FSST
// chunks (the main decode alone in the fused kernel: 2 % slower, A/B only),
// FLS_FUSED_FSST16 = waves of every 16 that start on FSST, FLS_FUSED_PIECE =
// FSST vectors per queue item, FLS_FUSED_WPC = waves per CU (0: as many as
// fit), FLS_FUSED_STATIC_PCT = % of the FSST vectors the FSST-first waves
// split statically before the queue, FLS_FUSED_MIN_VECS_PER_CU = the FSST
// vectors per CU below which the launch stays serial.
struct FusedCfg {
    // 0 off; 1 (default) launches with main chunks and FSST chunks of one
    // segmented kind; 2 (FLS_FUSED=1) also launches with only one of the two
    int mode = 1;
    uint32_t min_vecs_per_cu = 0;
    bool per16_set = false;  // FLS_FUSED_FSST16 given (else by launch size, launch_all)
    bool variant = false;    // a non-default FLS_FSST_VARIANT: no fused launch
    FusedLaunch how;
};
FusedCfg fused_cfg() {
    FusedCfg f;
    if (const char *e = getenv("FLS_FUSED")) f.mode = std::min(2, std::max(0, atoi(e) == 1 ? 2 : atoi(e)));
    if (const char *e = getenv("FLS_FUSED_FSST16")) {
        f.how.fsst_per16 = (uint32_t)std::min(16, std::max(0, atoi(e)));
        f.per16_set = true;
    }
    if (const char *e = getenv("FLS_FUSED_PIECE")) f.how.piece = (uint32_t)std::min(64, std::max(1, atoi(e)));
    if (const char *e = getenv("FLS_FUSED_WPC")) f.how.waves_per_cu = std::max(0, atoi(e));
    if (const char *e = getenv("FLS_FUSED_STATIC_PCT")) f.how.fsst_static_pct = (uint32_t)std::min(100, std::max(0, atoi(e)));
    if (const char *e = getenv("FLS_FUSED_STATIC_FIRST")) f.how.static_first = atoi(e) != 0;
    if (const char *e = getenv("FLS_FUSED_HALVING")) f.how.halving = atoi(e) != 0;
    if (const char *e = getenv("FLS_FUSED_TAIL")) f.how.tail_chunks = (uint32_t)std::max(0, atoi(e));
    if (const char *e = getenv("FLS_FUSED_TAIL_SPLIT")) f.how.tail_split = (uint32_t)std::min(64, std::max(1, atoi(e)));
    if (const char *e = getenv("FLS_FUSED_X")) f.how.x = atoi(e);
    if (const char *e = getenv("FLS_FUSED_MIN_VECS_PER_CU")) f.min_vecs_per_cu = (uint32_t)std::max(0, atoi(e));
    // an FSST kernel variant A/B (FLS_FSST_VARIANT, experiment library) runs
    // the standalone FSST kernels: the fused kernel holds only the default's
    // FSST part, so fusing would measure the default instead
    if (const char *e = getenv("FLS_FSST_VARIANT"))
        if (atoi(e) != kFsstDefault) f.variant = true;
    return f;
}

// CU-partitioned overlap: the main decode (HBM-bound) and the FSST kernels
// (VALU / LDS-bound) each start alone on their own CU set instead of sharing
// every CU's LDS and issue slots (the co-resident split lost to running them
// one after the other at the 8-GPU share, profiles/r3/abenv_sf12_split_r3zl.txt):
//   stream A (CUs with index mod 32 < m): full decode grid, then FSST;
//   stream B (the other CUs):             full FSST grid, then decode.
// Both kinds drain shared queues, so whichever set finishes its kind first
// joins the other.  A mask that takes m of every 32 CU indices gives each XCD
// the same share whether the mask's bits run XCD by XCD or round-robin over
// the XCDs (m a multiple of 8).
template <class LaunchGroup>
hipError_t launch_cu_split(const DevChunk *d_chunks, uint32_t nmain, const FsstCounts &fc, uint32_t *d_err,
                           const DecodeGeom &geom, hipStream_t stream, uint32_t *d_queue, SideStream *side,
                           const OverlapSplit &ov, int cus, const FsstLaunch (&how)[kFsstGroups],
                           LaunchGroup &launch_group) {
    const int m = ov.cu_split;
    uint32_t mask_a[8] = {}, mask_b[8] = {};
    int na = 0, nb = 0;
    for (int i = 0; i < std::min(cus, 256); ++i) {
        if (i % 32 < m) {
            mask_a[i / 32] |= 1u << (i % 32);
            ++na;
        } else {
            mask_b[i / 32] |= 1u << (i % 32);
            ++nb;
        }
    }
    if (na == 0 || nb == 0) return hipErrorInvalidValue;
    if (side->cu_m != m) {
        side->release_cu();
        hipError_t e = hipExtStreamCreateWithCUMask(&side->cu_a, 8, mask_a);
        if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&side->cu_b, 8, mask_b);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&side->join_a, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&side->join_b, hipEventDisableTiming);
        if (e != hipSuccess) {
            side->release_cu();
            return e;
        }
        side->cu_m = m;
    }
    const uint32_t shmem = 4 * (geom.p_bytes + geom.v_bytes);
    const int bpc = std::max(1, (geom.grid > 0 ? geom.grid : decode_grid_size(shmem)) / std::max(1, cus));
    DecodeGeom ga = geom, gb = geom;
    ga.grid = na * bpc;
    gb.grid = nb * bpc;
    FsstLaunch ha[kFsstGroups], hb[kFsstGroups];
    for (int g = 0; g < kFsstGroups; ++g) {
        ha[g] = hb[g] = how[g];
        ha[g].queue = hb[g].queue = d_queue + 1 + g;
        ha[g].reset_queue = hb[g].reset_queue = false;
        ha[g].grid_cus = na;
        hb[g].grid_cus = nb;
    }
    hipError_t e = hipMemsetAsync(d_queue, 0, kQueueWords * sizeof(uint32_t), stream);
    if (e == hipSuccess) e = hipEventRecord(side->fork, stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(side->cu_a, side->fork, 0);
    if (e == hipSuccess) e = hipStreamWaitEvent(side->cu_b, side->fork, 0);
    if (e == hipSuccess)
        e = launch_decode(d_chunks, nmain, d_err, ga, side->cu_a, d_queue, nullptr, SplitPlan(), true, ov.decode_prio);
    for (int g = 0; g < kFsstGroups && e == hipSuccess; ++g) e = launch_group(g, side->cu_b, hb[g]);
    if (e == hipSuccess)
        e = launch_decode(d_chunks, nmain, d_err, gb, side->cu_b, d_queue, nullptr, SplitPlan(), true, ov.decode_prio);
    for (int g = 0; g < kFsstGroups && e == hipSuccess; ++g) e = launch_group(g, side->cu_a, ha[g]);
    if (e == hipSuccess) e = hipEventRecord(side->join_a, side->cu_a);
    if (e == hipSuccess) e = hipEventRecord(side->join_b, side->cu_b);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, side->join_a, 0);
    if (e == hipSuccess) e = hipStreamWaitEvent(stream, side->join_b, 0);
    return e;
}

hipError_t launch_all(const DevChunk *d_chunks, uint32_t nmain, uint32_t ntotal, const FsstCounts &fc,
                      uint32_t *d_err, const DecodeGeom &geom, hipStream_t stream, uint32_t *d_queue, int64_t policy,
                      SplitPlan plan, const SideStream *side = nullptr) {
    // a guided plan only orders the serial launch: the overlapped and
    // CU-split launches drain whole chunks from a queue several grids share
    const uint32_t *d_split = plan.waves ? reinterpret_cast<const uint32_t *>(d_chunks + ntotal) : nullptr;
    const bool balanced = d_split && !plan.guided;
    const bool sp = (policy & POLICY_FSST_SP) != 0;
    const OverlapSplit ov = overlap_split();
    FsstLaunch how[kFsstGroups];
    for (int g = 0; g < kFsstGroups; ++g) {
        how[g].bytes_per_lane = (policy & POLICY_FSST16) ? 16 : 8;
        if (const char *fv = getenv("FLS_FSST_VARIANT")) how[g].variant = atoi(fv);  // fsst_config_check'ed
        how[g].small = g == 0 || g == 2;
        how[g].seg = g < 2;
        if (const char *sc = getenv("FLS_FSST_SEG_CAP")) how[g].seg_cap = atoi(sc);
    }
    auto launch_group = [&](int g, hipStream_t st, const FsstLaunch &h) -> hipError_t {
        const DevChunk *dc = d_chunks + nmain + fc.first(g);
        if (g == 2 && sp && !h.queue) return launch_fsst_sp(dc, fc.n[g], fc.vecs[g], d_err, st);
        return launch_fsst(dc, fc.n[g], fc.vecs[g], d_err, st, h);
    };
    const int cus = device_cus();
    const uint64_t fsst_vecs = fc.total_vecs();
    if (ov.cu_split > 0 && side && side->stream && nmain > 0 && fsst_vecs > 0 && !balanced && !sp &&
        !(policy & POLICY_STATIC))
        return launch_cu_split(d_chunks, nmain, fc, d_err, geom, stream, d_queue, const_cast<SideStream *>(side),
                               ov, cus, how, launch_group);
    // fused: one kernel pulling main chunks and FSST pieces from two queues
    // (launch_fused), when every FSST chunk is of one segmented kind
    {
        const FusedCfg fz = fused_cfg();
        int g1 = -1, ng = 0;
        for (int g = 0; g < kFsstGroups; ++g)
            if (fc.n[g]) {
                g1 = g;
                ++ng;
            }
        if (fz.mode > 0 && !fz.variant && ((ng == 1 && nmain > 0) || fz.mode == 2) && ng <= 1 && g1 < 2 && !balanced && !sp &&
            !(policy & POLICY_STATIC) &&
            fsst_vecs >= (uint64_t)fz.min_vecs_per_cu * (uint64_t)cus) {
            const int g = std::max(0, g1);  // (no FSST chunks: the main decode alone, in the fused kernel)
            // waves starting on FSST: 6 of 16 for large launches (SF100:
            // 21.79 ms against 21.93 with 5), 5 below 1,000 FSST vectors per
            // CU (SF12.5: 3.115 against 3.133 ms with 6; profiles/r5/)
            FusedLaunch how = fz.how;
            if (!fz.per16_set) how.fsst_per16 = fsst_vecs < 1000ull * (uint64_t)cus ? 5u : 6u;
            return launch_fused(d_chunks, nmain, d_chunks + nmain + fc.first(g), fc.n[g], fc.vecs[g], g == 0, d_err,
                                geom, stream, d_queue, how);
        }
    }
    const bool overlap = side && side->stream && ov.fsst_wpc > 0 && nmain > 0 && fsst_vecs > 0 &&
                         fsst_vecs >= (uint64_t)ov.min_vecs_per_cu * (uint64_t)cus && !balanced && !sp &&
                         !(policy & POLICY_STATIC);
    hipError_t e = hipSuccess;
    if (overlap) {
        DecodeGeom narrow = geom;
        const uint32_t shmem = 4 * (geom.p_bytes + geom.v_bytes);
        narrow.grid = std::min(geom.grid > 0 ? geom.grid : decode_grid_size(shmem), cus * ov.decode_bpc);
        e = hipMemsetAsync(d_queue, 0, kQueueWords * sizeof(uint32_t), stream);
        if (e == hipSuccess) e = hipEventRecord(side->fork, stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(side->stream, side->fork, 0);
        FsstLaunch narrow_how[kFsstGroups];
        for (int g = 0; g < kFsstGroups; ++g) {
            how[g].queue = d_queue + 1 + g;
            how[g].reset_queue = false;
            narrow_how[g] = how[g];
            narrow_how[g].waves_per_cu = ov.fsst_wpc;
        }
        // main stream: narrow decode, then full FSST
        // (a guided plan: both decode grids drain its items from the shared queue)
        const uint32_t *gs = d_split && plan.guided && ov.guided ? d_split : nullptr;
        const SplitPlan gp = gs ? plan : SplitPlan();
        if (e == hipSuccess)
            e = launch_decode(d_chunks, nmain, d_err, narrow, stream, d_queue, gs, gp, true, ov.decode_prio);
        // side stream: narrow FSST, then full decode
        for (int g = 0; g < kFsstGroups && e == hipSuccess; ++g) e = launch_group(g, side->stream, narrow_how[g]);
        if (e == hipSuccess)
            e = launch_decode(d_chunks, nmain, d_err, geom, side->stream, d_queue, gs, gp, true, ov.decode_prio);
        for (int g = 0; g < kFsstGroups && e == hipSuccess; ++g) e = launch_group(g, stream, how[g]);
        if (e == hipSuccess) e = hipEventRecord(side->join, side->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, side->join, 0);
        return e;
    }
    e = launch_decode(d_chunks, nmain, d_err, geom, stream, (policy & POLICY_STATIC) ? nullptr : d_queue, d_split, plan);
    // FSST groups in order; chunks whose strings are all <= 255 bytes without
    // segment tables go to the string-parallel kernel under POLICY_FSST_SP
    for (int g = 0; g < kFsstGroups && e == hipSuccess; ++g) e = launch_group(g, stream, how[g]);
    return e;
}

}  // namespace

fls_table::~fls_table() {
    if (profiled && ScanProf::on()) scan_prof().print();
    resident.clear();
    // the scan pipelines go back to the connection (synchronised first: their
    // copies may read the image or the pinned stage)
    for (ScanCtx *s : {&scan, &mat})
        for (auto &d : s->devs) {
            if (d) {
                d->sync();
                d->dimg.reset();  // the resident image stays with the open-file cache entry
            }
            if (res) res->give(std::move(d));
            d.reset();
        }
    if (registered) hipHostUnregister((void *)img);
    if (map) munmap(map, map_len);
}

// ------------------------------------------------------------------------------
// scan pipeline

namespace {

// May any row of row group rg satisfy term h?  (zone maps / dictionary)
bool term_may_match(const fls_table *t, uint32_t rg, const HostTerm &h) {
    const RowGroupMeta &r = t->meta.rgs[rg];
    const ChunkRef &ch = r.chunks[h.col];
    // NULLs: the chunk's validity flag, and the zone map's all-NULL mark
    const bool all_null = !r.zones.empty() && (r.zones[h.col].flags & ZM_ALL_NULL);
    if (h.op == OP_FALSE) return false;
    if (h.op == OP_IS_NULL) return chunk_has_validity(ch.hdr);
    if (h.op == OP_IS_NOT_NULL) return !all_null;
    if (all_null) return false;  // no valid row to compare
    if (h.kind == FK_STR) {
        if (ch.hdr.enc != ENC_DICT) return true;  // FSST: no statistics
        const uint8_t *aux = t->img + ch.off + ch.hdr.aux_off;
        for (uint32_t i = 0; i < ch.hdr.dict_count; ++i) {
            const uint8_t *p;
            uint32_t len;
            dict_string(aux, ch.hdr.dict_count, i, p, len);
            if (op_holds(h.op, cmp_bytes(p, len, (const uint8_t *)h.str.data(), (uint32_t)h.str.size())))
                return true;
        }
        return false;
    }
    if (r.zones.empty() || !(r.zones[h.col].flags & ZM_VALID)) return true;
    const ZoneMap &z = r.zones[h.col];
    int cmin, cmax;  // min vs constant, max vs constant
    if (h.kind == FK_INT) {
        cmin = cmp_int((int64_t)z.min, (int64_t)h.value);
        cmax = cmp_int((int64_t)z.max, (int64_t)h.value);
    } else if (h.kind == FK_UINT) {
        cmin = cmp_uint(z.min, h.value);
        cmax = cmp_uint(z.max, h.value);
    } else {
        const double nan = __builtin_nan("");
        const double lo = (z.flags & ZM_ALL_NAN) ? nan : as_double(z.min);
        const double hi = (z.flags & ZM_HAS_NAN) ? nan : as_double(z.max);
        cmin = cmp_float(lo, as_double(h.value));
        cmax = cmp_float(hi, as_double(h.value));
    }
    switch (h.op) {
    case OP_EQ: return cmin <= 0 && cmax >= 0;
    case OP_NE: return !(cmin == 0 && cmax == 0);
    case OP_LT: return cmin < 0;
    case OP_LE: return cmin <= 0;
    case OP_GT: return cmax > 0;
    default: return cmax >= 0;  // OP_GE
    }
}

// Every clause has a term that may match (terms sorted by clause).
bool rowgroup_may_match(const fls_table *t, uint32_t rg, const std::vector<HostTerm> &terms) {
    size_t i = 0;
    while (i < terms.size()) {
        bool any = false;
        const uint32_t cl = terms[i].clause;
        for (; i < terms.size() && terms[i].clause == cl; ++i) any = any || term_may_match(t, rg, terms[i]);
        if (!any) return false;
    }
    return true;
}

// The file's resident image on GPU dev (made on first use), or none: a table
// not read from a file, FLS_SCAN_RESIDENT_MB=0, or no room in the GPU's image
// budget (FLS_SCAN_RESIDENT_MB, default 65,536 MB, over every cached file)
// after evicting the least recently used images no running scan holds.  The
// image holds the file bytes of shard g of G: the row groups this GPU owns
// when the whole table is split over the connection's GPUs.
std::shared_ptr<DevImage> resident_image(fls_table *t, int dev, uint32_t g, uint32_t G) {
    if (!t->mapped) return nullptr;
    const uint64_t budget = resident_budget();
    const uint32_t N = (uint32_t)t->meta.rgs.size();
    G = std::max(1u, G);
    const uint32_t r0 = (uint32_t)((uint64_t)N * g / G), r1 = (uint32_t)((uint64_t)N * (g + 1) / G);
    if (budget == 0 || r0 >= r1) return nullptr;
    uint64_t lo, hi;
    rg_byte_range(t->meta, r0, r1, lo, hi);
    if (hi <= lo) return nullptr;
    const uint64_t need = hi - lo + kImagePad;
    ImageRegistry &R = image_registry();
    ResidentSet<DevImage>::Evicted ev;  // freed under the lock: the new image may need their memory
    std::lock_guard<std::mutex> lk(R.mu);
    if (auto p = R.set.find(t->mapped.get(), dev, lo, hi)) return p;
    // an image made for another split of the table that another scan decodes
    // from: use it (batches outside it stream); idle ones overlapping this
    // shard are replaced
    if (auto p = R.set.find_held_overlap(t->mapped.get(), dev, lo, hi)) return p;
    R.set.drop_overlap(t->mapped.get(), dev, lo, hi, ev);
    ev.clear();
    if (!R.set.make_room(dev, need, budget, ev)) return nullptr;
    ev.clear();
    if (hipSetDevice(dev) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    // leave at least half of the free HBM to the scans' own buffers: evict
    // more idle images (least recent first) while the new one would not
    for (;;) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        if (need <= free_b / 2) break;
        if (!R.set.evict_lru(dev, ev)) return nullptr;
        ev.clear();
    }
    auto di = std::make_shared<DevImage>();
    di->dev = dev;
    hipError_t e = hipMalloc((void **)&di->p, need);
    if (e == hipErrorOutOfMemory && R.set.release_idle(dev, ev) > 0) {
        (void)hipGetLastError();
        ev.clear();
        e = hipMalloc((void **)&di->p, need);
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        di->p = nullptr;
        return nullptr;
    }
    di->lo = lo;
    di->hi = hi;
    di->nrg = N;
    di->present.reset(new std::atomic<uint8_t>[N]);
    for (uint32_t r = 0; r < N; ++r) di->present[r].store(0);
    R.set.insert(t->mapped.get(), dev, lo, hi, need, di);
    if (debug_enabled())
        fprintf(stderr, "DEBUG: resident image of row groups [%u, %u) on GPU %d: %llu bytes (%llu of %llu MB in use)\n",
                r0, r1, dev, (unsigned long long)need, (unsigned long long)(R.set.used(dev) >> 20),
                (unsigned long long)(budget >> 20));
    return di;
}

int scan_setup(fls_table *t, ScanCtx &s, const std::vector<int> &devs, const uint8_t *col_mask, uint32_t rg0,
               uint32_t rg1, const std::vector<HostTerm> *filter) {
    ProfTimer prof(PROF_SETUP);
    t->profiled = t->profiled || ScanProf::on();
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    if (rg1 > t->meta.rgs.size() || rg0 > rg1) return fail(FLS_ERR_ARG, "row-group range [%u,%u) out of bounds", rg0, rg1);
    // tear down a previous scan on this context
    for (auto &dp : s.devs) {
        ScanDev &d = *dp;
        d.sync();
        for (auto &sl : d.slots) {
            sl.busy = false;
            sl.starved = false;
            sl.hb = nullptr;
        }
        // every host batch back to the pool (a row group still held from the
        // previous scan is invalid from here on, as documented in flsgpu.h)
        d.free_batches.clear();
        for (auto &b : d.batches) d.free_batches.push_back(b.get());
    }
    s.out.clear();
    s.ready.clear();
    s.mask.assign(ncols, 1);
    if (col_mask)
        for (uint32_t c = 0; c < ncols; ++c) s.mask[c] = col_mask[c] ? 1 : 0;
    s.terms.clear();
    if (filter) s.terms = *filter;
    s.dict_codes = filter != nullptr && t->dict_codes;  // scans (not materialize) only
    s.narrow = filter != nullptr && t->narrow;
    s.defer_records = filter != nullptr && t->defer_records;
    s.dmask = s.mask;
    for (auto &h : s.terms)
        if (h.op < OP_IS_NULL) s.dmask[h.col] = 1;
    // row-group pruning on zone maps / dictionaries
    s.rgs.clear();
    s.pruned = 0;
    for (uint32_t r = rg0; r < rg1; ++r) {
        if (s.terms.empty() || rowgroup_may_match(t, r, s.terms)) s.rgs.push_back(r);
        else s.pruned++;
    }
    s.cur = 0;
    s.held = -1;
    s.err_rc = 0;
    s.err_msg.clear();
    if (s.rgs.empty()) {  // an empty table or range, or every row group pruned: no device work
        s.active = true;
        return 0;
    }
    const uint32_t G = (uint32_t)devs.size(), n = (uint32_t)s.rgs.size();
    // one pipeline per GPU of this scan, borrowed from the connection (kept
    // from the previous scan of this context when it targets the same GPUs)
    bool same = s.devs.size() == G;
    for (uint32_t g = 0; same && g < G; ++g) same = s.devs[g] && s.devs[g]->dev == devs[g];
    if (!same) {
        for (auto &d : s.devs) t->res->give(std::move(d));
        s.devs.clear();
        for (uint32_t g = 0; g < G; ++g) s.devs.push_back(t->res->take(devs[g]));
    }
    s.batch = (uint32_t)std::max<int64_t>(1, knob_value("FLS_SCAN_BATCH"));
    s.early_refill = knob_value("FLS_SCAN_EARLY_REFILL") != 0;
    s.spin_wait = getenv("FLS_SCAN_SPIN_WAIT") && atoi(getenv("FLS_SCAN_SPIN_WAIT")) != 0;
    s.max_batches = (uint32_t)std::max<int64_t>(2, knob_value("FLS_SCAN_HOST_BATCHES"));
    s.nslots = (int)std::max<int64_t>(1, std::min<int64_t>(ScanDev::kMaxSlots, knob_value("FLS_SCAN_SLOTS")));
    for (uint32_t g = 0; g < G; ++g) {
        ScanDev &d = *s.devs[g];
        HIP_TRY(hipSetDevice(d.dev));
        if (!d.stream) HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        for (auto &sl : d.slots) {
            if (!sl.stream) HIP_TRY(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
            sl.d_out.resize(ncols);
        }
        // contiguous shard of the surviving row groups
        d.p0 = (uint32_t)((uint64_t)n * g / G);
        d.p1 = (uint32_t)((uint64_t)n * (g + 1) / G);
        d.next_p = d.p0;
        d.rg0 = d.p0 < d.p1 ? s.rgs[d.p0] : 0;
        d.rg1 = d.p0 < d.p1 ? s.rgs[d.p1 - 1] + 1 : 0;
        {   // the image holds this GPU's shard of the table over the connection's GPUs;
            // a GPU the connection lists k times holds k shards: pipeline g
            // takes the shard of the listing that is its own occurrence
            uint32_t occ = 0;
            for (uint32_t h = 0; h < g; ++h) occ += s.devs[h]->dev == d.dev;
            uint32_t shard = 0, seen = 0;
            bool in = false;
            for (uint32_t k = 0; k < (uint32_t)t->devices.size() && !in; ++k)
                if (t->devices[k] == d.dev && seen++ == occ) {
                    shard = k;
                    in = true;
                }
            ProfTimer pi(PROF_IMAGE);
            d.dimg = resident_image(t, d.dev, in ? shard : 0u, in ? (uint32_t)t->devices.size() : 1u);
        }
        int rc;
        {
            ProfTimer ps(PROF_STRTABS);
            rc = build_strtabs(t, d.dev, d.rg0, d.rg1, d.strtab, d.strtab_off, d.h_strtab);
        }
        if (rc) return rc;
        if (s.dict_codes && !d.ident.p) {
            std::vector<uint8_t> id(kIdent16 + 2 * 65536);
            for (uint32_t i = 0; i < 256; ++i) id[i] = (uint8_t)i;
            for (uint32_t i = 0; i < 65536; ++i) memcpy(&id[kIdent16 + 2 * i], &i, 2);
            HIP_TRY(d.ident.alloc(d.dev, id.size()));
            HIP_TRY(hipMemcpy(d.ident.p, id.data(), id.size(), hipMemcpyHostToDevice));
        }
        HIP_TRY(d.err.alloc(d.dev, 1));
        HIP_TRY(hipMemsetAsync(d.err.p, 0, sizeof(uint32_t), d.stream));
        HIP_TRY(hipStreamSynchronize(d.stream));
    }
    // batches are staged from the image into a pinned buffer per slot by the
    // connection's copy threads (enqueue_batch); FLS_SCAN_PIN=1 instead pins
    // the whole image once (hipHostRegister: no host copies afterwards, but
    // ~0.12 s per GB before the first batch can move)
    static const bool pin = getenv("FLS_SCAN_PIN") && atoi(getenv("FLS_SCAN_PIN")) != 0;
    if (pin && !t->pin_tried && t->len > 0) {
        t->pin_tried = true;
        if (hipHostRegister((void *)t->img, t->len, hipHostRegisterDefault) == hipSuccess) t->registered = true;
        else (void)hipGetLastError();
    }
    s.active = true;
    return 0;
}

// Filter descriptors of a batch: the terms over the slot's decoded columns,
// the delivered columns' compaction targets, then the constant strings.
int enqueue_filter(fls_table *t, ScanCtx &s, ScanDev &d, Slot &sl, uint64_t rows, uint64_t in_lo, uint64_t in_len) {
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    std::vector<DevOut> outs;
    for (uint32_t c = 0; c < ncols; ++c) {
        if (!col_selected(s.mask, c)) continue;
        DevOut o;
        memset(&o, 0, sizeof(o));
        o.src = sl.hb->narrowed[c] ? sl.d_narrow[c].p : sl.d_out[c].p;
        o.dst = sl.hb->h_out[c].p;
        o.ob = sl.hb->ob[c];
        outs.push_back(o);
    }
    // validity words of the batch rows for every filtered column with a NULL
    // in the batch (row groups start at whole vectors: rows / 64 words apart)
    sl.d_valid.resize(ncols);
    std::vector<uint8_t> need(ncols, 0);
    for (auto &h : s.terms) need[h.col] = 1;
    for (uint32_t c = 0; c < ncols; ++c) {
        bool any = false;
        for (uint32_t r = sl.rg0; need[c] && r < sl.rg0 + sl.nrg; ++r)
            any = any || chunk_has_validity(t->meta.rgs[r].chunks[c].hdr);
        if (!any) {
            need[c] = 0;
            continue;
        }
        HIP_TRY(sl.d_valid[c].alloc(d.dev, (rows + 63) / 64 + 16));
        for (uint32_t r = sl.rg0; r < sl.rg0 + sl.nrg; ++r) {
            const ChunkRef &ch = t->meta.rgs[r].chunks[c];
            uint64_t *dst = sl.d_valid[c].p + (t->meta.rgs[r].first_row - t->meta.rgs[sl.rg0].first_row) / 64;
            const size_t bytes = (size_t)kValidityVecBytes * ch.hdr.nvec;
            if (chunk_has_validity(ch.hdr))
                HIP_TRY(hipMemcpyAsync(dst, sl.in_dev + (ch.off - in_lo) + validity_off(ch.len, ch.hdr.nvec), bytes,
                                       hipMemcpyDeviceToDevice, sl.stream));
            else
                HIP_TRY(hipMemsetAsync(dst, 0xFF, bytes, sl.stream));
        }
    }
    const size_t nt = s.terms.size(), no = outs.size();
    size_t str_bytes = 0;
    for (auto &h : s.terms) str_bytes += (h.str.size() + 15) & ~size_t(15);
    const size_t bytes = nt * sizeof(DevTerm) + no * sizeof(DevOut) + str_bytes;
    HIP_TRY(sl.h_fdesc.alloc(bytes));
    HIP_TRY(sl.d_fdesc.alloc(d.dev, bytes));
    uint8_t *fd = sl.h_fdesc.p;
    DevTerm *terms = (DevTerm *)fd;
    size_t so = nt * sizeof(DevTerm) + no * sizeof(DevOut);
    for (size_t i = 0; i < nt; ++i) {
        const HostTerm &h = s.terms[i];
        DevTerm &dt = terms[i];
        memset(&dt, 0, sizeof(dt));
        dt.col = sl.d_out[h.col].p;
        dt.value = h.value;
        dt.kind = h.kind;
        dt.op = h.op;
        dt.ob = (uint8_t)out_bytes_of(t, h.col);
        dt.end_clause = (i + 1 == nt || s.terms[i + 1].clause != h.clause) ? 1 : 0;
        dt.valid = need[h.col] ? sl.d_valid[h.col].p : nullptr;
        if (h.kind == FK_STR) {
            memcpy(fd + so, h.str.data(), h.str.size());
            dt.str = sl.d_fdesc.p + so;
            dt.str_len = (uint32_t)h.str.size();
            so += (h.str.size() + 15) & ~size_t(15);
            if (sl.heap_bytes[h.col]) {  // FSST: long strings live in the batch heap
                dt.host_lo = (uint64_t)(uintptr_t)sl.hb->h_heap[h.col].p;
                dt.host_hi = dt.host_lo + sl.heap_bytes[h.col];
                dt.dev_delta = (int64_t)((uintptr_t)sl.d_heap[h.col].p - (uintptr_t)sl.hb->h_heap[h.col].p);
            } else {  // DICT: long strings point into the file image, uploaded as d_in
                dt.host_lo = (uint64_t)(uintptr_t)(t->img + in_lo);
                dt.host_hi = dt.host_lo + in_len;
                dt.dev_delta = (int64_t)((uintptr_t)sl.in_dev - (uintptr_t)(t->img + in_lo));
            }
        }
    }
    memcpy(fd + nt * sizeof(DevTerm), outs.data(), no * sizeof(DevOut));
    HIP_TRY(hipMemcpyAsync(sl.d_fdesc.p, fd, bytes, hipMemcpyHostToDevice, sl.stream));
    HostBatch &hb = *sl.hb;
    hb.nvec = (uint32_t)((rows + 1023) / 1024);
    HIP_TRY(sl.d_mask.alloc(d.dev, (size_t)hb.nvec * 16));
    HIP_TRY(sl.d_counts.alloc(d.dev, hb.nvec));
    HIP_TRY(hb.h_counts.alloc(hb.nvec));
    HIP_TRY(hb.h_sel.alloc(std::max<uint64_t>(rows, 1)));
    HIP_TRY(launch_filter((const DevTerm *)sl.d_fdesc.p, (uint32_t)nt, (uint32_t)rows, sl.d_mask.p, sl.d_counts.p,
                          d.err.p, sl.stream));
    HIP_TRY(launch_compact((const DevOut *)(sl.d_fdesc.p + nt * sizeof(DevTerm)), (uint32_t)no, sl.d_mask.p,
                           sl.d_counts.p, (uint32_t)rows, t->meta.rowgroup_size, hb.h_sel.p, sl.stream));
    HIP_TRY(hipMemcpyAsync(hb.h_counts.p, sl.d_counts.p, hb.nvec * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           sl.stream));
    hb.sel_ready = false;
    return 0;
}

// enqueue the next batch of device d into slot si: up to s.batch consecutive
// surviving row groups
// A slot's refill in two parts.  claim_batch (with s.mu held) takes the
// slot's next row groups and a host batch; fill_batch (without s.mu: the
// staging copy, descriptors, H2D, launches and D2H of a batch take about a
// millisecond, and every consumer's acquire and release needs s.mu) enqueues
// its work; the slot turns busy (visible to acquire) only once its event is
// recorded.  The read_fastlanes profile of round 3's inline refill: of 1.8 s
// of scan-thread time (16 threads, lineitem_full SF10), 1.2 s was waiting for
// the claim lock while one thread ran a refill (profiles/r4/).
int fill_batch(fls_table *t, ScanCtx &s, ScanDev &d, int si);
int claim_batch(fls_table *t, ScanCtx &s, ScanDev &d, int si) {
    Slot &sl = d.slots[si];
    sl.busy = false;
    sl.starved = false;
    sl.hb = nullptr;
    if (d.next_p >= d.p1) return 0;
    // host side from the pool; at the cap the refill waits for a release.
    // Slots past the first two never grow the pool: they run on host batches
    // consumers have handed back (a cold query's first batches would otherwise
    // wait for one more pinned allocation each; slots_r6az.txt)
    if (d.free_batches.empty()) {
        if (d.batches.size() >= s.max_batches || si >= 2) {
            sl.starved = true;
            return 0;
        }
        d.batches.push_back(std::make_unique<HostBatch>());
        d.free_batches.push_back(d.batches.back().get());
    }
    {   // test hook: FLS_TEST_FAIL_ENQUEUE=k fails the k-th batch enqueue of the
        // process (1-based) as an allocation failure would (tests/test_scan_errors.py)
        static std::atomic<long> n_enqueue{0};
        const char *f = getenv("FLS_TEST_FAIL_ENQUEUE");
        if (f && ++n_enqueue == atol(f)) return fail(FLS_ERR_NOMEM, "injected batch enqueue failure (FLS_TEST_FAIL_ENQUEUE)");
    }
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    sl.rg0 = s.rgs[d.next_p];
    sl.nrg = 1;
    while (sl.nrg < s.batch && d.next_p + sl.nrg < d.p1 && s.rgs[d.next_p + sl.nrg] == sl.rg0 + sl.nrg) sl.nrg++;
    d.next_p += sl.nrg;
    sl.hb = d.free_batches.back();
    d.free_batches.pop_back();
    HostBatch &hb = *sl.hb;
    hb.rg0 = sl.rg0;
    hb.nrg = sl.nrg;
    hb.handed = hb.released = 0;
    hb.h_out.resize(ncols);
    sl.filling = true;
    return 1;
}
// Both parts (the scan's first batches, a refill a release unblocks).
int enqueue_batch(fls_table *t, ScanCtx &s, ScanDev &d, int si) {
    const int c = claim_batch(t, s, d, si);
    if (c <= 0) return c;
    const int rc = fill_batch(t, s, d, si);
    d.slots[si].filling = false;
    d.slots[si].busy = rc == 0;
    return rc;
}
int fill_batch(fls_table *t, ScanCtx &s, ScanDev &d, int si) {
    ProfTimer prof(PROF_FILL), pdesc(PROF_FILL_DESC);
    Slot &sl = d.slots[si];
    HostBatch &hb = *sl.hb;
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    const bool filtered = !s.terms.empty();
    HIP_TRY(hipSetDevice(d.dev));
    // 1. H2D of the batch's compressed bytes
    // (resident image: nothing when every row group of the batch is there
    // already, else the upload goes into the image and marks them present)
    uint64_t lo, hi;
    rg_byte_range(t->meta, sl.rg0, sl.rg0 + sl.nrg, lo, hi);
    sl.in_base = lo;
    DevImage *di = d.dimg.get();
    if (di && (lo < di->lo || hi > di->hi)) di = nullptr;  // outside this GPU's image: streamed
    bool have = di != nullptr;
    for (uint32_t r = sl.rg0; have && r < sl.rg0 + sl.nrg; ++r) have = di->present[r].load(std::memory_order_acquire) != 0;
    hb.upload_resident.store(di != nullptr && !have);
    if (have) {
        sl.in_dev = di->p + (lo - di->lo);
        if (getenv("FLS_DEBUG"))
            fprintf(stderr, "DEBUG: scan batch of row groups [%u, %u) decoded from the HBM-resident image\n", sl.rg0,
                    sl.rg0 + sl.nrg);
    } else {
        uint8_t *dst;
        if (di) {
            dst = di->p + (lo - di->lo);
        } else {
            HIP_TRY(sl.d_in.alloc(d.dev, hi - lo + kImagePad));
            dst = sl.d_in.p;
        }
        const uint8_t *src = t->img + lo;
        if (!t->registered) {
            HIP_TRY(sl.h_stage.alloc(hi - lo));
            ProfTimer pc(PROF_STAGE_COPY, hi - lo);
            t->res->copy.copy(sl.h_stage.p, src, hi - lo);
            src = sl.h_stage.p;
        }
        // (by the DMA engines: a copy kernel here, 57.4 GB/s alone, waits for
        // CUs behind the other slot's decode and lost the overlap: the cold
        // 16-thread query ran 135 against 156 M rows/s, cold_copy_ab_r6ap.txt)
        HIP_TRY(hipMemcpyAsync(dst, src, hi - lo, hipMemcpyHostToDevice, sl.stream));
        sl.in_dev = dst;
    }
    // dictionary-coded delivery: a delivered DICT string column no filter term
    // reads goes over PCIe as 1- or 2-byte codes when every chunk of the batch
    // is DICT (DuckDB dictionary vectors over the host string_t dictionaries)
    hb.ob.assign(ncols, 0);
    hb.dict_ptrs.assign((size_t)sl.nrg * ncols, nullptr);
    hb.dict_sizes.assign((size_t)sl.nrg * ncols, 0);
    std::vector<uint8_t> code_w(ncols, 0), in_term(ncols, 0);
    for (auto &h : s.terms) in_term[h.col] = 1;
    for (uint32_t c = 0; c < ncols; ++c) {
        hb.ob[c] = (uint8_t)out_bytes_of(t, c);
        if (!s.dict_codes || !col_selected(s.mask, c) || in_term[c] || !type_is_string(t->meta.cols[c].type)) continue;
        bool all = true;
        uint32_t maxd = 0;
        for (uint32_t r = sl.rg0; r < sl.rg0 + sl.nrg; ++r) {
            const ChunkHeader &h = t->meta.rgs[r].chunks[c].hdr;
            all = all && h.enc == ENC_DICT;
            maxd = std::max(maxd, h.dict_count);
        }
        if (!all || maxd > 65536) continue;
        code_w[c] = hb.ob[c] = maxd <= 256 ? 1 : 2;
        for (uint32_t r = 0; r < sl.nrg; ++r) {
            const size_t i = (size_t)r * ncols + c;
            hb.dict_ptrs[i] = d.h_strtab.data() + d.strtab_off[(size_t)(sl.rg0 + r - d.rg0) * ncols + c];
            hb.dict_sizes[i] = t->meta.rgs[sl.rg0 + r].chunks[c].hdr.dict_count;
        }
    }
    // the decode's bytes per row (string_t / code width / the type's width);
    // hb.ob below is what crosses PCIe
    const std::vector<uint8_t> dob = hb.ob;
    // narrowed delivery: an integer column whose row groups' zone maps bound
    // every value within 2^8 / 2^16 / 2^32 of the row group's minimum crosses
    // PCIe as value - minimum in 1 / 2 / 4 bytes (narrow_kernel after the decode)
    hb.narrowed.assign(ncols, 0);
    hb.nbase.assign((size_t)sl.nrg * ncols, 0);
    for (uint32_t c = 0; s.narrow && c < ncols; ++c) {
        const uint8_t ty = t->meta.cols[c].type;
        if (!col_selected(s.mask, c) || type_is_string(ty) || type_is_float(ty) || hb.ob[c] < 2) continue;
        bool ok = true;
        uint64_t range = 0;
        for (uint32_t r = sl.rg0; ok && r < sl.rg0 + sl.nrg; ++r) {
            const auto &zs = t->meta.rgs[r].zones;
            ok = !zs.empty() && (zs[c].flags & ZM_VALID) && !(zs[c].flags & ZM_ALL_NULL);
            if (ok) range = std::max<uint64_t>(range, zs[c].max - zs[c].min);
        }
        const uint8_t nw = range < (1ull << 8) ? 1 : range < (1ull << 16) ? 2 : range < (1ull << 32) ? 4 : 8;
        if (!ok || nw >= hb.ob[c]) continue;
        hb.ob[c] = nw;
        hb.narrowed[c] = 1;
        for (uint32_t r = 0; r < sl.nrg; ++r) hb.nbase[(size_t)r * ncols + c] = t->meta.rgs[sl.rg0 + r].zones[c].min;
    }
    // FSST columns as string lengths: the narrow kernel takes the low 1 / 2 /
    // 4 bytes of each string_t record's length word (base 0); the records are
    // rebuilt over the copied heap on the consumer's thread (scan_acquire).
    // Unfiltered scans only (a filtered batch compacts its rows, and the heap
    // offsets of the delivered strings need every row's length).
    // On by default with narrowing (FLS_SCAN_STRLEN=0: string_t records over
    // the link).  Round 3 measured it neutral while the scan was bound by host
    // work (profiles/r3/bench_e2e_strlen_r3zj.json); with the compressed image
    // resident in HBM the 16-thread read_fastlanes is bound by the D2H link,
    // and the lengths (15 fewer bytes per lineitem row) measured 7.81e8 rows/s
    // against 6.78e8 (profiles/r4/e2e_arms_strlen_r4t.txt).
    hb.strlen_w.assign(ncols, 0);
    const bool strlen_on = knob_value("FLS_SCAN_STRLEN") != 0;
    for (uint32_t c = 0; strlen_on && s.narrow && s.terms.empty() && c < ncols; ++c) {
        if (!col_selected(s.mask, c) || !type_is_string(t->meta.cols[c].type) || hb.ob[c] != 16) continue;
        bool ok = true;
        uint64_t maxlen = 0;
        for (uint32_t r = sl.rg0; ok && r < sl.rg0 + sl.nrg; ++r) {
            ok = is_fsst(t, r, c);
            const ChunkRef &ch = t->meta.rgs[r].chunks[c];
            const uint8_t *meta = t->img + ch.off + ch.hdr.meta_off;
            for (uint32_t v = 0; ok && v < ch.hdr.nvec; ++v) {
                VecMeta vm;
                memcpy(&vm, meta + 32ull * v, 32);
                ok = vm.for_base >= 0 && vm.bw <= 32;
                maxlen = std::max<uint64_t>(maxlen, (uint64_t)vm.for_base + (vm.bw >= 32 ? 0xFFFFFFFFull : (1ull << vm.bw) - 1));
            }
        }
        if (!ok) continue;
        const uint8_t nw = maxlen <= 0xFF ? 1 : maxlen <= 0xFFFF ? 2 : 4;
        hb.ob[c] = nw;
        hb.narrowed[c] = 1;
        hb.strlen_w[c] = nw;
        for (uint32_t r = 0; r < sl.nrg; ++r) hb.nbase[(size_t)r * ncols + c] = 0;
    }
    hb.narrow_out = hb.narrowed;
    hb.ob_out = hb.ob;
    for (uint32_t c = 0; c < ncols; ++c)
        if (hb.strlen_w[c]) {
            hb.narrow_out[c] = 0;
            hb.ob_out[c] = 16;
        }
    // 2. decode into the slot's device columns (FSST columns also into a heap)
    const uint64_t max_rows = (uint64_t)s.batch * t->meta.rowgroup_size;
    sl.heap_bytes.assign(ncols, 0);
    sl.d_heap.resize(ncols);
    hb.h_heap.resize(ncols);
    std::vector<uint64_t> hoff((size_t)sl.nrg * ncols, 0);
    for (uint32_t c = 0; c < ncols; ++c) {
        if (!col_selected(s.dmask, c)) continue;
        const uint64_t nb = max_rows * out_bytes_of(t, c);
        HIP_TRY(sl.d_out[c].alloc(d.dev, nb));
        // the host column at the width that crosses PCIe (narrowed values,
        // dictionary codes, string lengths): pinned memory comes at ~6 GB/s
        // whatever the thread count (pin_alloc_r6ar.txt), and a cold query
        // allocates every host batch it holds
        if (col_selected(s.mask, c)) HIP_TRY(hb.h_out[c].alloc(max_rows * hb.ob[c]));
        for (uint32_t r = 0; r < sl.nrg; ++r) {
            hoff[(size_t)r * ncols + c] = sl.heap_bytes[c];
            if (is_fsst(t, sl.rg0 + r, c)) sl.heap_bytes[c] += t->meta.rgs[sl.rg0 + r].chunks[c].hdr.reserved1;
        }
        if (sl.heap_bytes[c]) {
            HIP_TRY(sl.d_heap[c].alloc(d.dev, sl.heap_bytes[c]));
            // (+16: scan_acquire reads a string's first 16 bytes whole)
            HIP_TRY(hb.h_heap[c].alloc(sl.heap_bytes[c] + 16));
        }
    }
    hb.heap_off = hoff;
    hb.h_rec.resize(ncols);
    hb.h_rec_cap.resize(ncols, 0);
    for (uint32_t c = 0; c < ncols; ++c)
        if (hb.strlen_w[c] && hb.h_rec_cap[c] < max_rows) {
            hb.h_rec[c].reset(new (std::nothrow) uint8_t[max_rows * 16]);
            if (!hb.h_rec[c]) return fail(FLS_ERR_NOMEM, "scan: no host memory for %llu string records",
                                          (unsigned long long)max_rows);
            hb.h_rec_cap[c] = max_rows;
        }
    std::vector<DevChunk> list;
    ByteCount bc;
    ProfTimer plist(PROF_FILL_LIST);
    for (uint32_t c = 0; c < ncols; ++c) {
        if (!col_selected(s.dmask, c)) continue;
        for (uint32_t r = sl.rg0; r < sl.rg0 + sl.nrg; ++r) {
            const ChunkRef &ch = t->meta.rgs[r].chunks[c];
            const uint64_t so = d.strtab_off[(size_t)(r - d.rg0) * ncols + c];
            const uint8_t *dict = so == UINT64_MAX ? nullptr : (const uint8_t *)(d.strtab.p + so);
            uint8_t *out = sl.d_out[c].p + (t->meta.rgs[r].first_row - t->meta.rgs[sl.rg0].first_row) * dob[c];
            const uint64_t ho = hoff[(size_t)(r - sl.rg0) * ncols + c];
            list.push_back(make_devchunk(t, r, c, sl.in_dev + (ch.off - lo), dict, out, &bc,
                                         sl.heap_bytes[c] ? sl.d_heap[c].p + ho : nullptr,
                                         sl.heap_bytes[c] ? hb.h_heap[c].p + ho : nullptr, code_w[c], d.ident.p));
        }
    }
    plist.stop();
    FsstCounts fsst;
    const int64_t policy = launch_policy(decode_policy(), list, bc.geom);
    const uint32_t nmain = order_for_launch(list, &fsst, policy);
    const size_t k = list.size();
    const SplitPlan plan = append_split(list, nmain, bc.geom, policy);
    pdesc.stop();
    const size_t kk = list.size();
    HIP_TRY(sl.h_chunks.alloc(kk));
    HIP_TRY(sl.d_chunks.alloc(d.dev, kk));
    if (kk) memcpy(sl.h_chunks.p, list.data(), kk * sizeof(DevChunk));
    if (!hb.done) HIP_TRY(hipEventCreateWithFlags(&hb.done, hipEventDisableTiming));
    if (ScanProf::on())
        for (hipEvent_t &e : hb.pt)
            if (!e) HIP_TRY(hipEventCreate(&e));
    HIP_TRY(hb.h_err.alloc(1));
    if (hb.pt[0]) HIP_TRY(hipEventRecord(hb.pt[0], sl.stream));
    HIP_TRY(hipMemcpyAsync(sl.d_chunks.p, sl.h_chunks.p, kk * sizeof(DevChunk), hipMemcpyHostToDevice, sl.stream));
    HIP_TRY(sl.queue.alloc(d.dev, kQueueWords));
    // (only batches with FSST work: a stale FLS_FSST_VARIANT must not fail
    // integer-only scans, nor cost every refill an environment parse)
    if (fsst.total_vecs() > 0)
        if (const int rc = fsst_config_check(policy)) return rc;
    HIP_TRY(launch_all(sl.d_chunks.p, nmain, (uint32_t)k, fsst, d.err.p, bc.geom, sl.stream, sl.queue.p, policy,
                       plan));
    const uint64_t rows = t->meta.rgs[sl.rg0 + sl.nrg - 1].first_row + t->meta.rgs[sl.rg0 + sl.nrg - 1].nrows -
                          t->meta.rgs[sl.rg0].first_row;
    // 2b. narrowed columns: value - base into their narrow copies
    {
        std::vector<uint32_t> nc;
        for (uint32_t c = 0; c < ncols; ++c)
            if (hb.narrowed[c]) nc.push_back(c);
        if (!nc.empty()) {
            sl.d_narrow.resize(ncols);
            const size_t bytes = nc.size() * (sizeof(DevNarrow) + 8ull * sl.nrg);
            HIP_TRY(sl.h_ndesc.alloc(bytes));
            HIP_TRY(sl.d_ndesc.alloc(d.dev, bytes));
            DevNarrow *dn = (DevNarrow *)sl.h_ndesc.p;
            uint64_t *bases = (uint64_t *)(sl.h_ndesc.p + nc.size() * sizeof(DevNarrow));
            for (size_t k = 0; k < nc.size(); ++k) {
                const uint32_t c = nc[k];
                HIP_TRY(sl.d_narrow[c].alloc(d.dev, max_rows * hb.ob[c]));
                memset(&dn[k], 0, sizeof(DevNarrow));
                dn[k].src = sl.d_out[c].p;
                dn[k].dst = sl.d_narrow[c].p;
                dn[k].base = (const uint64_t *)(sl.d_ndesc.p + nc.size() * sizeof(DevNarrow)) + k * sl.nrg;
                dn[k].ob = dob[c];
                dn[k].nw = hb.ob[c];
                dn[k].sign = type_is_signed(t->meta.cols[c].type) ? 1 : 0;
                for (uint32_t r = 0; r < sl.nrg; ++r) bases[k * sl.nrg + r] = hb.nbase[(size_t)r * ncols + c];
            }
            HIP_TRY(hipMemcpyAsync(sl.d_ndesc.p, sl.h_ndesc.p, bytes, hipMemcpyHostToDevice, sl.stream));
            HIP_TRY(launch_narrow((const DevNarrow *)sl.d_ndesc.p, (uint32_t)nc.size(), (uint32_t)rows,
                                  t->meta.rowgroup_size, d.err.p, sl.stream));
        }
    }
    if (filtered) {
        // 3a. select + compact the qualifying rows straight into pinned host memory
        int rc = enqueue_filter(t, s, d, sl, rows, lo, hi - lo);
        if (rc) return rc;
    }
    // 3. D2H into pinned host columns (and string heaps)
    if (hb.pt[1]) HIP_TRY(hipEventRecord(hb.pt[1], sl.stream));
    hb.prof_d2h = 0;
    {
        // by the copy kernel (FLS_SCAN_COPY_KERNEL; fls_filter.hpp), or the
        // DMA engines for a misaligned pair and with the knob at 0
        const bool by_kernel = knob_value("FLS_SCAN_COPY_KERNEL") != 0;
        std::vector<HostCopy> copies;
        auto d2h = [&](uint8_t *dst, const uint8_t *src, uint64_t bytes) -> hipError_t {
            hb.prof_d2h += bytes;
            if (by_kernel && !(((uintptr_t)dst | (uintptr_t)src) & 15)) {
                copies.push_back({src, dst, bytes});
                return hipSuccess;
            }
            return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, sl.stream);
        };
        for (uint32_t c = 0; c < ncols; ++c) {
            if (!col_selected(s.mask, c)) continue;
            if (!filtered)
                HIP_TRY(d2h(hb.h_out[c].p, hb.narrowed[c] ? sl.d_narrow[c].p : sl.d_out[c].p, rows * hb.ob[c]));
            if (sl.heap_bytes[c]) HIP_TRY(d2h(hb.h_heap[c].p, sl.d_heap[c].p, sl.heap_bytes[c]));
        }
        HIP_TRY(launch_host_copy(copies.data(), (uint32_t)copies.size(), sl.stream));
    }
    if (hb.pt[2]) {
        HIP_TRY(hipEventRecord(hb.pt[2], sl.stream));
        hb.prof_pending.store(true);
    }
    // the error flags ride along (sticky device flags: a batch sees its own
    // kernels' and any earlier ones'), so an acquire reads pinned memory
    // instead of a synchronous 4-byte copy per row group
    HIP_TRY(hipMemcpyAsync(hb.h_err.p, d.err.p, sizeof(uint32_t), hipMemcpyDeviceToHost, sl.stream));
    HIP_TRY(hipEventRecord(hb.done, sl.stream));
    hb.col_ptrs.assign((size_t)sl.nrg * ncols, nullptr);
    hb.valid_ptrs.assign((size_t)sl.nrg * ncols, nullptr);
    hb.vbits.resize((size_t)sl.nrg * ncols);
    if (!filtered)  // every row delivered: the image's bitmaps are the validity masks
        for (uint32_t r = 0; r < sl.nrg; ++r)
            for (uint32_t c = 0; c < ncols; ++c)
                if (col_selected(s.mask, c)) hb.valid_ptrs[(size_t)r * ncols + c] = chunk_validity_host(t, sl.rg0 + r, c);
    if (!filtered)
        for (uint32_t r = 0; r < sl.nrg; ++r)
            for (uint32_t c = 0; c < ncols; ++c)
                if (col_selected(s.mask, c))
                    hb.col_ptrs[(size_t)r * ncols + c] =
                        hb.h_out[c].p + (t->meta.rgs[sl.rg0 + r].first_row - t->meta.rgs[sl.rg0].first_row) * hb.ob[c];
    return 0;  // the caller marks the slot busy (under s.mu)
}

void build_records(const fls_table *t, HostBatch &hb, uint32_t rg) {
    // FSST columns delivered as lengths: this row group's string_t records,
    // rebuilt here (the consumer's thread) over the pinned heap copy -- inline
    // bytes for strings of <= 12 bytes, else a 4-byte prefix and the pointer --
    // vector by vector from each vector's heap offset (FsstVecHeader.heap_off)
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    for (uint32_t c = 0; c < ncols && !hb.strlen_w.empty(); ++c) {
        const uint8_t nw = hb.strlen_w[c];
        if (!nw) continue;
        const uint64_t i0 = t->meta.rgs[rg].first_row - t->meta.rgs[hb.rg0].first_row;
        const uint8_t *L = hb.h_out[c].p + i0 * nw;
        uint8_t *R = hb.h_rec[c].get() + i0 * 16;
        const ChunkRef &ch = t->meta.rgs[rg].chunks[c];
        const uint8_t *meta = t->img + ch.off + ch.hdr.meta_off;
        const uint8_t *heap = hb.h_heap[c].p + hb.heap_off[(size_t)(rg - hb.rg0) * ncols + c];
        const uint32_t nrows = t->meta.rgs[rg].nrows;
        for (uint32_t v = 0; v < ch.hdr.nvec; ++v) {
            VecMeta vm;
            memcpy(&vm, meta + 32ull * v, 32);
            FsstVecHeader fh;
            memcpy(&fh, t->img + ch.off + ch.hdr.aux_off + vm.aux_off, sizeof(fh));
            const uint8_t *hp = heap + fh.heap_off;
            uint64_t pos = 0;
            const uint32_t r1 = std::min(nrows, (v + 1) * kVectorSize);
            for (uint32_t i = v * kVectorSize; i < r1; ++i) {
                const uint32_t n = nw == 1 ? L[i] : nw == 2 ? ((const uint16_t *)L)[i] : ((const uint32_t *)L)[i];
                uint64_t a, b;
                memcpy(&a, hp + pos, 8);
                memcpy(&b, hp + pos + 8, 8);
                uint32_t w[4];
                w[0] = n;
                if (n <= 12) {
                    a &= n >= 8 ? ~0ull : (1ull << (8 * n)) - 1;
                    b &= n <= 8 ? 0ull : (1ull << (8 * (n - 8))) - 1;
                    w[1] = (uint32_t)a;
                    w[2] = (uint32_t)(a >> 32);
                    w[3] = (uint32_t)b;
                } else {
                    const uint64_t p = (uint64_t)(uintptr_t)(hp + pos);
                    w[1] = (uint32_t)a;
                    w[2] = (uint32_t)p;
                    w[3] = (uint32_t)(p >> 32);
                }
                memcpy(R + 16ull * i, w, 16);
                pos += n;
            }
        }
        hb.col_ptrs[(size_t)(rg - hb.rg0) * ncols + c] = R;
    }
}

int scan_start(fls_table *t, ScanCtx &s) {
    if (s.rgs.empty()) return 0;
    for (auto &d : s.devs)
        for (int si = 0; si < s.nslots; ++si) {
            int rc = enqueue_batch(t, s, *d, si);
            if (rc) return rc;
        }
    return 0;
}

// the device and host batch holding row group rg (a batch already released by
// its slot, or one a slot holds), or false if its batch is not enqueued
bool find_batch(ScanCtx &s, uint32_t rg, int &g, HostBatch *&hb) {
    for (auto &[dg, b] : s.ready)
        if (rg >= b->rg0 && rg < b->rg0 + b->nrg) {
            g = dg;
            hb = b;
            return true;
        }
    for (size_t i = 0; i < s.devs.size(); ++i)
        for (int j = 0; j < s.nslots; ++j) {
            const Slot &sl = s.devs[i]->slots[j];
            if (sl.busy && rg >= sl.rg0 && rg < sl.rg0 + sl.nrg) {
                g = (int)i;
                hb = sl.hb;
                return true;
            }
        }
    return false;
}

// filtered batch: selected-row offsets of its row groups from the per-vector
// counts (every row group of a batch but the table's last is whole vectors)
void batch_selection(fls_table *t, ScanCtx &s, HostBatch &hb) {
    std::lock_guard<std::mutex> lk(s.mu);
    if (hb.sel_ready) return;
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    hb.sel_off.assign(hb.nrg + 1, 0);
    uint32_t v = 0, acc = 0;
    for (uint32_t r = 0; r < hb.nrg; ++r) {
        hb.sel_off[r] = acc;
        const uint32_t nv = (t->meta.rgs[hb.rg0 + r].nrows + 1023) / 1024;
        for (uint32_t k = 0; k < nv && v < hb.nvec; ++k) acc += hb.h_counts.p[v++];
    }
    hb.sel_off[hb.nrg] = acc;
    for (uint32_t r = 0; r < hb.nrg; ++r)
        for (uint32_t c = 0; c < ncols; ++c)
            if (col_selected(s.mask, c))
                hb.col_ptrs[(size_t)r * ncols + c] = hb.h_out[c].p + (uint64_t)hb.sel_off[r] * hb.ob[c];
    hb.sel_ready = true;
}

// sticky scan error (call with s.mu held): every waiting and later acquire
// returns it instead of waiting for a batch that will never arrive
void set_scan_error(ScanCtx &s, int rc) {
    if (rc && !s.err_rc) {
        s.err_rc = rc;
        s.err_msg = fls_last_error();
    }
}

// Claim the next row group in order and wait until its batch is decoded and
// copied back.  Its buffers stay valid until scan_release(rg).  The first
// acquire that sees a batch's D2H complete refills the batch's slot (the
// device side is idle from then on; the batch's host side, its events and
// error flags are the HostBatch's), and the batch's other row groups are found
// on s.ready: the next batch's fill, decode and D2H overlap the hand-out of
// this one's, and no consumer waits on another one's release.
int scan_acquire(fls_table *t, ScanCtx &s, fls_rowgroup *out) {
    if (!s.active) return fail(FLS_ERR_STATE, "scan not started");
    int g = -1;
    uint32_t rg;
    HostBatch *hb = nullptr;
    {
        std::unique_lock<std::mutex> lk(s.mu);
        if (s.err_rc) return fail(s.err_rc, "%s", s.err_msg.c_str());
        if (s.cur >= s.rgs.size()) return 0;
        rg = s.rgs[s.cur++];
        // the batch holding rg is enqueued once its slot's previous batch has
        // completed (or, at the host-batch cap, once a batch is released)
        s.cv.wait(lk, [&] { return find_batch(s, rg, g, hb) || !s.active || s.err_rc != 0; });
        if (g < 0) {
            if (!s.active) return fail(FLS_ERR_STATE, "scan ended while waiting for row group %u", rg);
            return fail(s.err_rc, "%s", s.err_msg.c_str());
        }
    }
    ScanDev &d = *s.devs[g];
    auto wait_batch = [&]() -> int {
        HIP_TRY(hipSetDevice(d.dev));
        ProfTimer pw(PROF_WAIT);
        if (s.spin_wait) {  // poll the event (A/B knob FLS_SCAN_SPIN_WAIT: the blocking wait's wake-up latency)
            hipError_t q;
            while ((q = hipEventQuery(hb->done)) == hipErrorNotReady) std::this_thread::yield();
            HIP_TRY(q);
        } else {
            HIP_TRY(hipEventSynchronize(hb->done));
        }
        if (hb->prof_pending.exchange(false)) {  // the batch's stream times, once
            float dec = 0, d2h = 0;
            if (hipEventElapsedTime(&dec, hb->pt[0], hb->pt[1]) == hipSuccess &&
                hipEventElapsedTime(&d2h, hb->pt[1], hb->pt[2]) == hipSuccess) {
                ScanProf &p = scan_prof();
                p.ns[PROF_GPU_DECODE] += (uint64_t)(dec * 1e6);
                p.calls[PROF_GPU_DECODE] += 1;
                p.ns[PROF_D2H] += (uint64_t)(d2h * 1e6);
                p.bytes[PROF_D2H] += hb->prof_d2h;
                p.calls[PROF_D2H] += 1;
            }
        }
        const uint32_t err = *(volatile const uint32_t *)hb->h_err.p;
        if (err & KERR_FILTER_STR) return fail(FLS_ERR_FORMAT, "filter: string outside its batch heap (flags 0x%x)", err);
        if (err & KERR_NARROW)
            return fail(FLS_ERR_FORMAT, "corrupt chunk: a value outside its zone map in a narrowed column (flags 0x%x)", err);
        if (err & KERR_LDS_BASE) return fail(FLS_ERR_DEVICE, "FSST kernel: dynamic LDS not at address 0 (flags 0x%x)", err);
        if (err) return fail(FLS_ERR_FORMAT, "corrupt chunk detected while decoding (flags 0x%x)", err);
        return 0;
    };
    if (int rc = wait_batch()) {
        std::lock_guard<std::mutex> lk(s.mu);
        set_scan_error(s, rc);
        s.cv.notify_all();
        return rc;
    }
    ProfTimer seen(PROF_REFILL_LAT);  // this acquire saw the batch complete: until its refill starts
    // the batch's upload into the resident image is complete (its event covers
    // the H2D): later scans of this file may decode these row groups from it
    if (hb->upload_resident.exchange(false) && d.dimg)
        for (uint32_t r = hb->rg0; r < hb->rg0 + hb->nrg; ++r) d.dimg->present[r].store(1, std::memory_order_release);
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    out->rowgroup = rg;
    out->nrows = t->meta.rgs[rg].nrows;
    out->first_row = t->meta.row_offset + t->meta.rgs[rg].first_row;
    out->ncols = ncols;
    out->nrows_scanned = out->nrows;
    out->sel = nullptr;
    if (!s.terms.empty()) {
        batch_selection(t, s, *hb);
        const uint32_t i = rg - hb->rg0;
        out->nrows = hb->sel_off[i + 1] - hb->sel_off[i];
        out->sel = hb->h_sel.p + hb->sel_off[i];
    }
    out->columns = hb->col_ptrs.data() + (size_t)(rg - hb->rg0) * ncols;
    out->validity = hb->valid_ptrs.data() + (size_t)(rg - hb->rg0) * ncols;
    out->dict = hb->dict_ptrs.data() + (size_t)(rg - hb->rg0) * ncols;
    out->dict_size = hb->dict_sizes.data() + (size_t)(rg - hb->rg0) * ncols;
    out->dict_width = hb->ob_out.data();
    out->narrow = hb->narrow_out.data();
    out->narrow_base = hb->nbase.data() + (size_t)(rg - hb->rg0) * ncols;
    if (!s.defer_records) build_records(t, *hb, rg);
    if (out->sel) {  // filtered: the delivered rows' validity, gathered through sel
        const size_t i0 = (size_t)(rg - hb->rg0) * ncols;
        for (uint32_t c = 0; c < ncols; ++c) {
            const uint64_t *img = col_selected(s.mask, c) ? chunk_validity_host(t, rg, c) : nullptr;
            hb->valid_ptrs[i0 + c] = nullptr;
            if (!img) continue;
            std::vector<uint64_t> &w = hb->vbits[i0 + c];
            w.assign(std::max<size_t>(1, (out->nrows + 63) / 64), 0);
            bool any_null = false;
            for (uint32_t i = 0; i < out->nrows; ++i) {
                const uint32_t r = out->sel[i];
                const uint64_t b = (img[r >> 6] >> (r & 63)) & 1;
                w[i >> 6] |= b << (i & 63);
                any_null |= !b;
            }
            if (any_null) hb->valid_ptrs[i0 + c] = w.data();
        }
    }
    bool refill = false;
    int si = -1;
    std::shared_ptr<DevImage> done_img;  // dropped outside s.mu
    {
        std::lock_guard<std::mutex> lk(s.mu);
        s.out.emplace_back(rg, hb);
        const bool last = ++hb->handed == hb->nrg;
        // the batch's D2H is complete: if its slot still holds it, the slot
        // takes its next batch now (FLS_SCAN_EARLY_REFILL=0: once the batch's
        // last row group is handed out) and the batch moves to s.ready
        if (last || s.early_refill)
            for (int k = 0; k < s.nslots && si < 0; ++k)
                if (d.slots[k].busy && d.slots[k].hb == hb) si = k;
        if (si >= 0) {
            s.ready.emplace_back(g, hb);
            // a failed refill does not take this row group back: it is delivered,
            // and the error surfaces at the next acquire
            const int c = claim_batch(t, s, d, si);
            set_scan_error(s, c < 0 ? c : 0);
            refill = c == 1;
            // this GPU's last batch is decoded: the scan no longer holds its
            // resident image, which becomes evictable (the table may stay open)
            if (c == 0 && d.next_p >= d.p1 && d.dimg) {
                bool idle = true;
                for (int k = 0; k < s.nslots; ++k) idle = idle && !d.slots[k].busy && !d.slots[k].filling;
                if (idle) done_img = std::move(d.dimg);
            }
        }
        if (last)  // every row group of the batch handed out
            for (size_t i = 0; i < s.ready.size(); ++i)
                if (s.ready[i].second == hb) {
                    s.ready.erase(s.ready.begin() + (long)i);
                    break;
                }
        s.cv.notify_all();
    }
    if (!refill) seen.cancel();
    seen.stop();
    if (refill) {  // the slot's next batch, outside s.mu (claim_batch)
        Slot &sl = d.slots[si];
        const int rc = fill_batch(t, s, d, si);
        std::lock_guard<std::mutex> lk(s.mu);
        sl.filling = false;
        sl.busy = rc == 0;
        set_scan_error(s, rc);
        s.cv.notify_all();
    }
    return 1;
}

int scan_release(fls_table *t, ScanCtx &s, uint32_t rg) {
    std::lock_guard<std::mutex> lk(s.mu);
    auto it = std::find_if(s.out.begin(), s.out.end(), [&](const auto &o) { return o.first == rg; });
    if (!s.active || it == s.out.end()) return fail(FLS_ERR_ARG, "row group %u is not held by this scan", rg);
    HostBatch *hb = it->second;
    s.out.erase(it);
    if (++hb->released < hb->nrg) return 0;
    // every row group of the batch is back: its host side returns to the pool,
    // and a slot whose refill waited for one goes now
    int rc = 0;
    for (auto &dp : s.devs) {
        ScanDev &d = *dp;
        bool mine = false;
        for (auto &b : d.batches) mine = mine || b.get() == hb;
        if (!mine) continue;
        d.free_batches.push_back(hb);
        for (int si = 0; si < s.nslots && !rc; ++si)
            if (d.slots[si].starved) {
                rc = enqueue_batch(t, s, d, si);
                set_scan_error(s, rc);
            }
        break;
    }
    s.cv.notify_all();
    return rc;
}

// single-consumer form: releases the previously delivered row group
int scan_next(fls_table *t, ScanCtx &s, fls_rowgroup *out) {
    if (s.held >= 0) {
        const uint32_t prev = (uint32_t)s.held;
        s.held = -1;
        int rc = scan_release(t, s, prev);
        if (rc) return rc;
    }
    int rc = scan_acquire(t, s, out);
    if (rc == 1) s.held = out->rowgroup;
    return rc;
}

// fls_predicate[] -> host terms in the comparison domain, sorted by clause
int to_terms(const fls_table *t, const fls_predicate *p, uint32_t n, std::vector<HostTerm> &out) {
    out.clear();
    if (n && !p) return fail(FLS_ERR_ARG, "fls_scan_filter: NULL predicates");
    for (uint32_t i = 0; i < n; ++i) {
        if (p[i].col >= t->meta.cols.size()) return fail(FLS_ERR_ARG, "filter column %u out of range", p[i].col);
        if (p[i].op > FLS_CMP_FALSE) return fail(FLS_ERR_ARG, "filter operator %u unknown", p[i].op);
        HostTerm h;
        h.col = p[i].col;
        h.clause = p[i].clause;
        h.op = p[i].op;
        const uint8_t ty = t->meta.cols[h.col].type;
        if (type_is_string(ty)) {
            h.kind = FK_STR;
            if (p[i].str_len && !p[i].str) return fail(FLS_ERR_ARG, "filter on column %u: NULL string", h.col);
            if (p[i].str_len > 0xFFFFFFFFull) return fail(FLS_ERR_ARG, "filter string too long");
            if (p[i].str_len) h.str.assign(p[i].str, p[i].str_len);
        } else if (type_is_float(ty)) {
            h.kind = FK_FLOAT;
            double d;
            if (ty == TY_FLOAT) {
                float f;
                const uint32_t b = (uint32_t)p[i].value;
                memcpy(&f, &b, 4);
                d = f;
            } else {
                memcpy(&d, &p[i].value, 8);
            }
            memcpy(&h.value, &d, 8);
        } else {
            h.kind = type_is_signed(ty) ? FK_INT : FK_UINT;
            h.value = p[i].value;
        }
        out.push_back(std::move(h));
    }
    std::stable_sort(out.begin(), out.end(), [](const HostTerm &a, const HostTerm &b) { return a.clause < b.clause; });
    return 0;
}

int open_common(fls_connection *conn, fls_table *t, fls_table **out) {
    std::string why = parse_file(t->img, t->len, t->meta);
    if (!why.empty()) {
        delete t;
        return fail(FLS_ERR_FORMAT, "not a valid FastLanes file: %s", why.c_str());
    }
    t->devices = conn->devices;
    t->res = conn->res;
    for (auto &c : t->meta.cols) t->names.push_back(c.name);
    *out = t;
    if (debug_enabled())
        fprintf(stderr, "DEBUG: FLS file opened: %zu columns, %llu rows, %zu row groups\n", t->meta.cols.size(),
                (unsigned long long)t->meta.nrows, t->meta.rgs.size());
    return 0;
}

}  // namespace

// ------------------------------------------------------------------------------
// C-ABI

extern "C" {

const char *fls_last_error(void) { return last_error().c_str(); }

const char *fls_version(void) { return "fastlanes-mi355x 0.1.0 (gfx950)"; }

int fls_config_default(const char *name, int64_t *value) {
    const Knob *k = find_knob(name);
    if (!k || !value) return fail(FLS_ERR_ARG, "fls_config_default: '%s' is not a knob", name ? name : "(null)");
    *value = k->def;
    return 0;
}

int fls_config_value(const char *name, int64_t *value) {
    if (!find_knob(name) || !value) return fail(FLS_ERR_ARG, "fls_config_value: '%s' is not a knob", name ? name : "(null)");
    *value = knob_value(name);
    return 0;
}

int fls_config_count(void) { return (int)(sizeof(kKnobs) / sizeof(kKnobs[0])); }

const char *fls_config_name(int i) {
    return i >= 0 && i < fls_config_count() ? kKnobs[i].name : nullptr;
}

int fls_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int fls_device_alloc(int device, uint64_t bytes, void **ptr) {
    if (!ptr) return fail(FLS_ERR_ARG, "fls_device_alloc: NULL out");
    *ptr = nullptr;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipMalloc(ptr, std::max<uint64_t>(bytes, 1)));
    return 0;
}

int fls_device_free(int device, void *ptr) {
    if (!ptr) return 0;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipFree(ptr));
    return 0;
}

int fls_device_memcpy(int device, void *dst, const void *src, uint64_t bytes, int kind) {
    if (!dst || !src) return fail(FLS_ERR_ARG, "fls_device_memcpy: NULL pointer");
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                           : hipMemcpyDeviceToDevice;
    if (kind < 0 || kind > 2) return fail(FLS_ERR_ARG, "fls_device_memcpy: kind %d", kind);
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipMemcpy(dst, src, bytes, k));
    return 0;
}

int fls_connect(const int *devices, int ndevices, fls_connection **out) {
    if (!out) return fail(FLS_ERR_ARG, "fls_connect: NULL out");
    auto *c = new fls_connection();
    if (devices && ndevices > 0) c->devices.assign(devices, devices + ndevices);
    else c->devices.push_back(0);
    *out = c;
    return 0;
}

void fls_disconnect(fls_connection *conn) { delete conn; }

int fls_release_device_memory(int device, uint64_t *freed_bytes) {
    const uint64_t b = release_idle_images(device < 0 ? -1 : device);
    if (freed_bytes) *freed_bytes = b;
    return 0;
}

int fls_resident_info(int device, uint64_t *bytes, uint32_t *images) {
    ImageRegistry &R = image_registry();
    std::lock_guard<std::mutex> lk(R.mu);
    const int dv = device < 0 ? -1 : device;
    if (bytes) *bytes = R.set.used(dv);
    if (images) *images = (uint32_t)R.set.count(dv);
    return 0;
}

int fls_connection_trim(fls_connection *conn, uint64_t keep_bytes, uint64_t *idle_bytes) {
    if (!conn) return fail(FLS_ERR_ARG, "fls_connection_trim: NULL connection");
    {
        std::lock_guard<std::mutex> lk(conn->res->mu);
        conn->res->trim_locked(-1, (size_t)keep_bytes);
    }
    if (idle_bytes) *idle_bytes = conn->res->idle_pinned();
    return 0;
}

}  // extern "C"

namespace {
// The validated-file cache (MappedFile): the FLS_OPEN_CACHE most recently
// opened files (default 16, 0 = off) stay mapped with their metadata.  The
// key changes whenever the file is replaced or rewritten through the file
// system (inode, size, mtime in ns).
struct FileKey {
    uint64_t dev, ino, size;
    int64_t mtime_s, mtime_ns;
    bool operator==(const FileKey &o) const {
        return dev == o.dev && ino == o.ino && size == o.size && mtime_s == o.mtime_s && mtime_ns == o.mtime_ns;
    }
};
struct FileCache {
    std::mutex mu;
    std::vector<std::pair<FileKey, std::shared_ptr<MappedFile>>> lru;  // most recent last
    static size_t capacity() {
        static const size_t cap = (size_t)std::max<int64_t>(0, knob_value("FLS_OPEN_CACHE"));
        return cap;
    }
    std::shared_ptr<MappedFile> find(const FileKey &k) {
        std::lock_guard<std::mutex> lk(mu);
        for (size_t i = 0; i < lru.size(); ++i)
            if (lru[i].first == k) {
                auto hit = lru[i];
                lru.erase(lru.begin() + (long)i);
                lru.push_back(hit);
                return hit.second;
            }
        return nullptr;
    }
    void put(const FileKey &k, std::shared_ptr<MappedFile> m) {
        if (capacity() == 0) return;
        std::lock_guard<std::mutex> lk(mu);
        lru.emplace_back(k, std::move(m));
        while (lru.size() > capacity()) lru.erase(lru.begin());
    }
};
FileCache &file_cache() {
    static FileCache *c = new FileCache();  // process lifetime (tables may outlive static destruction order)
    return *c;
}
}  // namespace

extern "C" {

int fls_read_fls(fls_connection *conn, const char *path, fls_table **out) {
    if (!conn || !path || !out) return fail(FLS_ERR_ARG, "fls_read_fls: NULL argument");
    // map the file: opening reads only the footer and the chunk headers it
    // validates (DuckDB opens a file at bind and at init), the scan streams
    // the row groups it keeps
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return fail(FLS_ERR_IO, "Failed to open FastLanes file: %s", path);
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
        close(fd);
        return fail(FLS_ERR_IO, "Failed to open FastLanes file: %s", path);
    }
    const FileKey key{(uint64_t)st.st_dev, (uint64_t)st.st_ino, (uint64_t)st.st_size, (int64_t)st.st_mtim.tv_sec,
                      (int64_t)st.st_mtim.tv_nsec};
    if (FileCache::capacity() > 0 && st.st_size > 0) {
        if (std::shared_ptr<MappedFile> hit = file_cache().find(key)) {  // unchanged file: already validated
            close(fd);
            auto *t = new fls_table();
            t->mapped = hit;
            t->img = (const uint8_t *)hit->map;
            t->len = hit->len;
            t->meta = hit->meta;
            t->devices = conn->devices;
            t->res = conn->res;
            for (auto &c : t->meta.cols) t->names.push_back(c.name);
            *out = t;
            return 0;
        }
    }
    auto *t = new fls_table();
    const size_t n = (size_t)st.st_size;
    if (n > 0) {
        void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {  // e.g. a pipe-backed or special file system: read it
            t->owned.resize(n);
            size_t got = 0;
            while (got < n) {
                const ssize_t r = pread(fd, t->owned.data() + got, n - got, (off_t)got);
                if (r <= 0) break;
                got += (size_t)r;
            }
            if (got != n) { close(fd); delete t; return fail(FLS_ERR_IO, "short read of %s", path); }
            t->img = t->owned.data();
        } else {
            t->map = m;
            t->map_len = n;
            t->img = (const uint8_t *)m;
        }
    }
    close(fd);
    t->len = (uint64_t)n;
    const int rc = open_common(conn, t, out);
    if (rc == 0 && t->map && FileCache::capacity() > 0) {  // share the mapping and the validated metadata
        auto mf = std::make_shared<MappedFile>();
        mf->map = t->map;
        mf->len = t->map_len;
        mf->meta = t->meta;
        t->map = nullptr;  // owned by mf now
        t->mapped = mf;
        file_cache().put(key, std::move(mf));
    }
    return rc;
}

int fls_read_fls_image(fls_connection *conn, const void *img, uint64_t len, int copy, fls_table **out) {
    if (!conn || !img || !out) return fail(FLS_ERR_ARG, "fls_read_fls_image: NULL argument");
    auto *t = new fls_table();
    if (copy) {
        t->owned.assign((const uint8_t *)img, (const uint8_t *)img + len);
        t->img = t->owned.data();
    } else {
        t->img = (const uint8_t *)img;
    }
    t->len = len;
    return open_common(conn, t, out);
}

void fls_table_close(fls_table *t) { delete t; }

uint32_t fls_table_ncols(const fls_table *t) { return t ? (uint32_t)t->meta.cols.size() : 0; }
uint64_t fls_table_nrows(const fls_table *t) { return t ? t->meta.nrows : 0; }
uint64_t fls_table_row_offset(const fls_table *t) { return t ? t->meta.row_offset : 0; }
uint32_t fls_table_nrowgroups(const fls_table *t) { return t ? (uint32_t)t->meta.rgs.size() : 0; }
int64_t fls_table_rowgroup_rows(const fls_table *t, uint32_t rg) {
    if (!t || rg >= t->meta.rgs.size()) return fail(FLS_ERR_ARG, "row group %u out of range", rg);
    return t->meta.rgs[rg].nrows;
}

int fls_table_column(const fls_table *t, uint32_t col, fls_column_info *out) {
    if (!t || !out || col >= t->meta.cols.size()) return fail(FLS_ERR_ARG, "column %u out of range", col);
    const ColumnMeta &c = t->meta.cols[col];
    out->name = t->names[col].c_str();
    out->type = c.type;
    out->width = c.width;
    out->scale = c.scale;
    out->out_bytes = (uint8_t)type_out_bytes(c.type);
    return 0;
}

int fls_materialize(fls_table *t, uint32_t rg, const uint8_t *col_mask, fls_rowgroup *out) {
    if (!t || !out) return fail(FLS_ERR_ARG, "fls_materialize: NULL argument");
    if (rg >= t->meta.rgs.size()) return fail(FLS_ERR_ARG, "row group %u out of range", rg);
    // a one-row-group scan on the GPU that owns rg in a full-table sharding
    const uint32_t G = (uint32_t)t->devices.size(), N = (uint32_t)t->meta.rgs.size();
    uint32_t g = 0;
    while (g + 1 < G && rg >= (uint64_t)N * (g + 1) / G) ++g;
    int rc = scan_setup(t, t->mat, {t->devices[g]}, col_mask, rg, rg + 1, nullptr);
    if (!rc) rc = scan_start(t, t->mat);
    if (rc) return rc;
    rc = scan_next(t, t->mat, out);
    return rc == 1 ? 0 : (rc == 0 ? fail(FLS_ERR_STATE, "internal: empty materialize") : rc);
}

int fls_scan_begin(fls_table *t, const uint8_t *col_mask, uint32_t rg_begin, uint32_t rg_end) {
    if (!t) return fail(FLS_ERR_ARG, "fls_scan_begin: NULL table");
    int rc = scan_setup(t, t->scan, t->devices, col_mask, rg_begin, rg_end, &t->filter);
    if (rc) return rc;
    return scan_start(t, t->scan);
}

int fls_scan_filter(fls_table *t, const fls_predicate *preds, uint32_t n) {
    if (!t) return fail(FLS_ERR_ARG, "fls_scan_filter: NULL table");
    std::vector<HostTerm> terms;
    int rc = to_terms(t, preds, n, terms);
    if (rc) return rc;
    t->filter.swap(terms);
    return 0;
}

int fls_scan_pruned(const fls_table *t) {
    if (!t) return fail(FLS_ERR_ARG, "fls_scan_pruned: NULL table");
    return (int)t->scan.pruned;
}

int fls_table_zonemap(const fls_table *t, uint32_t rg, uint32_t col, uint64_t *min, uint64_t *max, uint32_t *flags) {
    if (!t || rg >= t->meta.rgs.size() || col >= t->meta.cols.size())
        return fail(FLS_ERR_ARG, "zone map (%u, %u) out of range", rg, col);
    const auto &z = t->meta.rgs[rg].zones;
    if (z.empty() || !(z[col].flags & (ZM_VALID | ZM_HAS_NULL | ZM_ALL_NULL))) return 0;
    if (min) *min = z[col].min;
    if (max) *max = z[col].max;
    if (flags) *flags = z[col].flags;
    return 1;
}

int fls_scan_narrow(fls_table *t, int enable) {
    if (!t) return fail(FLS_ERR_ARG, "fls_scan_narrow: NULL table");
    t->narrow = enable != 0;
    return 0;
}

int fls_scan_defer_records(fls_table *t, int enable) {
    if (!t) return fail(FLS_ERR_ARG, "fls_scan_defer_records: NULL table");
    t->defer_records = enable != 0;
    return 0;
}

int fls_scan_build_records(fls_table *t, const fls_rowgroup *rg) {
    if (!t || !rg) return fail(FLS_ERR_ARG, "fls_scan_build_records: NULL argument");
    HostBatch *hb = nullptr;
    {
        std::lock_guard<std::mutex> lk(t->scan.mu);
        for (const auto &o : t->scan.out)
            if (o.first == rg->rowgroup) hb = o.second;
    }
    if (!hb) return fail(FLS_ERR_ARG, "fls_scan_build_records: row group %u is not held by this scan", rg->rowgroup);
    if (t->scan.defer_records) build_records(t, *hb, rg->rowgroup);
    return 0;
}

int fls_scan_dict_codes(fls_table *t, int enable) {
    if (!t) return fail(FLS_ERR_ARG, "fls_scan_dict_codes: NULL table");
    t->dict_codes = enable != 0;
    return 0;
}

int fls_table_validity(const fls_table *t, uint32_t rg, uint32_t col, const uint64_t **words) {
    if (!t || rg >= t->meta.rgs.size() || col >= t->meta.cols.size())
        return fail(FLS_ERR_ARG, "validity (%u, %u) out of range", rg, col);
    const uint64_t *w = chunk_validity_host(t, rg, col);
    if (words) *words = w;
    return w ? 1 : 0;
}

int fls_rowgroup_may_match(const fls_table *t, uint32_t rg, const fls_predicate *preds, uint32_t n) {
    if (!t || rg >= t->meta.rgs.size()) return fail(FLS_ERR_ARG, "row group %u out of range", rg);
    std::vector<HostTerm> terms;
    int rc = to_terms(t, preds, n, terms);
    if (rc) return rc;
    return rowgroup_may_match(t, rg, terms) ? 1 : 0;
}

int fls_scan_next(fls_table *t, fls_rowgroup *out) {
    if (!t || !out) return fail(FLS_ERR_ARG, "fls_scan_next: NULL argument");
    return scan_next(t, t->scan, out);
}

int fls_scan_acquire(fls_table *t, fls_rowgroup *out) {
    if (!t || !out) return fail(FLS_ERR_ARG, "fls_scan_acquire: NULL argument");
    return scan_acquire(t, t->scan, out);
}

int fls_scan_release(fls_table *t, uint32_t rowgroup) {
    if (!t) return fail(FLS_ERR_ARG, "fls_scan_release: NULL table");
    return scan_release(t, t->scan, rowgroup);
}

// ---- device-resident mode -------------------------------------------------

}  // extern "C"

namespace {

// ---- HBM placement of the resident output columns --------------
// The decode's write stream runs at a speed set by where the driver placed
// the output buffers (the same decode at the same virtual addresses: 2.63-3.13
// ms on lineitem_full SF12.5 from one allocation to the next,
// profiles/r6/placement_*.txt).  A candidate set of output columns is rated by
// probe_placement: the decode's chunk-order write stream against a linear fill
// of the same buffers (the fill runs at the same speed on every placement, so
// the ratio q rates the placement on this box).  Up to FLS_PLACEMENT_TRIES
// sets (default 8) are tried, the best kept, the search ending early once
// q >= FLS_PLACEMENT_GOOD / 1000 (default 990: at 0.93-0.97 some placements
// still decoded slowly, profiles/r6/placement_q_sf25_r6q.txt).
int placement_tries() { return (int)std::max<int64_t>(1, knob_value("FLS_PLACEMENT_TRIES")); }

struct PlacementRating {
    float chunk_ms = 0, fill_ms = 0;
    double q = 0;
};

int rate_outputs(const fls_table *t, const Resident &r, const std::vector<DevBuf<uint8_t>> &outs,
                 PlacementRating &pr) {
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    std::vector<ProbeRegion> reg;
    for (uint32_t c = 0; c < ncols; ++c)
        for (uint32_t g = r.rg0; g < r.rg1; ++g) {
            const uint64_t ob = out_bytes_of(t, c);
            const uint64_t bytes = (t->meta.rgs[g].nrows * ob) & ~1023ull;
            if (bytes) reg.push_back({outs[c].p + (t->meta.rgs[g].first_row - r.first_row) * ob, bytes});
        }
    // the decode's queue order: largest output first
    std::stable_sort(reg.begin(), reg.end(), [](const ProbeRegion &a, const ProbeRegion &b) { return a.bytes > b.bytes; });
    DevBuf<ProbeRegion> d;
    HIP_TRY(d.alloc(r.dev, reg.size()));
    HIP_TRY(hipMemcpy(d.p, reg.data(), reg.size() * sizeof(ProbeRegion), hipMemcpyHostToDevice));
    std::vector<uint8_t *> bufs(ncols);
    std::vector<uint64_t> sizes(ncols);
    for (uint32_t c = 0; c < ncols; ++c) {
        bufs[c] = outs[c].p;
        sizes[c] = (r.rows * out_bytes_of(t, c)) & ~4095ull;
    }
    HIP_TRY(probe_placement(d.p, (uint32_t)reg.size(), bufs.data(), sizes.data(), ncols, 2, r.stream, &pr.chunk_ms,
                            &pr.fill_ms));
    pr.q = pr.chunk_ms > 0 ? pr.fill_ms / pr.chunk_ms : 0;
    return 0;
}

int decode_part(fls_table *t, Resident &r, const std::vector<uint8_t> &mask);

// A candidate set rated by one real decode launch of every column (the
// launch after a warm-up one, HIP events): at SF100 the write probe rated every
// set >= 0.99 while the main columns still decoded up to 5 % slower on some
// sets (profiles/r6/placement_sels_sf100_r6w.txt), and four sets rated by
// their decode differed by 3-4 % within one upload, the kept one decoding
// within 0.3 % of its rating afterwards (placement_dec_sf100_r6x.txt).  The
// launch's errors are not the upload's: a failure (ms < 0) falls back to the
// write probe.
float decode_rating(fls_table *t, Resident &r) {
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    const std::vector<uint8_t> mask(ncols, 1);
    r.h_chunks.clear();  // descriptors point at the current outputs
    const uint32_t ev0 = r.ev_used;
    struct RatingScope {
        RatingScope() { rating_launch() = true; }
        ~RatingScope() { rating_launch() = false; }
    } scope;
    // two warm-up launches (a fresh set decodes ~4 % slower at first), then
    // the fastest of three
    constexpr int kWarm = 2, kTimed = 3;
    bool ok = true;
    for (int i = 0; i < kWarm + kTimed && ok; ++i) ok = decode_part(t, r, mask) == 0;
    ok = ok && hipStreamSynchronize(r.stream) == hipSuccess;
    float ms = -1;
    for (int i = kWarm; i < kWarm + kTimed && ok; ++i) {
        float x = 0;
        ok = hipEventElapsedTime(&x, r.ev_pool[ev0 + 2 * i], r.ev_pool[ev0 + 2 * i + 1]) == hipSuccess;
        if (ok && (ms < 0 || x < ms)) ms = x;
    }
    uint32_t e = 0;
    ok = ok && hipMemcpy(&e, r.err.p, sizeof(e), hipMemcpyDeviceToHost) == hipSuccess && e == 0;
    (void)hipGetLastError();
    (void)hipMemset(r.err.p, 0, sizeof(uint32_t));
    r.ev_used = ev0;
    r.h_chunks.clear();
    return ok ? ms : -1.0f;
}

// A candidate placement: a new set of output columns, new FSST heaps
// (FLS_PLACEMENT_HEAPS, default 1) and a new copy of the compressed image
// (FLS_PLACEMENT_IMAGE, default 1): with all three re-drawn the decode-rated
// SF100 step ran 20.65-20.75 ms against 20.91-21.05 for outputs alone, four
// interleaved bench runs each (profiles/r6/ab_placement_candidates_r6af.txt).
// swap_into exchanges it with the part's current buffers.
struct Candidate {
    std::vector<DevBuf<uint8_t>> out, heap;
    DevBuf<uint8_t> img;
    void clear() {
        out.clear();
        heap.clear();
        img.release();
    }
    void swap_into(Resident &r) {
        std::swap(r.d_out, out);
        if (!heap.empty()) std::swap(r.d_heap, heap);
        if (img.p) {
            std::swap(r.img.p, img.p);
            std::swap(r.img.n, img.n);
            std::swap(r.img.dev, img.dev);
        }
    }
};
bool placement_flag(const char *name) { return knob_value(name) != 0; }

// a new candidate (plain hipMalloc: a speculative set must not evict cached
// images), or false when it does not fit
bool alloc_candidate(const fls_table *t, const Resident &r, uint64_t set_bytes, Candidate &cand) {
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    const bool heaps = placement_flag("FLS_PLACEMENT_HEAPS"), image = placement_flag("FLS_PLACEMENT_IMAGE");
    uint64_t extra = image ? r.img.n : 0;
    for (uint32_t c = 0; heaps && c < ncols; ++c) extra += r.d_heap[c].p ? r.d_heap[c].n : 0;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < set_bytes + extra + (set_bytes + extra) / 8 + (1ull << 30)) {
        (void)hipGetLastError();
        return false;  // no room for a second set
    }
    cand.clear();
    auto make = [&](DevBuf<uint8_t> &b, size_t n) {
        if (hipMalloc((void **)&b.p, std::max<size_t>(1, n)) != hipSuccess) {
            (void)hipGetLastError();
            b.p = nullptr;
            return false;
        }
        b.n = n;
        b.dev = r.dev;
        return true;
    };
    cand.out.resize(ncols);
    bool ok = true;
    for (uint32_t c = 0; c < ncols && ok; ++c) ok = make(cand.out[c], r.rows * out_bytes_of(t, c));
    if (ok && heaps) {
        cand.heap.resize(ncols);
        for (uint32_t c = 0; c < ncols && ok; ++c)
            if (r.d_heap[c].p) ok = make(cand.heap[c], r.d_heap[c].n);
    }
    if (ok && image) ok = make(cand.img, r.img.n) && hipMemcpy(cand.img.p, r.img.p, r.img.n, hipMemcpyDeviceToDevice) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        cand.clear();  // frees the ones made
    }
    return ok;
}

int choose_placement(fls_table *t, Resident &r) {
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    uint64_t set_bytes = 0;
    for (uint32_t c = 0; c < ncols; ++c) set_bytes += r.rows * out_bytes_of(t, c);
    if (set_bytes < (256ull << 20)) return 0;  // small outputs: nothing to gain
    const bool dbg = getenv("FLS_DEBUG") != nullptr;
    // 1. by decode time: FLS_PLACEMENT_DECODE sets (default 6), the fastest kept
    const int ndec = (int)std::max<int64_t>(0, knob_value("FLS_PLACEMENT_DECODE"));
    float best_ms = ndec > 1 ? decode_rating(t, r) : -1.0f;
    if (best_ms > 0) {
        if (dbg) fprintf(stderr, "DEBUG: placement dev %d set 0: decode %.3f ms\n", r.dev, best_ms);
        int kept = 0;
        Candidate cand;
        for (int k = 1; k < ndec && alloc_candidate(t, r, set_bytes, cand); ++k) {
            cand.swap_into(r);  // the candidate decodes in place of the current set
            const float ms = decode_rating(t, r);
            if (dbg) fprintf(stderr, "DEBUG: placement dev %d set %d: decode %.3f ms\n", r.dev, k, ms);
            if (ms > 0 && ms < best_ms) {
                best_ms = ms;  // keep it: the previous set is freed with cand
                kept = k;
            } else {
                cand.swap_into(r);  // back to the current set; the candidate goes
            }
            cand.clear();
        }
        r.placement_ms = best_ms;
        if (dbg) fprintf(stderr, "DEBUG: placement dev %d kept set %d (decode %.3f ms)\n", r.dev, kept, best_ms);
        return 0;
    }
    // 2. by the write probe: up to FLS_PLACEMENT_TRIES sets, stop at q >= good
    const int tries = placement_tries();
    if (tries <= 1) return 0;
    const double good = knob_value("FLS_PLACEMENT_GOOD") / 1000.0;  // per mille
    PlacementRating best;
    if (const int rc = rate_outputs(t, r, r.d_out, best)) return rc;
    if (dbg)
        fprintf(stderr, "DEBUG: placement dev %d set 0: chunk order %.3f ms, fill %.3f ms, q %.3f\n", r.dev,
                best.chunk_ms, best.fill_ms, best.q);
    int kept = 0;
    Candidate cand;
    for (int k = 1; k < tries && best.q < good && alloc_candidate(t, r, set_bytes, cand); ++k) {
        PlacementRating pr;
        if (const int rc = rate_outputs(t, r, cand.out, pr)) return rc;
        if (dbg)
            fprintf(stderr, "DEBUG: placement dev %d set %d: chunk order %.3f ms, fill %.3f ms, q %.3f\n", r.dev, k,
                    pr.chunk_ms, pr.fill_ms, pr.q);
        if (pr.q > best.q) {
            cand.swap_into(r);  // the previous set is freed with cand
            best = pr;
            kept = k;
        }
        cand.clear();
    }
    r.placement_q = best.q;
    if (dbg) fprintf(stderr, "DEBUG: placement dev %d kept set %d (q %.3f)\n", r.dev, kept, best.q);
    return 0;
}

// Upload one GPU's part: row groups [rg0, rg1) verbatim, their string_t
// tables, HBM output columns and FSST heaps.
int upload_part(fls_table *t, Resident &r) {
    HIP_TRY(hipSetDevice(r.dev));
    if (!r.stream) HIP_TRY(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
    uint64_t lo, hi;
    rg_byte_range(t->meta, r.rg0, r.rg1, lo, hi);
    r.base = lo;
    HIP_TRY(r.img.alloc(r.dev, hi - lo + kImagePad));
    HIP_TRY(hipMemcpy(r.img.p, t->img + lo, hi - lo, hipMemcpyHostToDevice));
    std::vector<StrT> host;  // (the resident part keeps only the device tables)
    int rc = build_strtabs(t, r.dev, r.rg0, r.rg1, r.strtab, r.strtab_off, host);
    if (rc) return rc;
    HIP_TRY(r.err.alloc(r.dev, 1));
    HIP_TRY(hipMemset(r.err.p, 0, sizeof(uint32_t)));
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    r.first_row = t->meta.rgs[r.rg0].first_row;
    r.rows = t->meta.rgs[r.rg1 - 1].first_row + t->meta.rgs[r.rg1 - 1].nrows - r.first_row;
    r.d_out.resize(ncols);
    for (uint32_t c = 0; c < ncols; ++c) HIP_TRY(r.d_out[c].alloc(r.dev, r.rows * out_bytes_of(t, c)));
    // FSST heaps: chunk heaps back to back per column, host copy for string_t
    r.heap_off.assign((size_t)(r.rg1 - r.rg0) * ncols, 0);
    r.d_heap.resize(ncols);
    r.h_heap.resize(ncols);
    for (uint32_t c = 0; c < ncols; ++c) {
        uint64_t tot = 0;
        for (uint32_t g = r.rg0; g < r.rg1; ++g) {
            r.heap_off[(size_t)(g - r.rg0) * ncols + c] = tot;
            if (is_fsst(t, g, c)) tot += t->meta.rgs[g].chunks[c].hdr.reserved1;
        }
        if (tot) {
            HIP_TRY(r.d_heap[c].alloc(r.dev, tot));
            HIP_TRY(r.h_heap[c].alloc(tot));
        } else {
            r.d_heap[c].release();
            r.h_heap[c].release();
        }
    }
    r.h_chunks.clear();
    r.mask.clear();
    if (const int prc = choose_placement(t, r)) return prc;
    if (getenv("FLS_DEBUG")) {  // buffer placement (decode speed by buffer address)
        fprintf(stderr, "DEBUG: part dev %d rg [%u, %u) image %p %llu B\n", r.dev, r.rg0, r.rg1, (void *)r.img.p,
                (unsigned long long)(hi - lo));
        for (uint32_t c = 0; c < ncols; ++c)
            fprintf(stderr, "DEBUG:   col %u out %p %llu B heap %p\n", c, (void *)r.d_out[c].p,
                    (unsigned long long)(r.rows * out_bytes_of(t, c)), (void *)r.d_heap[c].p);
    }
    return 0;
}

// Enqueue one decode launch of the selected columns on part r (asynchronous).
int decode_part(fls_table *t, Resident &r, const std::vector<uint8_t> &mask) {
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    HIP_TRY(hipSetDevice(r.dev));
    const int64_t policy = decode_policy();
    if (mask != r.mask || r.h_chunks.empty() || policy != r.policy) {
        // (re)build the launch descriptor list: column-major task order, so
        // concurrent waves stream one column's consecutive row groups
        std::vector<DevChunk> chunks;
        ByteCount bc;
        for (uint32_t c = 0; c < ncols; ++c) {
            if (!mask[c]) continue;
            for (uint32_t g = r.rg0; g < r.rg1; ++g) {
                const ChunkRef &ch = t->meta.rgs[g].chunks[c];
                const uint64_t so = r.strtab_off[(size_t)(g - r.rg0) * ncols + c];
                const uint8_t *dict = so == UINT64_MAX ? nullptr : (const uint8_t *)(r.strtab.p + so);
                uint8_t *out = r.d_out[c].p + (t->meta.rgs[g].first_row - r.first_row) * out_bytes_of(t, c);
                const uint64_t ho = r.heap_off[(size_t)(g - r.rg0) * ncols + c];
                chunks.push_back(make_devchunk(t, g, c, r.img.p + (ch.off - r.base), dict, out, &bc,
                                               r.d_heap[c].p ? r.d_heap[c].p + ho : nullptr,
                                               r.h_heap[c].p ? r.h_heap[c].p + ho : nullptr));
            }
        }
        const int64_t lpol = launch_policy(policy, chunks, bc.geom);
        r.nmain = order_for_launch(chunks, &r.fsst, lpol);
        r.policy = policy;
        r.lpolicy = lpol;
        const size_t k = chunks.size();
        r.split = append_split(chunks, r.nmain, bc.geom, lpol);
        HIP_TRY(hipStreamSynchronize(r.stream));
        HIP_TRY(r.d_chunks.alloc(r.dev, chunks.size()));
        HIP_TRY(hipMemcpy(r.d_chunks.p, chunks.data(), chunks.size() * sizeof(DevChunk), hipMemcpyHostToDevice));
        chunks.resize(k);
        r.h_chunks.swap(chunks);
        r.mask = mask;
        r.bytes = bc;
    }
    if (r.ev_used + 2 > r.ev_pool.size()) {
        for (int i = 0; i < 2; ++i) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            r.ev_pool.push_back(e);
        }
    }
    // queue counters and the side stream exist before the timed region
    HIP_TRY(r.queue.alloc(r.dev, kQueueWords));
    if (!r.side.stream) {
        HIP_TRY(hipStreamCreateWithFlags(&r.side.stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&r.side.fork, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&r.side.join, hipEventDisableTiming));
    }
    if (r.fsst.total_vecs() > 0)
        if (const int rc = fsst_config_check(r.lpolicy)) return rc;
    hipEvent_t e0 = r.ev_pool[r.ev_used], e1 = r.ev_pool[r.ev_used + 1];
    r.ev_used += 2;
    HIP_TRY(hipEventRecord(e0, r.stream));
    HIP_TRY(launch_all(r.d_chunks.p, r.nmain, (uint32_t)r.h_chunks.size(), r.fsst, r.err.p, r.bytes.geom, r.stream,
                       r.queue.p, r.lpolicy, r.split, &r.side));
    HIP_TRY(hipEventRecord(e1, r.stream));
    return 0;
}

uint64_t resident_rows(const fls_table *t) {
    uint64_t n = 0;
    for (auto &r : t->resident) n += r->rows;
    return n;
}

const Resident *part_of(const fls_table *t, uint32_t part) {
    return t && part < t->resident.size() ? t->resident[part].get() : nullptr;
}

}  // namespace

extern "C" {

int fls_device_upload(fls_table *t, uint32_t rg_begin, uint32_t rg_end) {
    if (!t) return fail(FLS_ERR_ARG, "fls_device_upload: NULL table");
    if (rg_end > t->meta.rgs.size() || rg_begin >= rg_end)
        return fail(FLS_ERR_ARG, "row-group range [%u,%u) out of bounds", rg_begin, rg_end);
    // contiguous shards over the connection's GPUs, as a scan splits them
    const uint32_t G = (uint32_t)t->devices.size(), n = rg_end - rg_begin;
    t->resident.clear();
    t->launches = 0;
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t a = rg_begin + (uint32_t)((uint64_t)n * g / G), b = rg_begin + (uint32_t)((uint64_t)n * (g + 1) / G);
        if (a == b) continue;
        auto r = std::make_unique<Resident>();
        r->dev = t->devices[g];
        r->rg0 = a;
        r->rg1 = b;
        int rc = upload_part(t, *r);
        t->resident.push_back(std::move(r));
        if (rc) {
            t->resident.clear();
            return rc;
        }
    }
    return 0;
}

int fls_device_decode(fls_table *t, const uint8_t *col_mask) {
    if (!t) return fail(FLS_ERR_ARG, "fls_device_decode: NULL table");
    if (t->resident.empty()) return fail(FLS_ERR_STATE, "fls_device_decode before fls_device_upload");
    const uint32_t ncols = (uint32_t)t->meta.cols.size();
    std::vector<uint8_t> mask(ncols, 1);
    if (col_mask)
        for (uint32_t c = 0; c < ncols; ++c) mask[c] = col_mask[c] ? 1 : 0;
    for (auto &r : t->resident) {  // every GPU's launch is queued before any waits
        int rc = decode_part(t, *r, mask);
        if (rc) return rc;
    }
    t->launches++;
    return 0;
}

int fls_device_sync(fls_table *t, fls_decode_stats *stats) {
    if (!t) return fail(FLS_ERR_ARG, "fls_device_sync: NULL table");
    if (t->resident.empty()) return fail(FLS_ERR_STATE, "nothing uploaded");
    uint32_t err = 0;
    for (auto &r : t->resident) {
        HIP_TRY(hipSetDevice(r->dev));
        HIP_TRY(hipStreamSynchronize(r->stream));
        uint32_t e = 0;
        HIP_TRY(hipMemcpy(&e, r->err.p, sizeof(e), hipMemcpyDeviceToHost));
        err |= e;
    }
    if (stats) {
        // per launch the slowest GPU's time (the parts run concurrently)
        memset(stats, 0, sizeof(*stats));
        const uint32_t nl = t->resident[0]->ev_used / 2;
        double total = 0, last = 0;
        for (uint32_t i = 0; i < nl; ++i) {
            double span = 0;
            for (auto &r : t->resident) {
                if (2 * i + 1 >= r->ev_used) continue;
                float ms = 0;
                HIP_TRY(hipSetDevice(r->dev));
                HIP_TRY(hipEventElapsedTime(&ms, r->ev_pool[2 * i], r->ev_pool[2 * i + 1]));
                span = std::max(span, (double)ms);
            }
            total += span;
            last = span;
        }
        stats->kernel_ms = last;
        stats->kernel_ms_total = total;
        stats->timed_launches = nl;
        for (auto &r : t->resident) {
            stats->values += r->bytes.values;
            stats->packed_bytes += r->bytes.packed;
            stats->meta_bytes += r->bytes.meta;
            stats->out_bytes += r->bytes.out;
        }
        stats->launches = t->launches;
    }
    for (auto &r : t->resident) r->ev_used = 0;
    if (err & KERR_LDS_BASE) return fail(FLS_ERR_DEVICE, "FSST kernel: dynamic LDS not at address 0 (flags 0x%x)", err);
    if (err) return fail(FLS_ERR_FORMAT, "corrupt chunk detected while decoding (flags 0x%x)", err);
    return 0;
}

int fls_device_parts(const fls_table *t) { return t ? (int)t->resident.size() : 0; }

int fls_device_part(const fls_table *t, uint32_t part, fls_device_part_info *out) {
    const Resident *r = part_of(t, part);
    if (!r || !out) return fail(FLS_ERR_ARG, "resident part %u out of range", part);
    out->device = r->dev;
    out->rg_begin = r->rg0;
    out->rg_end = r->rg1;
    out->first_row = r->first_row;
    out->nrows = r->rows;
    return 0;
}

int fls_device_part_column(fls_table *t, uint32_t part, uint32_t col, void **dev_ptr, uint64_t *nbytes) {
    const Resident *r = part_of(t, part);
    if (!r || col >= r->d_out.size() || !r->d_out[col].p)
        return fail(FLS_ERR_ARG, "column %u of part %u not resident", col, part);
    if (dev_ptr) *dev_ptr = r->d_out[col].p;
    if (nbytes) *nbytes = r->rows * out_bytes_of(t, col);
    return 0;
}

int fls_device_part_heap(fls_table *t, uint32_t part, uint32_t col, void **dev_ptr, const void **host_ptr,
                         uint64_t *nbytes) {
    const Resident *r = part_of(t, part);
    if (!r || col >= r->d_out.size() || !r->d_out[col].p)
        return fail(FLS_ERR_ARG, "column %u of part %u not resident", col, part);
    const bool has = col < r->d_heap.size() && r->d_heap[col].p;
    if (dev_ptr) *dev_ptr = has ? r->d_heap[col].p : nullptr;
    if (host_ptr) *host_ptr = has ? r->h_heap[col].p : nullptr;
    if (nbytes) *nbytes = has ? r->d_heap[col].n : 0;
    return has ? 1 : 0;
}

// single-GPU accessors: the table's only part (a table split over several
// GPUs is addressed per part)
int fls_device_column(fls_table *t, uint32_t col, void **dev_ptr, uint64_t *nbytes) {
    if (t && t->resident.size() > 1)
        return fail(FLS_ERR_STATE, "table is resident on %zu GPUs: use fls_device_part_column", t->resident.size());
    return fls_device_part_column(t, 0, col, dev_ptr, nbytes);
}

int fls_device_heap(fls_table *t, uint32_t col, void **dev_ptr, const void **host_ptr, uint64_t *nbytes) {
    if (t && t->resident.size() > 1)
        return fail(FLS_ERR_STATE, "table is resident on %zu GPUs: use fls_device_part_heap", t->resident.size());
    return fls_device_part_heap(t, 0, col, dev_ptr, host_ptr, nbytes);
}

int fls_device_copy_out(fls_table *t, uint32_t col, uint64_t row, uint64_t n, void *host_dst) {
    if (!t || t->resident.empty() || col >= t->meta.cols.size() || !host_dst)
        return fail(FLS_ERR_ARG, "column %u not resident", col);
    const uint64_t total = resident_rows(t);
    if (row > total || n > total - row) return fail(FLS_ERR_ARG, "rows out of range");
    const int ob = out_bytes_of(t, col);
    uint64_t at = 0;  // first resident row of the part, counted over the parts
    for (auto &rp : t->resident) {
        Resident &r = *rp;
        const uint64_t a = std::max(row, at), b = std::min(row + n, at + r.rows);
        if (a < b) {
            HIP_TRY(hipSetDevice(r.dev));
            HIP_TRY(hipStreamSynchronize(r.stream));
            HIP_TRY(hipMemcpy((uint8_t *)host_dst + (a - row) * ob, r.d_out[col].p + (a - at) * ob, (b - a) * ob,
                              hipMemcpyDeviceToHost));
            // FSST: string_t pointers target the host copy of the part's heap
            if (col < r.d_heap.size() && r.d_heap[col].p)
                HIP_TRY(hipMemcpy(r.h_heap[col].p, r.d_heap[col].p, r.d_heap[col].n, hipMemcpyDeviceToHost));
        }
        at += r.rows;
    }
    return 0;
}

uint64_t fls_device_rows(const fls_table *t) { return t ? resident_rows(t) : 0; }

}  // extern "C"
