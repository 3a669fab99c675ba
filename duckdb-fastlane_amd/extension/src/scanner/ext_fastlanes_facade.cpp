// ext_fastlanes_facade.cpp -- ext_fastlane::FastLanesFacade (declared at
// reference src/include/fastlanes_facade.hpp:23-48, never implemented there).
//
// Reads stream every row group through the engine's GPU scan (fls_scan_*) and
// box values row-major as the intended scanner expects
// (src/scanner/scan_fastlanes.cpp:132-140).  Writes buffer DataChunks into
// 65,536-row row groups (src/writer/write_fastlane_stream.cpp:21-24) and hand
// them to the FastLanes writer (include/flswriter.h) on a background thread,
// kBatchRowGroups at a time (fls_writer_add_rowgroups encodes their chunks in
// parallel): a batch is encoded while the sink buffers the next one.
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <exception>
#include <functional>
#include <cstring>
#include <deque>
#include <future>
#include <atomic>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <algorithm>
#include "../../../../include/flsgpu.h"
#include "../../../../include/flswriter.h"
#include "../gpu_devices.hpp"
#include "duckdb/common/vector.hpp"
#include "fastlanes_facade.hpp"
#include "type_mapping.hpp"

namespace duckdb {
namespace ext_fastlane {

// FLS_COPY_PROFILE=1: where a COPY's time goes (sink copies, waits for the
// background writer, the final write), printed to stderr at finalizeFile
struct CopyProfile {
    bool on = std::getenv("FLS_COPY_PROFILE") != nullptr;
    double sink = 0, wait = 0, encode = 0, finish = 0, prep = 0, fixed = 0, str = 0;
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
};

// Growable byte buffer whose growth leaves the new bytes uninitialised: the
// sink overwrites them at once (std::vector::resize would zero them first,
// doubling the sink's memory traffic).
class RawBuf {
public:
    uint8_t *data() { return p_.get(); }
    const uint8_t *data() const { return p_.get(); }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    void clear() { n_ = 0; }
    // k more bytes at the end; returns where they start
    uint8_t *grow(size_t k) {
        if (n_ + k > cap_) {
            const size_t cap = std::max<size_t>({n_ + k, 2 * cap_, 4096});
            std::unique_ptr<uint8_t[]> q(new uint8_t[cap]);
            if (n_) memcpy(q.get(), p_.get(), n_);
            p_ = std::move(q);
            cap_ = cap;
        }
        uint8_t *at = p_.get() + n_;
        n_ += k;
        return at;
    }
    void shrink(size_t k) { n_ -= k; }

private:
    std::unique_ptr<uint8_t[]> p_;
    size_t n_ = 0, cap_ = 0;
};

// Helper threads for a lone sink (an ordered COPY has one): a DataChunk
// slice's columns are copied side by side instead of one after another (the
// one sink thread's copies were 63 % of an ordered COPY, copy_profile_r5k).
// A slice is ~50 us of work, less than waking a sleeping thread costs, so the
// helpers spin between slices and sleep after 2 ms without one.  run()
// publishes a job through a sequence number (odd while the job's fields
// change; helpers only join an even, new one, and leave the old one before
// the fields change).
class ColumnPool {
public:
    ~ColumnPool() { stop(); }
    int size() const { return (int)th_.size(); }
    void start(int helpers) {
        if (!th_.empty() || helpers <= 0) return;
        quit_ = false;
        for (int i = 0; i < helpers; ++i) th_.emplace_back([this] { loop(); });
    }
    // fn(0..n-1) on the caller and the helpers; returns when every call is
    // done, rethrowing on the caller the first exception a call threw (a
    // helper's bad_alloc must not end the process)
    void run(size_t n, const std::function<void(size_t)> &fn) {
        if (th_.empty() || n < 2) {
            for (size_t i = 0; i < n; ++i) fn(i);
            return;
        }
        const uint64_t g = seq_.load() + 1;
        seq_.store(g);  // odd: helpers stay out
        while (active_.load() != 0) spin();
        fn_ = &fn;
        n_ = n;
        next_.store(0);
        done_.store(0);
        seq_.store(g + 1);  // even: the job is open
        if (sleepers_.load() != 0) {
            std::lock_guard<std::mutex> lk(mu_);
            cv_.notify_all();
        }
        for (size_t i; (i = next_.fetch_add(1)) < n;) call(i);
        while (done_.load() != n) spin();
        if (failed_.load()) {
            failed_.store(false);
            std::exception_ptr e = std::move(error_);
            error_ = nullptr;
            std::rethrow_exception(e);
        }
    }

private:
    void call(size_t i) {
        try {
            (*fn_)(i);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu_);
            if (!failed_.exchange(true)) error_ = std::current_exception();
        }
        done_.fetch_add(1);
    }
    static void spin() {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    void loop() {
        uint64_t seen = seq_.load();
        auto idle = std::chrono::steady_clock::now();
        for (;;) {
            if (quit_.load()) return;
            const uint64_t g = seq_.load();
            if ((g & 1) == 0 && g != seen) {
                active_.fetch_add(1);
                if (seq_.load() == g) {
                    seen = g;
                    for (size_t i; (i = next_.fetch_add(1)) < n_;) call(i);
                }
                active_.fetch_sub(1);
                idle = std::chrono::steady_clock::now();
                continue;
            }
            if (std::chrono::steady_clock::now() - idle < std::chrono::milliseconds(2)) {
                spin();
                continue;
            }
            std::unique_lock<std::mutex> lk(mu_);
            sleepers_.fetch_add(1);
            cv_.wait_for(lk, std::chrono::milliseconds(100), [&] {
                const uint64_t x = seq_.load();
                return quit_.load() || ((x & 1) == 0 && x != seen);
            });
            sleepers_.fetch_sub(1);
            idle = std::chrono::steady_clock::now();
        }
    }
    void stop() {
        quit_.store(true);
        {
            std::lock_guard<std::mutex> lk(mu_);
            cv_.notify_all();
        }
        for (auto &t : th_) t.join();
        th_.clear();
    }
    std::vector<std::thread> th_;
    std::atomic<uint64_t> seq_{0};
    std::atomic<int> active_{0}, sleepers_{0};
    std::atomic<bool> quit_{false};
    const std::function<void(size_t)> *fn_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0}, done_{0};
    std::atomic<bool> failed_{false};
    std::exception_ptr error_;
    std::mutex mu_;
    std::condition_variable cv_;
};

class FastLanesFacade::Impl {
public:
    // read side
    fls_connection *conn = nullptr;
    fls_table *table = nullptr;
    std::vector<fls_column_info> cols;
    fls_rowgroup rg{};
    bool have_rg = false, eof = false;
    idx_t rg_pos = 0;
    // write side
    fls_writer *writer = nullptr;
    std::string out_path;
    std::string error;                               // why the last call returned false (lastError)
    bool finalized_ok = false;                       // the last finalizeFile wrote the file (finalizeOk)
    std::vector<LogicalType> wtypes;
    std::vector<std::string> wnames;
    Stage *own = nullptr;  // the serial path's stage (writeChunk(chunk), merges, the last row group)
    std::mutex hand;       // one batch hand-off at a time (flush_stage)
    std::mutex merge;      // one mergeStage at a time (it fills `own`)
    std::atomic<int> nstages{0};  // stages handed out (FLS_COPY_PROFILE times a lone sink only)
    idx_t rg_rows = 65536;
    // row groups per writer call (FLS_COPY_BATCH, default 8): one call encodes
    // every (row group, column) chunk in parallel, so a row group's slowest
    // column does not idle the writer's other threads
    idx_t batch_rgs = 8;
    // Bytes all sink stages together may buffer (FLS_COPY_STAGED_MB, default
    // 1024): past it, a stage hands its row groups over at its next row-group
    // boundary, so an unordered COPY on many threads stays within the budget
    // plus one row group per stage instead of batch_rgs row groups per thread.
    uint64_t staged_budget = 1ull << 30;
    std::atomic<uint64_t> staged{0}, staged_peak{0};  // bytes buffered by all stages (account)
    // Batches handed to the writer: each is a background task that assembles
    // its VARCHAR columns, waits for the previous batch's writer call (the
    // writer appends row groups in call order) and then calls the writer.  Up
    // to kMaxInflight batches are queued, so a sink that fills a stage while
    // the writer is busy keeps going instead of waiting; their buffers are
    // recycled through `spare`.
    struct Batch {
        std::vector<RawBuf> cols, rec, arena;
        std::vector<RawBuf> valid;  // per column: validity words of the batch rows, or empty (no NULL)
        std::vector<std::vector<uint32_t>> offs;  // per row group k: rows_k + 1 offsets from k * (rg_rows + 1)
        std::vector<std::vector<uint64_t>> base;  // per row group: its first byte in cols[c]
        // the writer call's arrays (a pipelined writer reads them after the call)
        std::vector<uint32_t> nrows;
        std::vector<const void *> data;
        std::vector<const uint32_t *> offs_p;
        std::vector<const uint64_t *> valid_p;
    };
    // Pipelined writer calls (fls_writer_set_pipelined; FLS_COPY_PIPELINE=0
    // turns them off): a call returns with its chunks still encoding, so the
    // batch it was given stays here until the next call (or the finish)
    // returns.  Touched only by the chained writer calls and after them.
    bool pipelined = true;
    std::unique_ptr<Batch> held;
    static constexpr size_t kMaxInflight = 3;
    std::deque<std::shared_future<std::string>> inflight;  // "" or the writer's error (fls_last_error is per thread)
    std::vector<std::unique_ptr<Batch>> spare;
    std::mutex spare_mu;
    CopyProfile prof;
    // a lone sink's column helpers (FLS_COPY_SINK_THREADS, default 4; 0 = none),
    // started at its first chunk; the sink holding cpool_mu uses them
    ColumnPool cpool;
    std::mutex cpool_mu;
    int cpool_threads = 4;
    double encode_s = 0;  // background writer calls (one at a time: the tasks are chained)
    // wait until at most `keep` batches are in flight, the time into *wait
    // (a profiled stage's own counter); false if one failed
    bool wait_pending(size_t keep = 0, double *wait = nullptr) {
        bool ok = true;
        while (inflight.size() > keep) {
            const double t0 = wait ? CopyProfile::now() : 0;
            const std::string e = inflight.front().get();
            inflight.pop_front();
            if (wait) *wait += CopyProfile::now() - t0;
            if (!e.empty()) {
                error = "FastLanes writer: " + e;
                ok = false;
            }
        }
        return ok;
    }

    void close_read() {
        if (table) fls_table_close(table);
        table = nullptr;
        conn = nullptr;  // the process-wide connection (SharedConnection) stays open
        have_rg = eof = false;
        rg_pos = 0;
    }
    bool flush_stage(Stage &st);
    bool stage_chunk(Stage &st, DataChunk &chunk);
    bool stage_full(Stage &st);
    static uint64_t staged_bytes(const Stage &st);
    void account(Stage &st);
    void reset_stage(Stage &st) const;
    ~Impl();
};

// Rows buffered by one sink thread for the next batch of row groups.
class FastLanesFacade::Stage {
public:
    std::vector<RawBuf> wcols;  // fixed-width buffered rows
    // VARCHAR columns: the sink keeps DuckDB's 16-byte string_t records (one
    // bulk copy per slice) and the bytes of the non-inlined strings, whose
    // pointer field it rewrites to their offset in warena; the background
    // task turns them into the writer's bytes + offsets, a thread per column
    std::vector<RawBuf> wrec, warena;
    // per column: validity words of the buffered rows (DuckDB's layout, bit r
    // = row r), allocated at the column's first NULL; empty: every row valid
    std::vector<RawBuf> wvalid;
    // string bytes per VARCHAR column in the stage's last (partial) row group:
    // the writer's offsets are 32-bit per row group
    std::vector<uint64_t> wbytes;
    idx_t wrows = 0;
    std::string error;
    uint64_t accounted = 0;  // this stage's bytes in Impl::staged
    // FLS_COPY_PROFILE times one stage (the first handed out, or the serial
    // path's): only its thread writes prof, and its writer waits count here
    bool profile = false;
    double wait = 0;
};

void FastLanesFacade::StageDeleter::operator()(Stage *st) const { delete st; }

FastLanesFacade::Impl::~Impl() {
    close_read();
    wait_pending();
    if (writer) fls_writer_free(writer);
    delete own;
}

void FastLanesFacade::Impl::reset_stage(Stage &st) const {
    for (auto *b : {&st.wcols, &st.wrec, &st.warena, &st.wvalid}) {
        b->resize(wtypes.size());
        for (auto &x : *b) x.clear();
    }
    st.wbytes.assign(wtypes.size(), 0);
    st.wrows = 0;
}

uint64_t FastLanesFacade::Impl::staged_bytes(const Stage &st) {
    uint64_t bytes = 0;
    for (auto *b : {&st.wcols, &st.wrec, &st.warena, &st.wvalid})
        for (auto &x : *b) bytes += x.size();
    return bytes;
}

// bring the stages' byte total up to date with this stage's buffers
void FastLanesFacade::Impl::account(Stage &st) {
    const uint64_t now = staged_bytes(st);
    const uint64_t total = staged.fetch_add(now - st.accounted) + (now - st.accounted);  // mod 2^64
    st.accounted = now;
    uint64_t peak = staged_peak.load();
    while (total > peak && !staged_peak.compare_exchange_weak(peak, total)) {
    }
}

// at a row-group boundary: a full batch, or any stage's rows while all stages
// together are over the staged-bytes budget, go to the writer
bool FastLanesFacade::Impl::stage_full(Stage &st) {
    account(st);
    if (st.wrows == 0 || st.wrows % rg_rows) return false;
    return st.wrows >= rg_rows * batch_rgs || staged.load() > staged_budget;
}

FastLanesFacade::FastLanesFacade() : pImpl(new Impl()) {}
FastLanesFacade::~FastLanesFacade() = default;

bool FastLanesFacade::openFile(const std::string &file_path) {
    Impl &s = *pImpl;
    s.close_read();
    s.conn = SharedConnection();
    if (!s.conn || fls_read_fls(s.conn, file_path.c_str(), &s.table) != 0) {
        s.close_read();
        return false;
    }
    s.cols.resize(fls_table_ncols(s.table));
    for (uint32_t c = 0; c < s.cols.size(); ++c) fls_table_column(s.table, c, &s.cols[c]);
    return true;
}

std::vector<LogicalType> FastLanesFacade::getColumnTypes() {
    std::vector<LogicalType> t;
    for (auto &c : pImpl->cols) t.push_back(TypeMapping::FastLanesToDuckDB(c.type, c.width, c.scale));
    return t;
}

std::vector<std::string> FastLanesFacade::getColumnNames() {
    std::vector<std::string> n;
    for (auto &c : pImpl->cols) n.emplace_back(c.name);
    return n;
}

static Value BoxValue(const fls_column_info &ci, const void *col, idx_t row) {
    const uint8_t *p = (const uint8_t *)col;
    auto ld = [p, row](auto x) {
        memcpy(&x, p + row * sizeof(x), sizeof(x));
        return x;
    };
    switch (ci.type) {
    case FLS_INT8: return Value::TINYINT(ld(int8_t()));
    case FLS_INT16: return Value::SMALLINT(ld(int16_t()));
    case FLS_INT32: return Value::INTEGER(ld(int32_t()));
    case FLS_INT64: return Value::BIGINT(ld(int64_t()));
    case FLS_UINT8: return Value::UTINYINT(ld(uint8_t()));
    case FLS_UINT16: return Value::USMALLINT(ld(uint16_t()));
    case FLS_UINT32: return Value::UINTEGER(ld(uint32_t()));
    case FLS_UINT64: return Value::UBIGINT(ld(uint64_t()));
    case FLS_DATE: return Value::DATE(date_t{ld(int32_t())});
    case FLS_DECIMAL: return Value::DECIMAL(ld(int64_t()), ci.width ? ci.width : 18, ci.scale);
    case FLS_FLOAT: return Value::FLOAT(ld(float()));
    case FLS_DOUBLE: return Value::DOUBLE(ld(double()));
    case FLS_BOOLEAN: return Value::BOOLEAN(ld(uint8_t()) != 0);
    case FLS_VARCHAR: {
        string_t s;
        memcpy(&s, p + 16 * row, 16);
        return Value(s.GetString());
    }
    case FLS_BLOB: {
        string_t s;
        memcpy(&s, p + 16 * row, 16);
        return Value::BLOB((const uint8_t *)s.GetData(), s.GetSize());
    }
    default: return Value();
    }
}

bool FastLanesFacade::readNextChunk(std::vector<Value> &values, idx_t &rows_read) {
    Impl &s = *pImpl;
    rows_read = 0;
    values.clear();
    if (!s.table || s.eof) return false;
    if (!s.have_rg || s.rg_pos >= s.rg.nrows) {
        if (!s.have_rg && fls_scan_begin(s.table, nullptr, 0, fls_table_nrowgroups(s.table)) != 0) return false;
        s.have_rg = true;
        const int rc = fls_scan_next(s.table, &s.rg);
        if (rc != 1) {
            s.eof = true;
            return false;
        }
        s.rg_pos = 0;
    }
    const idx_t n = std::min<idx_t>(STANDARD_VECTOR_SIZE, s.rg.nrows - s.rg_pos);
    values.reserve(n * s.cols.size());
    for (idx_t r = 0; r < n; ++r)
        for (size_t c = 0; c < s.cols.size(); ++c) {
            const idx_t row = s.rg_pos + r;
            const uint64_t *valid = s.rg.validity ? s.rg.validity[c] : nullptr;
            values.push_back(valid && !((valid[row / 64] >> (row % 64)) & 1) ? Value()
                                                                               : BoxValue(s.cols[c], s.rg.columns[c], row));
        }
    s.rg_pos += n;
    rows_read = n;
    return true;
}

void FastLanesFacade::closeFile() { pImpl->close_read(); }

const std::string &FastLanesFacade::lastError() const { return pImpl->error; }

bool FastLanesFacade::isValid() const { return pImpl->table != nullptr || pImpl->writer != nullptr; }

// ---- write path ------------------------------------------------------------

bool FastLanesFacade::createFile(const std::string &file_path, const std::vector<LogicalType> &types,
                                 const std::vector<std::string> &names) {
    Impl &s = *pImpl;
    if (types.size() != names.size() || types.empty()) return false;
    s.wait_pending();
    if (s.writer) fls_writer_free(s.writer);
    s.writer = fls_writer_new(0);
    // integer columns are chosen (ENC_AUTO) and encoded on the first GPU of
    // the extension's set when one is visible -- the file is byte-identical
    // to the CPU writer's (FLS_COPY_GPU=0 keeps the CPU)
    if (KnobValue("FLS_COPY_GPU") != 0 && fls_device_count() > 0) fls_writer_set_device(s.writer, GpuDevices()[0]);
    for (size_t c = 0; c < types.size(); ++c) {
        const uint8_t ft = TypeMapping::DuckDBToFastLanes(types[c]);
        if (!ft || fls_writer_add_column(s.writer, names[c].c_str(), ft, types[c].Width(), types[c].Scale(),
                                         FLS_ENC_AUTO) != 0) {
            fls_writer_free(s.writer);
            s.writer = nullptr;
            return false;
        }
    }
    // the file is written while the COPY runs (row groups stream to a
    // temporary file renamed over file_path at finalize); FLS_COPY_STREAM=0
    // writes it all at finalize instead
    s.pipelined = KnobValue("FLS_COPY_PIPELINE") != 0;
    if (s.pipelined) fls_writer_set_pipelined(s.writer, 1);
    if (KnobValue("FLS_COPY_STREAM") != 0 && fls_writer_set_output(s.writer, file_path.c_str()) != 0) {
        s.error = std::string("FastLanes writer: ") + fls_last_error();
        fls_writer_free(s.writer);
        s.writer = nullptr;
        return false;
    }
    s.out_path = file_path;
    s.wtypes = types;
    s.wnames = names;
    if (!s.own) s.own = new Stage();
    s.reset_stage(*s.own);
    s.own->accounted = 0;
    s.staged = 0;
    s.staged_peak = 0;
    s.batch_rgs = (idx_t)std::max<int64_t>(1, KnobValue("FLS_COPY_BATCH"));
    s.staged_budget = (uint64_t)std::max<int64_t>(1, KnobValue("FLS_COPY_STAGED_MB")) << 20;
    s.cpool_threads = (int)std::max<int64_t>(0, KnobValue("FLS_COPY_SINK_THREADS"));
    return true;
}

// Hand a stage's buffered row groups to the writer as a background task
// (queued behind at most kMaxInflight - 1 others; the writer calls run in
// hand-off order) and give the stage a recycled batch's buffers to keep filling.
bool FastLanesFacade::Impl::flush_stage(Stage &st) {
    if (st.wrows == 0) return true;
    std::lock_guard<std::mutex> guard(hand);
    if (!wait_pending(kMaxInflight - 1, st.profile ? &st.wait : nullptr)) {
        st.error = error;
        return false;
    }
    std::unique_ptr<Batch> bp;
    {
        std::lock_guard<std::mutex> g(spare_mu);
        if (!spare.empty()) {
            bp = std::move(spare.back());
            spare.pop_back();
        }
    }
    if (!bp) bp.reset(new Batch());
    Batch *b = bp.release();
    for (auto *x : {&b->cols, &b->rec, &b->arena, &b->valid}) x->resize(wtypes.size());
    b->offs.resize(wtypes.size());
    b->base.resize(wtypes.size());
    std::swap(b->cols, st.wcols);
    std::swap(b->rec, st.wrec);
    std::swap(b->arena, st.warena);
    std::swap(b->valid, st.wvalid);
    const uint32_t rows = (uint32_t)st.wrows;
    reset_stage(st);
    account(st);
    std::shared_future<std::string> prev = inflight.empty() ? std::shared_future<std::string>() : inflight.back();
    inflight.push_back(std::async(std::launch::async, [this, rows, b, prev]() {
        std::unique_ptr<Batch> own_b(b);
        auto recycle = [this, &own_b]() {
            std::lock_guard<std::mutex> g(spare_mu);
            spare.push_back(std::move(own_b));
        };
        const uint32_t nrg = (uint32_t)((rows + rg_rows - 1) / rg_rows);
        // VARCHAR columns: string_t records -> bytes + offsets, the offsets
        // restarting at 0 in each row group (the sink keeps a row group's
        // strings under 4 GiB); a thread per column
        auto assemble = [this, rows, nrg, b](size_t c) {
            const uint8_t *rec = b->rec[c].data();
            std::vector<uint32_t> &o = b->offs[c];
            std::vector<uint64_t> &base = b->base[c];
            o.resize((size_t)rows + nrg);
            base.resize(nrg);
            uint64_t total = 0;
            for (uint32_t k = 0; k < nrg; ++k) {
                const idx_t r0 = (idx_t)k * rg_rows, n = std::min<idx_t>(rg_rows, rows - r0);
                uint32_t *ok = o.data() + (size_t)k * (rg_rows + 1);
                ok[0] = 0;
                for (idx_t i = 0; i < n; ++i) {
                    uint32_t len;
                    memcpy(&len, rec + 16ull * (r0 + i), 4);
                    ok[i + 1] = ok[i] + len;
                }
                base[k] = total;
                total += ok[n];
            }
            RawBuf &col = b->cols[c];
            col.clear();
            uint8_t *dst = col.grow((size_t)total + string_t::INLINE_LENGTH);
            col.shrink(string_t::INLINE_LENGTH);
            for (uint32_t r = 0; r < rows; ++r) {
                const uint8_t *x = rec + 16ull * r;
                uint32_t len;
                memcpy(&len, x, 4);
                if (len <= string_t::INLINE_LENGTH) {
                    memcpy(dst, x + 4, string_t::INLINE_LENGTH);
                } else {
                    uint64_t off;
                    memcpy(&off, x + 8, 8);
                    memcpy(dst, b->arena[c].data() + off, len);
                }
                dst += len;
            }
        };
        std::vector<std::thread> th;
        for (size_t c = 0; c < wtypes.size(); ++c)
            if (TypeMapping::IsString(wtypes[c])) th.emplace_back(assemble, c);
        for (auto &t : th) t.join();
        // the writer takes batches in hand-off order; a failed batch fails the rest
        if (prev.valid()) {
            const std::string e = prev.get();
            if (!e.empty()) {
                recycle();
                return e;
            }
        }
        const double t0 = prof.on ? CopyProfile::now() : 0;
        // row group k of the batch: fixed-width columns at row k * rg_rows,
        // VARCHAR columns at their row group's first byte, with its offsets
        const size_t nc = wtypes.size();
        std::vector<uint32_t> nrows(nrg);
        std::vector<const void *> data((size_t)nrg * nc);
        std::vector<const uint32_t *> offs((size_t)nrg * nc, nullptr);
        for (uint32_t k = 0; k < nrg; ++k) {
            const idx_t r0 = (idx_t)k * rg_rows;
            nrows[k] = (uint32_t)std::min<idx_t>(rg_rows, rows - r0);
            for (size_t c = 0; c < nc; ++c) {
                if (TypeMapping::IsString(wtypes[c])) {
                    data[k * nc + c] = b->cols[c].empty() ? (const void *)"" : b->cols[c].data() + b->base[c][k];
                    offs[k * nc + c] = b->offs[c].data() + (size_t)k * (rg_rows + 1);
                } else {
                    const idx_t w = TypeMapping::GetFastLanesTypeSize(TypeMapping::DuckDBToFastLanes(wtypes[c]));
                    data[k * nc + c] = b->cols[c].data() + r0 * w;
                }
            }
        }
        // NULLs: row group k's validity words from word k * rg_rows / 64
        std::vector<const uint64_t *> valid((size_t)nrg * nc, nullptr);
        for (uint32_t k = 0; k < nrg; ++k)
            for (size_t c = 0; c < nc; ++c)
                if (!b->valid[c].empty())
                    valid[k * nc + c] = (const uint64_t *)b->valid[c].data() + (size_t)k * rg_rows / 64;
        const int rc = fls_writer_add_rowgroups_v(writer, nrg, nrows.data(), data.data(), offs.data(), valid.data());
        std::string e = rc == 0 ? std::string() : std::string(fls_last_error());
        if (prof.on) encode_s += CopyProfile::now() - t0;
        if (pipelined) {
            // this call has returned: the previous batch is free, this one
            // (and the arrays the call was given) stays until the next
            std::swap(b->nrows, nrows);
            std::swap(b->data, data);
            std::swap(b->offs_p, offs);
            std::swap(b->valid_p, valid);
            std::swap(held, own_b);
        }
        if (own_b) recycle();
        return e;
    }).share());
    return true;
}

// String bytes one row group of a column may hold (the writer's offsets are
// 32-bit per row group); FLS_TEST_STRING_LIMIT lowers it for tests
static uint64_t StringLimit() {
    static const uint64_t lim = [] {
        const char *e = std::getenv("FLS_TEST_STRING_LIMIT");
        return e ? std::strtoull(e, nullptr, 10) : (uint64_t)UINT32_MAX;
    }();
    return lim;
}

// Validity of stage rows [at, at + n) from `valid(i)` for i < n: the stage's
// words are allocated (every earlier row valid) at the column's first NULL
// and grow with the rows from then on (new words all valid).
template <class F>
static void StageValidity(RawBuf &words, idx_t at, idx_t n, bool any_null, F &&valid) {
    if (!any_null && words.empty()) return;
    const size_t need = 8 * ((at + n + 63) / 64);
    if (words.size() < need) {
        const size_t more = need - words.size();
        memset(words.grow(more), 0xFF, more);
    }
    if (!any_null) return;
    uint64_t *w = (uint64_t *)words.data();
    for (idx_t i = 0; i < n; ++i)
        if (!valid(i)) w[(at + i) / 64] &= ~(1ull << ((at + i) % 64));
}

// DuckDB's physical width of a fixed-size column (DECIMAL narrows with width)
static idx_t PhysicalWidth(const LogicalType &t) {
    if (t.id() == LogicalTypeId::DECIMAL) return t.Width() <= 4 ? 2 : t.Width() <= 9 ? 4 : 8;
    return TypeMapping::GetFastLanesTypeSize(TypeMapping::DuckDBToFastLanes(t));
}

// Copy a DataChunk into a stage; a full batch goes to the writer (a
// profiled stage accounts its time in prof).
bool FastLanesFacade::Impl::stage_chunk(Stage &st, DataChunk &chunk) {
    Impl &s = *this;
    const bool profile = st.profile;
    const double t_in = profile ? CopyProfile::now() : 0;
    struct Tally {  // sink time of this call, less its waits for the writer
        Impl &s;
        const Stage &st;
        double t_in, w_in;
        ~Tally() {
            if (st.profile) s.prof.sink += CopyProfile::now() - t_in - (st.wait - w_in);
        }
    } tally{s, st, t_in, st.wait};
    if (!s.writer || chunk.ColumnCount() != s.wtypes.size()) return false;
    double tp = t_in;
    auto lap = [&](double &acc) {  // profile: time since the last lap into acc
        if (!profile) return;
        const double t = CopyProfile::now();
        acc += t - tp;
        tp = t;
    };
    // A dictionary vector of strings (read_fastlanes' DICT columns) is read
    // through its selection: one gather of its records into the stage instead
    // of a flatten and a copy.  Every other vector is flattened.
    const size_t ncol = s.wtypes.size();
    std::vector<UnifiedVectorFormat> uf(ncol);
    std::vector<uint8_t> by_sel(ncol, 0);
    for (size_t c = 0; c < ncol; ++c) {
        Vector &v = chunk.data[c];
        if (v.GetVectorType() == VectorType::DICTIONARY_VECTOR && TypeMapping::IsString(s.wtypes[c])) {
            v.ToUnifiedFormat(chunk.size(), uf[c]);
            by_sel[c] = 1;
        } else {
            v.Flatten(chunk.size());
        }
    }
    lap(s.prof.prep);
    // A lone sink (an ordered COPY's, or the serial path's) copies a slice's
    // columns on the column helpers, VARCHAR columns first (the longest).
    // Per-column phase laps are taken only without them.
    std::unique_lock<std::mutex> par;
    if (s.cpool_threads > 0 && s.nstages.load() <= 1) {
        par = std::unique_lock<std::mutex>(s.cpool_mu, std::try_to_lock);
        if (par.owns_lock()) s.cpool.start(s.cpool_threads);
        else par = std::unique_lock<std::mutex>();
    }
    const bool on_pool = par.owns_lock() && s.cpool.size() > 0;
    std::vector<uint32_t> order;
    order.reserve(ncol);
    for (int pass = 0; pass < 2; ++pass)
        for (size_t c = 0; c < ncol; ++c)
            if (TypeMapping::IsString(s.wtypes[c]) == (pass == 0)) order.push_back((uint32_t)c);
    // column-major: append each column's slice up to the row-group boundary
    // in bulk; a full batch of row groups goes to the writer
    idx_t r0 = 0;
    while (r0 < chunk.size()) {
        // (a slice is at most one vector: the VARCHAR path's position list)
        const idx_t n = std::min<idx_t>({chunk.size() - r0, s.rg_rows - st.wrows % s.rg_rows, STANDARD_VECTOR_SIZE});
        std::atomic<int> too_long{-1};  // a VARCHAR column over the writer's 4 GiB per row group
        auto copy_col = [&](size_t c) {
            Vector &v = chunk.data[c];
            const LogicalType &t = s.wtypes[c];
            RawBuf &col = st.wcols[c];
            const ValidityMask &mask = by_sel[c] ? uf[c].validity : FlatVector::Validity(v);
            const SelectionVector *sel = by_sel[c] ? uf[c].sel : nullptr;
            auto row = [&](idx_t i) -> idx_t { return sel ? sel->get_index(r0 + i) : r0 + i; };
            const bool nulls = !mask.AllValid();
            StageValidity(st.wvalid[c], st.wrows, n, nulls, [&](idx_t i) { return mask.RowIsValid(row(i)); });
            if (TypeMapping::IsString(t)) {
                // the records in one copy or, for a dictionary vector, one
                // gather (a NULL row's record, undefined in DuckDB, becomes the
                // empty string); the non-inlined strings' bytes to the arena,
                // their pointer field := arena offset
                uint8_t *rec = st.wrec[c].grow(n * sizeof(string_t));
                if (sel) {
                    const string_t *d = (const string_t *)uf[c].data;
                    string_t *o = (string_t *)rec;
                    for (idx_t r = 0; r < n; ++r) o[r] = d[sel->get_index(r0 + r)];
                } else {
                    memcpy(rec, FlatVector::GetData<string_t>(v) + r0, n * sizeof(string_t));
                }
                if (nulls)
                    for (idx_t r = 0; r < n; ++r)
                        if (!mask.RowIsValid(row(r))) memset(rec + sizeof(string_t) * r, 0, sizeof(string_t));
                const string_t *str = (const string_t *)rec;
                // lengths and the positions of the non-inlined strings without
                // a data-dependent branch (inlined and pointer strings alternate
                // unpredictably in a column like l_shipinstruct), then their bytes
                uint32_t longs[STANDARD_VECTOR_SIZE];
                uint32_t nl = 0;
                uint64_t bytes = 0, lbytes = 0;
                for (idx_t r = 0; r < n; ++r) {
                    const uint32_t len = str[r].GetSize();
                    const bool lg = len > string_t::INLINE_LENGTH;
                    bytes += len;
                    lbytes += lg ? len : 0u;
                    longs[nl] = (uint32_t)r;
                    nl += lg ? 1u : 0u;
                }
                // the slice's arena bytes in one grow (a grow per string cost
                // the single ordered sink ~20 ns a string: l_comment's are all
                // non-inlined)
                RawBuf &ar = st.warena[c];
                uint64_t off = ar.size();
                uint8_t *dst = ar.grow(lbytes);
                for (uint32_t i = 0; i < nl; ++i) {
                    const uint32_t r = longs[i], len = str[r].GetSize();
                    memcpy(dst, str[r].GetData(), len);
                    memcpy(rec + sizeof(string_t) * r + 8, &off, 8);
                    dst += len;
                    off += len;
                }
                if (st.wbytes[c] + bytes > StringLimit()) {  // the writer's offsets are 32-bit
                    int none = -1;
                    too_long.compare_exchange_strong(none, (int)c);
                    return;
                }
                st.wbytes[c] += bytes;
                if (!on_pool) lap(s.prof.str);
                return;
            }
            // the physical bytes (FLOAT/DOUBLE bit-exact for ALP); DECIMAL widened to int64
            const idx_t w = TypeMapping::GetFastLanesTypeSize(TypeMapping::DuckDBToFastLanes(t));
            const idx_t pw = PhysicalWidth(t);
            const uint8_t *src = FlatVector::GetData<uint8_t>(v) + r0 * pw;
            uint8_t *dst = col.grow(n * w);
            if (pw == w) {
                memcpy(dst, src, n * w);
            } else {  // narrow DECIMAL: sign-extend
                for (idx_t i = 0; i < n; ++i) {
                    const int64_t x = pw == 2 ? (int64_t)((const int16_t *)src)[i] : (int64_t)((const int32_t *)src)[i];
                    memcpy(dst + 8 * i, &x, 8);
                }
            }
            if (!on_pool) lap(s.prof.fixed);
        };
        if (on_pool) {
            s.cpool.run(order.size(), [&](size_t k) { copy_col(order[k]); });
            lap(s.prof.str);  // (profiled: the helpers' slice time counts as VARCHAR)
        } else {
            for (size_t c = 0; c < ncol; ++c) copy_col(c);
        }
        if (too_long.load() >= 0) {
            st.error = "column \"" + s.wnames[too_long.load()] + "\" holds more than 4 GiB of strings in one row group";
            return false;
        }
        st.wrows += n;
        r0 += n;
        if (st.wrows % s.rg_rows == 0) st.wbytes.assign(s.wtypes.size(), 0);
        if (s.stage_full(st) && !s.flush_stage(st)) return false;
    }
    return true;
}

bool FastLanesFacade::writeChunk(DataChunk &chunk) {
    Impl &s = *pImpl;
    if (!s.own) return false;
    s.own->profile = s.prof.on;
    const bool ok = s.stage_chunk(*s.own, chunk);
    if (!ok) s.error = s.own->error;
    return ok;
}

FastLanesFacade::StagePtr FastLanesFacade::newStage() {
    Impl &s = *pImpl;
    StagePtr st(new Stage());
    s.reset_stage(*st);
    st->profile = s.prof.on && s.nstages.fetch_add(1) == 0;
    if (!s.prof.on) s.nstages.fetch_add(1);
    return st;
}

bool FastLanesFacade::writeChunk(Stage &stage, DataChunk &chunk) {
    Impl &s = *pImpl;
    return s.stage_chunk(stage, chunk);
}

const std::string &FastLanesFacade::stageError(const Stage &stage) const { return stage.error; }

// Append a stage's rows to `own` a row-group slice at a time (`own` may end a
// batch mid-merge and hand it over), the non-inlined strings' bytes re-based
// into own's arena.
bool FastLanesFacade::mergeStage(Stage &st) {
    Impl &s = *pImpl;
    if (!s.writer || !s.own) return false;
    std::lock_guard<std::mutex> guard(s.merge);
    if (st.profile) {
        s.prof.wait += st.wait;
        st.wait = 0;
    }
    Stage &o = *s.own;
    if (o.wrows == 0) {  // nothing to append to (the only sink of an ordered COPY): take the buffers
        std::swap(o.wcols, st.wcols);
        std::swap(o.wrec, st.wrec);
        std::swap(o.warena, st.warena);
        std::swap(o.wvalid, st.wvalid);
        std::swap(o.wbytes, st.wbytes);
        std::swap(o.wrows, st.wrows);
        std::swap(o.accounted, st.accounted);
        s.reset_stage(st);
        if (s.stage_full(o) && !s.flush_stage(o)) {
            st.error = o.error;
            return false;
        }
        return true;
    }
    const size_t nc = s.wtypes.size();
    // When own sits at a row-group boundary, st's complete row groups go to
    // the writer as they are (no copy: at the end of an unordered COPY every
    // sink's stage holds up to a batch of them, a GB in all at 16 sinks) and
    // only its partial last row group is copied into own.
    const idx_t full = o.wrows % s.rg_rows == 0 ? st.wrows / s.rg_rows * s.rg_rows : 0;
    idx_t r0 = full;
    while (r0 < st.wrows) {
        const idx_t n = std::min<idx_t>(st.wrows - r0, s.rg_rows - o.wrows % s.rg_rows);
        for (size_t c = 0; c < nc; ++c) {
            const RawBuf &sv = st.wvalid[c];
            StageValidity(o.wvalid[c], o.wrows, n, !sv.empty(), [&](idx_t i) {
                const idx_t r = r0 + i;
                return ((((const uint64_t *)sv.data())[r / 64] >> (r % 64)) & 1) != 0;
            });
            if (TypeMapping::IsString(s.wtypes[c])) {
                const uint8_t *src = st.wrec[c].data() + sizeof(string_t) * r0;
                uint8_t *rec = o.wrec[c].grow(n * sizeof(string_t));
                memcpy(rec, src, n * sizeof(string_t));
                uint64_t bytes = 0;
                for (idx_t r = 0; r < n; ++r) {
                    uint32_t len;
                    memcpy(&len, rec + sizeof(string_t) * r, 4);
                    bytes += len;
                    if (len <= string_t::INLINE_LENGTH) continue;
                    uint64_t off;
                    memcpy(&off, rec + sizeof(string_t) * r + 8, 8);
                    const uint64_t at = o.warena[c].size();
                    memcpy(o.warena[c].grow(len), st.warena[c].data() + off, len);
                    memcpy(rec + sizeof(string_t) * r + 8, &at, 8);
                }
                if (o.wbytes[c] + bytes > StringLimit()) {
                    st.error = "column \"" + s.wnames[c] + "\" holds more than 4 GiB of strings in one row group";
                    return false;
                }
                o.wbytes[c] += bytes;
            } else {
                const idx_t w = TypeMapping::GetFastLanesTypeSize(TypeMapping::DuckDBToFastLanes(s.wtypes[c]));
                memcpy(o.wcols[c].grow(n * w), st.wcols[c].data() + r0 * w, n * w);
            }
        }
        o.wrows += n;
        r0 += n;
        if (o.wrows % s.rg_rows == 0) o.wbytes.assign(nc, 0);
        if (s.stage_full(o) && !s.flush_stage(o)) {
            st.error = o.error;
            return false;
        }
    }
    if (full == 0) {
        s.reset_stage(st);
        s.account(st);
        return true;
    }
    // st keeps its rows [0, full): the copied tail goes, then st is a batch
    for (size_t c = 0; c < nc; ++c) {
        if (TypeMapping::IsString(s.wtypes[c])) {
            st.wrec[c].shrink(st.wrec[c].size() - full * sizeof(string_t));
        } else {
            const idx_t w = TypeMapping::GetFastLanesTypeSize(TypeMapping::DuckDBToFastLanes(s.wtypes[c]));
            st.wcols[c].shrink(st.wcols[c].size() - full * w);
        }
        if (!st.wvalid[c].empty()) st.wvalid[c].shrink(st.wvalid[c].size() - 8 * ((full + 63) / 64));
    }
    st.wbytes.assign(nc, 0);
    st.wrows = full;
    s.account(st);
    if (!s.flush_stage(st)) return false;  // (st.error set)
    s.reset_stage(st);
    s.account(st);
    return true;
}

bool FastLanesFacade::setRowGroupSize(idx_t rows) {
    Impl &s = *pImpl;
    if (!s.writer || !s.own || s.own->wrows != 0 || fls_writer_set_rowgroup_size(s.writer, (uint32_t)rows) != 0) return false;
    s.rg_rows = rows;
    return true;
}

void FastLanesFacade::finalizeFile() {
    Impl &s = *pImpl;
    s.finalized_ok = false;
    if (!s.writer) {
        s.error = "finalizeFile without createFile";
        return;
    }
    bool ok = s.own && s.flush_stage(*s.own);
    if (!ok && s.own) s.error = s.own->error;
    double final_wait = 0;
    ok = s.wait_pending(0, s.prof.on ? &final_wait : nullptr) && ok;
    const double t0 = s.prof.on ? CopyProfile::now() : 0;
    if (ok && fls_writer_finish_file(s.writer, s.out_path.c_str()) != 0) {
        s.error = std::string("FastLanes writer: ") + fls_last_error();
        ok = false;
    }
    if (s.prof.on) {
        s.prof.finish += CopyProfile::now() - t0;
        s.prof.wait += s.own->wait + final_wait;  // + the profiled stage's (mergeStage)
        fprintf(stderr,
                "COPY sink profile: DataChunk copies %.3f s (flatten + validity %.3f, fixed-width %.3f, VARCHAR %.3f), "
                "waits for the writer %.3f s, string assembly + writer calls %.3f s (background), file assembly + "
                "write %.3f s; peak staged %llu bytes\n",
                s.prof.sink, s.prof.prep, s.prof.fixed, s.prof.str, s.prof.wait, s.encode_s, s.prof.finish,
                (unsigned long long)s.staged_peak.load());
    }
    fls_writer_free(s.writer);  // (waits for a pipelined call's chunks)
    s.writer = nullptr;
    s.held.reset();
    s.finalized_ok = ok;
}

bool FastLanesFacade::finalizeOk() const { return pImpl->finalized_ok; }

}  // namespace ext_fastlane
}  // namespace duckdb
