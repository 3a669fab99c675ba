// read_fastlanes.cpp -- `read_fastlanes(path | [paths])` over the MI355X engine.
//
// Bind reads only footers (no GPU): typed schema via TypeMapping.  InitGlobal
// turns DuckDB's projected column_ids into the engine's column mask, so only
// projected columns are uploaded, decoded and copied back.  Scan is parallel
// (the reference pins MaxThreads to 1, src/scanner/scan_fastlanes.cpp:43-45):
// each DuckDB thread claims whole row groups from fls_scan_acquire
// (GPU-sharded, decoded ahead into pinned host memory) and emits
// STANDARD_VECTOR_SIZE-row DataChunks that REFERENCE the pinned row-group
// buffers (FlatVector::SetData, zero-copy: the decoded columns are already in
// DuckDB's physical layouts).  Each vector carries a RowGroupPin as its
// auxiliary buffer; the row group goes back to the engine (fls_scan_release)
// when the last vector referencing it is reset, so a chunk DuckDB keeps past
// the Scan call stays valid.  string_t records point into the file image
// (DICT) or the batch's pinned FSST heap, both kept alive by the same pin.
// DECIMAL(w<=9) columns are narrowed from the engine's int64 by a copy.  The
// batch index is the row group's position over all files, so DuckDB restores
// file order.  Error texts follow src/scanner/scan_fastlanes.cpp:62-97.
#include <glob.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>

#include "../../../../include/flsgpu.h"
#include "../gpu_devices.hpp"
#include "duckdb/common/exception.hpp"
#include "duckdb/common/string_util.hpp"
#include "duckdb/main/extension_util.hpp"
#include "duckdb/parallel/task_scheduler.hpp"
#include "duckdb/parser/expression/constant_expression.hpp"
#include "duckdb/parser/expression/function_expression.hpp"
#include "duckdb/parser/tableref/table_function_ref.hpp"
#include "duckdb/common/types/selection_vector.hpp"
#include "duckdb/planner/filter/conjunction_filter.hpp"
#include "duckdb/planner/filter/constant_filter.hpp"
#include "duckdb/planner/filter/in_filter.hpp"
#include "duckdb/planner/filter/null_filter.hpp"
#include "duckdb/planner/filter/optional_filter.hpp"
#include "duckdb/planner/table_filter.hpp"
#include "duckdb/planner/table_filter_state.hpp"
#include "duckdb/storage/table/column_segment.hpp"
#include "table_function/read_fastlanes.hpp"
#include "type_mapping.hpp"

namespace duckdb {
namespace ext_fastlane {

namespace {

// FLS_READ_PROFILE=1: where a scan thread's time goes (summed over threads,
// printed to stderr when the query's global state goes away): waiting for
// the claim lock, inside fls_scan_acquire (the GPU pipeline's hand-over),
// building deferred string_t records, filling the DataChunks by kind, and
// returning row groups (the RowGroupPin release).
struct ReadProfile {
    enum Phase { kLockWait, kAcquire, kRecords, kRelease, kEmitRef, kEmitDict, kEmitNarrow, kEmitCopy, kValidity,
                 kResidual, kScanTotal, kNumPhases };
    std::atomic<uint64_t> ns[kNumPhases] = {};
    std::atomic<uint64_t> rowgroups{0}, chunks{0}, rows{0};
    static bool on() {  // read per query (InitGlobal)
        const char *e = std::getenv("FLS_READ_PROFILE");
        return e && std::atoi(e) != 0;
    }
    static uint64_t now() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void print(idx_t threads) {
        static const char *names[kNumPhases] = {"lock wait", "fls_scan_acquire", "string_t records", "row-group release",
                                                "emit zero-copy", "emit dictionary", "emit narrowed (widen)",
                                                "emit copy (decimal)", "validity", "residual filters", "ReadScan total"};
        fprintf(stderr, "read_fastlanes profile: %llu row groups, %llu chunks, %llu rows, %llu threads (seconds summed over threads)\n",
                (unsigned long long)rowgroups.load(), (unsigned long long)chunks.load(), (unsigned long long)rows.load(),
                (unsigned long long)threads);
        for (int k = 0; k < kNumPhases; ++k) fprintf(stderr, "  %-24s %9.4f s\n", names[k], ns[k].load() * 1e-9);
    }
};
struct PhaseTimer {
    ReadProfile *p;
    int k;
    uint64_t t0;
    PhaseTimer(ReadProfile *prof, int phase) : p(prof), k(phase), t0(prof ? ReadProfile::now() : 0) {}
    ~PhaseTimer() {
        if (p) p->ns[k] += ReadProfile::now() - t0;
    }
};

// An open file on the process-wide engine connection (SharedConnection: its
// scan pipelines and pinned buffers carry over between queries).
struct OpenTable {
    fls_table *table = nullptr;
    ~OpenTable() {
        if (table) fls_table_close(table);
    }
    bool open(const std::string &path) {
        fls_connection *conn = SharedConnection();
        return conn && fls_read_fls(conn, path.c_str(), &table) == 0;
    }
};

struct ReadBindData : public TableFunctionData {
    vector<string> files;
    vector<LogicalType> types;
    vector<string> names;
    vector<fls_column_info> cols;
    // the first file as Bind opened it (mapped, validated): the first
    // InitGlobal takes it instead of opening the file a second time (an open
    // validates every chunk header: 10-30 ms at SF10); later ones reopen
    mutable std::mutex bound_lock;
    mutable std::shared_ptr<OpenTable> bound;
};

struct ReadGlobalState : public GlobalTableFunctionState {
    vector<column_t> column_ids;
    vector<idx_t> out_ids;               // output column -> position in column_ids
    std::vector<uint8_t> mask;           // delivered table columns
    std::vector<fls_predicate> preds;    // pushed-down filter (empty: none)
    bool narrow = false;                 // narrowed delivery of integer columns (fls_scan_narrow)
    std::deque<string> pred_strs;        // VARCHAR constants the predicates point at
    // pushed-down filters the engine cannot evaluate (e.g. EXPRESSION_FILTER):
    // applied on the host to every delivered chunk the way DuckDB's own scans
    // apply them (ColumnSegment::FilterSelection), so the query never fails
    // on an unknown filter and no row that fails one is delivered
    struct Residual {
        column_t id;
        const TableFilter *filter;  // owned by DuckDB's TableFilterSet (lives for the query)
    };
    vector<Residual> residual;
    std::vector<idx_t> rg_base;          // batch index of each file's first row group
    std::vector<std::shared_ptr<OpenTable>> tables;  // opened (mapped) at init, scanned in order
    idx_t total_rowgroups = 0;
    std::mutex lock;                     // file advance and row-group claims
    idx_t file_idx = 0;
    std::shared_ptr<OpenTable> cur;      // file being scanned (nullptr: open the next)
    idx_t MaxThreads() const override { return std::max<idx_t>(1, total_rowgroups); }
    std::unique_ptr<ReadProfile> prof;   // FLS_READ_PROFILE
    std::atomic<idx_t> threads{0};
    ~ReadGlobalState() override {
        if (prof) prof->print(threads.load());
    }
};

// A delivered row group's pinned buffers, held by the local state while it
// emits chunks and by every vector that references them.  The last holder
// hands the row group back to the engine, which then recycles its batch slot.
// A failed release (a batch refill that could not be enqueued) is sticky in
// the engine: the next fls_scan_acquire reports it as an IOException.
struct RowGroupPin : public VectorBuffer {
    std::shared_ptr<OpenTable> table;    // keeps the file (DICT string_t targets) open
    uint32_t rowgroup;
    RowGroupPin(std::shared_ptr<OpenTable> t, uint32_t rg)
        : VectorBuffer(VectorBufferType::OPAQUE_BUFFER), table(std::move(t)), rowgroup(rg) {}
    ~RowGroupPin() override { fls_scan_release(table->table, rowgroup); }
};

struct ReadLocalState : public LocalTableFunctionState {
    vector<unique_ptr<TableFilterState>> residual_state;  // one per ReadGlobalState::residual (per thread)
    buffer_ptr<RowGroupPin> pin;         // the row group being emitted (nullptr: none)
    fls_rowgroup rg{};
    fls_table *table = nullptr;          // the table rg came from (held by pin)
    idx_t rg_pos = 0;
    idx_t batch_index = 0;
};

void CollectPaths(const Value &v, vector<string> &files, const char *fn) {
    if (v.IsNull()) throw BinderException(string(fn) + " file paths must be strings");
    if (v.type().id() == LogicalTypeId::LIST) {
        for (auto &c : v.ListChildren()) CollectPaths(c, files, fn);
        return;
    }
    if (v.type() != LogicalType::VARCHAR) throw BinderException(string(fn) + " file paths must be strings");
    const string path = v.GetValue<string>();
    if (path.find_first_of("*?[") == string::npos) {
        files.push_back(path);
        return;
    }
    // glob pattern, expanded in sorted order like DuckDB's FileSystem::GlobFiles
    glob_t g{};
    const int rc = glob(path.c_str(), 0, nullptr, &g);
    vector<string> hits;
    if (rc == 0)
        for (size_t i = 0; i < g.gl_pathc; ++i) hits.emplace_back(g.gl_pathv[i]);
    globfree(&g);
    if (hits.empty()) throw IOException("No files found that match the pattern \"" + path + "\"");
    std::sort(hits.begin(), hits.end());
    files.insert(files.end(), hits.begin(), hits.end());
}

unique_ptr<FunctionData> ReadBind(ClientContext &, TableFunctionBindInput &input, vector<LogicalType> &return_types,
                                  vector<string> &names) {
    auto bind = make_uniq<ReadBindData>();
    for (auto &v : input.inputs) CollectPaths(v, bind->files, "read_fastlanes");
    if (bind->files.empty()) throw BinderException("read_fastlanes requires at least one file path");
    auto t = std::make_shared<OpenTable>();
    if (!t->open(bind->files[0])) throw BinderException("Failed to open FastLanes file: " + bind->files[0]);
    const uint32_t n = fls_table_ncols(t->table);
    bind->cols.resize(n);
    for (uint32_t c = 0; c < n; ++c) {
        fls_table_column(t->table, c, &bind->cols[c]);
        bind->types.push_back(TypeMapping::FastLanesToDuckDB(bind->cols[c].type, bind->cols[c].width, bind->cols[c].scale));
        bind->names.emplace_back(bind->cols[c].name);
        bind->cols[c].name = nullptr;  // owned by the table (names are copied above)
    }
    bind->bound = std::move(t);
    return_types = bind->types;
    names = bind->names;
    return std::move(bind);
}

// engine comparison of a DuckDB one; false: none (the filter stays on the host)
bool CompareOp(ExpressionType t, uint8_t &op) {
    switch (t) {
    case ExpressionType::COMPARE_EQUAL: op = FLS_CMP_EQ; return true;
    case ExpressionType::COMPARE_NOTEQUAL: op = FLS_CMP_NE; return true;
    case ExpressionType::COMPARE_LESSTHAN: op = FLS_CMP_LT; return true;
    case ExpressionType::COMPARE_LESSTHANOREQUALTO: op = FLS_CMP_LE; return true;
    case ExpressionType::COMPARE_GREATERTHAN: op = FLS_CMP_GT; return true;
    case ExpressionType::COMPARE_GREATERTHANOREQUALTO: op = FLS_CMP_GE; return true;
    default: return false;
    }
}

// `col <op> constant` with the constant in the column's physical type; false:
// a type the engine does not compare (the filter stays on the host)
bool MakeTerm(uint32_t col, uint32_t clause, uint8_t op, const Value &v, const LogicalType &type,
              std::deque<string> &strs, fls_predicate &p) {
    memset(&p, 0, sizeof(p));
    p.col = col;
    p.clause = clause;
    p.op = op;
    if (v.IsNull()) {  // a comparison with NULL is never true
        p.op = FLS_CMP_FALSE;
        return true;
    }
    switch (type.id()) {
    case LogicalTypeId::TINYINT: case LogicalTypeId::SMALLINT: case LogicalTypeId::INTEGER:
    case LogicalTypeId::BIGINT:
        p.value = (uint64_t)v.GetValue<int64_t>();
        break;
    case LogicalTypeId::UTINYINT: case LogicalTypeId::USMALLINT: case LogicalTypeId::UINTEGER:
    case LogicalTypeId::UBIGINT:
        p.value = v.GetValue<uint64_t>();
        break;
    case LogicalTypeId::BOOLEAN:  // u8 0 / 1
        p.value = v.GetValue<bool>() ? 1 : 0;
        break;
    case LogicalTypeId::DATE:
        p.value = (uint64_t)(int64_t)v.GetValue<date_t>().days;
        break;
    case LogicalTypeId::DECIMAL:  // DuckDB casts the constant to the column's DECIMAL type
        p.value = (uint64_t)(type.Width() <= 4   ? (int64_t)v.GetValueUnsafe<int16_t>()
                             : type.Width() <= 9 ? (int64_t)v.GetValueUnsafe<int32_t>()
                                                 : v.GetValueUnsafe<int64_t>());
        break;
    case LogicalTypeId::FLOAT: {
        const float f = v.GetValue<float>();
        uint32_t b;
        memcpy(&b, &f, 4);
        p.value = b;
        break;
    }
    case LogicalTypeId::DOUBLE: {
        const double d = v.GetValue<double>();
        memcpy(&p.value, &d, 8);
        break;
    }
    case LogicalTypeId::BLOB:  // the constant's bytes (StringValue::Get), compared unsigned like DuckDB
        if (v.type().id() != LogicalTypeId::BLOB) return false;
        strs.push_back(StringValue::Get(v));
        p.str = strs.back().data();
        p.str_len = strs.back().size();
        break;
    case LogicalTypeId::VARCHAR:
        strs.push_back(v.GetValue<string>());
        p.str = strs.back().data();
        p.str_len = strs.back().size();
        break;
    default: return false;
    }
    return true;
}

// one clause of OR-ed terms (constants, IN lists, IS [NOT] NULL); false: a
// term the engine cannot evaluate
bool AddOrTerms(const TableFilter &f, uint32_t col, uint32_t clause, const LogicalType &type,
                std::vector<fls_predicate> &out, std::deque<string> &strs) {
    fls_predicate p;
    switch (f.filter_type) {
    case TableFilterType::CONSTANT_COMPARISON: {
        auto &c = f.Cast<ConstantFilter>();
        uint8_t op;
        if (!CompareOp(c.comparison_type, op) || !MakeTerm(col, clause, op, c.constant, type, strs, p)) return false;
        out.push_back(p);
        break;
    }
    case TableFilterType::IN_FILTER:
        for (auto &v : f.Cast<InFilter>().values) {
            if (!MakeTerm(col, clause, FLS_CMP_EQ, v, type, strs, p)) return false;
            out.push_back(p);
        }
        break;
    case TableFilterType::IS_NULL:
    case TableFilterType::IS_NOT_NULL: {
        memset(&p, 0, sizeof(p));
        p.col = col;
        p.clause = clause;
        p.op = f.filter_type == TableFilterType::IS_NULL ? FLS_CMP_IS_NULL : FLS_CMP_IS_NOT_NULL;
        out.push_back(p);
        break;
    }
    case TableFilterType::CONJUNCTION_OR:
        for (auto &ch : f.Cast<ConjunctionOrFilter>().child_filters)
            if (!AddOrTerms(*ch, col, clause, type, out, strs)) return false;
        break;
    default: return false;
    }
    return true;
}

// TableFilter on one column -> clauses (AND of ORs); false: some part the
// engine cannot evaluate (the caller keeps the whole filter on the host)
bool AddFilter(const TableFilter &f, uint32_t col, const LogicalType &type, uint32_t &clause,
               std::vector<fls_predicate> &out, std::deque<string> &strs) {
    switch (f.filter_type) {
    case TableFilterType::CONJUNCTION_AND:
        for (auto &ch : f.Cast<ConjunctionAndFilter>().child_filters)
            if (!AddFilter(*ch, col, type, clause, out, strs)) return false;
        return true;
    case TableFilterType::OPTIONAL_FILTER:  // optional by definition: DuckDB re-checks it above the scan
        return true;
    case TableFilterType::CONSTANT_COMPARISON: case TableFilterType::IN_FILTER: case TableFilterType::IS_NULL:
    case TableFilterType::IS_NOT_NULL: case TableFilterType::CONJUNCTION_OR:
        return AddOrTerms(f, col, clause++, type, out, strs);
    default: return false;  // EXPRESSION_FILTER, STRUCT_EXTRACT, DYNAMIC_FILTER, ...
    }
}

unique_ptr<GlobalTableFunctionState> ReadInitGlobal(ClientContext &context, TableFunctionInitInput &input) {
    const auto &bind = input.bind_data->Cast<ReadBindData>();
    auto state = make_uniq<ReadGlobalState>();
    if (ReadProfile::on()) state->prof.reset(new ReadProfile());
    // Narrowed delivery trades host work (adding the base back while filling
    // each vector) for PCIe bytes: it pays when the scan is link-bound, with
    // several threads to widen (lineitem_full SF10: 16 threads 4.3 -> 5.6-5.9e8
    // rows/s; one thread 3.9 -> 2.7e8).  FLS_READ_NARROW=1 / 0 forces it.
    const char *nv = std::getenv("FLS_READ_NARROW");
    state->narrow = nv ? std::atoi(nv) != 0 : TaskScheduler::GetScheduler(context).NumberOfThreads() >= 4;
    state->column_ids = input.column_ids;
    if (input.projection_ids.empty()) {
        for (idx_t i = 0; i < input.column_ids.size(); ++i) state->out_ids.push_back(i);
    } else {
        state->out_ids = input.projection_ids;
    }
    state->mask.assign(bind.cols.size(), 0);
    for (auto pos : state->out_ids) {
        const column_t id = state->column_ids[pos];
        if (id != COLUMN_IDENTIFIER_ROW_ID && id < bind.cols.size()) state->mask[id] = 1;
    }
    if (input.filters) {
        uint32_t clause = 0;
        for (auto &entry : input.filters->filters) {
            const column_t id = state->column_ids[entry.first];
            if (id == COLUMN_IDENTIFIER_ROW_ID || id >= bind.cols.size())
                throw NotImplementedException("read_fastlanes: filter on a non-table column");
            // the engine takes the column's filter whole or not at all
            const size_t n0 = state->preds.size();
            const uint32_t c0 = clause;
            if (!AddFilter(*entry.second, (uint32_t)id, bind.types[id], clause, state->preds, state->pred_strs)) {
                state->preds.resize(n0);
                clause = c0;
                state->residual.push_back({id, entry.second.get()});
                state->mask[id] = 1;  // the host needs the column's values
            }
        }
    }
    // fail early on unreadable or schema-incompatible files
    std::shared_ptr<OpenTable> prebound;
    {
        std::lock_guard<std::mutex> lk(bind.bound_lock);
        prebound = std::move(bind.bound);
    }
    for (auto &f : bind.files) {
        auto t = (&f == &bind.files[0] && prebound) ? std::move(prebound) : std::make_shared<OpenTable>();
        if (!t->table && !t->open(f)) throw IOException("Failed to open FastLanes file: " + f);
        bool same = fls_table_ncols(t->table) == bind.cols.size();
        for (uint32_t c = 0; same && c < bind.cols.size(); ++c) {
            fls_column_info ci;
            fls_table_column(t->table, c, &ci);
            same = ci.type == bind.cols[c].type && ci.width == bind.cols[c].width && ci.scale == bind.cols[c].scale;
        }
        if (!same) throw IOException("FastLanes file " + f + " does not match the schema of " + bind.files[0]);
        state->rg_base.push_back(state->total_rowgroups);
        state->total_rowgroups += fls_table_nrowgroups(t->table);
        state->tables.push_back(std::move(t));
    }
    return std::move(state);
}

unique_ptr<LocalTableFunctionState> ReadInitLocal(ExecutionContext &context, TableFunctionInitInput &,
                                                  GlobalTableFunctionState *gstate) {
    auto l = make_uniq<ReadLocalState>();
    gstate->Cast<ReadGlobalState>().threads++;
    for (auto &r : gstate->Cast<ReadGlobalState>().residual)
        l->residual_state.push_back(TableFilterState::Initialize(context.client, *r.filter));
    return std::move(l);
}

// give back the local state's row group and claim the next one (in file and
// row-group order over all threads); false at the end of all files.  The
// global lock covers only the file advance: fls_scan_acquire is thread-safe
// and hands out row groups in order itself, and it may wait for a batch or
// enqueue the next one (the 16-thread profile showed two thirds of the scan
// threads' time waiting for this lock while it was held across the acquire).
bool NextRowGroup(const ReadBindData &bind, ReadGlobalState &g, ReadLocalState &l) {
    ReadProfile *prof = g.prof.get();
    {
        PhaseTimer t(prof, ReadProfile::kRelease);
        l.pin.reset();  // released now unless a chunk DuckDB still holds references it
    }
    while (true) {
        std::shared_ptr<OpenTable> cur;
        idx_t fidx;
        {
            const uint64_t tw = prof ? ReadProfile::now() : 0;
            std::lock_guard<std::mutex> guard(g.lock);
            if (prof) prof->ns[ReadProfile::kLockWait] += ReadProfile::now() - tw;
            if (!g.cur) {
                if (g.file_idx >= bind.files.size()) return false;
                auto t = std::move(g.tables[g.file_idx]);  // opened by InitGlobal
                if (fls_scan_filter(t->table, g.preds.data(), (uint32_t)g.preds.size()) != 0)
                    throw IOException(string("FastLanes scan failed: ") + fls_last_error());
                // DICT string columns as codes + dictionary (DuckDB dictionary
                // vectors: 1-2 bytes per row over PCIe instead of a 16-byte
                // string_t); FLS_READ_DICT=0 delivers string_t (A/B knob)
                static const bool codes = KnobValue("FLS_READ_DICT") != 0;
                // integer columns narrowed to their row groups' ranges (value -
                // base in 1-4 bytes, widened in EmitColumn), see ReadInitGlobal;
                // narrowed scans deliver FSST columns as lengths, their string_t
                // records built by the consuming thread (ReadScan)
                if (fls_scan_dict_codes(t->table, codes ? 1 : 0) != 0 ||
                    fls_scan_narrow(t->table, g.narrow ? 1 : 0) != 0 || fls_scan_defer_records(t->table, 1) != 0 ||
                    fls_scan_begin(t->table, g.mask.data(), 0, fls_table_nrowgroups(t->table)) != 0)
                    throw IOException(string("FastLanes scan failed: ") + fls_last_error());
                g.cur = std::move(t);
            }
            cur = g.cur;
            fidx = g.file_idx;
        }
        int rc;
        {
            PhaseTimer t(prof, ReadProfile::kAcquire);
            rc = fls_scan_acquire(cur->table, &l.rg);
        }
        if (rc < 0) throw IOException(string("FastLanes scan failed: ") + fls_last_error());
        if (rc == 1) {
            if (prof) prof->rowgroups++;
            l.table = cur->table;
            l.pin = make_buffer<RowGroupPin>(cur, l.rg.rowgroup);
            l.rg_pos = 0;
            l.batch_index = g.rg_base[fidx] + l.rg.rowgroup;
            return true;
        }
        // this file is done: the first thread to see it moves the scan on
        std::lock_guard<std::mutex> guard(g.lock);
        if (g.cur == cur) {
            g.cur.reset();  // closed once the last thread holding one of its row groups lets go
            g.file_idx++;
        }
    }
}

// rows [rg_pos, rg_pos + n) of table column id into vec: a reference to the
// pinned row group (zero-copy) or, for DECIMAL(w<=9), the engine's int64
// narrowed to DuckDB's physical width
void EmitColumn(const ReadBindData &bind, ReadLocalState &l, column_t id, Vector &vec, idx_t n,
                ReadProfile *prof = nullptr) {
    const idx_t ob = bind.cols[id].out_bytes;
    // NULLs: the delivered rows' validity words (rg_pos is a multiple of
    // STANDARD_VECTOR_SIZE, so whole words)
    if (const uint64_t *valid = l.rg.validity ? l.rg.validity[id] : nullptr) {
        PhaseTimer t(prof, ReadProfile::kValidity);
        auto &mask = FlatVector::Validity(vec);
        mask.Initialize(STANDARD_VECTOR_SIZE);
        memcpy(mask.GetData(), valid + l.rg_pos / 64, ValidityMask::EntryCount(n) * sizeof(validity_t));
    }
    const bool is_dict = l.rg.dict && l.rg.dict[id];
    const bool is_narrow = !is_dict && l.rg.narrow && l.rg.narrow[id];
    PhaseTimer t(prof, is_dict ? ReadProfile::kEmitDict
                       : is_narrow ? ReadProfile::kEmitNarrow
                       : vec.GetType().PhysicalSize() == ob ? ReadProfile::kEmitRef : ReadProfile::kEmitCopy);
    if (const void *dict = l.rg.dict ? l.rg.dict[id] : nullptr) {  // dictionary codes
        const uint8_t w = l.rg.dict_width[id];
        const uint8_t *codes = (const uint8_t *)l.rg.columns[id] + l.rg_pos * w;
        auto code = [codes, w](idx_t i) -> sel_t {
            return w == 1 ? codes[i] : (sel_t)(codes[2 * i] | (uint32_t)codes[2 * i + 1] << 8);
        };
        const string_t *entries = (const string_t *)dict;
        if (l.rg.validity && l.rg.validity[id]) {  // NULLs: flat strings beside the validity set above
            string_t *d = FlatVector::GetData<string_t>(vec);
            for (idx_t i = 0; i < n; ++i) d[i] = entries[code(i)];
            // long strings point into the mapped file image: keep the row
            // group (and its table) alive as long as the vector
            vec.SetAuxiliary(l.pin);
            return;
        }
        // the row group's dictionary as a vector over the engine's string_t
        // records, the rows a selection of it
        Vector dict_vec(vec.GetType(), (data_ptr_t)dict);
        dict_vec.SetAuxiliary(l.pin);
        SelectionVector sel(n);
        sel_t *sd = sel.data();  // u8 / u16 -> sel_t widening, vectorisable
        if (w == 1) {
            for (idx_t i = 0; i < n; ++i) sd[i] = codes[i];
        } else {
            const uint16_t *c16 = (const uint16_t *)codes;  // 2-byte aligned: rg_pos is even
            for (idx_t i = 0; i < n; ++i) sd[i] = c16[i];
        }
        vec.Slice(dict_vec, sel, n);
        return;
    }
    const idx_t phys = vec.GetType().PhysicalSize();
    if (l.rg.narrow && l.rg.narrow[id]) {  // narrowed: value = base + difference, into DuckDB's width
        const uint8_t w = l.rg.dict_width[id];
        const uint64_t base = l.rg.narrow_base[id];
        const uint8_t *q = (const uint8_t *)l.rg.columns[id] + l.rg_pos * w;
        uint8_t *d = FlatVector::GetData<uint8_t>(vec);
        auto widen = [&](auto narrow_t, auto phys_t) {
            using N = decltype(narrow_t);
            using P = decltype(phys_t);
            const N *src = (const N *)q;
            P *dst = (P *)d;
            for (idx_t i = 0; i < n; ++i) dst[i] = (P)(base + src[i]);
        };
        auto by_phys = [&](auto narrow_t) {
            switch (phys) {
            case 2: widen(narrow_t, uint16_t()); break;
            case 4: widen(narrow_t, uint32_t()); break;
            default: widen(narrow_t, uint64_t()); break;
            }
        };
        if (w == 1) by_phys(uint8_t());
        else if (w == 2) by_phys(uint16_t());
        else by_phys(uint32_t());
        return;
    }
    const uint8_t *src = (const uint8_t *)l.rg.columns[id] + l.rg_pos * ob;
    if (phys == ob) {
        FlatVector::SetData(vec, (data_ptr_t)src);
        vec.SetAuxiliary(l.pin);
        return;
    }
    const int64_t *v = (const int64_t *)src;
    if (phys == 4) {
        int32_t *d = FlatVector::GetData<int32_t>(vec);
        for (idx_t i = 0; i < n; ++i) d[i] = (int32_t)v[i];
    } else {
        int16_t *d = FlatVector::GetData<int16_t>(vec);
        for (idx_t i = 0; i < n; ++i) d[i] = (int16_t)v[i];
    }
}

void ReadScan(ClientContext &, TableFunctionInput &data, DataChunk &output) {
    const auto &bind = data.bind_data->Cast<ReadBindData>();
    auto &g = data.global_state->Cast<ReadGlobalState>();
    auto &l = data.local_state->Cast<ReadLocalState>();
    ReadProfile *prof = g.prof.get();
    PhaseTimer total(prof, ReadProfile::kScanTotal);
    for (;;) {  // until a chunk with rows (host-side filters can empty one) or the end
        output.Reset();
        // (a filtered row group can deliver no rows)
        while (!(l.pin && l.rg_pos < l.rg.nrows)) {
            if (!NextRowGroup(bind, g, l)) {
                output.SetCardinality(0);
                return;
            }
            // FSST columns delivered as lengths: their string_t records, on
            // this thread after NextRowGroup's lock (fls_scan_defer_records)
            PhaseTimer t(prof, ReadProfile::kRecords);
            if (fls_scan_build_records(l.table, &l.rg) != 0)
                throw IOException(string("FastLanes scan failed: ") + fls_last_error());
        }
        const idx_t n = std::min<idx_t>(STANDARD_VECTOR_SIZE, l.rg.nrows - l.rg_pos);
        for (idx_t j = 0; j < output.ColumnCount(); ++j) {
            const column_t id = j < g.out_ids.size() ? g.column_ids[g.out_ids[j]] : j;
            Vector &vec = output.data[j];
            if (id == COLUMN_IDENTIFIER_ROW_ID) {
                int64_t *rid = FlatVector::GetData<int64_t>(vec);
                for (idx_t i = 0; i < n; ++i)
                    rid[i] = (int64_t)(l.rg.first_row + (l.rg.sel ? l.rg.sel[l.rg_pos + i] : l.rg_pos + i));
                continue;
            }
            EmitColumn(bind, l, id, vec, n, prof);
        }
        idx_t approved = n;
        if (!g.residual.empty()) {
            PhaseTimer t(prof, ReadProfile::kResidual);
            // DuckDB's FilterSelection reads the incoming selection before it
            // writes one (SelectionVector(n) leaves the buffer uninitialised):
            // start from the identity over the chunk's rows
            SelectionVector sel(n);
            for (idx_t i = 0; i < n; ++i) sel.set_index(i, i);
            for (size_t k = 0; k < g.residual.size() && approved > 0; ++k) {
                const auto &r = g.residual[k];
                Vector col(bind.types[r.id]);
                EmitColumn(bind, l, r.id, col, n);
                UnifiedVectorFormat vdata;
                col.ToUnifiedFormat(n, vdata);
                ColumnSegment::FilterSelection(sel, col, vdata, *r.filter, *l.residual_state[k], n, approved);
            }
            if (approved < n) output.Slice(sel, approved);
        }
        l.rg_pos += n;
        if (prof) {
            prof->chunks++;
            prof->rows += approved;
        }
        output.SetCardinality(approved);
        if (approved > 0) return;
    }
}

OperatorPartitionData ReadPartitionData(ClientContext &, TableFunctionGetPartitionInput &input) {
    return OperatorPartitionData(input.local_state->Cast<ReadLocalState>().batch_index);
}

unique_ptr<TableRef> ReadFastlanesReplacementScan(ClientContext &, ReplacementScanInput &input,
                                                  optional_ptr<ReplacementScanData>) {
    const string path = ReplacementScan::GetFullPath(input);
    const string lower = StringUtil::Lower(path);
    if (!StringUtil::EndsWith(lower, ".fls") && !StringUtil::EndsWith(lower, ".fastlane")) return nullptr;
    auto ref = make_uniq<TableFunctionRef>();
    vector<unique_ptr<ParsedExpression>> args;
    args.push_back(make_uniq<ConstantExpression>(Value(path)));
    ref->function = make_uniq<FunctionExpression>("read_fastlanes", std::move(args));
    return std::move(ref);
}

}  // namespace

TableFunction ReadFastlanesFunction() {
    TableFunction fn("read_fastlanes", {LogicalType::VARCHAR}, ReadScan, ReadBind, ReadInitGlobal, ReadInitLocal);
    fn.get_partition_data = ReadPartitionData;
    fn.projection_pushdown = true;
    fn.filter_pushdown = true;
    fn.filter_prune = true;
    // accepted like the intended scanner's (src/scanner/scan_fastlanes.cpp:156),
    // which never reads it either: the schema always comes from the footer
    fn.named_parameters["auto_detect"] = LogicalType::BOOLEAN;
    return fn;
}

void RegisterReadFastlanes(DatabaseInstance &db) {
    TableFunction fn = ReadFastlanesFunction();
    ExtensionUtil::RegisterFunction(db, fn);
    fn.arguments = {LogicalType::LIST(LogicalType::VARCHAR)};
    ExtensionUtil::RegisterFunction(db, fn);
    DBConfig::GetConfig(db).replacement_scans.emplace_back(ReadFastlanesReplacementScan);
}

}  // namespace ext_fastlane
}  // namespace duckdb
