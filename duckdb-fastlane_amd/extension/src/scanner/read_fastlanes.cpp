// read_fastlanes.cpp -- `read_fastlanes(path | [paths])` over the MI355X engine.
//
// Bind reads only footers (no GPU): typed schema via TypeMapping.  InitGlobal
// turns DuckDB's projected column_ids into the engine's column mask, so only
// projected columns are uploaded, decoded and copied back.  Scan is parallel
// (the reference pins MaxThreads to 1, src/scanner/scan_fastlanes.cpp:43-45):
// each DuckDB thread claims whole row groups from fls_scan_acquire
// (GPU-sharded, decoded ahead into pinned host memory), fills
// STANDARD_VECTOR_SIZE-row DataChunks by memcpy of DuckDB's physical layouts
// and hands the row group back with fls_scan_release.  The batch index is the
// row group's position over all files, so DuckDB restores file order.
// string_t records point into the file image, kept alive by every thread that
// holds one of its row groups.  Error texts follow
// src/scanner/scan_fastlanes.cpp:62-97.
#include <glob.h>

#include <algorithm>
#include <cstring>
#include <mutex>

#include "../../../../include/flsgpu.h"
#include "../gpu_devices.hpp"
#include "duckdb/common/exception.hpp"
#include "duckdb/common/string_util.hpp"
#include "duckdb/main/extension_util.hpp"
#include "duckdb/parser/expression/constant_expression.hpp"
#include "duckdb/parser/expression/function_expression.hpp"
#include "duckdb/parser/tableref/table_function_ref.hpp"
#include "table_function/read_fastlanes.hpp"
#include "type_mapping.hpp"

namespace duckdb {
namespace ext_fastlane {

namespace {

struct OpenTable {
    fls_connection *conn = nullptr;
    fls_table *table = nullptr;
    ~OpenTable() {
        if (table) fls_table_close(table);
        if (conn) fls_disconnect(conn);
    }
    bool open(const std::string &path) {
        std::vector<int> devs = GpuDevices();
        return fls_connect(devs.data(), (int)devs.size(), &conn) == 0 &&
               fls_read_fls(conn, path.c_str(), &table) == 0;
    }
};

struct ReadBindData : public TableFunctionData {
    vector<string> files;
    vector<LogicalType> types;
    vector<string> names;
    vector<fls_column_info> cols;
};

struct ReadGlobalState : public GlobalTableFunctionState {
    vector<column_t> column_ids;
    std::vector<uint8_t> mask;
    std::vector<idx_t> rg_base;          // batch index of each file's first row group
    idx_t total_rowgroups = 0;
    std::mutex lock;                     // file advance and row-group claims
    idx_t file_idx = 0;
    std::shared_ptr<OpenTable> cur;      // file being scanned (nullptr: open the next)
    idx_t MaxThreads() const override { return std::max<idx_t>(1, total_rowgroups); }
};

struct ReadLocalState : public LocalTableFunctionState {
    std::shared_ptr<OpenTable> table;    // keeps the file (and its string_t targets) alive
    fls_rowgroup rg{};
    bool have_rg = false;
    idx_t rg_pos = 0;
    idx_t batch_index = 0;
    ~ReadLocalState() override {
        if (have_rg) fls_scan_release(table->table, rg.rowgroup);
    }
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
    OpenTable t;
    if (!t.open(bind->files[0])) throw BinderException("Failed to open FastLanes file: " + bind->files[0]);
    const uint32_t n = fls_table_ncols(t.table);
    bind->cols.resize(n);
    for (uint32_t c = 0; c < n; ++c) {
        fls_table_column(t.table, c, &bind->cols[c]);
        bind->types.push_back(TypeMapping::FastLanesToDuckDB(bind->cols[c].type, bind->cols[c].width, bind->cols[c].scale));
        bind->names.emplace_back(bind->cols[c].name);
        bind->cols[c].name = nullptr;  // owned by the closed table
    }
    return_types = bind->types;
    names = bind->names;
    return std::move(bind);
}

unique_ptr<GlobalTableFunctionState> ReadInitGlobal(ClientContext &, TableFunctionInitInput &input) {
    const auto &bind = input.bind_data->Cast<ReadBindData>();
    auto state = make_uniq<ReadGlobalState>();
    state->column_ids = input.column_ids;
    state->mask.assign(bind.cols.size(), 0);
    for (auto id : state->column_ids)
        if (id != COLUMN_IDENTIFIER_ROW_ID && id < bind.cols.size()) state->mask[id] = 1;
    // fail early on unreadable or schema-incompatible files
    for (auto &f : bind.files) {
        OpenTable t;
        if (!t.open(f)) throw IOException("Failed to open FastLanes file: " + f);
        bool same = fls_table_ncols(t.table) == bind.cols.size();
        for (uint32_t c = 0; same && c < bind.cols.size(); ++c) {
            fls_column_info ci;
            fls_table_column(t.table, c, &ci);
            same = ci.type == bind.cols[c].type && ci.width == bind.cols[c].width && ci.scale == bind.cols[c].scale;
        }
        if (!same) throw IOException("FastLanes file " + f + " does not match the schema of " + bind.files[0]);
        state->rg_base.push_back(state->total_rowgroups);
        state->total_rowgroups += fls_table_nrowgroups(t.table);
    }
    return std::move(state);
}

unique_ptr<LocalTableFunctionState> ReadInitLocal(ExecutionContext &, TableFunctionInitInput &,
                                                  GlobalTableFunctionState *) {
    return make_uniq<ReadLocalState>();
}

// give back the local state's row group and claim the next one (in file and
// row-group order over all threads); false at the end of all files
bool NextRowGroup(const ReadBindData &bind, ReadGlobalState &g, ReadLocalState &l) {
    if (l.have_rg) {
        l.have_rg = false;
        if (fls_scan_release(l.table->table, l.rg.rowgroup) != 0)
            throw IOException(string("FastLanes scan failed: ") + fls_last_error());
    }
    l.table.reset();
    std::lock_guard<std::mutex> guard(g.lock);
    while (true) {
        if (!g.cur) {
            if (g.file_idx >= bind.files.size()) return false;
            auto t = std::make_shared<OpenTable>();
            if (!t->open(bind.files[g.file_idx]))
                throw IOException("Failed to open FastLanes file: " + bind.files[g.file_idx]);
            if (fls_scan_begin(t->table, g.mask.data(), 0, fls_table_nrowgroups(t->table)) != 0)
                throw IOException(string("FastLanes scan failed: ") + fls_last_error());
            g.cur = std::move(t);
        }
        const int rc = fls_scan_acquire(g.cur->table, &l.rg);
        if (rc < 0) throw IOException(string("FastLanes scan failed: ") + fls_last_error());
        if (rc == 1) {
            l.table = g.cur;
            l.have_rg = true;
            l.rg_pos = 0;
            l.batch_index = g.rg_base[g.file_idx] + l.rg.rowgroup;
            return true;
        }
        g.cur.reset();  // closed once the last thread holding one of its row groups lets go
        g.file_idx++;
    }
}

void ReadScan(ClientContext &, TableFunctionInput &data, DataChunk &output) {
    const auto &bind = data.bind_data->Cast<ReadBindData>();
    auto &g = data.global_state->Cast<ReadGlobalState>();
    auto &l = data.local_state->Cast<ReadLocalState>();
    output.Reset();
    if (!(l.have_rg && l.rg_pos < l.rg.nrows) && !NextRowGroup(bind, g, l)) {
        output.SetCardinality(0);
        return;
    }
    const idx_t n = std::min<idx_t>(STANDARD_VECTOR_SIZE, l.rg.nrows - l.rg_pos);
    for (idx_t j = 0; j < output.ColumnCount(); ++j) {
        const column_t id = j < g.column_ids.size() ? g.column_ids[j] : j;
        Vector &vec = output.data[j];
        if (id == COLUMN_IDENTIFIER_ROW_ID) {
            int64_t *rid = FlatVector::GetData<int64_t>(vec);
            for (idx_t i = 0; i < n; ++i) rid[i] = (int64_t)(l.rg.first_row + l.rg_pos + i);
            continue;
        }
        const idx_t ob = bind.cols[id].out_bytes;
        memcpy(vec.GetData(), (const uint8_t *)l.rg.columns[id] + l.rg_pos * ob, n * ob);
    }
    l.rg_pos += n;
    output.SetCardinality(n);
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
    fn.filter_pushdown = false;
    fn.filter_prune = false;
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
