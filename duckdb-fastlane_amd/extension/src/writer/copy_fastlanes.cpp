// copy_fastlanes.cpp -- the FastLanes COPY TO function.
//
// Option handling follows the reference's intended writer
// (src/writer/write_fastlane_stream.cpp:65-107): ROW_GROUP_SIZE / CHUNK_SIZE
// (default 65,536, :21-24), ROW_GROUP_SIZE_BYTES (rows = bytes / 1024 bytes per
// row, :27), the same error texts.  Rows go through
// ext_fastlane::FastLanesFacade::createFile/writeChunk/finalizeFile into the CPU
// FastLanes writer (per-chunk encoding choice: FFOR / DELTA / DICT / RLE).
// ROW_GROUPS_PER_FILE rotates files as the reference registers it (:96-97,
// :267-289, rotate_files / rotate_next_file): DuckDB then writes a directory of
// files and asks, before every sink, whether the current file holds its row
// groups.
#include "writer/copy_fastlanes.hpp"

#include <atomic>
#include <mutex>

#include "duckdb/common/optional_idx.hpp"
#include "duckdb/common/string_util.hpp"
#include "duckdb/main/extension_util.hpp"
#include "fastlanes_facade.hpp"
#include "table_function/read_fastlanes.hpp"

namespace duckdb {
namespace ext_fastlane {

namespace {

struct FastlaneCopyBindData : public TableFunctionData {
    vector<LogicalType> sql_types;
    vector<string> column_names;
    idx_t row_group_size = 65536;
    optional_idx row_groups_per_file;
    static constexpr idx_t BYTES_PER_ROW = 1024;
};

struct FastlaneCopyGlobalState : public GlobalFunctionData {
    std::unique_ptr<FastLanesFacade> facade;
    string file_path;
    // rotation: rows sunk into this file (current_rowgroup = rows / row group
    // size), through the facade's serial path so that the file holds exactly
    // the rows sunk into it when DuckDB finalizes it
    std::atomic<idx_t> rows{0};
    std::mutex serial;
};

// Each sink thread copies its chunks into its own facade stage (created at the
// first sink: init_local does not see the global state); full batches of row
// groups go to the writer from the stage, the rest is merged at combine.
struct FastlaneCopyLocalState : public LocalFunctionData {
    FastLanesFacade::StagePtr stage;
};

idx_t ValidRowGroupSize(uint64_t rows) {
    if (rows == 0 || rows > 65536 || rows % 1024)
        throw BinderException("ROW_GROUP_SIZE must be a multiple of 1024 between 1024 and 65536 (FastLanes vectors)");
    return rows;
}

unique_ptr<FunctionData> CopyBind(ClientContext &, CopyFunctionBindInput &input, const vector<string> &names,
                                  const vector<LogicalType> &sql_types) {
    auto bind = make_uniq<FastlaneCopyBindData>();
    bool size_set = false;
    for (auto &opt : input.info.options) {
        const string name = StringUtil::Lower(opt.first);
        if (opt.second.size() != 1) throw BinderException(StringUtil::Upper(name) + " requires exactly one argument");
        const Value &v = opt.second[0];
        if (name == "row_group_size" || name == "chunk_size" || name == "row_group_size_bytes") {
            if (size_set) throw BinderException("ROW_GROUP_SIZE and ROW_GROUP_SIZE_BYTES are mutually exclusive");
            size_set = true;
            const uint64_t x = (uint64_t)std::stoull(v.ToString());
            bind->row_group_size = name == "row_group_size_bytes"
                                       ? ValidRowGroupSize(std::max<uint64_t>(1024, x / FastlaneCopyBindData::BYTES_PER_ROW / 1024 * 1024))
                                       : ValidRowGroupSize(x);
        } else if (name == "row_groups_per_file") {
            const uint64_t x = (uint64_t)std::stoull(v.ToString());
            if (x == 0) throw BinderException("ROW_GROUPS_PER_FILE must be at least 1");
            bind->row_groups_per_file = x;
        } else {
            throw BinderException("Unknown option for FastLanes: " + StringUtil::Upper(name));
        }
    }
    bind->sql_types = sql_types;
    bind->column_names = names;
    return std::move(bind);
}

unique_ptr<GlobalFunctionData> CopyInitGlobal(ClientContext &, FunctionData &bind_p, const string &path) {
    auto &bind = bind_p.Cast<FastlaneCopyBindData>();
    auto state = make_uniq<FastlaneCopyGlobalState>();
    state->facade = std::make_unique<FastLanesFacade>();
    if (!state->facade->createFile(path, bind.sql_types, bind.column_names) ||
        !state->facade->setRowGroupSize(bind.row_group_size)) {
        throw IOException("Failed to create FastLanes file: " + path);
    }
    state->file_path = path;
    return std::move(state);
}

unique_ptr<LocalFunctionData> CopyInitLocal(ExecutionContext &, FunctionData &) {
    return make_uniq<FastlaneCopyLocalState>();
}

void CopySink(ExecutionContext &, FunctionData &bind_p, GlobalFunctionData &gstate, LocalFunctionData &lstate,
              DataChunk &input) {
    auto &g = gstate.Cast<FastlaneCopyGlobalState>();
    auto &l = lstate.Cast<FastlaneCopyLocalState>();
    if (bind_p.Cast<FastlaneCopyBindData>().row_groups_per_file.IsValid()) {
        // rotating: no per-thread stage may carry rows past this file's finalize
        std::lock_guard<std::mutex> guard(g.serial);
        if (!g.facade->writeChunk(input)) {
            const std::string &why = g.facade->lastError();
            throw IOException("Failed to write chunk to FastLanes" + (why.empty() ? std::string() : ": " + why));
        }
        g.rows += input.size();
        return;
    }
    if (!l.stage) l.stage = g.facade->newStage();
    if (!g.facade->writeChunk(*l.stage, input)) {
        const std::string &why = g.facade->stageError(*l.stage);
        throw IOException("Failed to write chunk to FastLanes" + (why.empty() ? std::string() : ": " + why));
    }
}

void CopyCombine(ExecutionContext &, FunctionData &, GlobalFunctionData &gstate, LocalFunctionData &lstate) {
    auto &g = gstate.Cast<FastlaneCopyGlobalState>();
    auto &l = lstate.Cast<FastlaneCopyLocalState>();
    if (l.stage && !g.facade->mergeStage(*l.stage)) {
        const std::string &why = g.facade->stageError(*l.stage);
        throw IOException("Failed to write chunk to FastLanes" + (why.empty() ? std::string() : ": " + why));
    }
}

// The reference's mode callback (src/writer/write_fastlane_stream.cpp:251-260)
// answers PARALLEL without insertion order and BATCH for a batch-index source,
// but registers no prepare_batch / flush_batch, which DuckDB's batch copy
// calls; here an ordered COPY keeps the single (REGULAR) sink, and an
// unordered one runs sinks on every thread, each into its own stage (only the
// hand-off of full batches to the writer is serialised).
CopyFunctionExecutionMode CopyExecutionMode(bool preserve_insertion_order, bool /*supports_batch_index*/) {
    return preserve_insertion_order ? CopyFunctionExecutionMode::REGULAR_COPY_TO_FILE
                                    : CopyFunctionExecutionMode::PARALLEL_COPY_TO_FILE;
}

// The reference's rotation callbacks (write_fastlane_stream.cpp:267-289): a
// directory of files when ROW_GROUPS_PER_FILE is set (FILE_SIZE_BYTES too,
// which the reference never rotates on: DuckDB's own size check is absent
// for it, and so here), the next file once this one holds that many row
// groups
bool CopyRotateFiles(FunctionData &bind_p, const optional_idx &file_size_bytes) {
    return file_size_bytes.IsValid() || bind_p.Cast<FastlaneCopyBindData>().row_groups_per_file.IsValid();
}

bool CopyRotateNextFile(GlobalFunctionData &gstate, FunctionData &bind_p, const optional_idx &) {
    auto &bind = bind_p.Cast<FastlaneCopyBindData>();
    if (!bind.row_groups_per_file.IsValid()) return false;
    const idx_t current_rowgroup = gstate.Cast<FastlaneCopyGlobalState>().rows.load() / bind.row_group_size;
    return current_rowgroup >= bind.row_groups_per_file.GetIndex();
}

// Rows per batch: one row group (write_fastlane_stream.cpp:262-265)
idx_t CopyDesiredBatchSize(ClientContext &, FunctionData &bind_p) {
    return bind_p.Cast<FastlaneCopyBindData>().row_group_size;
}

void CopyFinalize(ClientContext &, FunctionData &bind_p, GlobalFunctionData &gstate) {
    auto &g = gstate.Cast<FastlaneCopyGlobalState>();
    // rotating: DuckDB asks rotate_next_file before the combine calls too, so
    // the last rotation can open a file nothing is sunk into; it is not written
    if (bind_p.Cast<FastlaneCopyBindData>().row_groups_per_file.IsValid() && g.rows.load() == 0) return;
    g.facade->finalizeFile();
    if (!g.facade->finalizeOk()) {
        const std::string &why = g.facade->lastError();
        throw IOException("Failed to finalize FastLanes file: " + g.file_path + (why.empty() ? std::string() : ": " + why));
    }
}

}  // namespace

void RegisterFastlaneCopyFunction(DatabaseInstance &db) {
    CopyFunction fn("fls");
    fn.copy_to_bind = CopyBind;
    fn.copy_to_initialize_global = CopyInitGlobal;
    fn.copy_to_initialize_local = CopyInitLocal;
    fn.copy_to_sink = CopySink;
    fn.copy_to_combine = CopyCombine;
    fn.copy_to_finalize = CopyFinalize;
    fn.execution_mode = CopyExecutionMode;
    fn.desired_batch_size = CopyDesiredBatchSize;
    fn.rotate_files = CopyRotateFiles;
    fn.rotate_next_file = CopyRotateNextFile;
    fn.copy_from_function = ReadFastlanesFunction;
    fn.extension = "fls";
    ExtensionUtil::RegisterFunction(db, fn);
    fn.name = "fastlane";
    fn.extension = "fastlane";
    ExtensionUtil::RegisterFunction(db, fn);
}

}  // namespace ext_fastlane
}  // namespace duckdb
