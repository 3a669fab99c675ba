// scan_fastlanes.cpp -- `scan_fastlanes(path)`: the table function the
// reference actually compiles (src/scan_fastlanes.cpp:24-84), kept
// behaviour-identical on top of the GPU facade:
//   * exactly one VARCHAR argument, else BinderException with the reference's
//     texts (:29-35); named parameter `file` accepted (:81);
//   * Bind opens the file to validate it and fails with
//     "Failed to open FastLanes file: <path>" (:40-43);
//   * schema is a single VARCHAR column named `data` (:46-47);
//   * InitGlobal re-opens (IOException with the same text on failure, :57-59);
//   * Scan streams FastLanesFacade::readNextChunk until it returns false
//     (:65-77): column 0 of row group 0, rendered as VARCHAR.
// The typed, all-row-group GPU scan is `read_fastlanes` (read_fastlanes.cpp).
#include "scan_fastlanes.hpp"

#include "duckdb/common/types/data_chunk.hpp"
#include "duckdb/main/extension_util.hpp"
#include "fastlanes_facade.hpp"

namespace duckdb {

namespace {

struct FastLanesBindData : public TableFunctionData {
    std::string file_path;
};

struct FastLanesScanState : public GlobalTableFunctionState {
    std::unique_ptr<FastLanesFacade> facade;
    bool initialized = false;
};

unique_ptr<FunctionData> FastLanesBind(ClientContext &, TableFunctionBindInput &input,
                                       vector<LogicalType> &return_types, vector<string> &return_names) {
    if (input.inputs.size() != 1) {
        throw BinderException("scan_fastlanes requires exactly one argument (file path)");
    }
    const Value &arg = input.inputs[0];
    if (arg.type() != LogicalType::VARCHAR) {
        throw BinderException("scan_fastlanes file path must be a string");
    }
    auto bind = make_uniq<FastLanesBindData>();
    bind->file_path = arg.GetValue<string>();
    {
        FastLanesFacade probe;  // validate now, like the reference's Bind
        if (!probe.openFile(bind->file_path)) {
            throw BinderException("Failed to open FastLanes file: " + bind->file_path);
        }
    }
    return_types.assign(1, LogicalType::VARCHAR);
    return_names.assign(1, "data");
    return std::move(bind);
}

unique_ptr<GlobalTableFunctionState> FastLanesInitGlobal(ClientContext &, TableFunctionInitInput &input) {
    const auto &bind = input.bind_data->Cast<FastLanesBindData>();
    auto state = make_uniq<FastLanesScanState>();
    state->facade = std::make_unique<FastLanesFacade>();
    if (!state->facade->openFile(bind.file_path)) {
        throw IOException("Failed to open FastLanes file: " + bind.file_path);
    }
    state->initialized = true;
    return std::move(state);
}

void FastLanesScan(ClientContext &, TableFunctionInput &data, DataChunk &output) {
    auto &state = data.global_state->Cast<FastLanesScanState>();
    if (!state.initialized || !state.facade || !state.facade->readNextChunk(output)) {
        output.SetCardinality(0);
    }
}

}  // namespace

void ScanFastLanes::Register(DatabaseInstance &db) {
    TableFunction fn("scan_fastlanes", {LogicalType::VARCHAR}, FastLanesScan, FastLanesBind, FastLanesInitGlobal);
    fn.named_parameters["file"] = LogicalType::VARCHAR;
    ExtensionUtil::RegisterFunction(db, fn);
}

}  // namespace duckdb
