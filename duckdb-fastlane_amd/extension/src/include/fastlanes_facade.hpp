//===----------------------------------------------------------------------===//
//                         DuckDB - fastlane (MI355X)
//
// include/fastlanes_facade.hpp -- the richer facade the reference declares but
// never implements (src/include/fastlanes_facade.hpp:23-48): typed schema,
// row-major boxed reads, and the write path.  Same API; implemented in
// scanner/ext_fastlanes_facade.cpp over the MI355X engine (reads) and the CPU
// FastLanes writer (writes).  No FastLanes or HIP type appears here.
//===----------------------------------------------------------------------===//
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "duckdb/common/types.hpp"
#include "duckdb/common/types/data_chunk.hpp"

namespace duckdb {
namespace ext_fastlane {

class FastLanesFacade {
private:
    class Impl;
    std::unique_ptr<Impl> pImpl;

public:
    FastLanesFacade();
    ~FastLanesFacade();

    // Reading: all row groups, all columns, typed
    bool openFile(const std::string &file_path);
    std::vector<LogicalType> getColumnTypes();
    std::vector<std::string> getColumnNames();
    // next <= STANDARD_VECTOR_SIZE rows, row-major: values[row * ncols + col]
    bool readNextChunk(std::vector<Value> &values, idx_t &rows_read);
    void closeFile();

    // Writing: 65,536-row row groups, encodings chosen per chunk
    bool createFile(const std::string &file_path, const std::vector<LogicalType> &types,
                    const std::vector<std::string> &names);
    bool writeChunk(DataChunk &chunk);
    // Not in the reference's header: rows per row group for the COPY option
    // ROW_GROUP_SIZE (multiple of 1024, <= 65536); call after createFile.
    bool setRowGroupSize(idx_t rows);
    // void, as the reference declares it (src/include/fastlanes_facade.hpp:44);
    // whether the file was written: finalizeOk(), why not: lastError().
    void finalizeFile();

    bool isValid() const;
    // Not in the reference's header: why the last writeChunk or finalizeFile
    // failed (empty when no reason was recorded), for COPY's error message.
    const std::string &lastError() const;
    // Not in the reference's header: true iff the last finalizeFile wrote the
    // file.
    bool finalizeOk() const;

    // Not in the reference's header: thread-local staging for COPY sinks.
    // Each sink thread copies its DataChunks into its own Stage; a Stage that
    // holds a full batch of row groups hands it to the writer (the hand-off is
    // serialised, the copies are not).  mergeStage moves a Stage's remaining
    // rows (fewer than one batch) into the facade's own buffers at row-group
    // boundaries, so only the file's last row group can be short.  With one
    // sink thread the file's row order is the input order; with several it is
    // the order batches complete (PARALLEL_COPY_TO_FILE: no order promised).
    class Stage;
    struct StageDeleter {
        void operator()(Stage *st) const;
    };
    using StagePtr = std::unique_ptr<Stage, StageDeleter>;
    StagePtr newStage();
    bool writeChunk(Stage &stage, DataChunk &chunk);
    bool mergeStage(Stage &stage);
    // why the last writeChunk(stage, ...) / mergeStage(stage) returned false
    const std::string &stageError(const Stage &stage) const;
};

}  // namespace ext_fastlane
}  // namespace duckdb
