//===----------------------------------------------------------------------===//
//                         DuckDB - fastlane (MI355X)
//
// fastlanes_facade.hpp -- the PIMPL seam of the compiled extension
// (reference src/fastlanes_facade.hpp:17-30), unchanged for its callers.
// Behind it the cwida/FastLanes library is replaced by the MI355X engine's
// C-ABI (include/flsgpu.h): no FastLanes or HIP type leaks into this header.
//===----------------------------------------------------------------------===//
#pragma once

#include <memory>
#include <string>

#include "duckdb/common/types.hpp"
#include "duckdb/common/types/data_chunk.hpp"

namespace duckdb {

class FastLanesFacade {
public:
    FastLanesFacade();
    ~FastLanesFacade();

    // Open `filename` and decode its first row group on the GPU.  false on any
    // error (never throws), like the reference.
    bool openFile(const std::string &filename);
    // Emit the next <= STANDARD_VECTOR_SIZE rows as VARCHAR; false at the end.
    bool readNextChunk(DataChunk &result);
    void closeFile();

private:
    struct Impl;
    std::unique_ptr<Impl> pImpl;
};

}  // namespace duckdb
