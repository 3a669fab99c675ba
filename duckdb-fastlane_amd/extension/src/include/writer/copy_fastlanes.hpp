//===----------------------------------------------------------------------===//
//                         DuckDB - fastlane (MI355X)
//
// writer/copy_fastlanes.hpp -- COPY ... TO 'x.fls' (FORMAT fls | fastlane).
// Counterpart of the reference's uncompiled copy function
// (src/include/write_fastlane_stream.hpp, src/writer/write_fastlane_stream.cpp:294-314).
//===----------------------------------------------------------------------===//
#pragma once

#include "duckdb/function/copy_function.hpp"

namespace duckdb {
namespace ext_fastlane {

void RegisterFastlaneCopyFunction(DatabaseInstance &db);

}  // namespace ext_fastlane
}  // namespace duckdb
