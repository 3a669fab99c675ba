//===----------------------------------------------------------------------===//
//                         DuckDB - fastlane (MI355X)
//
// table_function/read_fastlanes.hpp -- the typed, all-row-group, multi-file
// GPU scan.  Modelled on the reference's intended (uncompiled) scanner
// (src/include/table_function/scan_fastlanes.hpp:17-19,
// src/scanner/scan_fastlanes.cpp:151-185) under the north-star name
// `read_fastlanes`, with projection pushdown honoured (the reference sets
// projection_pushdown=true but ignores column_ids, :136,153).
//===----------------------------------------------------------------------===//
#pragma once

#include "duckdb/function/table_function.hpp"

namespace duckdb {
namespace ext_fastlane {

TableFunction ReadFastlanesFunction();
void RegisterReadFastlanes(DatabaseInstance &db);

}  // namespace ext_fastlane
}  // namespace duckdb
