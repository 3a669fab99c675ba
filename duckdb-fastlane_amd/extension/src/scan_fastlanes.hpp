//===----------------------------------------------------------------------===//
//                         DuckDB - fastlane (MI355X)
//
// scan_fastlanes.hpp -- registration of the compiled `scan_fastlanes`
// table function (reference src/scan_fastlanes.hpp:7-10).
//===----------------------------------------------------------------------===//
#pragma once

#include "duckdb/function/table_function.hpp"

namespace duckdb {

class ScanFastLanes {
public:
    static void Register(DatabaseInstance &db);
};

}  // namespace duckdb
