//===----------------------------------------------------------------------===//
//                         DuckDB - fastlane (MI355X)
//
// type_mapping.hpp -- FastLanes column types <-> DuckDB LogicalType.
// Counterpart of the reference's (uncompiled) src/include/type_mapping.hpp /
// src/type_mapping.cpp:64-142, expressed over the engine's fls_type ids
// (include/flswriter.h) instead of FastLanes' data_t.
//===----------------------------------------------------------------------===//
#pragma once

#include <cstdint>

#include "duckdb/common/types.hpp"

namespace duckdb {
namespace ext_fastlane {

struct TypeMapping {
    // fls_type (+ decimal width/scale) -> DuckDB logical type
    static LogicalType FastLanesToDuckDB(uint8_t fls_type, uint8_t width, uint8_t scale);
    // DuckDB logical type -> fls_type; returns 0 when the type has no FastLanes
    // encoding on this path
    static uint8_t DuckDBToFastLanes(const LogicalType &type);
    // bytes of one decoded value as delivered by the engine (string_t = 16)
    static idx_t GetFastLanesTypeSize(uint8_t fls_type);
    static bool IsSupported(const LogicalType &type) { return DuckDBToFastLanes(type) != 0; }
    // a column written as byte strings (VARCHAR, CHAR, BLOB: 16-byte string_t)
    static bool IsString(const LogicalType &type) {
        const uint8_t t = DuckDBToFastLanes(type);
        return t == 20 || t == 21;  // FLS_VARCHAR, FLS_BLOB
    }
};

}  // namespace ext_fastlane
}  // namespace duckdb
