// type_mapping.cpp -- see include/type_mapping.hpp.
#include "type_mapping.hpp"

#include "../../../include/flswriter.h"

namespace duckdb {
namespace ext_fastlane {

LogicalType TypeMapping::FastLanesToDuckDB(uint8_t t, uint8_t width, uint8_t scale) {
    switch (t) {
    case FLS_INT8: return LogicalType::TINYINT;
    case FLS_INT16: return LogicalType::SMALLINT;
    case FLS_INT32: return LogicalType::INTEGER;
    case FLS_INT64: return LogicalType::BIGINT;
    case FLS_UINT8: return LogicalType::UTINYINT;
    case FLS_UINT16: return LogicalType::USMALLINT;
    case FLS_UINT32: return LogicalType::UINTEGER;
    case FLS_UINT64: return LogicalType::UBIGINT;
    case FLS_BOOLEAN: return LogicalType::BOOLEAN;
    case FLS_DATE: return LogicalType::DATE;
    case FLS_DECIMAL: return LogicalType::DECIMAL(width ? width : 18, scale);
    case FLS_FLOAT: return LogicalType::FLOAT;
    case FLS_DOUBLE: return LogicalType::DOUBLE;
    case FLS_VARCHAR: return LogicalType::VARCHAR;
    case FLS_BLOB: return LogicalType::BLOB;
    default: return LogicalType::SQLNULL;
    }
}

uint8_t TypeMapping::DuckDBToFastLanes(const LogicalType &type) {
    switch (type.id()) {
    case LogicalTypeId::TINYINT: return FLS_INT8;
    case LogicalTypeId::SMALLINT: return FLS_INT16;
    case LogicalTypeId::INTEGER: return FLS_INT32;
    case LogicalTypeId::BIGINT: return FLS_INT64;
    case LogicalTypeId::UTINYINT: return FLS_UINT8;
    case LogicalTypeId::USMALLINT: return FLS_UINT16;
    case LogicalTypeId::UINTEGER: return FLS_UINT32;
    case LogicalTypeId::UBIGINT: return FLS_UINT64;
    case LogicalTypeId::BOOLEAN: return FLS_BOOLEAN;  // reference type_mapping.cpp:13-14
    case LogicalTypeId::DATE: return FLS_DATE;
    // DECIMAL(w<=18) is stored as its int64 physical value; narrower physical
    // widths are widened by the writer glue
    case LogicalTypeId::DECIMAL: return type.Width() <= 18 ? FLS_DECIMAL : 0;
    case LogicalTypeId::VARCHAR:
    case LogicalTypeId::CHAR: return FLS_VARCHAR;  // read back as VARCHAR, as the reference (:35-36, :89-90)
    case LogicalTypeId::BLOB:                      // BYTE_ARRAY (:40-42, :93-94)
    case LogicalTypeId::BIT: return FLS_BLOB;      // the bitstring's bytes; read back as BLOB, as the reference (:41-42)
    case LogicalTypeId::FLOAT: return FLS_FLOAT;    // ALP
    case LogicalTypeId::DOUBLE: return FLS_DOUBLE;  // ALP
    default: return 0;
    }
}

idx_t TypeMapping::GetFastLanesTypeSize(uint8_t t) {
    switch (t) {
    case FLS_INT8: case FLS_UINT8: case FLS_BOOLEAN: return 1;
    case FLS_INT16: case FLS_UINT16: return 2;
    case FLS_INT32: case FLS_UINT32: case FLS_DATE: case FLS_FLOAT: return 4;
    case FLS_INT64: case FLS_UINT64: case FLS_DECIMAL: case FLS_DOUBLE: return 8;
    case FLS_VARCHAR: case FLS_BLOB: return 16;
    default: return 0;
    }
}

}  // namespace ext_fastlane
}  // namespace duckdb
