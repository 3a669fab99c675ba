// fastlane_extension.cpp -- extension entry points (reference
// src/fastlane_extension.cpp:94-124): the same two C symbols and class.
// Load registers the reference's compiled `scan_fastlanes` plus what the
// reference wrote but never registered (:44-90): the SQL scalar
// `fastlane_version()` (:32-42, used at examples/basic_usage.sql:8), the typed
// GPU scan (here `read_fastlanes`, VARCHAR and LIST(VARCHAR)), the
// .fls/.fastlane replacement scan, and the COPY TO (FORMAT fls | fastlane)
// writer.
#define DUCKDB_EXTENSION_MAIN

#include "fastlane_extension.hpp"

#include "duckdb.hpp"
#include "gpu_devices.hpp"
#include "scan_fastlanes.hpp"
#include "table_function/read_fastlanes.hpp"
#include "writer/copy_fastlanes.hpp"

namespace duckdb {

namespace {
// SELECT fastlane_version(): the reference's constant text
// (src/fastlane_extension.cpp:38-41), one constant VARCHAR
void FastlaneVersionFn(DataChunk &, ExpressionState &, Vector &result) {
    result.SetValue(0, StringVector::AddString(result, "FastLanes Extension v1.0.0"));
    result.SetVectorType(VectorType::CONSTANT_VECTOR);
}
// SELECT fastlane_release_memory(): not in the reference.  Hands the pinned
// host memory the GPU scan keeps between queries back to the OS and frees the
// HBM-resident file images no running scan uses; returns the bytes of both
// still held (0 when no scan runs).
void FastlaneReleaseMemoryFn(DataChunk &, ExpressionState &, Vector &result) {
    const uint64_t left = ext_fastlane::ReleaseMemory();
    result.SetValue(0, Value::BIGINT((int64_t)left));
    result.SetVectorType(VectorType::CONSTANT_VECTOR);
}
}  // namespace

void FastlaneExtension::Load(DuckDB &db) {
    ExtensionUtil::RegisterFunction(*db.instance,
                                    ScalarFunction("fastlane_version", {}, LogicalType::VARCHAR, FastlaneVersionFn));
    ExtensionUtil::RegisterFunction(
        *db.instance, ScalarFunction("fastlane_release_memory", {}, LogicalType::BIGINT, FastlaneReleaseMemoryFn));
    ScanFastLanes::Register(*db.instance);
    ext_fastlane::RegisterReadFastlanes(*db.instance);
    ext_fastlane::RegisterFastlaneCopyFunction(*db.instance);
}

std::string FastlaneExtension::Name() { return "fastlane"; }

std::string FastlaneExtension::Version() const {
#ifdef EXT_VERSION_FASTLANE
    return EXT_VERSION_FASTLANE;
#else
    return "";
#endif
}

}  // namespace duckdb

extern "C" {

DUCKDB_EXTENSION_API void fastlane_init(duckdb::DatabaseInstance &db) {
    duckdb::DuckDB wrapper(db);
    duckdb::FastlaneExtension ext;
    ext.Load(wrapper);
}

DUCKDB_EXTENSION_API const char *fastlane_version() { return duckdb::DuckDB::LibraryVersion(); }
}
