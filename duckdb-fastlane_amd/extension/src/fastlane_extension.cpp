// fastlane_extension.cpp -- extension entry points (reference
// src/fastlane_extension.cpp:94-124): the same two C symbols and class.
// Load registers the reference's compiled `scan_fastlanes` plus what the
// reference wrote but never registered (:44-90): the typed GPU scan (here
// `read_fastlanes`, VARCHAR and LIST(VARCHAR)), the .fls/.fastlane replacement
// scan, and the COPY TO (FORMAT fls | fastlane) writer.
#define DUCKDB_EXTENSION_MAIN

#include "fastlane_extension.hpp"

#include "duckdb.hpp"
#include "scan_fastlanes.hpp"
#include "table_function/read_fastlanes.hpp"
#include "writer/copy_fastlanes.hpp"

namespace duckdb {

void FastlaneExtension::Load(DuckDB &db) {
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
