// DuckDB v1.3.2 include path served by the API shim (see duckdb_shim_core.hpp)
#pragma once
#include "duckdb_shim_core.hpp"
