//===----------------------------------------------------------------------===//
//                         DuckDB - fastlane (MI355X)
//
// fastlane_extension.hpp -- extension class (reference
// src/include/fastlane_extension.hpp:7-12), unchanged.
//===----------------------------------------------------------------------===//
#pragma once

#include "duckdb.hpp"

namespace duckdb {

class FastlaneExtension : public Extension {
public:
    void Load(DuckDB &db) override;
    std::string Name() override;
    std::string Version() const override;
};

}  // namespace duckdb
