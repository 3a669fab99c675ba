// tsan_copy.cpp -- ThreadSanitizer driver for the parallel COPY sink (host only, no GPU):
// builds the extension sources with -fsanitize=thread and runs a 1- and 4-thread
// COPY of 41,037 literal rows (row groups of 1024, batches queued to the writer).
//   cd duckdb-fastlane_amd && g++ -O1 -g -std=c++20 -fsanitize=thread -Iextension/duckdb_shim \
//     -Iextension/src/include -Iextension/src extension/src/*.cpp extension/src/scanner/*.cpp \
//     extension/src/writer/*.cpp extension/duckdb_shim/duckdb_shim.cpp extension/harness/fls_ext_harness.cpp \
//     ../scripts/tsan_copy.cpp -L. -lflsgpu -Wl,-rpath,$PWD -o /tmp/copy_tsan && /tmp/copy_tsan
// Result (round 2): no ThreadSanitizer reports, both COPYs rc 0 (profiles/r2/tsan_copy_r2.txt).
#include <cstdio>
#include <string>
#include <vector>
#include <cstdint>
extern "C" {
struct fls_ext_db;
fls_ext_db *fls_ext_open(void);
void fls_ext_close(fls_ext_db *);
const char *fls_ext_last_error(void);
int fls_ext_copy_values_mt(fls_ext_db *d, const char *format, const char *dst, int ncols, const char *const *names,
                           const char *const *type_names, int64_t nrows, const char *const *cells,
                           const char *const *opt_keys, const char *const *opt_vals, int nopts, int nthreads,
                           uint64_t *rows);
}
int main() {
    fls_ext_db *d = fls_ext_open();
    const int64_t n = 40 * 1024 + 77;
    std::vector<std::string> store(2 * n);
    std::vector<const char *> cells(2 * n);
    for (int64_t i = 0; i < n; ++i) {
        store[2 * i] = std::to_string(i * 7);
        store[2 * i + 1] = std::string((size_t)(i % 19), 'a' + (char)(i % 26));
        cells[2 * i] = store[2 * i].c_str();
        cells[2 * i + 1] = store[2 * i + 1].c_str();
    }
    const char *names[2] = {"a", "s"}, *types[2] = {"BIGINT", "VARCHAR"};
    const char *k[1] = {"row_group_size"}, *v[1] = {"1024"};
    for (int th : {1, 4}) {
        uint64_t rows = 0;
        int rc = fls_ext_copy_values_mt(d, "fls", "/tmp/tsan_copy_out.fls", 2, names, types, n, cells.data(), k, v, 1, th, &rows);
        printf("threads %d rc %d rows %llu %s\n", th, rc, (unsigned long long)rows, rc ? fls_ext_last_error() : "");
    }
    fls_ext_close(d);
}
