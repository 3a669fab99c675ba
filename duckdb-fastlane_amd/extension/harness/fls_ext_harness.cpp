// fls_ext_harness.cpp -- a minimal DuckDB-style executor for the extension,
// exported as a C-ABI so tests (and bench_e2e) can drive the glue exactly the
// way DuckDB's binder and pipeline executor call table functions:
//   lookup overload -> bind -> (projection pushdown) -> init_global ->
//   init_local -> function() until an empty chunk.
// It stands in for `duckdb` itself, which is absent from this container (the
// duckdb/ submodule is empty, .gitmodules:1-4).  SQL-level operators the
// reference test uses (COUNT, LIMIT, LIKE, LENGTH) are applied by the tests on
// the returned rows.
#include <sys/stat.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "fastlanes_facade.hpp"  // ext_fastlane::FastLanesFacade (include/fastlanes_facade.hpp)

// Source compatibility with the reference's declaration
// (src/include/fastlanes_facade.hpp:33-44): code that takes these members'
// addresses compiles against this facade unchanged.
static_assert(std::is_same<decltype(&duckdb::ext_fastlane::FastLanesFacade::finalizeFile),
                           void (duckdb::ext_fastlane::FastLanesFacade::*)()>::value,
              "void finalizeFile(), as the reference declares it");
static_assert(std::is_same<decltype(&duckdb::ext_fastlane::FastLanesFacade::openFile),
                           bool (duckdb::ext_fastlane::FastLanesFacade::*)(const std::string &)>::value,
              "bool openFile(const std::string &)");
static_assert(std::is_same<decltype(&duckdb::ext_fastlane::FastLanesFacade::getColumnTypes),
                           std::vector<duckdb::LogicalType> (duckdb::ext_fastlane::FastLanesFacade::*)()>::value,
              "std::vector<LogicalType> getColumnTypes()");
static_assert(std::is_same<decltype(&duckdb::ext_fastlane::FastLanesFacade::getColumnNames),
                           std::vector<std::string> (duckdb::ext_fastlane::FastLanesFacade::*)()>::value,
              "std::vector<std::string> getColumnNames()");
static_assert(std::is_same<decltype(static_cast<bool (duckdb::ext_fastlane::FastLanesFacade::*)(
                                        std::vector<duckdb::Value> &, duckdb::idx_t &)>(
                               &duckdb::ext_fastlane::FastLanesFacade::readNextChunk)),
                           bool (duckdb::ext_fastlane::FastLanesFacade::*)(std::vector<duckdb::Value> &,
                                                                           duckdb::idx_t &)>::value,
              "bool readNextChunk(std::vector<Value> &, idx_t &)");
static_assert(std::is_same<decltype(&duckdb::ext_fastlane::FastLanesFacade::closeFile),
                           void (duckdb::ext_fastlane::FastLanesFacade::*)()>::value,
              "void closeFile()");

#include "duckdb.hpp"

extern "C" void fastlane_init(duckdb::DatabaseInstance &db);

using namespace duckdb;

struct fls_ext_db {
    DatabaseInstance db;
    ClientContext ctx;
};

struct fls_ext_result {
    std::vector<std::string> names, types;
    std::vector<std::vector<std::string>> cells;  // row-major
    std::vector<std::vector<char>> valid;
};

namespace {

thread_local std::string g_err;

struct Query {
    std::string fn;
    vector<Value> args;
    bool raw = false;  // call the bind callback with the arguments as given
};

bool resolve_replacement(fls_ext_db *d, const std::string &table, Query &q) {
    for (auto &rs : d->db.config.replacement_scans) {
        ReplacementScanInput in{table};
        auto ref = rs.function(d->ctx, in, nullptr);
        if (!ref) continue;
        auto &tf = static_cast<TableFunctionRef &>(*ref);
        auto &fe = static_cast<FunctionExpression &>(*tf.function);
        q.fn = fe.function_name;
        for (auto &c : fe.children) q.args.push_back(static_cast<ConstantExpression &>(*c).value);
        return true;
    }
    return false;
}

// DuckDB's overload resolution, reduced to what these functions need: exact
// type match first, then implicit casts of scalar arguments to VARCHAR.
TableFunction *lookup(fls_ext_db *d, Query &q) {
    auto range = d->db.table_functions.equal_range(q.fn);
    if (range.first == range.second) throw BinderException("Table Function with name " + q.fn + " does not exist!");
    if (q.raw) return &range.first->second;
    for (auto it = range.first; it != range.second; ++it) {
        auto &f = it->second;
        if (f.arguments.size() != q.args.size()) continue;
        bool ok = true;
        for (size_t i = 0; i < q.args.size(); ++i) ok &= f.arguments[i] == q.args[i].type();
        if (ok) return &f;
    }
    for (auto it = range.first; it != range.second; ++it) {
        auto &f = it->second;
        if (f.arguments.size() != q.args.size()) continue;
        bool ok = true;
        for (size_t i = 0; i < q.args.size(); ++i)
            ok &= f.arguments[i] == LogicalType::VARCHAR && q.args[i].type().id() != LogicalTypeId::LIST;
        if (!ok) continue;
        for (auto &a : q.args) a = Value(a.ToString());  // implicit cast to VARCHAR
        return &f;
    }
    std::string sig = q.fn + "(";
    for (size_t i = 0; i < q.args.size(); ++i) sig += (i ? ", " : "") + q.args[i].type().ToString();
    throw BinderException("No function matches the given name and argument types '" + sig + ")'");
}

// ---- WHERE clauses handed to the scan as DuckDB TableFilters --------------
// A filter is (table column, expression text) with the expression one of
//   "<op> v"  (op = <> < <= > >=)     -> ConstantFilter
//   "IN v1|v2|..."                     -> InFilter
//   "OR <op> v|<op> v|..."             -> ConjunctionOrFilter of ConstantFilters
//   "ISNULL" / "ISNOTNULL"             -> IsNullFilter / IsNotNullFilter
//   "OPT <expr>"                       -> OptionalFilter(<expr>)
//   "EXPR MOD m r" / "EXPR LIKE s"     -> ExpressionFilter (v % m == r / VARCHAR
//                                         contains s): a filter the engine cannot
//                                         evaluate, applied on the host
// Several filters on one column AND together (TableFilterSet::PushFilter).
// Constants are cast to the column type, as DuckDB's binder does before
// pushing a comparison down: DATE 'YYYY-MM-DD', DECIMAL '12.34', 'nan'.
struct FilterSpec {
    int col;
    std::string expr;
};

int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = (unsigned)(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + (int64_t)doe - 719468;
}

Value parse_constant(const std::string &t, const LogicalType &type) {
    switch (type.id()) {
    case LogicalTypeId::TINYINT: return Value::TINYINT((int8_t)std::stoll(t));
    case LogicalTypeId::SMALLINT: return Value::SMALLINT((int16_t)std::stoll(t));
    case LogicalTypeId::INTEGER: return Value::INTEGER((int32_t)std::stoll(t));
    case LogicalTypeId::BIGINT: return Value::BIGINT(std::stoll(t));
    case LogicalTypeId::UTINYINT: return Value::UTINYINT((uint8_t)std::stoull(t));
    case LogicalTypeId::USMALLINT: return Value::USMALLINT((uint16_t)std::stoull(t));
    case LogicalTypeId::UINTEGER: return Value::UINTEGER((uint32_t)std::stoull(t));
    case LogicalTypeId::UBIGINT: return Value::UBIGINT(std::stoull(t));
    case LogicalTypeId::DATE: {
        int y, m, d;
        if (sscanf(t.c_str(), "%d-%d-%d", &y, &m, &d) == 3) return Value::DATE(date_t{(int32_t)days_from_civil(y, m, d)});
        return Value::DATE(date_t{(int32_t)std::stoll(t)});
    }
    case LogicalTypeId::DECIMAL: {
        // exact decimal text -> scaled integer (rounded half away from zero)
        const bool neg = !t.empty() && t[0] == '-';
        std::string digits = neg ? t.substr(1) : t;
        const size_t dot = digits.find('.');
        std::string ip = dot == std::string::npos ? digits : digits.substr(0, dot);
        std::string fp = dot == std::string::npos ? "" : digits.substr(dot + 1);
        const unsigned sc = type.Scale();
        bool up = fp.size() > sc && fp[sc] >= '5';
        fp.resize(sc, '0');
        int64_t v = std::stoll((ip.empty() ? "0" : ip) + fp) + (up ? 1 : 0);
        return Value::DECIMAL(neg ? -v : v, type.Width(), type.Scale());
    }
    case LogicalTypeId::FLOAT: return Value::FLOAT(std::strtof(t.c_str(), nullptr));
    case LogicalTypeId::DOUBLE: return Value::DOUBLE(std::strtod(t.c_str(), nullptr));
    case LogicalTypeId::VARCHAR: case LogicalTypeId::CHAR: return Value(t);
    case LogicalTypeId::BOOLEAN: return Value::BOOLEAN(t == "true" || t == "1");
    case LogicalTypeId::BIT: {  // '0' / '1' text -> DuckDB's bitstring (Bit::ToBit)
        const size_t n = t.size();
        const unsigned pad = (unsigned)((8 - n % 8) % 8);
        std::string b(1 + (n + pad) / 8, '\0');
        b[0] = (char)pad;
        for (unsigned i = 0; i < pad; ++i) b[1] |= (char)(1u << (7 - i));      // padding bits are set
        for (size_t i = 0; i < n; ++i)
            if (t[i] == '1') b[1 + (pad + i) / 8] |= (char)(1u << (7 - (pad + i) % 8));
        return Value::BIT((const uint8_t *)b.data(), b.size());
    }
    case LogicalTypeId::BLOB: {  // the harness passes BLOB bytes as hex digits
        std::string b;
        for (size_t i = 0; i + 1 < t.size(); i += 2) b += (char)std::stoi(t.substr(i, 2), nullptr, 16);
        return Value::BLOB((const uint8_t *)b.data(), b.size());
    }
    default: throw NotImplementedException("harness: no constant for " + type.ToString());
    }
}

ExpressionType parse_op(const std::string &op) {
    if (op == "=") return ExpressionType::COMPARE_EQUAL;
    if (op == "<>" || op == "!=") return ExpressionType::COMPARE_NOTEQUAL;
    if (op == "<") return ExpressionType::COMPARE_LESSTHAN;
    if (op == "<=") return ExpressionType::COMPARE_LESSTHANOREQUALTO;
    if (op == ">") return ExpressionType::COMPARE_GREATERTHAN;
    if (op == ">=") return ExpressionType::COMPARE_GREATERTHANOREQUALTO;
    throw BinderException("harness: unknown comparison " + op);
}

std::vector<std::string> split(const std::string &s, char sep) {
    std::vector<std::string> out;
    size_t a = 0;
    while (true) {
        const size_t b = s.find(sep, a);
        out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) return out;
        a = b + 1;
    }
}

// the shim's stand-in for a bound expression (DuckDB: `col % m = r`, `col LIKE '%s%'`)
struct ModExpression : public Expression {
    int64_t m, r;
    ModExpression(int64_t m, int64_t r) : m(m), r(r) {}
    bool EvaluateRow(const Value &v) const override { return !v.IsNull() && v.GetInt64() % m == r; }
};
struct ContainsExpression : public Expression {
    std::string sub;
    explicit ContainsExpression(std::string s) : sub(std::move(s)) {}
    bool EvaluateRow(const Value &v) const override {
        return !v.IsNull() && v.GetValue<std::string>().find(sub) != std::string::npos;
    }
};

unique_ptr<TableFilter> parse_filter(const std::string &e, const LogicalType &type) {
    auto head = [&](const char *kw) { return e.rfind(kw, 0) == 0; };
    if (head("EXPR MOD ")) {
        long long m = 0, r = 0;
        if (sscanf(e.c_str() + 9, "%lld %lld", &m, &r) != 2 || m == 0) throw BinderException("harness: bad '" + e + "'");
        return make_uniq<ExpressionFilter>(make_uniq<ModExpression>(m, r));
    }
    if (head("EXPR LIKE ")) return make_uniq<ExpressionFilter>(make_uniq<ContainsExpression>(e.substr(10)));
    if (e == "ISNULL") return make_uniq<IsNullFilter>();
    if (e == "ISNOTNULL") return make_uniq<IsNotNullFilter>();
    if (head("OPT ")) return make_uniq<OptionalFilter>(parse_filter(e.substr(4), type));
    if (head("IN ")) {
        vector<Value> vals;
        for (auto &v : split(e.substr(3), '|')) vals.push_back(parse_constant(v, type));
        return make_uniq<InFilter>(std::move(vals));
    }
    if (head("OR ")) {
        auto f = make_uniq<ConjunctionOrFilter>();
        for (auto &part : split(e.substr(3), '|')) f->child_filters.push_back(parse_filter(part, type));
        return std::move(f);
    }
    const size_t sp = e.find(' ');
    if (sp == std::string::npos) throw BinderException("harness: bad filter '" + e + "'");
    return make_uniq<ConstantFilter>(parse_op(e.substr(0, sp)), parse_constant(e.substr(sp + 1), type));
}

// run the query; sink(batch_index, chunk, pick, n) receives every produced
// chunk.  With nthreads > 1 the scan runs the way DuckDB's pipeline executor
// runs a parallel source: min(nthreads, MaxThreads()) threads, each with its own
// local state, all pulling from one global state; the sink is then called
// concurrently and orders results by batch index itself.
template <class Sink>
void execute(fls_ext_db *d, Query &q, const std::vector<int> &proj, int64_t limit, std::vector<std::string> &names,
             std::vector<LogicalType> &types, Sink sink, int nthreads = 1,
             const std::vector<FilterSpec> &where = {}) {
    TableFunction *f = lookup(d, q);
    d->ctx.threads = std::max(1, nthreads);  // the database's worker threads for this query
    named_parameter_map_t named;
    TableFunctionBindInput bin{q.args, named};
    vector<LogicalType> rtypes;
    vector<string> rnames;
    auto bind = f->bind(d->ctx, bin, rtypes, rnames);
    vector<column_t> ids;
    if (proj.empty()) {
        for (column_t c = 0; c < rtypes.size(); ++c) ids.push_back(c);
    } else {
        for (int p : proj) {
            if (p < 0) ids.push_back(COLUMN_IDENTIFIER_ROW_ID);
            else if ((size_t)p < rtypes.size()) ids.push_back((column_t)p);
            else throw BinderException("projection index out of range");
        }
    }
    // without pushdown the function produces every column and we project after
    vector<column_t> fn_ids = ids;
    if (!f->projection_pushdown) {
        fn_ids.clear();
        for (column_t c = 0; c < rtypes.size(); ++c) fn_ids.push_back(c);
    }
    // WHERE: filter columns join column_ids (after the projected ones); with
    // filter_prune the chunk holds only the projected positions
    TableFilterSet filter_set;
    vector<idx_t> projection_ids;
    if (!where.empty()) {
        if (!f->filter_pushdown) throw NotImplementedException("harness: " + q.fn + " takes no filters");
        const size_t nproj_ids = fn_ids.size();
        for (auto &w : where) {
            if (w.col < 0 || (size_t)w.col >= rtypes.size()) throw BinderException("filter column out of range");
            size_t pos = 0;
            while (pos < fn_ids.size() && fn_ids[pos] != (column_t)w.col) ++pos;
            if (pos == fn_ids.size()) fn_ids.push_back((column_t)w.col);
            filter_set.PushFilter(pos, parse_filter(w.expr, rtypes[w.col]));
        }
        if (f->filter_prune && fn_ids.size() > nproj_ids)
            for (idx_t i = 0; i < nproj_ids; ++i) projection_ids.push_back(i);
    }
    TableFunctionInitInput iin{bind.get(), fn_ids, projection_ids, where.empty() ? nullptr : &filter_set};
    auto gstate = f->init_global ? f->init_global(d->ctx, iin) : nullptr;
    vector<LogicalType> chunk_types;
    for (size_t i = 0; i < (projection_ids.empty() ? fn_ids.size() : projection_ids.size()); ++i) {
        const column_t id = fn_ids[projection_ids.empty() ? i : projection_ids[i]];
        chunk_types.push_back(id == COLUMN_IDENTIFIER_ROW_ID ? LogicalType::BIGINT : rtypes[id]);
    }
    for (auto id : ids) {
        names.push_back(id == COLUMN_IDENTIFIER_ROW_ID ? "rowid" : rnames[id]);
        types.push_back(id == COLUMN_IDENTIFIER_ROW_ID ? LogicalType::BIGINT : rtypes[id]);
    }
    std::vector<size_t> pick;  // output column -> chunk column
    for (auto id : ids) {
        size_t k = 0;
        while (fn_ids[k] != id) ++k;
        pick.push_back(k);
    }
    int threads = 1;
    if (nthreads > 1 && limit < 0 && gstate)
        threads = (int)std::min<idx_t>((idx_t)nthreads, gstate->MaxThreads());
    OperatorPartitionInfo pinfo;
    auto worker = [&](int64_t lim) {
        ExecutionContext ectx(d->ctx);
        auto lstate = f->init_local ? f->init_local(ectx, iin, gstate.get()) : nullptr;
        DataChunk chunk;
        chunk.Initialize(chunk_types);
        int64_t produced = 0;
        while (lim < 0 || produced < lim) {
            chunk.Reset();
            TableFunctionInput tin{bind.get(), lstate.get(), gstate.get()};
            f->function(d->ctx, tin, chunk);
            if (chunk.size() == 0) break;
            idx_t batch = 0;
            if (f->get_partition_data) {
                TableFunctionGetPartitionInput pin{bind.get(), lstate.get(), gstate.get(), pinfo};
                batch = f->get_partition_data(d->ctx, pin).batch_index;
            }
            const idx_t take = lim < 0 ? chunk.size() : std::min<idx_t>(chunk.size(), (idx_t)(lim - produced));
            sink(batch, chunk, pick, take);
            produced += (int64_t)take;
        }
    };
    if (threads == 1) {
        worker(limit);
        return;
    }
    std::vector<std::thread> pool;
    std::vector<std::string> errs(threads);
    for (int i = 0; i < threads; ++i)
        pool.emplace_back([&, i] {
            try {
                worker(-1);
            } catch (const std::exception &e) {
                errs[i] = e.what();
            }
        });
    for (auto &th : pool) th.join();
    for (auto &e : errs)
        if (!e.empty()) throw Exception(e);
}

Query make_query(fls_ext_db *d, const char *fn, const char *const *args, int nargs, int as_list) {
    Query q;
    if (!fn) {
        if (nargs != 1 || !resolve_replacement(d, args[0], q))
            throw Exception("Catalog Error: Table with name " + std::string(nargs ? args[0] : "?") + " does not exist!");
        return q;
    }
    q.fn = fn;
    q.raw = as_list == 2;
    if (as_list == 1) {
        vector<Value> items;
        for (int i = 0; i < nargs; ++i) items.push_back(Value(args[i] ? args[i] : ""));
        q.args.push_back(Value::LIST(LogicalType::VARCHAR, items));
    } else {
        for (int i = 0; i < nargs; ++i) {
            const std::string a = args[i] ? args[i] : "";
            // "\x01" prefix marks an INTEGER literal (to exercise type checks)
            if (!a.empty() && a[0] == '\x01') q.args.push_back(Value::INTEGER(std::atoi(a.c_str() + 1)));
            else q.args.push_back(Value(a));
        }
    }
    return q;
}

}  // namespace

extern "C" {

const char *fls_ext_last_error(void) { return g_err.c_str(); }

fls_ext_db *fls_ext_open(void) {
    auto *d = new fls_ext_db();
    try {
        fastlane_init(d->db);  // what DuckDB calls on LOAD fastlane
    } catch (const std::exception &e) {
        g_err = e.what();
        delete d;
        return nullptr;
    }
    return d;
}

void fls_ext_close(fls_ext_db *d) { delete d; }

int fls_ext_has_function(fls_ext_db *d, const char *name) { return d && d->db.table_functions.count(name) ? 1 : 0; }

// 1 when every overload of table function fn registers named parameter name
// with logical type id type_id (0: any type)
int fls_ext_has_named_parameter(fls_ext_db *d, const char *fn, const char *name, int type_id) {
    if (!d) return 0;
    auto range = d->db.table_functions.equal_range(fn);
    if (range.first == range.second) return 0;
    for (auto it = range.first; it != range.second; ++it) {
        auto p = it->second.named_parameters.find(name);
        if (p == it->second.named_parameters.end()) return 0;
        if (type_id && (int)p->second.id() != type_id) return 0;
    }
    return 1;
}

// The copy function's execution mode for (preserve_insertion_order,
// supports_batch_index) as DuckDB's planner asks it (0 REGULAR, 1 PARALLEL,
// 2 BATCH, -1 no callback / no function) and its desired batch size for the
// given COPY options (-1 without the callback)
int fls_ext_copy_mode(fls_ext_db *d, const char *fmt, int preserve, int batch_index, const char *const *opt_keys,
                      const char *const *opt_vals, int nopts, int64_t *batch_rows) {
    if (!d) return -1;
    auto it = d->db.copy_functions.find(fmt);
    if (it == d->db.copy_functions.end() || !it->second.execution_mode) return -1;
    CopyFunction &cf = it->second;
    *batch_rows = -1;
    if (cf.desired_batch_size && cf.copy_to_bind) {
        CopyInfo info;
        for (int i = 0; i < nopts; ++i) info.options[StringUtil::Lower(opt_keys[i])].push_back(Value(opt_vals[i]));
        CopyFunctionBindInput cbin{info};
        auto bind = cf.copy_to_bind(d->ctx, cbin, vector<string>{"a"}, vector<LogicalType>{LogicalType::INTEGER});
        *batch_rows = (int64_t)cf.desired_batch_size(d->ctx, *bind);
    }
    return (int)cf.execution_mode(preserve != 0, batch_index != 0);
}

// SELECT name() for a zero-argument scalar function: its one VARCHAR value
// rendered into buf (cap bytes); -1 when there is no such function
int fls_ext_scalar0(fls_ext_db *d, const char *name, char *buf, int cap) {
    if (!d) return -1;
    auto it = d->db.scalar_functions.find(name);
    if (it == d->db.scalar_functions.end() || !it->second.arguments.empty()) return -1;
    try {
        DataChunk args;
        args.SetCardinality(1);
        ExpressionState state;
        Vector result(it->second.return_type);
        it->second.function(args, state, result);
        const string v = result.GetValue(0).ToString();
        snprintf(buf, cap, "%s", v.c_str());
        return (int)v.size();
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

static std::vector<FilterSpec> make_where(const int *fcols, const char *const *fexprs, int nfilters) {
    std::vector<FilterSpec> w;
    for (int i = 0; i < nfilters; ++i) w.push_back(FilterSpec{fcols[i], fexprs[i] ? fexprs[i] : ""});
    return w;
}

int fls_ext_query_where(fls_ext_db *d, const char *fn, const char *const *args, int nargs, int as_list,
                        const int *proj, int nproj, const int *fcols, const char *const *fexprs, int nfilters,
                        int64_t limit, int nthreads, fls_ext_result **out);

int fls_ext_query_mt(fls_ext_db *d, const char *fn, const char *const *args, int nargs, int as_list, const int *proj,
                     int nproj, int64_t limit, int nthreads, fls_ext_result **out) {
    return fls_ext_query_where(d, fn, args, nargs, as_list, proj, nproj, nullptr, nullptr, 0, limit, nthreads, out);
}

int fls_ext_query_where(fls_ext_db *d, const char *fn, const char *const *args, int nargs, int as_list,
                        const int *proj, int nproj, const int *fcols, const char *const *fexprs, int nfilters,
                        int64_t limit, int nthreads, fls_ext_result **out) {
    try {
        const std::vector<FilterSpec> where = make_where(fcols, fexprs, nfilters);
        Query q = make_query(d, fn, args, nargs, as_list);
        auto *r = new fls_ext_result();
        std::unique_ptr<fls_ext_result> guard(r);
        std::vector<LogicalType> types;
        std::vector<int> pv(proj, proj + (proj ? nproj : 0));
        struct Part {
            std::vector<std::vector<std::string>> cells;
            std::vector<std::vector<char>> valid;
        };
        std::mutex mu;
        std::map<idx_t, Part> parts;  // batch index -> rows in arrival order (one thread per batch)
        execute(d, q, pv, limit, r->names, types, [&](idx_t batch, DataChunk &c, const std::vector<size_t> &pick, idx_t n) {
            Part local;
            for (idx_t i = 0; i < n; ++i) {
                local.cells.emplace_back();
                local.valid.emplace_back();
                for (size_t k : pick) {
                    Value v = c.data[k].GetValue(i);
                    local.valid.back().push_back(!v.IsNull());
                    local.cells.back().push_back(v.IsNull() ? std::string() : v.ToString());
                }
            }
            std::lock_guard<std::mutex> g(mu);
            Part &p = parts[batch];
            for (auto &x : local.cells) p.cells.push_back(std::move(x));
            for (auto &x : local.valid) p.valid.push_back(std::move(x));
        }, nthreads, where);
        for (auto &b : parts) {
            for (auto &x : b.second.cells) r->cells.push_back(std::move(x));
            for (auto &x : b.second.valid) r->valid.push_back(std::move(x));
        }
        for (auto &t : types) r->types.push_back(t.ToString());
        *out = guard.release();
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

// an argument starting with '\x01' is an INTEGER literal (type errors).
// as_list: 0 = scalar VARCHAR arguments, 1 = one LIST(VARCHAR) argument,
// 2 = raw: bypass overload resolution and casts (reaches the bind checks).
int fls_ext_query(fls_ext_db *d, const char *fn, const char *const *args, int nargs, int as_list, const int *proj,
                  int nproj, int64_t limit, fls_ext_result **out) {
    return fls_ext_query_mt(d, fn, args, nargs, as_list, proj, nproj, limit, 1, out);
}

int64_t fls_ext_result_rows(const fls_ext_result *r) { return (int64_t)r->cells.size(); }
int fls_ext_result_cols(const fls_ext_result *r) { return (int)r->names.size(); }
const char *fls_ext_result_name(const fls_ext_result *r, int c) { return r->names[c].c_str(); }
const char *fls_ext_result_type(const fls_ext_result *r, int c) { return r->types[c].c_str(); }
const char *fls_ext_result_value(const fls_ext_result *r, int64_t row, int col) {
    return r->valid[row][col] ? r->cells[row][col].c_str() : nullptr;
}
void fls_ext_result_free(fls_ext_result *r) { delete r; }

// The typed facade's read API exactly as the reference's intended scanner
// drives it (src/scanner/scan_fastlanes.cpp:82-83,126: openFile,
// getColumnTypes / getColumnNames at bind, then readNextChunk(values,
// rows_read) until it returns false): every boxed value as Value::ToString
// (NULL -> a null cell), the rows of each readNextChunk call in chunk_rows
// (up to max_chunks of them, *nchunks = the number of calls that returned
// rows).  max_rows < 0: the whole file.
int fls_ext_facade_read(const char *path, int64_t max_rows, fls_ext_result **out, int64_t *chunk_rows,
                        int max_chunks, int *nchunks) {
    using duckdb::ext_fastlane::FastLanesFacade;
    *out = nullptr;
    *nchunks = 0;
    FastLanesFacade f;
    if (!f.openFile(path)) {
        g_err = std::string("openFile failed: ") + path;
        return -1;
    }
    const std::vector<duckdb::LogicalType> types = f.getColumnTypes();
    const std::vector<std::string> names = f.getColumnNames();
    if (types.size() != names.size() || types.empty()) {
        g_err = "getColumnTypes / getColumnNames disagree";
        return -1;
    }
    auto *r = new fls_ext_result;
    r->names = names;
    for (auto &t : types) r->types.push_back(t.ToString());
    const size_t nc = types.size();
    std::vector<duckdb::Value> vals;
    duckdb::idx_t n = 0;
    int k = 0;
    while (f.readNextChunk(vals, n)) {
        if (vals.size() != n * nc || n == 0 || n > STANDARD_VECTOR_SIZE) {
            g_err = "readNextChunk: " + std::to_string(vals.size()) + " values for " + std::to_string(n) + " rows";
            delete r;
            return -1;
        }
        if (k < max_chunks) chunk_rows[k] = (int64_t)n;
        ++k;
        for (duckdb::idx_t i = 0; i < n; ++i) {
            std::vector<std::string> row(nc);
            std::vector<char> ok(nc, 1);
            for (size_t c = 0; c < nc; ++c) {
                const duckdb::Value &v = vals[i * nc + c];
                if (v.IsNull()) ok[c] = 0;
                else row[c] = v.ToString();
            }
            r->cells.push_back(std::move(row));
            r->valid.push_back(std::move(ok));
        }
        if (max_rows >= 0 && (int64_t)r->cells.size() >= max_rows) break;
    }
    f.closeFile();
    *nchunks = k;
    *out = r;
    return 0;
}

// Stream a query without materialising it: rows, a checksum of the result
// and wall seconds.  The checksum is a polynomial hash per column over the
// values in result order (string_t hashed by content), folded across chunks
// with H(A|B) = H(A) + P^|A| H(B), so it is independent of chunk and batch
// boundaries and of how many threads scanned: chunks are hashed where they are
// produced and folded in (batch index, arrival-within-batch) order.
namespace {
constexpr uint64_t kPoly = 0x9E3779B97F4A7C15ull | 1;
uint64_t upow(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    for (; e; e >>= 1, b *= b)
        if (e & 1) r *= b;
    return r;
}
uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
struct ChunkHash {
    uint64_t n = 0;
    std::vector<uint64_t> col;
};
ChunkHash hash_chunk(DataChunk &c, const std::vector<size_t> &pick, idx_t cnt) {
    ChunkHash r;
    r.n = cnt;
    for (size_t k : pick) {
        Vector &v = c.data[k];
        v.Flatten(cnt);  // dictionary vectors (read_fastlanes' DICT string columns)
        uint64_t h = 0, pw = 1;
        if (v.GetType().id() == LogicalTypeId::VARCHAR || v.GetType().id() == LogicalTypeId::BLOB) {
            const string_t *s = FlatVector::GetData<string_t>(v);
            for (idx_t i = 0; i < cnt; ++i, pw *= kPoly) {
                uint64_t f = 1469598103934665603ull;
                const char *p = s[i].GetData();
                for (uint32_t j = 0; j < s[i].GetSize(); ++j) f = (f ^ (uint8_t)p[j]) * 1099511628211ull;
                h += pw * mix(f ^ s[i].GetSize());
            }
        } else {
            const idx_t w = v.GetType().PhysicalSize();
            const uint8_t *p = v.GetData();
            for (idx_t i = 0; i < cnt; ++i, pw *= kPoly) {
                uint64_t x = 0;
                memcpy(&x, p + i * w, w);
                h += pw * mix(x);
            }
        }
        r.col.push_back(h);
    }
    return r;
}
}  // namespace

extern "C" int fls_ext_scan_count_where(fls_ext_db *d, const char *fn, const char *path, const int *proj, int nproj,
                                        const int *fcols, const char *const *fexprs, int nfilters, int nthreads,
                                        uint64_t *rows, uint64_t *checksum, double *seconds);

extern "C" int fls_ext_scan_count_mt(fls_ext_db *d, const char *fn, const char *path, const int *proj, int nproj,
                                     int nthreads, uint64_t *rows, uint64_t *checksum, double *seconds) {
    return fls_ext_scan_count_where(d, fn, path, proj, nproj, nullptr, nullptr, 0, nthreads, rows, checksum, seconds);
}

extern "C" int fls_ext_scan_count_where(fls_ext_db *d, const char *fn, const char *path, const int *proj, int nproj,
                                        const int *fcols, const char *const *fexprs, int nfilters, int nthreads,
                                        uint64_t *rows, uint64_t *checksum, double *seconds) {
    try {
        const std::vector<FilterSpec> where = make_where(fcols, fexprs, nfilters);
        const char *args[1] = {path};
        Query q = make_query(d, fn, args, 1, 0);
        std::vector<std::string> names;
        std::vector<LogicalType> types;
        std::vector<int> pv(proj, proj + (proj ? nproj : 0));
        std::mutex mu;
        std::map<idx_t, std::vector<ChunkHash>> parts;
        auto t0 = std::chrono::steady_clock::now();
        execute(d, q, pv, -1, names, types, [&](idx_t batch, DataChunk &c, const std::vector<size_t> &pick, idx_t cnt) {
            ChunkHash h = hash_chunk(c, pick, cnt);
            std::lock_guard<std::mutex> g(mu);
            parts[batch].push_back(std::move(h));
        }, nthreads, where);
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t n = 0;
        std::vector<uint64_t> acc(names.size(), 0);
        for (auto &b : parts)
            for (auto &ch : b.second) {
                const uint64_t pw = upow(kPoly, n);
                for (size_t j = 0; j < acc.size(); ++j) acc[j] += pw * ch.col[j];
                n += ch.n;
            }
        uint64_t h = 1469598103934665603ull;
        for (uint64_t x : acc) h = (h ^ x) * 1099511628211ull;
        *rows = n;
        *checksum = (h ^ n) * 1099511628211ull;
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

// DataChunk delivery rate: the scan through the executor with a sink that
// only counts rows (no checksum, no copy), i.e. what the table function itself
// costs a DuckDB pipeline.
extern "C" int fls_ext_scan_rows(fls_ext_db *d, const char *fn, const char *path, const int *proj, int nproj,
                                 int nthreads, uint64_t *rows, double *seconds) {
    try {
        const char *args[1] = {path};
        Query q = make_query(d, fn, args, 1, 0);
        std::vector<std::string> names;
        std::vector<LogicalType> types;
        std::vector<int> pv(proj, proj + (proj ? nproj : 0));
        std::atomic<uint64_t> n{0};
        auto t0 = std::chrono::steady_clock::now();
        execute(d, q, pv, -1, names, types, [&](idx_t, DataChunk &, const std::vector<size_t> &, idx_t cnt) {
            n += cnt;
        }, nthreads);
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        *rows = n;
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

// The scan with a sink that KEEPS a reference to every chunk it receives
// (DataChunk::Reference, as an operator that buffers its input would) and
// hashes them all only after the scan has ended: zero-copy vectors must stay
// valid while referenced, whatever the engine recycled meanwhile (ADVICE r1:
// FSST strings pointing into a recycled batch heap).  Same checksum as
// fls_ext_scan_count.
extern "C" int fls_ext_scan_hold(fls_ext_db *d, const char *fn, const char *path, int nthreads, uint64_t *rows,
                                 uint64_t *checksum, double *seconds) {
    try {
        const char *args[1] = {path};
        Query q = make_query(d, fn, args, 1, 0);
        std::vector<std::string> names;
        std::vector<LogicalType> types;
        std::mutex mu;
        std::map<idx_t, std::vector<std::pair<std::unique_ptr<DataChunk>, idx_t>>> held;
        std::vector<size_t> pick0;
        auto t0 = std::chrono::steady_clock::now();
        execute(d, q, {}, -1, names, types, [&](idx_t batch, DataChunk &c, const std::vector<size_t> &pick, idx_t cnt) {
            auto h = std::make_unique<DataChunk>();
            h->Reference(c);
            std::lock_guard<std::mutex> g(mu);
            pick0 = pick;
            held[batch].emplace_back(std::move(h), cnt);
        }, nthreads);
        *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t n = 0;
        std::vector<uint64_t> acc(names.size(), 0);
        for (auto &b : held)
            for (auto &ch : b.second) {
                ChunkHash hc = hash_chunk(*ch.first, pick0, ch.second);
                const uint64_t pw = upow(kPoly, n);
                for (size_t j = 0; j < acc.size(); ++j) acc[j] += pw * hc.col[j];
                n += hc.n;
            }
        uint64_t h = 1469598103934665603ull;
        for (uint64_t x : acc) h = (h ^ x) * 1099511628211ull;
        *rows = n;
        *checksum = (h ^ n) * 1099511628211ull;
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

extern "C" int fls_ext_scan_count(fls_ext_db *d, const char *fn, const char *path, const int *proj, int nproj,
                                  uint64_t *rows, uint64_t *checksum, double *seconds) {
    return fls_ext_scan_count_mt(d, fn, path, proj, nproj, 1, rows, checksum, seconds);
}

// COPY (SELECT <proj> FROM fn(src)) TO dst (FORMAT format, key value, ...):
// bind -> init_global -> init_local -> sink per chunk -> combine -> finalize,
// the order DuckDB's PhysicalCopyToFile drives a CopyFunction.  Option values
// are passed as VARCHAR (DuckDB hands the parsed constants; the bind parses).
int fls_ext_copy_mt(fls_ext_db *d, const char *fn, const char *src, const int *proj, int nproj, const char *format,
                    const char *dst, const char *const *opt_keys, const char *const *opt_vals, int nopts,
                    int nthreads, uint64_t *rows);

int fls_ext_copy(fls_ext_db *d, const char *fn, const char *src, const int *proj, int nproj, const char *format,
                 const char *dst, const char *const *opt_keys, const char *const *opt_vals, int nopts,
                 uint64_t *rows) {
    return fls_ext_copy_mt(d, fn, src, proj, nproj, format, dst, opt_keys, opt_vals, nopts, 1, rows);
}

}  // extern "C"

// DuckDB's PhysicalCopyToFile target for a COPY without PARTITION_BY: one
// global state, or, when the function rotates files (rotate_files), a
// directory of files dst/data_0.<ext>, data_1.<ext>, ... (DuckDB's default
// FILENAME_PATTERN) where every sink first asks rotate_next_file under the
// global lock and a full file is finalized once its in-flight sinks are done
// (WriteRotateInternal).
struct CopyTarget {
    struct File {
        unique_ptr<GlobalFunctionData> g;
        std::shared_mutex rw;  // sinks into this file: shared; its finalize: exclusive
    };
    fls_ext_db *d;
    CopyFunction &cf;
    FunctionData &bind;
    std::string dst;
    bool rotate = false;
    idx_t next = 0;
    std::mutex mu;
    std::shared_ptr<File> cur;
    CopyTarget(fls_ext_db *d_, CopyFunction &cf_, FunctionData &bind_, const char *dst_)
        : d(d_), cf(cf_), bind(bind_), dst(dst_ ? dst_ : "") {
        rotate = cf.rotate_files && cf.rotate_files(bind, optional_idx());
        if (rotate && mkdir(dst.c_str(), 0777) != 0 && errno != EEXIST)
            throw IOException("Cannot create directory \"" + dst + "\"");
        cur = open();
    }
    std::shared_ptr<File> open() {
        auto f = std::make_shared<File>();
        const std::string path = rotate ? dst + "/data_" + std::to_string(next++) + "." + cf.extension : dst;
        f->g = cf.copy_to_initialize_global(d->ctx, bind, path);
        return f;
    }
    template <class F>
    void write(F &&fun) {
        for (;;) {
            std::unique_lock<std::mutex> g(mu);
            std::shared_ptr<File> f = cur;
            if (rotate && cf.rotate_next_file && cf.rotate_next_file(*f->g, bind, optional_idx())) {
                cur = open();
                g.unlock();
                std::unique_lock<std::shared_mutex> x(f->rw);
                cf.copy_to_finalize(d->ctx, bind, *f->g);
                continue;
            }
            std::shared_lock<std::shared_mutex> in(f->rw);
            g.unlock();
            fun(*f->g);
            return;
        }
    }
    void finalize() { cf.copy_to_finalize(d->ctx, bind, *cur->g); }
};

extern "C" {

// nthreads > 1: an unordered COPY, the scan on up to nthreads threads (the
// parallel source) and each thread sinking into its own local state, as
// DuckDB's pipeline runs PhysicalCopyToFile with PARALLEL_COPY_TO_FILE.
int fls_ext_copy_mt(fls_ext_db *d, const char *fn, const char *src, const int *proj, int nproj, const char *format,
                    const char *dst, const char *const *opt_keys, const char *const *opt_vals, int nopts,
                    int nthreads, uint64_t *rows) {
    try {
        const std::string fmt = StringUtil::Lower(format ? format : "");
        auto it = d->db.copy_functions.find(fmt);
        if (it == d->db.copy_functions.end())
            throw CatalogException("Copy Function with name " + fmt + " does not exist!");
        CopyFunction &cf = it->second;
        CopyInfo info;
        for (int i = 0; i < nopts; ++i) info.options[StringUtil::Lower(opt_keys[i])].push_back(Value(opt_vals[i]));
        const char *args[1] = {src};
        Query q = make_query(d, fn, args, 1, 0);
        std::vector<int> pv(proj, proj + (proj ? nproj : 0));
        // the source's schema (a bind-only pass, as DuckDB binds the SELECT first)
        std::vector<std::string> names;
        std::vector<LogicalType> types;
        {
            TableFunction *f = lookup(d, q);
            named_parameter_map_t named;
            TableFunctionBindInput bin{q.args, named};
            vector<LogicalType> rtypes;
            vector<string> rnames;
            f->bind(d->ctx, bin, rtypes, rnames);
            if (pv.empty()) {
                names.assign(rnames.begin(), rnames.end());
                types.assign(rtypes.begin(), rtypes.end());
            } else {
                for (int p : pv) {
                    if (p < 0 || (size_t)p >= rtypes.size()) throw BinderException("projection index out of range");
                    names.push_back(rnames[p]);
                    types.push_back(rtypes[p]);
                }
            }
        }
        CopyFunctionBindInput cbin{info};
        auto bind = cf.copy_to_bind(d->ctx, cbin, vector<string>(names.begin(), names.end()),
                                    vector<LogicalType>(types.begin(), types.end()));
        CopyTarget target(d, cf, *bind, dst);
        if (nthreads < 1) nthreads = 1;
        if (nthreads > 1 && (!cf.execution_mode ||
                             cf.execution_mode(false, false) != CopyFunctionExecutionMode::PARALLEL_COPY_TO_FILE))
            throw NotImplementedException("harness: " + fmt + " has no parallel COPY sink");
        ExecutionContext ectx(d->ctx);
        // one local state (and projection chunk) per sink thread
        struct Local {
            unique_ptr<LocalFunctionData> state;
            DataChunk out;
        };
        std::mutex lmu;
        std::map<std::thread::id, std::unique_ptr<Local>> locals;
        auto local = [&]() -> Local & {
            std::lock_guard<std::mutex> g(lmu);
            auto &l = locals[std::this_thread::get_id()];
            if (!l) {
                l = std::make_unique<Local>();
                l->state = cf.copy_to_initialize_local(ectx, *bind);
                l->out.Initialize(vector<LogicalType>(types.begin(), types.end()));
            }
            return *l;
        };
        std::atomic<uint64_t> n{0};
        std::vector<std::string> n2;
        std::vector<LogicalType> t2;
        execute(d, q, pv, -1, n2, t2, [&](idx_t, DataChunk &c, const std::vector<size_t> &pick, idx_t cnt) {
            Local &l = local();
            bool identity = pick.size() == c.ColumnCount() && cnt == c.size();
            for (size_t k = 0; identity && k < pick.size(); ++k) identity = pick[k] == k;
            DataChunk *sunk = &c;
            if (!identity) {
                DataChunk &out = l.out;
                out.Reset();
                for (size_t k = 0; k < pick.size(); ++k)
                    for (idx_t i = 0; i < cnt; ++i) out.data[k].SetValue(i, c.data[pick[k]].GetValue(i));
                out.SetCardinality(cnt);
                sunk = &out;
            }
            target.write([&](GlobalFunctionData &g) { cf.copy_to_sink(ectx, *bind, g, *l.state, *sunk); });
            n += cnt;
        }, nthreads);
        if (locals.empty()) local();  // an empty source still has one sink
        for (auto &kv : locals)
            if (cf.copy_to_combine)
                target.write([&](GlobalFunctionData &g) { cf.copy_to_combine(ectx, *bind, g, *kv.second->state); });
        target.finalize();
        if (rows) *rows = n.load();
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

// COPY (SELECT * FROM (VALUES ...) t(names)) TO dst (FORMAT format): literal
// rows, cells[row * ncols + col] as text or NULL for SQL NULL, in one chunk per
// STANDARD_VECTOR_SIZE rows.  Types: INTEGER, BIGINT, DOUBLE, VARCHAR.
int fls_ext_copy_values_mt(fls_ext_db *d, const char *format, const char *dst, int ncols, const char *const *names,
                           const char *const *type_names, int64_t nrows, const char *const *cells,
                           const char *const *opt_keys, const char *const *opt_vals, int nopts, int nthreads,
                           uint64_t *rows);

int fls_ext_copy_values(fls_ext_db *d, const char *format, const char *dst, int ncols, const char *const *names,
                        const char *const *type_names, int64_t nrows, const char *const *cells, uint64_t *rows) {
    return fls_ext_copy_values_mt(d, format, dst, ncols, names, type_names, nrows, cells, nullptr, nullptr, 0, 1,
                                  rows);
}

// The same with COPY options and nthreads sink threads, as DuckDB's
// PhysicalCopyToFile runs a parallel sink: each thread its own local state,
// chunk k sunk by thread k % nthreads, combine per local state, then finalize.
// nthreads > 1 needs the function to answer PARALLEL_COPY_TO_FILE for an
// unordered COPY (preserve_insertion_order = false).
int fls_ext_copy_values_mt(fls_ext_db *d, const char *format, const char *dst, int ncols, const char *const *names,
                           const char *const *type_names, int64_t nrows, const char *const *cells,
                           const char *const *opt_keys, const char *const *opt_vals, int nopts, int nthreads,
                           uint64_t *rows) {
    try {
        const std::string fmt = StringUtil::Lower(format ? format : "");
        auto it = d->db.copy_functions.find(fmt);
        if (it == d->db.copy_functions.end())
            throw CatalogException("Copy Function with name " + fmt + " does not exist!");
        CopyFunction &cf = it->second;
        if (nthreads < 1) nthreads = 1;
        if (nthreads > 1 && (!cf.execution_mode ||
                             cf.execution_mode(false, false) != CopyFunctionExecutionMode::PARALLEL_COPY_TO_FILE))
            throw NotImplementedException("harness: " + fmt + " has no parallel COPY sink");
        vector<string> cn;
        vector<LogicalType> ct;
        for (int c = 0; c < ncols; ++c) {
            const std::string tn = StringUtil::Upper(type_names[c]);
            cn.emplace_back(names[c]);
            unsigned w = 0, sc = 0;
            if (tn == "INTEGER") ct.push_back(LogicalType::INTEGER);
            else if (tn == "BIGINT") ct.push_back(LogicalType::BIGINT);
            else if (tn == "DOUBLE") ct.push_back(LogicalType::DOUBLE);
            else if (tn == "VARCHAR") ct.push_back(LogicalType::VARCHAR);
            else if (tn == "BOOLEAN") ct.push_back(LogicalType::BOOLEAN);
            else if (tn == "BLOB") ct.push_back(LogicalType::BLOB);
            else if (tn == "BIT") ct.push_back(LogicalType::BIT);
            else if (tn == "CHAR") ct.push_back(LogicalType(LogicalTypeId::CHAR));
            else if (tn == "TINYINT") ct.push_back(LogicalType::TINYINT);
            else if (tn == "SMALLINT") ct.push_back(LogicalType::SMALLINT);
            else if (tn == "UTINYINT") ct.push_back(LogicalType::UTINYINT);
            else if (tn == "UBIGINT") ct.push_back(LogicalType::UBIGINT);
            else if (tn == "FLOAT") ct.push_back(LogicalType::FLOAT);
            else if (tn == "DATE") ct.push_back(LogicalType::DATE);
            else if (sscanf(tn.c_str(), "DECIMAL(%u,%u)", &w, &sc) == 2) ct.push_back(LogicalType::DECIMAL(w, sc));
            else throw BinderException("harness: unsupported VALUES type " + tn);
        }
        CopyInfo info;
        for (int i = 0; i < nopts; ++i) info.options[StringUtil::Lower(opt_keys[i])].push_back(Value(opt_vals[i]));
        CopyFunctionBindInput cbin{info};
        auto bind = cf.copy_to_bind(d->ctx, cbin, cn, ct);
        CopyTarget target(d, cf, *bind, dst);
        auto worker = [&](int t) {
            ExecutionContext ectx(d->ctx);
            auto lstate = cf.copy_to_initialize_local(ectx, *bind);
            DataChunk chunk;
            chunk.Initialize(ct);
            const int64_t step = (int64_t)STANDARD_VECTOR_SIZE * nthreads;
            for (int64_t r0 = (int64_t)STANDARD_VECTOR_SIZE * t; r0 < nrows; r0 += step) {
                const idx_t n = (idx_t)std::min<int64_t>(STANDARD_VECTOR_SIZE, nrows - r0);
                chunk.Reset();
                for (int c = 0; c < ncols; ++c)
                    for (idx_t i = 0; i < n; ++i) {
                        const char *x = cells[(r0 + (int64_t)i) * ncols + c];
                        Value v;
                        if (!x) v = Value();
                        else if (ct[c].id() == LogicalTypeId::INTEGER) v = Value::INTEGER(std::atoi(x));
                        else if (ct[c].id() == LogicalTypeId::BIGINT) v = Value::BIGINT(std::atoll(x));
                        else if (ct[c].id() == LogicalTypeId::DOUBLE) v = Value::DOUBLE(std::atof(x));
                        else if (ct[c].id() == LogicalTypeId::VARCHAR) v = Value(std::string(x));
                        else v = parse_constant(x, ct[c]);
                        chunk.data[c].SetValue(i, v);
                    }
                chunk.SetCardinality(n);
                target.write([&](GlobalFunctionData &g) { cf.copy_to_sink(ectx, *bind, g, *lstate, chunk); });
            }
            if (cf.copy_to_combine)
                target.write([&](GlobalFunctionData &g) { cf.copy_to_combine(ectx, *bind, g, *lstate); });
        };
        if (nthreads == 1) {
            worker(0);
        } else {
            std::vector<std::thread> pool;
            std::vector<std::string> errs(nthreads);
            for (int t = 0; t < nthreads; ++t)
                pool.emplace_back([&, t] {
                    try {
                        worker(t);
                    } catch (const std::exception &e) {
                        errs[t] = e.what();
                    }
                });
            for (auto &th : pool) th.join();
            for (auto &e : errs)
                if (!e.empty()) throw Exception(e);
        }
        target.finalize();
        if (rows) *rows = (uint64_t)nrows;
        return 0;
    } catch (const std::exception &e) {
        g_err = e.what();
        return -1;
    }
}

int fls_ext_has_copy_function(fls_ext_db *d, const char *name) {
    return d && d->db.copy_functions.count(name) ? 1 : 0;
}

}  // extern "C"
