// duckdb_shim_core.hpp -- the slice of the DuckDB v1.3.2 C++ extension API the
// FastLanes glue uses, declared from public knowledge of
// DuckDB because the duckdb/ submodule is empty (.gitmodules:1-4).  It lets
// the glue in ../ compile and run unchanged in this container; against a real
// DuckDB v1.3.2 the glue compiles with DuckDB's own headers instead (same
// include paths: "duckdb.hpp", "duckdb/function/table_function.hpp", ...).
// Only the behaviour the glue and the tests observe is modelled: flat vectors,
// Value casts to VARCHAR, string_t, table-function callbacks, replacement
// scans, exceptions.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace duckdb {

using std::move;
using std::string;
template <class T>
using vector = std::vector<T>;
template <class T, class D = std::default_delete<T>>
using unique_ptr = std::unique_ptr<T, D>;
template <class T>
using shared_ptr = std::shared_ptr<T>;
template <class T>
using optional_ptr = T *;
using idx_t = uint64_t;
using column_t = uint64_t;
using data_ptr_t = uint8_t *;
using const_data_ptr_t = const uint8_t *;

constexpr idx_t STANDARD_VECTOR_SIZE = 2048;
constexpr column_t COLUMN_IDENTIFIER_ROW_ID = (column_t)-1;

template <class T, class... Args>
unique_ptr<T> make_uniq(Args &&...args) {
    return std::unique_ptr<T>(new T(std::forward<Args>(args)...));
}
template <class T, class... Args>
shared_ptr<T> make_shared_ptr(Args &&...args) {
    return std::make_shared<T>(std::forward<Args>(args)...);
}

// ---- exceptions ----------------------------------------------------------
class Exception : public std::runtime_error {
public:
    explicit Exception(const string &msg) : std::runtime_error(msg) {}
};
class BinderException : public Exception {
public:
    explicit BinderException(const string &msg) : Exception(msg) {}
};
class IOException : public Exception {
public:
    explicit IOException(const string &msg) : Exception(msg) {}
};
class InvalidInputException : public Exception {
public:
    explicit InvalidInputException(const string &msg) : Exception(msg) {}
};
class InternalException : public Exception {
public:
    explicit InternalException(const string &msg) : Exception(msg) {}
};
class CatalogException : public Exception {
public:
    explicit CatalogException(const string &msg) : Exception("Catalog Error: " + msg) {}
};
class NotImplementedException : public Exception {
public:
    explicit NotImplementedException(const string &msg) : Exception(msg) {}
};

// ---- types -----------------------------------------------------------------
enum class LogicalTypeId : uint8_t {
    INVALID = 0, SQLNULL, BOOLEAN, TINYINT, SMALLINT, INTEGER, BIGINT, UTINYINT, USMALLINT, UINTEGER,
    UBIGINT, DATE, FLOAT, DOUBLE, DECIMAL, VARCHAR, LIST, CHAR, BLOB, BIT
};

struct LogicalType {
    LogicalType() : id_(LogicalTypeId::INVALID) {}
    LogicalType(LogicalTypeId id) : id_(id) {}  // NOLINT (implicit like DuckDB)
    LogicalTypeId id() const { return id_; }
    bool operator==(const LogicalType &o) const {
        if (id_ != o.id_) return false;
        if (id_ == LogicalTypeId::DECIMAL) return width_ == o.width_ && scale_ == o.scale_;
        if (id_ == LogicalTypeId::LIST) return child_ && o.child_ && *child_ == *o.child_;
        return true;
    }
    bool operator!=(const LogicalType &o) const { return !(*this == o); }
    static LogicalType DECIMAL(uint8_t w, uint8_t s) {
        LogicalType t(LogicalTypeId::DECIMAL);
        t.width_ = w;
        t.scale_ = s;
        return t;
    }
    static LogicalType LIST(const LogicalType &child) {
        LogicalType t(LogicalTypeId::LIST);
        t.child_ = std::make_shared<LogicalType>(child);
        return t;
    }
    uint8_t Width() const { return width_; }
    uint8_t Scale() const { return scale_; }
    idx_t PhysicalSize() const;   // bytes per value in a flat vector
    string ToString() const;

    static const LogicalType SQLNULL, BOOLEAN, TINYINT, SMALLINT, INTEGER, BIGINT, UTINYINT, USMALLINT,
        UINTEGER, UBIGINT, DATE, FLOAT, DOUBLE, VARCHAR, BLOB, BIT;

private:
    LogicalTypeId id_;
    uint8_t width_ = 0, scale_ = 0;
    shared_ptr<LogicalType> child_;
};

// DuckDB string_t: 16 bytes, inlined up to 12 characters
struct string_t {
    static constexpr uint32_t INLINE_LENGTH = 12;
    string_t() { memset(this, 0, sizeof(*this)); }
    string_t(const char *data, uint32_t len) {
        memset(this, 0, sizeof(*this));
        value.inlined.length = len;
        if (len <= INLINE_LENGTH) {
            if (len) memcpy(value.inlined.inlined, data, len);
        } else {
            memcpy(value.pointer.prefix, data, 4);
            value.pointer.ptr = const_cast<char *>(data);
        }
    }
    uint32_t GetSize() const { return value.inlined.length; }
    const char *GetData() const {
        return GetSize() <= INLINE_LENGTH ? value.inlined.inlined : value.pointer.ptr;
    }
    string GetString() const { return string(GetData(), GetSize()); }
    union {
        struct {
            uint32_t length;
            char prefix[4];
            char *ptr;
        } pointer;
        struct {
            uint32_t length;
            char inlined[12];
        } inlined;
    } value;
};
static_assert(sizeof(string_t) == 16, "string_t is 16 bytes");

struct date_t {
    int32_t days;
};

// ---- Value -----------------------------------------------------------------
class Value {
public:
    Value() : type_(LogicalType::SQLNULL), is_null_(true) {}
    Value(const string &s) : type_(LogicalType::VARCHAR), is_null_(false), str_(s) {}  // NOLINT
    Value(const char *s) : Value(string(s)) {}                                          // NOLINT
    Value(const string_t &s) : Value(s.GetString()) {}                                  // NOLINT (DuckDB: Value(string_t))
    static Value INTEGER(int32_t v) { return Value(LogicalType::INTEGER, (int64_t)v); }
    static Value BIGINT(int64_t v) { return Value(LogicalType::BIGINT, v); }
    static Value TINYINT(int8_t v) { return Value(LogicalType::TINYINT, (int64_t)v); }
    static Value SMALLINT(int16_t v) { return Value(LogicalType::SMALLINT, (int64_t)v); }
    static Value UTINYINT(uint8_t v) { return Value(LogicalType::UTINYINT, (int64_t)v); }
    static Value USMALLINT(uint16_t v) { return Value(LogicalType::USMALLINT, (int64_t)v); }
    static Value UINTEGER(uint32_t v) { return Value(LogicalType::UINTEGER, (int64_t)v); }
    static Value UBIGINT(uint64_t v) { return Value(LogicalType::UBIGINT, (int64_t)v); }
    static Value DATE(date_t d) { return Value(LogicalType::DATE, (int64_t)d.days); }
    static Value DECIMAL(int64_t v, uint8_t w, uint8_t s) { return Value(LogicalType::DECIMAL(w, s), v); }
    static Value FLOAT(float v) { Value x(LogicalType::FLOAT, 0); x.dbl_ = v; return x; }
    static Value DOUBLE(double v) { Value x(LogicalType::DOUBLE, 0); x.dbl_ = v; return x; }
    static Value BOOLEAN(bool v) { return Value(LogicalType::BOOLEAN, (int64_t)v); }
    // DuckDB's Value::BLOB(const_data_ptr_t, idx_t): the raw bytes
    // DuckDB's BIT value: the bitstring's bytes (byte 0 = padding bit count,
    // the padding bits at the top of byte 1 set), as Bit::ToBit stores them
    static Value BIT(const uint8_t *data, idx_t len) {
        Value x(LogicalType::BIT, 0);
        x.str_.assign((const char *)data, len);
        return x;
    }
    static Value BLOB(const uint8_t *data, idx_t len) {
        Value x(LogicalType::BLOB, 0);
        x.str_.assign((const char *)data, len);
        return x;
    }
    static Value LIST(const LogicalType &child, vector<Value> items) {
        Value x(LogicalType::LIST(child), 0);
        x.list_ = std::move(items);
        return x;
    }

    const LogicalType &type() const { return type_; }
    bool IsNull() const { return is_null_; }
    template <class T>
    T GetValue() const;
    int64_t GetInt64() const { return int_; }
    template <class T>
    T GetValueUnsafe() const { return (T)int_; }
    double GetDouble() const { return dbl_; }
    const vector<Value> &ListChildren() const { return list_; }
    // DuckDB's VARCHAR rendering of the value (the cast Vector::SetValue applies)
    string ToString() const;

    friend struct StringValue;

private:
    Value(LogicalType t, int64_t v) : type_(std::move(t)), is_null_(false), int_(v) {}
    LogicalType type_;
    bool is_null_;
    int64_t int_ = 0;
    double dbl_ = 0;
    string str_;
    vector<Value> list_;
};
// DuckDB StringValue::Get: the bytes of a VARCHAR or BLOB value
struct StringValue {
    static const string &Get(const Value &v) { return v.str_; }
};
template <>
inline string Value::GetValue<string>() const { return is_null_ ? string() : (type_.id() == LogicalTypeId::VARCHAR ? str_ : ToString()); }
template <>
inline int64_t Value::GetValue<int64_t>() const { return int_; }
template <>
inline int32_t Value::GetValue<int32_t>() const { return (int32_t)int_; }
template <>
inline bool Value::GetValue<bool>() const { return int_ != 0; }
template <>
inline uint64_t Value::GetValue<uint64_t>() const { return (uint64_t)int_; }
template <>
inline double Value::GetValue<double>() const { return dbl_; }
template <>
inline float Value::GetValue<float>() const { return (float)dbl_; }
template <>
inline date_t Value::GetValue<date_t>() const { return date_t{(int32_t)int_}; }


// ---- vectors ---------------------------------------------------------------
enum class VectorType : uint8_t { FLAT_VECTOR, CONSTANT_VECTOR, DICTIONARY_VECTOR };

// DuckDB v1.3.2 common/types/vector_buffer.hpp: a buffer a Vector can hold
// on to.  OPAQUE_BUFFER subclasses keep foreign memory alive while a vector
// points into it (FlatVector::SetData + Vector::SetAuxiliary, as the Arrow
// scan does for zero-copy columns).
enum class VectorBufferType : uint8_t { STANDARD_BUFFER, STRING_BUFFER, OPAQUE_BUFFER };
class VectorBuffer {
public:
    explicit VectorBuffer(VectorBufferType type = VectorBufferType::STANDARD_BUFFER) : type_(type) {}
    virtual ~VectorBuffer() = default;
    VectorBufferType GetBufferType() const { return type_; }

private:
    VectorBufferType type_;
};
template <class T>
using buffer_ptr = shared_ptr<T>;
template <class T, class... Args>
buffer_ptr<T> make_buffer(Args &&...args) {
    return std::make_shared<T>(std::forward<Args>(args)...);
}

using sel_t = uint32_t;
// DuckDB common/types/selection_vector.hpp: row indices, owned (shared by
// copies, like DuckDB's SelectionData buffer) or borrowed (SelectionVector(sel_t *))
class SelectionVector {
public:
    SelectionVector() = default;
    explicit SelectionVector(sel_t *sel) : ptr_(sel) {}
    // DuckDB allocates the buffer and leaves it uninitialised (a DEBUG build
    // fills it with sel_t max): poisoned here too, so code that reads an
    // index it never wrote fails under the shim as it would in DuckDB
    explicit SelectionVector(idx_t count)
        : owned_(std::make_shared<vector<sel_t>>(count, std::numeric_limits<sel_t>::max())) {
        ptr_ = owned_->data();
    }
    // DuckDB's SelectionVector::Initialize(sel_t *) / (const SelectionVector &)
    void Initialize(sel_t *sel) {
        owned_.reset();
        ptr_ = sel;
    }
    void Initialize(const SelectionVector &other) {
        owned_ = other.owned_;
        ptr_ = other.ptr_;
    }
    idx_t get_index(idx_t i) const { return ptr_ ? ptr_[i] : i; }
    void set_index(idx_t i, idx_t loc) { ptr_[i] = (sel_t)loc; }
    sel_t *data() { return ptr_; }
    const sel_t *data() const { return ptr_; }

private:
    sel_t *ptr_ = nullptr;
    shared_ptr<vector<sel_t>> owned_;
};

// DuckDB common/types/validity_mask.hpp: one bit per row (1 = valid) in
// 64-bit words, no words allocated while every row is valid
using validity_t = uint64_t;
class ValidityMask {
public:
    static constexpr idx_t BITS_PER_VALUE = 64;
    explicit ValidityMask(idx_t capacity = STANDARD_VECTOR_SIZE) : capacity_(capacity) {}
    static idx_t EntryCount(idx_t count) { return (count + BITS_PER_VALUE - 1) / BITS_PER_VALUE; }
    bool AllValid() const { return !data_; }
    bool CheckAllValid(idx_t count) const {
        if (!data_) return true;
        for (idx_t i = 0; i < count / BITS_PER_VALUE; ++i)
            if (data_[i] != ~validity_t(0)) return false;
        const idx_t rest = count % BITS_PER_VALUE;
        return !rest || (data_[count / BITS_PER_VALUE] | (~validity_t(0) << rest)) == ~validity_t(0);
    }
    validity_t *GetData() const { return data_; }
    // own words for capacity rows, every row valid
    void Initialize(idx_t capacity) {
        capacity_ = capacity;
        owned_ = std::make_shared<vector<validity_t>>(EntryCount(capacity), ~validity_t(0));
        data_ = owned_->data();
    }
    void Initialize() { Initialize(capacity_); }
    void Reset() {
        data_ = nullptr;
        owned_.reset();
    }
    bool RowIsValid(idx_t row) const { return !data_ || ((data_[row / BITS_PER_VALUE] >> (row % BITS_PER_VALUE)) & 1); }
    void SetInvalid(idx_t row) {
        if (!data_) Initialize();
        data_[row / BITS_PER_VALUE] &= ~(validity_t(1) << (row % BITS_PER_VALUE));
    }
    void SetValid(idx_t row) {
        if (data_) data_[row / BITS_PER_VALUE] |= validity_t(1) << (row % BITS_PER_VALUE);
    }
    void Set(idx_t row, bool valid) { valid ? SetValid(row) : SetInvalid(row); }
    // a private copy of other's words
    void Copy(const ValidityMask &other, idx_t count) {
        if (!other.data_) {
            Reset();
            return;
        }
        Initialize(std::max(capacity_, count));
        std::copy(other.data_, other.data_ + EntryCount(count), data_);
    }
    idx_t Capacity() const { return capacity_; }

private:
    idx_t capacity_;
    validity_t *data_ = nullptr;
    shared_ptr<vector<validity_t>> owned_;
};

class Vector {
public:
    explicit Vector(LogicalType type, idx_t capacity = STANDARD_VECTOR_SIZE);
    // DuckDB Vector(const LogicalType &, data_ptr_t): a flat vector over
    // memory it does not own
    Vector(LogicalType type, data_ptr_t data);
    Vector(Vector &&o) noexcept;
    Vector(const Vector &) = delete;
    Vector &operator=(const Vector &) = delete;
    const LogicalType &GetType() const { return type_; }
    void SetValue(idx_t index, const Value &val);
    Value GetValue(idx_t index) const;
    data_ptr_t GetData() { return data_ptr_; }
    const uint8_t *GetData() const { return data_ptr_; }
    // FlatVector::SetData: point the vector at memory it does not own (valid
    // while the auxiliary buffer, or the caller, keeps it alive)
    void SetDataPtr(data_ptr_t p) { data_ptr_ = p; }
    void SetAuxiliary(buffer_ptr<VectorBuffer> b) { auxiliary_ = std::move(b); }
    // Vector::Reference: share other's data (and the buffer keeping it alive);
    // the shim's own storage is not shareable, so owned data is copied
    void Reference(const Vector &other);
    buffer_ptr<VectorBuffer> GetAuxiliary() const { return auxiliary_; }
    bool RowIsValid(idx_t i) const {
        return vtype_ == VectorType::DICTIONARY_VECTOR ? child_->RowIsValid(dict_sel_.get_index(i))
                                                       : validity_.RowIsValid(i);
    }
    void SetValid(idx_t i, bool v) { validity_.Set(i, v); }
    // DuckDB Vector::Slice(other, sel, count): this becomes a DICTIONARY_VECTOR,
    // row i = other's row sel[i] (other is referenced, not copied)
    void Slice(const Vector &other, const SelectionVector &sel, idx_t count);
    // DuckDB Vector::Flatten(count): a dictionary vector materialised flat
    void Flatten(idx_t count);
    const Vector &DictionaryChild() const { return *child_; }
    const SelectionVector &DictionarySel() const { return dict_sel_; }
    ValidityMask &Validity() { return validity_; }
    const ValidityMask &Validity() const { return validity_; }
    void ToUnifiedFormat(idx_t count, struct UnifiedVectorFormat &format) const;
    void SetVectorType(VectorType t) { vtype_ = t; }
    VectorType GetVectorType() const { return vtype_; }
    idx_t Capacity() const { return capacity_; }
    void Reset();
    // string heap owned by this vector (StringVector::AddString)
    string_t AddString(const string &s);
    void KeepAlive(shared_ptr<void> p) { keep_.push_back(std::move(p)); }

private:
    LogicalType type_;
    idx_t capacity_;
    vector<uint8_t> data_;
    data_ptr_t data_ptr_;                 // data_.data(), or foreign memory (SetData)
    buffer_ptr<VectorBuffer> auxiliary_;  // keeps foreign memory alive
    ValidityMask validity_;
    shared_ptr<Vector> child_;        // DICTIONARY_VECTOR: the dictionary
    SelectionVector dict_sel_;        // ... and the rows' entries
    std::deque<string> heap_;
    vector<shared_ptr<void>> keep_;
    VectorType vtype_ = VectorType::FLAT_VECTOR;
};

struct DictionaryVector {
    static const SelectionVector &SelVector(const Vector &v) { return v.DictionarySel(); }
    static const Vector &Child(const Vector &v) { return v.DictionaryChild(); }
};

struct FlatVector {
    template <class T>
    static T *GetData(Vector &v) { return reinterpret_cast<T *>(v.GetData()); }
    static void SetData(Vector &v, data_ptr_t data) { v.SetDataPtr(data); }
    static void SetNull(Vector &v, idx_t i, bool is_null) { v.SetValid(i, !is_null); }
    static bool IsNull(const Vector &v, idx_t i) { return !v.RowIsValid(i); }
    static ValidityMask &Validity(Vector &v) { return v.Validity(); }
    static const ValidityMask &Validity(const Vector &v) { return v.Validity(); }
    static void SetValidity(Vector &v, const ValidityMask &m) { v.Validity() = m; }
};
struct StringVector {
    static string_t AddString(Vector &v, const string &s) { return v.AddString(s); }
    static void AddBuffer(Vector &v, shared_ptr<void> keep) { v.KeepAlive(std::move(keep)); }
};

class DataChunk {
public:
    vector<Vector> data;
    idx_t ColumnCount() const { return data.size(); }
    idx_t size() const { return count_; }
    void SetCardinality(idx_t n) { count_ = n; }
    void InitializeEmpty(const vector<LogicalType> &types) {
        data.clear();
        for (auto &t : types) data.emplace_back(t);
        count_ = 0;
    }
    void Initialize(const vector<LogicalType> &types) { InitializeEmpty(types); }
    void Flatten() {  // DuckDB DataChunk::Flatten: every vector flat
        for (auto &v : data) v.Flatten(count_);
    }
    void Reset() {
        for (auto &v : data) v.Reset();
        count_ = 0;
    }
    // DataChunk::Reference: this chunk's vectors reference other's
    void Reference(const DataChunk &other) {
        data.clear();
        for (auto &v : other.data) {
            data.emplace_back(v.GetType());
            data.back().Reference(v);
        }
        count_ = other.count_;
    }
    vector<LogicalType> GetTypes() const {
        vector<LogicalType> t;
        for (auto &v : data) t.push_back(v.GetType());
        return t;
    }
    // keep rows sel[0, count) (DuckDB turns the vectors into dictionary
    // vectors over the same data; the shim copies the selected rows)
    void Slice(const class SelectionVector &sel, idx_t count);

private:
    idx_t count_ = 0;
};

// ---- functions -------------------------------------------------------------
class ClientContext {
public:
    int32_t threads = 1;  // the shim's stand-in for the database's worker threads (SET threads)
};
// DuckDB parallel/task_scheduler.hpp: NumberOfThreads()
class TaskScheduler {
public:
    static TaskScheduler &GetScheduler(ClientContext &context) {
        static thread_local TaskScheduler s;
        s.n_ = context.threads;
        return s;
    }
    int32_t NumberOfThreads() const { return n_; }

private:
    int32_t n_ = 1;
};
class ExecutionContext {
public:
    ClientContext &client;
    explicit ExecutionContext(ClientContext &c) : client(c) {}
};
class DatabaseInstance;

struct FunctionData {
    virtual ~FunctionData() = default;
    template <class T>
    T &Cast() { return static_cast<T &>(*this); }
    template <class T>
    const T &Cast() const { return static_cast<const T &>(*this); }
};
struct TableFunctionData : public FunctionData {
    vector<column_t> column_ids;
};
struct GlobalTableFunctionState {
    virtual ~GlobalTableFunctionState() = default;
    virtual idx_t MaxThreads() const { return 1; }
    template <class T>
    T &Cast() { return static_cast<T &>(*this); }
};
struct LocalTableFunctionState {
    virtual ~LocalTableFunctionState() = default;
    template <class T>
    T &Cast() { return static_cast<T &>(*this); }
};

using named_parameter_map_t = std::unordered_map<string, Value>;
using named_parameter_type_map_t = std::unordered_map<string, LogicalType>;

// ---- pushed-down table filters (duckdb/planner/table_filter.hpp and
// duckdb/planner/filter/*.hpp).  TableFilterSet::filters is keyed by the
// position in TableFunctionInitInput::column_ids.
enum class ExpressionType : uint8_t {
    COMPARE_EQUAL = 25, COMPARE_NOTEQUAL = 26, COMPARE_LESSTHAN = 27, COMPARE_GREATERTHAN = 28,
    COMPARE_LESSTHANOREQUALTO = 29, COMPARE_GREATERTHANOREQUALTO = 30
};
enum class TableFilterType : uint8_t {
    CONSTANT_COMPARISON = 0, IS_NULL = 1, IS_NOT_NULL = 2, CONJUNCTION_OR = 3, CONJUNCTION_AND = 4,
    STRUCT_EXTRACT = 5, OPTIONAL_FILTER = 6, IN_FILTER = 7, DYNAMIC_FILTER = 8, EXPRESSION_FILTER = 9
};
class TableFilter {
public:
    explicit TableFilter(TableFilterType t) : filter_type(t) {}
    virtual ~TableFilter() = default;
    TableFilterType filter_type;
    template <class T>
    T &Cast() { return static_cast<T &>(*this); }
    template <class T>
    const T &Cast() const { return static_cast<const T &>(*this); }
};
class ConstantFilter : public TableFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::CONSTANT_COMPARISON;
    ConstantFilter(ExpressionType comparison_type, Value constant)
        : TableFilter(TYPE), comparison_type(comparison_type), constant(std::move(constant)) {}
    ExpressionType comparison_type;
    Value constant;
};
class IsNullFilter : public TableFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::IS_NULL;
    IsNullFilter() : TableFilter(TYPE) {}
};
class IsNotNullFilter : public TableFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::IS_NOT_NULL;
    IsNotNullFilter() : TableFilter(TYPE) {}
};
class ConjunctionFilter : public TableFilter {
public:
    explicit ConjunctionFilter(TableFilterType t) : TableFilter(t) {}
    vector<unique_ptr<TableFilter>> child_filters;
};
class ConjunctionOrFilter : public ConjunctionFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::CONJUNCTION_OR;
    ConjunctionOrFilter() : ConjunctionFilter(TYPE) {}
};
class ConjunctionAndFilter : public ConjunctionFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::CONJUNCTION_AND;
    ConjunctionAndFilter() : ConjunctionFilter(TYPE) {}
};
class InFilter : public TableFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::IN_FILTER;
    explicit InFilter(vector<Value> values) : TableFilter(TYPE), values(std::move(values)) {}
    vector<Value> values;
};
class OptionalFilter : public TableFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::OPTIONAL_FILTER;
    explicit OptionalFilter(unique_ptr<TableFilter> child = nullptr) : TableFilter(TYPE), child_filter(std::move(child)) {}
    unique_ptr<TableFilter> child_filter;
};
class TableFilterSet {
public:
    std::map<idx_t, unique_ptr<TableFilter>> filters;
    // a second filter on one column AND-s with the first (TableFilterSet::PushFilter)
    void PushFilter(idx_t column_index, unique_ptr<TableFilter> filter) {
        auto it = filters.find(column_index);
        if (it == filters.end()) {
            filters[column_index] = std::move(filter);
            return;
        }
        if (it->second->filter_type != TableFilterType::CONJUNCTION_AND) {
            auto conj = make_uniq<ConjunctionAndFilter>();
            conj->child_filters.push_back(std::move(it->second));
            it->second = std::move(conj);
        }
        it->second->Cast<ConjunctionAndFilter>().child_filters.push_back(std::move(filter));
    }
};

// ---- residual filters: what DuckDB's own scans use for filters a scan
// cannot apply natively (v1.3.2 planner/filter/expression_filter.hpp,
// planner/table_filter_state.hpp, storage/table/column_segment.hpp,
// common/types/selection_vector.hpp).  The shim evaluates row by row through
// Value; Expression here is a stand-in the harness builds (DuckDB's
// ExpressionFilter holds a bound planner Expression run by an executor).
struct UnifiedVectorFormat {
    const SelectionVector *sel = nullptr;
    const_data_ptr_t data = nullptr;
    ValidityMask validity;
};
class Expression {
public:
    virtual ~Expression() = default;
    virtual bool EvaluateRow(const Value &v) const = 0;  // shim stand-in
};
class ExpressionFilter : public TableFilter {
public:
    static constexpr TableFilterType TYPE = TableFilterType::EXPRESSION_FILTER;
    explicit ExpressionFilter(unique_ptr<Expression> e) : TableFilter(TYPE), expr(std::move(e)) {}
    unique_ptr<Expression> expr;
};
struct TableFilterState {
    virtual ~TableFilterState() = default;
    static unique_ptr<TableFilterState> Initialize(ClientContext &context, const TableFilter &filter);
};
class ColumnSegment {
public:
    // keep the approved_tuple_count rows of sel for which the filter holds
    // (sel compacted in place); returns the new approved_tuple_count
    static idx_t FilterSelection(SelectionVector &sel, Vector &vector, UnifiedVectorFormat &vdata,
                                 const TableFilter &filter, TableFilterState &filter_state, idx_t scan_count,
                                 idx_t &approved_tuple_count);
};

struct TableFunctionBindInput {
    vector<Value> &inputs;
    named_parameter_map_t &named_parameters;
};
struct TableFunctionInitInput {
    optional_ptr<const FunctionData> bind_data;
    const vector<column_t> &column_ids;
    // filter_prune: positions in column_ids the output chunk holds (empty = all)
    vector<idx_t> projection_ids = {};
    optional_ptr<TableFilterSet> filters = nullptr;
};
struct TableFunctionInput {
    optional_ptr<const FunctionData> bind_data;
    optional_ptr<LocalTableFunctionState> local_state;
    optional_ptr<GlobalTableFunctionState> global_state;
};

using table_function_bind_t = unique_ptr<FunctionData> (*)(ClientContext &, TableFunctionBindInput &,
                                                           vector<LogicalType> &, vector<string> &);
using table_function_init_global_t = unique_ptr<GlobalTableFunctionState> (*)(ClientContext &,
                                                                             TableFunctionInitInput &);
using table_function_init_local_t = unique_ptr<LocalTableFunctionState> (*)(ExecutionContext &,
                                                                           TableFunctionInitInput &,
                                                                           GlobalTableFunctionState *);
using table_function_t = void (*)(ClientContext &, TableFunctionInput &, DataChunk &);

// order-preserving parallel scans (DuckDB v1.3 get_partition_data)
struct OperatorPartitionInfo {
    bool batch_index = true;
    bool RequiresBatchIndex() const { return batch_index; }
};
struct OperatorPartitionData {
    explicit OperatorPartitionData(idx_t batch_index) : batch_index(batch_index) {}
    idx_t batch_index;
};
struct TableFunctionGetPartitionInput {
    optional_ptr<const FunctionData> bind_data;
    optional_ptr<LocalTableFunctionState> local_state;
    optional_ptr<GlobalTableFunctionState> global_state;
    const OperatorPartitionInfo &partition_info;
};
using table_function_get_partition_data_t = OperatorPartitionData (*)(ClientContext &,
                                                                      TableFunctionGetPartitionInput &);

class TableFunction {
public:
    TableFunction(string name, vector<LogicalType> arguments, table_function_t function,
                  table_function_bind_t bind = nullptr, table_function_init_global_t init_global = nullptr,
                  table_function_init_local_t init_local = nullptr)
        : name(std::move(name)), arguments(std::move(arguments)), function(function), bind(bind),
          init_global(init_global), init_local(init_local) {}
    string name;
    vector<LogicalType> arguments;
    named_parameter_type_map_t named_parameters;
    table_function_t function;
    table_function_bind_t bind;
    table_function_init_global_t init_global;
    table_function_init_local_t init_local;
    table_function_get_partition_data_t get_partition_data = nullptr;
    bool projection_pushdown = false;
    bool filter_pushdown = false;
    bool filter_prune = false;
    void *in_out_function = nullptr;
};

struct ExpressionState {};
using scalar_function_t = void (*)(DataChunk &, ExpressionState &, Vector &);
class ScalarFunction {
public:
    ScalarFunction(string name, vector<LogicalType> arguments, LogicalType return_type, scalar_function_t fn)
        : name(std::move(name)), arguments(std::move(arguments)), return_type(std::move(return_type)),
          function(fn) {}
    string name;
    vector<LogicalType> arguments;
    LogicalType return_type;
    scalar_function_t function;
};

// ---- copy functions (COPY ... TO 'x' (FORMAT name, options)) ----------------
struct GlobalFunctionData {
    virtual ~GlobalFunctionData() = default;
    template <class T>
    T &Cast() { return static_cast<T &>(*this); }
};
struct LocalFunctionData {
    virtual ~LocalFunctionData() = default;
    template <class T>
    T &Cast() { return static_cast<T &>(*this); }
};
struct CopyInfo {
    std::map<string, vector<Value>> options;  // option name -> values
};
struct CopyFunctionBindInput {
    const CopyInfo &info;
};
using copy_to_bind_t = unique_ptr<FunctionData> (*)(ClientContext &, CopyFunctionBindInput &, const vector<string> &,
                                                    const vector<LogicalType> &);
using copy_to_initialize_global_t = unique_ptr<GlobalFunctionData> (*)(ClientContext &, FunctionData &,
                                                                      const string &);
using copy_to_initialize_local_t = unique_ptr<LocalFunctionData> (*)(ExecutionContext &, FunctionData &);
using copy_to_sink_t = void (*)(ExecutionContext &, FunctionData &, GlobalFunctionData &, LocalFunctionData &,
                                DataChunk &);
using copy_to_combine_t = void (*)(ExecutionContext &, FunctionData &, GlobalFunctionData &, LocalFunctionData &);
using copy_to_finalize_t = void (*)(ClientContext &, FunctionData &, GlobalFunctionData &);
enum class CopyFunctionExecutionMode : uint8_t { REGULAR_COPY_TO_FILE, PARALLEL_COPY_TO_FILE, BATCH_COPY_TO_FILE };
using copy_to_execution_mode_t = CopyFunctionExecutionMode (*)(bool preserve_insertion_order, bool supports_batch_index);
using copy_desired_batch_size_t = idx_t (*)(ClientContext &, FunctionData &);

// DuckDB common/optional_idx.hpp
class optional_idx {
public:
    optional_idx() = default;
    optional_idx(idx_t i) : i_(i) {}  // NOLINT (implicit like DuckDB)
    bool IsValid() const { return i_ != kInvalid; }
    idx_t GetIndex() const {
        if (!IsValid()) throw InternalException("Attempting to get the index of an optional_idx that is not set");
        return i_;
    }

private:
    static constexpr idx_t kInvalid = ~(idx_t)0;
    idx_t i_ = kInvalid;
};
// file rotation (v1.3.2 function/copy_function.hpp): rotate_files says the COPY
// writes a directory of files; rotate_next_file, asked before every sink, says
// the current file is complete
using copy_rotate_files_t = bool (*)(FunctionData &bind_data, const optional_idx &file_size_bytes);
using copy_rotate_next_file_t = bool (*)(GlobalFunctionData &gstate, FunctionData &bind_data,
                                         const optional_idx &file_size_bytes);

class CopyFunction {
public:
    explicit CopyFunction(string name) : name(std::move(name)) {}
    string name;
    string extension;
    copy_to_bind_t copy_to_bind = nullptr;
    copy_to_initialize_global_t copy_to_initialize_global = nullptr;
    copy_to_initialize_local_t copy_to_initialize_local = nullptr;
    copy_to_sink_t copy_to_sink = nullptr;
    copy_to_combine_t copy_to_combine = nullptr;
    copy_to_finalize_t copy_to_finalize = nullptr;
    copy_to_execution_mode_t execution_mode = nullptr;
    copy_desired_batch_size_t desired_batch_size = nullptr;
    copy_rotate_files_t rotate_files = nullptr;
    copy_rotate_next_file_t rotate_next_file = nullptr;
    std::function<TableFunction()> copy_from_function;  // COPY ... FROM
};

// ---- replacement scans -----------------------------------------------------
class ParsedExpression {
public:
    virtual ~ParsedExpression() = default;
};
class ConstantExpression : public ParsedExpression {
public:
    explicit ConstantExpression(Value v) : value(std::move(v)) {}
    Value value;
};
class FunctionExpression : public ParsedExpression {
public:
    FunctionExpression(string name, vector<unique_ptr<ParsedExpression>> children)
        : function_name(std::move(name)), children(std::move(children)) {}
    string function_name;
    vector<unique_ptr<ParsedExpression>> children;
};
class TableRef {
public:
    virtual ~TableRef() = default;
};
class TableFunctionRef : public TableRef {
public:
    unique_ptr<ParsedExpression> function;
};
struct ReplacementScanInput {
    string table_name;
};
struct ReplacementScanData {
    virtual ~ReplacementScanData() = default;
};
using replacement_scan_t = unique_ptr<TableRef> (*)(ClientContext &, ReplacementScanInput &,
                                                    optional_ptr<ReplacementScanData>);
struct ReplacementScan {
    ReplacementScan(replacement_scan_t fn) : function(fn) {}  // NOLINT
    replacement_scan_t function;
    static string GetFullPath(const ReplacementScanInput &input) { return input.table_name; }
};

struct DBConfig {
    vector<ReplacementScan> replacement_scans;
    static DBConfig &GetConfig(DatabaseInstance &db);
};

class DatabaseInstance {
public:
    DBConfig config;
    std::multimap<string, TableFunction> table_functions;
    std::multimap<string, ScalarFunction> scalar_functions;
    std::map<string, CopyFunction> copy_functions;
};

class DuckDB {
public:
    explicit DuckDB(DatabaseInstance &db) : instance(&db, [](DatabaseInstance *) {}) {}
    shared_ptr<DatabaseInstance> instance;
    static const char *LibraryVersion() { return "v1.3.2"; }
};

class Extension {
public:
    virtual ~Extension() = default;
    virtual void Load(DuckDB &db) = 0;
    virtual std::string Name() = 0;
    virtual std::string Version() const { return ""; }
};

struct ExtensionUtil {
    static void RegisterFunction(DatabaseInstance &db, TableFunction fn) {
        db.table_functions.emplace(fn.name, std::move(fn));
    }
    static void RegisterFunction(DatabaseInstance &db, ScalarFunction fn) {
        db.scalar_functions.emplace(fn.name, std::move(fn));
    }
    static void RegisterFunction(DatabaseInstance &db, CopyFunction fn) {
        db.copy_functions.emplace(fn.name, std::move(fn));
    }
};

struct StringUtil {
    static string Lower(const string &s);
    static string Upper(const string &s);
    static bool EndsWith(const string &s, const string &suffix) {
        return s.size() >= suffix.size() && s.compare(s.size() - suffix.size(), suffix.size(), suffix) == 0;
    }
};

}  // namespace duckdb

#ifndef DUCKDB_EXTENSION_API
#define DUCKDB_EXTENSION_API __attribute__((visibility("default")))
#endif
