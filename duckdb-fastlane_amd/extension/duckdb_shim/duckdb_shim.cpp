// duckdb_shim.cpp -- implementation of the DuckDB v1.3.2 API slice declared in
// duckdb_shim_core.hpp (flat vectors, Value -> VARCHAR casts, string heap).
#include <algorithm>
#include <cctype>
#include <cstdio>

#include "duckdb_shim_core.hpp"

namespace duckdb {

const LogicalType LogicalType::SQLNULL(LogicalTypeId::SQLNULL);
const LogicalType LogicalType::BOOLEAN(LogicalTypeId::BOOLEAN);
const LogicalType LogicalType::TINYINT(LogicalTypeId::TINYINT);
const LogicalType LogicalType::SMALLINT(LogicalTypeId::SMALLINT);
const LogicalType LogicalType::INTEGER(LogicalTypeId::INTEGER);
const LogicalType LogicalType::BIGINT(LogicalTypeId::BIGINT);
const LogicalType LogicalType::UTINYINT(LogicalTypeId::UTINYINT);
const LogicalType LogicalType::USMALLINT(LogicalTypeId::USMALLINT);
const LogicalType LogicalType::UINTEGER(LogicalTypeId::UINTEGER);
const LogicalType LogicalType::UBIGINT(LogicalTypeId::UBIGINT);
const LogicalType LogicalType::DATE(LogicalTypeId::DATE);
const LogicalType LogicalType::FLOAT(LogicalTypeId::FLOAT);
const LogicalType LogicalType::DOUBLE(LogicalTypeId::DOUBLE);
const LogicalType LogicalType::VARCHAR(LogicalTypeId::VARCHAR);
const LogicalType LogicalType::BLOB(LogicalTypeId::BLOB);
const LogicalType LogicalType::BIT(LogicalTypeId::BIT);

idx_t LogicalType::PhysicalSize() const {
    switch (id_) {
    case LogicalTypeId::BOOLEAN: case LogicalTypeId::TINYINT: case LogicalTypeId::UTINYINT: return 1;
    case LogicalTypeId::SMALLINT: case LogicalTypeId::USMALLINT: return 2;
    case LogicalTypeId::INTEGER: case LogicalTypeId::UINTEGER: case LogicalTypeId::DATE:
    case LogicalTypeId::FLOAT: return 4;
    case LogicalTypeId::BIGINT: case LogicalTypeId::UBIGINT: case LogicalTypeId::DOUBLE: return 8;
    case LogicalTypeId::DECIMAL: return width_ <= 4 ? 2 : width_ <= 9 ? 4 : 8;
    case LogicalTypeId::VARCHAR: case LogicalTypeId::CHAR: case LogicalTypeId::BLOB: case LogicalTypeId::BIT: return 16;
    default: return 8;
    }
}

string LogicalType::ToString() const {
    switch (id_) {
    case LogicalTypeId::SQLNULL: return "NULL";
    case LogicalTypeId::BOOLEAN: return "BOOLEAN";
    case LogicalTypeId::TINYINT: return "TINYINT";
    case LogicalTypeId::SMALLINT: return "SMALLINT";
    case LogicalTypeId::INTEGER: return "INTEGER";
    case LogicalTypeId::BIGINT: return "BIGINT";
    case LogicalTypeId::UTINYINT: return "UTINYINT";
    case LogicalTypeId::USMALLINT: return "USMALLINT";
    case LogicalTypeId::UINTEGER: return "UINTEGER";
    case LogicalTypeId::UBIGINT: return "UBIGINT";
    case LogicalTypeId::DATE: return "DATE";
    case LogicalTypeId::FLOAT: return "FLOAT";
    case LogicalTypeId::DOUBLE: return "DOUBLE";
    case LogicalTypeId::DECIMAL: return "DECIMAL(" + std::to_string(width_) + "," + std::to_string(scale_) + ")";
    case LogicalTypeId::VARCHAR: return "VARCHAR";
    case LogicalTypeId::CHAR: return "CHAR";
    case LogicalTypeId::BLOB: return "BLOB";
    case LogicalTypeId::BIT: return "BIT";
    case LogicalTypeId::LIST: return (child_ ? child_->ToString() : string("?")) + "[]";
    default: return "INVALID";
    }
}

namespace {

// civil-from-days (Howard Hinnant), DuckDB renders DATE as YYYY-MM-DD
string date_to_string(int32_t days) {
    int64_t z = (int64_t)days + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const unsigned doe = (unsigned)(z - era * 146097);
    const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = (int64_t)yoe + era * 400;
    const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const unsigned mp = (5 * doy + 2) / 153;
    const unsigned d = doy - (153 * mp + 2) / 5 + 1;
    const unsigned m = mp < 10 ? mp + 3 : mp - 9;
    y += (m <= 2);
    char buf[32];
    snprintf(buf, sizeof(buf), "%04lld-%02u-%02u", (long long)y, m, d);
    return buf;
}

string decimal_to_string(int64_t v, uint8_t scale) {
    if (scale == 0) return std::to_string(v);
    const bool neg = v < 0;
    uint64_t a = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    uint64_t p = 1;
    for (int i = 0; i < scale; ++i) p *= 10;
    string frac = std::to_string(a % p);
    frac.insert(0, scale - frac.size(), '0');
    return (neg ? "-" : "") + std::to_string(a / p) + "." + frac;
}

// DuckDB's Blob::ToString: printable ASCII as is, other bytes (and the
// quote and backslash characters) as \xHH
string blob_to_string(const string &b) {
    static const char *hex = "0123456789ABCDEF";
    string r;
    for (unsigned char c : b) {
        if (c >= 32 && c <= 126 && c != '\\' && c != '\'' && c != '"') {
            r += (char)c;
        } else {
            r += "\\x";
            r += hex[c >> 4];
            r += hex[c & 15];
        }
    }
    return r;
}

// DuckDB's Bit::ToString: the bits after the padding, most significant first
string bit_to_string(const string &b) {
    string r;
    if (b.size() < 2) return r;
    const unsigned pad = (uint8_t)b[0];
    for (size_t i = pad; i < 8 * (b.size() - 1); ++i) r += ((uint8_t)b[1 + i / 8] >> (7 - i % 8)) & 1 ? '1' : '0';
    return r;
}

// DuckDB prints doubles with the shortest round-tripping representation
string double_to_string(double v) {
    char buf[64];
    for (int prec = 1; prec <= 17; ++prec) {
        snprintf(buf, sizeof(buf), "%.*g", prec, v);
        if (strtod(buf, nullptr) == v) break;
    }
    return buf;
}

}  // namespace

string Value::ToString() const {
    if (is_null_) return "NULL";
    switch (type_.id()) {
    case LogicalTypeId::VARCHAR: case LogicalTypeId::CHAR: return str_;
    case LogicalTypeId::BLOB: return blob_to_string(str_);
    case LogicalTypeId::BIT: return bit_to_string(str_);
    case LogicalTypeId::BOOLEAN: return int_ ? "true" : "false";
    case LogicalTypeId::UBIGINT: return std::to_string((uint64_t)int_);
    case LogicalTypeId::DATE: return date_to_string((int32_t)int_);
    case LogicalTypeId::DECIMAL: return decimal_to_string(int_, type_.Scale());
    case LogicalTypeId::FLOAT: return double_to_string((float)dbl_);
    case LogicalTypeId::DOUBLE: return double_to_string(dbl_);
    case LogicalTypeId::LIST: {
        string s = "[";
        for (size_t i = 0; i < list_.size(); ++i) s += (i ? ", " : "") + list_[i].ToString();
        return s + "]";
    }
    default: return std::to_string(int_);
    }
}

Vector::Vector(LogicalType type, idx_t capacity)
    : type_(std::move(type)), capacity_(capacity), data_(capacity * type_.PhysicalSize(), 0),
      data_ptr_(data_.data()), validity_(capacity) {}

Vector::Vector(LogicalType type, data_ptr_t data)
    : type_(std::move(type)), capacity_(STANDARD_VECTOR_SIZE), data_ptr_(data), validity_(STANDARD_VECTOR_SIZE) {}

void Vector::Slice(const Vector &other, const SelectionVector &sel, idx_t count) {
    auto child = std::make_shared<Vector>(other.GetType(), (idx_t)0);
    child->Reference(other);
    Reset();
    type_ = other.GetType();
    child_ = std::move(child);
    dict_sel_ = sel;
    vtype_ = VectorType::DICTIONARY_VECTOR;
    (void)count;
}

void Vector::Flatten(idx_t count) {
    if (vtype_ != VectorType::DICTIONARY_VECTOR) return;
    const idx_t w = type_.PhysicalSize();
    std::shared_ptr<Vector> child = std::move(child_);
    const SelectionVector sel = dict_sel_;
    Reset();  // own storage, all valid
    if (data_.size() < count * w) data_.resize(count * w);
    capacity_ = std::max(capacity_, count);
    data_ptr_ = data_.data();
    // typed gathers (DuckDB's flatten is a typed copy too)
    const uint8_t *src = child->GetData();
    auto gather = [&](auto x) {
        using T = decltype(x);
        T *d = reinterpret_cast<T *>(data_ptr_);
        const T *c = reinterpret_cast<const T *>(src);
        for (idx_t i = 0; i < count; ++i) d[i] = c[sel.get_index(i)];
    };
    switch (w) {
    case 1: gather(uint8_t()); break;
    case 2: gather(uint16_t()); break;
    case 4: gather(uint32_t()); break;
    case 8: gather(uint64_t()); break;
    case 16: gather(string_t()); break;
    default:
        for (idx_t i = 0; i < count; ++i) memcpy(data_ptr_ + i * w, src + sel.get_index(i) * w, w);
    }
    if (!child->Validity().AllValid())
        for (idx_t i = 0; i < count; ++i)
            if (!child->RowIsValid(sel.get_index(i))) validity_.SetInvalid(i);
    keep_.push_back(child);  // strings still point into the dictionary's memory
}

Vector::Vector(Vector &&o) noexcept
    : type_(std::move(o.type_)), capacity_(o.capacity_), data_(std::move(o.data_)), auxiliary_(std::move(o.auxiliary_)),
      validity_(std::move(o.validity_)), child_(std::move(o.child_)), dict_sel_(std::move(o.dict_sel_)),
      heap_(std::move(o.heap_)), keep_(std::move(o.keep_)), vtype_(o.vtype_) {
    // a moved std::vector keeps its storage, so an owned data pointer stays valid
    data_ptr_ = o.data_ptr_;
    o.data_ptr_ = nullptr;
}

// DataChunk::Reset -> Vector::ResetFromCache in DuckDB: back to the vector's
// own buffer, dropping any foreign data pointer and its auxiliary holder
void Vector::Reset() {
    data_ptr_ = data_.data();
    auxiliary_.reset();
    validity_.Reset();
    child_.reset();
    dict_sel_ = SelectionVector();
    heap_.clear();
    keep_.clear();
    vtype_ = VectorType::FLAT_VECTOR;
}

void Vector::Reference(const Vector &o) {
    if (o.vtype_ == VectorType::DICTIONARY_VECTOR) {  // share the dictionary and the selection
        type_ = o.type_;
        child_ = o.child_;
        dict_sel_ = o.dict_sel_;
        vtype_ = o.vtype_;
        return;
    }
    type_ = o.type_;
    validity_ = o.validity_;  // shared words, as DuckDB's Reference shares the validity buffer
    vtype_ = o.vtype_;
    if (o.auxiliary_) {  // foreign data kept alive by its holder: share it
        data_ptr_ = o.data_ptr_;
        auxiliary_ = o.auxiliary_;
        return;
    }
    const size_t w = type_.PhysicalSize();
    data_.assign(o.data_ptr_, o.data_ptr_ + o.capacity_ * w);
    capacity_ = o.capacity_;
    data_ptr_ = data_.data();
    keep_ = o.keep_;
    if (type_.PhysicalSize() == 16 && type_.id() != LogicalTypeId::DECIMAL &&
        type_.id() != LogicalTypeId::LIST) {  // strings of o's heap into this one's
        string_t *sv = reinterpret_cast<string_t *>(data_ptr_);
        for (idx_t i = 0; i < capacity_; ++i)
            if (validity_.RowIsValid(i) && sv[i].GetSize() > string_t::INLINE_LENGTH) sv[i] = AddString(sv[i].GetString());
    }
}

string_t Vector::AddString(const string &s) {
    if (s.size() <= string_t::INLINE_LENGTH) return string_t(s.data(), (uint32_t)s.size());
    heap_.push_back(s);
    return string_t(heap_.back().data(), (uint32_t)heap_.back().size());
}

void Vector::SetValue(idx_t i, const Value &v) {
    if (i >= capacity_) throw InternalException("Vector::SetValue out of range");
    if (v.IsNull()) {
        validity_.SetInvalid(i);
        return;
    }
    validity_.SetValid(i);
    uint8_t *p = data_ptr_ + i * type_.PhysicalSize();
    switch (type_.id()) {
    case LogicalTypeId::VARCHAR: case LogicalTypeId::CHAR: {
        // implicit cast to VARCHAR, as DuckDB's Vector::SetValue does
        string_t s = AddString(v.GetValue<string>());
        memcpy(p, &s, sizeof(s));
        break;
    }
    case LogicalTypeId::BLOB: case LogicalTypeId::BIT: {
        if (v.type().id() != type_.id())
            throw InternalException("Vector::SetValue: " + type_.ToString() + " needs a " + type_.ToString() + " value");
        string_t s = AddString(StringValue::Get(v));
        memcpy(p, &s, sizeof(s));
        break;
    }
    case LogicalTypeId::FLOAT: { float f = (float)v.GetDouble(); memcpy(p, &f, 4); break; }
    case LogicalTypeId::DOUBLE: { double d = v.GetDouble(); memcpy(p, &d, 8); break; }
    default: {
        int64_t x = v.GetInt64();
        memcpy(p, &x, type_.PhysicalSize());
    }
    }
}

Value Vector::GetValue(idx_t i) const {
    if (vtype_ == VectorType::DICTIONARY_VECTOR) return child_->GetValue(dict_sel_.get_index(i));
    if (!validity_.RowIsValid(i)) return Value();
    const uint8_t *p = data_ptr_ + i * type_.PhysicalSize();
    auto ld = [p](auto x) { memcpy(&x, p, sizeof(x)); return x; };
    switch (type_.id()) {
    case LogicalTypeId::VARCHAR: case LogicalTypeId::CHAR: return Value(ld(string_t()).GetString());
    case LogicalTypeId::BLOB: {
        const string_t s = ld(string_t());
        return Value::BLOB((const uint8_t *)s.GetData(), s.GetSize());
    }
    case LogicalTypeId::BIT: {
        const string_t s = ld(string_t());
        return Value::BIT((const uint8_t *)s.GetData(), s.GetSize());
    }
    case LogicalTypeId::BOOLEAN: return Value::BOOLEAN(ld(uint8_t()) != 0);
    case LogicalTypeId::TINYINT: return Value::TINYINT(ld(int8_t()));
    case LogicalTypeId::SMALLINT: return Value::SMALLINT(ld(int16_t()));
    case LogicalTypeId::INTEGER: return Value::INTEGER(ld(int32_t()));
    case LogicalTypeId::BIGINT: return Value::BIGINT(ld(int64_t()));
    case LogicalTypeId::UTINYINT: return Value::UTINYINT(ld(uint8_t()));
    case LogicalTypeId::USMALLINT: return Value::USMALLINT(ld(uint16_t()));
    case LogicalTypeId::UINTEGER: return Value::UINTEGER(ld(uint32_t()));
    case LogicalTypeId::UBIGINT: return Value::UBIGINT(ld(uint64_t()));
    case LogicalTypeId::DATE: return Value::DATE(date_t{ld(int32_t())});
    case LogicalTypeId::FLOAT: return Value::FLOAT(ld(float()));
    case LogicalTypeId::DOUBLE: return Value::DOUBLE(ld(double()));
    case LogicalTypeId::DECIMAL: {
        const idx_t w = type_.PhysicalSize();
        int64_t x = w == 2 ? ld(int16_t()) : w == 4 ? ld(int32_t()) : ld(int64_t());
        return Value::DECIMAL(x, type_.Width(), type_.Scale());
    }
    default: return Value();
    }
}

DBConfig &DBConfig::GetConfig(DatabaseInstance &db) { return db.config; }

string StringUtil::Upper(const string &s) {
    string r(s);
    std::transform(r.begin(), r.end(), r.begin(), [](unsigned char c) { return (char)std::toupper(c); });
    return r;
}

string StringUtil::Lower(const string &s) {
    string r(s);
    std::transform(r.begin(), r.end(), r.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    return r;
}

}  // namespace duckdb

// ---- residual filters ------------------------------------------------------
namespace duckdb {

namespace {
const SelectionVector &incremental_sel() {
    static const SelectionVector s;  // empty: identity
    return s;
}

// -1 / 0 / 1 for comparable non-null values of one logical type
int compare_values(const Value &a, const Value &b) {
    switch (a.type().id()) {
    case LogicalTypeId::BLOB: {
        const string &x = StringValue::Get(a), &y = StringValue::Get(b);  // bytes compare as unsigned (memcmp)
        return x < y ? -1 : x > y ? 1 : 0;
    }
    case LogicalTypeId::VARCHAR: {
        const string x = a.GetValue<string>(), y = b.GetValue<string>();
        return x < y ? -1 : x > y ? 1 : 0;
    }
    case LogicalTypeId::FLOAT: case LogicalTypeId::DOUBLE: {
        const double x = a.GetDouble(), y = b.GetDouble();
        if (x != x || y != y) return (x != x) - (y != y);  // NaN sorts above everything, NaN = NaN
        return x < y ? -1 : x > y ? 1 : 0;
    }
    case LogicalTypeId::UBIGINT: {
        const uint64_t x = a.GetValue<uint64_t>(), y = b.GetValue<uint64_t>();
        return x < y ? -1 : x > y ? 1 : 0;
    }
    default: {
        const int64_t x = a.GetInt64(), y = b.GetInt64();
        return x < y ? -1 : x > y ? 1 : 0;
    }
    }
}

bool eval_filter(const TableFilter &f, const Value &v) {
    switch (f.filter_type) {
    case TableFilterType::IS_NULL: return v.IsNull();
    case TableFilterType::IS_NOT_NULL: return !v.IsNull();
    case TableFilterType::CONSTANT_COMPARISON: {
        auto &c = f.Cast<ConstantFilter>();
        if (v.IsNull() || c.constant.IsNull()) return false;
        const int r = compare_values(v, c.constant);
        switch (c.comparison_type) {
        case ExpressionType::COMPARE_EQUAL: return r == 0;
        case ExpressionType::COMPARE_NOTEQUAL: return r != 0;
        case ExpressionType::COMPARE_LESSTHAN: return r < 0;
        case ExpressionType::COMPARE_LESSTHANOREQUALTO: return r <= 0;
        case ExpressionType::COMPARE_GREATERTHAN: return r > 0;
        case ExpressionType::COMPARE_GREATERTHANOREQUALTO: return r >= 0;
        }
        return false;
    }
    case TableFilterType::IN_FILTER:
        if (v.IsNull()) return false;
        for (auto &x : f.Cast<InFilter>().values)
            if (!x.IsNull() && compare_values(v, x) == 0) return true;
        return false;
    case TableFilterType::CONJUNCTION_AND:
        for (auto &ch : f.Cast<ConjunctionAndFilter>().child_filters)
            if (!eval_filter(*ch, v)) return false;
        return true;
    case TableFilterType::CONJUNCTION_OR:
        for (auto &ch : f.Cast<ConjunctionOrFilter>().child_filters)
            if (eval_filter(*ch, v)) return true;
        return false;
    case TableFilterType::EXPRESSION_FILTER: return f.Cast<ExpressionFilter>().expr->EvaluateRow(v);
    default: return true;  // optional / dynamic: may be skipped, DuckDB re-checks above the scan
    }
}
}  // namespace

void Vector::ToUnifiedFormat(idx_t, UnifiedVectorFormat &format) const {
    if (vtype_ == VectorType::DICTIONARY_VECTOR) {
        format.sel = &dict_sel_;
        format.data = child_->GetData();
        format.validity = child_->Validity();
        return;
    }
    format.sel = &incremental_sel();
    format.data = GetData();
    format.validity = validity_;
}

unique_ptr<TableFilterState> TableFilterState::Initialize(ClientContext &, const TableFilter &) {
    return make_uniq<TableFilterState>();
}

idx_t ColumnSegment::FilterSelection(SelectionVector &sel, Vector &vector, UnifiedVectorFormat &, const TableFilter &filter,
                                     TableFilterState &, idx_t, idx_t &approved_tuple_count) {
    // as DuckDB's: reads the incoming selection (rows 0..approved-1 of it,
    // so every one of them must be set) and hands back a new one
    SelectionVector new_sel(approved_tuple_count);
    idx_t kept = 0;
    for (idx_t i = 0; i < approved_tuple_count; ++i) {
        const idx_t row = sel.get_index(i);
        if (row >= vector.Capacity()) throw InternalException("FilterSelection: selection index out of range");
        if (eval_filter(filter, vector.GetValue(row))) new_sel.set_index(kept++, row);
    }
    sel.Initialize(new_sel);
    approved_tuple_count = kept;
    return kept;
}

void DataChunk::Slice(const SelectionVector &sel, idx_t count) {
    vector<Vector> nd;
    nd.reserve(data.size());
    for (auto &v : data) {
        Vector nv(v.GetType());
        for (idx_t i = 0; i < count; ++i) nv.SetValue(i, v.GetValue(sel.get_index(i)));
        nd.push_back(std::move(nv));
    }
    data.swap(nd);
    count_ = count;
}

}  // namespace duckdb
