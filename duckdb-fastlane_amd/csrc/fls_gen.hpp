// fls_gen.hpp -- seeded, counter-based synthetic workloads (host + device).
//
// The reference ships no data (its only fixture, third_party/fastlanes/data/
// fls/data.fls used by test/sql/fastlane.test:15-66, lives in an empty
// submodule), so every workload of BASELINE.json is generated here.  All
// values are pure functions of (seed, row), which lets
//   * the CPU writer encode any row-group shard independently (multi-GPU
//     sharding, parallel encode), and
//   * a GPU check kernel regenerate the ground truth next to the decoded
//     output at full size (1e9 rows, SF100) without a host copy.
// Integer codecs are lossless, so the generator output IS the expected decode.
//
// Workloads (BASELINE.json "configs"):
//   c1       INT32 "value" = 1,000,000 + U[0,128)              (FFOR, W=7)
//   lineitem TPC-H-like lineitem, 15 columns (l_comment excluded: FSST is a
//            later row); row counts match dbgen at SF 0.01/1/
//            10/100; value distributions follow the TPC-H spec (4.2.3).
//   c3       INT64 sorted keys, orderkey model (1-7 rows per key, keys dense in
//            blocks of 8 per 32)                                (DELTA)
//   c4       VARCHAR l_shipmode-like, uniform over 7 values     (DICT, W=3)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#define FLS_HD __host__ __device__ __forceinline__

namespace fls {
namespace gen {

constexpr uint64_t kSeed = 42;

// stream ids (one independent random stream per attribute)
enum Stream : uint32_t {
    S_NLINES = 1, S_PART = 2, S_SUPP = 3, S_QTY = 4, S_DISC = 5, S_TAX = 6,
    S_ODATE = 7, S_SDATE = 8, S_CDATE = 9, S_RDATE = 10, S_RFLAG = 11,
    S_INSTR = 12, S_MODE = 13, S_C1 = 20, S_C4 = 21,
};

FLS_HD uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
FLS_HD uint64_t rnd(uint64_t seed, uint32_t stream, uint64_t ctr) {
    return mix64(ctr * 0xD1342543DE82EF95ull + (seed * 0x632BE59BD9B4E019ull ^ (uint64_t)stream << 40));
}
// uniform integer in [lo, hi] (inclusive); 64-bit modulo bias is negligible here
FLS_HD int64_t uni(uint64_t r, int64_t lo, int64_t hi) {
    return lo + (int64_t)(r % (uint64_t)(hi - lo + 1));
}

// ---- orders model: blocks of 8 orders hold exactly 32 lineitems ----------
// Each order has 1..7 lines (mean 4, TPC-H 4.2.3: O_ORDERKEY has 1-7 lines);
// orderkeys are dense 8 per 32 (TPC-H sparse key space).  A block's line
// counts are a random composition of 32 into 8 parts in [1,7] obtained from
// 20 random unit transfers out of (4,...,4); this keeps row -> order O(8).
FLS_HD void block_lines(uint64_t seed, uint64_t blk, uint32_t n[8]) {
    for (int i = 0; i < 8; ++i) n[i] = 4;
    uint64_t r = rnd(seed, S_NLINES, blk);
    uint64_t r2 = rnd(seed, S_NLINES, blk ^ 0x8000000000000000ull);
    for (int j = 0; j < 20; ++j) {
        uint64_t src = j < 10 ? r : r2;
        int sh = 6 * (j % 10);
        uint32_t a = (uint32_t)(src >> sh) & 7u, b = (uint32_t)(src >> (sh + 3)) & 7u;
        if (a != b && n[a] > 1 && n[b] < 7) { n[a]--; n[b]++; }
    }
}
struct OrderPos {
    uint64_t order;    // 0-based order index
    uint32_t line;     // 0-based line number within the order
};
FLS_HD OrderPos row_order(uint64_t seed, uint64_t row) {
    uint64_t blk = row >> 5;
    uint32_t pos = (uint32_t)(row & 31);
    uint32_t n[8];
    block_lines(seed, blk, n);
    uint32_t o = 0;
    while (pos >= n[o]) { pos -= n[o]; ++o; }
    return OrderPos{blk * 8 + o, pos};
}
FLS_HD int64_t orderkey(uint64_t order) { return (int64_t)((order >> 3) * 32 + (order & 7) + 1); }

// ---- lineitem ----------------------------------------------------------
constexpr int32_t kStartDate = 8035;    // 1992-01-01 (days since 1970-01-01)
constexpr int32_t kEndDate = 10591;     // 1998-12-31
constexpr int32_t kCurrentDate = 9298;  // 1995-06-17

struct LineitemParams {
    uint64_t seed;
    uint64_t nrows;   // total rows
    int64_t n_part;   // SF * 200,000
    int64_t n_supp;   // SF * 10,000
};

struct LineitemRow {
    int64_t orderkey;
    int32_t partkey, suppkey, linenumber;
    int64_t quantity, extendedprice, discount, tax;  // DECIMAL(15,2) cents
    uint32_t returnflag, linestatus;                 // dictionary codes
    int32_t shipdate, commitdate, receiptdate;
    uint32_t shipinstruct, shipmode;
};

constexpr int kLineitemCols = 15;

FLS_HD void lineitem_row_at(const LineitemParams &p, uint64_t row, OrderPos op, LineitemRow &o) {
    o.orderkey = orderkey(op.order);
    o.linenumber = (int32_t)op.line + 1;
    const int64_t pk = uni(rnd(p.seed, S_PART, row), 1, p.n_part);
    o.partkey = (int32_t)pk;
    // TPC-H 4.2.3: supplier i of part: (P + (i * (S/4 + (P-1)/S))) mod S + 1
    const int64_t S = p.n_supp;
    const int64_t i = uni(rnd(p.seed, S_SUPP, row), 0, 3);
    o.suppkey = (int32_t)((pk + (i * (S / 4 + (pk - 1) / S))) % S + 1);
    const int64_t qty = uni(rnd(p.seed, S_QTY, row), 1, 50);
    o.quantity = qty * 100;
    // P_RETAILPRICE = (90000 + ((P/10) mod 20001) + 100 * (P mod 1000)) / 100
    const int64_t rp = 90000 + ((pk / 10) % 20001) + 100 * (pk % 1000);
    o.extendedprice = qty * rp;
    o.discount = uni(rnd(p.seed, S_DISC, row), 0, 10);
    o.tax = uni(rnd(p.seed, S_TAX, row), 0, 8);
    const int32_t odate = (int32_t)uni(rnd(p.seed, S_ODATE, op.order), kStartDate, kEndDate - 151);
    o.shipdate = odate + (int32_t)uni(rnd(p.seed, S_SDATE, row), 1, 121);
    o.commitdate = odate + (int32_t)uni(rnd(p.seed, S_CDATE, row), 30, 90);
    o.receiptdate = o.shipdate + (int32_t)uni(rnd(p.seed, S_RDATE, row), 1, 30);
    // returnflag dict {A,N,R}; linestatus dict {F,O}
    o.returnflag = o.receiptdate <= kCurrentDate ? ((rnd(p.seed, S_RFLAG, row) & 1) ? 2u : 0u) : 1u;
    o.linestatus = o.shipdate > kCurrentDate ? 1u : 0u;
    o.shipinstruct = (uint32_t)uni(rnd(p.seed, S_INSTR, row), 0, 3);
    o.shipmode = (uint32_t)uni(rnd(p.seed, S_MODE, row), 0, 6);
}
FLS_HD void lineitem_row(const LineitemParams &p, uint64_t row, LineitemRow &o) {
    lineitem_row_at(p, row, row_order(p.seed, row), o);
}

// Sequential walk over rows: block line counts computed once per 32 rows.
struct OrderWalker {
    uint64_t seed, blk;
    uint32_t n[8], o, pos;
    FLS_HD void start(uint64_t s, uint64_t row) {
        seed = s;
        blk = row >> 5;
        block_lines(seed, blk, n);
        pos = (uint32_t)(row & 31);
        o = 0;
        while (pos >= n[o]) { pos -= n[o]; ++o; }
    }
    FLS_HD OrderPos cur() const { return OrderPos{blk * 8 + o, pos}; }
    FLS_HD void next() {
        if (++pos >= n[o]) {
            pos = 0;
            if (++o == 8) { o = 0; ++blk; block_lines(seed, blk, n); }
        }
    }
};

// raw column value (integers: value; VARCHAR: dictionary code)
FLS_HD int64_t lineitem_col(const LineitemRow &o, int col) {
    switch (col) {
    case 0: return o.orderkey;
    case 1: return o.partkey;
    case 2: return o.suppkey;
    case 3: return o.linenumber;
    case 4: return o.quantity;
    case 5: return o.extendedprice;
    case 6: return o.discount;
    case 7: return o.tax;
    case 8: return o.returnflag;
    case 9: return o.linestatus;
    case 10: return o.shipdate;
    case 11: return o.commitdate;
    case 12: return o.receiptdate;
    case 13: return o.shipinstruct;
    default: return o.shipmode;
    }
}

// ---- single-column workloads -------------------------------------------
FLS_HD int64_t c1_value(uint64_t seed, uint64_t row) { return 1000000 + uni(rnd(seed, S_C1, row), 0, 127); }
FLS_HD int64_t c3_value(uint64_t seed, uint64_t row) { return orderkey(row_order(seed, row).order); }
FLS_HD int64_t c4_code(uint64_t seed, uint64_t row) { return uni(rnd(seed, S_C4, row), 0, 6); }

}  // namespace gen
}  // namespace fls
