// fls_alp.hpp -- ALP decimal-exponent constants shared by the encoder (host),
// the decoder (device) and, as a literal copy, the oracle.
//
// ALP (Afroozeh, Kuffo, Boncz, "ALP: Adaptive Lossless floating-Point
// Compression", SIGMOD 2024) stores a double n as the integer
// d = round(n * 10^e * 10^-f) when (double)d * 10^f * 10^-e reproduces n
// bit for bit, otherwise as an exception.  Decode multiplies left to right in
// the value's own precision; the encoder verifies with exactly that
// expression, so every IEEE-correct implementation (x86 SSE2, gfx950 VALU)
// reproduces the original bits.
#pragma once

// 10^i, exact in binary64 for i <= 22 (binary32 for i <= 10)
#define FLS_ALP_F10_D                                                                                        \
    1.0, 10.0, 100.0, 1000.0, 10000.0, 100000.0, 1000000.0, 10000000.0, 100000000.0, 1000000000.0,          \
        10000000000.0, 100000000000.0, 1000000000000.0, 10000000000000.0, 100000000000000.0,                 \
        1000000000000000.0, 10000000000000000.0, 100000000000000000.0, 1000000000000000000.0
// nearest binary64 to 10^-i
#define FLS_ALP_IF10_D                                                                                       \
    1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001, 0.0000000001,     \
        0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001, 0.000000000000001,                \
        0.0000000000000001, 0.00000000000000001, 0.000000000000000001
#define FLS_ALP_F10_F                                                                                        \
    1.0f, 10.0f, 100.0f, 1000.0f, 10000.0f, 100000.0f, 1000000.0f, 10000000.0f, 100000000.0f,                \
        1000000000.0f, 10000000000.0f
#define FLS_ALP_IF10_F                                                                                       \
    1.0f, 0.1f, 0.01f, 0.001f, 0.0001f, 0.00001f, 0.000001f, 0.0000001f, 0.00000001f, 0.000000001f,         \
        0.0000000001f

namespace fls {
constexpr int kAlpMaxExpD = 18;  // exponents 0..18 for DOUBLE
constexpr int kAlpMaxExpF = 10;  // exponents 0..10 for FLOAT
}  // namespace fls
