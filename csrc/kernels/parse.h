// Device-side parsers of Hivemall feature strings (shared by ingest.hip and its probes).
// Semantics are those of the host parser (csrc/host/hashing.cpp parse_int / parse_float):
// integers exactly, decimals only when the result is provably the host's (float)strtod.
#pragma once
#include <stdint.h>

namespace hm {

__device__ __forceinline__ bool dev_parse_int(const uint8_t* p, int n, int64_t* out) {
    if (n <= 0 || n > 19) return false;
    int i = 0;
    bool neg = false;
    if (p[0] == '-' || p[0] == '+') { neg = p[0] == '-'; i = 1; if (n == 1) return false; }
    int64_t v = 0;
    for (; i < n; ++i) {
        const int c = p[i];
        if (c < '0' || c > '9') return false;
        v = v * 10 + (c - '0');
    }
    *out = neg ? -v : v;
    return true;
}

// Decimal "[+-]digits[.digits][(e|E)[+-]digits]" -> float, through double like strtod.  Exact
// (Clinger fast path: mantissa < 2^53, |power of ten| <= 22, one correctly rounded double
// operation) or refused, so the result always equals the host's (float)strtod.  Written as
// three straight scans (find the exponent marker, mantissa, exponent): the single-loop form
// with a mid-loop break refused every exponent on gfx950 (benchmarks/parse_probe.py).
__device__ __forceinline__ bool dev_parse_float(const uint8_t* p, int n, float* out) {
    if (n <= 0 || n > 63) return false;
    int ep = n;                                   // exponent marker position (n = none)
    for (int i = 0; i < n; ++i) {
        const int c = p[i];
        if (c == 'e' || c == 'E') { ep = i; break; }
    }
    int i = 0;
    bool neg = false;
    if (p[0] == '-' || p[0] == '+') { neg = p[0] == '-'; i = 1; }
    uint64_t m = 0;
    int digits = 0, frac = 0, nd = 0;
    bool dot = false;
    for (; i < ep; ++i) {
        const int c = p[i];
        if (c == '.') {
            if (dot) return false;
            dot = true;
            continue;
        }
        const unsigned d = (unsigned)(c - '0');
        if (d > 9u) return false;
        ++nd;
        if (dot) ++frac;
        if (m == 0 && d == 0) continue;           // leading zeros
        if (++digits > 19) return false;
        m = m * 10 + d;
    }
    if (nd == 0) return false;
    int e10 = 0;
    if (ep < n) {
        int j = ep + 1;
        bool eneg = false;
        if (j < n && (p[j] == '-' || p[j] == '+')) { eneg = p[j] == '-'; ++j; }
        if (j >= n || n - j > 4) return false;    // |exponent| < 10^4 (the fast path needs <= 22)
        for (; j < n; ++j) {
            const unsigned d = (unsigned)(p[j] - '0');
            if (d > 9u) return false;
            e10 = e10 * 10 + (int)d;
        }
        if (eneg) e10 = -e10;
    }
    const int e = e10 - frac;
    if (m >= (1ull << 53) || e > 22 || e < -22) return false;
    double pw = 1.0;                              // 10^|e| <= 10^22: every step exact
    for (int k = e < 0 ? -e : e; k > 0; --k) pw *= 10.0;
    double d = (double)m;
    d = e >= 0 ? d * pw : d / pw;
    *out = (float)(neg ? -d : d);
    return true;
}

__device__ __forceinline__ int find_colon(const uint8_t* s, int len, int from) {
    for (int i = from; i < len; ++i)
        if (s[i] == ':') return i;
    return -1;
}

}  // namespace hm
