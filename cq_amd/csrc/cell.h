// cell.h -- typed CSV cell semantics of the reference cq, as device functions.
//
// Everything the SELECT hot path needs to turn raw CSV field bytes into the
// reference's typed values and to compare/aggregate them bit-exactly:
//   * parse_cell      infer_type + parse_value   (reference csv_reader.c:133-240)
//   * parse_date      sscanf("%d-%d-%d" ...)      (reference date_utils.c:26-100)
//   * to_int / to_dbl strtoll / strtod           (correctly rounded: Clinger fast
//                     path, Eisel-Lemire 128-bit product, exact big-integer
//                     midpoint comparison for >19-digit significands)
//   * compare         value_compare              (reference csv_reader.c:98-130)
//   * arith           binary/unary arithmetic    (evaluator_expressions.c:101-263)
//   * group key       printf-canonical key identity (evaluator_aggregates.c:122-141)
//
// Compiled twice: by hipcc for gfx950 (CQ_HD = __device__) inside the kernels,
// and by g++ for the host unit tests (tests/test_cell_host.py), which check this
// exact code against glibc strtod/strtoll/sscanf on millions of inputs.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CQ_HD __device__ __forceinline__
#define CQ_HDM __device__ __forceinline__     // member functions
#define CQ_POW5_ATTR static __device__
#else
#define CQ_HD static inline
#define CQ_HDM inline
#define CQ_POW5_ATTR static
#endif

#include "pow5_table.h"

namespace cq {

enum : uint32_t { K_NULL = 0, K_INT = 1, K_DBL = 2, K_STR = 3, K_DATE = 4 };

// One typed cell. STRING: bits = address of the first (trimmed) byte, len = bytes.
// DATE: bits = y << 32 | m << 16 | d.  INT/DBL: bits = the 64-bit pattern.
struct Cell {
    uint32_t kind;
    uint32_t len;
    uint64_t bits;
};

CQ_HD Cell cell_null() { Cell c; c.kind = K_NULL; c.len = 0; c.bits = 0; return c; }
CQ_HD Cell cell_int(int64_t v) { Cell c; c.kind = K_INT; c.len = 0; c.bits = (uint64_t)v; return c; }
CQ_HD Cell cell_dbl(double v) {
    Cell c; c.kind = K_DBL; c.len = 0;
    union { double d; uint64_t u; } x; x.d = v; c.bits = x.u;
    return c;
}
CQ_HD double as_dbl(uint64_t b) { union { double d; uint64_t u; } x; x.u = b; return x.d; }
CQ_HD uint64_t dbl_bits(double d) { union { double d; uint64_t u; } x; x.d = d; return x.u; }
CQ_HD int64_t as_int(uint64_t b) { return (int64_t)b; }
CQ_HD const uint8_t* str_ptr(const Cell& c) { return (const uint8_t*)(uintptr_t)c.bits; }

// C-locale isspace / isdigit (the reference calls them on plain char; glibc maps
// bytes >= 0x80 to non-space/non-digit either way)
CQ_HD bool is_space(uint32_t c) { return c == 0x20 || (c >= 0x09 && c <= 0x0d); }
CQ_HD bool is_digit(uint32_t c) { return c - '0' < 10u; }

// ------------------------------------------------------------ 64x64 -> 128
struct U128 { uint64_t hi, lo; };
CQ_HD U128 mul128(uint64_t a, uint64_t b) {
    U128 r;
#if defined(__HIPCC__)
    r.lo = a * b;
    r.hi = __umul64hi(a, b);
#else
    unsigned __int128 p = (unsigned __int128)a * b;
    r.lo = (uint64_t)p;
    r.hi = (uint64_t)(p >> 64);
#endif
    return r;
}
CQ_HD int clz64(uint64_t x) {
#if defined(__HIPCC__)
    return __clzll((long long)x);
#else
    return __builtin_clzll(x);
#endif
}

// ------------------------------------------------------------ strtoll
// glibc strtoll(s, NULL, 10): isspace*, [+-], digits; saturates at the int64 limits.
CQ_HD int64_t to_int(const uint8_t* s) {
    while (is_space(*s)) s++;
    bool neg = false;
    if (*s == '+' || *s == '-') { neg = *s == '-'; s++; }
    uint64_t v = 0;
    bool ovf = false;
    const uint64_t lim = neg ? 9223372036854775808ULL : 9223372036854775807ULL;
    for (; is_digit(*s); s++) {
        uint32_t d = *s - '0';
        if (!ovf) {
            if (v > (lim - d) / 10) ovf = true;
            else v = v * 10 + d;
        }
    }
    if (ovf) return neg ? (int64_t)0x8000000000000000ULL : (int64_t)0x7fffffffffffffffULL;
    return neg ? (int64_t)(0 - v) : (int64_t)v;
}

// ------------------------------------------------------------ strtod
// Eisel-Lemire: w * 10^q -> binary64 (w != 0 and exact).  Returns false only
// when w was truncated and (w, w+1) round differently (caller resolves exactly).
CQ_HD uint64_t el_compute(int64_t q, uint64_t w, bool* ok_exact_hint) {
    // returns IEEE bits (positive), w != 0
    (void)ok_exact_hint;
    if (q < CQ_POW5_QMIN) return 0;
    if (q > CQ_POW5_QMAX) return 0x7ff0000000000000ULL;
    int lz = clz64(w);
    w <<= lz;
    int idx = 2 * (int)(q - CQ_POW5_QMIN);
    U128 first = mul128(w, cq_pow5_128[idx]);
    const uint64_t precision_mask = 0xFFFFFFFFFFFFFFFFULL >> 55;
    if ((first.hi & precision_mask) == precision_mask) {
        U128 second = mul128(w, cq_pow5_128[idx + 1]);
        first.lo += second.hi;
        if (second.hi > first.lo) first.hi++;
    }
    int upperbit = (int)(first.hi >> 63);
    int shift = upperbit + 64 - 52 - 3;
    uint64_t mant = first.hi >> shift;
    int32_t power = (int32_t)(((152170 + 65536) * q) >> 16) + 63;
    int32_t p2 = power + upperbit - lz + 1023;   // minimum_exponent = -1023
    if (p2 <= 0) {                                // subnormal
        if (-p2 + 1 >= 64) return 0;
        mant >>= -p2 + 1;
        mant += (mant & 1);
        mant >>= 1;
        p2 = (mant < (1ULL << 52)) ? 0 : 1;
        return ((uint64_t)p2 << 52) | (mant & ((1ULL << 52) - 1));
    }
    if (first.lo <= 1 && q >= -4 && q <= 23 && (mant & 3) == 1) {
        if ((mant << shift) == first.hi) mant &= ~1ULL;
    }
    mant += (mant & 1);
    mant >>= 1;
    if (mant >= (2ULL << 52)) { mant = 1ULL << 52; p2++; }
    mant &= ~(1ULL << 52);
    if (p2 >= 0x7ff) return 0x7ff0000000000000ULL;
    return ((uint64_t)p2 << 52) | mant;
}

// Exact comparison of the decimal (digits d[0..nd), value D * 10^E) with the
// binary midpoint (2m+1) * 2^(e2-1).  Returns -1, 0, +1.  Big integers of 32-bit
// limbs; only used for >19-significant-digit inputs whose rounding is ambiguous.
#define CQ_BIG_LIMBS 136
struct Big { uint32_t n; uint32_t w[CQ_BIG_LIMBS]; };
CQ_HD void big_set(Big& b, uint64_t v) {
    b.n = 0;
    while (v) { b.w[b.n++] = (uint32_t)v; v >>= 32; }
}
CQ_HD void big_muladd(Big& b, uint32_t m, uint32_t a) {
    uint64_t carry = a;
    for (uint32_t i = 0; i < b.n; i++) {
        uint64_t t = (uint64_t)b.w[i] * m + carry;
        b.w[i] = (uint32_t)t;
        carry = t >> 32;
    }
    if (carry && b.n < CQ_BIG_LIMBS) b.w[b.n++] = (uint32_t)carry;
}
CQ_HD void big_shl(Big& b, uint32_t s) {
    uint32_t limbs = s / 32, bits = s % 32;
    if (b.n == 0) return;
    if (bits) {
        uint32_t carry = 0;
        for (uint32_t i = 0; i < b.n; i++) {
            uint32_t nw = (b.w[i] << bits) | carry;
            carry = b.w[i] >> (32 - bits);
            b.w[i] = nw;
        }
        if (carry && b.n < CQ_BIG_LIMBS) b.w[b.n++] = carry;
    }
    if (limbs) {
        uint32_t nn = b.n + limbs;
        if (nn > CQ_BIG_LIMBS) nn = CQ_BIG_LIMBS;
        for (int i = (int)nn - 1; i >= 0; i--) b.w[i] = (i >= (int)limbs) ? b.w[i - limbs] : 0;
        b.n = nn;
    }
}
CQ_HD void big_mulpow5(Big& b, int32_t e) {
    while (e >= 13) { big_muladd(b, 1220703125u, 0); e -= 13; }   // 5^13
    uint32_t p = 1;
    while (e-- > 0) p *= 5;
    if (p != 1) big_muladd(b, p, 0);
}
CQ_HD int big_cmp(const Big& a, const Big& b) {
    uint32_t an = a.n, bn = b.n;
    while (an && a.w[an - 1] == 0) an--;
    while (bn && b.w[bn - 1] == 0) bn--;
    if (an != bn) return an < bn ? -1 : 1;
    for (int i = (int)an - 1; i >= 0; i--)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
}

// s: first byte of the digit run (after sign); parse grammar digits[.digits][e[+-]digits]
// again, feeding every significant digit (capped at 780) into a big integer.
CQ_HD int cmp_decimal_midpoint(const uint8_t* s, uint64_t m, int32_t e2) {
    Big L, R;
    L.n = 0;
    int32_t dexp = 0, nd = 0;
    bool started = false, sticky = false;
    const uint8_t* p = s;
    for (;; p++) {
        uint32_t c = *p;
        if (is_digit(c)) {
            if (!started && c == '0') continue;
            started = true;
            if (nd < 780) { big_muladd(L, 10, c - '0'); nd++; }
            else { dexp++; if (c != '0') sticky = true; }
        } else break;
    }
    if (*p == '.') {
        for (p++; is_digit(*p); p++) {
            uint32_t c = *p;
            if (!started && c == '0') { dexp--; continue; }
            started = true;
            if (nd < 780) { big_muladd(L, 10, c - '0'); nd++; dexp--; }
            else if (c != '0') sticky = true;
        }
    }
    if (*p == 'e' || *p == 'E') {
        const uint8_t* q = p + 1;
        bool en = false;
        if (*q == '+' || *q == '-') { en = *q == '-'; q++; }
        if (is_digit(*q)) {
            int32_t ev = 0;
            for (; is_digit(*q); q++) if (ev < 100000) ev = ev * 10 + (*q - '0');
            dexp += en ? -ev : ev;
        }
    }
    // compare L * 10^dexp  vs  (2m+1) * 2^(e2-1)
    big_set(R, 2 * m + 1);
    int32_t a2 = dexp - (e2 - 1);   // power of two on the left after factoring 10 = 2*5
    if (dexp >= 0) big_mulpow5(L, dexp);
    else big_mulpow5(R, -dexp);
    if (a2 >= 0) big_shl(L, (uint32_t)a2);
    else big_shl(R, (uint32_t)(-a2));
    int c = big_cmp(L, R);
    if (c == 0 && sticky) c = 1;
    return c;
}

// glibc strtod(s, NULL) for the grammar reachable from a cell the reference typed
// DOUBLE: isspace*, [+-], digits, '.', digits, optional exponent.  Round-to-nearest-even.
CQ_HD double to_dbl(const uint8_t* s) {
    while (is_space(*s)) s++;
    bool neg = false;
    if (*s == '+' || *s == '-') { neg = *s == '-'; s++; }
    const uint8_t* digits_start = s;
    uint64_t w = 0;
    int32_t nsig = 0, dexp = 0;
    bool trunc = false, started = false;
    const uint8_t* p = s;
    for (; is_digit(*p); p++) {
        uint32_t d = *p - '0';
        if (!started && d == 0) continue;
        started = true;
        if (nsig < 19) { w = w * 10 + d; nsig++; }
        else { dexp++; if (d) trunc = true; }
    }
    if (*p == '.') {
        for (p++; is_digit(*p); p++) {
            uint32_t d = *p - '0';
            if (!started && d == 0) { dexp--; continue; }
            started = true;
            if (nsig < 19) { w = w * 10 + d; nsig++; dexp--; }
            else if (d) trunc = true;
        }
    }
    if (*p == 'e' || *p == 'E') {
        const uint8_t* q = p + 1;
        bool en = false;
        if (*q == '+' || *q == '-') { en = *q == '-'; q++; }
        if (is_digit(*q)) {
            int32_t ev = 0;
            for (; is_digit(*q); q++) if (ev < 100000) ev = ev * 10 + (*q - '0');
            dexp += en ? -ev : ev;
        }
    }
    double r;
    if (w == 0) {
        r = 0.0;
    } else if (!trunc && w <= (1ULL << 53) && dexp >= -22 && dexp <= 22) {
        // Clinger: both operands exact, one correctly rounded IEEE operation
        const double p10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        r = dexp >= 0 ? (double)w * p10[dexp] : (double)w / p10[-dexp];
    } else {
        uint64_t b = el_compute(dexp, w, nullptr);
        if (trunc) {
            uint64_t b2 = el_compute(dexp, w + 1, nullptr);
            if (b2 != b && (b & 0x7ff0000000000000ULL) != 0x7ff0000000000000ULL) {
                // exact: the answer is b or its successor; compare with their midpoint
                uint64_t ex = b >> 52, fr = b & ((1ULL << 52) - 1);
                uint64_t m = ex ? (fr | (1ULL << 52)) : fr;
                int32_t e2 = ex ? (int32_t)ex - 1075 : -1074;
                int c = cmp_decimal_midpoint(digits_start, m, e2);
                if (c > 0 || (c == 0 && (m & 1))) b = b + 1;
            }
        }
        r = as_dbl(b);
    }
    return neg ? -r : r;
}

// ------------------------------------------------------------ dates (sscanf %d)
// glibc scanf %d: skip isspace, [+-], >= 1 digit; `width` bounds the characters
// consumed after the skipped whitespace (sign included).  Value is (int) of the long.
CQ_HD bool scan_d(const char*& s, int width, int& out) {
    while (is_space((uint8_t)*s)) s++;
    int used = 0;
    bool neg = false;
    if ((*s == '+' || *s == '-') && used < width) { neg = *s == '-'; s++; used++; }
    if (!(used < width && is_digit((uint8_t)*s))) return false;
    int64_t v = 0;
    while (used < width && is_digit((uint8_t)*s)) { v = v * 10 + (*s - '0'); s++; used++; }
    out = (int)(uint32_t)(uint64_t)(neg ? -v : v);
    return true;
}
CQ_HD bool valid_ymd(int y, int m, int d) {
    if (y < 1000 || y > 9999 || m < 1 || m > 12 || d < 1) return false;
    const int dm[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    bool leap = (y % 4 == 0 && y % 100 != 0) || (y % 400 == 0);
    int lim = (m == 2 && leap) ? 29 : dm[m - 1];
    return d <= lim;
}
// three %d separated by literal `sep`; returns the number of conversions (sscanf count)
CQ_HD int scan3(const char* s, char sep, int& a, int& b, int& c) {
    if (!scan_d(s, 1 << 30, a)) return 0;
    if (*s != sep) return 1;
    s++;
    if (!scan_d(s, 1 << 30, b)) return 1;
    if (*s != sep) return 2;
    s++;
    if (!scan_d(s, 1 << 30, c)) return 2;
    return 3;
}
// parse_date on a NUL-terminated, already trimmed string (date_utils.c:88-100)
CQ_HD bool parse_date(const char* s, int& Y, int& M, int& D) {
    int y, m, d;
    if (scan3(s, '-', y, m, d) == 3 && valid_ymd(y, m, d)) { Y = y; M = m; D = d; return true; }
    if (scan3(s, '/', m, d, y) == 3 && valid_ymd(y, m, d)) { Y = y; M = m; D = d; return true; }
    if (scan3(s, '/', d, m, y) == 3 && valid_ymd(y, m, d)) { Y = y; M = m; D = d; return true; }
    const char* t = s;
    int v;
    if (scan_d(t, 8, v)) {
        d = v % 100; v /= 100; m = v % 100; v /= 100; y = v;
        if (valid_ymd(y, m, d)) { Y = y; M = m; D = d; return true; }
    }
    return false;
}
CQ_HD uint64_t date_bits(int y, int m, int d) {
    return ((uint64_t)(uint32_t)y << 32) | ((uint64_t)(uint32_t)m << 16) | (uint32_t)d;
}

// ------------------------------------------------------------ the cell parser
// parse_value(str, len) (csv_reader.c:195-240) where f = field start and len the
// reference's field_len.  Numbers are converted from f with no length bound, as
// strtoll/strtod do in the reference; the buffer is '\n'-padded past its end.
CQ_HD Cell parse_cell(const uint8_t* f, uint32_t len) {
    if (len == 0) return cell_null();
    // every date format starts with sscanf's %d: [space*][+-]digit (a field that
    // cannot is not copied into the NUL-terminated scratch buffer at all)
    uint32_t d0 = 0;
    while (d0 < len && is_space(f[d0])) d0++;
    if (d0 < len && (f[d0] == '+' || f[d0] == '-')) d0++;
    if (len >= 8 && len <= 10 && d0 < len && is_digit(f[d0])) {
        char b[11];
        uint32_t n = 0;
        for (uint32_t i = 0; i < len; i++) { b[i] = (char)f[i]; if (!f[i]) break; n = i + 1; }
        b[n] = 0;
        uint32_t s = 0;
        while (s < n && is_space((uint8_t)b[s])) s++;
        while (n > s && is_space((uint8_t)b[n - 1])) b[--n] = 0;
        int y, m, d;
        if (parse_date(b + s, y, m, d)) {
            Cell c; c.kind = K_DATE; c.len = 0; c.bits = date_bits(y, m, d);
            return c;
        }
    }
    uint32_t i = 0;
    bool dot = false, dig = false, num = true;
    while (i < len && is_space(f[i])) i++;
    if (i < len && (f[i] == '+' || f[i] == '-')) i++;
    if (i < len) {
        while (i < len && !is_space(f[i])) {
            uint32_t ch = f[i];
            if (is_digit(ch)) dig = true;
            else if (ch == '.' && !dot) dot = true;
            else { num = false; break; }
            i++;
        }
        while (i < len && is_space(f[i])) i++;
        if (num && dig && i == len) return dot ? cell_dbl(to_dbl(f)) : cell_int(to_int(f));
    }
    // STRING: cq_strndup stops at NUL, then trim_whitespace
    uint32_t n = 0;
    while (n < len && f[n]) n++;
    uint32_t s = 0;
    while (s < n && is_space(f[s])) s++;
    while (n > s && is_space(f[n - 1])) n--;
    Cell c;
    c.kind = K_STR;
    c.len = n - s;
    c.bits = (uint64_t)(uintptr_t)(f + s);
    return c;
}

// ------------------------------------------------------------ comparison
CQ_HD int str_cmp(const uint8_t* a, uint32_t la, const uint8_t* b, uint32_t lb) {
    uint32_t n = la < lb ? la : lb;
    for (uint32_t i = 0; i < n; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return la == lb ? 0 : (la < lb ? -1 : 1);
}
CQ_HD double num_of(const Cell& c) { return c.kind == K_INT ? (double)as_int(c.bits) : as_dbl(c.bits); }
CQ_HD bool is_num(const Cell& c) { return c.kind == K_INT || c.kind == K_DBL; }

// value_compare (csv_reader.c:98-130): returns <0, 0, >0
CQ_HD int compare(const Cell& a, const Cell& b) {
    if (a.kind == K_NULL && b.kind == K_NULL) return 0;
    if (a.kind == K_NULL) return -1;
    if (b.kind == K_NULL) return 1;
    if (a.kind == K_DATE && b.kind == K_DATE) {
        int ay = (int)(a.bits >> 32), by = (int)(b.bits >> 32);
        if (ay != by) return ay - by;
        int am = (int)((a.bits >> 16) & 0xffff), bm = (int)((b.bits >> 16) & 0xffff);
        if (am != bm) return am - bm;
        return (int)(a.bits & 0xffff) - (int)(b.bits & 0xffff);
    }
    if (is_num(a) && is_num(b)) {
        double x = num_of(a), y = num_of(b);
        return x < y ? -1 : (x > y ? 1 : 0);
    }
    if (a.kind == K_STR && b.kind == K_STR) return str_cmp(str_ptr(a), a.len, str_ptr(b), b.len);
    return 0;
}

// ------------------------------------------------------------ arithmetic
enum : uint32_t { AR_ADD = 0, AR_SUB, AR_MUL, AR_DIV, AR_MOD, AR_AND, AR_OR, AR_XOR };

CQ_HD double fmod_exact(double x, double y) {
#if defined(__HIPCC__)
    return fmod(x, y);
#else
    return __builtin_fmod(x, y);
#endif
}

// evaluate_expression BINARY_OP (evaluator_expressions.c:320-426)
CQ_HD Cell arith(uint32_t op, const Cell& l, const Cell& r) {
    if (!is_num(l) || !is_num(r)) return cell_null();
    bool li = l.kind == K_INT, ri = r.kind == K_INT;
    double lv = num_of(l), rv = num_of(r);
    double res = 0;
    switch (op) {
        case AR_ADD: res = lv + rv; break;
        case AR_SUB: res = lv - rv; break;
        case AR_MUL: res = lv * rv; break;
        case AR_DIV:
            if (rv == 0) return cell_null();
            res = lv / rv;
            break;
        case AR_MOD:
            if (li && ri) {
                int64_t b = as_int(r.bits);
                if (b == 0) return cell_null();
                int64_t a = as_int(l.bits);
                return cell_int(b == -1 ? 0 : a % b);   // x86 traps on INT64_MIN % -1; 0 otherwise
            }
            if (rv == 0) return cell_null();
            res = fmod_exact(lv, rv);
            break;
        case AR_AND: case AR_OR: case AR_XOR: {
            if (!(li && ri)) return cell_null();
            int64_t a = as_int(l.bits), b = as_int(r.bits);
            return cell_int(op == AR_AND ? (a & b) : op == AR_OR ? (a | b) : (a ^ b));
        }
        default: return cell_null();
    }
    // both INTEGER and the double result integral -> INTEGER ((long long) cast on x86-64)
    if (li && ri && res >= -9223372036854775808.0 && res < 9223372036854775808.0 &&
        res == (double)(int64_t)res)
        return cell_int((int64_t)res);
    return cell_dbl(res);
}

CQ_HD Cell negate(const Cell& x) {
    if (x.kind == K_INT) return cell_int((int64_t)(0 - x.bits));
    if (x.kind == K_DBL) return cell_dbl(-as_dbl(x.bits));
    return cell_null();
}

// ------------------------------------------------------------ LIKE / ILIKE
CQ_HD uint32_t lower(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
// match_pattern (evaluator_conditions.c:16-59) over (ptr,len) strings
CQ_HD bool like(const uint8_t* s, uint32_t sl, const uint8_t* p, uint32_t pl, bool cs) {
    uint32_t si = 0, pi = 0;
    int64_t star = -1, ss = 0;
    while (si < sl) {
        if (pi < pl && p[pi] == '%') { star = pi++; ss = si; }
        else if (pi < pl && p[pi] == '_') { si++; pi++; }
        else {
            bool m = pi < pl && (cs ? s[si] == p[pi] : lower(s[si]) == lower(p[pi]));
            if (m) { si++; pi++; }
            else if (star >= 0) { pi = (uint32_t)star + 1; si = (uint32_t)(++ss); }
            else return false;
        }
    }
    while (pi < pl && p[pi] == '%') pi++;
    return pi == pl;
}

// ------------------------------------------------------------ group keys
// Key identity of the reference's printf-canonical group key text
// (evaluator_aggregates.c:122-141): two cells share a group iff their key texts
// are equal.  Text classes share one namespace: STR (trimmed bytes, first 255),
// NULL (the text "NULL") and DATE ("%04d-%02d-%02d": a STRING cell such as
// " 2024-01-05 " -- 12 raw bytes, too long for the date test -- groups with the
// DATE 2024-01-05).  INT (%lld) and DBL (%.6f) texts can never equal a string's
// (every numeric-looking field is typed numeric), so they keep binary payloads:
// INT the value, DBL sign + round-half-even(|x|*1e6) below 2^43 where the text
// is exact, and the value itself above (GK_BIG), where distinct doubles never
// share a text.
enum : uint32_t { GK_STR = 0, GK_INT = 1, GK_DBL = 2, GK_BIG = 3, GK_COMP = 4, GK_LONG = 5, GK_ALL = 7 };

// A group key in 16 bytes + class/length.  Text keys of at most 16 bytes (all
// NULL and DATE keys, most strings) are stored inline, little-endian, zero
// padded, so equality is two 64-bit compares.  Longer text keys (GK_LONG) keep
// the address of their bytes in w0 and a 64-bit content hash in w1.  INT / DBL
// / BIG keep their canonical payload in w0.
struct GKey {
    uint32_t cls;
    uint32_t len;       // text classes: bytes (<= 255)
    uint64_t w0;
    uint64_t w1;
};

CQ_HD uint32_t gk_clslen(const GKey& k) { return (k.cls << 16) | k.len; }

// round-half-even(|x| * 1e6) for |x| < 2^43 (exact in 128-bit): glibc printf
// formats the exact binary value and breaks exact ties to even.
CQ_HD uint32_t bit128(const U128& p, uint32_t k) {
    return k < 64 ? (uint32_t)((p.lo >> k) & 1) : (uint32_t)((p.hi >> (k - 64)) & 1);
}
CQ_HD uint64_t micro_units(double ax) {
    uint64_t b = dbl_bits(ax);
    uint32_t ex = (uint32_t)(b >> 52);
    uint64_t m = b & ((1ULL << 52) - 1);
    int32_t e;
    if (ex == 0) e = -1074;
    else { m |= 1ULL << 52; e = (int32_t)ex - 1075; }
    if (m == 0) return 0;
    U128 p = mul128(m, 1000000ULL);                 // < 2^73
    if (e >= 0) return p.lo << e;                    // unreachable below 2^43 (kept total)
    uint32_t sh = (uint32_t)(-e);
    if (sh >= 75) return 0;                          // p / 2^sh < 1/4
    uint64_t q = sh >= 64 ? (p.hi >> (sh - 64)) : ((p.lo >> sh) | (p.hi << (64 - sh)));
    uint32_t k = sh - 1;                             // round bit position
    uint32_t round = bit128(p, k);
    bool sticky;
    if (k == 0) sticky = false;
    else if (k <= 64) sticky = (k == 64 ? p.lo : (p.lo & ((1ULL << k) - 1))) != 0;
    else sticky = p.lo != 0 || (p.hi & ((1ULL << (k - 64)) - 1)) != 0;
    if (round && (sticky || (q & 1))) q++;
    return q;
}

CQ_HD uint64_t mix64(uint64_t h) {
    h ^= h >> 33; h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ULL;
    h ^= h >> 33;
    return h;
}

CQ_HD uint64_t fnv_bytes(const uint8_t* p, uint32_t n) {
    uint64_t h = 1469598103934665603ULL;
    for (uint32_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ULL; }
    return h;
}

// text key from bytes (trimmed STRING cell, the literal "NULL", a rendered DATE)
CQ_HD GKey text_key(const uint8_t* p, uint32_t len) {
    GKey k;
    if (len > 255) len = 255;
    k.len = len;
    if (len <= 16) {
        k.cls = GK_STR;
        uint64_t w0 = 0, w1 = 0;
        for (uint32_t i = 0; i < len; i++) {
            uint64_t b = p[i];
            if (i < 8) w0 |= b << (8 * i);
            else w1 |= b << (8 * (i - 8));
        }
        k.w0 = w0;
        k.w1 = w1;
    } else {
        k.cls = GK_LONG;
        k.w0 = (uint64_t)(uintptr_t)p;
        k.w1 = fnv_bytes(p, len);
    }
    return k;
}

CQ_HD GKey date_key(uint64_t bits) {   // "%04d-%02d-%02d" packed inline
    uint32_t y = (uint32_t)(bits >> 32), m = (uint32_t)((bits >> 16) & 0xffff), d = (uint32_t)(bits & 0xffff);
    uint8_t t[10];
    t[0] = (uint8_t)('0' + (y / 1000) % 10); t[1] = (uint8_t)('0' + (y / 100) % 10);
    t[2] = (uint8_t)('0' + (y / 10) % 10);   t[3] = (uint8_t)('0' + y % 10);
    t[4] = '-'; t[5] = (uint8_t)('0' + (m / 10) % 10); t[6] = (uint8_t)('0' + m % 10);
    t[7] = '-'; t[8] = (uint8_t)('0' + (d / 10) % 10); t[9] = (uint8_t)('0' + d % 10);
    return text_key(t, 10);
}

CQ_HD GKey group_key(const Cell& c) {
    GKey k;
    k.len = 0;
    k.w1 = 0;
    switch (c.kind) {
        case K_NULL: { const uint8_t t[4] = {'N', 'U', 'L', 'L'}; k = text_key(t, 4); break; }
        case K_INT: k.cls = GK_INT; k.w0 = c.bits; break;
        case K_DATE: k = date_key(c.bits); break;
        case K_DBL: {
            double x = as_dbl(c.bits);
            double ax = x < 0 ? -x : x;
            bool neg = (c.bits >> 63) != 0;
            if (ax < 8796093022208.0) { k.cls = GK_DBL; k.w0 = micro_units(ax) | ((uint64_t)neg << 63); }
            else { k.cls = GK_BIG; k.w0 = c.bits; }
            break;
        }
        default: k = text_key((const uint8_t*)(uintptr_t)c.bits, c.len); break;
    }
    return k;
}

// Two multiplies.  Multiplicative hashing mixes every input bit only into the
// TOP bits of the product, so the result is rotated: its low bits (the table
// index) are the product's top 24 bits; the high 32 bits (the slot tag) are
// only a filter before the full key compare.
CQ_HD uint64_t gk_hash(const GKey& k) {
    const uint64_t a = k.cls == GK_LONG ? 0 : k.w0;      // GK_LONG: w0 is an address, w1 the content hash
    const uint64_t x = a ^ (a >> 29) ^ (k.w1 * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)gk_clslen(k) << 7);
    const uint64_t h = x * 0xD6E8FEB86659FD93ULL;
    return (h >> 40) | (h << 24);
}

// Composite GROUP BY key (evaluator.c:113-212): the reference joins the parts'
// key texts with '\t' and groups by the joined text.  Here the key is a 128-bit
// digest of the parts' canonical keys (GK_COMP, len = part count): exact parts
// (inline text, numbers, dates) enter with their whole identity, long text parts
// with two independent 64-bit content hashes.  Equal texts give equal digests;
// unequal ones collide with probability ~2^-128 per pair.  A text part holding a
// tab could make two different part lists join to the same text, so kernels flag
// it and the host refuses the plan.
CQ_HD uint64_t bytes_hash2(const uint8_t* p, uint32_t n) {
    uint64_t h = 0x2545F4914F6CDD1DULL ^ n;
    for (uint32_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001B3ULL + (h >> 29);
    return mix64(h);
}
struct CompKey {
    uint64_t a = 0x6A09E667F3BCC908ULL, b = 0xBB67AE8584CAA73BULL;
    CQ_HDM void add(const GKey& k) {
        uint64_t x0 = k.w0, x1 = k.w1;
        if (k.cls == GK_LONG) x0 = bytes_hash2((const uint8_t*)(uintptr_t)k.w0, k.len);   // w1: FNV of the bytes
        const uint64_t t = ((uint64_t)gk_clslen(k) << 1) | 1;
        a = mix64(a ^ t) ^ x0;
        a = mix64(a ^ (x1 * 0x9E3779B97F4A7C15ULL));
        b = mix64(b + x1) ^ (t * 0xC2B2AE3D27D4EB4FULL);
        b = mix64(b ^ (x0 + 0x165667B19E3779F9ULL));
    }
};
CQ_HD GKey comp_key(const CompKey& c, uint32_t nparts) {
    GKey k;
    k.cls = GK_COMP;
    k.len = nparts;
    k.w0 = c.a;
    k.w1 = c.b;
    return k;
}
CQ_HD bool text_has_tab(const Cell& c) {
    if (c.kind != K_STR) return false;
    const uint8_t* p = (const uint8_t*)(uintptr_t)c.bits;
    const uint32_t n = c.len < 255 ? c.len : 255;
    for (uint32_t i = 0; i < n; i++)
        if (p[i] == '\t') return true;
    return false;
}

// A composite key whose text parts hold a tab (evaluator.c:124 joins the parts with
// '\t', so two different part lists can join to the same text): the joined text
// itself, rendered as evaluator.c:127-170 renders each part (NULL "NULL", %lld,
// %.6f, %04d-%02d-%02d, the string up to its first NUL or 255 bytes), hashed as one
// byte stream into two independent 64-bit lanes.  A list with a tab inside a part
// never joins to the same text as a list without one (its text has more tabs), so
// these keys (GK_COMP, len = part count | COMPT_FLAG) never meet the per-part
// digests.  Every cell renders (true); a DOUBLE through dbl_text, cut at 255 bytes.
constexpr uint32_t COMPT_FLAG = 0x8000;
struct TextHash {
    uint64_t a = 0xCBF29CE484222325ULL, b = 0x84222325CBF29CE4ULL;
    CQ_HDM void byte(uint8_t c) {
        a = (a ^ c) * 0x100000001B3ULL;
        b = (b ^ (c + 0x5Bu)) * 0x1000000000000B3ULL;
    }
    CQ_HDM void bytes(const uint8_t* p, uint32_t n) { for (uint32_t i = 0; i < n; i++) byte(p[i]); }
    CQ_HDM void dec(uint64_t v, int mind) {          // decimal digits, zero padded to mind
        uint8_t t[20];
        int n = 0;
        do { t[n++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
        while (n < mind) t[n++] = '0';
        while (n) byte(t[--n]);
    }
};
// bytes [lo, lo + 16) of a rendered joined text and its whole length: two joined
// texts are compared exactly window by window (scan.hip joined_text_equal)
struct TextWindow {
    uint64_t lo, pos = 0, w0 = 0, w1 = 0;
    CQ_HDM explicit TextWindow(uint64_t l) : lo(l) {}
    CQ_HDM void byte(uint8_t c) {
        const uint64_t k = pos - lo;                  // (wraps above 16 before the window)
        if (k < 8) w0 |= (uint64_t)c << (8 * k);
        else if (k < 16) w1 |= (uint64_t)c << (8 * (k - 8));
        pos++;
    }
    CQ_HDM void bytes(const uint8_t* p, uint32_t n) { for (uint32_t i = 0; i < n; i++) byte(p[i]); }
    CQ_HDM void dec(uint64_t v, int mind) {
        uint8_t t[20];
        int n = 0;
        do { t[n++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
        while (n < mind) t[n++] = '0';
        while (n) byte(t[--n]);
    }
};
// glibc's "%.6f" of a double, exactly (the binary value rounded half-even to 6
// decimals): below 2^43 through micro_units; from 2^43 the value m * 2^e has at most
// 9 fraction bits (integer part below 2^53, fraction f / 2^k rounded in 32-bit
// arithmetic) or is an integer, rendered from base-10^9 limbs (up to 309 digits);
// inf / nan as glibc prints them
template <class H>
CQ_HD void dbl_text(H& h, uint64_t bits) {
    const uint32_t ex = (uint32_t)((bits >> 52) & 0x7FF);
    const uint64_t frac = bits & ((1ULL << 52) - 1);
    if (bits >> 63) h.byte('-');
    if (ex == 0x7FF) {
        if (frac) h.bytes((const uint8_t*)"nan", 3);
        else h.bytes((const uint8_t*)"inf", 3);
        return;
    }
    const double ax = as_dbl(bits & ~(1ULL << 63));
    if (ax < 8796093022208.0) {                         // < 2^43
        const uint64_t u = micro_units(ax);
        h.dec(u / 1000000ULL, 1);
        h.byte('.');
        h.dec(u % 1000000ULL, 6);
        return;
    }
    const uint64_t m = frac | (1ULL << 52);             // (normal: >= 2^43)
    const int32_t e = (int32_t)ex - 1075;
    if (e < 0) {                                        // 2^43 <= x < 2^53: k = -e <= 9 fraction bits
        const uint32_t k = (uint32_t)(-e);
        uint64_t ip = m >> k;
        const uint64_t f = m & ((1ULL << k) - 1);
        const uint64_t n = f * 1000000ULL;               // < 2^29
        uint64_t q = n >> k;
        const uint64_t r = n & ((1ULL << k) - 1), half = 1ULL << (k - 1);
        if (r > half || (r == half && (q & 1))) q++;
        if (q == 1000000ULL) { ip++; q = 0; }
        h.dec(ip, 1);
        h.byte('.');
        h.dec(q, 6);
        return;
    }
    if (e <= 11) {                                      // m * 2^e < 2^64
        h.dec(m << e, 1);
    } else {                                            // base-10^9 limbs, least significant first
        uint32_t L[36];
        uint32_t nl = 2;
        L[0] = (uint32_t)(m % 1000000000ULL);
        L[1] = (uint32_t)(m / 1000000000ULL);           // (m < 2^53 < 10^18)
        for (int32_t left = e; left > 0;) {
            const uint32_t s = left > 29 ? 29u : (uint32_t)left;
            uint64_t carry = 0;
            for (uint32_t i = 0; i < nl; i++) {
                const uint64_t v = ((uint64_t)L[i] << s) + carry;
                L[i] = (uint32_t)(v % 1000000000ULL);
                carry = v / 1000000000ULL;
            }
            while (carry && nl < 36) { L[nl++] = (uint32_t)(carry % 1000000000ULL); carry /= 1000000000ULL; }
            left -= (int32_t)s;
        }
        while (nl > 1 && L[nl - 1] == 0) nl--;
        h.dec(L[nl - 1], 1);
        for (uint32_t i = nl - 1; i-- > 0;) h.dec(L[i], 9);
    }
    h.bytes((const uint8_t*)".000000", 7);
}

// a key part's text as the reference's `char key_part[256]` holds it: snprintf
// keeps the first 255 bytes (a %.6f of a double above ~1e248 is longer)
template <class H>
struct Cap255 {
    H& h;
    uint32_t n;
    CQ_HDM void byte(uint8_t c) {
        if (n < 255) h.byte(c);
        n++;
    }
    CQ_HDM void bytes(const uint8_t* p, uint32_t k) { for (uint32_t i = 0; i < k; i++) byte(p[i]); }
    CQ_HDM void dec(uint64_t v, int mind) {
        uint8_t t[20];
        int k = 0;
        do { t[k++] = (uint8_t)('0' + v % 10); v /= 10; } while (v);
        while (k < mind) t[k++] = '0';
        while (k) byte(t[--k]);
    }
};

template <class H>
CQ_HD bool joined_text_add(H& h, const Cell& c, bool first) {
    if (!first) h.byte('\t');
    switch (c.kind) {
        case K_NULL: h.bytes((const uint8_t*)"NULL", 4); break;
        case K_INT: {
            const int64_t v = (int64_t)c.bits;
            if (v < 0) h.byte('-');
            h.dec(v < 0 ? 0ULL - (uint64_t)v : (uint64_t)v, 1);
            break;
        }
        case K_DBL: {
            Cap255<H> cp{h, 0};
            dbl_text(cp, c.bits);
            break;
        }
        case K_DATE: {
            const int32_t y = (int32_t)(c.bits >> 32);
            const uint32_t m = (uint32_t)((c.bits >> 16) & 0xffff), d = (uint32_t)(c.bits & 0xffff);
            if (y < 0) h.byte('-');
            h.dec(y < 0 ? (uint64_t)(-(int64_t)y) : (uint64_t)y, y < 0 ? 3 : 4);
            h.byte('-');
            h.dec(m, 2);
            h.byte('-');
            h.dec(d, 2);
            break;
        }
        default: {
            const uint8_t* p = (const uint8_t*)(uintptr_t)c.bits;
            const uint32_t n = c.len < 255 ? c.len : 255;
            for (uint32_t i = 0; i < n && p[i]; i++) h.byte(p[i]);
            break;
        }
    }
    return true;
}
CQ_HD GKey joined_text_key(const TextHash& h, uint32_t nparts) {
    GKey k;
    k.cls = GK_COMP;
    k.len = nparts | COMPT_FLAG;
    k.w0 = mix64(h.a ^ (h.b >> 17));
    k.w1 = mix64(h.b + 0x9E3779B97F4A7C15ULL * h.a);
    return k;
}

CQ_HD bool gk_equal(const GKey& a, const GKey& b) {
    if (a.cls != b.cls || a.len != b.len || a.w1 != b.w1) return false;
    if (a.w0 == b.w0) return true;
    if (a.cls != GK_LONG) return false;
    const uint8_t* p = (const uint8_t*)(uintptr_t)a.w0;
    const uint8_t* q = (const uint8_t*)(uintptr_t)b.w0;
    for (uint32_t i = 0; i < a.len; i++)
        if (p[i] != q[i]) return false;
    return true;
}

}  // namespace cq
