// pytext.h -- byte-exact restatements of the Python text primitives the
// reference's file formats rely on: universal-newline line iteration,
// str.strip() (Unicode whitespace), str.split(sep), float(), and the
// shortest round-trip repr of a double.  Host code only.
#pragma once

#include <algorithm>
#include <cfloat>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <system_error>
#include <vector>

namespace di::py {

// Decode one UTF-8 code point starting at s[i] (no validation beyond length).
inline uint32_t decode_at(std::string_view s, size_t i, size_t *len) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) { *len = 1; return c; }
    int n = (c >= 0xF0) ? 4 : (c >= 0xE0) ? 3 : (c >= 0xC0) ? 2 : 1;
    if (i + n > s.size()) { *len = 1; return c; }
    uint32_t cp = (n == 2) ? (c & 0x1F) : (n == 3) ? (c & 0x0F) : (n == 4) ? (c & 0x07) : c;
    for (int k = 1; k < n; ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
    *len = (size_t)n;
    return cp;
}

// str.isspace() for one code point (CPython's _PyUnicode_IsWhitespace table).
inline bool is_space(uint32_t c) {
    switch (c) {
        case 0x09: case 0x0A: case 0x0B: case 0x0C: case 0x0D: case 0x1C: case 0x1D:
        case 0x1E: case 0x1F: case 0x20: case 0x85: case 0xA0: case 0x1680: case 0x2028:
        case 0x2029: case 0x202F: case 0x205F: case 0x3000:
            return true;
        default:
            return c >= 0x2000 && c <= 0x200A;
    }
}

// str.strip() with no argument.
inline std::string_view strip(std::string_view s) {
    size_t a = 0, len;
    while (a < s.size()) {
        uint32_t c = decode_at(s, a, &len);
        if (!is_space(c)) break;
        a += len;
    }
    size_t b = s.size();
    while (b > a) {
        size_t st = b - 1;
        while (st > a && ((unsigned char)s[st] & 0xC0) == 0x80) --st;
        uint32_t c = decode_at(s, st, &len);
        if (st + len != b || !is_space(c)) break;
        b = st;
    }
    return s.substr(a, b - a);
}

// str.split(sep) with a non-empty separator.
inline void split(std::string_view s, std::string_view sep, std::vector<std::string_view> &out) {
    out.clear();
    size_t pos = 0;
    for (;;) {
        size_t f = s.find(sep, pos);
        if (f == std::string_view::npos) {
            out.push_back(s.substr(pos));
            return;
        }
        out.push_back(s.substr(pos, f - pos));
        pos = f + sep.size();
    }
}

// Iterate lines the way Python text files do (universal newlines: \n, \r\n, \r).
// The callback receives each line WITHOUT its terminator.  A trailing
// terminator does not produce an extra empty line.
template <class F>
inline void for_each_line(std::string_view buf, F &&f) {
    size_t i = 0, n = buf.size();
    while (i < n) {
        size_t j = i;
        while (j < n && buf[j] != '\n' && buf[j] != '\r') ++j;
        f(buf.substr(i, j - i));
        if (j < n && buf[j] == '\r' && j + 1 < n && buf[j + 1] == '\n') ++j;
        i = j + 1;
    }
}

// Lines for_each_line yields over buf (for a prefix that ends at a line boundary: the
// number of lines before it).  Used on error paths to place a line in the whole file.
inline int64_t count_lines(std::string_view buf) {
    int64_t n = 0;
    for_each_line(buf, [&](std::string_view) { ++n; });
    return n;
}

// Cut buf into at most `parts` ranges of whole lines: boundaries right after a line
// terminator (\n, a \r\n pair, a lone \r), so for_each_line over the ranges in order
// yields exactly the lines of the whole buffer.  Returns the cut positions (first 0,
// last buf.size()).
inline std::vector<size_t> line_chunks(std::string_view buf, int parts) {
    const size_t n = buf.size();
    std::vector<size_t> cut{0};
    auto boundary = [&](size_t b) {  // a line starts at b
        if (b == 0 || b >= n) return true;
        const char c = buf[b - 1];
        return c == '\n' || (c == '\r' && buf[b] != '\n');
    };
    for (int p = 1; p < parts; ++p) {
        size_t b = std::max(cut.back(), n * (size_t)p / (size_t)parts);
        while (b < n && !boundary(b)) ++b;
        if (b > cut.back() && b < n) cut.push_back(b);
    }
    cut.push_back(n);
    return cut;
}

// float(text): strict decimal/inf/nan literal with optional surrounding
// whitespace.  Digit-group underscores (PEP 515) are accepted as Python does.
// Fast path (the formats' own numbers): plain [digits][.digits] with a mantissa below
// 2^53 and at most 22 fraction digits is m / 10^k in one correctly rounded division
// (both exact doubles: Clinger's fast path) -- the value strtod returns.
inline bool parse_float(std::string_view s, double *out) {
    {
        static constexpr double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                           1e8,  1e9,  1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                           1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        uint64_t m = 0;
        int nd = 0, frac = -1;
        bool fast = !s.empty();
        for (char c : s) {
            if (c >= '0' && c <= '9') {
                if (++nd > 19) {
                    fast = false;
                    break;
                }
                m = m * 10 + (uint64_t)(c - '0');
                if (frac >= 0) ++frac;
            } else if (c == '.' && frac < 0) {
                frac = 0;
            } else {
                fast = false;
                break;
            }
        }
        const int k = frac < 0 ? 0 : frac;
        if (fast && nd > 0 && m <= (1ull << 53) && k <= 22) {
            *out = (double)m / p10[k];
            return true;
        }
        // 54..64-bit mantissas (17-19 digits, e.g. repr of a float32 as a double): one
        // x87 extended division (64-bit mantissa, m and 10^k exact) rounded to double.
        // The double rounding is exact unless the extended quotient is itself a midpoint
        // between two doubles (its low 11 bits 0x400): then strtod decides.
        // (host code: the x87 80-bit format -- a 64-bit significand whose low 8 bytes the
        // memcpy below reads; IEEE quad (aarch64) or double-double long doubles are not
        // that format and take strtod)
        if constexpr (LDBL_MANT_DIG == 64 && sizeof(long double) >= 10) {
            if (fast && nd > 0 && k <= 22) {
                const long double q = (long double)m / (long double)p10[k];
                uint64_t mant;  // the x87 format's explicit 64-bit significand (low 8 bytes)
                std::memcpy(&mant, &q, 8);
                if ((mant & 0x7FFu) != 0x400u) {
                    *out = (double)q;
                    return true;
                }
            }
        }
    }
    s = strip(s);
    if (s.empty()) return false;
    char buf[128];
    size_t m = 0;
    bool prev_digit = false;
    for (size_t i = 0; i < s.size(); ++i) {
        char c = s[i];
        if (c == '_') {  // only between two digits
            bool next_digit = i + 1 < s.size() && s[i + 1] >= '0' && s[i + 1] <= '9';
            if (!prev_digit || !next_digit) return false;
            prev_digit = false;
            continue;
        }
        if (m + 1 >= sizeof buf) return false;
        buf[m++] = c;
        prev_digit = c >= '0' && c <= '9';
    }
    buf[m] = 0;
    // reject hex floats and other strtod extensions Python does not accept
    for (size_t i = 0; i < m; ++i) {
        char c = buf[i];
        if (c == 'x' || c == 'X' || c == 'p' || c == 'P') return false;
    }
    char *end = nullptr;
    double v = std::strtod(buf, &end);
    if (end != buf + m) return false;
    *out = v;
    return true;
}

// repr(float): shortest round-trip digits; fixed notation for exponents in
// [-4, 16), scientific otherwise ('1e-05', '1e+16'); '.0' on integral values.
inline void repr_double(double v, std::string &out) {
    if (std::isnan(v)) { out += "nan"; return; }
    if (std::isinf(v)) { out += v < 0 ? "-inf" : "inf"; return; }
    char sci[64];
    auto r = std::to_chars(sci, sci + sizeof sci, v, std::chars_format::scientific);
    *r.ptr = 0;
    // sci = [-]d[.ddd]e(+|-)XX
    const char *p = sci;
    bool neg = *p == '-';
    if (neg) ++p;
    std::string digits;
    const char *e = std::strchr(p, 'e');
    for (const char *q = p; q < e; ++q)
        if (*q != '.') digits += *q;
    int exp10 = std::atoi(e + 1);
    // strip trailing zeros of the mantissa (to_chars shortest already does)
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    if (neg) out += '-';
    const int nd = (int)digits.size();
    if (exp10 >= -5 + 1 && exp10 < 16) {  // CPython: -4 <= exp < 16
        if (exp10 >= 0) {
            if (nd <= exp10 + 1) {
                out += digits;
                out.append((size_t)(exp10 + 1 - nd), '0');
                out += ".0";
            } else {
                out.append(digits, 0, (size_t)exp10 + 1);
                out += '.';
                out.append(digits, (size_t)exp10 + 1, std::string::npos);
            }
        } else {
            out += "0.";
            out.append((size_t)(-exp10 - 1), '0');
            out += digits;
        }
    } else {
        out += digits[0];
        if (nd > 1) {
            out += '.';
            out.append(digits, 1, std::string::npos);
        }
        out += 'e';
        out += exp10 < 0 ? '-' : '+';
        int a = exp10 < 0 ? -exp10 : exp10;
        if (a < 10) out += '0';
        out += std::to_string(a);
    }
}

}  // namespace di::py
