// java_digits.h -- Integer.parseInt's digit test (Character.digit(ch, 10)) over the UTF-8 bytes of an algs4
// file, shared by the host parser (bfsx_api.cpp) and the GPU tokenizer (kernels_parse.hip).
//
// GraphFileUtil.convert reads the file through InputStreamReader (GraphFileUtil.java:46: the platform
// charset, UTF-8 on Linux) and parses tokens with Integer.parseInt (:48,62-63), which walks the String's
// UTF-16 chars and accepts every char Character.digit(ch, 10) maps to 0..9: the ASCII digits and every
// other BMP char of Unicode category Nd -- "١٢" (Arabic-Indic) or "１２" (fullwidth) parse as 12.  A
// supplementary digit (4-byte UTF-8) is two surrogate chars, neither a digit, and a malformed sequence
// decodes to U+FFFD: both make the token a NumberFormatException, as here.
// The Nd blocks are Java 8's (Unicode 6.2): the BMP blocks added in Unicode 7.0 (Sinhala Lith U+0DE6,
// Myanmar Tai Laing U+A9F0) are not digits to that runtime and are not digits here.
#pragma once

#include <cstdint>

namespace bfsx {

// zero code point of every BMP decimal-digit block (each block is ten consecutive code points)
#define BFSX_JAVA_ND_ZEROS                                                                                \
    0x0030, 0x0660, 0x06F0, 0x07C0, 0x0966, 0x09E6, 0x0A66, 0x0AE6, 0x0B66, 0x0BE6, 0x0C66, 0x0CE6,   \
        0x0D66, 0x0E50, 0x0ED0, 0x0F20, 0x1040, 0x1090, 0x17E0, 0x1810, 0x1946, 0x19D0, 0x1A80, 0x1A90, \
        0x1B50, 0x1BB0, 0x1C40, 0x1C50, 0xA620, 0xA8D0, 0xA900, 0xA9D0, 0xAA50, 0xABF0, 0xFF10

// Digit value of the char starting at b[i] (advancing i past its bytes), or -1 when the char is not a
// decimal digit, the sequence is malformed or runs past e.
__host__ __device__ inline int java_digit(const unsigned char *b, int64_t &i, int64_t e) {
    const unsigned c = b[i];
    if (c < 0x80u) {
        i++;
        return (c >= '0' && c <= '9') ? (int)(c - '0') : -1;
    }
    uint32_t cp;
    int len;
    if ((c & 0xE0u) == 0xC0u) {
        cp = c & 0x1Fu;
        len = 2;
    } else if ((c & 0xF0u) == 0xE0u) {
        cp = c & 0x0Fu;
        len = 3;
    } else {
        return -1; // a supplementary char (4-byte form) or a stray continuation / invalid lead byte
    }
    if (i + len > e) return -1;
    for (int k = 1; k < len; k++) {
        const unsigned x = b[i + k];
        if ((x & 0xC0u) != 0x80u) return -1;
        cp = (cp << 6) | (x & 0x3Fu);
    }
    if ((len == 2 && cp < 0x80u) || (len == 3 && (cp < 0x800u || (cp >= 0xD800u && cp <= 0xDFFFu)))) return -1;
    i += len;
    const uint32_t zeros[] = {BFSX_JAVA_ND_ZEROS};
    for (uint32_t z : zeros)
        if (cp >= z && cp < z + 10u) return (int)(cp - z);
    return -1;
}

// Integer.parseInt over the exact token [s, e): an optional ASCII sign, >= 1 digit, the int32 range.
__host__ __device__ inline bool java_parse_int(const unsigned char *b, int64_t s, int64_t e, int64_t &out) {
    if (s >= e) return false;
    bool neg = false;
    if (b[s] == '+' || b[s] == '-') {
        neg = b[s] == '-';
        if (++s == e) return false;
    }
    int64_t val = 0;
    while (s < e) {
        const int d = java_digit(b, s, e);
        if (d < 0) return false;
        val = val * 10 + d;
        if (val > 2147483648LL) return false;
    }
    if (neg) val = -val;
    if (val > 2147483647LL) return false;
    out = val;
    return true;
}

} // namespace bfsx
