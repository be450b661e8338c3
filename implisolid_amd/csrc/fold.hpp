// fold.hpp -- the serial float sum  s = 0; for k: s += e[k]  (compute_average_edge_length,
// centroids_projection.cpp:70-82), bit for bit, without walking the chain term by term.
//
// While the running sum s stays in one binade [2^(E-1), 2^E), the float grid there has spacing
// u = 2^(E-24) and s is a multiple of u, so for a term e >= 0 with s + e < 2^E
//     fl(s + e) = s + u * round(e / u)
// -- the rounding of e / u is independent of s unless e / u is exactly halfway (then round-half-even
// looks at the parity of s / u + floor(e / u)).  A run of terms thus adds the integer sum of their
// rounded quotients, valid when no term is a tie and the final s / u stays below 2^24 (the partial
// sums are monotone, and each exact partial sum is below its rounded one + 1/2, so no step leaves
// the binade).  The device tabulates, per chunk of kFoldChunk terms and per binade of a window,
// that integer sum (clamped at 2^24: larger sums are never usable) and flags (a tie, a term too
// large, negative or inf, a NaN) -- integer arithmetic on the float bits, exact.  The host then
// walks the chunks with the exact s, a chunk in O(1) from the table, and only chunks with a tie or
// a binade crossing term by term (about one chunk per doubling of s).  A NaN term makes the sum
// NaN (its payload, quieted) wherever it enters; after an inf term only a NaN can change the sum.
#pragma once
#include <stdint.h>
#ifndef __HIPCC_RTC__
#include <cmath>
#endif

#if defined(__HIPCC__)
#define IMPLI_FOLD_HD __host__ __device__
#else
#define IMPLI_FOLD_HD
#endif

namespace impli {

constexpr int kFoldChunk = 256;    // terms per table row (one wave, 4 per lane)
constexpr int kFoldBinades = 6;    // binades per chunk: E in [base, base + 6), base = the binade of a
                                   // double-precision estimate of the sum before the chunk, minus 3
                                   // (the float chain drifts from it by well under a factor 2)
constexpr uint8_t kFoldTie = 1, kFoldOverflow = 2, kFoldNaN = 4;
constexpr uint32_t kFoldCap = 1u << 24;

// round-half-up(e * 2^(24 - E)) (clamped at 2^24), and whether it was a tie, too large (>= 2^31,
// negative, inf) or NaN; e * 2^(24 - E) = M * 2^sh with M the 24-bit significand
IMPLI_FOLD_HD inline uint32_t fold_term(uint32_t bits, int E, uint8_t& flags) {
    const uint32_t ex = (bits >> 23) & 0xffu, frac = bits & 0x7fffffu;
    flags = 0;
    if (ex == 0xffu) { flags = frac ? kFoldNaN : kFoldOverflow; return 0u; }   // NaN / inf
    if (bits & 0x80000000u) {                      // negative (-0 contributes 0 exactly)
        if (bits & 0x7fffffffu) flags = kFoldOverflow;
        return 0u;
    }
    if (ex == 0u && frac == 0u) return 0u;         // +0
    const uint64_t M = (uint64_t)(frac | (ex ? 0x800000u : 0u));
    const int sh = (ex ? (int)ex : 1) - 150 + 24 - E;   // e = M 2^((ex or 1) - 150)
    if (sh >= 0) {
        if (sh >= 8) { flags = kFoldOverflow; return kFoldCap; }   // >= 2^31
        const uint64_t r = M << sh;
        return r >= kFoldCap ? kFoldCap : (uint32_t)r;
    }
    const int d = -sh;
    if (d > 25) return 0u;                          // below half the spacing: rounds to 0
    const uint64_t half = (uint64_t)1 << (d - 1), rem = M & (((uint64_t)1 << d) - 1);
    if (rem == half) flags = kFoldTie;
    return (uint32_t)((M + half) >> d);
}

IMPLI_FOLD_HD inline uint32_t fold_add(uint32_t a, uint32_t b) {   // saturating at kFoldCap
    const uint32_t s = a + b;
    return s >= kFoldCap ? kFoldCap : s;
}

// the window base of a chunk from the estimate of the sum before it (frexp exponent minus 3; a
// zero / tiny / non-finite estimate gives a base no chain value uses: the chunk goes term by term)
IMPLI_FOLD_HD inline int fold_base(double est) {
    if (!(est >= 0x1p-100) || !(est <= 0x1p100)) return -1000;
    int E = 0;
    double m = est;
    while (m >= 1.0) { m *= 0.5; ++E; }
    while (m < 0.5) { m *= 2.0; --E; }
    return E - 3;
}

// one table cell (host reference; the device kernel splits the chunk over a wave)
IMPLI_FOLD_HD inline void fold_cell(const float* e, int64_t n, int64_t chunk, int base, int b, uint32_t& sum,
                                    uint8_t& flags) {
    const int E = base + b;
    sum = 0;
    flags = 0;
    const int64_t k0 = chunk * kFoldChunk, k1 = k0 + kFoldChunk < n ? k0 + kFoldChunk : n;
    for (int64_t k = k0; k < k1; ++k) {
        uint32_t bits;
        __builtin_memcpy(&bits, &e[k], 4);
        uint8_t f;
        sum = fold_add(sum, fold_term(bits, E, f));
        flags |= f;
    }
}

IMPLI_FOLD_HD inline int64_t fold_chunks(int64_t n) { return (n + kFoldChunk - 1) / kFoldChunk; }

#ifndef __HIPCC_RTC__
// the serial chain, from the table (sum, flags: [chunk][binade]) and the terms themselves
inline float fold_walk(const float* e, int64_t n, const int32_t* base, const uint32_t* sum, const uint8_t* flags,
                       int64_t* table_chunks = nullptr) {
    float s = 0.f;
    const int64_t nc = fold_chunks(n);
    for (int64_t c = 0; c < nc; ++c) {
        const int64_t k0 = c * kFoldChunk, k1 = k0 + kFoldChunk < n ? k0 + kFoldChunk : n;
        if (flags[c * kFoldBinades] & kFoldNaN) {      // (the NaN flag is set in every binade)
            for (int64_t k = k0; k < k1; ++k) {        // the first NaN term decides the result
                if (e[k] != e[k]) return s + e[k];
                s += e[k];
            }
        }
        if (s >= 0x1p-100f && s <= 0x1p100f) {
            int E;
            (void)std::frexp(s, &E);                   // s in [2^(E-1), 2^E): spacing 2^(E-24)
            const int b = E - base[c];
            if (b >= 0 && b < kFoldBinades && !flags[c * kFoldBinades + b]) {
                const int64_t su = (int64_t)std::ldexp((double)s, 24 - E);   // in [2^23, 2^24)
                const int64_t t = su + (int64_t)sum[c * kFoldBinades + b];
                if (t < (int64_t)kFoldCap) {
                    s = (float)std::ldexp((double)t, E - 24);   // exact: t < 2^24 in this binade
                    if (table_chunks) ++*table_chunks;
                    continue;
                }
            }
        } else if (s == INFINITY) {                    // only a later NaN can change it
            for (int64_t cc = c; cc < nc; ++cc)
                if (flags[cc * kFoldBinades] & kFoldNaN)
                    for (int64_t k = cc * kFoldChunk; k < n; ++k)
                        if (e[k] != e[k]) return s + e[k];
            return s;
        }
        for (int64_t k = k0; k < k1; ++k) s += e[k];
    }
    return s;
}
#endif

}  // namespace impli
