// fold.hpp -- the serial float sum  s = 0; for k: s += e[k]  (compute_average_edge_length,
// centroids_projection.cpp:70-82), bit for bit, without walking the chain term by term.
//
// While the running sum s stays in one binade [2^(E-1), 2^E), the float grid there has spacing
// u = 2^(E-24) and s = x u for an integer x in [2^23, 2^24).  For a term e >= 0 with s + e < 2^E
//     fl(s + e) = u (x + m)                        if e / u is within 1/2 of the integer m,
//     fl(s + e) = u (x + m + ((x + m) & 1))        if e / u = m + 1/2 exactly (a tie: to even).
// So a term acts on x as x -> x + c[x & 1] with the pair c = (c_even, c_odd): (m, m) for a
// non-tie, (m + (m & 1), m + 1 - (m & 1)) for a tie.  Such maps compose into maps of the same form
// (fold_compose), so a run of terms is one pair, valid as long as the result stays below 2^24
// (partial values are monotone, and each exact partial sum is within 1/2 of its rounded one, so no
// step leaves the binade before the value reaches 2^24).  The device tabulates, per chunk of
// kFoldChunk terms and per binade of a window, the chunk's pair (clamped at 2^24: larger values are
// never usable) and a flag for terms the pair cannot express (too large, negative, inf, NaN) --
// integer arithmetic on the float bits, exact.  The walk then takes chunks in O(1) from the table
// and goes term by term only through chunks where s crosses a binade or a term is flagged.  A NaN
// term makes the sum NaN (its payload, quieted) wherever it enters; after an inf term only a NaN
// can change the sum.
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
constexpr int kFoldBinades = 4;    // binades per chunk: E in [base, base + 4), base = the binade of a
                                   // double-precision estimate of the sum before the chunk, minus 1
                                   // (the float chain drifts from it by well under a factor 2, and the
                                   // chunk may take it up two binades more)
constexpr uint8_t kFoldBad = 1, kFoldNaN = 4;   // a term the pair cannot express; a NaN term
constexpr uint32_t kFoldCap = 1u << 24;

struct FoldPair {
    uint32_t c0, c1;   // increment of x when x is even / odd
};

IMPLI_FOLD_HD inline uint32_t fold_sat(uint32_t a) { return a >= kFoldCap ? kFoldCap : a; }

// f, then g (values clamped at 2^24: a clamped value only means "reaches the binade's end")
IMPLI_FOLD_HD inline FoldPair fold_compose(FoldPair f, FoldPair g) {
    FoldPair h;
    h.c0 = fold_sat(f.c0 + ((f.c0 & 1u) ? g.c1 : g.c0));          // x even: x + f.c0 has f.c0's parity
    h.c1 = fold_sat(f.c1 + (((f.c1 + 1u) & 1u) ? g.c1 : g.c0));   // x odd: parity of 1 + f.c1
    return h;
}

// the pair of one term in binade E (spacing 2^(E-24)), and flags: kFoldBad for a term too large
// (>= 2^31 spacings), negative, inf or NaN, with kFoldNaN for NaN; e = M 2^(ex-150), M the 24-bit
// significand
IMPLI_FOLD_HD inline FoldPair fold_pair_term(uint32_t bits, int E, uint8_t& flags) {
    // branch-free (every case computed, then selected: the walk runs this in a single wave's
    // dependent chain, where divergent branches cost more than the arithmetic); 32-bit throughout:
    // M < 2^24, so M << sh (sh < 8) < 2^31 and M + half (d <= 25) < 2^25
    const uint32_t ex = (bits >> 23) & 0xffu, frac = bits & 0x7fffffu;
    const bool special = ex == 0xffu;                   // NaN / inf
    const bool neg = (bits >> 31) != 0u;
    const bool zero = (bits & 0x7fffffffu) == 0u;       // +-0 contributes 0 exactly
    const uint32_t M = frac | (ex ? 0x800000u : 0u);
    const int sh = (ex ? (int)ex : 1) - 150 + 24 - E;
    const int d = -sh;
    const int dc = d < 1 ? 1 : (d > 25 ? 25 : d);
    const uint32_t half = 1u << (dc - 1), rem = M & ((1u << dc) - 1u), m = M >> dc;
    const bool tie = rem == half;                       // exactly half a spacing: to even
    const uint32_t rr = (M + half) >> dc;
    const uint32_t a0 = d > 25 ? 0u : (tie ? m + (m & 1u) : rr);   // below half the spacing: nothing
    const uint32_t a1 = d > 25 ? 0u : (tie ? m + 1u - (m & 1u) : rr);
    const bool big = sh >= 8;                           // >= 2^31 spacings
    const uint32_t left = big ? kFoldCap : fold_sat(M << (sh < 0 ? 0 : (sh > 7 ? 7 : sh)));
    const bool kill = special || neg || zero;
    FoldPair p;
    p.c0 = kill ? 0u : (sh >= 0 ? left : a0);
    p.c1 = kill ? 0u : (sh >= 0 ? left : a1);
    flags = special ? (frac ? (uint8_t)(kFoldBad | kFoldNaN) : kFoldBad)
                    : ((zero || !(neg || big)) ? (uint8_t)0 : kFoldBad);
    return p;
}

// the window base of a chunk from the estimate of the sum before it (frexp exponent minus 1; a
// zero / tiny / non-finite estimate gives a base no chain value uses: the chunk goes term by term)
IMPLI_FOLD_HD inline int fold_base(double est) {
    if (!(est >= 0x1p-100) || !(est <= 0x1p100)) return -1000;
    int E = 0;
    double m = est;
    while (m >= 1.0) { m *= 0.5; ++E; }
    while (m < 0.5) { m *= 2.0; --E; }
    return E - 1;
}

// one table cell, in term order (host reference; the device kernel splits the chunk over a wave)
IMPLI_FOLD_HD inline void fold_cell(const float* e, int64_t n, int64_t chunk, int base, int b, FoldPair& pair,
                                    uint8_t& flags) {
    const int E = base + b;
    pair = FoldPair{0u, 0u};
    flags = 0;
    const int64_t k0 = chunk * kFoldChunk, k1 = k0 + kFoldChunk < n ? k0 + kFoldChunk : n;
    for (int64_t k = k0; k < k1; ++k) {
        uint32_t bits;
        __builtin_memcpy(&bits, &e[k], 4);
        uint8_t f;
        pair = fold_compose(pair, fold_pair_term(bits, E, f));
        flags |= f;
    }
}

IMPLI_FOLD_HD inline int64_t fold_chunks(int64_t n) { return (n + kFoldChunk - 1) / kFoldChunk; }

#ifndef __HIPCC_RTC__
// the serial chain, from the table (pairs, flags: [chunk][binade]) and the terms themselves
inline float fold_walk(const float* e, int64_t n, const int32_t* base, const FoldPair* pairs, const uint8_t* flags,
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
                const uint32_t x = (uint32_t)std::ldexp((double)s, 24 - E);   // in [2^23, 2^24)
                const FoldPair p = pairs[c * kFoldBinades + b];
                const uint64_t t = (uint64_t)x + ((x & 1u) ? p.c1 : p.c0);
                if (t < (uint64_t)kFoldCap) {
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
