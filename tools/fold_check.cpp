// fold_check.cpp -- the chunk-table fold (implisolid_amd/csrc/fold.hpp) against the serial float
// chain on many seeded arrays: typical edge lengths, wide log-uniform spreads, exact ties (integer
// and half-integer terms near binade tops), zeros, subnormals, huge values, inf and NaN, sizes from
// 0 to 10^6.  Prints "mismatches N"; the table is computed by the same fold_cell (term pairs,
// ties to even as parity-dependent increments) the device's table kernel computes.
//     g++ -O2 -ffp-contract=off -std=c++17 tools/fold_check.cpp -o fold_check && ./fold_check
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <random>
#include <vector>

#include "../implisolid_amd/csrc/fold.hpp"

static float serial(const std::vector<float>& e) {
    float s = 0.f;
    for (float x : e) s += x;
    return s;
}

static int64_t g_table_chunks = 0, g_chunks = 0;
static float table_fold(const std::vector<float>& e) {
    const int64_t n = (int64_t)e.size(), nc = impli::fold_chunks(n);
    std::vector<impli::FoldPair> sum((size_t)(nc * impli::kFoldBinades));
    std::vector<uint8_t> fl((size_t)(nc * impli::kFoldBinades));
    std::vector<int32_t> base((size_t)nc);
    double est = 0.0;   // the device's estimate: chunk sums in double, exclusive prefix
    for (int64_t c = 0; c < nc; ++c) {
        base[(size_t)c] = impli::fold_base(est);
        double cs = 0.0;
        for (int64_t k = c * impli::kFoldChunk; k < std::min(n, (c + 1) * impli::kFoldChunk); ++k) cs += (double)e[(size_t)k];
        est += cs;
        for (int b = 0; b < impli::kFoldBinades; ++b)
            impli::fold_cell(e.data(), n, c, base[(size_t)c], b, sum[(size_t)(c * impli::kFoldBinades + b)],
                             fl[(size_t)(c * impli::kFoldBinades + b)]);
    }
    g_chunks += nc;
    return impli::fold_walk(e.data(), n, base.data(), sum.data(), fl.data(), &g_table_chunks);
}

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main() {
    std::mt19937_64 rng(20261016);
    int64_t mismatches = 0, cases = 0, fast_checked = 0;
    auto check = [&](const std::vector<float>& e, const char* what) {
        const float a = serial(e), b = table_fold(e);
        ++cases;
        const bool same = bits(a) == bits(b) || (a != a && b != b && (bits(a) | 0x400000u) == (bits(b) | 0x400000u));
        if (!same) {
            ++mismatches;
            if (mismatches < 10) std::printf("MISMATCH %s n=%zu serial=%a table=%a\n", what, e.size(), a, b);
        }
        fast_checked += (int64_t)e.size();
    };
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (int t = 0; t < 400; ++t) {
        const int64_t n = (int64_t)(U(rng) * (t < 300 ? 5000 : 400000));
        std::vector<float> e((size_t)n);
        const int kind = t % 8;
        for (int64_t k = 0; k < n; ++k) {
            const double x = U(rng);
            switch (kind) {
                case 0: e[(size_t)k] = (float)(0.0144 * (0.5 + x)); break;                 // edge lengths
                case 1: e[(size_t)k] = (float)std::exp2(-30.0 + 60.0 * x); break;          // wide spread
                case 2: e[(size_t)k] = (float)std::floor(1 + 8 * x); break;                 // integers: ties at 2^24+
                case 3: e[(size_t)k] = (float)(std::floor(1 + 64 * x) * 0.5); break;        // half integers
                case 4: e[(size_t)k] = x < 0.3 ? 0.f : (float)(1e-3 * x); break;            // zeros
                case 5: e[(size_t)k] = x < 0.01 ? (float)(1e-40 * x) : (float)(3.0 * x); break;   // subnormals
                case 6: e[(size_t)k] = (float)std::ldexp(1.0, (int)(x * 40) - 20); break;   // powers of two: ties
                default: e[(size_t)k] = (float)(x * x * 100.0); break;
            }
        }
        check(e, "random");
    }
    // binade tops: a big start then terms around half the spacing
    for (int t = 0; t < 200; ++t) {
        const int E = 1 + (int)(U(rng) * 30);
        std::vector<float> e;
        e.push_back((float)std::ldexp(1.0, E) * (float)(0.5 + 0.49 * U(rng)));
        const double u = std::ldexp(1.0, E - 24);
        const int64_t n = 1000 + (int64_t)(U(rng) * 20000);
        for (int64_t k = 0; k < n; ++k) {
            const double x = U(rng);
            e.push_back((float)(x < 0.5 ? u * (0.5 + (int)(x * 8)) : u * x * 3));
        }
        check(e, "ties");
    }
    // specials
    check({}, "empty");
    check({1.f}, "one");
    check({0.f, -0.f, 0.f}, "zeros");
    {
        std::vector<float> e(100000, 0.0144f);
        e[50000] = INFINITY;
        check(e, "inf");
        e[70000] = NAN;
        check(e, "inf+nan");
        e[20000] = std::nanf("0x1234");
        check(e, "nan payload");
    }
    {
        std::vector<float> e(3000000, 1.0f);   // past 2^24 the terms stop counting (ties to even)
        check(e, "saturation");
    }
    std::printf("cases %lld terms %lld chunks %lld from the table %lld mismatches %lld\n", (long long)cases,
                (long long)fast_checked, (long long)g_chunks, (long long)g_table_chunks, (long long)mismatches);
    return mismatches != 0;
}
