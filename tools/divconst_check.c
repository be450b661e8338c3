/* divconst_check.c -- exhaustive check of the division-by-constant identity the device code uses
 * (ifunc_device.hpp div_const / div_const_d):
 *     q0 = x * R,  R = RN(1/D);   q = fma(fma(-q0, D, x), R, q0)   (q0 itself when not finite)
 * must equal the IEEE quotient x / D for every input the call site can see.  f32 sites divide a
 * float by D: all 2^32 bit patterns are checked.  The f64 site (double mushroom) divides the exact
 * double square of a float: all 2^32 floats x, a = (double)x * x.  NaN == NaN counts as equal.
 *   gcc -O2 -mfma -ffp-contract=off -pthread tools/divconst_check.c -o /tmp/divconst_check -lm
 *   /tmp/divconst_check [threads] [all]   -> one line per constant: mismatches
 * Result (8 threads, ~20 s for the f64 site): the f64 site has 0 mismatches, so the double
 * mushroom's three divisions use the identity.  The f32 sites (kept under `all` as the record) fail
 * on subnormal and near-subnormal inputs (0.2f: 8.2 M of 2^32), so those divisions stay IEEE.
 * (A property check of the device arithmetic against IEEE division, not a reference restatement.) */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef struct { int f64; float D; uint64_t lo, hi, bad; uint32_t first_bad; } job_t;

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static void* run(void* p) {
    job_t* j = (job_t*)p;
    const float D = j->D;
    const float R = 1.0f / D;
    const double Dd = (double)D, Rd = 1.0 / Dd;
    for (uint64_t u = j->lo; u < j->hi; ++u) {
        const float x = f_of((uint32_t)u);
        if (!j->f64) {
            const float want = x / D;
            const float q0 = x * R;
            const float got = isfinite(q0) ? fmaf(fmaf(-q0, D, x), R, q0) : q0;
            if (!(want == got || (isnan(want) && isnan(got))) || (want == 0 && signbit(want) != signbit(got))) {
                if (!j->bad) j->first_bad = (uint32_t)u;
                ++j->bad;
            }
        } else {
            const double a = (double)x * (double)x;
            const double want = a / Dd;
            const double q0 = a * Rd;
            const double got = isfinite(q0) ? fma(fma(-q0, Dd, a), Rd, q0) : q0;
            if (!(want == got || (isnan(want) && isnan(got))) || (want == 0 && signbit(want) != signbit(got))) {
                if (!j->bad) j->first_bad = (uint32_t)u;
                ++j->bad;
            }
        }
    }
    return NULL;
}

static uint64_t check(int f64, float D, int threads, uint32_t* first) {
    pthread_t t[64];
    job_t jb[64];
    const uint64_t n = 1ull << 32, per = n / (uint64_t)threads;
    for (int k = 0; k < threads; ++k) {
        jb[k] = (job_t){f64, D, per * (uint64_t)k, k == threads - 1 ? n : per * (uint64_t)(k + 1), 0, 0};
        pthread_create(&t[k], NULL, run, &jb[k]);
    }
    uint64_t bad = 0;
    *first = 0;
    for (int k = 0; k < threads; ++k) {
        pthread_join(t[k], NULL);
        if (jb[k].bad && !bad) *first = jb[k].first_bad;
        bad += jb[k].bad;
    }
    return bad;
}

int main(int argc, char** argv) {
    int threads = 8;
    if (argc > 1) sscanf(argv[1], "%d", &threads);
    const int all = argc > 2 && !strcmp(argv[2], "all");
    if (threads < 1 || threads > 64) threads = 8;
    const float pi = (float)3.1415926535897;   /* screw.hpp:20 */
    struct { const char* site; int f64; float D; } cases[] = {
        {"torus x / rx (0.2f)", 0, 0.2f},
        {"screw theta / pi2", 0, pi * 2},
        {"double mushroom grad -2x / a2 (0.2f*0.2f)", 0, 0.2f * 0.2f},
        {"rabbit (X - o) / gs (0.75f)", 0, 0.75f},
        {"double mushroom sq_exact(x) / (double)a2", 1, 0.2f * 0.2f},
    };
    int fail = 0;
    for (size_t c = 0; c < sizeof cases / sizeof cases[0]; ++c) {
        if (!all && !cases[c].f64) continue;
        uint32_t first;
        const uint64_t bad = check(cases[c].f64, cases[c].D, threads, &first);
        printf("%-45s D=%.9g %s mismatches %llu%s", cases[c].site, (double)cases[c].D, cases[c].f64 ? "f64" : "f32",
               (unsigned long long)bad, bad ? "" : "\n");
        if (bad) printf(" (first input bits 0x%08x)\n", first);
        fail |= bad != 0;
    }
    return fail;
}
