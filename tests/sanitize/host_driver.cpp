// host_driver.cpp -- TEST INFRASTRUCTURE: drives the library's host code (the code that takes the
// untrusted strings of the C ABI) under AddressSanitizer + UndefinedBehaviorSanitizer on the CPU.
//
// Built by tests/sanitize/Makefile from the product's own sources (implisolid_amd/csrc/host.cpp,
// jit.cpp, json.hpp); no GPU call is made: the JIT part only generates kernel source text.
//
// Input on stdin: records separated by a line holding only "%%".  The first line of a record is
// its kind, the rest its payload:
//   settings        <mc-settings JSON>       parse_mc_settings (polygoniser_settings.hpp:147-305)
//   mp5 | mp5i      <MP5 JSON>               compile_mp5 (object_factory.hpp:56-758), ignore_root_matrix
//                                            false / true, then the JIT's brick (shape and baked) and
//                                            point kernel sources for the compiled program
//   slab R z0 z1                             slab_range
//   partition R rank n                       slab_partition
//   matrix f0 .. f11                         invert_matrix12 (basic_functions.hpp:77-128)
//   rand seed n                              GlibcRand: n draws vs a seeded copy skipped by n
// One output line per record: "ok ..." or "error ...".  Any sanitizer report aborts the process
// (-fno-sanitize-recover), which the test sees as a non-zero exit.
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "host.hpp"
#include "jit.hpp"

using namespace impli;

static void run(const std::string& kind, const std::string& payload) {
    std::istringstream in(payload);
    try {
        if (kind == "settings") {
            const MCSettings s = parse_mc_settings(payload.c_str());
            std::printf("ok settings R=%d repeats=%d iters=%d proj=%d qem=%d subdiv=%d\n", s.resolution, s.overall_repeats,
                        s.vresampl_iters, (int)s.projection, (int)s.qem, (int)s.subdiv);
        } else if (kind == "mp5" || kind == "mp5i") {
            const Program p = compile_mp5(payload.c_str(), kind == "mp5i");
            const std::string a = TreeJit::kernel_source(p, false), b = TreeJit::kernel_source(p, true),
                              c = TreeJit::point_source(p);
            std::printf("ok mp5 instr=%d depth=%d mats=%d csg=%d src=%zu/%zu/%zu\n", p.n_instr, p.max_depth, p.n_mats, p.n_csg,
                        a.size(), b.size(), c.size());
        } else if (kind == "slab") {
            int R, z0, z1;
            in >> R >> z0 >> z1;
            const SlabRange r = slab_range(R, z0, z1);
            std::printf("ok slab %d %d %d\n", r.z0, r.z1, r.halo);
        } else if (kind == "partition") {
            int R, rank, n;
            in >> R >> rank >> n;
            const SlabRange r = slab_partition(R, rank, n);
            std::printf("ok partition %d %d %d\n", r.z0, r.z1, r.halo);
        } else if (kind == "matrix") {
            float m[12], o[12];
            for (float& v : m) in >> v;
            const bool ok = invert_matrix12(m, o);
            std::printf("ok matrix %d %a\n", (int)ok, ok ? (double)o[3] : 0.0);
        } else if (kind == "rand") {
            unsigned seed;
            unsigned long long n;
            in >> seed >> n;
            GlibcRand a(seed), b(seed);
            for (unsigned long long k = 0; k < n; ++k) (void)a.next();
            b.skip(n);
            std::printf("ok rand %d %d\n", (int)a.next(), (int)b.next());
        } else {
            std::printf("error unknown record kind\n");
        }
    } catch (const std::exception& e) {
        std::string w = e.what();
        if (w.size() > 120) w.resize(120);
        for (char& ch : w)
            if (ch == '\n') ch = ' ';
        std::printf("error %s\n", w.c_str());
    }
}

int main() {
    std::string line, kind, payload;
    bool have = false;
    auto flush = [&] {
        if (have) run(kind, payload);
        have = false;
        kind.clear();
        payload.clear();
    };
    while (std::getline(std::cin, line)) {
        if (line == "%%") {
            flush();
            continue;
        }
        if (!have) {
            have = true;
            const size_t sp = line.find(' ');
            kind = line.substr(0, sp);
            if (sp != std::string::npos) payload = line.substr(sp + 1);
            continue;
        }
        payload += (payload.empty() ? "" : "\n") + line;
    }
    flush();
    return 0;
}
