// jit.cpp -- code generation and hipRTC compilation of tree kernels (see jit.hpp).
#include "jit.hpp"
#include "kernels.hpp"

#include <hip/hiprtc.h>

#include <chrono>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <set>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <vector>

#include "generated/jit_headers.inc"

namespace impli {

namespace {

// types and macros hipRTC does not provide (the headers skip their system includes under it)
const char* kPrelude = R"(
typedef signed char int8_t;
typedef unsigned char uint8_t;
typedef short int16_t;
typedef unsigned short uint16_t;
typedef int int32_t;
typedef unsigned int uint32_t;
typedef long int64_t;
typedef unsigned long uint64_t;
#ifndef INFINITY
#define INFINITY __builtin_huge_valf()
#endif
)";

struct Node {
    bool leaf = false;
    int type = 0, mat = 0, csg = -1, prm = 0;
    int child[2] = {-1, -1};
};

// post-order program -> tree: XFORM(m) PRIM(t) is a leaf; XFORM(m) <a> <b> CSG(t) an inner node
int parse(const Program& p, int pc, std::vector<Node>& nodes, int& next) {
    if (pc >= p.n_instr || p.instr[pc].op != OP_XFORM) throw std::runtime_error("jit: malformed program");
    Node n;
    n.mat = p.instr[pc].mat;
    if (pc + 1 < p.n_instr && p.instr[pc + 1].op == OP_PRIM) {
        n.leaf = true;
        n.type = p.instr[pc + 1].type;
        n.prm = p.instr[pc + 1].prm;
        next = pc + 2;
    } else {
        int p1 = 0, p2 = 0;
        n.child[0] = parse(p, pc + 1, nodes, p1);
        n.child[1] = parse(p, p1, nodes, p2);
        if (p2 >= p.n_instr || p.instr[p2].op != OP_CSG) throw std::runtime_error("jit: malformed program");
        n.type = p.instr[p2].type;
        n.csg = p.instr[p2].csg;
        next = p2 + 1;
    }
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}

// a primitive's parameter row (Instr::prm) is passed as a pointer into the matrix array M
std::string with_params(const std::string& call, int prm) {
    const size_t k = call.find("P, ");
    if (k == std::string::npos) return call;
    return call.substr(0, k) + "M + " + std::to_string(12 * prm) + ", " + call.substr(k + 3);
}

const char* prim_call(int t) {
    switch (t) {
        case NT_ELLIPSOID: return "egg_f(";
        case NT_CUBE: return "cube_f(tab, ";
        case NT_CYLINDER: return "cyl_f(";
        case NT_CONE: return "cone_f(";
        case NT_HEART: return "heart_f(";
        case NT_TORUS: return "torus_f(";
        case NT_DMUSHROOM: return "dm_f(";
        case NT_SCREW: return "screw_f(P, ";
        case NT_HALF_PLANE: return "hp_f(P, ";
        case NT_TETRA: return "tet_f(P, ";
        case NT_METABALLS: return "meta_f(P, ";
        default: throw std::runtime_error("jit: unknown primitive");
    }
}

// One row of xform() (matrix_vector_product, basic_functions.hpp:140-177):
//     ((m0 x + m1 y) + m2 z) + m3
// specialised on the row's pattern, its values staying data (M + i).  Exact whatever the inputs:
//   - a coefficient equal to 0 contributes a zero: dropping it can only change the sign of an
//     intermediate zero, and the row's final + m3 (kept) gives the same result unless m3 is -0
//     (then the full expression is emitted);
//   - 1 * v == v exactly;
//   - an identity row (only 1 * v, m3 == +0) is v itself: coordinates are never -0 (sample
//     coordinates are a - b differences, every emitted row ends with + m3 != -0), so v + 0 == v.
std::string xform_row(const float* m, int base, const std::string& x, const std::string& y, const std::string& z) {
    const std::string v[3] = {x, y, z};
    auto is_bits = [](float f, uint32_t b) { uint32_t u; std::memcpy(&u, &f, 4); return u == b; };
    const float t = m[3];
    auto at = [&](int k) { return "M[" + std::to_string(base + k) + "]"; };
    if (is_bits(t, 0x80000000u) || !std::isfinite(t))   // -0 (or non-finite) translation: generic
        return "((" + at(0) + " * " + x + " + " + at(1) + " * " + y + ") + " + at(2) + " * " + z + ") + " + at(3);
    std::vector<std::string> terms;
    int ones = 0;
    for (int k = 0; k < 3; ++k) {
        if (!std::isfinite(m[k])) return "((" + at(0) + " * " + x + " + " + at(1) + " * " + y + ") + " + at(2) + " * " + z + ") + " + at(3);
        if (m[k] == 0.f) continue;
        if (m[k] == 1.f) { terms.push_back(v[k]); ++ones; }
        else terms.push_back(at(k) + " * " + v[k]);
    }
    if (terms.size() == 1 && ones == 1 && is_bits(t, 0u)) return terms[0];   // identity row
    std::string e;
    for (size_t k = 0; k < terms.size(); ++k) e = k == 0 ? terms[0] : "(" + e + " + " + terms[k] + ")";
    return terms.empty() ? "(0.f + " + at(3) + ")" : "(" + e + " + " + at(3) + ")";
}

// The interval row of xform_iv() (ifunc_interval.hpp), specialised like xform_row(): mulc(v, 1)
// is v, a zero coefficient adds a [+-0, +-0] term (only zero endpoint signs can differ, which no
// decision or class depends on), the final ivc(m3) and settle_point stay; an identity row is v.
std::string xform_iv_row(const float* m, int base, const std::string& p) {
    const std::string v[3] = {p + ".x", p + ".y", p + ".z"};
    auto is_bits = [](float f, uint32_t b) { uint32_t u; std::memcpy(&u, &f, 4); return u == b; };
    auto at = [&](int k) { return "M[" + std::to_string(base + k) + "]"; };
    const std::string generic = "settle_point(add(add(add(mulc(" + v[0] + ", " + at(0) + "), mulc(" + v[1] + ", " +
                                at(1) + ")), mulc(" + v[2] + ", " + at(2) + ")), ivc(" + at(3) + ")))";
    const float t = m[3];
    if (is_bits(t, 0x80000000u) || !std::isfinite(t)) return generic;
    std::vector<std::string> terms;
    int ones = 0;
    for (int k = 0; k < 3; ++k) {
        if (!std::isfinite(m[k])) return generic;
        if (m[k] == 0.f) continue;
        if (m[k] == 1.f) { terms.push_back(v[k]); ++ones; }
        else terms.push_back("mulc(" + v[k] + ", " + at(k) + ")");
    }
    if (terms.size() == 1 && ones == 1 && is_bits(t, 0u)) return terms[0];
    std::string e;
    for (size_t k = 0; k < terms.size(); ++k) e = k == 0 ? terms[0] : "add(" + e + ", " + terms[k] + ")";
    return terms.empty() ? "settle_point(ivc(" + at(3) + "))" : "settle_point(add(" + e + ", ivc(" + at(3) + ")))";
}

struct Emitter {
    const std::vector<Node>& nodes;
    const Program& prog;
    std::ostringstream out;
    int counter = 0;

    // emits the code of node `i` evaluated at point (x, y, z); returns the variable holding f
    std::string emit(int i, const std::string& x, const std::string& y, const std::string& z, int ind) {
        const Node& n = nodes[i];
        const int id = counter++;
        const std::string pad(ind, ' ');
        const std::string q = "q" + std::to_string(id), f = "f" + std::to_string(id);
        // matrix_vector_product (basic_functions.hpp:140-177), rows specialised by xform_row()
        const float* mm = prog.mats[n.mat];
        out << pad << "const V3 " << q << " = V3{" << xform_row(mm, 12 * n.mat, x, y, z) << ",\n" << pad << "    "
            << xform_row(mm + 4, 12 * n.mat + 4, x, y, z) << ",\n" << pad << "    "
            << xform_row(mm + 8, 12 * n.mat + 8, x, y, z) << "};\n";
        if (n.leaf) {
            std::string call = n.type == NT_LID         ? "lid_f(" + q + ".z)"
                               : n.type == NT_EXTRUSION ? with_params("extr_f(P, ", n.prm) + q + ".x, " + q + ".y)"
                                                        : with_params(prim_call(n.type), n.prm) + q + ".x, " + q + ".y, " + q + ".z)";
            out << pad << "const float " << f << " = " << call << ";\n";
            return f;
        }
        const std::string m = "m" + std::to_string(id), a = "a" + std::to_string(id), b = "b" + std::to_string(id);
        out << pad << "float " << f << ";\n" << pad << "{\n";
        out << pad << "  const uint32_t " << m << " = mode_of(modes, " << n.csg << ");\n";
        out << pad << "  float " << a << " = 0.f, " << b << " = 0.f;\n";
        out << pad << "  if (" << m << " != PM_RIGHT) {\n";
        const std::string fa = emit(n.child[0], q + ".x", q + ".y", q + ".z", ind + 4);
        out << pad << "    " << a << " = " << fa << ";\n" << pad << "  }\n";
        out << pad << "  if (" << m << " != PM_LEFT) {\n";
        const std::string fb = emit(n.child[1], q + ".x", q + ".y", q + ".z", ind + 4);
        out << pad << "    " << b << " = " << fb << ";\n" << pad << "  }\n";
        // transformed_union.hpp:48 / transformed_intersection.hpp:50 / transformed_subtract.hpp:52
        std::string sel, right = b;
        if (n.type == NT_UNION) sel = "(" + a + " > " + b + ") ? " + a + " : " + b;
        else if (n.type == NT_INTERSECTION) sel = "(" + a + " > " + b + ") ? " + b + " : " + a;
        else {
            sel = "(" + a + " < -" + b + ") ? " + a + " : -" + b;
            right = "-" + b;
        }
        out << pad << "  " << f << " = (" << m << " == PM_BOTH) ? (" << sel << ") : (" << m << " == PM_LEFT) ? " << a
            << " : " << right << ";\n";
        out << pad << "}\n";
        return f;
    }
};

const char* prim_iv_call(int t) {
    switch (t) {
        case NT_ELLIPSOID: return "egg_iv(";
        case NT_CUBE: return "cube_iv(tab, tab_range, ";
        case NT_CYLINDER: return "cyl_iv(";
        case NT_CONE: return "cone_iv(";
        case NT_HEART: return "heart_iv(";
        case NT_TORUS: return "torus_iv(";
        case NT_DMUSHROOM: return "dm_iv(";
        case NT_SCREW: return "screw_iv(P, ";
        case NT_LID: return "lid_iv(";
        case NT_HALF_PLANE: return "hp_iv(P, ";
        case NT_TETRA: return "tet_iv(P, ";
        case NT_METABALLS: return "meta_iv(P, ";
        case NT_EXTRUSION: return "extr_iv(P, ";
        default: throw std::runtime_error("jit: unknown primitive");
    }
}

// Interval version of the tree (eval_iv, ifunc_interval.hpp): the same primitive bounds, settle()
// and CSG decisions, so modes and classes are bit-identical to the interpreter's.
struct IvEmitter {
    const std::vector<Node>& nodes;
    const Program& prog;
    std::ostringstream out;
    int counter = 0;

    std::string emit(int i, const std::string& p, int ind) {
        const Node& n = nodes[i];
        const int id = counter++;
        const std::string pad(ind, ' ');
        const std::string q = "q" + std::to_string(id), r = "r" + std::to_string(id);
        const float* mm = prog.mats[n.mat];
        out << pad << "const Box " << q << " = Box{" << xform_iv_row(mm, 12 * n.mat, p) << ",\n" << pad << "    "
            << xform_iv_row(mm + 4, 12 * n.mat + 4, p) << ",\n" << pad << "    "
            << xform_iv_row(mm + 8, 12 * n.mat + 8, p) << "};\n";
        if (n.leaf) {
            out << pad << "const Iv " << r << " = settle(" << with_params(prim_iv_call(n.type), n.prm) << q << "));\n";
            return r;
        }
        const std::string m = "m" + std::to_string(id), a = "a" + std::to_string(id), b = "b" + std::to_string(id);
        out << pad << "Iv " << r << ";\n" << pad << "{\n";
        out << pad << "  const uint32_t " << m << " = mode_of(modes_in, " << n.csg << ");\n";
        out << pad << "  Iv " << a << " = Iv{0.f, 0.f}, " << b << " = Iv{0.f, 0.f};\n";
        out << pad << "  if (" << m << " != PM_RIGHT) {\n";
        const std::string ra = emit(n.child[0], q, ind + 4);
        out << pad << "    " << a << " = " << ra << ";\n" << pad << "  }\n";
        out << pad << "  if (" << m << " != PM_LEFT) {\n";
        const std::string rb = emit(n.child[1], q, ind + 4);
        out << pad << "    " << b << " = " << rb << ";\n" << pad << "  }\n";
        out << pad << "  if (" << m << " == PM_BOTH) {\n";
        out << pad << "    const uint32_t d = csg_decide(" << n.type << ", " << a << ", " << b << ", " << r << ");\n";
        if (n.csg >= 0 && n.csg < kMaxPruned) out << pad << "    modes |= (uint64_t)d << " << 2 * n.csg << ";\n";
        else out << pad << "    (void)d;\n";
        out << pad << "  } else if (" << m << " == PM_LEFT) {\n" << pad << "    " << r << " = " << a << ";\n";
        out << pad << "  } else {\n" << pad << "    " << r << " = " << (n.type == NT_DIFFERENCE ? "neg(" + b + ")" : b)
            << ";\n" << pad << "  }\n";
        out << pad << "}\n";
        return r;
    }
};

void rtc_check(hiprtcResult r, const char* what) {
    if (r != HIPRTC_SUCCESS) throw std::runtime_error(std::string(what) + ": " + hiprtcGetErrorString(r));
}

}  // namespace

TreeJit& TreeJit::instance() {
    static TreeJit j;
    return j;
}

TreeJit::TreeJit() {
    const char* e = std::getenv("IMPLISOLID_JIT");
    enabled_ = !(e && e[0] == '0');
}

std::string TreeJit::kernel_source(const Program& p) {
    std::vector<Node> nodes;
    int next = 0;
    const int root = parse(p, 0, nodes, next);
    if (next != p.n_instr) throw std::runtime_error("jit: trailing instructions");
    Emitter em{nodes, p};
    const std::string f = em.emit(root, "x0", "y0", "z0", 4);
    IvEmitter iv{nodes, p};
    const std::string r = iv.emit(root, "p0", 4);
    std::ostringstream s;
    if (const char* e = std::getenv("IMPLISOLID_EVAL_PAIR")) s << "#define IMPLI_EVAL_PAIR " << (e[0] == '1' ? 1 : 0) << "\n";
    s << kPrelude << "#include \"eval_bricks.hpp\"\n#include \"ifunc_interval.hpp\"\n#include \"brick_modes.hpp\"\n"
      << "namespace impli {\nusing namespace dev;\n"
      << "__device__ __forceinline__ float tree_f(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "                                        uint64_t modes, float x0, float y0, float z0) {\n"
      << em.out.str() << "    return " << f << ";\n}\n"
      << "struct JitEval {\n    const float* M;\n    const float* tab;\n"
      << "    __device__ __forceinline__ float operator()(uint64_t m, float x, float y, float z) const {\n"
      << "        return tree_f(M, tab, m, x, y, z);\n    }\n};\n"
      << "__device__ __forceinline__ Iv tree_iv(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "                                      float2 tab_range, Box p0, uint64_t modes_in, uint64_t& modes) {\n"
      << "    modes = modes_in;\n"
      << iv.out.str() << "    return " << r << ";\n}\n"
      << "struct JitIv {\n    const float* M;\n    const float* tab;\n    float2 tab_range;\n"
      << "    __device__ __forceinline__ Iv operator()(Box p, uint64_t mi, uint64_t& m) const {\n"
      << "        return tree_iv(M, tab, tab_range, p, mi, m);\n    }\n};\n"
      << "}  // namespace impli\n"
      << "extern \"C\" __global__ __launch_bounds__(" << kEvalBlock << ") void impli_eval_bricks(\n"
      << "    const float* M, const float* tab, impli::GridDesc g, impli::BrickGrid bg, const uint64_t* modes,\n"
      << "    const uint32_t* list, const uint32_t* count, float* field, void* signs) {\n"
      << "    impli::eval_bricks_body(impli::JitEval{M, tab}, g, bg, modes, list, count, field, signs);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void impli_coarse_modes(\n"
      << "    const float* M, const float* tab, float2 tab_range, impli::GridDesc g, impli::BrickGrid cg,\n"
      << "    uint64_t* cmodes, uint8_t* ccls, uint32_t* clist, uint32_t* counters) {\n"
      << "    impli::coarse_modes_body(impli::JitIv{M, tab, tab_range}, g, cg, cmodes, ccls, clist, counters);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void impli_brick_refine(\n"
      << "    const float* M, const float* tab, float2 tab_range, impli::GridDesc g, impli::BrickGrid bg,\n"
      << "    impli::BrickGrid cg, const uint64_t* cmodes, const uint32_t* clist, const uint32_t* ccount,\n"
      << "    uint64_t* modes, uint8_t* cls) {\n"
      << "    impli::brick_refine_body(impli::JitIv{M, tab, tab_range}, g, bg, cg, cmodes, clist, ccount, modes, cls);\n}\n"
;
    return s.str();
}

std::vector<char> TreeJit::compile(const std::string& src) {
    hiprtcProgram prog = nullptr;
    rtc_check(hiprtcCreateProgram(&prog, src.c_str(), "impli_tree.hip", kJitNumHeaders, kJitHeaderSources,
                                  kJitHeaderNames),
              "hiprtcCreateProgram");
    // the static library's floating-point contract: no FMA contraction, IEEE division/sqrt
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 4, opts);
    if (r != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        throw std::runtime_error("hiprtcCompileProgram: " + log.substr(0, 4000));
    }
    size_t code_size = 0;
    std::vector<char> code;
    try {
        rtc_check(hiprtcGetCodeSize(prog, &code_size), "hiprtcGetCodeSize");
        code.resize(code_size);
        rtc_check(hiprtcGetCode(prog, code.data()), "hiprtcGetCode");
    } catch (...) {
        hiprtcDestroyProgram(&prog);
        throw;
    }
    hiprtcDestroyProgram(&prog);
    if (const char* dir = std::getenv("IMPLISOLID_JIT_DUMP")) {   // diagnostics: keep source + code object
        static int n = 0;
        const std::string base = std::string(dir) + "/tree_" + std::to_string(n++);
        if (FILE* f = std::fopen((base + ".hip").c_str(), "w")) { std::fwrite(src.data(), 1, src.size(), f); std::fclose(f); }
        if (FILE* f = std::fopen((base + ".co").c_str(), "wb")) { std::fwrite(code.data(), 1, code.size(), f); std::fclose(f); }
    }
    return code;
}

TreeJit::Kernels TreeJit::kernels(const Program& p) {
    if (!enabled_) return Kernels{};
    std::string src;
    try {
        src = kernel_source(p);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "implisolid: tree JIT skipped (%s)\n", e.what());
        return Kernels{};
    }
    std::lock_guard<std::mutex> lock(mu_);
    auto it = cache_.find(src);
    if (it != cache_.end()) return it->second.k;
    Entry ent;
    const auto t0 = std::chrono::steady_clock::now();
    try {
        const std::vector<char> code = compile(src);
        if (hipModuleLoadData(&ent.mod, code.data()) != hipSuccess) throw std::runtime_error("hipModuleLoadData failed");
        if (hipModuleGetFunction(&ent.k.bricks, ent.mod, "impli_eval_bricks") != hipSuccess ||
            hipModuleGetFunction(&ent.k.coarse, ent.mod, "impli_coarse_modes") != hipSuccess ||
            hipModuleGetFunction(&ent.k.refine, ent.mod, "impli_brick_refine") != hipSuccess)
            throw std::runtime_error("hipModuleGetFunction failed");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "implisolid: tree JIT failed, using the interpreter (%s)\n", e.what());
        ent.k = Kernels{};
    }
    compile_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (ent.k.bricks) ++n_compiled_;
    cache_.emplace(src, ent);
    return ent.k;
}

void TreeJit::precompile(const std::vector<Program>& progs, int threads) {
    if (!enabled_) return;
    std::vector<std::string> srcs;
    {
        std::set<std::string> seen;
        std::lock_guard<std::mutex> lock(mu_);
        for (const Program& p : progs) {
            std::string src;
            try {
                src = kernel_source(p);
            } catch (const std::exception&) {
                continue;   // kernels() logs and falls back for this shape
            }
            if (!cache_.count(src) && seen.insert(src).second) srcs.push_back(std::move(src));
        }
    }
    if (srcs.empty()) return;
    std::vector<std::vector<char>> codes(srcs.size());
    std::vector<std::string> errs(srcs.size());
    std::atomic<size_t> next{0};
    const auto t0 = std::chrono::steady_clock::now();
    auto work = [&] {
        for (size_t i; (i = next++) < srcs.size();) {
            try {
                codes[i] = compile(srcs[i]);
            } catch (const std::exception& e) {
                errs[i] = e.what();
            }
        }
    };
    const int nt = std::max(1, std::min<int>(threads, (int)srcs.size()));
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    std::lock_guard<std::mutex> lock(mu_);
    for (size_t i = 0; i < srcs.size(); ++i) {
        Entry ent;
        if (!codes[i].empty() && hipModuleLoadData(&ent.mod, codes[i].data()) == hipSuccess &&
            hipModuleGetFunction(&ent.k.bricks, ent.mod, "impli_eval_bricks") == hipSuccess &&
            hipModuleGetFunction(&ent.k.coarse, ent.mod, "impli_coarse_modes") == hipSuccess &&
            hipModuleGetFunction(&ent.k.refine, ent.mod, "impli_brick_refine") == hipSuccess) {
            ++n_compiled_;
        } else {
            std::fprintf(stderr, "implisolid: tree JIT failed, using the interpreter (%s)\n",
                         errs[i].empty() ? "module load failed" : errs[i].substr(0, 400).c_str());
            ent.k = Kernels{};
        }
        cache_.emplace(srcs[i], ent);
    }
    compile_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void TreeJit::launch_bricks(hipFunction_t fn, const float* d_mats, const float* d_rabbit, const GridDesc& g,
                            const BrickGrid& bg, const uint64_t* d_modes, const uint32_t* d_list,
                            const uint32_t* d_count, float* d_field, void* d_signs, unsigned blocks, hipStream_t s) {
    if (bg.n_bricks <= 0) return;
    GridDesc gg = g;
    BrickGrid bb = bg;
    void* args[] = {(void*)&d_mats, (void*)&d_rabbit, (void*)&gg, (void*)&bb, (void*)&d_modes,
                    (void*)&d_list, (void*)&d_count, (void*)&d_field, (void*)&d_signs};
    if (hipModuleLaunchKernel(fn, blocks, 1, 1, kEvalBlock, 1, 1, 0, s, args, nullptr) != hipSuccess)
        throw std::runtime_error("hipModuleLaunchKernel(impli_eval_bricks) failed");
}

void TreeJit::launch(hipFunction_t fn, unsigned blocks, void** args, hipStream_t s, const char* what) {
    if (hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, s, args, nullptr) != hipSuccess)
        throw std::runtime_error(std::string("hipModuleLaunchKernel(") + what + ") failed");
}

}  // namespace impli
