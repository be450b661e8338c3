// jit.cpp -- code generation and hipRTC compilation of tree kernels (see jit.hpp).
#include "jit.hpp"
#include "kernels.hpp"

#include <hip/hiprtc.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <sstream>
#include <stdexcept>
#include <thread>
#include <vector>

#include <dirent.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>
#include <dlfcn.h>

#include "generated/jit_headers.inc"

namespace impli {

#define IMPLI_HIP_THROW(x) do { if ((x) != hipSuccess) throw std::runtime_error(#x " failed"); } while (0)

static const char* const kEvalWavesAttr = " __attribute__((amdgpu_waves_per_eu(8)))";

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
        case NT_SCREW_TBB: return "tbb_f(P, ";
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
// a float as an exact literal of its bit pattern (value-baked kernels)
std::string float_literal(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    char buf[48];
    std::snprintf(buf, sizeof buf, "__builtin_bit_cast(float, 0x%08xu)", u);
    return buf;
}

std::string xform_row(const float* m, int base, const std::string& x, const std::string& y, const std::string& z,
                      bool bake) {
    const std::string v[3] = {x, y, z};
    auto is_bits = [](float f, uint32_t b) { uint32_t u; std::memcpy(&u, &f, 4); return u == b; };
    const float t = m[3];
    auto at = [&](int k) { return bake ? float_literal(m[k]) : "M[" + std::to_string(base + k) + "]"; };
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
std::string xform_iv_row(const float* m, int base, const std::string& p, bool bake) {
    const std::string v[3] = {p + ".x", p + ".y", p + ".z"};
    auto is_bits = [](float f, uint32_t b) { uint32_t u; std::memcpy(&u, &f, 4); return u == b; };
    auto at = [&](int k) { return bake ? float_literal(m[k]) : "M[" + std::to_string(base + k) + "]"; };
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
    bool bake;
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
        out << pad << "const V3 " << q << " = V3{" << xform_row(mm, 12 * n.mat, x, y, z, bake) << ",\n" << pad << "    "
            << xform_row(mm + 4, 12 * n.mat + 4, x, y, z, bake) << ",\n" << pad << "    "
            << xform_row(mm + 8, 12 * n.mat + 8, x, y, z, bake) << "};\n";
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

// The point tree at two samples of one column (a brick's two layers, same x and y) under the same
// modes: each node's code for both samples in the same wave-uniform branches, so the two
// dependency chains interleave and the compiler shares whatever does not depend on z (the screw
// shares its atan2f through screw_f2 / tbb_f2).  Per sample, exactly the operations of emit().
struct PairEmitter {
    const std::vector<Node>& nodes;
    const Program& prog;
    bool bake;
    std::ostringstream out;
    int counter = 0;

    // returns the variables holding f at sample a and at sample b
    std::pair<std::string, std::string> emit(int i, const std::string& xa, const std::string& ya, const std::string& za,
                                             const std::string& xb, const std::string& yb, const std::string& zb, int ind) {
        const Node& n = nodes[i];
        const int id = counter++;
        const std::string pad(ind, ' ');
        const std::string q = "q" + std::to_string(id), f = "f" + std::to_string(id);
        const std::string qb = q + "b", fb = f + "b";
        const float* mm = prog.mats[n.mat];
        for (int s = 0; s < 2; ++s) {
            const std::string& x = s ? xb : xa;
            const std::string& y = s ? yb : ya;
            const std::string& z = s ? zb : za;
            out << pad << "const V3 " << (s ? qb : q) << " = V3{" << xform_row(mm, 12 * n.mat, x, y, z, bake) << ",\n"
                << pad << "    " << xform_row(mm + 4, 12 * n.mat + 4, x, y, z, bake) << ",\n" << pad << "    "
                << xform_row(mm + 8, 12 * n.mat + 8, x, y, z, bake) << "};\n";
        }
        if (n.leaf) {
            if (n.type == NT_SCREW || n.type == NT_SCREW_TBB) {
                out << pad << "float " << f << ", " << fb << ";\n" << pad
                    << with_params(n.type == NT_SCREW ? "screw_f2(P, " : "tbb_f2(P, ", n.prm) << q << ".x, " << q << ".y, "
                    << q << ".z, " << qb << ".x, " << qb << ".y, " << qb << ".z, " << f << ", " << fb << ");\n";
                return {f, fb};
            }
            for (int s = 0; s < 2; ++s) {
                const std::string& v = s ? qb : q;
                std::string call = n.type == NT_LID         ? "lid_f(" + v + ".z)"
                                   : n.type == NT_EXTRUSION ? with_params("extr_f(P, ", n.prm) + v + ".x, " + v + ".y)"
                                                            : with_params(prim_call(n.type), n.prm) + v + ".x, " + v + ".y, " + v + ".z)";
                out << pad << "const float " << (s ? fb : f) << " = " << call << ";\n";
            }
            return {f, fb};
        }
        const std::string m = "m" + std::to_string(id), a = "a" + std::to_string(id), b = "b" + std::to_string(id);
        const std::string ab = a + "b", bb = b + "b";
        out << pad << "float " << f << ", " << fb << ";\n" << pad << "{\n";
        out << pad << "  const uint32_t " << m << " = mode_of(modes, " << n.csg << ");\n";
        out << pad << "  float " << a << " = 0.f, " << b << " = 0.f, " << ab << " = 0.f, " << bb << " = 0.f;\n";
        out << pad << "  if (" << m << " != PM_RIGHT) {\n";
        const auto fa = emit(n.child[0], q + ".x", q + ".y", q + ".z", qb + ".x", qb + ".y", qb + ".z", ind + 4);
        out << pad << "    " << a << " = " << fa.first << ";\n" << pad << "    " << ab << " = " << fa.second << ";\n"
            << pad << "  }\n";
        out << pad << "  if (" << m << " != PM_LEFT) {\n";
        const auto fr = emit(n.child[1], q + ".x", q + ".y", q + ".z", qb + ".x", qb + ".y", qb + ".z", ind + 4);
        out << pad << "    " << b << " = " << fr.first << ";\n" << pad << "    " << bb << " = " << fr.second << ";\n"
            << pad << "  }\n";
        for (int s = 0; s < 2; ++s) {
            const std::string& A = s ? ab : a;
            const std::string& B = s ? bb : b;
            std::string sel, right = B;
            if (n.type == NT_UNION) sel = "(" + A + " > " + B + ") ? " + A + " : " + B;
            else if (n.type == NT_INTERSECTION) sel = "(" + A + " > " + B + ") ? " + B + " : " + A;
            else {
                sel = "(" + A + " < -" + B + ") ? " + A + " : -" + B;
                right = "-" + B;
            }
            out << pad << "  " << (s ? fb : f) << " = (" << m << " == PM_BOTH) ? (" << sel << ") : (" << m
                << " == PM_LEFT) ? " << A << " : " << right << ";\n";
        }
        out << pad << "}\n";
        return {f, fb};
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
        case NT_SCREW_TBB: return "tbb_iv(P, ";
        default: throw std::runtime_error("jit: unknown primitive");
    }
}

// Interval version of the tree (eval_iv, ifunc_interval.hpp): the same primitive bounds, settle()
// and CSG decisions, so modes and classes are bit-identical to the interpreter's.
struct IvEmitter {
    const std::vector<Node>& nodes;
    const Program& prog;
    bool bake;
    std::ostringstream out;
    int counter = 0;

    std::string emit(int i, const std::string& p, int ind) {
        const Node& n = nodes[i];
        const int id = counter++;
        const std::string pad(ind, ' ');
        const std::string q = "q" + std::to_string(id), r = "r" + std::to_string(id);
        const float* mm = prog.mats[n.mat];
        out << pad << "const Box " << q << " = Box{" << xform_iv_row(mm, 12 * n.mat, p, bake) << ",\n" << pad << "    "
            << xform_iv_row(mm + 4, 12 * n.mat + 4, p, bake) << ",\n" << pad << "    "
            << xform_iv_row(mm + 8, 12 * n.mat + 8, p, bake) << "};\n";
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

// Point version of the tree (eval_f / eval_fg of ifunc_device.hpp, straight-line): every node's
// transform is the generic xform() -- points may be NaN (OB02 vertices of singular faces), and
// dropping a zero coefficient would stop a NaN the interpreter propagates -- no pruning modes, and
// with `grad` the gradient: the leaf's M^-T prim_g, the CSG's selected child (the difference's
// second negated) under the node's M^-T (transformed_*.hpp:73-93).
const char* prim_g_call(int t) {
    switch (t) {
        case NT_ELLIPSOID: return "egg_g(";
        case NT_CUBE: return "cube_g(";
        case NT_CYLINDER: return "cyl_g(";
        case NT_CONE: return "cone_g(";
        case NT_HEART: return "heart_g(";
        case NT_TORUS: return "torus_g(";
        case NT_DMUSHROOM: return "dm_g(";
        case NT_SCREW: return "screw_g(P, ";
        case NT_HALF_PLANE: return "hp_g(P, ";
        case NT_TETRA: return "tet_g(P, ";
        case NT_METABALLS: return "meta_g(P, ";
        case NT_SCREW_TBB: return "tbb_g(P, ";
        default: throw std::runtime_error("jit: unknown primitive");
    }
}

// The point modules' transforms (xform / grad_xform, ifunc_device.hpp) written out per matrix.  A
// coefficient that is exactly 1 multiplies as the identity (1 * v == v: what constant folding makes
// of a baked module), exact zeros are literals (0 * v is kept: its sign and NaN cases), every other
// entry is read from M; the rows keep xform's operation order ((m0 x + m1 y) + m2 z) + m3.  Points
// may be non-finite here, so no term is dropped (unlike xform_row's finite sample rows).
std::string pt_coef(const float* m, int base, int k, const std::string& v) {
    uint32_t u;
    std::memcpy(&u, &m[k], 4);
    if (u == 0x3f800000u) return v;
    if (u == 0u) return "0.f * " + v;
    if (u == 0x80000000u) return "-0.f * " + v;
    return "M[" + std::to_string(base + k) + "] * " + v;
}
std::string pt_const(const float* m, int base, int k) {
    uint32_t u;
    std::memcpy(&u, &m[k], 4);
    if (u == 0u) return "0.f";
    if (u == 0x80000000u) return "-0.f";
    return "M[" + std::to_string(base + k) + "]";
}
std::string pt_xform(const float* m, int base, const std::string& x, const std::string& y, const std::string& z) {
    std::string r[3];
    for (int i = 0; i < 3; ++i)
        r[i] = "((" + pt_coef(m, base, 4 * i, x) + " + " + pt_coef(m, base, 4 * i + 1, y) + ") + " +
               pt_coef(m, base, 4 * i + 2, z) + ") + " + pt_const(m, base, 4 * i + 3);
    return "V3{" + r[0] + ", " + r[1] + ", " + r[2] + "}";
}
// grad_xform: inv^T g, row i = (m_i g.x + m_{4+i} g.y) + m_{8+i} g.z (g a V3 variable)
std::string pt_grad_xform(const float* m, int base, const std::string& g) {
    std::string r[3];
    for (int i = 0; i < 3; ++i)
        r[i] = "(" + pt_coef(m, base, i, g + ".x") + " + " + pt_coef(m, base, 4 + i, g + ".y") + ") + " +
               pt_coef(m, base, 8 + i, g + ".z");
    return "V3{" + r[0] + ", " + r[1] + ", " + r[2] + "}";
}

struct PtEmitter {
    const std::vector<Node>& nodes;
    const Program& prog;
    bool grad;
    std::ostringstream out;
    int counter = 0;

    // returns the variable holding f; the gradient is "g" + the same id
    std::string emit(int i, const std::string& x, const std::string& y, const std::string& z, int ind) {
        const Node& n = nodes[i];
        const int id = counter++;
        const std::string pad(ind, ' ');
        const std::string q = "q" + std::to_string(id), f = "f" + std::to_string(id), g = "g" + std::to_string(id);
        const float* mm = prog.mats[n.mat];
        const int mb = 12 * n.mat;
        out << pad << "const V3 " << q << " = " << pt_xform(mm, mb, x, y, z) << ";\n";
        if (n.leaf) {
            const std::string call = n.type == NT_LID         ? "lid_f(" + q + ".z)"
                                     : n.type == NT_EXTRUSION ? with_params("extr_f(P, ", n.prm) + q + ".x, " + q + ".y)"
                                                              : with_params(prim_call(n.type), n.prm) + q + ".x, " + q + ".y, " + q + ".z)";
            out << pad << "const float " << f << " = " << call << ";\n";
            if (grad) {
                const std::string gc = n.type == NT_LID         ? std::string("V3{0.f, 0.f, 1.f}")
                                       : n.type == NT_EXTRUSION ? with_params("extr_g(P, ", n.prm) + q + ".x, " + q + ".y)"
                                                                : with_params(prim_g_call(n.type), n.prm) + q + ".x, " + q + ".y, " + q + ".z)";
                out << pad << "const V3 t" << g << " = " << gc << ";\n";
                out << pad << "const V3 " << g << " = " << pt_grad_xform(mm, mb, "t" + g) << ";\n";
            }
            return f;
        }
        const std::string fa = emit(n.child[0], q + ".x", q + ".y", q + ".z", ind);
        const std::string fb = emit(n.child[1], q + ".x", q + ".y", q + ".z", ind);
        std::string sel;
        if (n.type == NT_UNION) sel = "(" + fa + " > " + fb + ") ? " + fa + " : " + fb;
        else if (n.type == NT_INTERSECTION) sel = "(" + fa + " > " + fb + ") ? " + fb + " : " + fa;
        else sel = "(" + fa + " < -" + fb + ") ? " + fa + " : -" + fb;
        out << pad << "const float " << f << " = " << sel << ";\n";
        if (grad) {
            const std::string ga = "g" + fa.substr(1), gb = "g" + fb.substr(1);
            const std::string gbs = n.type == NT_DIFFERENCE ? "V3{-" + gb + ".x, -" + gb + ".y, -" + gb + ".z}" : gb;
            out << pad << "const V3 t" << g << " = csg_first(" << n.type << ", " << fa << ", " << fb << ") ? " << ga << " : "
                << gbs << ";\n";
            out << pad << "const V3 " << g << " = " << pt_grad_xform(mm, mb, "t" + g) << ";\n";
        }
        return f;
    }
};

void rtc_check(hiprtcResult r, const char* what) {
    if (r != HIPRTC_SUCCESS) throw std::runtime_error(std::string(what) + ": " + hiprtcGetErrorString(r));
}

}  // namespace

TreeJit& TreeJit::instance() {
    static TreeJit* j = new TreeJit();   // never destroyed: workers are joined at exit (shutdown)
    return *j;
}

TreeJit::TreeJit() {
    if (const char* e = std::getenv("IMPLISOLID_JIT")) mode_.store(e[0] == '0' ? kOff : e[0] == '1' ? kSync : kAsync);
    if (const char* e = std::getenv("IMPLISOLID_JIT_BAKE")) set_bake(e[0] - '0');
    if (const char* e = std::getenv("IMPLISOLID_JIT_MAX_MODULES")) set_max_modules(std::atoi(e));
    const char* d = std::getenv("IMPLISOLID_JIT_CACHE");
    if (d && (!std::strcmp(d, "off") || !std::strcmp(d, "0"))) {
        disk_dir_.clear();
    } else if (d && d[0]) {
        disk_dir_ = d;
    } else if (const char* x = std::getenv("XDG_CACHE_HOME")) {
        disk_dir_ = std::string(x) + "/implisolid_amd";
    } else if (const char* h = std::getenv("HOME")) {
        disk_dir_ = std::string(h) + "/.cache/implisolid_amd";
    }
}

double TreeJit::compile_seconds() const { return compile_us_.load() * 1e-6; }

namespace {

uint64_t fnv1a(const char* p, size_t n, uint64_t h = 1469598103934665603ull) {
    for (size_t i = 0; i < n; ++i) { h ^= (unsigned char)p[i]; h *= 1099511628211ull; }
    return h;
}

// the device's architecture string (gcnArchName), once per device
std::string device_arch(int device) {
    static std::mutex mu;
    static std::map<int, std::string> names;
    std::lock_guard<std::mutex> lock(mu);
    auto it = names.find(device);
    if (it != names.end()) return it->second;
    hipDeviceProp_t prop{};
    std::string name = hipGetDeviceProperties(&prop, device) == hipSuccess ? std::string(prop.gcnArchName) : "unknown";
    names.emplace(device, name);
    return name;
}

// FNV-1a over the source, the headers it includes, the compile options, the hipRTC version and
// the device's architecture: the disk cache key
std::string source_hash(const std::string& src, int device) {
    uint64_t h = fnv1a(src.data(), src.size());
    for (int k = 0; k < kJitNumHeaders; ++k) h = fnv1a(kJitHeaderSources[k], std::strlen(kJitHeaderSources[k]), h);
    int major = 0, minor = 0;
    (void)hiprtcVersion(&major, &minor);
    const std::string tag = "--offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 v5 (points: -disable-promote-alloca-to-lds) hiprtc " + std::to_string(major) +
                            "." + std::to_string(minor) + " " + device_arch(device);
    h = fnv1a(tag.data(), tag.size(), h);
    char buf[32];
    std::snprintf(buf, sizeof buf, "%016llx", (unsigned long long)h);
    return buf;
}

// the integrity record stored beside a cached code object: its size and FNV-1a hash
std::string code_meta(const std::vector<char>& code) {
    char buf[64];
    std::snprintf(buf, sizeof buf, "%zu %016llx", code.size(), (unsigned long long)fnv1a(code.data(), code.size()));
    return buf;
}

bool read_file(const std::string& path, std::vector<char>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    const bool ok = n > 0 && std::fread(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

void write_file_atomic(const std::string& dir, const std::string& name, const std::vector<char>& data) {
    std::string path;   // mkdir -p
    for (size_t i = 1; i <= dir.size(); ++i)
        if (i == dir.size() || dir[i] == '/') (void)::mkdir(dir.substr(0, i).c_str(), 0755);
    // unique per process, thread and call: concurrent writers of one entry never share a temp file
    static std::atomic<uint64_t> counter{0};
    const std::string tmp = dir + "/." + name + "." + std::to_string((long)::getpid()) + "." +
                            std::to_string(std::hash<std::thread::id>()(std::this_thread::get_id())) + "." +
                            std::to_string(counter.fetch_add(1)) + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return;
    const bool ok = std::fwrite(data.data(), 1, data.size(), f) == data.size();
    std::fclose(f);
    if (!ok || std::rename(tmp.c_str(), (dir + "/" + name).c_str()) != 0) std::remove(tmp.c_str());
}

// The disk cache keeps at most IMPLISOLID_JIT_CACHE_MAX code objects (default 2048): once per
// process, before its first write, the least recently used entries beyond that (by modification
// time; a disk hit refreshes it) are removed with their .src / .meta files, down to 3/4 of the cap.
void trim_disk_cache(const std::string& dir) {
    size_t cap = 2048;
    if (const char* e = std::getenv("IMPLISOLID_JIT_CACHE_MAX")) cap = (size_t)std::max(16L, std::atol(e));
    DIR* d = ::opendir(dir.c_str());
    if (!d) return;
    std::vector<std::pair<long long, std::string>> cos;   // (mtime ns, name)
    while (const dirent* ent = ::readdir(d)) {
        const std::string nm = ent->d_name;
        if (nm.size() < 4 || nm.compare(nm.size() - 3, 3, ".co") != 0 || nm[0] == '.') continue;
        struct stat st{};
        if (::stat((dir + "/" + nm).c_str(), &st) != 0) continue;
        cos.emplace_back((long long)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec, nm);
    }
    ::closedir(d);
    if (cos.size() <= cap) return;
    std::sort(cos.begin(), cos.end());
    const size_t drop = cos.size() - cap * 3 / 4;
    for (size_t i = 0; i < drop; ++i) {
        const std::string base = dir + "/" + cos[i].second;
        std::remove(base.c_str());
        std::remove((base + ".src").c_str());
        std::remove((base + ".meta").c_str());
    }
}

}  // namespace

void TreeJit::build(Slot* slot) {
    const auto t0 = std::chrono::steady_clock::now();
    try {
        std::vector<char> code;
        const std::string name = source_hash(slot->src, slot->device) + ".co";
        // the disk copy is only trusted with its source beside it (a hash collision cannot alias) and
        // with its size and checksum matching the integrity record written after it
        std::vector<char> src_on_disk, meta_on_disk;
        bool from_disk = false;
        if (!disk_dir_.empty() && read_file(disk_dir_ + "/" + name, code) &&
            read_file(disk_dir_ + "/" + name + ".src", src_on_disk) &&
            std::string(src_on_disk.begin(), src_on_disk.end()) == slot->src &&
            read_file(disk_dir_ + "/" + name + ".meta", meta_on_disk) &&
            std::string(meta_on_disk.begin(), meta_on_disk.end()) == code_meta(code)) {
            ++n_disk_;
            from_disk = true;
            (void)::utimes((disk_dir_ + "/" + name).c_str(), nullptr);   // recently used (trim order)
        }
        auto compile_and_store = [&](const std::string& src) {
            code = compile(src);
            compile_us_ += (int64_t)(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
            ++n_compiled_;
            if (!disk_dir_.empty()) {
                static std::once_flag trimmed;
                std::call_once(trimmed, [this] { trim_disk_cache(disk_dir_); });
                write_file_atomic(disk_dir_, name + ".src", std::vector<char>(slot->src.begin(), slot->src.end()));
                write_file_atomic(disk_dir_, name, code);
                const std::string m = code_meta(code);
                write_file_atomic(disk_dir_, name + ".meta", std::vector<char>(m.begin(), m.end()));
            }
        };
        if (!from_disk) compile_and_store(slot->src);
        // the process is exiting (shutdown() joins this worker): load nothing into a runtime that
        // is being torn down
        {
            std::lock_guard<std::mutex> lock(mu_);
            if (stop_) {
                slot->failed.store(true, std::memory_order_release);
                return;
            }
        }
        int prev = 0;
        (void)hipGetDevice(&prev);
        if (prev != slot->device) IMPLI_HIP_THROW(hipSetDevice(slot->device));
        Kernels k;
        PointKernels pk;
        auto load = [&](const std::vector<char>& co) {
            bool ok = hipModuleLoadData(&slot->mod, co.data()) == hipSuccess;
            if (ok && slot->kind == kBricks)
                ok = hipModuleGetFunction(&k.bricks, slot->mod, "impli_eval_bricks") == hipSuccess &&
                     hipModuleGetFunction(&k.coarse, slot->mod, "impli_coarse_modes") == hipSuccess &&
                     hipModuleGetFunction(&k.refine, slot->mod, "impli_brick_refine") == hipSuccess;
            if (ok && slot->kind == kPoints)
                ok = hipModuleGetFunction(&pk.cnormals, slot->mod, "impli_pt_centroid_normals") == hipSuccess &&
                     hipModuleGetFunction(&pk.prep, slot->mod, "impli_pt_project_prep") == hipSuccess &&
                     hipModuleGetFunction(&pk.early, slot->mod, "impli_pt_project_early") == hipSuccess &&
                     hipModuleGetFunction(&pk.early2, slot->mod, "impli_pt_project_early2") == hipSuccess &&
                     hipModuleGetFunction(&pk.late, slot->mod, "impli_pt_project_late") == hipSuccess &&
                     hipModuleGetFunction(&pk.normals, slot->mod, "impli_pt_normals_at") == hipSuccess &&
                     hipModuleGetFunction(&pk.points, slot->mod, "impli_pt_points") == hipSuccess;
            return ok;
        };
        bool ok = load(code);
        if (!ok && from_disk) {   // a cached object that does not load: compile it again and rewrite the entry
            if (slot->mod) (void)hipModuleUnload(slot->mod);
            slot->mod = nullptr;
            from_disk = false;
            compile_and_store(slot->src);
            ok = load(code);
        }
        // the eval kernel asks for eight waves per SIMD; a tree whose code then spills to scratch is
        // compiled again without the request (stored under the same source key: deterministic)
        const size_t at = slot->src.find(" __attribute__((amdgpu_waves_per_eu(");
        const size_t at_end = at == std::string::npos ? at : slot->src.find(")))", at);
        int scratch = 0;
        if (ok && slot->kind == kBricks && at_end != std::string::npos &&
            hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, k.bricks) == hipSuccess && scratch > 0) {
            (void)hipModuleUnload(slot->mod);
            slot->mod = nullptr;
            std::string plain = slot->src;
            plain.erase(at, at_end + 3 - at);
            code = compile(plain);
            if (!disk_dir_.empty()) {
                write_file_atomic(disk_dir_, name, code);
                const std::string m = code_meta(code);
                write_file_atomic(disk_dir_, name + ".meta", std::vector<char>(m.begin(), m.end()));
            }
            ok = load(code);
        }
        if (prev != slot->device) (void)hipSetDevice(prev);
        if (!ok) throw std::runtime_error("hipModuleLoadData / hipModuleGetFunction failed");
        slot->k = k;
        slot->pk = pk;
        slot->ready.store(true, std::memory_order_release);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "implisolid: tree JIT failed, using the interpreter (%s)\n", std::string(e.what()).substr(0, 400).c_str());
        slot->failed.store(true, std::memory_order_release);
    }
}

void TreeJit::worker() {
    for (;;) {
        Slot* slot = nullptr;
        {
            std::unique_lock<std::mutex> lock(mu_);
            cv_.wait(lock, [this] { return stop_ || !queue_.empty(); });
            if (queue_.empty()) return;   // stop_ and drained
            slot = queue_.front();
            queue_.pop_front();
            ++busy_;
        }
        build(slot);
        {
            std::lock_guard<std::mutex> lock(mu_);
            --busy_;
        }
        idle_cv_.notify_all();
    }
}

void TreeJit::shutdown() {   // at exit: drop queued work, finish what is compiling, join
    {
        std::lock_guard<std::mutex> lock(mu_);
        stop_ = true;
        for (Slot* s : queue_) s->failed.store(true);
        queue_.clear();
    }
    cv_.notify_all();
    for (auto& t : workers_)
        if (t.joinable()) t.join();
    workers_.clear();
}

// A caller stream being captured into a graph (torch.cuda.CUDAGraph captures in global mode) must
// not see the device synchronisation an unload needs: eviction then waits for a request made outside
// a capture.  Only the caller's own stream is asked (querying the null stream during a capture would
// itself invalidate it); a null caller stream is taken as not capturing.
bool TreeJit::defer_eviction(hipStream_t stream) {
    if (!stream) return false;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess) {
        (void)hipGetLastError();
        return true;
    }
    return st != hipStreamCaptureStatusNone;
}

TreeJit::Slot* TreeJit::request(const Program& p, int kind, bool bake, hipStream_t stream) {
    const int m = mode();
    if (m == kOff) return nullptr;
    std::string src;
    try {
        src = kind == kPoints ? point_source(p, bake) : kernel_source(p, bake);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "implisolid: tree JIT skipped (%s)\n", e.what());
        return nullptr;
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    // the disk-cache key's device architecture, queried here on the caller's thread: a worker then
    // makes no HIP runtime call before its compile is done (at exit it makes none at all, build())
    (void)device_arch(dev);
    Slot* slot = nullptr;
    bool fresh = false;
    std::vector<Slot*> evict;
    {
        std::lock_guard<std::mutex> lock(mu_);
        const std::string key = std::to_string(dev) + "\n" + src;
        auto it = cache_.find(key);
        if (it != cache_.end()) {
            slot = it->second;
        } else {
            slot = new Slot();
            slot->kind = kind;
            slot->src = std::move(src);
            slot->key = key;
            slot->device = dev;
            cache_.emplace(key, slot);
            fresh = true;
        }
        // the reference is taken under the same lock as the lookup: a slot found here is held
        // before any other request can evict it (evict_locked takes only slots with refs == 0)
        ++slot->refs;
        slot->last_use = ++tick_;
        // modules are unloaded at trim points (trim(): set_object, wait_idle), where the device is
        // synchronised anyway -- never here, where another thread may hold a global-mode graph
        // capture the unload's device synchronisation would invalidate.  Only a cache four times
        // over its bound (a process that never reaches a trim point) is trimmed here, and not
        // while the caller's own stream captures.
        if ((int)cache_.size() > 4 * max_modules_.load()) evict_locked(evict, defer_eviction(stream));
        if (fresh) {
            if (m == kAsync && !stop_) {
                queue_.push_back(slot);
                if (workers_.empty()) {   // a small pool, started on first use
                    // hipRTC loads its compiler (comgr, the builtins) at the first compile; loaded now,
                    // their static destructors are registered before the exit handler below, so at
                    // exit shutdown() joins a worker still compiling before the compiler is torn down
                    // (exiting with a compile in flight otherwise crashed in the compiler)
                    static const bool preloaded = [] {
                        (void)dlopen("libamd_comgr.so.3", RTLD_NOW | RTLD_GLOBAL);
                        (void)dlopen("libhiprtc-builtins.so.7", RTLD_NOW | RTLD_GLOBAL);
                        return true;
                    }();
                    (void)preloaded;
                    const unsigned hw = std::thread::hardware_concurrency();
                    const int n = (int)std::max(1u, std::min(4u, hw ? hw / 2 : 1u));
                    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { worker(); });
                    std::atexit([] { TreeJit::instance().shutdown(); });
                }
            }
        }
    }
    unload(evict);
    if (fresh && m == kAsync) cv_.notify_one();
    if (fresh && (m == kSync || stop_)) {
        build(slot);
        // another thread's sync request for the same source waits on idle_cv_ (the lock orders the
        // notification after its predicate check)
        { std::lock_guard<std::mutex> lock(mu_); }
        idle_cv_.notify_all();
    }
    if (m == kSync) {   // a slot queued earlier in async mode: wait for it
        std::unique_lock<std::mutex> lock(mu_);
        idle_cv_.wait(lock, [slot] { return slot->ready.load() || slot->failed.load(); });
    }
    return slot;
}

void TreeJit::evict_locked(std::vector<Slot*>& out, bool defer) {
    // the least recently requested finished slots nobody holds, down to 3/4 of the bound (one
    // eviction pays for many requests); queued or compiling slots are never taken.  Deferred (a
    // graph capture is in progress): nothing is taken now; the next request outside a capture
    // trims the cache.
    if (defer) {
        ++n_deferred_;
        return;
    }
    std::vector<Slot*> idle;
    for (auto& kv : cache_) {
        Slot* s = kv.second;
        if (s->refs == 0 && (s->ready.load(std::memory_order_acquire) || s->failed.load(std::memory_order_acquire)))
            idle.push_back(s);
    }
    std::sort(idle.begin(), idle.end(), [](const Slot* a, const Slot* b) { return a->last_use < b->last_use; });
    const size_t target = (size_t)max_modules_ * 3 / 4;
    for (Slot* s : idle) {
        if (cache_.size() <= target) break;
        cache_.erase(s->key);
        out.push_back(s);
    }
}

void TreeJit::unload(std::vector<Slot*>& slots) {
    // nothing references these slots: their last users synchronised before releasing them, and the
    // device is synchronised once more so no kernel of an unloaded module can still be in flight
    if (slots.empty()) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    std::map<int, bool> synced;
    for (Slot* s : slots) {
        if (s->mod) {
            if (!synced[s->device]) {
                (void)hipSetDevice(s->device);
                const hipError_t e = hipDeviceSynchronize();
                if (e != hipSuccess)   // an earlier kernel's fault surfaces here: report it where it shows
                    std::fprintf(stderr, "implisolid: device synchronisation before a module unload failed: %s\n",
                                 hipGetErrorString(e));
                synced[s->device] = true;
            }
            (void)hipSetDevice(s->device);
            (void)hipModuleUnload(s->mod);
        }
        delete s;
        n_evicted_.fetch_add(1);
    }
    (void)hipSetDevice(prev);
    slots.clear();
}

void TreeJit::release(Slot* slot) {
    if (!slot) return;
    std::lock_guard<std::mutex> lock(mu_);
    if (slot->refs > 0) --slot->refs;
}

int TreeJit::modules() const {
    std::lock_guard<std::mutex> lock(mu_);
    return (int)cache_.size();
}

void TreeJit::wait_idle() {
    {
        std::unique_lock<std::mutex> lock(mu_);
        idle_cv_.wait(lock, [this] { return queue_.empty() && busy_ == 0; });
    }
    trim();
}

void TreeJit::trim() {
    std::vector<Slot*> evict;
    {
        std::lock_guard<std::mutex> lock(mu_);
        if ((int)cache_.size() > max_modules_.load()) evict_locked(evict, false);
    }
    unload(evict);
}

std::vector<TreeJit::Slot*> TreeJit::precompile(const std::vector<Program>& progs, int threads) {
    if (mode() == kOff) return {};
    // register and queue every program's module (async), then drain the queue with extra threads
    const int saved = mode();
    mode_.store(kAsync);
    // the slots stay held (returned to the caller, who releases them once the batch's engines have
    // taken their own references):
    // a batch larger than the module bound must not evict its own early modules before its warm run
    std::vector<Slot*> held;
    for (const Program& p : progs) held.push_back(request(p, kBricks, bake() == kBakeAlways));
    mode_.store(saved);
    // let the pool drain the queue, with extra threads for a large batch
    std::vector<std::thread> extra;
    const int n_extra = std::max(0, std::min<int>(threads, (int)progs.size()) - 4);
    for (int i = 0; i < n_extra; ++i) extra.emplace_back([this] {
        for (;;) {
            Slot* slot = nullptr;
            {
                std::lock_guard<std::mutex> lock(mu_);
                if (queue_.empty()) return;
                slot = queue_.front();
                queue_.pop_front();
                ++busy_;
            }
            build(slot);
            {
                std::lock_guard<std::mutex> lock(mu_);
                --busy_;
            }
            idle_cv_.notify_all();
        }
    });
    for (auto& t : extra) t.join();
    wait_idle();
    return held;
}

// The eval kernel's occupancy request: eight waves per SIMD (64 VGPRs).  The config-4 tree's pair
// code needs 79 without it (six waves) and runs 1 us faster with it (22.6 -> 21.6 us, no scratch:
// the compiler rematerialises and keeps more in SGPR lanes); build() drops the request for a tree
// that would spill to scratch.  IMPLISOLID_EVAL_WAVES=n (diagnostics) asks for n, 0 for none.
static std::string eval_waves_attr() {
    const char* e = std::getenv("IMPLISOLID_EVAL_WAVES");
    if (!e || !*e) return kEvalWavesAttr;
    const int n = std::atoi(e);
    return n > 0 ? " __attribute__((amdgpu_waves_per_eu(" + std::to_string(n) + ")))" : "";
}

std::string TreeJit::kernel_source(const Program& p, bool bake) {
    std::vector<Node> nodes;
    int next = 0;
    const int root = parse(p, 0, nodes, next);
    if (next != p.n_instr) throw std::runtime_error("jit: trailing instructions");
    Emitter em{nodes, p, bake};
    const std::string f = em.emit(root, "x0", "y0", "z0", 4);
    IvEmitter iv{nodes, p, bake};
    const std::string r = iv.emit(root, "p0", 4);
    PairEmitter pe{nodes, p, bake};
    const auto f2 = pe.emit(root, "x0", "y0", "z0", "x0", "y0", "z1", 4);
    std::ostringstream s;
    if (const char* e = std::getenv("IMPLISOLID_EVAL_PAIR")) s << "#define IMPLI_EVAL_PAIR " << (e[0] == '1' ? 1 : 0) << "\n";
    if (const char* e = std::getenv("IMPLISOLID_REFINE_WAVE_MODES"))
        s << "#define IMPLI_REFINE_WAVE_MODES " << (e[0] == '1' ? 1 : 0) << "\n";
    s << kPrelude << "#include \"eval_bricks.hpp\"\n#include \"ifunc_interval.hpp\"\n#include \"brick_modes.hpp\"\n"
      << "namespace impli {\nusing namespace dev;\n"
      << "__device__ __forceinline__ float tree_f(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "                                        uint64_t modes, float x0, float y0, float z0) {\n"
      << em.out.str() << "    return " << f << ";\n}\n"
      << "__device__ __forceinline__ void tree_f2(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "                                        uint64_t modes, float x0, float y0, float z0, float z1,\n"
      << "                                        float& out0, float& out1) {\n"
      << pe.out.str() << "    out0 = " << f2.first << ";\n    out1 = " << f2.second << ";\n}\n"
      << "struct JitEval {\n    const float* M;\n    const float* tab;\n"
      << "    __device__ __forceinline__ float operator()(uint64_t m, float x, float y, float z) const {\n"
      << "        return tree_f(M, tab, m, x, y, z);\n    }\n"
      << "    __device__ __forceinline__ void pair(uint64_t m, float x, float y, float z0, float z1, float& f0,\n"
      << "                                         float& f1) const {\n"
      << "        tree_f2(M, tab, m, x, y, z0, z1, f0, f1);\n    }\n};\n"
      << "__device__ __forceinline__ Iv tree_iv(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "                                      float2 tab_range, Box p0, uint64_t modes_in, uint64_t& modes) {\n"
      << "    modes = modes_in;\n"
      << iv.out.str() << "    return " << r << ";\n}\n"
      << "struct JitIv {\n    const float* M;\n    const float* tab;\n    float2 tab_range;\n"
      << "    __device__ __forceinline__ Iv operator()(Box p, uint64_t mi, uint64_t& m) const {\n"
      << "        return tree_iv(M, tab, tab_range, p, mi, m);\n    }\n};\n"
      << "}  // namespace impli\n"
      << "extern \"C\" __global__ __launch_bounds__(" << kEvalBlock << ")" << eval_waves_attr() << " void impli_eval_bricks(\n"
      << "    const float* M, const float* tab, impli::GridDesc g, impli::BrickGrid bg, const uint64_t* modes,\n"
      << "    const uint32_t* list, const uint32_t* count, float* field, void* signs, impli::ClaimCtx cc) {\n"
      << "    impli::eval_bricks_body(impli::JitEval{M, tab}, g, bg, cc, modes, list, count, field, signs);\n}\n"
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

// the point modules' early pass: the two-loop form (project_early_body); IMPLISOLID_EARLY_SM=1
// selects the single loop (project_early_sm_body, measured slower: DESIGN "OB02 on the GPU"), its
// faces per wave chunk IMPLISOLID_EARLY_CHUNK
bool early_single_loop() {
    static const bool on = [] {
        const char* e = std::getenv("IMPLISOLID_EARLY_SM");
        return e ? std::atoi(e) != 0 : false;
    }();
    return on;
}
int early_chunk() {
    static const int c = [] {
        const char* e = std::getenv("IMPLISOLID_EARLY_CHUNK");
        const int v = e ? std::atoi(e) : 64;
        return v < 16 ? 16 : v > 4096 ? 4096 : v;
    }();
    return c;
}

std::string TreeJit::point_source(const Program& p, bool bake) {
    std::vector<Node> nodes;
    int next = 0;
    const int root = parse(p, 0, nodes, next);
    if (next != p.n_instr) throw std::runtime_error("jit: trailing instructions");
    PtEmitter ef{nodes, p, false};
    const std::string f = ef.emit(root, "x0", "y0", "z0", 4);
    PtEmitter eg{nodes, p, true};
    const std::string fg = eg.emit(root, "x0", "y0", "z0", 4);
    std::ostringstream s;
    // IMPLISOLID_PT_WAVES=n (experiments): an occupancy request of n waves per SIMD on the search
    // passes (none by default)
    static const int pt_waves = [] {
        const char* e = std::getenv("IMPLISOLID_PT_WAVES");
        return e ? std::atoi(e) : 0;
    }();
    const std::string occ = pt_waves > 0 ? " __attribute__((amdgpu_waves_per_eu(" + std::to_string(pt_waves) + ")))" : "";
    const char* early = early_single_loop() ? "project_early_sm_body" : "project_early_body";
    // IMPLISOLID_PT_FG_WAVES=n: an occupancy request of n waves per SIMD on the f + gradient passes
    // at arbitrary points (centroid normals, normals at the projected centroids)
    static const int fg_waves = [] {
        const char* e = std::getenv("IMPLISOLID_PT_FG_WAVES");
        return e ? std::atoi(e) : 0;
    }();
    const std::string occ_fg = fg_waves > 0 ? " __attribute__((amdgpu_waves_per_eu(" + std::to_string(fg_waves) + ")))" : "";
    // baked (a hot object's module): the matrices and parameter rows as a constexpr table of exact
    // literals, so every transform reads immediates -- the same operations on the same values (no
    // term is dropped: 0 * NaN stays NaN), but no loop-invariant matrix values held in registers
    // (the early search pass: 189 -> ~130 VGPRs for config 3's tree, two -> three waves per SIMD)
    std::string table, mparam = "M";
    if (bake) {
        std::ostringstream t;
        const int nm = std::max(1, (int)p.n_mats);
        t << "__device__ constexpr float kMb[" << 12 * nm << "] = {";
        for (int i = 0; i < nm; ++i)
            for (int k = 0; k < 12; ++k) t << (i || k ? ",\n    " : "\n    ") << float_literal(i < p.n_mats ? p.mats[i][k] : 0.f);
        t << "};\n";
        table = t.str();
        mparam = "M_unused";
    }
    const std::string mbind = bake ? "    const float* const M = kMb;\n" : "";
    // IMPLISOLID_PROJ_GROUP=2 / 8 (experiments): the searches' lanes per face in this module
    static const int proj_group = [] {
        const char* e = std::getenv("IMPLISOLID_PROJ_GROUP");
        const int v = e ? std::atoi(e) : 0;
        return v == 2 || v == 8 ? v : 0;
    }();
    if (proj_group) s << "#define IMPLI_PROJ_GROUP " << proj_group << "\n";
    s << kPrelude << "#include \"ob02_device.hpp\"\n"
      << "namespace impli {\nusing namespace dev;\n" << table
      << "__device__ __forceinline__ float tree_pf(const float* __restrict__ " << mparam << ", const float* __restrict__ tab,\n"
      << "                                         float x0, float y0, float z0) {\n"
      << mbind << ef.out.str() << "    return " << f << ";\n}\n"
      << "__device__ __forceinline__ float tree_pfg(const float* __restrict__ " << mparam << ", const float* __restrict__ tab,\n"
      << "                                          float x0, float y0, float z0, V3& g_out) {\n"
      << mbind << eg.out.str() << "    g_out = g" << fg.substr(1) << ";\n    return " << fg << ";\n}\n"
      << "struct JitPt {\n    const float* M;\n    const float* tab;\n"
      << "    __device__ __forceinline__ float f(float x, float y, float z) const { return tree_pf(M, tab, x, y, z); }\n"
      << "    __device__ __forceinline__ float fg(float x, float y, float z, V3& g) const { return tree_pfg(M, tab, x, y, z, g); }\n"
      << "};\n}  // namespace impli\n"
      << "using impli::JitPt;\nusing impli::ob::ProjArgs;\n"
      << "extern \"C\" __global__ __launch_bounds__(256)" << occ_fg << " void impli_pt_centroid_normals(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "    const float* v, const int32_t* f, const int64_t* rng, float* C, float* N) {\n"
      << "    impli::ob::centroid_normals_body(JitPt{M, tab}, v, f, rng, C, N);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void impli_pt_project_prep(const float* __restrict__ M, const float* __restrict__ tab, ProjArgs a) {\n"
      << "    impli::ob::project_prep_body(JitPt{M, tab}, a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256)" << occ << " void impli_pt_project_early(const float* __restrict__ M, const float* __restrict__ tab, ProjArgs a) {\n"
      << "    impli::ob::" << early << "(JitPt{M, tab}, a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256)" << occ << " void impli_pt_project_early2(const float* __restrict__ M, const float* __restrict__ tab, ProjArgs a) {\n"
      << "    impli::ob::project_early_body<2>(JitPt{M, tab}, a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256)" << occ << " void impli_pt_project_late(const float* __restrict__ M, const float* __restrict__ tab, ProjArgs a) {\n"
      << "    impli::ob::project_late_body(JitPt{M, tab}, a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256)" << occ_fg << " void impli_pt_normals_at(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "    const float* P, const int64_t* rng, float* G, const uint32_t* pend, int mode) {\n"
      << "    impli::ob::normals_at_body(JitPt{M, tab}, P, rng, G, pend, mode);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void impli_pt_points(const float* __restrict__ M, const float* __restrict__ tab,\n"
      << "    const float* xyz, int64_t n, float* f, float* grad) {\n"
      << "    impli::ob::points_body(JitPt{M, tab}, xyz, n, f, grad);\n}\n";
    return s.str();
}

std::vector<char> TreeJit::compile(const std::string& src) {
    hiprtcProgram prog = nullptr;
    rtc_check(hiprtcCreateProgram(&prog, src.c_str(), "impli_tree.hip", kJitNumHeaders, kJitHeaderSources,
                                  kJitHeaderNames),
              "hiprtcCreateProgram");
    // the static library's floating-point contract: no FMA contraction, IEEE division/sqrt.  Point
    // modules: no promotion of private arrays to LDS -- whether the compiler promoted them varied
    // from process to process for the same source (18 KB per workgroup on the rabbit's trees, their
    // f + gradient passes 3-5x slower: profiles/r05zf_*), so it is ruled out explicitly.
    const bool points = src.find("impli_pt_project_early") != std::string::npos;
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17", "-mllvm",
                          "-disable-promote-alloca-to-lds"};
    const hiprtcResult r = hiprtcCompileProgram(prog, points ? 6 : 4, opts);
    // hipRTC loads its compiler libraries at the first compile, and their static destructors run at
    // exit before the handlers registered earlier: shutdown() (which joins a worker still compiling)
    // is registered once more now, so it runs before those destructors (a process that exited with
    // a compile in flight crashed in the compiler's torn-down state).  shutdown() is idempotent.
    static std::once_flag exit_hook;
    std::call_once(exit_hook, [] { std::atexit([] { TreeJit::instance().shutdown(); }); });
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

void TreeJit::launch_bricks(hipFunction_t fn, const float* d_mats, const float* d_rabbit, const GridDesc& g,
                            const BrickGrid& bg, const uint64_t* d_modes, const uint32_t* d_list,
                            const uint32_t* d_count, float* d_field, void* d_signs, const ClaimCtx& cc, unsigned blocks,
                            hipStream_t s) {
    if (bg.n_bricks <= 0) return;
    GridDesc gg = g;
    BrickGrid bb = bg;
    ClaimCtx c = cc;
    void* args[] = {(void*)&d_mats, (void*)&d_rabbit, (void*)&gg, (void*)&bb, (void*)&d_modes,
                    (void*)&d_list, (void*)&d_count, (void*)&d_field, (void*)&d_signs, (void*)&c};
    if (hipModuleLaunchKernel(fn, blocks, 1, 1, kEvalBlock, 1, 1, 0, s, args, nullptr) != hipSuccess)
        throw std::runtime_error("hipModuleLaunchKernel(impli_eval_bricks) failed");
}

void TreeJit::launch(hipFunction_t fn, unsigned blocks, void** args, hipStream_t s, const char* what) {
    if (hipModuleLaunchKernel(fn, blocks, 1, 1, 256, 1, 1, 0, s, args, nullptr) != hipSuccess)
        throw std::runtime_error(std::string("hipModuleLaunchKernel(") + what + ") failed");
}

}  // namespace impli
