// program.hpp -- the implicit-function tree compiled to a flat, wave-uniform node program.
//
// The reference evaluates its tree of virtual implicit_function objects node by node over whole
// batches, copying the batch at every transformed node (prepare_inner_vectors,
// basic_functions.hpp:361-379).  Here the tree (object_factory.hpp:56-758) is compiled once on the
// host into a post-order program that every lane of a wave interprets in lock step: the program
// counter, the stack depths and the matrices are uniform, so they live in SGPRs and the
// per-sample state (point stack, value stack) lives in VGPRs.
//
//   XFORM k   push M_k^-1 * top-point            (the node's own inverse matrix)
//   PRIM t    pop point, push f_t(point)         (egg, rabbit cube, cylinder, cone, heart, torus,
//                                                 double mushroom, screw, top/bottom lid, half plane;
//                                                 parameters in mats[prm])
//   CSG t     pop point, pop f2, f1, push f1 (op) f2   (Union / Intersection / Difference)
//
// With gradients enabled every value slot carries (f, gx, gy, gz) and every XFORM'd node applies
// M^-T to the selected gradient on the way up, exactly like eval_gradient in
// transformed_union.hpp:54-84 (children's f and grad are computed once and reused).
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#endif

namespace impli {

enum NodeType : int32_t {
    NT_UNION = 0,
    NT_INTERSECTION = 1,
    NT_DIFFERENCE = 2,
    NT_ELLIPSOID = 3,
    NT_CUBE = 4,
    NT_CYLINDER = 5,
    NT_CONE = 6,
    NT_HEART = 7,
    NT_TORUS = 8,
    NT_DMUSHROOM = 9,
    NT_SCREW = 10,        // screw.hpp (identity transformation_matrix), params {twist, r0, delta}
    NT_LID = 11,          // top_bottom_lid.hpp
    NT_HALF_PLANE = 12,   // half_plane.hpp, params {unit plane_vector, plane_point}
    NT_TETRA = 13,        // tetrahedron.hpp, params {a, b, c, d} x 4 oriented planes
    NT_METABALLS = 14,    // meta_balls_Rydgard.hpp, params {x, y, z, strength, subtract} x 4 balls
    NT_EXTRUSION = 15,    // extrusion.hpp + convex_polygon.hpp, params {n, (nx, ny, n0) x n}
    NT_SCREW_TBB = 16,    // inf_top_bot_bound.hpp over the screw ("screw_gradient_wrong"), params
                          // {twist, r0, delta} then (next row) the node's inverse matrix
};

enum OpCode : int32_t {
    OP_XFORM = 0,
    OP_PRIM = 1,
    OP_CSG = 2,
};

struct Instr {
    int16_t op;          // OpCode
    int16_t type;        // PRIM/CSG: NodeType; XFORM: XformPattern of its matrix
    int16_t mat;         // index of the node's inverse matrix (XFORM: the one to apply)
    int16_t csg;         // OP_CSG: index of this CSG node (pruning modes), else -1
    int16_t skip_csg;    // XFORM that starts a CSG operand: that CSG node's index, else -1
    int16_t skip_child;  // ... operand 0 or 1
    int16_t skip_to;     // ... first instruction after the operand's subtree
    int16_t prm;         // OP_PRIM: row of mats[] holding the primitive's parameters (raw floats)
};
static_assert(sizeof(Instr) == 16, "Instr layout");

// XFORM instructions: the pattern of the node's matrix, set by compile_mp5 (host.cpp).  XF_DIAG:
// every off-diagonal coefficient of the three rows is +-0, every translation is finite and not -0
// and every diagonal coefficient finite -- a scale + translate, whose rows the brick interpreters
// evaluate as m_dd v + m_d3 (xform_diag): at the finite sample points of a brick that is the full
// row's value (a zero coefficient adds a +-0, which the row's final + m_d3 != -0 absorbs), exactly
// the row the JIT emits for such a matrix (jit.cpp xform_row).  Points that may be NaN or infinite
// (OB02 vertices) keep the full rows.  Limit: "finite" holds for a nested transform's input only
// while no outer transform overflows the float range: a scale chain taking a grid coordinate past
// 3.4e38 makes a coordinate +-inf, where the full row gives 0 * inf = NaN and this row a finite value
// (ADVICE r04).  Such a tree has no surface at any float resolution; its field is not compared with
// the reference there (parity unpinned in that corner).
enum XformPattern : int16_t { XF_GENERIC = 0, XF_DIAG = 1 };

// Per-brick pruning: 2 bits per CSG node (index < kMaxPruned): both operands, left only, right only.
enum PruneMode : uint32_t { PM_BOTH = 0, PM_LEFT = 1, PM_RIGHT = 2 };
constexpr int kMaxPruned = 32;

constexpr int kMaxProgram = 256;   // instructions
constexpr int kMaxDepth = 16;      // point/value stack depth (tree depth + 1)

// Device-resident program (one per object).  Matrices are the inverse transforms
// (inv_transf_matrix), row-major 3x4.
struct Program {
    int32_t n_instr;
    int32_t max_depth;
    int32_t n_mats;
    int32_t n_csg;
    Instr instr[kMaxProgram];
    float mats[kMaxProgram][12];
};

}  // namespace impli
