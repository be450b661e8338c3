// kernels.hpp -- launch-side declarations of the MI355X kernels (all on one HIP stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "program.hpp"

namespace impli {

// Sampling grid of MarchingCubes (marching_cubes.hpp:175-243, 1662-1698) for one Z-slab.
//   res = R + 5 samples per axis; cells c in [1, res-3] per axis (render_geometry :1033-1039),
//   m = R + 2 cells per axis.  Cells touch samples [1, res-2]; those are stored (n = R + 3 per
//   axis, x fastest), the ring s in {1, res-2} holding seal_exterior's -1e7 (:895-963), so every
//   corner load is unconditional.  Samples 0 and res-1 are never read by any cell.
struct GridDesc {
    int R, res, n, m;            // n = R + 3 stored samples per axis, m = R + 2 cells per axis
    float w[3];                  // widthx/y/z = (max - min) / R
    float lo[3];                 // box min
    float i0[3];                 // render offsets xi0 = min / w - 2   (:1026-1028)
    int cz0, cz1;                // cell layers handled by this slab [cz0, cz1) (incl. halo layer)
    int cz_emit;                 // first layer whose faces / vertices this slab emits
    int fz0, fz1;                // stored sample layers [fz0, fz1) = [cz0, cz1 + 1)
    int64_t n_cells;             // m * m * (cz1 - cz0)
};

GridDesc make_grid(int R, const float box[6], int cz0, int cz1, int cz_emit);

// per-case marching-cubes data derived from the Bourke tables
struct CaseInfo {
    uint8_t ntri;
    uint8_t nown;       // crossing edges among the cell's owned edges 5, 6, 10
    int8_t rank[3];     // first-use rank of owned slot (edge 5, 6, 10) or -1
    uint8_t pad;
    uint8_t tri[15];    // Bourke edge ids, 3 per triangle
    uint8_t pad2[11];
};
static_assert(sizeof(CaseInfo) == 32, "CaseInfo layout");
void build_case_table(CaseInfo out[256]);

// K1: field at the slab's stored samples
void launch_eval_field(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g, float* d_field,
                       hipStream_t s);
// direct evaluation at arbitrary points (implicit values / gradients)
// pruned field evaluation: bricks of kBX x kBY x kBZ stored samples (x fastest)
constexpr int kBX = 16, kBY = 4, kBZ = 4;
enum BrickClass : uint8_t { kBrickMixed = 0, kBrickPos = 1, kBrickNeg = 2, kBrickNoFill = 4 };
// fill[b] (written by the pruned eval): kBrickPos / kBrickNeg if the brick was sign-filled --
// then no cell corner in it needs its exact value and MC may take the sign from fill -- else 0.
struct BrickGrid { int nbx, nby, nbz, n_bricks; };
BrickGrid brick_grid(const GridDesc& g);
void launch_eval_field_pruned(const Program* d_prog, int depth, const float* d_rabbit, float2 tab_range,
                              const GridDesc& g, uint64_t* d_modes, uint8_t* d_cls, uint8_t* d_fill, int sign_fill,
                              float* d_field, hipStream_t s, hipEvent_t mid = nullptr);
void launch_eval_points(const Program* d_prog, int depth, const float* d_rabbit, const float* d_xyz, int64_t n,
                        float* d_f, float* d_grad /* nullable: values only */, hipStream_t s);

// MC pipeline
constexpr int kUnitCells = 1024;       // cells per counting unit (contiguous in linear cell order)
constexpr int kScanUPT = 8;            // units per lane in the unit scan
constexpr int kScanBlock = 1024 * kScanUPT;
struct MCBuffers {
    const float* field;
    const uint8_t* fill;     // per brick of the field (BrickGrid nbx x nby x nbz), see BrickClass
    int nbx, nby;
    uint8_t* ci;             // cube index per cell (n_cells)
    uint4* unit_cnt;         // per unit {own, tri, act, halo own}; scanned in place to exclusive bases
    uint32_t* scan_blk;      // 8 per scan block: partial sums (5 components), then exclusive bases
    uint32_t* active_units;  // compacted list of units with work
    uint32_t* counters;      // [0] n_active_units, [1] halo own, [2..5] totals own/tri/act/halo
    uint32_t* vid3;          // 3 * n_cells
    uint4* records;          // active cells: {L, ci, fbase, 0}
    float* verts;            // 3 * cap_v
    int32_t* faces;          // 3 * cap_f
    int64_t cap_v, cap_f, cap_rec;
    const uint32_t* offsets; // device [Voff, Foff] of this slab in the global numbering
    uint32_t* overflow;      // set to 1 if a capacity was exceeded
};
void launch_mc_count(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s);
void launch_mc_scan(const GridDesc& g, const MCBuffers& b, hipStream_t s);
void launch_mc_emit(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s,
                    hipEvent_t mid = nullptr /* recorded between the vertex and face kernels */);

inline int64_t n_units(const GridDesc& g) { return (g.n_cells + kUnitCells - 1) / kUnitCells; }
inline int64_t n_scan_blocks(const GridDesc& g) { return (n_units(g) + kScanBlock - 1) / kScanBlock; }

}  // namespace impli
