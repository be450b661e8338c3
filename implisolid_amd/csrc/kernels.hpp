// kernels.hpp -- launch-side declarations of the MI355X kernels (all on one HIP stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grid.hpp"
#include "program.hpp"

namespace impli {

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
BrickGrid brick_grid(const GridDesc& g);
// K1a: interval pass -- per-brick CSG pruning modes and sign class
void launch_brick_modes(const Program* d_prog, int depth, const float* d_rabbit, float2 tab_range, const GridDesc& g,
                        uint64_t* d_modes, uint8_t* d_cls, hipStream_t s);
// K1b (interpreter): brick-pruned field; the JIT variant is TreeJit::launch_bricks (jit.hpp)
void launch_eval_bricks_interp(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g,
                               const uint64_t* d_modes, const uint8_t* d_cls, uint8_t* d_fill, int sign_fill,
                               float* d_field, void* d_signs, hipStream_t s);
// sign bitmap of a fully written field (unpruned path)
void launch_signs_from_field(const GridDesc& g, const float* d_field, uint64_t* d_signs, hipStream_t s);
void launch_eval_points(const Program* d_prog, int depth, const float* d_rabbit, const float* d_xyz, int64_t n,
                        float* d_f, float* d_grad /* nullable: values only */, hipStream_t s);

// MC pipeline.  Cells are numbered L = row * m + (x - 1), row = (z - cz0) * m + (y - 1); a unit is
// kUnitRows consecutive rows (contiguous in linear order), processed by one wave.
constexpr int kUnitRows = 4;
constexpr int kScanUPT = 8;            // units per lane in the unit scan
constexpr int kScanBlock = 1024 * kScanUPT;
struct MCBuffers {
    const float* field;
    const uint64_t* signs;   // sign bitmap of the stored samples (grid.hpp)
    uint4* unit_cnt;         // per unit {own, tri, act, halo own}; scanned in place to exclusive bases
    uint32_t* scan_blk;      // 8 per scan block: partial sums (5 components), then exclusive bases
    uint32_t* counters;      // [0] unused, [1] halo own, [2..5] totals own/tri/act/halo
    uint32_t* vid3;          // 3 * n_cells: slab-local vertex ids (vid - H, mod 2^32); faces add Voff
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

__host__ __device__ inline int64_t n_rows(const GridDesc& g) { return (int64_t)g.m * (g.cz1 - g.cz0); }
__host__ __device__ inline int64_t n_units(const GridDesc& g) { return (n_rows(g) + kUnitRows - 1) / kUnitRows; }
inline int64_t n_scan_blocks(const GridDesc& g) { return (n_units(g) + kScanBlock - 1) / kScanBlock; }

}  // namespace impli
