// kernels.hpp -- launch-side declarations of the MI355X kernels (all on one HIP stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grid.hpp"
#include "mc_types.hpp"
#include "program.hpp"

namespace impli {

GridDesc make_grid(int R, const float box[6], int cz0, int cz1, int cz_emit);

void build_case_table(CaseInfo out[256]);

// K1: field at the slab's stored samples
void launch_eval_field(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g, float* d_field,
                       hipStream_t s);
// direct evaluation at arbitrary points (implicit values / gradients)
BrickGrid brick_grid(const GridDesc& g);
// K1a: interval pass -- per-brick CSG pruning modes and sign class (coarse boxes, then the bricks
// of mixed coarse boxes)
BrickGrid coarse_grid(const GridDesc& g);
// JIT-compiled interval kernels for the shape (jit.hpp); null members -> interpreter
struct JitIntervalKernels {
    hipFunction_t coarse = nullptr, refine = nullptr;
};
void launch_brick_modes(const Program* d_prog, int depth, const float* d_rabbit, float2 tab_range, const GridDesc& g,
                        uint64_t* d_cmodes, uint8_t* d_ccls, uint32_t* d_clist, uint32_t* d_counters, uint64_t* d_modes,
                        uint8_t* d_cls, hipStream_t s, const JitIntervalKernels* jit = nullptr,
                        hipEvent_t after_coarse = nullptr /* recorded between the two kernels (timing) */);
// K1b: neighbour rule -> fill[b], the list of bricks to evaluate, constant sign bits of the rest
void launch_brick_fill(const GridDesc& g, const uint8_t* d_ccls, const uint64_t* d_cmodes, const uint8_t* d_cls,
                       const uint64_t* d_modes, int sign_fill, uint8_t* d_fill, uint32_t* d_list, uint64_t* d_lmodes,
                       uint32_t* d_count, void* d_signs, uint32_t* d_umark, uint32_t mark_id, hipStream_t s);
// K1c (interpreter): the listed bricks; the JIT variant is TreeJit::launch_bricks (jit.hpp)
constexpr int kEvalBlock = 256;   // lanes per block of the brick eval kernels
// whole waves (a partial wave would share the next block's brick index), within __launch_bounds__
static_assert(kEvalBlock % 64 == 0 && kEvalBlock <= 256, "kEvalBlock: whole waves, at most 256 lanes");
unsigned eval_bricks_grid(const GridDesc& g);
void launch_eval_bricks_interp(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g,
                               const uint64_t* d_modes, const uint32_t* d_list, const uint32_t* d_count,
                               float* d_field, void* d_signs, const ClaimCtx& cc, hipStream_t s);
// sign bitmap of a fully written field (unpruned path)
void launch_signs_from_field(const GridDesc& g, const float* d_field, uint64_t* d_signs, hipStream_t s);
void launch_eval_points(const Program* d_prog, int depth, const float* d_rabbit, const float* d_xyz, int64_t n,
                        float* d_f, float* d_grad /* nullable: values only */, hipStream_t s);
// diagnostics: glibc sinf (0) / atanf (1) / atan2f (2) restatements on device operands
void launch_libm_probe(int which, const float* d_a, const float* d_b, int64_t n, float* d_out, hipStream_t s);
void launch_cos_probe(const double* d_a, int64_t n, double* d_out, hipStream_t s);

// K2 (count per group) and K2b (group bases + flat list of non-empty units)
void launch_mc_count(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s);
void launch_mc_scan(const GridDesc& g, const MCBuffers& b, hipStream_t s);
// K3 and K4
void launch_mc_verts(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s);
void launch_mc_faces(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s);

// One object's device state for the merged launches of an object stream (BASELINE config 5): every
// stage of eval + MC runs once for all objects, block row y = object y (same grid for all objects,
// each with its own node program, buffers and counters; the interpreter kernels, since every
// object has its own tree).
struct ObjArgs {
    const Program* prog;
    uint64_t* cmodes;
    uint8_t* ccls;
    uint32_t* clist;
    uint64_t* modes;
    uint8_t* cls;
    uint8_t* fill;
    uint32_t* blist;
    uint64_t* lmodes;
    uint32_t* umark;
    uint32_t mark_id;
    float* field;
    void* signs;
    uint32_t* counters;
    uint32_t* claimed;   // the merged eval's claimed candidates, appended at counters[kClaimedWord]
    MCBuffers mc;
};
// eval (interval passes, fill, listed bricks) and MC (count, scan, vertices, faces) of n objects;
// blocks per object are capped for the grid-stride kernels (small grids: most blocks would idle)
// Node-stack capacity: 9 slots for objects of depth <= 9 (the smallest capacity the compiler
// still indexes through VGPR index mode rather than select chains; the eval then runs four waves
// per SIMD, 128 VGPRs and a small spill), else the interpreter's 12 or 16
// every object's counter block (kCounterWords words) into d_out[n][kCounterWords]
void launch_gather_counters(const ObjArgs* d_objs, int n, uint32_t* d_out, hipStream_t s);
// device byte ranges to clear, one block each (an object stream's fresh engines' resets in one
// launch instead of a memset call per buffer); p 16-byte aligned, n <= kZeroPieceBytes
struct ZeroPiece { uint64_t p; uint32_t n, pad; };
constexpr uint32_t kZeroPieceBytes = 1u << 16;
void launch_zero_pieces(const ZeroPiece* d_pieces, int n, hipStream_t s);
void launch_batch_eval(const ObjArgs* d_objs, int n, int depth, int vdepth, const float* d_rabbit, float2 tab_range, const GridDesc& g,
                       int sign_fill, hipStream_t s);
constexpr int kBatchShallowDepth = 9;
// merged object streams: the shallow class as this many pipelines on separate streams (abi.hip;
// the deep class is always one more).  Config 5: 2 / 3 / 4 pipelines 0.58 / 0.64 / 0.85 ms against
// 0.545 for one (profiles/r04x_*): concurrent merged kernels contend more than they overlap.
constexpr int kBatchGroups = 1;
void launch_batch_mc(const ObjArgs* d_objs, int n, const CaseInfo* d_cases, const GridDesc& g, hipStream_t s);

}  // namespace impli
