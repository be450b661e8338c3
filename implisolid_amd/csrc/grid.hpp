// grid.hpp -- sampling grid and brick decomposition shared by the static kernels and the
// JIT-compiled ones (device-safe: no host declarations).
#pragma once
#ifndef __HIPCC_RTC__   // hipRTC (jit.cpp) provides these through its prelude
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

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

// pruned field evaluation: bricks of kBX x kBY x kBZ stored samples (x fastest).  8 x 8 x 2 bricks
// under 8 x 8 x 16 coarse boxes measured fastest at R = 512 on config 4 (594 vs 575 Gvox/s for
// 8 x 8 x 4 under 8 x 8 x 16; 8 x 8 x 8 under 8 x 8 x 16: 449): small bricks cut the evaluated
// samples (4.3 % vs 6.8 %), the JIT interval pass keeps their bounds cheap.
#ifndef IMPLI_BRICK_X
#define IMPLI_BRICK_X 8
#define IMPLI_BRICK_Y 8
#define IMPLI_BRICK_Z 2
#endif
constexpr int kBX = IMPLI_BRICK_X, kBY = IMPLI_BRICK_Y, kBZ = IMPLI_BRICK_Z;
// the interval pass runs first over coarse boxes of kBX x kBY x (kCZ kBZ) samples and refines
// only the coarse boxes of mixed sign into bricks
constexpr int kCZ = 8;
static_assert(kBX * kBY == 64 && (kBX == 8 || kBX == 16 || kBX == 32), "a brick layer is one wave");
// the engine's counter block (u32 words): [0, 12) marching-cubes counters (mc_types.hpp),
// [12] brick-list length, [13] mixed coarse-box list length, [14] its copy for statistics,
// [16, 20) output overflow flags.
// The pruned eval zeroes it without a memset: the coarse pass's first block clears every word but
// [13], which it appends to; the fill kernel clears [13] once the refine pass has read it.
constexpr int kBrickListWord = 12, kCoarseListWord = 13, kOverflowWord = 16, kCounterWords = 32;
// [15]: the merged object-stream eval's claimed candidates (eval_listed_deferred)
constexpr int kClaimedWord = 15;
enum BrickClass : uint8_t { kBrickMixed = 0, kBrickPos = 1, kBrickNeg = 2, kBrickNoFill = 4 };
// fill[b] (written by the pruned eval) = class | fill class << 4 | flags.  Fill class kBrickPos /
// kBrickNeg: the brick's sign pieces are constant (no cell corner in it needs its exact value unless
// it is a claimed candidate) -- 0: listed, evaluated.
//   kBrickCandidate: sign-definite, and every face neighbour of another class is of mixed class.
//     Its values are needed only where a mixed neighbour's face samples take the other sign: the
//     mixed neighbour's wave checks that after its own evaluation and evaluates the candidate.
//   kBrickClaimed: set (atomically) by the first such wave.
enum BrickFlag : uint8_t { kBrickCandidate = 8, kBrickClaimed = 0x80 };
struct BrickGrid { int nbx, nby, nbz, n_bricks; };
// what a listed mixed brick's wave needs to find and evaluate its claimed neighbours
struct ClaimCtx {
    uint8_t* fill;            // null: no candidates (every brick that needs values is listed)
    const uint8_t* ccls;      // coarse classes: a brick of a mixed coarse box has refined modes
    const uint64_t* bmodes;   // per-brick modes (refine pass)
    const uint64_t* cmodes;   // per-coarse-box modes
    int cnbx, cplane;         // coarse grid: boxes per row, per layer
};
// list entry: brick index | kListCheck if the brick is of mixed class (its wave claims candidates)
constexpr uint32_t kListCheck = 0x80000000u;

// Field storage, brick-major: brick (bx, by, bz) of the slab's brick grid holds its kBX x kBY x kBZ
// stored samples contiguously (x fastest, then y, then layer), so one brick layer is kBX kBY floats
// (256 B: two whole 128 B lines).  The eval kernel's wave stores whole lines and a cell's corners
// mostly share lines.  Brick b's samples start at b * kBrickSamples (b as numbered by brick_of).
constexpr int kBrickSamples = kBX * kBY * kBZ;
__host__ __device__ inline int64_t field_index(const GridDesc& g, int sx, int sy, int layer) {
    const int nbx = (g.n + kBX - 1) / kBX, nby = (g.n + kBY - 1) / kBY;
    const int64_t b = (int64_t)(sx / kBX) + (int64_t)nbx * ((sy / kBY) + (int64_t)nby * (layer / kBZ));
    return b * kBrickSamples + ((layer % kBZ) * kBY + (sy % kBY)) * kBX + (sx % kBX);
}
// field_index = field_layer_term + field_y_term + field_x_term (the x and y terms stay below 2^31:
// one brick layer of the slab)
__host__ __device__ inline uint32_t field_x_term(int sx) {
    return (uint32_t)(sx / kBX) * kBrickSamples + (uint32_t)(sx % kBX);
}
__host__ __device__ inline uint32_t field_y_term(const GridDesc& g, int sy) {
    return (uint32_t)(sy / kBY) * (uint32_t)((g.n + kBX - 1) / kBX) * kBrickSamples + (uint32_t)(sy % kBY) * kBX;
}
__host__ __device__ inline int64_t field_layer_term(const GridDesc& g, int layer) {
    const int64_t nbx = (g.n + kBX - 1) / kBX, nby = (g.n + kBY - 1) / kBY;
    return (int64_t)(layer / kBZ) * nbx * nby * kBrickSamples + (int64_t)(layer % kBZ) * (kBX * kBY);
}
__host__ __device__ inline int64_t field_samples(const GridDesc& g) {   // allocation, padded bricks included
    const int64_t nbx = (g.n + kBX - 1) / kBX, nby = (g.n + kBY - 1) / kBY;
    const int64_t nbz = (g.fz1 - g.fz0 + kBZ - 1) / kBZ;
    return nbx * nby * (nbz > 0 ? nbz : 0) * kBrickSamples;
}

// Sign bitmap of the stored samples (bit set <=> sample < 0, MC's cube-index test): per stored
// sample row (layer, y) `sign_row_words(g)` 64-bit words, sample x at bit x % 64 of word x / 64.
// The eval kernels write it as kBX-bit pieces (one per brick row).
__host__ __device__ inline int sign_row_words(const GridDesc& g) { return (g.n + 63) / 64; }

}  // namespace impli
