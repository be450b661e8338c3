// mc_types.hpp -- marching-cubes data shared by the static kernels and the JIT module
// (device-safe: no host declarations).
#pragma once
#include "grid.hpp"
#include "program.hpp"

namespace impli {

// per-case marching-cubes data derived from the Bourke tables
struct CaseInfo {
    uint8_t ntri;
    uint8_t nown;       // crossing edges among the cell's owned edges 5, 6, 10
    int8_t rank[3];     // first-use rank of owned slot (edge 5, 6, 10) or -1
    uint8_t pad;
    uint8_t tri[15];    // Bourke edge ids, 3 per triangle
    uint8_t owners;     // bit o: the case uses an edge owned by owner cell o (mc.hip k_mc_faces)
    uint8_t pad2[10];
};
static_assert(sizeof(CaseInfo) == 32, "CaseInfo layout");
// MC pipeline.  Cells are numbered L = row * m + (x - 1), row = (z - cz0) * m + (y - 1); a unit is
// kUnitRows consecutive rows (contiguous in linear order), processed by one wave.
constexpr int kUnitRows = 4;
constexpr int kGroupUnits = 64;        // units per group: one count block; the group scan's element
constexpr int kVertsWaves = 4;         // waves per verts block (grid-stride over the unit list)
constexpr int kVertsMaxBlocks = 4096;  // cells grid cap (2048: +1 us at 512^3)
constexpr int kScanParts = 6;          // group sums scanned: own, tri, act, halo own, heavy / light unit parts
// A unit with more than kHeavyCells active cells takes several 64-cell windows, so its parts live
// 2-3x longer than a one-window part: the flat list holds them first (from the front) and the
// light ones after them (placed from the list's end backwards), so the longest parts start in
// the vertex pass's first wave generation instead of trailing it.
constexpr uint32_t kHeavyCells = 64;
// A non-empty unit with many active cells is handed to several waves ("parts"): part p of P takes
// the unit's 64-cell windows w with w % P == p (the other windows only advance its bases).
constexpr int kPartCells = 128;        // active cells per part
constexpr int kMaxParts = 8;          // (part and part count: 4 bits each in upart)
constexpr int kChunkMaskBits = 24;     // chunks per row the vertex pass can skip by mask (R <= 1533)
struct MCBuffers {
    const float* field;
    const uint64_t* signs;   // sign bitmap of the stored samples (grid.hpp)
    uint4* unit_cnt;         // per group, its non-empty units {unit in group, own, tri, act bases} (k_mc_count)
    uint32_t* unit_part;     // ... and their parts: in-group part base | part count << 16
    uint32_t* unit_cmask;    // ... and their chunks holding non-trivial cells (bit c, c < kChunkMaskBits)
    uint32_t* scan_blk;      // [kScanParts + 1][n_groups]: group sums (own, tri, act, halo own, parts),
                             // then the group's non-empty unit count (not scanned)
    uint4* ulist;            // all parts of the non-empty units in order: {unit, vbase, fbase, abase}
    uint32_t* upart;         // ... part index | part count << 4 | the unit's chunk mask << 8 (k_unit_scan)
    uint32_t cap_parts;      // ulist / upart entries: heavy parts at [0, H), light at [cap - L, cap)
    const uint32_t* umark;   // [unit][chunk]: the 64-cell chunks of a unit whose cells touch an evaluated
    uint32_t mark_id;        // brick hold mark_id (k_brick_fill); null: every chunk is counted (dense eval)
    uint32_t* counters;      // [0] unit parts, [1] halo own (read by the vertex pass), [2..5] totals
                             // own/tri/act/halo (copied as one block; [5] == [1]), [6] non-empty units,
                             // [7] heavy unit parts (the flat list's front)
    uint32_t* vid;           // 3 * n_cells: per cell id L, the slab-local ids (vid - H, mod 2^32) of its
                             // owned edges 5, 6, 10, written for the cells owning a crossing edge (halo
                             // layer included; unused slots undefined) -- the face pass reads an owner's
                             // triple straight from its cell id
    uint4* records;          // active cells: {L, ci, fbase, cell row}
    float* verts;            // 3 * cap_v
    int32_t* faces;          // 3 * cap_f
    int64_t cap_v, cap_f, cap_rec;
    const uint32_t* offsets; // device [Voff, Foff] of this slab in the global numbering, or
    const uint32_t* gathered;  // the all-gathered counts uint32[rank+][4] of the slabs (copy_counts
    int rank;                  // layout): Voff = sum over lower ranks of (own incl. halo - halo)
    uint32_t* overflow;      // set to 1 if a capacity was exceeded
};
__host__ __device__ inline int64_t n_rows(const GridDesc& g) { return (int64_t)g.m * (g.cz1 - g.cz0); }
__host__ __device__ inline int64_t n_units(const GridDesc& g) { return (n_rows(g) + kUnitRows - 1) / kUnitRows; }
__host__ __device__ inline int64_t n_groups(const GridDesc& g) { return (n_units(g) + kGroupUnits - 1) / kGroupUnits; }
// 64-cell chunks per cell row (chunk c: the cells whose low corner is stored sample 64 c + j)
__host__ __device__ inline int n_chunks(const GridDesc& g) { return (g.m + 63) / 64; }
constexpr int kMaxChunks = 128;   // per row (R <= 8189): the count kernel's candidate list in LDS

}  // namespace impli
