// mc.hip -- marching cubes with the reference's vertex numbering, without any map.
//
// Reference: render_geometry / polygonize_single_cube / flush_geometry_queue
// (marching_cubes.hpp:518-718, 1019-1072, 1520-1658).  The reference walks cells in z->y->x order,
// emits triangle corners in Bourke-table order and numbers a vertex the first time its edge code
// (3*ijk + axis) is seen, through a std::map.
//
// Owner rule: the first cell to reference a crossing grid edge is the lowest-index
// cell containing it, i.e. the cell that holds it as local edge 5 (Y at corner (1,0,1)), 6 (X at
// (0,1,1)) or 10 (Z at (1,1,0)).  So vertex ids = exclusive scan over cells of "owned crossing
// edges", ordered inside a cell by first use in that cell's triangle list; face offsets =
// exclusive scan of triangle counts.  A vertex's coordinates are computed by its owner cell with
// the owner's fx/fy/fz, exactly as the reference's first emission did.
//
// Signs come from the eval's sign bitmap (grid.hpp), 64 cells per bit operation; only the ~1 % of
// non-trivial cells (corner signs not all equal) do per-cell work.  A unit = kUnitRows cell rows.
//   K2 k_mc_count : per unit the sums of owned edges, triangles, active cells, halo-owned edges.
//   K2b k_unit_scan: per group, its global bases (sum of the groups before it) and its non-empty
//       units in order in the flat list.
//   K3 k_mc_cells : per unit, the non-trivial cells in cell order (selected in parallel): owned
//                   vertex positions (field values read only at crossing edges), records {cell,
//                   case, face base, row} of the active cells with their owned-id triples beside
//                   them (record order), and the item table (per row and 64-cell chunk: the mask
//                   and first record index of its non-trivial cells).
//   K4 k_mc_faces : per active cell, gathers the vertex ids of its triangle corners from the
//                   owner cells' triples, found by record index through the item table.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "eval_bricks.hpp"
#include "ifunc_device.hpp"
#include "kernels.hpp"
#include "mc_device.hpp"
#include "batch_device.hpp"

namespace impli {

GridDesc make_grid(int R, const float box[6], int cz0, int cz1, int cz_emit) {
    GridDesc g{};
    g.R = R;
    g.res = R + 5;
    g.n = R + 3;
    g.m = R + 2;
    for (int a = 0; a < 3; ++a) {
        const float width = box[2 * a + 1] - box[2 * a];   // init(): marching_cubes.hpp:231-243
        g.w[a] = width / (float)R;
        g.lo[a] = box[2 * a];
        g.i0[a] = box[2 * a] / g.w[a] - 2.f;                // render_geometry :1026-1028
    }
    g.cz0 = cz0;
    g.cz1 = cz1;
    g.cz_emit = cz_emit;
    g.fz0 = cz0;        // cells [cz0, cz1) touch sample layers [cz0, cz1]
    g.fz1 = cz1 + 1;
    g.n_cells = (int64_t)g.m * g.m * (cz1 - cz0);
    return g;
}

void build_case_table(CaseInfo out[256]) {
    for (int ci = 0; ci < 256; ++ci) {
        CaseInfo c{};
        const char* s = IMPLI_MC_TRI_CASES[ci];
        int n = 0;
        for (; s[n]; ++n) c.tri[n] = (uint8_t)((s[n] <= '9') ? s[n] - '0' : s[n] - 'a' + 10);
        c.ntri = (uint8_t)(n / 3);
        c.rank[0] = c.rank[1] = c.rank[2] = -1;
        int r = 0;
        for (int k = 0; k < n; ++k) {
            const int e = c.tri[k];
            const int slot = (e == 5) ? 0 : (e == 6) ? 1 : (e == 10) ? 2 : -1;
            if (slot >= 0 && c.rank[slot] < 0) c.rank[slot] = (int8_t)r++;
        }
        c.nown = (uint8_t)r;
        static const int owner_of_edge[12] = {5, 4, 4, 6, 2, 0, 0, 1, 3, 2, 0, 1};   // = c_edge_owner_idx
        for (int k = 0; k < n; ++k) c.owners = (uint8_t)(c.owners | (1u << owner_of_edge[c.tri[k]]));
        // k_mc_count relies on two table properties (checked here for every case): the owned
        // edges a case's triangles use are exactly its crossing owned edges (Bourke edges 5 =
        // corners 5-6, 6 = 6-7, 10 = 2-6), and every non-trivial case has a triangle.
        auto neg = [ci](int k) { return (ci >> k) & 1; };
        const int crossing = (neg(5) ^ neg(6)) + (neg(6) ^ neg(7)) + (neg(2) ^ neg(6));
        // ... and the triangle count is E - 2 P (mc_device.hpp chunk_triangles)
        int ec = 0, ei = 0, v = 0, ff = 0, opp = 0;
        for (const auto& e : kCubeEdges) { ec += neg(e[0]) ^ neg(e[1]); ei += neg(e[0]) & neg(e[1]); }
        for (int k = 0; k < 8; ++k) v += neg(k);
        for (const auto& f : kCubeFaces) ff += neg(f[0]) & neg(f[1]) & neg(f[2]) & neg(f[3]);
        for (const auto& o : kCubeOpposite) opp += (v == 6 && !neg(o[0]) && !neg(o[1])) ? 1 : 0;
        const int ntri_formula = (ci == 0 || ci == 255) ? 0 : ec - 2 * (v - ei + ff + 2 * opp);
        if (crossing != c.nown || (c.ntri > 0) != (ci != 0 && ci != 255) || ntri_formula != c.ntri)
            throw std::runtime_error("marching cubes: case table violates the count kernel's assumptions");
        out[ci] = c;
    }
}

namespace {

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// K2: one block per group of kGroupUnits units; lanes take the group's items (row, 64-cell chunk)
// round robin, so every lane has work (a wave per unit would leave 64 - 4 nch lanes idle).  Only
// the 64-cell chunks of a unit whose cells touch an evaluated brick are visited (b.umark, marked per
// (unit, chunk) by k_brick_fill): all others are trivial.  Owned
// vertices and triangles of a chunk are popcounts of corner-mask expressions (chunk_triangles).
// Per-unit sums through LDS atomics.
//   -> unit_cnt[64 group + k] = k-th non-empty unit of the group {unit in group, own / tri / act
//      exclusive bases in the group}; scan_blk[c][group] = the group's sums (own, tri, act, halo
//      own, non-empty units), read by k_unit_scan.
__device__ __forceinline__ void mc_count_body(const GridDesc& g, const MCBuffers& b) {
    __shared__ uint32_t s_u[kGroupUnits][4];
    __shared__ uint32_t s_cm[kGroupUnits];   // per unit: its chunks holding non-trivial cells (bit c)
    __shared__ uint16_t s_fp[kGroupUnits * kMaxChunks];   // the group's candidate (unit, chunk) pairs
    __shared__ uint32_t s_nf;
    const int t = threadIdx.x, nt_ = blockDim.x;   // triangle counts: chunk_triangles (checked against the table)
    for (int k = t; k < 4 * kGroupUnits; k += nt_) (&s_u[0][0])[k] = 0u;
    for (int k = t; k < kGroupUnits; k += nt_) s_cm[k] = 0u;
    if (t == 0) s_nf = 0u;
    const int64_t G = blockIdx.x;
    const int nch = n_chunks(g);
    const int64_t rows = n_rows(g), nu = n_units(g);
    const int64_t row0 = G * kGroupUnits * kUnitRows;
    __syncthreads();
    // candidates: the (unit, chunk) pairs whose cells touch an evaluated brick (the others hold no
    // non-trivial cell), appended in any order (the counts are sums); a wave's appends take one
    // LDS atomic
    for (int p0 = 0; p0 < kGroupUnits * nch; p0 += nt_) {
        const int p = p0 + t, ui = p / nch, c = p - ui * nch;
        const int64_t u = G * kGroupUnits + ui;
        const bool cand = p < kGroupUnits * nch && u < nu && (!b.umark || b.umark[u * nch + c] == b.mark_id);
        const uint64_t m = __ballot(cand);
        uint32_t base = 0;
        if ((t & 63) == 0 && m) base = atomicAdd(&s_nf, (uint32_t)__popcll((unsigned long long)m));
        base = __shfl(base, 0, 64);
        if (cand) s_fp[base + __popcll((unsigned long long)(m & ((1ull << (t & 63)) - 1ull)))] = (uint16_t)(ui * kMaxChunks + c);
    }
    __syncthreads();
    const int n_items = (int)s_nf * kUnitRows;
    for (int i = t; i < n_items; i += nt_) {
        ChunkBits k;
        const uint32_t pr = s_fp[i / kUnitRows];
        const int ui = (int)(pr / kMaxChunks), c = (int)(pr % kMaxChunks);
        const int rb = ui * kUnitRows + i % kUnitRows;
        const bool ok = row0 + rb < rows;
        // out-of-range rows read a valid chunk (row 0) and drop it: no branch around loads
        load_chunk(g, b.signs, ok ? row0 + rb : 0, c, k);
        if (!ok) k.nt = 0;
        if (!k.nt) continue;
        if (c < kChunkMaskBits) atomicOr(&s_cm[ui], 1u << c);
        // owned vertices = crossing owned edges (build_case_table checks the identity):
        // edge 5 = corners 5-6 (t01, t11), 6 = 6-7 (t11, s11), 10 = 2-6 (t10, t11)
        const unsigned own = (unsigned)(__popcll((unsigned long long)((k.t01 ^ k.t11) & k.nt)) +
                                        __popcll((unsigned long long)((k.s11 ^ k.t11) & k.nt)) +
                                        __popcll((unsigned long long)((k.t10 ^ k.t11) & k.nt)));
        unsigned tri = 0, act = 0, hal = 0;
        if (k.z >= g.cz_emit) {
            act = (unsigned)__popcll((unsigned long long)k.nt);   // every non-trivial case has a triangle
            tri = chunk_triangles(k);
        } else {
            hal = own;
        }
        uint32_t* d = s_u[ui];
        if (own) atomicAdd(&d[0], own);
        if (tri) { atomicAdd(&d[1], tri); atomicAdd(&d[2], act); }
        if (hal) atomicAdd(&d[3], hal);
    }
    __syncthreads();
    if (t < 64) {   // wave 0, one lane per unit of the group (kGroupUnits == 64; blockDim >= 64)
        const int64_t u = G * kGroupUnits + t;
        const uint32_t own = s_u[t][0], tri = s_u[t][1], act = s_u[t][2], hal = s_u[t][3];
        const bool ne = u < nu && (own | tri) != 0;
        // the group's non-empty units in order, with their exclusive bases inside the group
        const uint32_t eo = wave_incl_scan<uint32_t>(own, t) - own;
        const uint32_t et = wave_incl_scan<uint32_t>(tri, t) - tri;
        const uint32_t ea = wave_incl_scan<uint32_t>(act, t) - act;
        const uint64_t m = __ballot(ne);
        const uint32_t pos = (uint32_t)__popcll((unsigned long long)(m & ((1ull << t) - 1ull)));
        // parts: a unit's active cells split into runs of kPartCells for separate waves; heavy
        // units' parts (mc_types.hpp kHeavyCells) and light units' parts counted apart
        const uint32_t parts = ne ? min((uint32_t)kMaxParts, max(1u, (act + kPartCells - 1) / kPartCells)) : 0u;
        const bool heavy = act > kHeavyCells;
        const uint32_t ph = heavy ? parts : 0u, pl = heavy ? 0u : parts;
        const uint32_t eph = wave_incl_scan<uint32_t>(ph, t) - ph, epl = wave_incl_scan<uint32_t>(pl, t) - pl;
        if (ne) {
            b.unit_cnt[G * kGroupUnits + pos] = make_uint4((uint32_t)t, eo, et, ea);
            b.unit_part[G * kGroupUnits + pos] = (heavy ? eph : epl) | (parts << 16) | ((uint32_t)heavy << 20);
            b.unit_cmask[G * kGroupUnits + pos] = s_cm[t];
        }
        const uint32_t sums[kScanParts + 1] = {__shfl(eo + own, 63, 64), __shfl(et + tri, 63, 64),
                                               __shfl(ea + act, 63, 64), wave_sum(hal), __shfl(eph + ph, 63, 64),
                                               __shfl(epl + pl, 63, 64), (uint32_t)__popcll((unsigned long long)m)};
        if (t <= kScanParts) {
            const uint32_t v = t == 0 ? sums[0] : t == 1 ? sums[1] : t == 2 ? sums[2] : t == 3 ? sums[3]
                             : t == 4 ? sums[4] : t == 5 ? sums[5] : sums[6];
            b.scan_blk[(int64_t)t * gridDim.x + G] = v;
        }
    }
}
__global__ __launch_bounds__(512) void k_mc_count(GridDesc g, MCBuffers b) { mc_count_body(g, b); }

// K2b: one block per group.  Its global bases are the sums of the groups before it, read straight
// from L2 (kScanParts x G words, all loads in flight together; nothing waits on another block), then
// its non-empty units go to their place in the flat ordered list.  Groups without non-empty units
// exit at once; the last group writes the totals.  (A single-block scan plus a flatten kernel took
// 7.3 + 4.5 us at 512^3; a decoupled look-back inside k_mc_count, 28 us more: its status words
// cross the XCDs' L2s at memory latency, one round trip per 64 groups walked.)
constexpr int kScanBlock = 256;
constexpr int kScanRows = kScanParts + 1;   // + the non-empty unit counts (summed for statistics)
template <int BS = kScanBlock>
__device__ __forceinline__ void unit_scan_body(const GridDesc& g, const MCBuffers& b) {
    static_assert(BS >= kGroupUnits, "a lane per unit of the group");
    __shared__ uint32_t s_part[BS / 64][kScanRows];
    __shared__ uint32_t s_base[kScanRows];
    const int64_t G = blockIdx.x, ng = n_groups(g);
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const bool last = G == ng - 1;
    const uint32_t nne = b.scan_blk[kScanParts * ng + G];   // non-empty units of the group
    if (nne == 0 && !last) return;   // uniform
    const uint4 e = b.unit_cnt[G * kGroupUnits + (t < (int)nne ? t : 0)];
    const uint32_t pp = b.unit_part[G * kGroupUnits + (t < (int)nne ? t : 0)];
    const uint32_t cm = b.unit_cmask[G * kGroupUnits + (t < (int)nne ? t : 0)];
    uint32_t acc[kScanRows] = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll 4
    for (int64_t i = t; i < G; i += BS)
#pragma unroll
        for (int c = 0; c < kScanRows; ++c) acc[c] += b.scan_blk[c * ng + i];
#pragma unroll
    for (int c = 0; c < kScanRows; ++c) {
        const uint32_t s = wave_sum(acc[c]);
        if (lane == 0) s_part[wid][c] = s;
    }
    __syncthreads();
    if (t < kScanRows) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < BS / 64; ++w) s += s_part[w][t];
        s_base[t] = s;
    }
    __syncthreads();
    if (t < (int)nne) {
        const uint4 ent = make_uint4((uint32_t)(G * kGroupUnits) + e.x, s_base[0] + e.y, s_base[1] + e.z, s_base[2] + e.w);
        const uint32_t P = (pp >> 16) & 15u;
        const bool heavy = (pp >> 20) & 1u;
        // heavy parts from the list's front, light parts from its end backwards
        const uint32_t r = (heavy ? s_base[4] : s_base[5]) + (pp & 0xffffu);
        for (uint32_t q = 0; q < P; ++q) {
            const uint32_t at = heavy ? r + q : b.cap_parts - 1u - (r + q);
            b.ulist[at] = ent;
            b.upart[at] = q | (P << 4) | (cm << 8);
        }
    }
    if (last && t == 0) {
        const uint32_t nh = s_base[4] + b.scan_blk[4 * ng + G];
        b.counters[7] = nh;                                       // heavy parts (the list's front)
        b.counters[0] = nh + s_base[5] + b.scan_blk[5 * ng + G];  // unit parts
        b.counters[1] = s_base[3] + b.scan_blk[3 * ng + G];       // halo-owned vertices (ids below the slab's first)
        b.counters[2] = s_base[0] + b.scan_blk[G];                // owned vertices incl. halo
        b.counters[3] = s_base[1] + b.scan_blk[ng + G];           // triangles
        b.counters[4] = s_base[2] + b.scan_blk[2 * ng + G];       // active cells (face records)
        b.counters[5] = s_base[3] + b.scan_blk[3 * ng + G];       // = [1]: [2, 6) is the totals block
                                                                  // copy_counts / read_counts take whole
        b.counters[6] = s_base[6] + nne;                          // non-empty units (statistics)
    }
}
__global__ __launch_bounds__(kScanBlock) void k_unit_scan(GridDesc g, MCBuffers b) { unit_scan_body<>(g, b); }

__global__ __launch_bounds__(64 * kVertsWaves) __attribute__((amdgpu_waves_per_eu(6))) void k_mc_cells(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    mc_cells_body(cases, g, b);
}

// The face grid: the XCD remap below is a permutation of the blocks only when it is a multiple of 8.
constexpr unsigned kFacesBlocks = 2048;
static_assert(kFacesBlocks % 8 == 0, "k_mc_faces' XCD remap needs a multiple of 8 blocks");

// Bourke edge e of a cell is owned (edge 5, 6 or 10) by one of 7 cells: the cell itself, or its
// neighbour at -x, -y, -x-y, -z, -y-z, -x-z; owner index and owned slot per edge
__constant__ uint8_t c_edge_owner_idx[12] = {5, 4, 4, 6, 2, 0, 0, 1, 3, 2, 0, 1};
__constant__ uint8_t c_edge_slot[12] = {1, 0, 1, 0, 1, 0, 1, 0, 2, 2, 2, 2};

// K4: one lane per active cell, XCD-aware (the dispatcher puts block b on XCD b % 8, so XCD x takes
// the x-th eighth of the records in cell order and the owner cells it gathers from stay in its L2).
// A lane needs the owned-id triples of the owner cells its case uses (at most 7): the vertex pass
// wrote every owning cell's triple at its cell id (vid), so an owner's triple is one load at the
// cell id L minus the owner's offset (-x: 1, -y: m, -z: m^2; an owner in the halo layer below the
// slab's first emitted one is a cell of the slab like any other).  Round 6: this replaced the
// record-ordered triples and the (row, 64-cell chunk) item table that found an owner's record --
// one dependent round trip (record -> items -> triples) fewer.  Every address is formed before any
// load is used (a load under a divergent branch waits alone); an owner the case does not use reads
// the cell's own triple.  The 12 edges' ids go to LDS, and each triangle is one 12-byte store.
// one active-cell record i of a slab: its triangles with the vertex ids of their corners
__device__ __forceinline__ void face_record(const CaseInfo* s_case, uint32_t (*s_w)[256], const GridDesc& g,
                                            const MCBuffers& b, uint32_t Voff, uint32_t i) {
    const int t = threadIdx.x;
    const uint4 r = b.records[i];
    const uint32_t L = r.x, ci = r.y, fbase = r.z;
    const CaseInfo& C = s_case[ci];
    const int ntri = C.ntri;
    if (fbase + ntri > (uint64_t)b.cap_f) { *b.overflow = 1u; return; }
    const uint32_t need = C.owners;
    const uint32_t m = (uint32_t)g.m, m2 = m * m;
    // owners 1..6: -x, -y, -x-y, -z, -y-z, -x-z
    const uint32_t d[6] = {1u, m, m + 1u, m2, m2 + m, m2 + 1u};
    const IdTriple* vid = reinterpret_cast<const IdTriple*>(b.vid);
    IdTriple w[7];
    w[0] = vid[L];
#pragma unroll
    for (int q = 0; q < 6; ++q) w[q + 1] = vid[((need >> (q + 1)) & 1u) ? L - d[q] : L];
#pragma unroll
    for (int e = 0; e < 12; ++e) {
        const IdTriple& q = w[c_edge_owner_idx[e]];
        const int sl = c_edge_slot[e];
        s_w[e][t] = sl == 0 ? q.a : sl == 1 ? q.b : q.c;
    }
    int32_t* out = b.faces + 3 * (size_t)fbase;
    for (int k = 0; k < ntri; ++k) {
        IdTriple f;
        f.a = Voff + s_w[C.tri[3 * k]][t];
        f.b = Voff + s_w[C.tri[3 * k + 1]][t];
        f.c = Voff + s_w[C.tri[3 * k + 2]][t];
        *reinterpret_cast<IdTriple*>(out + 3 * k) = f;
    }
}

__device__ __forceinline__ void mc_faces_body(const CaseInfo* __restrict__ cases, const GridDesc& g, const MCBuffers& b) {
    __shared__ CaseInfo s_case[256];
    __shared__ uint32_t s_w[12][256];   // per lane: the vertex id of each of its cell's 12 edges
    const int t = threadIdx.x;
    s_case[t] = cases[t];
    __syncthreads();
    const uint32_t n_rec = b.counters[4];
    const uint32_t lim = n_rec < (uint64_t)b.cap_rec ? n_rec : (uint32_t)b.cap_rec;
    uint32_t Voff = b.offsets ? b.offsets[0] : 0u;
    if (b.gathered)
        for (int r = 0; r < b.rank; ++r) Voff += b.gathered[4 * r] - b.gathered[4 * r + 3];
    const uint32_t nb = gridDim.x, lb = (blockIdx.x % 8u) * (nb / 8u) + blockIdx.x / 8u;
    const uint32_t per = (lim + nb - 1u) / nb, i_end = min(lim, (lb + 1u) * per);
    for (uint32_t i = lb * per + t; i < i_end; i += 256) face_record(s_case, s_w, g, b, Voff, i);
}

__global__ __launch_bounds__(256) void k_mc_faces(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    mc_faces_body(cases, g, b);
}

// ---- merged launches of an object stream (ObjArgs, kernels.hpp): block row y = object y ----------
__global__ __launch_bounds__(512) void k_mc_count_b(const ObjArgs* __restrict__ objs, GridDesc g) {
    mc_count_body(g, objs[blockIdx.y].mc);
}
template <int B>
__global__ __launch_bounds__(B) void k_unit_scan_b(const ObjArgs* __restrict__ objs, GridDesc g) {
    unit_scan_body<B>(g, objs[blockIdx.y].mc);
}
// vertex pass: one flat index over every object's unit parts (batch_device.hpp), a wave per part
__global__ __launch_bounds__(64 * kVertsWaves) void k_mc_cells_b(const CaseInfo* __restrict__ cases,
                                                                const ObjArgs* __restrict__ objs, int n, GridDesc g) {
    __shared__ uint32_t s_cw[256];
    __shared__ uint64_t s_bits[kVertsWaves][9][64];
    __shared__ uint32_t s_excl[kVertsWaves][64];
    __shared__ uint32_t s_pre[kMaxBatchObjects + 4];
    const int t = threadIdx.x, wid = t >> 6;
    for (int k = t; k < 256; k += blockDim.x) s_cw[k] = case_word(cases[k]);
    const uint32_t total = batch_prefix(objs, n, 0, 1u, 0xffffffffu, s_pre);   // counters[0]: unit parts
    for (uint32_t e = blockIdx.x * kVertsWaves + wid; e < total; e += gridDim.x * kVertsWaves) {
        const int k = __builtin_amdgcn_readfirstlane(batch_object_of(s_pre, n, e));
        mc_cells_part(s_cw, g, objs[k].mc, e - s_pre[k], s_bits[wid], s_excl[wid]);
    }
}
// every object's counter block into one array (config 5's setup reads all of them with one copy)
__global__ __launch_bounds__(256) void k_gather_counters(const ObjArgs* __restrict__ objs, int n, uint32_t* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n * kCounterWords) out[i] = objs[i / kCounterWords].counters[i % kCounterWords];
}
__global__ __launch_bounds__(256) void k_zero_pieces(const ZeroPiece* __restrict__ pieces) {
    const ZeroPiece z = pieces[blockIdx.x];
    uint8_t* p = reinterpret_cast<uint8_t*>(z.p);
    const uint32_t n16 = z.n / 16;
    for (uint32_t i = threadIdx.x; i < n16; i += 256) reinterpret_cast<uint4*>(p)[i] = uint4{0, 0, 0, 0};
    for (uint32_t i = n16 * 16 + threadIdx.x; i < z.n; i += 256) p[i] = 0;
}
// face pass: one flat index over every object's records, a lane per record
__global__ __launch_bounds__(256) void k_mc_faces_b(const CaseInfo* __restrict__ cases, const ObjArgs* __restrict__ objs,
                                                    int n, GridDesc g) {
    __shared__ CaseInfo s_case[256];
    __shared__ uint32_t s_w[12][256];
    __shared__ uint32_t s_pre[kMaxBatchObjects + 4];
    const int t = threadIdx.x;
    s_case[t] = cases[t];
    const uint32_t total = batch_prefix(objs, n, 4, 1u, 0xffffffffu, s_pre);   // counters[4]: active cells
    for (uint32_t gi = blockIdx.x * 256 + t; gi < total; gi += gridDim.x * 256) {
        const int k = batch_object_of(s_pre, n, gi);
        const MCBuffers& b = objs[k].mc;
        const uint32_t i = gi - s_pre[k];
        if (i >= (uint64_t)b.cap_rec) { *b.overflow = 1u; continue; }
        face_record(s_case, s_w, g, b, b.offsets ? b.offsets[0] : 0u, i);
    }
}

}  // namespace

void launch_mc_count(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    const int64_t ng = n_groups(g);
    if (ng == 0) return;
    // lanes over the items of a group (kGroupUnits kUnitRows rows x nch chunks), whole waves, at
    // most 512: twice the resident groups of 1024-lane blocks
    const int items = kGroupUnits * kUnitRows * ((g.m + 63) / 64);
    const unsigned threads = (unsigned)std::min(512, (items + 63) / 64 * 64);
    (void)d_cases;
    k_mc_count<<<(unsigned)ng, threads, 0, s>>>(g, b);
}

void launch_mc_scan(const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    const int64_t ng = n_groups(g);
    if (ng > 0) k_unit_scan<<<(unsigned)ng, kScanBlock, 0, s>>>(g, b);
}

void launch_mc_faces(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    k_mc_faces<<<kFacesBlocks, 256, 0, s>>>(d_cases, g, b);
}

void launch_mc_verts(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    const int64_t nu = n_units(g);
    if (nu > 0) {
        k_mc_cells<<<(unsigned)std::min<int64_t>((nu + kVertsWaves - 1) / kVertsWaves, kVertsMaxBlocks),
                     64 * kVertsWaves, 0, s>>>(d_cases, g, b);
    }
}

}  // namespace impli

namespace impli {

// grids of the flat merged vertex / face kernels
constexpr unsigned kBatchCellBlocks = 4096, kBatchFaceBlocks = 2048;
constexpr int kBatchCountLanes = 128;

void launch_gather_counters(const ObjArgs* d_objs, int n, uint32_t* d_out, hipStream_t s) {
    if (n > 0) k_gather_counters<<<(unsigned)((n * kCounterWords + 255) / 256), 256, 0, s>>>(d_objs, n, d_out);
}

void launch_zero_pieces(const ZeroPiece* d_pieces, int n, hipStream_t s) {
    if (n > 0) k_zero_pieces<<<(unsigned)n, 256, 0, s>>>(d_pieces);
}

void launch_batch_mc(const ObjArgs* d_objs, int n, const CaseInfo* d_cases, const GridDesc& g, hipStream_t s) {
    const int64_t ng = n_groups(g), nu = n_units(g);
    if (ng == 0 || n <= 0) return;
    // An object's grid is small (128^3: 2 chunks per row, 63 groups): most of a group's (unit, chunk)
    // pairs are unmarked, so its count block loops over few items, and block count x waves is what
    // costs -- n objects' groups as blocks of kBatchCountLanes lanes (the single-grid path's 512-lane
    // blocks: 4x the waves of a 512^3 grid's count for the same samples).  The scan of <= 64 groups
    // reads them with one wave.
    const int items = kGroupUnits * kUnitRows * ((g.m + 63) / 64);
    const unsigned threads = (unsigned)std::min(kBatchCountLanes, (items + 63) / 64 * 64);
    k_mc_count_b<<<dim3((unsigned)ng, (unsigned)n), threads, 0, s>>>(d_objs, g);
    if (ng <= 64) k_unit_scan_b<64><<<dim3((unsigned)ng, (unsigned)n), 64, 0, s>>>(d_objs, g);
    else k_unit_scan_b<kScanBlock><<<dim3((unsigned)ng, (unsigned)n), kScanBlock, 0, s>>>(d_objs, g);
    (void)nu;
    k_mc_cells_b<<<kBatchCellBlocks, 64 * kVertsWaves, 0, s>>>(d_cases, d_objs, n, g);
    k_mc_faces_b<<<kBatchFaceBlocks, 256, 0, s>>>(d_cases, d_objs, n, g);
}

}  // namespace impli
