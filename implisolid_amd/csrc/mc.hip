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
//   K2b k_scan_*  : exclusive scan of the unit sums (partial sums, top level, apply).
//   K3 k_mc_verts : per unit, the non-trivial cells in cell order: owned vertex positions (field
//                   values read only at crossing edges), the dense vid3[cell][slot] table, records.
//   K4 k_mc_faces : per active cell, gathers the vertex ids of its triangle corners from vid3 of
//                   the owner cells.
#include <cstdlib>

#include "eval_bricks.hpp"
#include "ifunc_device.hpp"
#include "kernels.hpp"
#include "mc_device.hpp"

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
        out[ci] = c;
    }
}

namespace {

// K2: one wave per unit (kUnitRows rows).  Items (row, 64-cell chunk) are spread over the lanes;
// only non-trivial cells (~1 %) look at the case table.  -> unit_cnt[u] = {own, tri, act, halo own}
__global__ __launch_bounds__(256) void k_mc_count(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    const int lane = threadIdx.x & 63;
    const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u >= n_units(g)) return;
    const int nch = (g.m + 63) / 64;
    const int64_t rows = n_rows(g);
    unsigned own = 0, tri = 0, act = 0, hal = 0;
    for (int i = lane; i < kUnitRows * nch; i += 64) {
        const int64_t row = u * kUnitRows + i / nch;
        if (row >= rows) break;
        ChunkBits k;
        load_chunk(g, b.signs, row, i % nch, k);
        uint64_t nt = k.nt;
        const bool emit = k.z >= g.cz_emit;
        while (nt) {
            const int j = __ffsll((unsigned long long)nt) - 1;
            nt &= nt - 1;
            unsigned ntri;
            const unsigned no = case_counts(cases, chunk_ci(k, j), ntri);
            own += no;
            if (emit) { tri += ntri; act += ntri ? 1u : 0u; }
            else hal += no;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        own += __shfl_down(own, o, 64);
        tri += __shfl_down(tri, o, 64);
        act += __shfl_down(act, o, 64);
        hal += __shfl_down(hal, o, 64);
    }
    if (lane == 0) b.unit_cnt[u] = make_uint4(own, tri, act, hal);
}

// ---- unit scan: partial sums per scan block, top-level scan, apply ----
struct Cnt5 { uint32_t c[5]; };
__device__ __forceinline__ Cnt5 unit_c5(uint4 v) {
    Cnt5 r;
    r.c[0] = v.x; r.c[1] = v.y; r.c[2] = v.z; r.c[3] = v.w; r.c[4] = (v.x | v.y) ? 1u : 0u;
    return r;
}

// inclusive block scan (1024 lanes) of 5 components; returns exclusive, fills total
__device__ __forceinline__ Cnt5 block_scan5(Cnt5 v, Cnt5& total, uint32_t (*s_w)[16]) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    Cnt5 incl;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        incl.c[c] = wave_incl_scan<uint32_t>(v.c[c], lane);
        if (lane == 63) s_w[c][wid] = incl.c[c];
    }
    __syncthreads();
    Cnt5 ex;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        uint32_t pre = 0, tt = 0;
        for (int w = 0; w < 16; ++w) {
            const uint32_t x = s_w[c][w];
            if (w < wid) pre += x;
            tt += x;
        }
        ex.c[c] = pre + incl.c[c] - v.c[c];
        total.c[c] = tt;
    }
    __syncthreads();
    return ex;
}

__global__ __launch_bounds__(1024) void k_scan_partial(const uint4* __restrict__ cnt, int64_t nu, uint32_t* __restrict__ blk) {
    __shared__ uint32_t s_w[5][16];
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanUPT;
    Cnt5 sum = {{0, 0, 0, 0, 0}};
    for (int i = 0; i < kScanUPT; ++i)
        if (base + i < nu) {
            const Cnt5 c = unit_c5(cnt[base + i]);
            for (int k = 0; k < 5; ++k) sum.c[k] += c.c[k];
        }
    Cnt5 tot;
    (void)block_scan5(sum, tot, s_w);
    if (threadIdx.x == 0)
        for (int k = 0; k < 5; ++k) blk[8 * blockIdx.x + k] = tot.c[k];
}

__global__ __launch_bounds__(64) void k_scan_top(uint32_t* __restrict__ blk, int nb, uint32_t* __restrict__ counters) {
    if (threadIdx.x != 0) return;
    uint32_t run[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < nb; ++b)
        for (int k = 0; k < 5; ++k) {
            const uint32_t v = blk[8 * b + k];
            blk[8 * b + k] = run[k];
            run[k] += v;
        }
    counters[0] = run[4];
    counters[1] = run[3];
    counters[2] = run[0];
    counters[3] = run[1];
    counters[4] = run[2];
    counters[5] = run[3];
}

__global__ __launch_bounds__(1024) void k_scan_apply(uint4* __restrict__ cnt, int64_t nu, const uint32_t* __restrict__ blk) {
    __shared__ uint32_t s_w[5][16];
    const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanUPT;
    uint4 v[kScanUPT];
    Cnt5 sum = {{0, 0, 0, 0, 0}};
    for (int i = 0; i < kScanUPT; ++i) {
        v[i] = (base + i < nu) ? cnt[base + i] : make_uint4(0, 0, 0, 0);
        const Cnt5 c = unit_c5(v[i]);
        for (int k = 0; k < 5; ++k) sum.c[k] += c.c[k];
    }
    Cnt5 tot;
    Cnt5 run = block_scan5(sum, tot, s_w);
    for (int k = 0; k < 5; ++k) run.c[k] += blk[8 * blockIdx.x + k];
    for (int i = 0; i < kScanUPT; ++i) {
        if (base + i >= nu) break;
        const Cnt5 c = unit_c5(v[i]);
        cnt[base + i] = make_uint4(run.c[0], run.c[1], run.c[2], run.c[3]);
        for (int k = 0; k < 5; ++k) run.c[k] += c.c[k];
    }
}

__global__ __launch_bounds__(256) void k_mc_verts(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    mc_verts_body(cases, g, b);
}

// owner offset (dx, dy, dz subtracted) and owned slot of each Bourke edge
__constant__ int8_t c_edge_owner[12][4] = {
    {0, 1, 1, 1}, {0, 0, 1, 0}, {0, 0, 1, 1}, {1, 0, 1, 0}, {0, 1, 0, 1}, {0, 0, 0, 0},
    {0, 0, 0, 1}, {1, 0, 0, 0}, {1, 1, 0, 2}, {0, 1, 0, 2}, {0, 0, 0, 2}, {1, 0, 0, 2},
};

__global__ __launch_bounds__(256) void k_mc_faces(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    __shared__ CaseInfo s_case[256];
    __shared__ int32_t s_off[12];
    __shared__ int32_t s_slot[12];
    const int t = threadIdx.x;
    s_case[t] = cases[t];
    if (t < 12) {
        const int64_t m = g.m;
        s_off[t] = (int32_t)(c_edge_owner[t][0] + c_edge_owner[t][1] * m + c_edge_owner[t][2] * m * m);
        s_slot[t] = c_edge_owner[t][3];
    }
    __syncthreads();
    const uint32_t n_rec = b.counters[4];
    const uint32_t lim = n_rec < (uint64_t)b.cap_rec ? n_rec : (uint32_t)b.cap_rec;
    const uint32_t Voff = b.offsets ? b.offsets[0] : 0u;
    for (uint32_t i = blockIdx.x * 256 + t; i < lim; i += gridDim.x * 256) {
        const uint4 r = b.records[i];
        const uint32_t L = r.x, ci = r.y, fbase = r.z;
        const CaseInfo& C = s_case[ci];
        if (fbase + C.ntri > (uint64_t)b.cap_f) { *b.overflow = 1u; continue; }
        int32_t* out = b.faces + 3 * (size_t)fbase;
        for (int k = 0; k < 3 * C.ntri; ++k) {
            const int e = C.tri[k];
            const uint32_t owner = L - (uint32_t)s_off[e];
            out[k] = (int32_t)(Voff + b.vid3[(size_t)owner * 3 + s_slot[e]]);
        }
    }
}

}  // namespace

void launch_mc_count(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    const int64_t nu = n_units(g);
    if (nu == 0) return;
    k_mc_count<<<(unsigned)((nu + 3) / 4), 256, 0, s>>>(d_cases, g, b);
}

void launch_mc_scan(const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    const int64_t nu = n_units(g), nb = n_scan_blocks(g);
    if (nb > 0) k_scan_partial<<<(unsigned)nb, 1024, 0, s>>>(b.unit_cnt, nu, b.scan_blk);
    k_scan_top<<<1, 64, 0, s>>>(b.scan_blk, (int)nb, b.counters);
    if (nb > 0) k_scan_apply<<<(unsigned)nb, 1024, 0, s>>>(b.unit_cnt, nu, b.scan_blk);
}

void launch_mc_faces(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    k_mc_faces<<<2048, 256, 0, s>>>(d_cases, g, b);
}

void launch_mc_verts(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    const int64_t nu = n_units(g);
    if (nu > 0) k_mc_verts<<<(unsigned)((nu + 3) / 4), 256, 0, s>>>(d_cases, g, b);
}

}  // namespace impli
