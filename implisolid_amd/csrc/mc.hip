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

#include "ifunc_device.hpp"
#include "kernels.hpp"

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

// stored sample (sx, sy, sz) -- sample indices in [1, res-2], the sealed ring included
__device__ __forceinline__ int sample_index(const GridDesc& g, int sx, int sy, int sz) {
    return (sx - 1) + (sy - 1) * g.n + (sz - g.fz0) * g.n * g.n;   // the field is < 2^31 elements
}
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// owned-edge and triangle counts of a cube index
__device__ __forceinline__ unsigned case_counts(const CaseInfo* __restrict__ cases, unsigned ci, unsigned& ntri) {
    const uint16_t v = *reinterpret_cast<const uint16_t*>(&cases[ci]);   // {ntri, nown}
    ntri = v & 255u;
    return v >> 8;
}

// 64 consecutive cells of one cell row, as sign bits.  For cell j (x = 64 c + 1 + j) the corners
// are stored samples x-1 and x of the rows (y, z), (y+1, z), (y, z+1), (y+1, z+1): bit j of s.. and
// t.. (t = s shifted by one sample).  nt marks the non-trivial cells (corner signs not all equal).
struct ChunkBits {
    uint64_t s00, t00, s10, t10, s01, t01, s11, t11, nt;
    int y, z, x0;   // cell row and first cell x of the chunk
};

__device__ __forceinline__ void load_chunk(const GridDesc& g, const uint64_t* __restrict__ signs, int64_t row, int c,
                                           ChunkBits& k) {
    const int rw = sign_row_words(g);
    k.y = (int)(row % g.m) + 1;
    k.z = (int)(row / g.m) + g.cz0;
    k.x0 = 64 * c + 1;
    const int64_t r00 = ((int64_t)(k.z - g.fz0) * g.n + (k.y - 1)) * rw;   // (layer, stored y) -> word index
    const int64_t rows[4] = {r00, r00 + rw, r00 + (int64_t)g.n * rw, r00 + (int64_t)g.n * rw + rw};
    uint64_t s[4], t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t w = signs[rows[q] + c];
        const uint64_t nx = (c + 1 < rw) ? signs[rows[q] + c + 1] : 0ull;
        s[q] = w;
        t[q] = (w >> 1) | (nx << 63);
    }
    k.s00 = s[0]; k.t00 = t[0]; k.s10 = s[1]; k.t10 = t[1]; k.s01 = s[2]; k.t01 = t[2]; k.s11 = s[3]; k.t11 = t[3];
    const uint64_t all = s[0] & t[0] & s[1] & t[1] & s[2] & t[2] & s[3] & t[3];
    const uint64_t any = s[0] | t[0] | s[1] | t[1] | s[2] | t[2] | s[3] | t[3];
    const int left = g.m - 64 * c;   // cells of this chunk inside the row
    const uint64_t valid = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
    k.nt = any & ~all & valid;
}

// cube index of cell j of a chunk, corner bits as polygonize_single_cube (:553-560)
__device__ __forceinline__ unsigned chunk_ci(const ChunkBits& k, int j) {
    return (unsigned)((k.s00 >> j) & 1u) | ((unsigned)((k.t00 >> j) & 1u) << 1) | ((unsigned)((k.s10 >> j) & 1u) << 3) |
           ((unsigned)((k.t10 >> j) & 1u) << 2) | ((unsigned)((k.s01 >> j) & 1u) << 4) |
           ((unsigned)((k.t01 >> j) & 1u) << 5) | ((unsigned)((k.s11 >> j) & 1u) << 7) |
           ((unsigned)((k.t11 >> j) & 1u) << 6);
}

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

// K3: one wave per unit.  Lanes find the non-trivial cells of their (row, chunk) items; a wave scan
// orders them (cell order) into an LDS list, processed 64 at a time: a second wave scan of (owned
// edges, triangles, active) gives every cell its vertex / face / record base, all written in
// parallel.  Corner values are read from the field only for owned crossing edges.
__device__ __forceinline__ unsigned long long pack4(unsigned a, unsigned b, unsigned c, unsigned d) {
    return (unsigned long long)a | ((unsigned long long)b << 16) | ((unsigned long long)c << 32) |
           ((unsigned long long)d << 48);
}
__device__ __forceinline__ unsigned fld(unsigned long long p, int i) { return (unsigned)(p >> (16 * i)) & 0xffffu; }

constexpr int kListCap = 1024;   // LDS list entries per wave (a window; larger units loop)

__global__ __launch_bounds__(256) void k_mc_verts(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    __shared__ CaseInfo s_case[256];
    __shared__ uint32_t s_list[4][kListCap];   // per wave: ci | j << 8 | item << 14
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    s_case[t] = cases[t];
    __syncthreads();
    const int64_t u = (int64_t)blockIdx.x * 4 + wid;
    if (u >= n_units(g)) return;
    const uint32_t H = b.counters[1];
    const int nch = (g.m + 63) / 64;
    const int64_t rows = n_rows(g);
    const uint4 base = b.unit_cnt[u];   // exclusive {vbase, fbase, abase, hbase}
    uint32_t vrun0 = base.x, frun0 = base.y, arun0 = base.z;
    uint32_t* list = s_list[wid];
    const int items = kUnitRows * nch;
    for (int i0 = 0; i0 < items; i0 += 64) {
        const int i = i0 + lane;
        ChunkBits k;
        k.nt = 0;
        int64_t row = -1;
        if (i < items) {
            row = u * kUnitRows + i / nch;
            if (row < rows) load_chunk(g, b.signs, row, i % nch, k);
        }
        const uint32_t cnt = (uint32_t)__popcll((unsigned long long)k.nt);
        const uint32_t incl = wave_incl_scan<uint32_t>(cnt, lane);
        const uint32_t total = __shfl(incl, 63, 64);
        for (uint32_t w0 = 0; w0 < total; w0 += kListCap) {
            // this window's entries, in cell order
            uint32_t pos = incl - cnt;
            uint64_t nt = k.nt;
            while (nt) {
                const int j = __ffsll((unsigned long long)nt) - 1;
                nt &= nt - 1;
                if (pos >= w0 && pos < w0 + kListCap)
                    list[pos - w0] = chunk_ci(k, j) | ((uint32_t)j << 8) | ((uint32_t)i << 14);
                ++pos;
            }
            __builtin_amdgcn_wave_barrier();
            const uint32_t n_list = (total - w0 < (uint32_t)kListCap) ? total - w0 : (uint32_t)kListCap;
            for (uint32_t e0 = 0; e0 < n_list; e0 += 64) {
                const uint32_t e = e0 + (uint32_t)lane;
                const bool has = e < n_list;
                const uint32_t ent = has ? list[e] : 0u;
                const unsigned ci = ent & 255u;
                const int j = (int)((ent >> 8) & 63u), it = (int)(ent >> 14);
                const int64_t erow = u * kUnitRows + it / nch;
                const int x = 64 * (it % nch) + 1 + j;
                const int y = (int)(erow % g.m) + 1, z = (int)(erow / g.m) + g.cz0;
                const uint32_t L = (uint32_t)(erow * g.m + (x - 1));
                const CaseInfo& C = s_case[ci];
                const bool emit = has && z >= g.cz_emit;
                const unsigned own = has ? C.nown : 0u, tri = emit ? C.ntri : 0u, act = (emit && C.ntri) ? 1u : 0u;
                const unsigned long long p = pack4(own, tri, act, 0u);
                const unsigned long long inc = wave_incl_scan<unsigned long long>(p, lane);
                const unsigned long long pre = inc - p, tot = __shfl(inc, 63, 64);
                if (has && own) {
                    const uint32_t vrun = vrun0 + fld(pre, 0);
                    const float fx = ((float)x + g.i0[0]) * g.w[0];
                    const float fy = ((float)y + g.i0[1]) * g.w[1];
                    const float fz = ((float)z + g.i0[2]) * g.w[2];
                    const float fx2 = fx + g.w[0], fy2 = fy + g.w[1], fz2 = fz + g.w[2];
                    const int n = g.n, nn = g.n * g.n;
                    const float* q = b.field + sample_index(g, x, y, z);
                    const float f7 = q[nn + n + 1];
#pragma unroll
                    for (int slot = 0; slot < 3; ++slot) {
                        const int r = C.rank[slot];
                        if (r < 0) continue;
                        const uint32_t vid = vrun + (uint32_t)r;
                        b.vid3[(size_t)L * 3 + slot] = vid - H;
                        if (!emit) continue;
                        const uint32_t out = vid - H;
                        if (out >= (uint64_t)b.cap_v) { *b.overflow = 1u; continue; }
                        float px, py, pz;
                        if (slot == 0) {        // edge 5: VIntY at qxz, (fx2, fy + mu*dy, fz2), field5 -> field7
                            const float f5 = q[nn + 1];
                            const float mu = (0.f - f5) / (f7 - f5);
                            px = fx2; py = fy + mu * g.w[1]; pz = fz2;
                        } else if (slot == 1) { // edge 6: VIntX at qyz, (fx + mu*dx, fy2, fz2), field6 -> field7
                            const float f6 = q[nn + n];
                            const float mu = (0.f - f6) / (f7 - f6);
                            px = fx + mu * g.w[0]; py = fy2; pz = fz2;
                        } else {                // edge 10: VIntZ at qxy, (fx2, fy2, fz + mu*dz), field3 -> field7
                            const float f3 = q[n + 1];
                            const float mu = (0.f - f3) / (f7 - f3);
                            px = fx2; py = fy2; pz = fz + mu * g.w[2];
                        }
                        b.verts[3 * (size_t)out] = px;
                        b.verts[3 * (size_t)out + 1] = py;
                        b.verts[3 * (size_t)out + 2] = pz;
                    }
                }
                if (act) {
                    const uint32_t arun = arun0 + fld(pre, 2);
                    if (arun < (uint64_t)b.cap_rec) b.records[arun] = make_uint4(L, ci, frun0 + fld(pre, 1), 0u);
                    else *b.overflow = 1u;
                }
                vrun0 += fld(tot, 0);
                frun0 += fld(tot, 1);
                arun0 += fld(tot, 2);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
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

void launch_mc_emit(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s, hipEvent_t mid) {
    const int64_t nu = n_units(g);
    if (nu > 0) k_mc_verts<<<(unsigned)((nu + 3) / 4), 256, 0, s>>>(d_cases, g, b);
    if (mid) (void)hipEventRecord(mid, s);
    k_mc_faces<<<2048, 256, 0, s>>>(d_cases, g, b);
}

}  // namespace impli
