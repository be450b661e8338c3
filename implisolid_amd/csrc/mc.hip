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
//   K2 k_mc_count : per 1024-cell unit (contiguous in linear order) the sums of owned edges,
//                   triangles and active cells; units with work are appended to a list.
//   K2b k_mc_scan : exclusive scan of the unit sums (one workgroup).
//   K3 k_mc_verts : per active unit, in-unit block scan; writes owned vertex positions, the
//                   dense vid3[cell][slot] table and one record per active cell.
//   K4 k_mc_faces : per active cell, gathers the three vertex ids of every triangle corner from
//                   vid3 of the owner cell.
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
__device__ __forceinline__ float corner(const float* __restrict__ field, const GridDesc& g, int sx, int sy, int sz) {
    return field[sample_index(g, sx, sy, sz)];
}

struct CellVals {
    float f[8];   // f0=q f1=qx f2=qy f3=qxy f4=qz f5=qxz f6=qyz f7=qxyz
};

__device__ __forceinline__ unsigned load_cell(const float* __restrict__ field, const GridDesc& g, int cx, int cy, int cz,
                                              CellVals& v) {
    const int n = g.n, nn = g.n * g.n;
    const float* q = field + sample_index(g, cx, cy, cz);
    v.f[0] = q[0];
    v.f[1] = q[1];
    v.f[2] = q[n];
    v.f[3] = q[n + 1];
    v.f[4] = q[nn];
    v.f[5] = q[nn + 1];
    v.f[6] = q[nn + n];
    v.f[7] = q[nn + n + 1];
    unsigned ci = 0;   // polygonize_single_cube :553-560
    if (v.f[0] < 0.f) ci |= 1;
    if (v.f[1] < 0.f) ci |= 2;
    if (v.f[2] < 0.f) ci |= 8;
    if (v.f[3] < 0.f) ci |= 4;
    if (v.f[4] < 0.f) ci |= 16;
    if (v.f[5] < 0.f) ci |= 32;
    if (v.f[6] < 0.f) ci |= 128;
    if (v.f[7] < 0.f) ci |= 64;
    return ci;
}

__device__ __forceinline__ void cell_coords(const GridDesc& g, uint32_t L, int& cx, int& cy, int& cz) {
    const uint32_t m = (uint32_t)g.m, mm = m * m;
    const uint32_t zr = L / mm, rem = L - zr * mm;
    const uint32_t yr = rem / m;
    cx = 1 + (int)(rem - yr * m);
    cy = 1 + (int)yr;
    cz = g.cz0 + (int)zr;
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

// exclusive block scan over 256 lanes (4 waves); returns prefix, sets total
__device__ __forceinline__ unsigned long long block_excl_scan(unsigned long long v, unsigned long long& total,
                                                              unsigned long long* lds4) {
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const unsigned long long incl = wave_incl_scan<unsigned long long>(v, lane);
    if (lane == 63) lds4[wid] = incl;
    __syncthreads();
    unsigned long long pre = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const unsigned long long s = lds4[w];
        if (w < wid) pre += s;
        total += s;
    }
    __syncthreads();
    return pre + incl - v;
}

constexpr unsigned long long kF = 20;   // packed counter field width
__device__ __forceinline__ unsigned long long pack3(unsigned own, unsigned tri, unsigned act) {
    return (unsigned long long)own | ((unsigned long long)tri << kF) | ((unsigned long long)act << (2 * kF));
}
__device__ __forceinline__ unsigned f_own(unsigned long long p) { return (unsigned)(p & ((1ull << kF) - 1)); }
__device__ __forceinline__ unsigned f_tri(unsigned long long p) { return (unsigned)((p >> kF) & ((1ull << kF) - 1)); }
__device__ __forceinline__ unsigned f_act(unsigned long long p) { return (unsigned)(p >> (2 * kF)); }

// cube index from the negative-corner masks of the four sample rows around a run of cells:
// bit k of r00/r10/r01/r11 = sample x0+k of rows (y,z), (y+1,z), (y,z+1), (y+1,z+1) is < 0
__device__ __forceinline__ unsigned ci_from_rows(unsigned r00, unsigned r10, unsigned r01, unsigned r11, int k) {
    const unsigned a = (r00 >> k) & 3u, b = (r10 >> k) & 3u, c = (r01 >> k) & 3u, d = (r11 >> k) & 3u;
    // corners q(1) qx(2) | qy(8) qxy(4) | qz(16) qxz(32) | qyz(128) qxyz(64)
    return (a & 1u) | ((a >> 1) << 1) | ((b & 1u) << 3) | ((b >> 1) << 2) | ((c & 1u) << 4) | ((c >> 1) << 5) |
           ((d & 1u) << 7) | ((d >> 1) << 6);
}

// K2: one 256-thread block per 1024-cell unit, 4 consecutive cells per thread.  Runs of 4 cells
// in one row share their corners (20 loads instead of 32); if every brick the run touches was
// sign-filled by the eval with one sign, the cube indices are known without touching the field.
// owned-edge and triangle counts of a cube index; trivial cells (ci 0 / 255, ~99 % of them) skip
// the table read
__device__ __forceinline__ unsigned case_counts(const CaseInfo* __restrict__ cases, unsigned ci, unsigned& ntri) {
    if (ci == 0u || ci == 255u) { ntri = 0; return 0; }
    const uint16_t v = *reinterpret_cast<const uint16_t*>(&cases[ci]);   // {ntri, nown}
    ntri = v & 255u;
    return v >> 8;
}

__global__ __launch_bounds__(256) void k_mc_count(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    __shared__ uint4 s_red[4];
    const int t = threadIdx.x;
    const uint32_t u = blockIdx.x;
    const uint32_t L0 = u * kUnitCells + 4u * (uint32_t)t;
    unsigned own = 0, tri = 0, act = 0, halo_own = 0;
    if (L0 < (uint64_t)g.n_cells) {
        int cx, cy, cz;
        cell_coords(g, L0, cx, cy, cz);
        uint32_t ci4 = 0;
        if (cx + 3 <= g.m && L0 + 3 < (uint64_t)g.n_cells) {
            // stored coordinates of the run's first corner; the run reads x0 .. x0+4
            const int x0 = cx - 1, y0 = cy - 1, z0 = cz - g.fz0;
            const int bx0 = x0 / kBX, bx1 = (x0 + 4) / kBX, by0 = y0 / kBY, by1 = (y0 + 1) / kBY;
            const int bz0 = z0 / kBZ, bz1 = (z0 + 1) / kBZ;
            const int sby = b.nbx, sbz = b.nbx * b.nby;
            const uint8_t* fb = b.fill;
            unsigned f_and = 3u, f_or = 0u;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const unsigned v = fb[((k & 1) ? bx1 : bx0) + ((k & 2) ? by1 : by0) * sby + ((k & 4) ? bz1 : bz0) * sbz];
                f_and &= v;
                f_or |= v;
            }
            const unsigned f0 = f_or;
            if (f0 != 0u && f_and == f_or) {   // all eight equal and non-zero
                // all touched bricks filled with one sign: every corner has that sign
                ci4 = (f0 == kBrickNeg) ? 0xffffffffu : 0u;
            } else {
                const int n = g.n, nn = n * n;
                const float* q = b.field + (x0 + y0 * n + z0 * nn);
                unsigned r00 = 0, r10 = 0, r01 = 0, r11 = 0;
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    r00 |= (q[k] < 0.f ? 1u : 0u) << k;
                    r10 |= (q[n + k] < 0.f ? 1u : 0u) << k;
                    r01 |= (q[nn + k] < 0.f ? 1u : 0u) << k;
                    r11 |= (q[nn + n + k] < 0.f ? 1u : 0u) << k;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) ci4 |= ci_from_rows(r00, r10, r01, r11, k) << (8 * k);
            }
            unsigned o = 0, tr = 0, ac = 0;
            if (ci4 != 0u && ci4 != 0xffffffffu) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    unsigned nt;
                    o += case_counts(cases, (ci4 >> (8 * k)) & 255u, nt);
                    tr += nt;
                    ac += nt ? 1u : 0u;
                }
            }
            own = o;
            if (cz >= g.cz_emit) { tri = tr; act = ac; }
            else halo_own = o;
        } else {
            // the run crosses a row end (or the slab end): cell by cell
            int x = cx, y = cy, z = cz;
            for (int k = 0; k < 4; ++k) {
                if (L0 + k >= (uint64_t)g.n_cells) break;
                CellVals v;
                const unsigned ci = load_cell(b.field, g, x, y, z, v);
                ci4 |= ci << (8 * k);
                unsigned nt;
                const unsigned no = case_counts(cases, ci, nt);
                own += no;
                if (z >= g.cz_emit) { tri += nt; act += nt ? 1u : 0u; }
                else halo_own += no;
                if (++x > g.m) { x = 1; if (++y > g.m) { y = 1; ++z; } }
            }
        }
        *reinterpret_cast<uint32_t*>(b.ci + L0) = ci4;   // ci has >= 64 bytes of padding
    }
    const int lane = t & 63, wid = t >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        own += __shfl_down(own, o, 64);
        tri += __shfl_down(tri, o, 64);
        act += __shfl_down(act, o, 64);
        halo_own += __shfl_down(halo_own, o, 64);
    }
    if (lane == 0) s_red[wid] = make_uint4(own, tri, act, halo_own);
    __syncthreads();
    if (t == 0) {
        uint4 sm = s_red[0];
        for (int w = 1; w < 4; ++w) { sm.x += s_red[w].x; sm.y += s_red[w].y; sm.z += s_red[w].z; sm.w += s_red[w].w; }
        b.unit_cnt[u] = sm;
    }
}

// ---- unit scan: partial sums per scan block, top-level scan, apply + compaction of active units ----
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

__global__ __launch_bounds__(1024) void k_scan_apply(uint4* __restrict__ cnt, int64_t nu, const uint32_t* __restrict__ blk,
                                                     uint32_t* __restrict__ active) {
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
        if (c.c[4]) active[run.c[4]] = (uint32_t)(base + i);
        for (int k = 0; k < 5; ++k) run.c[k] += c.c[k];
    }
}

// K3: one wave per active unit (persistent loop).  Phase 1: each lane loads 16 cube indices
// (one 16-byte load) and the wave compacts the unit's non-trivial cells (ci != 0, 255 -- about
// 1 % of all cells) into an LDS list, in cell order.  Phase 2: lanes take list entries 64 at a
// time; a wave scan of (owned edges, triangles, active) gives each cell its vertex / face /
// record base, and the cells' vertices and records are written in parallel.
__device__ __forceinline__ unsigned long long pack4(unsigned a, unsigned b, unsigned c, unsigned d) {
    return (unsigned long long)a | ((unsigned long long)b << 16) | ((unsigned long long)c << 32) |
           ((unsigned long long)d << 48);
}
__device__ __forceinline__ unsigned fld(unsigned long long p, int i) { return (unsigned)(p >> (16 * i)) & 0xffffu; }

__global__ __launch_bounds__(256) void k_mc_verts(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    __shared__ CaseInfo s_case[256];
    __shared__ uint32_t s_list[4][kUnitCells];   // per wave: (cell offset in unit) | ci << 16
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    s_case[t] = cases[t];
    __syncthreads();
    const uint32_t n_active = b.counters[0];
    const uint32_t H = b.counters[1];
    const uint64_t halo_cells = (uint64_t)g.m * g.m * (uint64_t)(g.cz_emit - g.cz0);
    uint32_t* list = s_list[wid];
    constexpr int CPL = kUnitCells / 64;   // 16 cells per lane
    for (uint32_t a = blockIdx.x * 4 + wid; a < n_active; a += gridDim.x * 4) {
        const uint32_t u = b.active_units[a];
        const uint4 base = b.unit_cnt[u];   // exclusive {vbase, fbase, abase, hbase}
        const uint32_t U0 = u * kUnitCells;
        const uint32_t L0 = U0 + lane * CPL;
        uint32_t w[4] = {0, 0, 0, 0};
        if (L0 + CPL <= (uint64_t)g.n_cells) {
            const uint4 q = *reinterpret_cast<const uint4*>(b.ci + L0);
            w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w;
        } else {
            for (int k = 0; k < CPL; ++k)
                if (L0 + k < (uint64_t)g.n_cells) w[k >> 2] |= (uint32_t)b.ci[L0 + k] << (8 * (k & 3));
        }
        // non-trivial cells of this lane
        uint32_t mask = 0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 255u;
            mask |= (c != 0u && c != 255u) ? (1u << k) : 0u;
        }
        const uint32_t cnt = (uint32_t)__popc(mask);
        const uint32_t incl = wave_incl_scan<uint32_t>(cnt, lane);
        const uint32_t n_list = __shfl(incl, 63, 64);
        uint32_t pos = incl - cnt;
        while (mask) {
            const int k = __ffs(mask) - 1;
            mask &= mask - 1;
            list[pos++] = (uint32_t)(lane * CPL + k) | (((w[k >> 2] >> (8 * (k & 3))) & 255u) << 16);
        }
        __builtin_amdgcn_wave_barrier();
        uint32_t vrun0 = base.x, frun0 = base.y, arun0 = base.z;
        for (uint32_t e0 = 0; e0 < n_list; e0 += 64) {
            const uint32_t e = e0 + (uint32_t)lane;
            const bool has = e < n_list;
            const uint32_t ent = has ? list[e] : 0u;
            const uint32_t L = U0 + (ent & 0xffffu);
            const unsigned ci = ent >> 16;
            const CaseInfo& C = s_case[ci];
            const bool emit = has && (uint64_t)L >= halo_cells;
            const unsigned own = has ? C.nown : 0u, tri = emit ? C.ntri : 0u, act = (emit && C.ntri) ? 1u : 0u;
            const unsigned long long p = pack4(own, tri, act, 0u);
            const unsigned long long inc = wave_incl_scan<unsigned long long>(p, lane);
            const unsigned long long pre = inc - p, tot = __shfl(inc, 63, 64);
            if (has) {
                int x, y, z;
                cell_coords(g, L, x, y, z);
                uint32_t vrun = vrun0 + fld(pre, 0);
                if (own) {
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
            }
            vrun0 += fld(tot, 0);
            frun0 += fld(tot, 1);
            arun0 += fld(tot, 2);
        }
        __builtin_amdgcn_wave_barrier();
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
    k_mc_count<<<(unsigned)nu, 256, 0, s>>>(d_cases, g, b);
}

void launch_mc_scan(const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    const int64_t nu = n_units(g), nb = n_scan_blocks(g);
    if (nb > 0) k_scan_partial<<<(unsigned)nb, 1024, 0, s>>>(b.unit_cnt, nu, b.scan_blk);
    k_scan_top<<<1, 64, 0, s>>>(b.scan_blk, (int)nb, b.counters);
    if (nb > 0) k_scan_apply<<<(unsigned)nb, 1024, 0, s>>>(b.unit_cnt, nu, b.scan_blk, b.active_units);
}

void launch_mc_faces(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    k_mc_faces<<<2048, 256, 0, s>>>(d_cases, g, b);
}

void launch_mc_emit(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s, hipEvent_t mid) {
    const int64_t nu = n_units(g);
    k_mc_verts<<<(unsigned)(nu < 4096 ? (nu > 0 ? nu : 1) : 4096), 256, 0, s>>>(d_cases, g, b);
    if (mid) (void)hipEventRecord(mid, s);
    k_mc_faces<<<2048, 256, 0, s>>>(d_cases, g, b);
}

}  // namespace impli
