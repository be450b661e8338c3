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
    g.n = R + 1;
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
    const int lo = cz0 < 2 ? 2 : cz0, hi = (cz1 > g.res - 3 ? g.res - 3 : cz1) + 1;
    g.fz0 = lo;
    g.fz1 = hi > lo ? hi : lo;
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

__device__ __forceinline__ float corner(const float* __restrict__ field, const GridDesc& g, int sx, int sy, int sz) {
    const bool in = (unsigned)(sx - 2) <= (unsigned)g.R && (unsigned)(sy - 2) <= (unsigned)g.R &&
                    (unsigned)(sz - 2) <= (unsigned)g.R;
    return in ? field[(size_t)(sx - 2) + (size_t)(sy - 2) * g.n + (size_t)(sz - g.fz0) * g.n * g.n] : -10000000.0f;
}

struct CellVals {
    float f[8];   // f0=q f1=qx f2=qy f3=qxy f4=qz f5=qxz f6=qyz f7=qxyz
};

__device__ __forceinline__ unsigned load_cell(const float* __restrict__ field, const GridDesc& g, int cx, int cy, int cz,
                                              CellVals& v) {
    v.f[0] = corner(field, g, cx, cy, cz);
    v.f[1] = corner(field, g, cx + 1, cy, cz);
    v.f[2] = corner(field, g, cx, cy + 1, cz);
    v.f[3] = corner(field, g, cx + 1, cy + 1, cz);
    v.f[4] = corner(field, g, cx, cy, cz + 1);
    v.f[5] = corner(field, g, cx + 1, cy, cz + 1);
    v.f[6] = corner(field, g, cx, cy + 1, cz + 1);
    v.f[7] = corner(field, g, cx + 1, cy + 1, cz + 1);
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

__global__ __launch_bounds__(256) void k_mc_count(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    __shared__ uint8_t s_ntri[256], s_nown[256];
    __shared__ unsigned long long s_red[4];
    __shared__ unsigned s_halo[4];
    const int t = threadIdx.x;
    s_ntri[t] = cases[t].ntri;
    s_nown[t] = cases[t].nown;
    __syncthreads();
    const uint32_t u = blockIdx.x;
    unsigned own = 0, tri = 0, act = 0, halo_own = 0;
#pragma unroll
    for (int k = 0; k < kUnitCells / 256; ++k) {
        const uint32_t L = u * kUnitCells + k * 256 + t;
        if (L < (uint64_t)g.n_cells) {
            int cx, cy, cz;
            cell_coords(g, L, cx, cy, cz);
            CellVals v;
            const unsigned ci = load_cell(b.field, g, cx, cy, cz, v);
            const unsigned no = s_nown[ci], nt = s_ntri[ci];
            own += no;
            if (cz >= g.cz_emit) { tri += nt; act += nt ? 1u : 0u; }
            else halo_own += no;
        }
    }
    // block reduce
    unsigned long long p = pack3(own, tri, act);
    const int lane = t & 63, wid = t >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) p += __shfl_down(p, o, 64);
    unsigned h = halo_own;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) h += __shfl_down(h, o, 64);
    if (lane == 0) { s_red[wid] = p; s_halo[wid] = h; }
    __syncthreads();
    if (t == 0) {
        const unsigned long long s = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        const unsigned hs = s_halo[0] + s_halo[1] + s_halo[2] + s_halo[3];
        b.unit_cnt[3 * u + 0] = f_own(s);
        b.unit_cnt[3 * u + 1] = f_tri(s);
        b.unit_cnt[3 * u + 2] = f_act(s);
        if (s) b.active_units[atomicAdd(&b.counters[0], 1u)] = u;
        if (hs) atomicAdd(&b.counters[1], hs);
    }
}

// exclusive scan of unit_cnt (3 components) in place, one workgroup of 1024 lanes
// (unit sums fit 20-bit packed fields, slab totals do not: three separate 32-bit scans here)
__global__ __launch_bounds__(1024) void k_mc_scan(uint32_t* __restrict__ cnt, int64_t nu, uint32_t* __restrict__ counters) {
    __shared__ uint32_t s_w[3][16];
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int64_t chunk = (nu + 1023) / 1024;
    const int64_t a = t * chunk, e = (a + chunk < nu) ? a + chunk : nu;
    uint32_t sum[3] = {0, 0, 0};
    for (int64_t i = a; i < e; ++i)
        for (int c = 0; c < 3; ++c) sum[c] += cnt[3 * i + c];
    uint32_t run[3], tot[3];
    for (int c = 0; c < 3; ++c) {
        const uint32_t incl = wave_incl_scan<uint32_t>(sum[c], lane);
        if (lane == 63) s_w[c][wid] = incl;
        run[c] = incl - sum[c];
    }
    __syncthreads();
    for (int c = 0; c < 3; ++c) {
        uint32_t pre = 0, tt = 0;
        for (int w = 0; w < 16; ++w) {
            if (w < wid) pre += s_w[c][w];
            tt += s_w[c][w];
        }
        run[c] += pre;
        tot[c] = tt;
    }
    for (int64_t i = a; i < e; ++i)
        for (int c = 0; c < 3; ++c) {
            const uint32_t v = cnt[3 * i + c];
            cnt[3 * i + c] = run[c];
            run[c] += v;
        }
    if (t == 0) {
        counters[2] = tot[0];
        counters[3] = tot[1];
        counters[4] = tot[2];
        counters[5] = counters[1];
    }
}

__global__ __launch_bounds__(256) void k_mc_verts(const CaseInfo* __restrict__ cases, GridDesc g, MCBuffers b) {
    __shared__ CaseInfo s_case[256];
    __shared__ unsigned long long s_scan[4];
    const int t = threadIdx.x;
    s_case[t] = cases[t];
    __syncthreads();
    const uint32_t n_active = b.counters[0];
    const uint32_t H = b.counters[1];
    const uint32_t Voff = b.offsets ? b.offsets[0] : 0u;
    for (uint32_t a = blockIdx.x; a < n_active; a += gridDim.x) {
        const uint32_t u = b.active_units[a];
        const uint32_t vb = b.unit_cnt[3 * u], fb = b.unit_cnt[3 * u + 1], ab = b.unit_cnt[3 * u + 2];
        unsigned long long run = 0;
        for (int k = 0; k < kUnitCells / 256; ++k) {
            const uint32_t L = u * kUnitCells + k * 256 + t;
            const bool valid = L < (uint64_t)g.n_cells;
            int cx = 0, cy = 0, cz = 0;
            unsigned ci = 0;
            CellVals v;
            if (valid) {
                cell_coords(g, L, cx, cy, cz);
                ci = load_cell(b.field, g, cx, cy, cz, v);
            }
            const CaseInfo& C = s_case[ci];
            const bool emit = valid && cz >= g.cz_emit;
            const unsigned own = valid ? C.nown : 0u;
            const unsigned tri = emit ? C.ntri : 0u;
            const unsigned act = (emit && C.ntri) ? 1u : 0u;
            unsigned long long tot;
            const unsigned long long pre = run + block_excl_scan(pack3(own, tri, act), tot, s_scan);
            run += tot;
            if (own) {
                const uint32_t vloc = vb + f_own(pre);   // slab-local id, halo vertices first
                // render_geometry :1044-1053 and the owner's VIntX/Y/Z (:400-495)
                const float fx = ((float)cx + g.i0[0]) * g.w[0];
                const float fy = ((float)cy + g.i0[1]) * g.w[1];
                const float fz = ((float)cz + g.i0[2]) * g.w[2];
                const float fx2 = fx + g.w[0], fy2 = fy + g.w[1], fz2 = fz + g.w[2];
#pragma unroll
                for (int slot = 0; slot < 3; ++slot) {
                    const int r = C.rank[slot];
                    if (r < 0) continue;
                    const uint32_t vid = vloc + (uint32_t)r;
                    b.vid3[(size_t)L * 3 + slot] = Voff + vid - H;
                    if (!emit) continue;
                    const uint32_t out = vid - H;
                    if (out >= (uint64_t)b.cap_v) { *b.overflow = 1u; continue; }
                    float px, py, pz;
                    if (slot == 0) {        // edge 5: VIntY at qxz, (fx2, fy + mu*dy, fz2), field5 -> field7
                        const float mu = (0.f - v.f[5]) / (v.f[7] - v.f[5]);
                        px = fx2; py = fy + mu * g.w[1]; pz = fz2;
                    } else if (slot == 1) { // edge 6: VIntX at qyz, (fx + mu*dx, fy2, fz2), field6 -> field7
                        const float mu = (0.f - v.f[6]) / (v.f[7] - v.f[6]);
                        px = fx + mu * g.w[0]; py = fy2; pz = fz2;
                    } else {                // edge 10: VIntZ at qxy, (fx2, fy2, fz + mu*dz), field3 -> field7
                        const float mu = (0.f - v.f[3]) / (v.f[7] - v.f[3]);
                        px = fx2; py = fy2; pz = fz + mu * g.w[2];
                    }
                    b.verts[3 * (size_t)out] = px;
                    b.verts[3 * (size_t)out + 1] = py;
                    b.verts[3 * (size_t)out + 2] = pz;
                }
            }
            if (act) {
                const uint32_t ri = ab + f_act(pre);
                if (ri < (uint64_t)b.cap_rec) b.records[ri] = make_uint4(L, ci, fb + f_tri(pre), 0u);
                else *b.overflow = 1u;
            }
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
    for (uint32_t i = blockIdx.x * 256 + t; i < lim; i += gridDim.x * 256) {
        const uint4 r = b.records[i];
        const uint32_t L = r.x, ci = r.y, fbase = r.z;
        const CaseInfo& C = s_case[ci];
        if (fbase + C.ntri > (uint64_t)b.cap_f) { *b.overflow = 1u; continue; }
        int32_t* out = b.faces + 3 * (size_t)fbase;
        for (int k = 0; k < 3 * C.ntri; ++k) {
            const int e = C.tri[k];
            const uint32_t owner = L - (uint32_t)s_off[e];
            out[k] = (int32_t)b.vid3[(size_t)owner * 3 + s_slot[e]];
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
    k_mc_scan<<<1, 1024, 0, s>>>(b.unit_cnt, n_units(g), b.counters);
}

void launch_mc_emit(const CaseInfo* d_cases, const GridDesc& g, const MCBuffers& b, hipStream_t s) {
    k_mc_verts<<<2048, 256, 0, s>>>(d_cases, g, b);
    k_mc_faces<<<2048, 256, 0, s>>>(d_cases, g, b);
}

}  // namespace impli
