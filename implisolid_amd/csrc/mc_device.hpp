// mc_device.hpp -- device side of marching cubes shared by the static kernels (mc.hip) and the
// JIT module (jit.cpp): sign-bitmap chunks and the vertex-emission body (K3).
#pragma once
#include "eval_bricks.hpp"
#include "mc_types.hpp"

namespace impli {

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// three owned-edge vertex ids, one 12-byte access
struct __attribute__((packed, aligned(4))) IdTriple { uint32_t a, b, c; };

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
    const int r32 = (int)row;   // rows of a slab: m x layers < 2^31 (cells < 2^32, slab_range)
    k.y = r32 % g.m + 1;
    k.z = r32 / g.m + g.cz0;
    k.x0 = 64 * c + 1;
    const int64_t r00 = ((int64_t)(k.z - g.fz0) * g.n + (k.y - 1)) * rw;   // (layer, stored y) -> word index
    const int64_t rows[4] = {r00, r00 + rw, r00 + (int64_t)g.n * rw, r00 + (int64_t)g.n * rw + rw};
    // all eight loads issued before any use (a conditional load becomes a branch with its own
    // wait, serialising the rows): past a row's last word the next row's first word (or the
    // bitmap's tail padding) is read and discarded
    uint64_t w[4], nx[4], s[4], t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        w[q] = signs[rows[q] + c];
        nx[q] = signs[rows[q] + c + 1];
    }
    // arithmetic mask, not a select: a select of a loaded value is turned back into a load under
    // a branch
    const uint64_t keep = 0ull - (uint64_t)(c + 1 < rw);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        s[q] = w[q];
        t[q] = (w[q] >> 1) | ((nx[q] & keep) << 63);
    }
    k.s00 = s[0]; k.t00 = t[0]; k.s10 = s[1]; k.t10 = t[1]; k.s01 = s[2]; k.t01 = t[2]; k.s11 = s[3]; k.t11 = t[3];
    const uint64_t all = s[0] & t[0] & s[1] & t[1] & s[2] & t[2] & s[3] & t[3];
    const uint64_t any = s[0] | t[0] | s[1] | t[1] | s[2] | t[2] | s[3] | t[3];
    const int left = g.m - 64 * c;   // cells of this chunk inside the row
    const uint64_t valid = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
    k.nt = any & ~all & valid;
}

// Bourke cube edges / faces / opposite corner pairs (corner k = bit k of the cube index)
constexpr int kCubeEdges[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {4, 5}, {5, 6},
                                   {6, 7}, {7, 4}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
constexpr int kCubeFaces[6][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {0, 1, 5, 4}, {1, 2, 6, 5}, {2, 3, 7, 6}, {3, 0, 4, 7}};
constexpr int kCubeOpposite[4][2] = {{0, 6}, {1, 7}, {2, 4}, {3, 5}};

// Triangles of the non-trivial cells of a chunk, all 64 at once.  In the table a case with E
// crossing edges has E - 2 P triangles, P its polygons: the connected components of its negative
// corners, V - E_int + F_full (independent cycles of the induced cube subgraph are its full
// faces), except the four cases with exactly two opposite positive corners, whose six-cycle the
// table splits into two triangles (P = 2).  Checked for all 256 cases by build_case_table.
__device__ __forceinline__ unsigned chunk_triangles(const ChunkBits& k) {
    const uint64_t c[8] = {k.s00, k.t00, k.t10, k.s10, k.s01, k.t01, k.t11, k.s11};   // corner k of each cell
    const uint64_t nt = k.nt;
    int ec = 0, ei = 0, v = 0, ff = 0, opp = 0;
#pragma unroll
    for (int e = 0; e < 12; ++e) {
        const uint64_t a = c[kCubeEdges[e][0]], b = c[kCubeEdges[e][1]];
        ec += __popcll((unsigned long long)((a ^ b) & nt));
        ei += __popcll((unsigned long long)(a & b & nt));
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) v += __popcll((unsigned long long)(c[q] & nt));
#pragma unroll
    for (int f = 0; f < 6; ++f)
        ff += __popcll((unsigned long long)(c[kCubeFaces[f][0]] & c[kCubeFaces[f][1]] & c[kCubeFaces[f][2]] &
                                            c[kCubeFaces[f][3]] & nt));
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const int a = kCubeOpposite[o][0], b = kCubeOpposite[o][1];
        uint64_t rest = ~c[a] & ~c[b] & nt;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q != a && q != b) rest &= c[q];
        opp += __popcll((unsigned long long)rest);
    }
    return (unsigned)(ec - 2 * (v - ei + ff + 2 * opp));
}

// cube index of cell j of a chunk, corner bits as polygonize_single_cube (:553-560)
__device__ __forceinline__ unsigned chunk_ci(const ChunkBits& k, int j) {
    return (unsigned)((k.s00 >> j) & 1u) | ((unsigned)((k.t00 >> j) & 1u) << 1) | ((unsigned)((k.s10 >> j) & 1u) << 3) |
           ((unsigned)((k.t10 >> j) & 1u) << 2) | ((unsigned)((k.s01 >> j) & 1u) << 4) |
           ((unsigned)((k.t01 >> j) & 1u) << 5) | ((unsigned)((k.s11 >> j) & 1u) << 7) |
           ((unsigned)((k.t11 >> j) & 1u) << 6);
}

// K3: one wave per unit.  Lanes find the non-trivial cells of their (row, chunk) items; the cells
// are then taken in cell order, 64 at a time: a wave scan of (owned edges, triangles, active)
// gives every cell its vertex / face / record base; owned vertices are
// placed from the owner cell's fx/fy/fz (the reference's first emission) (halo cells, below the
// slab's first emitted layer: ids only), active cells get a record {L, ci, face base}; the ids of a
// cell owning a crossing edge go to the dense per-cell table (vid), where the face pass reads its
// owners' ids by cell id.  (A separate one-lane-per-active-cell
// position pass measured 2 us slower.)
// a window's (owned edges <= 3, triangles <= 5, active <= 1) per cell, packed for one 32-bit scan:
// over 64 cells the sums stay below 2^8 (192), 2^10 (320) and 2^7 (64)
constexpr int kPackShift[3] = {0, 8, 18};
constexpr unsigned kPackMask[3] = {0xffu, 0x3ffu, 0x7fu};
__device__ __forceinline__ unsigned pack3(unsigned own, unsigned tri, unsigned act) {
    return own | (tri << 8) | (act << 18);
}
__device__ __forceinline__ unsigned fld(unsigned p, int i) { return (p >> kPackShift[i]) & kPackMask[i]; }

// position of the r-th set bit of x (r < popcount(x))
__device__ __forceinline__ int select_bit(uint64_t x, uint32_t r) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) {
        const uint32_t c = (uint32_t)__popcll((unsigned long long)(x & ((1ull << w) - 1ull)));
        if (r >= c) { r -= c; x >>= w; pos += w; }
    }
    return pos;
}

// Waves take the parts of the non-empty units from the flat list (k_unit_scan) grid-stride: every
// resident wave gets an equal share whatever the surface's distribution over groups, and a heavy
// unit (up to ~2000 cells) is spread over up to kMaxParts waves instead of serialising its 64-cell
// windows, each with a field round trip, on one.  A
// unit's items (row, 64-cell chunk) go to LDS with their exclusive cell counts; each lane then
// finds its own cell -- the item by binary search, the cell by selecting the bit -- so cells are
// listed in cell order 64 at a time, with no lane looping over a dense chunk's bits.
// one part e of the flat unit list, by the calling wave (s_case: the case table in LDS; bits /
// excl: the wave's LDS scratch)
// the case facts the vertex pass needs, one word per case: nown (bits 0-1), ntri (2-4), and the
// rank of owned edge slot s + 1 (0: unused) in bits 5 + 3 s (an 8 KB CaseInfo table in LDS held
// the cells kernel to five waves per SIMD)
__device__ __forceinline__ uint32_t case_word(const CaseInfo& c) {
    uint32_t w = (uint32_t)c.nown | ((uint32_t)c.ntri << 2);
    for (int s = 0; s < 3; ++s) w |= (uint32_t)(c.rank[s] + 1) << (5 + 3 * s);
    return w;
}

__device__ __forceinline__ void mc_cells_part(const uint32_t* s_cw, const GridDesc& g, const MCBuffers& b, uint32_t e,
                                              uint64_t (*bits)[64], uint32_t* excl) {
    const int lane = threadIdx.x & 63;
    const uint32_t H = b.counters[1];
    const int nch = (g.m + 63) / 64;
    const int64_t rows = n_rows(g);
    const int items = kUnitRows * nch;
    {
        // the e-th part: heavy parts from the list's front, then the light ones from its end
        const uint32_t nh = b.counters[7];
        e = e < nh ? e : b.cap_parts - 1u - (e - nh);
        const uint4 ent = b.ulist[e];   // {unit, vbase, fbase, abase}
        // part | parts << 4 | chunk mask << 8: this wave emits windows w % parts == part; the unit's
        // chunks without a non-trivial cell (k_mc_count) are not loaded
        const uint32_t up = b.upart[e];
        const uint32_t part = up & 15u, parts = (up >> 4) & 15u;
        const uint32_t cmask = nch <= kChunkMaskBits ? up >> 8 : ~0u;
        const int64_t u = ent.x;
        uint32_t vrun0 = ent.y, frun0 = ent.z, arun0 = ent.w;
        uint32_t win = 0;   // 64-cell window index within the unit
        for (int i0 = 0; i0 < items; i0 += 64) {
            const int i = i0 + lane;
            ChunkBits k;
            k.nt = 0;
            k.z = 0;
            const int64_t irow = u * kUnitRows + i / nch;
            const int ic = i % nch;
            if (i < items) {
                if (irow < rows && (ic >= kChunkMaskBits || ((cmask >> ic) & 1u))) load_chunk(g, b.signs, irow, ic, k);
            }
            const uint32_t cnt = (uint32_t)__popcll((unsigned long long)k.nt);
            const uint32_t incl = wave_incl_scan<uint32_t>(cnt, lane);
            const uint32_t total = __shfl(incl, 63, 64);
            __builtin_amdgcn_wave_barrier();   // the previous batch's LDS reads are done
            bits[0][lane] = k.s00; bits[1][lane] = k.t00; bits[2][lane] = k.s10; bits[3][lane] = k.t10;
            bits[4][lane] = k.s01; bits[5][lane] = k.t01; bits[6][lane] = k.s11; bits[7][lane] = k.t11;
            bits[8][lane] = k.nt;
            excl[lane] = incl - cnt;
            __builtin_amdgcn_wave_barrier();
            for (uint32_t e0 = 0; e0 < total; e0 += 64, ++win) {
                const bool mine = win % parts == part;   // uniform: other windows only advance the bases
                const uint32_t ce = e0 + (uint32_t)lane;
                const bool has = ce < total;
                // the item holding cell ce: the last item whose exclusive count is <= ce (items
                // without cells share the next one's count, so the last such item has cells)
                int q = 0;
#pragma unroll
                for (int step = 32; step > 0; step >>= 1)
                    if (excl[q + step] <= ce) q += step;
                const int j = has ? select_bit(bits[8][q], ce - excl[q]) : 0;
                const unsigned ci =
                    has ? (unsigned)((bits[0][q] >> j) & 1u) | ((unsigned)((bits[1][q] >> j) & 1u) << 1) |
                              ((unsigned)((bits[3][q] >> j) & 1u) << 2) | ((unsigned)((bits[2][q] >> j) & 1u) << 3) |
                              ((unsigned)((bits[4][q] >> j) & 1u) << 4) | ((unsigned)((bits[5][q] >> j) & 1u) << 5) |
                              ((unsigned)((bits[7][q] >> j) & 1u) << 6) | ((unsigned)((bits[6][q] >> j) & 1u) << 7)
                        : 0u;   // chunk_ci of item q, cell j
                const int it = i0 + q;
                const int64_t erow = u * kUnitRows + it / nch;
                const int x = 64 * (it % nch) + 1 + j;
                const int z = (int)erow / g.m + g.cz0;
                const uint32_t L = (uint32_t)(erow * g.m + (x - 1));
                const uint32_t cw = s_cw[ci];
                const unsigned c_nown = cw & 3u, c_ntri = (cw >> 2) & 7u;
                const bool emit = has && z >= g.cz_emit;
                const unsigned own = has ? c_nown : 0u, tri = emit ? c_ntri : 0u, act = (emit && c_ntri) ? 1u : 0u;
                const unsigned p = pack3(own, tri, act);
                const unsigned inc = wave_incl_scan<unsigned>(p, lane);
                const unsigned pre = inc - p, tot = __shfl(inc, 63, 64);
                const uint32_t vrun = vrun0 + fld(pre, 0);
                if (mine) {
                    const int y = (int)erow % g.m + 1;
                    const int sx = x - 1, sy = y - 1, sl = z - g.fz0;
                    // corners 7 (1,1,1), 5 (1,0,1), 6 (0,1,1), 3 (1,1,0) of the brick-major field
                    // (grid.hpp field_index, split into per-axis terms); lanes without a cell read
                    // sample 0
                    const int cx = has ? sx : 0, cy = has ? sy : 0, cl = has ? sl : 0, d = has ? 1 : 0;
                    const uint32_t fx0 = field_x_term(cx), fx1 = field_x_term(cx + d);
                    const uint32_t fy0 = field_y_term(g, cy), fy1 = field_y_term(g, cy + d);
                    const int64_t fl0 = field_layer_term(g, cl), fl1 = field_layer_term(g, cl + d);
                    const float r7 = b.field[fl1 + (fy1 + fx1)];
                    const float r5 = b.field[fl1 + (fy0 + fx1)];
                    const float r6 = b.field[fl1 + (fy1 + fx0)];
                    const float r3 = b.field[fl0 + (fy1 + fx1)];
                    const bool sx1 = sealed_xy(g, sx + 1), sy1 = sealed_xy(g, sy + 1), sz1 = sealed_z(g, sl + 1);
                    const bool sx0 = sealed_xy(g, sx), sy0 = sealed_xy(g, sy), sz0 = sealed_z(g, sl);
                    const float f7 = (sx1 || sy1 || sz1) ? kSealed : r7;
                    const float f5 = (sx1 || sy0 || sz1) ? kSealed : r5;
                    const float f6 = (sx0 || sy1 || sz1) ? kSealed : r6;
                    const float f3 = (sx1 || sy1 || sz0) ? kSealed : r3;
                    // the cell's owned ids (slot order 5, 6, 10; an unused slot's word is never read)
                    uint32_t ids[3];
#pragma unroll
                    for (int slot = 0; slot < 3; ++slot) ids[slot] = vrun + (uint32_t)((cw >> (5 + 3 * slot)) & 7u) - 1u - H;
                    if (has && own) {
                        const float fx = ((float)x + g.i0[0]) * g.w[0];
                        const float fy = ((float)y + g.i0[1]) * g.w[1];
                        const float fz = ((float)z + g.i0[2]) * g.w[2];
                        const float fx2 = fx + g.w[0], fy2 = fy + g.w[1], fz2 = fz + g.w[2];
#pragma unroll
                        for (int slot = 0; slot < 3; ++slot) {
                            const int r = (int)((cw >> (5 + 3 * slot)) & 7u) - 1;
                            if (r < 0 || !emit) continue;
                            const uint32_t out = ids[slot];
                            if (out >= (uint64_t)b.cap_v) { *b.overflow = 1u; continue; }
                            float px, py, pz;
                            if (slot == 0) { const float mu = (0.f - f5) / (f7 - f5); px = fx2; py = fy + mu * g.w[1]; pz = fz2; }
                            else if (slot == 1) { const float mu = (0.f - f6) / (f7 - f6); px = fx + mu * g.w[0]; py = fy2; pz = fz2; }
                            else { const float mu = (0.f - f3) / (f7 - f3); px = fx2; py = fy2; pz = fz + mu * g.w[2]; }
                            b.verts[3 * (size_t)out] = px; b.verts[3 * (size_t)out + 1] = py; b.verts[3 * (size_t)out + 2] = pz;
                        }
                        // the cell's owned ids by cell id (halo cells too: the slab's layer below its
                        // first emitted one), where the face pass looks its owners up
                        *reinterpret_cast<IdTriple*>(b.vid + (size_t)L * 3) = IdTriple{ids[0], ids[1], ids[2]};
                    }
                    if (act) {   // an active cell: its record, at its record index
                        const uint32_t arun = arun0 + fld(pre, 2);
                        if (arun < (uint64_t)b.cap_rec) b.records[arun] = make_uint4(L, ci, frun0 + fld(pre, 1), (uint32_t)erow);
                        else *b.overflow = 1u;
                    }
                }
                vrun0 += fld(tot, 0);
                frun0 += fld(tot, 1);
                arun0 += fld(tot, 2);
            }
        }
    }
}

__device__ __forceinline__ void mc_cells_body(const CaseInfo* __restrict__ cases, const GridDesc& g, const MCBuffers& b) {
    __shared__ uint32_t s_cw[256];
    __shared__ uint64_t s_bits[kVertsWaves][9][64];   // per wave and item: the 8 corner words + nt
    __shared__ uint32_t s_excl[kVertsWaves][64];      // per wave and item: cells in the items before it
    const int t = threadIdx.x, wid = t >> 6;
    const uint32_t n_ne = b.counters[0];              // non-empty units
    const uint32_t w0 = blockIdx.x * kVertsWaves;
    if (w0 >= n_ne) return;                           // uniform over the block
    for (int k = t; k < 256; k += blockDim.x) s_cw[k] = case_word(cases[k]);
    __syncthreads();
    for (uint32_t e = w0 + wid; e < n_ne; e += gridDim.x * kVertsWaves) mc_cells_part(s_cw, g, b, e, s_bits[wid], s_excl[wid]);
}

}  // namespace impli
