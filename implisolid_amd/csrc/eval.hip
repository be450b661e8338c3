// eval.hip -- implicit-function field evaluation on gfx950.
//
// k_eval_field : one lane per stored (interior) sample of the slab; the node program is
//                interpreted in lock step by the whole wave (uniform scalar loads of the
//                program and matrices), the result is written once, coalesced, x fastest.
//                Replaces prepare_grid + eval_shape (marching_cubes.hpp:1662-1725) -- the
//                reference's res^3 x 12 B point grid and its per-node batch copies never exist.
// k_brick_modes / k_eval_field_pruned: the same field, computed per brick of kBX x kBY x kBZ
//                samples.  A first pass bounds every node of the program over each brick
//                (ifunc_interval.hpp), records which CSG operands provably win and the brick's
//                sign class; the second pass (one wave per brick) skips the losing subtrees.
//                Level 1: bit-identical to k_eval_field (test_pruned_field_identical).
//                Level 2 (sign_fill): bricks that are sign-definite together with their face
//                neighbours get +-1 instead of exact values -- no cell edge touching them changes
//                sign, so marching cubes reads only their sign and the mesh is bit-identical
//                (test_sign_fill_field_equivalent + every MC parity test).
// k_eval_points: arbitrary points (direct-eval ABI, mcc2.cpp:815-911) with optional gradient.
#include <algorithm>
#include <stdexcept>
#include <cstddef>
#include <cstdlib>

#include "ifunc_device.hpp"
#include "ifunc_interval.hpp"
#include "eval_bricks.hpp"
#include "brick_modes.hpp"
#include "kernels.hpp"
#include "jit.hpp"
#include "batch_device.hpp"

namespace impli {

using namespace dev;

// one wave per brick layer (64 stored samples, lane = (y % 8) * 8 + x % 8), in storage order: the
// wave writes its 256 contiguous bytes (this unpruned path also calibrates the PMC write counter,
// tools/pmc_traffic.py)
template <int D>
__global__ __launch_bounds__(256) void k_eval_field(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                    GridDesc g, BrickGrid bg, float* __restrict__ field) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // brick layer: brick w / kBZ, layer w % kBZ
    const int lane = threadIdx.x & 63;
    if (w >= (int64_t)bg.n_bricks * kBZ) return;
    int bx, by, bz;
    brick_of((int)(w / kBZ), bg, bx, by, bz);
    const int sx = bx * kBX + lane % kBX, sy = by * kBY + lane / kBX, layer = bz * kBZ + (int)(w % kBZ);
    float f = kSealed;
    if (sx < g.n && sy < g.n && layer < g.fz1 - g.fz0 &&
        !(sealed_xy(g, sx) || sealed_xy(g, sy) || sealed_z(g, layer)))
        f = 0.f + eval_f<D>(prog, tab, sample_xy(g, 0, sx), sample_xy(g, 1, sy), sample_z(g, layer));
    field[w * (kBX * kBY) + lane] = f;   // eval_shape: field (zero) += value
}

// A program pointer loaded from memory (ObjArgs::prog of a merged object stream) is generic: loads
// through it are flat vector loads, so every instruction fetch of the interpreter was a memory round
// trip and its fields and stack indices VGPR values.  The program is read-only during a launch, so
// the merged kernels read it through the constant address space (scalar loads, uniform indices).
typedef const __attribute__((address_space(4))) Program* ProgC;
__device__ __forceinline__ ProgC prog_const(const Program* p) { return (ProgC)p; }

template <int D, class ProgP = const Program*>
struct InterpIv {   // the interval interpreter (ifunc_interval.hpp eval_iv)
    ProgP prog;
    const float* tab;
    float2 tab_range;
    __device__ __forceinline__ Iv operator()(Box p, uint64_t modes_in, uint64_t& modes) const {
        return eval_iv<D>(prog, tab, tab_range, p, modes_in, modes);
    }
};

template <int D>
__global__ __launch_bounds__(256) void k_coarse_modes(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                      float2 tab_range, GridDesc g, BrickGrid cg,
                                                      uint64_t* __restrict__ cmodes, uint8_t* __restrict__ ccls,
                                                      uint32_t* __restrict__ clist, uint32_t* __restrict__ counters) {
    coarse_modes_body(InterpIv<D>{prog, tab, tab_range}, g, cg, cmodes, ccls, clist, counters);
}

template <int D>
__global__ __launch_bounds__(256) void k_brick_refine(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                      float2 tab_range, GridDesc g, BrickGrid bg, BrickGrid cg,
                                                      const uint64_t* __restrict__ cmodes,
                                                      const uint32_t* __restrict__ clist,
                                                      const uint32_t* __restrict__ ccount, uint64_t* __restrict__ modes,
                                                      uint8_t* __restrict__ cls) {
    // wave-uniform starting modes: uniform skips, so the interpreter's instruction fetch stays scalar
    brick_refine_body<InterpIv<D>, true>(InterpIv<D>{prog, tab, tab_range}, g, bg, cg, cmodes, clist, ccount, modes, cls);
}

template <int D, class ProgP = const Program*>
struct InterpEval {   // the node-program interpreter with per-brick operand skipping
    ProgP prog;
    const float* tab;
    __device__ __forceinline__ float operator()(uint64_t m, float x, float y, float z) const {
        return eval_f_pruned<D>(prog, tab, m, x, y, z);
    }
};

// A brick column's two samples in one pass of the interpreter: one instruction decode, one mode
// test and one primitive dispatch serve both, and the two dependency chains sit in the same basic
// blocks, so they interleave.  Per sample the operations are exactly eval_f_pruned's (bit-identical).
__device__ __forceinline__ void prim_f2(int t, const float* __restrict__ tab, const float* __restrict__ prm, float x0,
                                        float y0, float z0, float x1, float y1, float z1, float& a, float& b) {
    switch (t) {
        case NT_ELLIPSOID: a = egg_f(x0, y0, z0); b = egg_f(x1, y1, z1); return;
        case NT_CUBE: a = cube_f(tab, x0, y0, z0); b = cube_f(tab, x1, y1, z1); return;
        case NT_CYLINDER: a = cyl_f(x0, y0, z0); b = cyl_f(x1, y1, z1); return;
        case NT_CONE: a = cone_f(x0, y0, z0); b = cone_f(x1, y1, z1); return;
        case NT_HEART: a = heart_f(x0, y0, z0); b = heart_f(x1, y1, z1); return;
        case NT_TORUS: a = torus_f(x0, y0, z0); b = torus_f(x1, y1, z1); return;
        case NT_SCREW: a = screw_f(prm, x0, y0, z0); b = screw_f(prm, x1, y1, z1); return;
        case NT_LID: a = lid_f(z0); b = lid_f(z1); return;
        case NT_HALF_PLANE: a = hp_f(prm, x0, y0, z0); b = hp_f(prm, x1, y1, z1); return;
        case NT_TETRA: a = tet_f(prm, x0, y0, z0); b = tet_f(prm, x1, y1, z1); return;
        case NT_METABALLS: a = meta_f(prm, x0, y0, z0); b = meta_f(prm, x1, y1, z1); return;
        case NT_EXTRUSION: a = extr_f(prm, x0, y0); b = extr_f(prm, x1, y1); return;
        case NT_SCREW_TBB: a = tbb_f(prm, x0, y0, z0); b = tbb_f(prm, x1, y1, z1); return;
        default: a = dm_f(x0, y0, z0); b = dm_f(x1, y1, z1); return;
    }
}

// D: the point stacks' capacity (tree depth + 1); V: the value stacks' (the most values a postfix
// program holds at once, Engine::vdepth(): a Sethi-Ullman-like count, usually well below D)
template <int D, class ProgP, int V = D>
__device__ __forceinline__ void eval_f2_pruned(ProgP __restrict__ prog, const float* __restrict__ tab,
                                               uint64_t modes, float x, float y, float z0, float z1, float& r0,
                                               float& r1) {
    float px0[D], py0[D], pz0[D], px1[D], py1[D], pz1[D], vf0[V], vf1[V];
    int sp = 0, vp = 0;
    px0[0] = x; py0[0] = y; pz0[0] = z0;
    px1[0] = x; py1[0] = y; pz1[0] = z1;
    const int n = prog->n_instr;
    for (int pc = 0; pc < n; ++pc) {
        const Instr I = instr_at(prog, pc);
        if (I.skip_csg >= 0) {
            const uint32_t m = mode_of(modes, I.skip_csg);
            if (m == (I.skip_child ? (uint32_t)PM_LEFT : (uint32_t)PM_RIGHT)) {
                pc = I.skip_to - 1;
                continue;
            }
        }
        if (I.op == OP_XFORM) {
            const float* M = mat_row(prog, I.mat);
            const bool diag = I.type == XF_DIAG;
            const V3 q0 = diag ? xform_diag(M, px0[sp], py0[sp], pz0[sp]) : xform(M, px0[sp], py0[sp], pz0[sp]);
            const V3 q1 = diag ? xform_diag(M, px1[sp], py1[sp], pz1[sp]) : xform(M, px1[sp], py1[sp], pz1[sp]);
            ++sp;
            px0[sp] = q0.x; py0[sp] = q0.y; pz0[sp] = q0.z;
            px1[sp] = q1.x; py1[sp] = q1.y; pz1[sp] = q1.z;
        } else if (I.op == OP_PRIM) {
            float a, b;
            prim_f2(I.type, tab, mat_row(prog, I.prm), px0[sp], py0[sp], pz0[sp], px1[sp], py1[sp], pz1[sp], a, b);
            vf0[vp] = a; vf1[vp] = b;
            ++vp;
            --sp;
        } else {
            --sp;
            const uint32_t m = mode_of(modes, I.csg);
            if (m == PM_BOTH) {
                --vp;
                const float a2 = vf0[vp], a1 = vf0[vp - 1], b2 = vf1[vp], b1 = vf1[vp - 1];
                if (I.type == NT_UNION) {
                    vf0[vp - 1] = (a1 > a2) ? a1 : a2; vf1[vp - 1] = (b1 > b2) ? b1 : b2;
                } else if (I.type == NT_INTERSECTION) {
                    vf0[vp - 1] = (a1 > a2) ? a2 : a1; vf1[vp - 1] = (b1 > b2) ? b2 : b1;
                } else {
                    vf0[vp - 1] = (a1 < -a2) ? a1 : -a2; vf1[vp - 1] = (b1 < -b2) ? b1 : -b2;
                }
            } else if (m == PM_RIGHT && I.type == NT_DIFFERENCE) {
                vf0[vp - 1] = -vf0[vp - 1];
                vf1[vp - 1] = -vf1[vp - 1];
            }
        }
    }
    r0 = vf0[0];
    r1 = vf1[0];
}

template <int D, class ProgP = const Program*, int V = D>
struct InterpEval2 : InterpEval<D, ProgP> {   // the interpreter with the layer pair (eval_bricks.hpp eval_pair)
    __device__ __forceinline__ void pair(uint64_t m, float x, float y, float z0, float z1, float& f0, float& f1) const {
        eval_f2_pruned<D, ProgP, V>(this->prog, this->tab, m, x, y, z0, z1, f0, f1);
    }
};

// the interpreter's brick eval (merged streams, and single objects until their module is loaded):
// both layers per pass unless IMPLISOLID_INTERP_PAIR=0
static bool interp_pair() {
    static const bool on = [] {
        const char* s = std::getenv("IMPLISOLID_INTERP_PAIR");
        return !(s && std::atoi(s) == 0);
    }();
    return on;
}

template <int D, bool Pair>
__global__ __launch_bounds__(kEvalBlock) void k_eval_field_pruned(const Program* __restrict__ prog,
                                                           const float* __restrict__ tab, GridDesc g, BrickGrid bg,
                                                           const uint64_t* __restrict__ modes,
                                                           const uint32_t* __restrict__ list,
                                                           const uint32_t* __restrict__ count,
                                                           float* __restrict__ field, void* __restrict__ signs,
                                                           ClaimCtx cc) {
    if constexpr (Pair) eval_bricks_body(InterpEval2<D>{{prog, tab}}, g, bg, cc, modes, list, count, field, signs);
    else eval_bricks_body(InterpEval<D>{prog, tab}, g, bg, cc, modes, list, count, field, signs);
}

// Per brick: its class (inherited from a sign-definite coarse box, or refined), the neighbour rule
// (brick_modes.hpp), fill[b] = class | fill class << 4, and either the constant sign pieces of a
// sign-filled brick or an entry in the list of bricks to evaluate (with its modes, so the eval
// kernel reads them in list order).
//
// One thread per sign word of a brick row: the kFillP bricks (bx = kFillP c ...) whose pieces make
// up word c of the row's sample rows.  The class bytes of the bricks and of their neighbour rows
// (y +- 1, z +- 1) are kFillP consecutive bytes each (one unaligned 8-byte load per row), and the
// word is the same for every sample row of the brick row: kBY kBZ whole-word stores, consecutive
// lanes on consecutive words.  Listed bricks get a zero placeholder piece that the eval kernel
// overwrites (stream order); bytes past a row's last brick are bitmap padding (never read as a cell
// corner).  List appends are aggregated per block: one atomic per block (same-address atomics
// serialise: a wave-level append measured +30 us); the units a listed brick marks depend on its
// row only, so a thread marks them once.
constexpr int kFillBlock = 256;
constexpr int kFillP = 64 / kBX;   // bricks (sign pieces) per sign word
static_assert(kFillP <= 8, "one 8-byte class load per row");

struct RowSeal { bool has, only; };   // sealed_class's row terms (y, z) of a brick row
__device__ __forceinline__ RowSeal row_seal(const GridDesc& g, int by, int bz) {
    const BrickBox q = brick_box(g, 0, by, bz, kBZ);
    return RowSeal{q.y0 == 0 || q.y1 == g.n - 1 || g.fz0 + q.z0 <= 1 || g.fz0 + q.z1 >= g.res - 2,
                   q.y0 == g.n - 1 || (q.z0 == q.z1 && (g.fz0 + q.z0 <= 1 || g.fz0 + q.z0 >= g.res - 2))};
}
// brick_class_of (brick_modes.hpp) from the row's terms and the brick's x terms
__device__ __forceinline__ uint32_t class_adj(uint8_t c, uint8_t r, bool has, bool only) {
    if (c == kBrickMixed) return r;
    uint32_t v = only ? (uint32_t)kBrickNeg : (uint32_t)c;
    if (has && v == kBrickPos) v |= kBrickNoFill;
    return v;
}
__device__ __forceinline__ uint64_t load_row_bytes(const uint8_t* p) {   // kFillP bytes, any alignment
    uint64_t v = 0;
    __builtin_memcpy(&v, p, kFillP);
    return v;
}

__device__ __forceinline__ void brick_fill_body(const GridDesc& g, const BrickGrid& bg, const BrickGrid& cg,
                                                const uint8_t* __restrict__ ccls, const uint64_t* __restrict__ cmodes,
                                                const uint8_t* __restrict__ cls, const uint64_t* __restrict__ modes,
                                                int sign_fill, uint8_t* __restrict__ fill, uint32_t* __restrict__ list,
                                                uint64_t* __restrict__ lmodes, uint32_t* __restrict__ count,
                                                sign_piece_t* __restrict__ signs, uint32_t* __restrict__ ccount_reset,
                                                uint32_t* __restrict__ umark, uint32_t mark_id) {
    __shared__ uint32_t wsum[kFillBlock / 64], wbase[kFillBlock / 64];
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // the refine pass has read it; kept in [14] for stats
        ccount_reset[1] = ccount_reset[0];
        ccount_reset[0] = 0u;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rw = sign_row_words(g), layers = g.fz1 - g.fz0;
    const int plane = bg.nbx * bg.nby, cplane = cg.nbx * cg.nby;
    const int64_t item = (int64_t)blockIdx.x * kFillBlock + threadIdx.x;
    const bool valid = item < (int64_t)bg.nby * bg.nbz * rw;
    int c = 0, by = 0, bz = 0, nv = 0, bx0 = 0, b0 = 0;
    uint32_t own[kFillP], fc[kFillP];
    uint64_t oc = 0;   // the row's coarse class bytes
    if (valid) {
        c = (int)(item % rw);
        const int rr = (int)(item / rw);
        by = rr % bg.nby;
        bz = rr / bg.nby;
        bx0 = kFillP * c;
        nv = min(kFillP, bg.nbx - bx0);   // >= 1: rw words cover nbx bricks
        b0 = bx0 + by * bg.nbx + bz * plane;
        const int cb0 = bx0 + by * cg.nbx + (bz / kCZ) * cplane;
        const int yl = by > 0 ? by - 1 : by, yh = by + 1 < bg.nby ? by + 1 : by;
        const int zl = bz > 0 ? bz - 1 : bz, zh = bz + 1 < bg.nbz ? bz + 1 : bz;
        // rows: own, y - 1, y + 1, z - 1, z + 1 (a neighbour outside the grid is the row itself)
        const int rb[5] = {b0, b0 + (yl - by) * bg.nbx, b0 + (yh - by) * bg.nbx, b0 + (zl - bz) * plane,
                           b0 + (zh - bz) * plane};
        const int rc[5] = {cb0, cb0 + (yl - by) * cg.nbx, cb0 + (yh - by) * cg.nbx,
                           bx0 + by * cg.nbx + (zl / kCZ) * cplane, bx0 + by * cg.nbx + (zh / kCZ) * cplane};
        const int ry[5] = {by, yl, yh, by, by}, rz[5] = {bz, bz, bz, zl, zh};
        uint64_t rcls[5], rccl[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            rcls[k] = load_row_bytes(cls + rb[k]);
            rccl[k] = load_row_bytes(ccls + rc[k]);
        }
        // x neighbours of the word's first and last brick (the brick itself at the grid's edge)
        const int xl = bx0 > 0 ? bx0 - 1 : bx0, xh = bx0 + nv < bg.nbx ? bx0 + nv : bx0 + nv - 1;
        const uint8_t lcls = cls[b0 + xl - bx0], lccl = ccls[cb0 + xl - bx0];
        const uint8_t hcls = cls[b0 + xh - bx0], hccl = ccls[cb0 + xh - bx0];
        oc = rccl[0];
        RowSeal rs[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) rs[k] = row_seal(g, ry[k], rz[k]);
        auto xs_has = [&](int x) { return x * kBX == 0 || min(x * kBX + kBX - 1, g.n - 1) == g.n - 1; };
        auto xs_only = [&](int x) { return x * kBX == g.n - 1; };
        uint32_t nb[5][kFillP];
#pragma unroll
        for (int j = 0; j < kFillP; ++j) {
            const int x = bx0 + j;
            const bool hx = xs_has(x), ox = xs_only(x);
#pragma unroll
            for (int k = 0; k < 5; ++k)
                nb[k][j] = class_adj((uint8_t)(rccl[k] >> (8 * j)), (uint8_t)(rcls[k] >> (8 * j)), hx || rs[k].has,
                                     ox || rs[k].only);
        }
        const uint32_t left = class_adj(lccl, lcls, xs_has(xl) || rs[0].has, xs_only(xl) || rs[0].only);
        const uint32_t right = class_adj(hccl, hcls, xs_has(xh) || rs[0].has, xs_only(xh) || rs[0].only);
#pragma unroll
        for (int j = 0; j < kFillP; ++j) {
            own[j] = nb[0][j];
            const uint32_t xm = j == 0 ? left : nb[0][j - 1];
            const uint32_t xp = j + 1 < nv ? nb[0][j + 1] : right;
            // sign-filled: all six neighbours of its class; candidate: the others all of mixed class
            uint32_t f = kBrickMixed, cand = 0;
            const uint32_t o = own[j] & 3u;
            if (sign_fill && o != kBrickMixed && !(own[j] & kBrickNoFill)) {
                const uint32_t nn[6] = {xm & 3u, xp & 3u, nb[1][j] & 3u, nb[2][j] & 3u, nb[3][j] & 3u, nb[4][j] & 3u};
                bool same = true, other_def = false;
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    same &= nn[k] == o;
                    other_def |= nn[k] != o && nn[k] != kBrickMixed;
                }
                if (same || !other_def) f = o;
                if (!same && !other_def) cand = kBrickCandidate;
            }
            fc[j] = f | (cand << 8);
        }
    }
    // listed bricks of this word; their modes are loaded now and land while the list slot is fetched
    uint32_t emask = 0;
    uint64_t lm[kFillP];
#pragma unroll
    for (int j = 0; j < kFillP; ++j) {
        lm[j] = 0;
        if (valid && j < nv && (fc[j] & 3u) == kBrickMixed) {
            emask |= 1u << j;
            const int b = b0 + j, cb = bx0 + j + by * cg.nbx + (bz / kCZ) * cplane;
            lm[j] = ((uint8_t)(oc >> (8 * j)) == kBrickMixed) ? modes[b] : cmodes[cb];
        }
    }
    // block-aggregated list append: the wave's exclusive prefix of the per-thread counts (<= 8)
    // from the bit planes of the counts, one atomic per block
    const uint32_t cnt = (uint32_t)__popc(emask);
    uint32_t excl = 0, wtot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t bits = __ballot((cnt >> k) & 1u);
        excl += (uint32_t)__popcll(bits & ((1ull << lane) - 1ull)) << k;
        wtot += (uint32_t)__popcll(bits) << k;
    }
    if (lane == 0) wsum[w] = wtot;
    __syncthreads();
    uint32_t base = 0;
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < kFillBlock / 64; ++k) t += wsum[k];
        if (t) base = atomicAdd(count, t);
    }
    // the stores drain while the atomic is in flight
    if (valid) {
        uint64_t fv = 0, wv = 0;
#pragma unroll
        for (int j = 0; j < kFillP; ++j) {
            fv |= (uint64_t)(uint8_t)(own[j] | ((fc[j] & 3u) << 4) | (fc[j] >> 8)) << (8 * j);
            if (j < nv && (fc[j] & 3u) == kBrickNeg) wv |= (uint64_t)(sign_piece_t)~(sign_piece_t)0 << (kBX * j);
        }
        if (nv == kFillP) {
            __builtin_memcpy(fill + b0, &fv, kFillP);
        } else {
            for (int j = 0; j < nv; ++j) fill[b0 + j] = (uint8_t)(fv >> (8 * j));
        }
        if (sign_fill) {
            uint64_t* words = reinterpret_cast<uint64_t*>(signs);
            const int y1 = min(by * kBY + kBY, g.n), z1 = min(bz * kBZ + kBZ, layers);
            for (int zz = bz * kBZ; zz < z1; ++zz)
                for (int yy = by * kBY; yy < y1; ++yy) words[((size_t)zz * g.n + yy) * rw + c] = wv;
        }
    }
    if (threadIdx.x == 0) {
        for (int k = 0; k < kFillBlock / 64; ++k) {
            wbase[k] = base;
            base += wsum[k];
        }
    }
    __syncthreads();
    if (emask) {
        uint32_t i = wbase[w] + excl;
#pragma unroll
        for (int j = 0; j < kFillP; ++j) {
            if (!((emask >> j) & 1u)) continue;
            // mixed-class bricks claim their candidate neighbours after their own evaluation
            list[i] = (uint32_t)(b0 + j) | ((own[j] & 3u) == kBrickMixed && sign_fill ? kListCheck : 0u);
            lmodes[i] = lm[j];
            ++i;
        }
        // MC (unit, chunk) pairs whose cells have a corner in a listed brick of this word: cell
        // rows sy in [by kBY - 1, by kBY + kBY - 1], cell layers lz in [bz kBZ - 1, bz kBZ + kBZ - 1],
        // chunk c (cells 64 c ... 64 c + 63 by their low corner) and, when the word's first brick is
        // listed, chunk c - 1 (its last cell reaches sample 64 c)
        const int m = g.m, cl = g.cz1 - g.cz0, nch = n_chunks(g);
        const int sy0 = max(by * kBY - 1, 0), sy1 = min(by * kBY + kBY - 1, m - 1);
        const bool own_chunk = c < nch, prev_chunk = c > 0 && (emask & 1u) && c - 1 < nch;
        for (int lz = max(bz * kBZ - 1, 0); lz <= min(bz * kBZ + kBZ - 1, cl - 1); ++lz)
            for (int u = (lz * m + sy0) / kUnitRows; u <= (lz * m + sy1) / kUnitRows; ++u) {
                if (own_chunk) umark[(size_t)u * nch + c] = mark_id;
                if (prev_chunk) umark[(size_t)u * nch + c - 1] = mark_id;
            }
    }
}
// one thread per sign word of every brick row
static unsigned fill_grid(const GridDesc& g) {
    const BrickGrid bg = brick_grid(g);
    return (unsigned)(((int64_t)bg.nby * bg.nbz * sign_row_words(g) + kFillBlock - 1) / kFillBlock);
}
__global__ __launch_bounds__(kFillBlock) void k_brick_fill(GridDesc g, BrickGrid bg, BrickGrid cg,
                                                           const uint8_t* __restrict__ ccls,
                                                           const uint64_t* __restrict__ cmodes,
                                                           const uint8_t* __restrict__ cls,
                                                           const uint64_t* __restrict__ modes, int sign_fill,
                                                           uint8_t* __restrict__ fill, uint32_t* __restrict__ list,
                                                           uint64_t* __restrict__ lmodes, uint32_t* __restrict__ count,
                                                           sign_piece_t* __restrict__ signs,
                                                           uint32_t* __restrict__ ccount_reset,
                                                           uint32_t* __restrict__ umark, uint32_t mark_id) {
    brick_fill_body(g, bg, cg, ccls, cmodes, cls, modes, sign_fill, fill, list, lmodes, count, signs, ccount_reset,
                    umark, mark_id);
}

// ---- merged launches of an object stream (ObjArgs, kernels.hpp): block row y = object y ----------
template <int D>
__global__ __launch_bounds__(256) void k_coarse_modes_b(const ObjArgs* __restrict__ objs, const float* __restrict__ tab,
                                                        float2 tab_range, GridDesc g, BrickGrid cg) {
    const ObjArgs& o = objs[blockIdx.y];
    coarse_modes_body(InterpIv<D, ProgC>{prog_const(o.prog), tab, tab_range}, g, cg, o.cmodes, o.ccls, o.clist, o.counters);
}
template <int D>
__global__ __launch_bounds__(256) void k_brick_refine_b(const ObjArgs* __restrict__ objs, int n, const float* __restrict__ tab,
                                                        float2 tab_range, GridDesc g, BrickGrid bg, BrickGrid cg) {
    __shared__ uint32_t s_pre[kMaxBatchObjects + 4];
    constexpr uint32_t kItems = kCZ * kRefineSplit;   // items per listed coarse box
    const uint32_t total = batch_prefix(objs, n, kCoarseListWord, kItems, (uint32_t)cg.n_bricks, s_pre, 64u);
    // whole waves iterate (a brick's layer lanes shuffle together); object ranges are padded to
    // whole waves, so a wave's object, program and starting modes are uniform (WaveModes): the
    // interval interpreter's instruction fetch is scalar and its skips do not diverge
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~63u); i0 < total; i0 += gridDim.x * 256) {
        const int k = __builtin_amdgcn_readfirstlane(batch_object_of(s_pre, n, i0));
        const ObjArgs& o = objs[k];
        const uint32_t i = i0 + (threadIdx.x & 63u) - s_pre[k];
        const bool live = i < min(o.counters[kCoarseListWord], (uint32_t)cg.n_bricks) * kItems;
        brick_refine_item<InterpIv<D, ProgC>, true>(InterpIv<D, ProgC>{prog_const(o.prog), tab, tab_range}, g, bg, cg,
                                                    o.cmodes, o.clist, o.modes, o.cls, live ? i : 0u, live);
    }
}
__global__ __launch_bounds__(kFillBlock) void k_brick_fill_b(const ObjArgs* __restrict__ objs, GridDesc g, BrickGrid bg,
                                                             BrickGrid cg, int sign_fill) {
    const ObjArgs& o = objs[blockIdx.y];
    brick_fill_body(g, bg, cg, o.ccls, o.cmodes, o.cls, o.modes, sign_fill, o.fill, o.blist, o.lmodes,
                    o.counters + kBrickListWord, static_cast<sign_piece_t*>(o.signs), o.counters + kCoarseListWord,
                    o.umark, o.mark_id);
}
// W: the occupancy request (four waves per SIMD at stack depth 9: 128 VGPRs and 28 B of scratch,
// 0.531 -> 0.507 ms per config-5 pass against three waves without scratch; five spill far more: 1.0 ms)
template <int D, bool Pair, int W, int V = D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void k_eval_field_pruned_b(
    const ObjArgs* __restrict__ objs, int n, const float* __restrict__ tab, GridDesc g, BrickGrid bg) {
    __shared__ uint32_t s_pre[kMaxBatchObjects + 4];
    const uint32_t total = batch_prefix(objs, n, kBrickListWord, 1u, (uint32_t)bg.n_bricks, s_pre);
    const uint32_t stride = gridDim.x * 4;
    for (uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); i < total; i += stride) {
        const int k = __builtin_amdgcn_readfirstlane(batch_object_of(s_pre, n, i));
        const ObjArgs& o = objs[k];
        const uint32_t li = i - s_pre[k];
        // Pair: both layers in one pass of the interpreter (InterpEval2; twice the node stacks in VGPRs)
        const ClaimCtx cc{o.fill, o.ccls, o.modes, o.cmodes, bg.nbx, bg.nbx * bg.nby};
        eval_listed_deferred<InterpEval2<D, ProgC, V>, Pair>(InterpEval2<D, ProgC, V>{{prog_const(o.prog), tab}}, g, bg, cc,
                                                          o.blist[li], o.lmodes[li], o.field,
                                                          static_cast<sign_piece_t*>(o.signs), o.claimed,
                                                          o.counters + kClaimedWord, (uint32_t)bg.n_bricks);
    }
}
// the claimed candidates of every object (eval_listed_deferred), one wave per candidate: values
// only -- their sign pieces are constant and already written -- with the candidate's own modes
template <int D, bool Pair, int V = D>
__global__ __launch_bounds__(256) void k_eval_claimed_b(const ObjArgs* __restrict__ objs, int n,
                                                        const float* __restrict__ tab, GridDesc g, BrickGrid bg) {
    __shared__ uint32_t s_pre[kMaxBatchObjects + 4];
    const uint32_t total = batch_prefix(objs, n, kClaimedWord, 1u, (uint32_t)bg.n_bricks, s_pre);
    const uint32_t stride = gridDim.x * 4;
    for (uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); i < total; i += stride) {
        const int k = __builtin_amdgcn_readfirstlane(batch_object_of(s_pre, n, i));
        const ObjArgs& o = objs[k];
        const int cur = (int)__builtin_amdgcn_readfirstlane(o.claimed[i - s_pre[k]]);
        int cx, cy, cz;
        brick_of(cur, bg, cx, cy, cz);
        const int cb = cx + cy * bg.nbx + (cz / kCZ) * bg.nbx * bg.nby;   // the coarse box (same x, y grid)
        const uint64_t m = o.ccls[cb] == kBrickMixed ? o.modes[cur] : o.cmodes[cb];
        uint64_t neg[kBZ], valid;
        eval_one_brick<InterpEval2<D, ProgC, V>, Pair>(InterpEval2<D, ProgC, V>{{prog_const(o.prog), tab}}, g, bg, cur, m, o.field,
                                                    static_cast<sign_piece_t*>(o.signs), false, neg, valid);
    }
}

// sign bitmap of a fully evaluated field (unpruned path), in storage order: one wave per brick
// layer reads its 256 contiguous bytes (the PMC fetch calibration, tools/pmc_traffic.py) and writes
// the layer's kBY sign pieces, as the pruned eval does
__global__ __launch_bounds__(256) void k_signs_from_field(GridDesc g, BrickGrid bg, const float* __restrict__ field,
                                                          sign_piece_t* __restrict__ signs) {
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= (int64_t)bg.n_bricks * kBZ) return;
    int bx, by, bz;
    brick_of((int)(w / kBZ), bg, bx, by, bz);
    const int layer = bz * kBZ + (int)(w % kBZ);
    const int sx = bx * kBX + lane % kBX;
    const bool neg = sx < g.n && field[w * (kBX * kBY) + lane] < 0.f;
    const uint64_t bits = __ballot(neg);
    const int row_pieces = (64 / kBX) * sign_row_words(g);
    if (lane < kBY && layer < g.fz1 - g.fz0) {
        const int yy = by * kBY + lane;
        if (yy < g.n) signs[((size_t)layer * g.n + yy) * row_pieces + bx] = (sign_piece_t)(bits >> (kBX * lane));
    }
}

template <int D>
__global__ __launch_bounds__(256) void k_eval_points(const Program* __restrict__ prog, const float* __restrict__ tab,
                                                     const float* __restrict__ xyz, int64_t n, float* __restrict__ f,
                                                     float* __restrict__ grad) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (grad) {
        V3 g;
        const float v = eval_fg<D>(prog, tab, x, y, z, g);
        if (f) f[i] = v;
        grad[3 * i] = g.x; grad[3 * i + 1] = g.y; grad[3 * i + 2] = g.z;
    } else {
        f[i] = eval_f<D>(prog, tab, x, y, z);
    }
}

// Stack capacity actually instantiated.  Below 12 slots LLVM lowers the uniform-index stack
// accesses to v_cndmask select chains (8 compares + 8 selects per access); from 12 slots on it
// uses VGPR index mode (s_set_gpr_idx_on + one v_mov), measured 1.7x faster on the config-4 tree.
// IMPLISOLID_EVAL_DEPTH overrides the floor (experiments).
static int eval_depth(int depth) {
    static int floor_d = [] {
        const char* s = std::getenv("IMPLISOLID_EVAL_DEPTH");
        return s ? std::atoi(s) : 12;
    }();
    return depth > floor_d ? depth : floor_d;
}

void launch_eval_field(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g, float* d_field,
                       hipStream_t s) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    const unsigned grid = (unsigned)(((int64_t)bg.n_bricks * kBZ + 3) / 4);   // 4 brick layers per block
    depth = eval_depth(depth);
    if (depth <= 4) k_eval_field<4><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_field);
    else if (depth <= 8) k_eval_field<8><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_field);
    else if (depth <= 12) k_eval_field<12><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_field);
    else k_eval_field<16><<<grid, 256, 0, s>>>(d_prog, d_rabbit, g, bg, d_field);
}

BrickGrid brick_grid(const GridDesc& g) {
    BrickGrid bg;
    bg.nbx = (g.n + kBX - 1) / kBX;
    bg.nby = (g.n + kBY - 1) / kBY;
    bg.nbz = (g.fz1 - g.fz0 + kBZ - 1) / kBZ;
    if (bg.nbz < 0) bg.nbz = 0;
    bg.n_bricks = bg.nbx * bg.nby * bg.nbz;
    return bg;
}

BrickGrid coarse_grid(const GridDesc& g) {
    BrickGrid cg = brick_grid(g);
    cg.nbz = (g.fz1 - g.fz0 + kBZ * kCZ - 1) / (kBZ * kCZ);
    if (cg.nbz < 0) cg.nbz = 0;
    cg.n_bricks = cg.nbx * cg.nby * cg.nbz;
    return cg;
}

void launch_brick_modes(const Program* d_prog, int depth, const float* d_rabbit, float2 tab_range, const GridDesc& g,
                        uint64_t* d_cmodes, uint8_t* d_ccls, uint32_t* d_clist, uint32_t* d_counters, uint64_t* d_modes,
                        uint8_t* d_cls, hipStream_t s, const JitIntervalKernels* jit, hipEvent_t after_coarse) {
    BrickGrid bg = brick_grid(g), cg = coarse_grid(g);
    if (bg.n_bricks <= 0) {
        if (after_coarse) (void)hipEventRecord(after_coarse, s);
        return;
    }
    uint32_t* d_ccount = d_counters + kCoarseListWord;
    depth = eval_depth(depth);
    const unsigned tc = (unsigned)((cg.n_bricks + 255) / 256);
    const unsigned tr = (unsigned)std::min<int64_t>(((int64_t)cg.n_bricks * kCZ * kRefineSplit + 255) / 256, 4096);
    if (jit && jit->coarse && jit->refine) {
        GridDesc gg = g;
        const float* d_mats = reinterpret_cast<const float*>(reinterpret_cast<const char*>(d_prog) + offsetof(Program, mats));
        void* ca[] = {&d_mats, &d_rabbit, &tab_range, &gg, &cg, &d_cmodes, &d_ccls, &d_clist, &d_counters};
        TreeJit::launch(jit->coarse, tc, ca, s, "impli_coarse_modes");
        if (after_coarse) (void)hipEventRecord(after_coarse, s);
        void* ra[] = {&d_mats, &d_rabbit, &tab_range, &gg, &bg, &cg, &d_cmodes, &d_clist, &d_ccount, &d_modes, &d_cls};
        TreeJit::launch(jit->refine, tr, ra, s, "impli_brick_refine");
        return;
    }
#define IMPLI_MODES(DD)                                                                                           \
    do {                                                                                                          \
        k_coarse_modes<DD><<<tc, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, cg, d_cmodes, d_ccls, d_clist,     \
                                              d_counters);                                                        \
        if (after_coarse) (void)hipEventRecord(after_coarse, s);                                              \
        k_brick_refine<DD><<<tr, 256, 0, s>>>(d_prog, d_rabbit, tab_range, g, bg, cg, d_cmodes, d_clist, d_ccount, \
                                              d_modes, d_cls);                                                    \
    } while (0)
    if (depth <= 4) IMPLI_MODES(4);
    else if (depth <= 8) IMPLI_MODES(8);
    else if (depth <= 12) IMPLI_MODES(12);
    else IMPLI_MODES(16);
#undef IMPLI_MODES
}

void launch_signs_from_field(const GridDesc& g, const float* d_field, uint64_t* d_signs, hipStream_t s) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    k_signs_from_field<<<(unsigned)(((int64_t)bg.n_bricks * kBZ + 3) / 4), 256, 0, s>>>(
        g, bg, d_field, reinterpret_cast<sign_piece_t*>(d_signs));
}

void launch_brick_fill(const GridDesc& g, const uint8_t* d_ccls, const uint64_t* d_cmodes, const uint8_t* d_cls,
                       const uint64_t* d_modes, int sign_fill, uint8_t* d_fill, uint32_t* d_list, uint64_t* d_lmodes,
                       uint32_t* d_count, void* d_signs, uint32_t* d_umark, uint32_t mark_id, hipStream_t s) {
    const BrickGrid bg = brick_grid(g), cg = coarse_grid(g);
    if (bg.n_bricks <= 0) return;
    k_brick_fill<<<fill_grid(g), kFillBlock, 0, s>>>(g, bg, cg, d_ccls, d_cmodes, d_cls, d_modes, sign_fill, d_fill, d_list,
                                                   d_lmodes, d_count, static_cast<sign_piece_t*>(d_signs),
                                                   d_count - kBrickListWord + kCoarseListWord, d_umark, mark_id);
}

unsigned eval_bricks_grid(const GridDesc& g) {   // blocks of kEvalBlock lanes, one brick per wave
    const int nb = brick_grid(g).n_bricks;
    const unsigned wpb = kEvalBlock / 64, cap = 16384u / wpb;
    const unsigned want = (unsigned)((nb + wpb - 1) / wpb);
    return want < cap ? (want ? want : 1u) : cap;   // grid-stride over the list
}

void launch_eval_bricks_interp(const Program* d_prog, int depth, const float* d_rabbit, const GridDesc& g,
                               const uint64_t* d_modes, const uint32_t* d_list, const uint32_t* d_count,
                               float* d_field, void* d_signs, const ClaimCtx& cc, hipStream_t s) {
    const BrickGrid bg = brick_grid(g);
    if (bg.n_bricks <= 0) return;
    depth = eval_depth(depth);
    const unsigned eb = eval_bricks_grid(g);
#define IMPLI_EVAL_PRUNED(DD)                                                                                      \
    do {                                                                                                           \
        if (interp_pair())                                                                                         \
            k_eval_field_pruned<DD, true><<<eb, kEvalBlock, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_list,      \
                                                                    d_count, d_field, d_signs, cc);                \
        else                                                                                                       \
            k_eval_field_pruned<DD, false><<<eb, kEvalBlock, 0, s>>>(d_prog, d_rabbit, g, bg, d_modes, d_list,     \
                                                                     d_count, d_field, d_signs, cc);               \
    } while (0)
    if (depth <= 4) IMPLI_EVAL_PRUNED(4);
    else if (depth <= 8) IMPLI_EVAL_PRUNED(8);
    else if (depth <= 12) IMPLI_EVAL_PRUNED(12);
    else IMPLI_EVAL_PRUNED(16);
#undef IMPLI_EVAL_PRUNED
}

// flat merged kernels (refine, eval): a fixed grid over all objects' items
// (eval grid 2048 blocks: 0.531 ms per config-5 pass against 0.546 at 4096, 0.550 at 1536 and 0.537
// at 3072; the claimed pass 1024: 0.529 against 0.532 at 2048 and 0.537 at 4096 -- profiles/r04ap_*,
// r04aq_*, r04ar_*)
constexpr unsigned kBatchRefineBlocks = 2048, kBatchEvalBlocks = 2048, kBatchClaimedBlocks = 1024;

// value stacks of their own capacity for the shallow class (IMPLISOLID_BATCH_VSTACK=0: the point
// stacks' capacity, as before round 5)
static bool batch_vstack() {
    static const bool on = [] {
        const char* v = std::getenv("IMPLISOLID_BATCH_VSTACK");
        return !(v && std::atoi(v) == 0);
    }();
    return on;
}

void launch_batch_eval(const ObjArgs* d_objs, int n, int depth, int vdepth, const float* d_rabbit, float2 tab_range,
                       const GridDesc& g, int sign_fill, hipStream_t s) {
    const BrickGrid bg = brick_grid(g), cg = coarse_grid(g);
    if (bg.n_bricks <= 0 || n <= 0) return;
    if (n > kMaxBatchObjects) throw std::runtime_error("merged object stream: more than 1024 objects per launch");
    const dim3 gc((unsigned)((cg.n_bricks + 255) / 256), (unsigned)n);
    const dim3 gf(fill_grid(g), (unsigned)n);
#define IMPLI_BATCH_EVAL(DD, WW, VV)                                                                               \
    do {                                                                                                           \
        k_coarse_modes_b<DD><<<gc, 256, 0, s>>>(d_objs, d_rabbit, tab_range, g, cg);                               \
        k_brick_refine_b<DD><<<kBatchRefineBlocks, 256, 0, s>>>(d_objs, n, d_rabbit, tab_range, g, bg, cg);         \
        k_brick_fill_b<<<gf, kFillBlock, 0, s>>>(d_objs, g, bg, cg, sign_fill);                                    \
        if (interp_pair()) {                                                                                       \
            k_eval_field_pruned_b<DD, true, WW, VV><<<kBatchEvalBlocks, 256, 0, s>>>(d_objs, n, d_rabbit, g, bg);  \
            k_eval_claimed_b<DD, true, VV><<<kBatchClaimedBlocks, 256, 0, s>>>(d_objs, n, d_rabbit, g, bg);        \
        } else {                                                                                                   \
            k_eval_field_pruned_b<DD, false, WW, VV><<<kBatchEvalBlocks, 256, 0, s>>>(d_objs, n, d_rabbit, g, bg); \
            k_eval_claimed_b<DD, false, VV><<<kBatchClaimedBlocks, 256, 0, s>>>(d_objs, n, d_rabbit, g, bg);       \
        }                                                                                                          \
    } while (0)
    // stack capacity: kBatchShallowDepth slots for shallow objects (kernels.hpp), else the
    // interpreter's floor (12: VGPR index mode) or 16; the shallow class's value stacks by their own
    // depth (6 covers every config-5 object of that class)
    // the value stacks (private arrays of V slots) must hold the deepest program's values: vdepth is
    // the unpruned run's high-water mark (Engine::vdepth, program_vdepth), and a pruned run skips an
    // operand subtree together with its CSG node's pop, so it never holds more (checked
    // here rather than assumed -- a future n-ary node would otherwise overflow them silently)
    auto need = [&](int V, int D) {
        if (vdepth > V || depth > D)
            throw std::runtime_error("merged eval: a program's stacks exceed the kernel's (" + std::to_string(vdepth) + " values, depth " +
                                     std::to_string(depth) + ")");
    };
    if (depth <= kBatchShallowDepth) {
        if (batch_vstack() && vdepth <= 6) { need(6, kBatchShallowDepth); IMPLI_BATCH_EVAL(kBatchShallowDepth, 4, 6); }
        else { need(kBatchShallowDepth, kBatchShallowDepth); IMPLI_BATCH_EVAL(kBatchShallowDepth, 4, kBatchShallowDepth); }
    } else if (depth <= 12) {
        need(12, 12);
        IMPLI_BATCH_EVAL(12, 2, 12);
    } else {
        need(16, 16);
        IMPLI_BATCH_EVAL(16, 1, 16);
    }
#undef IMPLI_BATCH_EVAL
}

void launch_eval_points(const Program* d_prog, int depth, const float* d_rabbit, const float* d_xyz, int64_t n,
                        float* d_f, float* d_grad, hipStream_t s) {
    if (n <= 0) return;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    depth = eval_depth(depth);
    if (depth <= 4) k_eval_points<4><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
    else if (depth <= 8) k_eval_points<8><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
    else if (depth <= 12) k_eval_points<12><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
    else k_eval_points<16><<<blocks, 256, 0, s>>>(d_prog, d_rabbit, d_xyz, n, d_f, d_grad);
}

// diagnostics: the screw family's restated glibc float functions on n operands (which: 0 sinf(a),
// 1 atanf(a), 2 atan2f(a, b)) -- the GPU test compares them with the oracle's, pattern by pattern
__global__ __launch_bounds__(256) void k_libm_probe(int which, const float* __restrict__ a, const float* __restrict__ b,
                                                     int64_t n, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = which == 0 ? dev::glibc_sinf(a[i]) : which == 1 ? dev::glibc_atanf(a[i]) : dev::glibc_atan2f(a[i], b[i]);
}

void launch_libm_probe(int which, const float* d_a, const float* d_b, int64_t n, float* d_out, hipStream_t s) {
    if (n <= 0) return;
    k_libm_probe<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(which, d_a, d_b, n, d_out);
}

// diagnostics: the restated glibc double cos (the screw gradient's) on n arguments
__global__ __launch_bounds__(256) void k_cos_probe(const double* __restrict__ a, int64_t n, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = dev::glibc_cos(a[i]);
}

void launch_cos_probe(const double* d_a, int64_t n, double* d_out, hipStream_t s) {
    if (n <= 0) return;
    k_cos_probe<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(d_a, n, d_out);
}

}  // namespace impli
