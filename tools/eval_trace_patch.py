#!/usr/bin/env python3
"""Diagnostics variant (tools/build_variant.sh evaltrace ... with PATCH_PY=tools/eval_trace_patch.py):
the eval kernel records per-wave timestamps (s_memrealtime, 100 MHz) -- wave start, list entry
loaded, first brick evaluated, claims decided, wave end -- and its brick / claimed counts into a
buffer that Engine::eval_field dumps to $IMPLISOLID_EVAL_TRACE after the launch.  Never part of
the library; tools/eval_trace.py reads the dump.  Run from the variant copy's implisolid_amd/."""
import re

p = "csrc/grid.hpp"
s = open(p).read()
s = s.replace("    int cnbx, cplane;         // coarse grid: boxes per row, per layer\n};",
              "    int cnbx, cplane;         // coarse grid: boxes per row, per layer\n    uint64_t* trace;          // diagnostics: per-wave timestamps\n};")
open(p, "w").write(s)

p = "csrc/eval_bricks.hpp"
s = open(p).read()
old = """    sign_piece_t* signs = static_cast<sign_piece_t*>(signs_raw);
    const uint32_t nb = *count;"""
new = """    sign_piece_t* signs = static_cast<sign_piece_t*>(signs_raw);
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint32_t nb = *count;"""
assert old in s
s = s.replace(old, new)
old = """    for (; i < nb; i += stride) {
        const uint32_t e = __builtin_amdgcn_readfirstlane(b_next);
        const uint64_t m64 = m_next;
        if (i + stride < nb) {
            b_next = list[i + stride];
            m_next = modes[i + stride];
        }
        eval_listed<Eval, Pair>(ev, g, bg, cc, e, m64, field, signs);
    }
}"""
new = """    const uint32_t wave_id = blockIdx.x * wpb + (threadIdx.x >> 6);
    uint64_t t_list = 0, t_first = 0, t_claim = 0;
    uint32_t n_done = 0, n_claimed = 0;
    for (; i < nb; i += stride) {
        const uint32_t e = __builtin_amdgcn_readfirstlane(b_next);
        if (!n_done) t_list = __builtin_amdgcn_s_memrealtime();
        const uint64_t m64 = m_next;
        if (i + stride < nb) {
            b_next = list[i + stride];
            m_next = modes[i + stride];
        }
        n_claimed += eval_listed_traced<Eval, Pair>(ev, g, bg, cc, e, m64, field, signs, n_done == 0 ? &t_first : nullptr,
                                                    n_done == 0 ? &t_claim : nullptr);
        ++n_done;
    }
    if (cc.trace && (threadIdx.x & 63) == 0) {
        uint64_t* r = cc.trace + 8 * (uint64_t)wave_id;
        r[0] = t_start; r[1] = t_list; r[2] = t_first; r[3] = t_claim; r[4] = __builtin_amdgcn_s_memrealtime();
        r[5] = n_done; r[6] = n_claimed; r[7] = 1;
    }
}"""
assert old in s
s = s.replace(old, new)
# a traced copy of eval_listed: timestamps after the first brick and after its claims; returns claims
old = "template <class Eval, bool Pair = IMPLI_EVAL_PAIR != 0>\n__device__ __forceinline__ void eval_bricks_body("
traced = '''template <class Eval, bool Pair = IMPLI_EVAL_PAIR != 0>
__device__ __forceinline__ uint32_t eval_listed_traced(const Eval& ev, const GridDesc& g, const BrickGrid& bg, const ClaimCtx& cc,
                                                       uint32_t entry, uint64_t m64, float* __restrict__ field,
                                                       sign_piece_t* __restrict__ signs, uint64_t* t_first, uint64_t* t_claim) {
    const int b = (int)(entry & ~kListCheck);
    const bool check = (entry & kListCheck) && cc.fill;
    int cur = b;
    uint64_t mcur = m64;
    uint32_t claimed = 0, nclaimed = 0;
    for (bool first = true;; first = false) {
        uint64_t neg[kBZ], valid;
        eval_one_brick<Eval, Pair>(ev, g, bg, cur, mcur, field, signs, first, neg, valid);
        if (first && t_first) *t_first = __builtin_amdgcn_s_memrealtime();
        if (first && check) claimed = claim_neighbours(g, bg, cc, b, neg, valid);
        if (first && t_claim) *t_claim = __builtin_amdgcn_s_memrealtime();
        if (first) nclaimed = (uint32_t)__popc(claimed);
        if (!claimed) break;
        const int d = __builtin_ctz(claimed);
        claimed &= claimed - 1u;
        const int ax = d >> 1, up = d & 1;
        const int step = ax == 0 ? 1 : ax == 1 ? bg.nbx : bg.nbx * bg.nby;
        cur = up ? b + step : b - step;
        int cx, cy, cz;
        brick_of(cur, bg, cx, cy, cz);
        const int cb = cx + cy * cc.cnbx + (cz / kCZ) * cc.cplane;
        mcur = cc.ccls[cb] == kBrickMixed ? cc.bmodes[cur] : cc.cmodes[cb];
    }
    return nclaimed;
}

'''
assert old in s
s = s.replace(old, traced + old, 1)
open(p, "w").write(s)

p = "csrc/engine.hip"
s = open(p).read()
old = """        const ClaimCtx cc{level >= 2 ? fill_.as<uint8_t>() : nullptr, ccls_.as<uint8_t>(), modes_.as<uint64_t>(),
                          cmodes_.as<uint64_t>(), bg.nbx, bg.nbx * bg.nby};"""
new = """        static DevBuf trace_buf;
        static const char* trace_path = std::getenv("IMPLISOLID_EVAL_TRACE");
        const size_t trace_bytes = (size_t)65536 * 8 * sizeof(uint64_t);
        if (trace_path && !trace_buf.p) {
            trace_buf.reserve(trace_bytes);
        }
        if (trace_path) IMPLI_HIP(hipMemsetAsync(trace_buf.p, 0, trace_bytes, s));
        const ClaimCtx cc{level >= 2 ? fill_.as<uint8_t>() : nullptr, ccls_.as<uint8_t>(), modes_.as<uint64_t>(),
                          cmodes_.as<uint64_t>(), bg.nbx, bg.nbx * bg.nby, trace_path ? trace_buf.as<uint64_t>() : nullptr};"""
assert old in s
s = s.replace(old, new)
old = """            launch_eval_bricks_interp(prog_.as<Program>(), depth_, rabbit_.as<float>(), grid_, lmodes_.as<uint64_t>(),
                                      blist_.as<uint32_t>(), d_count, field_.as<float>(), signs_.p, cc, s);
        }"""
new = """            launch_eval_bricks_interp(prog_.as<Program>(), depth_, rabbit_.as<float>(), grid_, lmodes_.as<uint64_t>(),
                                      blist_.as<uint32_t>(), d_count, field_.as<float>(), signs_.p, cc, s);
        }
        if (trace_path) {
            std::vector<uint64_t> h(trace_bytes / 8);
            IMPLI_HIP(hipStreamSynchronize(s));
            IMPLI_HIP(hipMemcpy(h.data(), trace_buf.p, trace_bytes, hipMemcpyDeviceToHost));
            if (FILE* f = std::fopen(trace_path, "wb")) { std::fwrite(h.data(), 8, h.size(), f); std::fclose(f); }
        }"""
assert old in s
s = s.replace(old, new)
if "#include <cstdio>" not in s:
    s = "#include <cstdio>\n#include <cstdlib>\n#include <vector>\n" + s
open(p, "w").write(s)

p = "csrc/eval.hip"
s = open(p).read()
s = s.replace("const ClaimCtx cc{o.fill, o.ccls, o.modes, o.cmodes, bg.nbx, bg.nbx * bg.nby};",
              "const ClaimCtx cc{o.fill, o.ccls, o.modes, o.cmodes, bg.nbx, bg.nbx * bg.nby, nullptr};")
open(p, "w").write(s)
print("patched")
