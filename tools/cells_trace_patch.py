#!/usr/bin/env python3
"""Diagnostics variant (tools/build_variant.sh cellstrace ... with PATCH_PY=tools/cells_trace_patch.py):
the vertex pass (k_mc_cells) records per unit part (s_memrealtime, 100 MHz) -- part start, its
list entry in hand, its sign words in hand (after the wave scan that uses them), its windows
done (field loads used, stores issued), and its non-trivial cells and windows -- into a buffer
that Engine::emit_verts dumps to $IMPLISOLID_CELLS_TRACE.  Never part of the library;
tools/cells_trace.py reads the dump.  Run from the variant copy's implisolid_amd/."""

p = "csrc/mc_types.hpp"
s = open(p).read()
old = "    uint32_t* overflow;      // set to 1 if a capacity was exceeded\n};"
assert old in s
s = s.replace(old, "    uint32_t* overflow;      // set to 1 if a capacity was exceeded\n    uint64_t* trace;         // diagnostics\n};")
open(p, "w").write(s)

p = "csrc/mc_device.hpp"
s = open(p).read()
old = """    {
        const uint4 ent = b.ulist[e];   // {unit, vbase, fbase, abase}"""
new = """    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();
    uint64_t tr1 = 0, tr2 = 0;
    uint32_t tr_cells = 0, tr_windows = 0;
    {
        const uint4 ent = b.ulist[e];   // {unit, vbase, fbase, abase}"""
assert old in s
s = s.replace(old, new)
old = """        const int64_t u = ent.x;
        uint32_t vrun0 = ent.y, frun0 = ent.z, arun0 = ent.w;"""
new = """        const int64_t u = ent.x;
        uint32_t vrun0 = ent.y, frun0 = ent.z, arun0 = ent.w;
        asm volatile("" ::"v"(ent.x), "v"(up));
        tr1 = __builtin_amdgcn_s_memrealtime();"""
assert old in s
s = s.replace(old, new)
old = """            const uint32_t cnt = (uint32_t)__popcll((unsigned long long)k.nt);
            const uint32_t incl = wave_incl_scan<uint32_t>(cnt, lane);
            const uint32_t total = __shfl(incl, 63, 64);"""
new = """            const uint32_t cnt = (uint32_t)__popcll((unsigned long long)k.nt);
            const uint32_t incl = wave_incl_scan<uint32_t>(cnt, lane);
            const uint32_t total = __shfl(incl, 63, 64);
            asm volatile("" ::"v"(total));
            if (!tr2) tr2 = __builtin_amdgcn_s_memrealtime();
            tr_cells += total;
            tr_windows += (total + 63u) / 64u;"""
assert old in s
s = s.replace(old, new)
old = """                vrun0 += fld(tot, 0);
                frun0 += fld(tot, 1);
                arun0 += fld(tot, 2);
            }
        }
    }
}"""
new = """                vrun0 += fld(tot, 0);
                frun0 += fld(tot, 1);
                arun0 += fld(tot, 2);
            }
        }
    }
    if (b.trace && lane == 0 && e < 262144u) {
        uint64_t* r = b.trace + 8 * (uint64_t)e;
        r[0] = tr0; r[1] = tr1; r[2] = tr2; r[3] = __builtin_amdgcn_s_memrealtime();
        r[4] = tr_cells; r[5] = tr_windows; r[6] = blockIdx.x; r[7] = 1;
    }
}"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)

p = "csrc/engine.hip"
s = open(p).read()
old = """void Engine::emit_verts(hipStream_t s) {   // vertex positions and ids are slab-local: no offsets
    MCBuffers b = buffers();
    mark(6, s);
    launch_mc_verts(cases_.as<CaseInfo>(), grid_, b, s);"""
new = """void Engine::emit_verts(hipStream_t s) {   // vertex positions and ids are slab-local: no offsets
    MCBuffers b = buffers();
    static DevBuf trace_buf;
    static const char* trace_path = std::getenv("IMPLISOLID_CELLS_TRACE");
    const size_t trace_bytes = (size_t)262144 * 8 * sizeof(uint64_t);
    if (trace_path && !trace_buf.p) trace_buf.reserve(trace_bytes);
    if (trace_path) IMPLI_HIP(hipMemsetAsync(trace_buf.p, 0, trace_bytes, s));
    b.trace = trace_path ? trace_buf.as<uint64_t>() : nullptr;
    mark(6, s);
    launch_mc_verts(cases_.as<CaseInfo>(), grid_, b, s);
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
print("patched")
