#!/usr/bin/env python3
"""Config 4s (config 3's tree on the shifted box) at 512^3 in a fresh process: a never-seen
object's first build_geometry, then edits (the same tree with a root translation nudged: the tree
structure's unbaked modules, compiled by then), one profiled edit (stages drained), and the steady
state of a hot object after the JIT and bake.   usage: python tools/first_build_probe.py [R]"""
import copy
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def nudged(shape, k):
    """the shape with its root matrix's translation moved by k * 1e-7 (a different program: no
    tree module of it is compiled yet; the mesh stays essentially the same)"""
    s = copy.deepcopy(shape)
    m = s.get("matrix")
    if isinstance(m, list) and len(m) >= 12:
        m[3] = float(m[3]) + k * 1e-7
    else:
        s["matrix"] = [1, 0, 0, k * 1e-7, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]
    return s


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    import implisolid_amd as I
    from implisolid_amd import scenes
    shape, mc = scenes.config3_shifted(R)
    out = {"R": R}
    t0 = time.perf_counter()
    I.make_geometry(shape, mc)
    out["first_build_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    t0 = time.perf_counter()
    I.make_geometry(shape, mc)
    out["second_build_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    print(json.dumps(out), flush=True)
    # edits: the same tree with other matrix values.  The first nudge moves a translation off an
    # exact 0, which the modules are specialised on (xform_row, pt_xform): its modules compile in the
    # background (interpreter meanwhile); the timed edits after it reuse them
    I.jit_wait()
    I.make_geometry(nudged(shape, 5), mc)
    I.jit_wait()
    ts = []
    for k in (2, 3, 4):
        t0 = time.perf_counter()
        I.make_geometry(nudged(shape, k), mc)
        ts.append(time.perf_counter() - t0)
    out["edit_build_ms"] = round(min(ts) * 1e3, 3)
    # a never-seen shape again, profiled (stage boundaries drained)
    I.ob02_profile(True)
    t0 = time.perf_counter()
    I.make_geometry(nudged(shape, 1), mc)
    out["profiled_first_build_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    out["profiled_first_stats"] = I.last_build_stats()
    I.ob02_profile(False)
    print(json.dumps(out), flush=True)
    I.jit_wait()
    for _ in range(5):
        I.make_geometry(shape, mc)
    I.jit_wait()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        I.make_geometry(shape, mc)
        ts.append(time.perf_counter() - t0)
    out["steady_ms"] = round(min(ts) * 1e3, 3)
    I.ob02_profile(True)
    I.make_geometry(shape, mc)
    out["profiled_steady_stats"] = I.last_build_stats()
    I.ob02_profile(False)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
