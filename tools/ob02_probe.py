#!/usr/bin/env python3
"""End-to-end build_geometry timings (host-resident result, PCIe included) for the OB02 configs:
config 2 (union sphere+rabbit, 128^3, MC + 3 x [resample, project, QEM]) and config 3 (twist tree,
256^3, same loop), plus MC-only and subdivision variants; then one profiled build of each (stream
drained per stage) for the per-stage breakdown and the projection's evaluation count.
usage: python tools/ob02_probe.py [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    torch.cuda.init()
    cases = [("config2 R128 MC only", scenes.union_sphere_cube(), scenes.mc_settings(128, 1.0)),
             ("config2 R128 MC+3xOB02", *scenes.config2(128)),
             ("config3 R256 MC only", scenes.config3_tree(), scenes.mc_settings(256, 1.0)),
             ("config3 R256 MC+3xOB02", *scenes.config3(256)),
             ("config3s R256 MC+3xOB02 (shifted box: live projection)", *scenes.config3_shifted(256))]
    sub = dict(scenes.config2(128)[1])
    sub["subdiv"] = {"enabled": 1}
    sub["debug"] = {"post_subdiv_noise": 0.01}
    cases.append(("config2 R128 MC+3xOB02+subdiv", scenes.union_sphere_cube(), sub))
    for name, shape, mc in cases:
        I.make_geometry(shape, mc)   # warm (buffers; the tree module compiles in the background)
        I.jit_wait()
        I.make_geometry(shape, mc)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            v, f = I.make_geometry(shape, mc)
            ts.append(time.perf_counter() - t0)
        st = I.last_build_stats()
        print("%-32s V %8d F %8d  build_geometry %.2f ms (min of %d)  cap hits %d" % (
            name, len(v), len(f), min(ts) * 1e3, reps, st["bisection_cap_hits"]), flush=True)
    I.ob02_profile(True)
    for name, shape, mc in cases:
        if "OB02" not in name:
            continue
        I.make_geometry(shape, mc)
        st = I.last_build_stats()
        print("profile %-24s %s" % (name, json.dumps(st)), flush=True)
    I.ob02_profile(False)


if __name__ == "__main__":
    main()
