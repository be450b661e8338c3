#!/usr/bin/env python3
"""Config 4's OB02 build at 512^3 (scenes.config3_shifted(512): MC + 3 x [resample, project, QEM]),
warm, then `reps` builds (for a kernel trace); --baked: after the hot-object bake.
usage: python tools/ob02_r512_probe.py [reps] [--baked] [--R 256]  (--R: config 3s's tree at that resolution)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import implisolid_amd as I
    from implisolid_amd import scenes
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
    R = int(sys.argv[sys.argv.index("--R") + 1]) if "--R" in sys.argv else 512
    shape, mc = scenes.config3_shifted(R)
    I.make_geometry(shape, mc)
    I.jit_wait()
    I.make_geometry(shape, mc)
    if "--baked" in sys.argv:   # a hot object: after 4 builds its modules are baked (background compile)
        for _ in range(4):
            I.make_geometry(shape, mc)
        I.jit_wait()
        I.make_geometry(shape, mc)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        I.make_geometry_views(shape, mc)
        ts.append((time.perf_counter() - t0) * 1e3)
    print("config4s R%d MC+3xOB02 build_geometry min %.3f ms median %.3f ms" % (R, min(ts), sorted(ts)[len(ts) // 2]),
          flush=True)


if __name__ == "__main__":
    main()
