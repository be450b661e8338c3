#!/usr/bin/env python3
"""The projection's search balance (diagnostics): profiled build_geometry of config 3s at 256^3 and
config 4s at 512^3 with IMPLISOLID_PROJ_STATS=1 -- per projection the evaluations per face, the
bound a wave's longest face sets (16 faces per wave) and the faces left for the late pass.
    IMPLISOLID_PROJ_STATS=1 python tools/proj_stats_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import implisolid_amd as I
    from implisolid_amd import scenes
    for R in (256, 512):
        shape, mc = scenes.config3_shifted(R)
        I.make_geometry(shape, mc)
        I.jit_wait()
        I.ob02_profile(True)
        try:
            print("R", R, flush=True)
            sys.stderr.flush()
            I.make_geometry(shape, mc)
            print(I.last_build_stats(), flush=True)
        finally:
            I.ob02_profile(False)


if __name__ == "__main__":
    main()
