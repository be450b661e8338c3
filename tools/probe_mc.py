#!/usr/bin/env python3
"""Diagnostics of the config-4 pipeline: slab counters and brick statistics.
    python tools/probe_mc.py [R ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import implisolid_amd as I
    from implisolid_amd import scenes
    for R in [int(a) for a in sys.argv[1:]] or [512]:
        shape, mc = scenes.config4(R)
        s = I.Slab(shape, mc)
        s.eval()
        s.count()
        st = s.stats()
        s.emit()
        nv, nf, of = s.counts()
        print(json.dumps({"R": R, "verts": nv, "faces": nf, "stats": st, "bricks": s.brick_stats(), "jit": s.used_jit()}))
        s.close()


if __name__ == "__main__":
    main()
