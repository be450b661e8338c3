#!/usr/bin/env python3
"""The edge-length fold alone (implisolid_debug_fold) on the edge lengths of real MC meshes: config 3
on the shifted box at 256^3 and config 4 (the same tree) at 512^3, in the reference's term order
(|a-b|, |a-c|, |c-b| per face, centroids_projection.cpp:70-82).  With IMPLISOLID_FOLD_STATS=1 the
library prints the walk's step counts and cycle split; under rocprofv3 --kernel-trace the kernels'
durations.  Checks the sum bit for bit against numpy's sequential float32 accumulate.
    python tools/fold_mesh_probe.py [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def terms(v, f):
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    n = lambda d: np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
    return np.stack([n(a - b), n(a - c), n(c - b)], 1).reshape(-1)


def main():
    import implisolid_amd as I
    from implisolid_amd import scenes
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for R in (256, 512):
        shape, mc = scenes.config3_shifted(R)
        mc = dict(mc, vresampl={"iters": 0, "c": 1.0}, projection={"enabled": 0}, qem={"enabled": 0})
        v, f = I.make_geometry(shape, mc)
        e = terms(v.astype(np.float32), f)
        ref = np.add.accumulate(e, dtype=np.float32)[-1]
        for _ in range(reps):
            s, tc = I.debug_fold(e)
        print("R", R, "terms", e.size, "chunks", (e.size + 255) // 256, "from table", tc,
              "exact", bool(np.float32(s).view(np.uint32) == ref.view(np.uint32)), flush=True)


if __name__ == "__main__":
    main()
