#!/usr/bin/env python3
"""Diagnostics for the config-4 pipeline at one resolution: slab counters (active units, totals)
and brick statistics.  python tools/probe_mc.py [R]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    shape, mc = scenes.config4(R)
    s = I.Slab(shape, mc)
    s.eval(); s.count(); s.emit()
    nv, nf, of = s.counts()
    c = torch.empty(16, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ptr = I.lib().implisolid_slab_counters(s.h)
    import numpy as np
    h = np.zeros(16, np.uint32)
    torch.cuda.cudart().cudaMemcpy(h.ctypes.data, ptr, 64, 2) if hasattr(torch.cuda, "cudart") else None
    print({"R": R, "verts": nv, "faces": nf, "counters": h.tolist(), "bricks": s.brick_stats(),
           "units": (s.R + 2) ** 2 * (s.cz1 - s.cz0) // 1024})


if __name__ == "__main__":
    main()
