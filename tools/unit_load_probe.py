#!/usr/bin/env python3
"""Distribution of non-trivial cells per MC unit (kUnitRows rows) for config 4: the vertex-pass
load balance.  usage: python tools/unit_load_probe.py [R]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    torch.cuda.init()
    shape, mc = scenes.config4(R)
    s = I.Slab(shape, mc)
    s.eval()
    sg = s.read_signs().astype(bool)          # n*n*layers, x fastest
    n = R + 3
    sg = sg.reshape(-1, n, n)                 # [layer, y, x]
    c = sg[:-1, :-1, :-1]
    allv = c & sg[:-1, :-1, 1:] & sg[:-1, 1:, :-1] & sg[:-1, 1:, 1:] & sg[1:, :-1, :-1] & sg[1:, :-1, 1:] & sg[1:, 1:, :-1] & sg[1:, 1:, 1:]
    anyv = c | sg[:-1, :-1, 1:] | sg[:-1, 1:, :-1] | sg[:-1, 1:, 1:] | sg[1:, :-1, :-1] | sg[1:, :-1, 1:] | sg[1:, 1:, :-1] | sg[1:, 1:, 1:]
    nt = anyv & ~allv                         # [cell z, cell y, cell x]
    per_row = nt.sum(axis=2).reshape(-1)
    per_unit = np.add.reduceat(per_row, np.arange(0, per_row.size, 4))
    ne = per_unit[per_unit > 0]
    print("cells", int(nt.sum()), "units", per_unit.size, "non-empty", ne.size)
    print("per non-empty unit: mean %.1f  p50 %d  p90 %d  p99 %d  max %d" % (
        ne.mean(), np.percentile(ne, 50), np.percentile(ne, 90), np.percentile(ne, 99), ne.max()))
    print("units > 256 cells:", int((ne > 256).sum()), " cells in them:", int(ne[ne > 256].sum()))
    s.close()


if __name__ == "__main__":
    main()
