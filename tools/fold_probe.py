#!/usr/bin/env python3
"""The device edge-length fold alone (implisolid_debug_fold) on synthetic terms of several sizes,
for a kernel trace: python tools/fold_probe.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import implisolid_amd as I
    rng = np.random.default_rng(1)
    for n in (1000, 30000, 340000, 1000000):
        e = (0.0144 * (0.5 + rng.uniform(size=n))).astype(np.float32)
        for _ in range(3):
            s, tc = I.debug_fold(e)
        ref = np.add.accumulate(e, dtype=np.float32)[-1]
        print(n, "chunks", (n + 255) // 256, "from table", tc, "exact", bool(np.float32(s).view(np.uint32) == ref.view(np.uint32)), flush=True)


if __name__ == "__main__":
    main()
