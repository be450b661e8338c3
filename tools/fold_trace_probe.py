#!/usr/bin/env python3
"""The device fold walk's step trace (IMPLISOLID_FOLD_TRACE=1 prints it) on synthetic edge-length
terms: python tools/fold_trace_probe.py [n]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import implisolid_amd as I
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 340000
    rng = np.random.default_rng(1)
    e = (0.0144 * (0.5 + rng.uniform(size=n))).astype(np.float32)
    est = np.cumsum(e.astype(np.float64))
    cross = [int(np.searchsorted(est, 2.0 ** k)) for k in range(-8, 20) if est[-1] > 2.0 ** k > est[0]]
    print("estimate crosses powers of two at terms", cross, "chunks", [c // 256 for c in cross], flush=True)
    print(I.debug_fold(e), flush=True)


if __name__ == "__main__":
    main()
