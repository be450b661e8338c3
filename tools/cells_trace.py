#!/usr/bin/env python3
"""Per-part timeline of the vertex pass (diagnostics): run with the cellstrace variant library
(tools/cells_trace_patch.py) as IMPLISOLID_LIB, config 4 at R; every vertex pass dumps its unit
parts' records {start, list entry in hand, sign words in hand, end, non-trivial cells, windows,
block} (100 MHz s_memrealtime ticks) to $IMPLISOLID_CELLS_TRACE.  Prints the phase durations, the
parts per wave and the generations of the last step.   usage: python tools/cells_trace.py [R] [steps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import numpy as np
    import torch
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    path = os.environ.setdefault("IMPLISOLID_CELLS_TRACE", "/tmp/cells_trace.bin")
    import implisolid_amd as I
    from implisolid_amd import scenes
    shape, mc = scenes.config4(R)
    s = I.Slab(shape, mc)
    sp = torch.cuda.current_stream().cuda_stream
    for k in range(steps):
        s.eval(sp); s.count(sp); s.emit(0, sp)
        if k == 3:
            I.jit_wait()
    torch.cuda.synchronize()
    d = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    d = d[d[:, 7] == 1]
    t0_, t1_, t2_, t3_, cells, wins, blk = [d[:, k].astype(np.int64) for k in range(7)]
    base = t0_.min()
    us = lambda x: x * 0.01
    ph = {"entry": t1_ - t0_, "signs": t2_ - t1_, "windows": t3_ - t2_, "part": t3_ - t0_}
    out = {"R": R, "parts": int(len(d)), "span_us": round(us(t3_.max() - base), 2),
           "phase_us": {k: {"mean": round(us(v.mean()), 2), "p50": round(us(np.median(v)), 2),
                            "p90": round(us(np.percentile(v, 90)), 2), "max": round(us(v.max()), 2)} for k, v in ph.items()},
           "cells_per_part": {"mean": round(float(cells.mean()), 1), "max": int(cells.max())},
           "windows_per_part": {str(k): int((wins == k).sum()) for k in range(0, int(wins.max()) + 1)},
           "start_us_percentiles": [round(us(np.percentile(t0_ - base, q)), 2) for q in (0, 25, 50, 75, 90, 99, 100)],
           "end_us_percentiles": [round(us(np.percentile(t3_ - base, q)), 2) for q in (0, 25, 50, 75, 90, 99, 100)],
           "parts_started_after_first_end": int((t0_ > t3_.min()).sum())}
    # per-window cost: parts with w windows, mean windows phase
    out["windows_phase_by_count"] = {str(w): round(us(ph["windows"][wins == w].mean()), 2)
                                     for w in range(1, min(8, int(wins.max())) + 1) if (wins == w).any()}
    # waves / parts in flight per microsecond of the kernel's span, and how many had started
    bins = np.arange(0, int(us(t3_.max() - t0_.min())) + 2)
    rs, re_ = us(t0_ - t0_.min()), us(t3_ - t0_.min())
    out["in_flight_per_us"] = [int(((rs <= b + 0.5) & (re_ > b + 0.5)).sum()) for b in bins]
    out["started_by_us"] = [int((rs <= b + 0.5).sum()) for b in bins]
    print(json.dumps(out))
    s.close()


if __name__ == "__main__":
    main()
