#!/usr/bin/env python3
"""Per-slab kernel durations of tools/slab_probe.py from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/slab_probe.py 512 10 1,2,4,8 balanced
    python3 tools/slab_trace.py OUT/run_kernel_trace.csv 10 1,2,4,8 > summary.txt

slab_probe runs every rank's slab one after another on one GPU; each slab run dispatches a fixed
number of eval+MC steps (3 warm + 1 + `steps` direct + 3 + `steps` graph replays + 5 timed), and the
balanced cuts' interval pass (no eval kernel) before each N.  A step is the kernel sequence from a
coarse-modes kernel to the face kernel; steps are assigned to (N, rank) in that order, and per slab
the median duration of every kernel over its direct and replayed steps is printed, with the sum
(the slab's kernel critical path: the kernels run back to back on one stream).
"""
import csv
import re
import statistics
import sys

SHORT = {"impli_coarse_modes": "coarse", "k_coarse_modes": "coarse", "impli_brick_refine": "refine",
         "k_brick_refine": "refine", "k_brick_fill": "fill", "impli_eval_bricks": "eval", "k_eval_bricks": "eval",
         "k_mc_count": "count", "k_unit_scan": "scan", "k_mc_cells": "cells", "k_mc_faces": "faces"}
ORDER = ["coarse", "refine", "fill", "eval", "count", "scan", "cells", "faces"]


SHORT["k_eval_field_pruned"] = "eval"
_PAT = re.compile(r"\b(" + "|".join(sorted(SHORT, key=len, reverse=True)) + r")\b")


def short(name):
    m = _PAT.search(name)
    return SHORT[m.group(1)] if m else None


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    ns = [int(x) for x in sys.argv[3].split(",")]
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            k = short(r["Kernel_Name"])
            if k:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    # split into steps: a step starts at a coarse kernel; keep the ones that evaluate (eval kernel)
    seqs, cur = [], None
    for s, e, k in rows:
        if k == "coarse":
            cur = {}
            seqs.append(cur)
        if cur is not None:
            cur.setdefault(k, []).append((e - s) / 1000.0)
    full = [q for q in seqs if "eval" in q and "faces" in q]
    per_run = 3 + 1 + steps + 3 + steps + 5
    i = 0
    print("# tools/slab_probe.py R %d 1 step = coarse..faces; %d eval+MC steps per slab run; median us per kernel"
          % (steps, per_run))
    for n in ns:
        worst = None
        for rank in range(n):
            run = full[i:i + per_run]
            i += per_run
            if len(run) < per_run:
                print("# trace ended early at N=%d rank %d" % (n, rank))
                return
            timed = run[4:4 + steps] + run[4 + steps + 3:4 + 2 * steps + 3]
            med = {k: statistics.median(sum(x.get(k, [0.0])) for x in timed) for k in ORDER}
            tot = sum(med.values())
            worst = max(worst or 0.0, tot)
            print("N=%d rank=%d " % (n, rank) + "  ".join("%s=%.1f" % (k, med[k]) for k in ORDER) + "  sum=%.1f" % tot)
        print("N=%d slowest slab kernel sum %.1f us" % (n, worst))


if __name__ == "__main__":
    main()
