#!/usr/bin/env python3
"""HBM traffic per eval+MC step from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, one pass each).

    python tools/pmc_traffic.py --fetch D1 --write D2 [--cal-fetch D3 --cal-write D4] --R 512 \\
        > profiles/traffic_r01.json

D1/D2: `bench.py --skip-256 --no-cpu-baseline` (default pruning) under `rocprofv3 --pmc FETCH_SIZE`
and `--pmc WRITE_SIZE`.  D3/D4: the same with `--prune 0`, whose dense kernels move a known byte
count (k_eval_field stores exactly 4 B per stored sample, k_signs_from_field loads exactly that
field): they calibrate the counters for this code's 4-byte-per-lane accesses, a width
MI355X_MICROARCH.md (HBM) lists as uncalibrated.  Without them the guide's rule is applied
(FETCH_SIZE doubled, WRITE_SIZE as is).  Counters are in KiB as rocprofv3 reports them.

Only the launches of the R-sized config-4 grid are kept: the bench times that grid first, and
each kernel's launches are averaged over those dispatches.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {   # substring of the demangled name -> engine phase (Engine::kernel_times names)
    "impli_coarse_modes": "brick_modes", "impli_brick_refine": "brick_modes", "k_coarse_modes": "brick_modes",
    "k_brick_refine": "brick_modes", "k_brick_fill": "brick_modes",
    "impli_eval_bricks": "eval_field", "k_eval_field_pruned": "eval_field", "k_eval_field": "eval_field",
    "k_signs_from_field": "eval_field",
    "k_mc_count": "mc_count", "k_scan_groups": "mc_scan", "k_unit_flatten": "mc_scan", "k_unit_scan": "mc_scan",
    "k_mc_verts": "mc_verts", "k_mc_cells": "mc_verts", "k_mc_faces": "mc_faces",
}


def short(name):
    base = name.replace("(anonymous namespace)", "").split("(")[0].split("<")[0]
    for k in sorted(KERNELS, key=len, reverse=True):
        if base.endswith(k):
            return k
    return None


def load(d, counter):
    """kernel short name -> list of per-dispatch values (bytes/1024 as reported), dispatch order"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under " + d)
    rows = []
    for r in csv.DictReader(open(files[0])):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        if k:
            rows.append((int(r.get("Dispatch_Id", 0) or 0), k, float(r["Counter_Value"])))
    rows.sort()
    acc = collections.defaultdict(list)
    for _, k, v in rows:
        acc[k].append(v)
    return acc


def per_launch(acc, n_first):
    """mean over the first n_first dispatches of each kernel (the R-sized grid's steps)"""
    return {k: sum(v[:n_first]) / len(v[:n_first]) for k, v in acc.items() if v}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--cal-fetch")
    ap.add_argument("--cal-write")
    ap.add_argument("--R", type=int, default=512)
    ap.add_argument("--launches", type=int, default=4, help="dispatches per kernel of the R grid to average")
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--lib", help="the profiled library: its SHA-256 is recorded, so bench.py can tell whether the "
                                  "traffic figures describe the library it runs")
    a = ap.parse_args()
    kib = 1024.0
    fr, fw = 2.0, 1.0   # MI355X_MICROARCH.md: FETCH_SIZE counts half of wide streaming reads
    cal = None
    if a.cal_fetch and a.cal_write:
        n = a.R + 3
        known = 4.0 * n * n * n   # stored samples x 4 B (field of a whole-grid slab, n layers)
        cf = per_launch(load(a.cal_fetch, "FETCH_SIZE"), a.launches)
        cw = per_launch(load(a.cal_write, "WRITE_SIZE"), a.launches)
        fr = known / (kib * cf["k_signs_from_field"])
        fw = known / (kib * cw["k_eval_field"])
        cal = {"known_bytes": known, "fetch_factor": round(fr, 4), "write_factor": round(fw, 4),
               "how": "unpruned path: k_signs_from_field loads, k_eval_field stores exactly 4 B per stored sample"}
    fetch = per_launch(load(a.fetch, "FETCH_SIZE"), a.launches)
    write = per_launch(load(a.write, "WRITE_SIZE"), a.launches)
    # the tree JIT compiles in the background while the first warmup steps run the interpreter
    # kernels: when a JIT kernel ran, its interpreter twin's (warmup-only) dispatches are not part
    # of the timed step and would double-count the phase
    twins = {"impli_coarse_modes": "k_coarse_modes", "impli_brick_refine": "k_brick_refine",
             "impli_eval_bricks": "k_eval_field_pruned"}
    dropped = []
    for jk, ik in twins.items():
        if (jk in fetch or jk in write) and (ik in fetch or ik in write):
            fetch.pop(ik, None)
            write.pop(ik, None)
            dropped.append(ik)
    kern = {}
    for k in sorted(set(fetch) | set(write)):
        kern[k] = {"phase": KERNELS[k], "fetch_bytes": round(fr * kib * fetch.get(k, 0.0)),
                   "write_bytes": round(fw * kib * write.get(k, 0.0))}
        kern[k]["bytes"] = kern[k]["fetch_bytes"] + kern[k]["write_bytes"]
    phases = collections.defaultdict(float)
    for k, v in kern.items():
        phases[v["phase"]] += v["bytes"]
    out = {"workload_R": a.R, "tree_seed": a.seed, "pipeline_bytes": round(sum(phases.values())),
           "phase_bytes": {k: round(v) for k, v in sorted(phases.items())}, "kernels": kern,
           "calibration": cal or "guide rule: FETCH_SIZE x2, WRITE_SIZE x1",
           "dropped_warmup_interpreter_kernels": dropped,
           "note": __doc__.strip().splitlines()[0]}
    if a.lib:
        import hashlib
        out["lib_sha256"] = hashlib.sha256(open(a.lib, "rb").read()).hexdigest()
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
