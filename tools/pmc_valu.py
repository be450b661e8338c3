#!/usr/bin/env python3
"""VALU utilisation and wave-state breakdown per kernel from one rocprofv3 SQ counter pass.

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \\
        SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d D -o run -- python3 bench.py ...
    python tools/pmc_valu.py D > profiles/valu_<tag>.json

SURVEY.md H6 asks for VALU utilisation beside the HBM fraction.  Per kernel (summed over its
dispatches): `valu_busy` = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of a wave's life spent
issuing VALU work), `wait_mem` = SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barriers),
`wait_issue` = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (ready but not issued: dependencies, pipe
limits), `valu_insts_per_wave`.  The wait shares and SQ_ACTIVE_INST_ANY are disjoint
(MI355X_MICROARCH.md, rocprofv3 PMC slots).
"""
import collections
import csv
import glob
import json
import os
import sys

NAMES = ("impli_coarse_modes", "impli_brick_refine", "k_brick_fill", "impli_eval_bricks", "k_mc_count",
         "k_unit_scan", "k_mc_cells", "k_mc_faces")


def short(name):
    base = name.replace("(anonymous namespace)", "").split("(")[0].split("<")[0]
    for k in NAMES:
        if base.endswith(k):
            return k
    return None


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under " + d)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(files[0])):
        k = short(r["Kernel_Name"])
        if not k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id"))
    out = {}
    for k in NAMES:
        c = acc.get(k)
        if not c or not c["SQ_WAVE_CYCLES"]:
            continue
        wc = c["SQ_WAVE_CYCLES"]
        out[k] = {"dispatches": len(disp[k]),
                  "waves_per_dispatch": round(c["SQ_WAVES"] / max(1, len(disp[k]))),
                  "valu_busy": round(c["SQ_ACTIVE_INST_VALU"] / wc, 3),
                  "active_any": round(c["SQ_ACTIVE_INST_ANY"] / wc, 3),
                  "wait_mem": round(c["SQ_WAIT_ANY"] / wc, 3),
                  "wait_issue": round(c["SQ_WAIT_INST_ANY"] / wc, 3),
                  "valu_insts_per_wave": round(c["SQ_INSTS_VALU"] / max(1.0, c["SQ_WAVES"]))}
    json.dump({"note": __doc__.strip().splitlines()[0], "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
