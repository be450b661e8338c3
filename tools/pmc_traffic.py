#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py <fetch_dir> <write_dir> > profiles/traffic_r01.json

Counters are read as rocprofv3 reports them (kilobytes) and converted to bytes.  gfx950
correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of wide coalesced
streaming reads, so fetched bytes are doubled; WRITE_SIZE is taken as is.  Our kernels mostly use
4-byte-per-lane accesses, a width the guide lists as uncalibrated -- the figures are an estimate,
comparable between kernels and rounds.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def short(name):
    for k in ("k_brick_modes", "k_eval_field_pruned", "k_eval_field", "k_mc_count", "k_scan_partial", "k_scan_top",
              "k_scan_apply", "k_mc_verts", "k_mc_faces"):
        if k + "<" in name or k + "(" in name:
            return k
    return None


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    names = {"k_brick_modes": "brick_modes", "k_eval_field_pruned": "eval_field", "k_eval_field": "eval_field",
             "k_mc_count": "mc_count", "k_mc_verts": "mc_verts", "k_mc_faces": "mc_faces",
             "k_scan_partial": "mc_scan", "k_scan_top": "mc_scan", "k_scan_apply": "mc_scan"}
    out = {"fetch_bytes": {}, "write_bytes": {}, "bytes_per_launch": {}}
    for full in set(fetch) | set(write):
        k = short(full)
        if not k:
            continue
        key = names[k]
        fb = 2.0 * 1024.0 * fetch.get(full, 0.0)
        wb = 1024.0 * write.get(full, 0.0)
        out["fetch_bytes"][key] = out["fetch_bytes"].get(key, 0.0) + fb
        out["write_bytes"][key] = out["write_bytes"].get(key, 0.0) + wb
    for k in out["fetch_bytes"]:
        out["bytes_per_launch"][k] = out["fetch_bytes"][k] + out["write_bytes"].get(k, 0.0)
    out["note"] = __doc__.strip().splitlines()[0]
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
