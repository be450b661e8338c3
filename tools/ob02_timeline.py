#!/usr/bin/env python3
"""Timeline of one build_geometry with the OB02 loop (config 2 at 128^3, config 3s at 256^3):
where the wall time of a build goes -- kernels, copies, and the gaps between them.

  run:      rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run -- \
                python3 tools/ob02_timeline.py run
  analyse:  python3 tools/ob02_timeline.py analyse DIR

The run does 3 warm builds per config, then 5 traced builds separated by 30 ms of idle host time;
the analysis splits the trace at those idle gaps and prints, for the median build of each config,
its span, the busy time (union of kernel and copy intervals), the largest gaps and the operations
before them."""
import csv
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    torch.cuda.init()
    for name, (shape, mc) in (("config2", scenes.config2(128)), ("config3s", scenes.config3_shifted(256))):
        for _ in range(3):
            I.make_geometry(shape, mc)
            I.jit_wait()
        time.sleep(0.1)
        walls = []
        for _ in range(5):
            t0 = time.perf_counter()
            I.make_geometry(shape, mc)
            walls.append((time.perf_counter() - t0) * 1e3)
            time.sleep(0.03)
        print(name, "wall ms", [round(w, 3) for w in walls], flush=True)
        time.sleep(0.2)


def analyse(d):
    ops = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                        "copy %s %s B" % (r.get("Direction", "?"), r.get("Bytes", "?"))))
    ops.sort()
    builds, cur = [], [ops[0]]
    for o in ops[1:]:
        if o[0] - max(p[1] for p in cur[-8:]) > 10_000_000:   # > 10 ms idle: a new build
            builds.append(cur)
            cur = []
        cur.append(o)
    builds.append(cur)
    # the last 10 groups are the traced builds (5 per config); earlier ones are warm-up
    traced = builds[-10:]
    for name, grp in (("config2", traced[:5]), ("config3s", traced[5:])):
        spans = sorted(((b[-1][1] - b[0][0]), i) for i, b in enumerate(grp))
        b = grp[spans[len(spans) // 2][1]]
        t0 = b[0][0]
        busy, end = 0, t0
        gaps = []
        prev = None
        for s, e, n in b:
            if s > end:
                gaps.append((s - end, prev, n))
            busy += max(0, e - max(s, end))
            end = max(end, e)
            prev = n
        kern = sum(e - s for s, e, n in b if not n.startswith("copy"))
        copies = [(e - s, n) for s, e, n in b if n.startswith("copy")]
        print("%s: span %.1f us, busy %.1f us, kernels %d (%.1f us), copies %d (%.1f us), gaps %.1f us" % (
            name, (b[-1][1] - t0) / 1e3, busy / 1e3, sum(1 for o in b if not o[2].startswith("copy")), kern / 1e3,
            len(copies), sum(c[0] for c in copies) / 1e3, sum(g[0] for g in gaps) / 1e3))
        for g, p, n in sorted(gaps, reverse=True)[:12]:
            print("   gap %7.1f us  after %-45s before %s" % (g / 1e3, (p or "")[:45], n[:45]))
        for c in sorted(copies, reverse=True)[:6]:
            print("   %7.1f us %s" % (c[0] / 1e3, c[1]))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        analyse(sys.argv[2])
