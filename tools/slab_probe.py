#!/usr/bin/env python3
"""Time every rank's slab of config 4 on one GPU (no collectives): the per-rank compute of the
N-GPU Z-slab run, to see how the kernel sequence scales and how well the cuts balance it.

    python tools/slab_probe.py [R] [steps] [nranks,...] [equal|balanced|both]

Per N: the cuts, each rank's ms per step (eval + count + emit, launch-stream wall time over
`steps` steps) and per-kernel HIP-event times, max / min over ranks, and the strong-scaling bound
t(1 rank) / max over ranks.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ns = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4, 8]
    modes = {"both": ["equal", "balanced"]}.get(sys.argv[4] if len(sys.argv) > 4 else "both",
                                                 [sys.argv[4] if len(sys.argv) > 4 else "balanced"])
    shape, mc = scenes.config4(R)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    out = {"R": R, "steps": steps}
    t1 = None
    for n in ns:
        for mode in (modes if n > 1 else ["equal"]):
            cuts = I.slab_balance(shape, mc, n) if mode == "balanced" else None
            ranks = {}
            for rank in range(n):
                s = I.Slab(shape, mc, rank, n, cuts=cuts)
                for _ in range(3):
                    s.eval(sp); s.count(sp); s.emit(0, sp)
                s.counts(sp)
                s.eval(sp); s.count(sp); s.emit(0, sp)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    s.eval(sp); s.count(sp); s.emit(0, sp)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / steps * 1e3
                # the same step replayed as one hipGraph (one launch call per step instead of ~10)
                g = torch.cuda.CUDAGraph()
                cs = torch.cuda.Stream()
                cs.wait_stream(stream)
                with torch.cuda.stream(cs):
                    g.capture_begin()
                    s.eval(cs.cuda_stream); s.count(cs.cuda_stream); s.emit(0, cs.cuda_stream)
                    g.capture_end()
                stream.wait_stream(cs)
                for _ in range(3):
                    g.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    g.replay()
                torch.cuda.synchronize()
                ms_graph = (time.perf_counter() - t0) / steps * 1e3
                del g
                s.set_timing(True)
                per = []
                for _ in range(5):
                    s.eval(sp); s.count(sp); s.emit(0, sp)
                    per.append(s.kernel_times())
                s.set_timing(False)
                k = {key: round(sum(p[key] for p in per) / len(per), 4) for key in per[0]}
                ranks[rank] = {"layers": [s.cz_emit, s.cz1], "ms": round(ms, 4), "ms_graph": round(ms_graph, 4),
                               "kernel_ms": k}
                s.close()
            mss = [r["ms"] for r in ranks.values()]
            msg = [r["ms_graph"] for r in ranks.values()]
            if n == 1:
                t1 = mss[0]
            out["%d/%s" % (n, mode)] = {"cuts": cuts, "max_ms": max(mss), "min_ms": min(mss),
                                        "max_ms_graph": max(msg), "min_ms_graph": min(msg),
                                        "max_over_min": round(max(mss) / min(mss), 3),
                                        "strong_bound": round(t1 / max(mss), 2) if t1 else None, "ranks": ranks}
            print(n, mode, "max %.4f min %.4f ratio %.2f | graph max %.4f min %.4f" % (
                max(mss), min(mss), max(mss) / min(mss), max(msg), min(msg)), file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
