#!/usr/bin/env python3
"""Time one rank's slab of config 4 on one GPU (no collectives): the per-rank compute of the
N-GPU Z-slab run, to see how the kernel sequence scales before any RCCL cost.

    python tools/slab_probe.py [R] [steps] [nranks,...]
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
    shape, mc = scenes.config4(R)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    out = {}
    ns = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4, 8]
    for n in ns:
        for rank in sorted({0, n // 2, n - 1}):
            s = I.Slab(shape, mc, rank, n)
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
            s.set_timing(True)
            per = []
            for _ in range(5):
                s.eval(sp); s.count(sp); s.emit(0, sp)
                per.append(s.kernel_times())
            s.set_timing(False)
            k = {key: round(sum(p[key] for p in per) / len(per), 4) for key in per[0]}
            out["%d/%d" % (rank, n)] = {"ms": round(ms, 4), "kernel_ms": k}
            s.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
