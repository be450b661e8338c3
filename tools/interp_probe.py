#!/usr/bin/env python3
"""Time the interpreter path of one object (no tree module: implisolid_set_jit(0)), as a
never-seen shape runs until its module is loaded: config 4 at R, eval only and the whole step.

    IMPLISOLID_INTERP_PAIR=0|1 python tools/interp_probe.py [R] [steps]
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
    I.set_jit(0)
    shape, mc = scenes.config4(R)
    sp = torch.cuda.current_stream().cuda_stream
    s = I.Slab(shape, mc, 0, 1)
    for _ in range(3):
        s.eval(sp); s.count(sp); s.emit(0, sp)
    torch.cuda.synchronize()
    out = {"R": R, "pair": os.environ.get("IMPLISOLID_INTERP_PAIR", "1"), "used_jit": bool(s.used_jit())}
    t0 = time.perf_counter()
    for _ in range(steps):
        s.eval(sp)
    torch.cuda.synchronize()
    out["eval_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 4)
    t0 = time.perf_counter()
    for _ in range(steps):
        s.eval(sp); s.count(sp); s.emit(0, sp)
    torch.cuda.synchronize()
    out["step_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 4)
    out["counts"] = [int(x) for x in s.counts(sp)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
