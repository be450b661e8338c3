#!/usr/bin/env python3
"""The interval passes of config 4's tree at a few resolutions with the tree module compiled
synchronously (and baked, IMPLISOLID_JIT_BAKE=1 to bake): per-kernel HIP-event times, printed as
they come.  python tools/coarse_probe.py [R ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    I.set_jit(1)
    Rs = [int(a) for a in sys.argv[1:]] or [64, 256, 512]
    sp = torch.cuda.current_stream().cuda_stream
    for R in Rs:
        shape, mc = scenes.config4(R)
        s = I.Slab(shape, mc, 0, 1)
        t0 = time.perf_counter()
        s.eval(sp); s.count(sp); s.emit(0, sp)
        torch.cuda.synchronize()
        print("R", R, "first step %.3f s" % (time.perf_counter() - t0), "module", s.jit_module(), flush=True)
        for _ in range(3):
            s.eval(sp); s.count(sp); s.emit(0, sp)
        torch.cuda.synchronize()
        s.set_timing(True)
        per = []
        for _ in range(5):
            s.eval(sp); s.count(sp); s.emit(0, sp)
            per.append(s.kernel_times_each())
        s.set_timing(False)
        print("R", R, {k: round(sum(p[k] for p in per) / len(per) * 1e3, 1) for k in per[0]}, flush=True)
        s.close()


if __name__ == "__main__":
    main()
