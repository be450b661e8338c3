#!/usr/bin/env python3
"""Config 5 (64-object stream @128^3) variants on one GPU: streams x graphs on/off.
usage: python tools/config5_probe.py [n_objects] [R]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    torch.cuda.init()
    objs = scenes.config5_objects(n, R)
    shapes, mc = [o[0] for o in objs], objs[0][1]
    sp = torch.cuda.current_stream().cuda_stream
    I.set_jit(0)   # merged launches: the interpreter kernels
    b = I.Batch(shapes, mc, n_streams=0)
    for _ in range(3):
        b.run(sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        b.run(sp)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    print("merged launches (interpreter)  %.3f ms / %d objects  (%.1f us/object, %.0f Mvox/s)" %
          (ms, n, ms * 1e3 / n, n * R ** 3 / ms / 1e3), flush=True)
    b.close()
    I.set_jit(2)
    for graphs in (True, False):
        if graphs:
            os.environ.pop("IMPLISOLID_NO_GRAPH", None)
        else:
            os.environ["IMPLISOLID_NO_GRAPH"] = "1"
        for ns in (1, 2, 4, 8):
            b = I.Batch(shapes, mc, n_streams=ns)
            for _ in range(3):
                b.run(sp)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                b.run(sp)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 20 * 1e3
            print("graphs=%d streams=%d  %.3f ms / %d objects  (%.1f us/object, %.0f Mvox/s) jit %.1fs" %
                  (b.graphs, ns, ms, n, ms * 1e3 / n, n * R ** 3 / ms / 1e3, b.jit_seconds), flush=True)
            b.close()


if __name__ == "__main__":
    main()
