"""Probe: P independent whole-grid builds of config 4 on P HIP streams of ONE GPU.

Every kernel of one build is latency-bound (few waves per SIMD, dependent memory round trips), so
the chip is mostly idle inside each one.  P builds of the object, each with its own engine
(buffers) on its own stream, overlap those kernels.  Prints the time per build (ms) for direct
launches and for the P-stream step replayed as one hipGraph, and checks every build's mesh against
the one-stream mesh byte for byte.
    python tools/concurrent_probe.py [R] [P ...]
"""
import sys
import time

import numpy as np
import torch

import implisolid_amd as I
from implisolid_amd import scenes


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    Ps = [int(a) for a in sys.argv[2:]] or [1, 2, 3, 4]
    dev = torch.device("cuda", 0)
    main_s = torch.cuda.current_stream(dev)
    shape, mc = scenes.config4(R)
    ref = None
    for P in Ps:
        slabs = [I.Slab(shape, mc) for _ in range(P)]
        streams = [torch.cuda.Stream(dev) for _ in range(P)]
        ev_start = torch.cuda.Event()
        ev_end = [torch.cuda.Event() for _ in range(P)]
        cur = {"s": main_s}

        def step():
            ms = cur["s"]
            ev_start.record(ms)
            for p in range(P):
                st = streams[p]
                st.wait_event(ev_start)
                slabs[p].eval(st.cuda_stream)
                slabs[p].count(st.cuda_stream)
                slabs[p].emit(0, st.cuda_stream)
                ev_end[p].record(st)
            for p in range(P):
                ms.wait_event(ev_end[p])

        for _ in range(3):
            step()
        I.jit_wait()
        for _ in range(6):
            step()
        I.jit_wait()   # the hot object's baked module (bake mode 2)
        for _ in range(3):
            step()
        torch.cuda.synchronize(dev)
        if any(sl.counts(0)[2] for sl in slabs):   # first call sized the outputs: once more
            step()
        torch.cuda.synchronize(dev)
        res = {}
        for mode in ("direct", "graph"):
            run = step
            if mode == "graph":
                graph = torch.cuda.CUDAGraph()
                cs = torch.cuda.Stream(dev)
                cs.wait_stream(main_s)
                with torch.cuda.stream(cs):
                    cur["s"] = cs
                    graph.capture_begin()
                    step()
                    graph.capture_end()
                cur["s"] = main_s
                main_s.wait_stream(cs)
                run = graph.replay
                for _ in range(3):
                    run()
            torch.cuda.synchronize(dev)
            times = []
            for rep in range(3):
                t0 = time.perf_counter()
                for _ in range(50):
                    run()
                torch.cuda.synchronize(dev)
                times.append((time.perf_counter() - t0) / 50 * 1e3 / P)
            res[mode] = round(min(times), 4)
        same = True
        for sl in slabs:
            nv, nf, of = sl.counts(0)
            assert not of
            v, f = sl.download(nv, nf, 0)
            if ref is None:
                ref = (v, f)
            same = same and v.shape == ref[0].shape and f.shape == ref[1].shape and \
                np.array_equal(v.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(f, ref[1])
        print("R=%d P=%d ms/build %s  V=%d F=%d identical=%s" % (R, P, res, len(ref[0]), len(ref[1]), same), flush=True)
        for sl in slabs:
            sl.close()


if __name__ == "__main__":
    main()
