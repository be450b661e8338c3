"""Probe: config 4 at R = 512 split into S balanced Z-slabs on S HIP streams of ONE GPU.

Each slab's latency-bound kernels run beside the other slabs' (the pipeline of one slab leaves
most of the chip idle in its interval, fill, count and scan kernels).  The face pass of slab s
needs the counts of the slabs below it: each slab copies its counts into row s of one device
array and records an event; slab s's stream waits for the events of slabs < s.  Prints the step
time per S and checks that the concatenated slab meshes equal the one-slab mesh byte for byte.
    python tools/streams_probe.py [S ...] [--graph]   (--graph: each step replayed as one hipGraph)
"""
import sys
import time

import numpy as np
import torch

import implisolid_amd as I
from implisolid_amd import scenes


def main():
    use_graph = "--graph" in sys.argv
    Ss = [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [1, 2, 3, 4]
    dev = torch.device("cuda", 0)
    main_s = torch.cuda.current_stream(dev)
    shape, mc = scenes.config4(512)
    ref = None
    for S in Ss:
        cuts = I.slab_balance(shape, mc, S) if S > 1 else None
        slabs = [I.Slab(shape, mc, s, S, cuts=cuts) for s in range(S)]
        streams = [main_s] if S == 1 else [torch.cuda.Stream(dev) for _ in range(S)]
        gath = torch.zeros(S, 4, dtype=torch.int32, device=dev)
        ev_cnt = [torch.cuda.Event() for _ in range(S)]
        ev_end = [torch.cuda.Event() for _ in range(S)]
        ev_start = torch.cuda.Event()

        def step():
            if S == 1:
                sp = main_s.cuda_stream
                slabs[0].eval(sp)
                slabs[0].count(sp)
                slabs[0].emit(0, sp)
                return
            ev_start.record(main_s)
            for s in range(S):
                st = streams[s]
                st.wait_event(ev_start)
                slabs[s].eval(st.cuda_stream)
                slabs[s].count(st.cuda_stream)
                slabs[s].copy_counts(gath[s].data_ptr(), st.cuda_stream)
                ev_cnt[s].record(st)
                slabs[s].emit_verts(st.cuda_stream)
            for s in range(S):
                st = streams[s]
                for t in range(s):
                    st.wait_event(ev_cnt[t])
                slabs[s].emit_faces(0, gath.data_ptr(), s, st.cuda_stream)
                ev_end[s].record(st)
            for s in range(S):
                main_s.wait_event(ev_end[s])

        for _ in range(3):
            step()
        I.jit_wait()
        for _ in range(3):
            step()
        I.jit_wait()
        for _ in range(3):
            step()
        torch.cuda.synchronize(dev)
        grew = any(sl.counts(0)[2] for sl in slabs)
        if grew:
            step()
        torch.cuda.synchronize(dev)
        run = step
        if use_graph:   # the whole multi-stream step as one graph: no host launch cost per kernel
            graph = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream(dev)
            cs.wait_stream(main_s)
            outer = main_s
            with torch.cuda.stream(cs):
                main_s = cs
                graph.capture_begin()
                step()
                graph.capture_end()
            main_s = outer
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
            times.append((time.perf_counter() - t0) / 50 * 1e3)
        vs, fs = [], []
        for sl in slabs:
            nv, nf, of = sl.counts(0)
            assert not of
            v, f = sl.download(nv, nf, 0)
            vs.append(v)
            fs.append(f)
        V, F = np.concatenate(vs), np.concatenate(fs)
        if ref is None:
            ref = (V, F)
        same = V.shape == ref[0].shape and F.shape == ref[1].shape and np.array_equal(V.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(F, ref[1])
        print("S=%d cuts=%s ms/step %s  V=%d F=%d identical=%s" % (S, cuts, [round(t, 4) for t in times], len(V), len(F), same), flush=True)
        for sl in slabs:
            sl.close()


if __name__ == "__main__":
    main()
