#!/usr/bin/env python3
"""One GPU, one build split into K balanced Z-slabs run concurrently on K HIP streams (the
multi-GPU slab decomposition inside one device): each stream evaluates and counts its slab, copies
its counts into a shared device table, emits its vertices, then -- after the counts of the slabs
below it -- its faces with global ids.  The whole step is captured once as a hipGraph and
replayed.  Prints per K: ms per build, and whether the concatenated mesh equals K = 1's.

    python tools/subslab_probe.py [R] [steps] [K,...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import numpy as np
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ks = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 3, 4, 6, 8]
    dev = torch.device("cuda", 0)
    shape, mc = scenes.config4(R)
    main_s = torch.cuda.current_stream(dev)
    ref = None
    out = {"R": R, "steps": steps, "runs": []}
    for K in ks:
        cuts = I.slab_balance(shape, mc, K) if K > 1 else None
        slabs = [I.Slab(shape, mc, k, K, cuts=cuts) for k in range(K)]
        streams = [torch.cuda.Stream(dev) for _ in range(K)]
        gath = torch.zeros(K, 4, dtype=torch.int32, device=dev)
        fork = torch.cuda.Event()
        counted = [torch.cuda.Event() for _ in range(K)]
        done = [torch.cuda.Event() for _ in range(K)]

        def step(ms):
            fork.record(ms)
            for k in range(K):
                st = streams[k]
                st.wait_event(fork)
                slabs[k].eval(st.cuda_stream)
                slabs[k].count(st.cuda_stream)
                slabs[k].copy_counts(gath[k].data_ptr(), st.cuda_stream)
                counted[k].record(st)
            for k in range(K):
                st = streams[k]
                slabs[k].emit_verts(st.cuda_stream)
                for q in range(k):
                    st.wait_event(counted[q])
                slabs[k].emit_faces(0, gath.data_ptr(), k, st.cuda_stream)
                done[k].record(st)
            for k in range(K):
                ms.wait_event(done[k])

        for _ in range(3):
            step(main_s)
        I.jit_wait()
        for _ in range(3):
            step(main_s)
        torch.cuda.synchronize(dev)
        if any(s.counts(0)[2] for s in slabs):
            step(main_s)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step(main_s)
        torch.cuda.synchronize(dev)
        ms_direct = (time.perf_counter() - t0) / steps * 1e3
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(main_s)
        with torch.cuda.stream(cs):
            g.capture_begin()
            step(cs)
            g.capture_end()
        main_s.wait_stream(cs)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize(dev)
        ms_graph = (time.perf_counter() - t0) / steps * 1e3
        vs, fs = [], []
        for s in slabs:
            nv, nf, of = s.counts(0)
            assert not of
            v, f = s.download(nv, nf, 0)
            vs.append(v)
            fs.append(f)
        V, F = np.concatenate(vs), np.concatenate(fs)
        if ref is None:
            ref = (V, F)
        same = V.shape == ref[0].shape and F.shape == ref[1].shape and np.array_equal(V.view(np.uint32), ref[0].view(np.uint32)) \
            and np.array_equal(F, ref[1])
        row = {"K": K, "cuts": cuts, "ms_direct": round(ms_direct, 4), "ms_graph": round(ms_graph, 4),
               "gvox_per_s": round(R ** 3 / (ms_graph * 1e-3) / 1e9, 1), "verts": int(len(V)), "faces": int(len(F)),
               "mesh_equals_K1": bool(same)}
        out["runs"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
        del g
        for s in slabs:
            s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
