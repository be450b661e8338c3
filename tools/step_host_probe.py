#!/usr/bin/env python3
"""Price the host side of the N > 1 bench step on one GPU: one rank's slab of config 4 stepped
(a) kernels only, direct launches; (b) the bench's N > 1 step -- copy_counts, the count all-gather
over RCCL (a world-1 "nccl" group: the same enqueue path, no peer), the vertex pass, the face pass
-- direct; (c) that step captured once as a hipGraph (RCCL collective inside the capture) and
replayed.  Each row: ms per step over `steps` back-to-back steps, launch-stream wall time.

    python tools/step_host_probe.py [R] [steps] [nranks] [rank,...]

The gathered-count rows of the other ranks stay zero (world 1), so the faces' global ids are
offset wrongly; the kernels' work and the launch sequence are the bench's.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    import torch.distributed as dist
    import implisolid_amd as I
    from implisolid_amd import scenes, distributed as D
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    ranks = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 2]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29655")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    shape, mc = scenes.config4(R)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    cuts = I.slab_balance(shape, mc, n) if n > 1 else None
    out = {"R": R, "steps": steps, "nranks": n, "cuts": cuts, "ranks": {}}
    for rank in ranks:
        s = I.Slab(shape, mc, rank, n, cuts=cuts)
        cnt = torch.zeros(4, dtype=torch.int32, device=dev)
        gath = torch.zeros(n, 4, dtype=torch.int32, device=dev)

        def kern(st):
            s.eval(st); s.count(st); s.emit(0, st)

        def full(st):
            s.eval(st); s.count(st)
            s.copy_counts(cnt.data_ptr(), st)
            work = D.gather_counts_async(cnt, gath[0:1].view(-1))
            s.emit_verts(st)
            if work is not None:
                work.wait()
            s.emit_faces(0, gath.data_ptr(), rank, st)

        class _Cai:   # the slab's totals block [2, 6) of its counters, as a tensor without a copy
            __cuda_array_interface__ = {"shape": (4,), "typestr": "<i4", "data": (s.counters_ptr() + 8, False),
                                        "version": 3, "strides": None}
        tot = torch.as_tensor(_Cai(), device=dev)

        def sync_early(st):   # the all-gather on the launch stream (async_op=False), before the vertex pass
            s.eval(st); s.count(st)
            dist.all_gather_into_tensor(gath[0:1].view(-1), tot)
            s.emit_verts(st)
            s.emit_faces(0, gath.data_ptr(), rank, st)

        def sync_late(st):    # ... after it
            s.eval(st); s.count(st)
            s.emit_verts(st)
            dist.all_gather_into_tensor(gath[0:1].view(-1), tot)
            s.emit_faces(0, gath.data_ptr(), rank, st)

        def async_nocopy(st):   # the bench's order without copy_counts
            s.eval(st); s.count(st)
            work = D.gather_counts_async(tot, gath[0:1].view(-1))
            s.emit_verts(st)
            if work is not None:
                work.wait()
            s.emit_faces(0, gath.data_ptr(), rank, st)

        def timed(fn):
            for _ in range(5):
                fn()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize(dev)
            return (time.perf_counter() - t0) / steps * 1e3

        for _ in range(3):
            kern(sp)
        I.jit_wait()
        s.counts(sp)
        row = {"layers": [s.cz_emit, s.cz1]}
        row["kernels_direct_ms"] = round(timed(lambda: kern(sp)), 4)
        row["step_direct_ms"] = round(timed(lambda: full(sp)), 4)
        row["step_sync_early_ms"] = round(timed(lambda: sync_early(sp)), 4)
        row["step_sync_late_ms"] = round(timed(lambda: sync_late(sp)), 4)
        row["step_async_nocopy_ms"] = round(timed(lambda: async_nocopy(sp)), 4)
        # host cost alone: the launch loop's wall time without waiting (queue depth permitting)
        t0 = time.perf_counter()
        for _ in range(steps):
            full(sp)
        row["step_host_enqueue_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 4)
        torch.cuda.synchronize(dev)
        for name, fn in (("kernels_graph_ms", kern), ("step_graph_ms", full), ("step_sync_late_graph_ms", sync_late)):
            try:
                g = torch.cuda.CUDAGraph()
                cs = torch.cuda.Stream(dev)
                cs.wait_stream(stream)
                with torch.cuda.stream(cs):
                    g.capture_begin()
                    fn(cs.cuda_stream)
                    g.capture_end()
                stream.wait_stream(cs)
                row[name] = round(timed(g.replay), 4)
                del g
            except Exception as exc:   # capture refused: record why
                torch.cuda.synchronize(dev)
                row[name] = None
                row[name + "_error"] = str(exc)[:300]
        # the bench's N > 1 form: two graphs (eval + count + vertex pass; face pass) with the
        # all-gather launched between their replays on the same stream
        try:
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream(dev)
            cs.wait_stream(stream)
            with torch.cuda.stream(cs):
                g1.capture_begin()
                s.eval(cs.cuda_stream); s.count(cs.cuda_stream); s.emit_verts(cs.cuda_stream)
                g1.capture_end()
                g2.capture_begin()
                s.emit_faces(0, gath.data_ptr(), rank, cs.cuda_stream)
                g2.capture_end()
            stream.wait_stream(cs)

            def two():
                g1.replay()
                dist.all_gather_into_tensor(gath[0:1].view(-1), tot)
                g2.replay()
            row["step_two_graphs_ms"] = round(timed(two), 4)
            t0 = time.perf_counter()
            for _ in range(steps):
                two()
            row["step_two_graphs_host_enqueue_ms"] = round((time.perf_counter() - t0) / steps * 1e3, 4)
            torch.cuda.synchronize(dev)
            del g1, g2
        except Exception as exc:
            torch.cuda.synchronize(dev)
            row["step_two_graphs_error"] = str(exc)[:300]
        s.close()
        out["ranks"][rank] = row
        print(json.dumps({rank: row}), file=sys.stderr, flush=True)
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
