#!/usr/bin/env python3
"""Benchmark: eval + marching cubes (Mvoxels/s) of the config-4 scene on 1..N MI355X.

Workload (BASELINE.json configs[3], the largest single-GPU configuration the metric is quoted on):
config 3's seeded 21-node MP5 CSG tree at R = 512 over the box [-1, 1]^3.  One step = field
evaluation of the (R+1)^3 stored samples + marching-cubes count / scan / vertex + face emission,
with the mesh left resident in HBM (no host copy in the timed region).

N > 1 (torchrun, one process per GPU, RCCL): the cell layers are split into Z-slabs at balanced
cuts (one interval pass of the whole grid, computed alike by every rank).  Each rank recomputes one
halo cell layer below its slab; the only exchange in the step is an all-gather of the per-slab
(vertex, face) counts on the launch stream, which gives every rank its global numbering offsets on
the device.  The headline is weak scaling (the task's bench contract for a path that partitions:
per-GPU work fixed as N grows): the grid grows to R_N = round(R N^(1/3)) -- 645^3 / 813^3 / 1024^3
at 2 / 4 / 8 ranks, ~R^3 voxels per rank -- and `value` is all R_N^3 voxels over the max-over-ranks
step time.  Strong scaling of BASELINE config 4 (the R = 512 grid over N GPUs) is reported beside it
under "strong"; --strong swaps the two.  After the timed steps each mesh is gathered to rank 0
(distributed.gather_mesh, timed as "gather_ms") and checked against the oracle's summary of the
same workload.

Prints ONE JSON line (rank 0).  Extra fields: per-kernel times from HIP events on the launch
stream, the HBM roofline of the eval+MC kernel sequence (SURVEY.md 8d's algorithmic bytes), and
the CPU baseline (the oracle restatement, single thread, on a bounded sample of the same workload).
"""
import argparse
import json
import os
import re
import sys
import time

import numpy as np

T_START = time.perf_counter()   # the bench's total wall time is reported from here (legs_wall_s)


def progress(what):
    """A progress line on stderr (rank 0): a cold box compiles every tree module on first use, and
    a run that prints nothing for minutes reads as hung.  The JSON line stays alone on stdout."""
    if os.environ.get("RANK", "0") == "0":
        print("bench: %s (%.1f s)" % (what, time.perf_counter() - T_START), file=sys.stderr, flush=True)
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def jit_wait(I, what="tree-module compiles"):
    """I.jit_wait() with a progress line every 20 s while it blocks: on a box with an empty JIT cache
    the headline's modules compile before the first leg starts (the ctypes call releases the GIL)."""
    import threading
    t = threading.Thread(target=I.jit_wait, daemon=True)
    t.start()
    while True:
        t.join(20.0)
        if not t.is_alive():
            return
        progress("waiting for %s" % what)


HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md)
# kernel (profile short name) -> the engine's timed phase (Slab.KERNELS; tools/pmc_traffic.py)
KERNEL_PHASE = {"impli_coarse_modes": "brick_modes", "impli_brick_refine": "brick_modes", "k_brick_fill": "brick_modes",
                "impli_eval_bricks": "eval_field", "k_eval_field_pruned": "eval_field", "k_mc_count": "mc_count",
                "k_unit_scan": "mc_scan", "k_mc_cells": "mc_verts", "k_mc_faces": "mc_faces"}

# algorithmic FP ops per sample for one instruction of the node program
OP_FLOPS = {"xform": 18, "csg": 2, 3: 9, 4: 45, 5: 24, 6: 20, 7: 24, 8: 14, 9: 12,
            10: 90, 11: 3, 12: 8}   # 10 screw (atan2f + sinf + 25), 11 lid, 12 half plane


def program_flops(shape):
    import implisolid_amd as I
    n_instr, depth, n_mats, _ = I.program_info(shape)
    # count leaves / CSG nodes from the JSON (the program has one XFORM per node)
    def walk(d):
        t = d["type"]
        if "children" in d:
            kids = d["children"]
            n = len(kids) - 1 if t == "Union" else 1
            return OP_FLOPS["csg"] * n + OP_FLOPS["xform"] * n + sum(walk(c) for c in (kids if t == "Union" else kids[:2]))
        x, c = OP_FLOPS["xform"], OP_FLOPS["csg"]
        composite = {"screw": (c + x) + (x + OP_FLOPS[10]) + (x + OP_FLOPS[11]),
                     "inf_screw": x + OP_FLOPS[10],
                     "screw_diff_two_plane": 2 * (c + x) + (x + OP_FLOPS[10]) + 2 * (x + OP_FLOPS[12]),
                     "top_bottom_lid": x + OP_FLOPS[11], "half_plane": x + OP_FLOPS[12],
                     "screw_gradient_wrong": x + OP_FLOPS[10] + OP_FLOPS[11] + c}
        if t in composite:
            return composite[t]
        code = {"iellipsoid": 3, "ellipsoid": 3, "cube": 4, "icube": 4, "icylinder": 5, "cylinder": 5, "icone": 6,
                "cone": 6, "iheart": 7, "itorus": 8, "implicit_double_mushroom": 9}[t]
        return OP_FLOPS["xform"] + OP_FLOPS[code]
    return walk(shape), n_instr, depth


def cpu_baseline(shape, target_s=20.0):
    """Oracle (CPU restatement, 1 thread) eval + MC of the same tree on a bounded sample."""
    import oracle
    oracle.build()
    tree = oracle.mp5_to_nodes(json.dumps(shape))
    box = [-1.0, 1.0] * 3
    R = 48
    t0 = time.perf_counter()
    oracle.marching_cubes(tree, R, box)
    dt = time.perf_counter() - t0
    # scale the sample so it runs about target_s seconds
    R = int(max(48, min(512, R * (target_s / max(dt, 1e-3)) ** (1 / 3))))
    t0 = time.perf_counter()
    v, f = oracle.marching_cubes(tree, R, box)
    dt = time.perf_counter() - t0
    return {"value": R ** 3 / dt / 1e6, "unit": "Mvoxels/s", "cores": 1, "kind": "port",
            "sample": "oracle restatement (C, 1 thread) eval+MC of the same tree at %d^3 on this host (%.1f s, %d faces)"
                      % (R, dt, f.shape[0]), "host": host_info()}, (R, v, f)


_C5_WORKER = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import oracle
from implisolid_amd import scenes
objs = scenes.config5_objects(64, 128)
for k in map(int, sys.argv[2].split(",")):
    shape, _ = objs[k]
    t0 = time.perf_counter()
    v, f = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(shape)), 128, [-1.0, 1.0] * 3)
    print(json.dumps([k, time.perf_counter() - t0, int(v.shape[0]), int(f.shape[0])]), flush=True)
"""


def config5_cpu_baseline(n_objects=64):
    """config 5's CPU figure on N = cores processes -- the oracle polygonises the 64
    objects at 128^3 (the whole stream, not a sample) on as many worker processes as this process
    may use (the affinity mask, capped by OMP_NUM_THREADS, which the GPU box sets to its CPU share).
    Each worker is a plain child interpreter (subprocess, nothing inherited from this process's GPU
    context, no multiprocessing semaphores or resource tracker) taking every cores-th object; all of
    them are reaped before this returns."""
    import subprocess
    import oracle
    oracle.build()
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        cores = min(cores, int(cap))
    cores = max(1, min(cores, n_objects))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    t0 = time.perf_counter()
    procs = [subprocess.Popen([sys.executable, "-c", _C5_WORKER, ROOT,
                               ",".join(str(k) for k in range(w, n_objects, cores))],
                              stdout=subprocess.PIPE, text=True, env=env) for w in range(cores)]
    rows = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=600)
            if p.returncode != 0:
                raise RuntimeError("config-5 oracle worker exited with %d" % p.returncode)
            rows += [json.loads(line) for line in out.splitlines() if line.strip()]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    wall = time.perf_counter() - t0
    if len(rows) != n_objects:
        raise RuntimeError("config-5 oracle workers returned %d of %d objects" % (len(rows), n_objects))
    one = sum(r[1] for r in rows)
    return {"value": round(n_objects / wall, 2), "unit": "objects/s", "cores": cores, "kind": "port",
            "sample": "oracle restatement (C): all %d config-5 objects at 128^3, eval+MC, the objects dealt over "
                      "%d worker processes (%.2f s wall incl. process start; %.1f s summed per-object CPU time = %.2f "
                      "objects/s on one core)" % (n_objects, cores, wall, one, n_objects / one),
            "mvoxels_per_s": round(n_objects * 128 ** 3 / wall / 1e6, 2),
            "faces": sum(r[3] for r in rows)}


def host_info():
    """The host the CPU baseline ran on: logical CPUs (nproc), the CPUs this process may use, and
    the model name (lscpu) -- SURVEY.md 8d asks for the core count beside the one-thread figure."""
    import subprocess
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except Exception:
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k.strip().lower().replace(" ", "_").replace("(s)", "s")] = v.strip()
    except Exception:
        pass
    return info


def mesh_parity(v, f, v_ref, f_ref):
    """max|v - v_ref| over the vertices and whether the face arrays are identical (the metric's
    max|v-v_ref|).  Non-finite reference vertices (OB02 on a tree whose singular
    point lands on a grid sample: a zero gradient that normalize_1111 divides by)
    must be non-finite at the same rows; the difference is taken over the finite ones."""
    same_shape = v.shape == v_ref.shape and f.shape == f_ref.shape
    out = {"verts": int(v_ref.shape[0]), "faces": int(f_ref.shape[0]),
           "faces_identical": bool(same_shape and np.array_equal(f, f_ref)), "max_abs_v_diff": None}
    if same_shape:
        fin, fin_ref = np.isfinite(v).all(1), np.isfinite(v_ref).all(1)
        both = fin & fin_ref
        out["max_abs_v_diff"] = float(np.abs(v[both].astype(np.float64) - v_ref[both]).max()) if both.any() else 0.0
        if not fin_ref.all():
            out["nonfinite_ref_verts"] = int((~fin_ref).sum())
            out["nonfinite_rows_identical"] = bool(np.array_equal(fin, fin_ref))
    return out


def headline_parity(name, v, f):
    """The whole mesh against the oracle's committed summary of the same workload
    (tests/golden/headline_summaries.json, made by tests/golden/make_headline.py), if there is one."""
    import hashlib
    path = os.path.join(ROOT, "tests", "golden", "headline_summaries.json")
    try:
        s = json.load(open(path))[name]
    except Exception:
        return {"checked": False, "why": "no oracle summary for " + name}
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    same = sha(v) == s["sha256_verts"]
    diff = 0.0 if same else None
    over = "all vertices" if same else "the summary's 4096 sampled rows"
    full = None
    if not same and len(v) == s["n_verts"]:   # the oracle's full vertex array, where one is committed
        try:
            full = np.load(os.path.join(ROOT, "tests", "golden", "headline_ob02_verts.npz"))[name]
        except Exception:
            full = None
    if full is not None:
        v = np.asarray(v)
        fin = np.isfinite(full).all(1)
        d = np.abs(v[fin].astype(np.float64) - full[fin])
        diff = float(d.max(initial=0.0))
        over = "all vertices (the oracle's full array): %.5f of the rows bit-identical" % float((d == 0).all(1).mean())
        if not np.array_equal(np.isfinite(v).all(1), fin):
            diff = float("inf")
    elif not same and len(v) == s["n_verts"]:
        # the oracle's 4096 sampled rows (trees with a twist: the gradient's double cos)
        try:
            smp = np.load(os.path.join(ROOT, "tests", "golden", "headline_samples.npz"))
            idx, vs = smp[name + "_idx"], smp[name + "_v"]
            ok = np.isfinite(vs).all(1)
            diff = float(np.abs(np.asarray(v)[idx][ok].astype(np.float64) - vs[ok]).max(initial=0.0))
        except Exception:
            diff = None
    return {"checked": True, "against": "oracle summary " + name, "verts": int(len(v)), "faces": int(len(f)),
            "faces_identical": sha(f) == s["sha256_faces"], "verts_identical": same,
            "max_abs_v_diff": diff, "v_diff_over": over}


def copy_attainable(dev, nbytes=1 << 30, reps=10):
    """Measured device-to-device copy rate (GB/s, read + write bytes): the attainable HBM figure
    SURVEY.md 8d asks to report beside the 8 TB/s peak."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    return round(gbs, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--resolution", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--skip-256", action="store_true", help="do not also time R=256")
    ap.add_argument("--prune", type=int, default=None, help="pruning level 0/1/2 (default: library default 2)")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: the headline is weak scaling (R_N = R N^(1/3), ~R^3 voxels per rank; the default) "
                         "rather than strong scaling of the R grid (BASELINE config 4); the other is reported "
                         "beside it either way, both with the gathered mesh checked against the oracle")
    ap.add_argument("--strong", action="store_true", help="N > 1: strong scaling of the R grid as the headline")
    ap.add_argument("--equal-slabs", action="store_true", help="N > 1: equal-layer slabs instead of balanced cuts")
    ap.add_argument("--skip-config5", action="store_true", help="do not time the 64-object stream (config 5)")
    ap.add_argument("--config5-streams", type=int, default=8)
    ap.add_argument("--skip-ob02", action="store_true", help="do not time build_geometry with the OB02 loop")
    ap.add_argument("--skip-concurrent", action="store_true",
                    help="do not time P concurrent builds of the headline object on P streams (serving throughput)")
    ap.add_argument("--bake", type=int, default=None,
                    help="tree modules with the matrices baked in: 0 never, 1 every object, 2 hot objects (library default)")
    ap.add_argument("--graph", action="store_true",
                    help="N = 1: replay the step as a hipGraph (an A/B switch; direct launches are the default)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import implisolid_amd as I
    from implisolid_amd import distributed as D
    from implisolid_amd import scenes

    if args.prune is not None:
        I.set_pruning(args.prune)
    if args.bake is not None:
        I.set_jit_bake(args.bake)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    # one GPU per rank; IMPLISOLID_DIST_BACKEND=gloo rehearses several ranks on fewer GPUs
    backend = os.environ.get("IMPLISOLID_DIST_BACKEND", "nccl")
    dev_index = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def run(R, steps, warmup, scene=None, gather=False):
        shape, mc = scene if scene is not None else scenes.config4(R)
        # N > 1: balanced Z-slab cuts from one interval pass of the whole grid, computed by every
        # rank alike (no exchange; implisolid_slab_balance), unless --equal-slabs
        cuts = None
        t_cut = 0.0
        if world > 1 and not args.equal_slabs:
            t0 = time.perf_counter()
            cuts = D.balanced_cuts(shape, mc, world)
            t_cut = time.perf_counter() - t0
        slab = I.Slab(shape, mc, rank, world, cuts=cuts)
        gath = torch.zeros(world, 4, dtype=torch.int32, device=dev)
        totals = D.counts_tensor(slab, dev) if backend == "nccl" else None
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]

        def step(e=None):
            if e: e[0].record(stream)
            slab.eval(sp)
            if e: e[1].record(stream)
            slab.count(sp)
            if e: e[2].record(stream)
            if world > 1:
                # the vertex pass (slab-local ids), then the 16 B/rank count all-gather on the same
                # stream, straight from the engine's counters (D.gather_counts_inline: an async
                # gather on RCCL's own stream cost 16 us more per step in cross-stream events);
                # the face pass forms this slab's vertex offset from the gathered counts
                slab.emit_verts(sp)
                if totals is not None:
                    D.gather_counts_inline(totals, gath)
                else:   # gloo rehearsal: host round trip of a copy
                    cnt = torch.zeros(4, dtype=torch.int32, device=dev)
                    slab.copy_counts(cnt.data_ptr(), sp)
                    torch.cuda.synchronize(dev)
                    D.gather_counts_inline(cnt, gath)
                slab.emit_faces(0, gath.data_ptr(), rank, sp)
            else:
                slab.emit(0, sp)
            if e: e[3].record(stream)

        progress("headline R=%d: warmup" % R)
        # warmup (first call sizes the output buffers); the tree module compiles in the background
        # meanwhile (async JIT) -- wait for it, so the timed steps run the compiled kernels
        for _ in range(max(1, warmup)):
            step()
        jit_wait(I)
        for _ in range(max(1, warmup)):
            step()
        # a hot object's baked module (bake mode 2) is requested after a few evals: wait for it too
        jit_wait(I)
        for _ in range(max(1, warmup)):
            step()
        # no compilation may run beside the timed steps (host threads compiling next to the launch
        # loop; a fresh box's first 256^3 line once read 0.18 ms against 0.065 ms on the next run):
        # warm up until a round schedules no compile and loads no module
        def jit_count():
            st = I.jit_stats()
            return st["compiled"] + st["disk_hits"]
        for _ in range(3):
            done = jit_count()
            for _ in range(max(1, warmup)):
                step()
            jit_wait(I)
            if jit_count() == done:
                break
        nv, nf, grew = slab.counts(sp)
        if grew:
            step()
        torch.cuda.synchronize(dev)
        # --graph (one GPU): the step's launches are captured once as a hipGraph and replayed --
        # every replay recomputes everything; the graph only changes how the kernels are launched
        graph = None
        if world == 1 and args.graph:
            try:
                graph = torch.cuda.CUDAGraph()
                cs = torch.cuda.Stream(dev)
                cs.wait_stream(stream)
                with torch.cuda.stream(cs):
                    graph.capture_begin()
                    slab.eval(cs.cuda_stream)
                    slab.count(cs.cuda_stream)
                    slab.emit(0, cs.cuda_stream)
                    graph.capture_end()
                stream.wait_stream(cs)
                for _ in range(2):
                    graph.replay()
                torch.cuda.synchronize(dev)
            except Exception as exc:   # capture unavailable: direct launches
                print("bench: hipGraph capture failed (%s); launching directly" % exc, file=sys.stderr)
                graph = None
                torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        # the timed steps carry no event records (each record is a queue marker: ~4 us per step
        # at 512^3 with four of them); the phase split is timed on extra steps afterwards
        t0 = time.perf_counter()
        if graph is not None:
            for k in range(steps):
                graph.replay()
        else:
            for k in range(steps):
                step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        nv, nf, of = slab.counts(sp)
        if of:
            raise RuntimeError("output overflow in the timed region")
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        tot = torch.tensor([nv, nf], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.all_reduce(tot)
        el = float(t.item())
        n_phase = min(steps, 10)   # phase split (eval / count + scan / emit): extra steps with events
        for k in range(n_phase):
            if graph is not None:
                ev[k][0].record(stream)
                graph.replay()
                ev[k][3].record(stream)
            else:
                step(ev[k])
        torch.cuda.synchronize(dev)
        ev = ev[:n_phase]
        if graph is not None:   # one interval per replay: eval + count + scan + emit
            kms = {"step_graph": float(np.mean([e[0].elapsed_time(e[3]) for e in ev]))}
        else:
            kms = {"eval": float(np.mean([e[0].elapsed_time(e[1]) for e in ev])),
                   "mc_count_scan": float(np.mean([e[1].elapsed_time(e[2]) for e in ev])),
                   "mc_emit": float(np.mean([e[2].elapsed_time(e[3]) for e in ev]))}
        # per-kernel durations: HIP events recorded by the engine between its launches on this
        # stream, over a few extra steps after the timed region (so it is not perturbed)
        slab.set_timing(True)
        per, per_each = [], []
        for _ in range(5):
            step()
            per.append(slab.kernel_times())
            per_each.append(slab.kernel_times_each())
        slab.set_timing(False)
        kernel_ms = {k: float(np.mean([p[k] for p in per])) for k in per[0]}
        each_ms = {k: float(np.mean([p[k] for p in per_each])) for k in per_each[0]}
        # the emission kernels are idempotent once counted (same positions, ids and records from
        # the same counts): each launched 20 times back to back between two events, which prices
        # one launch without the per-kernel event markers' queue gaps
        repeat_ms = {}
        for name, fn in (("k_mc_cells", lambda: slab.emit_verts(sp)),
                         ("k_mc_faces", lambda: slab.emit_faces(0, gath.data_ptr() if world > 1 else 0, rank, sp))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn()
            e0.record(stream)
            for _ in range(20):
                fn()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            repeat_ms[name] = e0.elapsed_time(e1) / 20
        info = dict(R=R, nv=int(tot[0]), nf=int(tot[1]), elapsed=el, kernels_ms=kms, kernel_ms=kernel_ms, each_ms=each_ms, repeat_ms=repeat_ms,
                    shape=shape, slab_layers=slab.cz1 - slab.cz_emit, depth=slab.depth, bricks=slab.brick_stats(),
                    graph=graph is not None, cuts=cuts, cut_s=t_cut,
                    fz=(slab.fz0, slab.fz1), jit=slab.used_jit(), jit_module=slab.jit_module(), stats=slab.stats())
        if world > 1:
            # every rank's own step time (the max over ranks is the headline's): the balance
            rt = torch.tensor([el], dtype=torch.float64, device=dev)
            allt = [torch.zeros_like(rt) for _ in range(world)]
            dist.all_gather(allt, rt)
            info["rank_ms"] = [round(float(x.item()) / steps * 1e3, 4) for x in allt]
        if gather and world > 1:
            # the output gather to rank 0 (the C ABI's host-resident result; outside the timed step):
            # then parity of the whole N-GPU mesh against the oracle's summary of the same workload
            step()
            torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            res = D.gather_mesh(slab, gath, rank, world)
            info["gather_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
            if rank == 0:
                info["parity"] = headline_parity("config4_mc_r%d" % R, *res)
        slab.close()
        return info

    # N > 1: the headline is weak scaling (R_N = R N^(1/3), ~R^3 voxels per rank: the per-GPU work
    # stays that of one GPU; the task's contract for a path that partitions); strong scaling of config
    # 4 (the R grid over N GPUs, BASELINE config 4) is reported beside it (--strong swaps them).  Both gather their mesh to rank 0 after the timed steps
    # and check it against the oracle's summary of the same grid (tests/golden/make_headline.py holds
    # config4_mc_r512 / r645 / r813 / r1024)
    legs = {}

    def leg(name, fn):
        progress("%s ..." % name)
        t0 = time.perf_counter()
        r = fn()
        legs[name] = round(time.perf_counter() - t0, 2)
        return r
    weak = world > 1 and not args.strong
    R_weak = int(round(args.resolution * world ** (1.0 / 3.0)))
    main_run = leg("headline", lambda: run(R_weak if weak else args.resolution, args.steps, args.warmup, gather=True))
    side_run = None
    if world > 1:
        side_run = leg("side", lambda: run(args.resolution if weak else R_weak, args.steps, args.warmup, gather=True))
    r256 = leg("r256", lambda: run(256, args.steps, args.warmup)) if (not args.skip_256 and args.resolution != 256 and world == 1) else None
    # a dense-surface data point: config 2's scene (sphere u rabbit, ~1.5 M vertices) at the same R
    rdense = None if (args.skip_256 or world > 1) else leg("union_scene", lambda: run(
        args.resolution, args.steps, args.warmup, scene=(scenes.union_sphere_cube(), scenes.mc_settings(args.resolution, 1.0))))

    # serving throughput: P independent builds of the config-4 object, each with its own engine
    # (buffers) on its own HIP stream, the P-stream step replayed as one hipGraph.  Every kernel of
    # one build is latency-bound (few waves per SIMD, dependent memory round trips), so builds
    # overlap.  Every build recomputes everything; each one's mesh is checked against the first.
    def run_concurrent(R, P, steps):
        shape, mc = scenes.config4(R)
        slabs = [I.Slab(shape, mc) for _ in range(P)]
        try:
            streams = [torch.cuda.Stream(dev) for _ in range(P)]
            ev_start, ev_end = torch.cuda.Event(), [torch.cuda.Event() for _ in range(P)]
            main_s = torch.cuda.current_stream(dev)

            def step(ms):
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
                for _ in range(4):
                    step(main_s)
                jit_wait(I)
            torch.cuda.synchronize(dev)
            if any(sl.counts(0)[2] for sl in slabs):   # the first call sized the outputs
                step(main_s)
            torch.cuda.synchronize(dev)
            graph = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream(dev)
            cs.wait_stream(main_s)
            with torch.cuda.stream(cs):
                graph.capture_begin()
                step(cs)
                graph.capture_end()
            main_s.wait_stream(cs)
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                graph.replay()
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) / steps * 1e3 / P
            meshes = []
            for sl in slabs:
                nv, nf, of = sl.counts(0)
                if of:
                    raise RuntimeError("concurrent builds: output overflow")
                meshes.append(sl.download(nv, nf, 0))
            v0, f0 = meshes[0]
            same = all(v.shape == v0.shape and f.shape == f0.shape and np.array_equal(v.view(np.uint32), v0.view(np.uint32))
                       and np.array_equal(f, f0) for v, f in meshes[1:])
            return {"resolution": R, "builds": P, "ms_per_build": round(ms, 4),
                    "value": round(R ** 3 / (ms * 1e-3) / 1e6, 2), "unit": "Mvoxels/s",
                    "verts": int(len(v0)), "faces": int(len(f0)), "meshes_identical": bool(same)}
        finally:
            for sl in slabs:
                sl.close()
    conc = None
    if world == 1 and not args.skip_concurrent:
        conc = leg("concurrent", lambda: [run_concurrent(args.resolution, 4, args.steps)] +
                   ([] if args.skip_256 or args.resolution == 256 else [run_concurrent(256, 8, args.steps)]))

    # config 5: a stream of 64 seeded random MP5 objects at 128^3, eval + MC, each object's
    # pipeline captured once in a hipGraph and replayed (objects round-robin over a few streams).
    # Headline: the interpreter kernels (no per-object compilation, so nothing is left out of the
    # rate); beside it the JIT tier, whose hipRTC time for the 64 shapes is reported and folded
    # into an objects/s over one pass that includes it.
    def run_batch(objs, jit_mode, n_streams):
        I.set_jit(jit_mode)
        setup_cold = None
        # the objects arrive as JSON text, the form the reference's polygonize entry takes them in
        # (the generator's dicts serialised before the clock starts)
        texts = [json.dumps(o[0]) for o in objs]
        try:
            t0 = time.perf_counter()
            batch = I.Batch(texts, objs[0][1], n_streams=n_streams)
            setup_s = time.perf_counter() - t0
            if n_streams == 0:
                # merged launches: the stream's next batch of objects in this process -- created again,
                # every object parsed, set up and run once -- with the device-memory pool holding the
                # previous batch's buffers (the serving steady state); the first creation is reported
                # beside it (its buffers come from hipMalloc)
                batch.close()
                setup_cold = setup_s
                t0 = time.perf_counter()
                batch = I.Batch(texts, objs[0][1], n_streams=n_streams)
                setup_s = time.perf_counter() - t0
        finally:
            I.set_jit(2)
        for _ in range(max(1, args.warmup)):
            batch.run(sp)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            batch.run(sp)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        tv = tf = 0
        for i in range(batch.n):
            a, b_, of = batch.counts(i)
            if of:
                raise RuntimeError("config 5: object %d overflowed" % i)
            tv, tf = tv + a, tf + b_
        ms5 = el / args.steps * 1e3
        res = {"objects_per_s": round(batch.n / (ms5 * 1e-3), 1), "value": round(batch.n * 128 ** 3 / (ms5 * 1e-3) / 1e6, 2),
               "unit": "Mvoxels/s", "ms_per_stream": round(ms5, 4), "graphs": batch.graphs, "merged": batch.merged,
               "verts": tv, "faces": tf,
               "setup_s": round(setup_s, 4), "jit_compile_s": round(batch.jit_seconds, 2),
               "objects_per_s_incl_setup": round(batch.n / (ms5 * 1e-3 + setup_s), 1)}
        if setup_cold is not None:
            res["setup_s_first_batch"] = round(setup_cold, 4)
            res["objects_per_s_incl_setup_first_batch"] = round(batch.n / (ms5 * 1e-3 + setup_cold), 1)
            res["setup_note"] = ("setup_s: implisolid_batch_create of the 64 objects (JSON text) as the stream's next "
                                 "batch in this process (programs parsed, engines set up, one merged pass sizing the outputs; the "
                                 "device-memory pool serves the previous batch's buffers); setup_s_first_batch: the "
                                 "process's first batch (buffers from hipMalloc)")
        n_streams = batch.n_streams
        batch.close()
        return res, n_streams

    # N > 1: the OB02 loop on Z-slabs (config 3 on the shifted box, live projection, at 256^3): the
    # slabs' MC meshes all-gathered to every rank, then resampling / projection / QEM per owned vertex
    # range with the owned vertices all-gathered after each vertex-moving step
    # (distributed.ob02_sharded); wall time of the loop (max over ranks) and parity of rank 0's mesh
    # against the oracle's committed summary
    ob02_sharded = None
    if world > 1 and not args.skip_ob02:
        def run_ob02_sharded(Re=256):
            shape, mc = scenes.config3_shifted(Re)
            cuts = D.balanced_cuts(shape, mc, world)
            slab = I.Slab(shape, mc, rank, world, cuts=cuts)
            cnt = torch.zeros(4, dtype=torch.int32, device=dev)
            gath = torch.zeros(world, 4, dtype=torch.int32, device=dev)
            for _ in range(2):   # the second pass runs with outputs sized by the first
                slab.eval(sp); slab.count(sp); slab.counts(sp)
                slab.copy_counts(cnt.data_ptr(), sp)
                torch.cuda.synchronize(dev)
                work = D.gather_counts_async(cnt, gath)
                slab.emit_verts(sp)
                if work is not None:
                    work.wait()
                torch.cuda.synchronize(dev)
                slab.emit_faces(0, gath.data_ptr(), rank, sp)
                slab.counts(sp)
            V, F, voff, foff = D.allgather_mesh(slab, gath, rank, world, dev)
            slab.close()
            res = None
            for _ in range(4):   # warm: the shard's point modules (baked once hot, as in the ob02 leg)
                D.ob02_sharded(shape, mc, V, F, voff, rank, world)
            jit_wait(I)
            times = []
            for _ in range(3):
                dist.barrier()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                res = D.ob02_sharded(shape, mc, V, F, voff, rank, world)
                t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                times.append(float(t.item()))
            out_ = {"workload": "config %s on the shifted box (scenes.config3_shifted) at %d^3: MC on %d balanced Z-slabs, "
                                "then 3 x [resample, project, QEM] sharded by owned vertex ranges"
                                % ("3" if Re == 256 else "4", Re, world),
                    "ob02_ms": round(min(times) * 1e3, 3), "verts": int(V.numel() // 3), "faces": int(F.numel() // 3),
                    "owned_verts": [int(voff[r + 1] - voff[r]) for r in range(world)]}
            if rank == 0:
                out_["parity"] = headline_parity("config3s_ob02_r256" if Re == 256 else "config4s_ob02_r512", *res)
            return out_
        try:
            ob02_sharded = leg("ob02_sharded", run_ob02_sharded)
        except Exception as exc:   # reported, never the reason the bench line is lost
            ob02_sharded = {"error": repr(exc)[:300]}
        try:   # config 4's size
            ob02_sharded["r512"] = leg("ob02_sharded_r512", lambda: run_ob02_sharded(512))
        except Exception as exc:
            ob02_sharded["r512"] = {"error": repr(exc)[:300]}
        D.release_shards()   # the kept shard handles' streams and buffers are not the later legs'

    # N = 1: the sharded OB02 loop's 8-rank critical path, estimated on this GPU: config 3
    # on the shifted box at 256^3, its MC mesh owned by the 8 balanced slabs' vertex ranges, every
    # shard stepped one at a time (distributed.ob02_shards_local, HIP events on the shard's stream)
    # with the exchanges of distributed.ob02_plan as device copies.  The 8-rank loop time is the sum
    # over steps of the slowest shard, plus the exchanges priced by a stated model (the all-gather's
    # bytes over xGMI); the same loop on one shard is the single-GPU figure beside it.
    ob02_est = None
    if world == 1 and not args.skip_ob02:
        def run_ob02_estimate(Re=256, n=8):
            from implisolid_amd import distributed as D
            shape, mc = scenes.config3_shifted(Re)
            cuts = D.balanced_cuts(shape, mc, n)
            nvs = []
            for r in range(n):
                sl = I.Slab(shape, mc, r, n, cuts=cuts)
                nvs.append(sl.run()[0])
                sl.close()
            mc_only = dict(mc, vresampl={"iters": 0, "c": 1.0}, projection={"enabled": 0}, qem={"enabled": 0},
                           subdiv={"enabled": 0})
            v_mc, f_mc = I.make_geometry(shape, mc_only)
            assert sum(nvs) == len(v_mc)
            V = torch.from_numpy(v_mc.reshape(-1).copy()).to(dev)
            F = torch.from_numpy(f_mc.reshape(-1).copy()).to(dev)
            voff = np.concatenate([[0], np.cumsum(nvs)]).astype(np.int64)
            for _ in range(4):   # warm: point modules (baked once hot, as in the ob02 leg), tables
                D.ob02_shards_local(shape, mc, V, F, voff, timing=True)
            jit_wait(I)
            v, f, st8 = D.ob02_shards_local(shape, mc, V, F, voff, timing=True)
            _, _, st1 = D.ob02_shards_local(shape, mc, V, F, [0, len(v_mc)], timing=True)
            crit = sum(max(x["shard_ms"]) for x in st8["steps"])
            one = sum(max(x["shard_ms"]) for x in st1["steps"])
            # exchange model: RCCL all-gather / p2p on one node, 25 us per exchange + the bytes a rank
            # receives at 50 GB/s (a conservative share of its xGMI links; not measured here)
            nbytes = st8["exchange_bytes"]
            per_rank = [b / n for b in nbytes]
            ex_ms = sum(0.025 + pb / 50e9 * 1e3 for pb in per_rank)
            return {"workload": "config %s on the shifted box (scenes.config3_shifted) at %d^3, 3 x [resample, project, "
                                "QEM], the MC mesh's vertices owned by the 8 balanced Z-slabs" % ("3" if Re == 256 else "4", Re),
                    "shards": n, "owned_verts": nvs, "steps": [x["step"] + ":" + str(x["exchange"]) for x in st8["steps"]],
                    "loop_compute_ms_8": round(crit, 4), "loop_compute_ms_1": round(one, 4),
                    "step_max_ms": [max(x["shard_ms"]) for x in st8["steps"]],
                    "attach_ms_max_8": max(st8["attach_ms"]), "attach_ms_1": st1["attach_ms"][0],
                    "exchange_bytes_per_rank": [round(b) for b in per_rank],
                    "exchange_model_ms": round(ex_ms, 4),
                    "exchange_model": "25 us latency per exchange + received bytes at 50 GB/s per rank (a model, not "
                                      "measured: one GPU here)",
                    "estimate_ms_8": round(crit + ex_ms + max(st8["attach_ms"]), 4),
                    "single_ms": round(one + st1["attach_ms"][0], 4),
                    "parity": headline_parity("config3s_ob02_r256" if Re == 256 else "config4s_ob02_r512", v, f)}
        try:
            ob02_est = leg("ob02_sharded_estimate", run_ob02_estimate)
        except Exception as exc:   # an estimate, never the reason the bench line is lost
            ob02_est = {"error": repr(exc)[:300]}
        try:   # config 4's size: the 512^3 mesh
            ob02_est["r512"] = leg("ob02_sharded_estimate_r512", lambda: run_ob02_estimate(512))
        except Exception as exc:
            ob02_est["r512"] = {"error": repr(exc)[:300]}
        from implisolid_amd import distributed as D_
        # the 16 kept shard handles hold 32 HIP streams; left alive, they crowded the process's
        # hardware queues and the config-5 leg's two pipelines ran 0.85 instead of 0.50 ms per pass
        D_.release_shards()

    c5 = None
    if world == 1 and not args.skip_config5:
        objs = scenes.config5_objects(64, 128)
        c5, _ = leg("config5_merged", lambda: run_batch(objs, 0, 0))
        c5["workload"] = ("config5: 64 seeded random MP5 objects (scenes.config5_objects, 1-12 leaves) at 128^3, eval+MC, "
                          "interpreter kernels (no per-object compilation), merged launches: each stage once for all "
                          "64 objects")
        c5["graphs_interpreter"], _ = leg("config5_graphs_interpreter", lambda: run_batch(objs, 0, args.config5_streams))
        c5["jit"], ns5 = leg("config5_graphs_jit", lambda: run_batch(objs, 1, args.config5_streams))
        c5["jit"]["workload"] = "JIT tree kernels, hipGraph per object over %d streams" % ns5

    # First-call latency of a never-seen shape (async JIT: the interpreter kernels run at once, the
    # module compiles in the background): build_geometry (eval + MC, host-resident result) of fresh
    # random trees at R 32 and 128, against the oracle on one host core for the same call
    first = None
    progress("first_call ...")
    t_leg = time.perf_counter()
    if world == 1 and not args.skip_ob02:
        import oracle
        oracle.build()
        first = {}
        for k, Rf in enumerate((32, 128)):
            shape = scenes.random_tree(990001 + k, 10)
            mc = scenes.mc_settings(Rf, 1.0)
            t0 = time.perf_counter()
            v, f = I.make_geometry(shape, mc)
            t_gpu = time.perf_counter() - t0
            t0 = time.perf_counter()
            vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
            t_cpu = time.perf_counter() - t0
            first["r%d" % Rf] = {"gpu_first_call_ms": round(t_gpu * 1e3, 3), "cpu_oracle_ms": round(t_cpu * 1e3, 3),
                                 "faces_identical": bool(np.array_equal(f, fr)),
                                 "verts_identical": bool(np.array_equal(v.view(np.uint32), vr.view(np.uint32)))}
        jit_wait(I)
        first["jit"] = I.jit_stats()
        legs["first_call"] = round(time.perf_counter() - t_leg, 2)

    # end-to-end build_geometry of the config-4 tree (eval + MC) through the C ABI,
    # to a host-resident mesh (PCIe included), at 256^3 and 512^3 -- the reference's unit of work
    e2e = None
    progress("end_to_end ...")
    t_leg = time.perf_counter()
    if world == 1 and not args.skip_ob02:
        e2e = {}
        for Re in (256, 512):
            shape, mc = scenes.config4(Re)
            # warm: the object turns hot after a few builds (bake mode 2) and its baked module
            # compiles on host threads; builds timed beside that compile read up to 2x slower
            # (BENCH_r03: median 1.89 vs min 0.92 ms), so the timed builds start once it is loaded
            for _ in range(2):
                for _ in range(5):
                    I.make_geometry(shape, mc)
                jit_wait(I)
            # the C ABI as the reference's front end uses it (implisolid_main.js:227-237): build_geometry,
            # then the mesh read through get_v_ptr / get_f_ptr in the library's (pinned) result buffers
            # (build_geometry_views_ms; build_geometry_copy_out_ms adds get_v / get_f copies)
            ts = []
            for _ in range(7):
                t0 = time.perf_counter()
                v, f = I.make_geometry_views(shape, mc)
                ts.append(time.perf_counter() - t0)
            par = headline_parity("config4_mc_r%d" % Re, v, f)
            # ... and with the mesh copied out into fresh numpy arrays (get_v / get_f)
            tc = []
            for _ in range(7):
                t0 = time.perf_counter()
                v, f = I.make_geometry(shape, mc)
                tc.append(time.perf_counter() - t0)
            e2e["r%d" % Re] = {"build_geometry_views_ms": round(min(ts) * 1e3, 3), "median_ms": round(float(np.median(ts)) * 1e3, 3),
                               "mvoxels_per_s": round(Re ** 3 / min(ts) / 1e6, 1), "verts": int(len(v)), "faces": int(len(f)),
                               "build_geometry_copy_out_ms": round(min(tc) * 1e3, 3),
                               "parity": par, "parity_copy_out": headline_parity("config4_mc_r%d" % Re, v, f)}
        legs["end_to_end"] = round(time.perf_counter() - t_leg, 2)

    # configs 2 and 3 through the C ABI: build_geometry (MC + 3 x [resample, project, QEM]) to a
    # host-resident mesh, PCIe included; the oracle times config 2 on one host core beside it
    ob02 = None
    progress("ob02 ...")
    t_leg = time.perf_counter()
    # config 3 on its dyadic box keeps every centroid (NaN average edge length from the reference's
    # NaN normals at a singular sample); on the box shifted by 0.003 the alpha
    # search and bisection run on every face (config3s)
    ob02_legs = (("config2_r128", scenes.config2(128)), ("config3_r256", scenes.config3(256)),
                 ("config3s_r256", scenes.config3_shifted(256)), ("config4s_r512", scenes.config3_shifted(512)))
    # the oracle takes ~60 s for the 512^3 loop: that leg is checked against the committed summary
    # of the same workload (tests/golden/make_headline.py config4s_ob02_r512) instead of a live run
    ob02_summary = {"config4s_r512": "config4s_ob02_r512"}
    if world == 1 and not args.skip_ob02:
        ob02 = {}
        for key, (shape, mc) in ob02_legs:
            # the first build of the shape: its tree modules compile in the background (interpreter
            # kernels meanwhile) and the projection's perturbation table is drawn for this face count
            t0 = time.perf_counter()
            I.make_geometry(shape, mc)
            t_first = time.perf_counter() - t0
            jit_wait(I)
            # the steady state of a hot object (refined build after build): after 4 builds its brick
            # and point modules are rebuilt with its matrices baked in (implisolid_set_jit_bake's
            # default), compiled in the background; wait for them
            for _ in range(4):
                I.make_geometry(shape, mc)
            jit_wait(I)
            I.make_geometry(shape, mc)
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                v, f = I.make_geometry(shape, mc)
                ts.append(time.perf_counter() - t0)
            # the same build with the mesh read in place (get_v_ptr / get_f_ptr, the reference front
            # end's reads, implisolid_main.js:227-237) instead of copied into fresh arrays
            tv = []
            for _ in range(3):
                t0 = time.perf_counter()
                I.make_geometry_views(shape, mc)
                tv.append(time.perf_counter() - t0)
            ob02[key] = {"build_geometry_ms": round(min(ts) * 1e3, 3), "build_geometry_views_ms": round(min(tv) * 1e3, 3),
                         "first_build_ms": round(t_first * 1e3, 3),
                         "verts": int(len(v)), "faces": int(len(f)),
                         "steps": "MC + 3 x [vertex resampling, centroid projection, QEM]",
                         "note": "build_geometry_ms: the mesh copied into fresh arrays (get_v / get_f); "
                                 "build_geometry_views_ms: read in place (get_v_ptr / get_f_ptr)"}
            if key in ob02_summary:
                ob02[key]["parity"] = headline_parity(ob02_summary[key], v, f)
            # one profiled build (stream drained at every stage boundary): per-stage times, the
            # projection's evaluation count, and SURVEY.md 8d's per-iteration algorithmic bytes over them
            # (resample 60 F + 28 V, project (24 + 12 k) F with k evaluations per face, QEM (12 + 36 deg) V)
            I.ob02_profile(True)
            try:
                I.make_geometry(shape, mc)
                st = I.last_build_stats()
            finally:
                I.ob02_profile(False)
            reps = mc["overall_repeats"]
            F, V = len(f), len(v)
            sm = st["stage_ms"]
            k_ev = st["projection_evals"] / max(1, F * reps)
            alg = {"resample": reps * (60.0 * F + 28.0 * V), "project": reps * (24.0 + 12.0 * k_ev) * F,
                   "qem": reps * (12.0 + 36.0 * 6.0) * V}
            ob02[key]["profile"] = {
                "stage_ms": {k: round(x, 4) for k, x in sm.items()},
                "projection_evals": st["projection_evals"], "evals_per_face_per_repeat": round(k_ev, 2),
                "projection_gevals_per_s": round(st["projection_evals"] / max(1e-9, sm["project"] * 1e-3) / 1e9, 3),
                "alg_gbs": {k: round(b / max(1e-9, sm[k] * 1e-3) / 1e9, 2) for k, b in alg.items()},
                "bisection_cap_hits": st["bisection_cap_hits"], "jit_point_launches": st["jit_launches"],
                "note": "profiled build: the stream is drained at each stage boundary (edge_fold includes the "
                        "projection's prep pass, which overlaps the host fold in unprofiled builds)"}
        ob02["config3s_r256"]["workload"] = "config 3 with its box shifted by 0.003 (scenes.config3_shifted): finite average edge length, live alpha search + bisection"
        ob02["config4s_r512"]["workload"] = ("config 4: the same tree at 512^3 on the shifted box, the same loop; parity "
                                             "against the oracle's committed summary (the oracle ran %.1f s for it "
                                             "in the build container, one core)" % json.load(open(os.path.join(
                                                 ROOT, "tests", "golden", "headline_summaries.json")))["config4s_ob02_r512"]["oracle_s"])
        legs["ob02"] = round(time.perf_counter() - t_leg, 2)
        if not args.no_cpu_baseline:
            # the oracle runs every configuration on this host: its time on one core, and max|v - v_ref|
            # and face identity of the GPU result against it
            import oracle
            oracle.build()
            progress("ob02_cpu_oracle ...")
            t_leg = time.perf_counter()
            for key, (shape, mc) in ob02_legs:
                if key in ob02_summary:
                    continue
                v, f = I.make_geometry(shape, mc)
                t0 = time.perf_counter()
                v_ref, f_ref = oracle.polygonize(json.dumps(shape), json.dumps(mc))
                ob02[key]["cpu_oracle_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
                ob02[key]["parity"] = mesh_parity(v, f, v_ref, f_ref)
            legs["ob02_cpu_oracle"] = round(time.perf_counter() - t_leg, 2)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    R = main_run["R"]
    ms = main_run["elapsed"] / args.steps * 1e3
    value = R ** 3 / (ms * 1e-3) / 1e6
    kms = main_run["kernels_ms"]
    kern = main_run["kernel_ms"]
    _, n_instr, depth = program_flops(main_run["shape"])
    # rank-0 slab: stored samples (n = R+3 per axis incl. the sealed ring), cells, bricks
    n_side = R + 3
    samples = n_side * n_side * (main_run["fz"][1] - main_run["fz"][0])
    cells = (R + 2) ** 2 * main_run["slab_layers"]
    bricks_total, bricks_mixed, bricks_filled = main_run["bricks"]
    nv, nf = main_run["nv"], main_run["nf"]
    # Roofline (task contract 4).  The dominant kernel is the one with the largest
    # average duration (engine HIP events on the launch stream, 5 extra steps after the timed
    # region: Slab.kernel_times_each).  Its `achieved` = its ALGORITHMIC bytes per launch over that
    # duration; algorithmic bytes per kernel:
    #   impli_eval_bricks  4 B per evaluated sample (the listed + claimed bricks x 128 samples)
    #   k_brick_fill       the sign bitmap of the grid, 1 bit per stored sample
    #   k_mc_cells         20 B per vertex: its 12 B position + the 2 x 4 B field values of its edge
    #   k_mc_faces         12 B per face
    # (the interval passes, count and scan produce only per-box / per-unit metadata: no figure).
    # `traffic` = that kernel's HBM bytes per launch from the committed PMC summary
    # (tools/profile_round.sh; FETCH_SIZE x2 and WRITE_SIZE calibrated as MI355X_MICROARCH.md
    # prescribes), with `traffic_current` saying whether it was taken on this very library.
    # Beside it, the pass: the counter bytes of all eight kernels and SURVEY.md 8d's
    # dense-equivalent bytes B = 8 (R+1)^3 + 12 V + 12 F over the kernel sequence's time.
    b_pipe = (8.0 * (R + 1) ** 3 + 12.0 * nv + 12.0 * nf) / world
    t_kern = sum(kms.values()) * 1e-3
    each = main_run["each_ms"]
    dom = max(each, key=each.get)
    # the newest committed PMC summaries (tools/profile_round.sh <tag> -> profiles/traffic_<tag>.json,
    # profiles/valu_<tag>.json), if they were taken on this workload
    import glob
    import hashlib

    def tag_key(path):   # r03w < r03z < r03aa < r03ab: round, then suffix length, then suffix
        m = re.match(r"\D*_r(\d+)([a-z]*)\.json$", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")

    lib_sha = hashlib.sha256(open(I.LIB_PATH, "rb").read()).hexdigest()

    def newest(pattern, prefer_sha=None):
        fs = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=tag_key)
        docs = []
        for f in fs:
            try:
                docs.append((os.path.basename(f), json.load(open(f))))
            except Exception:
                pass
        if prefer_sha:   # the profile of this very library, if one is committed
            for name, doc in reversed(docs):
                if isinstance(doc, dict) and doc.get("lib_sha256") == prefer_sha:
                    return name, doc
        return docs[-1] if docs else (None, None)
    tname, tj = newest("traffic_r*.json", lib_sha)
    if not (tj and tj.get("workload_R") == R and tj.get("tree_seed") == scenes.CONFIG3_SEED):
        tname, tj = None, None
    traffic_current = bool(tj and tj.get("lib_sha256") == lib_sha)
    vname, vj = newest("valu_r*.json")
    if tname:   # the VALU pass of the same profiling run as the traffic, when there is one
        vpath = os.path.join(ROOT, "profiles", tname.replace("traffic_", "valu_"))
        if os.path.exists(vpath):
            vname, vj = os.path.basename(vpath), json.load(open(vpath))
    traffic = tj.get("pipeline_bytes") if tj else None
    k_traffic = {k: v["bytes"] for k, v in tj.get("kernels", {}).items()} if tj else {}
    valu = vj.get("kernels", {}) if vj else {}
    evaluated = (bricks_total - bricks_filled) * 128
    alg = {"impli_eval_bricks": 4.0 * evaluated, "k_brick_fill": samples / 8.0,
           "k_mc_cells": 20.0 * nv / world, "k_mc_faces": 12.0 * nf / world}
    per_kernel = {}
    for k, ms_k in each.items():
        row = {"ms": round(ms_k, 4)}
        if k in alg:
            row["alg_bytes"] = round(alg[k])
            row["alg_gbs"] = round(alg[k] / (ms_k * 1e-3) / 1e9, 1)
            row["alg_frac"] = round(row["alg_gbs"] / HBM_PEAK_GBS, 4)
        if k in k_traffic:
            row["traffic"] = k_traffic[k]
            row["traffic_gbs"] = round(k_traffic[k] / (ms_k * 1e-3) / 1e9, 1)
            row["traffic_frac"] = round(row["traffic_gbs"] / HBM_PEAK_GBS, 4)
            if k in alg:
                row["traffic_over_alg"] = round(k_traffic[k] / max(1.0, alg[k]), 2)
        if k in valu:
            row["valu_busy"] = valu[k].get("valu_busy")
            if "valu_insts_per_wave" in valu[k] and "waves_per_dispatch" in valu[k]:
                # VALU issue roofline: wave instructions x 2 cycles each (a wave64 VALU op on a SIMD-32,
                # MI355X_MICROARCH.md) over the 1024 SIMDs x 2.4 GHz for the kernel's time -- a lower
                # bound of the VALU pipe's occupancy (f64 and transcendental ops take longer)
                row["valu_issue_frac"] = round(valu[k]["valu_insts_per_wave"] * valu[k]["waves_per_dispatch"] * 2.0
                                               / (1024 * 2.4e9 * ms_k * 1e-3), 4)
        per_kernel[k] = row
    for k, v in main_run["repeat_ms"].items():
        per_kernel[k]["ms_repeated_launches"] = round(v, 4)
    dom_alg = alg.get(dom)
    # the dominant kernel's duration: from 20 back-to-back launches where it is idempotent
    # (emission kernels), else from the per-kernel events
    dom_ms = main_run["repeat_ms"].get(dom, each[dom])
    achieved = dom_alg / (dom_ms * 1e-3) / 1e9 if dom_alg else None
    pass_achieved = traffic / t_kern / 1e9 if traffic else None
    out = {
        "metric": "Mvoxels/s (eval+MC) at 256^3 & 512^3",
        "value": round(value, 2),
        "unit": "Mvoxels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": "config4: seeded ~20-node MP5 CSG tree with twist/union/difference (scenes.config4, seed 20251015), box [-1,1]^3, "
                        "R=%d, eval+MC, mesh resident in HBM%s" % (
                            R, (", weak scaling: R = %d N^(1/3), ~%d^3 voxels per rank" % (args.resolution, args.resolution))
                            if weak else (", strong scaling: the grid over %d balanced Z-slabs" % world) if world > 1 else ""),
            "resolution": R, "voxels": R ** 3, "samples": (R + 1) ** 3, "cells": (R + 2) ** 3,
            "verts": nv, "faces": nf, "program_instr": n_instr, "tree_depth": depth,
            "parallelism": "zslab%d" % world,
            "voxels_per_rank": R ** 3 // world,
        },
        "kernels_ms": {k: round(v, 4) for k, v in kms.items()},
        "kernel_ms": {k: round(v, 4) for k, v in kern.items()},
        "kernel_ms_each": {k: round(v, 4) for k, v in main_run["each_ms"].items()},
        "eval_kernel": {"shape": "jit", "baked": "jit (object's module, matrices as literals)"}.get(
            main_run["jit_module"], "interpreter"),
        "launch": "hipGraph replay of the step" if main_run["graph"] else "direct launches",
        "bricks": {"total": bricks_total, "mixed": bricks_mixed, "sign_filled": bricks_filled,
                   "evaluated_sample_frac": round(1.0 - bricks_filled / max(1, bricks_total), 4),
                   "mixed_coarse_boxes": main_run["stats"]["mixed_coarse_boxes"]},
        "mc": {"units": main_run["stats"]["units"], "nonempty_units": main_run["stats"]["nonempty_units"],
               "active_cells": main_run["stats"]["act"]},
        # bound: what the counters show.  The path is elementwise / scan / gather work priced against
        # HBM (roofline_class), but every kernel of the pruned pass is latency- or issue-bound:
        # the pass moves 0.14 of peak by its counter bytes (pass_frac) and the dominant kernel's
        # VALU is mostly idle
        "roofline": {"bound": "latency", "roofline_class": "hbm", "kernel": dom, "dominant_kernel": dom,
                     "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": k_traffic.get(dom), "traffic_source": tname, "traffic_current": traffic_current,
                     "alg_bytes_per_launch": round(dom_alg) if dom_alg else None, "launch_ms": round(dom_ms, 4),
                     "launch_ms_method": "20 back-to-back launches between two HIP events on the launch stream"
                                         if dom in main_run["repeat_ms"] else "HIP events around the kernel on the launch stream",
                     "limiter": "latency: dependent memory round trips at few waves per SIMD (DESIGN.md section 3)",
                     "valu_source": vname,
                     "per_kernel": per_kernel,
                     "kernel_share": {k: round(v / max(1e-9, sum(each.values())), 3) for k, v in each.items()},
                     "pass_frac": round(pass_achieved / HBM_PEAK_GBS, 4) if pass_achieved else None,
                     "pass_frac_note": "the whole eval+MC pass: PMC counter bytes of its kernels over their time "
                                       "(the honest pass figure; pass.effective_frac is the dense-equivalent, > 1)",
                     "pass": {"kernels": "the eval+MC kernel sequence (8 kernels), HIP events around eval / count+scan / emit",
                              "launch_ms": round(t_kern * 1e3, 4), "traffic": traffic,
                              "achieved": round(pass_achieved, 1) if pass_achieved else None,
                              "frac": round(pass_achieved / HBM_PEAK_GBS, 4) if pass_achieved else None,
                              "effective_bytes": b_pipe, "effective_achieved": round(b_pipe / t_kern / 1e9, 1),
                              "effective_frac": round(b_pipe / t_kern / 1e9 / HBM_PEAK_GBS, 4),
                              "effective_note": "SURVEY.md 8d's dense-equivalent bytes 8 (R+1)^3 + 12 V + 12 F; the pruned "
                                                "pass never moves most of them, so this is not a roofline fraction"}},
    }
    if world > 1:
        out["slabs"] = {"cuts": main_run["cuts"], "balanced": main_run["cuts"] is not None,
                        "cut_probe_s": round(main_run["cut_s"], 4), "rank_ms": main_run.get("rank_ms"),
                        "max_over_min": round(max(main_run["rank_ms"]) / max(1e-9, min(main_run["rank_ms"])), 3)}
        if "gather_ms" in main_run:
            out["gather_ms"] = main_run["gather_ms"]
        if "parity" in main_run:
            out["parity"] = main_run["parity"]
    if side_run:
        mss = side_run["elapsed"] / args.steps * 1e3
        out["strong" if weak else "weak"] = {
            "resolution": side_run["R"], "value": round(side_run["R"] ** 3 / (mss * 1e-3) / 1e6, 2),
            "ms_per_step": round(mss, 4), "scaling": "strong" if weak else "weak",
            "rank_ms": side_run.get("rank_ms"), "cuts": side_run["cuts"]}
        for k in ("gather_ms", "parity"):
            if k in side_run:
                out["strong" if weak else "weak"][k] = side_run[k]
    if rdense:
        msd = rdense["elapsed"] / args.steps * 1e3
        out["value_union_scene"] = round(R ** 3 / (msd * 1e-3) / 1e6, 2)
        out["union_scene"] = {"workload": "config 2 scene (sphere u rabbit) at R=%d, eval+MC" % R, "ms_per_step": round(msd, 4),
                              "verts": rdense["nv"], "faces": rdense["nf"],
                              "kernel_ms": {k: round(v, 4) for k, v in rdense["kernel_ms"].items()}}
    if r256:
        ms256 = r256["elapsed"] / args.steps * 1e3
        out["value_256"] = round(256 ** 3 / (ms256 * 1e-3) / 1e6, 2)
        out["ms_per_step_256"] = round(ms256, 4)
    if conc:
        out["concurrent_builds"] = {
            "workload": "P independent builds of the config-4 object (own engine each) on P HIP streams, "
                        "the P-stream step replayed as one hipGraph: serving throughput, every build "
                        "recomputed (the headline above is one build at a time)",
            "runs": conc}
    if c5:
        out["config5"] = c5
    if ob02:
        out["ob02"] = ob02
    if ob02_sharded:
        out["ob02_sharded"] = ob02_sharded
    if ob02_est:
        out["ob02_sharded_estimate"] = ob02_est
    if e2e:
        out["end_to_end"] = dict(e2e, workload="config4 tree, build_geometry (eval + MC) to host-resident verts/faces: "
                                               "build_geometry_views_ms = the ABI call with the mesh read through get_v_ptr / "
                                               "get_f_ptr (the reference front end's path, no copy); "
                                               "build_geometry_copy_out_ms adds get_v / get_f copies into fresh arrays")
    if first:
        out["first_call"] = dict(first, workload="never-seen random 10-leaf trees, build_geometry eval+MC, "
                                                 "async JIT (interpreter kernels on the first call)")
    if world == 1 and not args.no_cpu_baseline:
        progress("cpu_baseline ...")
        t0 = time.perf_counter()
        out["cpu_baseline"], (Rs, v_ref, f_ref) = cpu_baseline(main_run["shape"])
        legs["cpu_baseline"] = round(time.perf_counter() - t0, 2)
        # the GPU mesh of the same tree at the sample's resolution against the oracle's
        v, f = I.make_geometry(main_run["shape"], scenes.mc_settings(Rs, 1.0))
        out["parity"] = dict(mesh_parity(v, f, v_ref, f_ref), resolution=Rs,
                             workload="config4 tree, eval+MC: GPU (build_geometry) vs the oracle")
    else:
        out["cpu_baseline"] = None
    if c5 and not args.no_cpu_baseline:
        progress("config5_cpu_baseline ...")
        t0 = time.perf_counter()
        c5["cpu_baseline"] = config5_cpu_baseline()
        legs["config5_cpu_baseline"] = round(time.perf_counter() - t0, 2)
    out["roofline"]["copy_attainable"] = copy_attainable(dev)
    out["legs_wall_s"] = dict(legs, total=round(time.perf_counter() - T_START, 2))
    # child processes still alive at the end (the config-5 CPU workers are reaped; the driver has
    # reported one process left behind after the bench): named here, if any
    try:
        import psutil
        out["children_at_exit"] = [" ".join(c.cmdline()[:3]) for c in psutil.Process().children(recursive=True)]
    except Exception as exc:   # psutil missing or a child gone mid-listing
        out["children_at_exit"] = "unavailable: %s" % exc
    # the compact summary last, so a log's tail always holds it (the driver keeps the last 8 KB)
    summ = {"value": out["value"], "unit": out["unit"], "ms_per_step": out["ms_per_step"], "n_gpus": world,
            "scaling": out["scaling"], "dominant_kernel_frac": out["roofline"].get("frac")}
    for k in ("strong", "weak"):
        if k in out:
            summ[k] = {"value": out[k]["value"], "ms_per_step": out[k]["ms_per_step"]}
    if "config5" in out:
        c = out["config5"]
        summ["config5"] = {k: c.get(k) for k in ("objects_per_s", "objects_per_s_incl_setup",
                                                 "objects_per_s_incl_setup_first_batch", "ms_per_stream")}
    if "ob02" in out:
        summ["ob02_build_ms"] = {k: v.get("build_geometry_ms") for k, v in out["ob02"].items() if isinstance(v, dict)}
        summ["ob02_first_build_ms"] = {k: v.get("first_build_ms") for k, v in out["ob02"].items() if isinstance(v, dict)}
        summ["ob02_build_views_ms"] = {k: v.get("build_geometry_views_ms") for k, v in out["ob02"].items() if isinstance(v, dict)}
    if "ob02_sharded_estimate" in out:
        e = out["ob02_sharded_estimate"]
        summ["ob02_8shard_estimate_ms"] = {"r256": [e.get("estimate_ms_8"), e.get("single_ms")],
                                           "r512": [e.get("r512", {}).get("estimate_ms_8"), e.get("r512", {}).get("single_ms")]}
    out["summary"] = summ
    print(json.dumps(out), flush=True)
    print("bench summary: " + json.dumps(summ), file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
