"""Multi-GPU Z-slab numbering exchange (one process per GPU, torch.distributed over RCCL).

The only data-path exchange of the sharded polygoniser: after each rank has
counted its slab (``Slab.count``), every rank needs the number of vertices and faces emitted by
the ranks below it, so that its vertex ids and face rows continue the global z-major numbering of
the single-GPU result.  16 bytes per rank are all-gathered and reduced on the device; nothing
else crosses xGMI until the (optional) output gather.

Counts layout (``Slab.copy_counts``): int32 [own vertices incl. halo, faces, active cells,
halo-owned vertices].  A rank's emitted vertex count is own - halo.
"""
import torch
import torch.distributed as dist


def gather_counts(local_counts, world, group=None):
    """All-gather the per-rank int32[4] counts -> int32[world, 4] on the same device."""
    out = torch.empty(world, local_counts.numel(), dtype=local_counts.dtype, device=local_counts.device)
    if dist.get_backend(group) == "gloo":
        parts = list(out.unbind(0))
        dist.all_gather(parts, local_counts, group=group)
        return torch.stack(parts)
    dist.all_gather_into_tensor(out, local_counts, group=group)
    return out


def gather_counts_async(local_counts, out, group=None):
    """Start the all-gather of the per-rank counts into `out` (int32[world, 4], rank order);
    returns a work handle (wait() orders the caller's stream after it) or None when the backend
    completed it synchronously.  The face pass reads `out` directly (Slab.emit_faces
    d_gathered), so the vertex pass can run while the gather is in flight."""
    if dist.get_backend(group) == "gloo":
        parts = list(out.unbind(0))
        dist.all_gather(parts, local_counts, group=group)
        return None
    return dist.all_gather_into_tensor(out, local_counts, group=group, async_op=True)


def counts_tensor(slab, device):
    """The slab's totals block (its counter words [2, 6): own incl. halo, faces, active cells,
    halo own -- the copy_counts layout) as an int32[4] tensor over the engine's own memory, no copy
    (``__cuda_array_interface__``).  Valid while the slab lives; every count() rewrites it."""
    class _Totals:
        __cuda_array_interface__ = {"shape": (4,), "typestr": "<i4", "data": (slab.counters_ptr() + 8, False),
                                    "version": 3, "strides": None}
    return torch.as_tensor(_Totals(), device=device)


def gather_counts_inline(totals, out, group=None):
    """All-gather the per-rank counts into `out` (int32[world, 4]) on the caller's current stream
    (a blocking-style collective: RCCL enqueues it on the launch stream; the host does not wait).
    Measured on one MI355X (world 1, 1/8 of config 4 at 512^3, tools/step_host_probe.py): the
    async form on the process group's own stream with copy_counts cost 21.6 us per step over the
    kernels (cross-stream events), this one 5.3 us (profiles/r04d_step_host_probe.json)."""
    if dist.get_backend(group) == "gloo":   # gloo: host tensors round trip (tests on the CPU)
        parts = list(out.unbind(0))
        dist.all_gather(parts, totals, group=group)
        return
    dist.all_gather_into_tensor(out.view(-1), totals, group=group)


def offsets_from_counts(gathered, rank, out=None):
    """Exclusive prefix over ranks: int32 [vertex offset, face offset] for `rank` (on device)."""
    v = gathered[:, 0] - gathered[:, 3]
    f = gathered[:, 1]
    if out is None:
        out = torch.zeros(2, dtype=gathered.dtype, device=gathered.device)
    out[0] = v[:rank].sum()
    out[1] = f[:rank].sum()
    return out


def global_offsets(local_counts, rank, world, group=None, out=None):
    """gather_counts + offsets_from_counts; returns (offsets int32[2], gathered int32[world, 4])."""
    g = gather_counts(local_counts, world, group)
    return offsets_from_counts(g, rank, out), g


def balanced_cuts(shape, mc_settings, world):
    """Balanced Z-slab cuts for `world` ranks (implisolid_slab_balance): every rank runs the same
    interval pass of the whole grid on its own GPU and gets the same cuts, so the partition needs
    no exchange.  Pass them to ``Slab(..., rank, world, cuts=cuts)``."""
    import implisolid_amd as I
    return I.slab_balance(shape, mc_settings, world)


def gather_mesh(slab, gathered, rank, world, group=None, stream=0):
    """Gather every rank's emitted mesh to rank 0 in rank order (the multi-GPU result of the C ABI's
    build_geometry, mcc2.cpp:446-525).  `gathered` is the all-gathered counts tensor int32[world, 4]
    (gather_counts); the faces must have been emitted with global vertex ids (Slab.emit_faces with
    the gathered counts), so concatenation is the whole single-GPU mesh, byte for byte.

    RCCL: point-to-point device buffers (rank r sends its slab to rank 0 over xGMI; rank 0 receives
    all slabs concurrently into slices of one buffer).  gloo (CPU rehearsal): the same through host
    copies.  Returns (verts float32 [V, 3], faces int32 [F, 3]) numpy arrays on rank 0, None elsewhere."""
    import numpy as np
    g = gathered.to("cpu").numpy().astype(np.int64)
    nv = g[:, 0] - g[:, 3]
    nf = g[:, 1]
    gloo = dist.get_backend(group) == "gloo"
    dev = gathered.device if not gloo else torch.device("cpu")
    if gloo:
        v_np, f_np = slab.download(int(nv[rank]), int(nf[rank]), stream)
        v_loc, f_loc = torch.from_numpy(v_np.reshape(-1)), torch.from_numpy(f_np.reshape(-1))
    else:
        v_loc = torch.empty(int(nv[rank]) * 3, dtype=torch.float32, device=dev)
        f_loc = torch.empty(int(nf[rank]) * 3, dtype=torch.int32, device=dev)
        slab.copy_mesh(v_loc.data_ptr(), f_loc.data_ptr(), int(nv[rank]), int(nf[rank]), stream)
        # the copy ran on `stream` (any caller stream, not necessarily torch's current one): wait
        # for that stream before the send reads the buffers
        if stream:
            torch.cuda.ExternalStream(stream, device=dev).synchronize()
        else:
            torch.cuda.synchronize(dev)
    if rank != 0:   # empty parts are skipped on both sides (both know the sizes)
        works = [dist.isend(t, 0, group=group) for t in (v_loc, f_loc) if t.numel()]
        for w in works:
            w.wait()
        return None
    voff = np.concatenate([[0], np.cumsum(nv)])
    foff = np.concatenate([[0], np.cumsum(nf)])
    V = torch.empty(int(voff[-1]) * 3, dtype=torch.float32, device=dev)
    F = torch.empty(int(foff[-1]) * 3, dtype=torch.int32, device=dev)
    V[:int(nv[0]) * 3].copy_(v_loc)
    F[:int(nf[0]) * 3].copy_(f_loc)
    works = []
    for r in range(1, world):
        for t in (V[int(voff[r]) * 3:int(voff[r + 1]) * 3], F[int(foff[r]) * 3:int(foff[r + 1]) * 3]):
            if t.numel():
                works.append(dist.irecv(t, r, group=group))
    for w in works:
        w.wait()
    return V.cpu().numpy().reshape(-1, 3), F.cpu().numpy().reshape(-1, 3)


def allgather_mesh(slab, gathered, rank, world, device, group=None, stream=0):
    """Every rank's emitted slab mesh to every rank, concatenated in rank order (the whole MC mesh,
    byte-identical to one GPU), as device tensors (verts float32 [V*3], faces int32 [F*3]) on
    `device` -- the input of the sharded OB02 loop.  Padded equal-size all-gathers (RCCL), or host
    copies under gloo."""
    import numpy as np
    g = gathered.to("cpu").numpy().astype(np.int64)
    nv = g[:, 0] - g[:, 3]
    nf = g[:, 1]
    voff = np.concatenate([[0], np.cumsum(nv)])
    foff = np.concatenate([[0], np.cumsum(nf)])
    gloo = dist.get_backend(group) == "gloo"
    if gloo:
        v_np, f_np = slab.download(int(nv[rank]), int(nf[rank]), stream)
        v_loc, f_loc = torch.from_numpy(v_np.reshape(-1)), torch.from_numpy(f_np.reshape(-1))
    else:
        v_loc = torch.empty(int(nv[rank]) * 3, dtype=torch.float32, device=device)
        f_loc = torch.empty(int(nf[rank]) * 3, dtype=torch.int32, device=device)
        slab.copy_mesh(v_loc.data_ptr(), f_loc.data_ptr(), int(nv[rank]), int(nf[rank]), stream)
        if stream:
            torch.cuda.ExternalStream(stream, device=device).synchronize()
        else:
            torch.cuda.synchronize(device)
    V = _allgather_segments(v_loc, voff * 3, world, group)
    F = _allgather_segments(f_loc, foff * 3, world, group)
    return V.to(device), F.to(device), voff, foff


def _allgather_segments(local, offs, world, group=None):
    """All-gather of rank-ordered segments of different lengths (offs: element offsets, world + 1):
    each rank's segment padded to the longest, one equal-size all-gather, then concatenated."""
    n = [int(offs[r + 1] - offs[r]) for r in range(world)]
    m = max(1, max(n))
    pad = torch.zeros(m, dtype=local.dtype, device=local.device)
    pad[:local.numel()] = local
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out = torch.stack(parts)
    else:
        out = torch.empty(world, m, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r, :n[r]] for r in range(world)])


def ob02_plan(st):
    """The OB02 loop's steps in grand_algorithm's order (mcc2.cpp:309-444, polygonizer_algorithm_ob02.hpp
    :74-157): overall_repeats x [vresampl.iters x resampling ("R"); projection ("P", + QEM)], and the
    exchange each vertex-moving step needs before the next step that reads vertices:
      - before a resampling, only its halo (the vertices of the faces whose centroids its weights
        read, Ob02Shard.halo()): "halo";
      - before a projection (the edge-length fold reads every vertex) or at the end: "full".
    A projection without QEM moves no vertex (exchange None).  Returns [(step, exchange), ...]."""
    steps = []
    for _ in range(st["overall_repeats"]):
        steps += ["R"] * st["vresampl_iters"]
        if st["projection"]:
            steps.append("P")
    out = []
    for k, step in enumerate(steps):
        moves = step == "R" or st["qem"]
        nxt = next((x for x in steps[k + 1:] if x == "R" or x == "P"), None)
        out.append((step, None if not moves else "halo" if nxt == "R" else "full"))
    # a step that moves nothing leaves the previous exchange's coverage; the step after a "halo"
    # exchange is always a resampling, which reads only the halo
    return out


def shard_transfers(voff, halos, rank, kind="halo"):
    """The vertex ranges one exchange moves for `rank` (a pure function: every exchange path --
    ob02_sharded over RCCL and over gloo, and ob02_shards_local's device copies -- takes its ranges
    from here).  voff: the owned-range offsets (world + 1); halos[q]: (h0, h1), the vertex range
    rank q's next resampling reads (Ob02Shard.halo()).
      kind "halo": rank sends q the owned vertices inside q's halo, and receives from q q's owned
                   vertices inside its own halo;
      kind "full": rank sends its whole owned range to every q and receives every q's.
    Returns (sends, recvs): lists of (peer, a, b) vertex ranges [a, b), non-empty, peers ascending.
    What r sends q is exactly what q receives from r (tests/test_cpu.py::test_shard_transfers_*)."""
    world = len(voff) - 1
    v0, v1 = int(voff[rank]), int(voff[rank + 1])
    sends, recvs = [], []
    for q in range(world):
        if q == rank:
            continue
        q0, q1 = int(voff[q]), int(voff[q + 1])
        if kind == "halo":
            a, b = max(v0, int(halos[q][0])), min(v1, int(halos[q][1]))        # my owned vertices q reads
            c, d = max(q0, int(halos[rank][0])), min(q1, int(halos[rank][1]))  # q's owned vertices I read
        elif kind == "full":
            a, b, c, d = v0, v1, q0, q1
        else:
            raise ValueError("kind must be 'halo' or 'full'")
        if a < b:
            sends.append((q, a, b))
        if c < d:
            recvs.append((q, c, d))
    return sends, recvs


_SHARDS = {}   # (device, slot) -> (object key, Ob02Shard): one kept handle per slot and device


def shard_handle(shape, mc_settings, slot=0, device=None):
    """The rank's OB02 shard handle for this object, created once and reused by later builds, as
    build_geometry keeps its one refinement state (abi.hip g_ob02): a fresh handle allocates every
    device buffer, its side stream and events on its first attach and projection (0.3-0.8 ms per
    shard), a reused one only re-attaches the mesh.  At most one handle is kept per (device, slot):
    a build of another object (shape or settings) closes the slot's previous handle, so a caller
    that builds many shapes holds no more buffers and streams than one object's.  release_shards()
    frees them all; a loop that raises drops its handle (ob02_sharded, ob02_shards_local)."""
    import json
    import implisolid_amd as I
    dev = (torch.cuda.current_device() if torch.cuda.is_available() else -1) if device is None else int(device)
    okey = (json.dumps(shape, sort_keys=True), json.dumps(mc_settings, sort_keys=True))
    kept = _SHARDS.get((dev, int(slot)))
    if kept is not None and kept[0] == okey and kept[1].h:
        return kept[1]
    if kept is not None:
        kept[1].close()
    ob = I.Ob02Shard(shape, mc_settings)
    _SHARDS[(dev, int(slot))] = (okey, ob)
    return ob


def drop_shard(ob):
    """Close a kept handle and forget it (a loop that failed part-way: its state is not reused)."""
    for k, (_, kept) in list(_SHARDS.items()):
        if kept is ob:
            del _SHARDS[k]
    ob.close()


def release_shards():
    """Close every kept shard handle (shard_handle)."""
    for _, ob in _SHARDS.values():
        ob.close()
    _SHARDS.clear()


def ob02_sharded(shape, mc_settings, V, F, voff, rank, world, group=None, on_step=None, halo=True):
    """The OB02 loop (ob02_plan) over Z-slab shards: every rank holds the whole mesh and owns its
    slab's vertices [voff[rank], voff[rank + 1]).  Stream-ordered: the loop runs on the shard's HIP
    stream (Ob02Shard.attach / resample_async / project_async) with no host synchronisation per
    step, on a copy of V that is the shard's working vertex array in place.  After a vertex-moving
    step the owned ranges are exchanged into that array on the same stream:
      - "full": every rank's owned range padded to one equal row, one all-gather (RCCL), unpacked by
        one kernel (Ob02Shard.unpack);
      - "halo" (halo=True, before a resampling): point-to-point sends of the owned vertices each
        neighbour's next resampling reads (its one-ring halo), batched (RCCL group).
    Subdivision runs once on rank 0 after the loop (it reads every face).  gloo (the CPU-side
    rehearsal) stages the same exchanges through host copies.  Returns rank 0's final (verts,
    faces) numpy arrays, None elsewhere; byte-identical to the single-device loop."""
    import numpy as np
    import implisolid_amd as I
    st = I.parse_settings(mc_settings)
    device = V.device
    cuda = device.type == "cuda"
    gloo = dist.get_backend(group) == "gloo"
    nv, nf = V.numel() // 3, F.numel() // 3
    voff = [int(x) for x in voff]
    v0, v1 = voff[rank], voff[rank + 1]
    W = V.clone()   # the working array (updated in place)
    ob = shard_handle(shape, mc_settings, device=device.index if cuda else None)
    ok = False
    try:
        cur = torch.cuda.current_stream(device) if cuda else None
        ob.attach(W.data_ptr(), nv, F.data_ptr(), nf, v0, v1, cur.cuda_stream if cur is not None else 0)
        s_ob = torch.cuda.ExternalStream(ob.stream(), device=device) if cuda else None
        # every rank's halo (host, once)
        h = torch.tensor(list(ob.halo()), dtype=torch.int64, device=device if not gloo else "cpu")
        hs = [torch.zeros_like(h) for _ in range(world)]
        dist.all_gather(hs, h, group=group)
        H = [(int(x[0]), int(x[1])) for x in hs]
        m = 3 * max(1, max(voff[r + 1] - voff[r] for r in range(world)))

        def full_exchange():
            if gloo:
                s_ob.synchronize()
                own = torch.zeros(m, dtype=torch.float32)
                own[:3 * (v1 - v0)] = W[3 * v0:3 * v1].cpu()
                parts = [torch.empty(m, dtype=torch.float32) for _ in range(world)]
                dist.all_gather(parts, own, group=group)
                rows = torch.stack(parts).to(device)
                torch.cuda.current_stream(device).synchronize()
                ob.unpack(rows.data_ptr(), m, voff, rank)
                s_ob.synchronize()
                return
            with torch.cuda.stream(s_ob):
                own = torch.zeros(m, dtype=torch.float32, device=device)
                own[:3 * (v1 - v0)].copy_(W[3 * v0:3 * v1])
                rows = torch.empty(world, m, dtype=torch.float32, device=device)
                dist.all_gather_into_tensor(rows, own, group=group)
                ob.unpack(rows.data_ptr(), m, voff, rank)

        def halo_exchange():
            sends, recvs = shard_transfers(voff, H, rank, "halo")
            if gloo:
                s_ob.synchronize()
                host = W.cpu()
                ops = [dist.P2POp(dist.isend, host[3 * a:3 * b].clone(), q, group=group) for q, a, b in sends]
                got = [(a, b, torch.empty(3 * (b - a), dtype=torch.float32)) for q, a, b in recvs]
                ops += [dist.P2POp(dist.irecv, t, q, group=group) for (q, _, _), (_, _, t) in zip(recvs, got)]
                for r in (dist.batch_isend_irecv(ops) if ops else []):
                    r.wait()
                for a, b, t in got:
                    W[3 * a:3 * b].copy_(t.to(device))
                torch.cuda.current_stream(device).synchronize()
                return
            ops = [dist.P2POp(dist.isend, W[3 * a:3 * b], q, group=group) for q, a, b in sends]
            ops += [dist.P2POp(dist.irecv, W[3 * a:3 * b], q, group=group) for q, a, b in recvs]
            if not ops:
                return
            with torch.cuda.stream(s_ob):
                for r in dist.batch_isend_irecv(ops):
                    r.wait()

        plan = ob02_plan(st)
        reps = st["overall_repeats"]
        per_rep = len(plan) // reps if reps else 0
        for k, (step, ex) in enumerate(plan):
            if step == "R":
                ob.resample_async()
            else:
                ob.project_async()
            if ex == "full" or (ex == "halo" and not halo):
                full_exchange()
            elif ex == "halo":
                halo_exchange()
            if on_step and per_rep:
                on_step({"R": "resample", "P": "project"}[step], k // per_rep)
        if st["subdiv"] and st["overall_repeats"] >= 1 and rank == 0:   # polygonize_step_3, last repeat: noise x 10
            ob.subdivide(float(st["post_subdiv_noise"]) * 10.0)
        res = ob.download() if rank == 0 else None
        if cuda:
            s_ob.synchronize()
        ok = True
        return res
    finally:
        if cuda and ob.h:
            torch.cuda.ExternalStream(ob.stream(), device=device).synchronize()   # W lives until the loop is done
        if not ok:
            drop_shard(ob)   # a half-attached handle is not reused


def ob02_shards_local(shape, mc_settings, V, F, voff, halo=True, timing=False):
    """The sharded loop of ob02_sharded with every shard in this process, on one GPU (tests and the
    bench's 8-rank estimate; shard r's handle is shard_handle(..., slot=r), kept across calls): shard r owns [voff[r], voff[r + 1]) and steps on its own HIP stream;
    the exchanges of ob02_plan are device copies between the shards' arrays (full: every owned range
    to every shard; halo: each shard's halo from its owners).  timing=True: every shard's step is
    timed with HIP events on its stream, run one shard at a time (so the shards do not share the
    GPU), giving each step's slowest shard.  Returns (shard 0's final verts, faces, stats)."""
    import numpy as np
    import implisolid_amd as I
    st = I.parse_settings(mc_settings)
    device = V.device
    nv, nf = V.numel() // 3, F.numel() // 3
    voff = [int(x) for x in voff]
    n = len(voff) - 1
    Ws = [V.clone() for _ in range(n)]
    obs = [shard_handle(shape, mc_settings, slot=r, device=device.index) for r in range(n)]
    stats = {"steps": [], "exchange_bytes": []}
    ok = False
    try:
        import time
        cur = torch.cuda.current_stream(device)
        torch.cuda.synchronize(device)
        attach_ms = []
        for r, ob in enumerate(obs):   # one at a time: each shard's load + topology + ranges
            t0 = time.perf_counter()
            ob.attach(Ws[r].data_ptr(), nv, F.data_ptr(), nf, voff[r], voff[r + 1], cur.cuda_stream)
            torch.cuda.ExternalStream(ob.stream(), device=device).synchronize()
            attach_ms.append((time.perf_counter() - t0) * 1e3)
        stats["attach_ms"] = [round(t, 4) for t in attach_ms]
        streams = [torch.cuda.ExternalStream(ob.stream(), device=device) for ob in obs]
        H = [ob.halo() for ob in obs]
        stats["halo"] = H

        def exchange(kind):
            for s in streams:
                s.synchronize()
            moved = 0
            for r in range(n):
                for q, a, b in shard_transfers(voff, H, r, kind)[1]:
                    Ws[r][3 * a:3 * b].copy_(Ws[q][3 * a:3 * b])
                    moved += 12 * (b - a)
            torch.cuda.synchronize(device)
            return moved

        for step, ex in ob02_plan(st):
            times = []
            for r, ob in enumerate(obs):
                if timing:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(streams[r])
                ob.resample_async() if step == "R" else ob.project_async()
                if timing:
                    e1.record(streams[r])
                    e1.synchronize()
                    times.append(e0.elapsed_time(e1))
            if ex:
                stats["exchange_bytes"].append(exchange("full" if ex == "full" or not halo else "halo"))
            stats["steps"].append({"step": step, "exchange": ex if (halo or ex is None) else "full",
                                   "shard_ms": [round(t, 4) for t in times]})
        if st["subdiv"] and st["overall_repeats"] >= 1:
            obs[0].subdivide(float(st["post_subdiv_noise"]) * 10.0)
        v, f = obs[0].download()
        ok = True
        return v, f, stats
    finally:
        torch.cuda.synchronize(device)   # the shards' streams are done with Ws
        if not ok:
            for ob in obs:
                drop_shard(ob)
