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


def ob02_sharded(shape, mc_settings, V, F, voff, rank, world, group=None, on_step=None):
    """The OB02 loop (grand_algorithm's order, mcc2.cpp:309-444 / polygonizer_algorithm_ob02.hpp:74-157:
    overall_repeats x [vresampl.iters x resampling; projection (+ QEM)]; subdivision on the last
    repeat) over Z-slab shards: every rank holds the whole mesh and owns its slab's vertices
    [voff[rank], voff[rank + 1]); after each step that moves vertices the owned ranges are
    all-gathered (12 B per vertex), so every rank starts the next step from the same mesh.
    Subdivision runs once on rank 0 after the loop (it reads every face).  Returns rank 0's final
    (verts, faces) numpy arrays, None elsewhere; byte-identical to the single-device loop."""
    import implisolid_amd as I
    st = I.parse_settings(mc_settings)
    device = V.device
    nv, nf = V.numel() // 3, F.numel() // 3
    v0, v1 = int(voff[rank]), int(voff[rank + 1])
    ob = I.Ob02Shard(shape, mc_settings)
    try:
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        ob.load(V.data_ptr(), nv, F.data_ptr(), nf, v0, v1)
        buf = torch.empty(nv * 3, dtype=torch.float32, device=device)

        def exchange():
            ob.get_verts(buf.data_ptr())
            own = buf[3 * v0:3 * v1]
            src = own if dist.get_backend(group) != "gloo" else own.cpu()
            full = _allgather_segments(src, voff * 3, world, group).to(device)
            buf.copy_(full)
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            ob.set_verts(buf.data_ptr())

        reps = st["overall_repeats"]
        for rep in range(reps):
            for _ in range(st["vresampl_iters"]):
                ob.resample()
                exchange()
            if on_step:
                on_step("resample", rep)
            if st["projection"]:
                ob.project()
                if st["qem"]:
                    exchange()
                if on_step:
                    on_step("project", rep)
            if st["subdiv"] and (reps <= 1 or rep == reps - 1):
                if rank == 0:   # polygonize_step_3: noise on the last repeat, scaled by 10
                    ob.subdivide(float(st["post_subdiv_noise"]) * 10.0 if rep == reps - 1 else 0.0)
        return ob.download() if rank == 0 else None
    finally:
        ob.close()
