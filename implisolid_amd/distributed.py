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
