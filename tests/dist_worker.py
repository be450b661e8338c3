"""Worker of the multi-process GPU test (tests/test_gpu_parity.py::test_multiprocess_slabs_gloo).

Launched by ``python -m torch.distributed.run --nproc-per-node N ... tests/dist_worker.py OUT R
[balanced]``: one process per rank, every rank on cuda:(LOCAL_RANK mod the visible devices) --
several ranks share the one GPU of a test box -- and torch.distributed over
IMPLISOLID_DIST_BACKEND (gloo for the rehearsal, nccl = RCCL on a multi-GPU node).  Each rank runs
bench.py's multi-GPU step on its Z-slab of config 3's tree (balanced cuts from one interval pass,
eval, count, the vertex pass, the count all-gather on the launch stream, the face pass with the
gathered counts), then the mesh is gathered to rank 0, which writes it to OUT (.npz).

With the flag "ob02" the scene is config 2 (sphere u rabbit, MC + 3 x [resample, project, QEM]): the
slabs' MC meshes are all-gathered to every rank, the OB02 loop runs sharded by owned vertex ranges
(distributed.ob02_sharded: the owned vertices all-gathered after every vertex-moving step) and rank 0
writes the refined mesh.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    import implisolid_amd as I
    from implisolid_amd import distributed as D
    from implisolid_amd import scenes

    out_path, R = sys.argv[1], int(sys.argv[2])
    balanced = "balanced" in sys.argv[3:]
    ob02 = "ob02" in sys.argv[3:]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("IMPLISOLID_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    shape, mc = scenes.config2(R) if ob02 else (scenes.config3_tree(), scenes.mc_settings(R, 1.0))
    cuts = D.balanced_cuts(shape, mc, world) if balanced else None
    slab = I.Slab(shape, mc, rank, world, cuts=cuts)
    sp = torch.cuda.current_stream(dev).cuda_stream
    cnt = torch.zeros(4, dtype=torch.int32, device=dev)
    gath = torch.zeros(world, 4, dtype=torch.int32, device=dev)
    totals = D.counts_tensor(slab, dev) if backend == "nccl" else None
    for _ in range(2):   # the second pass runs with outputs sized by the first
        slab.eval(sp)
        slab.count(sp)
        slab.counts(sp)
        # bench.py's step: the vertex pass, then the counts' all-gather on the launch stream (RCCL:
        # straight from the engine's counters; gloo: a copy, host-synchronised), then the face pass
        slab.emit_verts(sp)
        if totals is not None:
            D.gather_counts_inline(totals, gath)
        else:
            slab.copy_counts(cnt.data_ptr(), sp)
            torch.cuda.current_stream(dev).synchronize()
            D.gather_counts_inline(cnt, gath)
        slab.emit_faces(0, gath.data_ptr(), rank, sp)
        nv, nf, of = slab.counts(sp)
    assert not of
    if ob02:
        V, F, voff, foff = D.allgather_mesh(slab, gath, rank, world, dev)
        res = D.ob02_sharded(shape, mc, V, F, voff, rank, world)
    else:
        res = D.gather_mesh(slab, gath, rank, world)
    if rank == 0:
        v, f = res
        np.savez(out_path, verts=v, faces=f, cuts=np.asarray(cuts or [], np.int32), gathered=gath.cpu().numpy())
    slab.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
