"""Worker of the multi-process GPU test (tests/test_gpu_parity.py::test_multiprocess_slabs_gloo).

Launched by ``python -m torch.distributed.run --nproc-per-node N ... tests/dist_worker.py OUT R
[balanced]``: one process per rank, every rank on cuda:(LOCAL_RANK mod the visible devices) --
several ranks share the one GPU of a test box -- and torch.distributed over
IMPLISOLID_DIST_BACKEND (gloo for the rehearsal, nccl = RCCL on a multi-GPU node).  Each rank runs
bench.py's multi-GPU step on its Z-slab of config 3's tree (balanced cuts from one interval pass,
eval, count, the count all-gather in flight while the vertex pass runs, the face pass with the
gathered counts), then the mesh is gathered to rank 0, which writes it to OUT (.npz).
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
    balanced = len(sys.argv) > 3 and sys.argv[3] == "balanced"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("IMPLISOLID_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    shape, mc = scenes.config3_tree(), scenes.mc_settings(R, 1.0)
    cuts = D.balanced_cuts(shape, mc, world) if balanced else None
    slab = I.Slab(shape, mc, rank, world, cuts=cuts)
    sp = torch.cuda.current_stream(dev).cuda_stream
    cnt = torch.zeros(4, dtype=torch.int32, device=dev)
    gath = torch.zeros(world, 4, dtype=torch.int32, device=dev)
    for _ in range(2):   # the second pass runs with outputs sized by the first
        slab.eval(sp)
        slab.count(sp)
        slab.counts(sp)
        slab.copy_counts(cnt.data_ptr(), sp)
        torch.cuda.current_stream(dev).synchronize()
        work = D.gather_counts_async(cnt, gath)
        slab.emit_verts(sp)
        if work is not None:
            work.wait()
        torch.cuda.current_stream(dev).synchronize()
        slab.emit_faces(0, gath.data_ptr(), rank, sp)
        nv, nf, of = slab.counts(sp)
    assert not of
    res = D.gather_mesh(slab, gath, rank, world)
    if rank == 0:
        v, f = res
        np.savez(out_path, verts=v, faces=f, cuts=np.asarray(cuts or [], np.int32), gathered=gath.cpu().numpy())
    slab.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
