#!/usr/bin/env python3
"""The bench's 8-rank OB02 estimate in detail: config 3 on the shifted box at 256^3, the MC mesh's
vertices owned by the balanced Z-slabs, the sharded loop stepped one shard at a time on one GPU
(distributed.ob02_shards_local, timing=True).  Prints every step's per-shard milliseconds for n
shards and for one shard (the single-device loop), and the attach times.  Run it under
rocprofv3 --kernel-trace to see which kernels make up a shard's step.

    python tools/ob02_shard_probe.py [n] [R]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import numpy as np
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes, distributed as D
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    dev = torch.device("cuda", 0)
    shape, mc = scenes.config3_shifted(R)
    cuts = D.balanced_cuts(shape, mc, n)
    nvs = []
    for r in range(n):
        sl = I.Slab(shape, mc, r, n, cuts=cuts)
        nvs.append(sl.run()[0])
        sl.close()
    mc_only = dict(mc, vresampl={"iters": 0, "c": 1.0}, projection={"enabled": 0}, qem={"enabled": 0},
                   subdiv={"enabled": 0})
    v_mc, f_mc = I.make_geometry(shape, mc_only)
    V = torch.from_numpy(v_mc.reshape(-1).copy()).to(dev)
    F = torch.from_numpy(f_mc.reshape(-1).copy()).to(dev)
    voff = np.concatenate([[0], np.cumsum(nvs)]).astype(np.int64)
    D.ob02_shards_local(shape, mc, V, F, voff, timing=True)
    I.jit_wait()
    out = {"n": n, "R": R, "owned": nvs}
    for name, vo in (("n", voff), ("one", [0, len(v_mc)])):
        _, _, st = D.ob02_shards_local(shape, mc, V, F, vo, timing=True)
        out[name] = {"attach_ms": st["attach_ms"], "steps": st["steps"]}
        print(json.dumps({name: out[name]}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
