#!/usr/bin/env python3
"""Config 5's setup: implisolid_batch_create of the 64 seeded objects at 128^3 (merged launches),
timed three times in one process, each followed by one pass; IMPLISOLID_BATCH_TIMING=1 prints the
setup's phases (engines, set_object, set_grid, warm runs).   usage: python tools/batch_setup_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    objs = scenes.config5_objects(64, 128)
    texts = [json.dumps(o[0]) for o in objs]   # JSON text, as bench.py hands them over
    I.set_jit(0)
    sp = torch.cuda.current_stream().cuda_stream
    out = []
    for k in range(3):
        t0 = time.perf_counter()
        b = I.Batch(texts, objs[0][1], n_streams=0)
        setup = time.perf_counter() - t0
        b.run(sp)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        b.run(sp)
        torch.cuda.synchronize()
        run = time.perf_counter() - t1
        b.close()
        out.append({"setup_ms": round(setup * 1e3, 3), "pass_ms": round(run * 1e3, 3)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
