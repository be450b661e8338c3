#!/usr/bin/env python3
"""Config 5 merged launches only (for rocprofv3 kernel stats).  usage: python tools/config5_merged_probe.py [n] [R] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import implisolid_amd as I
    from implisolid_amd import scenes
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    torch.cuda.init()
    objs = scenes.config5_objects(n, R)
    sp = torch.cuda.current_stream().cuda_stream
    I.set_jit(0)
    b = I.Batch([o[0] for o in objs], objs[0][1], n_streams=0)
    for _ in range(3):
        b.run(sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        b.run(sp)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    print("merged: %.3f ms / %d objects (%.0f objects/s)" % (ms, n, n / ms * 1e3), flush=True)


if __name__ == "__main__":
    main()
