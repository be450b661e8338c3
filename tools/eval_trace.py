#!/usr/bin/env python3
"""Per-wave timeline of the eval kernel (diagnostics): run with the evaltrace variant library
(tools/eval_trace_patch.py) as IMPLISOLID_LIB, config 4 at R; every eval dumps the waves' records
{start, list entry loaded, first brick evaluated, claims decided, end, bricks, claimed} (100 MHz
s_memrealtime ticks) to $IMPLISOLID_EVAL_TRACE.  Prints the phase durations and the wave
generations of the last step.   usage: python tools/eval_trace.py [R] [steps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import numpy as np
    import torch
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    path = os.environ.setdefault("IMPLISOLID_EVAL_TRACE", "/tmp/eval_trace.bin")
    import implisolid_amd as I
    from implisolid_amd import scenes
    shape, mc = scenes.config4(R)
    s = I.Slab(shape, mc)
    sp = torch.cuda.current_stream().cuda_stream
    for k in range(steps):
        s.eval(sp); s.count(sp); s.emit(0, sp)
        if k == 3:
            I.jit_wait()
    torch.cuda.synchronize()
    d = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    d = d[d[:, 7] == 1]
    st, tl, tf, tc, te, nb, ncl = [d[:, k].astype(np.int64) for k in range(7)]
    t0 = st.min()
    us = lambda x: x * 0.01   # 100 MHz ticks -> us
    work = nb > 0
    out = {"R": R, "waves": int(len(d)), "waves_with_bricks": int(work.sum()), "jit_module": s.jit_module(),
           "span_us": round(us(te.max() - t0), 2),
           "bricks_per_wave": {str(k): int((nb == k).sum()) for k in range(0, int(nb.max()) + 1)},
           "claimed_per_wave": {str(k): int((ncl[work] == k).sum()) for k in range(0, int(ncl.max()) + 1)}}
    w = work
    ph = {"start_to_list": tl[w] - st[w], "first_eval": tf[w] - tl[w], "claims": tc[w] - tf[w], "rest": te[w] - tc[w],
          "lifetime": te[w] - st[w]}
    out["phase_us"] = {k: {"mean": round(us(v.mean()), 2), "p50": round(us(np.median(v)), 2), "p90": round(us(np.percentile(v, 90)), 2),
                           "max": round(us(v.max()), 2)} for k, v in ph.items()}
    claimers = w & (ncl > 0)
    out["rest_us_claimers"] = round(us((te[claimers] - tc[claimers]).mean()), 2) if claimers.any() else None
    out["rest_us_nonclaimers"] = round(us((te[w & (ncl == 0)] - tc[w & (ncl == 0)]).mean()), 2)
    first_end = te[w].min()
    out["start_us_percentiles"] = [round(us(np.percentile(st - t0, q)), 2) for q in (0, 25, 50, 75, 90, 99, 100)]
    out["end_us_percentiles"] = [round(us(np.percentile(te - t0, q)), 2) for q in (0, 25, 50, 75, 90, 99, 100)]
    out["waves_started_after_first_end"] = int((st > first_end).sum())
    # waves / parts in flight per microsecond of the kernel's span, and how many had started
    bins = np.arange(0, int(us(te.max() - st.min())) + 2)
    rs, re_ = us(st - st.min()), us(te - st.min())
    out["in_flight_per_us"] = [int(((rs <= b + 0.5) & (re_ > b + 0.5)).sum()) for b in bins]
    out["started_by_us"] = [int((rs <= b + 0.5).sum()) for b in bins]
    print(json.dumps(out))
    s.close()


if __name__ == "__main__":
    main()
