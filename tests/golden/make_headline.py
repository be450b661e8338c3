#!/usr/bin/env python3
"""Headline-size golden summaries (TEST INFRASTRUCTURE): the exact workloads bench.py times.

The C oracle (oracle/, the CPU restatement of the reference; "parity unpinned")
polygonises each configuration once here; the summary pins the GPU result in
tests/test_gpu_parity.py::test_headline_* without running the oracle on the GPU box (its 512^3
run alone takes ~16 s of CPU):

  config4_mc_r512   config 3/4's twist tree, R = 512, eval + MC          (the bench headline)
  config4_mc_r256   the same tree at R = 256, eval + MC                  (the metric's 256^3 point)
  config4_mc_r645 / r813 / r1024   the same tree at bench.py's weak-scaling grids for 2 / 4 / 8
                    ranks (R_N = round(512 N^(1/3))), eval + MC; r1024 also pins the one-GPU test
                    of the eight balanced slabs of the 1024^3 grid
  config3_ob02_r256 config 3 (the tree, R = 256, MC + 3 x [resample, project, QEM])
  config2_ob02_r128 config 2 (sphere u rabbit, R = 128, MC + 3 x [resample, project, QEM])
  config3s_ob02_r256 config 3 with its box shifted by 0.003 (scenes.config3_shifted): no singular
                    sample, every vertex finite, so the alpha search and bisection run on every face
  config4_ob02_r512 / config4s_ob02_r512   config 4: the same tree at R = 512 through the same
                    loop, on the dyadic box and on the box shifted by 0.003
  config5_mc_r128   config 5's 64 objects at 128^3, eval + MC: per object V / F and the SHA-256s

Per configuration: V / F counts, SHA-256 of the face array, SHA-256 of the vertex array (for the
bit-exact cases), the non-finite vertex rows (OB02 on the tree: reference behaviour at singular
points), the float64 sum of the finite vertices, and 4096 seeded sampled vertex rows
with their values (the tolerance check for trees holding a twist, whose gradient uses the double
cos).  OB02 meshes with more than 21 845 faces are past the reference's short edge-id wrap
(DESIGN.md §5): the oracle, like the GPU, follows the intended semantics there.

    python tests/golden/make_headline.py        # adds missing entries; --all recomputes every one

headline_ob02_verts.npz holds the full vertex arrays of the two OB02 meshes of the twist tree
(config3_ob02_r256, config3s_ob02_r256) for the every-row tolerance check.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

N_SAMPLE = 4096


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def configs():
    from implisolid_amd import scenes
    return {
        "config4_mc_r512": scenes.config4(512),
        "config4_mc_r256": scenes.config4(256),
        # the weak-scaling grids of bench.py at N = 2, 4, 8 ranks: R_N = round(512 N^(1/3))
        "config4_mc_r645": scenes.config4(645),
        "config4_mc_r813": scenes.config4(813),
        "config4_mc_r1024": scenes.config4(1024),
        "config3_ob02_r256": scenes.config3(256),
        "config2_ob02_r128": scenes.config2(128),
        "config3s_ob02_r256": scenes.config3_shifted(256),
        # config 4's tree at 512^3 through the whole OB02 loop (BASELINE config 4 "eval + MC (+ OB02)")
        "config4_ob02_r512": scenes.config3(512),
        "config4s_ob02_r512": scenes.config3_shifted(512),
    }


def summarize(v, f, seed):
    fin = np.isfinite(v).all(1)
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(v.shape[0], size=min(N_SAMPLE, v.shape[0]), replace=False)).astype(np.int64)
    return {
        "n_verts": int(v.shape[0]), "n_faces": int(f.shape[0]),
        "sha256_faces": sha(f), "sha256_verts": sha(v),
        "nonfinite_rows": [int(i) for i in np.flatnonzero(~fin)],
        "finite_sum": [float(x) for x in v[fin].astype(np.float64).sum(0)],
    }, idx, v[idx]


def config5_summary():
    """Config 5's object stream: each of the 64 objects' eval + MC mesh (oracle.marching_cubes)."""
    import oracle
    from implisolid_amd import scenes
    objs = scenes.config5_objects(64, 128)
    rows = []
    t0 = time.perf_counter()
    for shape, mc in objs:
        v, f = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(shape)), 128, [-1.0, 1.0] * 3)
        rows.append({"n_verts": int(v.shape[0]), "n_faces": int(f.shape[0]), "sha256_faces": sha(f), "sha256_verts": sha(v)})
    return {"workload": "scenes.config5_objects(64, 128): eval + MC of each object, box [-1, 1]^3",
            "objects": rows, "oracle_s": round(time.perf_counter() - t0, 1)}


def main():
    import oracle
    oracle.build()
    redo = "--all" in sys.argv
    path_s, path_a = os.path.join(HERE, "headline_summaries.json"), os.path.join(HERE, "headline_samples.npz")
    out, arrays = {}, {}
    if not redo and os.path.exists(path_s):
        out = json.load(open(path_s))
        arrays = dict(np.load(path_a))
    for k, (name, (shape, mc)) in enumerate(configs().items()):
        if name in out:
            continue
        t0 = time.perf_counter()
        v, f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
        s, idx, vs = summarize(v, f, 20251015 + k)
        s.update(shape=shape, mc=mc, oracle_s=round(time.perf_counter() - t0, 1))
        out[name] = s
        arrays[name + "_idx"], arrays[name + "_v"] = idx, vs
        print(name, s["n_verts"], s["n_faces"], "non-finite", len(s["nonfinite_rows"]), "%.1f s" % s["oracle_s"])
    # the full vertex arrays of the OB02 meshes of trees with a twist (their vertices are compared to
    # 1e-5, the twist's gradient going through the double cos): every row, not only the samples
    path_v = os.path.join(HERE, "headline_ob02_verts.npz")
    full = dict(np.load(path_v)) if (not redo and os.path.exists(path_v)) else {}
    for name in ("config3_ob02_r256", "config3s_ob02_r256", "config4s_ob02_r512"):
        if name in full:
            continue
        shape, mc = out[name]["shape"], out[name]["mc"]
        v, f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
        assert sha(f) == out[name]["sha256_faces"]
        full[name] = v
        print(name, "full vertex array", v.shape)
    np.savez_compressed(path_v, **full)
    if "config5_mc_r128" not in out:
        out["config5_mc_r128"] = config5_summary()
        print("config5_mc_r128", sum(o["n_faces"] for o in out["config5_mc_r128"]["objects"]), "faces",
              "%.1f s" % out["config5_mc_r128"]["oracle_s"])
    with open(path_s, "w") as fh:
        json.dump(out, fh, indent=1)
    np.savez_compressed(path_a, **arrays)


if __name__ == "__main__":
    main()
