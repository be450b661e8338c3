#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (TEST INFRASTRUCTURE).

The reference ships no tests, fixtures or golden data and cannot be built here (SURVEY.md §4,
§8c), so these vectors come from the CPU restatements: the C oracle (oracle/) for everything, and
the independent numpy restatement (tests/np_restate.py) must agree with it where it covers the
stage (field + marching cubes).  They pin both restatements against regressions; the GPU path is
compared with them in tests/test_gpu_parity.py.  "parity unpinned" applies (Oracle).

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def point_trees():
    from implisolid_amd import scenes
    out = {"sphere": {"type": "iellipsoid", "matrix": scenes.EYE},
           "union_sphere_cube": scenes.union_sphere_cube(),
           "config3_tree": scenes.random_tree(scenes.CONFIG3_SEED, 10)}   # the tree without its twist
    for t in ["iellipsoid", "icylinder", "icone", "itorus", "implicit_double_mushroom", "iheart", "cube"]:
        out["leaf_" + t] = {"type": t, "matrix": scenes.st(0.5, 0.125, -0.0625, 0.03125)}
    return out


def main():
    import oracle
    import np_restate
    from implisolid_amd import scenes
    oracle.build()

    # 1. config 1 (sphere, box +-0.6, R 32): full mesh
    shape, mc = scenes.config1()
    v, f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    v2, f2 = np_restate.polygonize_mc(shape, 32, [-0.6, 0.6] * 3)
    assert np.array_equal(f, f2) and np.array_equal(v.view(np.uint32), v2.view(np.uint32))
    np.savez_compressed(os.path.join(HERE, "config1_mc.npz"), verts=v, faces=f,
                        shape=json.dumps(shape), mc=json.dumps(mc))

    # 2. point evaluation (f and gradient) on seeded points, per tree
    trees = point_trees()
    rng = np.random.default_rng(20251015)
    pts = rng.uniform(-1.1, 1.1, size=(4096, 3)).astype(np.float32)
    arrays = {"points": pts}
    for name, sh in trees.items():
        tree = oracle.mp5_to_nodes(json.dumps(sh))
        fo = oracle.eval_implicit(tree, pts)
        fn = np_restate.evaluate(sh, pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy())
        assert np.array_equal(fo.view(np.uint32), fn.view(np.uint32)), name
        arrays["f_" + name] = fo
        arrays["g_" + name] = oracle.eval_gradient(tree, pts)
    # the twist family (oracle only: the numpy restatement has no glibc sinf / atan2f)
    for name, sh in {"twist": scenes.twist(1, 0, 0, 0), "twist_small_pitch": scenes.twist(0.5, 0.125, 0, 0.0625, pitch=0.0625),
                     "config3_twist_tree": scenes.config3_tree()}.items():
        trees[name] = sh
        tree = oracle.mp5_to_nodes(json.dumps(sh))
        arrays["f_" + name] = oracle.eval_implicit(tree, pts)
        arrays["g_" + name] = oracle.eval_gradient(tree, pts)
    np.savez_compressed(os.path.join(HERE, "points_eval.npz"), trees=json.dumps(trees), **arrays)

    # 3. config 2's scene at R 32 through the whole OB02 loop (3 repeats, resample+project+QEM)
    shape, mc = scenes.config2(32)
    taps = {}
    v, f = oracle.polygonize(json.dumps(shape), json.dumps(mc), taps=taps)
    np.savez_compressed(os.path.join(HERE, "config2_r32_ob02.npz"), verts=v, faces=f,
                        shape=json.dumps(shape), mc=json.dumps(mc),
                        **{"tap_" + k: np.asarray(a) for k, a in taps.items()})

    # 5. subdivision (step 3): config 1 with subdiv on and the default noise 0.01 (x10 on the last
    #    repeat), rand() seeded with srand(1); and config 2 at R 24 with subdivision after 3 repeats
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    sub = {}
    for name, (shape, mc) in [("config1", (scenes.config1()[0], scenes.mc_settings(32, 0.6, subdiv=1,
                                                                                  post_subdiv_noise=0.01))),
                              ("config2_r24", (scenes.union_sphere_cube(),
                                               scenes.mc_settings(24, 1.0, vresampl_iters=1, vresampl_c=0.4,
                                                                  projection=1, qem=1, overall_repeats=3,
                                                                  subdiv=1, post_subdiv_noise=0.01)))]:
        oracle.srand(1)
        v, f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
        libc.srand(1)
        sub[name + "_verts"], sub[name + "_faces"] = v, f
        sub[name + "_shape"], sub[name + "_mc"] = json.dumps(shape), json.dumps(mc)
    # the numpy restatement agrees on the MC-only case (subdivision of the MC mesh)
    shape, mc = scenes.config1()
    v0, f0 = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    libc.srand(1)
    d = [libc.rand() for _ in range(3 * sub["config1_verts"].shape[0])]
    v2, f2 = np_restate.subdivide(v0, f0, np.float32(np.float32(0.01) * np.float32(10.0)), d)
    assert np.array_equal(f2, sub["config1_faces"]) and np.array_equal(v2.view(np.uint32), sub["config1_verts"].view(np.uint32))
    np.savez_compressed(os.path.join(HERE, "subdiv.npz"), **sub)

    # 4. marching-cubes summaries at larger sizes (counts + SHA-256 of the arrays)
    summary = {}
    for name, sh, R, box in [("config2_mc_r128", scenes.union_sphere_cube(), 128, [-1, 1] * 3),
                             ("config3_mc_r96", scenes.config3()[0], 96, [-1, 1] * 3)]:
        v, f = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(sh)), R, box)
        summary[name] = {"shape": sh, "R": R, "box": box, "n_verts": int(v.shape[0]), "n_faces": int(f.shape[0]),
                         "sha256_faces": sha(f), "sha256_verts": sha(v)}
    with open(os.path.join(HERE, "mc_summaries.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
