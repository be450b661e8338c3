"""How much of the pruned eval's work marching cubes actually needs (config-4 tree).

Runs the 512^3 grid at pruning level 1 (every sample exact), takes the sample signs, and marks the
samples that end a sign-changing axis edge (the only field values marching cubes reads).  Prints,
per 8x8x2 brick, how many bricks hold such a sample, how many need only one of their two layers, and
the level-2 pipeline's listed-brick count for comparison.

    python tools/needed_probe.py [R]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import implisolid_amd as ia
from implisolid_amd import scenes


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    shape, mc = scenes.config4(R) if callable(getattr(scenes, "config4", None)) else (scenes.config3_tree(), None)
    if mc is None:
        mc = scenes.mc_settings(R, 1.0)
    ia.set_pruning(2)
    s = ia.Slab(shape, mc)
    s.eval()
    bricks, mixed, filled = s.brick_stats()
    sg = s.read_signs().astype(bool)
    s.close()
    s_exact = sg
    L, n, _ = sg.shape
    need = np.zeros_like(sg)
    for ax in range(3):
        a = np.moveaxis(sg, ax, 0)
        nv = np.moveaxis(need, ax, 0)
        d = a[1:] != a[:-1]
        nv[1:] |= d
        nv[:-1] |= d
    del sg
    Lp, npad = (L + 1) // 2 * 2, (n + 7) // 8 * 8
    pad = np.zeros((Lp, npad, npad), bool)
    pad[:L, :n, :n] = need
    del need
    # brick classes from the exact signs (0 positive, 1 negative, 2 mixed) and the neighbour rule
    sp = np.ones((Lp, npad, npad), bool)   # padding: negative like the sealed ring
    sp[:L, :n, :n] = s_exact
    sb = sp.reshape(Lp // 2, 2, npad // 8, 8, npad // 8, 8)
    allneg, anyneg = sb.all(axis=(1, 3, 5)), sb.any(axis=(1, 3, 5))
    cls = np.where(allneg, 1, np.where(anyneg, 2, 0)).astype(np.int8)
    del sp, sb

    def nb(ax, d):   # neighbour class along axis ax (edge: the brick itself)
        c = np.moveaxis(cls, ax, 0)
        o = c.copy()
        if d < 0:
            o[1:] = c[:-1]
        else:
            o[:-1] = c[1:]
        return np.moveaxis(o, 0, ax)
    definite = cls != 2
    dx = (nb(2, -1) != cls) | (nb(2, 1) != cls) | (nb(1, -1) != cls) | (nb(1, 1) != cls)
    dzl, dzh = nb(0, -1) != cls, nb(0, 1) != cls
    listed_exact = ~definite | dx | dzl | dzh
    half = definite & ~dx & (dzl ^ dzh)
    b = pad.reshape(Lp // 2, 2, npad // 8, 8, npad // 8, 8)
    per_layer = b.any(axis=(3, 5))            # (bz, 2, by, bx)
    any_b = per_layer.any(axis=1)
    one_layer = any_b & ~per_layer.all(axis=1)
    cnt = b.sum(axis=(1, 3, 5))
    out = {
        "R": R,
        "bricks": int(bricks),
        "interval_mixed": int(mixed),
        "listed": int(bricks - filled),
        "needed_samples": int(pad.sum()),
        "bricks_with_needed": int(any_b.sum()),
        "bricks_needing_one_layer": int(one_layer.sum()),
        "needed_per_needed_brick_mean": float(cnt[any_b].mean()),
        "exact_mixed_bricks": int((~definite).sum()),
        "exact_listed_bricks": int(listed_exact.sum()),
        "exact_listed_half_bricks_z_only": int(half.sum()),
        "definite_bricks_with_needed": int((any_b & definite).sum()),
        "mixed_bricks_with_needed": int((any_b & ~definite).sum()),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
