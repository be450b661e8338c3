"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit-exact.

Integer/index outputs (faces) must be identical; float outputs (field values, gradients,
vertices) must be bit-identical too, because both sides execute the same IEEE operations in the
reference's order (no FMA contraction, correctly rounded division/sqrt).
"""
import json

import numpy as np
import pytest

from conftest import mesh_edges

pytestmark = pytest.mark.gpu


def _trees():
    from implisolid_amd import scenes
    out = {
        "sphere": {"type": "iellipsoid", "matrix": scenes.EYE},
        "union_sphere_cube": scenes.union_sphere_cube(),
        "config3_tree": scenes.config3()[0],
    }
    for t in ["iellipsoid", "icylinder", "icone", "itorus", "implicit_double_mushroom", "iheart", "cube"]:
        out["leaf_" + t] = {"type": t, "matrix": scenes.st(0.5, 0.125, -0.0625, 0.03125)}
    out["difference"] = {"type": "Difference", "matrix": scenes.st(1, 0.015625, 0, 0), "children": [
        {"type": "icylinder", "matrix": scenes.st(0.5, 0, 0, 0)}, {"type": "iellipsoid", "matrix": scenes.st(0.5, 0.25, 0, 0)}]}
    out["intersection"] = {"type": "Intersection", "matrix": scenes.EYE, "children": [
        {"type": "itorus", "matrix": scenes.st(0.25, 0, 0, 0)}, {"type": "icone", "matrix": scenes.st(1, 0, 0, -0.25)}]}
    out.update(SCREW_TREES)
    return out


def _screw_trees():
    from implisolid_amd import scenes
    tw = scenes.twist(1, 0, 0, 0)
    return {
        "twist": tw,
        "twist_small_pitch": scenes.twist(0.5, 0.125, 0, 0.0625, pitch=0.0625),   # sinf arguments > 120
        "twist_two_plane": dict(tw, type="screw_diff_two_plane"),
        "twist_inf": dict(scenes.twist(0.5, 0, 0.25, 0), type="inf_screw", pitch=0.25),
        "twist_tbb": {"type": "Union", "matrix": scenes.EYE, "children": [   # screw_gradient_wrong
            dict(scenes.twist(0.5, 0, 0.25, 0.0625), type="screw_gradient_wrong", pitch=0.25),
            {"type": "iellipsoid", "matrix": scenes.st(0.25, -0.25, -0.25, 0)}]},
        "half_plane": {"type": "Intersection", "matrix": scenes.EYE, "children": [
            {"type": "iellipsoid", "matrix": scenes.EYE},
            {"type": "half_plane", "matrix": scenes.st(0.5, 0, 0.125, 0), "plane_vector": [0, 1, 2],
             "plane_point": [0, 0, 0.25]}]},
        "lid": {"type": "Intersection", "matrix": scenes.EYE, "children": [
            {"type": "icylinder", "matrix": scenes.st(1, 0, 0, 0.5)},
            {"type": "top_bottom_lid", "matrix": scenes.st(1, 0, 0, 0)}]},
        "tetrahedron": scenes.tetrahedron(),
        "meta_balls": scenes.meta_balls(),
        "meta_balls_t": scenes.meta_balls(0.5, (0.125, 0, 0), time=2.5),
        "extrusion": scenes.extrusion(6),
        "extrusion_tri": {"type": "Union", "matrix": scenes.EYE, "children": [
            scenes.extrusion(3, 0.5, (0.25, 0, 0)), scenes.tetrahedron(0.5, (-0.25, 0, 0))]},
    }


# the screw gradient (screw.hpp:152-160) calls the double cos: glibc's in the oracle, its restatement
# on the device (ifunc_device.hpp glibc_cos, test_device_cos_bit_exact) -- every value, gradient and
# mesh is compared bit for bit
SCREW_TREES = _screw_trees()
TREES = _trees()


@pytest.mark.parametrize("name", sorted(TREES))
def test_eval_points_bit_exact(impli, oracle, name):
    shape = TREES[name]
    rng = np.random.default_rng(1234)
    pts = rng.uniform(-1.1, 1.1, size=(60000, 3)).astype(np.float32)
    tree = oracle.mp5_to_nodes(json.dumps(shape))
    f_ref = oracle.eval_implicit(tree, pts)
    g_ref = oracle.eval_gradient(tree, pts)
    with impli.ImplicitService(shape) as svc:
        f, g = svc.eval(pts, gradient=True)
        f2 = svc.eval(pts)
    assert np.array_equal(f.view(np.uint32), f_ref.view(np.uint32)), np.flatnonzero(f != f_ref)[:10]
    assert np.array_equal(f2.view(np.uint32), f_ref.view(np.uint32))
    # every gradient bit for bit, twists included (the screw gradient's double cos is glibc's,
    # restated: test_device_cos_bit_exact)
    assert np.array_equal(g.view(np.uint32), g_ref.view(np.uint32)), np.flatnonzero((g != g_ref).any(1))[:10]


def _same_bits(a, b):
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def _pattern_windows(centres, half=20000):
    return np.concatenate([np.arange(c - half, c + half, dtype=np.int64) for c in centres]).astype(np.uint32)


def test_device_libm_bit_exact(impli, oracle):
    """The screw family's glibc sinf / atanf / atan2f restatements on the device (branch-free
    selections, one division) against the oracle's (pinned to the host glibc by test_cpu), over a
    stride through every float pattern, dense windows around every range boundary, both signs,
    and seeded atan2f pairs including x == 1, zeros, infinities and NaN."""
    stride = np.arange(0, 1 << 32, 257, dtype=np.uint64).astype(np.uint32)
    sin_b = [0x39800000, 0x3f490fdb, 0x42f00000, 0x7f800000]                      # 2^-12, pi/4, 120, inf
    atan_b = [0x31000000, 0x3ee00000, 0x3f300000, 0x3f980000, 0x401c0000, 0x4c000000, 0x7f800000]
    for which, bounds in ((0, sin_b), (1, atan_b)):
        w = _pattern_windows(bounds)
        pats = np.concatenate([stride, w, w | np.uint32(0x80000000)])
        a = pats.view(np.float32)
        got, ref = impli.debug_libm(which, a), oracle.libm_apply(which, a)
        bad = ~_same_bits(got, ref)
        assert not bad.any(), (which, pats[bad][:8], got[bad][:4], ref[bad][:4])
    rng = np.random.default_rng(99)
    n = 1 << 21
    ys = [rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32),
          rng.uniform(-4, 4, n).astype(np.float32), (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-40, 40, n)).astype(np.float32)]
    xs = [rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32),
          rng.uniform(-4, 4, n).astype(np.float32), (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-40, 40, n)).astype(np.float32)]
    # |y / x| near atanf's boundaries, x == 1 (atanf(y) path), and the special operands
    t = np.array([0x3ee00000, 0x3f300000, 0x3f980000, 0x401c0000], np.uint32).view(np.float32)
    xr = rng.uniform(0.5, 2, n).astype(np.float32)
    yr = (xr * rng.choice(t, n) * (1 + rng.uniform(-1e-6, 1e-6, n))).astype(np.float32) * rng.choice([-1, 1], n).astype(np.float32)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 1e-30, -1e-30, 1e30, -1e30, 2.0], np.float32)
    gy, gx = np.meshgrid(sp, sp)
    Y = np.concatenate(ys + [yr, yr, ys[2], gy.ravel()]).astype(np.float32)
    X = np.concatenate(xs + [xr, -xr, np.ones(n, np.float32), gx.ravel()]).astype(np.float32)
    got, ref = impli.debug_libm(2, Y, X), oracle.libm_apply(2, Y, X)
    bad = ~_same_bits(got, ref)
    assert not bad.any(), (Y[bad][:4], X[bad][:4], got[bad][:4], ref[bad][:4])


def test_device_cos_bit_exact(impli, oracle):
    """The screw gradient's double cos on the device (ifunc_device.hpp glibc_cos: glibc 2.35's __cos,
    x86_64 FMA variant, restated) against the oracle's restatement (pinned to the host cos by
    test_cpu.test_cos_restatement_matches_glibc) and the host cos itself: every branch, dense bit
    windows around the branch boundaries and the multiples of pi/2, the screw's own arguments
    (pi x phase), signed zeros, infinities and NaN.  |x| >= 105414336 (__branred) is not restated."""
    rng = np.random.default_rng(2026)
    n = 1 << 21
    edges = np.array([2.0 ** -27, 0.85546875, 2.426265, np.pi / 4, np.pi / 2, np.pi, 3 * np.pi / 2, 2 * np.pi,
                      0.126, 1e3, 105414335.9])
    win = (edges.view(np.int64)[:, None] + np.arange(-4096, 4096)[None, :]).ravel().view(np.float64)
    x = np.concatenate([rng.uniform(-8, 8, n), rng.uniform(-200, 200, n), rng.uniform(-1e8, 1e8, n // 4),
                        np.pi * rng.uniform(-6, 6, n), (rng.uniform(-1, 1, n) * 2.0 ** rng.integers(-40, 2, n)),
                        win, -win, np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-300, -1e-300])])
    # __branred takes every |x| whose high word is >= 0x419921fb, i.e. |x| >= 105414336: not restated
    x = np.where(np.isfinite(x) & (np.abs(x) >= 105414336.0), 0.5, x)   # inf and NaN stay
    got, ref, host = impli.debug_cos(x), oracle.cos_apply(x), oracle.cos_apply(x, glibc=True)
    same = lambda a, b: (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))
    assert same(ref, host).all()
    bad = ~same(got, ref)
    assert not bad.any(), (bad.sum(), x[bad][:6], got[bad][:3], ref[bad][:3])


def _has_twist(shape):
    return "screw" in json.dumps(shape)


def _fold_arrays():
    """Seeded edge-length-fold inputs in the spirit of tools/fold_check.cpp: typical edge lengths,
    wide spreads, integer and half-integer terms (ties), zeros, subnormals, powers of two, binade
    tops with terms at half the spacing, inf / NaN payloads, saturation past 2^24."""
    rng = np.random.default_rng(20261017)
    out = []
    for t in range(48):
        n = int(rng.uniform() * (5000 if t < 32 else 300000))
        x = rng.uniform(size=n)
        kind = t % 8
        e = [0.0144 * (0.5 + x), np.exp2(-30.0 + 60.0 * x), np.floor(1 + 8 * x), np.floor(1 + 64 * x) * 0.5,
             np.where(x < 0.3, 0.0, 1e-3 * x), np.where(x < 0.01, 1e-40 * x, 3.0 * x),
             np.ldexp(1.0, (x * 40).astype(np.int64) - 20), x * x * 100.0][kind]
        out.append(("random%d" % kind, e.astype(np.float32)))
    for t in range(24):
        E = 1 + int(rng.uniform() * 30)
        u = np.ldexp(1.0, E - 24)
        n = 1000 + int(rng.uniform() * 20000)
        x = rng.uniform(size=n)
        body = np.where(x < 0.5, u * (0.5 + (x * 8).astype(np.int64)), u * x * 3)
        head = np.float32(np.ldexp(1.0, E) * (0.5 + 0.49 * rng.uniform()))
        out.append(("ties", np.concatenate([[head], body]).astype(np.float32)))
    out += [("empty", np.zeros(0, np.float32)), ("one", np.ones(1, np.float32)),
            ("zeros", np.array([0.0, -0.0, 0.0], np.float32)), ("leading zeros", np.r_[np.zeros(5000), 0.01 * np.ones(700)].astype(np.float32))]
    e = np.full(100000, 0.0144, np.float32)
    e[50000] = np.inf
    out.append(("inf", e.copy()))
    e[70000] = np.nan
    out.append(("inf+nan", e.copy()))
    e[20000] = np.frombuffer(np.uint32(0x7f801234).tobytes(), np.float32)[0]   # signalling NaN, payload 0x1234
    out.append(("nan payload", e.copy()))
    out.append(("saturation", np.ones(3000000, np.float32)))
    return out


def test_device_edge_fold_matches_serial_chain(impli):
    """The projection's average-edge-length fold (compute_average_edge_length, cp:70-82: s = 0;
    s += e[k], float, in order) as the device computes it -- chunk table plus one-wave walk, no host
    round trip -- against the serial float chain (numpy's add.accumulate is strictly sequential), bit
    for bit; NaN results compared up to the quiet bit (x86 addss returns the NaN operand quieted)."""
    for name, e in _fold_arrays():
        ref = np.add.accumulate(e, dtype=np.float32)[-1] if e.size else np.float32(0.0)
        got, _ = impli.debug_fold(e)
        a, b = np.float32(ref).view(np.uint32), np.float32(got).view(np.uint32)
        if np.isnan(ref):
            assert np.isnan(got) and (int(a) | 0x400000) == (int(b) | 0x400000), (name, hex(int(a)), hex(int(b)))
        else:
            assert a == b, (name, e.size, float(ref), float(got))
    # a typical mesh's terms: most chunks come from the table
    e = _fold_arrays()[0][1]
    big = np.tile(e, 100)
    got, tc = impli.debug_fold(big)
    assert np.float32(got).view(np.uint32) == np.add.accumulate(big, dtype=np.float32)[-1].view(np.uint32)
    assert tc > 0.5 * (big.size // 256), tc


def test_direct_eval_abi_matches_reference_semantics(impli, oracle):
    shape = TREES["union_sphere_cube"]
    pts = np.random.default_rng(5).uniform(-1, 1, size=(1000, 3)).astype(np.float32)
    tree = oracle.mp5_to_nodes(json.dumps(shape))
    with impli.ImplicitService(shape) as svc:
        f = svc.query_implicit_values(pts)
        n = svc.query_normals(pts, normalize_and_invert=True)
    assert np.array_equal(f, oracle.eval_implicit(tree, pts))
    g = oracle.eval_gradient(tree, pts)
    nrm = np.sqrt(g[:, 0] * g[:, 0] + g[:, 1] * g[:, 1] + g[:, 2] * g[:, 2]).astype(np.float32)
    fac = np.where(nrm > 0.0001, (-1.0 / nrm.astype(np.float64)).astype(np.float32), np.float32(-42.0))
    assert np.array_equal(n, (g * fac[:, None]).astype(np.float32))


def test_set_x_limit_and_errors(impli):
    L = impli.lib()
    assert L.set_object(b'{"type":"iellipsoid","matrix":[1,0,0,0,0,1,0,0,0,0,1,0]}', False) == 1
    assert L.set_object(b'{"type":"iellipsoid","matrix":[1,0,0,0,0,1,0,0,0,0,1,0]}', False) == 0
    big = np.zeros((50000, 3), np.float32)
    assert not L.set_x(big.ctypes.data, 50000)          # mcc2.cpp:770 limit kept
    assert L.set_x(big.ctypes.data, 49999)
    L.unset_x()
    assert not L.unset_object(2)
    assert L.unset_object(1)


def _mc_compare(impli, oracle, shape, mc):
    v, f = impli.make_geometry(shape, mc)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    assert f.shape == fr.shape and v.shape == vr.shape, (f.shape, fr.shape, v.shape, vr.shape)
    assert np.array_equal(f, fr)
    assert np.array_equal(v.view(np.uint32), vr.view(np.uint32)), np.abs(v - vr).max()
    return v, f


def test_config1_sphere_mc(impli, oracle):
    from implisolid_amd import scenes
    shape, mc = scenes.config1()
    v, f = _mc_compare(impli, oracle, shape, mc)
    assert v.shape == (3318, 3) and f.shape == (6632, 3)
    _, cnt = mesh_edges(f)
    assert (cnt == 2).all()


@pytest.mark.parametrize("R", [32, 64, 128])
def test_union_sphere_cube_mc(impli, oracle, R):
    from implisolid_amd import scenes
    _mc_compare(impli, oracle, scenes.union_sphere_cube(), scenes.mc_settings(R, 1.0))


@pytest.mark.parametrize("seed", [20251015, 7, 11, 13])
def test_random_tree_mc(impli, oracle, seed):
    from implisolid_amd import scenes
    _mc_compare(impli, oracle, scenes.random_tree(seed, 10), scenes.mc_settings(48, 1.0))


@pytest.mark.parametrize("name", sorted(SCREW_TREES))
def test_screw_family_mc(impli, oracle, name):
    """Twist / lid / half-plane trees: field values are bit-exact (glibc sinf / atan2f restated),
    so the meshes are too."""
    from implisolid_amd import scenes
    for R in (40, 97):
        _mc_compare(impli, oracle, SCREW_TREES[name], scenes.mc_settings(R, 0.7))


def test_config3_twist_tree_mc(impli, oracle):
    from implisolid_amd import scenes
    for R in (48, 128):
        _mc_compare(impli, oracle, scenes.config3_tree(), scenes.mc_settings(R, 1.0))


def test_anisotropic_box_mc(impli, oracle):
    from implisolid_amd import scenes
    mc = scenes.mc_settings(40, 1.0)
    mc["box"] = {"xmin": -0.7, "xmax": 0.9, "ymin": -1.1, "ymax": 0.6, "zmin": -0.55, "zmax": 0.8}
    _mc_compare(impli, oracle, scenes.union_sphere_cube(), mc)


def test_empty_and_full(impli, oracle):
    from implisolid_amd import scenes
    # surface entirely outside the box -> empty mesh; box inside the solid -> sealed shell only
    far = {"type": "iellipsoid", "matrix": scenes.st(0.25, 3.0, 0, 0)}
    v, f = _mc_compare(impli, oracle, far, scenes.mc_settings(16, 1.0))
    assert len(f) == 0 and len(v) == 0
    big = {"type": "iellipsoid", "matrix": scenes.st(8, 0, 0, 0)}
    _mc_compare(impli, oracle, big, scenes.mc_settings(16, 1.0))


def test_hot_object_switches_to_baked_module(impli):
    """Bake mode 2 (default): a slab evaluating the same object runs the shape module first, then
    (after a few evals, compiled in the background) the object's baked module -- with the same
    field, signs and mesh bit for bit; bake mode 0 never switches."""
    import hashlib
    from implisolid_amd import scenes
    mc = scenes.mc_settings(64, 1.0)
    shape = TREES["config3_64"] if "config3_64" in TREES else scenes.config3_tree()
    try:
        for bake in (2, 0):
            impli.set_jit_bake(bake)
            s = impli.Slab(shape, mc)
            try:
                kinds, outs = [], []
                for _ in range(8):
                    s.eval()
                    kinds.append(s.jit_module())
                    outs.append((s.read_field(), s.read_signs()))
                    impli.jit_wait()
                nv, nf = s.run()
                v, f = s.download(nv, nf)
            finally:
                s.close()
            assert ("baked" in kinds) == (bake == 2), kinds
            assert kinds[-1] == ("baked" if bake == 2 else "shape"), kinds
            fa, sa = outs[0]
            for fb, sb in outs[1:]:
                assert np.array_equal(fa.view(np.uint32), fb.view(np.uint32))
                assert np.array_equal(sa, sb)
            key = hashlib.sha256(np.ascontiguousarray(f).tobytes() + np.ascontiguousarray(v).tobytes()).hexdigest()
            if bake == 2:
                ref = key
            else:
                assert key == ref
    finally:
        impli.set_jit_bake(2)


@pytest.mark.parametrize("level", [1, 2])
@pytest.mark.parametrize("name", sorted(TREES))
def test_jit_field_matches_interpreter(impli, name, level):
    """The hipRTC-compiled tree kernels (interval pass and field) -- per-shape modules (matrices
    read from memory) and per-object modules with the matrices baked in as literals -- and the
    interpreter produce the same field, sign bitmap and brick classes bit for bit."""
    from implisolid_amd import scenes
    mc = scenes.mc_settings(48, 1.0)
    out = []
    impli.set_pruning(level)
    try:
        for mode, bake in ((0, False), (1, False), (1, True)):
            impli.set_jit(mode)
            impli.set_jit_bake(bake)
            s = impli.Slab(TREES[name], mc)
            try:
                s.eval()
                assert s.used_jit() == bool(mode)
                out.append((s.read_field(), s.read_signs(), s.brick_stats()))
            finally:
                s.close()
    finally:
        impli.set_jit(2)
        impli.set_jit_bake(2)
        impli.set_pruning(2)
    fa, sa, ba = out[0]
    for fb, sb, bb in out[1:]:
        assert np.array_equal(fa.view(np.uint32), fb.view(np.uint32)), np.flatnonzero(fa != fb)[:10]
        assert np.array_equal(sa, sb)
        assert ba == bb


def test_jit_module_bound_unloads_idle_modules(impli, oracle):
    """The loaded-module bound: with one baked module per object and room for 8, polygonising 14
    objects one after another unloads the least recently used idle modules (never one a live slab
    holds); an object seen again is rebuilt (disk cache or hipRTC) with the same mesh, which is the
    oracle's."""
    import hashlib
    from implisolid_amd import scenes
    mc = scenes.mc_settings(32, 1.0)
    shapes = [scenes.random_tree(515000 + k, 3) for k in range(14)]
    impli.set_jit(1)
    impli.set_jit_bake(1)
    impli.set_jit_max_modules(8)
    ev0 = impli.jit_stats()["evicted"]

    def mesh(shape):
        s = impli.Slab(shape, mc)
        try:
            nv, nf = s.run()
            assert s.used_jit()
            st = impli.jit_stats()
            assert st["modules"] <= 9, st   # the bound, plus the module just requested
            return s.download(nv, nf)
        finally:
            s.close()

    try:
        first = mesh(shapes[0])
        held = impli.Slab(shapes[1], mc)   # a live slab's module is never unloaded
        try:
            held.run()
            for sh in shapes[2:]:
                mesh(sh)
            assert impli.jit_stats()["evicted"] > ev0
            nv, nf = held.run()            # its module is still loaded: no fault, same kernels
            vh, fh = held.download(nv, nf)
        finally:
            held.close()
        again = mesh(shapes[0])
    finally:
        impli.set_jit_max_modules(1024)
        impli.set_jit(2)
        impli.set_jit_bake(2)
    for (v, f), sh in ((first, shapes[0]), (again, shapes[0]), ((vh, fh), shapes[1])):
        vr, fr = oracle.polygonize(json.dumps(sh), json.dumps(mc))
        assert np.array_equal(f, fr) and np.array_equal(v.view(np.uint32), vr.view(np.uint32))
    assert hashlib.sha256(first[1].tobytes()).digest() == hashlib.sha256(again[1].tobytes()).digest()


def test_jit_module_bound_two_threads(impli, oracle):
    """The module bound under concurrent requests: two host threads polygonise 10
    different objects each through their own slabs (ctypes drops the GIL inside the library), with
    one baked module per object and room for 8.  A request that finds its slot takes the reference
    under the lookup's lock, so another thread's eviction can never unload a module in use: every
    mesh is the oracle's."""
    import threading
    from implisolid_amd import scenes
    mc = scenes.mc_settings(32, 1.0)
    shapes = [[scenes.random_tree(616000 + 100 * t + k, 3) for k in range(10)] for t in range(2)]
    out = [[None] * 10 for _ in range(2)]
    errs = []

    def work(t):
        try:
            for k, sh in enumerate(shapes[t]):
                for _ in range(2):   # the second pass finds the slot (or a rebuilt one) in the cache
                    s = impli.Slab(sh, mc)
                    try:
                        nv, nf = s.run()
                        out[t][k] = s.download(nv, nf)
                    finally:
                        s.close()
        except Exception as e:   # reported by the main thread
            errs.append(e)

    impli.set_jit(1)
    impli.set_jit_bake(1)
    impli.set_jit_max_modules(8)
    try:
        th = [threading.Thread(target=work, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        impli.set_jit_max_modules(1024)
        impli.set_jit(2)
        impli.set_jit_bake(2)
    assert not errs, errs
    for t in range(2):
        for k, sh in enumerate(shapes[t]):
            vr, fr = oracle.polygonize(json.dumps(sh), json.dumps(mc))
            v, f = out[t][k]
            assert np.array_equal(f, fr) and np.array_equal(v.view(np.uint32), vr.view(np.uint32)), (t, k)


@pytest.mark.parametrize("level", [1, 2])
def test_same_grid_new_object_resets_buffers(impli, oracle, level):
    """build_geometry of one object, then of another on the same grid: the engine keeps
    an unchanged grid's buffers only while the object is unchanged too, so the second object never
    reads the first one's signs (at pruning level 1 the unlisted bricks' sign words are not
    rewritten).  Both meshes, and the first object's again, are the oracle's."""
    from implisolid_amd import scenes
    impli.set_pruning(level)
    try:
        mc = scenes.mc_settings(56, 1.0)
        a, b = scenes.union_sphere_cube(), scenes.config3()[0]
        for sh in (a, b, a, b):
            _mc_compare(impli, oracle, sh, mc)
    finally:
        impli.set_pruning(2)


def test_jit_async_first_call_then_compiled(impli, oracle):
    """Async JIT (the default): a never-seen shape is polygonised at once with the interpreter
    kernels while its module compiles in the background; after jit_wait() the same slab's eval runs
    the compiled kernels.  Both meshes are the oracle's."""
    from implisolid_amd import scenes
    shape = scenes.random_tree(424242, 7)      # a shape no other test compiles
    mc = scenes.mc_settings(40, 1.0)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    impli.set_jit(2)
    s = impli.Slab(shape, mc)
    try:
        s.eval()
        first = s.used_jit()
        s.count()
        nv, nf, _ = s.counts()
        s.emit()
        v0, f0 = s.download(*s.counts()[:2])
        impli.jit_wait()
        s.eval()
        assert s.used_jit() and not first
        s.count()
        s.emit()
        v1, f1 = s.download(*s.counts()[:2])
    finally:
        s.close()
    for v, f in ((v0, f0), (v1, f1)):
        assert np.array_equal(f, fr) and np.array_equal(v.view(np.uint32), vr.view(np.uint32))


@pytest.mark.parametrize("level", [0, 1, 2])
def test_mc_identical_at_every_pruning_level(impli, oracle, level):
    from implisolid_amd import scenes
    impli.set_pruning(level)
    try:
        _mc_compare(impli, oracle, scenes.config3()[0], scenes.mc_settings(64, 1.0))
        _mc_compare(impli, oracle, scenes.union_sphere_cube(), scenes.mc_settings(50, 1.0))
    finally:
        impli.set_pruning(2)


@pytest.mark.parametrize("seed", list(range(300, 312)))
def test_pruning_levels_agree_random_twist_trees(impli, seed):
    """Random trees with twists at odd and even resolutions (partial bricks and coarse boxes at the
    grid's ends, one-layer top bricks): the default pipeline -- per-layer refinement, neighbour
    candidates claimed by their mixed neighbours, chunk marks -- gives the unpruned mesh bit for bit."""
    from implisolid_amd import scenes
    shape = scenes.random_tree(seed, 4 + seed % 9, twist_leaves=True)
    R = [23, 31, 45, 66, 37, 52][seed % 6]
    mc = scenes.mc_settings(R, 1.0)
    out = []
    try:
        for level in (0, 2):
            impli.set_pruning(level)
            out.append(impli.make_geometry(shape, mc))
    finally:
        impli.set_pruning(2)
    (v0, f0), (v2, f2) = out
    assert np.array_equal(f0, f2) and np.array_equal(v0.view(np.uint32), v2.view(np.uint32))


@pytest.mark.parametrize("nranks", [2, 3, 5])
def test_zslab_split_identical(impli, oracle, nranks):
    """Z-slab decomposition (one-layer recomputed halo, global offsets) == single GPU."""
    from implisolid_amd import scenes
    shape, mc = scenes.union_sphere_cube(), scenes.mc_settings(64, 1.0)
    ref_v, ref_f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    slabs = [impli.Slab(shape, mc, r, nranks) for r in range(nranks)]
    counts = []
    for s in slabs:
        s.eval()
        s.count()
        counts.append(s.counts()[:2])
    voff = np.concatenate([[0], np.cumsum([c[0] for c in counts])])
    foff = np.concatenate([[0], np.cumsum([c[1] for c in counts])])
    vs, fs, st = [], [], []
    for r, s in enumerate(slabs):
        s.set_offsets(int(voff[r]), int(foff[r]))
        s.emit()
        nv, nf, of = s.counts()
        assert not of
        v, f = s.download(nv, nf)
        vs.append(v)
        fs.append(f)
        st.append(s.stats())
        s.close()
    v = np.concatenate(vs)
    f = np.concatenate(fs)
    assert np.array_equal(f, ref_f)
    assert np.array_equal(v.view(np.uint32), ref_v.view(np.uint32))
    # every counter slot: the halo count the vertex pass reads is the totals block's; the slabs'
    # owned-minus-halo vertices, triangles and active cells add up to the oracle's mesh
    for k, c in enumerate(st):
        assert c["halo_own"] == c["halo_own_verts_pass"], k
        assert (c["halo_own"] == 0) == (k == 0), k
        assert c["unit_parts"] >= c["nonempty_units"] > 0, k
    assert sum(c["own"] - c["halo_own"] for c in st) == len(ref_v)
    assert sum(c["tri"] for c in st) == len(ref_f)
    one = impli.Slab(shape, mc, 0, 1)
    one.eval()
    one.count()
    assert sum(c["act"] for c in st) == one.stats()["act"]
    one.close()


@pytest.mark.parametrize("nranks", [2, 5])
def test_zslab_gathered_counts_identical(impli, oracle, nranks):
    """The multi-GPU step's emit path: vertex pass, then the face pass taking its vertex offset
    from every slab's gathered counts on the device == single GPU."""
    import torch
    from implisolid_amd import scenes
    shape, mc = scenes.config3(64)[0], scenes.mc_settings(64, 1.0)
    ref_v, ref_f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    slabs = [impli.Slab(shape, mc, r, nranks) for r in range(nranks)]
    gath = torch.zeros(nranks, 4, dtype=torch.int32, device="cuda")
    for r, s in enumerate(slabs):
        s.eval()
        s.count()
        s.counts()   # sizes the output buffers
        s.copy_counts(gath[r].data_ptr())
    torch.cuda.synchronize()
    vs, fs = [], []
    for r, s in enumerate(slabs):
        s.emit_verts()
        s.emit_faces(0, gath.data_ptr(), r)
        nv, nf, of = s.counts()
        assert not of
        v, f = s.download(nv, nf)
        vs.append(v)
        fs.append(f)
        s.close()
    assert np.array_equal(np.concatenate(fs), ref_f)
    assert np.array_equal(np.concatenate(vs).view(np.uint32), ref_v.view(np.uint32))


def _ob02_compare(impli, oracle, shape, mc, exact=None):
    """Faces bit-exact; vertices bit-exact (exact=False: within 1e-5, the north-star vertex
    tolerance).  Non-finite reference vertices (a
    zero gradient at a singular point that lands on a grid sample: normalize_1111 divides by its
    norm, normalise_inplace.hpp:60-70) must be non-finite in the same rows."""
    if exact is None:
        exact = True   # twists too: the screw gradient's double cos is glibc's, restated
    v, f = impli.make_geometry(shape, mc)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    assert np.array_equal(f, fr)
    fin = np.isfinite(vr).all(1)
    assert np.array_equal(np.isfinite(v).all(1), fin)
    v_, vr_ = v[fin], vr[fin]
    bad = np.flatnonzero((v_ != vr_).any(1))
    if exact:
        assert bad.size == 0, (bad.size, bad[:10], np.abs(v_ - vr_).max())
    elif v_.size:
        assert np.abs(v_ - vr_).max() < 1e-5, (bad.size, np.abs(v_ - vr_).max())
    return v, vr


def test_ob02_resampling_only(impli, oracle):
    from implisolid_amd import scenes
    mc = scenes.mc_settings(40, 1.0, vresampl_iters=2, vresampl_c=0.4)
    _ob02_compare(impli, oracle, scenes.union_sphere_cube(), mc)


@pytest.mark.parametrize("edit", ["boundary", "nonmanifold", "degenerate"])
def test_ob02_resampling_irregular_topology(impli, oracle, edit):
    """Faces of faces from the umbrellas (ob02.hip k_fof_umbrella) on meshes marching cubes never
    makes -- boundary edges (faces removed), edges of three or four faces (faces repeated, one
    reversed), degenerate faces with a repeated vertex -- give the oracle's resampling bit for bit
    (first / last face of an edge and its half-edge count, mesh_algorithms.hpp:111-121)."""
    import torch
    from implisolid_amd import scenes
    shape = scenes.union_sphere_cube()
    mc = scenes.mc_settings(24, 1.0, vresampl_iters=1, vresampl_c=0.4)
    v, f = impli.make_geometry(shape, scenes.mc_settings(24, 1.0))
    f = f.copy()
    if edit == "boundary":
        f = np.delete(f, [5, 17, 40], axis=0)
    elif edit == "nonmanifold":
        f = np.concatenate([f, f[[3, 9]], f[[20]][:, ::-1]])
    else:
        f = np.concatenate([f, [[f[7, 0], f[7, 0], f[7, 1]], [f[11, 2], f[11, 1], f[11, 2]]]])
    f = np.ascontiguousarray(f, dtype=np.int32)
    tree = oracle.mp5_to_nodes(json.dumps(shape))
    vr, _ = oracle.vertex_resampling(tree, v, f, 0.4)
    V = torch.from_numpy(v.reshape(-1).copy()).cuda()
    F = torch.from_numpy(f.reshape(-1).copy()).cuda()
    ob = impli.Ob02Shard(shape, mc)
    try:
        ob.load(V.data_ptr(), len(v), F.data_ptr(), len(f), 0, len(v))
        ob.resample()
        vg, fg = ob.download()
    finally:
        ob.close()
    assert np.array_equal(fg, f)
    same = (vg.view(np.uint32) == vr.view(np.uint32)) | (np.isnan(vg) & np.isnan(vr))
    assert same.all(), (edit, np.argwhere(~same)[:5])


def test_ob02_projection_no_qem(impli, oracle):
    from implisolid_amd import scenes
    mc = scenes.mc_settings(40, 1.0, vresampl_iters=1, vresampl_c=0.4, projection=1, qem=0)
    _ob02_compare(impli, oracle, scenes.union_sphere_cube(), mc)
    ref_tree = oracle.mp5_to_nodes(json.dumps(scenes.union_sphere_cube()))
    p = impli.get_pointset("post_p_centroids")
    assert p is not None and p.shape[1] == 3


@pytest.mark.parametrize("repeats", [1, 2])
def test_ob02_pointsets_taken_in_order(impli, oracle, repeats):
    """The reference's STORE_POINTSET records (configs.hpp:106, centroids_projection.cpp:1238-1285)
    are copied on a stream of their own in build_geometry: each must still hold the array as it was
    at its point of the loop.  Checked against what they must equal: the final vertices
    (post_qem_verts), the mesh after the last resampling (pre_qem_verts: the projection moves no
    vertex; with one repeat, the result of the same loop without projection), the centroids of that
    mesh (pre_p_centroids, f32 in compute_centroids' order).  (The resampling records keep the
    process's first build, vertex_resampling.hpp:176-211, so they are not this build's.)"""
    from implisolid_amd import scenes
    shape, mc = scenes.config2(40)
    mc = dict(mc, overall_repeats=repeats)
    v, f = impli.make_geometry(shape, mc)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    bits = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
    assert np.array_equal(f, fr) and np.array_equal(bits(v), bits(vr))
    ps = {k: impli.get_pointset(k) for k in ("pre_p_centroids", "post_p_centroids", "pre_qem_verts", "post_qem_verts")}
    assert np.array_equal(bits(ps["post_qem_verts"]), bits(v))
    pre = ps["pre_qem_verts"]
    c = pre[f]
    cen = ((c[:, 0] + c[:, 1]) + c[:, 2]) / np.float32(3.0)
    assert np.array_equal(bits(ps["pre_p_centroids"]), bits(cen))
    assert ps["post_p_centroids"].shape == (len(f), 3)
    if repeats == 1:
        v_res, _ = impli.make_geometry(shape, dict(mc, projection={"enabled": 0}, qem={"enabled": 0}))
        assert np.array_equal(bits(pre), bits(v_res))


@pytest.mark.parametrize("R", [32, 48])
def test_ob02_full_config2_shape(impli, oracle, R):
    from implisolid_amd import scenes
    shape, mc = scenes.config2(R)
    _ob02_compare(impli, oracle, shape, mc)


@pytest.mark.parametrize("name", ["twist", "twist_two_plane", "half_plane", "tetrahedron", "meta_balls", "extrusion"])
def test_ob02_screw_family(impli, oracle, name):
    from implisolid_amd import scenes
    mc = scenes.mc_settings(40, 0.7, vresampl_iters=1, vresampl_c=0.4, projection=1, qem=1, overall_repeats=2)
    _ob02_compare(impli, oracle, SCREW_TREES[name], mc)


def test_ob02_config3_tree_small(impli, oracle):
    from implisolid_amd import scenes
    shape, mc = scenes.config3(40)
    _ob02_compare(impli, oracle, shape, mc)


def test_ob02_config3_nonfinite_rows(impli, oracle):
    """config 3 at R = 64: centroids of degenerate faces sit exactly on singular points of the tree
    (zero gradient), so the reference's resampling produces non-finite vertices (668 of 5524 after 3
    repeats); the GPU reproduces the same rows, faces and every finite vertex."""
    from implisolid_amd import scenes
    shape, mc = scenes.config3(64)
    v, vr = _ob02_compare(impli, oracle, shape, mc)
    assert (~np.isfinite(vr).all(1)).sum() > 0


@pytest.fixture
def sync_jit(impli):
    """JIT in sync mode: every new shape's modules are compiled before its first use, so the JIT
    kernels (not the interpreter) run from the first call."""
    impli.set_jit(1)
    yield
    impli.set_jit(2)


@pytest.mark.parametrize("bake", [False, True])
@pytest.mark.parametrize("name", ["config2_48", "config3_64", "twist_tbb", "meta_balls"])
def test_ob02_point_jit_matches_oracle(impli, oracle, sync_jit, name, bake):
    """The OB02 passes over the JIT point module (ob02_device.hpp bodies over straight-line tree
    code) give the oracle's mesh -- config 3 at 64 includes the non-finite rows (NaN centroids
    through the unspecialised transforms).  bake: the module with the object's matrices as literals
    (a hot object's, here from the first build) -- the same operations on the same values."""
    from implisolid_amd import scenes
    if name == "config2_48":
        shape, mc = scenes.config2(48)
    elif name == "config3_64":
        shape, mc = scenes.config3(64)
    else:
        shape = SCREW_TREES[name]
        mc = scenes.mc_settings(40, 0.7, vresampl_iters=1, vresampl_c=0.4, projection=1, qem=1, overall_repeats=2)
    if bake:
        impli.set_jit_bake(1)
    try:
        _ob02_compare(impli, oracle, shape, mc)
    finally:
        impli.set_jit_bake(2)
    assert impli.last_build_stats()["jit_launches"] > 0


def test_ob02_hot_object_switches_to_baked_point_module(impli, oracle):
    """The default bake policy: an object built again and again gets its point module rebuilt with
    its matrices baked in (in the background, after 4 builds' worth of OB02 steps) and switches to
    it; every build's mesh is the oracle's, before and after the switch."""
    from implisolid_amd import scenes
    shape, mc = scenes.config3_shifted(64)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    for k in range(7):
        v, f = impli.make_geometry(shape, mc)
        assert np.array_equal(f, fr) and np.array_equal(v.view(np.uint32), vr.view(np.uint32)), k
        if k == 4:
            impli.jit_wait()   # the baked modules requested during builds 4-5 are loaded from here on


@pytest.mark.parametrize("bake", [False, True])
@pytest.mark.parametrize("name", ["config3_tree", "union_sphere_cube", "twist_tbb", "extrusion_tri", "leaf_cube"])
def test_eval_points_jit_bit_exact(impli, oracle, sync_jit, name, bake):
    """Direct evaluation through the JIT point module, including non-finite coordinates (the
    interpreter's transforms propagate NaN through zero coefficients, and so must the JIT's -- with
    the matrices baked in as literals too)."""
    shape = TREES[name]
    rng = np.random.default_rng(77)
    pts = rng.uniform(-1.1, 1.1, size=(20000, 3)).astype(np.float32)
    pts[:50, 1] = np.nan
    pts[50:100, 0] = np.inf
    pts[100:150, 2] = -np.inf
    tree = oracle.mp5_to_nodes(json.dumps(shape))
    f_ref, g_ref = oracle.eval_implicit(tree, pts), oracle.eval_gradient(tree, pts)
    if bake:
        impli.set_jit_bake(1)
    try:
        with impli.ImplicitService(shape) as svc:
            f, g = svc.eval(pts, gradient=True)
    finally:
        impli.set_jit_bake(2)
    assert np.array_equal(f.view(np.uint32), f_ref.view(np.uint32)) or np.array_equal(
        np.isnan(f), np.isnan(f_ref)) and np.array_equal(f[~np.isnan(f)], f_ref[~np.isnan(f_ref)])
    ok = np.isfinite(g_ref).all(1)
    assert np.array_equal(np.isfinite(g).all(1), ok)
    assert np.array_equal(g[ok].view(np.uint32), g_ref[ok].view(np.uint32))


def _field(impli, shape, mc, level, signs=False):
    impli.set_pruning(level)
    try:
        s = impli.Slab(shape, mc)
        s.eval()
        f = s.read_field()
        sg = s.read_signs()
        s.close()
    finally:
        impli.set_pruning(2)
    if level < 2:   # the sign bitmap always matches a fully written field
        assert np.array_equal(sg.astype(bool), f < 0)
    return (f, sg) if signs else f


def _needed_samples(f):
    """Stored samples whose exact value marching cubes can read: the ends of a sign-changing
    axis edge (the sealed ring is stored, so every edge a cell has lies inside the array)."""
    neg = f < 0
    need = np.zeros_like(neg)
    for ax in range(3):
        a = np.moveaxis(neg, ax, 0)
        nv = np.moveaxis(need, ax, 0)
        d = a[1:] != a[:-1]
        nv[1:] |= d
        nv[:-1] |= d
    return need


@pytest.mark.parametrize("name", sorted(TREES))
def test_pruned_field_identical(impli, name):
    """Per-brick interval pruning must not change a single bit of the field."""
    from implisolid_amd import scenes
    for R, box in [(64, None), (37, {"xmin": -0.7, "xmax": 0.9, "ymin": -1.1, "ymax": 0.6, "zmin": -0.55, "zmax": 0.8})]:
        mc = scenes.mc_settings(R, 1.0)
        if box:
            mc["box"] = box
        a = _field(impli, TREES[name], mc, 1)
        b = _field(impli, TREES[name], mc, 0)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), np.flatnonzero(a != b)[:10]
        c, cs = _field(impli, TREES[name], mc, 2, signs=True)
        assert np.array_equal(cs.astype(bool), b < 0)
        need = _needed_samples(b)
        assert np.array_equal(c[need].view(np.uint32), b[need].view(np.uint32))


@pytest.mark.parametrize("seed", list(range(100, 124)))
def test_pruned_field_random_trees(impli, seed):
    from implisolid_amd import scenes
    shape = scenes.random_tree(seed, 3 + seed % 10)
    mc = scenes.mc_settings(48, 1.0)
    a = _field(impli, shape, mc, 1)
    b = _field(impli, shape, mc, 0)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), np.flatnonzero(a != b)[:10]
    c, cs = _field(impli, shape, mc, 2, signs=True)
    assert np.array_equal(cs.astype(bool), b < 0)
    need = _needed_samples(b)
    assert np.array_equal(c[need].view(np.uint32), b[need].view(np.uint32))


@pytest.mark.parametrize("pitch,delta_ratio,off", [(0.5, 1.5, (0, 0, 0)), (-0.3, 1.5, (0.2, -0.1, 0.05)),
                                                   (0.0625, 3.0, (0, 0.3, 0)), (2.0, 1.2, (-0.25, 0, 0.1)),
                                                   (-4.0, 2.0, (0.1, 0.1, -0.2))])
def test_pruned_field_twist_phase_bounds(impli, pitch, delta_ratio, off):
    """The screw's interval bound follows the sine's phase over the brick (screw_sin_iv): unions
    and differences of twists with other leaves must keep every needed field bit."""
    from implisolid_amd import scenes
    tw = scenes.twist(0.8, *off, pitch=pitch, delta_ratio=delta_ratio)
    for shape in (tw,
                  {"type": "Union", "matrix": scenes.EYE, "children": [tw, scenes.twist(0.5, 0.3, 0.2, 0.1, pitch=-pitch)]},
                  {"type": "Difference", "matrix": scenes.EYE,
                   "children": [tw, dict(scenes.twist(0.4, -0.1, 0, 0, pitch=pitch * 0.7), type="screw_gradient_wrong")]}):
        mc = scenes.mc_settings(56, 1.0)
        a = _field(impli, shape, mc, 1)
        b = _field(impli, shape, mc, 0)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), np.flatnonzero(a != b)[:10]
        c, cs = _field(impli, shape, mc, 2, signs=True)
        assert np.array_equal(cs.astype(bool), b < 0)
        need = _needed_samples(b)
        assert np.array_equal(c[need].view(np.uint32), b[need].view(np.uint32))


# ---- against the committed golden fixtures (tests/golden/make_golden.py) ---------------------------
def _golden(name):
    import os
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name)


def test_golden_config1_gpu(impli):
    g = np.load(_golden("config1_mc.npz"))
    v, f = impli.make_geometry(str(g["shape"]), str(g["mc"]))
    assert np.array_equal(f, g["faces"]) and np.array_equal(v.view(np.uint32), g["verts"].view(np.uint32))


def test_golden_points_gpu(impli):
    g = np.load(_golden("points_eval.npz"))
    trees = json.loads(str(g["trees"]))
    for name, sh in trees.items():
        with impli.ImplicitService(sh) as svc:
            f, gr = svc.eval(g["points"], gradient=True)
        assert np.array_equal(f.view(np.uint32), g["f_" + name].view(np.uint32)), name
        assert np.array_equal(gr.view(np.uint32), g["g_" + name].view(np.uint32)), name


def test_golden_config2_ob02_gpu(impli):
    g = np.load(_golden("config2_r32_ob02.npz"))
    v, f = impli.make_geometry(str(g["shape"]), str(g["mc"]))
    assert np.array_equal(f, g["faces"]) and np.array_equal(v.view(np.uint32), g["verts"].view(np.uint32))
    p = impli.get_pointset("post_p_centroids")
    assert np.array_equal(p.view(np.uint32), g["tap_post_p_centroids"][-1].view(np.uint32))


def test_golden_mc_summaries_gpu(impli):
    import hashlib
    from implisolid_amd import scenes
    d = json.load(open(_golden("mc_summaries.json")))
    for name, s in d.items():
        mc = scenes.mc_settings(s["R"], 1.0)
        v, f = impli.make_geometry(s["shape"], mc)
        assert (len(v), len(f)) == (s["n_verts"], s["n_faces"]), name
        assert hashlib.sha256(np.ascontiguousarray(f).tobytes()).hexdigest() == s["sha256_faces"], name
        assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == s["sha256_verts"], name


def test_node_addon_config1_gpu(impli):
    import os
    import shutil
    import subprocess
    if not (shutil.which("node") and os.path.exists("/usr/include/node/node_api.h")):
        pytest.skip("node or node headers absent")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "bindings", "node")], check=True)
    g = np.load(_golden("config1_mc.npz"))
    js = ("const {make_geometry} = require('./bindings/node/impli1.js');"
          "const fs = require('fs');"
          "make_geometry(process.argv[1], process.argv[2], (v, f) => {"
          "  fs.writeFileSync(process.argv[3], Buffer.from(v.buffer));"
          "  fs.writeFileSync(process.argv[4], Buffer.from(f.buffer)); });")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        vp, fp = os.path.join(d, "v.bin"), os.path.join(d, "f.bin")
        r = subprocess.run(["node", "-e", js, str(g["shape"]), str(g["mc"]), vp, fp], cwd=root,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        v = np.fromfile(vp, np.float32).reshape(-1, 3)
        f = np.fromfile(fp, np.uint32).reshape(-1, 3).astype(np.int32)
    assert np.array_equal(f, g["faces"]) and np.array_equal(v.view(np.uint32), g["verts"].view(np.uint32))


def test_progress_callbacks_match_oracle_stages(impli, oracle):
    """build_geometry_u reports the mesh where the reference's send_mesh_back_to_client does
    (mcc2.cpp:351, 372, 390): after marching cubes, after each repeat's resampling and after each
    projection -- 1 + 2 x 3 updates for config 2 -- carrying the call specs' ids.  The MC update and
    the after-projection updates equal the oracle run with 0..3 repeats; the last is the result."""
    from implisolid_amd import scenes
    shape, mc = scenes.config2(32)
    specs = {"progressCallback_id": 7, "call_id": 3, "shape_id": 11}
    v, f, ups = impli.make_geometry_progressive(shape, mc, json.dumps(specs))
    assert len(ups) == 1 + 2 * mc["overall_repeats"]
    assert all(u[2:] == (7, 11, 3) for u in ups)
    stages = [(0, scenes.mc_settings(32, 1.0))]
    for r in (1, 2, 3):
        stages.append((2 * r, dict(mc, overall_repeats=r)))
    for k, m in stages:
        vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(m))
        uv, uf = ups[k][0], ups[k][1]
        assert np.array_equal(uf, fr), k
        assert np.array_equal(uv.view(np.uint32), vr.view(np.uint32)), k
    assert np.array_equal(v.view(np.uint32), ups[-1][0].view(np.uint32)) and np.array_equal(f, ups[-1][1])
    # no call specs: -1 ids; config 1 (1 repeat, 0 resampling iterations, no projection) reports
    # after MC and after the repeat's (empty) resampling loop, as the reference does
    _, _, ups = impli.make_geometry_progressive(*scenes.config1(), None)
    assert len(ups) == 2 and all(u[2:] == (-1, -1, -1) for u in ups)


def test_node_addon_progressive_gpu(impli):
    """The worker path from JavaScript: build_geometry_u with call specs and a progress function,
    called like wwapi.send_progress_update (js/worker_api.js:399-416)."""
    import os
    import shutil
    import subprocess
    from implisolid_amd import scenes
    if not (shutil.which("node") and os.path.exists("/usr/include/node/node_api.h")):
        pytest.skip("node or node headers absent")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "bindings", "node")], check=True)
    shape, mc = scenes.config2(24)
    js = ("const {impli1} = require('./bindings/node/impli1.js');"
          "const seen = [];"
          "impli1.build_geometry_u(process.argv[1], process.argv[2], JSON.stringify({progressCallback_id: 5, call_id: 2, shape_id: 9}),"
          "  (v, f, pid, sid, cid) => seen.push([v.length / 3, f.length / 3, pid, sid, cid]));"
          "console.log(JSON.stringify({seen, nv: impli1.get_v_size(), nf: impli1.get_f_size()}));"
          "impli1.finish_geometry();")
    r = subprocess.run(["node", "-e", js, json.dumps(shape), json.dumps(mc)], cwd=root, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(out["seen"]) == 7 and all(s[2:] == [5, 9, 2] for s in out["seen"])
    assert out["seen"][-1][:2] == [out["nv"], out["nf"]]


# ---- step 3: subdivision (my_subdiv_, centroids_projection.cpp:1314-1367) -------------------------
def _subdiv_compare(impli, oracle, shape, mc, seed):
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    impli.srand(seed)
    v, f = impli.make_geometry(shape, mc)
    # hipRTC (LLVM's Process::GetRandomNumber) calls the process-global srand()/rand(): let the
    # background compile of this shape finish before the oracle draws from glibc's generator
    impli.jit_wait()
    oracle.srand(seed)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    assert np.array_equal(f, fr)
    bad = np.flatnonzero((v.view(np.uint32) != vr.view(np.uint32)).any(1))
    assert bad.size == 0, (bad.size, bad[:10], np.abs(v - vr).max())
    # both generators continue from the same state
    assert [impli.rand() for _ in range(5)] == [libc.rand() for _ in range(5)]
    return v, f


@pytest.mark.parametrize("noise", [0.0, 0.01, 0.5])
def test_subdivision_config1(impli, oracle, noise):
    from implisolid_amd import scenes
    mc = scenes.mc_settings(32, 0.6, subdiv=1, post_subdiv_noise=noise)
    v, f = _subdiv_compare(impli, oracle, scenes.config1()[0], mc, 1)
    assert f.shape == (4 * 6632, 3) and v.shape == (3318 + 3 * 6632 // 2, 3)


@pytest.mark.parametrize("R", [24, 96])
def test_subdivision_after_ob02(impli, oracle, R):
    """config 2's loop with subdivision on the last of 3 repeats (polygonize_step_3, noise x10)."""
    from implisolid_amd import scenes
    mc = scenes.mc_settings(R, 1.0, vresampl_iters=1, vresampl_c=0.4, projection=1, qem=1, overall_repeats=3,
                            subdiv=1, post_subdiv_noise=0.01)
    _subdiv_compare(impli, oracle, scenes.union_sphere_cube(), mc, 20251015)


def test_subdivision_mc_only_large_and_empty(impli, oracle):
    """R 160 (~4k noise lanes: every row of the jump table) and an empty mesh (noise on nothing)."""
    from implisolid_amd import scenes
    shape = scenes.union_sphere_cube()
    _subdiv_compare(impli, oracle, shape, scenes.mc_settings(160, 1.0, subdiv=1, post_subdiv_noise=0.02), 3)
    far = {"type": "iellipsoid", "matrix": scenes.st(0.25, 5, 5, 5)}
    v, f = _subdiv_compare(impli, oracle, far, scenes.mc_settings(16, 1.0, subdiv=1, post_subdiv_noise=0.01), 4)
    assert v.shape[0] == 0 and f.shape[0] == 0


def test_subdivision_repeats_without_last(impli, oracle):
    """overall_repeats 1 subdivides once with noise; default settings (subdiv on) go through it."""
    from implisolid_amd import scenes
    shape = scenes.config3(24)[0]
    mc = scenes.mc_settings(24, 1.0, vresampl_iters=1, vresampl_c=0.4, projection=1, qem=0, overall_repeats=1,
                            subdiv=1, post_subdiv_noise=0.01)
    _subdiv_compare(impli, oracle, shape, mc, 77)


def test_golden_subdivision_gpu(impli):
    g = np.load(_golden("subdiv.npz"))
    for name in ["config1", "config2_r24"]:
        impli.srand(1)
        v, f = impli.make_geometry(str(g[name + "_shape"]), str(g[name + "_mc"]))
        assert np.array_equal(f, g[name + "_faces"]), name
        assert np.array_equal(v.view(np.uint32), g[name + "_verts"].view(np.uint32)), name


# ---- object stream (config 5): hipGraph-captured per-object pipelines --------------------------
@pytest.mark.parametrize("n_streams", [0, 3])
def test_batch_stream_matches_oracle(impli, oracle, n_streams):
    """The object stream, merged launches (n_streams 0: one launch per stage for all objects, block
    row = object) and per-object graphs over streams: every object's mesh is the oracle's."""
    from implisolid_amd import scenes
    objs = scenes.config5_objects(10, 56) + [(scenes.config3_tree(), scenes.mc_settings(56, 1.0))]
    shapes, mc = [o[0] for o in objs], objs[0][1]
    with impli.Batch(shapes, mc, n_streams=n_streams) as b:
        assert b.n == len(shapes) and b.merged == (n_streams == 0)
        for rep in range(2):                   # replays give the same meshes
            b.run()
            for i, sh in enumerate(shapes):
                v, f = b.download(i)
                vr, fr = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(sh)), 56, [-1, 1] * 3)
                assert np.array_equal(f, fr), (rep, i)
                assert np.array_equal(v.view(np.uint32), vr.view(np.uint32)), (rep, i)


def _depth_class_objects():
    """Objects of every depth class of the merged batch (abi.hip implisolid_batch: stacks of 9, 12 and
    16 slots, the deeper classes on the batch's side stream) with rotated and sheared matrices (x and
    y rows that read z, so the layer pair's samples differ in every coordinate)."""
    import math
    import random
    from implisolid_amd import scenes
    rng = random.Random(4242)

    def rot(a, b, t):
        ca, sa, cb, sb = math.cos(a), math.sin(a), math.cos(b), math.sin(b)
        return [ca, -sa * cb, sa * sb, t[0], sa, ca * cb, -ca * sb, t[1], 0.0, sb, cb, t[2]]

    def chain(n):   # a left-deep chain: tree depth n
        node = scenes.random_leaf(rng)
        for k in range(n - 1):
            op = ("Union", "Difference", "Intersection")[k % 3]
            leaf = scenes.random_leaf(rng)
            if op == "Intersection":
                leaf = {"type": "iellipsoid", "matrix": scenes.st(2.0, 0.0, 0.0, 0.0)}
            node = {"type": op, "matrix": rot(0.1 * k, 0.05 * k, (0, 0, 0)) if k % 4 == 1 else list(scenes.EYE),
                    "children": [node, leaf]}
        return node

    objs = [scenes.random_tree(11, 5), chain(9), chain(12), chain(14), scenes.random_tree(3, 30),
            {"type": "Union", "matrix": rot(0.7, 0.4, (0.05, -0.03, 0.02)),
             "children": [scenes.random_tree(5, 6), scenes.random_leaf(rng)]},
            scenes.random_leaf(rng)]
    depths = sorted(scenes.tree_stats(o)[2] for o in objs)
    # stack depth = tree depth + 1: every class present (<= 9, 10..12, 13..16 slots)
    assert depths[0] <= 8 and any(9 <= d <= 11 for d in depths) and depths[-1] >= 12, depths
    return objs


def test_batch_depth_classes_against_oracle(impli, oracle):
    """The merged batch over objects of all three interpreter depth classes, with rotated node
    matrices: each object's mesh is the oracle's, byte for byte, on two replays (the side-stream
    fork and join of the deeper classes replayed)."""
    from implisolid_amd import scenes
    objs = _depth_class_objects()
    mc = scenes.mc_settings(40, 1.0)
    with impli.Batch(objs, mc, n_streams=0) as b:
        assert b.n == len(objs) and b.merged
        for rep in range(2):
            b.run()
            for i, sh in enumerate(objs):
                v, f = b.download(i)
                vr, fr = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(sh)), 40, [-1, 1] * 3)
                assert len(fr) > 0, i
                assert np.array_equal(f, fr), (rep, i)
                assert np.array_equal(v.view(np.uint32), vr.view(np.uint32)), (rep, i)


_EXIT_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
import torch
torch.cuda.is_available()
import implisolid_amd as I
from implisolid_amd import scenes
v, f = I.make_geometry(*scenes.config3(24))
print(len(v), len(f), flush=True)
"""


def test_exit_with_compiles_in_flight(tmp_path):
    """A process that exits right after its first build -- its tree modules still compiling on the
    JIT's worker threads (an empty disk cache) -- exits cleanly: the exit handler joins the workers
    and they load nothing into the runtime being torn down (it crashed or hung before)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, IMPLISOLID_JIT_CACHE=str(tmp_path / "jit"))
    r = subprocess.run([sys.executable, "-c", _EXIT_SCRIPT, root], env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.split() == ["698", "1384"], r.stdout   # config 3 at 24^3 (the oracle's mesh size)


_INTERP_SCRIPT = r"""
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import implisolid_amd as I
from implisolid_amd import scenes
objs = scenes.config5_objects(8, 48)
shapes, mc = [o[0] for o in objs], objs[0][1]
I.set_jit(0)
out = []
with I.Batch(shapes, mc, n_streams=0) as b:
    b.run()
    for i in range(len(shapes)):
        v, f = b.download(i)
        out.append(hashlib.sha256(v.tobytes() + f.tobytes()).hexdigest())
v, f = I.make_geometry(scenes.config3_tree(), scenes.mc_settings(48, 1.0))
out.append(hashlib.sha256(v.tobytes() + f.tobytes()).hexdigest())
print(" ".join(out))
"""


def test_interpreter_switches_identical():
    """The interpreter's diagnostic switch (IMPLISOLID_INTERP_PAIR=0: one layer per pass, read once
    per process) gives the meshes of the default layer pair: merged object stream and a single
    object on the interpreter kernels (set_jit(0)), each in a fresh process."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for pair in ("1", "0"):
        env = dict(os.environ, IMPLISOLID_INTERP_PAIR=pair)
        r = subprocess.run([sys.executable, "-c", _INTERP_SCRIPT, root], env=env, capture_output=True,
                           text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        res[pair] = r.stdout.split()
    assert len(res["1"]) == 9 and res["1"] == res["0"]


# ---- the bench's own workloads at their full sizes (tests/golden/make_headline.py) -----------------
_HEADLINE = None


def _headline():
    global _HEADLINE
    if _HEADLINE is None:
        _HEADLINE = (json.load(open(_golden("headline_summaries.json"))), np.load(_golden("headline_samples.npz")))
    return _HEADLINE


@pytest.mark.parametrize("name", ["config4_mc_r512", "config4_mc_r256", "config3_ob02_r256", "config3s_ob02_r256",
                                  "config2_ob02_r128", "config4_ob02_r512", "config4s_ob02_r512"])
def test_headline_against_oracle_summary(impli, name):
    """The exact meshes bench.py times (config 4's tree at 512^3 and 256^3, eval + MC) and the OB02
    legs it reports (config 3 at 256^3, config 2 at 128^3, 3 repeats of resample + project + QEM),
    against the oracle's summaries: faces and vertices byte-identical (SHA-256; twist trees included:
    the screw gradient's double cos is glibc's, restated), the twist tree's OB02 meshes also row by
    row against the oracle's full arrays (headline_ob02_verts.npz); a mesh with the reference's
    non-finite rows (config 3): those rows at the same positions, every finite row bit
    for bit (a NaN's payload bits are the producer's, so no SHA over them)."""
    import hashlib
    summ, samples = _headline()
    s = summ[name]
    v, f = impli.make_geometry(s["shape"], s["mc"])
    assert (len(v), len(f)) == (s["n_verts"], s["n_faces"])
    assert hashlib.sha256(np.ascontiguousarray(f).tobytes()).hexdigest() == s["sha256_faces"]
    fin = np.isfinite(v).all(1)
    assert np.flatnonzero(~fin).tolist() == s["nonfinite_rows"]
    idx, vs = samples[name + "_idx"], samples[name + "_v"]
    if not s["nonfinite_rows"]:   # (NaN payload bits are the producer's: compared by position below)
        assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == s["sha256_verts"]
    ok = np.isfinite(vs).all(1)
    assert np.abs(v[idx][ok].astype(np.float64) - vs[ok]).max(initial=0.0) < 1e-5
    full = np.load(_golden("headline_ob02_verts.npz"))
    if name in full.files:   # the twist tree's OB02 meshes: every row, not only the samples
        vr = full[name]
        assert np.array_equal(np.isfinite(vr).all(1), fin)
        bad = np.flatnonzero((v[fin].view(np.uint32) != vr[fin].view(np.uint32)).any(1))
        assert bad.size == 0, (bad.size, bad[:10])   # every finite row bit for bit
    tot = v[fin].astype(np.float64).sum(0)
    assert np.abs(tot - np.array(s["finite_sum"])).max() < 1e-5 * max(1, fin.sum())


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["config3s_ob02_r256", "config4s_ob02_r512"])
def test_config3_shifted_projection_live(impli, name):
    """Config 3 at 256^3 and config 4 at 512^3 on the shifted box (scenes.config3_shifted): the
    average edge length stays finite, so the projection runs its alpha search and bisection on the
    faces (many evaluations per face and repeat, not config 3's one), and the mesh is still the
    oracle's (faces and vertices SHA-256, every vertex finite)."""
    summ, samples = _headline()
    s = summ[name]
    impli.ob02_profile(True)
    try:
        v, f = impli.make_geometry(s["shape"], s["mc"])
        st = impli.last_build_stats()
    finally:
        impli.ob02_profile(False)
    assert _sha(f) == s["sha256_faces"] and np.isfinite(v).all() and s["nonfinite_rows"] == []
    assert _sha(v) == s["sha256_verts"]
    idx, vs = samples[name + "_idx"], samples[name + "_v"]
    assert np.array_equal(v[idx].astype(np.float64), vs)
    evals_per_face = st["projection_evals"] / (len(f) * s["mc"]["overall_repeats"])
    # config 3's dyadic box: one evaluation per face (every centroid kept); live: 20 at 256^3, 9 at
    # 512^3 (the finer mesh's centroids sit closer to the surface: earlier hits, shorter bisections)
    assert evals_per_face > 5, evals_per_face


@pytest.mark.parametrize("n_streams", [0, 8])
def test_config5_stream_against_oracle_summary(impli, n_streams):
    """Config 5 at its stated size: the 64 seeded objects at 128^3 (scenes.config5_objects(64, 128)),
    eval + MC as one merged launch per stage (n_streams 0, the bench headline) and as per-object
    hipGraphs over 8 streams: every object's faces and vertices byte-identical to the oracle's
    (tests/golden/make_headline.py), on two replays."""
    from implisolid_amd import scenes
    summ, _ = _headline()
    rows = summ["config5_mc_r128"]["objects"]
    objs = scenes.config5_objects(64, 128)
    shapes, mc = [o[0] for o in objs], objs[0][1]
    with impli.Batch(shapes, mc, n_streams=n_streams) as b:
        assert b.n == 64 and b.merged == (n_streams == 0)
        for rep in range(2):
            b.run()
            for i, row in enumerate(rows):
                v, f = b.download(i)
                assert (len(v), len(f)) == (row["n_verts"], row["n_faces"]), (rep, i)
                assert _sha(f) == row["sha256_faces"] and _sha(v) == row["sha256_verts"], (rep, i)


@pytest.mark.parametrize("R,nslabs,balanced", [(512, 8, True), (512, 8, False), (645, 2, True), (813, 4, True),
                                                (1024, 8, True)])
def test_config4_slabs_against_summary(impli, R, nslabs, balanced):
    """bench.py's N-GPU partitions on one GPU: config 4's grid as N Z-slabs (balanced cuts from the
    interval pass, or equal layers), each with its recomputed halo layer and global offsets; the
    concatenated mesh is the oracle's config4_mc_r<R> byte for byte.  645^3 / 813^3 / 1024^3 over
    2 / 4 / 8 slabs are the weak-scaling headline runs (R_N = round(512 N^(1/3))); 512^3 over 8 slabs
    is the strong-scaling line reported beside them (BASELINE config 4)."""
    from implisolid_amd import scenes
    summ, _ = _headline()
    s = summ["config4_mc_r%d" % R]
    shape, mc = scenes.config4(R)
    assert shape == s["shape"]
    cuts = impli.slab_balance(shape, mc, nslabs) if balanced else None
    slabs = [impli.Slab(shape, mc, r, nslabs, cuts=cuts) for r in range(nslabs)]
    try:
        counts = []
        for sl in slabs:
            sl.eval()
            sl.count()
            counts.append(sl.counts()[:2])
        voff = np.concatenate([[0], np.cumsum([c[0] for c in counts])])
        foff = np.concatenate([[0], np.cumsum([c[1] for c in counts])])
        vs, fs = [], []
        for r, sl in enumerate(slabs):
            if cuts is not None:
                assert (sl.cz_emit, sl.cz1) == (cuts[r], cuts[r + 1])
            sl.set_offsets(int(voff[r]), int(foff[r]))
            sl.emit()
            nv, nf, of = sl.counts()
            assert not of and (nf > 0 or cuts is None)   # equal slabs: the bottom ones may hold no surface
            v, f = sl.download(nv, nf)
            vs.append(v)
            fs.append(f)
    finally:
        for sl in slabs:
            sl.close()
    v, f = np.concatenate(vs), np.concatenate(fs)
    assert (len(v), len(f)) == (s["n_verts"], s["n_faces"])
    assert _sha(f) == s["sha256_faces"] and _sha(v) == s["sha256_verts"]


def test_rebuild_sequence_consistent(impli):
    """Repeated builds of one object at growing and shrinking resolutions through the C ABI (one
    engine, its buffers reset between grids on the null stream while its kernels run on a
    non-blocking stream): every build of a resolution gives the same mesh.  Regression: a 256^3
    build right after a 512^3 one once raced its buffer resets and came back empty."""
    import hashlib
    from implisolid_amd import scenes
    shape = scenes.config3_tree()
    seen = {}
    for R in [64, 64, 64, 64, 64, 384, 192, 128, 192, 384, 192]:
        v, f = impli.make_geometry(shape, scenes.mc_settings(R, 1.0))
        key = (len(v), len(f), hashlib.sha256(np.ascontiguousarray(f).tobytes()).hexdigest())
        assert len(f) > 0, R
        assert seen.setdefault(R, key) == key, R
        impli.jit_wait()


# ---- multi-GPU: balanced slabs, multi-device build_geometry, multi-process ranks -------------------
def test_balanced_slabs_identical(impli, oracle):
    """Balanced Z-slab cuts (one interval pass of the whole grid) split config 3's tree at R 96 into
    4 unequal slabs whose concatenated meshes are the oracle's, byte for byte; the estimated work
    is better balanced than with equal layers."""
    from implisolid_amd import scenes
    shape, mc = scenes.config3_tree(), scenes.mc_settings(96, 1.0)
    cuts = impli.slab_balance(shape, mc, 4)
    assert cuts[0] == 1 and cuts[-1] == 96 + 3 and all(b > a for a, b in zip(cuts, cuts[1:]))
    assert cuts == impli.slab_balance(shape, mc, 4)          # deterministic: every rank agrees
    ref_v, ref_f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    slabs = [impli.Slab(shape, mc, r, 4, cuts=cuts) for r in range(4)]
    counts = []
    for s in slabs:
        s.eval()
        s.count()
        counts.append(s.counts()[:2])
    voff = np.concatenate([[0], np.cumsum([c[0] for c in counts])])
    foff = np.concatenate([[0], np.cumsum([c[1] for c in counts])])
    vs, fs = [], []
    for r, s in enumerate(slabs):
        assert (s.cz_emit, s.cz1) == (cuts[r], cuts[r + 1])
        s.set_offsets(int(voff[r]), int(foff[r]))
        s.emit()
        nv, nf, of = s.counts()
        assert not of
        v, f = s.download(nv, nf)
        vs.append(v)
        fs.append(f)
        s.close()
    assert np.array_equal(np.concatenate(fs), ref_f)
    assert np.array_equal(np.concatenate(vs).view(np.uint32), ref_v.view(np.uint32))


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0, 0]])
def test_multi_device_build_geometry(impli, oracle, devices):
    """build_geometry with implisolid_set_devices: marching cubes over balanced Z-slabs on several
    devices (here the box's one GPU repeated), concatenated on the host == the oracle; the OB02
    steps then run on the first device on the gathered mesh == the single-device result."""
    from implisolid_amd import scenes
    shape, mc = scenes.config3(56)
    mc_only = scenes.mc_settings(56, 1.0)
    v1, f1 = impli.make_geometry(shape, mc)
    try:
        impli.set_devices(devices)
        v, f = impli.make_geometry(shape, mc_only)
        vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc_only))
        assert np.array_equal(f, fr) and np.array_equal(v.view(np.uint32), vr.view(np.uint32))
        v2, f2 = impli.make_geometry(shape, mc)
        assert np.array_equal(f2, f1)
        assert np.array_equal(v2.view(np.uint32), v1.view(np.uint32))
    finally:
        impli.set_devices(None)


@pytest.mark.parametrize("world,balanced", [(2, True), (3, False)])
def test_multiprocess_ob02_sharded_gloo(impli, oracle, tmp_path, world, balanced):
    """OB02 on Z-slabs: `world` fresh processes build config 2 at R = 64 (sphere u rabbit, MC + 3 x
    [resample, project, QEM]) -- their slabs' MC meshes all-gathered to every rank, then the OB02 loop
    sharded by owned vertex ranges (each rank resamples and QEMs its slab's vertices over the faces
    touching them; the edge-length fold on every rank; owned vertices all-gathered after every step
    that moves them) -- and rank 0's refined mesh is the single-GPU oracle's byte for byte."""
    import os
    import socket
    import subprocess
    import sys
    from implisolid_amd import scenes
    R = 64
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = str(tmp_path / "mesh.npz")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, IMPLISOLID_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "tests", "dist_worker.py"),
           out, str(R), "ob02"] + (["balanced"] if balanced else [])
    r = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    g = np.load(out)
    shape, mc = scenes.config2(R)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    assert np.array_equal(g["faces"], fr)
    assert np.array_equal(g["verts"].view(np.uint32), vr.view(np.uint32))


@pytest.mark.parametrize("mode", ["slabs", "ob02"])
def test_rccl_world1_pipeline(impli, oracle, tmp_path, mode):
    """The multi-GPU step over RCCL itself (backend "nccl"), on the one GPU a test box has: world 1
    under torch.distributed.run -- the counts' all_gather_into_tensor on the launch stream straight
    from the engine's counters (distributed.counts_tensor / gather_counts_inline),
    the mesh gather to rank 0, and for OB02 the slab meshes' and the owned vertices' padded
    all-gathers -- gives the oracle's mesh byte for byte.  (Point-to-point sends need a second GPU.)"""
    import os
    import socket
    import subprocess
    import sys
    from implisolid_amd import scenes
    R = 64 if mode == "ob02" else 72
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = str(tmp_path / "mesh.npz")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, IMPLISOLID_DIST_BACKEND="nccl", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "tests", "dist_worker.py"),
           out, str(R)] + (["ob02"] if mode == "ob02" else [])
    r = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    g = np.load(out)
    shape, mc = scenes.config2(R) if mode == "ob02" else (scenes.config3_tree(), scenes.mc_settings(R, 1.0))
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    assert np.array_equal(g["faces"], fr)
    assert np.array_equal(g["verts"].view(np.uint32), vr.view(np.uint32))


def test_ob02_shard_owning_nothing(impli):
    """A shard whose owned range is empty (load_shard with v0 == v1): no work faces, no centroid
    faces, its halo the empty owned range, and its steps leave every vertex as loaded."""
    import torch
    from implisolid_amd import scenes
    shape, mc = scenes.config2(48)
    v_mc, f_mc = impli.make_geometry(shape, scenes.mc_settings(48, 1.0))
    nv, nf = len(v_mc), len(f_mc)
    V = torch.from_numpy(v_mc.reshape(-1).copy()).cuda()
    F = torch.from_numpy(f_mc.reshape(-1).copy()).cuda()
    for at in (0, nv // 2, nv):
        ob = impli.Ob02Shard(shape, mc)
        try:
            ob.load(V.data_ptr(), nv, F.data_ptr(), nf, at, at)
            assert ob.ranges() == (at, at, 0, 0, 0, 0)
            assert ob.halo() == (at, at)
            ob.resample()
            ob.project()
            out = torch.empty_like(V)
            ob.get_verts(out.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), v_mc.reshape(-1).view(np.uint32))
        finally:
            ob.close()


def test_ob02_shards_in_one_process(impli, oracle):
    """The sharded OB02 loop without processes: config 2 at R = 48 as 3 and 5 vertex-range shards on
    one GPU, stepped together with the owned ranges exchanged on the host after every vertex-moving
    step -- the same mesh as build_geometry and the oracle, byte for byte; the shards' work-face
    ranges cover their vertices' umbrellas and stay within the slabs plus one layer."""
    import torch
    from implisolid_amd import scenes
    shape, mc = scenes.config2(48)
    st = impli.parse_settings(mc)
    v_mc, f_mc = impli.make_geometry(shape, scenes.mc_settings(48, 1.0))
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    for nshard in (3, 5):
        nv, nf = len(v_mc), len(f_mc)
        voff = np.linspace(0, nv, nshard + 1).astype(np.int64)
        V = torch.from_numpy(v_mc.reshape(-1).copy()).cuda()
        F = torch.from_numpy(f_mc.reshape(-1).copy()).cuda()
        obs = [impli.Ob02Shard(shape, mc) for _ in range(nshard)]
        # the ranges the device finds, against the host's: work faces = the faces touching an owned
        # vertex; centroid faces = those and their edge neighbours; halo = those faces' vertices
        edge_faces = {}
        for j, (a, b, c) in enumerate(f_mc.tolist()):
            for e in ((a, b), (b, c), (c, a)):
                edge_faces.setdefault((min(e), max(e)), []).append(j)
        for r, ob in enumerate(obs):
            ob.load(V.data_ptr(), nv, F.data_ptr(), nf, int(voff[r]), int(voff[r + 1]))
            v0, v1, w0, w1, c0, c1 = ob.ranges()
            assert (v0, v1) == (voff[r], voff[r + 1])
            touch = np.flatnonzero(((f_mc >= v0) & (f_mc < v1)).any(1))
            assert (w0, w1) == (int(touch[0]), int(touch[-1]) + 1)
            near, near2 = set(range(w0, w1)), set(range(w0, w1))   # every face on a shared edge / manifold edges only
            for j in range(w0, w1):
                a, b, c = f_mc[j].tolist()
                for e in ((a, b), (b, c), (c, a)):
                    fs = edge_faces[(min(e), max(e))]
                    near.update(fs)
                    if len(fs) == 2:
                        near2.update(fs)
            assert min(near) <= c0 <= min(near2) and max(near2) + 1 <= c1 <= max(near) + 1
            h0, h1 = ob.halo()
            assert (h0, h1) == (min(v0, int(f_mc[c0:c1].min())), max(v1, int(f_mc[c0:c1].max()) + 1))
        bufs = [torch.empty(nv * 3, dtype=torch.float32, device="cuda") for _ in obs]

        def exchange():
            full = torch.empty(nv * 3, dtype=torch.float32, device="cuda")
            for r, ob in enumerate(obs):
                ob.get_verts(bufs[r].data_ptr())
                full[3 * voff[r]:3 * voff[r + 1]] = bufs[r][3 * voff[r]:3 * voff[r + 1]]
            torch.cuda.synchronize()
            for ob in obs:
                ob.set_verts(full.data_ptr())

        for rep in range(st["overall_repeats"]):
            for _ in range(st["vresampl_iters"]):
                for ob in obs:
                    ob.resample()
                exchange()
            for ob in obs:
                ob.project()
            exchange()
        v, f = obs[0].download()
        for ob in obs:
            ob.close()
        assert np.array_equal(f, fr)
        assert np.array_equal(v.view(np.uint32), vr.view(np.uint32)), nshard


@pytest.mark.parametrize("nshard,halo,scene", [(3, True, "config2_48"), (5, True, "config2_48"), (8, True, "config2_48"),
                                               (5, False, "config2_48"), (8, True, "config3s_64"), (4, True, "subdiv_40")])
def test_ob02_stream_ordered_shards(impli, oracle, nshard, halo, scene):
    """The stream-ordered sharded loop (distributed.ob02_shards_local: every shard attached to its own
    copy of the mesh, stepped on its own stream without host synchronisation, the exchanges of
    ob02_plan -- the one-ring halo before a resampling, every owned range before a projection and
    at the end -- as device copies) is build_geometry's mesh and the oracle's, byte for byte, at 3 to
    8 shards, with and without the halo-only exchanges, with subdivision after the loop."""
    import torch
    from implisolid_amd import distributed as D
    from implisolid_amd import scenes
    if scene == "config2_48":
        shape, mc = scenes.config2(48)
    elif scene == "config3s_64":
        shape, mc = scenes.config3_shifted(64)
    else:
        shape, mc = scenes.config2(40)
        mc = dict(mc, subdiv={"enabled": 1})
    v_mc, f_mc = impli.make_geometry(shape, dict(mc, vresampl={"iters": 0, "c": 1.0}, projection={"enabled": 0},
                                                 qem={"enabled": 0}, subdiv={"enabled": 0}))
    impli.srand(4711)   # subdivision noise: glibc rand() from the same state on both sides
    oracle.srand(4711)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    nv = len(v_mc)
    voff = np.linspace(0, nv, nshard + 1).astype(np.int64)
    V = torch.from_numpy(v_mc.reshape(-1).copy()).cuda()
    F = torch.from_numpy(f_mc.reshape(-1).copy()).cuda()
    plan = D.ob02_plan(impli.parse_settings(mc))
    assert plan and plan[-1][1] in ("full", None)
    v, f, stats = D.ob02_shards_local(shape, mc, V, F, voff, halo=halo)
    assert np.array_equal(f, fr)
    fin = np.isfinite(vr).all(1)
    assert np.array_equal(np.isfinite(v).all(1), fin)
    assert np.array_equal(v[fin].view(np.uint32), vr[fin].view(np.uint32)), (nshard, halo, scene)
    if halo and any(ex == "halo" for _, ex in plan):
        full = 12 * nv * (nshard - 1) / nshard * nshard   # bytes a full exchange moves
        assert min(stats["exchange_bytes"]) < full / 4    # the halo exchanges move a fraction


@pytest.mark.parametrize("world,balanced", [(2, True), (3, False)])
def test_multiprocess_slabs_gloo(impli, oracle, tmp_path, world, balanced):
    """`world` fresh processes (torch.distributed.run, all on this box's GPU, gloo backend) run the
    bench's multi-GPU step -- balanced or equal Z-slabs, eval, count, the vertex pass, the count
    all-gather, the face pass with the gathered counts -- and gather the mesh to rank 0
    (distributed.gather_mesh): byte-identical to the oracle."""
    import os
    import socket
    import subprocess
    import sys
    from implisolid_amd import scenes
    R = 72
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    out = str(tmp_path / "mesh.npz")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, IMPLISOLID_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "tests", "dist_worker.py"),
           out, str(R)] + (["balanced"] if balanced else [])
    r = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    g = np.load(out)
    shape, mc = scenes.config3_tree(), scenes.mc_settings(R, 1.0)
    vr, fr = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    assert np.array_equal(g["faces"], fr)
    assert np.array_equal(g["verts"].view(np.uint32), vr.view(np.uint32))
    if balanced:
        assert len(g["cuts"]) == world + 1


def test_geometry_views_generation(impli):
    """make_geometry_views' arrays are read-only views into the library's result buffers, valid until
    the next build: copy_geometry_views copies current ones and refuses stale ones."""
    from implisolid_amd import scenes
    v, f = impli.make_geometry_views(*scenes.config1())
    assert not v.flags.writeable and impli.views_current(v) and impli.views_current(f[1:])
    vc, fc = impli.copy_geometry_views(v, f)
    v2, f2 = impli.make_geometry(*scenes.config1())
    assert np.array_equal(vc, v2) and np.array_equal(fc, f2)
    impli.make_geometry_views(*scenes.config2(48))
    assert not impli.views_current(v)
    with pytest.raises(impli.ImplisolidError):
        impli.copy_geometry_views(v, f)


def test_shard_handles_bounded(impli):
    """distributed.shard_handle keeps one handle per (device, slot): the same object reuses it, another
    object closes it (its buffers and streams freed), release_shards() closes the rest."""
    from implisolid_amd import distributed as D, scenes
    D.release_shards()
    a = D.shard_handle(scenes.config1()[0], scenes.config1()[1], slot=0)
    assert D.shard_handle(scenes.config1()[0], scenes.config1()[1], slot=0) is a
    b = D.shard_handle(scenes.config3_tree(), scenes.config1()[1], slot=0)
    assert b is not a and a.h is None and b.h
    c = D.shard_handle(scenes.config3_tree(), scenes.config1()[1], slot=1)
    assert len(D._SHARDS) == 2
    D.drop_shard(c)
    assert c.h is None and len(D._SHARDS) == 1
    D.release_shards()
    assert b.h is None and not D._SHARDS


def test_config4_ob02_r512_sharded_against_summary(impli):
    """Config 4's OB02 loop at its own size: the tree at 512^3 on the shifted box (live alpha search
    and bisection), the MC mesh's vertices owned by the 8 balanced Z-slabs' ranges, every shard
    stepped on its own stream with the halo / full exchanges (distributed.ob02_shards_local, the
    bench's 8-rank estimate), against the oracle's summary (tests/golden/make_headline.py
    config4s_ob02_r512): faces and vertices byte-identical (SHA-256)."""
    import torch
    from implisolid_amd import distributed as D
    summ, _ = _headline()
    s = summ["config4s_ob02_r512"]
    shape, mc = s["shape"], s["mc"]
    cuts = D.balanced_cuts(shape, mc, 8)
    nvs = []
    for r in range(8):
        sl = impli.Slab(shape, mc, r, 8, cuts=cuts)
        nvs.append(sl.run()[0])
        sl.close()
    mc_only = dict(mc, vresampl={"iters": 0, "c": 1.0}, projection={"enabled": 0}, qem={"enabled": 0},
                   subdiv={"enabled": 0})
    v_mc, f_mc = impli.make_geometry(shape, mc_only)
    assert sum(nvs) == len(v_mc)
    V = torch.from_numpy(v_mc.reshape(-1).copy()).cuda()
    F = torch.from_numpy(f_mc.reshape(-1).copy()).cuda()
    voff = np.concatenate([[0], np.cumsum(nvs)]).astype(np.int64)
    v, f, _ = D.ob02_shards_local(shape, mc, V, F, voff)
    assert _sha(f) == s["sha256_faces"] and np.isfinite(v).all()
    assert _sha(v) == s["sha256_verts"]
