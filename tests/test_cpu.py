"""CPU suite (no GPU): the oracle against the golden vectors and the independent numpy
restatement, the host logic of the C ABI, the library's exported symbols, and the multi-rank
numbering exchange over gloo (world size 2 and 3)."""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, mesh_edges

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import np_restate  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def _u32(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


# ---- tables and libm-level pins -------------------------------------------------------------------
@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference tree not mounted")
def test_tables_extracted_from_reference():
    """generated/tables.h == the reference's MC tables (marching_cubes.hpp:1207-1502) and rabbit
    table (cube.hpp:68-72)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "extract_tables.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_mc_tables_self_consistent():
    # every case's triangle list uses exactly the edges whose endpoints differ in sign
    for c, t in enumerate(np_restate.TRI):
        assert len(t) % 3 == 0
        used = {int(ch, 16) for ch in t}
        crossing = {e for e, (a, b, _, _) in enumerate(np_restate.EDGES)
                    if bool(c & np_restate.CORNER_BIT[a]) != bool(c & np_restate.CORNER_BIT[b])}
        assert used == crossing, c


def test_acosf_restatement_matches_glibc_strided(oracle):
    # vertex_resampling.hpp:75 std::acos(float): the restated glibc-2.35 acosf, every 61st pattern
    assert oracle.acosf_check(0, 61, (1 << 32) // 61) == 0


@pytest.mark.slow
@pytest.mark.skipif(not os.environ.get("IMPLISOLID_SLOW"), reason="exhaustive (~50 s): set IMPLISOLID_SLOW=1")
def test_acosf_restatement_matches_glibc_exhaustive(oracle):
    assert oracle.acosf_check(0, 1, 1 << 32) == 0


# ---- oracle vs the independent numpy restatement ------------------------------------------------
def _trees():
    from implisolid_amd import scenes
    t = {"sphere": ({"type": "iellipsoid", "matrix": scenes.EYE}, [-0.6, 0.6] * 3, 32),
         "union_sphere_cube": (scenes.union_sphere_cube(), [-1, 1] * 3, 40),
         "config3_tree": (scenes.random_tree(scenes.CONFIG3_SEED, 10), [-1, 1] * 3, 40),   # without twists
         "anisotropic": (scenes.union_sphere_cube(), [-0.7, 0.9, -1.1, 0.6, -0.55, 0.8], 36)}
    for seed in (7, 11, 13, 101, 102):
        t["random_%d" % seed] = (scenes.random_tree(seed, 3 + seed % 10), [-1, 1] * 3, 40)
    return t


TREES = _trees()


@pytest.mark.parametrize("name", sorted(TREES))
def test_oracle_field_and_mc_match_numpy_restatement(oracle, name):
    shape, box, R = TREES[name]
    tree = oracle.mp5_to_nodes(json.dumps(shape))
    F, w = np_restate.field(shape, R, box)
    Fo = oracle.mc_field(tree, R, box)
    assert np.array_equal(_u32(F), _u32(Fo))
    v, f = np_restate.marching_cubes(F, w, box, R)
    vo, fo = oracle.marching_cubes(tree, R, box)
    assert np.array_equal(f, fo)
    assert np.array_equal(_u32(v), _u32(vo))


def test_point_eval_matches_numpy_restatement(oracle):
    rng = np.random.default_rng(3)
    pts = rng.uniform(-1.3, 1.3, size=(20000, 3)).astype(np.float32)
    for name, (shape, _, _) in TREES.items():
        fo = oracle.eval_implicit(oracle.mp5_to_nodes(json.dumps(shape)), pts)
        fn = np_restate.evaluate(shape, pts[:, 0].copy(), pts[:, 1].copy(), pts[:, 2].copy())
        assert np.array_equal(_u32(fo), _u32(fn)), name


# ---- golden fixtures ------------------------------------------------------------------------------
def test_golden_config1(oracle):
    g = np.load(os.path.join(GOLDEN, "config1_mc.npz"))
    v, f = oracle.polygonize(str(g["shape"]), str(g["mc"]))
    assert v.shape == (3318, 3) and f.shape == (6632, 3)
    assert np.array_equal(f, g["faces"]) and np.array_equal(_u32(v), _u32(g["verts"]))


def test_golden_point_values(oracle):
    g = np.load(os.path.join(GOLDEN, "points_eval.npz"))
    trees = json.loads(str(g["trees"]))
    pts = g["points"]
    for name, sh in trees.items():
        tree = oracle.mp5_to_nodes(json.dumps(sh))
        assert np.array_equal(_u32(oracle.eval_implicit(tree, pts)), _u32(g["f_" + name])), name
        assert np.array_equal(_u32(oracle.eval_gradient(tree, pts)), _u32(g["g_" + name])), name


def test_golden_config2_ob02(oracle):
    g = np.load(os.path.join(GOLDEN, "config2_r32_ob02.npz"))
    taps = {}
    v, f = oracle.polygonize(str(g["shape"]), str(g["mc"]), taps=taps)
    assert np.array_equal(f, g["faces"]) and np.array_equal(_u32(v), _u32(g["verts"]))
    assert np.array_equal(_u32(np.asarray(taps["post_p_centroids"])), _u32(g["tap_post_p_centroids"]))


def test_golden_mc_summaries(oracle):
    import hashlib
    d = json.load(open(os.path.join(GOLDEN, "mc_summaries.json")))
    for name, s in d.items():
        v, f = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(s["shape"])), s["R"], s["box"])
        assert (v.shape[0], f.shape[0]) == (s["n_verts"], s["n_faces"]), name
        assert hashlib.sha256(np.ascontiguousarray(f).tobytes()).hexdigest() == s["sha256_faces"], name
        assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == s["sha256_verts"], name
    # SURVEY.md §8a (independent numpy estimate): config 2 scene at R=128 -> V 56 684, F 113 360
    assert (d["config2_mc_r128"]["n_verts"], d["config2_mc_r128"]["n_faces"]) == (56684, 113360)
    assert 56684 - 113360 // 2 == 4          # Euler characteristic: two sphere-like components


def test_golden_subdivision(oracle):
    """Step 3 (my_subdiv_) through polygonize with the oracle's glibc rand() seeded by srand(1)."""
    g = np.load(os.path.join(GOLDEN, "subdiv.npz"))
    for name in ["config1", "config2_r24"]:
        oracle.srand(1)
        v, f = oracle.polygonize(str(g[name + "_shape"]), str(g[name + "_mc"]))
        assert np.array_equal(f, g[name + "_faces"]) and np.array_equal(_u32(v), _u32(g[name + "_verts"])), name
    # config 1: V' = V + E, F' = 4F on a closed mesh (E = 3F/2)
    assert g["config1_verts"].shape == (3318 + 3 * 6632 // 2, 3) and g["config1_faces"].shape == (4 * 6632, 3)


def _ragged_mesh(rng, nv=40, nf=90):
    v = rng.uniform(-1, 1, (nv, 3)).astype(np.float32)
    f = rng.integers(0, nv, (nf, 3)).astype(np.int32)
    f[5] = [3, 3, 7]                     # degenerate face: edge (3, 3)
    f[6] = [7, 3, 3]
    return v, f


@pytest.mark.parametrize("amp", [0.0, 0.1, 3.0])
def test_subdivide_oracle_matches_numpy(oracle, amp):
    """The oracle's 1-to-4 subdivision + randomize_verts == the vectorised numpy restatement, on
    the config-1 mesh and on a ragged mesh (boundary edges, edges in > 2 faces, degenerate faces)."""
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    shape, mc = __import__("implisolid_amd.scenes", fromlist=["x"]).config1()
    v0, f0 = oracle.polygonize(json.dumps(shape), json.dumps(mc))
    for v, f in [(v0, f0), _ragged_mesh(np.random.default_rng(3))]:
        oracle.srand(99)
        V, F = oracle.subdivide(v, f, amp)
        libc.srand(99)
        d = [libc.rand() for _ in range(3 * V.shape[0])]
        V2, F2 = np_restate.subdivide(v, f, amp, d)
        assert np.array_equal(F, F2) and np.array_equal(_u32(V), _u32(V2))
    # empty mesh: no faces, the vertices still get their noise
    oracle.srand(5)
    V, F = oracle.subdivide(v0[:10], np.zeros((0, 3), np.int32), 1.0)
    libc.srand(5)
    V2, _ = np_restate.subdivide(v0[:10], np.zeros((0, 3), np.int32), 1.0, [libc.rand() for _ in range(30)])
    assert F.shape == (0, 3) and np.array_equal(_u32(V), _u32(V2))


def test_library_rand_matches_glibc(impli):
    """The library's process-global rand() (host.hpp GlibcRand) == glibc rand() after the same
    srand, including the O(log n) jump-ahead the GPU noise kernel's lanes use."""
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    for seed in [0, 1, 7, 123456789, 0xDEADBEEF]:
        libc.srand(seed)
        impli.srand(seed)
        assert [libc.rand() for _ in range(2000)] == [impli.rand() for _ in range(2000)], seed
        for n in [1, 30, 31, 62, 248, 15872, 100003]:
            for _ in range(n):
                libc.rand()
            impli.rand_skip(n)
            assert libc.rand() == impli.rand(), (seed, n)


# ---- glibc float math of the screw family (or_libm.c; the device copies are compared on the GPU) ---
def test_libm_restatements_match_glibc_strided(oracle):
    # screw.hpp: std::sin(float) (x86_64 FMA variant of sinf) and std::atan2(float, float)
    assert oracle.libm_check(0, 0, 61, (1 << 32) // 61) == 0      # sinf, every 61st pattern
    assert oracle.libm_check(1, 7, 61, (1 << 32) // 61) == 0      # atanf
    assert oracle.libm_check(2, 1, 1, 2_000_000) == 0             # atan2f, seeded pairs


@pytest.mark.slow
@pytest.mark.skipif(not os.environ.get("IMPLISOLID_SLOW"), reason="exhaustive (~2 min): set IMPLISOLID_SLOW=1")
def test_libm_restatements_match_glibc_exhaustive(oracle):
    assert oracle.libm_check(0, 0, 1, 1 << 32) == 0
    assert oracle.libm_check(1, 0, 1, 1 << 32) == 0
    assert oracle.libm_check(2, 2, 1, 100_000_000) == 0


def test_cos_restatement_matches_glibc(oracle):
    """The screw gradient's double cos (screw.hpp:178-180): glibc 2.35's __cos, x86_64 FMA variant,
    restated from the host libm's __cos_fma (or_libm.c or_cos; its table from libm by
    tools/extract_sincostab.py) -- bit for bit against the host cos on seeded arguments spanning
    every branch (|x| < 2^-27, do_cos, do_sin near pi/2, the reduced range with its TAYLOR_SIN
    path) and the screw's own range (pi x a phase of a few units).  2 G arguments gave 0 mismatches
    (DESIGN.md section 4)."""
    for seed, lim in ((1, 4.0), (2, 64.0), (3, 1e4), (4, 1e8)):
        assert oracle.cos_check(seed, 2_000_000, lim) == 0, (seed, lim)
    x = np.array([0.0, -0.0, 1e-300, 2.0 ** -27, -(2.0 ** -27), 0.85546875, -0.85546875, 2.426265, np.pi / 2,
                  -np.pi, 105414349.0, 1e300, np.inf, -np.inf, np.nan])
    a, b = oracle.cos_apply(x), oracle.cos_apply(x, glibc=True)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)) or np.array_equal(np.isnan(a), np.isnan(b))


def test_sincostab_header_matches_libm():
    """csrc/generated/sincostab.h is glibc's __sincostab as this image's libm holds it."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "extract_sincostab.py")], capture_output=True,
                         text=True, check=True).stdout
    assert open(os.path.join(root, "implisolid_amd", "csrc", "generated", "sincostab.h")).read() == out


def _screw_family():
    from implisolid_amd import scenes
    tw = scenes.twist(1, 0, 0, 0)
    return {"screw": tw, "screw_diff_two_plane": dict(tw, type="screw_diff_two_plane"),
            "inf_screw": dict(tw, type="inf_screw", pitch=0.25),
            "half_plane": {"type": "Intersection", "matrix": scenes.EYE, "children": [
                {"type": "iellipsoid", "matrix": scenes.EYE},
                {"type": "half_plane", "matrix": scenes.st(0.5, 0, 0.125, 0), "plane_vector": [0, 1, 2],
                 "plane_point": [0, 0, 0.25]}]},
            "lid": {"type": "Intersection", "matrix": scenes.EYE, "children": [
                {"type": "icylinder", "matrix": scenes.st(1, 0, 0, 0.5)},
                {"type": "top_bottom_lid", "matrix": scenes.st(1, 0, 0, 0)}]},
            "config3_twist": scenes.config3_tree(),
            "tetrahedron": scenes.tetrahedron(), "meta_balls": scenes.meta_balls(), "extrusion": scenes.extrusion(6),
            "extrusion_tri": scenes.extrusion(3, scale=0.5),
            "screw_gradient_wrong": dict(scenes.twist(1, 0, 0, 0.0625), type="screw_gradient_wrong")}


@pytest.mark.parametrize("name", sorted(_screw_family()))
def test_screw_family_oracle_meshes_closed(oracle, name):
    """The twist (screw), lid and half-plane nodes give closed edge-manifold MC meshes."""
    shape = _screw_family()[name]
    v, f = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(shape)), 48, [-0.7, 0.7] * 3)
    assert len(f) > 1000
    _, cnt = mesh_edges(f)
    assert (cnt == 2).all()


def test_screw_values_follow_the_reference_formula(oracle):
    """Spot values of screw.hpp's field at its constants: f = r0 + delta sin(2 pi (t/pitch) - theta)
    - r, with r0 = 1/3, delta = 1/6 (delta_ratio 1.5), t = z + 1/2; the lid cuts |z| > 1/2."""
    from implisolid_amd import scenes
    tree = oracle.mp5_to_nodes(json.dumps(dict(scenes.twist(1, 0, 0, 0), type="inf_screw")))
    rng = np.random.default_rng(4)
    p = rng.uniform(-0.6, 0.6, (2000, 3)).astype(np.float32)
    f = oracle.eval_implicit(tree, p).astype(np.float64)
    x, y, z = p[:, 0].astype(np.float64), p[:, 1].astype(np.float64), p[:, 2].astype(np.float64)
    ref = 1 / 3 + (1 / 6) * np.sin(2 * np.pi * ((z + 0.5) / 0.5) - np.arctan2(y, x)) - np.hypot(x, y)
    assert np.abs(f - ref).max() < 2e-6


def test_screw_gradient_wrong_semantics(oracle):
    """inf_top_bot_bound over the screw (object_factory.hpp:435-479, inf_top_bot_bound.hpp:65-166):
    the value is min(screw, -lid) at x' = T^-1 x, and the gradient ignores which operand won --
    (0, 0, -/+1) outside |z'| < 0.5, the screw's gradient with T^-T applied twice inside."""
    from implisolid_amd import scenes
    sh = dict(scenes.twist(0.5, 0, 0, 0.125), type="screw_gradient_wrong")
    tree = oracle.mp5_to_nodes(json.dumps(sh))
    inf = oracle.mp5_to_nodes(json.dumps(dict(sh, type="inf_screw")))
    rng = np.random.default_rng(8)
    p = rng.uniform(-0.6, 0.6, (4000, 3)).astype(np.float32)
    zl = (p[:, 2] - np.float32(0.125)) * np.float32(2)               # z' = T^-1 x (scale 1/2, exact)
    lid = np.maximum(zl - np.float32(0.5), -(zl + np.float32(0.5)))
    fs = oracle.eval_implicit(inf, p)
    f = oracle.eval_implicit(tree, p)
    assert np.array_equal(f, np.where(-lid < fs, -lid, fs).astype(np.float32))
    g, gs = oracle.eval_gradient(tree, p), oracle.eval_gradient(inf, p)
    up, dn = zl >= 0.5, zl <= -0.5
    mid = ~(up | dn)
    assert up.any() and dn.any() and mid.any()
    assert np.array_equal(g[up], np.tile([0, 0, -2], (up.sum(), 1)).astype(np.float32))
    assert np.array_equal(g[dn], np.tile([0, 0, 2], (dn.sum(), 1)).astype(np.float32))
    assert np.array_equal(g[mid], gs[mid] * np.float32(2))           # T^-T = 2 I once more


def test_screw_factory_errors(impli):
    from implisolid_amd import scenes
    bad = dict(scenes.twist(1, 0, 0, 0))
    del bad["v"]
    with pytest.raises(impli.ImplisolidError, match="missing"):
        impli.program_info(bad)
    assert impli.program_info(scenes.twist(1, 0, 0, 0))[:3] == (6, 3, 4)   # XFORM Diff + 2 leaves, 1 param row


# ---- mesh properties ------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["sphere", "union_sphere_cube", "config3_tree"])
def test_mc_output_is_closed_edge_manifold(oracle, name):
    shape, box, R = TREES[name]
    v, f = oracle.marching_cubes(oracle.mp5_to_nodes(json.dumps(shape)), R, box)
    _, cnt = mesh_edges(f)
    assert (cnt == 2).all()
    assert (np.bincount(f.ravel(), minlength=len(v)) > 0).all()      # every vertex referenced
    if name == "sphere":
        assert len(v) - len(f) // 2 == 2                              # Euler characteristic


def test_owner_rule_matches_first_appearance_order():
    """The GPU numbering rule: a vertex is created by the cell owning its edge (local edge 5, 6 or
    10), ordered by owner cell z-major.  First-appearance ids must be non-decreasing in owner layer,
    which is what lets Z-slabs number independently and concatenate."""
    for name in ["union_sphere_cube", "config3_tree", "random_7"]:
        shape, box, R = TREES[name]
        F, w = np_restate.field(shape, R, box)
        v, f, codes = np_restate.mc_with_codes(F, w, box, R)
        z = np_restate.owner_cell_z(codes, R)
        assert (np.diff(z) >= 0).all(), name


def test_ob02_properties(oracle):
    """Projected centroids lie on the surface to the bisection tolerance (configs.hpp:33)."""
    from implisolid_amd import scenes
    shape, mc = scenes.config2(32)
    taps = {}
    oracle.polygonize(json.dumps(shape), json.dumps(mc), taps=taps)
    tree = oracle.mp5_to_nodes(json.dumps(shape))
    cen = np.asarray(taps["post_p_centroids"][-1])
    fv = np.abs(oracle.eval_implicit(tree, cen))
    assert np.median(fv) <= 1e-4 and (fv <= 1e-4).mean() > 0.95


# ---- host logic of the C ABI (no GPU calls) -------------------------------------------------------
def _header_functions():
    txt = open(os.path.join(ROOT, "include", "implisolid.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"typedef[^;]*;", "", txt)   # function-pointer typedefs declare no symbol
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\([^;{]*\)\s*;", txt, flags=re.M)
    return sorted(set(names))


def test_abi_exports_every_declared_symbol(impli):
    names = _header_functions()
    assert len(names) >= 40, names
    L = impli.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) <= set(impli.ABI_SYMBOLS) | {"main"}, set(names) - set(impli.ABI_SYMBOLS)


def test_host_matrix_inverse_matches_oracle(impli, oracle):
    """compile_mp5's inverse (host C++) == the oracle's LU restatement, bit for bit, including
    general (rotation + shear) matrices where the LU operation order matters."""
    rng = np.random.default_rng(11)
    for trial in range(40):
        m = rng.uniform(-1, 1, 12).astype(np.float32)
        m[[0, 5, 10]] += np.float32(2.0)
        shape = {"type": "iellipsoid", "matrix": [float(x) for x in m]}
        n_instr, depth, n_mats, mats = impli.program_info(shape)
        tree = oracle.mp5_to_nodes(json.dumps(shape))
        ref = np.array(tree[0][tree[1]].minv[:], np.float32)
        assert np.array_equal(_u32(mats[0]), _u32(ref)), trial


def test_program_compiles_reference_factory_semantics(impli):
    from implisolid_amd import scenes
    # n-ary union -> left-deep chain: 3 children = 2 union nodes
    u3 = {"type": "Union", "matrix": scenes.EYE, "children": [
        {"type": "iellipsoid", "matrix": scenes.EYE}, {"type": "icone", "matrix": scenes.EYE},
        {"type": "itorus", "matrix": scenes.EYE}]}
    n_instr, depth, n_mats, _ = impli.program_info(u3)
    assert n_instr == 3 * 2 + 2 * 2     # 3 leaves (XFORM + PRIM) + 2 unions (XFORM + CSG)
    for bad, msg in [({"type": "bogus", "matrix": scenes.EYE}, "Invalid"),
                     ({"type": "screw", "matrix": scenes.EYE}, "missing"),
                     ({"type": "sdf_3d", "matrix": scenes.EYE}, "outside the implemented"),
                     ({"type": "iellipsoid"}, "matrix")]:
        with pytest.raises(Exception) as e:
            impli.program_info(bad)
        assert msg.lower() in str(e.value).lower(), str(e.value)


def test_settings_parser_matches_oracle(impli, oracle):
    from implisolid_amd import scenes
    cases = [scenes.config1()[1], scenes.config2(64)[1],
             dict(scenes.mc_settings(40, 1.0), resolution="40", ignore_root_matrix="true"),
             dict(scenes.mc_settings(40, 1.0), overall_repeats=0)]
    for mc in cases:
        a = impli.parse_settings(mc)
        b = oracle.parse_mc_settings(json.dumps(mc))
        assert [np.float32(x) for x in a["box"]] == [np.float32(x) for x in b.box]
        assert (a["resolution"], a["overall_repeats"], a["vresampl_iters"]) == (b.resolution, b.overall_repeats, b.vresampl_iters)
        assert (bool(a["projection"]), bool(a["qem"]), bool(a["subdiv"]), bool(a["ignore_root_matrix"])) == \
               (b.projection, b.qem, b.subdiv, b.ignore_root_matrix)
        assert a["vresampl_c"] == b.vresampl_c
    for bad in [dict(scenes.mc_settings(40, 1.0), resolution=40.5), dict(scenes.mc_settings(40, 1.0), resolution=2),
                {"resolution": 40}, dict(scenes.mc_settings(40, 1.0), qem={"enabled": 1})]:
        with pytest.raises(Exception):
            impli.parse_settings(bad)
        with pytest.raises(ValueError):
            oracle.parse_mc_settings(json.dumps(bad))


def test_invalid_settings_abort_in_reference_mode(impli):
    """Error mode 0 (the default for C callers) aborts like polygoniser_settings.hpp:297-301."""
    code = ("import ctypes, implisolid_amd as I; L = I.lib(); L.implisolid_set_error_mode(0); "
            "import numpy as np; b=(ctypes.c_float*6)(); i=(ctypes.c_int32*7)(); f=(ctypes.c_float*2)(); "
            "L.implisolid_parse_settings(b'{\"resolution\": 40}', b, i, f)")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode != 0 and "Abort" in r.stderr


def test_slab_partition_covers_all_layers(impli):
    for R in (16, 61, 512):
        for n in (1, 2, 3, 8):
            parts = [impli.slab_partition(R, r, n) for r in range(n)]
            layers = [z for (z0, z1, _) in parts for z in range(z0, z1)]
            assert layers == list(range(1, R + 3))                  # cells 1 .. res-3
            assert [h for (_, _, h) in parts] == [0] + [1] * (n - 1)


def test_slab_32bit_cell_limit(impli):
    """A slab's cell ids, vertex ids and face rows are 32-bit: one slab may hold < 2^32 cells
    (halo layer included).  R = 1623 fits one GPU (1625^3 cells); R = 1624 and R = 2000 must be
    split, and 2 slabs of R = 2000 (2002^2 x 1002 cells each) fit."""
    assert impli.slab_partition(1623, 0, 1) == (1, 1626, 0)
    for R in (1624, 2000):
        with pytest.raises(impli.ImplisolidError, match="2\\^32"):
            impli.slab_partition(R, 0, 1)
    assert impli.slab_partition(2000, 1, 2)[2] == 1
    with pytest.raises(impli.ImplisolidError):
        impli.slab_partition(2000, 0, 3000)   # more slabs than layers


def _layer_work(listed, bpl, cuts):
    w = np.asarray(listed, np.float64) / 2 + 0.02 * bpl / 2   # cell layer c costs sample layer c - 1
    return [w[cuts[r] - 1:cuts[r + 1] - 1].sum() for r in range(len(cuts) - 1)]


def test_balanced_cuts_from_layer_work(impli):
    """Balanced Z-slab cuts (engine.hip cuts_from_layer_work): they cover the cell layers
    1 .. R + 2 in order with at least one layer per slab, split a uniform load into equal slabs,
    and keep a surface concentrated in the middle layers within 1.3x max / min."""
    R, bpl = 512, 65 * 65
    L = R + 2
    for n in (1, 2, 3, 8):
        cuts = impli.cuts_from_layer_work(np.full(R + 3, 100), bpl, R, n)
        assert cuts[0] == 1 and cuts[-1] == R + 3 and all(b > a for a, b in zip(cuts, cuts[1:]))
        sizes = np.diff(cuts)
        assert sizes.max() - sizes.min() <= 1
    z = np.arange(R + 3)
    listed = (3000 * np.exp(-((z - 0.55 * R) / (0.18 * R)) ** 2)).astype(np.int64)   # surface mid-grid
    for n in (2, 4, 8):
        cuts = impli.cuts_from_layer_work(listed, bpl, R, n)
        w = _layer_work(listed, bpl, cuts)
        assert max(w) / min(w) < 1.3, (n, cuts, w)
        eq = [impli.slab_partition(R, r, n)[0] for r in range(n)] + [L + 1]
        weq = _layer_work(listed, bpl, eq)
        assert max(w) < max(weq)                                  # better than equal layers
    # degenerate inputs: all work in one layer; as many slabs as layers
    one = np.zeros(R + 3, np.int64)
    one[100] = 10 ** 6
    cuts = impli.cuts_from_layer_work(one, bpl, R, 8)
    assert all(b > a for a, b in zip(cuts, cuts[1:])) and cuts[-1] == R + 3
    cuts = impli.cuts_from_layer_work(np.ones(18), 16, 15, 17)
    assert cuts == list(range(1, 19))
    with pytest.raises(impli.ImplisolidError):
        impli.cuts_from_layer_work(np.ones(18), 16, 15, 18)


# ---- multi-rank numbering exchange (gloo, CPU) -----------------------------------------------------
def _slab_counts(codes, faces_cell_z, R, z0, z1, halo):
    """counts int32[4] a rank's Slab.count() produces: own vertices incl. halo, faces, -, halo."""
    oz = np_restate.owner_cell_z(codes, R)
    own = int(((oz >= z0 - halo) & (oz < z1)).sum())
    hal = int(((oz >= z0 - halo) & (oz < z0)).sum())
    nf = int(((faces_cell_z >= z0) & (faces_cell_z < z1)).sum())
    return [own, nf, 0, hal]


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import implisolid_amd as I
    from implisolid_amd import distributed as D
    from implisolid_amd import scenes
    import np_restate as N
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        shape, box, R = scenes.union_sphere_cube(), [-1, 1] * 3, 40
        F, w = N.field(shape, R, box)
        v, f, codes = N.mc_with_codes(F, w, box, R)
        oz = N.owner_cell_z(codes, R)          # owner layer of every vertex (first-appearance order)
        ci_layers = _face_layers(F, R)         # cell layer of every face (emission order)
        z0, z1, halo = I.slab_partition(R, rank, world)
        cnt = torch.tensor(_slab_counts(codes, ci_layers, R, z0, z1, halo), dtype=torch.int32)
        offs, gathered = D.global_offsets(cnt, rank, world)
        # expected: this rank's vertices/faces start where the global first-appearance numbering
        # places its first owned vertex / first face
        exp_v = int((oz < z0).sum())
        exp_f = int((ci_layers < z0).sum())
        # the bench's path: async gather into a [world, 4] buffer; the face kernel's vertex offset
        # is the sum over lower ranks of (own incl. halo - halo) (mc.hip k_mc_faces)
        g2 = torch.zeros(world, 4, dtype=torch.int32)
        work = D.gather_counts_async(cnt, g2)
        if work is not None:
            work.wait()
        voff_dev = int(sum(int(g2[r, 0]) - int(g2[r, 3]) for r in range(rank)))
        ok = (int(offs[0]) == exp_v and int(offs[1]) == exp_f and int(gathered[:, 1].sum()) == len(f)
              and int((gathered[:, 0] - gathered[:, 3]).sum()) == len(v) and torch.equal(g2, gathered)
              and voff_dev == exp_v)
        q.put((rank, ok, [int(offs[0]), int(offs[1])], [exp_v, exp_f]))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e), None))


def _face_layers(F, R):
    """cell layer zi of every face, in emission order (z-major cells, table order)."""
    res = R + 5
    n = res - 3
    corner = [F[1 + dz:1 + dz + n, 1 + dy:1 + dy + n, 1 + dx:1 + dx + n] for dx, dy, dz in np_restate.CORNER_OFF]
    ci = np.zeros((n, n, n), np.int64)
    for k in range(8):
        ci |= np.where(corner[k] < np.float32(0), np_restate.CORNER_BIT[k], 0)
    ntri = np.array([len(t) // 3 for t in np_restate.TRI])
    per_cell = ntri[ci.ravel()]
    zi = np.arange(per_cell.size) // (n * n) + 1
    return np.repeat(zi, per_cell)


@pytest.mark.parametrize("world", [2, 3])
def test_zslab_offsets_gloo(world):
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, got, exp in sorted(res):
        assert ok, (rank, got, exp)


# ---- JavaScript binding (N-API addon over the C ABI) -----------------------------------------------
def _node_ok():
    import shutil
    return shutil.which("node") and os.path.exists("/usr/include/node/node_api.h")


@pytest.mark.skipif(not _node_ok(), reason="node or node headers absent")
def test_node_addon_exports(impli):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "bindings", "node")], check=True)
    js = ("const {impli1, native} = require('./bindings/node/impli1.js');"
          "impli1.set_error_mode(1);"
          "const ok = native.program_info(JSON.stringify({type:'iellipsoid', matrix:[1,0,0,0,0,1,0,0,0,0,1,0]}));"
          "const bad = native.program_info('{\"type\":\"bogus\",\"matrix\":[1,0,0,0,0,1,0,0,0,0,1,0]}');"
          "console.log(JSON.stringify({keys: Object.keys(native), ok, bad, err: impli1.last_error()}));")
    r = subprocess.run(["node", "-e", js], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    need = {"build_geometry", "build_geometry_u", "get_v_size", "get_f_size", "get_v", "get_f", "finish_geometry", "set_object",
            "unset_object", "set_x", "unset_x", "calculate_implicit_values", "get_values",
            "calculate_implicit_gradients", "get_gradients", "get_pointset", "about"}
    assert need <= set(out["keys"])
    assert out["ok"] == 2 and out["bad"] == -1 and "Invalid object" in out["err"]


def test_jit_tree_kernels_compile_for_gfx950(impli):
    """Host-only: the generated tree kernel compiles with hipRTC for several shapes."""
    from implisolid_amd import scenes
    for shape in [{"type": "iellipsoid", "matrix": scenes.EYE}, scenes.union_sphere_cube(), scenes.config3()[0],
                  scenes.random_tree(7, 10)]:
        n, secs, src = impli.jit_compile(shape)
        assert n > 1000 and "impli_eval_bricks" in src, src[:500]
        assert "impli_coarse_modes" in src and "impli_brick_refine" in src
        # the brick pair's tree code (both layers in one pass) and the eval kernel's occupancy request
        assert "tree_f2(M, tab, m, x, y, z0, z1, f0, f1)" in src
        assert "__launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void impli_eval_bricks" in src


def test_jit_pair_code_shares_the_screw_atan2f(impli):
    """Host-only: a twist leaf's pair code calls screw_f2 (one atan2f for both layers when their
    (ab1, ab0) agree); the baked source of an object holds the same calls with literal matrices."""
    from implisolid_amd import scenes
    shape = scenes.twist(1, 0, 0, 0)
    _, _, src = impli.jit_compile(shape)
    assert "screw_f2(M + " in src
    impli.set_jit_bake(1)
    try:
        _, _, baked = impli.jit_compile(scenes.config3()[0])
    finally:
        impli.set_jit_bake(2)
    assert "screw_f2(M + " in baked and "__builtin_bit_cast(float, 0x" in baked


def test_headline_summary_oracle_regression(oracle):
    """The cheapest headline fixture (config 2, R 128, 3 OB02 repeats; tests/golden/make_headline.py)
    still reproduces from the oracle -- the GPU tests compare against these summaries."""
    import hashlib
    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "headline_summaries.json")))
    s = d["config2_ob02_r128"]
    v, f = oracle.polygonize(json.dumps(s["shape"]), json.dumps(s["mc"]))
    assert (len(v), len(f)) == (s["n_verts"], s["n_faces"])
    assert hashlib.sha256(np.ascontiguousarray(f).tobytes()).hexdigest() == s["sha256_faces"]
    assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == s["sha256_verts"]


def test_fold_table_exact(tmp_path):
    """The OB02 edge-length fold from the device's chunk table (implisolid_amd/csrc/fold.hpp) equals
    the serial float chain bit for bit on 600+ seeded arrays: edge-length-like terms, wide spreads,
    engineered ties near binade tops, zeros, subnormals, inf, NaN payloads, saturation past 2^24
    (tools/fold_check.cpp; most chunks taken from the table, the rest term by term)."""
    exe = str(tmp_path / "fold_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", os.path.join(ROOT, "tools", "fold_check.cpp"),
                    "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr
    table = int(r.stdout.split("from the table")[1].split()[0])
    assert table > 50000, r.stdout


def test_divconst_identity_exhaustive(tmp_path):
    """The double mushroom's divisions by its constant use q0 = a R, q = fma(fma(-q0, D, a), R, q0)
    (ifunc_device.hpp div_sq_const); it must equal the IEEE quotient for the square of every float
    (all 2^32 bit patterns, tools/divconst_check.c)."""
    exe = str(tmp_path / "divconst_check")
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-pthread", os.path.join(ROOT, "tools", "divconst_check.c"),
                    "-o", exe, "-lm"], check=True)
    r = subprocess.run([exe, str(min(8, os.cpu_count() or 1))], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_ob02_exchange_plan(impli):
    """distributed.ob02_plan (the sharded OB02 loop's exchanges): after a vertex-moving step, the
    one-ring halo when the next step is a resampling (it reads only the vertices of the faces whose
    centroids its weights use), every owned range when the next is a projection (the edge-length
    fold reads every edge) and at the end (rank 0 returns the whole mesh); a projection without
    QEM moves nothing."""
    from implisolid_amd import distributed as D
    from implisolid_amd import scenes
    st = impli.parse_settings(scenes.config2(64)[1])   # 3 x [1 resampling, projection + QEM]
    assert D.ob02_plan(st) == [("R", "full"), ("P", "halo"), ("R", "full"), ("P", "halo"), ("R", "full"), ("P", "full")]
    two = impli.parse_settings(scenes.mc_settings(32, 1.0, vresampl_iters=2, vresampl_c=0.4, projection=1, qem=0,
                                                  overall_repeats=2))
    assert D.ob02_plan(two) == [("R", "halo"), ("R", "full"), ("P", None), ("R", "halo"), ("R", "full"), ("P", None)]
    proj_only = impli.parse_settings(scenes.mc_settings(32, 1.0, projection=1, qem=1, overall_repeats=2))
    assert D.ob02_plan(proj_only) == [("P", "full"), ("P", "full")]
    assert D.ob02_plan(impli.parse_settings(scenes.mc_settings(32, 1.0))) == []


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_transfers_symmetric_and_covering(world):
    """distributed.shard_transfers (the ranges every exchange path of the sharded OB02 loop moves:
    RCCL point-to-point / all-gather, gloo, and the one-process device copies): what rank r sends q
    is what q receives from r, nothing is sent to oneself, and after a halo exchange each rank holds
    its whole halo (own range plus the received ranges tile it exactly); a full exchange gives every
    rank every other rank's owned range."""
    from implisolid_amd import distributed as D
    rng = np.random.default_rng(world)
    for trial in range(200):
        cuts = np.sort(rng.integers(0, 5000, size=world - 1))
        voff = [0] + [int(c) for c in cuts] + [5000]
        halos = []
        for r in range(world):   # a halo reaches a little below and above the owned range
            lo = max(0, voff[r] - int(rng.integers(0, 400)))
            hi = min(5000, voff[r + 1] + int(rng.integers(0, 400)))
            halos.append((lo, hi) if voff[r] < voff[r + 1] else (0, 0))
        for kind in ("halo", "full"):
            plans = [D.shard_transfers(voff, halos, r, kind) for r in range(world)]
            for r, (sends, recvs) in enumerate(plans):
                assert all(q != r and a < b for q, a, b in sends + recvs)
                for q, a, b in sends:
                    assert (r, a, b) in plans[q][1]
                    assert voff[r] <= a and b <= voff[r + 1]
                for q, a, b in recvs:
                    assert (r, a, b) in plans[q][0]
                    assert voff[q] <= a and b <= voff[q + 1]
                have = np.zeros(5000, bool)
                have[voff[r]:voff[r + 1]] = True
                for q, a, b in recvs:
                    assert not have[a:b].any()
                    have[a:b] = True
                want = np.zeros(5000, bool)
                if kind == "full":
                    want[:] = True
                else:
                    want[halos[r][0]:halos[r][1]] = True
                    want[voff[r]:voff[r + 1]] = True
                assert np.array_equal(have, want)
