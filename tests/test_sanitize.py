"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

The C ABI takes untrusted strings (polygoniser_settings.hpp:147-305 parses the mc-settings JSON,
object_factory.hpp:56-758 the MP5 shape JSON); the library's host side that reads them -- the JSON
DOM (json.hpp), the settings parser and MP5 compiler (host.cpp), the JIT's source generation from
the compiled program (jit.cpp), slab ranges, the float LU inverse and glibc rand -- is built with
-fsanitize=address,undefined,float-cast-overflow (tests/sanitize/Makefile) and driven with every
shape and settings string the other tests use, plus malformed, truncated, deeply nested, oversized
and out-of-range ones.  The oracle restatement (oracle/*.c) gets the same build, loaded into a
Python process with libasan preloaded, and polygonises a few scenes through MC and OB02.

Any sanitizer report aborts the process (-fno-sanitize-recover=all), so a clean exit is the check.
The run found two undefined float-to-int conversions (an out-of-range "resolution" and extrusion
"size"), now rejected as the reference's intent requires, and an unbounded parser recursion.
"""
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


@pytest.fixture(scope="module")
def san_build():
    if not shutil.which("g++"):
        pytest.skip("no g++")
    r = subprocess.run(["make", "-s", "-C", SAN, "-j4"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(SAN, "build")


def _shapes():
    from implisolid_amd import scenes
    out = [scenes.config1()[0], scenes.config2(64)[0], scenes.config3()[0], scenes.union_sphere_cube(),
           scenes.tetrahedron(), scenes.meta_balls(), scenes.extrusion(6), scenes.twist(1, 0, 0, 0)]
    out += [scenes.random_tree(7000 + k, 1 + k % 12) for k in range(24)]
    out += [o[0] for o in scenes.config5_objects(8, 32)]
    tw = scenes.twist(0.5, 0, 0.25, 0.0625)
    out += [dict(tw, type="screw_diff_two_plane"), dict(tw, type="inf_screw"), dict(tw, type="screw_gradient_wrong"),
            {"type": "half_plane", "matrix": scenes.EYE, "plane_vector": [0, 1, 2], "plane_point": [0, 0, 0.25]},
            {"type": "top_bottom_lid", "matrix": scenes.EYE}]
    return out


def _malformed(valid_shape, valid_settings):
    eye = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]
    s = json.dumps(valid_shape)
    cases = []
    # every truncation of a valid document (stride 3) and a few byte flips
    cases += [("mp5", s[:k]) for k in range(0, len(s), 3)]
    cases += [("settings", valid_settings[:k]) for k in range(0, len(valid_settings), 2)]
    for k in range(0, len(s), 7):
        cases.append(("mp5", s[:k] + "\x01" + s[k + 1:]))
        cases.append(("mp5", s[:k] + '"' + s[k:]))
    # nesting far past any bound, in arrays and objects and as MP5 node trees
    cases += [("mp5", "[" * 100000), ("mp5", "{\"a\":" * 50000 + "1" + "}" * 50000), ("settings", "[" * 300 + "]" * 300)]
    node = {"type": "iellipsoid", "matrix": eye}
    for _ in range(40):
        node = {"type": "Intersection", "matrix": eye, "children": [node, {"type": "icone", "matrix": eye}]}
    cases.append(("mp5", json.dumps(node)))
    cases.append(("mp5", json.dumps({"type": "Union", "matrix": eye, "children": [{"type": "iellipsoid", "matrix": eye}] * 5000})))
    # oversized / odd matrices, numbers no float or int holds, wrong types
    for m in ([1e39] * 12, [float("nan")] * 12, ["x"] * 12, [1] * 11, [0.5] * 4000, [[1]] * 12, [], "matrix",
              [0] * 12, [1e-45] * 12, [3.4e38, 0, 0, 0, 0, 3.4e38, 0, 0, 0, 0, 3.4e38, 1e38]):
        cases.append(("mp5", json.dumps({"type": "iellipsoid", "matrix": m}).replace("NaN", "nan")))
    for size in ("1e30", "-1e30", "nan", "inf", "2", "41", "40", "\"7\"", "3.99"):
        cases.append(("mp5", '{"type":"extrusion","size":%s,"matrix":%s}' % (size, json.dumps(eye))))
    for t in ("screw", "tetrahedron", "meta_balls", "half_plane", "sdf_3d", "rawjscode", "", "Union", "Difference"):
        cases.append(("mp5", json.dumps({"type": t, "matrix": eye})))
        cases.append(("mp5", json.dumps({"type": t, "matrix": eye, "children": [], "pitch": "a", "delta_ratio": 0,
                                         "corners": [[1e39, "x"], 5], "plane_vector": [0, 0, 0], "plane_point": 1,
                                         "v": 1, "profile": 1, "end_type": 1, "time": "t"})))
    cases.append(("mp5", '{"type":"iellipsoid","matrix":[1,0,0,0,0,1,0,0,0,0,1,0],"s":"\\u12"}'))
    cases.append(("mp5", '{"type":"iellipsoid","matrix":[1,0,0,0,0,1,0,0,0,0,1,0],"s":"\\uzzzz\\ud800\\\\"}'))
    cases.append(("mp5", "\x00"))
    cases.append(("mp5", ""))
    for res in ("1e20", "-1e20", "nan", "inf", "2147483648", "-2147483649", "65536", "3.5", "\"12\"", "true", "9" * 40):
        cases.append(("settings", '{"resolution": %s, "overall_repeats": 99999999999999, "vresampl": {"iters": %s}}'
                      % (res, res)))
    cases.append(("settings", '{"box": {"xmin": "nan", "xmax": 1e39}, "resolution": 8}'))
    cases.append(("settings", '{"qem": {"enabled": 1}, "projection": {"enable": 1}}'))
    return cases


def _run_driver(path, records):
    text = "\n%%\n".join(k + "\n" + p if k in ("settings", "mp5", "mp5i") else k + " " + p for k, p in records)
    r = subprocess.run([os.path.join(path, "host_driver")], input=text.encode("latin-1", "replace"),
                       capture_output=True, env=ENV, timeout=600)
    return r.returncode, r.stdout.decode(errors="replace").splitlines(), r.stderr.decode(errors="replace")


def test_host_code_under_sanitizers(san_build):
    from implisolid_amd import scenes
    shapes = _shapes()
    settings = [scenes.config1()[1], scenes.config2(64)[1], scenes.config3(256)[1], scenes.mc_settings(512, 1.0)]
    records = []
    for sh in shapes:
        records += [("mp5", json.dumps(sh)), ("mp5i", json.dumps(sh))]
    records += [("settings", json.dumps(st)) for st in settings]
    records += _malformed(scenes.config3()[0], json.dumps(settings[2]))
    for R, z0, z1 in ((32, 1, 35), (512, 1, 515), (512, 200, 260), (1623, 1, 1626), (1700, 1, 1703), (512, 0, 10),
                      (512, 10, 5), (2, 1, 2), (-5, 1, 2), (2147483647, 1, 2147483647)):
        records.append(("slab", "%d %d %d" % (R, z0, z1)))
    for R, rank, n in ((512, 0, 8), (512, 7, 8), (512, 8, 8), (512, -1, 8), (10, 0, 64), (512, 0, 0), (0, 0, 1)):
        records.append(("partition", "%d %d %d" % (R, rank, n)))
    import numpy as np
    rng = np.random.default_rng(5)
    for _ in range(200):
        m = rng.standard_normal(12) * 10.0 ** rng.integers(-40, 40, 12)
        records.append(("matrix", " ".join("%.9g" % x for x in m)))
    records += [("matrix", " ".join(["0"] * 12)), ("matrix", " ".join(["1e38"] * 12)), ("matrix", " ".join(["nan"] * 12))]
    records += [("rand", "%d %d" % (seed, n)) for seed, n in ((1, 0), (1, 1000), (0, 31), (12345, 1 << 20), (7, 3))]
    rc, out, err = _run_driver(san_build, records)
    assert rc == 0, err[-3000:]
    assert "runtime error" not in err and "AddressSanitizer" not in err, err[-3000:]
    assert len(out) == len(records), (len(out), len(records), err[-2000:])
    # the valid inputs compile; the reference's abort cases are errors, never crashes
    n_valid = 2 * len(shapes)
    assert all(line.startswith("ok mp5") for line in out[:n_valid]), [l for l in out[:n_valid] if not l.startswith("ok")][:5]
    assert all(line.startswith("ok settings") for line in out[n_valid:n_valid + len(settings)])
    tail = out[n_valid + len(settings):]
    assert any("nested too deeply" in line for line in tail)
    assert any("err3" in line for line in tail)           # resolution 1e20: not an integer, no UB
    assert any("extrusion: Invalid size" in line for line in tail)
    for line in out:
        if line.startswith("ok rand"):
            a, b = line.split()[2:4]
            assert a == b                                    # skip(n) == n draws


def test_oracle_under_sanitizers(san_build):
    """The oracle's C restatement (MC, OB02 resampling / projection / QEM, subdivision, eval and
    gradients) in a Python process with the sanitizer runtime preloaded."""
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not asan or not os.path.exists(asan):
        pytest.skip("libasan not found")
    script = r"""
import json, sys
sys.path.insert(0, %r)
import numpy as np
import oracle
oracle._LIB_PATH = %r
from implisolid_amd import scenes
shapes = [scenes.config1()[0], scenes.config3()[0], scenes.union_sphere_cube(), scenes.twist(1, 0, 0, 0),
          scenes.meta_balls(), scenes.extrusion(5), scenes.tetrahedron()]
rng = np.random.default_rng(3)
pts = rng.uniform(-1.2, 1.2, (4000, 3)).astype(np.float32)
pts[::97] = np.nan
for sh in shapes:
    t = oracle.mp5_to_nodes(json.dumps(sh))
    oracle.eval_implicit(t, pts); oracle.eval_gradient(t, pts)
    v, f = oracle.marching_cubes(t, 20, [-1.0, 1.0] * 3)
shape, mc = scenes.config2(24)
v, f = oracle.polygonize(json.dumps(shape), json.dumps(mc))
shape3, mc3 = scenes.config3_shifted(20)
v3, f3 = oracle.polygonize(json.dumps(shape3), json.dumps(mc3))
mc = dict(mc, subdiv={"enabled": 1})
v2, f2 = oracle.polygonize(json.dumps(shape), json.dumps(mc))
print("ok", len(v), len(f), len(v2), len(f2))
""" % (ROOT, os.path.join(san_build, "liboracle_asan.so"))
    env = dict(ENV, LD_PRELOAD=asan)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.stdout[-500:], r.stderr[-3000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
