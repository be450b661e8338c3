"""CPU oracle for the implicit-surface polygoniser hot path -- TEST INFRASTRUCTURE ONLY.

This package restates the reference (ynotstartups/implisolid, ``js_iteration_2/``) on the CPU so the
MI355X path can be checked against it.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it; the product (``implisolid_amd``) never does.

* ``oracle/*.c`` (built to ``oracle/build/liboracle.so`` by ``oracle/Makefile``): implicit-function
  evaluation, marching cubes with first-appearance numbering, vertex resampling, centroid
  projection + bisection, QEM.  Each C function cites the reference file:line it restates.
* this module: the MP5-JSON factory (``object_factory.hpp:56-758``) and the mc-settings parser
  (``polygoniser_settings.hpp:147-305``) restated in Python, the ``grand_algorithm`` driver
  (``mcc2.cpp:309-444``) and ctypes bindings.

Parity status: **parity unpinned** -- the reference ships no tests, fixtures or golden vectors and
cannot be compiled here (Boost/Eigen/emscripten.h are absent; header stand-ins are not allowed), so
the oracle is a restatement checked by construction, by property tests and by the exhaustive
glibc-acosf check (see DESIGN.md "Oracle").
"""
import ctypes
import json
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

(UNION, INTERSECTION, DIFFERENCE, ELLIPSOID, CUBE, CYLINDER, CONE, HEART, TORUS, DMUSHROOM, SCREW, LID, HALF_PLANE,
 TETRA, METABALLS, EXTRUSION, SCREW_TBB) = range(17)

# MP5 "type" strings accepted by object_factory.hpp:86-653 for the plain-arithmetic node families.
PRIMITIVE_TYPES = {
    "implicit_double_mushroom": DMUSHROOM,   # object_factory.hpp:86-100
    "icube": CUBE, "cube": CUBE,             # :110-119
    "icylinder": CYLINDER, "cylinder": CYLINDER,  # :121-132
    "iellipsoid": ELLIPSOID, "ellipsoid": ELLIPSOID,  # :134-143
    "icone": CONE, "cone": CONE,             # :144-152
    "iheart": HEART,                         # :153-162
    "itorus": TORUS,                         # :163-173
}
# types the reference knows but this build does not evaluate (Eigen-based or JS callbacks)
KNOWN_UNSUPPORTED = {"sdf_3d", "rawjscode"}


class OrNode(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("child", ctypes.c_int32 * 2),
                ("m", ctypes.c_float * 12), ("minv", ctypes.c_float * 12), ("prm", ctypes.c_float * 128)]


class OrMesh(ctypes.Structure):
    _fields_ = [("verts", ctypes.POINTER(ctypes.c_float)), ("faces", ctypes.POINTER(ctypes.c_int32)),
                ("nv", ctypes.c_int64), ("nf", ctypes.c_int64)]


_lib = None


def build():
    """Compile oracle/*.c (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int32)
        npp = ctypes.POINTER(OrNode)
        L.or_invert_matrix.argtypes = [fp, fp]
        L.or_tree_prepare.argtypes = [npp, ctypes.c_int]
        L.or_eval.argtypes = [npp, ctypes.c_int, fp, ctypes.c_int64, fp]
        L.or_grad.argtypes = [npp, ctypes.c_int, fp, ctypes.c_int64, fp]
        L.or_acosf.argtypes = [ctypes.c_float]
        L.or_acosf.restype = ctypes.c_float
        L.or_acosf_check.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.or_acosf_check.restype = ctypes.c_int64
        for fn in ("or_sinf", "or_atanf"):
            getattr(L, fn).argtypes = [ctypes.c_float]
            getattr(L, fn).restype = ctypes.c_float
        L.or_atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
        L.or_atan2f.restype = ctypes.c_float
        L.or_libm_check.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.or_libm_check.restype = ctypes.c_int64
        L.or_libm_apply.argtypes = [ctypes.c_int, fp, fp, ctypes.c_int64, fp]
        L.or_libm_apply.restype = None
        L.or_cos.argtypes = [ctypes.c_double]
        L.or_cos.restype = ctypes.c_double
        L.or_cos_check.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double]
        L.or_cos_check.restype = ctypes.c_int64
        L.or_cos_apply.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int64, ctypes.POINTER(ctypes.c_double),
                                   ctypes.c_int]
        L.or_cos_apply.restype = None
        L.or_marching_cubes.argtypes = [npp, ctypes.c_int, ctypes.c_int, fp, ctypes.POINTER(OrMesh)]
        L.or_mesh_free.argtypes = [ctypes.POINTER(OrMesh)]
        L.or_mc_field.argtypes = [npp, ctypes.c_int, ctypes.c_int, fp, fp]
        L.or_vertex_resampling.argtypes = [npp, ctypes.c_int, ctypes.c_float, fp, ctypes.c_int64, ip,
                                           ctypes.c_int64, fp]
        L.or_centroids_projection.argtypes = [npp, ctypes.c_int, fp, ctypes.c_int64, ip, ctypes.c_int64,
                                              ctypes.c_int, fp, fp]
        L.or_subdivide.argtypes = [fp, ctypes.c_int64, ip, ctypes.c_int64, ctypes.c_float,
                                   ctypes.POINTER(fp), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ip)]
        L.or_srand.argtypes = [ctypes.c_uint]
        L.or_rand.restype = ctypes.c_int
        L.or_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


# ---------------------------------------------------------------------------------------------
# number parsing: boost::property_tree get_value<float> reads with a C++ stream (strtof semantics)
_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]


def strtof(s):
    s = str(s).strip()
    b = s.encode()
    end = ctypes.c_char_p()
    v = _libc.strtof(b, ctypes.byref(end))
    return np.float32(v)


def _loads(text):
    """JSON with numbers kept as their source text (ptree stores strings)."""
    if isinstance(text, (dict, list)):
        return text
    return json.loads(text, parse_float=str, parse_int=str)


def _matrix12(d):
    """getMatrix12 object_factory.hpp:21-30: the first 12 entries (16-entry matrices overflow the
    reference's REAL[12], F8b -- we accept 12 or 16 and use the first 12)."""
    vals = d.get("matrix")
    if vals is None or len(vals) < 12:
        raise ValueError("MP5 node needs a 12- or 16-entry 'matrix'")
    return [strtof(v) for v in vals[:12]]


EYE12 = [np.float32(v) for v in (1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0)]


def _screw_params(d):
    """screw::getScrewParameters (screw.hpp:380-470) + the constructor (:222-330), in float:
    outer = |v| = 1 (v = (0,1,0)), inner = outer / delta_ratio, r0 = inner / 2,
    delta = outer / 2 - inner / 2, twist_rate = pitch.  "matrix", "v", "profile" and "end_type"
    must be present (ptree get_child / get throw); their values are unused."""
    for k in ("matrix", "v", "pitch", "profile", "end_type", "delta_ratio"):
        if k not in d:
            raise ValueError("screw: missing %r" % k)
    f = np.float32
    pitch, ratio = strtof(d["pitch"]), strtof(d["delta_ratio"])
    outer = f(1.0)
    inner = f(outer / ratio)
    r0 = f(inner / f(2))
    delta = f(f(outer / f(2)) - f(inner / f(2)))
    return [pitch, r0, delta]


def _half_plane_params(pv, pp):
    """half_plane constructor (half_plane.hpp:96-125): plane_vector / plane_vector.norm() in float,
    the norm reduced as a0 + (a1 + a2)."""
    f = np.float32
    v = [strtof(a) for a in pv]
    n = np.sqrt(f(v[0] * v[0] + f(v[1] * v[1] + v[2] * v[2])))
    return [f(a / n) for a in v] + [strtof(a) for a in pp]


_libm = ctypes.CDLL("libm.so.6")
for _fn, _t in (("sin", ctypes.c_double), ("cos", ctypes.c_double), ("sqrt", ctypes.c_double),
                ("sinf", ctypes.c_float), ("cosf", ctypes.c_float)):
    getattr(_libm, _fn).argtypes = [_t]
    getattr(_libm, _fn).restype = _t


def _tetra_params(d, m12):
    """tetrahedron (tetrahedron.hpp:20-128): the corners (getCorners, object_factory.hpp:32-45; a
    missing corner stays 0) moved by the forward matrix (matrix_vector_product, basic_functions.hpp:
    140-177), the four planes of calculatePlaneCoefficients, each multiplied by the sign (tolerance
    ROOT_TOLERANCE, configs.hpp:33) of its value at the opposite corner."""
    f = np.float32
    c = [[f(0)] * 3 for _ in range(4)]
    for i, corner in enumerate(d.get("corners", [])[:4]):
        for j, v in enumerate(corner[:3]):
            c[i][j] = strtof(v)
    m = [f(v) for v in m12]
    p = [[f(f(f(f(m[4 * r] * q[0]) + f(m[4 * r + 1] * q[1])) + f(m[4 * r + 2] * q[2])) + m[4 * r + 3]) for r in range(3)]
         for q in c]

    def coef(P1, P2, P3):
        x1, y1, z1 = P1
        x2, y2, z2 = P2
        x3, y3, z3 = P3
        a = f(f(f(f(f(y1 * z2) - f(y1 * z3)) - f(y2 * z1)) + f(y2 * z3)) + f(y3 * z1)) - f(y3 * z2)
        b = f(f(f(f(f(x1 * z3) - f(x1 * z2)) + f(x2 * z1)) - f(x2 * z3)) - f(x3 * z1)) + f(x3 * z2)
        cc = f(f(f(f(f(x1 * y2) - f(x1 * y3)) - f(x2 * y1)) + f(x2 * y3)) + f(x3 * y1)) - f(x3 * y2)
        dd = f(f(f(f(f(f(x1 * y3) * z2) - f(f(x1 * y2) * z3)) + f(f(x2 * y1) * z3)) - f(f(x2 * y3) * z1))
               - f(f(x3 * y1) * z2)) + f(f(x3 * y2) * z1)
        return [a, b, cc, dd]

    planes = [coef(p[1], p[2], p[3]), coef(p[0], p[2], p[3]), coef(p[0], p[1], p[3]), coef(p[0], p[1], p[2])]
    tol = f(0.001 / 10.0)
    out = []
    for k in range(4):
        a, b, cc, dd = planes[k]
        v = f(f(f(f(a * p[k][0]) + f(b * p[k][1])) + f(cc * p[k][2])) + dd)
        sg = f(1) if v > tol else (f(-1) if v < -tol else f(0))
        out += [f(a * sg), f(b * sg), f(cc * sg), f(dd * sg)]
    return out


def _metaball_params(d):
    """meta_ball_Rydgard (meta_balls_Rydgard.hpp:27-60) with 4 blobs, scale 1 and `time` (default
    0.1): the ball centres in double (libm sin / cos) stored to float; strength 1.2 / ((sqrt(4) - 1)
    / 4 + 1), subtract 12."""
    f = np.float32
    time = strtof(d["time"]) if "time" in d else f(0.1)
    t, D, half = float(time), float(f(1)), float(f(0.5))
    out = []
    for i in range(4):
        bx = _libm.sin(i + 1.26 * t * (1.03 + 0.5 * _libm.cos(0.21 * i))) * 0.27 * D + 0.5 - half
        by = abs(_libm.cos(i + 1.12 * t * _libm.cos(1.22 + 0.1424 * i))) * 0.77 * D - half
        bz = _libm.cos(i + 1.32 * t * 0.1 * _libm.sin(0.92 + 0.53 * i)) * 0.27 * D + 0.5 - half
        strength = 1.2 / ((_libm.sqrt(4) - 1) / 4 + 1)
        out += [f(bx), f(by), f(bz), f(strength), f(12)]
    return out


def _extrusion_params(d):
    """extrusion(eye, size) (extrusion.hpp:61-94): a regular `size`-gon of radius 0.5 starting at
    (0, 0.5), counter-clockwise, corners from polarToCartesian (basic_functions.hpp:33-36: cosf /
    sinf of a float angle); convex_polygon::update_inner_data (:77-93) edge normals in float with
    1/d divided in double."""
    f = np.float32
    if "size" not in d:
        raise ValueError("extrusion: missing 'size'")
    size = int(strtof(d["size"]))
    if size < 3:
        raise ValueError("extrusion: Invalid size")
    if size > 40:
        raise ValueError("extrusion: size above 40 is not supported")
    PI = f(3.141592653589793238463)
    rot = f(f(2 * PI) / f(size))
    cx, cy = [f(0)], [f(0.5)]
    for i in range(1, size):
        theta = f(float(PI) / 2.0 + float(f(f(i) * rot)))
        cx.append(f(f(0.5) * f(_libm.cosf(theta))))
        cy.append(f(f(0.5) * f(_libm.sinf(theta))))
    out = [f(size)]
    for i in range(size):
        j = i + 1 if i < size - 1 else 0
        dx, dy = f(cx[j] - cx[i]), f(cy[j] - cy[i])
        dd = np.sqrt(f(f(dx * dx) + f(dy * dy)))
        dinv = f(1.0 / float(dd)) if dd > 0.00000001 else f(0)
        nx, ny = f(dy * dinv), f(-dx * dinv)
        out += [nx, ny, f(f(cx[i] * nx) + f(cy[i] * ny))]
    return out


def mp5_to_nodes(shape, ignore_root_matrix=False):
    """object_factory (object_factory.hpp:56-758) -> flat node list + root index."""
    nodes = []

    def add(t, m, c0=-1, c1=-1, prm=None):
        nodes.append((t, (c0, c1), m, prm or []))
        return len(nodes) - 1

    def build_node(d, ignore):
        t = d.get("type")
        if t in PRIMITIVE_TYPES:
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            return add(PRIMITIVE_TYPES[t], m)
        if t == "Union":                          # object_factory.hpp:537-580, left-deep chain
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            ch = d.get("children") or []
            if len(ch) < 2:
                raise ValueError("Union needs at least two children (one child is UB in the reference)")
            a = build_node(ch[0], False)
            for k in range(1, len(ch)):
                b = build_node(ch[k], False)
                if k == len(ch) - 1:
                    a = add(UNION, m, a, b)       # o_matrix of the last step is the object
                else:
                    a = add(UNION, list(EYE12), a, b)  # o_plain
            return a
        if t in ("Intersection", "Difference"):   # :581-653, binary (extra children ignored)
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            ch = d.get("children") or []
            if len(ch) < 2:
                raise ValueError("%s needs two children" % t)
            a = build_node(ch[0], False)
            b = build_node(ch[1], False)
            return add(INTERSECTION if t == "Intersection" else DIFFERENCE, m, a, b)
        if t in ("screw", "inf_screw", "screw_diff_two_plane"):
            prm = _screw_params(d)
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            if t == "inf_screw":                   # :189-215: the screw under its own matrix
                return add(SCREW, m, prm=prm)
            s = add(SCREW, list(EYE12), prm=prm)   # transformation_matrix forced to identity
            if t == "screw":                       # :304-351: subtract(screw, top_bottom_lid)
                return add(DIFFERENCE, m, s, add(LID, list(EYE12)))
            # :216-302: subtract(subtract(screw, half_plane z >= .25), half_plane z <= -.25)
            top = add(HALF_PLANE, list(EYE12), prm=_half_plane_params(["0", "0", "1"], ["0", "0", "0.25"]))
            first = add(DIFFERENCE, list(EYE12), s, top)
            bot = add(HALF_PLANE, list(EYE12), prm=_half_plane_params(["0", "0", "-1"], ["0", "0", "-0.25"]))
            return add(DIFFERENCE, m, first, bot)
        if t == "screw_gradient_wrong":            # :435-479: inf_top_bot_bound(T, screw(T)), no
            return add(SCREW_TBB, _matrix12(d), prm=_screw_params(d))   # ignore_root_matrix
        if t == "top_bottom_lid":                  # :480-506: the matrix is read, then unused
            _matrix12(d)
            return add(LID, list(EYE12))
        if t == "half_plane":                      # :396-434
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            return add(HALF_PLANE, m, prm=_half_plane_params(d["plane_vector"], d["plane_point"]))
        if t == "tetrahedron":                     # :175-188
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            return add(TETRA, list(EYE12), prm=_tetra_params(d, m))
        if t == "meta_balls":                      # :654-673
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            return add(METABALLS, m, prm=_metaball_params(d))
        if t == "extrusion":                       # :674-731: subtract(extrusion(eye, size), lid)
            m = _matrix12(d)
            if ignore:
                m = list(EYE12)
            e = add(EXTRUSION, list(EYE12), prm=_extrusion_params(d))
            return add(DIFFERENCE, m, e, add(LID, list(EYE12)))
        if t in KNOWN_UNSUPPORTED:
            raise NotImplementedError("MP5 type %r is outside the implemented node families" % t)
        raise ValueError("Invalid object you asked for: %r" % t)   # the reference abort()s

    root = build_node(_loads(shape), ignore_root_matrix)
    arr = (OrNode * len(nodes))()
    for i, (t, (c0, c1), m, prm) in enumerate(nodes):
        for k, v in enumerate(prm):
            arr[i].prm[k] = float(v)
        arr[i].type = t
        arr[i].child[0] = c0
        arr[i].child[1] = c1
        for k in range(12):
            arr[i].m[k] = float(m[k])
    lib().or_tree_prepare(arr, len(nodes))
    return arr, root


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def invert_matrix(m12):
    a = np.ascontiguousarray(m12, dtype=np.float32)
    o = np.zeros(12, np.float32)
    lib().or_invert_matrix(_fp(a), _fp(o))
    return o


def eval_implicit(tree, pts):
    nodes, root = tree
    p = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 3)
    f = np.empty(p.shape[0], np.float32)
    lib().or_eval(nodes, root, _fp(p), p.shape[0], _fp(f))
    return f


def eval_gradient(tree, pts):
    nodes, root = tree
    p = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 3)
    g = np.empty((p.shape[0], 3), np.float32)
    lib().or_grad(nodes, root, _fp(p), p.shape[0], _fp(g))
    return g


def acosf(x):
    return np.float32(lib().or_acosf(float(x)))


def acosf_check(start, stride, count):
    """Mismatches of the acosf restatement against the host libm over a strided bit-pattern range."""
    return int(lib().or_acosf_check(start, stride, count))


def mc_field(tree, resolution, box):
    nodes, root = tree
    res = resolution + 5
    out = np.empty(res ** 3, np.float32)
    b = np.asarray(box, np.float32)
    if lib().or_mc_field(nodes, root, resolution, _fp(b), _fp(out)) != 0:
        raise MemoryError
    return out.reshape(res, res, res)


def marching_cubes(tree, resolution, box):
    nodes, root = tree
    b = np.asarray(box, np.float32)
    m = OrMesh()
    if lib().or_marching_cubes(nodes, root, resolution, _fp(b), ctypes.byref(m)) != 0:
        raise MemoryError
    v = np.ctypeslib.as_array(m.verts, shape=(m.nv * 3,)).copy().reshape(-1, 3) if m.nv else np.zeros((0, 3), np.float32)
    f = np.ctypeslib.as_array(m.faces, shape=(m.nf * 3,)).copy().reshape(-1, 3) if m.nf else np.zeros((0, 3), np.int32)
    lib().or_mesh_free(ctypes.byref(m))
    return v.astype(np.float32), f.astype(np.int32)


def vertex_resampling(tree, verts, faces, c):
    nodes, root = tree
    v = np.ascontiguousarray(verts, dtype=np.float32).copy()
    f = np.ascontiguousarray(faces, dtype=np.int32)
    cen = np.empty((f.shape[0], 3), np.float32)
    if lib().or_vertex_resampling(nodes, root, float(np.float32(c)), _fp(v), v.shape[0], _ip(f), f.shape[0], _fp(cen)):
        raise MemoryError
    return v, cen


def centroids_projection(tree, verts, faces, enable_qem):
    nodes, root = tree
    v = np.ascontiguousarray(verts, dtype=np.float32).copy()
    f = np.ascontiguousarray(faces, dtype=np.int32)
    cen = np.empty((f.shape[0], 3), np.float32)
    avg = np.zeros(1, np.float32)
    if lib().or_centroids_projection(nodes, root, _fp(v), v.shape[0], _ip(f), f.shape[0], int(bool(enable_qem)),
                                     _fp(cen), _fp(avg)):
        raise MemoryError
    return v, cen, float(avg[0])


def libm_check(which, start, stride, count):
    """Mismatches of the restated glibc sinf (0) / atanf (1) over bit patterns start + k*stride,
    or atan2f (2) over `count` seeded random pairs, against this host's libm."""
    return int(lib().or_libm_check(int(which), int(start), int(stride), int(count)))


def libm_apply(which, a, b=None):
    """The restated glibc sinf (0) / atanf (1) / atan2f (2: atan2f(a, b)) on float32 arrays."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(a if b is None else b, dtype=np.float32)
    out = np.empty_like(a)
    fpp = ctypes.POINTER(ctypes.c_float)
    lib().or_libm_apply(int(which), a.ctypes.data_as(fpp), b.ctypes.data_as(fpp), a.size, out.ctypes.data_as(fpp))
    return out


def cos_check(seed, count, lim=64.0):
    """Mismatches of the restated glibc double cos (x86_64 FMA variant) against this host's cos over
    `count` seeded arguments (or_libm.c or_cos_check)."""
    return int(lib().or_cos_check(int(seed), int(count), float(lim)))


def cos_apply(a, glibc=False):
    """The restated glibc double cos (glibc=False) or the host's own cos (True) on a float64 array."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    dpp = ctypes.POINTER(ctypes.c_double)
    lib().or_cos_apply(a.ctypes.data_as(dpp), a.size, out.ctypes.data_as(dpp), int(bool(glibc)))
    return out


def srand(seed):
    """glibc srand() of this process (the state randomize_verts' rand() calls draw from)."""
    lib().or_srand(int(seed))


def rand():
    return int(lib().or_rand())


def subdivide(verts, faces, amplitude):
    """my_subdiv_ (centroids_projection.cpp:1314-1367): 1-to-4 subdivision + randomize_verts noise
    drawn from this process's glibc rand()."""
    v = np.ascontiguousarray(verts, dtype=np.float32)
    f = np.ascontiguousarray(faces, dtype=np.int32)
    vo = ctypes.POINTER(ctypes.c_float)()
    fo = ctypes.POINTER(ctypes.c_int32)()
    n = ctypes.c_int64(0)
    if lib().or_subdivide(_fp(v), v.shape[0], _ip(f), f.shape[0], float(np.float32(amplitude)),
                          ctypes.byref(vo), ctypes.byref(n), ctypes.byref(fo)):
        raise MemoryError
    nv, nf = n.value, 4 * f.shape[0]
    V = np.ctypeslib.as_array(vo, shape=(nv * 3,)).copy().reshape(-1, 3) if nv else np.zeros((0, 3), np.float32)
    F = np.ctypeslib.as_array(fo, shape=(nf * 3,)).copy().reshape(-1, 3) if nf else np.zeros((0, 3), np.int32)
    lib().or_free(ctypes.cast(vo, ctypes.c_void_p))
    lib().or_free(ctypes.cast(fo, ctypes.c_void_p))
    return V.astype(np.float32), F.astype(np.int32)


# ---------------------------------------------------------------------------------------------
# polygoniser_settings.hpp:147-305 parse_mc_properties_json
class MCSettings:
    def __init__(self):
        self.box = [np.float32(-1), np.float32(1)] * 3
        self.resolution = 28
        self.ignore_root_matrix = False
        self.overall_repeats = 1
        self.vresampl_iters = 0
        self.vresampl_c = np.float32(1.0)
        self.projection = False
        self.qem = False
        self.subdiv = True
        self.post_subdiv_noise = np.float32(0.01)


def _get(d, path):
    cur = d
    for k in path.split("."):
        if not isinstance(cur, dict) or k not in cur:
            return None
        cur = cur[k]
    return cur


def _get_int(d, path, default):
    v = _get(d, path)
    if v is None or isinstance(v, (dict, list)):
        return default
    try:
        s = str(v).strip()
        if not s.lstrip("-").isdigit():
            return default
        return int(s)
    except ValueError:
        return default


def _get_float(d, path, default):
    v = _get(d, path)
    if v is None or isinstance(v, (dict, list)):
        return default
    try:
        float(str(v))
    except ValueError:
        return default
    return strtof(v)


def parse_mc_settings(text):
    d = _loads(text)
    s = MCSettings()
    box = [_get_float(d, "box." + k, None) for k in ("xmin", "xmax", "ymin", "ymax", "zmin", "zmax")]
    if any(v is None for v in box):
        raise ValueError("Error: missing or incorrect values in mc_parameters_json (box)")
    s.box = [np.float32(v) for v in box]
    r = _get_float(d, "resolution", np.float32(-1))
    ri = int(r)
    if ri == -1:
        ri = 28
    if np.float32(ri) != r:
        raise ValueError("Error: resolution must be integer")
    if ri <= 2:
        raise ValueError("Error: resolution must be > 2")
    s.resolution = ri
    s.vresampl_c = _get_float(d, "vresampl.c", np.float32(1.0))
    s.vresampl_iters = _get_int(d, "vresampl.iters", 0)

    def rb(name, default):
        v = _get_int(d, name, -1)
        return default if v == -1 else bool(v)
    s.projection = rb("projection.enabled", False)
    s.qem = rb("qem.enabled", False)
    s.subdiv = rb("subdiv.enabled", True)
    s.post_subdiv_noise = _get_float(d, "debug.post_subdiv_noise", np.float32(0.01))
    s.overall_repeats = _get_int(d, "overall_repeats", 1)
    irm = _get(d, "ignore_root_matrix")
    s.ignore_root_matrix = str(irm).strip() in ("true", "1") if irm is not None else False
    if s.qem and not s.projection:
        raise ValueError("Invalid settings: QEM will not be applied if centroid projection is disabled")
    return s


def polygonize(shape_json, mc_json, taps=None):
    """grand_algorithm (mcc2.cpp:309-444): MC, then overall_repeats x [resampling x iters;
    projection (+QEM); subdivision when enabled and (overall_repeats <= 1 or last)].  Subdivision
    noise draws from this process's glibc rand() (call srand() first for a fixed sequence)."""
    s = parse_mc_settings(mc_json)
    tree = mp5_to_nodes(shape_json, s.ignore_root_matrix)
    v, f = marching_cubes(tree, s.resolution, s.box)
    if taps is not None:
        taps["mc_verts"] = v.copy()
    for rep in range(s.overall_repeats):
        for _ in range(s.vresampl_iters):
            v, _c = vertex_resampling(tree, v, f, s.vresampl_c)
        if s.projection:
            v, cen, _avg = centroids_projection(tree, v, f, s.qem)
            if taps is not None:
                taps.setdefault("post_p_centroids", []).append(cen)
        if s.subdiv and (s.overall_repeats <= 1 or rep == s.overall_repeats - 1):
            # polygonize_step_3 (polygonizer_algorithm_ob02.hpp:119-157): REAL actual_noise =
            # is_last ? post_subdiv_noise * 10.0f : 0
            is_last = rep == s.overall_repeats - 1
            noise = np.float32(s.post_subdiv_noise * np.float32(10.0)) if is_last else np.float32(0)
            v, f = subdivide(v, f, noise)
    return v, f
