"""implisolid_amd -- MI355X-native implicit-surface polygoniser (Python host side).

The product is the shared library ``implisolid_amd/lib/libimplisolid_mi355x.so`` (HIP, gfx950),
whose C ABI (``include/implisolid.h``) is a drop-in for ImpliSolid's ``mcc2.cpp`` interface.  This
module binds it with ctypes and mirrors the reference's JavaScript front-end calls for the same
path (``implisolid_main.js``: ``make_geometry`` :201-249, ``query_implicit_values`` :291-333,
``query_a_normal`` :335-368), so Python callers get the reference's behaviour.

There is no CPU fallback: if the library is missing or no GPU is present the calls raise.
"""
import ctypes
import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libimplisolid_mi355x.so")
LIB_PATH = os.environ.get("IMPLISOLID_LIB") or LIB_PATH   # experiments: an alternative build

# every symbol declared in include/implisolid.h
ABI_SYMBOLS = [
    "build_geometry", "build_geometry_u", "get_v_size", "get_f_size", "get_f", "get_v", "finish_geometry",
    "get_f_ptr", "get_v_ptr", "set_object", "unset_object", "set_x", "unset_x", "calculate_implicit_values",
    "get_values_ptr", "get_values_size", "calculate_implicit_gradients", "get_gradients_ptr",
    "get_gradients_size", "get_pointset_ptr", "get_pointset_size", "about", "implisolid_last_error",
    "implisolid_set_error_mode", "implisolid_eval_points", "implisolid_program_info",
    "implisolid_slab_create", "implisolid_slab_destroy", "implisolid_slab_eval", "implisolid_slab_count",
    "implisolid_slab_emit", "implisolid_slab_emit_verts", "implisolid_slab_emit_faces", "implisolid_slab_counters", "implisolid_slab_counts", "implisolid_slab_grid",
    "implisolid_slab_verts", "implisolid_slab_faces", "implisolid_slab_field", "implisolid_slab_set_offsets",
    "implisolid_slab_download", "implisolid_slab_copy_counts", "implisolid_slab_read_field", "implisolid_set_pruning",
    "implisolid_parse_settings", "implisolid_slab_partition", "implisolid_slab_brick_stats",
    "implisolid_slab_set_timing", "implisolid_slab_kernel_times", "implisolid_jit_compile",
    "implisolid_slab_used_jit", "implisolid_set_jit", "implisolid_slab_stats", "implisolid_slab_read_signs",
    "implisolid_srand", "implisolid_rand", "implisolid_rand_skip",
    "implisolid_batch_create", "implisolid_batch_run", "implisolid_batch_info", "implisolid_batch_counts",
    "implisolid_batch_download", "implisolid_batch_destroy",
    "implisolid_slab_create_range", "implisolid_slab_balance", "implisolid_cuts_from_layer_work", "implisolid_set_devices",
    "implisolid_slab_copy_mesh", "implisolid_set_jit_bake", "implisolid_jit_wait", "implisolid_jit_stats",
    "implisolid_set_jit_max_modules", "implisolid_jit_modules",
    "implisolid_set_progress_callback", "implisolid_ob02_profile", "implisolid_last_build_stats",
    "implisolid_jit_compile_points", "implisolid_debug_libm", "implisolid_debug_cos", "implisolid_slab_stats_n",
    "implisolid_slab_kernel_times_each", "implisolid_debug_fold",
    "implisolid_ob02_create", "implisolid_ob02_destroy", "implisolid_ob02_load", "implisolid_ob02_resample",
    "implisolid_ob02_project", "implisolid_ob02_subdivide", "implisolid_ob02_counts", "implisolid_ob02_ranges",
    "implisolid_ob02_get_verts", "implisolid_ob02_set_verts", "implisolid_ob02_download",
    "implisolid_ob02_attach", "implisolid_ob02_stream", "implisolid_ob02_resample_async", "implisolid_ob02_project_async",
    "implisolid_ob02_unpack", "implisolid_ob02_halo",
]

# implisolid_progress_callback (include/implisolid.h): verts, n_verts, faces, n_faces,
# progress_callback_id, shape_id, call_id, user
PROGRESS_CALLBACK = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)

_lib = None


class ImplisolidError(RuntimeError):
    pass


def build(jobs=8):
    """Compile the HIP library in-tree (make -C implisolid_amd)."""
    import subprocess
    subprocess.run(["make", "-s", "-j%d" % jobs, "-C", _HERE], check=True)


def lib():
    """The loaded C ABI.  Raises if the HIP library has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("implisolid_amd: %s is missing -- run implisolid_amd.build() (make -C implisolid_amd)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    c_char_p, c_int, c_bool, c_void_p = ctypes.c_char_p, ctypes.c_int, ctypes.c_bool, ctypes.c_void_p
    fp = ctypes.POINTER(ctypes.c_float)
    ip = ctypes.POINTER(ctypes.c_int32)
    up = ctypes.POINTER(ctypes.c_uint32)
    sig = {
        "build_geometry": ([c_char_p, c_char_p], None),
        "build_geometry_u": ([c_char_p, c_char_p, c_char_p], None),
        "get_v_size": ([], c_int), "get_f_size": ([], c_int),
        "get_f": ([ip, c_int], None), "get_v": ([fp, c_int], None),
        "finish_geometry": ([], None), "get_f_ptr": ([], c_void_p), "get_v_ptr": ([], c_void_p),
        "set_object": ([c_char_p, c_bool], c_int), "unset_object": ([c_int], c_bool),
        "set_x": ([c_void_p, c_int], c_bool), "unset_x": ([], None),
        "calculate_implicit_values": ([], None), "get_values_ptr": ([], c_void_p), "get_values_size": ([], c_int),
        "calculate_implicit_gradients": ([c_bool], None), "get_gradients_ptr": ([], c_void_p),
        "get_gradients_size": ([], c_int), "get_pointset_ptr": ([c_char_p], c_void_p),
        "get_pointset_size": ([c_char_p], c_int), "about": ([], None),
        "implisolid_last_error": ([], c_char_p), "implisolid_set_error_mode": ([c_int], None),
        "implisolid_eval_points": ([fp, ctypes.c_int64, fp, fp], c_int),
        "implisolid_debug_libm": ([c_int, fp, fp, ctypes.c_int64, fp], c_int),
        "implisolid_debug_cos": ([ctypes.POINTER(ctypes.c_double), ctypes.c_int64, ctypes.POINTER(ctypes.c_double)], c_int),
        "implisolid_debug_fold": ([fp, ctypes.c_int64, fp, ctypes.POINTER(ctypes.c_int64)], c_int),
        "implisolid_ob02_create": ([c_char_p, c_char_p], c_void_p),
        "implisolid_ob02_destroy": ([c_void_p], None),
        "implisolid_ob02_load": ([c_void_p, c_void_p, ctypes.c_int64, c_void_p, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_int64], c_int),
        "implisolid_ob02_resample": ([c_void_p], c_int),
        "implisolid_ob02_project": ([c_void_p], c_int),
        "implisolid_ob02_subdivide": ([c_void_p, ctypes.c_float], c_int),
        "implisolid_ob02_counts": ([c_void_p, ctypes.POINTER(ctypes.c_int64)], c_int),
        "implisolid_ob02_ranges": ([c_void_p, ctypes.POINTER(ctypes.c_int64)], c_int),
        "implisolid_ob02_get_verts": ([c_void_p, c_void_p], c_int),
        "implisolid_ob02_set_verts": ([c_void_p, c_void_p], c_int),
        "implisolid_ob02_download": ([c_void_p, fp, ip], c_int),
        "implisolid_ob02_attach": ([c_void_p, c_void_p, ctypes.c_int64, c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int64, c_void_p], c_int),
        "implisolid_ob02_stream": ([c_void_p], c_void_p),
        "implisolid_ob02_resample_async": ([c_void_p], c_int),
        "implisolid_ob02_project_async": ([c_void_p], c_int),
        "implisolid_ob02_unpack": ([c_void_p, c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), c_int, c_int], c_int),
        "implisolid_ob02_halo": ([c_void_p, ctypes.POINTER(ctypes.c_int64)], c_int),
        "implisolid_program_info": ([c_char_p, c_int, ip, fp], c_int),
        "implisolid_slab_create": ([c_char_p, c_char_p, c_int, c_int], c_void_p),
        "implisolid_slab_destroy": ([c_void_p], None),
        "implisolid_slab_eval": ([c_void_p, c_void_p], c_int),
        "implisolid_slab_count": ([c_void_p, c_void_p], c_int),
        "implisolid_slab_emit": ([c_void_p, c_void_p, c_void_p], c_int),
        "implisolid_slab_emit_verts": ([c_void_p, c_void_p], c_int),
        "implisolid_slab_emit_faces": ([c_void_p, c_void_p, c_void_p, c_int, c_void_p], c_int),
        "implisolid_slab_counters": ([c_void_p], c_void_p),
        "implisolid_slab_counts": ([c_void_p, c_void_p, up], c_int),
        "implisolid_slab_grid": ([c_void_p, ip], c_int),
        "implisolid_slab_verts": ([c_void_p], c_void_p),
        "implisolid_slab_faces": ([c_void_p], c_void_p),
        "implisolid_slab_field": ([c_void_p], c_void_p),
        "implisolid_slab_set_offsets": ([c_void_p, ctypes.c_uint32, ctypes.c_uint32], c_int),
        "implisolid_slab_download": ([c_void_p, fp, ip, c_void_p], c_int),
        "implisolid_slab_copy_counts": ([c_void_p, c_void_p, c_void_p], c_int),
        "implisolid_slab_read_field": ([c_void_p, fp, ctypes.c_int64], ctypes.c_int64),
        "implisolid_set_pruning": ([c_int], None),
        "implisolid_parse_settings": ([c_char_p, fp, ip, fp], c_int),
        "implisolid_slab_partition": ([c_int, c_int, c_int, ip], c_int),
        "implisolid_slab_brick_stats": ([c_void_p, ctypes.POINTER(ctypes.c_int64)], c_int),
        "implisolid_slab_set_timing": ([c_void_p, c_int], c_int),
        "implisolid_slab_used_jit": ([c_void_p], c_int),
        "implisolid_slab_stats": ([c_void_p, ctypes.POINTER(ctypes.c_int64)], c_int),
        "implisolid_slab_read_signs": ([c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int64], ctypes.c_int64),
        "implisolid_set_jit": ([c_int], None),
        "implisolid_jit_compile": ([c_char_p, ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double)],
                                   ctypes.c_int64),
        "implisolid_slab_kernel_times": ([c_void_p, fp], c_int),
        "implisolid_slab_kernel_times_each": ([c_void_p, fp], c_int),
        "implisolid_slab_stats_n": ([c_void_p, ctypes.POINTER(ctypes.c_int64), c_int], c_int),
        "implisolid_srand": ([ctypes.c_uint], None),
        "implisolid_rand": ([], c_int),
        "implisolid_rand_skip": ([ctypes.c_uint64], None),
        "implisolid_batch_create": ([ctypes.POINTER(c_char_p), c_int, c_char_p, c_int], c_void_p),
        "implisolid_batch_run": ([c_void_p, c_void_p], c_int),
        "implisolid_batch_info": ([c_void_p, ip, ctypes.POINTER(ctypes.c_double)], c_int),
        "implisolid_batch_counts": ([c_void_p, c_int, up], c_int),
        "implisolid_batch_download": ([c_void_p, c_int, fp, ip], c_int),
        "implisolid_batch_destroy": ([c_void_p], None),
        "implisolid_slab_create_range": ([c_char_p, c_char_p, c_int, c_int], c_void_p),
        "implisolid_slab_balance": ([c_char_p, c_char_p, c_int, ip], c_int),
        "implisolid_cuts_from_layer_work": ([ctypes.POINTER(ctypes.c_int64), c_int, ctypes.c_int64, c_int, c_int, ip], c_int),
        "implisolid_set_devices": ([ip, c_int], c_int),
        "implisolid_slab_copy_mesh": ([c_void_p, c_void_p, c_void_p, ctypes.c_int64, ctypes.c_int64, c_void_p], c_int),
        "implisolid_set_jit_bake": ([c_int], None),
        "implisolid_jit_wait": ([], None),
        "implisolid_jit_stats": ([ip, ctypes.POINTER(ctypes.c_double)], None),
        "implisolid_set_jit_max_modules": ([ctypes.c_int], None),
        "implisolid_jit_modules": ([ip], None),
        "implisolid_set_progress_callback": ([PROGRESS_CALLBACK, c_void_p], None),
        "implisolid_ob02_profile": ([c_int], None),
        "implisolid_jit_compile_points": ([c_char_p, ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double)],
                                          ctypes.c_int64),
        "implisolid_last_build_stats": ([ctypes.POINTER(ctypes.c_double)], c_int),
    }
    for name, (args, res) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            # an older experimental build (IMPLISOLID_LIB, same-box A/B runs) lacks the newest entry
            # points: only its callers fail; the in-tree library exports every one (test_cpu)
            if os.environ.get("IMPLISOLID_LIB"):
                continue
            raise
        f.argtypes = args
        f.restype = res
    L.implisolid_set_error_mode(1)   # Python callers get exceptions instead of abort()
    _lib = L
    return L


def _s(x):
    if isinstance(x, (dict, list)):
        x = json.dumps(x)
    return x.encode() if isinstance(x, str) else x


def _check():
    err = lib().implisolid_last_error()
    if err:
        raise ImplisolidError(err.decode(errors="replace"))


def parse_settings(mc_settings):
    """Host-side mc-settings parse (no GPU): dict of the parsed values; raises on invalid input."""
    L = lib()
    box = (ctypes.c_float * 6)()
    ints = (ctypes.c_int32 * 7)()
    fl = (ctypes.c_float * 2)()
    if L.implisolid_parse_settings(_s(mc_settings), box, ints, fl) != 0:
        raise ImplisolidError(last_error())
    keys = ["resolution", "ignore_root_matrix", "overall_repeats", "vresampl_iters", "projection", "qem", "subdiv"]
    out = {k: int(v) for k, v in zip(keys, ints)}
    out["box"] = [np.float32(b) for b in box]
    out["vresampl_c"] = np.float32(fl[0])
    out["post_subdiv_noise"] = np.float32(fl[1])
    return out


def slab_partition(R, rank, nranks):
    """(z0, z1, halo): the cell layers a rank owns in the Z-slab decomposition."""
    out = (ctypes.c_int32 * 3)()
    if lib().implisolid_slab_partition(int(R), int(rank), int(nranks), out) != 0:
        raise ImplisolidError(last_error())
    return int(out[0]), int(out[1]), int(out[2])


def slab_balance(shape, mc_settings, nranks):
    """Balanced Z-slab cuts [1, ..., R + 3] (nranks + 1 cell-layer boundaries) from one interval
    pass of the whole grid on the current device; rank r owns layers [cuts[r], cuts[r + 1])."""
    out = (ctypes.c_int32 * (int(nranks) + 1))()
    if lib().implisolid_slab_balance(_s(shape), _s(mc_settings), int(nranks), out) != 0:
        raise ImplisolidError(last_error())
    return [int(x) for x in out]


def cuts_from_layer_work(listed, bricks_per_layer, R, nranks):
    """Host only: the balanced cuts from per-sample-layer listed-brick counts (R + 3 layers)."""
    a = np.ascontiguousarray(listed, dtype=np.int64)
    out = (ctypes.c_int32 * (int(nranks) + 1))()
    if lib().implisolid_cuts_from_layer_work(a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), len(a),
                                             int(bricks_per_layer), int(R), int(nranks), out) != 0:
        raise ImplisolidError(last_error())
    return [int(x) for x in out]


def set_devices(ids):
    """The HIP devices build_geometry's marching cubes runs on (balanced Z-slabs, slab r on
    ids[r]; a device may repeat).  None or one device: the current device only."""
    ids = list(ids or [])
    arr = (ctypes.c_int32 * max(1, len(ids)))(*ids)
    if lib().implisolid_set_devices(arr if ids else None, len(ids)) != 0:
        raise ImplisolidError(last_error())


def set_jit(mode):
    """Tree-kernel JIT mode for objects set from now on: False/0 off (interpreter), True/1 sync
    (compile before the first eval), 2 async (the library default: compile in the background, the
    interpreter meanwhile)."""
    lib().implisolid_set_jit(int(mode))


def set_jit_bake(mode):
    """Tree modules with the object's matrices baked in as literals: 0 never (one module per shape),
    1 every object, 2 (default) hot objects -- an object evaluated 4 times by the same engine gets its
    baked module (compiled in the background in async mode).  True / False mean 1 / 0."""
    lib().implisolid_set_jit_bake(int(mode))


def jit_wait():
    """Block until every scheduled tree-kernel compilation has finished."""
    lib().implisolid_jit_wait()


def jit_stats():
    out = (ctypes.c_int32 * 4)()
    secs = ctypes.c_double(0)
    lib().implisolid_jit_stats(out, ctypes.byref(secs))
    mods = (ctypes.c_int32 * 3)()
    lib().implisolid_jit_modules(mods)
    return {"mode": out[0], "bake": int(out[1]), "compiled": out[2], "disk_hits": out[3], "compile_s": secs.value,
            "modules": mods[0], "max_modules": mods[1], "evicted": mods[2]}


def set_jit_max_modules(n):
    """Bound the loaded tree modules (least recently requested unheld ones are unloaded past it)."""
    lib().implisolid_set_jit_max_modules(int(n))


def jit_compile(shape, points=False):
    """Host-only: (code-object bytes, compile seconds, generated source) of the shape's tree kernel
    module (points=True: its point module)."""
    L = lib()
    buf = ctypes.create_string_buffer(1 << 20)
    secs = ctypes.c_double(0)
    fn = L.implisolid_jit_compile_points if points else L.implisolid_jit_compile
    n = fn(_s(shape), buf, len(buf), ctypes.byref(secs))
    if n < 0:
        raise ImplisolidError(last_error())
    return int(n), float(secs.value), buf.value.decode()


def set_pruning(level):
    """Per-brick pruning level of the field evaluation: 0 off, 1 CSG operand pruning (field
    bit-identical), 2 (default) + sign-filled bricks (mesh bit-identical).  True means 2."""
    if level is True:
        level = 2
    lib().implisolid_set_pruning(int(level))


def srand(seed):
    """Seed the library's glibc-compatible rand() (the generator the subdivision noise draws from,
    randomize_verts basic_functions.hpp:551-557).  Host only."""
    lib().implisolid_srand(int(seed) & 0xFFFFFFFF)


def rand():
    return int(lib().implisolid_rand())


def rand_skip(n):
    """Discard n draws of the library's rand() (O(log n) jump-ahead)."""
    lib().implisolid_rand_skip(int(n))


def last_error():
    return lib().implisolid_last_error().decode(errors="replace")


# ---- mesh API (implisolid_main.js make_geometry :201-249) -----------------------------------------
def make_geometry(shape, mc_settings):
    """Polygonise an MP5 shape; returns (verts float32 [V,3], faces int32 [F,3]) host copies."""
    L = lib()
    L.finish_geometry()             # implisolid_main.js:214-217
    _VIEW_GEN[0] += 1   # earlier make_geometry_views arrays are stale from here on
    L.build_geometry(_s(shape), _s(mc_settings))
    _check()
    nv, nf = L.get_v_size(), L.get_f_size()
    v = np.empty((nv, 3), np.float32)
    f = np.empty((nf, 3), np.int32)
    if nv:
        L.get_v(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), nv)
    if nf:
        L.get_f(f.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), nf)
    L.finish_geometry()
    return v, f


_VIEW_GEN = [0]   # build_geometry calls through make_geometry_views: the generation of its views


def make_geometry_views(shape, mc_settings):
    """build_geometry as the reference's front end reads it (implisolid_main.js:227-237): the mesh is
    left in the library's result buffers (pinned host memory) and returned as read-only numpy views
    over get_v_ptr / get_f_ptr -- no copy.  The views are valid until the next build_geometry or
    finish_geometry (a larger next build frees the pinned buffers they point into): keep them with
    copy_geometry_views(v, f), which refuses stale views; views_current(v) tells whether a view
    still holds the last build's mesh."""
    L = lib()
    _VIEW_GEN[0] += 1
    L.finish_geometry()
    L.build_geometry(_s(shape), _s(mc_settings))
    _check()
    nv, nf = L.get_v_size(), L.get_f_size()
    v = np.ctypeslib.as_array(ctypes.cast(L.get_v_ptr(), ctypes.POINTER(ctypes.c_float)), shape=(nv, 3)) if nv \
        else np.zeros((0, 3), np.float32)
    f = np.ctypeslib.as_array(ctypes.cast(L.get_f_ptr(), ctypes.POINTER(ctypes.c_int32)), shape=(nf, 3)) if nf \
        else np.zeros((0, 3), np.int32)
    v, f = v.view(_GeometryView), f.view(_GeometryView)
    for a in (v, f):
        a.flags.writeable = False
        a._gen = _VIEW_GEN[0]
    return v, f


class _GeometryView(np.ndarray):
    """A read-only numpy view into the library's result buffers (make_geometry_views), tagged with the
    build generation that made it."""
    _gen = -1

    def __array_finalize__(self, obj):
        self._gen = getattr(obj, "_gen", -1)


def views_current(a):
    """True while a make_geometry_views array still holds the last build's mesh."""
    return getattr(a, "_gen", -1) == _VIEW_GEN[0]


def copy_geometry_views(v, f):
    """Owned copies of make_geometry_views' arrays; raises if another build has replaced them."""
    if not (views_current(v) and views_current(f)):
        raise ImplisolidError("geometry views are stale: a later build_geometry replaced the mesh they point into")
    return np.array(v, dtype=np.float32, copy=True), np.array(f, dtype=np.int32, copy=True)


def make_geometry_progressive(shape, mc_settings, call_specs=None):
    """build_geometry_u with a progress hook (the reference's worker path, worker_api.js:315-345 and
    send_progress_update :399-416): returns (verts, faces, updates), updates = the intermediate
    meshes the library reported -- after marching cubes, after each repeat's vertex resampling and
    after each centroid projection -- as (verts, faces, progressCallback_id, shape_id, call_id)."""
    L = lib()
    updates = []

    def hook(vp, nv, fp_, nf, pid, sid, cid, user):
        v = np.ctypeslib.as_array(vp, shape=(nv * 3,)).copy().reshape(nv, 3) if nv else np.zeros((0, 3), np.float32)
        f = np.ctypeslib.as_array(fp_, shape=(nf * 3,)).copy().reshape(nf, 3) if nf else np.zeros((0, 3), np.int32)
        updates.append((v, f, int(pid), int(sid), int(cid)))

    cb = PROGRESS_CALLBACK(hook)
    L.finish_geometry()
    L.implisolid_set_progress_callback(cb, None)
    try:
        _VIEW_GEN[0] += 1
        L.build_geometry_u(_s(shape), _s(mc_settings), _s(call_specs if call_specs is not None else {}))
    finally:
        L.implisolid_set_progress_callback(PROGRESS_CALLBACK(), None)
    _check()
    nv, nf = L.get_v_size(), L.get_f_size()
    v = np.empty((nv, 3), np.float32)
    f = np.empty((nf, 3), np.int32)
    if nv:
        L.get_v(v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), nv)
    if nf:
        L.get_f(f.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), nf)
    L.finish_geometry()
    return v, f, updates


OB02_STAGES = ("topology", "resample", "edge_fold", "project", "qem", "subdiv", "fetch")


def ob02_profile(on):
    """Per-stage wall times and evaluation counts of the OB02 steps for following builds (drains
    the stream at every stage boundary: for breakdowns, not for timing whole builds)."""
    lib().implisolid_ob02_profile(1 if on else 0)


def last_build_stats():
    """Diagnostics of the last build_geometry: bisection cap hits, projection evaluations and stage
    times (profiled builds), the last average edge length, faces and vertices."""
    out = (ctypes.c_double * 13)()
    if lib().implisolid_last_build_stats(out) != 0:
        raise ImplisolidError(last_error())
    d = {"bisection_cap_hits": int(out[0]), "projection_evals": int(out[1]), "avg_edge": float(out[2]),
         "faces": int(out[10]), "verts": int(out[11]), "jit_launches": int(out[12])}
    d["stage_ms"] = dict(zip(OB02_STAGES, [float(x) for x in out[3:10]]))
    return d


def get_pointset(name):
    L = lib()
    n = L.get_pointset_size(_s(name))
    p = L.get_pointset_ptr(_s(name))
    if not p or n <= 0:
        return None
    return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), shape=(n * 3,)).copy().reshape(n, 3)


# ---- direct evaluation (implisolid_main.js:291-368) ---------------------------------------------------
class ImplicitService:
    """set_object / set_x / calculate_implicit_values / calculate_implicit_gradients."""

    def __init__(self, shape, ignore_root_matrix=False):
        L = lib()
        self.id = L.set_object(_s(shape), bool(ignore_root_matrix))
        if self.id != 1:
            raise ImplisolidError(last_error() or "set_object failed")

    def close(self):
        if self.id:
            lib().unset_object(self.id)
            self.id = 0

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def eval(self, pts, gradient=False):
        """Any number of points (additive implisolid_eval_points; no 50k limit)."""
        p = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 3)
        f = np.empty(p.shape[0], np.float32)
        g = np.empty((p.shape[0], 3), np.float32) if gradient else None
        fp = ctypes.POINTER(ctypes.c_float)
        rc = lib().implisolid_eval_points(p.ctypes.data_as(fp), p.shape[0], f.ctypes.data_as(fp),
                                          g.ctypes.data_as(fp) if gradient else None)
        if rc != 0:
            raise ImplisolidError(last_error())
        return (f, g) if gradient else f

    def query_implicit_values(self, pts):
        """The reference call sequence set_x / calculate_implicit_values / get_values / unset_x."""
        L = lib()
        p = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 3)
        if not L.set_x(p.ctypes.data_as(ctypes.c_void_p), p.shape[0]):
            raise ImplisolidError(last_error())
        try:
            L.calculate_implicit_values()
            _check()
            n = L.get_values_size()
            ptr = L.get_values_ptr()
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_float)), shape=(n,)).copy() if n else np.zeros(0, np.float32)
        finally:
            L.unset_x()

    def query_normals(self, pts, normalize_and_invert=True):
        L = lib()
        p = np.ascontiguousarray(pts, dtype=np.float32).reshape(-1, 3)
        if not L.set_x(p.ctypes.data_as(ctypes.c_void_p), p.shape[0]):
            raise ImplisolidError(last_error())
        try:
            L.calculate_implicit_gradients(bool(normalize_and_invert))
            _check()
            n = L.get_gradients_size()
            ptr = L.get_gradients_ptr()
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_float)), shape=(n,)).copy().reshape(-1, 3)
        finally:
            L.unset_x()


def debug_libm(which, a, b=None):
    """Diagnostics: the device restatements of glibc sinf (0) / atanf (1) / atan2f (2: atan2f(a, b))."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    bb = np.ascontiguousarray(b, dtype=np.float32) if b is not None else None
    if bb is not None and bb.shape != a.shape:
        raise ValueError("debug_libm: a and b differ in shape")
    out = np.empty_like(a)
    fp = ctypes.POINTER(ctypes.c_float)
    rc = lib().implisolid_debug_libm(int(which), a.ctypes.data_as(fp), bb.ctypes.data_as(fp) if bb is not None else None,
                                     a.size, out.ctypes.data_as(fp))
    if rc != 0:
        raise ImplisolidError(last_error())
    return out


def debug_cos(a):
    """Diagnostics: the device restatement of glibc's double cos (the screw gradient's) on a float64 array."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    dp = ctypes.POINTER(ctypes.c_double)
    rc = lib().implisolid_debug_cos(a.ctypes.data_as(dp), a.size, out.ctypes.data_as(dp))
    if rc != 0:
        raise ImplisolidError(last_error())
    return out


def debug_fold(terms):
    """Diagnostics: the projection's edge-length fold (s = 0; s += e[k], float, in order) on the
    device, as build_geometry computes it; returns (sum, chunks taken from the chunk table)."""
    e = np.ascontiguousarray(terms, dtype=np.float32).reshape(-1)
    out = (ctypes.c_float * 1)()
    tc = ctypes.c_int64(0)
    fp = ctypes.POINTER(ctypes.c_float)
    rc = lib().implisolid_debug_fold(e.ctypes.data_as(fp), e.size, out, ctypes.byref(tc))
    if rc != 0:
        raise ImplisolidError(last_error())
    return np.float32(out[0]), int(tc.value)


def program_info(shape, ignore_root_matrix=False):
    """Host-only: compile an MP5 tree; returns (n_instr, depth, n_mats, inverse matrices [n,12])."""
    L = lib()
    info = (ctypes.c_int32 * 4)()
    mats = np.zeros((256, 12), np.float32)
    rc = L.implisolid_program_info(_s(shape), int(bool(ignore_root_matrix)), info,
                                   mats.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    if rc != 0:
        raise ImplisolidError(last_error())
    return info[0], info[1], info[2], mats[:info[2]].copy()


# ---- device slab pipeline (bench / multi-GPU) -----------------------------------------------------
class Slab:
    """One Z-slab of one object on the current device.  Stream = a hipStream_t handle (int)."""

    def __init__(self, shape, mc_settings, rank=0, nranks=1, cuts=None):
        """cuts: nranks + 1 cell-layer boundaries (slab_balance) -- rank r takes [cuts[r], cuts[r+1]);
        None: the equal-layer split (slab_partition)."""
        if cuts is not None:
            if len(cuts) != nranks + 1:
                raise ImplisolidError("Slab: cuts must hold nranks + 1 boundaries")
            self.h = lib().implisolid_slab_create_range(_s(shape), _s(mc_settings), int(cuts[rank]), int(cuts[rank + 1]))
        else:
            self.h = lib().implisolid_slab_create(_s(shape), _s(mc_settings), int(rank), int(nranks))
        if not self.h:
            raise ImplisolidError(last_error())
        g = (ctypes.c_int32 * 8)()
        lib().implisolid_slab_grid(self.h, g)
        self.R, self.res, self.cz0, self.cz1, self.cz_emit, self.fz0, self.fz1, self.depth = list(g)

    def _rc(self, rc):
        if rc != 0:
            raise ImplisolidError(last_error())

    def eval(self, stream=0):
        self._rc(lib().implisolid_slab_eval(self.h, ctypes.c_void_p(stream)))

    def count(self, stream=0):
        self._rc(lib().implisolid_slab_count(self.h, ctypes.c_void_p(stream)))

    def emit(self, d_offsets=0, stream=0):
        self._rc(lib().implisolid_slab_emit(self.h, ctypes.c_void_p(d_offsets or None), ctypes.c_void_p(stream)))

    def emit_verts(self, stream=0):
        """vertex pass alone (slab-local ids, no offsets needed)"""
        self._rc(lib().implisolid_slab_emit_verts(self.h, ctypes.c_void_p(stream)))

    def emit_faces(self, d_offsets=0, d_gathered=0, rank=0, stream=0):
        """face pass: offsets from device [Voff, Foff], or from every rank's gathered counts"""
        self._rc(lib().implisolid_slab_emit_faces(self.h, ctypes.c_void_p(d_offsets or None),
                                                  ctypes.c_void_p(d_gathered or None), int(rank),
                                                  ctypes.c_void_p(stream)))

    def counters_ptr(self):
        return lib().implisolid_slab_counters(self.h)

    def counts(self, stream=0):
        out = (ctypes.c_uint32 * 3)()
        self._rc(lib().implisolid_slab_counts(self.h, ctypes.c_void_p(stream), out))
        return int(out[0]), int(out[1]), bool(out[2])

    def copy_counts(self, d_dst, stream=0):
        """async: counters [own incl. halo, faces, active, halo] -> device uint32[4] at d_dst"""
        self._rc(lib().implisolid_slab_copy_counts(self.h, ctypes.c_void_p(d_dst), ctypes.c_void_p(stream)))

    def copy_mesh(self, d_verts, d_faces, nv, nf, stream=0):
        """async device-to-device copy of the emitted mesh into caller-owned device buffers"""
        self._rc(lib().implisolid_slab_copy_mesh(self.h, ctypes.c_void_p(d_verts or None), ctypes.c_void_p(d_faces or None),
                                                 int(nv), int(nf), ctypes.c_void_p(stream)))

    def set_offsets(self, voff, foff):
        self._rc(lib().implisolid_slab_set_offsets(self.h, int(voff), int(foff)))

    def download(self, nv, nf, stream=0):
        v = np.empty((nv, 3), np.float32)
        f = np.empty((nf, 3), np.int32)
        self._rc(lib().implisolid_slab_download(self.h, v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                f.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.c_void_p(stream)))
        return v, f

    def run(self, stream=0):
        """eval + count + emit with the host-set offsets; returns (nv, nf) (blocking)."""
        self.eval(stream)
        self.count(stream)
        nv, nf, grew = self.counts(stream)
        self.emit(0, stream)
        nv, nf, of = self.counts(stream)
        if of:
            self.emit(0, stream)
            nv, nf, of = self.counts(stream)
            if of:
                raise ImplisolidError("slab output overflow")
        return nv, nf

    def verts_ptr(self):
        return lib().implisolid_slab_verts(self.h)

    def faces_ptr(self):
        return lib().implisolid_slab_faces(self.h)

    def field_ptr(self):
        return lib().implisolid_slab_field(self.h)

    KERNELS = ("brick_modes", "eval_field", "mc_count", "mc_scan", "mc_verts", "mc_faces")
    # one figure per kernel (Engine::kernel_times_each); names as in the rocprofv3 kernel trace
    EACH_KERNEL = ("impli_coarse_modes", "impli_brick_refine", "k_brick_fill", "impli_eval_bricks", "k_mc_count",
                   "k_unit_scan", "k_mc_cells", "k_mc_faces")

    def set_timing(self, on=True):
        self._rc(lib().implisolid_slab_set_timing(self.h, 1 if on else 0))

    def kernel_times(self):
        """ms per kernel of the last timed eval/count/emit (HIP events on the launch stream)."""
        out = (ctypes.c_float * 6)()
        self._rc(lib().implisolid_slab_kernel_times(self.h, out))
        return dict(zip(self.KERNELS, [float(x) for x in out]))

    def kernel_times_each(self):
        """ms per kernel (coarse, refine and fill split out of the brick pass) of the last timed calls."""
        out = (ctypes.c_float * 8)()
        self._rc(lib().implisolid_slab_kernel_times_each(self.h, out))
        return dict(zip(self.EACH_KERNEL, [float(x) for x in out]))

    def stats(self):
        """After count(): units, non-empty units, owned vertices, triangles, active cells, halo-owned,
        cells, mixed coarse boxes, halo-owned as the vertex pass reads it, unit parts."""
        out = (ctypes.c_int64 * 10)()
        n = lib().implisolid_slab_stats_n(self.h, out, 10)
        self._rc(-1 if n < 0 else 0)
        keys = ["units", "nonempty_units", "own", "tri", "act", "halo_own", "cells", "mixed_coarse_boxes",
                "halo_own_verts_pass", "unit_parts"]
        return dict(zip(keys, [int(x) for x in out]))

    def used_jit(self):
        return bool(lib().implisolid_slab_used_jit(self.h))

    def jit_module(self):
        """The tree kernels of the last eval: "interpreter", "shape" (JIT module per tree shape) or
        "baked" (the object's module with its matrices as literals)."""
        return ("interpreter", "shape", "baked")[lib().implisolid_slab_used_jit(self.h)]

    def brick_stats(self):
        """[bricks, mixed-sign bricks, sign-filled bricks] of the last eval."""
        out = (ctypes.c_int64 * 3)()
        self._rc(lib().implisolid_slab_brick_stats(self.h, out))
        return [int(x) for x in out]

    def read_signs(self):
        """Blocking host copy of the sample signs (1 where value < 0), shape (layers, n, n)."""
        L = lib()
        n = L.implisolid_slab_read_signs(self.h, None, 0)
        _check()
        out = np.empty(n, np.uint8)
        L.implisolid_slab_read_signs(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), n)
        _check()
        n_side = self.R + 3
        return out.reshape(-1, n_side, n_side)

    def read_field(self):
        """Blocking host copy of the stored field samples, shape (layers, n, n)."""
        L = lib()
        n = L.implisolid_slab_read_field(self.h, None, 0)
        _check()
        out = np.empty(n, np.float32)
        L.implisolid_slab_read_field(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n)
        _check()
        n_side = self.R + 3          # samples 1 .. res-2 per axis, the sealed ring included
        return out.reshape(-1, n_side, n_side)

    def close(self):
        if self.h:
            lib().implisolid_slab_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Ob02Shard:
    """The OB02 loop on one Z-slab shard (include/implisolid.h implisolid_ob02_*): load the whole MC
    mesh (device pointers) owning vertices [v0, v1); resample() / project() update the owned
    vertices; get_verts / set_verts move the current vertices to and from a device buffer for the
    exchange between steps (distributed.ob02_sharded drives the loop).  Every call blocks."""

    def __init__(self, shape, mc_settings):
        self.h = lib().implisolid_ob02_create(_s(shape), _s(mc_settings))
        if not self.h:
            raise ImplisolidError(last_error())

    def _rc(self, rc):
        if rc != 0:
            raise ImplisolidError(last_error())

    def load(self, d_verts, nv, d_faces, nf, v0, v1):
        self._rc(lib().implisolid_ob02_load(self.h, ctypes.c_void_p(d_verts), int(nv), ctypes.c_void_p(d_faces), int(nf),
                                            int(v0), int(v1)))

    def resample(self):
        self._rc(lib().implisolid_ob02_resample(self.h))

    def project(self):
        self._rc(lib().implisolid_ob02_project(self.h))

    def subdivide(self, amplitude):
        self._rc(lib().implisolid_ob02_subdivide(self.h, float(amplitude)))

    def counts(self):
        out = (ctypes.c_int64 * 2)()
        self._rc(lib().implisolid_ob02_counts(self.h, out))
        return int(out[0]), int(out[1])

    def ranges(self):
        """[v0, v1) owned vertices, [f0, f1) work faces, [c0, c1) centroid faces"""
        out = (ctypes.c_int64 * 6)()
        self._rc(lib().implisolid_ob02_ranges(self.h, out))
        return tuple(int(x) for x in out)

    # stream-ordered form (implisolid_ob02_attach ...): nothing below blocks the host
    def attach(self, d_verts, nv, d_faces, nf, v0, v1, after_stream=0):
        """The caller's device vertex array becomes the working one (updated in place; keep it alive);
        the handle's stream is ordered after `after_stream` by an event."""
        self._rc(lib().implisolid_ob02_attach(self.h, ctypes.c_void_p(d_verts), int(nv), ctypes.c_void_p(d_faces), int(nf),
                                              int(v0), int(v1), ctypes.c_void_p(after_stream)))

    def stream(self):
        """The handle's HIP stream (an int for torch.cuda.ExternalStream)."""
        return int(lib().implisolid_ob02_stream(self.h) or 0)

    def resample_async(self):
        self._rc(lib().implisolid_ob02_resample_async(self.h))

    def project_async(self):
        self._rc(lib().implisolid_ob02_project_async(self.h))

    def unpack(self, d_rows, row_len, voff, rank):
        """Copy every rank's row but `rank`'s (all-gathered owned ranges, equal rows of row_len floats)
        into the vertex array, on the handle's stream."""
        arr = (ctypes.c_int64 * len(voff))(*[int(x) for x in voff])
        self._rc(lib().implisolid_ob02_unpack(self.h, ctypes.c_void_p(d_rows), int(row_len), arr, len(voff) - 1, int(rank)))

    def halo(self):
        """[h0, h1): the vertices the next resampling reads."""
        out = (ctypes.c_int64 * 2)()
        self._rc(lib().implisolid_ob02_halo(self.h, out))
        return int(out[0]), int(out[1])

    def get_verts(self, d_dst):
        self._rc(lib().implisolid_ob02_get_verts(self.h, ctypes.c_void_p(d_dst)))

    def set_verts(self, d_src):
        self._rc(lib().implisolid_ob02_set_verts(self.h, ctypes.c_void_p(d_src)))

    def download(self):
        nv, nf = self.counts()
        v = np.empty((nv, 3), np.float32)
        f = np.empty((nf, 3), np.int32)
        self._rc(lib().implisolid_ob02_download(self.h, v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                f.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return v, f

    def close(self):
        if self.h:
            lib().implisolid_ob02_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    """A stream of objects polygonised with one mc-settings dict (BASELINE config 5).  n_streams=0:
    merged launches (every stage once for all objects, interpreter kernels); n_streams >= 1: one
    hipGraph per object (JIT tree kernels) replayed over that many streams.  run() is async on
    `stream`; counts()/download() block."""

    def __init__(self, shapes, mc_settings, n_streams=4):
        L = lib()
        enc = [_s(sh) for sh in shapes]
        arr = (ctypes.c_char_p * len(enc))(*enc)
        self.h = L.implisolid_batch_create(arr, len(enc), _s(mc_settings), int(n_streams))
        if not self.h:
            raise ImplisolidError(last_error() or "implisolid_batch_create failed")
        info = (ctypes.c_int32 * 4)()
        secs = ctypes.c_double(0)
        L.implisolid_batch_info(self.h, info, ctypes.byref(secs))
        self.n, self.n_streams, self.graphs, self.jit_seconds = int(info[0]), int(info[1]), bool(info[2]), secs.value
        self.merged = bool(info[3])

    def run(self, stream=None):
        if lib().implisolid_batch_run(self.h, stream) != 0:
            raise ImplisolidError(last_error())

    def counts(self, i):
        out = (ctypes.c_uint32 * 3)()
        if lib().implisolid_batch_counts(self.h, int(i), out) != 0:
            raise ImplisolidError(last_error())
        return int(out[0]), int(out[1]), bool(out[2])

    def download(self, i):
        nv, nf, of = self.counts(i)
        v = np.empty((nv, 3), np.float32)
        f = np.empty((nf, 3), np.int32)
        if lib().implisolid_batch_download(self.h, int(i), v.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                           f.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) != 0:
            raise ImplisolidError(last_error())
        return v, f

    def close(self):
        if self.h:
            lib().implisolid_batch_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
