"""Synthetic MP5 scenes and mc-settings for the BASELINE.json configurations.

All matrices are 12-entry row-major scale + translate with power-of-two scales and translations in
(1/64)Z, so the reference's float LU inverse (basic_functions.hpp:77-128) is exact whatever its
internals.  Rabbit ("cube") leaves are placed so every table read of the box stays in the table's
safe band (cube.hpp:222-250 reads foo[idx+1] past a row in the last band, F8d).
"""
import json
import random

EYE = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]

# rabbit table extent (cube.hpp:65-72): local coordinates must stay below origin + (size-1)*0.75
_RABBIT_SAFE_HI = (-10.2189 + 21 * 0.75, -6.6299 + 17 * 0.75, -2.5487 + 21 * 0.75)
_RABBIT_LO = (-10.2189, -6.6299, -2.5487)


def st(scale, tx, ty, tz):
    return [scale, 0, 0, tx, 0, scale, 0, ty, 0, 0, scale, tz]


def mc_settings(resolution, box=1.0, *, vresampl_iters=0, vresampl_c=1.0, projection=0, qem=0,
                overall_repeats=1, subdiv=0, post_subdiv_noise=0):
    return {
        "box": {"xmin": -box, "xmax": box, "ymin": -box, "ymax": box, "zmin": -box, "zmax": box},
        "resolution": resolution,
        "vresampl": {"iters": vresampl_iters, "c": vresampl_c},
        "projection": {"enabled": projection},
        "qem": {"enabled": qem},
        "subdiv": {"enabled": subdiv},
        "overall_repeats": overall_repeats,
        "debug": {"post_subdiv_noise": post_subdiv_noise},
    }


# configuration 1: single sphere (iellipsoid r = 0.5), box +-0.6, 32^3, MC only
def config1():
    return {"type": "iellipsoid", "matrix": list(EYE)}, mc_settings(32, 0.6)


# configuration 2: Union(sphere, rabbit cube), box +-1, 128^3, MC + 3 OB02 iterations
def union_sphere_cube():
    return {"type": "Union", "matrix": list(EYE), "children": [
        {"type": "iellipsoid", "matrix": st(1, -0.375, -0.25, 0.25)},
        {"type": "cube", "matrix": st(0.125, 0.5, 0.375, -0.5)},
    ]}


def config2(resolution=128):
    return union_sphere_cube(), mc_settings(resolution, 1.0, vresampl_iters=1, vresampl_c=0.4, projection=1, qem=1,
                                            overall_repeats=3)


LEAF_TYPES = ["iellipsoid", "icylinder", "icone", "itorus", "implicit_double_mushroom", "iheart", "cube"]


def _rabbit_ok(s, t, box):
    for a in range(3):
        hi = (box + 0.1 - t[a]) / s
        lo = (-box - 0.1 - t[a]) / s
        if hi >= _RABBIT_SAFE_HI[a] - 1e-3:
            return False
        del lo
    return True


TWIST_LEAF_TYPES = LEAF_TYPES + ["screw"]


def twist(scale, tx, ty, tz, pitch=0.5, delta_ratio=1.5):
    """The reference's "screw" node (object_factory.hpp:304-351): a sine-profile twisted rod of
    radius 1/2 cut to |z| <= 1/2 by top_bottom_lid, under the given scale + translation."""
    return {"type": "screw", "matrix": st(scale, tx, ty, tz), "v": [0, 2, 0], "pitch": pitch, "profile": "sin",
            "delta_ratio": delta_ratio, "end_type": "0"}


def tetrahedron(scale=1.0, t=(0, 0, 0)):
    """tetrahedron.hpp: corners moved by the node matrix."""
    return {"type": "tetrahedron", "matrix": st(scale, *t),
            "corners": [[-0.5, -0.375, -0.25], [0.5, -0.25, -0.375], [0, 0.5, -0.25], [0.125, 0, 0.5]]}


def meta_balls(scale=1.0, t=(0, 0, 0), time=0.1):
    """meta_balls_Rydgard.hpp: 4 moving blobs at `time`."""
    return {"type": "meta_balls", "matrix": st(scale, *t), "time": time}


def extrusion(size=6, scale=1.0, t=(0, 0, 0)):
    """extrusion.hpp: a regular size-gon prism of radius 1/2, cut to |z| <= 1/2."""
    return {"type": "extrusion", "matrix": st(scale, *t), "size": size}


def random_leaf(rng, box=1.0, types=LEAF_TYPES):
    while True:
        t = rng.choice(types)
        if t == "screw":
            s = rng.choice([0.25, 0.5])
            tr = [rng.randint(-32, 32) / 64.0 for _ in range(3)]
            return twist(s, *tr, pitch=rng.choice([0.25, 0.5]))
        s = rng.choice([0.125, 0.25, 0.5])
        tr = [rng.randint(-32, 32) / 64.0 for _ in range(3)]
        if t == "torus" or t == "itorus":
            # torus.hpp: r = 4, rx = 0.2 -> radius 0.8 in local units; keep it inside the box
            s = rng.choice([0.125, 0.25])
        if t == "iheart":
            s = rng.choice([0.25, 0.5])
        if t == "cube":
            # the rabbit SDF table spans ~16.5 x 13.5 x 16.5 local units: at scale 1/8 it is about
            # the box's size (config 2's rabbit); larger scales enclose the whole box in one solid
            s = 0.125
        if t == "cube" and not _rabbit_ok(s, tr, box):
            continue
        return {"type": t, "matrix": st(s, *tr)}


def _size(node):
    return 1 if "children" not in node else sum(_size(c) for c in node["children"])


def random_tree(seed, n_leaves=10, box=1.0, twist_leaves=False):
    """Random binary CSG tree with n_leaves leaves and n_leaves-1 Union / Difference /
    Intersection nodes.  Subtrees are paired at random from a pool (expected depth O(log n)).
    Difference keeps the larger operand first; Intersection clips with a large ellipsoid leaf so
    the result stays non-empty; the root is a Union.  twist_leaves adds the "screw" node to the
    leaf types and makes the first leaf one."""
    rng = random.Random(seed)
    types = TWIST_LEAF_TYPES if twist_leaves else LEAF_TYPES
    pool = [random_leaf(rng, box, types) for _ in range(n_leaves)]
    if twist_leaves and not any(p["type"] == "screw" for p in pool):
        pool[0] = random_leaf(rng, box, ["screw"])
    while len(pool) > 1:
        i, j = rng.sample(range(len(pool)), 2)
        a, b = pool[i], pool[j]
        rest = [p for k, p in enumerate(pool) if k not in (i, j)]
        r = rng.random()
        op = "Union" if (r < 0.55 or not rest) else ("Difference" if r < 0.85 else "Intersection")
        m = list(EYE) if rng.random() < 0.6 else st(1, *[rng.randint(-4, 4) / 64.0 for _ in range(3)])
        if op == "Difference" and _size(b) > _size(a):
            a, b = b, a
        if op == "Intersection":
            clip = {"type": "iellipsoid", "matrix": st(rng.choice([1.5, 2.0]), *[rng.randint(-8, 8) / 64.0 for _ in range(3)])}
            node = {"type": "Union", "matrix": m, "children": [{"type": "Intersection", "matrix": list(EYE), "children": [a, clip]}, b]}
        else:
            node = {"type": op, "matrix": m, "children": [a, b]}
        pool = rest + [node]
    return pool[0]


CONFIG3_SEED = 20251015


def config3_tree():
    """~20-node MP5 CSG tree with twist / union / difference (BASELINE.json config 3): 10 leaves
    including at least one twist ("screw", 3 reference nodes each) and 9 CSG nodes."""
    return random_tree(CONFIG3_SEED, 10, twist_leaves=True)


def config3(resolution=256):
    return config3_tree(), mc_settings(resolution, 1.0, vresampl_iters=1, vresampl_c=0.4, projection=1,
                                                      qem=1, overall_repeats=3)


def config3_shifted(resolution=256, shift=0.003):
    """Config 3 with its box moved by a non-dyadic offset (every axis [-1 + shift, 1 + shift]).

    On the dyadic box [-1, 1]^3 a double mushroom's singular point lands exactly on a grid sample:
    the zero gradient there makes the reference's NaN normals, the average
    edge length is NaN from the first repeat, make_alpha_list (centroids_projection.cpp:144-194)
    returns an empty list and the projection keeps every centroid.  Shifted, no sample is singular,
    every vertex stays finite, and the alpha search and the bisection run on every face."""
    shape, mc = config3(resolution)
    mc["box"] = {k: v + shift for k, v in mc["box"].items()}
    return shape, mc


def config4(resolution=512):
    """config 3's tree at 512^3, eval + MC (the Z-slab scaling workload)."""
    return config3_tree(), mc_settings(resolution, 1.0)


def config5_objects(n=64, resolution=128):
    out = []
    for k in range(n):
        rng = random.Random(CONFIG3_SEED + k)
        leaves = rng.randint(1, 12)
        shape = random_tree(CONFIG3_SEED + k, leaves) if leaves > 1 else random_leaf(rng)
        out.append((shape, mc_settings(resolution, 1.0)))
    return out


def tree_stats(shape):
    """(nodes, leaves, depth)"""
    if "children" not in shape:
        return 1, 1, 1
    st_ = [tree_stats(c) for c in shape["children"]]
    return 1 + sum(s[0] for s in st_), sum(s[1] for s in st_), 1 + max(s[2] for s in st_)


def dumps(x):
    return json.dumps(x)
