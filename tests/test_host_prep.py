"""Product host prep (C++ in librtamd.so, no GPU calls) against the oracle's restatement (CPU only):
scene loading (SceneSpec::to_scene, scene.rs:357-441), OBJ loading, transforms and the octree
(geometry.rs:1145-1216) must be bit-identical; malformed inputs must fail with an error code,
never crash (the reference panics)."""
import os

import numpy as np
import pytest

from conftest import REPO, scene_path


@pytest.mark.parametrize("name", ["cornell_box", "cubes", "flying_unicorn"])
def test_scene_prep_matches_oracle(name, rt, oracle_scenes):
    s = rt.Scene.from_toml(scene_path(name))
    o = oracle_scenes[name]
    info = s.info()
    assert info["objects"] == len(o.objects) and info["light"] == o.light == 8
    for i, kind in enumerate(o.objects):
        if kind not in ("mesh", "cube", "prism"):
            continue
        m = s.mesh(i)
        st = o.mesh_stats(i)
        kind_o, child_o, off_o, cnt_o, refs_o = o.mesh_octree(i)
        verts_o, idx_o = o.mesh_vertices(i)
        assert np.array_equal(m["vertices"], verts_o)  # bitwise: transforms replicated exactly
        assert np.array_equal(m["indices"].astype(np.int64), idx_o.astype(np.int64))
        assert np.array_equal(m["bbox"], st["bbox"]) and m["surface_area"] == st["surface_area"]
        assert np.array_equal(m["kind"], kind_o) and np.array_equal(m["child"], child_o)
        assert np.array_equal(m["leaf_cnt"], cnt_o) and np.array_equal(m["refs"], refs_o)


def test_unicorn_info(rt):
    info = rt.Scene.from_toml(scene_path("flying_unicorn")).info()
    assert (info["nodes"], info["parents"], info["leaves"], info["refs"]) == (47183, 9540, 37643, 187766)
    assert info["max_leaf"] == 12 and info["max_depth"] == 10


def _write(tmp_path, text, name="s.toml"):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


GOOD = """
[camera]
pos = [50, 52, 295.6]   # integers are accepted for f64 fields (serde)
dir = [0.0, -0.042612, -1.0]
[[objects]]
brdf = { type = "diffuse", kd = [0.75, 0.25, 0.25] }
geometry = { type = "plane", pos = [1.0, 0.0, 0.0], n = [-1.0, 0.0, 0.0] }
[[objects]]
emitted = [50.0, 50.0, 50.0]
brdf = { type = "diffuse", kd = [0.0, 0.0, 0.0] }
geometry = { type = "sphere", pos = [50.0, 70.0, 100.0], r = 4.0 }
transforms = [
    { translate = [1, 0, 0] },
    { scale = 2.0 },
]
"""


def test_toml_subset_parses(rt, tmp_path):
    s = rt.Scene.from_toml(_write(tmp_path, GOOD))
    assert s.info()["objects"] == 2 and s.info()["light"] == 1


@pytest.mark.parametrize("text,needle", [
    ("[camera]\npos=[0,0,0]\n", "dir"),
    (GOOD.replace('"diffuse", kd = [0.75', '"velvet", kd = [0.75'), "velvet"),
    (GOOD.replace("[0.0, -0.042612, -1.0]", "[0.0, -1.0]"), "3"),
    (GOOD.replace("{ scale = 2.0 }", "{ shear = 2.0 }"), "shear"),
    (GOOD.replace("emitted = [50.0, 50.0, 50.0]", "emitted = [0.0, 0.0, 0.0]"), "emitting"),
    (GOOD.replace('type = "sphere", pos', 'type = "plane", n = [0,1,0], pos').replace(", r = 4.0", ""), "plane"),
    ("[camera\npos = [1,2,3]\n", "line"),
    (GOOD + "\n[camera]\n", "twice"),
])
def test_toml_errors(rt, tmp_path, text, needle):
    with pytest.raises(rt.RtError) as e:
        rt.Scene.from_toml(_write(tmp_path, text))
    assert needle in str(e.value)


def test_obj_errors(rt, tmp_path):
    (tmp_path / "assets").mkdir()
    base = GOOD + '\n[[objects]]\nbrdf = { type = "diffuse", kd = [1,1,1] }\ngeometry = { type = "mesh", path = "m.obj" }\n'
    p = _write(tmp_path, base)
    with pytest.raises(rt.RtError) as e:
        rt.Scene.from_toml(p)
    assert e.value.code == -4  # RT_E_IO: missing asset
    for bad in ["v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 4\n", "v 0 0 x\n", "v 0 0 0\nf 1//1 1 1\n", "f 1 2\n"]:
        (tmp_path / "assets" / "m.obj").write_text(bad)
        with pytest.raises(rt.RtError):
            rt.Scene.from_toml(p)
    (tmp_path / "assets" / "m.obj").write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf 1/1/1 +2/2/2 3\n")
    s = rt.Scene.from_toml(p)
    m = s.mesh(2)
    assert m["indices"].tolist() == [[0, 1, 2]]


@pytest.mark.parametrize("face,ok", [
    ("f 1/1/1 +2/2/2 3", True),        # usize::from_str accepts one leading '+'
    ("f 1 2 +3", True),
    ("f 1 2 +", False),                # '+' alone
    ("f 1 2 ++3", False),
    ("f 1 2 -3", False),               # no sign for usize
    ("f 1 2 18446744073709551616", False),  # usize::MAX + 1: PosOverflow
    ("f 1 2 3/", False),               # empty part after '/'
    ("f 1 2 3x", False),
])
def test_obj_face_index_parse_product_and_oracle_agree(rt, oracle, tmp_path, face, ok):
    """geometry.rs:698-701 parse_face (Rust `usize::from_str`): the product's OBJ reader and the
    oracle's restatement must accept and reject the same face tokens."""
    (tmp_path / "assets").mkdir()
    base = GOOD + '\n[[objects]]\nbrdf = { type = "diffuse", kd = [1,1,1] }\ngeometry = { type = "mesh", path = "m.obj" }\n'
    p = _write(tmp_path, base)
    (tmp_path / "assets" / "m.obj").write_text(f"v 0 0 0\nv 1 0 0\nv 0 1 0\n{face}\n")
    try:
        s = rt.Scene.from_toml(p)
        prod = s.mesh(2)["indices"].tolist() == [[0, 1, 2]]
    except rt.RtError:
        prod = False
    try:
        oracle.OracleScene(p)
        orc = True
    except RuntimeError:
        orc = False
    assert prod == ok and orc == ok


def test_scene_create_from_desc_matches_toml(rt):
    """rt_scene_create (the host-keeps-its-loader boundary) builds the same octree as the TOML path."""
    t = rt.Scene.from_toml(scene_path("flying_unicorn"))
    m = t.mesh(6)
    objs = []
    import tomli
    spec = tomli.load(open(scene_path("flying_unicorn"), "rb"))
    for o in spec["objects"]:
        g, b = o["geometry"], o["brdf"]
        d = dict(emitted=o.get("emitted", [0, 0, 0]), brdf_kind={"diffuse": 0, "specular": 1}[b["type"]],
                 k=b.get("kd", b.get("ks")))
        if g["type"] == "plane":
            d.update(geom_kind=1, pos=g["pos"], n=g["n"])
        elif g["type"] == "sphere":
            d.update(geom_kind=0, pos=g["pos"], r=g["r"])
        else:
            d.update(geom_kind=2, mesh=0)
        objs.append(d)
    mesh = dict(vertices=m["vertices"], indices=m["indices"], bbox_min=m["bbox"][:3], bbox_max=m["bbox"][3:],
                surface_area=m["surface_area"])
    s = rt.Scene.from_desc(spec["camera"]["pos"], spec["camera"]["dir"], objs, [mesh])
    m2 = s.mesh(6)
    assert np.array_equal(m2["child"], m["child"]) and np.array_equal(m2["refs"], m["refs"])
    assert s.info() == t.info()


def test_bad_desc_rejected(rt):
    with pytest.raises(rt.RtError):
        rt.Scene.from_desc([0, 0, 0], [0, 0, -1], [dict(geom_kind=2, mesh=3, emitted=[1, 1, 1])], [])


def test_root_order_sorting_network():
    """path_f64.h: root_order's 19-comparator network on (key, index) equals the reference's stable
    insertion sort (geometry.rs:1248-1260) — 0-1 principle over all binary keys plus random keys
    with ties. The network is read from the device source."""
    import itertools
    import random
    import re

    src = open(os.path.join(REPO, "raytracer-server_amd", "csrc", "device", "path_f64.h")).read()
    body = re.search(r"constexpr int net\[19\]\[2\] = \{(.*?)\};", src, re.S).group(1)
    net = [tuple(map(int, p)) for p in re.findall(r"\{(\d+), (\d+)\}", body)]
    assert len(net) == 19

    def network(keys):
        a = [(k, i) for i, k in enumerate(keys)]
        for x, y in net:
            if a[x] > a[y]:
                a[x], a[y] = a[y], a[x]
        return [i for _, i in a]

    def insertion(keys):
        order = list(range(8))
        for i in range(1, 8):
            for j in range(i, 0, -1):
                if keys[order[j - 1]] > keys[order[j]]:
                    order[j - 1], order[j] = order[j], order[j - 1]
                else:
                    break
        return order

    for bits in itertools.product([0, 1], repeat=8):
        assert network(list(bits)) == insertion(list(bits))
    rnd = random.Random(5)
    for _ in range(20000):
        keys = [rnd.choice([0.5, 1.0, 2.0, rnd.random()]) for _ in range(8)]
        assert network(keys) == insertion(keys)


EXTRA_ASSET_SCENE = """
[camera]
pos = [50.0, 52.0, 295.6]
dir = [0.0, -0.042612, -1.0]
[[objects]]
brdf = {{ type = "diffuse", kd = [0.75, 0.25, 0.25] }}
geometry = {{ type = "plane", pos = [1.0, 0.0, 0.0], n = [1.0, 0.0, 0.0] }}
[[objects]]
brdf = {{ type = "diffuse", kd = [0.25, 0.25, 0.75] }}
geometry = {{ type = "plane", pos = [99.0, 0.0, 0.0], n = [-1.0, 0.0, 0.0] }}
[[objects]]
brdf = {{ type = "diffuse", kd = [0.75, 0.75, 0.75] }}
geometry = {{ type = "plane", pos = [0.0, 0.0, 0.0], n = [0.0, 1.0, 0.0] }}
[[objects]]
brdf = {{ type = "diffuse", kd = [0.75, 0.75, 0.75] }}
geometry = {{ type = "plane", pos = [0.0, 81.6, 0.0], n = [0.0, -1.0, 0.0] }}
[[objects]]
brdf = {{ type = "diffuse", kd = [0.75, 0.75, 0.75] }}
geometry = {{ type = "plane", pos = [0.0, 0.0, 0.0], n = [0.0, 0.0, 1.0] }}
[[objects]]
brdf = {{ type = "diffuse", kd = [0.8, 0.7, 0.5] }}
geometry = {{ type = "mesh", path = "{asset}" }}
transforms = [
    {{ scale = {scale} }},
    {{ rotate_y = 0.6 }},
    {{ translate = [50.0, {ty}, 70.0] }},
]
[[objects]]
emitted = [50.0, 50.0, 50.0]
brdf = {{ type = "diffuse", kd = [0.0, 0.0, 0.0] }}
geometry = {{ type = "sphere", pos = [50.0, 70.0, 100.0], r = 4.0 }}
"""


def extra_asset_scene(tmp_path, asset):
    """A room around one of the reference's unused assets (scenes/assets/chair.obj, crewmate.obj:
    `v/vt/vn` faces, Blender exports)."""
    scale, ty = {"chair.obj": (30.0, 24.5), "crewmate.obj": (0.25, -73.7)}[asset]
    d = tmp_path / asset.split(".")[0]
    d.mkdir()
    os.symlink(os.path.join(REPO, "scenes", "assets"), d / "assets")
    p = d / "s.toml"
    p.write_text(EXTRA_ASSET_SCENE.format(asset=asset, scale=scale, ty=ty))
    return str(p)


@pytest.mark.parametrize("asset", ["chair.obj", "crewmate.obj"])
def test_extra_assets_prep_matches_oracle(asset, rt, oracle, tmp_path):
    """the reference's other OBJ assets load through the product's host prep
    exactly as through the oracle's restatement of Mesh::load + Octree::build."""
    p = extra_asset_scene(tmp_path, asset)
    s = rt.Scene.from_toml(p)
    o = oracle.OracleScene(p)
    m = s.mesh(5)
    kind_o, child_o, off_o, cnt_o, refs_o = o.mesh_octree(5)
    verts_o, idx_o = o.mesh_vertices(5)
    assert len(idx_o) > 100
    assert np.array_equal(m["vertices"], verts_o)
    assert np.array_equal(m["indices"].astype(np.int64), idx_o.astype(np.int64))
    assert np.array_equal(m["kind"], kind_o) and np.array_equal(m["child"], child_o)
    assert np.array_equal(m["leaf_cnt"], cnt_o) and np.array_equal(m["refs"], refs_o)


def test_root_order_grid_form_matches_insertion_sort():
    """path_f64.h root_order_grid (the visiting order from the 2x2x2 structure of the root octant
    centres, taken only when every consecutive radicand gap exceeds 2^-46 of the largest) restated
    in f64 and checked against the reference's stable insertion sort by mag(centre - origin)
    (geometry.rs:1248-1260) on random origins, origins near the root's mid-planes and near-equal
    deltas: whenever the grid form claims a result, it is the reference's order."""
    import math
    import random

    rnd = random.Random(11)
    lo, hi = [11.657, -2.801, 56.176], [52.06, 59.347, 91.408]  # the unicorn's root box

    def centres(lo, hi):
        mid = [(a + b) / 2.0 for a, b in zip(lo, hi)]
        cs = []
        for i in range(8):
            bmin = [mid[k] if (i >> (2 - k)) & 1 else lo[k] for k in range(3)]
            bmax = [hi[k] if (i >> (2 - k)) & 1 else mid[k] for k in range(3)]
            cs.append([(a + b) / 2.0 for a, b in zip(bmin, bmax)])
        return cs

    def reference(cs, o):
        key = []
        for c in cs:
            dv = [c[0] - o[0], c[1] - o[1], c[2] - o[2]]
            key.append(math.sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]))
        order = list(range(8))
        for i in range(1, 8):
            j = i
            while j > 0 and key[order[j - 1]] > key[order[j]]:
                order[j - 1], order[j] = order[j], order[j - 1]
                j -= 1
        return order

    def grid(cs, o):
        dl, far, nb = [], [], []
        for k in range(3):
            a, b = cs[0][k] - o[k], cs[4 >> k][k] - o[k]
            e0, e1 = a * a, b * b
            nb.append((4 >> k) if e1 < e0 else 0)
            dl.append(abs(e1 - e0))
            far.append(max(e0, e1))
        ax = sorted(range(3), key=lambda k: (dl[k], k))  # the device's 3 compare-swaps are a stable sort
        da, db, dc = (dl[k] for k in ax)
        A, B, C = (4 >> k for k in ax)
        sab = da + db
        gap = min(min(da, db - da), min(dc - db, abs(dc - sab)))
        ok = gap > 2.0 ** -46 * (far[0] + far[1] + far[2])
        N = nb[0] | nb[1] | nb[2]
        x3, x4 = ((N ^ A ^ B), (N ^ C)) if sab < dc else ((N ^ C), (N ^ A ^ B))
        return ok, [N, N ^ A, N ^ B, x3, x4, N ^ A ^ C, N ^ B ^ C, N ^ A ^ B ^ C]

    cs = centres(lo, hi)
    mid = [(a + b) / 2.0 for a, b in zip(lo, hi)]
    claimed = [0, 0, 0, 0]
    for n in range(60000):
        mode = n % 4
        o = [rnd.uniform(lo[k] - 30, hi[k] + 30) for k in range(3)]
        if mode == 1:  # on or next to a mid-plane
            k = rnd.randrange(3)
            o[k] = mid[k] + rnd.choice([0.0, 1e-13, -1e-13, 1e-9, 5e-16])
        elif mode == 2:  # two deltas nearly equal: |o_x - mid_x| ~ |o_y - mid_y| (equal half-extents scaled)
            t = rnd.uniform(0.1, 20)
            o[0], o[1] = mid[0] + t, mid[1] + t * (hi[0] - lo[0]) / (hi[1] - lo[1]) * rnd.choice([1.0, 1 + 1e-14])
        elif mode == 3:  # da + db ~ dc
            o = [mid[k] + rnd.uniform(-3, 3) for k in range(3)]
        ok, order = grid(cs, o)
        if ok:
            claimed[mode] += 1
            assert order == reference(cs, o), (o, order, reference(cs, o))
    assert claimed[0] > 0.999 * 15000 and claimed[3] > 0.99 * 15000  # random origins: the fast form almost always


def _speck_toml(tmp_path, n=64):
    """A mesh far smaller than its own cull padding: n triangles inside a 1e-8 cube at (1e6, 1e6, 1e6), whose
    cull padding is 1e-7 * 1e6 = 0.1 (rt_api.cpp pack_scene)."""
    rng = np.random.default_rng(3)
    lines = []
    for t in range(n):
        for _ in range(3):
            x, y, z = (1e6 + int(k) * 1e-9 for k in rng.integers(0, 10, 3))
            lines.append(f"v {x!r} {y!r} {z!r}")
        lines.append(f"f {3 * t + 1} {3 * t + 2} {3 * t + 3}")
    (tmp_path / "speck.obj").write_text("\n".join(lines) + "\n")
    text = """
[camera]
pos = [50.0, 52.0, 295.6]
dir = [0.0, -0.042612, -1.0]
[[objects]]
brdf = { type = "diffuse", kd = [0.9, 0.9, 0.9] }
geometry = { type = "mesh", path = "speck.obj" }
[[objects]]
emitted = [50.0, 50.0, 50.0]
brdf = { type = "diffuse", kd = [0.0, 0.0, 0.0] }
geometry = { type = "sphere", pos = [50.0, 70.0, 100.0], r = 4.0 }
"""
    return _write(tmp_path, text)


def test_slot_bound_codes_never_clamp_on_reference_meshes(rt, tmp_path):
    """rt_api.cpp make_slot: the walks decode every subtree-bound code as base + q * step (path_f64.h
    tight_lo / tight_hi), which encloses the subtree only if no code was clamped to the 16-bit range, so a
    scene keeps its slot tables only then. The reference meshes keep them (their codes lie in about
    [E / step, 2 E / step]); a mesh smaller than its own cull padding (1e-7 of its coordinates' scale), far
    from the origin, clamps and is walked through the plain child tables (the same result without the
    subtree culls)."""
    for name in ("flying_unicorn", "cubes"):
        assert rt.Scene.from_toml(scene_path(name)).info()["slot_tables"] == 1, name
    speck = rt.Scene.from_toml(_speck_toml(tmp_path), str(tmp_path)).info()
    assert speck["parents"] > 0  # an octree with slot rows to encode
    assert speck["slot_tables"] == 0


def test_tight_padding_commutes_with_max_min():
    """path_f64.h tight_padded_le: the slab test pads the interval ends once, f(max tn) <= g(min tf) with
    f(x) = x - 1e-9|x|, g(x) = x + 1e-9|x| in f64, instead of max f(tn) <= min g(tf) per axis. f and g are
    non-decreasing in IEEE f64 (checked here on adjacent doubles, signed zeros and a spread of magnitudes),
    so they commute with max / min and the two forms decide every test alike (checked on random slabs)."""
    rng = np.random.default_rng(7)
    f = lambda x: x - 1e-9 * np.abs(x)  # noqa: E731
    g = lambda x: x + 1e-9 * np.abs(x)  # noqa: E731
    x = np.concatenate([rng.standard_normal(200000) * 10.0 ** rng.integers(-300, 300, 200000),
                        np.array([0.0, -0.0, 5e-324, -5e-324, 1e308, -1e308])])
    x.sort()
    up = np.nextafter(x, np.inf)
    assert np.all(f(up) >= f(x)) and np.all(g(up) >= g(x))
    tn = rng.standard_normal((100000, 3)) * 10.0 ** rng.integers(-5, 8, (100000, 1))
    tf = tn + np.abs(rng.standard_normal((100000, 3))) * 10.0 ** rng.integers(-12, 3, (100000, 1))
    t0, t1 = np.maximum(0.0, tn.max(axis=1)), tf.min(axis=1)
    per_axis = np.maximum(0.0, f(tn).max(axis=1)) <= np.minimum(np.inf, g(tf).min(axis=1))
    assert np.array_equal(per_axis, f(t0) <= g(t1))
