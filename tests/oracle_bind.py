"""ctypes binding for the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module. The
scene TOML is parsed here with `tomli` (the reference parses it with the `toml` crate,
scene.rs:143-150); object construction, transforms, octree build and rendering happen in the
C++ oracle (oracle/oracle.cpp), which restates scene.rs:292-441 / geometry.rs.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.environ.get("RT_ORACLE_LIB") or os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None

_D = ctypes.POINTER(ctypes.c_double)
_I32 = ctypes.POINTER(ctypes.c_int32)
_I64 = ctypes.POINTER(ctypes.c_int64)
_U8 = ctypes.POINTER(ctypes.c_uint8)
_U32 = ctypes.POINTER(ctypes.c_uint32)


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if "RT_ORACLE_LIB" not in os.environ and (not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) <
                                                  os.path.getmtime(os.path.join(ORACLE_DIR, "oracle.cpp"))):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_scene_new.restype = ctypes.c_void_p
        L.orc_scene_new.argtypes = [_D, _D]
        L.orc_scene_free.argtypes = [ctypes.c_void_p]
        L.orc_scene_error.restype = ctypes.c_char_p
        L.orc_scene_error.argtypes = [ctypes.c_void_p]
        L.orc_add_object.restype = ctypes.c_int
        L.orc_add_object.argtypes = [ctypes.c_void_p, _D, ctypes.c_int, _D, _D, _D, _D, ctypes.c_int, _D,
                                     ctypes.c_char_p, ctypes.c_int, _I32, _D]
        L.orc_scene_finalize.restype = ctypes.c_int
        L.orc_scene_finalize.argtypes = [ctypes.c_void_p]
        L.orc_mesh_stats.restype = ctypes.c_int
        L.orc_mesh_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, _I64, _D, _D, _I64, _I64]
        L.orc_mesh_octree.restype = ctypes.c_int64
        L.orc_mesh_octree.argtypes = [ctypes.c_void_p, ctypes.c_int, _I32, _I32, _I32, _I32, _I32]
        L.orc_mesh_vertices.restype = ctypes.c_int
        L.orc_mesh_vertices.argtypes = [ctypes.c_void_p, ctypes.c_int, _D, _I32]
        L.orc_octants.argtypes = [_D, _D, _D]
        L.orc_philox.argtypes = [_U32, _U32, _U32]
        L.orc_draws.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                ctypes.c_int, _D]
        L.orc_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64, _D, _D, _D, _I32, _D, _D]
        L.orc_scene_set_mesh_accel.restype = None
        L.orc_scene_set_mesh_accel.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.orc_render.restype = ctypes.c_int64
        L.orc_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                 ctypes.c_int, _U8, _D, _I64]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(_D)


def _arr(v, n=3):
    a = np.zeros(n, dtype=np.float64)
    if v is not None:
        a[: len(v)] = v
    return a


_TF = {"translate": 0, "scale": 1, "rotate_x": 2, "rotate_y": 3, "rotate_z": 4}


class OracleScene:
    """Scene built by the oracle from a reference scene TOML (scene.rs:357 SceneSpec::to_scene)."""

    def __init__(self, toml_path, assets_dir=None, mesh_nearest=False):
        import tomli

        with open(toml_path, "rb") as f:
            spec = tomli.load(f)
        if assets_dir is None:
            assets_dir = os.path.join(os.path.dirname(os.path.abspath(toml_path)), "assets")
        L = lib()
        cam = spec["camera"]
        self.h = L.orc_scene_new(_dp(_arr(cam["pos"])), _dp(_arr(cam["dir"])))
        self.objects = []
        for o in spec["objects"]:
            b = o["brdf"]
            g = o["geometry"]
            bk = {"diffuse": 0, "specular": 1, "phong": 2}[b["type"]]
            k = _arr(b.get("kd") if bk == 0 else b.get("ks") if bk == 1 else None)
            ph = _arr([b["kd"], b["ks"], b["power"]] if bk == 2 else None)
            cd = _arr(b.get("color_d") if bk == 2 else None)
            cs = _arr(b.get("color_s") if bk == 2 else None)
            gt = g["type"]
            gp = np.zeros(6)
            path = None
            if gt == "sphere":
                gk = 0
                gp[:3] = g["pos"]
                gp[3] = g["r"]
            elif gt == "plane":
                gk = 1
                gp[:3] = g["pos"]
                gp[3:] = g["n"]
            elif gt == "mesh":
                gk = 2
                path = os.path.join(assets_dir, g["path"]).encode()
            elif gt == "cube":
                gk = 3
                gp[:3] = g["pos"]
                gp[3] = g["size"]
            elif gt == "prism":
                gk = 4
                gp[:3] = g["pos"]
                gp[3:] = g["size"]
            else:
                raise ValueError(gt)
            tfs = o.get("transforms", [])
            kinds = np.zeros(max(1, len(tfs)), dtype=np.int32)
            vals = np.zeros(3 * max(1, len(tfs)), dtype=np.float64)
            for i, t in enumerate(tfs):
                (name, val), = t.items()
                kinds[i] = _TF[name]
                if name == "translate":
                    vals[3 * i: 3 * i + 3] = val
                else:
                    vals[3 * i] = val
            em = _arr(o.get("emitted"))
            r = L.orc_add_object(self.h, _dp(em), bk, _dp(k), _dp(ph), _dp(cd), _dp(cs), gk, _dp(gp), path,
                                 len(tfs), kinds.ctypes.data_as(_I32), _dp(vals))
            if r < 0:
                raise RuntimeError(L.orc_scene_error(self.h).decode())
            self.objects.append(gt)
        self.light = L.orc_scene_finalize(self.h)
        if self.light < 0:
            raise RuntimeError(L.orc_scene_error(self.h).decode())
        if mesh_nearest:  # Mesh::intersect's `octree: None` branch (geometry.rs:886-903)
            L.orc_scene_set_mesh_accel(self.h, 0)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_scene_free(self.h)
            self.h = None

    def mesh_stats(self, obj):
        out = np.zeros(6, dtype=np.int64)
        bbox = np.zeros(6)
        sa = ctypes.c_double()
        nt = ctypes.c_int64()
        nv = ctypes.c_int64()
        r = lib().orc_mesh_stats(self.h, obj, out.ctypes.data_as(_I64), _dp(bbox), ctypes.byref(sa),
                                 ctypes.byref(nt), ctypes.byref(nv))
        assert r == 0
        return dict(nodes=int(out[0]), parents=int(out[1]), leaves=int(out[2]), refs=int(out[3]),
                    max_leaf=int(out[4]), max_depth=int(out[5]), bbox=bbox, surface_area=sa.value,
                    n_tris=nt.value, n_verts=nv.value)

    def mesh_octree(self, obj):
        st = self.mesh_stats(obj)
        n = st["nodes"]
        kind = np.zeros(n, dtype=np.int32)
        child = np.zeros(8 * n, dtype=np.int32)
        off = np.zeros(n, dtype=np.int32)
        cnt = np.zeros(n, dtype=np.int32)
        refs = np.zeros(max(1, st["refs"]), dtype=np.int32)
        P = lambda a: a.ctypes.data_as(_I32)
        lib().orc_mesh_octree(self.h, obj, P(kind), P(child), P(off), P(cnt), P(refs))
        return kind, child.reshape(n, 8), off, cnt, refs[: st["refs"]]

    def mesh_vertices(self, obj):
        st = self.mesh_stats(obj)
        v = np.zeros(3 * st["n_verts"])
        idx = np.zeros(3 * st["n_tris"], dtype=np.int32)
        lib().orc_mesh_vertices(self.h, obj, _dp(v), idx.ctypes.data_as(_I32))
        return v.reshape(-1, 3), idx.reshape(-1, 3)

    def trace(self, origins, dirs):
        o = np.ascontiguousarray(origins, dtype=np.float64)
        d = np.ascontiguousarray(dirs, dtype=np.float64)
        n = o.shape[0]
        t = np.zeros(n)
        ids = np.zeros(n, dtype=np.int32)
        pos = np.zeros((n, 3))
        nrm = np.zeros((n, 3))
        lib().orc_trace(self.h, n, _dp(o), _dp(d), _dp(t), ids.ctypes.data_as(_I32), _dp(pos), _dp(nrm))
        return t, ids, pos, nrm

    def render(self, width, height, spp, seed, tile=None, mis=False, threads=None, want_sub=True):
        x0, y0, tw, th = tile if tile is not None else (0, 0, width, height)
        rgb = np.zeros((th, tw, 3), dtype=np.uint8)
        sub = np.zeros((th, tw, 4, 3), dtype=np.float64) if want_sub else None
        casts = ctypes.c_int64()
        nthreads = threads if threads is not None else (os.cpu_count() or 1)
        verts = lib().orc_render(self.h, width, height, x0, y0, tw, th, spp, seed, int(mis), nthreads,
                                 rgb.ctypes.data_as(_U8), _dp(sub) if sub is not None else None,
                                 ctypes.byref(casts))
        return rgb, sub, dict(vertices=int(verts), casts=int(casts.value))


def octants(mn, mx):
    out = np.zeros(48)
    lib().orc_octants(_dp(_arr(mn)), _dp(_arr(mx)), _dp(out))
    return out.reshape(8, 2, 3)


def philox(ctr, key):
    c = np.array(ctr, dtype=np.uint32)
    k = np.array(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    P = lambda a: a.ctypes.data_as(_U32)
    lib().orc_philox(P(c), P(k), P(o))
    return [int(x) for x in o]


def draws(seed, pixel, sample, sub, n=8):
    """First n uniforms of the stream of (pixel, sample, subpixel) — RNG spec v2."""
    out = np.zeros(n)
    lib().orc_draws(seed, pixel, sample, sub, n, _dp(out))
    return out
