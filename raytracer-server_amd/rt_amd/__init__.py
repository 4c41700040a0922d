"""Python mirror of the reference's render interface over the C ABI (include/rt_ffi.h).

Reference interface it mirrors (SuneelFreimuth/raytracer-server):
  Scene.from_toml(path)                    <- Scene::from_toml            src/scene.rs:143-150
  sample_pixel(x, y, w, h, spp, scene)     <- sample_pixel + gamma        src/server.rs:320-368
  RenderJob(...).run(scene, w, h, spp)     <- RenderJob::run              src/server.rs:157-199
                                              (same 6-byte header + RGB8 chunk messages)
  Scene.trace_ray(origins, dirs)           <- Scene::trace_ray            src/scene.rs:272-289

Everything computes on the GPU through lib/librtamd.so; there is no CPU fallback. Importing this
module without the built library raises ImportError.
"""
import ctypes
import os
import struct

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_AMD_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "librtamd.so")

RT_OK = 0
RT_CANCELLED = 1
FLAG_MIS = 1 << 0
FLAG_MEGAKERNEL = 1 << 1
FLAG_FP32 = 1 << 2
FLAG_MESH_NEAREST = 1 << 3  # Mesh::intersect without the octree (geometry.rs:886-903), BVH on the device

BRDF_DIFFUSE, BRDF_SPECULAR, BRDF_PHONG = 0, 1, 2
GEOM_SPHERE, GEOM_PLANE, GEOM_MESH = 0, 1, 2

_D3 = ctypes.c_double * 3


class RenderParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("x0", ctypes.c_int32),
                ("y0", ctypes.c_int32), ("tile_w", ctypes.c_int32), ("tile_h", ctypes.c_int32),
                ("spp", ctypes.c_int32), ("seed", ctypes.c_uint64), ("flags", ctypes.c_uint32),
                ("device", ctypes.c_int32), ("row_step", ctypes.c_int32)]


class RenderStats(ctypes.Structure):
    _fields_ = [("samples", ctypes.c_int64), ("vertices", ctypes.c_int64), ("iterations", ctypes.c_int64),
                ("device_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double * 8),
                ("kernel_launches", ctypes.c_int64 * 8)]

    def as_dict(self):
        return dict(samples=self.samples, vertices=self.vertices, iterations=self.iterations,
                    device_ms=self.device_ms, kernel_ms=list(self.kernel_ms),
                    kernel_launches=list(self.kernel_launches))


class ObjectDesc(ctypes.Structure):
    _fields_ = [("emitted", _D3), ("brdf_kind", ctypes.c_int32), ("k", _D3), ("phong_kd", ctypes.c_double),
                ("phong_ks", ctypes.c_double), ("phong_power", ctypes.c_int32), ("color_d", _D3),
                ("color_s", _D3), ("geom_kind", ctypes.c_int32), ("pos", _D3), ("r", ctypes.c_double),
                ("n", _D3), ("mesh", ctypes.c_int32)]


class MeshDesc(ctypes.Structure):
    _fields_ = [("n_vertices", ctypes.c_uint32), ("vertices", ctypes.POINTER(ctypes.c_double)),
                ("n_triangles", ctypes.c_uint32), ("indices", ctypes.POINTER(ctypes.c_uint32)),
                ("bbox_min", _D3), ("bbox_max", _D3), ("surface_area", ctypes.c_double)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("cam_pos", _D3), ("cam_dir", _D3), ("n_objects", ctypes.c_uint32),
                ("objects", ctypes.POINTER(ObjectDesc)), ("n_meshes", ctypes.c_uint32),
                ("meshes", ctypes.POINTER(MeshDesc))]


_EXPORTS = ["rt_scene_load_toml", "rt_scene_create", "rt_scene_destroy", "rt_scene_info", "rt_scene_mesh",
            "rt_render", "rt_render_device", "rt_render_multi", "rt_band_plan", "rt_trace_rays", "rt_trace_rays_flags", "rt_last_error", "rt_abi_version",
            "rt_device_count"]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"rt_amd: native library not built: {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    L.rt_scene_load_toml.argtypes = [ctypes.c_char_p, ctypes.c_char_p, P(vp)]
    L.rt_scene_create.argtypes = [P(SceneDesc), P(vp)]
    L.rt_scene_destroy.argtypes = [vp]
    L.rt_scene_destroy.restype = None
    L.rt_scene_info.argtypes = [vp, P(ctypes.c_int64)]
    L.rt_scene_mesh.argtypes = [vp, ctypes.c_int32, P(ctypes.c_int64), P(ctypes.c_double), P(ctypes.c_double),
                                P(ctypes.c_double), P(ctypes.c_uint32), P(ctypes.c_int32), P(ctypes.c_int32),
                                P(ctypes.c_int32), P(ctypes.c_int32), P(ctypes.c_int32)]
    L.rt_render.argtypes = [vp, P(RenderParams), P(ctypes.c_uint8), P(ctypes.c_double), P(ctypes.c_int32),
                            P(RenderStats)]
    L.rt_render_device.argtypes = [vp, P(RenderParams), vp, vp, vp, P(RenderStats)]
    L.rt_render_multi.argtypes = [vp, P(RenderParams), P(ctypes.c_int32), ctypes.c_int32, ctypes.c_int32,
                                  P(ctypes.c_uint8), P(ctypes.c_int32), P(RenderStats)]
    L.rt_band_plan.restype = ctypes.c_int32
    L.rt_band_plan.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P(ctypes.c_int32),
                               P(ctypes.c_int32)]
    L.rt_trace_rays.argtypes = [vp, ctypes.c_int32, ctypes.c_int64, P(ctypes.c_double), P(ctypes.c_double),
                                P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_double), P(ctypes.c_double)]
    L.rt_trace_rays_flags.argtypes = [vp, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64, P(ctypes.c_double),
                                      P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_int32), P(ctypes.c_double),
                                      P(ctypes.c_double)]
    L.rt_last_error.restype = ctypes.c_char_p
    L.rt_last_error.argtypes = []
    L.rt_abi_version.argtypes = []
    L.rt_device_count.argtypes = []
    # diagnostics (include/rt_diag.h)
    if hasattr(L, "rt_selftest_arith"):  # absent from libraries built before it existed (A/B variants)
        L.rt_selftest_arith.argtypes = [ctypes.c_long, ctypes.c_ulonglong, P(ctypes.c_ulonglong)]
    if hasattr(L, "rt_selftest_arith_n"):
        L.rt_selftest_arith_n.argtypes = [ctypes.c_long, ctypes.c_ulonglong, P(ctypes.c_ulonglong), ctypes.c_int]
    if hasattr(L, "rt_selftest_tables"):
        L.rt_selftest_tables.argtypes = [P(ctypes.c_ulonglong), ctypes.c_int, P(ctypes.c_ulonglong)]
    if hasattr(L, "rt_debug_qcheck"):
        L.rt_debug_qcheck.argtypes = [P(ctypes.c_ulonglong)]
    if hasattr(L, "rt_debug_counters"):
        L.rt_debug_counters.argtypes = [P(ctypes.c_ulonglong)]
    if hasattr(L, "rt_debug_regions"):
        L.rt_debug_regions.argtypes = [P(ctypes.c_ulonglong)]
    if hasattr(L, "rt_debug_wave_times"):
        L.rt_debug_wave_times.argtypes = [P(ctypes.c_ulonglong), ctypes.c_int]
    if hasattr(L, "rt_debug_last_split"):
        L.rt_debug_last_split.argtypes = [P(ctypes.c_longlong)]
    return L


lib = _load()


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rt error {code}: {msg}")
        self.code = code


def _check(rc):
    if rc < 0:
        raise RtError(rc, lib.rt_last_error().decode(errors="replace"))
    return rc


def _ptr(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct)) if a is not None else None


class Scene:
    """Immutable scene (SceneSpec::to_scene, scene.rs:357). Share it freely across renders."""

    def __init__(self, handle):
        self._h = ctypes.c_void_p(handle)

    @classmethod
    def from_toml(cls, path, assets_dir=None):
        h = ctypes.c_void_p()
        _check(lib.rt_scene_load_toml(os.fsencode(path), os.fsencode(assets_dir) if assets_dir else None,
                                      ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def from_desc(cls, cam_pos, cam_dir, objects, meshes=()):
        """objects: list of dicts with ObjectDesc field names; meshes: list of dicts with keys
        vertices (n,3), indices (m,3), bbox_min, bbox_max, surface_area."""
        keep = []
        od = (ObjectDesc * max(1, len(objects)))()
        for i, o in enumerate(objects):
            for k, v in o.items():
                f = getattr(od[i], k)
                if isinstance(f, ctypes.Array):
                    for j, x in enumerate(v):
                        f[j] = x
                else:
                    setattr(od[i], k, v)
        md = (MeshDesc * max(1, len(meshes)))()
        for i, m in enumerate(meshes):
            v = np.ascontiguousarray(m["vertices"], dtype=np.float64)
            ix = np.ascontiguousarray(m["indices"], dtype=np.uint32)
            keep += [v, ix]
            md[i].n_vertices = v.shape[0]
            md[i].vertices = _ptr(v, ctypes.c_double)
            md[i].n_triangles = ix.shape[0]
            md[i].indices = _ptr(ix, ctypes.c_uint32)
            for j in range(3):
                md[i].bbox_min[j] = m["bbox_min"][j]
                md[i].bbox_max[j] = m["bbox_max"][j]
            md[i].surface_area = m["surface_area"]
        d = SceneDesc()
        for j in range(3):
            d.cam_pos[j] = cam_pos[j]
            d.cam_dir[j] = cam_dir[j]
        d.n_objects = len(objects)
        d.objects = od
        d.n_meshes = len(meshes)
        d.meshes = md
        h = ctypes.c_void_p()
        _check(lib.rt_scene_create(ctypes.byref(d), ctypes.byref(h)))
        return cls(h.value)

    def close(self):
        if self._h and self._h.value:
            lib.rt_scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def info(self):
        a = np.zeros(16, dtype=np.int64)
        _check(lib.rt_scene_info(self._h, _ptr(a, ctypes.c_int64)))
        keys = ["objects", "light", "meshes", "nodes", "parents", "leaves", "refs", "triangles", "vertices",
                "max_leaf", "max_depth", "slot_tables"]
        return {k: int(a[i]) for i, k in enumerate(keys)}

    def mesh(self, obj):
        counts = np.zeros(4, dtype=np.int64)
        bbox = np.zeros(6)
        sa = ctypes.c_double()
        _check(lib.rt_scene_mesh(self._h, obj, _ptr(counts, ctypes.c_int64), _ptr(bbox, ctypes.c_double),
                                 ctypes.byref(sa), None, None, None, None, None, None, None))
        nn, nr, nt, nv = (int(x) for x in counts)
        verts = np.zeros((nv, 3))
        idx = np.zeros((nt, 3), dtype=np.uint32)
        kind = np.zeros(nn, dtype=np.int32)
        child = np.zeros((nn, 8), dtype=np.int32)
        off = np.zeros(nn, dtype=np.int32)
        cnt = np.zeros(nn, dtype=np.int32)
        refs = np.zeros(max(1, nr), dtype=np.int32)
        I = ctypes.c_int32
        _check(lib.rt_scene_mesh(self._h, obj, None, None, None, _ptr(verts, ctypes.c_double),
                                 _ptr(idx, ctypes.c_uint32), _ptr(kind, I), _ptr(child, I), _ptr(off, I),
                                 _ptr(cnt, I), _ptr(refs, I)))
        return dict(bbox=bbox, surface_area=sa.value, vertices=verts, indices=idx, kind=kind, child=child,
                    leaf_off=off, leaf_cnt=cnt, refs=refs[:nr])

    def trace_ray(self, origins, dirs, device=0, mesh_nearest=False):
        o = np.ascontiguousarray(origins, dtype=np.float64).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, dtype=np.float64).reshape(-1, 3)
        n = o.shape[0]
        t = np.zeros(n)
        ids = np.zeros(n, dtype=np.int32)
        pos = np.zeros((n, 3))
        nrm = np.zeros((n, 3))
        D = ctypes.c_double
        _check(lib.rt_trace_rays_flags(self._h, device, FLAG_MESH_NEAREST if mesh_nearest else 0, n, _ptr(o, D),
                                       _ptr(d, D), _ptr(t, D), _ptr(ids, ctypes.c_int32), _ptr(pos, D), _ptr(nrm, D)))
        return t, ids, pos, nrm


def make_params(width, height, spp, seed=0x5EED, tile=None, flags=0, device=0, row_step=1):
    """tile = (x0, y0, tile_w, tile_h); with row_step k > 1, tile row i is screen row y0 + i*k."""
    x0, y0, tw, th = tile if tile is not None else (0, 0, width, height)
    return RenderParams(width, height, x0, y0, tw, th, spp, seed, flags, device, row_step)


def render(scene, width, height, spp, seed=0x5EED, tile=None, mis=False, megakernel=False, device=0,
           want_sub=False, cancel=None, row_step=1, mesh_nearest=False, fp32=False):
    """Renders a tile to host memory. Returns (rgb[th, tw, 3] u8, sub[th, tw, 4, 3] f64 or None, stats).
    mesh_nearest: Mesh::intersect's `octree: None` semantics (RT_FLAG_MESH_NEAREST, megakernel only).
    fp32: the f32 perf mode (RT_FLAG_FP32: statistical parity only; meshes with nearest-triangle semantics)."""
    flags = (FLAG_MIS if mis else 0) | (FLAG_MEGAKERNEL if megakernel else 0) | (FLAG_MESH_NEAREST if mesh_nearest else 0)
    flags |= FLAG_FP32 if fp32 else 0
    p = make_params(width, height, spp, seed, tile, flags, device, row_step)
    rgb = np.zeros((p.tile_h, p.tile_w, 3), dtype=np.uint8)
    sub = np.zeros((p.tile_h, p.tile_w, 4, 3), dtype=np.float64) if want_sub else None
    st = RenderStats()
    cflag = cancel if cancel is not None else None
    rc = _check(lib.rt_render(scene.handle, ctypes.byref(p), _ptr(rgb, ctypes.c_uint8), _ptr(sub, ctypes.c_double),
                              ctypes.byref(cflag) if cflag is not None else None, ctypes.byref(st)))
    out = st.as_dict()
    out["cancelled"] = rc == RT_CANCELLED
    return rgb, sub, out


def render_device(scene, params, d_rgb, d_sub=None, stream=None, stats=False):
    """Enqueues a render into device buffers (raw device pointers as ints) on a HIP stream handle."""
    st = RenderStats() if stats else None
    _check(lib.rt_render_device(scene.handle, ctypes.byref(params), ctypes.c_void_p(d_rgb),
                                ctypes.c_void_p(d_sub) if d_sub else None,
                                ctypes.c_void_p(stream) if stream else None,
                                ctypes.byref(st) if st is not None else None))
    return st.as_dict() if st is not None else None


def render_multi(scene, width, height, spp, devices, seed=0x5EED, tile=None, mis=False, band_rows=0, cancel=None,
                 row_step=1, fp32=False, mesh_nearest=False):
    """rt_render_multi: one worker thread per entry of `devices` (ordinals may repeat), bands of rows
    handed out dynamically, RGB8 gathered on the host. Returns (rgb[th, tw, 3] u8, stats)."""
    flags = FLAG_MEGAKERNEL | (FLAG_MIS if mis else 0) | (FLAG_FP32 if fp32 else 0) | \
        (FLAG_MESH_NEAREST if mesh_nearest else 0)
    p = make_params(width, height, spp, seed, tile, flags, devices[0], row_step)
    rgb = np.zeros((p.tile_h, p.tile_w, 3), dtype=np.uint8)
    devs = (ctypes.c_int32 * len(devices))(*devices)
    st = RenderStats()
    rc = _check(lib.rt_render_multi(scene.handle, ctypes.byref(p), devs, len(devices), band_rows,
                                    _ptr(rgb, ctypes.c_uint8), ctypes.byref(cancel) if cancel is not None else None,
                                    ctypes.byref(st)))
    out = st.as_dict()
    out["cancelled"] = rc == RT_CANCELLED
    return rgb, out


def band_plan(tile_h, n_workers, band_rows=0):
    """The band plan rt_render_multi hands out: (first tile row, rows) per band, in handout order."""
    n = lib.rt_band_plan(tile_h, n_workers, band_rows, 0, None, None)
    first = np.zeros(max(1, n), dtype=np.int32)
    rows = np.zeros(max(1, n), dtype=np.int32)
    lib.rt_band_plan(tile_h, n_workers, band_rows, n, _ptr(first, ctypes.c_int32), _ptr(rows, ctypes.c_int32))
    return first[:n].tolist(), rows[:n].tolist()


def sample_pixel(x, y, width, height, samples_per_pixel, scene, seed=0x5EED, mis=False):
    """server.rs:320-368 for one pixel: returns the gamma-corrected RGB8 triple of pixel (x, y) where
    y counts from the BOTTOM as in the reference (RenderJob::run passes height - row - 1)."""
    row = height - y - 1
    rgb, _, _ = render(scene, width, height, samples_per_pixel, seed, tile=(x, row, 1, 1), mis=mis)
    return tuple(int(c) for c in rgb[0, 0])


PIXELS_PER_MSG = 60  # server.rs:145


def chunk_messages(rgb, x0=0, y0=0):
    """Packs a rendered tile into the reference's binary messages (server.rs:173-190):
    [u8 type=0][u8 n][u16le x][u16le y][n x RGB8], rows top-first, 60-pixel windows."""
    th, tw, _ = rgb.shape
    for r in range(th):
        for x in range(0, tw, PIXELS_PER_MSG):
            n = min(PIXELS_PER_MSG, tw - x)
            yield struct.pack("<BBHH", 0, n, x0 + x, y0 + r) + rgb[r, x:x + n].tobytes()


class RenderJob:
    """RenderJob::run (server.rs:157-199) on the GPU: renders the frame, then yields the chunk
    messages the WebSocket server sends. `stop()` cancels between bounce iterations."""

    def __init__(self, device=0, seed=0x5EED):
        self.device = device
        self.seed = seed
        self._cancel = ctypes.c_int32(0)

    def stop(self):
        self._cancel.value = 1

    def run(self, scene, width, height, spp, mis=False):
        self._cancel.value = 0
        rgb, _, st = render(scene, width, height, spp, self.seed, mis=mis, device=self.device, cancel=self._cancel)
        if st["cancelled"]:
            return []
        return list(chunk_messages(rgb))


def selftest_arith(n=1 << 24, seed=0x5EED):
    """Device check of the exact-arithmetic shortcuts: (reciprocal, quotient, square-root mismatches)."""
    out = (ctypes.c_ulonglong * 3)()
    _check(lib.rt_selftest_arith_n(n, seed, out, 3))
    return int(out[0]), int(out[1]), int(out[2])


def selftest_tables(ptrs):
    """Device round trips of the per-call pointer views (include/rt_diag.h rt_selftest_tables): per address
    p, (tables() via the kernarg view, tables() of the by-value argument, the round-4 sign-extending form,
    kernarg ctab, kernarg node_slot [= p + 16], kernarg RenderArgs.tail_buf [= p + 32])."""
    n = len(ptrs)
    inp = (ctypes.c_ulonglong * n)(*ptrs)
    out = (ctypes.c_ulonglong * (6 * n))()
    _check(lib.rt_selftest_tables(inp, n, out))
    return [tuple(int(out[6 * i + k]) for k in range(6)) for i in range(n)]


def debug_qcheck():
    """RT_QCHECK builds: LDS hand-off protocol violation counters since the last call (4 ints), or
    None when the loaded library was built without the checks."""
    out = (ctypes.c_ulonglong * 4)()
    rc = lib.rt_debug_qcheck(out)
    if rc < 0:
        raise RtError(rc, "rt_debug_qcheck")
    return None if rc == 1 else [int(v) for v in out]


def debug_last_split():
    """The split tail of this thread's last f64 megakernel render (rt_diag.h rt_debug_last_split):
    dict(split=subpixels handed out as sample chunks, want=the kernel family's split before the scratch
    buffer capped it, chunk=samples per chunk)."""
    out = (ctypes.c_longlong * 3)()
    _check(lib.rt_debug_last_split(out))
    return dict(split=int(out[0]), want=int(out[1]), chunk=int(out[2]))


def device_count():
    return lib.rt_device_count()
