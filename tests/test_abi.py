"""The C ABI library loads and exports every entry point include/rt_ffi.h declares, and the ctypes
mirror's struct layouts match the header (compiled with gcc). CPU only: no compute calls."""
import ctypes
import os
import re
import subprocess

from conftest import REPO

HEADER = os.path.join(REPO, "include", "rt_ffi.h")


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rt_[a-z_0-9]+)\s*\(", text, re.M)))


def test_exports_every_declared_symbol(rt):
    names = declared()
    assert len(names) >= 11
    for n in names:
        assert hasattr(rt.lib, n), f"missing export {n}"
    assert rt.lib.rt_abi_version() == 3


def test_exports_diagnostics(rt):
    text = open(os.path.join(REPO, "include", "rt_diag.h")).read()
    names = re.findall(r"^int\s+(rt_[a-z_0-9]+)\s*\(", text, re.M)
    assert names == ["rt_selftest_arith_n", "rt_selftest_arith", "rt_selftest_tables", "rt_debug_qcheck",
                     "rt_debug_counters", "rt_debug_regions", "rt_debug_last_split",
                     "rt_debug_wave_times"]
    for n in names:
        assert hasattr(rt.lib, n), f"missing export {n}"
    assert rt.debug_qcheck() is None  # the product library is built without the protocol checks


def test_struct_layout_matches_header(rt, tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "rt_ffi.h"\nint main(void){'
                   'printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(rt_render_params), sizeof(rt_render_stats),'
                   'sizeof(rt_object_desc), sizeof(rt_mesh_desc), sizeof(rt_scene_desc),'
                   'offsetof(rt_render_params, seed), offsetof(rt_object_desc, mesh));return 0;}')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(rt.RenderParams), ctypes.sizeof(rt.RenderStats), ctypes.sizeof(rt.ObjectDesc),
            ctypes.sizeof(rt.MeshDesc), ctypes.sizeof(rt.SceneDesc), rt.RenderParams.seed.offset,
            rt.ObjectDesc.mesh.offset]
    assert got == want


def test_errors_are_codes_not_crashes(rt):
    h = ctypes.c_void_p()
    assert rt.lib.rt_scene_load_toml(b"/nonexistent.toml", None, ctypes.byref(h)) == -4
    assert b"nonexistent" in rt.lib.rt_last_error()
    assert rt.lib.rt_render(None, None, None, None, None, None) == -1


def test_render_multi_rejects_bad_device_ordinals(rt):
    """rt_render_multi checks every device ordinal against the visible HIP devices before it starts
    a worker: an ordinal no device has (negative, or >= the device count) is RT_E_INVAL with a message,
    never a crash; on a host without a GPU every call is RT_E_NODEVICE (-6), so a caller can tell
    'no GPU' from 'bad ordinal'."""
    from conftest import scene_path

    sc = rt.Scene.from_toml(scene_path("cornell_box"))
    p = rt.make_params(64, 48, 4, 1, (0, 0, 64, 48), rt.FLAG_MEGAKERNEL, 0, 1)
    out = (ctypes.c_uint8 * (64 * 48 * 3))()
    n = rt.lib.rt_device_count()
    for bad in (-1, n, n + 7, 1 << 30):
        devs = (ctypes.c_int32 * 2)(0, bad)
        rc = rt.lib.rt_render_multi(sc.handle, ctypes.byref(p), devs, 2, 0, out, None, None)
        if n == 0:
            assert rc == -6 and b"no HIP device" in rt.lib.rt_last_error()
        else:
            assert rc == -1 and b"out of range" in rt.lib.rt_last_error()


def test_scene_without_slot_tables_still_loads(rt, monkeypatch):
    """An octree whose node ids exceed the child-slot encoding loads without its slot tables (rt_scene_info
    [11] = 0) instead of failing; RT_TEST_SLOT_MAX_PID lowers the parent-ordinal limit to stand in for a mesh beyond the encoding.
    (The GPU test test_walk_culls_do_not_change_frames renders such a scene.)"""
    from conftest import scene_path

    assert rt.Scene.from_toml(scene_path("flying_unicorn")).info()["slot_tables"] == 1
    monkeypatch.setenv("RT_TEST_SLOT_MAX_PID", "1000")
    info = rt.Scene.from_toml(scene_path("flying_unicorn")).info()
    assert info["nodes"] == 47183 and info["slot_tables"] == 0


def test_band_plan_covers_tile_in_order(rt):
    """rt_render_multi's band plan (handed out in this order from a host atomic counter): the bands
    partition the tile's rows [0, tile_h) contiguously, in increasing order, each non-empty; about 8
    bands per worker by default."""
    for th in (1, 7, 37, 450, 1080, 4096):
        for workers in (1, 2, 3, 8):
            for band in (0, 1, 5, 64, 5000):
                first, rows = rt.band_plan(th, workers, band)
                assert first[0] == 0 and all(r > 0 for r in rows)
                assert all(first[i] + rows[i] == first[i + 1] for i in range(len(rows) - 1))
                assert first[-1] + rows[-1] == th
                if band > 0:
                    assert all(r == min(band, th) for r in rows[:-1])
                else:
                    assert len(rows) <= 8 * workers and (th < 8 * workers or len(rows) >= 4 * workers)
    assert rt.band_plan(0, 4, 0) == ([], [])


def test_product_library_reads_no_tuning_switches(rt):
    """The RT_* A/B switches (ab_knobs.h) are compiled into the A/B build only: the product library holds
    none of their names, so no environment variable can select another kernel or shape in a server
    process. Only the two RT_TEST_* hooks remain (they force the exact fallback tables of oversized
    octrees, for tests)."""
    blob = open(rt.LIB_PATH, "rb").read()
    names = set(re.findall(rb"RT_[A-Z0-9_]{3,}", blob))
    switches = {n for n in names if not n.startswith((b"RT_FLAG_", b"RT_TEST_", b"RT_E_", b"RT_OK"))}
    assert not switches, sorted(switches)
    assert not re.search(rb"RT_MK_", blob)
    ab = os.path.join(REPO, "raytracer-server_amd", "lib", "variants", "ab.so")
    if os.path.exists(ab):  # the A/B build does read them
        assert b"RT_MK_POOL" in open(ab, "rb").read()
