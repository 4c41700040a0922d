"""Diagnostic for the mesh megakernel (RT_DEBUG_COUNTERS + RT_DEBUG_TIMERS build, tools/gpu_task.sh
dbgbuild): wave iterations, lanes in the vertex phase, walk steps and walking lanes per step, and the
wave-time split between the walk phase, the vertex phase and the bookkeeping.
python tools/dbg_mesh.py <lib.so> SCENE W H SPP"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RT_AMD_LIB"] = sys.argv[1]
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

scene, w, h, spp = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
rt_amd.render(s, 64, 48, 4, megakernel=True)
c = (ctypes.c_ulonglong * 16)()
r = (ctypes.c_ulonglong * 64)()
rt_amd.lib.rt_debug_counters(c)
rt_amd.lib.rt_debug_regions(r)
rgb, _, st = rt_amd.render(s, w, h, spp, megakernel=True)
rt_amd.lib.rt_debug_counters(c)
rt_amd.lib.rt_debug_regions(r)
calls = max(1, c[0])
it = max(1, c[8])
print(f"{scene} {w}x{h}x{spp} {' '.join(k + '=' + v for k, v in os.environ.items() if k.startswith('RT_MK'))}: "
      f"device {st['device_ms']:.1f} ms, vertices {st['vertices']}, vertices/wave-iteration {st['vertices'] / it:.1f}")
print(f"  mesh calls {c[0]}, past cull {c[1] / calls:.3f}; per call: nodes {c[2] / calls:.2f} leaves {c[3] / calls:.2f} culled picks {c[6] / calls:.2f} "
      f"tris {c[4] / calls:.2f} steps {c[5] / calls:.2f}")
if scene != "cubes":
    print(f"  walk-pool queries: shadow {c[12]}, closest {c[13]}, closest right after the same vertex's shadow query {c[14]}")
print(f"  wave iterations {c[8]}: vertex-phase lanes/iteration {c[9] / it:.1f}, walk steps/iteration {c[10] / it:.2f}, "
      f"walking lanes/step {c[11] / max(1, c[10]):.1f}")
T = {0: "iteration", 1: "walk phase", 2: "vertex phase", 4: "refill + ticket", 7: "surface()", 9: "light_sample",
     10: "visible()", 11: "brdf_sample", 13: "trace: inv + planes", 14: "trace: spheres"}
if scene != "cubes":  # the walk-pool kernel (render_mesh_f64.hip, path_f64.h walk_step)
    T.update({3: "pool: take + park load", 5: "pool: park store + put", 6: "vertex: trace + mesh cull",
              8: "vertex: shade_vertex", 12: "walk: leaf triangles", 13: "walk: pop", 14: "walk: pick + descend",
              15: "walk: begin (root order)"})
if os.environ.get("RT_MK_POOL", "2") == "2" and scene != "cubes":  # the role-split pool (default) (k_megakernel_roles_f64)
    T.update({0: "shader: iteration", 1: "walker: walk step", 2: "shader: vertex work", 3: "shader: take + load",
              4: "walker: iteration", 5: "walker: refill"})
    print(f"  roles: shader iterations {c[8]}, lanes holding a path {c[9] / it:.1f}; walker steps {c[10]}, "
          f"walking lanes/step {c[11] / max(1, c[10]):.1f}")
if os.environ.get("RT_MK_FLAT", "1") != "0" and scene == "cubes":  # render_flat_f64.hip phases
    T.update({1: "A camera + analytic", 2: "P mesh queries", 3: "C shadow results + shade + bookkeeping",
              6: "barrier waits"})
    print(f"  flat kernel: query chunks/iteration {c[13] / it:.2f}, lanes per chunk {c[12] / max(1, c[13]):.1f}, "
          f"active lanes/iteration {c[9] / it:.1f}")
tot = max(1, r[32] or sum(r[33:48]))
for i in range(16):
    if r[32 + i]:
        print(f"  t{i:2d} {T.get(i, '?'):22s} {r[32 + i] / tot * 100:6.1f} %  ticks/iter {r[32 + i] / it:9.1f}")
