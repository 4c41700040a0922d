"""Diagnostic: traversal work per mesh trace on the GPU (RT_DEBUG_COUNTERS build) vs the oracle.
python tools/dbg_counters.py <lib.so> SCENE W H SPP"""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RT_AMD_LIB"] = sys.argv[1]
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa
scene, w, h, spp = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
c = (ctypes.c_ulonglong * 16)()
rt_amd.lib.rt_debug_counters(c)
rgb, _, st = rt_amd.render(s, w, h, spp, megakernel=True)
rt_amd.lib.rt_debug_counters(c)
calls = max(1, c[0])
print(f"{scene} {w}x{h}x{spp}: vertices {st['vertices']} mesh calls {c[0]} past cull {c[1]} "
      f"({c[1]/calls:.3f}); per call: nodes {c[2]/calls:.2f} boxes {c[3]/calls:.2f} tris {c[4]/calls:.2f}; "
      f"device {st['device_ms']:.1f} ms")
if c[8]:
    print(f"  mesh megakernel: {c[8]} wave iterations, vertex-phase lanes/iteration {c[9]/c[8]:.1f}, "
          f"walk steps/iteration {c[10]/c[8]:.2f}, walking lanes/step {c[11]/max(1, c[10]):.1f}")
