"""Diagnostic: lane utilisation per instrumented region of the megakernel (RT_DEBUG_COUNTERS build).
python tools/dbg_regions.py <lib.so> SCENE W H SPP [share=N/R]  (share: rank R's interleaved rows of N, bench.py's
partition)"""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["RT_AMD_LIB"] = sys.argv[1]
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa
NAMES = {0: "loop iteration", 1: "active lanes", 2: "fresh (begin path)", 3: "refill pass", 4: "sample end",
         5: "begin_sample fallback", 6: "shade: hit", 7: "shade: specular", 8: "shade: diffuse NEE",
         9: "shadow ray (Le*f != 0)", 10: "BSDF continuation", 11: "sphere sqrt part", 12: "trace_closest",
         13: "visible()"}
scene, w, h, spp = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
c = (ctypes.c_ulonglong * 64)()
rt_amd.lib.rt_debug_regions(c)
kw = {}
share = next((x for x in sys.argv[6:] if x.startswith("share=")), None)
if share:
    sn, sr = (int(v) for v in share[6:].split("/"))
    kw = dict(tile=(0, sr, w, (h - sr + sn - 1) // sn), row_step=sn)
rgb, _, st = rt_amd.render(s, w, h, spp, megakernel=True, **kw)
rt_amd.lib.rt_debug_regions(c)
it = max(1, c[0])
print(f"{scene} {w}x{h}x{spp}{' ' + share if share else ''}: vertices {st['vertices']}, wave iterations {c[0]}")
TNAMES = {0: "iteration", 1: "fresh block", 2: "trace_closest (main)", 3: "shade_vertex", 4: "refill pass",
          5: "bookkeeping (ticket/cancel)", 6: "sample-end block", 7: "surface()", 9: "light_sample", 10: "visible()",
          11: "brdf_sample", 13: "trace: inv + axis planes", 14: "trace: spheres"}
tot = max(1, c[32])
print("  wave time per region (share of the iteration; nested regions overlap):")
for i in range(32):
    if c[32 + i]:
        print(f"  t{i:2d} {TNAMES.get(i, '?'):28s} {c[32+i]/tot*100:6.1f} %   ticks/iter {c[32+i]/it:8.1f}")
for i in range(16):
    if c[2 * i]:
        print(f"  r{i:2d} {NAMES.get(i, '?'):24s} entries/iter {c[2*i]/it:6.3f}  lanes/entry {c[2*i+1]/c[2*i]:5.1f}"
              f"  lanes/iter {c[2*i+1]/it:5.1f}")
