"""One render through the C ABI for profiling runs:
python tools/prof_render.py SCENE W H SPP [mk|wf|f32] [mis] [nearest] [share=N/R]
  share=N/R  only rank R's interleaved rows of N (bench.py's partition: rows R, R + N, ...)

A small warm-up render of the same scene runs first (module load, scene upload), so the last
dispatch of the render kernel in a rocprofv3 pass is the measured render; the line printed at the
end carries its device time and exact path-vertex count (tools/pmc_report.py reads both)."""
import hashlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

scene, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
mode = sys.argv[5] if len(sys.argv) > 5 else "mk"
mis = "mis" in sys.argv[6:]
nearest = "nearest" in sys.argv[6:]  # RT_FLAG_MESH_NEAREST (BVH)
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
kw = dict(megakernel=(mode == "mk"), mis=mis, mesh_nearest=nearest, fp32=(mode == "f32"))
share = next((x for x in sys.argv[6:] if x.startswith("share=")), None)
if share:
    sn, sr = (int(v) for v in share[6:].replace("/", ":").split(":"))
    kw.update(tile=(0, sr, w, (h - sr + sn - 1) // sn), row_step=sn)
rt_amd.render(s, w, h, 4, **kw)  # warm-up at the same size (buffers allocated and touched)
rt_amd.render(s, w, h, spp, **kw)  # and at the same spp (the split tail's scratch allocated)
t = time.perf_counter()
rgb, _, st = rt_amd.render(s, w, h, spp, **kw)
dt = time.perf_counter() - t
n = st["samples"]
print(f"{scene} {w}x{h}x{spp} {mode}{' mis' if mis else ''}{' nearest' if nearest else ''}{' ' + share if share else ''}: {dt*1e3:.1f} ms wall, "
      f"{st['device_ms']:.1f} ms device, {n / st['device_ms'] / 1e3:.1f} Msamples/s, samples {n}, "
      f"vertices {st['vertices']}, {st['vertices'] / max(1, n):.3f} vertices/sample, iterations {st['iterations']}, "
      f"rgb sha1 {hashlib.sha1(rgb.tobytes()).hexdigest()[:12]}")
