"""Device time of one frame vs spp (each size rendered twice through rt_render; the second call is the
steady state): python tools/spp_probe.py SCENE W H SPP[,SPP...] [mis] [wf]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

scene, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
spps = [int(x) for x in sys.argv[4].split(",")]
mis = "mis" in sys.argv[5:]
mk = "wf" not in sys.argv[5:]
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
for spp in spps:
    for rep in range(2):
        _, _, st = rt_amd.render(s, w, h, spp, megakernel=mk, mis=mis)
        n = st["samples"]
        print(f"{scene} {w}x{h}x{spp}{' mis' if mis else ''}{'' if mk else ' wavefront'} call {rep}: {st['device_ms']:.1f} ms device, "
              f"{n / st['device_ms'] / 1e3:.1f} Msamples/s", flush=True)
