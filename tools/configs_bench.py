"""Every BASELINE.json config on one GPU (one process): Msamples/s per config, device time.
python tools/configs_bench.py [--quick] [--fp32]  (--fp32: the f32 perf mode; C5 is 4096x4096 at reduced spp on 1 GPU: stated in the line)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

quick = "--quick" in sys.argv
fp32 = "--fp32" in sys.argv
CONFIGS = [
    # (label, scene, w, h, spp, mis)
    ("C1 cornell 600x450 1spp (reference plumbing case: black frame)", "cornell_box", 600, 450, 1, False),
    ("C1' cornell 600x450 4spp", "cornell_box", 600, 450, 4, False),
    ("C2 cornell 1920x1080 256spp MIS on", "cornell_box", 1920, 1080, 256, True),
    ("C2' cornell 1920x1080 256spp MIS off", "cornell_box", 1920, 1080, 256, False),
    ("C3 cubes 1920x1080 1024spp MIS off", "cubes", 1920, 1080, 1024, False),
    ("C3 cubes 1920x1080 1024spp MIS on", "cubes", 1920, 1080, 1024, True),
    ("C4 unicorn 1920x1080 512spp", "flying_unicorn", 1920, 1080, 512, False),
    ("C5 unicorn 4096x4096 (64 of 4096 spp, 1 GPU)", "flying_unicorn", 4096, 4096, 64, False),
]
scenes = {}
for label, name, w, h, spp, mis in CONFIGS:
    if quick:
        spp = max(1, spp // 16) if spp > 4 else spp
    if name not in scenes:
        scenes[name] = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{name}.toml"))
    t = time.perf_counter()
    rgb, _, st = rt_amd.render(scenes[name], w, h, spp, megakernel=True, mis=mis, fp32=fp32)
    wall = time.perf_counter() - t
    n = st["samples"]
    rate = n / st["device_ms"] / 1e3 if st["device_ms"] > 0 and n else 0.0
    print(f"{label}{' [f32]' if fp32 else ''}: spp {spp}, {n} samples, {st['device_ms']:.1f} ms device, {wall*1e3:.1f} ms wall, "
          f"{rate:.1f} Msamples/s, {st['vertices'] / max(1, n):.3f} vertices/sample, mean RGB8 {rgb.mean():.2f}",
          flush=True)
