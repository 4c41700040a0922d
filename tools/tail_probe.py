"""Strong-scaling probe on one GPU: device time of rank r's interleaved-row share of the frame
(row_step = N) vs the whole frame, i.e. the per-rank efficiency the N-GPU bench can reach at best.
python tools/tail_probe.py [spp] [scene]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
scene = sys.argv[2] if len(sys.argv) > 2 else "cornell_box"
W, H = 1920, 1080
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
rt_amd.render(s, W, H, 4, megakernel=True)  # warm-up
_, _, full = rt_amd.render(s, W, H, spp, megakernel=True)
print(f"{scene} {W}x{H}x{spp}: full frame {full['device_ms']:.1f} ms")
for n in (2, 4, 8):
    worst = 0.0
    for r in (0, n - 1):
        th = (H - r + n - 1) // n
        _, _, st = rt_amd.render(s, W, H, spp, tile=(0, r, W, th), megakernel=True, row_step=n)
        worst = max(worst, st["device_ms"])
    print(f"  N={n}: rank share {worst:.1f} ms, ideal {full['device_ms'] / n:.1f} ms, efficiency {full['device_ms'] / n / worst:.3f}")
