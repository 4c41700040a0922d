"""Cost of the frame by row band: device time, path vertices per sample and time per vertex of each band of
rows rendered on its own (the bands an interleaved rank share or the split tail draws its subpixels from).
python tools/row_cost.py [scene] [spp] [bands] [W] [H]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell_box"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
bands = int(sys.argv[3]) if len(sys.argv) > 3 else 8
W = int(sys.argv[4]) if len(sys.argv) > 4 else 1920
H = int(sys.argv[5]) if len(sys.argv) > 5 else 1080
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
rt_amd.render(s, 64, 48, 4, megakernel=True)
_, _, full = rt_amd.render(s, W, H, spp, megakernel=True)
print(f"{scene} {W}x{H}x{spp}: full frame {full['device_ms']:.1f} ms, {full['vertices'] / full['samples']:.3f} vertices/sample, "
      f"{full['device_ms'] * 1e6 / full['vertices']:.4f} ns/vertex", flush=True)
for b in range(bands):
    y0, y1 = b * H // bands, (b + 1) * H // bands
    _, _, st = rt_amd.render(s, W, H, spp, tile=(0, y0, W, y1 - y0), megakernel=True)
    print(f"  rows {y0:5d}..{y1:5d}: {st['device_ms']:8.1f} ms ({st['device_ms'] / full['device_ms'] * bands:.3f} of "
          f"an equal share), {st['vertices'] / st['samples']:.3f} vertices/sample, "
          f"{st['device_ms'] * 1e6 / st['vertices']:.4f} ns/vertex", flush=True)
