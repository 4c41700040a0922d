"""Where a rank share's fixed ~10 ms goes: device time of the analytic megakernel on tiles of the
cornell frame, contiguous (row_step 1) and interleaved (row_step N), against the full frame's
per-sample rate. python tools/end_probe.py [spp] [scene]
RT_MK_TAIL / RT_MK_TAIL_CPS act only in the A/B build: run it with RT_AMD_LIB=.../lib/variants/ab.so."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
scene = sys.argv[2] if len(sys.argv) > 2 else "cornell_box"
W, H = 1920, 1080
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
rt_amd.render(s, 64, 48, 4, megakernel=True)
_, _, full = rt_amd.render(s, W, H, spp, megakernel=True)
per_row = full["device_ms"] / H
print(f"{scene} {W}x{H}x{spp} env TAIL={os.environ.get('RT_MK_TAIL', '-')} CPS={os.environ.get('RT_MK_TAIL_CPS', '-')}: "
      f"full {full['device_ms']:.1f} ms", flush=True)
for rows, step in ((540, 1), (540, 2), (270, 1), (135, 1), (135, 8), (68, 1), (34, 1)):
    _, _, st = rt_amd.render(s, W, H, spp, tile=(0, 0, W, rows), megakernel=True, row_step=step)
    print(f"  rows {rows:4d} step {step}: {st['device_ms']:7.1f} ms, linear {rows * per_row:7.1f}, "
          f"excess {st['device_ms'] - rows * per_row:5.1f} ms", flush=True)
