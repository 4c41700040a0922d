"""Where a rank share's fixed ~10 ms goes: device time of the analytic megakernel on tiles of the
cornell frame, contiguous (row_step 1) and interleaved (row_step N), against the full frame's
per-sample rate. python tools/end_probe.py [spp] [scene]
RT_MK_TAIL / RT_MK_TAIL_CPS act only in the A/B build: run it with RT_AMD_LIB=.../lib/variants/ab.so.

python tools/end_probe.py --waves [spp] [scene]: with the diagnostic build (lib/variants/dbg.so,
RT_DEBUG_TIMERS: rt_debug_wave_times), the wave-by-wave timeline of the full frame and of one 8-GPU rank's
share (135 rows, row_step 8): when the waves start and end, how much of the launch's wave-slot time lies after
a wave's end (the drain), and how long waves run with fewer than half of their lanes busy."""
import ctypes
import os
import sys

if "--waves" in sys.argv:
    sys.argv.remove("--waves")
    WAVES = True
    os.environ.setdefault("RT_AMD_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "raytracer-server_amd", "lib", "variants", "dbg.so"))
else:
    WAVES = False

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
scene = sys.argv[2] if len(sys.argv) > 2 else "cornell_box"
W, H = 1920, 1080
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
rt_amd.render(s, 64, 48, 4, megakernel=True)
if WAVES:
    import numpy as np

    NW = 8192

    def timeline(label, **kw):
        out = (ctypes.c_ulonglong * (5 * NW))()
        rt_amd.lib.rt_debug_wave_times(out, NW)  # clear
        _, _, st = rt_amd.render(s, W, H, spp, megakernel=True, **kw)
        plan = rt_amd.debug_last_split()
        assert rt_amd.lib.rt_debug_wave_times(out, NW) == 0, "not a RT_DEBUG_TIMERS build"
        raw = np.frombuffer(out, dtype=np.uint64).reshape(NW, 5)
        raw = raw[raw[:, 2] > 0]
        a = raw.astype(np.float64)
        t0 = a[:, 0].min()
        start, end, tk = (a[:, 0] - t0) / 1e5, (a[:, 2] - t0) / 1e5, (a[:, 3] - t0) / 1e5  # ms (100 MHz)
        half = np.where(raw[:, 1] == np.uint64(0xFFFFFFFFFFFFFFFF), a[:, 2], a[:, 1])
        half = (half - t0) / 1e5
        span = end.max()
        idle = (span - end).sum() / (len(end) * span)
        q = np.percentile(end, [0, 10, 50, 90, 99, 100])
        print(f"{label}: {st['device_ms']:.1f} ms device, {len(end)} waves, span {span:.1f} ms; starts within "
              f"{start.max():.2f} ms; wave ends (ms) min/p10/p50/p90/p99/max " + " / ".join(f"{v:.1f}" for v in q) +
              f"; wave-slot time after a wave's end {100 * idle:.1f}%; below half its lanes: mean "
              f"{(end - half).mean():.2f} ms, max {(end - half).max():.2f} ms; last unit handed out at "
              f"{tk.max():.1f} ms; split {plan}", flush=True)
        nsub = (kw.get("tile", (0, 0, W, H))[2] * kw.get("tile", (0, 0, W, H))[3]) * 4
        n_whole = nsub - plan["split"]
        cps = max(1, (spp // 4) // max(1, plan["chunk"]))
        for i in np.argsort(-end)[:6]:  # the last waves: their last unit (whole subpixel or a chunk of a split one)
            u = int(raw[i, 4])
            what = f"whole subpixel {u}" if u < n_whole else \
                f"chunk {(u - n_whole) % cps} of split subpixel {n_whole + (u - n_whole) // cps}"
            print(f"    wave {i}: end {end[i]:.1f} ms; its last lane took its last unit at {tk[i]:.1f} ms ({end[i] - tk[i]:.1f} "
                  f"ms before the wave's end): {what}", flush=True)

    timeline(f"{scene} {W}x{H}x{spp} full frame")
    for rows, step in ((135, 8), (135, 1), (540, 1)):
        timeline(f"  rows {rows} step {step}", tile=(0, 0, W, rows), row_step=step)
    sys.exit(0)
_, _, full = rt_amd.render(s, W, H, spp, megakernel=True)
per_row = full["device_ms"] / H
print(f"{scene} {W}x{H}x{spp} env TAIL={os.environ.get('RT_MK_TAIL', '-')} CPS={os.environ.get('RT_MK_TAIL_CPS', '-')}: "
      f"full {full['device_ms']:.1f} ms", flush=True)
for rows, step in ((540, 1), (540, 2), (270, 1), (135, 1), (135, 8), (68, 1), (34, 1)):
    _, _, st = rt_amd.render(s, W, H, spp, tile=(0, 0, W, rows), megakernel=True, row_step=step)
    print(f"  rows {rows:4d} step {step}: {st['device_ms']:7.1f} ms, linear {rows * per_row:7.1f}, "
          f"excess {st['device_ms'] - rows * per_row:5.1f} ms", flush=True)
