"""Cancel latency through rt_render (one render, then two concurrent renders sharing one flag):
python tools/cancel_probe.py [SCENE W H SPP DELAY]
Prints, per render, the time from start to return and whether it reported RT_CANCELLED."""
import ctypes
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell_box"
w, h, spp = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (1920, 1080, 2048)
delay = float(sys.argv[5]) if len(sys.argv) > 5 else 0.3
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
rt_amd.render(s, 64, 48, 4, megakernel=True)  # warm-up (module load, scene upload)

for n in (1, 2):
    flag = ctypes.c_int32(0)
    done = {}
    t0 = time.perf_counter()

    def run(k):
        _, _, st = rt_amd.render(s, w, h, spp, 0x5EED + k, megakernel=True, cancel=flag)
        done[k] = (time.perf_counter() - t0, st["cancelled"], st["device_ms"])

    timer = threading.Timer(delay, lambda: setattr(flag, "value", 1))
    timer.start()
    ts = [threading.Thread(target=run, args=(k,)) for k in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    timer.cancel()
    for k in range(n):
        print(f"{n} render(s): render {k} returned after {done[k][0]:.3f} s, cancelled {done[k][1]}, "
              f"device {done[k][2]:.1f} ms (flag raised at {delay:.2f} s)", flush=True)
