"""Is a rank share's fixed ~10 ms per launch an end phase or a clock ramp after idle? Times the N = 8
rank-0 share of cornell 1920x1080x1024 (a) after 200 ms of host idle and (b) enqueued right behind
another render on the same stream (no idle gap), with HIP events on that stream.
python tools/ramp_probe.py [N] [spp]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import torch  # noqa: E402
import rt_amd  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
W, H = 1920, 1080
torch.cuda.set_device(0)
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", "cornell_box.toml"))
th = (H + N - 1) // N
p = rt_amd.make_params(W, H, spp, 0x5EED, (0, 0, W, th), rt_amd.FLAG_MEGAKERNEL, 0, N)
full = rt_amd.make_params(W, H, spp, 0x5EED, (0, 0, W, H), rt_amd.FLAG_MEGAKERNEL, 0, 1)
rgb = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
rt_amd.render_device(s, p, rgb.data_ptr(), None, st.cuda_stream)
st.synchronize()
for rep in range(3):
    time.sleep(0.2)
    e[0].record(st)
    rt_amd.render_device(s, p, rgb.data_ptr(), None, st.cuda_stream)
    e[1].record(st)
    rt_amd.render_device(s, p, rgb.data_ptr(), None, st.cuda_stream)
    e[2].record(st)
    rt_amd.render_device(s, p, rgb.data_ptr(), None, st.cuda_stream)
    e[3].record(st)
    st.synchronize()
    print(f"N={N} share x3 back to back after idle: {e[0].elapsed_time(e[1]):.1f} / {e[1].elapsed_time(e[2]):.1f} / "
          f"{e[2].elapsed_time(e[3]):.1f} ms", flush=True)
time.sleep(0.2)
e[0].record(st)
rt_amd.render_device(s, full, rgb.data_ptr(), None, st.cuda_stream)
e[1].record(st)
st.synchronize()
print(f"full frame: {e[0].elapsed_time(e[1]):.1f} ms, /N {e[0].elapsed_time(e[1]) / N:.1f}", flush=True)
