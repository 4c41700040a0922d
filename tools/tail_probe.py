"""Strong-scaling probe on one GPU: device time of rank r's interleaved-row share of the frame
(row_step = N) vs the whole frame, i.e. the per-rank efficiency the N-GPU bench can reach at best
(the partition of server.rs:165-168 is by pixels; bench.py interleaves rows).

python tools/tail_probe.py [spp] [scene] [W] [H]
    full frame, then ranks 0 and N-1 of N = 2, 4, 8
python tools/tail_probe.py share SPP SCENE W H N RANK[,RANK...] [REF_SPP]
    only the given ranks' shares of N (e.g. C5: share 4096 flying_unicorn 4096 4096 8 0,7), plus the
    full frame at REF_SPP (default 64) as the single-GPU rate the shares are projected against"""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402


def share(s, W, H, spp, n, r):
    th = (H - r + n - 1) // n
    rgb, _, st = rt_amd.render(s, W, H, spp, tile=(0, r, W, th), megakernel=True, row_step=n)
    return st, hashlib.sha1(rgb.tobytes()).hexdigest()[:12]


if len(sys.argv) > 1 and sys.argv[1] == "share":
    spp, scene, W, H, n = int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
    ranks = [int(x) for x in sys.argv[7].split(",")]
    ref_spp = int(sys.argv[8]) if len(sys.argv) > 8 else 64
    s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
    rt_amd.render(s, 64, 48, 4, megakernel=True)  # warm-up
    _, _, ref = rt_amd.render(s, W, H, ref_spp, megakernel=True)
    ref_rate = ref["samples"] / ref["device_ms"] / 1e3
    print(f"{scene} {W}x{H}x{ref_spp} full frame: {ref['device_ms']:.1f} ms, {ref_rate:.1f} Msamples/s", flush=True)
    for r in ranks:
        st, dig = share(s, W, H, spp, n, r)
        rate = st["samples"] / st["device_ms"] / 1e3
        ideal = W * H * 4 * (spp // 4) / n / ref_rate / 1e3
        print(f"  {scene} {W}x{H}x{spp} rank {r} of {n}: {st['samples']} samples, {st['device_ms'] / 1e3:.2f} s device, "
              f"{rate:.1f} Msamples/s, vs the full frame's rate at {ref_spp} spp: ideal {ideal / 1e3:.2f} s, "
              f"efficiency {ideal / st['device_ms']:.3f}; rgb sha1 {dig}", flush=True)
    sys.exit(0)

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
scene = sys.argv[2] if len(sys.argv) > 2 else "cornell_box"
W = int(sys.argv[3]) if len(sys.argv) > 3 else 1920
H = int(sys.argv[4]) if len(sys.argv) > 4 else 1080
s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{scene}.toml"))
rt_amd.render(s, W, H, 4, megakernel=True)  # warm-up
_, _, full = rt_amd.render(s, W, H, spp, megakernel=True)
print(f"{scene} {W}x{H}x{spp}: full frame {full['device_ms']:.1f} ms", flush=True)
for n in (2, 4, 8):
    worst = 0.0
    for r in (0, n - 1):
        st, _ = share(s, W, H, spp, n, r)
        worst = max(worst, st["device_ms"])
    print(f"  N={n}: rank share {worst:.1f} ms, ideal {full['device_ms'] / n:.1f} ms, efficiency {full['device_ms'] / n / worst:.3f}",
          flush=True)
