"""Determinism stress of the megakernels' LDS hand-offs ("Hand-off protocol"): ROUNDS
rounds of 3 renders per scene enqueued back to back on two HIP streams (the launches overlap, blocks
of two kernels share the CUs, and which wave takes which queued query changes from run to run), every
frame compared byte for byte with the serial frame of the same seed. With RT_AMD_LIB pointing at the
RT_QCHECK build (lib/variants/qcheck.so) it also prints the protocol-violation counters
(rt_debug_qcheck: slot overwritten, over capacity, negative outstanding count, owner/taker mismatch).

python tools/determinism_stress.py [ROUNDS] [SCENE:W:H:SPP ...]"""
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import torch  # noqa: E402

import rt_amd  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cases = [c.split(":") for c in sys.argv[2:]] or [["cubes", "256", "192", "64"], ["flying_unicorn", "192", "144", "32"]]
SEED = 0x5EED
qcheck = rt_amd.debug_qcheck()  # clears the counters (zeros and no effect in the product build)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
total_bad = 0
for name, w, h, spp in cases:
    w, h, spp = int(w), int(h), int(spp)
    s = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{name}.toml"))
    ref = {k: rt_amd.render(s, w, h, spp, SEED + k, megakernel=True)[0] for k in range(3)}
    bad = 0
    for r in range(rounds):
        bufs = []
        for k in range(3):
            p = rt_amd.make_params(w, h, spp, SEED + k, None, rt_amd.FLAG_MEGAKERNEL, 0, 1)
            buf = torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()  # the zero fill (current stream) completes before the render's stream writes
            rt_amd.render_device(s, p, buf.data_ptr(), None, ((s1, s2)[(k + r) & 1]).cuda_stream)
            bufs.append(buf)
        torch.cuda.synchronize()
        for k in range(3):
            got = bufs[k].cpu().numpy()
            diff = np.argwhere(np.any(got != ref[k], axis=-1))
            if diff.size:
                bad += 1
                y, x = diff[0]
                print(f"  MISMATCH {name} round {r} seed +{k}: {len(diff)} pixels, first ({x}, {y}) "
                      f"{got[y, x].tolist()} vs {ref[k][y, x].tolist()}", flush=True)
    total_bad += bad
    digests = [hashlib.sha1(ref[k].tobytes()).hexdigest()[:12] for k in range(3)]
    print(f"{name} {w}x{h}x{spp}: {rounds * 3} concurrent renders, {bad} differ from the serial frames {digests}", flush=True)
print(f"qcheck counters (slot, capacity, pending<0, state): {rt_amd.debug_qcheck()}; mismatching frames {total_bad}", flush=True)
sys.exit(1 if total_bad else 0)
