"""Determinism of the megakernels' LDS hand-offs (the query pool of the flat-mesh kernel and the walk
pool of the deep-octree kernel, kernels/megakernel_common.h LdsQueue):

  * repeated concurrent renders on two HIP streams (the launches overlap on the device, blocks of the
    two kernels interleave on the CUs, and which wave evaluates which query changes from run to run)
    are byte-identical to the serial renders, for the cubes (query pool) and the unicorn (walk pool);
  * the same renders through the protocol-checking build (lib/variants/qcheck.so, -DRT_QCHECK=1, run
    in a subprocess with RT_AMD_LIB) report no violation: no ring slot is overwritten before it was
    taken, no queue exceeds its ring, no outstanding-query count goes negative, no owner/taker state
    mismatch (rt_diag.h: rt_debug_qcheck), and its frames equal the product library's.

A lane's result must not depend on which other lanes share its wave: DESIGN.md §5 (hand-off
protocol) argues why, and test_exact_division_shortcuts checks the wave-voted arithmetic shortcuts
(rcp_rn / qdiv / sqrt_rn take their fast path only when the whole wave qualifies) against the
library operations bit for bit.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO
from test_gpu_parity import SEED

pytestmark = pytest.mark.gpu

CASES = [("cubes", 256, 192, 64), ("flying_unicorn", 192, 144, 32)]


def _device_render(rt, torch, scene, w, h, spp, seed, stream):
    p = rt.make_params(w, h, spp, seed, None, rt.FLAG_MEGAKERNEL, 0, 1)
    buf = torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the zero fill (current stream) is done before the render's stream writes
    rt.render_device(scene, p, buf.data_ptr(), None, stream.cuda_stream)
    return buf


def _concurrent_rounds(rt, torch, scenes, rounds):
    """Per case, `rounds` x 3 renders on two streams (seeds 0, 1, 2 alternating streams), all compared
    with the serial frames; returns the serial frames' digests."""
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    digests = {}
    for name, w, h, spp in CASES:
        s = scenes[name]
        ref = {k: rt.render(s, w, h, spp, SEED + k, megakernel=True)[0] for k in range(3)}
        digests[name] = [hashlib.sha1(ref[k].tobytes()).hexdigest()[:12] for k in range(3)]
        for r in range(rounds):
            bufs = [_device_render(rt, torch, s, w, h, spp, SEED + k, (s1, s2)[(k + r) & 1]) for k in range(3)]
            torch.cuda.synchronize()
            for k in range(3):
                got = bufs[k].cpu().numpy()
                bad = np.argwhere(np.any(got != ref[k], axis=-1))
                assert bad.size == 0, (name, r, k, bad[:4].tolist(), got[tuple(bad[0])].tolist(), ref[k][tuple(bad[0])].tolist())
    return digests


def test_concurrent_renders_bit_identical(rt, gpu_scenes):
    import torch

    _concurrent_rounds(rt, torch, gpu_scenes, rounds=4)


_QCHECK_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.path.join(os.environ["RT_REPO"], "raytracer-server_amd"))
sys.path.insert(0, os.path.join(os.environ["RT_REPO"], "tests"))
import torch
import rt_amd
import test_gpu_determinism as T
scenes = {n: rt_amd.Scene.from_toml(os.path.join(os.environ["RT_REPO"], "scenes", n + ".toml")) for n, *_ in T.CASES}
rt_amd.debug_qcheck()
digests = T._concurrent_rounds(rt_amd, torch, scenes, rounds=2)
print(json.dumps({"qcheck": rt_amd.debug_qcheck(), "digests": digests}))
"""


def test_qcheck_build_reports_no_protocol_violation(rt, gpu_scenes):
    import torch

    lib = os.path.join(REPO, "raytracer-server_amd", "lib", "variants", "qcheck.so")
    if not os.path.exists(lib):
        pytest.skip("lib/variants/qcheck.so not built (make -C raytracer-server_amd qcheck)")
    env = dict(os.environ, RT_AMD_LIB=lib, RT_REPO=REPO, PYTHONPATH=os.path.join(REPO, "tests"))
    out = subprocess.run([sys.executable, "-c", _QCHECK_SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["qcheck"] == [0, 0, 0, 0], res
    # the checking build renders the product library's frames
    for name, w, h, spp in CASES:
        want = [hashlib.sha1(rt.render(gpu_scenes[name], w, h, spp, SEED + k, megakernel=True)[0].tobytes()).hexdigest()[:12]
                for k in range(3)]
        assert res["digests"][name] == want, name


_VARIANT_SCRIPT = r"""
import hashlib, json, os, sys
sys.path.insert(0, os.path.join(os.environ["RT_REPO"], "raytracer-server_amd"))
import rt_amd
out = {}
for name, w, h, spp in [("cubes", 160, 120, 32), ("flying_unicorn", 160, 120, 16)]:
    s = rt_amd.Scene.from_toml(os.path.join(os.environ["RT_REPO"], "scenes", name + ".toml"))
    out[name] = hashlib.sha1(rt_amd.render(s, w, h, spp, 0x5EED, megakernel=True)[0].tobytes()).hexdigest()[:12]
print(json.dumps(out))
"""


@pytest.mark.parametrize("env", [{"RT_MK_FPOOL": "0"}, {"RT_MK_POOL": "0"}, {"RT_MK_NOSPEC": "0"},
                                 {"RT_MK_FPOOL_REFILL": "0", "RT_MK_POOL_CAM_REFILL": "0"}])
def test_kernel_variants_render_the_default_frames(env):
    """The A/B kernel variants behind RT_* switches, which only the A/B build reads (ab_knobs.h:
    lib/variants/ab.so, -DRT_AB_KNOBS=1; read once per process, so each in a subprocess): the
    block-synchronous flat kernel (RT_MK_FPOOL=0), per-lane octree walks (RT_MK_POOL=0), the
    mirror-capable query-pool instance on the mirror-free cubes (RT_MK_NOSPEC=0: the default runs Cfg
    bit 32) and both pools without their camera-sample refill pass render byte-identical frames to the
    product library's defaults; the product library under the same switches renders them too (it
    reads none of them)."""
    ab = os.path.join(REPO, "raytracer-server_amd", "lib", "variants", "ab.so")
    assert os.path.exists(ab), f"{ab} not built (make -C raytracer-server_amd ab)"
    base = dict(os.environ, RT_REPO=REPO)
    for k in ("RT_MK_FPOOL", "RT_MK_POOL", "RT_MK_NOSPEC", "RT_MK_FPOOL_REFILL", "RT_MK_POOL_CAM_REFILL", "RT_AMD_LIB"):
        base.pop(k, None)
    runs = []
    for e in ({}, dict(env, RT_AMD_LIB=ab), env):
        out = subprocess.run([sys.executable, "-c", _VARIANT_SCRIPT], env=dict(base, **e), capture_output=True,
                             text=True, timeout=240)
        assert out.returncode == 0, out.stderr[-3000:]
        runs.append(json.loads(out.stdout.strip().splitlines()[-1]))
    assert runs[0] == runs[1], (env, runs)


# C3 / C4 at their full 1920x1080 (reduced spp): one render per scene, frame digests as JSON
_CULL_SCRIPT = """
import hashlib, json, os, sys
sys.path.insert(0, os.path.join(os.environ["RT_REPO"], "raytracer-server_amd"))
import rt_amd
out = {}
for name in ("cubes", "flying_unicorn"):
    s = rt_amd.Scene.from_toml(os.path.join(os.environ["RT_REPO"], "scenes", name + ".toml"))
    out[name + "/slots"] = s.info()["slot_tables"]
    out[name] = hashlib.sha1(rt_amd.render(s, 1920, 1080, 8, 0x5EED, megakernel=True)[0].tobytes()).hexdigest()[:12]
print(json.dumps(out))
"""
_cull_frames = {}


def _cull_run(lib=None, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("RT_TEST_SLOT_MAX_PID", "RT_AMD_LIB")}
    e.update(RT_REPO=REPO, **(env or {}))
    if lib:
        e["RT_AMD_LIB"] = lib
    out = subprocess.run([sys.executable, "-c", _CULL_SCRIPT], env=e, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("variant", ["walkref", "near64", "noslots", "noanc"])
def test_walk_culls_do_not_change_frames(variant):
    """The culls the mesh kernels add to the reference's octree walk (geometry.rs:1262-1273) are exact:
    the cubes (C3) and the unicorn (C4) at 1920x1080 render byte-identical frames without them —
      walkref: the octree walked in the reference's visiting order with no subtree-bounds culls
               (-DRT_WALK_TIGHT=0, lib/variants/walkref.so: node_kids walks);
      near64:  the per-mesh near tests in f64 (near_box) instead of f32 (near_mesh32), -DRT_NEAR32=0;
      noslots: the default library on a scene loaded without its slot tables (RT_TEST_SLOT_MAX_PID=0, the
               path a 2^23-node octree takes: the pool kernel's node_kids instance);
      noanc:   the role pool's walkers without their 16-bit LDS ancestor columns, popping through pid_up
               (RT_TEST_ANC_OFF=1: the path of octrees with more than 65536 parents)."""
    if "default" not in _cull_frames:
        _cull_frames["default"] = _cull_run()
    base = _cull_frames["default"]
    assert base["cubes/slots"] == 1 and base["flying_unicorn/slots"] == 1
    if variant == "noslots":
        got = _cull_run(env={"RT_TEST_SLOT_MAX_PID": "0"})
        assert got["flying_unicorn/slots"] == 0 and got["cubes/slots"] == 0
    elif variant == "noanc":
        got = _cull_run(env={"RT_TEST_ANC_OFF": "1"})
        assert got["flying_unicorn/slots"] == 1
    else:
        lib = os.path.join(REPO, "raytracer-server_amd", "lib", "variants", variant + ".so")
        assert os.path.exists(lib), f"{lib} not built (make -C raytracer-server_amd variants)"
        got = _cull_run(lib=lib)
    assert got["cubes"] == base["cubes"] and got["flying_unicorn"] == base["flying_unicorn"], (variant, base, got)
