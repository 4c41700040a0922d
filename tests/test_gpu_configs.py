"""GPU tests of the BASELINE.json configurations the headline bench does not cover (C1, C3, C5), at
their real frame sizes where the oracle can keep up, against the CPU oracle (f64 tolerances of
SURVEY §8c.1 via test_gpu_parity._assert_parity).

  C1  cornell_box 600x450 1 spp: the reference's all-black frame (spp/4 = 0, server.rs:332), and the
      same frame at 4 spp against the oracle on crops;
  C3  cubes 1920x1080 MIS on vs off: the MIS estimator against the oracle (both kernels), and MIS vs
      NEE with the SAME seeds — same expectation, per-pixel variance ratio reported;
  C5  flying_unicorn 4096x4096 tiled across 8 GPUs: one rank's interleaved share (row_step 8) against
      the oracle on crops, the 8 shares assembled equal to a single-call frame byte for byte, and the
      one-process multi-device path (rt_render_multi) equal to it as well.
"""
import json
import os

import numpy as np
import pytest

from conftest import REPO
from test_gpu_parity import SEED, _assert_parity, _render_pair

pytestmark = pytest.mark.gpu


def _record(name, data):
    """Measured values of a statistical test, kept with the run's output (gpurun_out/)."""
    d = os.path.join(REPO, "gpurun_out")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"test_{name}.json"), "w") as f:
        json.dump(data, f, indent=1)
    print(name, json.dumps(data))


def test_c1_cornell_600x450(rt, gpu_scenes, oracle_scenes):
    s, o = gpu_scenes["cornell_box"], oracle_scenes["cornell_box"]
    for mk in (True, False):
        rgb, _, st = rt.render(s, 600, 450, 1, SEED, megakernel=mk)
        assert rgb.shape == (450, 600, 3) and st["samples"] == 0 and not rgb.any()
    full, sub, st = rt.render(s, 600, 450, 4, SEED, megakernel=True, want_sub=True)
    assert st["samples"] == 600 * 450 * 4
    for (x0, y0, tw, th) in [(0, 0, 24, 16), (288, 217, 24, 16), (576, 434, 24, 16), (100, 300, 40, 8)]:
        rgb_o, sub_o, _ = o.render(600, 450, 4, SEED, tile=(x0, y0, tw, th))
        _assert_parity(full[y0:y0 + th, x0:x0 + tw], sub[y0:y0 + th, x0:x0 + tw], rgb_o, sub_o, f"C1 crop {x0},{y0}")
    wf, _, _ = rt.render(s, 600, 450, 4, SEED, megakernel=False)
    assert np.array_equal(wf, full)


@pytest.mark.parametrize("megakernel", [True, False], ids=["megakernel", "wavefront"])
def test_c3_cubes_mis_parity(megakernel, rt, gpu_scenes, oracle_scenes):
    rgb_g, sub_g, st, rgb_o, sub_o, st_o = _render_pair(rt, gpu_scenes["cubes"], oracle_scenes["cubes"], 96, 72, 16,
                                                        mis=True, megakernel=megakernel)
    assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
    _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"cubes/mis/{'mk' if megakernel else 'wf'}")
    # C3's full frame size at low spp: a crop against the oracle
    full, sub, _ = rt.render(gpu_scenes["cubes"], 1920, 1080, 4, SEED, mis=True, megakernel=megakernel, want_sub=True)
    crop = (700, 700, 24, 16)  # the cubes' region
    x0, y0, tw, th = crop
    rgb_o, sub_o, _ = oracle_scenes["cubes"].render(1920, 1080, 4, SEED, tile=crop, mis=True)
    _assert_parity(full[y0:y0 + th, x0:x0 + tw], sub[y0:y0 + th, x0:x0 + tw], rgb_o, sub_o, "cubes/mis 1080p crop")


def test_c3_cubes_mis_vs_nee_same_seed(rt, gpu_scenes):
    """MIS on vs off with the same seeds (BASELINE C3): per subpixel, K independent estimates (seeds)
    per mode. The two estimators have the same expectation (frame means within 4 standard errors) and
    the per-pixel variance ratio MIS/NEE is reported (whole frame and per 16x16 block)."""
    s = gpu_scenes["cubes"]
    w, h, spp, K = 128, 96, 32, 16
    est = {}
    for mis in (False, True):
        subs = [rt.render(s, w, h, spp, SEED + 1000 + k, want_sub=True, megakernel=True, mis=mis)[1] for k in range(K)]
        est[mis] = np.stack(subs)  # [K, h, w, 4, 3] subpixel means (before the clamp)
    m0, m1 = est[False].mean(axis=0), est[True].mean(axis=0)
    v0, v1 = est[False].var(axis=0, ddof=1), est[True].var(axis=0, ddof=1)
    n = K * h * w * 4
    se = np.sqrt((v0.sum(axis=(0, 1, 2)) + v1.sum(axis=(0, 1, 2))) / n ** 2 * K)  # per channel
    diff = m1.mean(axis=(0, 1, 2)) - m0.mean(axis=(0, 1, 2))
    ratio = float(v1.mean() / v0.mean())
    B = 16
    bv0 = v0.mean(axis=(2, 3)).reshape(h // B, B, w // B, B).mean(axis=(1, 3))
    bv1 = v1.mean(axis=(2, 3)).reshape(h // B, B, w // B, B).mean(axis=(1, 3))
    block = bv1 / np.maximum(bv0, 1e-30)
    _record("c3_mis_vs_nee", {"frame_mean_nee": m0.mean(axis=(0, 1, 2)).tolist(),
                              "frame_mean_mis": m1.mean(axis=(0, 1, 2)).tolist(), "se": se.tolist(),
                              "variance_ratio_mis_over_nee": ratio,
                              "block_ratio_min": float(block.min()), "block_ratio_median": float(np.median(block)),
                              "block_ratio_max": float(block.max()), "K": K, "spp": spp, "size": [w, h]})
    assert np.all(np.abs(diff) <= 4 * se + 1e-12), (diff, se)
    assert ratio < 1.0  # measured 0.917 (blocks 0.71 .. 1.00) on the first run, profiles/r02_c3_mis_vs_nee.json


C5_W = C5_H = 4096
C5_RANKS = 8


def _share(rank):
    """bench.partition's interleaved share of rank `rank` of 8: (y0, rows, row_step)."""
    return rank, (C5_H - rank + C5_RANKS - 1) // C5_RANKS, C5_RANKS


def test_c5_unicorn_share_against_oracle(rt, gpu_scenes, oracle_scenes):
    s, o = gpu_scenes["flying_unicorn"], oracle_scenes["flying_unicorn"]
    y0, th, step = _share(3)
    rgb, sub, st = rt.render(s, C5_W, C5_H, 4, SEED, tile=(0, y0, C5_W, th), row_step=step, megakernel=True,
                             want_sub=True)
    assert st["samples"] == C5_W * th * 4 and rgb.shape == (th, C5_W, 3)
    # crops of the share: share rows i0..i0+nr are screen rows y0 + i * 8 (the unicorn is near the centre)
    for (x0, i0, tw, nr) in [(2000, 250, 24, 6), (1500, 180, 24, 6), (0, 0, 16, 4), (4080, 508, 16, 4)]:
        rows = [o.render(C5_W, C5_H, 4, SEED, tile=(x0, y0 + (i0 + i) * step, tw, 1)) for i in range(nr)]
        rgb_o = np.concatenate([r[0] for r in rows])
        sub_o = np.concatenate([r[1] for r in rows])
        _assert_parity(rgb[i0:i0 + nr, x0:x0 + tw], sub[i0:i0 + nr, x0:x0 + tw], rgb_o, sub_o, f"C5 share crop {x0},{i0}")


def test_c5_shares_assemble_to_single_frame(rt, gpu_scenes):
    """The 8 interleaved shares (one per GPU in the C5 run) put back in row order equal one
    single-call render of the frame byte for byte; so does rt_render_multi (host-side band handout,
    two workers on this one device, sharing the scene)."""
    s = gpu_scenes["flying_unicorn"]
    full, _, _ = rt.render(s, C5_W, C5_H, 4, SEED, megakernel=True)
    frame = np.zeros_like(full)
    for r in range(C5_RANKS):
        y0, th, step = _share(r)
        part, _, _ = rt.render(s, C5_W, C5_H, 4, SEED, tile=(0, y0, C5_W, th), row_step=step, megakernel=True)
        frame[y0::step] = part
    assert np.array_equal(frame, full)
    multi, st = rt.render_multi(s, C5_W, C5_H, 4, [0, 0], SEED, band_rows=256)
    assert np.array_equal(multi, full) and st["samples"] == C5_W * C5_H * 4
