"""f32 perf mode vs the f64 path on the GPU (same seed): the statistics the parity test bounds.
The f64 GPU path equals the CPU oracle to 1e-9 (tests/test_gpu_parity.py), so it stands in for it
here; the test itself compares against the oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
import rt_amd  # noqa: E402


def stats(name, w, h, spp, mis=False):
    sc = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{name}.toml"))
    mesh = name == "flying_unicorn" or name == "cubes"
    rgb_d, sub_d, st_d = rt_amd.render(sc, w, h, spp, 0x5EED, mis=mis, megakernel=True, want_sub=True,
                                       mesh_nearest=mesh)
    rgb_f, sub_f, st_f = rt_amd.render(sc, w, h, spp, 0x5EED, mis=mis, want_sub=True, fp32=True)
    cd = np.clip(sub_d, 0, 1).mean(axis=2)  # clamped subpixel means averaged: pixel values (server.rs:360)
    cf = np.clip(sub_f, 0, 1).mean(axis=2)
    m_d, m_f = cd.mean(axis=(0, 1)), cf.mean(axis=(0, 1))
    diff = rgb_f.astype(int) - rgb_d.astype(int)
    same = np.all(diff == 0, axis=-1).mean()
    close = np.all(np.abs(diff) <= 1, axis=-1).mean()
    # 16x16 block means of the pixel values, paired difference vs its standard error
    B = 16
    hb, wb = h // B, w // B
    dd = (cf - cd)[:hb * B, :wb * B].reshape(hb, B, wb, B, 3)
    bm = dd.mean(axis=(1, 3))
    se = dd.std(axis=(1, 3)) / B
    z = np.abs(bm) / np.maximum(se, 1e-12)
    rel_blk = np.abs(bm) / np.maximum(cd[:hb * B, :wb * B].reshape(hb, B, wb, B, 3).mean(axis=(1, 3)), 1e-3)
    print(f"{name:15s} {w}x{h}x{spp} mis={mis}: mean rel diff {np.abs(m_f / m_d - 1).max():.5f}; RGB8 same "
          f"{same:.4f}, |d|<=1 {close:.4f}, mean|d| {np.abs(diff).mean():.3f}; block z max {z.max():.2f} "
          f"(>4: {(z > 4).mean():.4f}), block rel max {rel_blk.max():.4f}; vertices/sample f64 "
          f"{st_d['vertices'] / st_d['samples']:.3f} f32 {st_f['vertices'] / st_f['samples']:.3f}", flush=True)


if __name__ == "__main__":
    stats("cornell_box", 192, 144, 64)
    stats("cornell_box", 192, 144, 64, mis=True)
    stats("cubes", 192, 144, 64)
    stats("cubes", 192, 144, 64, mis=True)
    stats("flying_unicorn", 192, 144, 64)
    stats("cornell_box", 480, 270, 1024)
