"""The single-precision mesh cull (path_f64.h near_mesh32) passes every ray the f64
near_box passes: compiled and run on the host over 3 x 400k random rays at the reference scenes' mesh
boxes (half grazing a face within the f64 pad, some with axis-parallel direction components).
Round 3 ran 3 x 20M the same way: 0 rays culled by the f32 test that the f64 test passes."""
import os
import subprocess

from conftest import REPO


def test_near32_never_culls_what_near_box_passes(tmp_path):
    exe = str(tmp_path / "near32_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                    os.path.join(REPO, "tests", "near32_check.cpp")], check=True)
    out = subprocess.run([exe, "400000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "f64-pass-but-f32-cull 0" in out.stdout, out.stdout
