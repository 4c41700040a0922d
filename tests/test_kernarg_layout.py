"""The megakernels read their DevScene and RenderArgs arguments in place in the kernarg segment at fixed
offsets (megakernel_common.h: karg_scene at 0, karg_render_args at 248). The static_assert there checks
only the host-side sizeof / alignof arithmetic; this test reads the code objects' own argument metadata
(the AMDGPU .args notes of every kernel in lib/librtamd.so, no GPU needed) and checks that every kernel
that uses the views really takes a 248-byte DevScene at offset 0 and a RenderArgs at offset 248, so a
reordered or inserted parameter fails here instead of reading garbage scene pointers on the GPU."""
import os
import re
import subprocess

import pytest

from conftest import REPO

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(REPO, "raytracer-server_amd", "lib", "librtamd.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# kernels whose bodies call karg_scene() / karg_render_args() (RT_KARG_VIEW), by mangled-name stem
VIEW_KERNELS = ("k_megakernel_f64", "k_megakernel_mesh_f64", "k_megakernel_roles_f64", "k_megakernel_fpool_f64",
                "k_selftest_tables")
# superseded kernels compiled only into the A/B build (ab_knobs.h: lib/variants/ab.so)
AB_VIEW_KERNELS = ("k_megakernel_flat_f64",)
AB_LIB = os.path.join(REPO, "raytracer-server_amd", "lib", "variants", "ab.so")


def _kernels(tmp_path, lib=LIB):
    if not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("ROCm LLVM tools not installed")
    fb = tmp_path / "fatbin.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, str(fb)], check=True)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert starts, "no offload bundle in librtamd.so"
    out = {}
    for i, s in enumerate(starts):
        part = tmp_path / f"b{i}.bin"
        part.write_bytes(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = tmp_path / f"b{i}.co"
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                               text=True).stdout
        # one kernel per "- .agpr_count" item of amdhsa.kernels: its .args list, then its .name
        for item in notes.split("  - .agpr_count:")[1:]:
            name = re.search(r"^\s+\.name:\s+(\S+)", item, re.M)
            if not name:
                continue
            args = re.findall(r"- (?:\.\w+:.*\n\s+)*?\.offset:\s+(\d+)\n\s+\.size:\s+(\d+)", item)
            out[name.group(1)] = [(int(o), int(z)) for o, z in args]
    return out


@pytest.mark.parametrize("which", ["product", "ab"])
def test_kernarg_views_match_every_megakernel_signature(which, tmp_path):
    if which == "ab" and not os.path.exists(AB_LIB):
        pytest.skip("lib/variants/ab.so not built (make -C raytracer-server_amd ab)")
    ks = _kernels(tmp_path, LIB if which == "product" else AB_LIB)
    stems = VIEW_KERNELS + (AB_VIEW_KERNELS if which == "ab" else ())
    hits = {k: v for k, v in ks.items() if any(re.search(rf"\d{stem}I", k) or re.search(rf"\d{stem}E", k)
                                                for stem in stems)}
    # every megakernel family is present (the library instantiates each), the role-split pool included
    for stem in stems:
        assert any(re.search(rf"\d{stem}[IE]", k) for k in hits), f"no {stem} instance in the code objects"
    if which == "product":  # the superseded kernels are gone from the product library
        assert not any(stem in k for k in ks for stem in AB_VIEW_KERNELS)
    for name, args in hits.items():
        assert "NS_8DevSceneENS_10RenderArgsE" in name, f"{name}: (DevScene, RenderArgs) are not the first two parameters"
        assert args[0] == (0, 248), f"{name}: DevScene at {args[0]} (karg_scene reads offset 0, 248 bytes)"
        assert args[1][0] == 248 and args[1][1] == 176, f"{name}: RenderArgs at {args[1]} (karg_render_args: 248)"
    assert len(hits) >= 20
