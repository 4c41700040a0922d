"""Every BASELINE.json config on one GPU (one process): Msamples/s per config, device time.

python tools/configs_bench.py [--quick] [--fp32] [--json]
  --fp32  the f32 perf mode
  --json  one bench-style JSON line per config instead of the text line: value, roofline (SURVEY §8(d):
          88 B per camera sample + 280 B per path vertex over the device time; for mesh scenes also the
          scene bytes touched, 32 B per parent visit + 8 B per leaf + (4 + 36) B per triangle test, from
          the walk counters of the diagnostic build lib/variants/dbg.so run in a subprocess on the same workload;
          the compute block and the measured traffic (2 x FETCH_SIZE + WRITE_SIZE) from the newest committed PMC
          summary of exactly this workload, profiles/<round>_pmc_<scene>_<W>x<H>x<SPP>[_mis].json, else of the
          scene at another size, scaled per sample and labelled)
          and cpu_baseline (the config's line in profiles/r03_cpu_configs.log, tools/cpu_configs.py)
C5 is 4096x4096 at 64 of its 4096 spp on 1 GPU (stated in the line; the per-rank share at full spp is
tools/tail_probe.py share ...)."""
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))
sys.path.insert(0, REPO)
import rt_amd  # noqa: E402

import bench  # noqa: E402  (compute_block, constants)

quick = "--quick" in sys.argv
fp32 = "--fp32" in sys.argv
as_json = "--json" in sys.argv
CONFIGS = [
    # (label, scene, w, h, spp, mis)
    ("C1 cornell 600x450 1spp (reference plumbing case: black frame)", "cornell_box", 600, 450, 1, False),
    ("C1' cornell 600x450 4spp", "cornell_box", 600, 450, 4, False),
    ("C2 cornell 1920x1080 256spp MIS on", "cornell_box", 1920, 1080, 256, True),
    ("C2' cornell 1920x1080 256spp MIS off", "cornell_box", 1920, 1080, 256, False),
    ("C3 cubes 1920x1080 1024spp MIS off", "cubes", 1920, 1080, 1024, False),
    ("C3 cubes 1920x1080 1024spp MIS on", "cubes", 1920, 1080, 1024, True),
    ("C4 unicorn 1920x1080 512spp", "flying_unicorn", 1920, 1080, 512, False),
    ("C5 unicorn 4096x4096 (64 of 4096 spp, 1 GPU)", "flying_unicorn", 4096, 4096, 64, False),
]

_WALK_SCRIPT = r"""
import ctypes, json, os, sys
sys.path.insert(0, os.path.join(os.environ["RT_REPO"], "raytracer-server_amd"))
import rt_amd
s = rt_amd.Scene.from_toml(os.path.join(os.environ["RT_REPO"], "scenes", sys.argv[1] + ".toml"))
c = (ctypes.c_ulonglong * 16)()
rt_amd.render(s, 64, 48, 4, megakernel=True)
rt_amd.lib.rt_debug_counters(c)
_, _, st = rt_amd.render(s, int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[5]), megakernel=True, mis=sys.argv[4] == "1")
rt_amd.lib.rt_debug_counters(c)
print(json.dumps({"calls": c[0], "parent_visits": c[2], "leaves": c[3], "tri_tests": c[4], "vertices": st["vertices"],
                  "samples": st["samples"]}))
"""


def walk_counters(scene, w, h, mis, spp):
    """Per-vertex octree walk counters of the diagnostic build on the same workload (None if it is not built)."""
    lib = os.path.join(REPO, "raytracer-server_amd", "lib", "variants", "dbg.so")
    if not os.path.exists(lib):
        return None
    env = dict(os.environ, RT_AMD_LIB=lib, RT_REPO=REPO)
    out = subprocess.run([sys.executable, "-c", _WALK_SCRIPT, scene, str(w), str(h), "1" if mis else "0", str(spp)], env=env,
                         capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        return None
    return json.loads(out.stdout.strip().splitlines()[-1])


def _round_key(f):
    """Sort key of profiles/r<NN><tag>_pmc_*.json files: newest round, then newest tag, last (tags run a..z,
    then aa..az: a longer tag is newer)."""
    b = os.path.basename(f)
    tag = b.split("_pmc_")[0][3:]
    return (b[1:3], len(tag), tag, b)


def pmc_summary(scene, w, h, spp, mis):
    """The newest committed PMC summary (tools/pmc_report.py) of exactly this workload, else of the scene's
    megakernel at another size: (summary, path, exact)."""
    tag = f"{scene}_{w}x{h}x{spp}{'_mis' if mis else ''}"
    exact = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_{tag}.json")), key=_round_key)
    pat = os.path.join(REPO, "profiles", f"r*_pmc_{scene}_*{'_mis' if mis else ''}.json")
    other = sorted((f for f in glob.glob(pat) if mis or "_mis" not in os.path.basename(f)), key=_round_key)
    for files, is_exact in ((exact, True), (other, False)):
        for f in reversed(files):
            try:
                with open(f) as fh:
                    d = json.load(fh)
            except (OSError, ValueError):
                continue
            if d.get("valu_mix"):
                return d, os.path.relpath(f, REPO), is_exact
    return None, None, False


def cpu_rates():
    try:
        with open(os.path.join(REPO, "profiles", "r03_cpu_configs.log")) as f:
            return {d["config"]: d for d in (json.loads(x) for x in f if x.startswith("{"))}
    except (OSError, ValueError):
        return {}


scenes = {}
cpu = cpu_rates() if as_json else {}
for label, name, w, h, spp, mis in CONFIGS:
    if quick:
        spp = max(1, spp // 16) if spp > 4 else spp
    if name not in scenes:
        scenes[name] = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{name}.toml"))
    # the same render once untimed first: the kernel's code object loads on its first launch and the workspace
    # (subpixel means, split-tail scratch) is allocated for the frame's size, both inside the first render's events
    rt_amd.render(scenes[name], w, h, spp, megakernel=True, mis=mis, fp32=fp32)
    t = time.perf_counter()
    rgb, _, st = rt_amd.render(scenes[name], w, h, spp, megakernel=True, mis=mis, fp32=fp32)
    wall = time.perf_counter() - t
    n = st["samples"]
    rate = n / st["device_ms"] / 1e3 if st["device_ms"] > 0 and n else 0.0
    if not as_json:
        print(f"{label}{' [f32]' if fp32 else ''}: spp {spp}, {n} samples, {st['device_ms']:.1f} ms device, {wall*1e3:.1f} ms wall, "
              f"{rate:.1f} Msamples/s, {st['vertices'] / max(1, n):.3f} vertices/sample, mean RGB8 {rgb.mean():.2f}",
              flush=True)
        continue
    if n == 0:
        print(json.dumps({"config": label, "value": 0.0, "unit": "Msamples/s", "note": "spp/4 = 0: no samples"}), flush=True)
        continue
    sec = st["device_ms"] / 1e3
    line = {"metric": f"Msamples/sec {name} {w}x{h}x{spp}spp{' mis' if mis else ''}", "config_label": label,
            "value": round(rate, 3), "unit": "Msamples/s", "n_gpus": 1, "higher_is_better": True,
            "dtype": "f32" if fp32 else "f64", "data": "synthetic: reference scene file + counter-based RNG, seed 0x5eed",
            "config": {"workload": f"{name} {w}x{h}x{spp}spp", "scene": f"scenes/{name}.toml", "width": w, "height": h,
                       "spp": spp, "mis": mis, "mode": "megakernel" + ("-f32" if fp32 else ""),
                       "vertices": st["vertices"], "vertices_per_sample": round(st["vertices"] / n, 4),
                       "device_ms": round(st["device_ms"], 3)},
            }
    pmc, src, exact = pmc_summary(name, w, h, spp, mis) if not fp32 else (None, None, False)
    # only a PMC summary of exactly this workload prices the roofline (FP64 FLOP per vertex, measured traffic)
    mix = dict(pmc["valu_mix"], waits=pmc.get("waits"), source=pmc.get("kernel") or "") if (pmc and exact) else None
    hbm = pmc.get("hbm") if (pmc and exact) else None
    line["roofline"] = bench.roofline_block(
        mix, src, st["vertices"], n, st["device_ms"], hbm["bytes"] if hbm else None,
        f"{src}: 2 x FETCH_SIZE + WRITE_SIZE of this workload's launch", "k_megakernel", None,
        "valu_issue_f64" if not fp32 else "valu_issue_f32")
    if name != "cornell_box" and not fp32:
        wc = walk_counters(name, w, h, mis, spp)
        if wc and wc["vertices"] and wc["calls"] and not (wc["parent_visits"] or wc["leaves"] or wc["tri_tests"]):
            # flat meshes (the cubes): flat_query reads its mesh's triangles through scalar loads, outside the walk
            # counters, so the octree model has nothing to count
            line["roofline"]["scene_bytes"] = None
            line["roofline"]["scene_bytes_note"] = ("not applicable: every mesh is a flat octree, queried by flat_query "
                                                    "(scalar loads of <= 32 triangles per mesh), not walked")
        elif wc and wc["vertices"] and wc["calls"]:
            per_v = {k: wc[k] / wc["vertices"] for k in ("calls", "parent_visits", "leaves", "tri_tests")}
            sb_v = 32 * per_v["parent_visits"] + 8 * per_v["leaves"] + 40 * per_v["tri_tests"]
            line["roofline"]["scene_bytes"] = {
                "model": "SURVEY 8(d): 32 B per parent visit + 8 B per leaf + (4 + 36) B per triangle test (LDS / L2 / MALL, "
                         "not HBM)",
                "per_vertex": round(sb_v, 2), "GBps": round(sb_v * st["vertices"] / sec / 1e9, 2),
                "walks_per_vertex": round(per_v["calls"], 4),
                "per_walk": {k: round(wc[k] / max(1, wc["calls"]), 3) for k in ("parent_visits", "leaves", "tri_tests")},
                "source": "walk counters of lib/variants/dbg.so (RT_DEBUG_COUNTERS) on this workload"}
    if pmc:
        rf = line["roofline"]
        rf["compute"] = bench.compute_block(pmc["valu_mix"], st["vertices"], st["device_ms"])
        rf["compute"]["source"] = src if exact else f"{src} (another size of this scene: per-vertex mix only)"
        rf["compute"]["kernel"] = pmc.get("kernel")
        if pmc.get("waits"):
            rf["compute"]["simd_valu_busy"] = round(pmc["waits"]["simd_valu_busy"], 4)
            rf["compute"]["wait_any"] = round(pmc["waits"]["wait_any"], 4)
        if exact and pmc.get("l2_hit_rate") is not None:
            rf["l2_hit_rate"] = round(pmc["l2_hit_rate"], 4)
    c = cpu.get(label.split(" (")[0]) or next((v for k, v in cpu.items() if k.startswith(label.split(" (")[0])), None)
    if c:
        line["cpu_baseline"] = {"value": c["all_cores"]["Msamples_per_s"], "unit": "Msamples/s", "cores": c["cores"],
                                "kind": c["kind"], "sample": c["all_cores"]["sample"],
                                "single_thread": c["one_thread"], "source": "profiles/r03_cpu_configs.log"}
    print(json.dumps(line), flush=True)
