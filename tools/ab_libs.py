"""A/B of library builds on one GPU: python tools/ab_libs.py SCENE W H SPP LIB[,LIB...] [ROUNDS] [extra prof_render args]

Each LIB (a path to a librtamd.so build, e.g. lib/variants/base.so; "main" = lib/librtamd.so; an
optional "@VAR=VAL[+VAR=VAL]" suffix sets RT_* switches for that entry, e.g.
raytracer-server_amd/lib/variants/ab.so@RT_MK_POOL=1 — only the A/B build reads them, ab_knobs.h) renders
the same frame in its own process (tools/prof_render.py under RT_AMD_LIB), ROUNDS times in alternating
order, so clock drift hits every build alike. Prints device time, Msamples/s and the frame's sha1 per
run (identical digests = identical frames), then the median per build."""
import os
import re
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
scene, w, h, spp = sys.argv[1:5]
libs = sys.argv[5].split(",")
rounds = int(sys.argv[6]) if len(sys.argv) > 6 else 2
extra = sys.argv[7:]
rate = {lib: [] for lib in libs}
for r in range(rounds):
    for lib in (libs if r % 2 == 0 else libs[::-1]):
        name, _, sets = lib.partition("@")
        path = os.path.join(REPO, "raytracer-server_amd", "lib", "librtamd.so") if name == "main" else os.path.join(REPO, name)
        env = dict(os.environ, RT_AMD_LIB=path)
        env.update(kv.split("=", 1) for kv in sets.split("+") if kv)
        out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_render.py"), scene, w, h, spp,
                              os.environ.get("AB_MODE", "mk"), *extra],
                             env=env, capture_output=True, text=True, timeout=600)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-400:]
        m = re.search(r"([\d.]+) Msamples/s", line)
        if m:
            rate[lib].append(float(m.group(1)))
        print(f"{lib}: {line}", flush=True)
for lib in libs:
    if rate[lib]:
        print(f"median {lib}: {statistics.median(rate[lib]):.1f} Msamples/s over {len(rate[lib])} runs", flush=True)
