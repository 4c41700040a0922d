"""CPU baseline for every BASELINE.json config ("CPU Msamples/s next to the GPU number
for every config"): the CPU oracle (oracle/oracle.cpp, a line-by-line f64 restatement of the
reference's sample loop; the Rust reference cannot be built here) compiled for this host
(-O3 -march=native), timed on a bounded row band of each config's frame at reduced spp, on every
core this job may use (bench.host_cores()) and on 1 thread (the reference renders a job on one
task, server.rs:157-199). Cost is linear in spp and in rows, so the rate at reduced spp is the
config's rate; the spp used is stated per line.

python tools/cpu_configs.py [--seconds S]   (S: target seconds per all-core sample, default 8)
Prints one JSON line per config."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import bench  # noqa: E402  (host_cores, native_oracle)

CONFIGS = [
    # (label, scene, w, h, spp, mis, cpu spp)
    ("C1' cornell 600x450 4spp", "cornell_box", 600, 450, 4, False, 4),
    ("C2 cornell 1920x1080 256spp MIS on", "cornell_box", 1920, 1080, 256, True, 16),
    ("C2' cornell 1920x1080 256spp MIS off", "cornell_box", 1920, 1080, 256, False, 16),
    ("C3 cubes 1920x1080 1024spp MIS off", "cubes", 1920, 1080, 1024, False, 16),
    ("C3 cubes 1920x1080 1024spp MIS on", "cubes", 1920, 1080, 1024, True, 16),
    ("C4 unicorn 1920x1080 512spp", "flying_unicorn", 1920, 1080, 512, False, 16),
    ("C5 unicorn 4096x4096 4096spp (per-rank share rate = frame rate)", "flying_unicorn", 4096, 4096, 4096, False, 16),
]


def main():
    target = float(sys.argv[sys.argv.index("--seconds") + 1]) if "--seconds" in sys.argv else 8.0
    lib, flags = bench.native_oracle()
    if lib:
        os.environ["RT_ORACLE_LIB"] = lib
    import oracle_bind

    cores, source = bench.host_cores()
    scenes = {}
    for label, name, w, h, spp, mis, cspp in CONFIGS:
        if name not in scenes:
            scenes[name] = oracle_bind.OracleScene(os.path.join(REPO, "scenes", f"{name}.toml"))
        sc = scenes[name]
        res = {"config": label, "scene": name, "width": w, "height": h, "spp": spp, "mis": mis, "cpu_spp": cspp,
               "cores": cores, "cores_source": source, "host_cpus_visible": os.cpu_count(),
               "kind": "port", "compiler": f"g++ {flags}"}
        for threads, key, budget in ((cores, "all_cores", target), (1, "one_thread", target / 2)):
            rows = 2
            while True:  # grow the band until a sample takes about `budget` seconds (middle rows of the frame)
                rows = min(rows, h)
                y0 = (h - rows) // 2
                t0 = time.perf_counter()
                sc.render(w, h, cspp, 0x5EED, tile=(0, y0, w, rows), mis=mis, threads=threads, want_sub=False)
                dt = time.perf_counter() - t0
                if dt >= budget or rows == h:
                    break
                rows = max(rows + 1, int(rows * min(8.0, budget / max(dt, 1e-3))))
            reps = 1
            while dt < budget:  # the whole frame takes less than the budget: render it again until it does not
                t0 = time.perf_counter()
                sc.render(w, h, cspp, 0x5EED, tile=(0, y0, w, rows), mis=mis, threads=threads, want_sub=False)
                dt += time.perf_counter() - t0
                reps += 1
            n = w * rows * 4 * (cspp // 4) * reps
            res[key] = {"Msamples_per_s": round(n / dt / 1e6, 5), "threads": threads,
                        "sample": f"rows {y0}..{y0 + rows} at {cspp} spp x {reps} ({n} samples, {dt:.2f} s)"}
        print(json.dumps(res), flush=True)
    if lib:
        os.unlink(lib)


if __name__ == "__main__":
    main()
