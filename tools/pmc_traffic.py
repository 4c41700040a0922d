"""roofline.traffic for bench.py: HBM bytes per launch of the render kernel from the FETCH_SIZE and
WRITE_SIZE passes (separate rocprofv3 runs of `bench.py --steps 1 --warmup 0 --no-cpu-baseline`,
tools/gpu_task.sh benchpmc), merged into a JSON map {workload key: bytes}.

usage: python tools/pmc_traffic.py <fetch run_counter_collection.csv> <write ...csv> <key> [kernel-substring]
                                   [--out profiles/pmc_traffic.json]

Per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
counts half the bytes of wide reads, so it is doubled. The bench runs one untimed stats render before
its steps, so the LAST dispatch of the kernel in each pass is the timed step's. A value implying more
than the HBM peak over the dispatch's own duration is a counter fault and is refused.
"""
import csv
import json
import os
import sys

PEAK = 8.0e12


def last_value(path, kernel, counter):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not rows:
        raise SystemExit(f"{path}: no {counter} rows for {kernel}")
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    r = rows[-1]
    return float(r["Counter_Value"]) * 1024.0, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
        args.remove(out)
    fetch_csv, write_csv, key = args[0], args[1], args[2]
    kernel = args[3] if len(args) > 3 else "k_megakernel"
    fetch, t_f = last_value(fetch_csv, kernel, "FETCH_SIZE")
    write, t_w = last_value(write_csv, kernel, "WRITE_SIZE")
    fetch *= 2.0
    total = fetch + write
    rate = max(fetch / t_f, write / t_w)
    print(f"{key}: {kernel}: FETCH x2 {fetch / 1e6:.1f} MB ({t_f * 1e3:.1f} ms) + WRITE {write / 1e6:.1f} MB "
          f"({t_w * 1e3:.1f} ms) = {total / 1e6:.1f} MB per launch")
    if rate > PEAK:
        raise SystemExit("refused: above the HBM peak, counter fault")
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[key] = int(total)
    json.dump(d, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
