"""Derive roofline.traffic (HBM bytes per launch of the render kernel) from the FETCH_SIZE and
WRITE_SIZE passes of tools/gpu_profile.sh and store it in profiles/pmc_traffic.json.

usage: python tools/pmc_traffic.py <fetch run_counter_collection.csv> <write ...csv> <kernel_ms> <key>

Per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
counts half the bytes of wide reads, so it is doubled. The bench runs one untimed stats render before
its steps, so the LAST dispatch of the kernel in each pass is the timed step's. A value implying more
than the HBM peak over the kernel's duration is a counter fault and is refused (r01c recorded one).
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
    return float(rows[-1]["Counter_Value"]) * 1024.0


def main():
    fetch_csv, write_csv, kernel_ms, key = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    kernel = sys.argv[5] if len(sys.argv) > 5 else "k_megakernel_f64"
    fetch = 2.0 * last_value(fetch_csv, kernel, "FETCH_SIZE")
    write = last_value(write_csv, kernel, "WRITE_SIZE")
    total = fetch + write
    rate = total / (kernel_ms / 1e3)
    print(f"{kernel}: FETCH x2 {fetch / 1e6:.1f} MB + WRITE {write / 1e6:.1f} MB = {total / 1e6:.1f} MB per launch, "
          f"{rate / 1e9:.2f} GB/s over {kernel_ms:.1f} ms")
    if rate > PEAK:
        raise SystemExit("refused: above the HBM peak, counter fault")
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[key] = int(total)
    json.dump(d, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
