"""Per-kernel time and PMC HBM traffic from tools/gpu_wf_pmc.sh outputs (FETCH_SIZE x2 per the gfx950 note)."""
import collections
import csv
import re


def kname(s):
    m = re.search(r"(k_\w+|__amd_\w+)", s)
    return m.group(1) if m else s[:40]

t = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open("gpurun_out/wf_trace/run_kernel_trace.csv")):
    n = kname(r["Kernel_Name"])
    t[n][0] += 1
    t[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
f = collections.defaultdict(float)
w = collections.defaultdict(float)
for fn, d in [("gpurun_out/wf_fetch/run_counter_collection.csv", f), ("gpurun_out/wf_write/run_counter_collection.csv", w)]:
    for r in csv.DictReader(open(fn)):
        n = kname(r["Kernel_Name"])
        d[n] += float(r["Counter_Value"]) * 1024
for n, (c, ms) in sorted(t.items(), key=lambda x: -x[1][1]):
    fb, wb = 2 * f[n], w[n]
    rate = (fb + wb) / (ms / 1e3) / 1e9 if ms else 0.0
    print(f"{n:28s} calls {c:5d} {ms:9.2f} ms  fetch(x2) {fb / 1e9:8.3f} GB  write {wb / 1e9:8.3f} GB  -> {rate:8.1f} GB/s")
