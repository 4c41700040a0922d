"""Summarise rocprofv3 SQ counter passes (gpurun_out/pmc*/run_counter_collection.csv) for one kernel."""
import csv, glob, sys, collections
pat = sys.argv[1] if len(sys.argv) > 1 else "megakernel"
d = collections.defaultdict(float)
for f in sorted(glob.glob("gpurun_out/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r.get("Kernel_Name", ""):
            d[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(d): print(f"{k:28s} {d[k]:.4g}")
if d.get("SQ_ACTIVE_INST_VALU"):
    print("lane utilisation (THREAD_CYCLES_VALU / (64*ACTIVE_INST_VALU)):", d["SQ_THREAD_CYCLES_VALU"] / (64 * d["SQ_ACTIVE_INST_VALU"]))
    print("SALU/VALU instr:", d["SQ_INSTS_SALU"] / d["SQ_INSTS_VALU"])
    print("wait_any / wave_cycles:", d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"])
