"""Summarise the counter passes of `tools/gpu_task.sh pmc:SCENE:W:H:SPP` for the render kernel.

usage: python tools/pmc_report.py gpurun_out/<TAG> <key> [kernel-substring] [--out profiles/<file>.json]
                                  [--valu-key "<scene> <mode>" --valu-out profiles/pmc_valu.json]
(--pmc-file profiles/<name>.json records, in that map entry, the committed summary the mix comes from;
--valu-key merges the per-vertex instruction mix into the map bench.py's roofline.compute reads)

Per MI355X_MICROARCH.md:
  * HBM bytes = 2 x FETCH_SIZE (gfx950 counts half the bytes of wide reads) + WRITE_SIZE, both KiB;
  * L2 hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum);
  * effective clock = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / the dispatch's duration
    (Start/End timestamps of the same pass);
  * VALU issue occupancy: wave-instructions priced per class on a SIMD-32 (a wave64 instruction
    occupies its SIMD for 2 cycles at full rate): f64 add/mul/fma 4 cycles (FP64 vector = half the
    FP32 rate, 78.6 vs 157.3 TF), f64 transcendentals 8, 64-bit integer 4, every other VALU
    instruction 2 — over 1024 SIMDs x clock x duration;
  * FP64 FLOP rate = (ADD_F64 + MUL_F64 + 2 FMA_F64) x 64 x lane utilisation / duration, against
    78.6 TFLOP/s. Lane utilisation = SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU).
The measured dispatch is the LAST one of the kernel in each pass (tools/prof_render.py warms up
first). The path-vertex count comes from the `*_plain.log` line of the same workload.
"""
import csv
import glob
import json
import os
import re
import sys

COST = {"f64": 4, "trans_f64": 8, "int64": 4, "other": 2}
N_SIMD = 1024
FP64_PEAK = 78.6e12
HBM_PEAK = 8.0e12


def last_dispatch(path, kernel):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"{path}: no rows for {kernel}")
    last = max(int(r["Dispatch_Id"]) for r in rows)
    rows = [r for r in rows if int(r["Dispatch_Id"]) == last]
    vals = {r["Counter_Name"]: float(r["Counter_Value"]) for r in rows}
    dur_ns = int(rows[0]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    return vals, dur_ns, rows[0]["Kernel_Name"]


def report(d, key, kernel):
    c = {}
    durs = {}
    name = None
    for f in sorted(glob.glob(os.path.join(d, f"{key}_*", "run_counter_collection.csv"))):
        p = os.path.basename(os.path.dirname(f))[len(key) + 1:]
        v, dur, name = last_dispatch(f, kernel)
        c.update(v)
        durs[p] = dur
    plain = open(os.path.join(d, f"{key}_plain.log")).read()
    m = re.search(r"samples (\d+), vertices (\d+)", plain)
    samples, vertices = (int(m.group(1)), int(m.group(2))) if m else (None, None)
    if m is None:  # older log format: vertices/sample to 3 digits
        w, h, spp = (int(x) for x in re.search(r"(\d+)x(\d+)x(\d+)", plain).groups())
        samples = w * h * 4 * (spp // 4)
        vertices = int(float(re.search(r"([\d.]+) vertices/sample", plain).group(1)) * samples)
    dev_ms = float(re.search(r"([\d.]+) ms device", plain).group(1))
    dur = durs.get("fetch") or next(iter(durs.values()))
    out = {"workload": key, "kernel": name.split("(")[0], "unprofiled_device_ms": dev_ms,
           "profiled_kernel_ms": dur / 1e6, "samples": samples, "vertices": vertices}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch, write = 2 * 1024 * c["FETCH_SIZE"], 1024 * c["WRITE_SIZE"]
        out["hbm"] = {"fetch_bytes_x2": fetch, "write_bytes": write, "bytes": fetch + write,
                      "GBps": (fetch + write) / dur, "frac_of_8TBps": (fetch + write) / dur * 1e9 / HBM_PEAK}
    if "TCC_HIT_sum" in c:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        out["l2_requests"] = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
    if "GRBM_GUI_ACTIVE" in c:
        out["clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / dur
    if "SQ_INSTS_VALU" in c and "SQ_INSTS_VALU_FMA_F64" in c and "SQ_INSTS_VALU_INT64" in c:
        f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_FMA_F64"]
        tr = c["SQ_INSTS_VALU_TRANS_F64"]
        i64 = c["SQ_INSTS_VALU_INT64"]
        other = c["SQ_INSTS_VALU"] - f64 - tr - i64
        cyc = f64 * COST["f64"] + tr * COST["trans_f64"] + i64 * COST["int64"] + other * COST["other"]
        clk = out.get("clock_GHz", 2.1)
        lanes = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
        flops = (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2 * c["SQ_INSTS_VALU_FMA_F64"]) * 64 * lanes
        out["valu"] = {
            "insts": c["SQ_INSTS_VALU"], "f64_add_mul_fma": f64, "f64_trans": tr, "int64": i64, "other": other,
            "int32": c.get("SQ_INSTS_VALU_INT32"), "cvt": c.get("SQ_INSTS_VALU_CVT"),
            "salu": c.get("SQ_INSTS_SALU"), "lds": c.get("SQ_INSTS_LDS"), "smem": c.get("SQ_INSTS_SMEM"),
            "vmem": c.get("SQ_INSTS_VMEM"),
            "lane_utilisation": lanes, "issue_cycles": cyc, "cost_model_cycles": COST,
            "issue_frac": cyc / (N_SIMD * clk * dur),
            "fp64_tflops": flops / dur / 1e3, "fp64_frac": flops / (dur * 1e-9) / FP64_PEAK,
            "per_vertex": c["SQ_INSTS_VALU"] / vertices if vertices else None,
            "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"] if "SQ_WAVE_CYCLES" in c else None,
        }
        if vertices:
            out["valu_mix"] = {
                "per_vertex": {"f64": f64 / vertices, "trans_f64": tr / vertices, "int64": i64 / vertices,
                               "other": other / vertices},
                "fp64_flops_per_vertex": flops / vertices, "lane_utilisation": lanes, "clock_GHz": clk,
                "source": f"SQ PMC passes of tools/gpu_task.sh pmc:{key} (tools/pmc_report.py)"}
    if "SQ_WAIT_INST_LDS" in c and "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        # SQ cycle counters tick once per 4 cycles: resident waves per SIMD = 4 WAVE_CYCLES / (SIMDs x cycles)
        clk = out.get("clock_GHz") or 2.4
        wps = 4 * wc / (N_SIMD * clk * dur)
        out["waits"] = {  # fractions of the waves' resident cycles (pmcw passes)
            "waves_per_simd": wps, "clock_GHz_assumed": None if "clock_GHz" in out else clk,
            "wait_any": c["SQ_WAIT_ANY"] / wc, "wait_inst_any": c["SQ_WAIT_INST_ANY"] / wc,
            "wait_inst_lds": c["SQ_WAIT_INST_LDS"] / wc,
            "active_valu": c["SQ_ACTIVE_INST_VALU"] / wc, "active_salu": c["SQ_ACTIVE_INST_SCA"] / wc,
            "active_lds": c["SQ_ACTIVE_INST_LDS"] / wc, "active_vmem": c["SQ_ACTIVE_INST_VMEM"] / wc,
            # the SIMD's view: the share of its cycles with a VALU (SALU) instruction of some wave executing
            "simd_valu_busy": c["SQ_ACTIVE_INST_VALU"] / wc * wps, "simd_salu_busy": c["SQ_ACTIVE_INST_SCA"] / wc * wps,
            "lds_bank_conflict_cycles": c.get("SQ_LDS_BANK_CONFLICT", 0) / wc if "SQ_LDS_BANK_CONFLICT" in c else None,
            "source": "SQ_WAIT_ANY: a wave waiting on a dependency (s_waitcnt: memory / LDS / scalar loads); "
                      "SQ_WAIT_INST_ANY: a wave with a ready instruction waiting to issue (another wave holds the "
                      "unit); SQ_ACTIVE_INST_VALU: cycles a wave's VALU instruction executes"}
    return out


def main():
    args, skip = [], False
    for a in sys.argv[1:]:
        if skip:
            skip = False
        elif a.startswith("--"):
            skip = True
        else:
            args.append(a)
    d, key = args[0], args[1]
    kernel = args[2] if len(args) > 2 else "megakernel"
    r = report(d, key, kernel)
    if "waits" in r and "valu_mix" in r:
        r["valu_mix"]["waits"] = {k: r["waits"][k] for k in ("simd_valu_busy", "simd_salu_busy", "wait_any",
                                                              "wait_inst_any", "waves_per_simd")}
    print(json.dumps(r, indent=1))
    if "--out" in sys.argv:
        path = sys.argv[sys.argv.index("--out") + 1]
        json.dump(r, open(path, "w"), indent=1)
    if "--valu-key" in sys.argv and "valu_mix" in r:
        vk = sys.argv[sys.argv.index("--valu-key") + 1]
        path = sys.argv[sys.argv.index("--valu-out") + 1] if "--valu-out" in sys.argv else os.path.join(
            os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_valu.json")
        m = json.load(open(path)) if os.path.exists(path) else {}
        m[vk] = r["valu_mix"]
        if "--pmc-file" in sys.argv:  # the committed summary this mix came from (bench.py's roofline names it)
            m[vk]["pmc_file"] = sys.argv[sys.argv.index("--pmc-file") + 1]
        json.dump(m, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
