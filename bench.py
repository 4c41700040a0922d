"""Headline benchmark: Msamples/s of the path-tracing hot path on cornell_box 1920x1080x1024spp.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 launched by
torch.distributed.run, one rank per GPU. A step = one full render of the frame (scene resident in
HBM) with the RGB8 rows copied to the host and gathered to rank 0 there: rank r renders the
interleaved rows r, r+N, r+2N, ... of the frame (rt_render_params.row_step = N: every rank gets the
same mix of cheap and expensive rows; --partition stripes gives contiguous stripes). The process
group is gloo (host): the gather, the barriers and the max-over-ranks timing run over it, so no
RCCL collective is on the data path (north_star: "tiles gathered on the host"). Total work is
fixed: scaling = "strong". Rank 0 prints one JSON line.

roofline (dominant kernel = the render megakernel; kernel_ms = its average device time per launch,
HIP events recorded on the stream the kernel runs on). The megakernels keep every path in registers and
read a scene of a few KB (cornell) from cache, so HBM does not bind them; f64 VALU issue does
(the wait breakdown). The top-level fields therefore price the kernel against the FP64
vector peak, every figure measured (roofline_block()):
  * bound "fp64_valu": achieved = FP64 TFLOP/s of this run = the PMC-measured FP64 FLOP per path vertex
    of this exact command (profiles/pmc_valu.json: (ADD_F64 + MUL_F64 + 2 FMA_F64) x 64 x lane
    utilisation, tools/pmc_report.py) x this run's vertices (device counter) / kernel_ms; peak 78.6
    TFLOP/s (MI355X FP64 vector); frac = achieved / peak, in [0, 1]. simd_valu_busy (SQ_ACTIVE_INST_VALU x
    waves per SIMD, the SIMD's own VALU-busy share) stands beside it: an f64 path tracer also issues
    integer, compare, select and 64-bit move VALU work, so the FP64 fraction alone understates how
    full the VALU is;
  * traffic = the HBM bytes the PMC counters measured for one launch of this exact command
    (profiles/pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE, separate rocprofv3 passes over
    `bench.py --steps 1 --warmup 0`, tools/gpu_task.sh benchpmc), scaled to this rank's rows; null
    when no measurement exists; hbm.frac = traffic / kernel_ms / 8 TB/s;
  * wavefront_model: SURVEY §8(d)'s HBM model, 88 B per camera sample + 280 B per path vertex (the f32
    SoA wavefront's state traffic) over kernel_ms; its frac can exceed 1 (a kernel that keeps paths in
    registers beats the model), so it is a comparison, never the roofline fraction;
    model_ceiling_Msamples = 8 TB/s / (88 + 280 V), V = vertices per sample;
  * minimum_bytes_per_launch = the megakernel's own unavoidable traffic: the f64 subpixel means
    written (4 x 3 x 8 B per pixel) and read back by the finalize, plus the RGB8 frame;
  * compute = the instruction-class issue model (f64 add/mul/fma 4 cycles per wave64 instruction,
    f64 transcendental 8, 64-bit integer 4, other VALU 2) and the wait breakdown.
Without a PMC mix for the workload (wavefront mode, f32, an unprofiled size) the line falls back to
bound "hbm" with the measured traffic (or null), never the model.

cpu_baseline: the CPU oracle (a line-by-line f64 restatement of the reference's sample loop; the
reference itself is Rust and cannot be built here), compiled on this host with -O3 -march=native,
on a bounded row band of the same frame on every core this job may use (host_cores(): the cgroup CPU
quota, else the pool's declared share OMP_NUM_THREADS, else the affinity mask; os.cpu_count() is
reported beside it), and on 1 thread; rank 0 at N = 1 only.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))

HBM_PEAK_GBS = 8000.0
FP64_PEAK_TFLOPS = 78.6
N_SIMD = 1024
BYTES_PER_SAMPLE = 88
BYTES_PER_VERTEX = 280
VALU_COST = {"f64": 4, "trans_f64": 8, "int64": 4, "other": 2}  # cycles per wave64 instruction on a SIMD-32


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell_box")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    ap.add_argument("--mode", choices=["megakernel", "wavefront"], default=os.environ.get("RT_BENCH_MODE", "megakernel"))
    ap.add_argument("--mis", action="store_true")
    ap.add_argument("--fp32", action="store_true",
                    help="f32 perf mode (RT_FLAG_FP32, statistical parity only; not the headline f64 number)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=120)
    ap.add_argument("--cpu-spp", type=int, default=256)
    ap.add_argument("--cpu-rows-1t", type=int, default=4, help="rows of the one-thread CPU sample")
    ap.add_argument("--partition", choices=["interleave", "stripes"], default="interleave")
    return ap.parse_args()


def stripe(rank, world, height):
    y0 = rank * height // world
    y1 = (rank + 1) * height // world
    return y0, y1 - y0


def partition(rank, world, height, mode="interleave"):
    """Rows of rank `rank`: (y0, tile rows, row_step) — tile row i is screen row y0 + i * row_step."""
    if mode == "stripes" or world == 1:
        y0, th = stripe(rank, world, height)
        return y0, th, 1
    return rank, (height - rank + world - 1) // world, world


def assemble(parts, world, height, mode="interleave"):
    """Rank 0: puts the gathered row sets (each padded to the same row count) back into frame order."""
    import numpy as np

    frame = np.zeros((height,) + tuple(parts[0].shape[1:]), dtype=parts[0].dtype)
    for r, p in enumerate(parts):
        y0, th, step = partition(r, world, height, mode)
        frame[y0:y0 + (th - 1) * step + 1:step] = p[:th]
    return frame


def native_oracle():
    """The CPU oracle built for this host's CPU (-O3 -march=native); falls back to the
    portable build if the compiler is missing."""
    out = os.path.join(tempfile.gettempdir(), f"rt_liboracle_native_{os.getpid()}.so")
    cmd = ["g++", "-O3", "-march=native", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-shared",
           "-o", out, os.path.join(REPO, "oracle", "oracle.cpp"), "-lpthread"]
    try:
        subprocess.run(cmd, check=True, capture_output=True, timeout=120)
        return out, "-O3 -march=native"
    except (OSError, subprocess.SubprocessError):
        return None, "-O3 (portable build; -march=native compile failed)"


def host_cores():
    """(cores, source): the CPU share this job may use. A GPU box shows the whole machine's CPUs in
    os.cpu_count() / nproc but grants a job a share of them (cgroup quota, or the pool's declared
    OMP_NUM_THREADS); threads beyond the share only time-slice."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(per))), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return max(1, q // per), "cgroup cfs quota"
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < aff:
        return int(omp), "OMP_NUM_THREADS (the pool's CPU share per GPU job)"
    return aff, "sched_getaffinity"


def cpu_baseline(args):
    lib, flags = native_oracle()
    if lib:
        os.environ["RT_ORACLE_LIB"] = lib
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bind

    threads, cores_source = host_cores()
    sc = oracle_bind.OracleScene(os.path.join(REPO, "scenes", f"{args.scene}.toml"))
    rows = min(args.cpu_rows, args.height)
    y0 = (args.height - rows) // 2
    t0 = time.perf_counter()
    _, _, st = sc.render(args.width, args.height, args.cpu_spp, args.seed, tile=(0, y0, args.width, rows),
                         mis=args.mis, threads=threads, want_sub=False)
    dt = time.perf_counter() - t0
    samples = args.width * rows * 4 * (args.cpu_spp // 4)
    # SURVEY §8(d) also asks for one thread: the reference renders a job on one task (server.rs:157-199)
    rows1 = min(args.cpu_rows_1t, args.height)
    y1 = (args.height - rows1) // 2
    t1 = time.perf_counter()
    sc.render(args.width, args.height, args.cpu_spp, args.seed, tile=(0, y1, args.width, rows1), mis=args.mis,
              threads=1, want_sub=False)
    dt1 = time.perf_counter() - t1
    samples1 = args.width * rows1 * 4 * (args.cpu_spp // 4)
    if lib:
        os.unlink(lib)
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "cores_source": cores_source, "host_cpus_visible": os.cpu_count(),
            "sample": f"{args.scene} rows {y0}..{y0 + rows} of {args.width}x{args.height} at {args.cpu_spp} spp "
                      f"({samples} samples, {dt:.1f} s, f64, CPU oracle restating server.rs:320-368 + scene.rs + "
                      f"geometry.rs, g++ {flags})",
            "single_thread": {"value": samples1 / dt1 / 1e6, "cores": 1,
                              "sample": f"rows {y1}..{y1 + rows1} at {args.cpu_spp} spp ({samples1} samples, {dt1:.1f} s)"}}


def load_profile(name, key):
    try:
        with open(os.path.join(REPO, "profiles", name)) as f:
            return json.load(f).get(key)
    except (OSError, ValueError):
        return None


def compute_block(mix, vertices, kernel_ms):
    """f64 VALU issue occupancy and FP64 FLOP rate of this run from the PMC mix per path vertex."""
    rate = vertices / (kernel_ms / 1e3)  # path vertices per second
    cyc = sum(mix["per_vertex"][c] * VALU_COST[c] for c in VALU_COST) * rate
    clock = mix["clock_GHz"] * 1e9
    flops = mix["fp64_flops_per_vertex"] * rate
    out = {"bound": "valu_issue_f64", "issue_frac": round(cyc / (N_SIMD * clock), 4),
            "issue_cycles_per_s": round(cyc, 1), "clock_GHz": mix["clock_GHz"],
            "valu_inst_per_vertex": round(sum(mix["per_vertex"].values()), 2),
            "fp64_tflops": round(flops / 1e12, 3), "fp64_peak_tflops": FP64_PEAK_TFLOPS,
            "fp64_frac": round(flops / 1e12 / FP64_PEAK_TFLOPS, 4), "lane_utilisation": mix["lane_utilisation"],
            "cost_cycles": VALU_COST, "source": mix["source"]}
    if mix.get("waits"):  # the SIMD's measured view (SQ_ACTIVE_INST_VALU, SQ_WAIT_*: pmcw passes)
        w = mix["waits"]
        out["simd_valu_busy"] = round(w["simd_valu_busy"], 4)
        out["simd_salu_busy"] = round(w["simd_salu_busy"], 4)
        out["wave_wait_dependency"] = round(w["wait_any"], 4)
        out["wave_wait_issue"] = round(w["wait_inst_any"], 4)
        out["waits_source"] = ("SQ_ACTIVE_INST_VALU x waves/SIMD: share of SIMD cycles with a VALU instruction "
                               "executing; SQ_WAIT_ANY / SQ_WAIT_INST_ANY per resident wave-cycle")
    return out


def roofline_block(mix, mix_source, vertices, samples, kernel_ms, traffic, traffic_source, kernel, min_bytes,
                   binds):
    """The bench line's roofline object (module docstring). mix: a profiles/pmc_valu.json entry of this
    workload or None; vertices / samples: the launch's path vertices and camera samples; traffic: measured
    HBM bytes per launch or None."""
    sec = kernel_ms / 1e3
    model_bytes = BYTES_PER_SAMPLE * samples + BYTES_PER_VERTEX * vertices
    model_gbs = model_bytes / sec / 1e9
    hbm_gbs = traffic / sec / 1e9 if traffic else None
    out = {}
    if mix and mix.get("fp64_flops_per_vertex"):
        tflops = mix["fp64_flops_per_vertex"] * vertices / sec / 1e12
        out.update({"bound": "fp64_valu", "achieved": round(tflops, 3), "peak": FP64_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tflops / FP64_PEAK_TFLOPS, 4),
                    "frac_meaning": "measured FP64 FLOP rate of the kernel over the MI355X FP64 vector peak",
                    "fp64_flops_per_vertex": round(mix["fp64_flops_per_vertex"], 3),
                    "flops_source": f"{mix.get('pmc_file') or mix_source}: {mix.get('source', '')}"})
        if mix.get("waits"):
            out["simd_valu_busy"] = round(mix["waits"]["simd_valu_busy"], 4)
    else:
        out.update({"bound": "hbm", "achieved": round(hbm_gbs, 2) if hbm_gbs is not None else None,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(hbm_gbs / HBM_PEAK_GBS, 6) if hbm_gbs is not None else None,
                    "frac_meaning": "measured HBM bytes per launch over 8 TB/s (no PMC instruction mix for "
                                    "this workload)"})
    out.update({
        "traffic": int(traffic) if traffic else None,
        "traffic_source": traffic_source if traffic else None,
        "hbm": {"achieved_GBps": round(hbm_gbs, 3) if hbm_gbs is not None else None, "peak_GBps": HBM_PEAK_GBS,
                "frac": round(hbm_gbs / HBM_PEAK_GBS, 6) if hbm_gbs is not None else None},
        "minimum_bytes_per_launch": min_bytes,
        "wavefront_model_frac": round(model_gbs / HBM_PEAK_GBS, 4),
        "wavefront_model": {"achieved_GBps": round(model_gbs, 2), "bytes_per_launch": model_bytes,
                            "model": "SURVEY 8(d): 88 B per camera sample + 280 B per path vertex (f32 SoA "
                                     "wavefront state), vertices from this run's device counter; a comparison "
                                     "(> 1 means the kernel beats the streaming design), not bytes moved"},
        "model_ceiling_Msamples": round(HBM_PEAK_GBS * 1e9 / (BYTES_PER_SAMPLE + BYTES_PER_VERTEX * vertices /
                                                              samples) / 1e6, 1),
        "kernel": kernel, "kernel_ms": round(kernel_ms, 3), "binds": binds})
    return out


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # device map: rank -> its local GPU; RT_BENCH_DEVICE=k puts every rank on GPU k (a rehearsal of the
    # N-rank path on a one-GPU box: the frame digest must equal N = 1's, the timing means nothing)
    pinned = os.environ.get("RT_BENCH_DEVICE")
    device = int(pinned) if pinned not in (None, "") else (local if world > 1 else 0)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("gloo")  # host gather + barriers; no RCCL on the data path
    dev = torch.cuda.current_device()

    import rt_amd

    scene = rt_amd.Scene.from_toml(os.path.join(REPO, "scenes", f"{args.scene}.toml"))
    y0, th, row_step = partition(rank, world, args.height, args.partition)
    flags = (rt_amd.FLAG_MEGAKERNEL if args.mode == "megakernel" else 0) | (rt_amd.FLAG_MIS if args.mis else 0)
    flags |= rt_amd.FLAG_FP32 if args.fp32 else 0
    params = rt_amd.make_params(args.width, args.height, args.spp, args.seed, (0, y0, args.width, th), flags, dev,
                                row_step)
    max_rows = max(partition(r, world, args.height, args.partition)[1] for r in range(world))
    rgb = torch.zeros((max_rows, args.width, 3), dtype=torch.uint8, device="cuda")
    # two pinned host buffers: step k's rows are gathered to rank 0 (gloo, on the host) while step k + 1 renders
    # (stream order keeps the device buffer's next render behind this step's copy-back); the last step's gather
    # is inside the timed region, so every timed frame is complete on rank 0 when the clock stops
    hosts = [torch.zeros((max_rows, args.width, 3), dtype=torch.uint8).pin_memory() for _ in range(2)]
    host = hosts[0]
    stream = torch.cuda.current_stream()
    gathered = [torch.empty_like(host) for _ in range(world)] if (world > 1 and rank == 0) else None
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    kernel_ms = []
    pending = [None]  # the host buffer whose gather is still to be done
    last = [hosts[0]]  # the buffer of the last step (its frame: digest, N = 1)

    def flush():
        if world > 1 and pending[0] is not None:
            dist.gather(pending[0], gathered if rank == 0 else None, dst=0)  # host-side gather (gloo)
        pending[0] = None

    def step(i, timed):
        buf = hosts[i % 2]
        if timed:
            ev0.record(stream)
        rt_amd.render_device(scene, params, rgb.data_ptr(), None, stream.cuda_stream)
        if timed:
            ev1.record(stream)
        buf.copy_(rgb, non_blocking=True)  # the rank's rows to the host
        flush()  # the previous step's rows, while this one renders
        stream.synchronize()
        if timed:
            kernel_ms.append(ev0.elapsed_time(ev1))
        pending[0] = buf
        last[0] = buf

    # one untimed stats run: path-vertex count of this exact workload (device counter)
    st = rt_amd.render_device(scene, params, rgb.data_ptr(), None, stream.cuda_stream, stats=True)
    for i in range(args.warmup):
        step(i, False)
    flush()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    dev_ms = sum(kernel_ms) / max(1, len(kernel_ms))
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        v = torch.tensor([st["vertices"]], dtype=torch.int64)
        dist.all_reduce(v)
        total_vertices = int(v.item())
    else:
        total_vertices = st["vertices"]

    n_samples = args.width * args.height * 4 * (args.spp // 4)
    ms_per_step = wall * 1000.0 / args.steps
    value = n_samples / (wall / args.steps) / 1e6

    if rank == 0:
        # the frame: the gathered row sets put back in order; its digest is the same at every N
        if world > 1:
            frame = assemble([g.numpy() for g in gathered], world, args.height, args.partition)
        else:
            frame = last[0][:th].numpy()
        digest = hashlib.sha1(np.ascontiguousarray(frame).tobytes()).hexdigest()[:16]
        rank_samples = args.width * th * 4 * (args.spp // 4)
        workload = f"{args.scene} {args.width}x{args.height}x{args.spp}spp{' mis' if args.mis else ''}"
        mode = args.mode + ("-f32" if args.fp32 else "")
        kernel = "k_megakernel_f32" if args.fp32 else (
            "k_megakernel_f64" if args.mode == "megakernel" else "k_wf_extend+k_wf_shade")
        # traffic was measured at N = 1 on the whole frame: scale to this rank's share of the rows
        traffic_full = load_profile("pmc_traffic.json", f"{workload} {mode}")
        traffic = int(traffic_full * th / args.height) if traffic_full else None
        npix = args.width * th
        alg_bytes = npix * (2 * 12 * 8 + 3)  # f64 subpixel means written + read by the finalize, RGB8 out
        out = {
            "metric": "Msamples/sec (pixels x spp), cornell_box 1920x1080x1024spp" if args.scene == "cornell_box"
            and args.width == 1920 and args.height == 1080 and args.spp == 1024 and not args.fp32
            else f"Msamples/sec {workload}{' (f32 perf mode)' if args.fp32 else ''}",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32" if args.fp32 else "f64",
            "data": "synthetic: reference scene file + counter-based RNG (Philox4x32-10 -> xoroshiro128++), seed "
                    f"{args.seed:#x}",
            "config": {"workload": workload, "scene": f"scenes/{args.scene}.toml", "width": args.width,
                       "height": args.height, "spp": args.spp, "traced_spp": 4 * (args.spp // 4),
                       "mode": mode, "mis": args.mis,
                       "parallelism": f"{'interleaved rows' if args.partition == 'interleave' else 'row stripes'} x{world}"
                                      ", host gather (gloo)" if world > 1 else "1 GPU",
                       "frame_sha1": digest,
                       "device_map": f"every rank on GPU {device} (RT_BENCH_DEVICE: a rehearsal, timing not "
                                     "meaningful)" if pinned not in (None, "") else "rank -> LOCAL_RANK",
                       "vertices": total_vertices,
                       "vertices_per_sample": round(total_vertices / n_samples, 4)},
        }
        # the instruction mix of this exact command (benchpmc); only the exact workload prices the roofline
        mix_key = f"{workload} {mode}"
        mix = load_profile("pmc_valu.json", mix_key) if args.mode == "megakernel" else None
        out["roofline"] = roofline_block(
            mix, f"profiles/pmc_valu.json[{mix_key!r}]", st["vertices"], rank_samples, dev_ms, traffic,
            "profiles/pmc_traffic.json (2 x FETCH_SIZE + WRITE_SIZE per launch, rocprofv3 passes over this "
            "command)", kernel, alg_bytes,
            "valu_issue_f64" if args.mode == "megakernel" else "launches_and_state_traffic")
        if mix:
            out["roofline"]["compute"] = compute_block(mix, st["vertices"], dev_ms)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
