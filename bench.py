"""Headline benchmark: Msamples/s of the path-tracing hot path on cornell_box 1920x1080x1024spp.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 launched by
torch.distributed.run, one rank per GPU. A step = one full render of the frame (scene resident in
HBM; output RGB8 gathered to rank 0). Rank r renders the interleaved rows r, r+N, r+2N, ... of the
frame (rt_render_params.row_step = N: every rank gets the same mix of cheap and expensive rows;
--partition stripes gives contiguous stripes instead); no collective on the data path except the
final RGB8 gather the north_star prescribes. Total work is fixed: scaling = "strong". Rank 0
prints one JSON line.

roofline: dominant kernel = the render kernel(s). Algorithmic bytes follow SURVEY §8(d)'s canonical
SoA wavefront model, 88 B per camera sample + 280 B per path vertex, with the vertex count taken
from the device counter of the same workload; achieved = those bytes / device time measured with
HIP events on the stream the kernels run on. peak = 8.0 TB/s (MI355X HBM3E). traffic = PMC-derived
HBM bytes per launch from profiles/ (null when not collected for this mode).

cpu_baseline: the CPU oracle (a line-by-line f64 restatement of the reference's sample loop, the
reference itself is Rust and cannot be built here) on a bounded row band of the same frame, on
min(16, cpu_count) threads, rank 0 at N = 1 only.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))

HBM_PEAK_GBS = 8000.0
BYTES_PER_SAMPLE = 88
BYTES_PER_VERTEX = 280


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


def cpu_baseline(args):
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bind

    threads = max(1, min(16, os.cpu_count() or 1))
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
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{args.scene} rows {y0}..{y0 + rows} of {args.width}x{args.height} at {args.cpu_spp} spp "
                      f"({samples} samples, {dt:.1f} s, f64, CPU oracle restating server.rs:320-368 + scene.rs + geometry.rs)",
            "single_thread": {"value": samples1 / dt1 / 1e6, "cores": 1,
                              "sample": f"rows {y1}..{y1 + rows1} at {args.cpu_spp} spp ({samples1} samples, {dt1:.1f} s)"}}


def load_valu(workload_key):
    """VALU wave-instructions per path vertex of the dominant kernel, from the SQ PMC passes in
    profiles/ (tools/gpu_pmc_mk.sh -> profiles/pmc_valu.json), or None."""
    path = os.path.join(REPO, "profiles", "pmc_valu.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


def load_traffic(workload_key):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload_key)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
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
    stream = torch.cuda.current_stream()
    gathered = [torch.empty_like(rgb) for _ in range(world)] if (world > 1 and rank == 0) else None

    def step():
        rt_amd.render_device(scene, params, rgb.data_ptr(), None, stream.cuda_stream)
        if world > 1:
            dist.gather(rgb, gathered if rank == 0 else None, dst=0)

    # one untimed stats run: path-vertex count of this exact workload (device counter)
    st = rt_amd.render_device(scene, params, rgb.data_ptr(), None, stream.cuda_stream, stats=True)
    for _ in range(args.warmup):
        step()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    dev_ms = ev0.elapsed_time(ev1) / max(1, args.steps)
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        v = torch.tensor([st["vertices"]], dtype=torch.int64, device="cuda")
        dist.all_reduce(v)
        total_vertices = int(v.item())
    else:
        total_vertices = st["vertices"]

    # the frame (rank 0): the gathered row sets put back in order; its digest is the same at every N
    import hashlib

    if rank == 0:
        if world > 1:
            frame = assemble([g.cpu().numpy() for g in gathered], world, args.height, args.partition)
        else:
            frame = rgb[:th].cpu().numpy()
        digest = hashlib.sha1(frame.tobytes()).hexdigest()[:16]

    n_samples = args.width * args.height * 4 * (args.spp // 4)
    ms_per_step = wall * 1000.0 / args.steps
    value = n_samples / (wall / args.steps) / 1e6

    if rank == 0:
        rank_samples = args.width * th * 4 * (args.spp // 4)
        alg_bytes = BYTES_PER_SAMPLE * rank_samples + BYTES_PER_VERTEX * st["vertices"]
        achieved = alg_bytes / (dev_ms / 1e3) / 1e9
        workload = f"{args.scene} {args.width}x{args.height}x{args.spp}spp{' mis' if args.mis else ''}"
        mode = args.mode + ("-f32" if args.fp32 else "")
        kernel = "k_megakernel_f32" if args.fp32 else (
            "k_megakernel_f64" if args.mode == "megakernel" else "k_wf_extend+k_wf_shade")
        traffic = load_traffic(f"{workload} {mode}")
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
                       "parallelism": f"{'interleaved rows' if args.partition == 'interleave' else 'row stripes'} x{world}",
                       "frame_sha1": digest,
                       "vertices_per_sample": round(total_vertices / n_samples, 4)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": kernel,
                         "kernel_ms": round(dev_ms, 3),
                         "alg_bytes_per_launch": alg_bytes,
                         "model": "SURVEY 8(d): 88 B/sample + 280 B/vertex (canonical f32 SoA wavefront state)"},
        }
        # The megakernel's own bound is VALU issue: PMC instructions per vertex x the
        # vertex rate of this run, against 1024 SIMDs x one wave-instruction per 4 cycles at 2.4 GHz
        valu = load_valu(f"{args.scene} {mode}") if mode.startswith("megakernel") else None
        if valu:
            rate = valu["valu_inst_per_vertex"] * st["vertices"] / (dev_ms / 1e3)
            peak = 1024 * 2.4e9 / 4
            out["roofline"]["valu"] = {"achieved": round(rate / 1e9, 2), "peak": round(peak / 1e9, 2),
                                       "unit": "G wave-instr/s", "frac": round(rate / peak, 4),
                                       "inst_per_vertex": valu["valu_inst_per_vertex"], "source": valu["source"]}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
