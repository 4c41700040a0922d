"""The driver's N-rank bench path on the one GPU of the test box (bench.py:213-367; the reference's
row-band fan-out, server.rs:165-168): `torch.distributed.run --nproc-per-node 2 bench.py --gpus 2`, every
rank mapped to GPU 0 by RT_BENCH_DEVICE=0 before any GPU call in the child. Each rank sets its device,
joins the gloo group, renders its interleaved rows, copies them to pinned memory and gathers them on
rank 0, which assembles the frame: its digest must equal the N = 1 frame's. Both runs are fresh child
processes (the launcher starts before anything in them touches the GPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

ARGS = ["--steps", "1", "--warmup", "0", "--spp", "64", "--no-cpu-baseline"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench_line(cmd, env):
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, f"{' '.join(cmd)}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_bench_n_ranks_frame_equals_one_rank(world, gpu_scenes):
    env = {k: v for k, v in os.environ.items() if not k.startswith(("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_"))}
    env["RT_BENCH_DEVICE"] = "0"
    one = _bench_line([sys.executable, "bench.py", "--gpus", "1"] + ARGS, env)
    many = _bench_line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus",
                        str(world)] + ARGS, env)
    assert one["n_gpus"] == 1 and many["n_gpus"] == world
    assert many["config"]["parallelism"].startswith(f"interleaved rows x{world}")
    assert many["config"]["frame_sha1"] == one["config"]["frame_sha1"]
    assert many["config"]["vertices"] == one["config"]["vertices"]  # the ranks' counts summed over gloo
    assert many["value"] > 0 and many["roofline"]["bound"] == "hbm"
