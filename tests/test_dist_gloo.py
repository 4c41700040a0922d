"""Multi-rank image tiling (bench.py's N > 1 path) rehearsed on CPU with the gloo backend.

Each rank renders its rows (bench.partition: interleaved rows r, r+N, ... or contiguous stripes),
the row sets are gathered to rank 0 exactly as bench.py does (a host gather over a gloo process group:
no RCCL collective is on the data path), and the assembled frame
(bench.assemble) must equal a single-rank render byte for byte:
the RNG is keyed by the global pixel id, so the partition cannot change the image. The CPU oracle
stands in for the GPU renderer here (test infrastructure only)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, scene_path

W, H, SPP, SEED = 48, 37, 4, 0x5EED


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path, mode):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import oracle_bind

    y0, th, step = bench.partition(rank, world, H, mode)
    max_rows = max(bench.partition(r, world, H, mode)[1] for r in range(world))
    sc = oracle_bind.OracleScene(scene_path("cubes"))
    # the rank's rows (row_step > 1: one oracle call per screen row y0 + i*step)
    rows = [sc.render(W, H, SPP, SEED, tile=(0, y0 + i * step, W, 1), threads=1, want_sub=False)[0] for i in range(th)]
    rgb = np.concatenate(rows, axis=0)
    buf = torch.zeros((max_rows, W, 3), dtype=torch.uint8)
    buf[:th] = torch.from_numpy(rgb)
    gathered = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    if rank == 0:
        np.save(out_path, bench.assemble([g.numpy() for g in gathered], world, H, mode))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["interleave", "stripes"])
@pytest.mark.parametrize("world", [2, 3])
def test_partition_gather_equals_single_render(world, mode, tmp_path, oracle):
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, mode), nprocs=world, join=True)
    frame = np.load(out)
    ref, _, _ = oracle.OracleScene(scene_path("cubes")).render(W, H, SPP, SEED, want_sub=False)
    assert frame.shape == ref.shape and np.array_equal(frame, ref)


def test_stripes_cover_frame():
    sys.path.insert(0, REPO)
    import bench

    for world in (1, 2, 3, 4, 7, 8):
        rows = []
        for r in range(world):
            y0, th = bench.stripe(r, world, 1080)
            rows.extend(range(y0, y0 + th))
        assert rows == list(range(1080))
        for mode in ("interleave", "stripes"):
            rows = []
            for r in range(world):
                y0, th, step = bench.partition(r, world, 1080, mode)
                rows.extend(range(y0, y0 + (th - 1) * step + 1, step) if th else [])
            assert sorted(rows) == list(range(1080))
