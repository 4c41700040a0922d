"""GPU tests of the drop-in boundary's concurrency and front-ends:

  * concurrent rt_render_device calls on one scene and one device, on two HIP streams (one thread
    enqueueing both, and two host threads) equal their serial renders: each in-flight render keeps
    its own workspace (rt_ffi.h: a scene may be shared by concurrent renders);
  * rt_render_multi (one process, several workers, dynamic band handout, host gather) equals
    rt_render, with and without stats, and honours cancel;
  * the WebSocket server (rt_amd.server, the reference's server.rs protocol) rendering on the GPU
    through gpu_band_renderer, over a real socket, reassembled chunk by chunk and compared with the
    CPU oracle byte for byte; `stop_rendering` mid-frame cancels the job.
"""
import asyncio
import ctypes
import json
import struct
import threading
import time

import numpy as np
import pytest

from test_gpu_parity import SEED

pytestmark = pytest.mark.gpu


def _device_render(rt, torch, scene, w, h, spp, seed, stream, mis=False):
    p = rt.make_params(w, h, spp, seed, None, rt.FLAG_MEGAKERNEL | (rt.FLAG_MIS if mis else 0), 0, 1)
    buf = torch.zeros((h, w, 3), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the zero fill runs on the current stream: done before `stream` writes buf
    rt.render_device(scene, p, buf.data_ptr(), None, stream.cuda_stream)
    return buf


def test_concurrent_render_device_two_streams(rt, gpu_scenes):
    import torch

    s = gpu_scenes["cubes"]  # ~40 ms per render: the two launches overlap on the device
    w, h, spp = 256, 192, 64
    ref = {k: rt.render(s, w, h, spp, SEED + k, megakernel=True)[0] for k in range(4)}
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    # one thread, two streams, back to back (the second enqueue happens while the first kernel runs)
    for _ in range(2):
        a = _device_render(rt, torch, s, w, h, spp, SEED + 0, s1)
        b = _device_render(rt, torch, s, w, h, spp, SEED + 1, s2)
        c = _device_render(rt, torch, s, w, h, spp, SEED + 2, s1)
        torch.cuda.synchronize()
        assert np.array_equal(a.cpu().numpy(), ref[0])
        assert np.array_equal(b.cpu().numpy(), ref[1])
        assert np.array_equal(c.cpu().numpy(), ref[2])
    # two host threads, each with its own stream, three renders each
    out = {}

    def worker(tid, stream):
        bufs = [_device_render(rt, torch, s, w, h, spp, SEED + tid + 2 * i, stream) for i in range(2)]
        stream.synchronize()
        out[tid] = [b.cpu().numpy() for b in bufs]

    ts = [threading.Thread(target=worker, args=(t, st)) for t, st in ((0, s1), (1, s2))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for tid in (0, 1):
        for i in range(2):
            assert np.array_equal(out[tid][i], ref[tid + 2 * i]), (tid, i)


@pytest.mark.parametrize("name", ["cornell_box", "cubes"])
def test_render_multi_equals_render(name, rt, gpu_scenes):
    s = gpu_scenes[name]
    w, h, spp = 320, 240, 16
    ref, _, st_ref = rt.render(s, w, h, spp, SEED, megakernel=True)
    for devices, band in [([0], 0), ([0, 0], 7), ([0, 0, 0], 64)]:
        rgb, st = rt.render_multi(s, w, h, spp, devices, SEED, band_rows=band)
        assert np.array_equal(rgb, ref), (devices, band)
        assert st["samples"] == w * h * spp and st["vertices"] == st_ref["vertices"]
    # a tile with interleaved rows, several workers
    tile, step = (40, 2, 200, 60), 3
    want, _, _ = rt.render(s, w, h, spp, SEED, tile=tile, row_step=step, megakernel=True)
    got, _ = rt.render_multi(s, w, h, spp, [0, 0], SEED, tile=tile, row_step=step, band_rows=9)
    assert np.array_equal(got, want)


def test_render_multi_rejects_missing_device(rt, gpu_scenes):
    """An ordinal past the visible devices (here: device_count()) fails the whole call with RT_E_INVAL
    before any band runs, and the next call renders normally."""
    n = rt.device_count()
    with pytest.raises(rt.RtError, match="out of range"):
        rt.render_multi(gpu_scenes["cornell_box"], 64, 48, 4, [0, n], SEED)
    rgb, st = rt.render_multi(gpu_scenes["cornell_box"], 64, 48, 4, [0], SEED)
    assert st["samples"] == 64 * 48 * 4 and rgb.any()


def test_render_multi_cancel(rt, gpu_scenes):
    flag = ctypes.c_int32(0)
    timer = threading.Timer(0.3, lambda: setattr(flag, "value", 1))
    t0 = time.time()
    timer.start()
    _, st = rt.render_multi(gpu_scenes["cornell_box"], 1920, 1080, 2048, [0, 0], SEED, band_rows=16, cancel=flag)
    dt = time.time() - t0
    timer.cancel()
    assert st["cancelled"] and dt < 4.0, (st["cancelled"], dt)


# ---------------------------------------------------------------- WebSocket front-end on the GPU
W, H, SPP = 64, 48, 8


async def _session(srv, messages, rows, stop_after=None, timeout=20.0):
    from aiohttp import ClientSession, WSMsgType, web

    runner = web.AppRunner(srv.app())
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]
    got = []
    try:
        async with ClientSession() as cs:
            async with cs.ws_connect(f"http://127.0.0.1:{port}/") as ws:
                for m in messages:
                    await ws.send_str(m)
                while True:
                    try:
                        msg = await asyncio.wait_for(ws.receive(), timeout=timeout)
                    except asyncio.TimeoutError:
                        break
                    if msg.type != WSMsgType.BINARY:
                        break
                    got.append(msg.data)
                    if stop_after is not None and len(got) == stop_after:
                        await ws.send_str(json.dumps({"type": "stop_rendering"}))
                        timeout = 3.0  # after the stop, only chunks already in flight may arrive
                    if len(got) == rows:
                        break
    finally:
        await runner.cleanup()
    return got


def _assemble(msgs, w, h):
    frame = np.zeros((h, w, 3), dtype=np.uint8)
    for m in msgs:
        t, n, x, y = struct.unpack("<BBHH", m[:6])
        assert t == 0 and len(m) == 6 + 3 * n and n <= 60
        frame[y, x:x + n] = np.frombuffer(m[6:], dtype=np.uint8).reshape(n, 3)
    return frame


def test_ws_server_gpu_frame_equals_oracle(rt, gpu_scenes, oracle_scenes, monkeypatch):
    from rt_amd import server

    monkeypatch.setenv("RT_SEED", hex(SEED))
    srv = server.Server({"cornell_box": gpu_scenes["cornell_box"]}, renderer=server.gpu_band_renderer(device=0),
                        width=W, height=H, band_rows=8, log=lambda *_: None)
    msgs = asyncio.run(_session(srv, [json.dumps({"type": "render", "scene": "cornell_box", "spp": SPP})],
                                rows=H * 2))  # 64 px per row = 2 messages (60 + 4) per row
    assert len(msgs) == 2 * H
    frame = _assemble(msgs, W, H)
    ref, _, _ = oracle_scenes["cornell_box"].render(W, H, SPP, SEED, want_sub=False)
    assert np.array_equal(frame, ref)
    rows = [struct.unpack("<BBHH", m[:6])[3] for m in msgs]
    assert rows == sorted(rows)  # bands stream top to bottom, like the reference's fill


def test_ws_server_gpu_stop_rendering(rt, gpu_scenes, monkeypatch):
    from rt_amd import server

    monkeypatch.setenv("RT_SEED", hex(SEED))
    srv = server.Server({"cornell_box": gpu_scenes["cornell_box"]}, renderer=server.gpu_band_renderer(device=0),
                        width=600, height=450, band_rows=4, log=lambda *_: None)
    t0 = time.time()
    msgs = asyncio.run(_session(srv, [json.dumps({"type": "render", "scene": "cornell_box", "spp": 8192})],
                                rows=450 * 10, stop_after=10))  # 8192 spp: ~1.2 s per frame
    dt = time.time() - t0
    assert 10 <= len(msgs) < 450 * 10 and dt < 15.0, (len(msgs), dt)


def test_concurrent_cancellable_renders_share_one_flag(rt, gpu_scenes):
    """Two rt_render calls on two host threads share one cancel flag (the reference's per-job
    AtomicBool, server.rs:226-251, viewed as an i32). The flag is never registered with HIP: each
    render polls a pinned word of its own that its waiting thread copies the flag into, so one render
    ending cannot unmap the flag under the other. Flag clear: both frames equal their serial renders.
    Flag raised mid-render: both return RT_CANCELLED long before a full frame."""
    s = gpu_scenes["cornell_box"]
    w, h, spp = 256, 192, 64
    ref = [rt.render(s, w, h, spp, SEED + k, megakernel=True)[0] for k in range(2)]
    flag = ctypes.c_int32(0)
    out = {}

    def run(k, width, height, n):
        out[k] = rt.render(s, width, height, n, SEED + k, megakernel=True, cancel=flag)

    ts = [threading.Thread(target=run, args=(k, w, h, spp)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for k in range(2):
        assert np.array_equal(out[k][0], ref[k]) and not out[k][2]["cancelled"], k
    # 1920x1080 at 2048 spp: ~9 s per frame alone; the flag goes up after 0.3 s
    timer = threading.Timer(0.3, lambda: setattr(flag, "value", 1))
    t0 = time.time()
    timer.start()
    ts = [threading.Thread(target=run, args=(k, 1920, 1080, 2048)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.time() - t0
    timer.cancel()
    # two frames together would take ~18 s; the bound leaves room for a fresh box's first 1.7 GB workspace
    # allocations (the split-tail scratch of each render) without accepting a missed cancel
    assert out[0][2]["cancelled"] and out[1][2]["cancelled"] and dt < 6.0, \
        (out[0][2]["cancelled"], out[1][2]["cancelled"], dt, out[0][2]["device_ms"], out[1][2]["device_ms"])
