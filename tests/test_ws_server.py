"""WebSocket front-end (rt_amd.server, the §8f "next" row): the reference's protocol end to end on
CPU. The band renderer is the CPU oracle (test infrastructure) so no GPU is needed here; the GPU
renderer behind the same interface is exercised by tests/test_gpu_parity.py."""
import asyncio
import json
import struct

import numpy as np
import pytest

from conftest import scene_path

W, H, SPP, SEED = 60, 45, 4, 0x5EED


def _server(oracle, band_rows=8):
    from rt_amd import server

    scenes = {"cornell_box": oracle.OracleScene(scene_path("cornell_box"))}

    def render(scene, width, height, spp, seed, y0, rows, cancel):
        rgb, _, _ = scene.render(width, height, spp, SEED, tile=(0, y0, width, rows), threads=2, want_sub=False)
        return rgb

    return server.Server(scenes, renderer=render, width=W, height=H, band_rows=band_rows, log=lambda *_: None)


async def _session(srv, messages, stop_after=None):
    from aiohttp import web, ClientSession, WSMsgType

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
                        msg = await asyncio.wait_for(ws.receive(), timeout=5.0)
                    except asyncio.TimeoutError:
                        break
                    if msg.type != WSMsgType.BINARY:
                        break
                    got.append(msg.data)
                    if stop_after is not None and len(got) == stop_after:
                        await ws.send_str(json.dumps({"type": "stop_rendering"}))
                    if len(got) == H:
                        break
    finally:
        await runner.cleanup()
    return got


def test_render_protocol_roundtrip(oracle):
    srv = _server(oracle)
    got = asyncio.run(_session(srv, [json.dumps({"type": "render", "scene": "cornell_box", "spp": SPP})]))
    assert len(got) == H  # one 60-pixel message per row at W = 60
    frame = np.zeros((H, W, 3), dtype=np.uint8)
    for m in got:
        t, n, x, y = struct.unpack("<BBHH", m[:6])
        assert t == 0 and len(m) == 6 + 3 * n
        frame[y, x:x + n] = np.frombuffer(m[6:], dtype=np.uint8).reshape(n, 3)
    ref, _, _ = oracle.OracleScene(scene_path("cornell_box")).render(W, H, SPP, SEED, want_sub=False)
    assert np.array_equal(frame, ref)
    rows = [struct.unpack("<BBHH", m[:6])[3] for m in got]
    assert rows == sorted(rows)  # top to bottom, like the reference's fill


def test_stop_rendering_cancels(oracle):
    srv = _server(oracle, band_rows=4)
    got = asyncio.run(_session(srv, [json.dumps({"type": "render", "scene": "cornell_box", "spp": SPP})],
                               stop_after=4))
    assert 4 <= len(got) < H


def test_bad_messages(oracle):
    srv = _server(oracle)
    # unknown scene: ignored (the reference's job task panics); the connection stays usable
    got = asyncio.run(_session(srv, [json.dumps({"type": "render", "scene": "nope", "spp": 4}),
                                     json.dumps({"type": "render", "scene": "cornell_box", "spp": SPP})]))
    assert len(got) == H
    # malformed JSON ends the connection (the reference panics in the connection task)
    got = asyncio.run(_session(srv, ["{not json", json.dumps({"type": "render", "scene": "cornell_box", "spp": 4})]))
    assert got == []


def test_connection_ids(oracle):
    srv = _server(oracle)
    ids = {srv.new_id() for _ in range(200)}
    assert len(ids) == 200 and all(len(i) == 5 and len(set(i)) == 5 and i.islower() for i in ids)
