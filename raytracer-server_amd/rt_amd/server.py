"""WebSocket front-end on the C ABI: the reference's server.rs protocol, rendering on the GPU.

Mirrors src/server.rs of SuneelFreimuth/raytracer-server:
  * connection ids: 5 distinct lowercase letters (server.rs:63-78);
  * client messages (server.rs:121-126): {"type": "render", "scene": <name>, "spp": <int>} starts a
    job when none is running; {"type": "stop_rendering"} cancels the running job;
  * server messages (server.rs:173-190): binary [u8 type = 0][u8 n][u16le x][u16le y][n x RGB8],
    one per 60-pixel window of a screen row (row 0 = top);
  * frame size 600 x 450 (server.rs:29-30), spp semantics of sample_pixel (4*floor(spp/4) traced).
Differences, by design: the render runs on the GPU through rt_render in row bands (progressive
streaming, band by band, top to bottom), the cancel flag is also polled inside the render, and the
reference's panics (bad JSON, unknown scene) become logged errors.

Run:  PORT=8080 python -m rt_amd.server <scenes dir>
"""
import asyncio
import ctypes
import json
import os
import random
import string
import struct
import sys

import numpy as np

WIDTH = 600   # server.rs:29
HEIGHT = 450  # server.rs:30
PIXELS_PER_MSG = 60  # server.rs:145
SCENE_NAMES = ("cornell_box", "cubes", "flying_unicorn")  # main.rs:17


def chunk_messages(rgb, y0):
    """Binary messages for rows y0.. of a rendered band (server.rs:173-190)."""
    rows, width, _ = rgb.shape
    for r in range(rows):
        for x in range(0, width, PIXELS_PER_MSG):
            n = min(PIXELS_PER_MSG, width - x)
            yield struct.pack("<BBHH", 0, n, x, y0 + r) + rgb[r, x:x + n].tobytes()


def gpu_band_renderer(device=0, fp32=False):
    """Default band renderer: rt_render on `device` for rows [y0, y0 + rows). fp32: the f32 perf mode
    (RT_FLAG_FP32, statistical parity only) — server-wide, the protocol is unchanged."""
    import rt_amd

    def render(scene, width, height, spp, seed, y0, rows, cancel):
        rgb, _, st = rt_amd.render(scene, width, height, spp, seed, tile=(0, y0, width, rows),
                                   megakernel=True, device=device, cancel=cancel, fp32=fp32)
        return None if st["cancelled"] else rgb

    return render


class RenderJob:
    """server.rs:139-223: one job per connection, cancellable between bands."""

    def __init__(self, send, renderer, band_rows):
        self.send = send
        self.renderer = renderer
        self.band_rows = band_rows
        self.cancel = ctypes.c_int32(1)  # starts cancelled == not running (server.rs:148-149)

    def running(self):
        return self.cancel.value == 0

    def stop(self):
        self.cancel.value = 1

    async def run(self, scene, width, height, spp, seed):
        """Returns True when stopped before completion (server.rs:156)."""
        self.cancel.value = 0
        loop = asyncio.get_running_loop()
        for y0 in range(0, height, self.band_rows):
            if self.cancel.value:
                return True
            rows = min(self.band_rows, height - y0)
            rgb = await loop.run_in_executor(None, self.renderer, scene, width, height, spp, seed, y0, rows,
                                             self.cancel)
            if rgb is None or self.cancel.value:
                return True
            for msg in chunk_messages(rgb, y0):
                try:
                    await self.send(msg)
                except ConnectionError:
                    self.cancel.value = 1
                    return True
        self.cancel.value = 1
        return False


class Server:
    def __init__(self, scenes, renderer=None, width=WIDTH, height=HEIGHT, band_rows=32, log=print):
        self.scenes = scenes
        self.renderer = renderer or gpu_band_renderer()
        self.width = width
        self.height = height
        self.band_rows = band_rows
        self.connections = set()
        self.log = log

    def new_id(self):  # server.rs:63-78
        while True:
            cid = "".join(random.sample(string.ascii_lowercase, 5))
            if cid not in self.connections:
                self.connections.add(cid)
                return cid

    async def handle(self, request):
        from aiohttp import WSMsgType, web

        ws = web.WebSocketResponse()
        await ws.prepare(request)
        cid = self.new_id()
        self.log(f"[{cid}] Accepted connection.")
        job = RenderJob(ws.send_bytes, self.renderer, self.band_rows)
        task = None
        try:
            async for msg in ws:
                if msg.type != WSMsgType.TEXT:
                    continue
                self.log(f"[{cid}] New message: '{msg.data}'")
                try:
                    m = json.loads(msg.data)
                    kind = m["type"]
                except (ValueError, KeyError, TypeError):
                    self.log(f"[{cid}] failed to parse message")
                    break  # the reference panics here (server.rs:92): the connection ends
                if kind == "render" and not job.running():
                    name, spp = m.get("scene"), m.get("spp")
                    if name not in self.scenes or not isinstance(spp, int):
                        self.log(f"[{cid}] bad render request {m!r}")
                        continue
                    seed = int.from_bytes(os.urandom(8), "little") if "RT_SEED" not in os.environ \
                        else int(os.environ["RT_SEED"], 0)
                    self.log(f"[{cid}] Rendering...")
                    task = asyncio.ensure_future(self._run(cid, job, self.scenes[name], spp, seed))
                elif kind == "stop_rendering" and job.running():
                    job.stop()
                    self.log(f"[{cid}] Render cancelled.")
        finally:
            job.stop()
            if task is not None:
                await asyncio.gather(task, return_exceptions=True)
            self.connections.discard(cid)
            self.log(f"[{cid}] Disconnected.")
        return ws

    async def _run(self, cid, job, scene, spp, seed):
        cancelled = await job.run(scene, self.width, self.height, spp, seed)
        if not cancelled:
            self.log(f"[{cid}] Done rendering.")

    def app(self):
        from aiohttp import web

        app = web.Application()
        app.router.add_get("/", self.handle)
        return app


def main(argv=None):
    from aiohttp import web

    argv = argv if argv is not None else sys.argv[1:]
    if not argv:
        print("Usage: python -m rt_amd.server <scenes directory>", file=sys.stderr)
        return 2
    import rt_amd

    scene_dir = argv[0]
    scenes = {n: rt_amd.Scene.from_toml(os.path.join(scene_dir, f"{n}.toml")) for n in SCENE_NAMES}
    port = int(os.environ.get("PORT", "8080"))  # main.rs:38
    print(f"Listening on port {port}.")
    fp32 = os.environ.get("RT_PRECISION", "f64") == "f32"  # f64 (the reference's arithmetic) by default
    if fp32:
        # the f32 mode traces meshes with the nearest-triangle semantics
        # (geometry.rs:886-903), not the reference's first-hit octree walk (geometry.rs:1237-1295)
        print("RT_PRECISION=f32: f32 perf mode; meshes (flying_unicorn) use nearest-triangle hits, not the "
              "reference's octree semantics; frames differ statistically from server.rs", file=sys.stderr)
    web.run_app(Server(scenes, renderer=gpu_band_renderer(fp32=fp32)).app(), host="0.0.0.0", port=port, print=None)
    return 0


if __name__ == "__main__":
    sys.exit(main())
