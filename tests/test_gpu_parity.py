"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same seeded inputs.

Tolerances (SURVEY §8c.1, f64 mode):
  * Scene::trace_ray: object id, t, hit position and normal bit-identical on >= 99.9% of rays; the
    rest may differ only where device and host libm disagree in the last ulp (not expected: trace
    uses only + - * / sqrt, all correctly rounded on both sides);
  * subpixel means: |rel| <= 1e-9 on >= 99.9% of subpixels (the GPU walks the path forward, the
    oracle recurses like the reference: sums associate differently, ~1e-15);
  * RGB8 identical on >= 99.9% of pixels, |delta| <= 1 elsewhere, except pixels whose paths took a
    different branch because sin/cos differ by an ulp between ocml and glibc (counted, bounded).
Megakernel and wavefront run the same device code per sample and must agree bit for bit.
"""
import numpy as np
import pytest

from conftest import scene_path

pytestmark = pytest.mark.gpu

SEED = 0x5EED


def _rays_for(name, n, rng):
    """Camera-like rays, random rays inside the room, and rays aimed at the mesh region."""
    o = np.empty((n, 3))
    d = rng.normal(size=(n, 3))
    k = n // 3
    o[:k] = [50.0, 52.0, 295.6]
    d[:k] = np.column_stack([rng.uniform(-0.35, 0.35, k), rng.uniform(-0.3, 0.25, k), -np.ones(k)])
    o[k:2 * k] = rng.uniform([2, 1, 1], [98, 80, 200], size=(k, 3))
    # aimed at the unicorn / cubes region, from anywhere in the room
    tgt = rng.uniform([12, 0, 25], [92, 60, 92], size=(n - 2 * k, 3))
    o[2 * k:] = rng.uniform([2, 1, 1], [98, 80, 250], size=(n - 2 * k, 3))
    d[2 * k:] = tgt - o[2 * k:]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d


def test_exact_division_shortcuts(rt):
    """rcp_rn / qdiv / sqrt_rn (path_f64.h) against the IEEE operations on the device: 2^24 operands
    each, spanning every exponent of the shortcuts' ranges (sqrt_rn: [2^-767, 2^1024))."""
    assert rt.selftest_arith(1 << 24) == (0, 0, 0)


@pytest.mark.parametrize("name", ["cornell_box", "cubes", "flying_unicorn"])
def test_trace_ray_bit_exact(name, gpu_scenes, oracle_scenes):
    rng = np.random.default_rng(1234)
    o, d = _rays_for(name, 30000, rng)
    t_g, id_g, p_g, n_g = gpu_scenes[name].trace_ray(o, d)
    t_o, id_o, p_o, n_o = oracle_scenes[name].trace(o, d)
    assert (id_o >= 0).mean() > 0.99
    same_id = id_g == id_o
    exact = same_id & (t_g == t_o) & np.all(p_g == p_o, axis=1) & np.all(n_g == n_o, axis=1)
    assert same_id.mean() >= 0.999, f"object id mismatch on {np.count_nonzero(~same_id)} rays"
    assert exact.mean() >= 0.999, f"non bit-exact hits: {np.count_nonzero(~exact)}"


def _render_pair(rt, gpu_scene, oracle_scene, w, h, spp, tile=None, mis=False, megakernel=False):
    rgb_g, sub_g, st = rt.render(gpu_scene, w, h, spp, SEED, tile=tile, mis=mis, megakernel=megakernel,
                                 want_sub=True)
    rgb_o, sub_o, st_o = oracle_scene.render(w, h, spp, SEED, tile=tile, mis=mis)
    return rgb_g, sub_g, st, rgb_o, sub_o, st_o


def _assert_parity(rgb_g, sub_g, rgb_o, sub_o, what):
    rel = np.abs(sub_g - sub_o) / np.maximum(np.abs(sub_o), 1e-300)
    close_sub = np.all((rel <= 1e-9) | (np.abs(sub_g - sub_o) <= 1e-15), axis=-1)  # per subpixel
    frac_sub = close_sub.mean()
    diff = np.abs(rgb_g.astype(int) - rgb_o.astype(int))
    same_px = np.all(diff == 0, axis=-1).mean()
    assert frac_sub >= 0.999, f"{what}: only {frac_sub:.5f} of subpixels within 1e-9"
    assert same_px >= 0.999, f"{what}: only {same_px:.5f} of pixels RGB8-identical"
    # anything else must be a (rare) branch flip, not a systematic drift
    flipped = ~np.all(diff <= 1, axis=-1)
    assert flipped.mean() <= 0.001, f"{what}: {np.count_nonzero(flipped)} pixels differ by more than 1"


@pytest.mark.parametrize("name", ["cornell_box", "cubes", "flying_unicorn"])
@pytest.mark.parametrize("megakernel", [False, True], ids=["wavefront", "megakernel"])
def test_render_parity_small(name, megakernel, rt, gpu_scenes, oracle_scenes):
    w, h, spp = 96, 72, 16
    rgb_g, sub_g, st, rgb_o, sub_o, st_o = _render_pair(rt, gpu_scenes[name], oracle_scenes[name], w, h, spp,
                                                        megakernel=megakernel)
    assert st["samples"] == w * h * 4 * (spp // 4)
    # the GPU ends zero-throughput paths early (same radiance), so it counts at most the oracle's vertices
    assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
    _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"{name}/{'mk' if megakernel else 'wf'}")


@pytest.fixture(scope="module")
def oracle_nearest(oracle):
    """Oracle scenes whose meshes take Mesh::intersect's `octree: None` branch (geometry.rs:886-903)."""
    return {n: oracle.OracleScene(scene_path(n), mesh_nearest=True) for n in ("cubes", "flying_unicorn")}


@pytest.mark.parametrize("name", ["cubes", "flying_unicorn"])
def test_trace_mesh_nearest_bit_exact(name, gpu_scenes, oracle_nearest, oracle_scenes):
    """RT_FLAG_MESH_NEAREST: the device BVH returns the brute-force nearest triangle (strict <,
    ties to the lower index) — the same hits as the oracle's loop over every triangle, bit for bit."""
    rng = np.random.default_rng(4321)
    o, d = _rays_for(name, 30000 if name == "cubes" else 6000, rng)  # the oracle tests every triangle
    t_g, id_g, p_g, n_g = gpu_scenes[name].trace_ray(o, d, mesh_nearest=True)
    t_o, id_o, p_o, n_o = oracle_nearest[name].trace(o, d)
    exact = (id_g == id_o) & (t_g == t_o) & np.all(p_g == p_o, axis=1) & np.all(n_g == n_o, axis=1)
    assert exact.all(), f"{name}: {np.count_nonzero(~exact)} of {len(exact)} hits differ"
    # the two mesh semantics differ on some rays of the non-convex unicorn (the octree returns the
    # first subtree with a hit); on the convex cubes they coincide
    t_oct, id_oct, _, _ = oracle_scenes[name].trace(o, d)
    assert (np.count_nonzero(t_oct != t_o) > 0) == (name == "flying_unicorn")


@pytest.mark.parametrize("name", ["cubes", "flying_unicorn"])
def test_render_parity_mesh_nearest(name, rt, gpu_scenes, oracle_nearest):
    w, h, spp = (96, 72, 16) if name == "cubes" else (24, 18, 4)  # oracle: every triangle per mesh query
    rgb_g, sub_g, st = rt.render(gpu_scenes[name], w, h, spp, SEED, megakernel=True, mesh_nearest=True, want_sub=True)
    rgb_o, sub_o, st_o = oracle_nearest[name].render(w, h, spp, SEED)
    assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
    _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"{name}/nearest")
    with pytest.raises(rt.RtError):  # megakernel only
        rt.render(gpu_scenes[name], 8, 8, 4, SEED, megakernel=False, mesh_nearest=True)


def test_megakernel_equals_wavefront(rt, gpu_scenes):
    for name in ("cornell_box", "flying_unicorn"):
        a = rt.render(gpu_scenes[name], 128, 96, 8, SEED, want_sub=True, megakernel=True)
        b = rt.render(gpu_scenes[name], 128, 96, 8, SEED, want_sub=True, megakernel=False)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0]), name
        assert a[2]["vertices"] == b[2]["vertices"]


def test_split_tail_equals_wavefront(rt, gpu_scenes):
    """The megakernel hands out its last subpixels (up to one per resident lane, at most half the
    frame) as chunks of samples and sums their stored radiance afterwards in sample order
    (render_f64.hip: plan_tail, k_tail_sum_f64): the means must be the bits of the whole-subpixel
    sum. 96 samples per subpixel = 3 chunks of 32; the wavefront sums every subpixel in one lane.
    flying_unicorn runs the interleaved mesh megakernel, the others the analytic one."""
    for name in ("cornell_box", "cubes", "flying_unicorn"):
        for tile, step in [(None, 1), ((0, 1, 80, 20), 3)]:
            a = rt.render(gpu_scenes[name], 80, 60, 384, SEED, tile=tile, row_step=step, want_sub=True, megakernel=True)
            b = rt.render(gpu_scenes[name], 80, 60, 384, SEED, tile=tile, row_step=step, want_sub=True, megakernel=False)
            assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0]), (name, tile)
            assert a[2]["vertices"] == b[2]["vertices"]


@pytest.mark.parametrize("name,mis,spp", [("cornell_box", False, 256), ("cubes", False, 256),
                                          ("flying_unicorn", False, 256), ("chair_phong", True, 256),
                                          ("cornell_box", False, 308)])
def test_split_tail_parity_against_oracle(name, mis, spp, rt, gpu_scenes, oracle_scenes, oracle, tmp_path):
    """The split tail of every megakernel family against the oracle (1e-9 / RGB8), at 256 spp (64 samples per
    subpixel: the smallest spp that splits, plan_tail): chunk 0 of a split subpixel sums in place in sub_buf,
    the later chunks store each sample's radiance at tail_slot, and k_tail_sum_f64 continues chunk 0's partial
    sum. cornell: the analytic kernel (half the frame split); cubes: the 1024-thread query pool; the unicorn:
    the role-split pool (the whole frame split, six subpixels per path slot); a Phong chair with MIS: the
    512-thread Phong / MIS role-pool instance. 308 spp (77 samples per subpixel, 45 stored per split subpixel: an
    odd run, a partial last stage) takes k_tail_sum_f64's generic staging path. The launch must have split
    subpixels (rt_debug_last_split)."""
    if name == "chair_phong":
        from test_host_prep import extra_asset_scene

        p = extra_asset_scene(tmp_path, "chair.obj")
        text = open(p).read()
        floor = '{ type = "diffuse", kd = [0.75, 0.75, 0.75] }\ngeometry = { type = "plane", pos = [0.0, 0.0, 0.0]'
        assert floor in text
        text = text.replace(floor, floor.replace('{ type = "diffuse", kd = [0.75, 0.75, 0.75] }',
                                                 '{ type = "phong", kd = 0.5, ks = 0.3, power = 8, color_d = [0.7, 0.6, '
                                                 '0.5], color_s = [1.0, 1.0, 1.0] }'))
        open(p, "w").write(text)
        sc, orc = rt.Scene.from_toml(p), oracle.OracleScene(p)
    else:
        sc, orc = gpu_scenes[name], oracle_scenes[name]
    w, h = 32, 24
    tile = (0, 0, w, h) if name != "flying_unicorn" else None
    if name == "flying_unicorn":  # the mesh's part of the frame (a 32x24 crop of 640x480)
        w, h, tile = 640, 480, (300, 230, 32, 24)
    rgb_g, sub_g, st = rt.render(sc, w, h, spp, SEED, tile=tile, mis=mis, megakernel=True, want_sub=True)
    plan = rt.debug_last_split()
    nsub = tile[2] * tile[3] * 4
    assert plan["chunk"] == 32 and 0 < plan["split"] <= nsub, plan
    if name in ("flying_unicorn", "chair_phong"):
        assert plan["split"] == nsub, plan  # the walk kernels split the whole frame when it is this small
    rgb_o, sub_o, st_o = orc.render(w, h, spp, SEED, tile=tile, mis=mis)
    _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"{name}/split tail")


def test_tiling_invariance_and_determinism(rt, gpu_scenes):
    s = gpu_scenes["cubes"]
    w, h = 200, 150
    full, sub_full, _ = rt.render(s, w, h, 8, SEED, want_sub=True)
    again, sub_again, _ = rt.render(s, w, h, 8, SEED, want_sub=True)
    assert np.array_equal(sub_full, sub_again) and np.array_equal(full, again)
    tiles = [(0, 0, 64, 64), (64, 0, 136, 64), (0, 64, 200, 86), (37, 41, 19, 23)]
    for (x0, y0, tw, th) in tiles:
        t, sub_t, _ = rt.render(s, w, h, 8, SEED, tile=(x0, y0, tw, th), want_sub=True)
        assert np.array_equal(t, full[y0:y0 + th, x0:x0 + tw])
        assert np.array_equal(sub_t, sub_full[y0:y0 + th, x0:x0 + tw])
    # interleaved rows (bench.py's multi-GPU partition): tile row i = screen row y0 + i * row_step
    for mk in (True, False):
        for (y0, step, x0, tw) in [(0, 3, 0, 200), (2, 3, 0, 200), (1, 7, 50, 100)]:
            th = (h - y0 + step - 1) // step
            t, sub_t, _ = rt.render(s, w, h, 8, SEED, tile=(x0, y0, tw, th), want_sub=True, row_step=step,
                                    megakernel=mk)
            assert np.array_equal(t, full[y0::step, x0:x0 + tw])
            assert np.array_equal(sub_t, sub_full[y0::step, x0:x0 + tw])
    with pytest.raises(rt.RtError):  # last row outside the image
        rt.render(s, w, h, 8, SEED, tile=(0, 2, w, 50 + 1), row_step=3)


def test_spp_semantics(rt, gpu_scenes, oracle_scenes):
    s = gpu_scenes["cornell_box"]
    for spp in (0, 1, 3):  # server.rs:332 — spp/4 == 0 renders black (gamma(0) = 0.5 -> 0u8)
        rgb, _, st = rt.render(s, 64, 48, spp, SEED)
        assert st["samples"] == 0 and not rgb.any()
    a = rt.render(s, 64, 48, 4, SEED, want_sub=True)
    b = rt.render(s, 64, 48, 7, SEED, want_sub=True)
    assert np.array_equal(a[1], b[1])


def test_sample_pixel_and_chunks(rt, gpu_scenes, oracle_scenes):
    """sample_pixel and RenderJob.run (the reference's per-pixel seam and chunk loop, server.rs:157-199,
    320-368) against the CPU oracle's render of the same pixels, and against the full GPU frame."""
    s = gpu_scenes["cornell_box"]
    w, h, spp = 60, 45, 8
    full, sub_full, _ = rt.render(s, w, h, spp, SEED, want_sub=True)
    rgb_o, sub_o, _ = oracle_scenes["cornell_box"].render(w, h, spp, SEED)
    _assert_parity(full, sub_full, rgb_o, sub_o, "60x45 frame")
    # sample_pixel takes the reference's bottom-up y
    px = rt.sample_pixel(10, h - 1 - 7, w, h, spp, s, seed=SEED)
    assert px == tuple(int(c) for c in full[7, 10])
    assert np.all(np.abs(np.array(px) - rgb_o[7, 10].astype(int)) <= 1)
    msgs = rt.RenderJob(seed=SEED).run(s, w, h, spp)
    assert len(msgs) == h  # 60 px per message, one message per row at w = 60
    m = msgs[3]
    assert m[0] == 0 and m[1] == 60 and m[2:4] == (0).to_bytes(2, "little") and m[4:6] == (3).to_bytes(2, "little")
    assert m[6:] == full[3].tobytes()
    # every chunk against the oracle's frame (RGB8 within 1: the parity bound of _assert_parity)
    got = np.frombuffer(b"".join(bytes(x[6:]) for x in msgs), dtype=np.uint8).reshape(h, w, 3)
    assert np.abs(got.astype(int) - rgb_o.astype(int)).max() <= 1


def test_full_frame_properties(rt, gpu_scenes, oracle_scenes):
    """The bench frame size (1920x1080) at low spp: a crop equals an independent tile render and
    matches the oracle on that crop (the RNG is keyed by the global pixel id)."""
    s = gpu_scenes["cornell_box"]
    w, h, spp = 1920, 1080, 4
    full, sub_full, st = rt.render(s, w, h, spp, SEED, want_sub=True)
    assert st["samples"] == w * h * 4
    crop = (900, 500, 24, 16)
    x0, y0, tw, th = crop
    rgb_o, sub_o, _ = oracle_scenes["cornell_box"].render(w, h, spp, SEED, tile=crop)
    _assert_parity(full[y0:y0 + th, x0:x0 + tw], sub_full[y0:y0 + th, x0:x0 + tw], rgb_o, sub_o, "1080p crop")
    mean = full.reshape(-1, 3).mean(0)
    assert 60 < mean.mean() < 200


def test_mis_matches_nee_statistically(rt, gpu_scenes):
    """MIS (build-defined balance heuristic) must have the same expectation as the reference's NEE."""
    s = gpu_scenes["cornell_box"]
    w, h = 80, 60
    _, sub_nee, _ = rt.render(s, w, h, 512, SEED, want_sub=True)
    _, sub_mis, _ = rt.render(s, w, h, 512, SEED + 1, want_sub=True, mis=True)
    m_nee = sub_nee.mean(axis=(0, 1, 2))
    m_mis = sub_mis.mean(axis=(0, 1, 2))
    assert np.all(np.abs(m_mis - m_nee) / m_nee < 0.01), (m_nee, m_mis)


def test_mis_parity_small(rt, gpu_scenes, oracle_scenes):
    rgb_g, sub_g, st, rgb_o, sub_o, st_o = _render_pair(rt, gpu_scenes["cornell_box"], oracle_scenes["cornell_box"],
                                                        64, 48, 16, mis=True)
    _assert_parity(rgb_g, sub_g, rgb_o, sub_o, "cornell/mis")


@pytest.mark.parametrize("megakernel", [True, False], ids=["megakernel", "wavefront"])
def test_cancel(rt, gpu_scenes, megakernel):
    """RenderJob::stop semantics (server.rs:201-203): a set flag ends a long render early."""
    import ctypes
    import threading
    import time

    flag = ctypes.c_int32(0)
    timer = threading.Timer(0.3, lambda: setattr(flag, "value", 1))
    t0 = time.time()
    timer.start()
    _, _, st = rt.render(gpu_scenes["cornell_box"], 1920, 1080, 4096, SEED, megakernel=megakernel, cancel=flag)
    dt = time.time() - t0
    timer.cancel()
    assert st["cancelled"] and dt < 4.0, (st["cancelled"], dt)


# ---------------------------------------------------------------- f32 perf mode (RT_FLAG_FP32)
# Statistical parity only. The f32 kernel draws the same RNG streams in the same
# order (a draw is the top 24 bits of the f64 draw's 64-bit word), so its frame tracks the f64 frame
# path for path and the comparison is paired, pixel by pixel. Bounds (measured margins in DESIGN.md §10,
# profiles/r01h_fp32.log):
#   * per-channel image mean of the pixel values: |rel| <= 0.5%;
#   * 16x16-block means: |diff| <= 4 paired standard errors, or <= 1% of the block mean;
#   * RGB8 within 1 on >= 93% of pixels, mean |dRGB8| <= 0.3.
def _assert_fp32_stats(sub_f, sub_r, rgb_f, rgb_r, what):
    cf = np.clip(sub_f, 0, 1).mean(axis=2)  # pixel values before gamma (server.rs:358-360)
    cr = np.clip(sub_r, 0, 1).mean(axis=2)
    m_f, m_r = cf.mean(axis=(0, 1)), cr.mean(axis=(0, 1))
    assert np.all(np.abs(m_f - m_r) <= 0.005 * m_r), f"{what}: image means {m_f} vs {m_r}"
    h, w = cf.shape[:2]
    B = 16
    hb, wb = h // B, w // B
    d = (cf - cr)[:hb * B, :wb * B].reshape(hb, B, wb, B, 3)
    bm = np.abs(d.mean(axis=(1, 3)))
    se = d.std(axis=(1, 3)) / B
    ref = cr[:hb * B, :wb * B].reshape(hb, B, wb, B, 3).mean(axis=(1, 3))
    bad = (bm > 4 * se) & (bm > 0.01 * np.maximum(ref, 1e-3))
    assert bad.mean() <= 0.01, f"{what}: {np.count_nonzero(bad)} of {bad.size} block means off"
    diff = np.abs(rgb_f.astype(int) - rgb_r.astype(int))
    assert np.all(diff <= 1, axis=-1).mean() >= 0.93, f"{what}: RGB8 within 1 on too few pixels"
    assert diff.mean() <= 0.3, f"{what}: mean |dRGB8| {diff.mean():.3f}"


@pytest.mark.parametrize("name,mis", [("cornell_box", False), ("cornell_box", True), ("cubes", False),
                                      ("cubes", True)])
def test_fp32_statistical_parity(name, mis, rt, gpu_scenes, oracle_scenes, oracle_nearest):
    w, h, spp = 96, 80, 64
    rgb_f, sub_f, st = rt.render(gpu_scenes[name], w, h, spp, SEED, mis=mis, want_sub=True, fp32=True)
    assert st["samples"] == w * h * spp
    # cubes: the convex cubes give the same hits under both mesh semantics (test_trace_mesh_nearest_bit_exact)
    ref = oracle_scenes[name]
    rgb_o, sub_o, st_o = ref.render(w, h, spp, SEED, mis=mis)
    # the GPU ends zero-throughput paths early (the oracle keeps walking them, at zero radiance)
    assert 0.9 * st_o["vertices"] <= st["vertices"] <= 1.01 * st_o["vertices"]
    _assert_fp32_stats(sub_f, sub_o, rgb_f, rgb_o, f"{name}/f32{'/mis' if mis else ''}")


def test_fp32_statistical_parity_mesh(rt, gpu_scenes, oracle_nearest):
    """The unicorn in f32 (nearest-triangle meshes) against the f64 nearest-triangle path, which is
    bit-exact against the oracle's brute-force loop (test_render_parity_mesh_nearest), at a size the
    brute-force oracle cannot reach; plus a direct oracle check on a small tile."""
    sc = gpu_scenes["flying_unicorn"]
    w, h, spp = 192, 144, 64
    rgb_f, sub_f, st = rt.render(sc, w, h, spp, SEED, want_sub=True, fp32=True)
    rgb_d, sub_d, st_d = rt.render(sc, w, h, spp, SEED, want_sub=True, megakernel=True, mesh_nearest=True)
    assert abs(st["vertices"] / st_d["vertices"] - 1) < 0.01
    _assert_fp32_stats(sub_f, sub_d, rgb_f, rgb_d, "flying_unicorn/f32")
    rgb_f, sub_f, _ = rt.render(sc, 24, 18, 4, SEED, want_sub=True, fp32=True)
    rgb_o, sub_o, _ = oracle_nearest["flying_unicorn"].render(24, 18, 4, SEED)
    assert np.all(np.abs(rgb_f.astype(int) - rgb_o.astype(int)) <= 1, axis=-1).mean() >= 0.8


def test_fp32_rejects_unsupported(rt, gpu_scenes):
    """Phong BRDFs and mesh lights stay on the f64 path: RT_FLAG_FP32 returns RT_E_INVAL for them."""
    phong = rt.Scene.from_desc([50, 52, 295.6], [0, -0.042612, -1], [
        dict(geom_kind=1, pos=[0, 0, 0], n=[0, 1, 0], brdf_kind=2, phong_kd=0.5, phong_ks=0.3, phong_power=8,
             color_d=[0.7, 0.7, 0.7], color_s=[1, 1, 1]),
        dict(geom_kind=0, pos=[50, 70, 100], r=4, brdf_kind=0, k=[0, 0, 0], emitted=[50, 50, 50])])
    with pytest.raises(rt.RtError):
        rt.render(phong, 8, 8, 4, SEED, fp32=True)
    rt.render(phong, 8, 8, 4, SEED)  # the f64 path renders it


def test_fp32_cancel_and_tiling(rt, gpu_scenes):
    """The f32 kernel polls the cancel flag like the f64 megakernel, and its frame does not depend on
    the tiling (the RNG is keyed by global pixel, sample and subpixel)."""
    import ctypes
    import threading
    import time

    flag = ctypes.c_int32(0)
    timer = threading.Timer(0.3, lambda: setattr(flag, "value", 1))
    t0 = time.time()
    timer.start()
    _, _, st = rt.render(gpu_scenes["cornell_box"], 1920, 1080, 8192, SEED, fp32=True, cancel=flag)
    dt = time.time() - t0
    timer.cancel()
    assert st["cancelled"] and dt < 4.0, (st["cancelled"], dt)
    sc = gpu_scenes["cubes"]
    full, sub_full, _ = rt.render(sc, 96, 64, 8, SEED, fp32=True, want_sub=True)
    tile, sub_tile, _ = rt.render(sc, 96, 64, 8, SEED, tile=(32, 16, 40, 24), fp32=True, want_sub=True)
    assert np.array_equal(tile, full[16:40, 32:72]) and np.array_equal(sub_tile, sub_full[16:40, 32:72])


@pytest.mark.parametrize("asset", ["chair.obj", "crewmate.obj"])
def test_extra_assets_parity(asset, rt, oracle, tmp_path):
    """The reference's other OBJ assets in a room: f64 megakernel and wavefront
    against the oracle (1e-9 / RGB8 bounds of §8c.1), and the f32 mode against the f64
    nearest-triangle path (§8c.2 bounds)."""
    from test_host_prep import extra_asset_scene

    p = extra_asset_scene(tmp_path, asset)
    sc, orc = rt.Scene.from_toml(p), oracle.OracleScene(p)
    w, h, spp = 64, 48, 8
    rgb_o, sub_o, st_o = orc.render(w, h, spp, SEED)
    for mk in (True, False):
        rgb_g, sub_g, st = rt.render(sc, w, h, spp, SEED, megakernel=mk, want_sub=True)
        assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
        _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"{asset}/{'mk' if mk else 'wf'}")
    w, h, spp = 128, 96, 64
    rgb_f, sub_f, _ = rt.render(sc, w, h, spp, SEED, want_sub=True, fp32=True)
    rgb_d, sub_d, _ = rt.render(sc, w, h, spp, SEED, want_sub=True, megakernel=True, mesh_nearest=True)
    _assert_fp32_stats(sub_f, sub_d, rgb_f, rgb_d, f"{asset}/f32")


def test_two_deep_meshes_parity(rt, oracle, tmp_path):
    """Two deep octrees in one scene (chair.obj and crewmate.obj side by side): the walk pool takes
    queries that walk both meshes (a query's walks of the two octrees run one after the other, in the
    scene's object order, with the reference's tie rule between their hits); megakernel and wavefront
    against the oracle at the 1e-9 / RGB8 bounds."""
    import os
    from test_host_prep import EXTRA_ASSET_SCENE, REPO

    d = tmp_path / "two"
    d.mkdir()
    os.symlink(os.path.join(REPO, "scenes", "assets"), d / "assets")
    chair = EXTRA_ASSET_SCENE.format(asset="chair.obj", scale=30.0, ty=24.5)
    crew = EXTRA_ASSET_SCENE.format(asset="crewmate.obj", scale=0.25, ty=-73.7)
    mesh_obj = crew[crew.index("[[objects]]\nbrdf = { type = \"diffuse\", kd = [0.8, 0.7, 0.5] }"):]
    mesh_obj = mesh_obj[:mesh_obj.index("[[objects]]\nemitted")]
    text = chair.replace("translate = [50.0,", "translate = [28.0,") + mesh_obj.replace("translate = [50.0,", "translate = [72.0,")
    p = d / "s.toml"
    p.write_text(text)
    sc, orc = rt.Scene.from_toml(str(p)), oracle.OracleScene(str(p))
    assert len(sc.mesh(5)["kind"]) >= 64 and len(sc.mesh(7)["kind"]) >= 64  # both walked by the pool
    w, h, spp = 64, 48, 8
    rgb_o, sub_o, st_o = orc.render(w, h, spp, SEED)
    for mk in (True, False):
        rgb_g, sub_g, st = rt.render(sc, w, h, spp, SEED, megakernel=mk, want_sub=True)
        assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
        _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"two meshes/{'mk' if mk else 'wf'}")


@pytest.mark.parametrize("phong", [False, True], ids=["diffuse", "phong"])
def test_deep_mesh_mis_and_phong_parity(phong, rt, oracle, tmp_path):
    """The role-split pool's other instances on a deep octree (chair.obj): MIS on and off (the 768-thread
    instances with and without pdf_prev in the path record), and with Phong objects (a Phong floor and a
    Phong sphere: the 512-thread instances, render_mesh_f64.hip RoleShape), against the oracle at the
    1e-9 / RGB8 bounds (scene.rs:56-98 Phong lobes, scene.rs:186-215 MIS)."""
    from test_host_prep import extra_asset_scene

    p = extra_asset_scene(tmp_path, "chair.obj")
    text = open(p).read()
    if phong:
        floor = 'brdf = { type = "diffuse", kd = [0.75, 0.75, 0.75] }\ngeometry = { type = "plane", pos = [0.0, 0.0, 0.0], n = [0.0, 1.0, 0.0] }'
        assert floor in text
        text = text.replace(floor, floor.replace('{ type = "diffuse", kd = [0.75, 0.75, 0.75] }', '{ type = "phong", kd = 0.5, '
                                                 'ks = 0.3, power = 8, color_d = [0.7, 0.6, 0.5], color_s = [1.0, 1.0, 1.0] }'))
        text += ('[[objects]]\nbrdf = { type = "phong", kd = 0.2, ks = 0.7, power = 24, color_d = [0.9, 0.3, 0.3], '
                 'color_s = [1.0, 1.0, 1.0] }\ngeometry = { type = "sphere", pos = [22.0, 12.0, 60.0], r = 12.0 }\n')
        open(p, "w").write(text)
    sc, orc = rt.Scene.from_toml(p), oracle.OracleScene(p)
    assert len(sc.mesh(5)["kind"]) >= 64  # a deep octree: the role-split pool walks it
    w, h, spp = 64, 48, 8
    for mis in (False, True):
        rgb_o, sub_o, st_o = orc.render(w, h, spp, SEED, mis=mis)
        rgb_g, sub_g, st = rt.render(sc, w, h, spp, SEED, megakernel=True, mis=mis, want_sub=True)
        assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
        _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"chair/{'phong' if phong else 'diffuse'}/{'mis' if mis else 'nee'}")


# ---------------------------------------------------------------- reference quirks off the 3 scenes
QUIRK_SCENE = """
[camera]
pos = [0.0, 6.0, 60.0]
dir = [0.0, -0.1, -1.0]
[[objects]]
emitted = [12.0, 12.0, 12.0]
brdf = { type = "diffuse", kd = [0.0, 0.0, 0.0] }
geometry = { type = "cube", pos = [6.0, 14.0, -4.0], size = 4.0 }
transforms = [ { rotate_y = 0.3 } ]
[[objects]]
brdf = { type = "phong", kd = 0.5, ks = 0.3, power = 8, color_d = [0.7, 0.6, 0.5], color_s = [1.0, 1.0, 1.0] }
geometry = { type = "plane", pos = [0.0, -5.0, 0.0], n = [0.0, 1.0, 0.0] }
[[objects]]
brdf = { type = "diffuse", kd = [0.6, 0.6, 0.75] }
geometry = { type = "plane", pos = [0.0, 0.0, -30.0], n = [0.0, 0.0, 1.0] }
[[objects]]
brdf = { type = "phong", kd = 0.2, ks = 0.7, power = 24, color_d = [0.9, 0.3, 0.3], color_s = [1.0, 1.0, 1.0] }
geometry = { type = "sphere", pos = [-8.0, 0.0, 2.0], r = 5.0 }
[[objects]]
brdf = { type = "specular", ks = [0.95, 0.95, 0.95] }
geometry = { type = "sphere", pos = [9.0, -1.0, 6.0], r = 4.0 }
[[objects]]
brdf = { type = "diffuse", kd = [0.8, 0.8, 0.8] }
geometry = { type = "prism", pos = [-2.0, -5.0, -12.0], size = [6.0, 9.0, 5.0] }
"""


def test_phong_and_mesh_light_parity(rt, oracle, tmp_path):
    """Phong BRDFs with the reference's unrotated lobes (scene.rs:56-98) and a
    triangle-mesh emitter (the first emitting object is the light, scene.rs:129-137) sampled with
    WeightedIndex + Triangle::sample's missing `+ a` (geometry.rs:588-592, 622-635), on the f64
    megakernel and wavefront against the oracle at the 1e-9 / RGB8 bounds; MIS on and off."""
    p = tmp_path / "quirks.toml"
    p.write_text(QUIRK_SCENE)
    sc, orc = rt.Scene.from_toml(str(p)), oracle.OracleScene(str(p))
    assert sc.info()["light"] == 0 == orc.light and orc.objects[0] == "cube"
    w, h, spp = 64, 48, 16
    for mis in (False, True):
        rgb_o, sub_o, st_o = orc.render(w, h, spp, SEED, mis=mis)
        assert rgb_o.mean() > 5  # the frame is not black: light reaches the camera
        for mk in (True, False):
            rgb_g, sub_g, st = rt.render(sc, w, h, spp, SEED, megakernel=mk, mis=mis, want_sub=True)
            assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
            _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"quirks/{'mk' if mk else 'wf'}/{'mis' if mis else 'nee'}")


ROOT_LEAF_OBJ = """v 0 0 0
v 4 0 0
v 0 0 4
v 0 5 0
v 4 5 4
f 1 2 3
f 1 2 4
f 1 3 4
f 2 3 4
f 2 5 4
f 3 5 4
"""
ROOT_LEAF_SCENE = """
[camera]
pos = [50.0, 30.0, 160.0]
dir = [0.0, -0.1, -1.0]
[[objects]]
brdf = { type = "diffuse", kd = [0.75, 0.75, 0.75] }
geometry = { type = "plane", pos = [0.0, 0.0, 0.0], n = [0.0, 1.0, 0.0] }
[[objects]]
brdf = { type = "diffuse", kd = [0.75, 0.25, 0.25] }
geometry = { type = "plane", pos = [0.0, 0.0, 0.0], n = [0.0, 0.0, 1.0] }
[[objects]]
brdf = { type = "diffuse", kd = [0.9, 0.9, 0.9] }
geometry = { type = "mesh", path = "pyr.obj" }
transforms = [ { scale = 6.0 }, { scale = -0.8 }, { translate = [50.0, 20.0, 60.0] } ]
[[objects]]
emitted = [50.0, 50.0, 50.0]
brdf = { type = "diffuse", kd = [0.0, 0.0, 0.0] }
geometry = { type = "sphere", pos = [50.0, 70.0, 100.0], r = 4.0 }
"""


def test_root_leaf_mesh_with_scale_quirk(rt, oracle, tmp_path):
    """A mesh of <= 9 triangles is a single octree leaf, which the reference tests without any box
    (geometry.rs:1237-1241, 1276-1293). A negative `scale` below -0.5 leaves the stored bounding box
    smaller than the triangles (geometry.rs:503-506), so the device's early-out culls must use a box
    that encloses both (DevMesh::cull_box): trace_ray bit-exact against the oracle, with hits outside
    the stored box, in both mesh semantics, and a render at parity."""
    (tmp_path / "assets").mkdir()
    (tmp_path / "assets" / "pyr.obj").write_text(ROOT_LEAF_OBJ)
    p = tmp_path / "leaf.toml"
    p.write_text(ROOT_LEAF_SCENE)
    sc, orc = rt.Scene.from_toml(str(p)), oracle.OracleScene(str(p))
    info = sc.info()
    assert info["nodes"] == 1 and info["leaves"] == 1
    m = sc.mesh(2)
    lo, hi = m["bbox"][:3], m["bbox"][3:]
    v = m["vertices"]
    assert np.any(v < lo - 1e-9) and np.any(v > hi + 1e-9)  # the stored box no longer encloses the mesh
    rng = np.random.default_rng(77)
    n = 20000
    tgt = rng.uniform(v.min(0) - 1, v.max(0) + 1, size=(n, 3))
    o = rng.uniform([5, 2, 80], [95, 60, 200], size=(n, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t_g, id_g, p_g, n_g = sc.trace_ray(o, d)
    t_o, id_o, p_o, n_o = orc.trace(o, d)
    exact = (id_g == id_o) & (t_g == t_o) & np.all(p_g == p_o, axis=1) & np.all(n_g == n_o, axis=1)
    assert exact.all(), f"{np.count_nonzero(~exact)} of {n} hits differ"
    on_mesh = id_o == 2
    outside = on_mesh & np.any((p_o < lo - 1e-6) | (p_o > hi + 1e-6), axis=1)
    assert on_mesh.sum() > 1000 and outside.sum() > 100, (on_mesh.sum(), outside.sum())
    orc_n = oracle.OracleScene(str(p), mesh_nearest=True)
    t_g, id_g, p_g, n_g = sc.trace_ray(o, d, mesh_nearest=True)
    t_o, id_o, p_o, n_o = orc_n.trace(o, d)
    assert np.array_equal(id_g, id_o) and np.array_equal(t_g, t_o) and np.array_equal(p_g, p_o)
    rgb_o, sub_o, _ = orc.render(64, 48, 16, SEED)
    for mk in (True, False):
        rgb_g, sub_g, _ = rt.render(sc, 64, 48, 16, SEED, megakernel=mk, want_sub=True)
        _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"root-leaf/{'mk' if mk else 'wf'}")


def test_octree_first_hit_subtree_known_answer(rt, oracle, tmp_path):
    """The hand-derived octree case of tests/octree_kat.py (geometry.rs:1245-1295) on
    the device through rt_trace_rays: the walk returns the FARTHER triangle T_far, bit-identical to
    the oracle; the nearest-triangle mode (RT_FLAG_MESH_NEAREST) returns T_near."""
    import octree_kat as K

    path = K.write_scene(tmp_path)
    sc = rt.Scene.from_toml(path)
    info = sc.info()
    assert (info["nodes"], info["parents"], info["leaves"], info["refs"]) == (8, 3, 5, 14)
    o, d = K.rays()
    t_oct, t_near = K.expected_t(d)
    orc = oracle.OracleScene(path)
    for nearest, want, x0 in ((False, t_oct, K.T_FAR_X), (True, t_near, K.T_NEAR_X)):
        t_g, id_g, p_g, n_g = sc.trace_ray(o, d, mesh_nearest=nearest)
        t_o, id_o, p_o, n_o = (oracle.OracleScene(path, mesh_nearest=True) if nearest else orc).trace(o, d)
        assert list(id_g) == [0, 0] and np.allclose(t_g, want, rtol=1e-12, atol=0)
        assert abs(p_g[0, 0] - x0) < 1e-4
        assert np.array_equal(t_g, t_o) and np.array_equal(p_g, p_o) and np.array_equal(n_g, n_o)


SKINNY_SCENE = """
[camera]
pos = [50.0, 50.0, 300.0]
dir = [0.0, 0.0, -1.0]
[[objects]]
brdf = {{ type = "diffuse", kd = [0.8, 0.8, 0.8] }}
geometry = {{ type = "mesh", path = "{obj}" }}
[[objects]]
emitted = [50.0, 50.0, 50.0]
brdf = {{ type = "diffuse", kd = [0.0, 0.0, 0.0] }}
geometry = {{ type = "sphere", pos = [50.0, 5000.0, 50.0], r = 4.0 }}
"""


def _skinny_mesh_scene(tmp_path, n=3000, seed=7):
    """Needle triangles (length 1..10, width 1e-7..1e-3) in random orientations around (50, 50, 50): the
    meshes where the slot walk's subtree bounds (a triangle's vertex bounds padded by 1e-7 of the scene
    scale) sit closest to the triangles' own rounding."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(40.0, 60.0, size=(n, 3))
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    v = np.cross(u, rng.normal(size=(n, 3)))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    length = rng.uniform(1.0, 10.0, size=(n, 1))
    width = 10.0 ** rng.uniform(-7.0, -3.0, size=(n, 1))
    a, b, cc = c - 0.5 * length * u, c + 0.5 * length * u, c + width * v
    verts = np.stack([a, b, cc], axis=1).reshape(-1, 3)
    d = tmp_path / "skinny"
    (d / "assets").mkdir(parents=True)
    lines = [f"v {x!r} {y!r} {z!r}" for x, y, z in verts.tolist()]
    lines += [f"f {3 * i + 1} {3 * i + 2} {3 * i + 3}" for i in range(n)]
    (d / "assets" / "needles.obj").write_text("\n".join(lines) + "\n")
    p = d / "s.toml"
    p.write_text(SKINNY_SCENE.format(obj="needles.obj"))
    return str(p), verts.reshape(n, 3, 3)


def test_slot_walk_exact_on_grazing_rays(rt, oracle, tmp_path, monkeypatch):
    """The slot walk's subtree-bounds culls (kid_tight_hit, path_f64.h) on adversarial rays: a mesh of
    needle triangles, rays from far origins (1 to 1e5 scene units away) aimed at the triangles'
    vertices and edges — where a ray grazes a subtree's padded bounds — with and without ulp-scale
    offsets. The trace must be bit-identical to the walk without the culls (the same scene loaded
    without slot tables, RT_TEST_SLOT_MAX_PID=0: the reference's visiting order over node_kids) and to the
    oracle's walk (geometry.rs:1237-1295)."""
    path, tri = _skinny_mesh_scene(tmp_path)
    slots = rt.Scene.from_toml(path)
    monkeypatch.setenv("RT_TEST_SLOT_MAX_PID", "0")
    plain = rt.Scene.from_toml(path)
    monkeypatch.delenv("RT_TEST_SLOT_MAX_PID")
    assert slots.info()["slot_tables"] == 1 and plain.info()["slot_tables"] == 0
    assert slots.info()["parents"] > 8  # a deep octree
    rng = np.random.default_rng(11)
    n = 120000
    k = rng.integers(0, tri.shape[0], n)
    w = rng.uniform(size=(n, 1))
    kind = rng.integers(0, 3, n)
    tgt = np.where((kind == 0)[:, None], tri[k, rng.integers(0, 3, n)],                       # a vertex
                   np.where((kind == 1)[:, None], (1 - w) * tri[k, 0] + w * tri[k, 1],         # the long edge
                            (1 - w) * tri[k, 1] + w * tri[k, 2]))                             # a short edge
    tgt = tgt * (1.0 + rng.choice([0.0, 1.0, -1.0], size=(n, 1)) * 2.0 ** -52 * rng.integers(0, 8, (n, 1)))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = tgt - d * 10.0 ** rng.uniform(0.0, 5.0, size=(n, 1))
    t_s, id_s, p_s, n_s = slots.trace_ray(o, d)
    t_p, id_p, p_p, n_p = plain.trace_ray(o, d)
    assert (id_s == 0).mean() > 0.2  # many rays reach a needle
    assert np.array_equal(id_s, id_p) and np.array_equal(t_s, t_p), \
        f"slot walk differs from the node_kids walk on {np.count_nonzero((id_s != id_p) | (t_s != t_p))} rays"
    assert np.array_equal(p_s, p_p) and np.array_equal(n_s, n_p)
    t_o, id_o, p_o, n_o = oracle.OracleScene(path).trace(o, d)
    exact = (id_s == id_o) & (t_s == t_o) & np.all(p_s == p_o, axis=1) & np.all(n_s == n_o, axis=1)
    assert exact.all(), f"{np.count_nonzero(~exact)} of {n} rays differ from the oracle"


# Generic (non-axis) planes between the meshes in object order: the compact table's gen slots then mix
# analytic objects and meshes (CompactTab::gen_analytic / gen_mesh / gen_cull32), which the per-ray loops
# of both mesh kernels read instead of the objects.
TILTED_PLANE = """[[objects]]
brdf = {{ type = "diffuse", kd = [{k}, 0.7, 0.6] }}
geometry = {{ type = "plane", pos = [0.0, {y}, 0.0], n = [{nx}, 1.0, {nz}] }}
"""
GEN_CUBES_SCENE = """
[camera]
pos = [50.0, 52.0, 295.6]
dir = [0.0, -0.042612, -1.0]
[[objects]]
brdf = { type = "diffuse", kd = [0.75, 0.25, 0.25] }
geometry = { type = "plane", pos = [1.0, 0.0, 0.0], n = [-1.0, 0.0, 0.0] }
[[objects]]
brdf = { type = "diffuse", kd = [0.25, 0.25, 0.75] }
geometry = { type = "plane", pos = [99.0, 0.0, 0.0], n = [-1.0, 0.0, 0.0] }
[[objects]]
brdf = { type = "diffuse", kd = [0.75, 0.75, 0.75] }
geometry = { type = "plane", pos = [0.0, 0.0, 0.0], n = [0.0, 0.0, -1.0] }
""" + TILTED_PLANE.format(k=0.7, y=-2.0, nx=0.05, nz=0.02) + """
[[objects]]
brdf = { type = "diffuse", kd = [0.9, 0.9, 0.9] }
geometry = { type = "cube", pos = [20.5, 8.0, 40.5], size = 22.0 }
transforms = [ { rotate_y = 0.5 } ]
""" + TILTED_PLANE.format(k=0.6, y=80.0, nx=-0.03, nz=0.04) + """
[[objects]]
brdf = { type = "diffuse", kd = [0.9, 0.9, 0.9] }
geometry = { type = "cube", pos = [63.0, 6.0, 30.0], size = 20.0 }
transforms = [ { rotate_y = -0.6 } ]
[[objects]]
emitted = [50.0, 50.0, 50.0]
brdf = { type = "diffuse", kd = [0.0, 0.0, 0.0] }
geometry = { type = "sphere", pos = [50.0, 70.0, 100.0], r = 4.0 }
"""


def test_generic_planes_between_meshes_parity(rt, oracle, tmp_path):
    """Tilted planes (the generic intersector) placed before, between and after the meshes in object
    order, so the gen slots alternate analytic objects and meshes: the deep-octree walk pool (chair.obj)
    and the flat-mesh query pool (two cubes, the no-mirror 768-thread instance) against the oracle at the
    1e-9 / RGB8 bounds, megakernel and wavefront."""
    import os
    from test_host_prep import EXTRA_ASSET_SCENE, REPO

    d = tmp_path / "gen"
    d.mkdir()
    os.symlink(os.path.join(REPO, "scenes", "assets"), d / "assets")
    chair = EXTRA_ASSET_SCENE.format(asset="chair.obj", scale=30.0, ty=24.5)
    i = chair.index("[[objects]]\nbrdf = { type = \"diffuse\", kd = [0.8, 0.7, 0.5] }")
    j = chair.index("[[objects]]\nemitted")
    walk_text = (chair[:i] + TILTED_PLANE.format(k=0.7, y=-2.0, nx=0.05, nz=0.02) + chair[i:j] +
                 TILTED_PLANE.format(k=0.6, y=80.0, nx=-0.03, nz=0.04) + chair[j:])
    cases = {"walk pool": walk_text, "query pool": GEN_CUBES_SCENE}
    for what, text in cases.items():
        p = d / (what.replace(" ", "_") + ".toml")
        p.write_text(text)
        sc, orc = rt.Scene.from_toml(str(p)), oracle.OracleScene(str(p))
        w, h, spp = 64, 48, 8
        rgb_o, sub_o, st_o = orc.render(w, h, spp, SEED)
        assert rgb_o.mean() > 5
        for mk in (True, False):
            rgb_g, sub_g, st = rt.render(sc, w, h, spp, SEED, megakernel=mk, want_sub=True)
            assert 0.9 * st_o["vertices"] <= st["vertices"] <= st_o["vertices"]
            _assert_parity(rgb_g, sub_g, rgb_o, sub_o, f"generic planes/{what}/{'mk' if mk else 'wf'}")
