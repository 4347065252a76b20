"""GPU parity tests (MI355X): the HIP kernels through the C ABI against the FP64 oracle.

The oracle's Philox mode consumes the same random numbers as the device, so images compare
per pixel.  Tolerances (reference precision is binary64, Core.hs:29-31):
  * binary64 kernel (the default): >= 99.9 % of pixels within 1e-9 relative of the oracle
    (max(|ref|, 1e-3) scale) — the remaining pixels hold a sample whose path split on a
    decision within rounding of its threshold; the worst pixel within 2 L / spp of the oracle,
    L = the largest radiance one sample can carry in the scene (the brightest emitter or
    background; a divergent sample moves its pixel's mean by at most L / spp), i.e. at most
    two divergent samples in any pixel;
  * FP32 kernel (RT_EXEC_F32): >= 99 % of pixels within 1e-3 (relative above 1; >= 97 % on
    demo1's glass / metal spheres), the worst pixel within 4 L / spp + 1e-3;
  * both: per-channel 8x8-block RMSE against the oracle <= 0.5 x the seed-to-seed noise floor
    of the published renders (FP32 on the glass-cuboid test scene: 1.5 x), means within 0.5 %;
  * full-size Cornell box vs the reference's cornell_box_redirect.png: 8x8-block RMSE within
    1.5x the measured seed-to-seed noise floor, means within 1 %;
  * row-sharded renders, device lists and item chunkings are bit-identical; repeated renders
    are bit-identical; the 8-bit epilogue equals the host encoder bit for bit.
"""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, as_published, block8, pixel_agreement, record_measure

pytestmark = pytest.mark.gpu

import raytrace_amd as R  # noqa: E402
from raytrace_amd import scenes  # noqa: E402

# (name, scene, kwargs, FP32 per-pixel bar, L = the largest radiance of one sample: the Cornell
# light (15) or the background / sky (1))
CASES = [
    ("cornell", scenes.cornell_box, dict(spp=16, width=96), 0.99, 15.0),
    ("readme", scenes.readme_scene, dict(spp=16, width=120), 0.99, 1.0),
    ("demo1", scenes.demo1, dict(width=160, spp=8), 0.97, 1.0),
    ("bunny_cornell", scenes.bunny_cornell, dict(width=80, spp=8), 0.99, 15.0),
    ("pawn_fog", scenes.pawn_fog, dict(width=80, spp=8), 0.99, 1.0),
    ("pawn_test", scenes.pawn_test, dict(width=80, spp=8), 0.99, 1.0),
    ("demo2", scenes.demo2, dict(width=96, spp=8), 0.95, 7.0),
]


def _floor():
    with open(os.path.join(GOLDEN, "noise_floor.json")) as f:
        d = json.load(f)
    return {"cornell": np.array(d["cornell_box_redirect"]["block8_rmse"]),
            "readme": np.array(d["example_image"]["block8_rmse"])}


def assert_parity(img, ref, precision, need32=0.99, floor=None, what="", spp=8, lmax=1.0, floor_mult=0.5):
    """The file docstring's per-pixel, worst-pixel, block and mean bars."""
    assert img.shape == ref.shape
    assert img.dtype == (np.float64 if precision == "f64" else np.float32)
    assert np.isfinite(img).all(), what
    d = np.abs(img.astype(np.float64) - ref)
    if precision == "f64":
        rel = (d / np.maximum(np.abs(ref), 1e-3)).max(-1)
        frac = float((rel <= 1e-9).mean())
        assert frac >= 0.999, (what, frac)
        assert d.max() <= 2 * lmax / spp, (what, float(d.max()), 2 * lmax / spp)
    else:
        rel = (d / np.maximum(np.abs(ref), 1.0)).max(-1)
        frac = float((rel < 1e-3).mean())
        assert frac >= need32, (what, frac)
        assert d.max() <= 4 * lmax / spp + 1e-3, (what, float(d.max()), 4 * lmax / spp)
    if floor is not None and img.shape[0] >= 8 and img.shape[1] >= 8:
        rmse = np.sqrt(((block8(img.astype(np.float64)) - block8(ref)) ** 2).reshape(-1, 3).mean(0))
        assert (rmse <= floor_mult * floor).all(), (what, rmse, floor_mult * floor)
    np.testing.assert_allclose(img.reshape(-1, 3).mean(0), ref.reshape(-1, 3).mean(0), rtol=5e-3, atol=1e-6)


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from raytrace_amd import _lib
    _lib.load()
    return torch


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name,fn,kw,need,lmax", CASES, ids=[c[0] for c in CASES])
def test_gpu_matches_oracle_per_pixel(gpu, oracle_mod, name, fn, kw, need, lmax, precision):
    cs, world, seed = fn(**kw)
    img = R.raytrace(cs, world, seed, precision=precision)
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    assert_parity(img, ref, precision, need, _floor()["cornell"], name, kw["spp"], lmax)


# Every BASELINE config at its FULL resolution (reduced spp), compared with the oracle on every
# 8th row: the per-pixel, worst-pixel, 8x8-block (over the sampled rows) and mean bars.
FULL = [
    ("readme", scenes.readme_scene, dict(spp=8), "readme", 1.0),
    ("cornell", scenes.cornell_box, dict(spp=8), "cornell", 15.0),
    ("demo1", scenes.demo1, dict(spp=4), "cornell", 1.0),
    ("demo1_1200x800", scenes.demo1_1200x800, dict(spp=2), "cornell", 1.0),
    ("bunny_cornell", scenes.bunny_cornell, dict(spp=4), "cornell", 15.0),
    ("pawn_fog", scenes.pawn_fog, dict(spp=4), "cornell", 1.0),
    ("bunny_instances", scenes.bunny_instances, dict(spp=4, n=8), "cornell", 15.0),
    ("demo2", scenes.demo2, dict(spp=4), "cornell", 7.0),
]


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name,fn,kw,fl,lmax", FULL, ids=[c[0] for c in FULL])
def test_full_resolution_parity_on_row_subset(gpu, oracle_mod, name, fn, kw, fl, lmax, precision):
    from raytrace_amd.camera import image_height
    cs, world, seed = fn(**kw)
    h, w = image_height(cs), int(cs.cs_imageWidth)
    img = R.raytrace(cs, world, seed, precision=precision)
    assert img.shape == (h, w, 3)
    rows = np.arange(0, h, 8)
    pix = (rows[:, None] * w + np.arange(w)[None, :]).reshape(-1).astype(np.int32)
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX, pixels=pix).reshape(len(rows), w, 3)
    need = 0.97 if name.startswith("demo1") else 0.95 if name == "demo2" else 0.99
    assert_parity(img[rows], ref, precision, need, _floor()[fl], name, kw["spp"], lmax)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_gpu_matches_kernel_emulator(gpu, emu_mod, precision):
    """Same source (rt_trace.h) on the host: identical numbers up to FP contraction / libm (the
    device's refined hardware binary64 reciprocals and its sin / cos polynomial differ from the
    host's IEEE / libm results by ulps)."""
    cs, world, seed = scenes.cornell_box(spp=8, width=64)
    a = R.raytrace(cs, world, seed, precision=precision)
    b = emu_mod.render(cs, world, seed, precision=precision)
    if precision == "f64":
        rel = (np.abs(a - b) / np.maximum(np.abs(b), 1e-3)).max(-1)
        assert (rel <= 1e-9).mean() >= 0.999
    else:
        assert pixel_agreement(a, b, 1e-4) > 0.99


def test_full_cornell_matches_published_render(gpu, golden_stats):
    stats, floors = golden_stats
    cs, world, seed = scenes.cornell_box()
    img = R.raytrace(cs, world, seed)
    assert img.shape == (600, 600, 3) and img.dtype == np.float64
    lin = as_published(img, "sqrt")
    gold = np.load(os.path.join(GOLDEN, "cornell_box_redirect_block8.npy")).astype(np.float64)
    rmse = np.sqrt(((block8(lin) - gold) ** 2).reshape(-1, 3).mean(0))
    floor = np.array(floors["cornell_box_redirect"]["block8_rmse"])
    assert (rmse <= 1.5 * floor).all(), (rmse, floor)
    np.testing.assert_allclose(lin.reshape(-1, 3).mean(0), stats["images"]["cornell_box_redirect"]["linear_mean"],
                               rtol=0.01)


def test_readme_scene_matches_published_render(gpu, golden_stats):
    stats, floors = golden_stats
    cs, world, seed = scenes.readme_scene()
    lin = as_published(R.raytrace(cs, world, seed), "srgb")
    gold = np.load(os.path.join(GOLDEN, "example_image_block8.npy")).astype(np.float64)
    rmse = np.sqrt(((block8(lin) - gold) ** 2).reshape(-1, 3).mean(0))
    assert (rmse <= 1.5 * np.array(floors["example_image"]["block8_rmse"])).all(), rmse
    np.testing.assert_allclose(lin.reshape(-1, 3).mean(0), stats["images"]["example_image"]["linear_mean"], rtol=0.01)


def test_pawn_demo_matches_published_render(gpu, golden_stats):
    stats, _ = golden_stats
    cs, world, seed = scenes.pawn_test()
    lin = as_published(R.raytrace(cs, world, seed), "srgb")
    np.testing.assert_allclose(lin.reshape(-1, 3).mean(0), stats["images"]["pawn_demo"]["linear_mean"], rtol=0.01)
    gold = np.load(os.path.join(GOLDEN, "pawn_demo_block8.npy")).astype(np.float64)
    assert np.sqrt(((block8(lin) - gold) ** 2).mean()) < 0.02


def test_demo2_matches_published_render(gpu, golden_stats):
    """demo2 (test/Main.hs:259-321, the reference's test entry point demoTest) against its published
    demo2.png, 800 x 800.  The render is pinned where the image does not depend on the random world
    draw: the published ground boxes and ball cluster are not the ones the restated mkStdGen 1234
    stream draws (an earlier revision of the code, as for the other PNGs), but the light, the back
    wall seen through the camera-enclosing fog (constantMedium 0.0001 (sphere 0 5000): the
    ray-starts-inside case of Geometry.hs:313), the moving (motion-blurred) orange sphere and the
    image-textured earth (imageTexture of images/earthmap.jpg under transform . rotateY) are.
    Measured against the PNG (tools/demo2_fit.py, profiles/r4/demo2_fit.json): depth 50 and
    ~10^4 spp (the top band's pixel noise; depth 4, the test entry's, is 0.5-0.8 codes too dark
    there).  Bars, binary64 at depth 50 and 1000 spp:
      * linear mean within 3 standard deviations of the spread over world seeds
        (tests/golden/demo2_worlds.json, FP64 oracle);
      * 8x8-block RMSE against the PNG in the top band (rows 0-199: light, wall, fog, moving sphere)
        no larger than between two of our renders with different camera seeds (measured 0.74x), and
        in the earth's interior within 1.5x of it (measured 1.0-1.1x: the JPEG decoders differ)."""
    stats, _ = golden_stats
    with open(os.path.join(GOLDEN, "demo2_worlds.json")) as f:
        sd = np.array(json.load(f)["std_over_worlds"])
    pub = np.array(stats["images"]["demo2"]["linear_mean"])
    gold = np.load(os.path.join(GOLDEN, "demo2_block8.npy")).astype(np.float64)
    cs, world, seed = scenes.demo2(spp=1000, depth=50)
    a = as_published(R.raytrace(cs, world, seed), "sqrt")
    b = as_published(R.raytrace(cs, world, R.mkStdGen(12)), "sqrt")
    assert a.shape == (800, 800, 3)
    ba, bb = block8(a), block8(b)

    def rmse(x, y):
        return np.sqrt(((x - y) ** 2).reshape(-1, 3).mean(0))

    top_pub, top_seed = rmse(ba[:25], gold[:25]), rmse(ba[:25], bb[:25])
    earth = (slice(52, 64), slice(8, 20))
    earth_pub, earth_seed = rmse(ba[earth], gold[earth]), rmse(ba[earth], bb[earth])
    m = a.reshape(-1, 3).mean(0)
    record_measure("published_renders", dict(test="demo2", mean=m.tolist(), pub=pub.tolist(), world_sd=sd.tolist(),
                                             top_pub=top_pub.tolist(), top_seed=top_seed.tolist(),
                                             earth_pub=earth_pub.tolist(), earth_seed=earth_seed.tolist()))
    assert (np.abs(m - pub) <= 3 * sd).all(), (m, pub, sd)
    assert (top_pub <= top_seed).all(), (top_pub, top_seed)
    assert (earth_pub <= 1.5 * earth_seed).all(), (earth_pub, earth_seed)


def test_demo1_matches_published_render_statistically(gpu, golden_stats):
    """demo1 at the reference's 1200 x 675 x 500 against its published demo1.png.  The reference drew
    the world from newStdGen (test/Main.hs:184-185), so the spheres' placement cannot be reproduced:
    the quantised image's linear mean must lie within 3 standard deviations of the oracle's spread
    over world seeds (tests/golden/demo1_worlds.json, make_golden.py --demo1) of the published one,
    and the 8x8-block RMSE against demo1.png within 1.25x the RMSE between two of our own worlds (the
    large spheres, ground and sky agree; the small spheres are a different draw either way)."""
    stats, _ = golden_stats
    with open(os.path.join(GOLDEN, "demo1_worlds.json")) as f:
        spread = json.load(f)
    pub = np.array(stats["images"]["demo1"]["linear_mean"])
    gold = np.load(os.path.join(GOLDEN, "demo1_block8.npy")).astype(np.float64)
    lins = []
    for world_seed in (1, 2):
        cs, world, seed = scenes.demo1(seed=world_seed)
        lins.append(as_published(R.raytrace(cs, world, seed), "sqrt"))
    assert lins[0].shape == (675, 1200, 3)
    sd = np.array(spread["std_over_worlds"])
    means = [lin.reshape(-1, 3).mean(0) for lin in lins]
    rmse_pub = float(np.sqrt(((block8(lins[0]) - gold) ** 2).mean()))
    rmse_worlds = float(np.sqrt(((block8(lins[0]) - block8(lins[1])) ** 2).mean()))
    record_measure("published_renders", dict(test="demo1", means=[m.tolist() for m in means], pub=pub.tolist(),
                                             world_sd=sd.tolist(), rmse_pub=rmse_pub, rmse_worlds=rmse_worlds))
    for m in means:
        assert (np.abs(m - pub) <= 3 * sd).all(), (m, pub, sd)
    assert rmse_pub <= 1.25 * rmse_worlds, (rmse_pub, rmse_worlds)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_full_demo1_is_finite(gpu, precision):
    """demo1 at its full 1200x675x500: long total-internal-reflection chains inside the glass
    spheres stay finite (directions re-normalised after reflect / refract, rt_trace.h `unit`)."""
    cs, world, seed = scenes.demo1()
    img = R.raytrace(cs, world, seed, precision=precision)
    assert img.shape == (675, 1200, 3)
    assert np.isfinite(img).all()
    m = img.reshape(-1, 3).mean(0)
    assert (m > 0.3).all() and (m < 1.0).all()


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["cornell", "pawn_fog", "bunny_cornell", "demo1"])
def test_kernel_variants_bitwise_identical(knobs, gpu, monkeypatch, name, precision):
    """Flat / BVH-decoupled kernels: same per-path arithmetic, different schedule; fixed-point
    accumulation makes the images bit-identical.  (The lockstep BVH kernel, the reference schedule,
    is compiled into experiment builds only, RT_LOCKSTEP_KERNELS; the host emulator checks it,
    test_oracle_golden.py test_kernel_variants_render_bitwise_identical_images.)"""
    fn = {"cornell": scenes.cornell_box, "pawn_fog": scenes.pawn_fog, "bunny_cornell": scenes.bunny_cornell,
          "demo1": scenes.demo1}[name]
    cs, world, seed = fn(width=96, spp=8)
    imgs = []
    # the flat kernel tests cuboid faces as box groups, the BVH kernels run on a flat scene test
    # them one by one (same result up to rounding at the box edges): compare with box groups off
    monkeypatch.setenv("RT_AMD_NO_BOX", "1")
    for v in ("0", "2"):
        monkeypatch.setenv("RT_AMD_VARIANT", v)
        imgs.append(R.raytrace(cs, world, seed, precision=precision))
    for img in imgs[1:]:
        assert np.array_equal(img, imgs[0], equal_nan=True)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["bunny_cornell", "demo1"])
def test_large_primitive_prefix_is_exact(knobs, gpu, monkeypatch, name, precision):
    fn = {"bunny_cornell": scenes.bunny_cornell, "demo1": scenes.demo1}[name]
    cs, world, seed = fn(width=96, spp=8)
    monkeypatch.setenv("RT_AMD_NO_BOX", "1")  # exact claim: per-face tests in and out of the BVH
    a = R.raytrace(cs, world, seed, precision=precision)
    monkeypatch.setenv("RT_AMD_NO_PREFIX", "1")
    b = R.raytrace(cs, world, seed, precision=precision)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["cornell", "box_gallery"])
def test_box_groups_match_oracle(knobs, gpu, oracle_mod, monkeypatch, name, precision):
    fn = {"cornell": scenes.cornell_box, "box_gallery": scenes.box_gallery}[name]
    cs, world, seed = fn(width=96, spp=8)
    a = R.raytrace(cs, world, seed, precision=precision)
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    # FP32 on box_gallery's oblique glass cuboid at 8 spp: paths that split on a rounding-level
    # decision inside the glass carry the light's 15 to a different pixel, so the block bar is
    # the 1.5x of §8c's CPU-vs-reference test there; binary64 keeps 0.5x
    mult = 1.5 if (precision == "f32" and name == "box_gallery") else 0.5
    assert_parity(a, ref, precision, 0.99, _floor()["cornell"], name, 8, 15.0, mult)
    monkeypatch.setenv("RT_AMD_NO_BOX", "1")
    b = R.raytrace(cs, world, seed, precision=precision)
    assert pixel_agreement(a, b, 1e-9 if precision == "f64" else 1e-3) >= 0.995


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["cornell", "bunny_cornell"])
def test_item_chunk_does_not_change_the_image(knobs, gpu, monkeypatch, name, precision):
    """Items of 1, 3 (ragged: does not divide spp), 4 and 16 samples, and two item sizes: a
    different work split and commit order, the same fixed-point sums — bit-identical images."""
    fn = {"cornell": scenes.cornell_box, "bunny_cornell": scenes.bunny_cornell}[name]
    cs, world, seed = fn(width=64, spp=20)
    imgs = []
    for c in ("1", "3", "4", "16"):
        monkeypatch.setenv("RT_AMD_CHUNK", c)
        imgs.append(R.raytrace(cs, world, seed, precision=precision))
    # two item sizes (big items of 7 samples first, a tail of 3-sample items)
    monkeypatch.setenv("RT_AMD_CHUNK", "3")
    monkeypatch.setenv("RT_AMD_BIG_CHUNK", "7")
    monkeypatch.setenv("RT_AMD_TAIL_SAMPLES", "6")
    imgs.append(R.raytrace(cs, world, seed, precision=precision))
    for img in imgs[1:]:
        assert np.array_equal(img, imgs[0], equal_nan=True)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["cornell", "bunny_cornell"])
def test_tail_stealing_is_exact(knobs, gpu, monkeypatch, name, precision):
    """64 pixels x 600 samples: the queue drains at once and most samples are rendered by lanes
    that took them from another lane's item (rt_trace.h steal_sample, both lane loops).  One-sample
    items leave nothing to take; 16- and 64-sample items are split across the wave.  The stolen
    samples keep their pixel and sample index (the same Philox draws) and integer sums commute, so
    the images are bit-identical."""
    fn = {"cornell": scenes.cornell_box, "bunny_cornell": scenes.bunny_cornell}[name]
    cs, world, seed = fn(width=8, spp=600)
    imgs = []
    for c in ("1", "16", "64"):
        monkeypatch.setenv("RT_AMD_CHUNK", c)
        imgs.append(R.raytrace(cs, world, seed, precision=precision))
    for img in imgs[1:]:
        assert np.array_equal(img, imgs[0], equal_nan=True)
    assert np.isfinite(imgs[0]).all() and imgs[0].mean() > 0


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["cornell", "bunny_cornell", "pawn_fog"])
def test_commit_aggregation_is_exact(knobs, gpu, monkeypatch, name, precision):
    """Items summed per pixel in the waves' LDS slots before the commit atomics (rt_render_kernel.h
    WaveWork) against every item committed directly (RT_AMD_AGG=0): bit-identical images, with one
    item size (32 / 128 chunks per pixel: flat and BVH kernels aggregate) and with two sizes (a
    pool straddling the size boundary, big items of 8 samples: 8 per pixel)."""
    fn = {"cornell": scenes.cornell_box, "bunny_cornell": scenes.bunny_cornell, "pawn_fog": scenes.pawn_fog}[name]
    cs, world, seed = fn(width=96, spp=128)
    for env in ({}, {"RT_AMD_CHUNK": "1"}, {"RT_AMD_BIG_CHUNK": "8", "RT_AMD_TAIL_SAMPLES": "64"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        monkeypatch.delenv("RT_AMD_AGG", raising=False)
        a = R.raytrace(cs, world, seed, precision=precision)
        monkeypatch.setenv("RT_AMD_AGG", "0")
        b = R.raytrace(cs, world, seed, precision=precision)
        assert np.isfinite(a).all() and a.mean() > 0
        assert np.array_equal(a, b, equal_nan=True), (name, env)
        for k in env:
            monkeypatch.delenv(k)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["bunny_cornell", "demo1", "pawn_fog"])
def test_one_class_leaf_kernels_are_exact(knobs, gpu, monkeypatch, name, precision):
    """BVH kernels whose leaf test is specialised to the scene's one primitive class (RT_VAR_LEAF_TRI
    for the bunny and for pawn+fog — its media kernel, the fog sphere a single-leaf medium set
    tested generically — RT_VAR_LEAF_SPHERE for demo1) against the generic leaf test: the same
    arithmetic per primitive, so bit-identical images."""
    fn = {"bunny_cornell": scenes.bunny_cornell, "demo1": scenes.demo1, "pawn_fog": scenes.pawn_fog}[name]
    cs, world, seed = fn(width=96, spp=16)
    a = R.raytrace(cs, world, seed, precision=precision)
    monkeypatch.setenv("RT_AMD_LEAF_KIND", "0")
    b = R.raytrace(cs, world, seed, precision=precision)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["pawn_fog", "demo2"])
def test_media_events_in_shading_phase_are_exact(knobs, gpu, monkeypatch, name, precision):
    """The media events in the shading phase (rt_trace.h media_events_late) render the traversal
    loop's query-chain image bit for bit (RT_AMD_MEDIA_LATE=0)."""
    fn = {"pawn_fog": scenes.pawn_fog, "demo2": scenes.demo2}[name]
    cs, world, seed = fn(width=80, spp=8)
    a = R.raytrace(cs, world, seed, precision=precision)
    monkeypatch.setenv("RT_AMD_MEDIA_LATE", "0")
    b = R.raytrace(cs, world, seed, precision=precision)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_medium_boundary_alias_is_exact(knobs, gpu, monkeypatch, precision):
    cs, world, seed = scenes.pawn_fog(width=96, spp=8)
    a = R.raytrace(cs, world, seed, precision=precision)
    monkeypatch.setenv("RT_AMD_NO_ALIAS", "1")
    b = R.raytrace(cs, world, seed, precision=precision)
    assert np.array_equal(a, b, equal_nan=True)


def _image_scene():
    img = np.load(os.path.join(GOLDEN, "earthmap_128x64.npy")).astype(np.float32)
    tex = R.imageTexture(img)
    world = R.group([R.lambertian(tex) << R.sphere((0, 0, -2), 0.6),
                     R.lambertian(tex) << R.parallelogram((-2, -1, -3), (4, 0, 0), (0, 2.5, 0)),
                     R.lambertian(R.constantTexture(0.5)) << R.sphere((0, -100.6, -2), 100)])
    return R.defaultCameraSettings(cs_imageWidth=120, cs_samplesPerPixel=8, cs_background=R.sky), world, R.mkStdGen(3)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["noise_test", "image"])
def test_textured_scenes_match_oracle_per_pixel(gpu, oracle_mod, name, precision):
    """imageTexture (wrap, row flip) and the Perlin noise / marble textures (Texture.hs:31-78,
    Noise.hs) against the oracle on the same Philox numbers."""
    cs, world, seed = scenes.noise_test(width=160, spp=8) if name == "noise_test" else _image_scene()
    img = R.raytrace(cs, world, seed, precision=precision)
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    assert_parity(img, ref, precision, 0.99, _floor()["cornell"], name, 8, 1.0)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("kind", ["sphere", "triangle", "parallelogram", "mirror"])
def test_known_answer_hits(gpu, kind, precision):
    """The analytic known-answer scenes of test_oracle_golden on the GPU:
    pixels wholly inside / outside the primitive are exact."""
    from test_oracle_golden import _kat_scene
    cs, world, mask = _kat_scene(kind)
    out = R.raytrace(cs, world, R.mkStdGen(5), precision=precision)
    m = mask >= 0
    np.testing.assert_allclose(out[m], np.repeat(mask[m][:, None], 3, axis=1), atol=1e-12 if precision == "f64" else 1e-6)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_deterministic_shard_and_device_list_invariant(gpu, precision):
    """Repeated renders, row shards (one process per GPU) and device lists (one process, many
    GPUs: ABI v3 rt_exec.devices, here device 0 listed 2 and 3 times) all give the same image."""
    from raytrace_amd.ray import assemble_shards, render_shard
    cs, world, seed = scenes.cornell_box(spp=4, width=50)
    a = R.raytrace(cs, world, seed, precision=precision)
    b = R.raytrace(cs, world, seed, precision=precision)
    np.testing.assert_array_equal(a, b)
    for n, rb in [(2, 4), (3, 1), (8, 4)]:
        tiles = np.stack([render_shard(cs, world, seed, n, r, rb, precision=precision) for r in range(n)])
        np.testing.assert_array_equal(assemble_shards(tiles, 50, rb), a)
    for devs, rb in [([0, 0], 4), ([0, 0, 0], 1), ([0] * 8, 2)]:
        st = {}
        c = R.raytrace(cs, world, seed, precision=precision, devices=devs, row_block=rb, stats=st)
        np.testing.assert_array_equal(c, a)
        assert st["samples"] == 50 * 50 * 4
    d = R.raytrace(cs, world, R.mkStdGen(235), precision=precision)
    assert not np.array_equal(a, d)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_multi_device_scene_and_encoded_output(gpu, precision):
    """rt_multi_scene: one host build, resident across renders (no rebuild or re-upload on the
    second render), gather into the first device's framebuffer, and the 8-bit epilogue fused
    after the gather (rt_exec RT_EXEC_ENCODE8_*): bytes equal encode8 of the linear render."""
    cs, world, seed = scenes.bunny_cornell(width=64, spp=4)
    a = R.raytrace(cs, world, seed, precision=precision)
    for enc in ("srgb", "sqrt"):
        np.testing.assert_array_equal(R.raytrace(cs, world, seed, precision=precision, encode=enc), R.encode8(a, enc))
        np.testing.assert_array_equal(R.raytrace(cs, world, seed, precision=precision, encode=enc, devices=[0, 0, 0],
                                                 row_block=2), R.encode8(a, enc))
    m = R.MultiDeviceScene(world, [0] * 8)
    st1, st2 = {}, {}
    np.testing.assert_array_equal(m.render(cs, seed, precision=precision, row_block=1, stats=st1), a)
    np.testing.assert_array_equal(m.render(cs, seed, precision=precision, row_block=3, stats=st2), a)
    np.testing.assert_array_equal(m.render(cs, seed, precision=precision, encode="srgb"), R.encode8(a, "srgb"))
    # the second render re-uses the resident records: only the one-time build is reported again
    assert st2["upload_ms"] <= st1["upload_ms"] + 1.0, (st1, st2)
    assert st1["samples"] == st2["samples"] == 64 * 64 * 4
    m.close()
    # one entry, rendering an rt_exec shard: the multi-device call with a single device
    single = R.MultiDeviceScene(world, [0])
    np.testing.assert_array_equal(single.render(cs, seed, precision=precision), a)
    # a caller-held output buffer (poisoned between renders) is overwritten with the same frame
    buf = np.full(a.shape, np.nan, a.dtype)
    assert single.render(cs, seed, precision=precision, out=buf) is buf
    np.testing.assert_array_equal(buf, a)
    buf[:] = np.nan
    np.testing.assert_array_equal(single.render(cs, seed, precision=precision, out=buf), a)
    codes = np.full(a.shape, 7, np.uint8)
    np.testing.assert_array_equal(R.raytrace(cs, world, seed, precision=precision, encode="srgb", out=codes),
                                  R.encode8(a, "srgb"))
    single.close()


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_multi_device_scene_allocates_once(gpu, precision):
    """A resident rt_multi_scene keeps its tiles, workspaces, gather and 8-bit buffers, streams and
    events across renders: the first render allocates (rt_stats.device_allocs > 0), the next ones
    of the same or a smaller frame allocate nothing, a larger frame grows the buffers once; images
    bit-identical to the one-device render throughout."""
    cs, world, seed = scenes.bunny_cornell(width=48, spp=2)
    a = R.raytrace(cs, world, seed, precision=precision)
    m = R.MultiDeviceScene(world, [0, 0, 0])
    st = [{} for _ in range(4)]
    np.testing.assert_array_equal(m.render(cs, seed, precision=precision, stats=st[0]), a)
    np.testing.assert_array_equal(m.render(cs, seed, precision=precision, stats=st[1]), a)
    np.testing.assert_array_equal(m.render(cs, seed, precision=precision, encode="sqrt", stats=st[2]), R.encode8(a, "sqrt"))
    np.testing.assert_array_equal(m.render(cs, seed, precision=precision, encode="sqrt"), R.encode8(a, "sqrt"))
    big = cs.replace(cs_imageWidth=64)
    b = m.render(big, seed, precision=precision, stats=st[3])
    np.testing.assert_array_equal(b, R.raytrace(big, world, seed, precision=precision))
    again = {}
    m.render(big, seed, precision=precision, stats=again)
    m.render(cs, seed, precision=precision, stats=again)
    assert st[0]["device_allocs"] >= 4, st  # three tiles and workspaces, the gather
    assert st[1]["device_allocs"] == 0, st
    assert st[2]["device_allocs"] == 1, st  # the 8-bit buffer, once
    assert st[3]["device_allocs"] > 0 and again["device_allocs"] == 0, (st, again)
    m.close()


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_multi_device_copy_path(knobs, gpu, monkeypatch, precision):
    """The path of a shard whose device has no peer access to the first one (rt_api.hip
    multi_render: its own tile, then one strided hipMemcpy2DAsync into the frame), forced on one GPU
    with RT_AMD_COPY_SHARDS (bit k: shard k): every shard copied, and copied and direct shards
    writing the same frame.  Bit-identical to the one-device render, linear and encoded; the first
    render allocates the workspaces, the copied shards' tiles and the frame, the next ones nothing."""
    cs, world, seed = scenes.bunny_cornell(width=48, spp=2)
    a = R.raytrace(cs, world, seed, precision=precision)
    for devs, mask in (([0, 0], "-1"), ([0, 0, 0], "-1"), ([0, 0, 0], "0x5"), ([0] * 4, "0x2")):
        monkeypatch.setenv("RT_AMD_COPY_SHARDS", mask)
        m = R.MultiDeviceScene(world, devs)
        try:
            st = [{}, {}]
            for k in range(2):
                np.testing.assert_array_equal(m.render(cs, seed, precision=precision, row_block=2, stats=st[k]), a)
            np.testing.assert_array_equal(m.render(cs, seed, precision=precision, row_block=1), a)
            np.testing.assert_array_equal(m.render(cs, seed, precision=precision, encode="sqrt"), R.encode8(a, "sqrt"))
        finally:
            m.close()
        copied = len(devs) if mask == "-1" else bin(int(mask, 0)).count("1")
        assert st[0]["device_allocs"] == len(devs) + copied + 1, (devs, mask, st)
        assert st[1]["device_allocs"] == 0, (devs, mask, st)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_multi_device_distinct_gpus(gpu, precision):
    """A device list over DISTINCT GPUs: each peer device's resolve writes its rows straight into the
    first device's frame over xGMI (rt_api.hip multi_render).  [0, 1] and [0, 1, 0, 1], linear in
    both precisions and 8-bit, rendered twice (the resident buffers re-used across devices), each
    bit-identical to the one-device render.  Needs two GPUs: skipped on the one-GPU box, runs on the
    driver's multi-GPU node."""
    if gpu.cuda.device_count() < 2:
        pytest.skip("needs two visible GPUs")
    cs, world, seed = scenes.bunny_cornell(width=48, spp=2)
    a = R.raytrace(cs, world, seed, precision=precision)
    for devs in ([0, 1], [0, 1, 0, 1]):
        m = R.MultiDeviceScene(world, devs)
        try:
            for rb in (1, 2):
                st = {}
                np.testing.assert_array_equal(m.render(cs, seed, precision=precision, row_block=rb, stats=st), a)
            np.testing.assert_array_equal(m.render(cs, seed, precision=precision, encode="sqrt"), R.encode8(a, "sqrt"))
            np.testing.assert_array_equal(m.render(cs, seed, precision=precision, encode="sqrt"), R.encode8(a, "sqrt"))
        finally:
            m.close()
        assert st["device_allocs"] == 0, (devs, st)


@pytest.mark.parametrize("name,precision", [("cornell", "f64"), ("cornell", "f32"), ("bunny_cornell", "f64")])
def test_tile_beyond_2p24_pixels(gpu, oracle_mod, name, precision):
    """A one-GPU tile of more than 2^24 pixels (4100 x 4100): the item's tile-pixel word then uses
    bits 24-30, which the commit must not read as an aggregation slot code (rt_render_kernel.h
    WaveWork::aggregating).  The whole-frame render equals the same frame rendered as two shards of
    under 2^24 pixels each, bit for bit, and the oracle on sampled pixels."""
    from raytrace_amd.ray import assemble_shards, render_shard
    fn = {"cornell": scenes.cornell_box, "bunny_cornell": scenes.bunny_cornell}[name]
    cs, world, seed = fn(width=4100, spp=1, depth=3)
    assert 4100 * 4100 > 1 << 24
    a = R.raytrace(cs, world, seed, precision=precision)
    tiles = np.stack([render_shard(cs, world, seed, 2, r, 4, precision=precision) for r in range(2)])
    assert tiles.shape[1] * 4100 < 1 << 24
    np.testing.assert_array_equal(assemble_shards(tiles, 4100, 4), a)
    rows = np.array([0, 1, 2047, 4091, 4099])  # the last rows: tile pixels above 2^24
    pix = (rows[:, None] * 4100 + np.arange(0, 4100, 7)[None, :]).reshape(-1).astype(np.int32)
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX, pixels=pix)
    got = a.reshape(-1, 3)[pix].astype(np.float64)
    tol = 1e-9 if precision == "f64" else 1e-3
    rel = (np.abs(got - ref) / np.maximum(np.abs(ref), 1e-3 if precision == "f64" else 1.0)).max(-1)
    assert (rel <= tol).mean() >= 0.99, float((rel <= tol).mean())


def test_device_list_bvh_scene(gpu):
    cs, world, seed = scenes.bunny_cornell(width=64, spp=4)
    a = R.raytrace(cs, world, seed)
    np.testing.assert_array_equal(R.raytrace(cs, world, seed, devices=[0, 0, 0], row_block=1), a)


def test_edge_cases(gpu):
    cs, world, seed = scenes.cornell_box(spp=2, width=16)
    assert (R.raytrace(cs.replace(cs_maxRecursionDepth=0), world, seed) == 0).all()  # Ray.hs:176: black
    d1 = R.raytrace(cs.replace(cs_maxRecursionDepth=1), world, seed)
    assert set(np.unique(np.round(d1, 4))) <= {0.0, 7.5, 15.0}
    one = R.raytrace(cs.replace(cs_imageWidth=1), world, seed)
    assert one.shape == (1, 1, 3) and np.isfinite(one).all()
    tall = R.raytrace(cs.replace(cs_imageWidth=3, cs_aspectRatio=0.01), world, seed)
    assert tall.shape == (300, 3, 3)
    # a world that is a single sphere (root of the BVH is a leaf) under a sky background
    sky_world = R.lambertian(R.constantTexture(0.5)) << R.sphere((0, 0, -1), 0.5)
    img = R.raytrace(R.defaultCameraSettings(cs_imageWidth=32, cs_background=R.sky), sky_world, R.mkStdGen(1))
    assert np.isfinite(img).all() and img.max() <= 1.0 + 1e-12
    # background only: every sample sees const colour exactly, in both precisions
    empty_like = R.lightSource(R.constantTexture(0)) << R.sphere((0, 0, 100), 0.1)
    for precision in ("f64", "f32"):
        bg = R.raytrace(R.defaultCameraSettings(cs_imageWidth=8, cs_background=R.constBackground((0.25, 0.5, 1.0))),
                        empty_like, R.mkStdGen(3), precision=precision)
        np.testing.assert_array_equal(bg, np.broadcast_to(np.array([0.25, 0.5, 1.0]), bg.shape))


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_all_materials_against_oracle(gpu, oracle_mod, precision):
    """One sphere per reference material (Material.hs:41-129) over a checker floor, media included."""
    mats = [R.lightSource(R.constantTexture(4)), R.pitchBlack, R.lambertian(R.constantTexture((0.7, 0.3, 0.2))),
            R.lommelSeeliger(R.constantTexture(0.9)), R.mirror(R.constantTexture(0.8)),
            R.metal(0.3, R.constantTexture((0.8, 0.8, 0.9))), R.dielectric(1.5),
            R.transparent(R.constantTexture((0.9, 0.5, 0.5))), R.isotropic(R.constantTexture(0.8)),
            R.anisotropic(0.6, R.constantTexture(0.8))]
    objs = [R.lambertian(R.checkerTexture(10, 10, 0.2, 0.9)) << R.parallelogram((-10, -1, -10), (20, 0, 0), (0, 0, 20))]
    for k, m in enumerate(mats):
        x = -4.5 + k
        if m.kind in (8, 9):
            objs.append(m << R.constantMedium(1.5, R.sphere((x, -0.5, -4), 0.45)))
        else:
            objs.append(m << R.sphere((x, -0.5, -4), 0.45))
    world = R.group(objs)
    cs = R.defaultCameraSettings(cs_imageWidth=160, cs_aspectRatio=2.0, cs_samplesPerPixel=8, cs_background=R.sky,
                                 cs_center=(0, 1, 2), cs_lookAt=(0, -0.5, -4),
                                 cs_redirectTargets=[(0.2, (-5, 3, -5), (10, 0, 0), (0, 0, 2))])
    img = R.raytrace(cs, world, R.mkStdGen(9), precision=precision)
    ref = oracle_mod.render(cs, world, R.mkStdGen(9), mode=oracle_mod.RNG_PHILOX)
    assert_parity(img, ref, precision, 0.98, _floor()["cornell"], "materials", 8, 4.0)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("mats", [False, True])
def test_deep_bvh_against_oracle(gpu, oracle_mod, mats, precision):
    """A BVH 26 levels deep (spheres 8^k apart along the view axis): one 1024-lane workgroup of the
    4-wave binary64 / 8-wave FP32 (with the metal sphere) classes cannot hold its stacks beside the
    item sums, so the scene runs their 512-lane twins (RT_VAR_NARROW, rt_render_kernel.h)."""
    objs = [R.lambertian(R.constantTexture(0.5)) << R.sphere((0, -1000.5, -1), 1000)]
    for k in range(40):
        objs.append(R.lambertian(R.constantTexture((0.8, 0.3, 0.2))) << R.sphere((0.3 * (k % 3 - 1), 0.0, -2.0 - 8.0 ** k), 0.2))
    if mats:
        objs.append(R.metal(0.2, R.constantTexture(0.8)) << R.sphere((0.6, 0.1, -2.5), 0.3))
    world = R.group(objs)
    cs = R.defaultCameraSettings(cs_imageWidth=96, cs_aspectRatio=1.5, cs_samplesPerPixel=8, cs_background=R.sky,
                                 cs_center=(0, 0.3, 1), cs_lookAt=(0, 0, -3))
    st = {}
    img = R.raytrace(cs, world, R.mkStdGen(5), precision=precision, stats=st)
    assert st["max_stack"] >= 24, st  # deeper than a 1024-lane binary64 workgroup's stacks hold
    # the 512-lane twin ran (the FP32 sphere-leaf class without the full material set is a 768-lane
    # class: no twin)
    assert st["kernel_block"] == (512 if precision == "f64" or mats else 768), st
    ref = oracle_mod.render(cs, world, R.mkStdGen(5), mode=oracle_mod.RNG_PHILOX)
    assert_parity(img, ref, precision, 0.98, _floor()["cornell"], "deep_bvh", 8, 1.0)


def mixed_leaf_scene(width=160, spp=2):
    """A BVH scene whose leaves mix triangles and spheres (the generic-leaf kernel classes) with the
    full material set (metal, dielectric, mirror beside lambertian): the bunny mesh among 48
    spheres, sky background.  Test scene, not a reference scene."""
    mesh = scenes.load_mesh("bunny.obj")
    center = tuple(R.midpoint(i) for i in R.boundingBox(R.triangleMesh(mesh)))
    bunny = R.triangleMesh(R.transformVertices(R.scale(8) @ R.translate(tuple(-c for c in center)), mesh))
    objs = [R.lambertian(R.constantTexture(0.5)) << R.sphere((0, -1000.6, 0), 1000),
            R.lambertian(R.constantTexture((0.8, 0.6, 0.3))) << bunny]
    for k in range(48):
        x, z = -3.0 + 0.9 * (k % 8), -1.0 - 0.9 * (k // 8)
        m = [R.metal(0.1 * (k % 4), R.constantTexture(0.8)), R.dielectric(1.5), R.mirror(R.constantTexture(0.9)),
             R.lambertian(R.constantTexture((0.2, 0.4, 0.8)))][k % 4]
        objs.append(m << R.sphere((x, -0.35, z), 0.25))
    cs = R.defaultCameraSettings(cs_imageWidth=width, cs_aspectRatio=1.5, cs_samplesPerPixel=spp, cs_background=R.sky,
                                 cs_center=(0, 1.2, 3), cs_lookAt=(0, 0, -2))
    return cs, R.group(objs), R.mkStdGen(13)


DETERMINISM_SCENES = {
    # the instanced classes (FP32 spilled in a round-5 experiment build), the media kernels, demo1
    "bunny_instances": lambda: scenes.bunny_instances(spp=4, n=8),
    "pawn_fog": lambda: scenes.pawn_fog(width=200, spp=2),
    "demo1": lambda: scenes.demo1(width=300, spp=2),
    # classes that spilled VGPRs in the round-5 product build (profiles/r5/final/resources.txt): the
    # full-material generic-leaf class, the instanced classes with textures and the media query
    # chain (demo2 with RT_AMD_MEDIA_LATE=0), instances with textured leaves and the full material set
    "mixed_leaf": mixed_leaf_scene,
    "demo2_chain": lambda: scenes.demo2(width=160, spp=2, depth=4),
    "instance_gallery": lambda: scenes.instance_gallery(width=160, spp=2),
    "box_gallery": lambda: scenes.box_gallery(width=120, spp=2),
    "noise_test": lambda: scenes.noise_test(width=160, spp=2),
}


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", list(DETERMINISM_SCENES))
def test_renders_are_deterministic(knobs, gpu, name, precision):
    """The same frame twice is bit-identical (fixed-point sums make the image independent of the
    schedule).  A build whose FP32 instanced kernel spilled VGPRs rendered nondeterministically
    (profiles/r5/bigwg/README.md); since round 6 no dispatchable kernel spills (tests/test_spill_gate.py)
    and this check renders every kernel class that spilled before, and the bench configs' classes."""
    if name == "demo2_chain":
        knobs.setenv("RT_AMD_MEDIA_LATE", "0")
    cs, world, seed = DETERMINISM_SCENES[name]()
    a = R.raytrace(cs, world, seed, precision=precision)
    b = R.raytrace(cs, world, seed, precision=precision)
    assert np.array_equal(a, b, equal_nan=True), float(np.nanmax(np.abs(a - b)))


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_moving_and_transform_against_oracle(gpu, oracle_mod, precision):
    """`moving` (motion blur, Geometry.hs:449-456) and rotated textured spheres (sphereUV frame)."""
    tex = R.checkerTexture(8, 4, (0.9, 0.1, 0.1), (0.1, 0.1, 0.9))
    world = R.group([
        R.lambertian(R.constantTexture(0.5)) << R.sphere((0, -1000.5, -1), 1000),
        R.lambertian(tex) << R.moving((0, 0, 0), (0.6, 0, 0), R.sphere((-0.6, 0, -1.5), 0.5)),
        R.lambertian(tex) << R.transform(R.translate((0.8, 0, -1.2)) @ R.rotateX(R.degrees(60)),
                                         R.sphere((0, 0, 0), 0.4)),
        R.metal(0.1, R.constantTexture(0.8)) << R.moving((0, 0.2, 0), (0, -0.2, 0),
                                                         R.transform(R.rotateY(R.degrees(30)),
                                                                     R.cuboid(R.fromCorners((-2, -0.5, -3.5), (-1.2, 0.5, -2.7))))),
    ])
    cs = R.defaultCameraSettings(cs_imageWidth=128, cs_aspectRatio=1.5, cs_samplesPerPixel=8, cs_background=R.sky)
    img = R.raytrace(cs, world, R.mkStdGen(4), precision=precision)
    ref = oracle_mod.render(cs, world, R.mkStdGen(4), mode=oracle_mod.RNG_PHILOX)
    assert_parity(img, ref, precision, 0.98, _floor()["cornell"], "moving", 8, 1.0)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("n", [3, 8])
def test_two_level_instancing_against_oracle(gpu, oracle_mod, n, precision):
    """n x n rigid placements of ONE bunny object traced as rt_instances (world BVH over instance
    boxes -> object-space BLAS, ray moved by the inverse 3x4) against the oracle's walk of the
    reference's `transform` (Geometry.hs:382-391), and against the transforms baked into world
    triangles (instance_min=0)."""
    from raytrace_amd import scene as S
    cs, world, seed = scenes.bunny_instances(width=96, spp=8, n=n)
    inst = S.flatten(world)
    assert len(inst.instances) == n * n
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    img = R.raytrace(cs, inst, seed, precision=precision)
    assert_parity(img, ref, precision, 0.99, _floor()["cornell"], f"instances{n}", 8, 15.0)
    baked = R.raytrace(cs, S.flatten(world, instance_min=0), seed, precision=precision)
    assert_parity(baked, ref, precision, 0.99, _floor()["cornell"], f"baked{n}", 8, 15.0)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_instancing_edge_cases_against_oracle(gpu, oracle_mod, precision):
    """scenes.instance_gallery: placements by rotation, reflection (det -1), under a dielectric
    `<$`, and translation of one object with a textured sphere, a metal parallelogram and a mesh."""
    from raytrace_amd import scene as S
    cs, world, seed = scenes.instance_gallery(width=128, spp=8)
    flat = S.flatten(world)
    assert len(flat.instances) == 4
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    img = R.raytrace(cs, flat, seed, precision=precision)
    assert_parity(img, ref, precision, 0.99, _floor()["cornell"], "instance_gallery", 8, 1.0)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_device_scene_async_and_encode8_bit_exact(gpu, precision):
    torch = gpu
    from raytrace_amd import _lib
    cs, world, seed = scenes.cornell_box(spp=4, width=64)
    ds = R.DeviceScene(world)
    dt = torch.float64 if precision == "f64" else torch.float32
    out = torch.empty((64, 64, 3), dtype=dt, device="cuda")
    s = torch.cuda.current_stream()
    ds.render_async(cs, seed, out.data_ptr(), s.cuda_stream, precision=precision)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), R.raytrace(cs, world, seed, precision=precision))
    # RT_EXEC_SOLO (the synchronous call's work plan) renders the same bytes
    out2 = torch.full_like(out, float("nan"))
    ds.render_async(cs, seed, out2.data_ptr(), s.cuda_stream, precision=precision, solo=True)
    torch.cuda.synchronize()
    assert torch.equal(out2, out)
    big, bseed = cs.replace(cs_samplesPerPixel=200), seed  # (a frame with big items in both plans)
    for solo in (False, True):
        ds.render_async(big, bseed, (out if solo else out2).data_ptr(), s.cuda_stream, precision=precision, solo=solo)
    torch.cuda.synchronize()
    assert torch.equal(out2, out)
    # the render plus every code boundary (the host thresholds and their neighbours), NaN, +-inf,
    # negative and > 1 values: the device codes equal the host encoder's bit for bit
    x = np.linspace(0.0, 1.0, 4097)
    special = np.array([np.nan, np.inf, -np.inf, -1.0, -0.0, 0.0, 2.0, 1.0, 0.0031308, 0.04045, 1e-300])
    edges = []
    for enc in ("srgb", "sqrt"):
        for k in range(1, 256):  # bisect each code boundary on the host encoder
            lo, hi = 0.0, 1.0
            for _ in range(80):
                mid = 0.5 * (lo + hi)
                if R.encode8(np.array([mid]), enc)[0] >= k:
                    hi = mid
                else:
                    lo = mid
            edges += [lo, hi, np.nextafter(hi, 2.0), np.nextafter(lo, -1.0)]
    vals = np.concatenate([out.cpu().numpy().astype(np.float64).ravel(), x, special, np.array(edges)])
    if precision == "f32":
        vals = vals.astype(np.float32)
    dev = torch.from_numpy(np.ascontiguousarray(vals)).cuda()
    codes = torch.empty(vals.shape, dtype=torch.uint8, device="cuda")
    for enc, name in [(0, "srgb"), (1, "sqrt")]:
        _lib.check(_lib.load().rt_encode8_async(ctypes.c_void_p(dev.data_ptr()), 1 if precision == "f64" else 0,
                                                ctypes.c_void_p(codes.data_ptr()), vals.size, enc,
                                                ctypes.c_void_p(s.cuda_stream)))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(codes.cpu().numpy(), R.encode8(vals, name))
    ds.close()


def test_invalid_inputs_raise(gpu):
    cs, world, seed = scenes.cornell_box(spp=1, width=8)
    with pytest.raises(R.RtUnsupported):
        R.raytrace(cs, R.lambertian(R.solidTexture(lambda p: p)) << R.sphere((0, 0, 0), 1), seed)
    with pytest.raises(R.RtInvalid):
        R.raytrace(cs.replace(cs_samplesPerPixel=0), world, seed)
    with pytest.raises(R.RtInvalid):
        R.raytrace(cs, world, seed, devices=[0, 99])
