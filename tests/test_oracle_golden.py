"""Pins the FP64 oracle (oracle/rt_oracle.c) — the parity checker of the HIP path — against the
reference's own committed renders (the only result pins the reference has)
and against published known-answer vectors.

The reference's renders are noisy Monte-Carlo images and its RNG stream could not be reproduced
bit-for-bit offline (the splitmix/random restatement does not regenerate the PNG pixels), so
the render comparison is statistical: per-channel 8x8-block RMSE of the decoded linear images
within 1.5x the seed-to-seed noise floor measured for the same config (tests/golden/
noise_floor.json), and global means within 1 %.  The decoded images pass through the reference
writers' exact 8-bit quantisation (clipping at 1 included) before comparison.
"""
import os

import numpy as np
import pytest

import raytrace_amd as R
from conftest import GOLDEN, as_published, block8, pixel_agreement
from raytrace_amd import scenes
from raytrace_amd.camera import image_height


def _golden(name):
    import os
    from conftest import GOLDEN
    return np.load(os.path.join(GOLDEN, f"{name}_block8.npy")).astype(np.float64)


def test_philox_known_answer_vectors(oracle_mod):
    # Random123 kat_vectors, philox4x32 with 10 rounds
    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, want in kat:
        assert tuple(int(x) for x in oracle_mod.philox(ctr, key)) == want


def test_readme_scene_matches_example_image(oracle_mod, golden_stats):
    stats, floors = golden_stats
    cs, world, seed = scenes.readme_scene()
    img = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_SPLITMIX)
    assert img.shape == (338, 600, 3)
    lin = as_published(img, "srgb")
    mean = lin.reshape(-1, 3).mean(0)
    np.testing.assert_allclose(mean, stats["images"]["example_image"]["linear_mean"], rtol=0.01)
    rmse = np.sqrt(((block8(lin) - _golden("example_image")) ** 2).reshape(-1, 3).mean(0))
    floor = np.array(floors["example_image"]["block8_rmse"])
    assert (rmse <= 1.5 * floor).all(), (rmse, floor)


def test_cornell_band_matches_cornell_box_redirect(oracle_mod, golden_stats):
    """cornellBox 200 50 (test/Main.hs:188-218) on rows 152..447 at full spp."""
    stats, floors = golden_stats
    cs, world, seed = scenes.cornell_box()
    w = 600
    r0, r1 = 152, 448
    pix = (np.arange(r0, r1)[:, None] * w + np.arange(w)[None, :]).reshape(-1).astype(np.int32)
    out = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_SPLITMIX, pixels=pix)
    lin = as_published(out.reshape(r1 - r0, w, 3), "sqrt")
    gold = _golden("cornell_box_redirect")[r0 // 8: r1 // 8]
    rmse = np.sqrt(((block8(lin) - gold) ** 2).reshape(-1, 3).mean(0))
    floor = np.array(floors["cornell_box_redirect"]["block8_rmse"])
    assert (rmse <= 1.5 * floor).all(), (rmse, floor)
    np.testing.assert_allclose(block8(lin).reshape(-1, 3).mean(0), gold.reshape(-1, 3).mean(0), rtol=0.01)


def test_redirect_is_unbiased_against_noisy_render(oracle_mod, golden_stats):
    """cs_redirectTargets = [] reproduces cornell_box_noisy.png's statistics (README.md:71)."""
    stats, _ = golden_stats
    cs, world, seed = scenes.cornell_box(redirect=False)
    w, r0, r1 = 600, 200, 264
    pix = (np.arange(r0, r1)[:, None] * w + np.arange(w)[None, :]).reshape(-1).astype(np.int32)
    out = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_SPLITMIX, pixels=pix)
    lin = as_published(out.reshape(r1 - r0, w, 3), "sqrt")
    gold = _golden("cornell_box_noisy")[r0 // 8: r1 // 8]
    np.testing.assert_allclose(block8(lin).reshape(-1, 3).mean(0), gold.reshape(-1, 3).mean(0), rtol=0.03)


def test_pawn_demo_statistics(oracle_mod, golden_stats):
    """pawnTest (test/Main.hs:323-344): glass pawn with a red isotropic medium inside, at 1/10 spp;
    compared on 40x40-pixel blocks where the 1/10-spp noise is averaged out."""
    stats, _ = golden_stats
    cs, world, seed = scenes.pawn_test(spp=40)
    img = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_SPLITMIX)
    lin = as_published(img, "srgb")
    np.testing.assert_allclose(lin.reshape(-1, 3).mean(0), stats["images"]["pawn_demo"]["linear_mean"], rtol=0.01)
    gold = _golden("pawn_demo")  # 62 x 62 blocks of 8
    ours = block8(lin)
    g5 = gold[:60, :60].reshape(12, 5, 12, 5, 3).mean((1, 3))
    o5 = ours[:60, :60].reshape(12, 5, 12, 5, 3).mean((1, 3))
    assert np.abs(g5 - o5).max() < 0.02


def test_kernel_logic_matches_oracle_per_pixel(oracle_mod, emu_mod):
    """The kernel's own source (rt_trace.h) built for the host consumes the same Philox numbers as
    the oracle's Philox mode: almost every pixel agrees to 1e-3 (FP32 vs FP64 paths split only
    where a decision sits within rounding of its threshold)."""
    cases = [(scenes.cornell_box, dict(spp=16, width=96), 0.995),
             (scenes.readme_scene, dict(spp=16, width=120), 0.995),
             (scenes.demo1, dict(width=120, spp=8), 0.97),
             (scenes.bunny_cornell, dict(width=64, spp=8), 0.995),
             (scenes.pawn_fog, dict(width=64, spp=8), 0.99)]
    for fn, kw, need in cases:
        cs, world, seed = fn(**kw)
        got = emu_mod.render(cs, world, seed)
        ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
        assert got.shape == ref.shape
        assert np.isfinite(got).all()
        assert pixel_agreement(got, ref) >= need, fn.__name__
        np.testing.assert_allclose(got.reshape(-1, 3).mean(0), ref.reshape(-1, 3).mean(0), rtol=5e-3)


def test_glass_sphere_internal_reflection_chain_stays_finite(oracle_mod, emu_mod):
    """demo1 row 110 at the full 500 spp: sample 180 of pixel 513 bounces ~15 times by total
    internal reflection inside the big glass sphere.  The reference's sphere test assumes unit
    directions (Geometry.hs:64-68); FP32 rounding in reflect / refract used to grow |d| every
    bounce until the path diverged to a non-finite radiance.  The kernel re-normalises the
    directions that are unit in exact arithmetic, so the row stays finite and matches the FP64
    oracle on the same Philox numbers."""
    cs, world, seed = scenes.demo1()
    h, w = 675, cs.cs_imageWidth
    got = emu_mod.render(cs, world, seed, n_shards=h, shard=110, row_block=1)
    assert got.shape == (1, w, 3)
    assert np.isfinite(got).all()
    pix = (110 * w + np.arange(w)).astype(np.int32)
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX, pixels=pix)
    assert pixel_agreement(got.reshape(1, w, 3), ref.reshape(1, w, 3)) >= 0.97
    np.testing.assert_allclose(got[0, 513], ref.reshape(w, 3)[513], rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("name", ["cornell", "pawn_fog", "bunny_cornell"])
def test_kernel_variants_render_bitwise_identical_images(knobs, emu_mod, monkeypatch, name):
    """The three render-kernel variants (flat lockstep, BVH lockstep, BVH with traversal
    decoupled from shading) run the same per-path arithmetic in a different schedule; with
    fixed-point accumulation the images are bit-identical (host build of rt_trace.h)."""
    fn = {"cornell": scenes.cornell_box, "pawn_fog": scenes.pawn_fog, "bunny_cornell": scenes.bunny_cornell}[name]
    cs, world, seed = fn(width=48, spp=4)
    imgs = []
    # the flat kernel tests cuboid faces as box groups, the BVH kernels run on a flat scene test
    # them one by one (same result up to rounding at the box edges): compare with box groups off
    monkeypatch.setenv("RT_AMD_NO_BOX", "1")
    for v in ("0", "1", "2"):
        monkeypatch.setenv("RT_AMD_VARIANT", v)
        imgs.append(emu_mod.render(cs, world, seed))
    for img in imgs[1:]:
        assert np.array_equal(img, imgs[0], equal_nan=True)


@pytest.mark.parametrize("name", ["cornell", "readme"])
def test_two_size_items_render_the_same_image(knobs, emu_mod, monkeypatch, name):
    """Work items of two sizes (flat kernel; rt_build.cpp rt_host_plan_work: big items for the
    first samples of every pixel, small ones for the tail; rt_trace.h open_item) cover every
    (pixel, sample) exactly once: with fixed-point sums the image is bit-identical to one item
    size."""
    fn = {"cornell": scenes.cornell_box, "readme": scenes.readme_scene}[name]
    cs, world, seed = fn(width=40, spp=37)
    a = emu_mod.render(cs, world, seed)
    monkeypatch.setenv("RT_AMD_TAIL_ITEMS", "1")
    monkeypatch.setenv("RT_AMD_BIG_CHUNK", "5")
    b = emu_mod.render(cs, world, seed)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("variant", ["1", "2"])
def test_medium_boundary_alias_is_exact(knobs, emu_mod, monkeypatch, variant):
    """pawnTest's medium boundary is the dielectric surface itself; reusing the surface hit
    instead of traversing the boundary (DevMedium.alias_surface) gives the identical image."""
    cs, world, seed = scenes.pawn_fog(width=48, spp=4)
    monkeypatch.setenv("RT_AMD_VARIANT", variant)
    a = emu_mod.render(cs, world, seed)
    monkeypatch.setenv("RT_AMD_NO_ALIAS", "1")
    b = emu_mod.render(cs, world, seed)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name", ["pawn_fog", "pawn_test", "demo2"])
def test_media_events_in_shading_phase_are_exact(knobs, emu_mod, monkeypatch, name, precision):
    """BVH kernels whose media boundaries are the surface set or single leaves (pawn+fog: the
    pawn's interior aliases the surface, the fog is one sphere) run the segment's media events in
    the shading phase (rt_trace.h media_events_late) instead of the traversal loop's query chain:
    the same queries, draws and order, so the image is bit-identical (RT_AMD_MEDIA_LATE=0)."""
    fn = {"pawn_fog": scenes.pawn_fog, "pawn_test": scenes.pawn_test, "demo2": scenes.demo2}[name]
    cs, world, seed = fn(width=48, spp=4)
    a = emu_mod.render(cs, world, seed, precision=precision)
    monkeypatch.setenv("RT_AMD_MEDIA_LATE", "0")
    b = emu_mod.render(cs, world, seed, precision=precision)
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("variant", ["1", "2"])
@pytest.mark.parametrize("name", ["bunny_cornell", "demo1"])
def test_large_primitive_prefix_is_exact(knobs, emu_mod, monkeypatch, variant, name):
    """The surface set's large primitives (Cornell walls, demo1's ground sphere) tested before the
    BVH instead of inside it: the closest-hit key carries the global depth-first order, so the
    image is bit-identical, and the traversal does less work."""
    fn = {"bunny_cornell": scenes.bunny_cornell, "demo1": scenes.demo1}[name]
    cs, world, seed = fn(width=48, spp=4)
    monkeypatch.setenv("RT_AMD_VARIANT", variant)
    monkeypatch.setenv("RT_AMD_NO_BOX", "1")  # exact claim: per-face tests in and out of the BVH
    a, ca = emu_mod.render(cs, world, seed, counters=True)
    monkeypatch.setenv("RT_AMD_NO_PREFIX", "1")
    b, cb = emu_mod.render(cs, world, seed, counters=True)
    assert np.array_equal(a, b, equal_nan=True)
    assert ca["bvh_nodes"] < cb["bvh_nodes"]


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("name,kind", [("bunny_cornell", 1), ("demo1", 2), ("pawn_fog", 1), ("pawn_test", 1), ("bunny_instances", 0)])
def test_one_class_leaves_are_exact(knobs, emu_mod, monkeypatch, name, kind, precision):
    """The host picks one-class leaf kernels from the leaves below BVH nodes (pawn+fog: the pawn's
    triangles in the surface and medium sets; its fog sphere is a single-leaf medium set, tested
    generically), and they render the generic kernel's image bit for bit."""
    cs, world, seed = scenes.CONFIGS[name](width=40, spp=4)
    assert emu_mod.scene_info(world)["leaf_kind"] == kind
    a = emu_mod.render(cs, world, seed, precision=precision)
    monkeypatch.setenv("RT_AMD_LEAF_KIND", "0")
    b = emu_mod.render(cs, world, seed, precision=precision)
    assert np.isfinite(a).all() and a.mean() > 0
    assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("name", ["cornell", "box_gallery", "bunny_cornell"])
def test_box_groups_match_per_face_tests(knobs, oracle_mod, emu_mod, monkeypatch, name):
    """Cuboid faces and the Cornell walls tested as box groups (one slab test per box, DevBox)
    render the image of one parallelogram test per face up to FP32 rounding at the box edges,
    and match the FP64 oracle (which walks the reference's group of parallelograms) per pixel.
    box_gallery has rays inside a glass cuboid (exit faces) and a reflected (det -1) cuboid."""
    fn = {"cornell": scenes.cornell_box, "box_gallery": scenes.box_gallery, "bunny_cornell": scenes.bunny_cornell}[name]
    cs, world, seed = fn(width=64, spp=8)
    a, ca = emu_mod.render(cs, world, seed, counters=True)
    monkeypatch.setenv("RT_AMD_NO_BOX", "1")
    b, cb = emu_mod.render(cs, world, seed, counters=True)
    assert ca["prims_tested"] < cb["prims_tested"]
    assert np.isfinite(a).all()
    assert pixel_agreement(a, b) >= 0.995
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    assert pixel_agreement(a, ref) >= 0.995
    np.testing.assert_allclose(a.reshape(-1, 3).mean(0), ref.reshape(-1, 3).mean(0), rtol=5e-3)


@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("n", [1, 3, 8])
def test_two_level_instancing_matches_oracle(oracle_mod, emu_mod, n, precision):
    """n x n placements of ONE bunny object (rt_instance, 2-level BVH: world boxes -> object-space
    BLAS) against the oracle, which walks the reference's `transform` (ray into object space,
    Geometry.hs:382-391) on the same Philox numbers, and against the same scene with the
    transforms baked into world-space triangles (instance_min=0)."""
    from raytrace_amd import scene as S
    cs, world, seed = scenes.bunny_instances(width=48, spp=4, n=n)
    inst = S.flatten(world)
    baked = S.flatten(world, instance_min=0)
    assert len(inst.instances) == n * n and len(baked.instances) == 0
    assert len(inst.prims) < len(baked.prims) or n == 1
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    for flat in (inst, baked):
        got = emu_mod.render(cs, flat, seed, precision=precision)
        assert np.isfinite(got).all()
        if precision == "f64":
            rel = (np.abs(got - ref) / np.maximum(np.abs(ref), 1e-3)).max(-1)
            assert (rel <= 1e-9).mean() >= 0.999
        else:
            assert pixel_agreement(got, ref) >= 0.99
        np.testing.assert_allclose(got.reshape(-1, 3).mean(0), ref.reshape(-1, 3).mean(0), rtol=5e-3)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_instancing_edge_cases_match_oracle(oracle_mod, emu_mod, precision):
    """scenes.instance_gallery: one object with its own leaf materials placed by a rotation, a
    reflection (det -1), a rotation under a dielectric `<$` and a translation — a textured
    sphere's uv, the parallelogram's front side under the reflection and the outermost-material
    rule through instances, against the oracle's walk of the reference's closures."""
    from raytrace_amd import scene as S
    cs, world, seed = scenes.instance_gallery(width=96, spp=4)
    flat = S.flatten(world)
    assert len(flat.instances) == 4
    ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    got = emu_mod.render(cs, flat, seed, precision=precision)
    if precision == "f64":
        rel = (np.abs(got - ref) / np.maximum(np.abs(ref), 1e-3)).max(-1)
        assert (rel <= 1e-9).mean() >= 0.999
    else:
        assert pixel_agreement(got, ref) >= 0.99
    np.testing.assert_allclose(got.reshape(-1, 3).mean(0), ref.reshape(-1, 3).mean(0), rtol=5e-3)


def test_perlin_tables(oracle_mod):
    """The product's Perlin tables: three permutations of 0..255 (Noise.hs:60-92) and the 256
    gradients of Noise.hs:94-98, identical to the oracle's independent C restatement."""
    from raytrace_amd import perlin
    perm = perlin.permutations()
    assert perm.shape == (3, 256)
    for row in perm:
        assert sorted(row.tolist()) == list(range(256))
    g = perlin.gradients()
    assert np.array_equal(g, oracle_mod.perlin_gradients())
    assert np.allclose((g * g).sum(1), 1.0, atol=1e-12)


def test_textured_scenes_kernel_logic_matches_oracle(oracle_mod, emu_mod):
    """Noise / marble (noiseTest, test/Main.hs:63-86) and image textures: the kernel's source
    built for the host against the oracle, per pixel."""
    img = np.load(os.path.join(GOLDEN, "earthmap_128x64.npy")).astype(np.float32)
    tex = R.imageTexture(img)
    image_world = R.group([R.lambertian(tex) << R.sphere((0, 0, -2), 0.6),
                           R.lambertian(tex) << R.parallelogram((-2, -1, -3), (4, 0, 0), (0, 2.5, 0)),
                           R.lambertian(R.constantTexture(0.5)) << R.sphere((0, -100.6, -2), 100)])
    cases = [scenes.noise_test(width=96, spp=4),
             (R.defaultCameraSettings(cs_imageWidth=80, cs_samplesPerPixel=4, cs_background=R.sky), image_world,
              R.mkStdGen(3))]
    for cs, world, seed in cases:
        got = emu_mod.render(cs, world, seed)
        ref = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
        assert np.isfinite(got).all()
        assert pixel_agreement(got, ref) >= 0.99
        np.testing.assert_allclose(got.reshape(-1, 3).mean(0), ref.reshape(-1, 3).mean(0), rtol=5e-3)


def test_image_texture_lookup_wraps_and_flips(oracle_mod):
    """imageTexture (Texture.hs:31-41): (u, v) = (0, 0) is the bottom-left texel, coordinates
    wrap.  A camera looking straight at a unit quad textured with a 2 x 2 image of four
    colours sees them in image order (row 0 at the top)."""
    img = np.array([[[1, 0, 0], [0, 1, 0]], [[0, 0, 1], [1, 1, 0]]], np.float32)
    world = R.lightSource(R.imageTexture(img)) << R.parallelogram((-1, -1, -1), (2, 0, 0), (0, 2, 0))
    cs = R.defaultCameraSettings(cs_imageWidth=4, cs_aspectRatio=1.0, cs_samplesPerPixel=1,
                                 cs_vfov=2 * np.arctan(0.5), cs_center=(0, 0, 1), cs_lookAt=(0, 0, 0))
    out = oracle_mod.render(cs, world, R.mkStdGen(1), mode=oracle_mod.RNG_PHILOX)
    assert np.allclose(out[0, 0], [1, 0, 0]) and np.allclose(out[0, 3], [0, 1, 0])
    assert np.allclose(out[3, 0], [0, 0, 1]) and np.allclose(out[3, 3], [1, 1, 0])


def _kat_scene(kind):
    """Analytic known-answer scenes: an emitter of radiance 1 (or a
    mirror of albedo 0.5 in front of a large emitter) seen head-on by a 16 x 16 camera with a
    1:1 viewport of half-width 1 at distance 1, background 0.  Returns (world, mask) where
    mask[j, i] is 1 / 0.5 / 0 for pixels whose whole footprint lies inside / mirrored / outside
    the primitive (-1: straddles an edge, not checked).  The pixel jitter cannot move a sample out
    of its pixel footprint, so these pixels are exact whatever the random numbers."""
    import numpy as np
    n = 16
    light = R.lightSource(R.constantTexture(1.0))
    # pixel (j, i) covers x in [-1 + i/8, -1 + (i+1)/8], y in [1 - (j+1)/8, 1 - j/8] on the z = -1 plane
    xs0 = -1 + np.arange(n) / 8.0
    ys1 = 1 - np.arange(n) / 8.0
    X0, Y1 = np.meshgrid(xs0, ys1)
    X1, Y0 = X0 + 1 / 8.0, Y1 - 1 / 8.0
    mask = -np.ones((n, n))
    if kind == "sphere":   # Geometry.hs:58-94, radius 0.5 at the plane's centre (far side behind)
        world = light << R.sphere((0, 0, -1.5), 0.5)
        # conservative: inside if the pixel's rays all hit: angular radius asin(0.5/1.5) ~ 0.3398 at z=-1
        rr = np.tan(np.arcsin(0.5 / 1.5))
        far = np.maximum(np.maximum(np.hypot(X0, Y0), np.hypot(X1, Y1)), np.maximum(np.hypot(X0, Y1), np.hypot(X1, Y0)))
        near = np.hypot(np.clip(0, X0, X1), np.clip(0, Y0, Y1))
        mask[far < rr - 1e-3] = 1
        mask[near > rr + 1e-3] = 0
    elif kind == "triangle":  # planeShape with a, b >= 0, a + b <= 1 (Geometry.hs:117-151)
        world = light << R.triangle(((-0.5, -0.5, -1), (0, 0)), ((0.5, -0.5, -1), (1, 0)), ((-0.5, 0.5, -1), (0, 1)))
        inside = lambda x, y: (x >= -0.5) & (y >= -0.5) & (x + y <= 0.0)
        allin = inside(X0, Y0) & inside(X1, Y0) & inside(X0, Y1) & inside(X1, Y1)
        anyin = (X1 > -0.5) & (Y1 > -0.5) & (X0 + Y0 < 0.0)
        mask[allin] = 1
        mask[~anyin] = 0
    elif kind == "parallelogram":
        world = light << R.parallelogram((-0.5, -0.25, -1), (1.0, 0, 0), (0.25, 0.75, 0))
        def inside(x, y):
            b = (y + 0.25) / 0.75
            a = (x + 0.5) - 0.25 * b
            return (a >= 0) & (a <= 1) & (b >= 0) & (b <= 1)
        allin = inside(X0, Y0) & inside(X1, Y0) & inside(X0, Y1) & inside(X1, Y1)
        anyin = inside(X0, Y0) | inside(X1, Y0) | inside(X0, Y1) | inside(X1, Y1) | \
            ((X1 > -0.5) & (X0 < 0.75) & (Y1 > -0.25) & (Y0 < 0.5) & ~(X1 < -0.5 + 0.25 * (Y0 + 0.25) / 0.75) &
             ~(X0 > 0.5 + 0.25 * (Y1 + 0.25) / 0.75))
        mask[allin] = 1
        mask[~anyin] = 0
    else:  # mirror (Material.hs:64-67): albedo 0.5 mirror facing the camera, emitter behind the camera
        world = R.group([R.mirror(R.constantTexture(0.5)) << R.parallelogram((-0.5, -0.5, -1), (1, 0, 0), (0, 1, 0)),
                         light << R.parallelogram((-10, -10, 5), (0, 20, 0), (20, 0, 0))])
        allin = (X0 >= -0.5) & (X1 <= 0.5) & (Y0 >= -0.5) & (Y1 <= 0.5)
        mask[allin] = 0.5
        mask[(X1 <= -0.5) | (X0 >= 0.5) | (Y1 <= -0.5) | (Y0 >= 0.5)] = 0
    cs = R.defaultCameraSettings(cs_imageWidth=n, cs_aspectRatio=1.0, cs_samplesPerPixel=4, cs_vfov=np.pi / 2,
                                 cs_center=(0, 0, 0), cs_lookAt=(0, 0, -1), cs_focusDist=1.0,
                                 cs_background=R.constBackground(0.0), cs_maxRecursionDepth=5)
    return cs, world, mask


@pytest.mark.parametrize("kind", ["sphere", "triangle", "parallelogram", "mirror"])
def test_oracle_known_answer_hits(oracle_mod, kind):
    cs, world, mask = _kat_scene(kind)
    out = oracle_mod.render(cs, world, R.mkStdGen(5), mode=oracle_mod.RNG_PHILOX)
    assert out.shape == (16, 16, 3)
    m = mask >= 0
    assert m.sum() > 100 and (mask == (0.5 if kind == "mirror" else 1)).sum() > 4
    np.testing.assert_array_equal(out[m], np.repeat(mask[m][:, None], 3, axis=1))


def test_philox_and_splitmix_modes_agree_statistically(oracle_mod):
    """The device's direct samplers (Philox mode) and the reference's rejection samplers
    (splitmix mode) estimate the same image."""
    cs, world, seed = scenes.cornell_box(spp=64, width=150)
    a = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_PHILOX)
    b = oracle_mod.render(cs, world, seed, mode=oracle_mod.RNG_SPLITMIX)
    np.testing.assert_allclose(a.reshape(-1, 3).mean(0), b.reshape(-1, 3).mean(0), rtol=0.02)
    assert np.sqrt(((block8(np.minimum(a, 1)) - block8(np.minimum(b, 1))) ** 2).mean()) < 0.01


def test_oracle_edge_cases(oracle_mod):
    cs, world, seed = scenes.cornell_box(spp=2, width=16)
    # maxRecursionDepth 0: every sample is black, not background (Ray.hs:176)
    black = oracle_mod.render(cs.replace(cs_maxRecursionDepth=0, cs_background=__import__("raytrace_amd").constBackground(1.0)),
                              world, seed)
    assert (black == 0).all()
    # depth 1: only emission seen directly (the light) survives
    d1 = oracle_mod.render(cs.replace(cs_maxRecursionDepth=1), world, seed)
    assert set(np.unique(np.round(d1, 6))) <= {0.0, 7.5, 15.0}
    # width-1 image
    one = oracle_mod.render(cs.replace(cs_imageWidth=1), world, seed)
    assert one.shape == (1, 1, 3)


@pytest.mark.parametrize("name,boxes,prefix", [("cornell", 3, 0), ("box_gallery", 4, 0), ("bunny_cornell", 1, 6),
                                               ("demo1", 0, 1), ("pawn_fog", 0, 0), ("readme", 0, 0)])
def test_host_build_box_groups_and_prefix(emu_mod, name, boxes, prefix):
    """The host build finds the box groups (the Cornell walls = 5 faces of the 555-cube, every
    `cuboid`) and the BVH scenes' surface prefix (the walls and the light around the bunny,
    demo1's ground sphere; nothing for the pawn's triangles)."""
    cs, world, seed = scenes.CONFIGS[name]()
    info = emu_mod.scene_info(world)
    assert info["boxes"] == boxes and info["prefix"] == prefix, info
