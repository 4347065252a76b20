"""Host-side mirror of the reference API: camera set-up, boxes, bvhTree, matrices, OBJ parsing,
flattening (no GPU needed)."""
import math

import numpy as np
import pytest

import raytrace_amd as R
from raytrace_amd import geometry as G
from raytrace_amd import scene as S
from raytrace_amd import scenes
from raytrace_amd.camera import camera_basis, image_height


def test_image_height_bankers_rounding():
    # Ray.hs:123 `round (fromIntegral w / aspect)`: 600 / (16/9) = 337.5 -> 338 (round half even)
    assert image_height(R.defaultCameraSettings(cs_imageWidth=600, cs_aspectRatio=16 / 9)) == 338
    assert image_height(R.defaultCameraSettings(cs_imageWidth=5, cs_aspectRatio=2.0)) == 2   # 2.5 -> 2
    assert image_height(R.defaultCameraSettings(cs_imageWidth=7, cs_aspectRatio=2.0)) == 4   # 3.5 -> 4
    assert image_height(R.defaultCameraSettings(cs_imageWidth=120, cs_aspectRatio=16 / 9)) == 68


def test_camera_basis_cornell_known_answer():
    cs, _, _ = scenes.cornell_box()
    cb = camera_basis(cs)
    # vfov 40 deg, focusDist 10: viewport height 2*10*tan(20 deg)
    vh = 10 * math.tan(math.radians(40) / 2) * 2
    assert cb.height == 600
    np.testing.assert_allclose(cb.pixel_v, (0, -vh / 600, 0), atol=1e-15)
    np.testing.assert_allclose(cb.pixel_u, (-vh / 600, 0, 0), atol=1e-15)  # u = up x w points to -x here
    # the pixel centre of the middle of the image looks straight down +z
    mid = np.array(cb.top_left) + 300 * np.array(cb.pixel_u) + 300 * np.array(cb.pixel_v)
    np.testing.assert_allclose(mid, (278, 278, -790), atol=1e-9)
    assert cb.disk_u == (0.0, 0.0, 0.0) or np.allclose(cb.disk_u, 0)


def test_default_camera_settings_match_reference():
    cs = R.defaultCameraSettings()
    assert cs.cs_center == (0.0, 0.0, 0.0) and cs.cs_lookAt == (0.0, 0.0, -1.0) and cs.cs_up == (0.0, 1.0, 0.0)
    assert cs.cs_vfov == math.pi / 2 and cs.cs_aspectRatio == 1.0 and cs.cs_imageWidth == 100
    assert cs.cs_samplesPerPixel == 10 and cs.cs_maxRecursionDepth == 10
    assert cs.cs_defocusAngle == 0.0 and cs.cs_focusDist == 10.0 and cs.cs_redirectTargets == []
    assert cs.cs_background == R.constBackground(1.0)


def test_boxes_and_padding():
    q = R.parallelogram((0, 0, 0), (1, 0, 0), (0, 1, 0))
    # Geometry.hs:144 pads plane shapes by 1e-4 so flat boxes have volume
    assert q.bbox == ((-0.0001, 1.0001), (-0.0001, 1.0001), (-0.0001, 0.0001))
    s = R.sphere((1, 2, 3), 2)
    assert s.bbox == ((-1.0, 3.0), (0.0, 4.0), (1.0, 5.0))
    assert R.longestDim(((0, 1), (0, 3), (0, 2))) == R.Y
    assert R.longestDim(((0, 1), (0, 1), (0, 1))) == R.Z  # ties fall through to Z (Core.hs:37-40)
    with pytest.raises(ValueError):
        R.group([])
    with pytest.raises(ValueError):
        R.bvhTree([])


def test_bvh_tree_median_split_structure():
    # Geometry.hs:368-377: longest axis of the joined boxes, stable sort by midpoint, left = n div 2
    obs = [R.sphere((x, 0, 0), 0.1) for x in (3, 1, 2, 0, 4)]
    t = R.bvhTree(obs)
    assert isinstance(t, G.BvhNode)
    left, right = t.left, t.right
    # 5 objects: left gets 2 (x = 0, 1), right 3 (x = 2, 3, 4)
    xs_left = sorted(o.center[0] for o in _leaves(left))
    xs_right = sorted(o.center[0] for o in _leaves(right))
    assert xs_left == [0, 1] and xs_right == [2, 3, 4]
    assert R.bvhTree([obs[0]]) is obs[0]


def _leaves(g):
    if isinstance(g, (G.Sphere, G.PlaneShape)):
        return [g]
    out = []
    for c in G.children_of(g):
        out += _leaves(c)
    return out


def test_matrices_and_inverse():
    m = R.translate((265, 0, 295)) @ R.rotateY(R.degrees(15))
    inv = G.inv44(m)
    prod = np.array(G.mmul(m, inv))
    np.testing.assert_allclose(prod, np.eye(4), atol=1e-12)
    c, s = math.cos(R.degrees(15)), math.sin(R.degrees(15))
    assert m[0][0] == c and m[0][2] == s and m[2][0] == -s and m[0][3] == 265


def test_parse_obj_semantics():
    text = "# comment\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0 # trailing\nvt 0.5\nvt 0.25 0.75\nf 1 2 3 4\nf -4/1 -3/2 -2//\n"
    m = R.parseObj(text)
    assert len(m.vertices) == 4 and m.uvs == [(0.5, 0.0), (0.25, 0.75)]
    # the quad is fan-triangulated: (1,2,3), (1,3,4); negative indices count from the end
    assert m.faces[0] == ((0, None), (1, None), (2, None))
    assert m.faces[1] == ((0, None), (2, None), (3, None))
    assert m.faces[2] == ((0, 0), (1, 1), (2, None))


@pytest.mark.parametrize("text,msg", [
    ("v 0 0\n", "line 1: invalid 'v' statement"),
    ("v 0 0 0\nv 1 0 0\nf 1 2\n", "line 3: invalid 'f' statement (fewer than 3 vertices)"),
    ("v 0 0 0\nf 1 2 5\n", "line 2: index out of bounds: 2"),
    ("v 0 0 0\nv 0 0 0\nv 0 0 0\nf 1 2 x3\n", "line 4: expected number"),
    ("v 0 0 0\nv 0 0 0\nv 0 0 0\nf 1 2 3a\n", "line 4: unexpected character 'a'"),
    ("vt a\n", "line 1: invalid 'vt' statement"),
    ("v .5 0 0\n", "line 1: invalid 'v' statement"),  # Haskell's read rejects ".5"
])
def test_parse_obj_errors(text, msg):
    with pytest.raises(R.ObjParseError) as e:
        R.parseObj(text)
    assert str(e.value) == msg


def test_mesh_assets_parse():
    for name, nv, nf in [("bunny.obj", 2503, 4968), ("pawn.obj", 602, 1200)]:
        m = scenes.load_mesh(name)
        assert len(m.vertices) == nv and len(m.faces) == nf


def test_flatten_materials_outermost_wins_and_media_lifted():
    red = R.lambertian(R.constantTexture((1, 0, 0)))
    blue = R.lambertian(R.constantTexture((0, 0, 1)))
    inner = blue << R.sphere((0, 0, 0), 1)
    world = R.group([red << inner, R.isotropic(R.constantTexture(1)) << R.constantMedium(0.5, R.sphere((0, 0, 0), 3))])
    f = R.flatten(world)
    assert len(f.prims) == 2 and len(f.media) == 1
    surf = f.prims[f.prims["set"] == 0][0]
    assert f.materials[surf["material"]]["kind"] == 2
    tex = f.textures[f.materials[surf["material"]]["texture"]]
    assert tuple(tex["c0"]) == (1.0, 0.0, 0.0)  # the outer `<$` (red) wins, as fmap composition does
    assert f.prims[f.prims["set"] == 1][0]["material"] == -1
    assert f.media[0]["density"] == 0.5
    # depth-first orders: surface leaf 0, medium 1, boundary leaf 2
    assert sorted(f.prims["order"].tolist()) == [0, 2] and f.media[0]["order"] == 1


def test_flatten_bakes_rigid_transform_exactly():
    cube = R.cuboid(R.fromCorners((0, 0, 0), (165, 330, 165)))
    m = R.translate((265, 0, 295)) @ R.rotateY(R.degrees(15))
    f = R.flatten(R.lambertian(R.constantTexture(0.73)) << R.transform(m, cube))
    assert len(f.prims) == 6
    q0 = f.prims[0]["p"][:3]
    np.testing.assert_allclose(q0, G.mul_point(m[:3], (0.0, 0.0, 165.0)), rtol=0, atol=0)


def test_flatten_reflection_keeps_object_front_side():
    flip = G.M44(((-1, 0, 0, 0), (0, 1, 0, 0), (0, 0, 1, 0), (0, 0, 0, 1)))
    quad = R.parallelogram((0, 0, 0), (1, 0, 0), (0, 1, 0))  # normal +z
    f = R.flatten(R.lambertian(R.constantTexture(1)) << R.transform(flip, quad))
    p = f.prims[0]
    u, v = np.array(p["p"][3:6]), np.array(p["p"][6:9])
    # reference: object-space normal +z mapped by the (reflection) matrix stays +z
    assert np.cross(u, v)[2] > 0
    assert tuple(p["uv"]) == (0.0, 0.0, 0.0, 1.0, 1.0, 0.0)


def test_flatten_rejects_what_the_device_cannot_evaluate():
    with pytest.raises(R.RtUnsupported):
        R.flatten(R.lambertian(R.solidTexture(lambda p: p)) << R.sphere((0, 0, 0), 1))
    with pytest.raises(R.RtUnsupported):
        R.flatten(R.lambertian(R.constantTexture(1)) << R.transform(R.scale(2), R.sphere((0, 0, 0), 1)))
    with pytest.raises(R.RtInvalid):
        R.flatten(R.sphere((0, 0, 0), 1))  # no material
    with pytest.raises(TypeError):
        R.constantMedium(1.0, R.constantMedium(1.0, R.sphere((0, 0, 0), 1)))
    from raytrace_amd.camera import background_of
    with pytest.raises(R.RtUnsupported):
        background_of(R.defaultCameraSettings(cs_background=lambda ray: (0, 0, 0)))


def test_flatten_configs_sizes():
    assert len(R.flatten(scenes.cornell_box()[1]).prims) == 18
    f = R.flatten(scenes.pawn_fog()[1])
    assert len(f.media) == 2 and (f.prims["set"] == 0).sum() == 1200 and (f.prims["set"] == 1).sum() == 1200
    assert (f.prims["set"] == 2).sum() == 1
    # the dielectric surface and the medium boundary share geometric identities (self-skip)
    g0 = set(f.prims[f.prims["set"] == 0]["gid"].tolist())
    g1 = set(f.prims[f.prims["set"] == 1]["gid"].tolist())
    assert g0 == g1


def test_stdgen_split_and_random_ranges():
    g = R.mkStdGen(234)
    a, b = g.split()
    assert a.gamma == g.gamma and a.seed == (g.seed + 2 * g.gamma) % 2 ** 64
    x, g2 = g.random()
    assert 0.0 <= x <= 1.0 and g2 != g
    y, _ = g.randomR(-1.0, 1.0)
    assert -1.0 <= y <= 1.0
    assert R.mkStdGen(1).key() != R.mkStdGen(2).key()


def test_encode8_matches_reference_quantisation():
    # min(255, floor(256 * transfer(clamp01 x))) (measured on pawn_demo.png, tests/golden/make_golden.py)
    x = np.array([[[0.0, 0.8, 1.0], [2.0, -1.0, 0.25]]])
    np.testing.assert_array_equal(R.encode8(x, "sqrt"), [[[0, 228, 255], [255, 0, 128]]])
    np.testing.assert_array_equal(R.encode8(np.array([[[0.8, 1.0, 0.0]]]), "srgb"), [[[232, 255, 0]]])


def test_experiment_knobs_ignored_without_the_switch(emu_mod, monkeypatch):
    """The library reads its RT_AMD_* tuning knobs only with RT_AMD_EXPERIMENTS set (rt_internal.h
    rt_knob): with the switch unset, a scene renders identically whatever knobs a caller's
    environment holds (host build + kernel logic through the emulator); with it set they act."""
    from raytrace_amd import scenes
    cs, world, seed = scenes.bunny_cornell(width=24, spp=4)
    monkeypatch.delenv("RT_AMD_EXPERIMENTS", raising=False)
    base = emu_mod.render(cs, world, seed)
    info = emu_mod.scene_info(world)
    knobs = {"RT_AMD_NO_BOX": "1", "RT_AMD_NO_PREFIX": "1", "RT_AMD_VARIANT": "1", "RT_AMD_LEAF_MAX": "7",
             "RT_AMD_LEAF_KIND": "0", "RT_AMD_CHUNK": "3", "RT_AMD_AGG": "0", "RT_AMD_PREFIX_AREA": "0.9",
             "RT_AMD_LEAF_EXIT_PCT": "90", "RT_AMD_TRAV_PCT": "10", "RT_AMD_NO_ALIAS": "1", "RT_AMD_LDS_NODES": "0"}
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    assert emu_mod.scene_info(world) == info
    np.testing.assert_array_equal(emu_mod.render(cs, world, seed), base)
    monkeypatch.setenv("RT_AMD_EXPERIMENTS", "0")
    assert emu_mod.scene_info(world) == info
    monkeypatch.setenv("RT_AMD_EXPERIMENTS", "1")  # switched on, the knobs change the host build
    on = emu_mod.scene_info(world)
    assert on["prefix"] == 0 and on["boxes"] == 0 and on != info


def test_caller_output_buffer_is_checked():
    # raytrace(..., out=) / MultiDeviceScene.render(..., out=): the library writes the whole frame
    # into the caller's array, so anything it could not fill is refused before any device call
    from raytrace_amd.errors import RtInvalid
    from raytrace_amd.ray import _out_buffer
    buf = np.empty((4, 5, 3), np.float64)
    assert _out_buffer(buf, (4, 5, 3), np.float64) is buf
    assert _out_buffer(None, (4, 5, 3), np.uint8).dtype == np.uint8
    for bad in (np.empty((4, 5, 3), np.float32), np.empty((5, 4, 3)), np.empty((4, 5, 3, 1)),
                np.empty((4, 10, 3))[:, ::2], [[0.0]]):
        with pytest.raises(RtInvalid):
            _out_buffer(bad, (4, 5, 3), np.float64)
    ro = np.empty((4, 5, 3))
    ro.flags.writeable = False
    with pytest.raises(RtInvalid):
        _out_buffer(ro, (4, 5, 3), np.float64)
