"""The benchmark / parity scenes (BASELINE.json configs), built with the mirrored constructors
exactly as the reference writes them.  Each returns (CameraSettings, world, StdGen).

  readme_scene   README.md:41-55 (config 1, `example_image.png`)
  cornell_box    test/Main.hs:188-218 (config 2, `cornell_box_redirect.png`)
  demo1          test/Main.hs:136-186 (config 3; the reference seeds it with newStdGen,
                 here a fixed mkStdGen so the world is reproducible)
  bunny_cornell  config 4 (composed: Cornell walls + light + images/bunny.obj)
  pawn_fog       config 5 (composed: pawnTest, test/Main.hs:323-344, plus a fog sphere)
  pawn_test      test/Main.hs:323-344 verbatim (`pawn_demo.png`)
  demo2          test/Main.hs:259-321 verbatim (`demo2.png`; the reference's test entry point,
                 demoTest = demo2 "test_image.png" 400 250 4)
"""
from __future__ import annotations

import math
import os

from .camera import constBackground, defaultCameraSettings, grayFade, sky
from .core import V3, degrees, mkStdGen, midpoint, norm, sub
from .geometry import (boundingBox, bvhTree, cuboid, constantMedium, group, parallelogram, pureGeometry, readObj,
                       rotateX, rotateY, scale, sphere, transform, transformVertices, translate, triangleMesh)
from .geometry import moving
from .material import (checkerTexture, constantTexture, dielectric, imageTexture, isotropic, lambertian, lightSource,
                       marbleTexture, metal, mirror, noiseTexture)
from .core import fromCorners

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def readme_scene(width=600, spp=50):
    world = group([
        lambertian(checkerTexture(20, 10, 0.2, 0.8)) << sphere(V3(0, 0, 0), 1),
        lambertian(constantTexture(V3(0, 0.2, 0.5))) << sphere(V3(0, -1000, 0), 999),
        mirror(constantTexture(0.8)) << parallelogram(V3(-3.25, -1, -0.75), V3(1.25, 0, -1.25), V3(0, 2, 0)),
    ])
    settings = defaultCameraSettings(cs_center=V3(-0.75, 0, 2), cs_lookAt=V3(0, 0, -1), cs_aspectRatio=16 / 9,
                                     cs_imageWidth=width, cs_samplesPerPixel=spp)
    return settings, world, mkStdGen(100)


def cornell_walls(light_emit=15.0):
    red = lambertian(constantTexture(V3(0.65, 0.05, 0.05)))
    white = lambertian(constantTexture(V3(0.73, 0.73, 0.73)))
    green = lambertian(constantTexture(V3(0.12, 0.45, 0.15)))
    light = lightSource(constantTexture(V3(light_emit, light_emit, light_emit)))
    return [
        green << parallelogram(V3(555, 0, 0), V3(0, 555, 0), V3(0, 0, 555)),
        red << parallelogram(V3(0, 0, 0), V3(0, 555, 0), V3(0, 0, 555)),
        light << parallelogram(V3(343, 554, 332), V3(-130, 0, 0), V3(0, 0, -105)),
        white << parallelogram(V3(0, 0, 0), V3(555, 0, 0), V3(0, 0, 555)),
        white << parallelogram(V3(555, 555, 555), V3(-555, 0, 0), V3(0, 0, -555)),
        white << parallelogram(V3(0, 0, 555), V3(555, 0, 0), V3(0, 555, 0)),
    ], white


CORNELL_TARGETS = [(0.25, V3(343, 554, 332), V3(-130, 0, 0), V3(0, 0, -105))]


def cornell_settings(width=600, spp=200, depth=50, redirect=True):
    return defaultCameraSettings(
        cs_aspectRatio=1.0, cs_imageWidth=width, cs_samplesPerPixel=spp, cs_maxRecursionDepth=depth,
        cs_background=constBackground(V3(0, 0, 0)), cs_vfov=degrees(40), cs_center=V3(278, 278, -800),
        cs_lookAt=V3(278, 278, 0), cs_redirectTargets=list(CORNELL_TARGETS) if redirect else [])


def cornell_box(spp=200, depth=50, width=600, redirect=True):
    walls, white = cornell_walls()
    world = group(walls + [
        transform(translate(V3(265, 0, 295)) @ rotateY(degrees(15)),
                  white << cuboid(fromCorners(V3(0, 0, 0), V3(165, 330, 165)))),
        transform(translate(V3(130, 0, 65)) @ rotateY(degrees(-18)),
                  white << cuboid(fromCorners(V3(0, 0, 0), V3(165, 165, 165)))),
    ])
    return cornell_settings(width, spp, depth, redirect), world, mkStdGen(234)


def demo1_world(gen):
    """genWorld of test/Main.hs:150-168 evaluated with the splitmix StdGen; returns (world, gen')."""
    material_ground = lambertian(constantTexture(V3(0.5, 0.5, 0.5)))
    material_glass = dielectric(1.5)
    material_diffuse = lambertian(constantTexture(V3(0.4, 0.2, 0.1)))
    material_mirror = mirror(constantTexture(V3(0.7, 0.6, 0.5)))
    big = [
        material_ground << sphere(V3(0, -1000, 0), 1000),
        material_glass << sphere(V3(0, 1, 0), 1),
        material_diffuse << sphere(V3(-4, 1, 0), 1),
        material_mirror << sphere(V3(4, 1, 0), 1),
    ]
    small = []
    for a in range(-11, 11):
        for b in range(-11, 11):
            ox, gen = gen.randomR(0.0, 0.9)
            oz, gen = gen.randomR(0.0, 0.9)
            center = (float(a) + ox, 0.2, float(b) + oz)
            if norm(sub(center, V3(4, 0.2, 0))) <= 0.9:
                continue
            choose, gen = gen.random()
            if choose < 0.8:
                c1 = []
                for _ in range(3):
                    x, gen = gen.random()
                    c1.append(x)
                c2 = []
                for _ in range(3):
                    x, gen = gen.random()
                    c2.append(x)
                mat = lambertian(constantTexture(V3(c1[0] * c2[0], c1[1] * c2[1], c1[2] * c2[2])))
            elif choose < 0.95:
                fuzz, gen = gen.randomR(0.0, 0.5)
                col = []
                for _ in range(3):
                    x, gen = gen.randomR(0.5, 1.0)
                    col.append(x)
                mat = metal(fuzz, constantTexture(V3(*col)))
            else:
                mat = material_glass
            small.append(mat << sphere(center, 0.2))
    return bvhTree(big + small), gen


def demo1(width=1200, spp=500, depth=50, seed=1, aspect=16 / 9):
    """test/Main.hs:136-186 (aspect 16/9: 1200 x 675, the reference's own image size)."""
    world, gen2 = demo1_world(mkStdGen(seed))
    settings = defaultCameraSettings(
        cs_aspectRatio=aspect, cs_imageWidth=width, cs_samplesPerPixel=spp, cs_maxRecursionDepth=depth,
        cs_vfov=degrees(20), cs_center=V3(13, 2, 3), cs_lookAt=V3(0, 0, 0), cs_defocusAngle=degrees(0.6),
        cs_focusDist=10, cs_background=sky)
    return settings, world, gen2


def demo1_1200x800(width=1200, spp=500, depth=50, seed=1):
    """demo1 at BASELINE.json's 1200 x 800 (aspect 3/2).  The reference renders 1200 x 675
    (test/Main.hs:170-172, aspect 16/9); BASELINE.json's configs line says 1200x800, so both
    are provided."""
    return demo1(width=width, spp=spp, depth=depth, seed=seed, aspect=3 / 2)


def load_mesh(name):
    return readObj(os.path.join(DATA_DIR, name))


def bunny_cornell(width=800, spp=1000, depth=50):
    """Config 4 (composed, documented in DESIGN.md): the Cornell walls and light of config 2
    with images/bunny.obj centred on its bbox midpoint (as bunnyTest, test/Main.hs:376),
    rotated 30 degrees about y, scaled by 2000 and set on the floor at x = z = 278."""
    mesh = load_mesh("bunny.obj")
    center = tuple(midpoint(i) for i in boundingBox(triangleMesh(mesh)))
    m = rotateY(degrees(30)) @ scale(2000) @ translate(tuple(-c for c in center))
    m1 = transformVertices(m, mesh)
    ymin = min(v[1] for v in m1.vertices)
    mesh2 = transformVertices(translate(V3(278, -ymin, 278)), m1)
    walls, white = cornell_walls()
    world = group(walls + [white << triangleMesh(mesh2)])
    return cornell_settings(width, spp, depth, True), world, mkStdGen(234)


def _pawn_world(mesh, fog):
    pawn = triangleMesh(mesh)
    objs = [pureGeometry(dielectric(1.5) << pawn),
            isotropic(constantTexture(V3(1, 0, 0))) << constantMedium(5, pawn)]
    if fog:
        objs.append(isotropic(constantTexture(1)) << constantMedium(0.02, sphere(V3(0, 2.75, 0), 20)))
    return group(objs)


def bunny_instances(width=400, spp=64, depth=50, n=3):
    """Two-level instancing test scene (not a reference scene): the Cornell walls and light
    around an n x n grid of the SAME bunny mesh object (object space: centred)
    placed by rigid transforms (rotateY by a different angle, translate), with materials applied
    outside the transforms (lambertian colours, one mirror, one dielectric) — every placement is
    an rt_instance of one object (Geometry.hs:382-391).  The object is scaled 900 * 3 / n so the
    grid fits the room for any n."""
    mesh = load_mesh("bunny.obj")
    center = tuple(midpoint(i) for i in boundingBox(triangleMesh(mesh)))
    obj_mesh = transformVertices(scale(900 * 3 / max(n, 3)) @ translate(tuple(-c for c in center)), mesh)
    ymin = min(v[1] for v in obj_mesh.vertices)
    bunny = triangleMesh(obj_mesh)  # one object, shared by every placement below
    walls, white = cornell_walls()
    placed = []
    for i in range(n):
        for j in range(n):
            k = i * n + j
            x, z = 100 + 355 * (i + 0.5) / n, 100 + 355 * (j + 0.5) / n
            m = translate(V3(x, -ymin, z)) @ rotateY(degrees(40 * k))
            if k == 1:
                mat = mirror(constantTexture(V3(0.9, 0.9, 0.9)))
            elif k == n * n - 1:
                mat = dielectric(1.5)
            else:
                mat = lambertian(constantTexture(V3(0.3 + 0.07 * (k % 10), 0.5, 0.8 - 0.06 * (k % 10))))
            placed.append(mat << transform(m, bunny))
    world = group(walls + placed)
    return cornell_settings(width, spp, depth, redirect=True), world, mkStdGen(91)


def instance_gallery(width=160, spp=8, depth=20):
    """Two-level instancing edge cases (test scene, not a reference scene): ONE object with its
    own leaf materials — a bunny mesh (lambertian), a checker-textured sphere (sphereUV in object
    space) and a metal parallelogram — placed four times: a rotation, a reflection (x -> -x,
    det -1: the object's front sides must follow the reference's m-mapped normals), a rotation
    with a dielectric `<$` over the whole placement (the outermost material wins), and a
    translation; sky background."""
    from .geometry import M44
    mesh = load_mesh("bunny.obj")
    center = tuple(midpoint(i) for i in boundingBox(triangleMesh(mesh)))
    obj_mesh = transformVertices(scale(6) @ translate(tuple(-c for c in center)), mesh)
    obj = group([lambertian(constantTexture(V3(0.8, 0.6, 0.3))) << triangleMesh(obj_mesh),
                 lambertian(checkerTexture(8, 4, V3(0.9, 0.1, 0.1), V3(0.1, 0.1, 0.9))) << sphere(V3(0.9, 0.3, 0), 0.35),
                 metal(0.05, constantTexture(V3(0.8, 0.8, 0.8))) << parallelogram(V3(-1, -0.5, -0.8), V3(2, 0, 0),
                                                                                   V3(0, 1.2, 0))])
    reflect_x = M44(((-1, 0, 0, 0), (0, 1, 0, 0), (0, 0, 1, 0), (0, 0, 0, 1)))
    world = group([
        lambertian(constantTexture(V3(0.5, 0.5, 0.5))) << sphere(V3(0, -1000.6, 0), 1000),
        transform(translate(V3(-2.2, 0, -1)) @ rotateY(degrees(35)), obj),
        transform(translate(V3(0, 0, -1.5)) @ reflect_x @ rotateY(degrees(-20)), obj),
        dielectric(1.5) << transform(translate(V3(2.2, 0, -1)) @ rotateY(degrees(120)), obj),
        transform(translate(V3(0.3, 0.2, 1.2)), obj),
    ])
    settings = defaultCameraSettings(cs_center=V3(0, 1.5, 5), cs_lookAt=V3(0, 0.2, 0), cs_imageWidth=width,
                                     cs_vfov=degrees(50), cs_samplesPerPixel=spp, cs_maxRecursionDepth=depth,
                                     cs_background=sky)
    return settings, world, mkStdGen(17)


def pawn_test(width=500, spp=400, depth=20):
    mesh = transformVertices(scale(100), load_mesh("pawn.obj"))
    settings = defaultCameraSettings(cs_center=V3(0, 3.75, 5), cs_lookAt=V3(0, 2.75, 0), cs_imageWidth=width,
                                     cs_vfov=degrees(80), cs_samplesPerPixel=spp, cs_maxRecursionDepth=depth,
                                     cs_background=grayFade)
    return settings, _pawn_world(mesh, fog=False), mkStdGen(55)


def pawn_fog(width=800, spp=2000, depth=20):
    """Config 5 (composed): pawnTest plus an isotropic fog sphere (density 0.02, radius 20)
    enclosing the camera, which exercises the ray-starts-inside case (Geometry.hs:313)."""
    mesh = transformVertices(scale(100), load_mesh("pawn.obj"))
    settings = defaultCameraSettings(cs_center=V3(0, 3.75, 5), cs_lookAt=V3(0, 2.75, 0), cs_imageWidth=width,
                                     cs_vfov=degrees(80), cs_samplesPerPixel=spp, cs_maxRecursionDepth=depth,
                                     cs_background=grayFade)
    return settings, _pawn_world(mesh, fog=True), mkStdGen(55)


def noise_test(width=400, spp=100, depth=50, seed=7):
    """noiseTest (test/Main.hs:63-86): a Perlin-noise ground sphere and a marble ball.  The
    reference seeds it with newStdGen; this build fixes `seed`."""
    world = group([
        lambertian(noiseTexture(2, 2.0, V3(10, 0, 0), 0, 1)) << sphere(V3(0, -1000, 0), 1000),
        lambertian(marbleTexture(V3(0, 0, 1), 4, 0)) << sphere(V3(0, 2, 0), 2),
    ])
    settings = defaultCameraSettings(cs_aspectRatio=16 / 9, cs_imageWidth=width, cs_samplesPerPixel=spp,
                                     cs_maxRecursionDepth=depth, cs_background=sky, cs_vfov=degrees(20),
                                     cs_center=V3(13, 2, 3), cs_lookAt=V3(0, 0, 0))
    return settings, world, mkStdGen(seed)


def box_gallery(width=200, spp=16, depth=50):
    """Test scene for box groups (DevBox): the Cornell walls around a glass cuboid at an oblique
    orientation (rays inside it exit through a face), a fuzzy-metal cuboid under a reflecting
    transform (det -1) and a mirror cuboid.  Not a reference scene."""
    import numpy as np
    walls, white = cornell_walls()
    reflect_x = np.diag([-1.0, 1.0, 1.0, 1.0])
    world = group(walls + [
        transform(translate(V3(300, 120, 300)) @ rotateY(degrees(30)) @ rotateX(degrees(25)),
                  dielectric(1.5) << cuboid(fromCorners(V3(-60, -60, -60), V3(60, 60, 60)))),
        transform(translate(V3(420, 0, 120)) @ reflect_x @ rotateY(degrees(-20)),
                  metal(0.2, constantTexture(V3(0.8, 0.85, 0.9))) << cuboid(fromCorners(V3(0, 0, 0), V3(90, 200, 90)))),
        transform(translate(V3(90, 0, 380)) @ rotateY(degrees(40)),
                  mirror(constantTexture(V3(0.9, 0.9, 0.9))) << cuboid(fromCorners(V3(0, 0, 0), V3(120, 120, 120)))),
    ])
    return cornell_settings(width, spp, depth, redirect=True), world, mkStdGen(77)


def earthmap():
    """images/earthmap.jpg as readImage returns it (Ray.hs:241-245: linear RGB), from the decoded
    8-bit codes committed losslessly as data/earthmap.png (tests/golden/make_earthmap.py)."""
    from .ray import readImage
    return readImage(os.path.join(DATA_DIR, "earthmap.png"))


def demo2_world(gen, earth):
    """generateWorld of test/Main.hs:264-303 evaluated with the splitmix StdGen: 20 x 20 ground
    cuboids of random height (randomR (1, 101) each, i outer, j inner), then 1000 spheres of radius
    10 at V3 (randomR (0, 165)) points (linear's V3 instance draws x, y, z in turn) in a bvhTree
    under translate (V3 (-100) 270 395) . rotateY 15 degrees, the large objects, and two media:
    the camera-enclosing constantMedium 0.0001 (sphere 0 5000) and the blue fog inside the glass
    sphere `boundary`.  Returns (world, gen')."""
    ground = lambertian(constantTexture(V3(0.48, 0.83, 0.53)))
    white = lambertian(constantTexture(V3(0.73, 0.73, 0.73)))
    boxes = []
    for i in range(20):
        for j in range(20):
            x0, z0 = -1000.0 + i * 100.0, -1000.0 + j * 100.0
            y1, gen = gen.randomR(1.0, 101.0)
            boxes.append(cuboid(fromCorners(V3(x0, 0.0, z0), V3(x0 + 100.0, y1, z0 + 100.0))))
    balls = []
    for _ in range(1000):
        p = []
        for _ in range(3):
            x, gen = gen.randomR(0.0, 165.0)
            p.append(x)
        balls.append(sphere(V3(*p), 10))
    boundary = sphere(V3(360, 150, 145), 70)
    large = [
        lightSource(constantTexture(V3(7, 7, 7))) << parallelogram(*DEMO2_LIGHT),
        lambertian(constantTexture(V3(0.7, 0.3, 0.1))) << moving(V3(0, 0, 0), V3(30, 0, 0), sphere(V3(400, 400, 200), 50)),
        dielectric(1.5) << sphere(V3(260, 150, 45), 50),
        dielectric(1.5) << boundary,
        metal(1.0, constantTexture(V3(0.8, 0.8, 0.9))) << sphere(V3(0, 150, 145), 50),
        lambertian(imageTexture(earth)) << transform(translate(V3(400, 0, 400)) @ rotateY(math.pi / 2),
                                                     sphere(V3(0, 200, 0), 100)),
        lambertian(marbleTexture(V3(0, 0, 0.05), 4, 0)) << sphere(V3(220, 280, 300), 80),
    ]
    world = group([
        pureGeometry(group([ground << bvhTree(boxes),
                            white << transform(translate(V3(-100, 270, 395)) @ rotateY(degrees(15)), bvhTree(balls))]
                           + large)),
        isotropic(constantTexture(1)) << constantMedium(0.0001, sphere(V3(0, 0, 0), 5000)),
        isotropic(constantTexture(V3(0.2, 0.4, 0.9))) << constantMedium(0.2, boundary),
    ])
    return world, gen


DEMO2_LIGHT = (V3(123, 554, 147), V3(300, 0, 0), V3(0, 0, 265))


def demo2(width=800, spp=250, depth=4, seed=1234):
    """test/Main.hs:259-321: demo2 path imageWidth samplesPerPixel maxRecursionDepth, world from
    mkStdGen 1234 and the generator after it as raytrace's seed.  Defaults: demo2.png's 800 x 800
    with the reference's own test entry's spp and depth (demoTest: 250, 4); the published image's
    spp and depth are not stated (tests/test_gpu.py pins them against it)."""
    world, gen2 = demo2_world(mkStdGen(seed), earthmap())
    settings = defaultCameraSettings(
        cs_center=V3(478, 278, -600), cs_lookAt=V3(278, 278, 0), cs_vfov=degrees(40), cs_aspectRatio=1.0,
        cs_imageWidth=width, cs_samplesPerPixel=spp, cs_maxRecursionDepth=depth, cs_background=constBackground(0),
        cs_redirectTargets=[(0.25,) + DEMO2_LIGHT])
    return settings, world, gen2


CONFIGS = {
    "readme": readme_scene,
    "cornell": cornell_box,
    "demo1": demo1,
    "demo1_1200x800": demo1_1200x800,
    "bunny_cornell": bunny_cornell,
    "pawn_fog": pawn_fog,
    "pawn_test": pawn_test,
    "noise_test": noise_test,
    "box_gallery": box_gallery,
    "bunny_instances": bunny_instances,
    "instance_gallery": instance_gallery,
    "demo2": demo2,
}
