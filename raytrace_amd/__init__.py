"""raytrace_amd — MI355X-native drop-in for UnaryPlus/raytrace's per-pixel radiance loop.

The public names mirror the reference's modules (Graphics.Ray, .Core, .Geometry, .Material,
.Texture): build a scene with the same smart constructors, call `raytrace(settings, world,
seed)`, get the image.  The render runs in a hand-written HIP kernel for gfx950
(raytrace_amd/csrc/rt_kernel.hip) behind the C ABI of include/rt.h.
"""
from .camera import (Background, CameraSettings, constBackground, defaultCameraSettings, grayFade, image_height,
                     lerpYBackground, sky)
from .core import (V3, X, Y, Z, StdGen, allCorners, boxHull, boxJoin, component, degrees, fromCorners, infinity,
                   inInterval, longestDim, midpoint, mkStdGen, padBox, padInterval, reflect, shiftBox)
from .errors import RtDeviceError, RtError, RtInvalid, RtUnsupported
from .geometry import (M44, Mesh, ObjParseError, boundingBox, bvhNode, bvhTree, constantMedium, cuboid, group,
                       moving, parallelogram, parseObj, pureGeometry, readObj, rotateX, rotateY, rotateZ, scale,
                       sphere, transform, transformVertices, translate, triangle, triangleMesh, withMaterial)
from .material import (Material, Texture, anisotropic, checkerTexture, constantTexture, dielectric, imageTexture,
                       isotropic, lambertian, lightSource, lommelSeeliger, marbleTexture, metal, mirror, noiseTexture,
                       pitchBlack, solidTexture, transparent, uvTexture)
from .ray import DeviceScene, MultiDeviceScene, encode8, raytrace, readImage, render_shard, writeImage, writeImageSqrt
from .scene import FlatScene, flatten

__version__ = "0.1.0"
