"""CameraSettings (reference: src/Graphics/Ray.hs:40-98) and the camera set-up of `raytrace`
(Ray.hs:122-155), evaluated in binary64 in the reference's operation order.

`cs_background` is a closure `Ray -> Color` in the reference.  Only reifiable backgrounds
cross the device boundary: a constant colour and a lerp on the ray direction's y component,
which covers every background the reference's demos use (`const c`, `sky`, `grayFade`,
test/Main.hs:19-28).
"""
from __future__ import annotations

import dataclasses
import math
from typing import List, Tuple

from .core import V3, cross, divs, muls, neg, normalize, smul, sub

BG_CONST, BG_LERP_Y = 0, 1


@dataclasses.dataclass(frozen=True)
class Background:
    """kind BG_CONST: c0.  kind BG_LERP_Y: (1 - a) *^ c0 + a *^ c1 with a = 0.5 * (y + 1)."""
    kind: int
    c0: Tuple[float, float, float]
    c1: Tuple[float, float, float] = (0.0, 0.0, 0.0)


def constBackground(c) -> Background:
    """`const c`."""
    return Background(BG_CONST, V3(c))


def lerpYBackground(c0, c1) -> Background:
    return Background(BG_LERP_Y, V3(c0), V3(c1))


sky = lerpYBackground(1.0, (0.5, 0.7, 1.0))       # test/Main.hs:19-22
grayFade = lerpYBackground(0.0, 1.0)             # test/Main.hs:24-28 ((1-a)*0 + a*1 == a exactly)


@dataclasses.dataclass
class CameraSettings:
    """Ray.hs:40-68 (same field names)."""
    cs_center: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    cs_lookAt: Tuple[float, float, float] = (0.0, 0.0, -1.0)
    cs_up: Tuple[float, float, float] = (0.0, 1.0, 0.0)
    cs_vfov: float = math.pi / 2
    cs_aspectRatio: float = 1.0
    cs_imageWidth: int = 100
    cs_samplesPerPixel: int = 10
    cs_maxRecursionDepth: int = 10
    cs_background: Background = dataclasses.field(default_factory=lambda: constBackground(1.0))
    cs_defocusAngle: float = 0.0
    cs_focusDist: float = 10.0
    cs_redirectTargets: List[Tuple[float, tuple, tuple, tuple]] = dataclasses.field(default_factory=list)

    def replace(self, **kw) -> "CameraSettings":
        """Record update syntax `settings { cs_x = ... }`."""
        return dataclasses.replace(self, **kw)


def defaultCameraSettings(**overrides) -> CameraSettings:
    """Ray.hs:84-98."""
    return CameraSettings(**overrides)


def background_of(cs: CameraSettings) -> Background:
    bg = cs.cs_background
    if isinstance(bg, Background):
        return bg
    if callable(bg):
        from .errors import RtUnsupported
        raise RtUnsupported("cs_background is an arbitrary closure; only constBackground / lerpYBackground "
                            "(const, sky, grayFade) can be evaluated on the device")
    return constBackground(bg)


def image_height(cs: CameraSettings) -> int:
    """`round (fromIntegral cs_imageWidth / cs_aspectRatio)` with banker's rounding."""
    if not (cs.cs_aspectRatio > 0) or not math.isfinite(cs.cs_aspectRatio):
        from .errors import RtInvalid
        raise RtInvalid(f"aspect ratio {cs.cs_aspectRatio} must be positive and finite")
    return int(round(float(cs.cs_imageWidth) / cs.cs_aspectRatio))


@dataclasses.dataclass
class CameraBasis:
    width: int
    height: int
    center: tuple
    top_left: tuple
    pixel_u: tuple
    pixel_v: tuple
    disk_u: tuple
    disk_v: tuple


def camera_basis(cs: CameraSettings) -> CameraBasis:
    """Ray.hs:122-136, 153-155."""
    width = int(cs.cs_imageWidth)
    height = image_height(cs)
    if width <= 0 or height <= 0:
        from .errors import RtInvalid
        raise RtInvalid(f"image size {width}x{height} must be positive")
    center, look, up = V3(cs.cs_center), V3(cs.cs_lookAt), V3(cs.cs_up)
    vh = cs.cs_focusDist * math.tan(cs.cs_vfov / 2) * 2
    vw = vh * float(width) / float(height)
    w = normalize(sub(center, look))
    u = normalize(cross(up, w))
    v = cross(w, u)
    across = smul(vw, u)
    down = neg(smul(vh, v))
    top_left = sub(sub(sub(center, muls(w, cs.cs_focusDist)), divs(across, 2)), divs(down, 2))
    pixel_u = divs(across, float(width))
    pixel_v = divs(down, float(height))
    dr = cs.cs_focusDist * math.tan(cs.cs_defocusAngle / 2)
    return CameraBasis(width, height, center, top_left, pixel_u, pixel_v, muls(u, dr), muls(v, dr))
