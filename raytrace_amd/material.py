"""Graphics.Ray.Material and Graphics.Ray.Texture as reified descriptors.

Reference: src/Graphics/Ray/Material.hs:17-129, src/Graphics/Ray/Texture.hs:15-78.
The reference's materials and textures are closures; these constructors keep the names and
arguments and record WHICH closure was meant, so the device kernel can evaluate the same
formula with a `switch`.  `solidTexture` / `uvTexture` take arbitrary functions and cannot be
reified: they are accepted here but rejected (RtUnsupported) when a scene is flattened.
"""
from __future__ import annotations

from .core import V3

# material kinds (must match include/rt.h RT_MAT_*)
LIGHT, BLACK, LAMBERT, LOMMEL, MIRROR, METAL, DIELECTRIC, TRANSPARENT, ISOTROPIC, ANISOTROPIC = range(10)
MATERIAL_NAMES = ["lightSource", "pitchBlack", "lambertian", "lommelSeeliger", "mirror", "metal", "dielectric",
                  "transparent", "isotropic", "anisotropic"]

# texture kinds (include/rt.h RT_TEX_*)
TEX_CONSTANT, TEX_CHECKER, TEX_IMAGE, TEX_NOISE, TEX_MARBLE, TEX_CLOSURE = range(6)


def _color(c):
    return V3(c)


class Texture:
    __slots__ = ("kind", "c0", "c1", "nu", "nv", "params", "image", "fn")

    def __init__(self, kind, c0=(0.0, 0.0, 0.0), c1=(0.0, 0.0, 0.0), nu=0, nv=0, params=(), image=None, fn=None):
        self.kind = kind
        self.c0 = _color(c0)
        self.c1 = _color(c1)
        self.nu = int(nu)
        self.nv = int(nv)
        self.params = tuple(float(p) for p in params)
        self.image = image
        self.fn = fn

    def key(self):
        img = None if self.image is None else id(self.image)
        return (self.kind, self.c0, self.c1, self.nu, self.nv, self.params, img, id(self.fn) if self.fn else None)


def constantTexture(color) -> Texture:
    """Texture.hs:18-19."""
    return Texture(TEX_CONSTANT, color)


def checkerTexture(n_u: int, n_v: int, c0, c1) -> Texture:
    """Texture.hs:45-53."""
    return Texture(TEX_CHECKER, c0, c1, n_u, n_v)


def imageTexture(image) -> Texture:
    """Texture.hs:31-41 (an h x w x 3 linear-RGB array)."""
    return Texture(TEX_IMAGE, image=image)


def noiseTexture(k: int, freq: float, shift, color0, color1) -> Texture:
    """Texture.hs:56-67."""
    return Texture(TEX_NOISE, color0, color1, nu=k, params=(freq,) + tuple(V3(shift)))


def marbleTexture(direction, freq: float, shift) -> Texture:
    """Texture.hs:70-78."""
    return Texture(TEX_MARBLE, params=tuple(V3(direction)) + (freq,) + tuple(V3(shift)))


def solidTexture(fn) -> Texture:
    """Texture.hs:22-23 — an arbitrary closure: not reifiable for the device."""
    return Texture(TEX_CLOSURE, fn=fn)


def uvTexture(fn) -> Texture:
    """Texture.hs:26-27 — an arbitrary closure: not reifiable for the device."""
    return Texture(TEX_CLOSURE, fn=fn)


class Material:
    __slots__ = ("kind", "texture", "param")

    def __init__(self, kind, texture=None, param=0.0):
        self.kind = kind
        self.texture = texture if texture is not None else constantTexture(0.0)
        self.param = float(param)

    def __lshift__(self, geometry):
        """`material << geometry` ≡ the reference's `material <$ geometry`."""
        from .geometry import withMaterial
        return withMaterial(self, geometry)

    def key(self):
        return (self.kind, self.texture.key(), self.param)

    def __repr__(self):
        return f"{MATERIAL_NAMES[self.kind]}(param={self.param})"


def lightSource(tex: Texture) -> Material:
    """Material.hs:41-42."""
    return Material(LIGHT, tex)


pitchBlack = Material(BLACK)  # Material.hs:46-47


def lambertian(tex: Texture) -> Material:
    """Material.hs:51-53."""
    return Material(LAMBERT, tex)


def lommelSeeliger(tex: Texture) -> Material:
    """Material.hs:56-61."""
    return Material(LOMMEL, tex)


def mirror(tex: Texture) -> Material:
    """Material.hs:64-67."""
    return Material(MIRROR, tex)


def metal(fuzz: float, tex: Texture) -> Material:
    """Material.hs:72-78."""
    return Material(METAL, tex, fuzz)


def dielectric(ior: float) -> Material:
    """Material.hs:89-106."""
    return Material(DIELECTRIC, constantTexture(1.0), ior)


def transparent(tex: Texture) -> Material:
    """Material.hs:109-112."""
    return Material(TRANSPARENT, tex)


def isotropic(tex: Texture) -> Material:
    """Material.hs:116-118."""
    return Material(ISOTROPIC, tex)


def anisotropic(g: float, tex: Texture) -> Material:
    """Material.hs:124-129 (Henyey-Greenstein)."""
    return Material(ANISOTROPIC, tex, g)
