"""Graphics.Ray.Geometry as a deep embedding (reference: src/Graphics/Ray/Geometry.hs).

The reference's `Geometry m a` is a bounding box plus an opaque hit closure
(Geometry.hs:42), which cannot be shipped to a GPU.  Here every smart constructor keeps the
reference's NAME, ARGUMENTS and BOUNDING-BOX arithmetic but returns a descriptor node; the
tree of descriptors is what `raytrace_amd.scene` flattens into device buffers.  Hit
semantics live in the HIP kernel (raytrace_amd/csrc/rt_kernel.hip) and, for parity checking,
in the FP64 oracle (oracle/rt_oracle.c).

`mat <$ geom` (attach a material, outermost wins) is spelled `withMaterial(mat, geom)` or
`mat << geom`.
"""
from __future__ import annotations

import math
import re
from typing import List, Optional, Sequence, Tuple

from .core import (Box, Point3, Vec3, add, allCorners, boxHull, boxJoin, cross, fromCorners, longestDim,
                   midpoint, norm, padBox, shiftBox, sub)


class ObjParseError(ValueError):
    """`Left String` of parseObj / readObj (Geometry.hs:194-285)."""


class Geometry:
    """Base descriptor.  `bbox` follows the reference's `boundingBox` exactly."""

    is_random = False  # True for `Geometry (State StdGen)` (contains constantMedium)

    def boundingBox(self) -> Box:
        return self.bbox


def boundingBox(g: Geometry) -> Box:
    """Geometry.hs:54-55."""
    return g.bbox


class Sphere(Geometry):

    def __init__(self, center: Point3, radius: float):
        self.center = tuple(float(c) for c in center)
        self.radius = float(radius)
        diag = (self.radius, self.radius, self.radius)
        self.bbox = fromCorners(sub(self.center, diag), add(self.center, diag))


PARALLELOGRAM, TRIANGLE = 0, 1


class PlaneShape(Geometry):
    """planeShape q u v test getUV bbox (Geometry.hs:108-144) for the two reference tests."""


    def __init__(self, q, u, v, kind, bbox, uv0=(0.0, 0.0), uv1=(1.0, 0.0), uv2=(0.0, 1.0)):
        self.q = tuple(float(x) for x in q)
        self.u = tuple(float(x) for x in u)
        self.v = tuple(float(x) for x in v)
        self.kind = kind
        self.uv0 = tuple(float(x) for x in uv0)
        self.uv1 = tuple(float(x) for x in uv1)
        self.uv2 = tuple(float(x) for x in uv2)
        if norm(cross(self.u, self.v)) == 0:
            # the reference divides by |u x v| and would produce NaN normals (never hits)
            pass
        self.bbox = padBox(0.0001, bbox)


class Group(Geometry):

    def __init__(self, children: Sequence[Geometry]):
        self.children = list(children)
        self.bbox = boxJoin([c.bbox for c in self.children])
        self.is_random = any(c.is_random for c in self.children)


class BvhNode(Geometry):

    def __init__(self, left: Geometry, right: Geometry):
        self.left = left
        self.right = right
        self.bbox = boxJoin([left.bbox, right.bbox])
        self.is_random = left.is_random or right.is_random


class Transform(Geometry):

    def __init__(self, m, child: Geometry):
        self.m = tuple(tuple(float(x) for x in row) for row in m)
        self.m34 = self.m[:3]
        self.inv34 = inv44(self.m)[:3]
        self.child = child
        self.is_random = child.is_random
        self.bbox = boxHull([mul_point(self.m34, c) for c in allCorners(child.bbox)])


class Moving(Geometry):

    def __init__(self, v0: Vec3, v1: Vec3, child: Geometry):
        self.v0 = tuple(float(x) for x in v0)
        self.v1 = tuple(float(x) for x in v1)
        self.child = child
        self.is_random = child.is_random
        self.bbox = boxJoin([shiftBox(self.v0, child.bbox), shiftBox(self.v1, child.bbox)])


class ConstantMedium(Geometry):
    is_random = True

    def __init__(self, density: float, child: Geometry):
        if child.is_random:
            raise TypeError("constantMedium: the surface must be a pure geometry (Geometry Identity ())")
        self.density = float(density)
        self.child = child
        self.bbox = child.bbox


class WithMaterial(Geometry):

    def __init__(self, material, child: Geometry):
        self.material = material
        self.child = child
        self.is_random = child.is_random
        self.bbox = child.bbox


# ------------------------------------------------------------------ smart constructors

def sphere(center: Point3, radius: float) -> Geometry:
    """Geometry.hs:58-94."""
    return Sphere(center, radius)


def parallelogram(q: Point3, u: Vec3, v: Vec3) -> Geometry:
    """Geometry.hs:147-151."""
    q = tuple(float(x) for x in q)
    u = tuple(float(x) for x in u)
    v = tuple(float(x) for x in v)
    bbox = boxHull([q, add(q, u), add(q, v), add(add(q, u), v)])
    return PlaneShape(q, u, v, PARALLELOGRAM, bbox)


def triangle(a: Tuple[Point3, Tuple[float, float]], b, c) -> Geometry:
    """Geometry.hs:169-176; each argument is (corner, uv)."""
    (p0, uv0), (p1, uv1), (p2, uv2) = a, b, c
    p0 = tuple(float(x) for x in p0)
    p1 = tuple(float(x) for x in p1)
    p2 = tuple(float(x) for x in p2)
    s1 = sub(p1, p0)
    s2 = sub(p2, p0)
    return PlaneShape(p0, s1, s2, TRIANGLE, boxHull([p0, p1, p2]), uv0, uv1, uv2)


def cuboid(box: Box) -> Geometry:
    """Geometry.hs:154-166: a `group` of six parallelograms."""
    (xmin, xmax), (ymin, ymax), (zmin, zmax) = box
    dx = (xmax - xmin, 0.0, 0.0)
    dy = (0.0, ymax - ymin, 0.0)
    dz = (0.0, 0.0, zmax - zmin)
    ndx = (-dx[0], -0.0, -0.0)
    ndz = (-0.0, -0.0, -dz[2])
    return group([
        parallelogram((xmin, ymin, zmax), dx, dy),
        parallelogram((xmax, ymin, zmin), ndx, dy),
        parallelogram((xmin, ymin, zmin), dz, dy),
        parallelogram((xmax, ymin, zmax), ndz, dy),
        parallelogram((xmin, ymax, zmax), dx, ndz),
        parallelogram((xmin, ymin, zmin), dx, dz),
    ])


def group(obs: Sequence[Geometry]) -> Geometry:
    """Geometry.hs:335-347 (closest hit in list order; `group []` fails like foldl1')."""
    return Group(obs)


def bvhNode(left: Geometry, right: Geometry) -> Geometry:
    """Geometry.hs:351-363."""
    return BvhNode(left, right)


def bvhTree(obs: Sequence[Geometry]) -> Geometry:
    """Geometry.hs:368-377: median split on the longest axis of the joined boxes,
    stable `sortOn` of the bbox midpoint, left half = n `div` 2."""
    obs = list(obs)
    if not obs:
        raise ValueError("bvhTree: empty list")
    if len(obs) == 1:
        return obs[0]
    d = longestDim(boxJoin([o.bbox for o in obs]))
    obs2 = sorted(obs, key=lambda o: midpoint(o.bbox[d]))
    k = len(obs2) // 2
    return BvhNode(bvhTree(obs2[:k]), bvhTree(obs2[k:]))


def constantMedium(density: float, surface: Geometry) -> Geometry:
    """Geometry.hs:298-330."""
    return ConstantMedium(density, surface)


def pureGeometry(g: Geometry) -> Geometry:
    """Geometry.hs:50-51 (a type-level promotion; the identity on descriptors)."""
    return g


def transform(m, g: Geometry) -> Geometry:
    """Geometry.hs:382-391."""
    return Transform(m, g)


def moving(v0: Vec3, v1: Vec3, g: Geometry) -> Geometry:
    """Geometry.hs:449-456."""
    return Moving(v0, v1, g)


def withMaterial(material, g: Geometry) -> Geometry:
    """`material <$ g` (Functor instance, Geometry.hs:44-47)."""
    return WithMaterial(material, g)


# ------------------------------------------------------------------ matrices (M44 Double)

class M44(tuple):
    """A 4x4 row-major matrix; `a @ b` is linear's `a !*! b`."""

    def __new__(cls, rows):
        return super().__new__(cls, tuple(tuple(float(x) for x in r) for r in rows))

    def __matmul__(self, other):
        return M44(mmul(self, other))


def mmul(f, g):
    """linear's (!*!): row i = foldl' (^+^) zero (liftI2 (*^) f_i g)."""
    out = []
    for fi in f:
        acc = [0.0, 0.0, 0.0, 0.0]
        for k in range(4):
            for c in range(4):
                acc[c] = acc[c] + fi[k] * g[k][c]
        out.append(tuple(acc))
    return tuple(out)


def translate(v: Vec3) -> M44:
    x, y, z = v
    return M44(((1, 0, 0, x), (0, 1, 0, y), (0, 0, 1, z), (0, 0, 0, 1)))


def rotateX(angle: float) -> M44:
    c, s = math.cos(angle), math.sin(angle)
    return M44(((1, 0, 0, 0), (0, c, -s, 0), (0, s, c, 0), (0, 0, 0, 1)))


def rotateY(angle: float) -> M44:
    c, s = math.cos(angle), math.sin(angle)
    return M44(((c, 0, s, 0), (0, 1, 0, 0), (-s, 0, c, 0), (0, 0, 0, 1)))


def rotateZ(angle: float) -> M44:
    c, s = math.cos(angle), math.sin(angle)
    return M44(((c, -s, 0, 0), (s, c, 0, 0), (0, 0, 1, 0), (0, 0, 0, 1)))


def scale(a: float) -> M44:
    return M44(((a, 0, 0, 0), (0, a, 0, 0), (0, 0, a, 0), (0, 0, 0, 1)))


def inv44(m):
    """linear's `inv44` (cofactor expansion in the library's term order)."""
    (i00, i01, i02, i03), (i10, i11, i12, i13), (i20, i21, i22, i23), (i30, i31, i32, i33) = m
    s0 = i00 * i11 - i10 * i01
    s1 = i00 * i12 - i10 * i02
    s2 = i00 * i13 - i10 * i03
    s3 = i01 * i12 - i11 * i02
    s4 = i01 * i13 - i11 * i03
    s5 = i02 * i13 - i12 * i03
    c5 = i22 * i33 - i32 * i23
    c4 = i21 * i33 - i31 * i23
    c3 = i21 * i32 - i31 * i22
    c2 = i20 * i33 - i30 * i23
    c1 = i20 * i32 - i30 * i22
    c0 = i20 * i31 - i30 * i21
    det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0
    inv_det = 1 / det
    rows = (
        (i11 * c5 - i12 * c4 + i13 * c3, -(i01 * c5) + i02 * c4 - i03 * c3,
         i31 * s5 - i32 * s4 + i33 * s3, -(i21 * s5) + i22 * s4 - i23 * s3),
        (-(i10 * c5) + i12 * c2 - i13 * c1, i00 * c5 - i02 * c2 + i03 * c1,
         -(i30 * s5) + i32 * s2 - i33 * s1, i20 * s5 - i22 * s2 + i23 * s1),
        (i10 * c4 - i11 * c2 + i13 * c0, -(i00 * c4) + i01 * c2 - i03 * c0,
         i30 * s4 - i31 * s2 + i33 * s0, -(i20 * s4) + i21 * s2 - i23 * s0),
        (-(i10 * c3) + i11 * c1 - i12 * c0, i00 * c3 - i01 * c1 + i02 * c0,
         -(i30 * s3) + i31 * s1 - i32 * s0, i20 * s3 - i21 * s1 + i22 * s0),
    )
    return tuple(tuple(inv_det * x for x in r) for r in rows)


def mul_point(m34, p):
    """(m34 !* V4.point p): each row is the V4 dot ((a*x + b*y) + c*z) + d*1."""
    return tuple(r[0] * p[0] + r[1] * p[1] + r[2] * p[2] + r[3] * 1.0 for r in m34[:3])


def mul_vector(m34, v):
    return tuple(r[0] * v[0] + r[1] * v[1] + r[2] * v[2] + r[3] * 0.0 for r in m34[:3])


# ------------------------------------------------------------------ meshes

class Mesh:
    """Geometry.hs:179-184: vertex positions, texture coordinates, triangles of
    ((vertex index, Maybe uv index) x 3)."""


    def __init__(self, vertices, uvs, faces):
        self.vertices = [tuple(float(x) for x in v) for v in vertices]
        self.uvs = [tuple(float(x) for x in t) for t in uvs]
        self.faces = [tuple((int(i), None if j is None else int(j)) for i, j in f) for f in faces]

    def __repr__(self):
        return f"Mesh({len(self.vertices)} vertices, {len(self.uvs)} uvs, {len(self.faces)} triangles)"


def transformVertices(m, mesh: Mesh) -> Mesh:
    """Geometry.hs:187-190."""
    m34 = tuple(tuple(float(x) for x in r) for r in m)[:3]
    return Mesh([mul_point(m34, v) for v in mesh.vertices], mesh.uvs, mesh.faces)


# Haskell `readMaybe :: String -> Maybe Double` accepts an optional minus sign, digits, an
# optional fraction with digits on both sides, an optional exponent (and "Infinity"/"NaN").
_HS_DOUBLE = re.compile(r"^-?(\d+(\.\d+)?([eE][+-]?\d+)?|Infinity|NaN)$")


def _read_double(s: str) -> Optional[float]:
    if not _HS_DOUBLE.match(s):
        return None
    if s.endswith("Infinity"):
        return -math.inf if s.startswith("-") else math.inf
    if s.endswith("NaN"):
        return math.nan
    return float(s)


def _extract_nat(s: str):
    m = re.match(r"\d*", s)
    ds = m.group(0)
    if not ds:
        raise ObjParseError("expected number")
    return int(ds), s[len(ds):]


def _extract_int(s: str):
    if s.startswith("-"):
        i, rest = _extract_nat(s[1:])
        return -i, rest
    return _extract_nat(s)


def _process_ix(length: int, i: int) -> int:
    if 1 <= i <= length:
        return i - 1
    if -length <= i <= -1:
        return i + length
    raise ObjParseError("index out of bounds: " + str(i))


def _get_indices(num_vs: int, num_vts: int, s: str):
    i, rest = _extract_int(s)
    i2 = _process_ix(num_vs, i)
    if rest == "":
        return (i2, None)
    if rest.startswith("//"):
        return (i2, None)
    if rest.startswith("/"):
        j, _ = _extract_int(rest[1:])
        return (i2, _process_ix(num_vts, j))
    raise ObjParseError("unexpected character '" + rest[0] + "'")


def parseObj(text: str) -> Mesh:
    """Geometry.hs:207-285.  Raises ObjParseError with the reference's message on `Left`."""
    lines = [ln.split("#", 1)[0] for ln in text.split("\n")]
    if text.endswith("\n"):
        lines = lines[:-1]  # Haskell `lines` drops the empty tail
    vls, vtls, fls = [], [], []
    for k, line in enumerate(lines, start=1):
        if line.startswith("v "):
            vls.append((k, line[2:]))
        elif line.startswith("vt "):
            vtls.append((k, line[3:]))
        elif line.startswith("f "):
            fls.append((k, line[2:]))
    vs = []
    for k, line in vls:
        w = line.split()
        vals = [_read_double(x) for x in w[:3]]
        if len(w) < 3 or any(v is None for v in vals):
            raise ObjParseError(f"line {k}: invalid 'v' statement")
        vs.append(tuple(vals))
    vts = []
    for k, line in vtls:
        w = line.split()
        if len(w) == 1 and _read_double(w[0]) is not None:
            vts.append((_read_double(w[0]), 0.0))
            continue
        if len(w) >= 2 and _read_double(w[0]) is not None and _read_double(w[1]) is not None:
            vts.append((_read_double(w[0]), _read_double(w[1])))
            continue
        raise ObjParseError(f"line {k}: invalid 'vt' statement")
    faces = []
    for k, line in fls:
        try:
            idx = [_get_indices(len(vs), len(vts), w) for w in line.split()]
        except ObjParseError as e:
            raise ObjParseError(f"line {k}: {e}") from None
        if len(idx) < 3:
            raise ObjParseError(f"line {k}: invalid 'f' statement (fewer than 3 vertices)")
        first, rest = idx[0], idx[1:]
        for a, b in zip(rest, rest[1:]):
            faces.append((first, a, b))
    return Mesh(vs, vts, faces)


def readObj(path: str) -> Mesh:
    """Geometry.hs:194-195 (the error message is prefixed with the path)."""
    with open(path, "r") as f:
        text = f.read()
    try:
        return parseObj(text)
    except ObjParseError as e:
        raise ObjParseError(f"{path}, {e}") from None


def triangleMesh(mesh: Mesh) -> Geometry:
    """Geometry.hs:288-294: a bvhTree of triangles; missing uvs default to (0,0),(1,0),(0,1)."""
    tris = []
    for (i0, j0), (i1, j1), (i2, j2) in mesh.faces:
        uv0 = mesh.uvs[j0] if j0 is not None else (0.0, 0.0)
        uv1 = mesh.uvs[j1] if j1 is not None else (1.0, 0.0)
        uv2 = mesh.uvs[j2] if j2 is not None else (0.0, 1.0)
        tris.append(triangle((mesh.vertices[i0], uv0), (mesh.vertices[i1], uv1), (mesh.vertices[i2], uv2)))
    return bvhTree(tris)


def children_of(g: Geometry) -> List[Geometry]:
    if isinstance(g, Group):
        return g.children
    if isinstance(g, BvhNode):
        return [g.left, g.right]
    if isinstance(g, (Transform, Moving, ConstantMedium, WithMaterial)):
        return [g.child]
    return []
