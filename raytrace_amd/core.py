"""Core vocabulary of Graphics.Ray.Core (reference: src/Graphics/Ray/Core.hs).

Host-side values only: vectors are plain 3-tuples of Python floats (IEEE binary64, like
Haskell's `Double`), boxes are 3-tuples of (lo, hi) intervals.  Every helper follows the
reference's evaluation order so that scene constants computed here (bounding boxes,
transform matrices, camera basis) are bit-identical to the reference's.
"""
from __future__ import annotations

import math
from typing import Iterable, Sequence, Tuple

Vec3 = Tuple[float, float, float]
Point3 = Vec3
Color = Vec3
Interval = Tuple[float, float]
Box = Tuple[Interval, Interval, Interval]

infinity = math.inf  # Core.hs:21-22
pi = math.pi         # Haskell's `pi :: Double` = 3.141592653589793

X, Y, Z = 0, 1, 2    # Core.hs:32-33 `data Dim = X | Y | Z`


def V3(x, y=None, z=None) -> Vec3:
    """`V3 x y z`; `V3(c)` is the Num literal `fromInteger c` broadcast (e.g. `constantTexture 1`)."""
    if y is None and z is None:
        if isinstance(x, (tuple, list)):
            return (float(x[0]), float(x[1]), float(x[2]))
        return (float(x), float(x), float(x))
    return (float(x), float(y), float(z))


def degrees(x: float) -> float:
    """Core.hs:25-26 `degrees x = x * pi / 180`."""
    return x * math.pi / 180


def component(d: int, v: Vec3) -> float:
    return v[d]


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def neg(a):
    return (-a[0], -a[1], -a[2])


def smul(s, a):
    """`s *^ v`."""
    return (s * a[0], s * a[1], s * a[2])


def muls(a, s):
    """`v ^* s`."""
    return (a[0] * s, a[1] * s, a[2] * s)


def divs(a, s):
    """`v ^/ s` (component-wise division, as linear's `fmap (/ s)`)."""
    return (a[0] / s, a[1] / s, a[2] / s)


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def quadrance(a):
    return dot(a, a)


def norm(a):
    return math.sqrt(quadrance(a))


def normalize(v):
    """linear's `normalize`: unchanged when the quadrance is nearZero or nearZero (1 - quadrance)."""
    l = quadrance(v)
    if abs(l) <= 1e-12 or abs(1 - l) <= 1e-12:
        return v
    return divs(v, math.sqrt(l))


def hmax(x, y):
    """Haskell's default `max` for Double (`if x <= y then y else x`)."""
    return y if x <= y else x


def hmin(x, y):
    return x if x <= y else y


def reflect(normal: Vec3, v: Vec3) -> Vec3:
    """Core.hs:49-51."""
    return sub(v, smul(2 * dot(normal, v), normal))


# ------------------------------------------------------------------ intervals & boxes

def inInterval(ival: Interval, t: float) -> bool:
    """Core.hs:83-84 (open interval)."""
    return ival[0] < t < ival[1]


def midpoint(ival: Interval) -> float:
    return (ival[0] + ival[1]) / 2


def padInterval(p: float, ival: Interval) -> Interval:
    return (ival[0] - p, ival[1] + p)


def fromCorners(a: Point3, b: Point3) -> Box:
    """Core.hs:112-113."""
    return tuple((x, y) if x < y else (y, x) for x, y in zip(a, b))  # type: ignore[return-value]


def _join2(b1: Box, b2: Box) -> Box:
    return tuple((hmin(i1[0], i2[0]), hmax(i1[1], i2[1])) for i1, i2 in zip(b1, b2))  # type: ignore[return-value]


def boxJoin(boxes: Sequence[Box]) -> Box:
    """Core.hs:115-117 `foldl1'` of the component-wise hull; fails on [] like the reference."""
    boxes = list(boxes)
    if not boxes:
        raise ValueError("boxJoin: empty list (foldl1')")
    acc = boxes[0]
    for b in boxes[1:]:
        acc = _join2(acc, b)
    return acc


def boxHull(pts: Iterable[Point3]) -> Box:
    """Core.hs:120-125."""
    pts = list(pts)
    if not pts:
        raise ValueError("boxHull: empty list")
    out = []
    for d in range(3):
        vals = [p[d] for p in pts]
        lo = vals[0]
        hi = vals[0]
        for x in vals[1:]:
            lo = hmin(lo, x)
            hi = hmax(hi, x)
        out.append((lo, hi))
    return tuple(out)  # type: ignore[return-value]


def allCorners(box: Box):
    """Core.hs:128-132."""
    (a0, a1), (b0, b1), (c0, c1) = box
    return [(x, y, z) for x in (a0, a1) for y in (b0, b1) for z in (c0, c1)]


def padBox(p: float, box: Box) -> Box:
    return tuple(padInterval(p, i) for i in box)  # type: ignore[return-value]


def shiftBox(v: Vec3, box: Box) -> Box:
    return tuple((i[0] + x, i[1] + x) for x, i in zip(v, box))  # type: ignore[return-value]


def longestDim(box: Box) -> int:
    """Core.hs:143-144 with argMax (Core.hs:37-40)."""
    x, y, z = (i[1] - i[0] for i in box)
    if x > y:
        return X if x > z else Z
    return Y if y > z else Z


# ------------------------------------------------------------------ StdGen (splitmix)

_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = ((z ^ (z >> 33)) * 0xFF51AFD7ED558CCD) & _M64
    z = ((z ^ (z >> 33)) * 0xC4CEB9FE1A85EC53) & _M64
    return z ^ (z >> 33)


def _mix64v13(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _mix_gamma(z: int) -> int:
    z1 = _mix64v13(z) | 1
    n = bin(z1 ^ (z1 >> 1)).count("1")
    return z1 if n >= 24 else z1 ^ 0xAAAAAAAAAAAAAAAA


class StdGen:
    """`StdGen` = splitmix `SMGen seed gamma` (random >= 1.2).

    Only used to carry `raytrace`'s seed argument.  The device path keys its counter-based
    Philox stream with `key()`, a 64-bit digest of (seed, gamma); the oracle's splitmix
    mode consumes (seed, gamma) exactly like the reference.
    """

    __slots__ = ("seed", "gamma")

    def __init__(self, seed: int, gamma: int):
        self.seed = seed & _M64
        self.gamma = gamma & _M64

    def next_word64(self):
        s = (self.seed + self.gamma) & _M64
        return _mix64(s), StdGen(s, self.gamma)

    def split(self):
        """splitSMGen."""
        sp = (self.seed + self.gamma) & _M64
        spp = (sp + self.gamma) & _M64
        return StdGen(spp, self.gamma), StdGen(_mix64(sp), _mix_gamma(spp))

    def uniform01(self):
        w, g = self.next_word64()
        return float(w) / 18446744073709551615.0, g

    def random(self):
        """`random :: Double` (random-1.2/1.3: 1 - uniformDouble01M)."""
        x, g = self.uniform01()
        return 1 - x, g

    def randomR(self, lo: float, hi: float):
        if lo == hi:
            return lo, self
        x, g = self.uniform01()
        return x * lo + (1 - x) * hi, g

    def key(self) -> int:
        """64-bit Philox key for the device stream (a splitmix digest of the generator)."""
        return _mix64((self.seed ^ _mix64(self.gamma)) & _M64)

    def __repr__(self):
        return f"StdGen(seed=0x{self.seed:016x}, gamma=0x{self.gamma:016x})"

    def __eq__(self, other):
        return isinstance(other, StdGen) and (self.seed, self.gamma) == (other.seed, other.gamma)

    def __hash__(self):
        return hash((self.seed, self.gamma))


def mkStdGen(n: int) -> StdGen:
    """`mkStdGen n = StdGen (mkSMGen (fromIntegral n))`."""
    s = n & _M64
    return StdGen(_mix64(s), _mix_gamma((s + 0x9E3779B97F4A7C15) & _M64))
