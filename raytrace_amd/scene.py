"""Scene flattening: descriptor tree -> the C-ABI's SoA primitive arrays (include/rt.h).

The reference evaluates a tree of closures (group fold, bvhNode, transform, moving,
constantMedium, `<$`; Geometry.hs:298-456).  Its result for a ray is the CLOSEST hit in the
open interval, ties going to the earliest leaf in depth-first order (group folds keep the
earlier hit on equal t, bvhNode's right child must be strictly closer).  That result does not
depend on the tree's shape, so `flatten` bakes the tree into a flat primitive list — rigid
transforms and motion applied to the leaves, `<$` resolved (outermost wins), media lifted to a
top-level list with their boundary primitives in their own sets — and records each leaf's
depth-first `order` for tie-breaking.  The library then builds its own BVH over the list.

`serialize_tree` keeps the tree exactly as written; it feeds the FP64 oracle (tests only),
which walks the reference's own structure.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import geometry as G
from . import material as M
from .errors import RtInvalid, RtUnsupported

# ------------------------------------------------------------------ C-ABI record layouts (include/rt.h)
PRIM_SPHERE, PRIM_PARALLELOGRAM, PRIM_TRIANGLE = 0, 1, 2

PRIM_DTYPE = np.dtype([
    ("kind", "<i4"), ("material", "<i4"), ("set", "<i4"), ("motion", "<i4"),
    ("gid", "<i4"), ("order", "<i4"), ("uvframe", "<i4"), ("pad", "<i4"),
    ("p", "<f8", (9,)), ("uv", "<f8", (6,)),
], align=True)
MEDIUM_DTYPE = np.dtype([("density", "<f8"), ("material", "<i4"), ("order", "<i4")], align=True)
MATERIAL_DTYPE = np.dtype([("kind", "<i4"), ("texture", "<i4"), ("param", "<f8")], align=True)
TEXTURE_DTYPE = np.dtype([
    ("kind", "<i4"), ("nu", "<i4"), ("nv", "<i4"), ("image", "<i4"),
    ("c0", "<f8", (3,)), ("c1", "<f8", (3,)), ("params", "<f8", (8,)),
], align=True)
MOTION_DTYPE = np.dtype([("v0", "<f8", (3,)), ("v1", "<f8", (3,))], align=True)
INSTANCE_DTYPE = np.dtype([("blas", "<i4"), ("material", "<i4"), ("order", "<i4"), ("pad", "<i4"),
                           ("m", "<f8", (12,))], align=True)
INSTANCE_MIN_LEAVES = 64  # a rigid `transform` over at least this many leaves is instanced, not baked


def RT_SET_BLAS(b: int) -> int:
    return -1 - b
UVFRAME_DTYPE = np.dtype([("r", "<f8", (9,))], align=True)

RIGID_TOL = 1e-9


def _is_rigid(m34) -> bool:
    r = np.array([row[:3] for row in m34], dtype=np.float64)
    return bool(np.allclose(r.T @ r, np.eye(3), atol=RIGID_TOL, rtol=0))


def _compose(outer, inner):
    """outer . inner for 3x4 affine matrices (host precision; only used for baking)."""
    a = np.vstack([np.array(outer, dtype=np.float64), [0, 0, 0, 1]])
    b = np.vstack([np.array(inner, dtype=np.float64), [0, 0, 0, 1]])
    return (a @ b)[:3]


class _Tables:
    def __init__(self):
        self.materials: List[M.Material] = []
        self.mat_index: Dict[tuple, int] = {}
        self.textures: List[M.Texture] = []
        self.tex_index: Dict[tuple, int] = {}

    def texture(self, t: M.Texture) -> int:
        k = t.key()
        if k not in self.tex_index:
            self.tex_index[k] = len(self.textures)
            self.textures.append(t)
        return self.tex_index[k]

    def material(self, m: M.Material) -> int:
        k = m.key()
        if k not in self.mat_index:
            self.texture(m.texture)
            self.mat_index[k] = len(self.materials)
            self.materials.append(m)
        return self.mat_index[k]

    def material_array(self):
        a = np.zeros(len(self.materials), MATERIAL_DTYPE)
        for i, m in enumerate(self.materials):
            a[i]["kind"] = m.kind
            a[i]["texture"] = self.tex_index[m.texture.key()]
            a[i]["param"] = m.param
        return a

    def texture_array(self):
        """(rt_texture records, texels float32 (n, 3), rt_perlin record or None)."""
        a = np.zeros(len(self.textures), TEXTURE_DTYPE)
        texels = []
        n_texels = 0
        need_perlin = False
        for i, t in enumerate(self.textures):
            if t.kind == M.TEX_CLOSURE:
                raise RtUnsupported("solidTexture / uvTexture closures are not reifiable for the device "
                                    "(constant, checker, image, noise and marble textures are)")
            a[i]["kind"] = t.kind
            a[i]["nu"] = t.nu
            a[i]["nv"] = t.nv
            a[i]["image"] = -1
            a[i]["c0"] = t.c0
            a[i]["c1"] = t.c1
            p = list(t.params)[:8]
            a[i]["params"][: len(p)] = p
            if t.kind == M.TEX_IMAGE:
                img = np.ascontiguousarray(t.image, dtype=np.float32).reshape(t.image.shape[0], t.image.shape[1], 3)
                h, w = img.shape[:2]
                a[i]["nu"], a[i]["nv"], a[i]["image"] = w, h, n_texels
                texels.append(img.reshape(-1, 3))
                n_texels += h * w
            elif t.kind in (M.TEX_NOISE, M.TEX_MARBLE):
                need_perlin = True
        tex = np.concatenate(texels) if texels else np.zeros((0, 3), np.float32)
        perlin = None
        if need_perlin:
            from .perlin import perlin_record
            perlin = perlin_record()
        return a, tex, perlin


class FlatScene:
    """Flattened scene: numpy record arrays with the exact layout of include/rt.h."""

    def __init__(self, prims, media, materials, textures, motions, uvframes, n_surface, texels=None, perlin=None,
                 instances=None):
        self.instances = instances if instances is not None else np.zeros(0, INSTANCE_DTYPE)
        self.prims = prims
        self.media = media
        self.materials = materials
        self.textures = textures
        self.texels = texels if texels is not None else np.zeros((0, 3), np.float32)
        self.perlin = perlin
        self.motions = motions
        self.uvframes = uvframes
        self.n_surface = n_surface

    def __repr__(self):
        return (f"FlatScene({len(self.prims)} prims, {len(self.media)} media, {len(self.materials)} materials, "
                f"{len(self.textures)} textures, {len(self.instances)} instances)")


def _leaf_count(g, memo) -> int:
    k = id(g)
    if k not in memo:
        if isinstance(g, (G.Sphere, G.PlaneShape)):
            memo[k] = 1
        else:
            memo[k] = sum(_leaf_count(c, memo) for c in G.children_of(g))
    return memo[k]


def _bakes_only(g) -> bool:
    """Subtrees with `moving` or media stay baked (an instance has one rigid placement)."""
    if isinstance(g, (G.Moving, G.ConstantMedium)):
        return True
    return any(_bakes_only(c) for c in G.children_of(g))


def flatten(world: G.Geometry, instance_min: int = INSTANCE_MIN_LEAVES) -> FlatScene:
    """Bake the descriptor tree into the C-ABI's flat primitive lists (see module doc).

    Two-level instancing: a rigid `transform` over at least `instance_min` leaves (no `moving`
    or media inside, not itself inside a `moving`) becomes an rt_instance of an object whose
    leaves are flattened ONCE in object space (set RT_SET_BLAS(b)); the same child object under
    several transforms shares one object.  The device traces it under the instance's transform
    (exact up to rounding: the images equal the baked ones within 1e-12 in binary64).
    instance_min = 0 bakes every transform."""
    tabs = _Tables()
    instances: List[tuple] = []
    blas_of: Dict[int, Tuple[int, int, bool]] = {}  # id(child) -> (blas, leaves, every leaf has a material)
    leaf_memo: Dict[int, int] = {}
    prims: List[tuple] = []
    media: List[tuple] = []
    motions: List[tuple] = []
    uvframes: List[tuple] = []
    uvframe_index: Dict[tuple, int] = {}
    gids: Dict[tuple, int] = {}
    order = [0]

    def uvframe_of(m34) -> int:
        if m34 is None:
            return -1
        rt = tuple(float(m34[c][r]) for r in range(3) for c in range(3))  # R^T, row-major
        if rt not in uvframe_index:
            uvframe_index[rt] = len(uvframes)
            uvframes.append(rt)
        return uvframe_index[rt]

    def motion_of(mv) -> int:
        if mv is None:
            return -1
        motions.append(mv)
        return len(motions) - 1

    def gid_of(leaf, m34, mv, set_id) -> int:
        # an instanced object's leaves live in their own gid space (a ray leaving one skips only
        # that leaf of that instance; rt_build / rt_trace compare the instance too)
        key = (id(leaf), None if m34 is None else tuple(map(tuple, np.asarray(m34).tolist())), mv,
               set_id if set_id < 0 else 0)
        if key not in gids:
            gids[key] = len(gids)
        return gids[key]

    def walk(node, m34, mv, mat: Optional[int], set_id: int, leaf_out: list):
        if isinstance(node, G.WithMaterial):
            if set_id <= 0 and mat is None:
                mat = tabs.material(node.material)
            walk(node.child, m34, mv, mat, set_id, leaf_out)
        elif isinstance(node, G.Group):
            for c in node.children:
                walk(c, m34, mv, mat, set_id, leaf_out)
        elif isinstance(node, G.BvhNode):
            walk(node.left, m34, mv, mat, set_id, leaf_out)
            walk(node.right, m34, mv, mat, set_id, leaf_out)
        elif isinstance(node, G.Transform):
            if not _is_rigid(node.m34):
                raise RtUnsupported("transform with a non-Euclidean matrix (the reference documents Euclidean "
                                    "transforms only, Geometry.hs:379-381); use transformVertices for meshes")
            m2 = node.m34 if m34 is None else _compose(m34, node.m34)
            if (set_id == 0 and mv is None and instance_min > 0
                    and _leaf_count(node.child, leaf_memo) >= instance_min and not _bakes_only(node.child)):
                key = id(node.child)
                if key not in blas_of:
                    b = len(blas_of)
                    saved = order[0]
                    order[0] = 0
                    blas_leaves: list = []
                    walk(node.child, None, None, None, RT_SET_BLAS(b), blas_leaves)
                    n = order[0]
                    order[0] = saved
                    leaf_out.extend(blas_leaves)
                    blas_of[key] = (b, n, all(rec[1] is not None for rec in blas_leaves))
                b, n, own = blas_of[key]
                if mat is None and not own:
                    raise RtInvalid("a surface has no material (apply one with withMaterial / `<<`)")
                instances.append((b, -1 if mat is None else mat, order[0], m2))
                order[0] += n
                return
            walk(node.child, m2, mv, mat, set_id, leaf_out)
        elif isinstance(node, G.Moving):
            v0, v1 = node.v0, node.v1
            if m34 is not None:
                r = np.array(m34, dtype=np.float64)[:, :3]
                v0 = tuple((r @ np.array(v0)).tolist())
                v1 = tuple((r @ np.array(v1)).tolist())
            if mv is not None:
                v0 = tuple(a + b for a, b in zip(v0, mv[0]))
                v1 = tuple(a + b for a, b in zip(v1, mv[1]))
            walk(node.child, m34, (tuple(v0), tuple(v1)), mat, set_id, leaf_out)
        elif isinstance(node, G.ConstantMedium):
            if set_id != 0:
                raise RtInvalid("constantMedium inside a medium boundary")
            k = len(media)
            media.append(None)
            my_order = order[0]
            order[0] += 1
            media[k] = (node.density, mat, my_order)
            walk(node.child, m34, mv, None, k + 1, leaf_out)
        elif isinstance(node, G.Sphere):
            c = node.center
            if m34 is not None:
                c = G.mul_point(m34, c)
            rec = (M_SPHERE_KIND, mat, set_id, motion_of(mv), gid_of(node, m34, mv, set_id), order[0],
                   uvframe_of(m34), (c[0], c[1], c[2], node.radius, 0, 0, 0, 0, 0), (0,) * 6)
            order[0] += 1
            leaf_out.append(rec)
        elif isinstance(node, G.PlaneShape):
            q, u, v = node.q, node.u, node.v
            uv0, uv1, uv2 = node.uv0, node.uv1, node.uv2
            if node.kind == G.PARALLELOGRAM:
                uv0, uv1, uv2 = (0.0, 0.0), (1.0, 0.0), (0.0, 1.0)
            if m34 is not None:
                q = G.mul_point(m34, q)
                u = G.mul_vector(m34, u)
                v = G.mul_vector(m34, v)
                if np.linalg.det(np.array(m34, dtype=np.float64)[:, :3]) < 0:
                    # keep the reference's object-space front side under a reflection
                    u, v = v, u
                    uv1, uv2 = uv2, uv1
            kind = PRIM_PARALLELOGRAM if node.kind == G.PARALLELOGRAM else PRIM_TRIANGLE
            rec = (kind, mat, set_id, motion_of(mv), gid_of(node, m34, mv, set_id), order[0], -1,
                   tuple(q) + tuple(u) + tuple(v), tuple(uv0) + tuple(uv1) + tuple(uv2))
            order[0] += 1
            leaf_out.append(rec)
        else:
            raise RtUnsupported(f"geometry node {type(node).__name__} cannot be reified for the device")

    leaves: list = []
    walk(world, None, None, None, 0, leaves)
    # surface prims must carry a material (the reference's world has type Geometry m Material)
    for rec in leaves:
        if rec[2] == 0 and rec[1] is None:
            raise RtInvalid("a surface has no material (apply one with withMaterial / `<<`)")
    inst = np.zeros(len(instances), INSTANCE_DTYPE)
    for k, (b, m, od, m34) in enumerate(instances):
        inst[k]["blas"] = b
        inst[k]["material"] = m
        inst[k]["order"] = od
        inst[k]["m"] = np.asarray(m34, dtype=np.float64).reshape(-1)
    for k, (dens, mat, _) in enumerate(media):
        if mat is None:
            raise RtInvalid("a constantMedium has no material")
        if not (dens > 0):
            raise RtInvalid("constantMedium density must be positive")
        if not any(rec[2] == k + 1 for rec in leaves):
            raise RtInvalid("constantMedium with an empty boundary")
    prims = np.zeros(len(leaves), PRIM_DTYPE)
    for i, rec in enumerate(leaves):
        kind, mat, set_id, motion, gid, od, uvf, p, uv = rec
        prims[i]["kind"] = kind
        prims[i]["material"] = -1 if mat is None else mat
        prims[i]["set"] = set_id
        prims[i]["motion"] = motion
        prims[i]["gid"] = gid
        prims[i]["order"] = od
        prims[i]["uvframe"] = uvf
        prims[i]["p"] = p
        prims[i]["uv"] = uv
    med = np.zeros(len(media), MEDIUM_DTYPE)
    for k, (dens, mat, od) in enumerate(media):
        med[k]["density"] = dens
        med[k]["material"] = mat
        med[k]["order"] = od
    mot = np.zeros(len(motions), MOTION_DTYPE)
    for k, (v0, v1) in enumerate(motions):
        mot[k]["v0"] = v0
        mot[k]["v1"] = v1
    uvf = np.zeros(len(uvframes), UVFRAME_DTYPE)
    for k, r in enumerate(uvframes):
        uvf[k]["r"] = r
    n_surface = int(np.sum(prims["set"] == 0)) if len(prims) else 0
    tex, texels, perlin = tabs.texture_array()
    return FlatScene(prims, med, tabs.material_array(), tex, mot, uvf, n_surface, texels, perlin, inst)


M_SPHERE_KIND = PRIM_SPHERE

# ------------------------------------------------------------------ tree serialization (oracle input)
N_SPHERE, N_PLANE, N_GROUP, N_BVH, N_TRANSFORM, N_MOVING, N_MEDIUM, N_MATERIAL = range(8)
NI, ND = 4, 30


class SerializedTree:
    def __init__(self, node_i, node_d, children, root, materials, textures, n_media, texels=None, perlin=None):
        self.texels = texels if texels is not None else np.zeros((0, 3), np.float32)
        self.perlin = perlin
        self.node_i = node_i
        self.node_d = node_d
        self.children = children
        self.root = root
        self.materials = materials
        self.textures = textures
        self.n_media = n_media


def serialize_tree(world: G.Geometry) -> SerializedTree:
    """The reference's geometry tree as flat node arrays (layout documented in oracle/rt_oracle.c)."""
    tabs = _Tables()
    node_i: List[List[int]] = []
    node_d: List[List[float]] = []
    children: List[int] = []
    memo: Dict[int, int] = {}
    media_count = [0]
    contains_medium: Dict[int, bool] = {}

    def has_medium(n) -> bool:
        k = id(n)
        if k not in contains_medium:
            contains_medium[k] = isinstance(n, G.ConstantMedium) or any(has_medium(c) for c in G.children_of(n))
        return contains_medium[k]

    def emit(kind, ints, box, params) -> int:
        idx = len(node_i)
        ni = [kind] + list(ints) + [0] * (NI - 1 - len(ints))
        nd = [0.0] * ND
        if box is not None:
            nd[0:6] = [box[0][0], box[0][1], box[1][0], box[1][1], box[2][0], box[2][1]]
        nd[6:6 + len(params)] = params
        node_i.append(ni)
        node_d.append(nd)
        return idx

    def ser(n) -> int:
        # shared pure subtrees are emitted once; media get one node per occurrence (their own draws)
        if not has_medium(n) and id(n) in memo:
            return memo[id(n)]
        if isinstance(n, G.Sphere):
            idx = emit(N_SPHERE, [], n.bbox, list(n.center) + [n.radius])
        elif isinstance(n, G.PlaneShape):
            idx = emit(N_PLANE, [n.kind], n.bbox, list(n.q) + list(n.u) + list(n.v) + list(n.uv0) + list(n.uv1)
                       + list(n.uv2))
        elif isinstance(n, G.Group):
            kids = [ser(c) for c in n.children]
            first = len(children)
            children.extend(kids)
            idx = emit(N_GROUP, [first, len(kids)], n.bbox, [])
        elif isinstance(n, G.BvhNode):
            l, r = ser(n.left), ser(n.right)
            idx = emit(N_BVH, [l, r], n.bbox, [])
        elif isinstance(n, G.Transform):
            c = ser(n.child)
            idx = emit(N_TRANSFORM, [c], n.bbox, [x for row in n.m34 for x in row] + [x for row in n.inv34 for x in row])
        elif isinstance(n, G.Moving):
            c = ser(n.child)
            idx = emit(N_MOVING, [c], n.bbox, list(n.v0) + list(n.v1))
        elif isinstance(n, G.ConstantMedium):
            mi = media_count[0]
            media_count[0] += 1
            c = ser(n.child)
            idx = emit(N_MEDIUM, [c, mi], n.bbox, [n.density])
        elif isinstance(n, G.WithMaterial):
            c = ser(n.child)
            idx = emit(N_MATERIAL, [c, tabs.material(n.material)], n.bbox, [])
        else:
            raise RtUnsupported(f"cannot serialize {type(n).__name__}")
        memo[id(n)] = idx
        return idx

    root = ser(world)
    ni = np.array(node_i, dtype=np.int32).reshape(-1, NI)
    nd = np.array(node_d, dtype=np.float64).reshape(-1, ND)
    ch = np.array(children if children else [0], dtype=np.int32)
    tex, texels, perlin = tabs.texture_array()
    return SerializedTree(ni, nd, ch, root, tabs.material_array(), tex, media_count[0], texels, perlin)
