"""The C-ABI boundary: librt_amd.so loads without a GPU, exports every function include/rt.h
declares, and the record layouts the Python mirror writes match the header's C layout."""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np

from conftest import ROOT
from raytrace_amd import _lib
from raytrace_amd import scene as S

HEADER = os.path.join(ROOT, "include", "rt.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(rt_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.EXPORTED)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (rt_\w+)", out.stdout))
    assert set(names) <= exported
    assert L.rt_abi_version() == _lib.ABI_VERSION == 6


def test_host_only_entry_points_without_gpu():
    L = _lib.load()
    from raytrace_amd import scenes
    cs = _lib.camera_struct(scenes.readme_scene()[0])
    assert L.rt_image_height(ctypes.byref(cs)) == 338
    ex = _lib.exec_struct(n_shards=3, shard=1, row_block=4)
    assert L.rt_shard_rows(338, ctypes.byref(ex)) == 116       # ceil(ceil(338/4)/3)*4
    assert L.rt_shard_row(0, ctypes.byref(ex)) == 4 and L.rt_shard_row(5, ctypes.byref(ex)) == 17
    bad = _lib.exec_struct(n_shards=2, shard=2)
    assert L.rt_shard_rows(100, ctypes.byref(bad)) == _lib.RT_E_INVALID
    assert b"invalid" in L.rt_last_error()


C_LAYOUT = r"""
#include <stdio.h>
#include <stddef.h>
#include "rt.h"
#define P(T) printf(#T " %zu\n", sizeof(T))
#define O(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))
int main(void) {
  P(rt_prim); O(rt_prim, p); O(rt_prim, uv); O(rt_prim, uvframe);
  P(rt_medium); O(rt_medium, material);
  P(rt_material); O(rt_material, param);
  P(rt_texture); O(rt_texture, c0); O(rt_texture, params);
  P(rt_motion); P(rt_uvframe);
  P(rt_scene); O(rt_scene, prims); O(rt_scene, uvframes); O(rt_scene, texels); O(rt_scene, perlin);
  P(rt_perlin); O(rt_perlin, grad);
  P(rt_camera_settings); O(rt_camera_settings, image_width); O(rt_camera_settings, background_c0);
  O(rt_camera_settings, defocus_angle); O(rt_camera_settings, redirect_targets);
  P(rt_redirect_target); P(rt_exec); O(rt_exec, flags); O(rt_exec, devices); P(rt_stats); O(rt_stats, samples);
  O(rt_stats, device_allocs); O(rt_stats, kernel_block);
  return 0;
}
"""


def test_record_layouts_match_header():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "layout.c")
        exe = os.path.join(d, "layout")
        open(src, "w").write(C_LAYOUT)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, src], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    c = dict(line.rsplit(" ", 1) for line in out.strip().splitlines())
    c = {k: int(v) for k, v in c.items()}
    assert c["rt_prim"] == S.PRIM_DTYPE.itemsize
    assert c["rt_prim.p"] == S.PRIM_DTYPE.fields["p"][1] and c["rt_prim.uv"] == S.PRIM_DTYPE.fields["uv"][1]
    assert c["rt_prim.uvframe"] == S.PRIM_DTYPE.fields["uvframe"][1]
    assert c["rt_medium"] == S.MEDIUM_DTYPE.itemsize and c["rt_medium.material"] == S.MEDIUM_DTYPE.fields["material"][1]
    assert c["rt_material"] == S.MATERIAL_DTYPE.itemsize and c["rt_material.param"] == S.MATERIAL_DTYPE.fields["param"][1]
    assert c["rt_texture"] == S.TEXTURE_DTYPE.itemsize and c["rt_texture.c0"] == S.TEXTURE_DTYPE.fields["c0"][1]
    assert c["rt_texture.params"] == S.TEXTURE_DTYPE.fields["params"][1]
    assert c["rt_motion"] == S.MOTION_DTYPE.itemsize and c["rt_uvframe"] == S.UVFRAME_DTYPE.itemsize
    assert c["rt_scene"] == ctypes.sizeof(_lib.RtScene)
    assert c["rt_scene.uvframes"] == _lib.RtScene.uvframes.offset
    assert c["rt_scene.texels"] == _lib.RtScene.texels.offset and c["rt_scene.perlin"] == _lib.RtScene.perlin.offset
    from raytrace_amd.perlin import PERLIN_DTYPE
    assert c["rt_perlin"] == PERLIN_DTYPE.itemsize and c["rt_perlin.grad"] == PERLIN_DTYPE.fields["grad"][1]
    assert c["rt_camera_settings"] == ctypes.sizeof(_lib.RtCameraSettings)
    for f in ("image_width", "background_c0", "defocus_angle", "redirect_targets"):
        assert c[f"rt_camera_settings.{f}"] == getattr(_lib.RtCameraSettings, f).offset, f
    assert c["rt_redirect_target"] == ctypes.sizeof(_lib.RtRedirectTarget)
    assert c["rt_exec"] == ctypes.sizeof(_lib.RtExec)
    assert c["rt_exec.flags"] == _lib.RtExec.flags.offset and c["rt_exec.devices"] == _lib.RtExec.devices.offset
    assert c["rt_stats"] == ctypes.sizeof(_lib.RtStats) and c["rt_stats.samples"] == _lib.RtStats.samples.offset
    assert c["rt_stats.device_allocs"] == _lib.RtStats.device_allocs.offset
    assert c["rt_stats.kernel_block"] == _lib.RtStats.kernel_block.offset


def test_render_fails_loudly_without_a_device():
    """No CPU fallback: on a machine without a GPU the product path raises."""
    import torch
    if torch.cuda.is_available():
        return
    import pytest
    import raytrace_amd as R
    from raytrace_amd import scenes
    with pytest.raises(R.RtDeviceError):
        R.raytrace(*scenes.cornell_box(spp=1, width=4))
    with pytest.raises(R.RtDeviceError):
        R.DeviceScene(scenes.cornell_box()[1])


def test_scene_validation_errors_before_device():
    """rt_render validates the camera before touching the device (RT_E_INVALID / UNSUPPORTED)."""
    import pytest
    import raytrace_amd as R
    from raytrace_amd import scenes
    cs, world, seed = scenes.cornell_box(spp=1, width=4)
    with pytest.raises(R.RtInvalid):
        R.raytrace(cs.replace(cs_samplesPerPixel=0), world, seed)
    with pytest.raises(R.RtInvalid):
        R.raytrace(cs.replace(cs_aspectRatio=0.0), world, seed)
    with pytest.raises(R.RtUnsupported):
        R.raytrace(cs.replace(cs_redirectTargets=[(0.01, (0, 0, 0), (1, 0, 0), (0, 1, 0))] * 9), world, seed)
    with pytest.raises(ValueError):
        R.raytrace(cs, world, seed, precision="f16")
    with pytest.raises(R.RtUnsupported):  # column / row are 16-bit in the kernels
        R.raytrace(cs.replace(cs_imageWidth=65536, cs_aspectRatio=65536.0), world, seed)
    # a tile beyond 2^31 pixels (32-bit pixel ids) is refused before any buffer is written
    L = _lib.load()
    from raytrace_amd.scene import flatten
    big = cs.replace(cs_imageWidth=65535, cs_aspectRatio=65535 / 40000)
    c, sc, ex = _lib.camera_struct(big), _lib.scene_struct(flatten(world)), _lib.exec_struct()
    out = np.zeros(3)
    assert L.rt_render(ctypes.byref(c), ctypes.byref(sc), 1, ctypes.byref(ex), out.ctypes.data, None) == _lib.RT_E_UNSUPPORTED
    assert b"2^31" in L.rt_last_error()


def test_device_list_validation_before_device():
    """ABI v3 device lists: malformed lists are RT_E_INVALID before any device is touched."""
    import pytest
    from raytrace_amd import scenes
    L = _lib.load()
    cs, world, seed = scenes.cornell_box(spp=1, width=4)
    from raytrace_amd.scene import flatten
    c, sc = _lib.camera_struct(cs), _lib.scene_struct(flatten(world))
    out = np.zeros((4, 4, 3))
    ex = _lib.exec_struct(devices=[0, 0])
    ex.n_shards = 2  # a device list renders the whole image
    assert L.rt_render(ctypes.byref(c), ctypes.byref(sc), 1, ctypes.byref(ex), out.ctypes.data, None) == _lib.RT_E_INVALID
    assert b"n_shards" in L.rt_last_error()
    ex = _lib.exec_struct(devices=[0])
    ex.n_devices = 65
    assert L.rt_render(ctypes.byref(c), ctypes.byref(sc), 1, ctypes.byref(ex), out.ctypes.data, None) == _lib.RT_E_INVALID
    with pytest.raises(ValueError):
        _lib.exec_struct(precision="bf16")


def test_exec_flags_validated_before_device():
    """rt_exec.flags: an unknown bit, or both 8-bit encodings, is RT_E_INVALID (not a silent choice),
    before any device is touched."""
    from raytrace_amd import scenes
    from raytrace_amd.scene import flatten
    L = _lib.load()
    cs, world, seed = scenes.cornell_box(spp=1, width=4)
    c, sc = _lib.camera_struct(cs), _lib.scene_struct(flatten(world))
    out = np.zeros((4, 4, 3))
    for flags, msg in [(0x100, b"unknown"), (2 | 4, b"exclusive"), (1 | 2 | 4, b"exclusive")]:
        ex = _lib.exec_struct()
        ex.flags = flags
        assert L.rt_render(ctypes.byref(c), ctypes.byref(sc), 1, ctypes.byref(ex), out.ctypes.data, None) == _lib.RT_E_INVALID
        assert msg in L.rt_last_error(), (flags, L.rt_last_error())
    # RT_EXEC_SOLO is a known bit: the call gets past the flag check (and then fails only for want
    # of a device here, or renders on a GPU box)
    ex = _lib.exec_struct(solo=True)
    assert ex.flags == _lib.RT_EXEC_SOLO == 8
    rc = L.rt_render(ctypes.byref(c), ctypes.byref(sc), 1, ctypes.byref(ex), out.ctypes.data, None)
    assert rc != _lib.RT_E_INVALID or b"unknown" not in L.rt_last_error(), L.rt_last_error()


def test_haskell_binding_offsets_match_header():
    """hs/Graphics/Ray/Device.hs marshals the rt.h records by byte offset (GHC is absent here, so
    it cannot be compiled): every `-- LAYOUT <struct>[.<field>] <bytes>` line it declares must
    equal the C compiler's sizeof / offsetof, and its foreign imports must name exported symbols."""
    hs = open(os.path.join(ROOT, "hs", "Graphics", "Ray", "Device.hs")).read()
    decl = re.findall(r"^-- LAYOUT (\w+)(?:\.(\w+))? (\d+)$", hs, flags=re.M)
    assert len(decl) >= 30
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "rt.h"', "int main(void) {"]
    for st, field, _ in decl:
        expr = f"offsetof({st}, {field})" if field else f"sizeof({st})"
        lines.append(f'  printf("%zu\\n", {expr});')
    lines += ["  return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "hs_layout.c"), os.path.join(d, "hs_layout")
        open(src, "w").write("\n".join(lines) + "\n")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, src], check=True)
        got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    for (st, field, want), g in zip(decl, got):
        assert int(want) == g, (st, field, want, g)
    imports = re.findall(r'foreign import ccall (?:safe|unsafe) "(\w+)"', hs)
    assert set(imports) <= set(_lib.EXPORTED) and "rt_render" in imports
    assert 'error "' not in hs  # no unimplemented stubs


def test_haskell_binding_needs_no_reference_edit():
    """Device.hs embeds Noise.hs's permutation constants (the reference does not export them) and
    re-exports the reference's raw constructors as bundled pattern synonyms (custom geometries,
    materials and textures compile unchanged and render through the CPU fallback)."""
    import json
    hs = open(os.path.join(ROOT, "hs", "Graphics", "Ray", "Device.hs")).read()
    assert "import Graphics.Ray.Noise" not in hs
    with open(os.path.join(ROOT, "raytrace_amd", "data", "perlin_perm.json")) as f:
        perm = json.load(f)
    for name in ("permX", "permY", "permZ"):
        m = re.search(name + r"Table =\s*\[([^\]]*)\]", hs)
        assert m, name
        assert [int(x) for x in m.group(1).replace("\n", " ").split(",")] == perm[name], name
    for con in ("Geometry", "Material", "Texture"):
        assert f"{con}({con})" in hs and f"pattern {con} ::" in hs, con
        assert f"fromReference{con}" in hs
    # RT_E_UNSUPPORTED (-3) and RT_E_STACK (-5) go to the CPU path
    assert "code == -3 || code == -5" in hs
