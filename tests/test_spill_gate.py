"""The spill gate (tools/spill_gate.py) over the product library's kernel units: no render-kernel
instantiation that rt_render_kernel.h render_kernel_of can select may spill VGPRs or use scratch.

A round-5 experiment build whose FP32 instanced kernel spilled VGPRs rendered nondeterministically
(profiles/r5/bigwg, profiles/r6/nondet); every product class is kept spill-free since round 6.
The make rule writes the resource remarks next to each object; `make` here is a no-op when the
library is current (the driver's build() has normally run it), else it rebuilds the stale units."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raytrace_amd", "csrc")
OBJ = os.path.join(ROOT, "raytrace_amd", "_lib", "obj")


def test_no_render_kernel_spills():
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-C", CSRC, "-j", jobs], check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "spill_gate.py"), OBJ],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    table = open(os.path.join(OBJ, "resources.txt")).read().splitlines()[1:]
    # both precisions, flat and BVH classes, the narrow twins: the gate saw the whole library
    assert len(table) >= 150, len(table)
    assert any("rtk64::rt_render_kernel<0, 0, 0, false, false, 0, false>" in t for t in table)
    assert any("rtk64::rt_render_kernel<2, 0, 2, false, false, 1, true>" in t for t in table)
    for t in table:
        vgpr, vspill, sspill, scratch, occ = t.split()[-5:]
        assert vspill == "0" and scratch == "0", t


def test_gate_flags_a_spilling_kernel(tmp_path):
    # the parser on a synthetic remark block: a spilling instantiation fails the gate
    remark = ("x.h:1:1: remark: Function Name: _ZN3rtk16rt_render_kernelILi2ELi0ELi0ELb1ELb0ELi0ELb0EEEv13KernelParamsTIfE "
              "[-Rpass-analysis=kernel-resource-usage]\n")
    for k, v in (("VGPRs", 64), ("ScratchSize [bytes/lane]", 16), ("Occupancy [waves/SIMD]", 8), ("SGPRs Spill", 0),
                 ("VGPRs Spill", 4)):
        remark += f"x.h:1:1: remark:     {k}: {v} [-Rpass-analysis=kernel-resource-usage]\n"
    (tmp_path / "k.hip.o.res").write_text(remark)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "spill_gate.py"), str(tmp_path)],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "SPILL" in r.stderr, r.stdout + r.stderr
    assert "rtk::rt_render_kernel<2, 0, 0, true, false, 0, false> 64 4 0 16 8" in (tmp_path / "resources.txt").read_text()
