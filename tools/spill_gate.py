"""Build gate: no render-kernel instantiation of the product library may spill VGPRs.

The kernel translation units are compiled with -Rpass-analysis=kernel-resource-usage
(raytrace_amd/csrc/Makefile); their remarks land in <objdir>/<unit>.res.  This script parses them,
writes the resource table (<objdir>/resources.txt: kernel, VGPRs, VGPR spills, SGPR spills, scratch
bytes per lane, occupancy) and exits non-zero if any rt_render_kernel instantiation spills VGPRs
or uses scratch.  Every instantiation in these units is one rt_render_kernel.h render_kernel_of can
select, so the gate covers exactly the dispatchable kernels.

Why: a round-5 experiment build whose FP32 instanced kernel spilled 6 VGPRs rendered frames that
differed from run to run (profiles/r5/bigwg, profiles/r6/nondet).  The same class without spills is
bit-deterministic.  VGPR spill stores and reloads are exec-masked; one placed in a divergent region
and reloaded under a wider mask restores lanes the store never wrote.  SGPR spills go to VGPR lanes
through v_writelane / v_readlane, which ignore the exec mask, so they are reported but not gated.

usage: python tools/spill_gate.py <objdir> [--table-only]
"""
import glob
import os
import re
import subprocess
import sys

FIELDS = {
    "VGPRs": "vgpr",
    "VGPRs Spill": "vspill",
    "SGPRs Spill": "sspill",
    "ScratchSize [bytes/lane]": "scratch",
    "Occupancy [waves/SIMD]": "occ",
}


def parse(text: str) -> list[dict]:
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([^:]+?): (\S+) \[-Rpass-analysis", line)
        if m and cur is not None and m.group(1) in FIELDS:
            v = m.group(2)
            cur[FIELDS[m.group(1)]] = int(v) if v.isdigit() else v
    return rows


def demangle(names: list[str]) -> list[str]:
    tool = next((t for t in ("/opt/rocm/lib/llvm/bin/llvm-cxxfilt", "/usr/bin/c++filt") if os.path.exists(t)), None)
    if not names or tool is None:
        return names
    out = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return [o if o else n for o, n in zip(out, names)]


def main() -> int:
    objdir = sys.argv[1]
    rows = []
    for res in sorted(glob.glob(os.path.join(objdir, "*.res"))):
        rows += parse(open(res, errors="replace").read())
    kernels = [r for r in rows if "rt_render_kernel" in r["name"]]
    for r, d in zip(kernels, demangle([r["name"] for r in kernels])):
        r["pretty"] = d.replace("(KernelParamsT<double>)", "").replace("(KernelParamsT<float>)", "")
    kernels.sort(key=lambda r: r["pretty"])
    with open(os.path.join(objdir, "resources.txt"), "w") as f:
        f.write("# kernel vgpr vspill sspill scratch occ (tools/spill_gate.py)\n")
        for r in kernels:
            f.write(f"{r['pretty']} {r.get('vgpr')} {r.get('vspill')} {r.get('sspill')} {r.get('scratch')} {r.get('occ')}\n")
    if not kernels:
        print("spill_gate: no render-kernel resource remarks found in", objdir, file=sys.stderr)
        return 1
    bad = [r for r in kernels if r.get("vspill", 0) != 0 or r.get("scratch", 0) != 0]
    print(f"spill_gate: {len(kernels)} render-kernel instantiations, {len(bad)} with VGPR spills / scratch")
    for r in bad:
        print(f"  SPILL {r['pretty']}: {r.get('vgpr')} VGPRs, {r.get('vspill')} spilled, scratch {r.get('scratch')} B/lane, "
              f"occupancy {r.get('occ')}", file=sys.stderr)
    if "--table-only" in sys.argv:
        return 0
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
