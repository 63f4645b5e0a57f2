#!/usr/bin/env python3
"""Per-kernel resource usage from hipcc -Rpass-analysis=kernel-resource-usage remarks.

The Makefile writes the remarks of every compile to build/csrc/*.ru.txt; `parse`
turns them into {mangled name: {VGPRs, AGPRs, ScratchSize, Occupancy, ...}} and
the CLI prints a table (optionally filtered by a substring of the demangled name).
tests/test_resource_usage_cpu.py uses `load_build` to assert that the step and
resident kernels do not spill to scratch.

usage: resource_usage.py [FILTER]
"""
import glob
import os
import re
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
BUILD_DIR = os.path.normpath(os.path.join(_HERE, "..", "..", "build", "csrc"))
_FIELD = re.compile(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                    r"LDS Size \[bytes/block\]|TotalSGPRs|SGPRs Spill|VGPRs Spill): (\d+)")


def parse(text: str) -> dict:
    rows, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = rows.setdefault(m.group(1), {})
            continue
        m = _FIELD.search(line)
        if m and cur is not None:
            key = m.group(1) if m.group(1) in ("SGPRs Spill", "VGPRs Spill") else m.group(1).split()[0]
            cur[key] = int(m.group(2))
    return rows


def load_build(build_dir: str = BUILD_DIR) -> dict:
    rows = {}
    for p in sorted(glob.glob(os.path.join(build_dir, "*.ru.txt"))):
        with open(p) as f:
            rows.update(parse(f.read()))
    return rows


def loop_scratch(asm: str, name: str, min_depth: int = 1) -> dict:
    """Scratch (spill) instructions of kernel `name` in device assembly text (hipcc -S
    --cuda-device-only), split into those inside a loop nest at least `min_depth` deep
    (LLVM's `; in Loop: ... Depth=N` block comments) and the rest: {"loop": [...],
    "other": [...]} of instruction lines."""
    i = asm.index(name + ":")
    body = asm[i:asm.index(".Lfunc_end", i)]
    out, depth = {"loop": [], "other": []}, 0
    for line in body.splitlines():
        m = re.match(r"^(?:\.LBB\d+_\d+:|; %bb\.\d+:)(.*)", line)
        if m:
            d = re.search(r"in Loop:.*Depth=(\d+)", m.group(1))
            depth = int(d.group(1)) if d else 0
        elif "scratch_" in line:
            out["loop" if depth >= min_depth else "other"].append(line.strip())
    return out


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return [o.replace("nlspn::", "").replace("void ", "") for o in out[:len(names)]]


def main():
    filt = sys.argv[1] if len(sys.argv) > 1 else ""
    rows = load_build()
    names = sorted(rows)
    for n, d in zip(names, demangle(names)):
        if filt in d:
            r = rows[n]
            print(f"{d[:100]:100s} vgpr={r.get('VGPRs')} sgpr={r.get('TotalSGPRs')} scratch={r.get('ScratchSize')} "
                  f"occ={r.get('Occupancy')} lds={r.get('LDS')}")


if __name__ == "__main__":
    main()
