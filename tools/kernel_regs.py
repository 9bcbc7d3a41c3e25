#!/usr/bin/env python3
"""VGPR / AGPR counts, spills and scratch bytes of the kernels in a built unit's gfx950 code
object (the code object's metadata notes).  A kernel that spills reads and writes scratch in HBM
per step: the first thing to check when a layout change (e.g. 1,024-lane workgroups, 128 VGPRs
a lane) makes a kernel slower.

usage: python3 tools/kernel_regs.py <unit, e.g. ans_codecs_indep_enc> [name regex] [--spills]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = "/opt/rocm/lib/llvm/bin"


def notes(unit):
    with tempfile.TemporaryDirectory() as t:
        subprocess.check_call([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/f.bin",
                               os.path.join(ROOT, "shuffle-coding_amd", "build", unit + ".o")])
        subprocess.check_call([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/f.bin",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/k.co"])
        return subprocess.check_output([f"{B}/llvm-readelf", "--notes", f"{t}/k.co"], text=True)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    unit, pat = args[0], (args[1] if len(args) > 1 else ".")
    only_spills = "--spills" in sys.argv
    for blk in re.split(r"\n\s+- \.", notes(unit)):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or not re.search(pat, m.group(1)):
            continue
        g = lambda k: int((re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "0"])[1])  # noqa: E731
        sp = g("vgpr_spill_count") + g("sgpr_spill_count")
        if only_spills and not sp:
            continue
        print(f"vgpr {g('vgpr_count'):3d} agpr {g('agpr_count'):3d} spill {sp:4d} "
              f"scratch {g('private_segment_fixed_size'):4d}  {m.group(1)}")


if __name__ == "__main__":
    main()
