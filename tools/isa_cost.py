#!/usr/bin/env python3
"""Per-step ISA cost table of a fast kernel: the VALU instructions of one symbol step in the
built library's gfx950 code object, each with its measured issue cost (cycles per wave64
instruction per SIMD with many waves, profiles/r02_valu_microbench.txt, tools/microbench.hip).

usage: python3 tools/isa_cost.py <kernel mangled-name prefix> <step start regex> [obj=ans_kernels]
The step is the instruction sequence from the second match of <step start regex> in the
kernel's main loop to the next match (e.g. 'v_ffbh_u32' for the decoders, 'v_fma_f64' for the
encoders).  Prints a markdown table and the totals.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = "/opt/rocm/lib/llvm/bin"

# measured classes (profiles/r02_valu_microbench.txt); instructions not measured there take the
# class of their encoding: VOP3 / 3-operand / 64-bit ~4.4, simple VOP2 32-bit ~2.4
COST = {
    "v_add_u32": 2.86, "v_add_u32_e64": 2.60, "v_sub_u32": 2.50, "v_subrev_u32": 2.50, "v_xor_b32": 2.58,
    "v_and_b32": 2.32, "v_or_b32": 2.32, "v_lshrrev_b32": 2.40, "v_ashrrev_i32": 2.32, "v_lshlrev_b16": 2.33,
    "v_add_u16": 2.39, "v_lshlrev_b32": 4.17, "v_mul_lo_u32": 4.47, "v_mul_hi_u32": 4.43, "v_mul_u32_u24": 4.32,
    "v_mad_u64_u32": 5.47, "v_lshrrev_b64": 4.79, "v_lshlrev_b64": 4.79, "v_lshl_add_u64": 4.93, "v_fma_f64": 4.52,
    "v_fmac_f64": 4.52, "v_cvt_f64_u32": 4.27, "v_alignbyte_b32": 4.26, "v_perm_b32": 4.24, "v_add3_u32": 4.43,
    "v_lshl_or_b32": 4.32, "v_bfe_u32": 4.18, "v_mad_u32_u24": 4.42, "v_ffbh_u32": 4.10, "v_min_u32": 4.29,
    "v_max_u32": 4.18, "v_cndmask_b32": 4.57, "v_cmp": 4.77, "v_add_co_u32": 4.83, "v_addc_co_u32": 4.80,
    "v_sub_co_u32": 4.61, "v_and_or_b32": 4.39, "v_or3_b32": 4.27, "v_bfi_b32": 4.28, "v_lshl_add_u32": 4.41,
    "v_rcp_f64": 16.31, "v_mov_b32": 2.4, "v_mov_b64": 4.8,
}


def cost(op, line):
    base = op.split("_e32")[0].split("_e64")[0].split("_sdwa")[0]
    if base.startswith("v_cmp"):
        return COST["v_cmp"] + (0.3 if "64" in base.split("_")[-1] else 0.0)
    if "_sdwa" in op:
        return 4.3  # SDWA forms issue in the slow class (tools/b16_probe.hip)
    return COST.get(base, 4.4)


def disassemble(obj):
    with tempfile.TemporaryDirectory() as t:
        subprocess.check_call([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/f.bin",
                               os.path.join(ROOT, "shuffle-coding_amd", "build", obj + ".o")])
        subprocess.check_call([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/f.bin",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/k.co"])
        return subprocess.check_output([f"{B}/llvm-objdump", "-d", "--no-show-raw-insn", f"{t}/k.co"], text=True)


def main():
    name, start = sys.argv[1], sys.argv[2]
    obj = sys.argv[3] if len(sys.argv) > 3 else "ans_kernels"
    text = disassemble(obj).split("\n")
    i0 = next(i for i, ln in enumerate(text) if re.match(r"^[0-9a-f]+ <" + re.escape(name), ln))
    i1 = next(i for i in range(i0 + 1, len(text)) if re.match(r"^[0-9a-f]+ <", text[i]))
    body = [ln.split("//")[0].strip() for ln in text[i0 + 1:i1]]
    body = [ln for ln in body if ln]
    hits = [i for i, ln in enumerate(body) if re.search(start, ln)]
    a, b = hits[1], hits[2]
    rows, total_v, total_c, lds = [], 0, 0.0, 0
    for ln in body[a:b]:
        op = ln.split()[0]
        if op.startswith("v_"):
            c = cost(op, ln)
            total_v += 1
            total_c += c
            rows.append((ln, f"{c:.2f}"))
        elif op.startswith("ds_"):
            lds += 1
            rows.append((ln, "LDS"))
        else:
            rows.append((ln, ""))
    print(f"### {name} — one step ({start!r} to the next)\n")
    print("| instruction | issue cycles |\n|---|---|")
    for ln, c in rows:
        print(f"| `{ln}` | {c} |")
    print(f"\n**{total_v} VALU, {total_c:.1f} issue cycles, {lds} LDS instructions per step**")


if __name__ == "__main__":
    main()
