#!/usr/bin/env python3
"""Static instruction mix of a kernel's main loop in the built library (gfx950 code object):
the longest backward branch's body, i.e. the straight-line path a wave runs per iteration
(out-of-line blocks the compiler moved past the loop, such as the voted fix-up branches, are
not counted).  Prints VALU / SALU / LDS / VMEM counts, per symbol when the symbols per
iteration are given, and the VALU opcode histogram.

usage: python3 tools/loop_valu.py <unit, e.g. ans_launch_dec_u8> <mangled-name regex> [symbols per iteration]
"""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_cost import cost, disassemble  # noqa: E402


def main():
    unit, pat = sys.argv[1], sys.argv[2]
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    text = disassemble(unit).split("\n")
    starts = [i for i, ln in enumerate(text) if re.match(r"^[0-9a-f]+ <", ln)]
    cands = [i for i in starts if re.search(pat, text[i])]
    if not cands:
        sys.exit(f"no kernel matches {pat!r}")
    i0 = cands[0]
    i1 = next((i for i in starts if i > i0), len(text))
    print(text[i0])
    body = []
    for ln in text[i0 + 1:i1]:  # "\t<instruction>  // <address>: <encoding> ..."
        m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):", ln)
        if m:
            body.append((int(m.group(2), 16), m.group(1).strip()))
    addr_idx = {a: k for k, (a, _) in enumerate(body)}
    best = None
    for k, (a, ins) in enumerate(body):
        m = re.match(r"s_cbranch_\w+\s+(-?\d+)|s_branch\s+(-?\d+)", ins)
        if not m:
            continue
        off = int(m.group(1) or m.group(2))
        off = off - 65536 if off >= 32768 else off  # (printed as the unsigned 16-bit field)
        tgt = a + 4 + 4 * off
        if tgt < a and tgt in addr_idx:
            span = k - addr_idx[tgt]
            if best is None or span > best[0]:
                best = (span, addr_idx[tgt], k)
    if best is None:
        sys.exit("no loop")
    _, lo, hi = best
    hist = collections.Counter()
    n = collections.Counter()
    cyc = 0.0
    for _, ins in body[lo:hi + 1]:
        op = ins.split()[0] if ins else ""
        if op.startswith("v_"):
            n["valu"] += 1
            hist[op] += 1
            cyc += cost(op, ins)
        elif op.startswith("s_"):
            n["salu"] += 1
        elif op.startswith("ds_"):
            n["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            n["vmem"] += 1
    print(f"loop: {hi - lo + 1} instructions; " + ", ".join(f"{k} {v}" for k, v in sorted(n.items()))
          + f"; VALU issue cycles {cyc:.1f}")
    if per:
        print(f"per symbol ({per} per iteration): VALU {n['valu'] / per:.2f}, issue cycles {cyc / per:.1f}, "
              f"LDS {n['lds'] / per:.2f}")
    for op, c in hist.most_common():
        print(f"  {c:5d} {op}")


if __name__ == "__main__":
    main()
