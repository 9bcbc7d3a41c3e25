#!/usr/bin/env python3
"""Average VALU count and issue cycles per step of a kernel's unrolled main loop in the built
library: from the first occurrence of a per-step marker instruction (e.g. v_ffbh_u32 for the
decoders, v_fmac_f64 for the C3 encoder) over N steps, so the once-per-unit work (points, line
stores, output packing, deferred tests) is averaged in, where tools/isa_cost.py shows one step.

usage: python3 tools/loop_avg.py <unit> <mangled-name prefix> <marker> <steps>
"""
import re, sys
sys.path.insert(0, 'tools')
from isa_cost import disassemble, cost
t = disassemble(sys.argv[1]).split('\n')
i0 = next(i for i, l in enumerate(t) if re.match(r'^[0-9a-f]+ <' + sys.argv[2], l))
i1 = next(i for i in range(i0 + 1, len(t)) if re.match(r'^[0-9a-f]+ <', t[i]))
body = [l.split('//')[0].strip() for l in t[i0 + 1:i1]]
ff = [k for k, l in enumerate(body) if l.startswith(sys.argv[3])]
n = int(sys.argv[4])  # steps in the main loop, from the first marker
a, b = ff[0], ff[n]
v = [l for l in body[a:b] if l.startswith('v_')]
cyc = sum(cost(l.split()[0], l) for l in v)
print(f"{len(v) / n:.2f} VALU, {cyc / n:.1f} issue cycles per step over {n} steps (points, stores, packing included)")
