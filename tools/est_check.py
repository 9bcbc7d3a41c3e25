#!/usr/bin/env python3
"""Exact-rounding check (fractions) of the C3 decoder's bit-built quotient estimate (ans_fast.hpp
DecChain::renorm_div_u, kNormStd): q_m in {q - 1, q} over norms in [2^16, 2^31] and heads at
multiples of the norm, 2^12 around them and at random.  usage: python3 tools/est_check.py"""
# exhaustive-ish check of the decoder's shifted-head quotient estimate (from below, q_m in {q-1, q})
import random
from fractions import Fraction as F
MAGIC = 562949953421311.875  # 2^49 - 1/8
def est(x, n):
    rcp = 1.0 / n
    rcp8 = rcp * 0.125
    C = MAGIC - (2.0 ** 61) * rcp
    V = F(2 ** 64 + ((x >> 12) << 12))
    t = float(V * F(rcp8) + F(C))  # one rounding (fma)
    m = (F(t) - 2 ** 49) * 8
    assert m.denominator == 1, (x, n, t)
    return int(m)
def old(x, n):
    rcp8 = (1.0 / n) * 0.125
    t = float(F(float(x)) * F(rcp8) + F(MAGIC))  # xd = fl(x) (cvt/fma exact for hi*2^32+lo? fl(x) rounding)
    return int((F(t) - 2 ** 49) * 8)
random.seed(1)
bad = 0; cnt = 0; hits = {}
norms = [1 << 16, (1 << 16) + 1, 65537, 139224331, 134561356, (1 << 31) - 1, 1 << 31, 3 * 2 ** 29 + 7]
norms += [random.randrange(1 << 16, (1 << 31) + 1) for _ in range(300)]
for n in norms:
    K = (1 << 56) // n; L = n * K
    xs = [L, (1 << 64) - 1, (1 << 64) - 2]
    for _ in range(60):
        q = random.randrange(L // n, ((1 << 64) - 1) // n + 1)
        for d in (-2, -1, 0, 1, 2, 4095, 4096, 4097, -4095, -4096, -4097):
            x = q * n + d
            if L <= x < (1 << 64): xs.append(x)
        xs.append(random.randrange(L, 1 << 64))
    for x in xs:
        q = x // n
        m = est(x, n)
        cnt += 1
        k = m - q
        hits[k] = hits.get(k, 0) + 1
        if k not in (-1, 0):
            bad += 1
            if bad < 5: print("BAD", x, n, m, q)
print(cnt, "cases; q_m - q histogram", hits, "bad", bad)
