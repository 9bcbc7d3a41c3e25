"""Rates of the codecs beside Categorical on the GPU: Independent<Categorical>
with a table per position (src/codec.rs:366-403), IID<Uniform(2^40)> (src/codec.rs:13-49) and
IID<LogUniform(47)> (src/codec.rs:561-611, MaxBenfordIID's item).  Host-buffer API calls
(best of 3, round trip verified); the kernel times come from a rocprofv3 --kernel-trace --stats
run of this script (profiles/r03_codecs_kernel_stats.csv).  Prints one JSON line.
usage: python tools/codecs_bench.py [log2n_independent=26] [log2n_uniform=24]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "shuffle-coding_amd")]
import numpy as np  # noqa: E402

import ans_amd as A  # noqa: E402


def timed(fn, reps=3):
    best, out = None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, out


def main():
    li = int(sys.argv[1]) if len(sys.argv) > 1 else 26
    lu = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    L = 4096
    rng = np.random.default_rng(3)
    g = A.Gpu(0)
    res = {"chunk_len": L}

    # Independent: five 256-symbol tables (norm in the fast range), position k uses table k % 5
    n = 1 << li
    cats, ms = [], []
    for t in range(5):
        m = rng.integers(1, 1 << 16, 256).astype(np.uint64)
        ms.append(m)
        cats.append(A.Categorical(m))
    ts = A.GpuTableSet(g, cats)
    tids = (np.arange(n) % 5).astype(np.uint32)
    syms = np.empty(n, np.uint8)
    for t in range(5):
        p = ms[t].astype(np.float64)
        sel = tids == t
        syms[sel] = rng.choice(256, size=int(sel.sum()), p=p / p.sum())
    te, enc = timed(lambda: ts.encode_chunks(tids, syms, L))
    td, back = timed(lambda: ts.decode_chunks(tids, *enc, L, np.uint8))
    assert np.array_equal(back, syms)
    res["independent"] = {"symbols": n, "tables": 5, "table_symbols": 256, "sym_bytes": 1,
                          "encode_ms": round(1e3 * te, 2), "decode_ms": round(1e3 * td, 2),
                          "gib_s": round(n / (te + td) / 2**30, 3), "compressed_bytes": int(len(enc[0]))}

    # Uniform(2^40): u64 symbols
    n = 1 << lu
    gu = A.GpuUniform(g, 1 << 40)
    xs = rng.integers(0, 1 << 40, n, dtype=np.uint64)
    te, enc = timed(lambda: gu.encode_chunks(xs, L))
    td, back = timed(lambda: gu.decode_chunks(*enc, n, L, np.uint64))
    assert np.array_equal(back, xs)
    res["uniform_2^40"] = {"symbols": n, "sym_bytes": 8, "encode_ms": round(1e3 * te, 2),
                           "decode_ms": round(1e3 * td, 2), "gib_s": round(8 * n / (te + td) / 2**30, 3),
                           "compressed_bytes": int(len(enc[0]))}

    # LogUniform(47): bit lengths uniform over 0..47, the bits below the top one uniform
    bits = rng.integers(0, 48, n)
    low = rng.integers(0, 1 << 46, n, dtype=np.uint64)
    xs = np.where(bits == 0, 0, (np.uint64(1) << np.maximum(bits - 1, 0).astype(np.uint64)) |
                  (low & ((np.uint64(1) << np.maximum(bits - 1, 0).astype(np.uint64)) - np.uint64(1)))).astype(np.uint64)
    gl = A.GpuLogUniform(g, 47)
    te, enc = timed(lambda: gl.encode_chunks(xs, L))
    td, back = timed(lambda: gl.decode_chunks(*enc, n, L, np.uint64))
    assert np.array_equal(back, xs)
    res["loguniform_47"] = {"symbols": n, "sym_bytes": 8, "encode_ms": round(1e3 * te, 2),
                            "decode_ms": round(1e3 * td, 2), "gib_s": round(8 * n / (te + td) / 2**30, 3),
                            "compressed_bytes": int(len(enc[0]))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
